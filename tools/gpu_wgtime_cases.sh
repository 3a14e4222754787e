#!/bin/bash
# WGTIME debug build once, then per-workgroup timelines for several (split, n, p) cases.
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/wgt; mkdir -p $D
C=genomicbreedingmodels.jl_amd/csrc
for f in stats grm chol effects gibbs; do hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DGBM_DEBUG_WGTIME -c $C/$f.hip -o $D/$f.o || exit 1; done
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/capi.cpp -o $D/capi.o && hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/session.cpp -o $D/session.o || exit 1
hipcc --offload-arch=gfx950 -shared -fPIC $D/*.o -lrccl -o $D/libgbm.so || exit 1
for CASE in ${CASES:-1:5000:50000}; do
  IFS=: read -r S N P <<< "$CASE"
  if [ "$S" = auto ]; then unset GBM_GRM_SPLIT; else export GBM_GRM_SPLIT=$S; fi
  echo "== split $S n=$N p=$P"
  GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 200 python tools/${TOOL:-wgtime.py} $N $P || exit 1
done
