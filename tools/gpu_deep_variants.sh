# GRM deep-pipeline variants: build, parity (test_gpu_parity), SYRK timing
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/deep; mkdir -p $OUT
C=genomicbreedingmodels.jl_amd/csrc
for V in ${VARIANTS:-"8:4" "12:3"}; do
  IFS=: read -r DB DN <<< "$V"
  D=$OUT/bk${DB}_nb${DN}; mkdir -p $D
  for f in stats grm chol effects gibbs; do hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DGBM_DEEP_BK=$DB -DGBM_DEEP_NBUF=$DN -c $C/$f.hip -o $D/$f.o || exit 1; done
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/capi.cpp -o $D/capi.o && hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/session.cpp -o $D/session.o || exit 1
  hipcc --offload-arch=gfx950 -shared -fPIC $D/*.o -lrccl -o $D/libgbm.so || exit 1
  echo "== deep BK $DB NBUF $DN"
  GBM_GRM_KERNEL=w4 GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu 2>&1 | tail -1
  GBM_GRM_KERNEL=w4 GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 120 python tools/time_grm.py || exit 1
done
