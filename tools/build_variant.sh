#!/bin/bash
# Build a timing variant of libgbm from a modified copy of csrc: tools/build_variant.sh NAME DIR
# (DIR = a directory holding the csrc files to compile) -> variants/libgbm_NAME.so
set -e
NAME=$1; SRC=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/variants/build_$NAME; mkdir -p $OUT
pids=()
for f in stats.hip grm.hip grm_exact.hip chol.hip chol_flow.hip effects.hip gibbs.hip capi.cpp session.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$ROOT/genomicbreedingmodels.jl_amd/csrc -c $SRC/$f -o $OUT/$f.o ${VARIANT_FLAGS} &
  pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUT/*.o -lrccl -lrocprofiler-sdk-roctx -o $ROOT/variants/libgbm_$NAME.so
rm -rf $OUT
