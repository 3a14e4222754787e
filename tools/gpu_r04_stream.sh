#!/bin/bash
# Round 4: loci-streamed fits — small-shape parity tests, then C3 (50 000 x 600 000) on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_streamed.py \
  > gpurun_out/r04_stream_tests.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_large.py -k c3_full \
  > gpurun_out/r04_c3_full.log 2>&1
[ $? -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-host-path > gpurun_out/r04_bench_parity.json 2> gpurun_out/r04_bench_parity.err
