#!/bin/bash
# Distributed-factorisation rework: GPU parity tests, then the per-rank solve time at n = 50 000.
set -o pipefail
mkdir -p gpu_run_out gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_dist_solve.py tests/test_gpu_sharded.py tests/test_gpu_farming.py > gpurun_out/r04_dist_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/dist_solve_time.py 50000 8 4 2 > gpurun_out/r04_dist_solve_time.json 2> gpurun_out/r04_dist_solve_time.err
