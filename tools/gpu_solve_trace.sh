#!/bin/bash
# Kernel trace of the GBLUP solve at n = N (default 5000): busy time and launch gaps per kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/strace; mkdir -p $OUT
REPS=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- python3 tools/time_solve.py > $OUT/log 2> $OUT/err || { tail $OUT/err; exit 1; }
cat $OUT/log
python3 tools/solve_timeline.py $(find $OUT/t -name 'run_kernel_trace.csv' | head -1)
