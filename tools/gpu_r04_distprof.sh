#!/bin/bash
# Kernel trace of the per-rank distributed solve at n = 50 000, R = 8 (rank 0's work, copies for the
# all-gathers): where the per-rank time goes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/distprof
SKIP_REDUNDANT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/distprof -o dp -- python3 tools/dist_solve_time.py 50000 8 > gpurun_out/distprof/out.json 2> gpurun_out/distprof/err.txt || { tail gpurun_out/distprof/err.txt; exit 1; }
cat gpurun_out/distprof/out.json
f=$(find gpurun_out/distprof -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -c1-220
for t in 4096 12288; do
  GBM_DIST_TAIL_ROWS=$t SKIP_REDUNDANT=1 timeout -k 10 200 python3 tools/dist_solve_time.py 50000 8 > gpurun_out/distprof/tail$t.json 2>> gpurun_out/distprof/err.txt || exit 1
  echo "tail $t: $(cat gpurun_out/distprof/tail$t.json)"
done
