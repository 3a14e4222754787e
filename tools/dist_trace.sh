# Kernel trace of rank 0's distributed solve at n = 50 000, R = 8 (tools/dist_solve_time.py, the redundant solve
# skipped) into gpurun_out/dist_trace/; the per-launch CSV is analysed on the host (tools/dist_trace_stats.py).
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dist_trace
mkdir -p $OUT
N=${N:-50000}
R=${R:-8}
SKIP_REDUNDANT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 tools/dist_solve_time.py $N $R > $OUT/time.json 2> $OUT/time.err &&
cat $OUT/time.json
