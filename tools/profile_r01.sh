# rocprofv3 kernel-trace summary of the bench (no PMC), then separate PMC passes on the GRM.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit $?
find $OUT/trace -name "*stats*" | head
