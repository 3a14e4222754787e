#!/bin/bash
# Round 4: the C3 bench line on one GPU (loci-streamed), two chunk sizes, then a kernel trace.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/c3; mkdir -p $OUT
timeout -k 10 400 python bench.py --individuals 50000 --loci 600000 --stream-chunk 300000 --steps 2 --warmup 1 \
  --no-cpu-baseline > $OUT/bench_c300k.json 2> $OUT/bench_c300k.err || exit 1
timeout -k 10 500 python bench.py --individuals 50000 --loci 600000 --stream-chunk 75000 --steps 2 --warmup 1 \
  > $OUT/bench_c75k.json 2> $OUT/bench_c75k.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --individuals 50000 --loci 600000 --stream-chunk 300000 --steps 1 --warmup 1 --no-cpu-baseline \
  > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
python3 tools/rocprof_stats.py $OUT/trace --warmup 1 --steps 1 --csv $OUT/kernel_stats_timed.csv
