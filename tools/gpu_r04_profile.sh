#!/bin/bash
# Round 4 C2 profile set on HEAD: bench line, rocprofv3 kernel trace (warm-up excluded summary),
# PMC FETCH_SIZE / WRITE_SIZE passes (pmc_grm.json with the kernel-source hash), SQ counters.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/prof; mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
python3 tools/rocprof_stats.py $OUT/trace --warmup 2 --steps 5 --csv $OUT/kernel_stats_timed.csv || exit 1
bash tools/profile_pmc.sh > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
cp gpurun_out/pmc/pmc_grm.json $OUT/pmc_grm.json
bash tools/profile_sq.sh > $OUT/sq_summary.txt 2>&1 || { tail $OUT/sq_summary.txt; exit 1; }
cat $OUT/sq_summary.txt
