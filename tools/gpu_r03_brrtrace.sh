set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brrtr; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_brr.py -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 tools/brr_trace.py > $OUT/trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
cat $OUT/trace.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 60 > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
cat $OUT/prof.json
f=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1); head -6 "$f" | cut -c1-60,200-320
GBM_BRR_LA2=0 timeout -k 10 300 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 60 > $OUT/v3.json 2> $OUT/v3.err || { tail $OUT/v3.err; exit 1; }
cat $OUT/v3.json
GBM_BRR_OWN_R=4 timeout -k 10 300 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 60 > $OUT/r4.json 2> $OUT/r4.err || { tail $OUT/r4.err; exit 1; }
cat $OUT/r4.json
GBM_BRR_OWN_R=4 timeout -k 10 300 python3 tools/brr_trace.py > $OUT/trace_r4.json 2> $OUT/trace_r4.err || { tail $OUT/trace_r4.err; exit 1; }
cat $OUT/trace_r4.json
