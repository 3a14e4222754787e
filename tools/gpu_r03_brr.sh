# Round 3: BRR super-block sweep — sampler GPU tests, then C4-shape timing (n = 10 000,
# p = 100 000) of the super-block sweep against the 128-block sweep (GBM_BRR_SB=0), A/B on one box,
# then the rocprofv3 kernel stats of the super-block path.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brrsb; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_brr.py -m gpu > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 250 > $OUT/c4_sb_$r.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
  cat $OUT/c4_sb_$r.json
  GBM_BRR_SB=0 timeout -k 10 300 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 250 > $OUT/c4_128_$r.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
  cat $OUT/c4_128_$r.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 60 > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
f=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1); head -12 "$f"
