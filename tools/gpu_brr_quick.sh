# BRR: sampler GPU tests, then C4-shape timing (n = 10 000, p = 100 000) of the sweep, twice
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brrq; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_brr.py -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 250 > $OUT/c4_$r.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
  cat $OUT/c4_$r.json
done
