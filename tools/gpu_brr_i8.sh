# BRR byte-storage path: its GPU tests, then C4-shaped timing with byte and fp64 storage.
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brr8; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_brr.py -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 50 > $OUT/c4_i8.json 2> $OUT/c4_i8.err \
  && cat $OUT/c4_i8.json \
  && GBM_BRR_I8=0 timeout -k 10 300 python -u tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 50 > $OUT/c4_f64.json 2> $OUT/c4_f64.err \
  && cat $OUT/c4_f64.json
