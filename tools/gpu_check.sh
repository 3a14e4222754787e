# All -m gpu tests, then one default bench line (no CPU baseline). Usage: bash tools/gpu_check.sh [pytest -k expr]
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/check; mkdir -p $OUT
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread $K > $OUT/tests.log 2>&1; rc=$?
tail -4 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
