# The large-config GPU tests (C3 per-GPU shape, a full-size C5 fold, C4 5000 iterations) with
# their printed timings. Usage: bash tools/gpu_large.sh [pytest -k expr]
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/large; mkdir -p $OUT
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -v -s -m gpu --timeout 400 --timeout-method thread $K > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|C3|C4|C5|gbm_gblup|passed|failed" $OUT/tests.log | tail -20
[ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/tests.log | head -30; exit $rc; }
