# Dataflow factorisation: parity tests, then solve timings (dataflow vs launch-per-panel)
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/flow; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_chol_flow.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for N in 1000 3000 5000 10000 16000; do
  timeout -k 10 120 env N=$N P=2000 GBM_CHOL_FLOW_MAX=100000 python tools/time_solve.py 2>&1 | tail -1 || exit 1
  timeout -k 10 120 env N=$N P=2000 GBM_CHOL_FLOW_MAX=0 python tools/time_solve.py 2>&1 | tail -1 || exit 1
done
