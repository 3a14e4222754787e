# dataflow vs launch-per-panel solve times over n (choosing GBM_CHOL_FLOW_MAX)
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
for N in 5000 10000 16000 20000 26000; do
  timeout -k 10 120 env N=$N P=1000 REPS=3 GBM_CHOL_FLOW_MAX=100000 python tools/time_solve.py 2>&1 | tail -1 || exit 1
  timeout -k 10 120 env N=$N P=1000 REPS=3 GBM_CHOL_FLOW_MAX=0 python tools/time_solve.py 2>&1 | tail -1 || exit 1
done
