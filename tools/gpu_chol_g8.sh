# 8-panel Cholesky groups: GPU tests with the groups forced on small matrices, then the solve at
# C3 shape (n = 50 000), n = 20 000 and C2 for several GBM_CHOL_G8_LIM thresholds.
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/cholg8; mkdir -p $out
timeout -k 10 300 env GBM_CHOL_G8_LIM=0 GBM_CHOL_G4_LIM=0 GBM_UPD64_LIM=128 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > $out/tests_forced.log 2>&1 || { echo "forced-group tests failed"; tail -30 $out/tests_forced.log; exit 1; }
tail -1 $out/tests_forced.log
for n in 50000 20000; do
  for lim in -1 16384 8192 4096; do
    echo -n "n=$n g8lim=$lim: "; N=$n P=2000 REPS=2 GBM_CHOL_G8_LIM=$lim timeout -k 10 200 python tools/time_solve.py || exit 1
  done
done
for lim in -1 2048; do
  echo -n "n=5000 g8lim=$lim: "; N=5000 P=4000 REPS=5 GBM_CHOL_G8_LIM=$lim timeout -k 10 200 python tools/time_solve.py || exit 1
done
