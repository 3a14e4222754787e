set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chol_flow.py tests/test_gpu_parity.py > gpurun_out/r05/chol_tests.log 2>&1 || exit 1
for k in 1 2 3; do
  GBM_CHOL_FLOW_ORDER=4 REPS=20 timeout -k 10 60 python -u tools/time_solve.py >> gpurun_out/r05/chol_ab.txt 2>&1 || exit 1
  REPS=20 timeout -k 10 60 python -u tools/time_solve.py >> gpurun_out/r05/chol_ab.txt 2>&1 || exit 1
done
FLOW_DUMP=gpurun_out/r05/flow_dump_new.npy timeout -k 10 120 python -u tools/flow_timeline.py > gpurun_out/r05/flow_timeline_new.txt 2>&1
