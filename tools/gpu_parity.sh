set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/t1.log 2>&1; rc=$?
cat gpurun_out/t1.log | tail -40
exit $rc
