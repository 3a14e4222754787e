set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/t1.log 2>&1; rc=$?
tail -5 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?
cat gpurun_out/bench1.json; tail -20 gpurun_out/bench1.err
exit $rc
