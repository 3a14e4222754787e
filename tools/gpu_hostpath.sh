# pipelined host upload: its tests, then the bench's host-path timings (C2, pageable / pinned / int8)
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/hp; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_farming.py tests/test_gpu_fixtures.py tests/test_gpu_chol_flow.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/tests.log | head -20; exit $rc; }
for C in 0 -1 6250 12500; do
  echo "GBM_HOST_CHUNK=$C"
  timeout -k 10 300 env GBM_HOST_CHUNK=$C python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { tail $OUT/bench_$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$C.json')); print(d['ms_per_step'], d['stage_ms']['solve'], {k: round(v,2) for k,v in d['host_path'].items() if 'ms' in k})"
done
