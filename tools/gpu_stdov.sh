# overlapped standardisation: parity tests, then bench with and without the overlap
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/so; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/tests.log | head -20; exit $rc; }
for O in 1 0 1 0; do
  timeout -k 10 300 env GBM_STD_OVERLAP=$O python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/bench_$O.json 2> $OUT/bench_$O.err || { tail $OUT/bench_$O.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$O.json')); print('overlap $O', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['stage_ms'].items()})"
done
