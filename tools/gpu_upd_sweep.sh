set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/sweep; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for L in 0 2048 3968 6000; do
  GBM_UPD64_LIM=$L timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/b_$L.json 2>$OUT/b_$L.err || { tail $OUT/b_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$L.json')); print('lim $L', 'ms %.2f'%d['ms_per_step'], 'solve %.2f'%d['stage_ms']['solve'])"
done
