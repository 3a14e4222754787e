set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/edge; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_session.py -x -q -m gpu > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in 1 0 1 0; do
  GBM_GRM_EDGE_CONCURRENT=$c timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b$c.json 2> $OUT/b$c.err || { tail -3 $OUT/b$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$c.json')); print('conc=$c ms %.3f syrk %.3f reduce %.3f solve %.3f frac %.4f'%(d['ms_per_step'], d['stage_ms']['grm_syrk'], d['stage_ms']['grm_reduce'], d['stage_ms']['solve'], d['roofline']['frac']))"
done
