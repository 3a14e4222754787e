# Time prebuilt libgbm variants (build/var/*/libgbm.so, tools/build_variant.sh) on one GPU:
# GRM-parity tests with each, then the GRM launch alone and a short bench.
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/variants; mkdir -p $OUT
for D in ${VARS:-build/var/*}; do
  V=$(basename $D)
  GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > $OUT/$V.tests.log 2>&1 || { echo "$V: PARITY FAIL"; tail -5 $OUT/$V.tests.log; exit 1; }
  echo -n "$V: "; GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 200 python tools/time_grm.py ${GRM_SHAPE:-} || exit 1
  GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/$V.bench.json 2> $OUT/$V.bench.err || { tail -3 $OUT/$V.bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$V.bench.json')); print('   bench ms %.2f syrk %.2f solve %.2f frac %.3f'%(d['ms_per_step'], d['stage_ms']['grm_syrk'], d['stage_ms']['solve'], d['roofline']['frac']))"
done
