#!/bin/bash
# A/B: the one-row-per-wave standardisation (variants/libgbm_stdwave.so, -DGBM_STD_WAVE=1) against
# the in-tree library on the C2 bench (stage timings), after the streamed/parity tests on the variant.
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/stdwave; mkdir -p $OUT
export GBM_LIBGBM=$PWD/variants/libgbm_stdwave.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_streamed.py tests/test_gpu_fixtures.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2 3; do
  for v in base wave; do
    if [ $v = wave ]; then export GBM_LIBGBM=$PWD/variants/libgbm_stdwave.so; else unset GBM_LIBGBM; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail $OUT/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); s=d['stage_ms']; print('$v', '%.3f'%d['ms_per_step'], ' '.join('%s=%.3f'%(k,v) for k,v in s.items()))"
  done
done
