#!/bin/bash
# A/B of libgbm builds on one box: parity tests on the candidate (the in-tree library), then the C2
# bench alternating the candidate and variants/libgbm_base.so. TESTS overrides the test selection.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab; mkdir -p $OUT
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_chol_flow.py tests/test_gpu_dist_solve.py tests/test_gpu_fixtures.py"}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2 3; do
  for v in cand base; do
    if [ $v = base ]; then export GBM_LIBGBM=$PWD/variants/libgbm_base.so; else unset GBM_LIBGBM; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path ${BENCH_ARGS} > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail $OUT/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); s=d['stage_ms']; print('$v', '%.3f'%d['ms_per_step'], ' '.join('%s=%.3f'%(k,v) for k,v in s.items()))"
  done
done
