#!/bin/bash
# A/B/n of libgbm timing variants on one box: the C2 bench alternating the in-tree library ("cand")
# and variants/libgbm_<v>.so for v in $VARIANTS (default "base"), $ROUNDS rounds. No tests.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/abn; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in cand ${VARIANTS:-base}; do
    if [ $v = cand ]; then unset GBM_LIBGBM; else export GBM_LIBGBM=$PWD/variants/libgbm_$v.so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path ${BENCH_ARGS} > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail $OUT/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); s=d['stage_ms']; print('%-8s'%'$v', '%.3f'%d['ms_per_step'], ' '.join('%s=%.3f'%(k,v) for k,v in s.items()))"
  done
done
