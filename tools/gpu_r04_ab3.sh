#!/bin/bash
# Dataflow Cholesky A/B: in-tree (candidate) vs variants/libgbm_prebal.so
# (assistant, 1-step batches) vs variants/libgbm_flowhead.so (round-3 kernel); chol_flow tests on the
# in-tree and kb1 builds, C2 bench stage times, then the in-tree timeline.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab3; mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chol_flow.py"
timeout -k 10 300 $T > $OUT/t_tree.log 2>&1 || { tail -20 $OUT/t_tree.log; exit 1; }
GBM_LIBGBM=$PWD/variants/libgbm_prebal.so timeout -k 10 300 $T > $OUT/t_prebal.log 2>&1 || { tail -20 $OUT/t_prebal.log; exit 1; }
tail -n 1 $OUT/t_tree.log; tail -n 1 $OUT/t_prebal.log
for r in 1 2; do
  for v in tree prebal flowhead; do
    if [ $v = tree ]; then unset GBM_LIBGBM; else export GBM_LIBGBM=$PWD/variants/libgbm_$v.so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail $OUT/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); s=d['stage_ms']; print('$v', '%.3f'%d['ms_per_step'], ' '.join('%s=%.3f'%(k,v) for k,v in s.items()))"
  done
done
unset GBM_LIBGBM
timeout -k 10 200 python3 tools/flow_timeline.py > $OUT/flow.txt 2> $OUT/flow.err || { tail $OUT/flow.err; exit 1; }
cat $OUT/flow.txt
