#!/bin/bash
# A/B on one box: (1) the double-buffered row update (in-tree) vs single-buffered (variants/libgbm_rowsb.so)
# on the redundant and R = 8 distributed solves at n = 50 000; (2) the wave standardisation
# (variants/libgbm_stdwave.so) vs in-tree on the C2 bench; then the dataflow timeline.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab2; mkdir -p $OUT
for r in 1 2; do
  for v in cand rowsb; do
    if [ $v = rowsb ]; then export GBM_LIBGBM=$PWD/variants/libgbm_rowsb.so; else unset GBM_LIBGBM; fi
    timeout -k 10 300 python3 tools/dist_solve_time.py 50000 8 > $OUT/d_${v}_$r.json 2> $OUT/d_${v}_$r.err || { tail $OUT/d_${v}_$r.err; exit 1; }
    echo "$v $(cat $OUT/d_${v}_$r.json)"
  done
done
unset GBM_LIBGBM
GBM_LIBGBM=$PWD/variants/libgbm_stdwave.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_streamed.py > $OUT/t_wave.log 2>&1 || { tail -20 $OUT/t_wave.log; exit 1; }
for r in 1 2 3; do
  for v in base wave; do
    if [ $v = wave ]; then export GBM_LIBGBM=$PWD/variants/libgbm_stdwave.so; else unset GBM_LIBGBM; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail $OUT/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); s=d['stage_ms']; print('$v', '%.3f'%d['ms_per_step'], ' '.join('%s=%.3f'%(k,v) for k,v in s.items()))"
  done
done
unset GBM_LIBGBM
timeout -k 10 200 python3 tools/flow_timeline.py > $OUT/flow.txt 2> $OUT/flow.err || { tail $OUT/flow.err; exit 1; }
tail -8 $OUT/flow.txt
