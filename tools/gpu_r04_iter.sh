#!/bin/bash
# Iteration check: Cholesky / distributed tests, the dataflow timeline (with the assistant's
# timestamps), the per-rank distributed solve at n = 50 000, two C2 bench lines.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/iter; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_chol_flow.py tests/test_gpu_dist_solve.py tests/test_gpu_parity.py tests/test_gpu_sharded.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 tools/flow_timeline.py > $OUT/flow.txt 2> $OUT/flow.err || { tail $OUT/flow.err; exit 1; }
cat $OUT/flow.txt
timeout -k 10 300 python3 tools/dist_solve_time.py 50000 8 > $OUT/dist.json 2> $OUT/dist.err || { tail $OUT/dist.err; exit 1; }
cat $OUT/dist.json
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/b$r.json 2> $OUT/b$r.err || { tail $OUT/b$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b$r.json')); s=d['stage_ms']; print('%.3f'%d['ms_per_step'], ' '.join('%s=%.3f'%(k,v) for k,v in s.items()))"
done
