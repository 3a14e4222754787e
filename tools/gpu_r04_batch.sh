#!/bin/bash
# One box: the distributed-factorisation tests and per-rank timing, the standardisation A/B, the
# current dataflow-Cholesky timeline at C2's n, then the §8(f) next-row timings.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_r04_dist.sh || { tail -30 gpurun_out/r04_dist_tests.log; exit 1; }
tail -3 gpurun_out/r04_dist_tests.log; cat gpurun_out/r04_dist_solve_time.json
timeout -k 10 200 python3 tools/flow_timeline.py > gpurun_out/r04_flow_timeline.txt 2> gpurun_out/r04_flow_timeline.err || { tail gpurun_out/r04_flow_timeline.err; exit 1; }
head -3 gpurun_out/r04_flow_timeline.txt
bash tools/gpu_r04_stdwave.sh || exit 1
bash tools/gpu_r04_next.sh || { tail gpurun_out/r04_next_*.err; exit 1; }
cat gpurun_out/r04_next_rows.jsonl
