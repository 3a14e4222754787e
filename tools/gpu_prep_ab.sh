#!/bin/bash
# A/B of the exact GRM's prep kernels (transpose + U grid): the exact tests, then a rocprofv3 kernel summary
# of tools/exact_grm_time.py per GBM_XG_TNR value. Stops at the first failing GPU step.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prep
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prep/tests.log 2>&1 || { tail -30 gpurun_out/prep/tests.log; exit 1; }
tail -1 gpurun_out/prep/tests.log
for t in ${TNRS:-64 128 32}; do
  if [ "$t" = auto ]; then unset GBM_XG_TNR; else export GBM_XG_TNR=$t; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prep/p$t -o run -- python3 tools/exact_grm_time.py 5000 50000 exact > gpurun_out/prep/p$t.log 2>&1 || exit 1
  python3 tools/prof_db_summary.py gpurun_out/prep/p$t/run_results.db --skip-first > gpurun_out/prep/p$t.txt || exit 1
  echo "TNR $t"; grep -E 'xg_' gpurun_out/prep/p$t.txt | cut -c1-40,75-96
  tail -1 gpurun_out/prep/p$t.log | cut -c1-200
done
