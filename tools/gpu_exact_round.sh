#!/bin/bash
# One GPU call for the exact-GRM work: its tests, the unit-order A/B, a rocprofv3 kernel summary, PMC passes
# and a default bench line (fp64 headline + the exact path beside it). Stops at the first failing GPU step.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_streamed.py tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread > gpurun_out/exact_tests.log 2>&1 || { tail -30 gpurun_out/exact_tests.log; exit 1; }
tail -2 gpurun_out/exact_tests.log
if [ -z "$SKIP_AB" ]; then
for r in 1 2; do
  for cfg in "0 128 1 64" "0 128 1 128"; do
    set -- $cfg
    GBM_XG_BM=${4:-128} GBM_XG_SPLIT=$3 GBM_XG_ORDER=$1 GBM_XG_BK=$2 timeout -k 10 120 python3 tools/exact_grm_time.py 5000 50000 exact > gpurun_out/ab_$1_$2_$3_${4:-128}.json 2>&1 || { tail gpurun_out/ab_$1_$2_$3_${4:-128}.json; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_$1_$2_$3_${4:-128}.json').read().strip().splitlines()[-1]); print('order $1 bk $2 split $3 bm ${4:-128}', round(d['ms_per_step'],3), round(d['stage_ms']['grm_syrk'],3))"
  done
done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_exact5 -o run -- python3 tools/exact_grm_time.py 5000 50000 exact > gpurun_out/prof_exact5.log 2>&1 || exit 1
python3 tools/prof_db_summary.py gpurun_out/prof_exact5/run_results.db --skip-first | head -10
[ -n "$SKIP_PMC" ] || bash tools/gpu_exact_pmc.sh || exit 1
timeout -k 10 500 python bench.py --no-cpu-c3 --no-host-path > gpurun_out/bench_both.json 2> gpurun_out/bench_both.err || { tail gpurun_out/bench_both.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_both.json')); e=d.get('exact_grm_path',{})
print('fp64', round(d['ms_per_step'],3), d['parity'].get('pass'), 'exact', round(e.get('ms_per_step',0),3), e.get('parity',{}).get('pass'), e.get('parity',{}).get('rel_err_y_pred'), e.get('roofline',{}).get('frac'))"
