# parity tests -> bench -> rocprofv3 kernel stats (one GPU call per iteration)
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/iter; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value %.3e ms %.2f syrk %.2f frac %.3f'%(d['value'],d['ms_per_step'],d['roofline']['ms_per_launch'],d['roofline']['frac'])); print(d['stage_ms'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/iter/trace/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r['Name'][:50].ljust(50), r['Calls'].rjust(5), ('%.1f'%(float(r['AverageNs'])/1000)).rjust(9),'us', r['Percentage'][:5])
PY
