# Full round check on one GPU: all -m gpu tests, smoke(), default bench (with CPU baseline),
# rocprofv3 kernel stats of the same bench command.
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/full; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -4 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/full/trace/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r['Name'][:50].ljust(50), r['Calls'].rjust(5), ('%.1f'%(float(r['AverageNs'])/1000)).rjust(9),'us', r['Percentage'][:5])
PY
