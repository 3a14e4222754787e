# rocprofv3 kernel stats of the solve alone at large n (tools/time_solve.py)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/solveprof; mkdir -p $OUT
N=${N:-50000}
N=$N P=2000 REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o run -- python3 tools/time_solve.py > $OUT/out.txt 2> $OUT/err.txt || { tail $OUT/err.txt; exit 1; }
cat $OUT/out.txt
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/solveprof/t/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r['Name'][:50].ljust(50), r['Calls'].rjust(6), ('%.1f'%(float(r['AverageNs'])/1000)).rjust(9),'us', ('%.1f'%(float(r['TotalDurationNs'])/1e6)).rjust(8), 'ms', r['Percentage'][:5])
PY
