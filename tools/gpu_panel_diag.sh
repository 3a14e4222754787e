set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pdiag; mkdir -p $OUT
for D in 0 1 2 4 7; do
  GBM_PANEL_DIAG=$D timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/d$D -o run -- python3 tools/time_solve.py > $OUT/d$D.log 2>$OUT/d$D.err || { tail $OUT/d$D.err; exit 1; }
  cat $OUT/d$D.log
  python3 - $D <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/pdiag/d{sys.argv[1]}/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'panel' in r['Name'] or 'back_diag' in r['Name']:
        print('   ', r['Name'][:30], r['Calls'], '%.1f us'%(float(r['AverageNs'])/1000))
PY
done
