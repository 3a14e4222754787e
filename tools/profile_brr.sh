# rocprofv3 kernel stats of the BRR Gibbs sampler (kernel trace only)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brrprof; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o run -- python3 tools/bench_next.py brr --n 10000 --p 100000 --iters 10 > $OUT/b.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/brrprof/t/**/run_kernel_stats.csv', recursive=True)[0]
print('src', f)
for r in list(csv.DictReader(open(f)))[:10]:
    print(r['Name'][:50].ljust(50), r['Calls'].rjust(7), ('%.2f' % (float(r['AverageNs']) / 1000)).rjust(9), 'us', r['Percentage'][:5])
t = glob.glob('gpurun_out/brrprof/t/**/run_kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(t)) if 'brr_' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
st = [int(r['Start_Timestamp']) for r in rows]; en = [int(r['End_Timestamp']) for r in rows]
gaps = [st[i + 1] - en[i] for i in range(len(rows) - 1)]
import statistics
print('kernels', len(rows), 'median gap ns', statistics.median(gaps), 'mean gap', sum(gaps) / len(gaps))
PY
