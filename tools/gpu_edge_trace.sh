set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/edgetr; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/edgetr/t/**/run_kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
for r in rows:
    k=r['Kernel_Name']
    if 'syrk_kernel<2>' in k or 'edge' in k or 'slab_reduce' in k or 'standardize' in k:
        print(k[:40].ljust(40), r['Queue_Id'], int(r['Start_Timestamp'])/1e3, int(r['End_Timestamp'])/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
