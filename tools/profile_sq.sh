# SQ + GRBM counters for the GRM SYRK and dataflow Cholesky kernels (one PMC pass, no other trace domains)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/sq; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/sq/p1/**/*counter_collection*.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[r['Kernel_Name'][:120]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    if 'syrk' in k or 'panel' in k or 'chol_flow' in k:
        print(k, {c: '%.4g' % (sum(v) / len(v)) for c, v in d.items()})
PY
