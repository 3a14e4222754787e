#!/bin/bash
# PMC passes over the exact-GRM step (tools/exact_grm_time.py, exact path only), one counter group per run:
# FETCH_SIZE, WRITE_SIZE (HBM bytes; MI355X_MICROARCH.md §HBM), TCC_HIT/TCC_MISS (L2), and SQ busy/wait cycles.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_exact; mkdir -p $OUT
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/$tag -o run -- \
    python3 tools/exact_grm_time.py ${N:-5000} ${P:-50000} exact > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_exact/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "xg_" not in k and "chol" not in k and "marker" not in k:
        continue
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
