#!/bin/bash
# Beyond-L2 read bytes (FETCH_SIZE x2, gfx950 correction) of the GRM SYRK per split / size.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/fetch; mkdir -p $OUT
CASES=${CASES:-"auto:5000:50000 1:5000:50000 1:3968:50000"}
for CASE in $CASES; do
  IFS=: read -r S N P <<< "$CASE"
  if [ "$S" = auto ]; then unset GBM_GRM_SPLIT; else export GBM_GRM_SPLIT=$S; fi
  D=$OUT/${S//,/_}_$N; rm -rf $D
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D -o run -- python3 tools/time_grm.py $N $P > $D.log 2> $D.err || { tail -3 $D.err; exit 1; }
  python3 - $D "$CASE" <<'PY'
import csv, glob, sys
vals = []
for f in glob.glob(sys.argv[1] + '/**/*counter_collection*.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if r.get('Counter_Name') == 'FETCH_SIZE' and 'syrk_kernel<1>' in r.get('Kernel_Name', ''):
            vals.append(float(r['Counter_Value']))
print(sys.argv[2], 'launches', len(vals), 'beyond-L2 read GB per launch %.1f' % (2 * sum(vals) / len(vals) * 1024 / 1e9), open(sys.argv[1] + '.log').read().strip())
PY
done
