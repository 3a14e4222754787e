set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for o in 0 4x8 8x8 4x16 2x16 16x16; do
    GBM_XG_ORDER=$o timeout -k 10 120 python3 tools/exact_grm_time.py 5000 50000 exact > gpurun_out/ord_$o.json 2>&1 || { tail gpurun_out/ord_$o.json; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ord_$o.json').read().strip().splitlines()[-1]); print('order $o', round(d['ms_per_step'],3), round(d['stage_ms']['grm_syrk'],3))"
  done
done
