# C-ABI host-path A/B on one box: the bench's host_path timings with a variant library
# (argument 1) and with the in-tree one, alternating twice
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/hostab; mkdir -p $OUT
for r in 1 2; do
  for lib in "$1" ""; do
    GBM_LIBGBM=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python3 -c "import json; h=json.load(open('$OUT/b.json'))['host_path']; print('${lib:-in-tree}'.ljust(40), 'pageable %.2f pinned %.2f i8 %.2f h2d %.2f'%(h['ms_per_call_pageable_x'],h['ms_per_call_pinned_x'],h['ms_per_call_dosage_i8'],h['h2d_x_ms_pinned']))"
  done
done
