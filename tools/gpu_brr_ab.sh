# BRR A/B on one box: C4-shape timing with a variant library (argument 1, e.g. variants/libgbm_x.so)
# and with the in-tree one, alternating
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brrab; mkdir -p $OUT
for r in 1 2; do
  for lib in "$1" ""; do
    GBM_LIBGBM=$lib timeout -k 10 300 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 250 > $OUT/c4.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4.json')); print('${lib:-in-tree}', '%.3f ms/iter'%d['ms_per_iter'])"
  done
done
