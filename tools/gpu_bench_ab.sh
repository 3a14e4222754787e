# bench A/B on one box: the default C2 bench with a variant library (argument 1) and with the
# in-tree one, alternating twice; prints ms/step and the stage times that differ
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/benchab; mkdir -p $OUT
for r in 1 2; do
  for lib in "$1" ""; do
    GBM_LIBGBM=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); s=d['stage_ms']; print('${lib:-in-tree}'.ljust(32), 'ms %.3f syrk %.3f solve %.3f std %.3f eff %.3f'%(d['ms_per_step'],s['grm_syrk'],s['solve'],s['standardize'],s['effects']))"
  done
done
