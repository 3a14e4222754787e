# GRM loci-split candidates at C2 through the whole bench step (GBM_GRM_SPLIT overrides the
# planner; stage counts of 16 loci): ms/step, GRM stage, slab reduce
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/split; mkdir -p $OUT
SPLITS=${SPLITS:-"auto 1250,1125,450,180,90,30 1400,1050,420,170,85 1250,1250,400,150,75 1600,900,400,150,75 1100,1100,500,250,125,50 auto"}
for S in $SPLITS; do
  if [ "$S" = auto ]; then unset GBM_GRM_SPLIT; else export GBM_GRM_SPLIT=$S; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); s=d['stage_ms']; print('$S'.ljust(34), 'slices', d['config']['grm_slices'], 'ms %.3f syrk %.3f reduce %.3f'%(d['ms_per_step'],s['grm_syrk'],s['grm_reduce']))"
done
