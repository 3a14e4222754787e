# Build GRM-kernel variants (stage depth BK, waves per SIMD) on the box and bench each.
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/var; mkdir -p $OUT
C=genomicbreedingmodels.jl_amd/csrc
VARIANTS=${VARIANTS:-"16:2: 8:2:"}
for V in $VARIANTS; do
  IFS=: read -r BKV WPSV XDEF <<< "$V"
  set -- $BKV $WPSV
  D=$OUT/bk$1_w$2$XDEF; mkdir -p $D
  for f in stats grm chol effects gibbs; do hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DGBM_BK=$1 -DGBM_WPS=$2 ${XDEF:+-D${XDEF//+/ -D}} -c $C/$f.hip -o $D/$f.o || exit 1; done
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/capi.cpp -o $D/capi.o && hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/session.cpp -o $D/session.o || exit 1
  hipcc --offload-arch=gfx950 -shared -fPIC $D/*.o -lrccl -o $D/libgbm.so || exit 1
  if [ "$XDEF" = GBM_DEBUG_WGTIME ]; then GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 200 python tools/wgtime.py; continue; fi
  if [ "$XDEF" = GBM_DEBUG_FACTIME ]; then GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 200 python tools/factime.py; continue; fi
  case "$XDEF" in GBM_DEBUG_*|TIME*) echo -n "BK $1 WPS $2 $XDEF: "; GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 200 python tools/time_grm.py || exit 1; continue;; esac
  GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/b.json 2> $D/b.err || { tail -3 $D/b.err; continue; }
  python3 -c "import json; d=json.load(open('$D/b.json')); print('BK $1 WPS $2 $XDEF', 'ms %.2f syrk %.2f solve %.2f frac %.3f'%(d['ms_per_step'], d['stage_ms']['grm_syrk'], d['stage_ms']['solve'], d['roofline']['frac']))"
done
