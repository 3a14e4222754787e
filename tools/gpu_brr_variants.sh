# Build BRR-kernel timing variants and print the step kernel's average duration for each
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brrvar; mkdir -p $OUT
C=genomicbreedingmodels.jl_amd/csrc
for XDEF in ${VARIANTS:-NONE}; do
  D=$OUT/$XDEF; mkdir -p $D
  for f in stats grm chol effects gibbs; do hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -D$XDEF -c $C/$f.hip -o $D/$f.o || exit 1; done
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/capi.cpp -o $D/capi.o && hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/session.cpp -o $D/session.o || exit 1
  hipcc --offload-arch=gfx950 -shared -fPIC $D/*.o -lrccl -o $D/libgbm.so || exit 1
  GBM_LIBGBM=$PWD/$D/libgbm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/t -o run -- python3 tools/bench_next.py brr --n 10000 --p 20000 --iters 20 > $D/b.json 2> $D/err.log || { tail -3 $D/err.log; exit 1; }
  python3 - "$D" "$XDEF" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/t/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'brr_step' in r['Name']:
        print(sys.argv[2], 'brr_step avg us', '%.2f' % (float(r['AverageNs']) / 1000))
PY
done
