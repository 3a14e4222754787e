# BRR sweep timing-only variants (operand streams removed; results are not meaningful)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brrvar2; mkdir -p $OUT
for v in ${VARIANTS:-noM noXV noRows}; do
  GBM_LIBGBM=$PWD/build/var/$v/libgbm.so timeout -k 10 120 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 100 > $OUT/$v.json 2> $OUT/$v.err || { tail -3 $OUT/$v.err; exit 1; }
  echo $v $(python3 -c "import json;print(round(json.load(open('$OUT/$v.json'))['ms_per_iter'],3))")
done
timeout -k 10 120 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 100 > $OUT/base.json 2> $OUT/base.err && echo base $(python3 -c "import json;print(round(json.load(open('$OUT/base.json'))['ms_per_iter'],3))")
