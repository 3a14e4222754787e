# Dataflow Cholesky timing variants (tools/build_flow_variants.sh): the flow tests on the knob
# variants, then the C2 chain timeline of each.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/fv; mkdir -p $OUT
for v in v1 v2; do
  GBM_LIBGBM=$PWD/variants/libgbm_$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chol_flow.py -m gpu > $OUT/tests_$v.log 2>&1 || { tail -20 $OUT/tests_$v.log; exit 1; }
  tail -1 $OUT/tests_$v.log
done
for v in v0 v1 v2 v3 v0 v1; do
  GBM_LIBGBM=$PWD/variants/libgbm_$v.so timeout -k 10 200 python3 tools/flow_timeline.py > $OUT/flow_$v.txt 2> $OUT/flow_$v.err || { tail $OUT/flow_$v.err; exit 1; }
  echo "$v $(head -1 $OUT/flow_$v.txt) | $(grep 'own 16' $OUT/flow_$v.txt | awk '{print $7}' | tr '\n' ' ')"
done
