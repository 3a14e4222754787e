# weighted sum (msum) with its loads batched (default, GBM_WSUM_BATCH=8) vs one load per term (variants/libgbm_wsum1.so,
# built with -DGBM_WSUM_BATCH=1: the round-5 loop): effects stage time and fit digests, fp64 and exact stages
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for v in default wsum1; do
    if [ $v = default ]; then L=genomicbreedingmodels.jl_amd/gbm/libgbm.so; else L=variants/libgbm_$v.so; fi
    GBM_LIBGBM=$L timeout -k 10 200 python3 -u tools/fit_digest.py >> gpurun_out/wsum_ab.txt 2>/dev/null
  done
done
