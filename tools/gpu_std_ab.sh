# standardisation A/B: the default build (nontemporal row loads and Z stores) against plain / loads-only / stores-only
# variants (tools/build_std_variants.sh)
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for v in default plain ntld ntst; do
    if [ $v = default ]; then L=genomicbreedingmodels.jl_amd/gbm/libgbm.so; else L=variants/libgbm_std_$v.so; fi
    GBM_LIBGBM=$L timeout -k 10 120 python3 -u tools/time_standardize.py >> gpurun_out/std_ab.txt 2>/dev/null
  done
done
# the whole C2 step (the GRM reads Z right after): default vs plain build, alternating
for r in 1 2; do
  for v in default plain; do
    if [ $v = default ]; then L=genomicbreedingmodels.jl_amd/gbm/libgbm.so; else L=variants/libgbm_std_$v.so; fi
    GBM_LIBGBM=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cpu-c3 --no-host-path --no-exact \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],3), {k: round(v,4) for k, v in d['stage_ms'].items()})" >> gpurun_out/std_ab.txt
  done
done
