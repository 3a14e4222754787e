#!/bin/bash
# Cholesky panel-group sweep: GPU tests with the 4-panel groups forced on small matrices, then
# bench.py at C2 and at a C3-shaped n = 50 000 for several GBM_CHOL_G4_LIM thresholds.
set -o pipefail
out=gpurun_out/cholg
mkdir -p $out
timeout -k 10 600 env GBM_CHOL_G4_LIM=0 GBM_UPD64_LIM=128 python -m pytest tests -m gpu -x -q > $out/tests_forced.log 2>&1 || { echo "forced-group tests failed"; tail -30 $out/tests_forced.log; exit 1; }
tail -2 $out/tests_forced.log
for lim in -1 8192 4096 2048 1024; do
  timeout -k 10 300 env GBM_CHOL_G4_LIM=$lim python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/c2_$lim.json 2> $out/c2_$lim.err || exit 1
  python -c "import json;d=json.loads(open('$out/c2_$lim.json').read().strip().splitlines()[-1]);print('C2 lim=$lim', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})"
done
for lim in -1 8192 4096; do
  timeout -k 10 300 env GBM_CHOL_G4_LIM=$lim python bench.py --individuals 50000 --loci 75000 --steps 1 --warmup 1 --no-cpu-baseline > $out/c3_$lim.json 2> $out/c3_$lim.err || exit 1
  python -c "import json;d=json.loads(open('$out/c3_$lim.json').read().strip().splitlines()[-1]);print('C3 lim=$lim', round(d['ms_per_step'],1), {k:round(v,1) for k,v in d['stage_ms'].items()})"
done
