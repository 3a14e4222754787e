# GRM fused slab reduce: GPU tests, then an A/B of the C2 bench line (GBM_GRM_FUSED=0/1, alternating)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grm_fused.py > gpurun_out/fused_tests.log 2>&1
for v in 0 1 0 1; do
  GBM_GRM_FUSED=$v timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cpu-c3 --no-host-path --no-exact > gpurun_out/fused_bench_$v.tmp 2> gpurun_out/fused_bench_err.log
  tail -1 gpurun_out/fused_bench_$v.tmp | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'fused': '$v', 'ms_per_step': d['ms_per_step'], 'stage_ms': d['stage_ms'], 'frac': d['roofline']['frac'], 'parity': d.get('parity', {}).get('pass')}))" >> gpurun_out/fused_ab.jsonl
done
