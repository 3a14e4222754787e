# Round-2 final state: every -m gpu test, the 2-rank path, smoke, the default bench line
# (gpu_round_final), the large-config timings (-s), rocprofv3 kernel stats (gpu_iter), the
# FETCH/WRITE PMC passes (profile_pmc) and the SQ counters (profile_sq)
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round_final.sh || exit $?
mkdir -p gpurun_out/large
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q -s -m gpu --timeout 240 --timeout-method thread > gpurun_out/large/large.log 2>&1 || { tail -20 gpurun_out/large/large.log; exit 1; }
grep -E "C3|C4|C5|passed" gpurun_out/large/large.log
bash tools/gpu_iter.sh && bash tools/profile_pmc.sh && bash tools/profile_sq.sh
