# Round profile set: parity tests, bench, rocprofv3 kernel stats, PMC HBM bytes, SQ counters.
# Results copied into profiles/ by the caller (names per round).
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sq && bash tools/gpu_iter.sh && bash tools/profile_pmc.sh > /dev/null && bash tools/profile_sq.sh > gpurun_out/sq/summary.txt && cat gpurun_out/sq/summary.txt
