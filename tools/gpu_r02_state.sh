# Round state: every -m gpu test, the 2-rank path, smoke, the default bench line, rocprofv3 kernel
# stats (gpu_iter), the FETCH/WRITE PMC passes (profile_pmc)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round_final.sh && bash tools/gpu_iter.sh && bash tools/profile_pmc.sh
