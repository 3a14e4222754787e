set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round_final.sh && bash tools/gpu_iter.sh
