# round-5 check: solve tests and solve time after the k-loop restructuring (default build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05o
mkdir -p $O
timeout -k 5 120 python -c "import torch; torch.zeros(1, device='cuda'); print('warm')" &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chol_flow.py tests/test_gpu_parity.py tests/test_gpu_dist_solve.py tests/test_lmer_known_answers.py > $O/chol_tests.log 2>&1 &&
REPS=30 timeout -k 10 60 python -u tools/time_solve.py > $O/solve.txt 2>&1 &&
REPS=30 timeout -k 10 60 python -u tools/time_solve.py >> $O/solve.txt 2>&1
