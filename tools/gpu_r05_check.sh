# round-5 check: chain timeline with wave 1's hand-over stamps; solve time (untraced) unchanged
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05r
mkdir -p $O
timeout -k 5 120 python -c "import torch; torch.zeros(1, device='cuda'); print('warm')" &&
REPS=30 timeout -k 10 60 python -u tools/time_solve.py > $O/solve.txt 2>&1 &&
FLOW_DUMP=$O/flow.npy timeout -k 5 60 python -u tools/flow_timeline.py > $O/flow.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chol_flow.py > $O/chol_tests.log 2>&1
