# round-5 check: solve tests (dataflow orders), pipeline-depth variants with the branch-free ring, traced timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h
mkdir -p $O
timeout -k 5 120 python -c "import torch; torch.zeros(1, device='cuda'); print('warm')" &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chol_flow.py tests/test_gpu_parity.py tests/test_gpu_dist_solve.py tests/test_lmer_known_answers.py > $O/chol_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in s4 s8 s16; do
    echo "variant=$v" >> $O/stages.txt
    GBM_LIBGBM=$PWD/variants/libgbm_$v.so REPS=30 timeout -k 10 60 python -u tools/time_solve.py >> $O/stages.txt 2>&1 || exit 1
  done
done
FLOW_DUMP=$O/flow_5000.npy timeout -k 5 60 python -u tools/flow_timeline.py > $O/flow_5000.txt 2>&1
