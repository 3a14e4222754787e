# round-5 check: kernel trace of the distributed solve at n = 50 000, R = 8 (rank 0's share, one GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05v
mkdir -p $O
timeout -k 5 120 python -c "import torch; torch.zeros(1, device='cuda'); print('warm')" &&
SKIP_REDUNDANT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u tools/dist_solve_time.py 50000 8 > $O/dist.json 2> $O/dist.err
