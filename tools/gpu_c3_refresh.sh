# C3 on one GPU with the current code: loci-streamed fp64 and the exact GRM (one timed step each, no CPU legs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c3
mkdir -p $O
timeout -k 5 120 python -c "import torch; torch.zeros(1, device='cuda'); print('warm')" &&
timeout -k 10 500 python -u bench.py --individuals 50000 --loci 600000 --stream-chunk 75000 --steps 1 --warmup 1 --no-cpu-baseline --no-host-path --no-exact > $O/c3_fp64.json 2> $O/c3_fp64.err &&
timeout -k 10 300 python -u bench.py --individuals 50000 --loci 600000 --grm exact --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > $O/c3_exact.json 2> $O/c3_exact.err
