# round-5 check: SYRK operand staging by LDS DMA (base) vs through registers (timing variants), twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05t
mkdir -p $O
timeout -k 5 120 python -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
for rep in 1 2; do
  for v in g_base g_reg g_noload; do
    echo "variant=$v" >> $O/syrk.txt
    GBM_LIBGBM=$PWD/variants/libgbm_$v.so timeout -k 10 90 python -u tools/time_grm.py >> $O/syrk.txt 2>&1 || exit 1
  done
done
