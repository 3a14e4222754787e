# round-5 check: SYRK operand-pipeline variants (tools/build_grm_variants.sh), two passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05k
mkdir -p $O
timeout -k 5 120 python -c "import torch; torch.zeros(1, device='cuda'); print('warm')" || exit 1
for rep in 1 2; do
  for v in g_base g_pf g_r8 g_r8pf g_r8n3 g_r4 g_noload; do
    echo "variant=$v" >> $O/syrk.txt
    GBM_LIBGBM=$PWD/variants/libgbm_$v.so timeout -k 10 90 python -u tools/time_grm.py >> $O/syrk.txt 2>&1 || exit 1
  done
done
