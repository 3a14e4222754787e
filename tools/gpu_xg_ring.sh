# exact GEMM tile / ring variants: 64x64 (default), 128x64 with a 4- or 5-stage ring, BK = 256 (timing)
set -e
mkdir -p gpurun_out/xgr
for r in 1 2; do
  for v in d64 b128n4 b128n5 bk256; do
    L=variants/libgbm_xg_ns4.so; BM=64; BKK=128
    case $v in b128n4) BM=128;; b128n5) BM=128; L=variants/libgbm_xg_ns5.so;; bk256) BKK=256;; esac
    echo -n "$v " >> gpurun_out/xgr/t.txt
    GBM_LIBGBM=$L GBM_XG_BM=$BM GBM_XG_BK=$BKK timeout -k 10 200 python3 -u tools/time_grm_exact.py >> gpurun_out/xgr/t.txt 2>/dev/null
  done
done
GBM_LIBGBM=variants/libgbm_xg_ns5.so GBM_XG_BM=128 timeout -k 10 200 python3 -u tools/exact_digest.py >> gpurun_out/xgr/t.txt 2>&1
GBM_LIBGBM=variants/libgbm_xg_ns4.so timeout -k 10 200 python3 -u tools/exact_digest.py >> gpurun_out/xgr/t.txt 2>&1
