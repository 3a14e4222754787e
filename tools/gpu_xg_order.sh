# exact GEMM unit order sweep (GBM_XG_ORDER = AxB blocks of row x column blocks; 0 = row-major)
set -e
mkdir -p gpurun_out/xgo
for r in 1 2; do
  for o in 0 8x8 4x8 4x16 16x4 2x32 8x16; do
    echo -n "$o " >> gpurun_out/xgo/t.txt
    GBM_XG_ORDER=$o timeout -k 10 200 python3 -u tools/time_grm_exact.py >> gpurun_out/xgo/t.txt 2>/dev/null
  done
done
