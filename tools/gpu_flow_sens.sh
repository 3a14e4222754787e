# dataflow Cholesky sensitivity: solve time at C2 with the chain's identity columns removed (noy), the workers'
# operand loads removed (noload) or their MFMAs removed (nomfma), beside the unmodified kernel (timing only)
set -e
mkdir -p gpurun_out
for v in base noy noload nomfma base noy; do
  NS=5000 REPS=20 GBM_LIBGBM=variants/libgbm_$v.so timeout -k 10 120 python3 -u tools/flow_ab.py >> gpurun_out/flow_sens.jsonl 2>/dev/null
done
