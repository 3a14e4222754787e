# 2 ranks on the single GPU of the box over gloo: exercises bench.py's N>1 path (loci sharding,
# all-reduce wiring, max-over-ranks timing) with the real HIP kernels.
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dist; mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 3 --warmup 1 --individuals 2000 --loci 20000 --dist-backend gloo --same-device > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; cat $OUT/bench2.json; tail -5 $OUT/bench2.err; exit $rc
