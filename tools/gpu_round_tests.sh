# All -m gpu tests, then the 2-rank (gloo, one GPU) rehearsal of bench.py's N > 1 path at a
# ragged n (edge kernel + helper stream in both ranks).
set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/rt; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 3 --warmup 1 --individuals 3000 --loci 20000 --dist-backend gloo --same-device > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; cat $OUT/bench2.json; [ $rc -eq 0 ] || tail -5 $OUT/bench2.err; exit $rc
