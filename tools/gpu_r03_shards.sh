# Round 3: concurrent multi-shard C-ABI fit — farming tests, serial vs threaded timing, and the
# rocprofv3 kernel + memory-copy traces of both schedules (tools/overlap_from_trace.py).
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/shards; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_farming.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 200 python3 tools/two_shard_overlap.py > $OUT/timing.json 2> $OUT/timing.err || { tail $OUT/timing.err; exit 1; }
cat $OUT/timing.json
for m in 1 0; do
  MODES=$m REPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/t$m -o run -- python3 tools/two_shard_overlap.py > $OUT/tr$m.json 2> $OUT/tr$m.err || { tail $OUT/tr$m.err; exit 1; }
  python3 tools/overlap_from_trace.py $OUT/t$m "GBM_SHARD_THREADS=$m" | tee $OUT/overlap$m.json
done
