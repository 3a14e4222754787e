# Round 3 (re-entry): pipelined-leaf chain factor + leaf-by-leaf worker solves. The dataflow Cholesky's
# tests, its timeline at C2's n, then the whole -m gpu suite, smoke and the default bench line.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/chain2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_chol_flow.py -m gpu > $OUT/chol_tests.log 2>&1 || { tail -30 $OUT/chol_tests.log; exit 1; }
tail -2 $OUT/chol_tests.log
timeout -k 10 200 python3 tools/flow_timeline.py > $OUT/flow.txt 2> $OUT/flow.err || { tail $OUT/flow.err; exit 1; }
cat $OUT/flow.txt
[ -n "$CHOL_ONLY" ] && exit 0
TAG=chain2 bash tools/gpu_r03_full.sh
