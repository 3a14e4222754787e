# dataflow Cholesky: its GPU tests, the chain timeline at C2's n, and the C2 bench solve stage.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/chol; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_chol_flow.py -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 tools/flow_timeline.py > $OUT/flow.txt 2> $OUT/flow.err || { tail $OUT/flow.err; exit 1; }
cat $OUT/flow.txt
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cpu-c3 --no-host-path > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['ms_per_step'], d['stage_ms'])"
