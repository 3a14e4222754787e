# BRR: GPU tests, C4-shape timing (n = 10 000, p = 100 000; sweep and per-launch paths) and
# rocprofv3 kernel stats
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/brrnew; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_brr.py tests/test_gpu_large.py -m gpu -k "brr or c4 or C4" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 250 > $OUT/c4.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
cat $OUT/c4.json
GBM_BRR_SWEEP=0 timeout -k 10 300 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 250 > $OUT/c4_launch.json 2> $OUT/c4l.err || { tail $OUT/c4l.err; exit 1; }
cat $OUT/c4_launch.json
bash tools/profile_brr.sh
