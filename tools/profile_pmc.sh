# Separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the bench, as MI355X_MICROARCH.md §HBM prescribes.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > $OUT/bench_$C.json 2> $OUT/bench_$C.err || exit $?
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_grm.json && cat $OUT/pmc_grm.json
