# PMC passes over the BRR C4 iteration kernels (SQ wait/MFMA counters, then FETCH_SIZE) and the
# dataflow Cholesky timeline at C2's n. Timing tool only.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcprep; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/sq -o run -- python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 10 > $OUT/sq.json 2> $OUT/sq.err || { tail $OUT/sq.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 10 > $OUT/fetch.json 2> $OUT/fetch.err || { tail $OUT/fetch.err; exit 1; }
timeout -k 10 200 python3 tools/flow_timeline.py > $OUT/flow.txt 2> $OUT/flow.err || { tail $OUT/flow.err; exit 1; }
cat $OUT/flow.txt
