#!/bin/bash
# §8(f) next-row timings on one GPU after the round-4 changes (tools/bench_next.py).
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
O=gpurun_out/r04_next_rows.jsonl; : > $O
B="python -u tools/bench_next.py"
timeout -k 10 240 $B brr-c4 --n 10000 --p 100000 --iters 50 >> $O 2> gpurun_out/r04_next_brr.err &&
timeout -k 10 120 $B reml >> $O 2> gpurun_out/r04_next_reml.err &&
timeout -k 10 120 $B ridge --n 200 --p 1000 --traits 1 >> $O 2> gpurun_out/r04_next_ridge.err &&
timeout -k 10 180 $B cv >> $O 2> gpurun_out/r04_next_cv.err &&
timeout -k 10 300 $B cv-synth --n 20000 --p 300000 --traits 3 --folds 10 >> $O 2> gpurun_out/r04_next_cvsynth.err
