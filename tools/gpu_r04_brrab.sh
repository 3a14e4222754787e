#!/bin/bash
# BRR C4 A/B: in-tree gibbs.hip (round-4 pruned) vs variants/libgbm_brr3.so (round-3 gibbs.hip, same rest).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/brrab; mkdir -p $OUT
for r in 1 2; do
  for v in tree brr3; do
    if [ $v = tree ]; then unset GBM_LIBGBM; else export GBM_LIBGBM=$PWD/variants/libgbm_$v.so; fi
    timeout -k 10 200 python3 tools/bench_next.py brr-c4 --n 10000 --p 100000 --iters 300 > $OUT/$v$r.json 2> $OUT/$v$r.err || { tail $OUT/$v$r.err; exit 1; }
    echo "$v $(cat $OUT/$v$r.json)"
  done
done
