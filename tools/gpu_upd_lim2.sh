#!/bin/bash
# Sweep GBM_UPD64_LIM2 (64x64-tile K=128 pair updates below this many trailing rows) at n = 5000.
set -o pipefail
for L in -1 2560 3072 3584 4096 6000; do
  GBM_UPD64_LIM2=$L REPS=8 timeout -k 10 120 python tools/time_solve.py 2>/dev/null | sed "s/^/lim2=$L /" || exit 1
done
