# Round profile set on one MI355X (results under gpurun_out/round/, copied into profiles/ by the caller):
#  1. the default bench command under rocprofv3 --kernel-trace --stats, summarised with the warm-up launches
#     left out (tools/rocprof_stats.py);
#  2. PMC HBM bytes of the GRM (separate FETCH_SIZE / WRITE_SIZE passes, tools/profile_pmc.sh);
#  3. SQ + GRBM counters of the GRM / Cholesky kernels (tools/profile_sq.sh): MFMA busy fraction and, with the
#     kernel durations of pass 1, the average shader clock (GRBM_GUI_ACTIVE / 8 XCDs / duration).
# Every step under its own time limit, chained with &&.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/round
mkdir -p $OUT
STEPS=${STEPS:-5}
WARM=${WARM:-2}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps $STEPS --warmup $WARM > $OUT/bench.json 2> $OUT/bench.err &&
python3 tools/rocprof_stats.py $OUT/trace --warmup $WARM --steps $STEPS --step-start standardize_kernel --csv $OUT/kernel_stats_timed.csv > $OUT/kernel_stats_timed.txt &&
python3 tools/rocprof_stats.py $OUT/trace --warmup $WARM --steps $STEPS --step-start xg_stats_kernel --csv $OUT/kernel_stats_timed_exact.csv > $OUT/kernel_stats_timed_exact.txt &&
bash tools/profile_pmc.sh > $OUT/pmc.txt &&
bash tools/profile_sq.sh > $OUT/sq.txt &&
cat $OUT/kernel_stats_timed.txt | head -20 && cat $OUT/sq.txt
