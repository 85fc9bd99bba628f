# Hardware counters of the steady-state VGG-small training step (bench.py).
#  0. unprofiled-counter run with a kernel trace: autotune picks saved to a cache file, per-kernel
#     steady-state durations (trace_steps.py) -> durations.csv
#  1-3. rocprofv3 --pmc passes (SQ+GRBM, FETCH_SIZE, WRITE_SIZE + L2 hit/miss) replaying the same
#     picks from the cache, each under its own time limit
# then a per-kernel summary of the last 2 steps -> gpurun_out/pmc_step/summary.{txt,csv}; the raw
# per-dispatch CSVs are deleted (they exceed what gpurun copies back).
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_step
mkdir -p $OUT
export RAFIKI_TUNE_CACHE=$PWD/$OUT/tune.json
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- \
  python3 bench.py --steps 20 --warmup 5 --trials 0 --probe-trials 0 --no-serving --configs none > $OUT/t.log 2>&1
python3 scripts/trace_steps.py $(find $OUT/t -name '*kernel_trace.csv' | head -1) --steps 20 \
  --csv $OUT/durations.csv > $OUT/durations.txt
ARGS="bench.py --steps 2 --warmup 1 --trials 0 --probe-trials 0 --no-serving --configs none"
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p0 -o run -- python3 $ARGS > $OUT/p0.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p1 -o run -- python3 $ARGS > $OUT/p1.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p2 -o run -- python3 $ARGS > $OUT/p2.log 2>&1
# issue-side pass (instruction mix and stall shares); optional: the summary runs without it
P3=""
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
  SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p3 -o run -- python3 $ARGS > $OUT/p3.log 2>&1 && P3=$OUT/p3
python3 scripts/pmc_summary.py $OUT/p0 $OUT/p1 $OUT/p2 $P3 --steps 2 --durations $OUT/durations.csv \
  --csv $OUT/summary.csv > $OUT/summary.txt
rm -rf $OUT/t $OUT/p0 $OUT/p1 $OUT/p2 $OUT/p3
cat $OUT/durations.txt | head -3
cat $OUT/summary.txt
