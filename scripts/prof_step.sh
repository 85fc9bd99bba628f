#!/bin/bash
# Per-kernel steady-state time of the bench.py training step (fp32 default; pass extra bench args).
#   scripts/prof_step.sh <tag> [bench args...]   -> gpurun_out/prof_<tag>/durations.{txt,csv}
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- \
  python3 bench.py --steps 20 --warmup 5 --trials 0 --probe-trials 0 --no-serving --configs none "$@" > $OUT/t.log 2>&1
python3 scripts/trace_steps.py $(find $OUT/t -name '*kernel_trace.csv' | head -1) --steps 20 \
  --csv $OUT/durations.csv --seq $OUT/seq.txt > $OUT/durations.txt
rm -rf $OUT/t
tail -1 $OUT/t.log
cat $OUT/durations.txt | head -60
