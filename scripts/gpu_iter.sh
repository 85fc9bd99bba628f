#!/bin/bash
# One build -> measure iteration on the GPU box:
#   scripts/gpu_iter.sh <tag> [pytest targets...]
# runs the given GPU tests (if any), then the headline bench with a FRESH tune (every candidate's time per
# shape logged to gpurun_out/<tag>/tune.jsonl), then a per-kernel profile of the steady-state steps
# (scripts/prof_step.sh) against the database that run just wrote.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export RAFIKI_TUNE_CACHE=$PWD/$OUT/tune_db.json
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
RAFIKI_AUTOTUNE_LOG=$PWD/$OUT/tune.jsonl timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --trials 0 \
  --probe-trials 0 --no-serving > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-260
bash scripts/prof_step.sh $TAG > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
head -40 gpurun_out/prof_$TAG/durations.txt
