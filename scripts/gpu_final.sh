#!/bin/bash
# Round-end evidence: full GPU suite, smoke, default bench (the driver's command), step kernels + PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final; mkdir -p $O
# bash scripts/gpu_final.sh        : suite + smoke + default bench
# bash scripts/gpu_final.sh prof   : step kernel trace + PMC passes
if [ "$1" != "prof" ]; then
  bash scripts/gpu_suite.sh || exit 1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
    || { tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-300
fi
if [ "$1" = "prof" ]; then
  bash scripts/prof_step.sh final > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
  head -3 gpurun_out/prof_final/durations.txt
  bash scripts/pmc_step.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
  tail -1 gpurun_out/pmc_step/summary.txt
fi
