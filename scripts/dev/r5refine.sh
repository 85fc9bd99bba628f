#!/bin/bash
# whole-step re-ranking of the shipped VGG-small picks, then a same-box A/B shipped vs refined
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/refine
DST=rafiki_amd/tune/$(python3 -c "from rafiki_amd.ops import autotune; print(autotune.db_name())")
cp "$DST" gpurun_out/refine/shipped.json
timeout -k 10 800 python -u scripts/step_refine.py --out gpurun_out/refine > gpurun_out/refine/log.txt 2>&1 \
  || { tail -20 gpurun_out/refine/log.txt; exit 1; }
tail -2 gpurun_out/refine/log.txt
rm -f gpurun_out/ab_db/results.txt
bash scripts/dev/ab_db.sh gpurun_out/refine/shipped.json gpurun_out/refine/refined_db.json
