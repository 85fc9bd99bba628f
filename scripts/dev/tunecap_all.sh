#!/bin/bash
# Capture the shipped autotune database for the current kernel build: the default bench.py run (VGG-small
# step, HPO / probe trials, serving shapes) and the PG-GAN rounds at lods 3 and 0, into ONE file
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tunecap; mkdir -p $O
export RAFIKI_TUNE_CACHE=$PWD/$O/tune_db.json
timeout -k 10 900 python -u bench.py --gpus 1 --steps 50 --warmup 10 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 600 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --warmup 3 > $O/pgbench.log 2>&1 \
  || { tail -20 $O/pgbench.log; exit 1; }
tail -3 $O/pgbench.log | cut -c1-300
python3 -c "import json; print(len(json.load(open('$O/tune_db.json'))), 'entries')"
