#!/bin/bash
# capture a cold tune database over every shape of the default bench (trial, eval, serving) and the
# PG-GAN lod 3 / 0 rounds, then re-rank its near-tied VGG-step picks by whole-step time
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5k; mkdir -p $O
rm -f $O/cap_db.json
RAFIKI_TUNE_CACHE=$PWD/$O/cap_db.json timeout -k 10 600 python -u bench.py > $O/bench_cap.log 2>&1 || { tail -20 $O/bench_cap.log; exit 1; }
tail -1 $O/bench_cap.log | cut -c1-400
RAFIKI_TUNE_CACHE=$PWD/$O/cap_db.json timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 3,0 > $O/pg_cap.log 2>&1 || { tail -20 $O/pg_cap.log; exit 1; }
tail -1 $O/pg_cap.log | cut -c1-400
timeout -k 10 500 python -u scripts/step_refine.py --start $O/cap_db.json --out $O/refine > $O/refine.log 2>&1 || { tail -20 $O/refine.log; exit 1; }
tail -2 $O/refine.log
