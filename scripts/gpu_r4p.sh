#!/bin/bash
# PG-GAN after the fused loss head / in-place grads / Winograd resampling: tests, census, profiles, A/B
set -o pipefail
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ \
  > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/pggan_aten_census.py --lods 3,0 > $O/census.jsonl 2> $O/census.err || exit $?
for m in wino direct; do
  RAFIKI_PGGAN_RESAMPLE=$m timeout -k 10 400 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --warmup 3 \
    > $O/bench_$m.json 2> $O/bench_$m.err || exit $?
  cat $O/bench_$m.json
done
bash scripts/gpu_pggan_prof.sh 3 6 > $O/prof3.log 2>&1 || exit $?
bash scripts/gpu_pggan_prof.sh 0 4 > $O/prof0.log 2>&1 || exit $?
tail -4 $O/prof3.log $O/prof0.log
