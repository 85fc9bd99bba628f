#!/bin/bash
# PG-GAN evidence on one box: GPU tests, aten census, throughput (graphed / eager, resampling A/B), per-LOD
# kernel + PMC profiles, the data-parallel segmented round.  -> gpurun_out/pggan_ev/ + pgprof_lod{3,0}/ + pgdp/
set -o pipefail
O=gpurun_out/pggan_ev; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pg_gan_gpu.py \
  tests/test_resample_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/dev/pggan_aten_census.py --lods 3,0 > $O/census.jsonl 2> $O/census.err || exit $?
for spec in "RAFIKI_PGGAN_RESAMPLE=wino" "RAFIKI_PGGAN_RESAMPLE=direct"; do
  env $spec timeout -k 10 400 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --warmup 3 \
    > $O/bench_${spec#*=}.json 2> $O/bench_${spec#*=}.err || exit $?
done
timeout -k 10 400 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --warmup 3 --no-graph > $O/bench_eager.json \
  2> $O/bench_eager.err || exit $?
cat $O/bench_*.json
bash scripts/gpu_pggan_prof.sh 3 6 > $O/prof3.log 2>&1 || exit $?
bash scripts/gpu_pggan_prof.sh 0 4 > $O/prof0.log 2>&1 || exit $?
bash scripts/dev/gpu_pggan_dp.sh > $O/dp.log 2>&1 || exit $?
echo done
