#!/bin/bash
# PG-GAN: mix kernel + per-step weight-transform cache: tests, throughput, profiles
set -o pipefail
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pg_gan_gpu.py tests/test_resample_gpu.py \
  > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 400 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --warmup 3 --no-graph > $O/bench_eager.json \
  2> $O/bench_eager.err || exit $?
cat $O/bench_eager.json
bash scripts/gpu_pggan_prof.sh 3 6 > $O/prof3.log 2>&1 || exit $?
bash scripts/gpu_pggan_prof.sh 0 4 > $O/prof0.log 2>&1 || exit $?
echo done
