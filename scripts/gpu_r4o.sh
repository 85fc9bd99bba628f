#!/bin/bash
# PG-GAN: fused loss head + in-place bias/weight grads + leaky-ReLU PT Winograd: tests, census, throughput
set -o pipefail
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pg_gan_gpu.py \
  tests/test_x6p_gpu.py -k "wgan or in_place or lrelu or pixel or generator or discriminator" > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/pggan_aten_census.py --lods 3,0 > $O/census.jsonl 2> $O/census.err || exit $?
for m in wino direct; do
  RAFIKI_PGGAN_RESAMPLE=$m timeout -k 10 400 python -u scripts/bench_pg_gan.py --lods 3,0 --steps 10 --warmup 3 \
    > $O/bench_$m.json 2> $O/bench_$m.err || exit $?
  cat $O/bench_$m.json
done
