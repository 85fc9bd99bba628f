#!/bin/bash
# Capture a node tune database for every shape the driver's bench touches, and A/B it against the shipped
# picks on the same box:
#   fresh.json  every pick re-tuned in this run (the shipped seed moved aside): bench.py (VGG-small step,
#               trials, serving buckets, PG-GAN lod 3 / lod 0, MLP) + the per-rank PG-GAN minibatches of the
#               data-parallel phase at N = 2, 4, 8
#   A / B       the training step on fresh.json vs on the shipped seed, alternating (A B A B)
# -> gpurun_out/tunecap/{fresh.json, bench_fresh.json, ab.txt}
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/tunecap
mkdir -p $OUT /tmp/shipped_seed
mv rafiki_amd/tune/*.json /tmp/shipped_seed/
export RAFIKI_TUNE_CACHE=$PWD/$OUT/fresh.json
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_fresh.json 2> $OUT/bench_fresh.err
for mb in 256 128 64; do
  timeout -k 10 300 python scripts/bench_pg_gan.py --lods 3 --minibatch $mb --steps 3 --warmup 3 >> $OUT/pg_dp_shapes.jsonl 2>/dev/null
done
for mb in 32 16 8; do
  timeout -k 10 300 python scripts/bench_pg_gan.py --lods 0 --minibatch $mb --steps 3 --warmup 3 >> $OUT/pg_dp_shapes.jsonl 2>/dev/null
done
STEP="bench.py --steps 50 --warmup 10 --trials 0 --probe-trials 0 --no-serving --configs none"
for r in 1 2; do
  RAFIKI_TUNE_CACHE=$PWD/$OUT/fresh.json timeout -k 10 300 python $STEP > $OUT/a$r.json 2>/dev/null
  mv /tmp/shipped_seed/*.json rafiki_amd/tune/
  RAFIKI_TUNE_CACHE=off timeout -k 10 300 python $STEP > $OUT/b$r.json 2>/dev/null
  mv rafiki_amd/tune/*.json /tmp/shipped_seed/
done
mv /tmp/shipped_seed/*.json rafiki_amd/tune/
for f in a1 b1 a2 b2; do python3 -c "import json; d = json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'])"; done > $OUT/ab.txt
cat $OUT/ab.txt
