#!/bin/bash
# PG-GAN: at::native census per LOD, and the lod-0 resampling-conv route A/B (direct vs Winograd)
set -o pipefail
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 400 python -u scripts/pggan_aten_census.py --lods 3,0 > $O/census.jsonl 2> $O/census.err || exit $?
for m in direct wino auto; do
  RAFIKI_PGGAN_RESAMPLE=$m timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 0 --steps 10 --warmup 3 \
    > $O/lod0_$m.json 2> $O/lod0_$m.err || exit $?
  cat $O/lod0_$m.json
done
