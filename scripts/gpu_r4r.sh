#!/bin/bash
# tune-DB capture for the current kernel sources, the PG-GAN DP segmented round, the at::native census
set -o pipefail
O=gpurun_out/r4r; mkdir -p $O
bash scripts/gpu_tunecap.sh > $O/tunecap.log 2>&1 || { tail -5 $O/tunecap.log; exit 1; }
tail -2 $O/tunecap.log
bash scripts/gpu_pggan_dp.sh > $O/dp.log 2>&1 || { tail -5 $O/dp.log; exit 1; }
grep images_per_sec $O/dp.log | cut -c1-600
timeout -k 10 400 python -u scripts/pggan_aten_census.py --lods 3,0 > $O/census.jsonl 2> $O/census.err || exit $?
echo done
