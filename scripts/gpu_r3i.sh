# X6 candidates everywhere: PG-GAN lod 3 / lod 0 bench, VGG bench (pre-transformed paths up to 32x32 maps)
set -o pipefail
mkdir -p gpurun_out/r3i
RAFIKI_AUTOTUNE_LOG=$PWD/gpurun_out/r3i/pg_tune.jsonl timeout -k 10 400 python -u scripts/bench_pg_gan.py --lods 3,0 > gpurun_out/r3i/pg.log 2>&1 || exit $?
tail -1 gpurun_out/r3i/pg.log | cut -c1-600
RAFIKI_AUTOTUNE_LOG=$PWD/gpurun_out/r3i/vgg_tune.jsonl timeout -k 10 300 python -u bench.py --trials 0 --probe-trials 0 --no-serving > gpurun_out/r3i/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3i/bench.log | cut -c1-300
