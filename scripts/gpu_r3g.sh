# Round-3 pass 5: per-kernel step profile + autotune decisions of the VGG-small step and PG-GAN lod 0
set -o pipefail
mkdir -p gpurun_out/r3g
RAFIKI_AUTOTUNE_LOG=$PWD/gpurun_out/r3g/vgg_autotune.jsonl bash scripts/prof_step.sh vgg > gpurun_out/r3g/prof_vgg.log 2>&1 || exit $?
head -45 gpurun_out/prof_vgg/durations.txt | cut -c1-140
RAFIKI_AUTOTUNE_LOG=$PWD/gpurun_out/r3g/pg0_autotune.jsonl timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 0 --steps 4 > gpurun_out/r3g/pg0.log 2>&1 || exit $?
tail -1 gpurun_out/r3g/pg0.log | cut -c200-500
wc -l gpurun_out/r3g/*.jsonl
RAFIKI_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 3 --trials 1 --probe-trials 2 --no-serving > gpurun_out/r3g/bench_2rank_gloo.log 2>&1 || exit $?
grep -v "^\[rank1\]" gpurun_out/r3g/bench_2rank_gloo.log | tail -1 | cut -c1-600
timeout -k 10 400 python -u scripts/bench_predictor.py --out gpurun_out/r3g/predictor_qps.json > gpurun_out/r3g/qps.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/r3g/predictor_qps.json'));print({k:d.get(k) for k in ('http_native','http_asyncio','batcher')})"
timeout -k 10 400 python -u scripts/bench_predictor.py --replicas 2 --skip-http-asyncio --out gpurun_out/r3g/predictor_qps_2rep.json > gpurun_out/r3g/qps2.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/r3g/predictor_qps_2rep.json'));print({k:d.get(k) for k in ('http_native','batcher')})"
