# few-wave X6 tiles: numerics, VGG / PG-GAN bench with the node tune database captured under gpurun_out
set -o pipefail
mkdir -p gpurun_out/r3m
export RAFIKI_TUNE_CACHE=$PWD/gpurun_out/r3m/tune_node.json
timeout -k 10 300 python -u -m pytest tests/test_x6_gpu.py tests/test_winograd4_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3m/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3m/tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
RAFIKI_AUTOTUNE_LOG=$PWD/gpurun_out/r3m/pg_tune.jsonl timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 3,0 > gpurun_out/r3m/pg.log 2>&1 || exit $?
tail -1 gpurun_out/r3m/pg.log | cut -c150-600
RAFIKI_AUTOTUNE_LOG=$PWD/gpurun_out/r3m/vgg_tune.jsonl timeout -k 10 400 python -u bench.py > gpurun_out/r3m/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3m/bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py > gpurun_out/r3m/bench_warm.log 2>&1 || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/r3m/bench_warm.log').read().strip().split(chr(10))[-1])
print('warm', d['value'], d['ms_per_step'], d['trials_per_hour_measured'], d['trial_breakdown_s']['first_trial_rank0']['wall'], d['trial_breakdown_s']['steady_mean_rank0']['train'])"
