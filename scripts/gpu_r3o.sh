# round-close pass at HEAD: full GPU suite, PG-GAN + VGG benches capturing the node tune database under
# gpurun_out (shipped as the package seed for these kernel sources), warm-database bench
set -o pipefail
mkdir -p gpurun_out/r3o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3o/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3o/pytest_gpu.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
export RAFIKI_TUNE_CACHE=$PWD/gpurun_out/r3o/tune_node.json
timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 3,0 > gpurun_out/r3o/pg.log 2>&1 || exit $?
tail -1 gpurun_out/r3o/pg.log | cut -c150-600
RAFIKI_AUTOTUNE_LOG=$PWD/gpurun_out/r3o/vgg_tune.jsonl timeout -k 10 400 python -u bench.py > gpurun_out/r3o/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3o/bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py > gpurun_out/r3o/bench_warm.log 2>&1 || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/r3o/bench_warm.log').read().strip().split(chr(10))[-1])
print('warm', d['value'], d['ms_per_step'], d['trials_per_hour_measured'], d['trial_breakdown_s']['first_trial_rank0']['wall'], d['trial_breakdown_s']['steady_mean_rank0']['train'])"
bash scripts/prof_step.sh r3o > gpurun_out/r3o/prof.log 2>&1 || exit $?
head -30 gpurun_out/prof_r3o/durations.txt
