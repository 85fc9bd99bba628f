# PG-GAN lod 0 kernel trace + PMC with the X6 candidates; full bench with the node tune database captured
# under gpurun_out (to ship as the package seed for this kernel library)
set -o pipefail
mkdir -p gpurun_out/r3l
export RAFIKI_TUNE_CACHE=$PWD/gpurun_out/r3l/tune_node.json
bash scripts/gpu_pggan_prof.sh 0 > gpurun_out/r3l/pgprof.log 2>&1 || { tail -5 gpurun_out/r3l/pgprof.log; exit 1; }
cat gpurun_out/r3l/pgprof.log | cut -c1-160
timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 3,0 > gpurun_out/r3l/pg.log 2>&1 || exit $?
tail -1 gpurun_out/r3l/pg.log | cut -c150-600
timeout -k 10 400 python -u bench.py > gpurun_out/r3l/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3l/bench.log | cut -c1-300
timeout -k 10 400 python -u bench.py > gpurun_out/r3l/bench_warm.log 2>&1 || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/r3l/bench_warm.log').read().strip().split(chr(10))[-1])
print('warm', d['value'], d['trials_per_hour_measured'], d['trial_breakdown_s']['first_trial_rank0']['wall'], d['trial_breakdown_s']['steady_mean_rank0']['train'])"
