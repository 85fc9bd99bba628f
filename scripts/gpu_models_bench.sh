set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_pg_gan.py > gpurun_out/pg_gan_bench.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_predictor.py --out gpurun_out/predictor_qps.json > gpurun_out/predictor.log 2>&1
rc=$?
tail -1 gpurun_out/pg_gan_bench.log; tail -1 gpurun_out/predictor.log | cut -c1-1500
exit $rc
