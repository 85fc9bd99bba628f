set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/*.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_pg_gan.py > gpurun_out/pg_gan_bench.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_predictor.py --out gpurun_out/predictor_qps.json > gpurun_out/predictor.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/pg_gan_bench.log; tail -1 gpurun_out/predictor.log | cut -c1-1200
exit $rc
