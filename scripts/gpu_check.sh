set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log | tail -2; tail -2 gpurun_out/bench.log
exit $rc
