set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/*.log
timeout -k 10 300 python -u -m pytest tests/test_winograd4_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/w4_tests.log 2>&1 && \
timeout -k 10 180 python -u scripts/bench_winograd4.py gpurun_out/w4_bench.jsonl > gpurun_out/w4_bench.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --deselect tests/test_pg_gan_gpu.py::test_dp_round_with_rccl_allreduce_is_graph_captured > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1 && \
NCCL_DEBUG=INFO AMD_LOG_LEVEL=2 timeout -k 10 180 python -u -m pytest tests/test_pg_gan_gpu.py -x -v --timeout 120 --timeout-method thread -k test_dp_round_with_rccl > gpurun_out/dp_debug.log 2>&1
rc=$?
tail -3 gpurun_out/w4_tests.log; cat gpurun_out/w4_bench.log; tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -2 gpurun_out/bench.log; tail -3 gpurun_out/dp_debug.log
exit $rc
