set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_winograd_gpu.py tests/test_winograd4_gpu.py tests/test_f32_gpu.py tests/test_serving_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/sanity_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?
tail -1 gpurun_out/smoke.log; tail -2 gpurun_out/sanity_tests.log; tail -1 gpurun_out/bench.log | cut -c1-200
exit $rc
