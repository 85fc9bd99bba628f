set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/*.log
timeout -k 10 600 python -u -m pytest tests/test_winograd_gpu.py tests/test_engine_gpu.py tests/test_f32_gpu.py tests/test_serving_gpu.py tests/test_convergence_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/w_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
bash scripts/prof_step.sh stem8 > gpurun_out/prof.log 2>&1
rc=$?
tail -2 gpurun_out/w_tests.log; tail -1 gpurun_out/bench.log | cut -c1-250; head -32 gpurun_out/prof_stem8/durations.txt
exit $rc
