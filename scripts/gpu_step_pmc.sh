set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/*.log
timeout -k 10 400 python -u -m pytest tests/test_winograd_gpu.py tests/test_winograd4_gpu.py tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w_tests.log 2>&1 && \
timeout -k 10 180 python -u scripts/dev/bench_winograd4.py gpurun_out/w_bench.jsonl > gpurun_out/w_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
bash scripts/pmc_step.sh > gpurun_out/pmc.log 2>&1
rc=$?
tail -2 gpurun_out/w_tests.log; cat gpurun_out/w_bench.log; tail -1 gpurun_out/bench.log | cut -c1-200; cat gpurun_out/pmc_step/summary.txt | head -40
exit $rc
