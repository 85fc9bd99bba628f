set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/*.log
timeout -k 10 400 python -u -m pytest tests/test_winograd4_gpu.py tests/test_winograd_gpu.py tests/test_f32_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/w4_tests.log 2>&1 && \
RAFIKI_AUTOTUNE_LOG=gpurun_out/tune_w4.jsonl timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1 && \
bash scripts/prof_step.sh w4 > gpurun_out/prof.log 2>&1
rc=$?
tail -3 gpurun_out/w4_tests.log; tail -1 gpurun_out/bench.log; head -40 gpurun_out/prof_w4/durations.txt
exit $rc
