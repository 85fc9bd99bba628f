# 32-bit BN index math: fp32 kernel tests, step kernel trace
set -o pipefail
mkdir -p gpurun_out/r3n
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py tests/test_engine_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r3n/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3n/tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_step.sh r3n > gpurun_out/r3n/prof.log 2>&1 || exit $?
grep -E "bnf|wall/step" gpurun_out/prof_r3n/durations.txt; tail -3 gpurun_out/r3n/prof.log | cut -c1-200
timeout -k 10 200 python -u -m pytest tests/test_xconv_gpu.py -x -q -k writes_only --timeout 120 --timeout-method thread > gpurun_out/r3n/xc_canary.log 2>&1; tail -3 gpurun_out/r3n/xc_canary.log | cut -c1-300
