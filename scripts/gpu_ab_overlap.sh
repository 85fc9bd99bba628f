set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/*.log
timeout -k 10 400 python -u -m pytest tests/test_winograd_gpu.py tests/test_engine_gpu.py tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w_tests.log 2>&1 && \
timeout -k 10 240 python -u bench.py --trials 0 --no-serving > gpurun_out/bench_a.log 2>&1 && \
RAFIKI_OVERLAP_WGRAD=1 timeout -k 10 240 python -u bench.py --trials 0 --no-serving > gpurun_out/bench_b.log 2>&1 && \
timeout -k 10 240 python -u bench.py --trials 0 --no-serving > gpurun_out/bench_a2.log 2>&1 && \
RAFIKI_OVERLAP_WGRAD=1 bash scripts/prof_step.sh ovl > gpurun_out/prof_ovl.log 2>&1
rc=$?
tail -2 gpurun_out/w_tests.log; for f in a b a2; do tail -1 gpurun_out/bench_$f.log | cut -c1-220; done; head -30 gpurun_out/prof_ovl/durations.txt
exit $rc
