set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/*.log
RAFIKI_WINO_PIPE=1 timeout -k 10 400 python -u -m pytest tests/test_winograd_gpu.py tests/test_winograd4_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w_tests.log 2>&1 && \
RAFIKI_WINO_PIPE=1 timeout -k 10 180 python -u scripts/bench_winograd4.py gpurun_out/w_bench.jsonl > gpurun_out/w_bench.log 2>&1 && \
RAFIKI_WINO_PIPE=1 RAFIKI_AUTOTUNE_LOG=gpurun_out/tune.jsonl timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
RAFIKI_WINO_PIPE=1 bash scripts/prof_step.sh w2s > gpurun_out/prof.log 2>&1
rc=$?
tail -3 gpurun_out/w_tests.log; cat gpurun_out/w_bench.log; tail -1 gpurun_out/bench.log | cut -c1-300; head -30 gpurun_out/prof_w2s/durations.txt
exit $rc
