# Round-3 GPU pass: wgrad variant tests + per-layer bench, full GPU suite, bench (1 GPU), --gpus 2 fails fast
set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest tests/test_winograd4_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/r3c/w4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3c/w4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_wgrad4.py gpurun_out/r3c/wgrad4.jsonl > gpurun_out/r3c/wgrad4.log 2>&1 || exit $?
cat gpurun_out/r3c/wgrad4.log | cut -c1-220
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3c/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3c/pytest_gpu.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r3c/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3c/bench.log
timeout -k 10 120 python -u bench.py --gpus 2 > gpurun_out/r3c/bench2.log 2>&1
echo "gpus2 rc=$? (expected non-zero)"; tail -2 gpurun_out/r3c/bench2.log
exit 0
