# Round-3 GPU pass: full GPU suite, then the bench (1 GPU), then --gpus 2 must fail fast on 1 GPU
set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3b/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r3b/pytest_gpu.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r3b/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3b/bench.log
timeout -k 10 120 python -u bench.py --gpus 2 > gpurun_out/r3b/bench2.log 2>&1
echo "gpus2 rc=$? (expected non-zero)"; tail -2 gpurun_out/r3b/bench2.log
exit 0
