set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu_final.log
exit $rc
