set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_configs.py --configs 2,3e > gpurun_out/configs.log 2>&1
rc=$?
grep "^{" gpurun_out/configs.log | cut -c1-600
exit $rc
