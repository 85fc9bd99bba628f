set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/bnp_tests.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/bnp_bench_on.log 2>&1 &&
RAFIKI_BN_POOL_FUSE=0 timeout -k 10 200 python bench.py > gpurun_out/bnp_bench_off.log 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/bnp_bench_on2.log 2>&1
