#!/bin/bash
# wgrad loader remap: fp64 tests, variant timings, fresh-tune step bench + kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r5l
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd4_gpu.py tests/test_f32_gpu.py > gpurun_out/r5l/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r5l/pytest.log
timeout -k 10 300 python -u scripts/dev/wino4_variants.py > gpurun_out/r5l/variants.jsonl 2>&1 && grep wgrad gpurun_out/r5l/variants.jsonl && \
bash scripts/gpu_iter.sh r5l_it
