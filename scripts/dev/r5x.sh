#!/bin/bash
# normalise-on-load: numerics + engine parity, then the winograd4 / f32 suites
set -o pipefail
mkdir -p gpurun_out/r5x
timeout -k 10 400 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_bn_on_load_gpu.py \
  > gpurun_out/r5x/bnl.log 2>&1 || { tail -40 gpurun_out/r5x/bnl.log; exit 1; }
tail -3 gpurun_out/r5x/bnl.log
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_winograd4_gpu.py \
  tests/test_f32_gpu.py > gpurun_out/r5x/w4.log 2>&1; rc=$?
tail -15 gpurun_out/r5x/w4.log
exit $rc
