#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -v --timeout 150 --timeout-method thread > $O/serving.log 2>&1
rc=$?; echo "serving rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/serving.log | tail -40
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread --deselect tests/test_serving_gpu.py::test_native_front_end_npy_and_two_replicas_double_buffered > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -5 $O/suite.log; grep -E "FAILED|ERROR" $O/suite.log | head
