#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_serving_gpu.py tests/test_tagger_gpu.py tests/test_x6_gpu.py tests/test_engine_gpu.py > $O/pytest_fixed.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest_fixed.log; grep -E "FAILED|ERROR" $O/pytest_fixed.log | head
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log | cut -c1-700; exit $rc
