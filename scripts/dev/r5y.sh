#!/bin/bash
# full GPU suite + smoke + default bench on the shipped tune DB
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log | cut -c1-700; exit $rc
