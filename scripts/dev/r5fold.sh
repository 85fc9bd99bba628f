#!/bin/bash
# folded eval BN in the grouped ensemble: tests, then the default bench (serving phase QPS)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5fold; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_f32_gpu.py tests/test_serving_gpu.py \
  > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log | cut -c1-2000; exit $rc
