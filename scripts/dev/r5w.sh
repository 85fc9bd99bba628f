#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_serving_gpu.py -k "two_replicas or native" > $O/pytest_serving2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest_serving2.log; grep -E "^E " $O/pytest_serving2.log | head -5
case $rc in 124|137|134|139) exit $rc;; esac
bash scripts/dev/ab_db.sh scripts/dev/db_A_cap.json scripts/dev/db_B_fresh.json
cat gpurun_out/ab_db/results.txt
