#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 400 python -u scripts/dev/serve_replica_diag.py > $O/diag.log 2>&1
rc=$?; echo "diag rc=$rc"; grep "^{" $O/diag.log | cut -c1-1500
