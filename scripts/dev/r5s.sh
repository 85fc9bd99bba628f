#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 400 python -u scripts/dev/serve_diag.py > $O/serve_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; grep -v amdgpu.ids $O/serve_diag.log | cut -c1-300 | head -80
