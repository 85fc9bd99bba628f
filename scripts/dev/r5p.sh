#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5p; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 120 python -u scripts/dev/ext_event_diag.py > $O/ext_event.log 2>&1
rc=$?; echo "ext rc=$rc"; grep -v amdgpu.ids $O/ext_event.log | cut -c1-600; fatal $rc ext_event
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_graph_events_gpu.py tests/test_tagger_gpu.py tests/test_pg_gan_gpu.py tests/test_winograd_gpu.py tests/test_winograd4_gpu.py -k "events or overlapped or adam or dp_round or wgrad" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -30; fatal $rc pytest
timeout -k 10 300 python -u scripts/dev/wino4_variants.py > $O/variants.jsonl 2>&1
rc=$?; fatal $rc variants; grep wgrad $O/variants.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/dp -o dp -- python scripts/dev/pggan_dp_trace.py 2.0 > $O/dp.log 2>&1
rc=$?; echo "dp rc=$rc"; grep -v "^W2026" $O/dp.log | tail -3; fatal $rc dp_trace
f=$(find $O/dp -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/dev/dp_overlap_summary.py "$f" > $O/dp_overlap.txt 2>&1; cat $O/dp_overlap.txt
rm -rf $O/dp
