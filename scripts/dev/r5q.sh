#!/bin/bash
# verification (external events, Adam, DP round, wgrad remaps) + cold tune capture over the default bench
# and the PG-GAN lods; a timeout / crash ends the script
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5q; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 120 python -u scripts/dev/ext_event_diag.py > $O/ext_event.log 2>&1
rc=$?; echo "ext rc=$rc"; grep -v amdgpu.ids $O/ext_event.log | cut -c1-400; fatal $rc ext_event
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_graph_events_gpu.py tests/test_tagger_gpu.py tests/test_pg_gan_gpu.py tests/test_winograd_gpu.py tests/test_winograd4_gpu.py -k "events or overlapped or adam or dp_round or wgrad" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -20; fatal $rc pytest
timeout -k 10 200 python -u scripts/dev/wino4_variants.py > $O/variants.jsonl 2>&1
rc=$?; fatal $rc variants; grep wgrad $O/variants.jsonl | cut -c1-300
rm -f $O/cap_db.json
RAFIKI_TUNE_CACHE=$PWD/$O/cap_db.json timeout -k 10 500 python -u bench.py > $O/bench_cap.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_cap.log | cut -c1-600; fatal $rc bench
[ $rc -eq 0 ] || exit 1
RAFIKI_TUNE_CACHE=$PWD/$O/cap_db.json timeout -k 10 240 python -u scripts/bench_pg_gan.py --lods 3,0 > $O/pg_cap.log 2>&1
rc=$?; echo "pg rc=$rc"; tail -1 $O/pg_cap.log | cut -c1-600; fatal $rc pg_bench
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/dp -o dp -- python scripts/dev/pggan_dp_trace.py 2.0 > $O/dp.log 2>&1
rc=$?; echo "dp rc=$rc"; grep -v "^W2026" $O/dp.log | tail -2; fatal $rc dp_trace
f=$(find $O/dp -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/dev/dp_overlap_summary.py "$f" > $O/dp_overlap.txt 2>&1; cat $O/dp_overlap.txt
rm -rf $O/dp
