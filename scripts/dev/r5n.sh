#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5n; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 120 python -u scripts/dev/ext_event_diag.py > $O/ext_event.log 2>&1
rc=$?; echo "ext rc=$rc"; cat $O/ext_event.log | grep -v amdgpu.ids; fatal $rc ext_event
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_tagger_gpu.py tests/test_lstm_gpu.py tests/test_lstm_native_gpu.py tests/test_pg_gan_gpu.py -k "tagger or lstm or bilstm or embedding or dp_round" > $O/pytest_tagger.log 2>&1
rc=$?; echo "pytest tagger rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_tagger.log | tail -40; fatal $rc pytest_tagger
timeout -k 10 200 python scripts/dev/tagger_step.py --graph 1 > $O/step_graph.json 2>$O/step_graph.err
rc=$?; tail -3 $O/step_graph.err; fatal $rc tagger_graph
timeout -k 10 200 python scripts/dev/tagger_step.py --graph 0 > $O/step_eager.json 2>$O/step_eager.err
rc=$?; tail -3 $O/step_eager.err; fatal $rc tagger_eager
cat $O/step_graph.json $O/step_eager.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/dev/tagger_step.py --graph 1 --steps 100 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; fatal $rc tagger_prof
find $O/prof -name "*kernel_stats.csv" | head -2
