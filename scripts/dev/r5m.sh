#!/bin/bash
# combined: tagger step + overlapped DP reduce (r5j) and the wgrad loader remap (r5l); a step that
# times out or crashes ends the script, an ordinary failure is reported and the next phase runs
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5m; mkdir -p $O
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graph_events_gpu.py tests/test_tagger_gpu.py tests/test_lstm_gpu.py tests/test_lstm_native_gpu.py tests/test_pg_gan_gpu.py -k "events or overlapped or tagger or lstm or bilstm or embedding or dp_round" > $O/pytest_tagger.log 2>&1
rc=$?; echo "pytest tagger rc=$rc"; tail -25 $O/pytest_tagger.log; fatal $rc pytest_tagger
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_winograd4_gpu.py tests/test_f32_gpu.py > $O/pytest_wino.log 2>&1
rc=$?; echo "pytest wino rc=$rc"; tail -3 $O/pytest_wino.log; fatal $rc pytest_wino
timeout -k 10 200 python scripts/dev/tagger_step.py --graph 1 > $O/step_graph.json 2>$O/step_graph.err
rc=$?; fatal $rc tagger_graph
timeout -k 10 200 python scripts/dev/tagger_step.py --graph 0 > $O/step_eager.json 2>$O/step_eager.err
rc=$?; fatal $rc tagger_eager
cat $O/step_graph.json $O/step_eager.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/dev/tagger_step.py --graph 1 --steps 100 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; fatal $rc tagger_prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/dp -o dp -- python scripts/dev/pggan_dp_trace.py 2.0 > $O/dp.log 2>&1
rc=$?; echo "dp rc=$rc"; tail -3 $O/dp.log; fatal $rc dp_trace
f=$(find $O/dp -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/dev/dp_overlap_summary.py "$f" > $O/dp_overlap.txt 2>&1; cat $O/dp_overlap.txt
rm -rf $O/dp/*/ 2>/dev/null
timeout -k 10 300 python -u scripts/dev/wino4_variants.py > $O/variants.jsonl 2>&1
rc=$?; fatal $rc variants; grep wgrad $O/variants.jsonl
bash scripts/gpu_iter.sh r5m_it
