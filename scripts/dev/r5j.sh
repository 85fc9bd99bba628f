#!/bin/bash
# native tagger step + overlapped DP reduce: GPU tests, timing, rocprofv3 kernel census / overlap trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r5j
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tagger_gpu.py tests/test_lstm_gpu.py tests/test_lstm_native_gpu.py tests/test_pg_gan_gpu.py -k "tagger or lstm or bilstm or embedding or dp_round" > gpurun_out/r5j/pytest.log 2>&1
echo "pytest rc=$?"
tail -30 gpurun_out/r5j/pytest.log
timeout -k 10 200 python scripts/dev/tagger_step.py --graph 1 > gpurun_out/r5j/step_graph.json 2>gpurun_out/r5j/step_graph.err && \
timeout -k 10 200 python scripts/dev/tagger_step.py --graph 0 > gpurun_out/r5j/step_eager.json 2>gpurun_out/r5j/step_eager.err && \
cat gpurun_out/r5j/step_graph.json gpurun_out/r5j/step_eager.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5j/prof -o run -- python scripts/dev/tagger_step.py --graph 1 --steps 100 > gpurun_out/r5j/prof.log 2>&1
echo "prof rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5j/dp -o dp -- python scripts/dev/pggan_dp_trace.py 2.0 > gpurun_out/r5j/dp.log 2>&1
echo "dp rc=$?"
tail -3 gpurun_out/r5j/dp.log
f=$(find gpurun_out/r5j/dp -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/dev/dp_overlap_summary.py "$f" > gpurun_out/r5j/dp_overlap.txt 2>&1; cat gpurun_out/r5j/dp_overlap.txt
find gpurun_out/r5j/prof -name "*kernel_stats.csv" | head -3
