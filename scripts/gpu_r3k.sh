# Round-3 X6 pass: full GPU suite, default bench (trials + serving), step kernel trace + PMC, xconv engine diagnostic
set -o pipefail
mkdir -p gpurun_out/r3k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3k/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3k/pytest_gpu.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
RAFIKI_AUTOTUNE_LOG=$PWD/gpurun_out/r3k/vgg_tune.jsonl timeout -k 10 400 python -u bench.py > gpurun_out/r3k/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3k/bench.log | cut -c1-500
bash scripts/pmc_step.sh > gpurun_out/r3k/pmc.log 2>&1 || exit $?
head -40 gpurun_out/pmc_step/summary.txt
RAFIKI_TUNE_CACHE=off RAFIKI_XCONV=1 timeout -k 10 200 python -u scripts/diag_xconv_engine.py > gpurun_out/r3k/diag_xc.log 2>&1 || exit $?
cat gpurun_out/r3k/diag_xc.log | grep -v amdgpu.ids
