# Round-3 re-entry: full GPU suite, default bench, step kernel trace + PMC at HEAD
set -o pipefail
mkdir -p gpurun_out/r3h
timeout -k 10 200 python -u -m pytest tests/test_serving_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3h/pytest_serving.log 2>&1; tail -2 gpurun_out/r3h/pytest_serving.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3h/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3h/pytest_gpu.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r3h/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3h/bench.log | cut -c1-400
bash scripts/pmc_step.sh > gpurun_out/r3h/pmc.log 2>&1 || exit $?
head -50 gpurun_out/pmc_step/summary.txt
