set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/*.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
bash scripts/pmc_step.sh > gpurun_out/pmc.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log | cut -c1-300; head -3 gpurun_out/pmc_step/durations.txt; tail -1 gpurun_out/pmc_step/summary.txt
exit $rc
