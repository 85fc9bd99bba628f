set -o pipefail
bash scripts/gpu_r3i.sh || exit $?
bash scripts/gpu_pmc_xconv.sh > gpurun_out/r3i/pmc_xc.log 2>&1 || exit $?
cat gpurun_out/r3i/pmc_xc.log | cut -c1-900
