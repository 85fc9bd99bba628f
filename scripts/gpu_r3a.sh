# Round-3 first GPU pass: full GPU suite, bench at HEAD (1 GPU, and --gpus 2 must fail fast), step profile
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3a/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r3a/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r3a/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3a/bench.log | cut -c1-400
timeout -k 10 120 python -u bench.py --gpus 2 > gpurun_out/r3a/bench2.log 2>&1
echo "gpus2 rc=$? (expected non-zero)"; tail -2 gpurun_out/r3a/bench2.log
bash scripts/pmc_step.sh > gpurun_out/r3a/pmc.log 2>&1 || exit $?
cp -r gpurun_out/pmc_step gpurun_out/r3a/
