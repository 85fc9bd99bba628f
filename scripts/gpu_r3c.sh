# Round-3 GPU pass: targeted tests (new wgrad path, PG-GAN graphed-vs-eager), full GPU suite, bench, --gpus 2
set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest tests/test_winograd4_gpu.py tests/test_pg_gan_gpu.py -q -s -k "wgrad or graphed_rounds" --timeout 120 --timeout-method thread > gpurun_out/r3c/targeted.log 2>&1
rc=$?; grep -E "frob|passed|failed" gpurun_out/r3c/targeted.log | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread --deselect tests/test_pg_gan_gpu.py::test_graphed_rounds_match_eager > gpurun_out/r3c/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3c/pytest_gpu.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r3c/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3c/bench.log
timeout -k 10 120 python -u bench.py --gpus 2 > gpurun_out/r3c/bench2.log 2>&1
echo "gpus2 rc=$? (expected non-zero)"; tail -2 gpurun_out/r3c/bench2.log
exit 0
