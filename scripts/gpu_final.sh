# final check at HEAD: full GPU suite + smoke + bench --gpus 1
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/final/pytest_gpu.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/final/bench.log 2>&1 || exit $?
tail -1 gpurun_out/final/bench.log | cut -c1-300
