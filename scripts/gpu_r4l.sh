# r4l: tile-major Y' for the plane GEMM + output transform: tests, then the step (fresh tune) + profile
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_x6p_gpu.py tests/test_winograd4_gpu.py tests/test_f32_gpu.py -x -q \
  --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_iter.sh r4l_it
