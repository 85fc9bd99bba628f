# r4e: new-kernel tests (head / x6p / native LSTM / serving), the x6p GEMM sweep, then the headline step
# with a fresh tune + its per-kernel profile
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_x6p_gpu.py tests/test_head_gpu.py tests/test_lstm_native_gpu.py \
  tests/test_serving_gpu.py tests/test_winograd4_gpu.py tests/test_pg_gan_gpu.py tests/test_f32_gpu.py \
  -x -q -s --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_x6p.py $O/x6p.jsonl > $O/b0.log 2>&1 || { tail -5 $O/b0.log; exit 1; }
bash scripts/gpu_iter.sh r4e_it
