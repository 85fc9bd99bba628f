cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5f
RAFIKI_TUNE_CACHE=off timeout -k 10 200 python -u scripts/dev/nobn_diag2.py > gpurun_out/r5f/diag2.log 2>&1
echo "diag rc=$?"; tail -2 gpurun_out/r5f/diag2.log | cut -c1-600
timeout -k 10 400 python -u -m pytest tests/test_winograd4_gpu.py tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5f/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r5f/pytest.log
timeout -k 10 200 python -u scripts/dev/wino4_variants.py > gpurun_out/r5f/variants.jsonl 2>&1 && cat gpurun_out/r5f/variants.jsonl
