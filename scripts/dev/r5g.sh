cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5g
timeout -k 10 200 python -u scripts/dev/nobn_diag3.py > gpurun_out/r5g/diag3.log 2>&1
echo "diag rc=$?"; cat gpurun_out/r5g/diag3.log | grep -v amdgpu.ids | head -40
timeout -k 10 500 python -u -m pytest tests/test_winograd4_gpu.py tests/test_f32_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5g/pytest.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/r5g/pytest.log
bash scripts/gpu_iter.sh r5g_it
