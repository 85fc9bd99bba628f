cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5i
timeout -k 10 400 python -u -m pytest tests/test_winograd4_gpu.py tests/test_f32_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5i/pytest.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/r5i/pytest.log
timeout -k 10 300 python -u scripts/dev/wino4_variants.py > gpurun_out/r5i/variants.jsonl 2>&1; cat gpurun_out/r5i/variants.jsonl
bash scripts/gpu_iter.sh r5i_it
