cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5h
timeout -k 10 200 python -u scripts/dev/nobn_diag3.py 2 > gpurun_out/r5h/diag3.log 2>&1
echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/r5h/diag3.log | head -40 | cut -c1-400
timeout -k 10 300 python -u -m pytest tests/test_winograd4_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r5h/pytest.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/r5h/pytest.log
timeout -k 10 200 python -u scripts/dev/wino4_variants.py > gpurun_out/r5h/variants.jsonl 2>&1; cat gpurun_out/r5h/variants.jsonl
