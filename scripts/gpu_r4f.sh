# r4f: the gather_batch fix (serving / engine tests), then x6p supply diagnostics: operands shared by all
# groups (L2-resident), no-DMA and no-MFMA timing builds
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_serving_gpu.py tests/test_x6p_gpu.py \
  -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
C="3,2,1;3,3,1;0,2,1;0,3,1;8,2,1;7,2,1;19,2,1"
X6P_CFGS="$C" X6P_SHARED=1 timeout -k 10 200 python -u scripts/bench_x6p.py $O/x6p_shared.jsonl > $O/b1.log 2>&1 || exit 1
for d in 1 2; do
  X6P_CFGS="3,2,1;3,3,1;0,2,1;0,3,1" RAFIKI_X6P_DBG=$d timeout -k 10 200 python -u scripts/bench_x6p.py \
    $O/x6p_dbg$d.jsonl > $O/b$((d+1)).log 2>&1 || exit 1
done
echo r4f-done
