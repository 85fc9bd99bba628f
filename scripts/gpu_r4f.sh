# r4f: the gather_batch fix (serving / engine tests) and the warp-specialised x6p tiles, then x6p supply
# diagnostics: the new tiles, operands shared by all groups (L2-resident), no-DMA and no-MFMA timing builds
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_x6p_gpu.py tests/test_engine_gpu.py tests/test_head_gpu.py \
  -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
W="9,2,1;9,3,1;10,2,1;10,3,1;11,2,1;11,3,1;12,2,1;12,3,1;9,3,2;9,3,4;10,3,2;11,3,2;26,2,1;28,2,1;3,2,1;0,3,1;8,2,1"
X6P_CFGS="$W" timeout -k 10 200 python -u scripts/bench_x6p.py $O/x6p_ws.jsonl > $O/b0.log 2>&1 || exit 1
X6P_CFGS="3,2,1;0,3,1;8,2,1;9,3,1;12,3,1" X6P_SHARED=1 timeout -k 10 200 python -u scripts/bench_x6p.py \
  $O/x6p_shared.jsonl > $O/b1.log 2>&1 || exit 1
for d in 1 2; do
  X6P_CFGS="3,2,1;3,3,1;0,2,1;0,3,1" RAFIKI_X6P_DBG=$d timeout -k 10 200 python -u scripts/bench_x6p.py \
    $O/x6p_dbg$d.jsonl > $O/b$((d+1)).log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for f in ('x6p_ws', 'x6p_shared', 'x6p_dbg1', 'x6p_dbg2'):
    for l in open('gpurun_out/r4f/%s.jsonl' % f):
        d = json.loads(l)
        print(f, d['name'], d['best'], d['us'], d['pct_x6_peak'], {k: v for k, v in sorted(d['all'].items(), key=lambda kv: kv[1])[:6]})
PY
timeout -k 10 600 python -u -m pytest tests/test_serving_gpu.py -q --timeout 150 --timeout-method thread \
  > $O/pytest_serving.log 2>&1
rc=$?; echo "serving rc=$rc"; tail -3 $O/pytest_serving.log
echo r4f-done
