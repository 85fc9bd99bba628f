# r4m: the x6s GEMM (fp32 operands split once per element in the workgroup): tests, x6s vs x6p sweep, step
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_x6p_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
X6S=1 timeout -k 10 200 python -u scripts/bench_x6p.py $O/x6s.jsonl > $O/b0.log 2>&1 || { tail -5 $O/b0.log; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r4m/x6s.jsonl'):
    d = json.loads(l)
    print(d['name'], d['best'], d['us'], d['pct_x6_peak'], sorted(d['all'].items(), key=lambda kv: kv[1])[:6])
PY
bash scripts/gpu_iter.sh r4m_it tests/test_winograd4_gpu.py tests/test_f32_gpu.py
