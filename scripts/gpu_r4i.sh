# r4i: x6p epilogue on buffer stores (tests + sweep), then the headline step with a fresh tune + profile
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_x6p_gpu.py tests/test_head_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
X6P_CFGS="3,2,1;3,3,1;0,3,1;9,3,1;12,3,1;35,2,1;32,3,1;8,2,1" timeout -k 10 200 python -u scripts/bench_x6p.py \
  $O/x6p.jsonl > $O/b0.log 2>&1 || { tail -5 $O/b0.log; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r4i/x6p.jsonl'):
    d = json.loads(l)
    print(d['name'], d['best'], d['us'], d['pct_x6_peak'], sorted(d['all'].items(), key=lambda kv: kv[1]))
PY
bash scripts/gpu_iter.sh r4i_it
