# x6p: tests incl. the persistent tiles, per-block phase stamps (RAFIKI_X6P_DBG=4) of tiles 0 / 3, then the
# persistent tiles against the best so far
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_x6p_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
X6P_SHAPES=c5f,c7f,c5w X6P_CFGS="3,2,1;3,3,1;0,2,1;0,3,1" RAFIKI_X6P_DBG=4 timeout -k 10 200 \
  python -u scripts/bench_x6p.py $O/stamps.jsonl > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
P="32,2,1;32,3,1;33,2,1;33,3,1;34,2,1;34,3,1;35,2,1;35,3,1;32,3,2;33,3,2;34,3,2;35,3,2;48,2,1;49,2,1;51,2,1;51,3,1;3,2,1;12,3,1;9,3,1"
X6P_CFGS="$P" timeout -k 10 300 python -u scripts/bench_x6p.py $O/pers.jsonl > $O/b2.log 2>&1 || { tail -20 $O/b2.log; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r4h/stamps.jsonl'):
    d = json.loads(l)
    print(d['name'], d['M'], d['N'], d['K'], d['all'])
    for k, v in d.get('phases', {}).items():
        print('  ', k, {a: round(b, 1) for a, b in v.items()})
for l in open('gpurun_out/r4h/pers.jsonl'):
    d = json.loads(l)
    print(d['name'], d['best'], d['us'], d['pct_x6_peak'], sorted(d['all'].items(), key=lambda kv: kv[1])[:8])
PY
