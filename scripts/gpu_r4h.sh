# x6p per-block phase stamps (RAFIKI_X6P_DBG=4): prologue / K loop / epilogue cycles, clock, concurrency
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
X6P_SHAPES=c5f,c7f,c5w X6P_CFGS="3,2,1;3,3,1;0,2,1;0,3,1" RAFIKI_X6P_DBG=4 timeout -k 10 200 \
  python -u scripts/bench_x6p.py $O/stamps.jsonl > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r4h/stamps.jsonl'):
    d = json.loads(l)
    print(d['name'], d['M'], d['N'], d['K'], d['all'])
    for k, v in d.get('phases', {}).items():
        print('  ', k, {a: round(b, 1) for a, b in v.items()})
PY
