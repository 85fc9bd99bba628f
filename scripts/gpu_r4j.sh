# r4j: serving tests + predictor QPS (1 and 2 replicas) with pre-captured staged graphs; PG-GAN per-kernel +
# counter profiles (incl. HBM fetch/write) at LOD 3 and LOD 0
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/bench_predictor.py --replicas 1 --out $O/qps_1rep.json > $O/qps1.log 2>&1 || { tail -5 $O/qps1.log; exit 1; }
timeout -k 10 400 python3 -u scripts/bench_predictor.py --replicas 2 --skip-http-asyncio --out $O/qps_2rep.json > $O/qps2.log 2>&1 || { tail -5 $O/qps2.log; exit 1; }
python3 -c "
import json
for f in ('qps_1rep', 'qps_2rep'):
    d = json.load(open('gpurun_out/r4j/%s.json' % f))
    print(f, json.dumps(d.get('http_native')), json.dumps(d.get('http_asyncio', {}).get('npy_batch128_8clients')))
"
timeout -k 10 700 bash scripts/gpu_pggan_prof.sh 3 6 > $O/pg3.log 2>&1 || { tail -5 $O/pg3.log; exit 1; }
tail -4 $O/pg3.log
timeout -k 10 900 bash scripts/gpu_pggan_prof.sh 0 4 > $O/pg0.log 2>&1 || { tail -5 $O/pg0.log; exit 1; }
tail -4 $O/pg0.log
