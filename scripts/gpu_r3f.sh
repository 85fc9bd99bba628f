# Round-3 pass 4: new PG-GAN tests, PG-GAN bench, predictor QPS with 2 replicas, full GPU suite, bench
set -o pipefail
mkdir -p gpurun_out/r3f
timeout -k 10 300 python -u -m pytest tests/test_pg_gan_gpu.py -q -s -k "graphed_rounds or lrelu_gate or in_place or resampling" --timeout 150 --timeout-method thread > gpurun_out/r3f/tests.log 2>&1
rc=$?; grep -E "frob|passed|failed|Error" gpurun_out/r3f/tests.log | tail -6; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_pg_gan.py --lods 3,0 > gpurun_out/r3f/pg.log 2>&1 || exit $?
tail -1 gpurun_out/r3f/pg.log | cut -c300-700
timeout -k 10 400 python -u scripts/bench_predictor.py --replicas 2 --out gpurun_out/r3f/predictor_qps_2rep.json > gpurun_out/r3f/qps.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/r3f/predictor_qps_2rep.json'));print({k:d.get(k) for k in ('http_native','http_asyncio','batcher')})"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r3f/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3f/pytest_gpu.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
