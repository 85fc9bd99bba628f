# X6 split-bf16 K loop: numerics vs fp64, per-layer timing vs the f32 loop, bench with and without
set -o pipefail
mkdir -p gpurun_out/x6
timeout -k 10 300 python -u -m pytest tests/test_x6_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/x6/tests.log 2>&1
rc=$?; tail -3 gpurun_out/x6/tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/dev/bench_x6.py --out gpurun_out/x6/layers.jsonl > gpurun_out/x6/layers.log 2>&1 || exit $?
python -c "
import json
for l in open('gpurun_out/x6/layers.jsonl'):
    r=json.loads(l); print(r['layer'],r['pass'],r['f32_us'],r['x6_us'],r['speedup'],'%.2e %.2e'%(r['err_f32'],r['err_x6']),r['x6_cfg'])"
timeout -k 10 300 python -u bench.py --trials 0 --probe-trials 0 --no-serving > gpurun_out/x6/bench_x6.log 2>&1 || exit $?
tail -1 gpurun_out/x6/bench_x6.log | cut -c1-300
