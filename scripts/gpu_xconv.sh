# halo-tiled X6 conv: numerics, per-layer timing vs the implicit GEMM loops, bench with autotune log
set -o pipefail
mkdir -p gpurun_out/xc
timeout -k 10 300 python -u -m pytest tests/test_xconv_gpu.py tests/test_x6_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xc/tests.log 2>&1
rc=$?; tail -3 gpurun_out/xc/tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_x6.py --out gpurun_out/xc/layers.jsonl > gpurun_out/xc/layers.log 2>&1 || exit $?
python -c "
import json
for l in open('gpurun_out/xc/layers.jsonl'):
    r=json.loads(l); print(r['layer'],r['pass'],'f32',r['f32_us'],'x6',r['x6_us'],'xconv',r['xconv_us'],r['xconv_cfg'],r['err_xconv'])"
true

