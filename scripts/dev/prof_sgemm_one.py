"""Run one fp32 conv GEMM config N times (rocprofv3 counter collection / wall timing).

usage: python scripts/dev/prof_sgemm_one.py <layer> <fwd|dgrad|wgrad> <tile> <nst> [splits] [reps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from rafiki_amd.ops import f32 as S  # noqa: E402

LAYERS = [(4, 64, 32), (64, 64, 32), (64, 128, 16), (128, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4),
          (512, 512, 4)]
li, pas, tile, nst = int(sys.argv[1]), sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
splits = int(sys.argv[5]) if len(sys.argv) > 5 else 1
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
cin, cout, hw = LAYERS[li]
B = 256
M = B * hw * hw
x = torch.randn(B, hw, hw, cin, device='cuda')
w = torch.randn(cout, 3, 3, cin, device='cuda') * 0.05
dy = torch.randn(B, hw, hw, cout, device='cuda')
wt = torch.randn(cin, 9 * cout, device='cuda') * 0.05
out_f = torch.empty(B, hw, hw, cout, device='cuda')
out_d = torch.empty(B, hw, hw, cin, device='cuda')
N = 9 * cin
slab = torch.empty(splits, cout, N, device='cuda')


def run():
    if pas == 'fwd':
        S.sgemm(S.KIND_CONV, x, w, out_f, M, cout, 9 * cin, cin, 9 * cin, cout, tile=tile, nst=nst, H=hw, W=hw, C=cin,
                taps=9)
    elif pas == 'dgrad':
        S.sgemm(S.KIND_CONV, dy, wt, out_d, M, cin, 9 * cout, cout, 9 * cout, cin, tile=tile, nst=nst, H=hw, W=hw,
                C=cout, taps=9)
    else:
        S.sgemm(S.KIND_WGRAD, dy, x, slab, cout, N, M, cout, cin, N, tile=tile, nst=nst, splits=splits,
                slab_stride=cout * N, H=hw, W=hw, C=cin, taps=9)


run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    run()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print('L{} {} tile={} nst={} s={}: {:.1f} us  {:.1f} TF'.format(li, pas, tile, nst, splits, dt * 1e6,
                                                               2.0 * M * cout * 9 * cin / dt / 1e12))
