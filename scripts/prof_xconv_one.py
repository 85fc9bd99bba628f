"""One VGG-small conv shape through the halo-tiled X6 conv (each cfg) and the Winograd F(4x4) forward,
a few launches each, for rocprofv3 counter passes.  usage: prof_xconv_one.py [layer]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rafiki_amd.ops import f32 as S  # noqa: E402
from scripts.bench_sgemm import LAYERS  # noqa: E402

li = int(sys.argv[1]) if len(sys.argv) > 1 else 1
cin, cout, hw = LAYERS[li]
B = 256
x = torch.randn(B, hw, hw, cin, device='cuda')
w = torch.randn(cout, 3, 3, cin, device='cuda') * 0.05
planes = S.xconv_planes(w)
u4 = S.wino4_u(w.reshape(cout, 9 * cin))
y = torch.empty(B, hw, hw, cout, device='cuda')
for cfg in [c[0] for c in S._xconv_cands(hw, hw, cin, cout, B * hw * hw)]:
    for _ in range(3):
        S.xconv(x, planes, cfg=S.XCONV - cfg, out=y)
for _ in range(3):
    S.wino4_conv(x, u4, out=y, variant=0)
torch.cuda.synchronize()
print('done')
