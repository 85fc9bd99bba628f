"""Run one igemm configuration N times (for rocprofv3 counter collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from rafiki_amd.ops import functional as F
layer, pas, tile, reps = int(sys.argv[1]), sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 10
# tile: igemm tile code (int) or 'h<bn_bit>g<grid>' for the halo conv (rk_hconv)
hcfg = (int(tile[1]), int(tile[3:])) if tile.startswith('h') else None
tile = 0 if hcfg else int(tile)
LAYERS = [(8, 64, 32), (64, 64, 32), (64, 128, 16), (128, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4)]
cin, cout, hw = LAYERS[layer]
B = 256
x = torch.randn(B, hw, hw, cin, device='cuda').bfloat16()
w = (torch.randn(cout, 3, 3, cin, device='cuda') * 0.05).bfloat16()
dy = torch.randn(B, hw, hw, cout, device='cuda').bfloat16()
M = B * hw * hw
for _ in range(reps):
    if pas == 'fwd':
        y = torch.empty(B, hw, hw, cout, device='cuda', dtype=torch.bfloat16)
        if hcfg:
            F.hconv(0, x, w, y, M, cout, 9 * cin, 9 * cin, hw, hw, cin, bn_bit=hcfg[0], grid=hcfg[1])
        else:
            F.igemm(F.KIND_CONV_FWD, 0, x, w, y, M, cout, 9 * cin, cin, 9 * cin, cout, H=hw, W=hw, C=cin, taps=9, tile=tile)
    elif pas == 'dgrad':
        dx = torch.empty(B, hw, hw, cin, device='cuda', dtype=torch.bfloat16)
        if hcfg:
            F.hconv(1, dy, w, dx, M, cin, 9 * cout, 9 * cin, hw, hw, cout, bn_bit=hcfg[0], grid=hcfg[1])
        else:
            F.igemm(F.KIND_CONV_DGRAD, 0, dy, w, dx, M, cin, 9 * cout, cout, 9 * cin, cin, H=hw, W=hw, C=cout, taps=9, Cb=cout, tile=tile)
    else:
        s = 8
        slab = torch.empty((s, cout, 9 * cin), device='cuda')
        F.igemm(F.KIND_CONV_WGRAD, 1, dy, x, slab, cout, 9 * cin, M, cout, 0, 9 * cin, H=hw, W=hw, C=cin, taps=9, splits=s, slab_stride=cout * 9 * cin, tile=tile)
torch.cuda.synchronize()
print('done')
