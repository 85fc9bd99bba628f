"""Fused F(4x4) forward variants on the VGG-small 32x32 / 16x16 shapes: standard vs blocked weight sets
(variants 0/1 vs 3/4), BN-statistics epilogue; one JSON line per (shape, variant)."""
import json
import sys

import torch

sys.path.insert(0, '.')
from rafiki_amd.ops import f32 as S  # noqa: E402


def t(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for (N, H, Ci, Co) in [(256, 32, 64, 64), (256, 16, 64, 128), (256, 16, 128, 128), (256, 16, 128, 64),
                       (256, 8, 128, 256), (256, 8, 256, 256)]:
    x = torch.randn(N, H, H, Ci, device='cuda')
    w = torch.randn(Co, 9 * Ci, device='cuda') * (1.0 / (9 * Ci)) ** 0.5
    u, ub = S.wino4_u(w), S.wino4b_u(w)
    acc = torch.zeros((S.bn_slots(Co), 2, Co), dtype=torch.float64, device='cuda')
    ref = S.wino4_conv(x, u, variant=1)
    r = dict(N=N, H=H, Ci=Ci, Co=Co)
    for v in (0, 1, 3, 4, 5):
        uu = ub if v >= 3 else u
        r['v%d_us' % v] = round(t(lambda: S.wino4_conv(x, uu, stats=acc, variant=v, n_out=Co)), 1)
        y = S.wino4_conv(x, uu, variant=v, n_out=Co)
        r['v%d_diff' % v] = float((y - ref).abs().max())
    print(json.dumps(r), flush=True)

# weight gradient: variants 0 (32x32), 1 (64x32), 2 (32x32 software-pipelined), best split each
for (N, H, Ci, Co) in [(256, 32, 64, 64), (256, 16, 64, 128), (256, 16, 128, 128), (256, 8, 128, 256),
                       (256, 32, 8, 64)]:
    x = torch.randn(N, H, H, Ci, device='cuda')
    dy = torch.randn(N, H, H, Co, device='cuda')
    dw = torch.empty(Co, 9 * Ci, device='cuda')
    ref = torch.empty_like(dw)
    S.wino4_wgrad(dy, x, ref, splits=1, variant=0)
    r = dict(kind='wgrad', N=N, H=H, Ci=Ci, Co=Co)
    cands = S._wino4_wgrad_cands(N, H, H, Co, Ci)
    for v in (0, 1, 2):
        ts = {}
        for c in cands:
            if c[1] != v:
                continue
            ts[c[2]] = t(lambda: S.wino4_wgrad(dy, x, dw, splits=c[2], variant=v))
        if ts:
            sb = min(ts, key=ts.get)
            S.wino4_wgrad(dy, x, dw, splits=sb, variant=v)
            r['v%d_us' % v], r['v%d_splits' % v] = round(ts[sb], 1), sb
            r['v%d_rel' % v] = float((dw - ref).norm() / ref.norm())
    print(json.dumps(r), flush=True)
