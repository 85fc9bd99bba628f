"""Normalise-on-load cost: the fused F(4x4) forward variants 3-5 (flags = stats) with and without the BN
prologue, and the F(4x4) wgrad variants with and without xpro, on the VGG-small batch-256 layer shapes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from rafiki_amd.ops import f32 as S  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


out = []
for N, H, C, Co in ((256, 32, 64, 64), (256, 16, 128, 128), (256, 8, 256, 256), (256, 4, 512, 512)):
    y = torch.randn(N, H, H, C, device='cuda')
    co = torch.stack([y.mean((0, 1, 2)), torch.ones(C, device='cuda'), torch.rand(C, device='cuda') + 0.5,
                      torch.randn(C, device='cuda') * 0.2]).contiguous()
    w = torch.randn(Co, 9 * C, device='cuda') * 0.05
    u = S.wino4b_u(w)
    acc = torch.zeros((S.bn_slots(Co), 2, Co), dtype=torch.float64, device='cuda')
    o = torch.empty(N, H, H, Co, device='cuda')
    for v in (3, 4, 5):
        t0 = timeit(lambda: S.wino4_conv(y, u, out=o, stats=acc, variant=v, n_out=Co))
        t1 = timeit(lambda: S.wino4_conv(y, u, out=o, stats=acc, variant=v, n_out=Co, pro=co))
        r = dict(op='fwd', shape=[N, H, C, Co], variant=v, us=round(t0, 1), us_pro=round(t1, 1))
        print(json.dumps(r), flush=True)
        out.append(r)
    dy = torch.randn(N, H, H, Co, device='cuda')
    g = torch.empty(Co, 9 * C, device='cuda')
    for _, v, s in S._wino4_wgrad_cands(N, H, H, Co, C):
        t0 = timeit(lambda: S.wino4_wgrad(dy, y, g, splits=s, variant=v))
        t1 = timeit(lambda: S.wino4_wgrad(dy, y, g, splits=s, variant=v, xpro=co))
        r = dict(op='wgrad', shape=[N, H, C, Co], variant=v, splits=s, us=round(t0, 1), us_pro=round(t1, 1))
        print(json.dumps(r), flush=True)
        out.append(r)
