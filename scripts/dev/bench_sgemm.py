"""Per-layer fp32 conv GEMM throughput of every sgemm config on the VGG-small shapes (batch 256).

usage: python scripts/dev/bench_sgemm.py [--layers 0,1,...] [--passes fwd,dgrad,wgrad] [--reps 10]
Prints one line per (layer, pass, config): microseconds and TFLOP/s (f32 MFMA peak 157.3).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from rafiki_amd.ops import f32 as S  # noqa: E402
from rafiki_amd.ops.graphs import capture  # noqa: E402

LAYERS = [(4, 64, 32), (64, 64, 32), (64, 128, 16), (128, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4),
          (512, 512, 4)]


def time_fn(fn, reps):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with capture(g):
        for _ in range(reps):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / (2 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--layers', default='0,1,2,3,4,5,6,7')
    ap.add_argument('--passes', default='fwd,dgrad,wgrad')
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--batch', type=int, default=256)
    a = ap.parse_args()
    B = a.batch
    dev = 'cuda'
    for li in [int(v) for v in a.layers.split(',')]:
        cin, cout, hw = LAYERS[li]
        M = B * hw * hw
        x = torch.randn(B, hw, hw, cin, device=dev)
        w = torch.randn(cout, 3, 3, cin, device=dev) * 0.05
        dy = torch.randn(B, hw, hw, cout, device=dev)
        wt = torch.randn(cin, 9 * cout, device=dev) * 0.05
        flop = 2.0 * M * cout * 9 * cin
        for pas in a.passes.split(','):
            if pas == 'dgrad' and li == 0:
                continue
            res = []
            if pas == 'fwd':
                y = torch.empty(B, hw, hw, cout, device=dev)
                for cfg in S._cands(M, cout, big=cin % 32 == 0):
                    fn = lambda cfg=cfg: S.sgemm(S.KIND_CONV, x, w, y, M, cout, 9 * cin, cin, 9 * cin, cout,
                                                 tile=cfg[0], nst=cfg[1], H=hw, W=hw, C=cin, taps=9)
                    res.append((cfg, time_fn(fn, a.reps)))
            elif pas == 'dgrad':
                dx = torch.empty(B, hw, hw, cin, device=dev)
                for cfg in S._cands(M, cin, big=True):
                    fn = lambda cfg=cfg: S.sgemm(S.KIND_CONV, dy, wt, dx, M, cin, 9 * cout, cout, 9 * cout, cin,
                                                 tile=cfg[0], nst=cfg[1], H=hw, W=hw, C=cout, taps=9)
                    res.append((cfg, time_fn(fn, a.reps)))
            else:
                N = 9 * cin
                out = torch.empty(cout, N, device=dev)
                for cfg in S._cands(cout, N, splittable=True, K=M, big=True):
                    tile, nst, s = cfg
                    slab = torch.empty(max(1, s), cout, N, device=dev)

                    def fn(tile=tile, nst=nst, s=s, slab=slab):
                        if s == 1:
                            S.sgemm(S.KIND_WGRAD, dy, x, out, cout, N, M, cout, cin, N, tile=tile, nst=nst, H=hw,
                                    W=hw, C=cin, taps=9)
                        else:
                            S.sgemm(S.KIND_WGRAD, dy, x, slab, cout, N, M, cout, cin, N, tile=tile, nst=nst,
                                    splits=s, slab_stride=cout * N, H=hw, W=hw, C=cin, taps=9)
                            S.reduce_slabs(slab, out)
                    res.append((cfg, time_fn(fn, a.reps)))
            res.sort(key=lambda r: r[1])
            for cfg, us in res[:6]:
                print('L{} {:6s} cin={:3d} cout={:3d} hw={:2d} cfg={} {:8.1f} us {:6.1f} TF'.format(
                    li, pas, cin, cout, hw, cfg, us, flop / us / 1e6), flush=True)


if __name__ == '__main__':
    main()
