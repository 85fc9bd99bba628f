"""Per-layer microbenchmark of the igemm kernels (VGG-small shapes, batch 256) for every tile.

Prints TFLOP/s per (layer, pass, tile, splits) so tile heuristics and kernel changes can be judged
on the real shapes.  Usage: python scripts/dev/bench_igemm.py [--batch 256] [--reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from rafiki_amd.ops import functional as F

ap = argparse.ArgumentParser()
ap.add_argument('--batch', type=int, default=256)
ap.add_argument('--reps', type=int, default=20)
ap.add_argument('--passes', default='fwd,dgrad,wgrad')
ap.add_argument('--variants', default='0,1,2,3,32,33,34,35,64,65,66,67')
ap.add_argument('--layers', default='0,1,2,3,4,5,6,7')
ap.add_argument('--satom', action='store_true', help='forward statistics as fp64 atomic slots (training path; '
                'required by the wave-K-split tiles 68/36)')
args = ap.parse_args()
VARIANTS = [int(v) for v in args.variants.split(',')]

LAYERS = [(8, 64, 32), (64, 64, 32), (64, 128, 16), (128, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4),
          (512, 512, 4)]
dev = 'cuda'
B = args.batch


def timeit(fn):
    """GPU time per launch, measured on a captured hipGraph (no host launch overhead)."""
    from rafiki_amd.ops import autotune
    return autotune._time_graph(None, lambda _: fn(), args.reps) * 1e3  # us


best_total = 0.0
for li, (cin, cout, hw) in enumerate(LAYERS):
    if str(li) not in args.layers.split(','):
        continue
    x = torch.randn(B, hw, hw, cin, device=dev).bfloat16()
    w = (torch.randn(cout, 3, 3, cin, device=dev) * 0.05).bfloat16()
    dy = torch.randn(B, hw, hw, cout, device=dev).bfloat16()
    M = B * hw * hw
    flops = 2.0 * M * cout * 9 * cin
    y = torch.empty(B, hw, hw, cout, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(B, hw, hw, cin, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(cout, 9 * cin, device=dev)
    line = []
    if 'fwd' in args.passes:
        res = {}
        for t in VARIANTS:
            if args.satom:
                stats = F.bn_acc_buffer(cout, dev)
                fl = F.FLAG_STATS | F.FLAG_SATOM | ((stats.shape[0] - 1) << 12)
            else:
                stats = torch.empty((F.stats_rows(M, cout, t), 2, cout), device=dev)
                fl = F.FLAG_STATS
            res[t] = timeit(lambda: F.igemm(F.KIND_CONV_FWD, 0, x, w, y, M, cout, 9 * cin, cin, 9 * cin, cout,
                                            stats=stats, H=hw, W=hw, C=cin, taps=9, flags=fl, tile=t))
        b = min(res, key=res.get)
        best_total += res[b]
        print('c{} fwd   M={:6d} N={:4d} K={:5d} '.format(li, M, cout, 9 * cin) +
              ' '.join('t{}:{:6.1f}us/{:5.0f}TF'.format(t, v, flops / v / 1e6) for t, v in res.items()) +
              '  heur=t{}'.format(F.pick_tile(M, cout)))
    if 'dgrad' in args.passes and li > 0:
        res = {}
        for t in VARIANTS:
            res[t] = timeit(lambda: F.igemm(F.KIND_CONV_DGRAD, 0, dy, w, dx, M, cin, 9 * cout, cout, 9 * cin, cin,
                                            H=hw, W=hw, C=cout, taps=9, Cb=cout, tile=t))
        b = min(res, key=res.get)
        best_total += res[b]
        print('c{} dgrad M={:6d} N={:4d} K={:5d} '.format(li, M, cin, 9 * cout) +
              ' '.join('t{}:{:6.1f}us/{:5.0f}TF'.format(t, v, flops / v / 1e6) for t, v in res.items()) +
              '  heur=t{}'.format(F.pick_tile(M, cin)))
    if 'wgrad' in args.passes:
        res = {}
        Mw, Nw, Kw = cout, 9 * cin, M
        for t in VARIANTS:
            for s in (2, 4, 8, 16, 32):
                slab = torch.empty((s, Mw, Nw), device=dev)

                def run():
                    F.igemm(F.KIND_CONV_WGRAD, 1, dy, x, slab, Mw, Nw, Kw, cout, 0, Nw, H=hw, W=hw, C=cin, taps=9,
                            splits=s, slab_stride=Mw * Nw, tile=t)
                    F.reduce_slabs(slab, dw)
                res[(t, s)] = timeit(run)
        b = min(res, key=res.get)
        best_total += res[b]
        top = sorted(res.items(), key=lambda kv: kv[1])[:4]
        print('c{} wgrad M={:4d} N={:5d} K={:6d} '.format(li, Mw, Nw, Kw) +
              ' '.join('t{}s{}:{:6.1f}us/{:5.0f}TF'.format(k[0], k[1], v, flops / v / 1e6) for k, v in top))
print('sum of best per-pass times: {:.1f} us'.format(best_total))
