"""Cost of the fused BatchNorm-statistics epilogue (fp64 atomic slots) in the VGG-small conv forwards.

For each layer's tuned forward config, times the same kernel with and without FLAG_STATS|FLAG_SATOM
(hipGraph-timed, host overhead excluded).  Usage: python scripts/dev/bench_stats_cost.py [--batch 256]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from rafiki_amd.ops import autotune
from rafiki_amd.ops import functional as F

ap = argparse.ArgumentParser()
ap.add_argument('--batch', type=int, default=256)
ap.add_argument('--reps', type=int, default=20)
args = ap.parse_args()
LAYERS = [(8, 64, 32), (64, 64, 32), (64, 128, 16), (128, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4),
          (512, 512, 4)]
B = args.batch
for li, (cin, cout, hw) in enumerate(LAYERS):
    x = torch.randn(B, hw, hw, cin, device='cuda').bfloat16()
    w = (torch.randn(cout, 9 * cin, device='cuda') * 0.05).bfloat16()
    acc = F.bn_acc_buffer(cout, 'cuda')
    y = torch.empty(B, hw, hw, cout, device='cuda', dtype=torch.bfloat16)
    F.conv_fwd(x, w, stats_acc=acc, out=y)  # tunes
    M, K = B * hw * hw, 9 * cin
    key = ('cf', M, cout, K, hw, hw, cin, 9, 'acc')
    cfg = autotune.lookup(key)
    flags_on = F.FLAG_STATS | F.FLAG_SATOM | ((acc.shape[0] - 1) << 12)
    res = {}
    for name, fl in (('stats', flags_on), ('plain', 0)):
        def run(_):
            if cfg[0] == 'h':
                F.hconv(0, x, w, y, M, cout, K, K, hw, hw, cin, stats=acc if fl else None, flags=fl, bn_bit=cfg[1],
                        grid=cfg[2])
            elif cfg[0] == 'k':
                return
            else:
                F.igemm(F.KIND_CONV_FWD, 0, x, w, y, M, cout, K, cin, K, cout, stats=acc if fl else None, H=hw, W=hw,
                        C=cin, taps=9, flags=fl, tile=cfg[0])
        res[name] = autotune._time_graph(None, run, args.reps) * 1e3
    print('c{} cfg={} stats {:6.1f} us  plain {:6.1f} us  (atomic epilogue {:+5.1f} us)'.format(
        li, cfg, res['stats'], res['plain'], res['stats'] - res['plain']), flush=True)
