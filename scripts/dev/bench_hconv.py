"""Per-layer timing of the halo-tiled conv (rk_hconv) against the best implicit-GEMM config, for
the VGG-small layer shapes at batch 256 (forward with BN stats, and data-gradient).
usage: python scripts/dev/bench_hconv.py [--batch 256]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

from rafiki_amd.ops import autotune, functional as F

LAYERS = [(32, 64, 64), (16, 64, 128), (16, 128, 128), (8, 128, 256), (8, 256, 256), (4, 256, 512), (4, 512, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    a = ap.parse_args()
    dev = 'cuda'
    rows = []
    for hw, cin, cout in LAYERS:
        B = a.batch
        M, K = B * hw * hw, 9 * cin
        x = torch.randn(B, hw, hw, cin, device=dev).bfloat16()
        w = (torch.randn(cout, K, device=dev) * 0.02).bfloat16()
        y = torch.empty(B, hw, hw, cout, device=dev, dtype=torch.bfloat16)
        stats = torch.empty(M // 64 * 2, 2, cout, device=dev)
        dy = torch.randn(B, hw, hw, cout, device=dev).bfloat16()
        dx = torch.empty(B, hw, hw, cin, device=dev, dtype=torch.bfloat16)
        for kind in ('fwd', 'dgrad', 'wgrad'):
            if kind == 'wgrad':
                gw = torch.empty(cout, K, device=dev)
                cands = F._split_candidates(cout, K, M) + F._hconv_wgrad_candidates(B, hw, hw, cin, cout, 9)

                def run(cfg):
                    if cfg[0] == 'hw':
                        slab = torch.empty((cfg[1], cout, K), device=dev)
                        F.hconv_wgrad(dy, x, slab, cfg[1])
                        F.reduce_slabs(slab, gw)
                        return
                    t, s = cfg
                    slab = torch.empty((s, cout, K), device=dev)
                    F.igemm(F.KIND_CONV_WGRAD, 1, dy, x, slab, cout, K, M, cout, 0, K, H=hw, W=hw, C=cin, taps=9,
                            splits=s, slab_stride=cout * K, tile=t)
                    F.reduce_slabs(slab, gw)
                N, C = cout, cin
            elif False:
                pass
            elif kind == 'fwd':
                N, C = cout, cin
                cands = F._tile_candidates(M, N) + F._hconv_candidates(M, N, hw, hw, C, 9)

                def run(cfg):
                    if cfg[0] == 'h':
                        F.hconv(0, x, w, y, M, N, K, K, hw, hw, C, stats=stats, flags=F.FLAG_STATS, bn_bit=cfg[1],
                                grid=cfg[2])
                    else:
                        F.igemm(F.KIND_CONV_FWD, 0, x, w, y, M, N, K, C, K, N, stats=stats, H=hw, W=hw, C=C, taps=9,
                                flags=F.FLAG_STATS, tile=cfg[0])
            else:
                N, C = cin, cout
                cands = F._tile_candidates(M, N) + F._hconv_candidates(M, N, hw, hw, C, 9)

                def run(cfg):
                    if cfg[0] == 'h':
                        F.hconv(1, dy, w, dx, M, N, 9 * C, 9 * N, hw, hw, C, bn_bit=cfg[1], grid=cfg[2])
                    else:
                        F.igemm(F.KIND_CONV_DGRAD, 0, dy, w, dx, M, N, 9 * C, C, 9 * N, N, H=hw, W=hw, C=C, taps=9,
                                Cb=C, tile=cfg[0])
            times = {}
            for _ in range(2):
                for c in cands:
                    t = autotune._time_graph(c, run, 5) * 1e3
                    times[c] = min(times.get(c, 1e9), t)
            ig = min((t, c) for c, t in times.items() if c[0] not in ('h', 'hw'))
            hc = [(t, c) for c, t in times.items() if c[0] in ('h', 'hw')]
            hb = min(hc) if hc else (float('nan'), None)
            flops = 2.0 * M * cin * cout * 9
            r = {'layer': f'{hw}x{hw} {cin}->{cout}', 'kind': kind, 'igemm_us': round(ig[0], 2), 'igemm_cfg': ig[1],
                 'hconv_us': round(hb[0], 2), 'hconv_cfg': hb[1],
                 'igemm_tflops': round(flops / ig[0] / 1e6, 1),
                 'hconv_tflops': round(flops / hb[0] / 1e6, 1) if hc else None,
                 'all_h': {str(c): round(t, 2) for t, c in hc}}
            rows.append(r)
            print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
