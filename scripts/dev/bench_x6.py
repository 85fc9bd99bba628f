"""Per-layer best config of the f32-MFMA K loop vs the X6 split-bf16 K loop (sgemm.hip) on the
VGG-small conv shapes (batch 256: forward, data gradient, weight gradient) and the pre-transformed
Winograd batched GEMM shapes, with each loop's error against an fp64 reference on the same data.

usage: python scripts/dev/bench_x6.py [--layers 0,...,7] [--out file.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as TF  # noqa: E402

from rafiki_amd.ops import f32 as S  # noqa: E402
from scripts.bench_sgemm import LAYERS, time_fn  # noqa: E402


def rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


def best(cands, make, reps):
    res = []
    for cfg in cands:
        try:
            res.append((time_fn(make(cfg), reps), cfg))
        except Exception as e:  # noqa: BLE001
            print('  cfg', cfg, 'failed:', e, flush=True)
    res.sort()
    return res[0] if res else (float('inf'), None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--layers', default='0,1,2,3,4,5,6,7')
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--out', default='')
    a = ap.parse_args()
    B, dev = a.batch, 'cuda'
    fout = open(a.out, 'a') if a.out else None
    for li in [int(v) for v in a.layers.split(',')]:
        cin, cout, hw = LAYERS[li]
        if cin % 8:
            cin = 8
        M = B * hw * hw
        x = torch.randn(B, hw, hw, cin, device=dev)
        w = torch.randn(cout, 3, 3, cin, device=dev) / (3 * cin ** 0.5)
        dy = torch.randn(B, hw, hw, cout, device=dev)
        wt = torch.randn(cin, 9 * cout, device=dev) / (3 * cout ** 0.5)
        flop = 2.0 * M * cout * 9 * cin
        for pas in ('fwd', 'dgrad', 'wgrad'):
            if pas == 'dgrad' and li == 0:
                continue
            if pas == 'fwd':
                y = torch.empty(B, hw, hw, cout, device=dev)
                cands = S._cands(M, cout, big=cin % 32 == 0)

                def make(cfg):
                    return lambda: S.sgemm(S.KIND_CONV, x, w, y, M, cout, 9 * cin, cin, 9 * cin, cout, tile=cfg[0],
                                           nst=cfg[1], H=hw, W=hw, C=cin, taps=9)
                out = y
            elif pas == 'dgrad':
                dx = torch.empty(B, hw, hw, cin, device=dev)
                cands = S._cands(M, cin, big=cout % 32 == 0)

                def make(cfg):
                    return lambda: S.sgemm(S.KIND_CONV, dy, wt, dx, M, cin, 9 * cout, cout, 9 * cout, cin,
                                           tile=cfg[0], nst=cfg[1], H=hw, W=hw, C=cout, taps=9)
                out = dx
            else:
                N = 9 * cin
                ow = torch.empty(cout, N, device=dev)
                cands = S._cands(cout, N, splittable=True, K=M, big=True)
                slabs = {}

                def make(cfg):
                    tile, nst, s = cfg
                    if s > 1 and s not in slabs:
                        slabs[s] = torch.empty(s, cout, N, device=dev)

                    def fn():
                        if s == 1:
                            S.sgemm(S.KIND_WGRAD, dy, x, ow, cout, N, M, cout, cin, N, tile=tile, nst=nst, H=hw, W=hw,
                                    C=cin, taps=9)
                        else:
                            S.sgemm(S.KIND_WGRAD, dy, x, slabs[s], cout, N, M, cout, cin, N, tile=tile, nst=nst,
                                    splits=s, slab_stride=cout * N, H=hw, W=hw, C=cin, taps=9)
                            S.reduce_slabs(slabs[s], ow)
                    return fn
                out = ow
            c32 = [c for c in cands if c[0] < S.X6]
            c6 = [c for c in cands if c[0] >= S.X6]
            t32, cfg32 = best(c32, make, a.reps)
            make(cfg32)()
            torch.cuda.synchronize()
            r32 = out.clone()
            t6, cfg6 = best(c6, make, a.reps)
            make(cfg6)()
            torch.cuda.synchronize()
            r6 = out.clone()
            # fp64 reference of the op
            if pas == 'fwd':
                ref = TF.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), padding=1)
                ref = ref.permute(0, 2, 3, 1)
            elif pas == 'dgrad':
                w2 = wt.double().reshape(cin, 3, 3, cout).permute(0, 3, 1, 2)
                ref = TF.conv2d(dy.double().permute(0, 3, 1, 2), w2, padding=1).permute(0, 2, 3, 1)
            else:
                xd = x.double().permute(0, 3, 1, 2)
                wz = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, device=dev, requires_grad=True)
                (gw,) = torch.autograd.grad(TF.conv2d(xd, wz, padding=1), wz, dy.double().permute(0, 3, 1, 2))
                ref = gw.permute(0, 2, 3, 1).reshape(cout, 9 * cin)
            # halo-tiled X6 conv (fwd / dgrad)
            tx, cfgx, ex = float('inf'), None, None
            if pas != 'wgrad' and S.xconv_ok(hw, hw, cin if pas == 'fwd' else cout, cout if pas == 'fwd' else cin, M, True):
                if pas == 'fwd':
                    planes = S.xconv_planes(w)
                    xin, oshape = x, (B, hw, hw, cout)
                else:
                    wfull = wt.reshape(cin, 3, 3, cout).permute(3, 1, 2, 0).flip(1, 2).contiguous()  # [cout][3][3][cin]
                    planes = S.xconv_planes(wfull, dgrad=True)
                    xin, oshape = dy, (B, hw, hw, cin)
                ox = torch.empty(oshape, device=dev)
                xc = S._xconv_cands(hw, hw, xin.shape[-1], oshape[-1], M, True)
                tx, cfgx = best(xc, lambda cfg: (lambda: S.xconv(xin, planes, cfg=S.XCONV - cfg[0], out=ox)), a.reps)
                if cfgx is not None:
                    S.xconv(xin, planes, cfg=S.XCONV - cfgx[0], out=ox)
                    torch.cuda.synchronize()
                    ex = rel(ox, ref)
            rec = {'layer': li, 'pass': pas, 'cin': cin, 'cout': cout, 'hw': hw,
                   'f32_us': round(t32, 2), 'f32_cfg': cfg32, 'f32_tflops': round(flop / t32 / 1e6, 1),
                   'x6_us': round(t6, 2), 'x6_cfg': cfg6, 'x6_tflops': round(flop / t6 / 1e6, 1),
                   'speedup': round(t32 / t6, 3), 'err_f32': rel(r32, ref), 'err_x6': rel(r6, ref),
                   'xconv_us': round(tx, 2), 'xconv_cfg': cfgx, 'err_xconv': ex,
                   'xconv_tflops': round(flop / tx / 1e6, 1) if tx < float('inf') else None}
            print(json.dumps(rec), flush=True)
            if fout:
                fout.write(json.dumps(rec) + '\n')
                fout.flush()


if __name__ == '__main__':
    main()
