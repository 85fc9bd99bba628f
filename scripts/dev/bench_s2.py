"""Throughput of the stride-2 gather convolutions (S2 / S2T / S2W) and the 3x3 conv at the PG-GAN
shapes (fmap 512, 32x32 -> 16x16, batch 128 = real + fake D batch).  Prints TFLOP/s per config."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from rafiki_amd.ops import f32 as S  # noqa: E402
from rafiki_amd.ops.graphs import capture  # noqa: E402


def time_fn(fn, reps=5):
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
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shapes', default='128,32,512,512;128,16,512,512;64,32,256,512')
    a = ap.parse_args()
    dev = 'cuda'
    for sh in a.shapes.split(';'):
        N, H, Ci, Co = [int(v) for v in sh.split(',')]
        x = torch.randn(N, H, H, Ci, device=dev)
        W = torch.randn(Co, 16 * Ci, device=dev) * 0.02
        g = torch.randn(N, H // 2, H // 2, Co, device=dev)
        w3 = torch.randn(Co, 9 * Ci, device=dev) * 0.02
        fl_s2 = 2.0 * N * (H // 2) ** 2 * Co * 16 * Ci
        fl_3 = 2.0 * N * H * H * Co * 9 * Ci
        rows = [('s2 fwd', lambda: S.s2_conv(x, W), fl_s2),
                ('s2t (adjoint)', lambda: S.s2t_conv(g, W), fl_s2 / 4),   # 4 of 16 taps per output pixel
                ('s2 wgrad', lambda: S.s2_wgrad(x, g), fl_s2),
                ('conv3x3 fwd', lambda: S.conv_fwd(x, w3), fl_3)]
        for name, fn, fl in rows:
            us = time_fn(fn)
            print('N={} H={} Ci={} Co={} {:14s} {:9.1f} us {:6.1f} TF'.format(N, H, Ci, Co, name, us, fl / us / 1e6),
                  flush=True)


if __name__ == '__main__':
    main()
