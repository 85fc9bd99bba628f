"""F(4x4,3x3) vs F(2x2,3x3) fused Winograd fp32 convs on the VGG-small layer shapes (batch 256, BN
statistics epilogue), with each kernel's relative error against an fp64 reference on a slice.
usage: python scripts/dev/bench_winograd4.py [out.jsonl]"""
import json
import sys

sys.path.insert(0, '.')
import torch  # noqa: E402
import torch.nn.functional as TF  # noqa: E402

from rafiki_amd.ops import _lib, f32 as S  # noqa: E402

_lib.lib()


def t(fn, reps=20):
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


res = []
for (N, H, C, K) in [(256, 32, 64, 64), (256, 16, 64, 128), (256, 16, 128, 128), (256, 8, 128, 256),
                     (256, 8, 256, 256), (256, 4, 256, 512), (256, 4, 512, 512)]:
    x = torch.randn(N, H, H, C, device='cuda')
    w = torch.randn(K, 9 * C, device='cuda') * (1.0 / (9 * C)) ** 0.5
    u = torch.empty(16, K, C, device='cuda')
    ut = torch.empty(16, C, K, device='cuda')
    S.wino_weights(w, u, ut)
    u4 = S.wino4_u(w)
    acc = torch.zeros((S.bn_slots(K), 2, K), dtype=torch.float64, device='cuda')
    r = dict(N=N, H=H, C=C, K=K)
    for v in (0, 1, 2, 3, 4, 5):
        r['w2_v%d_us' % v] = round(t(lambda: S.wino_conv(x, u, stats=acc, variant=v)), 1)
    for v in (0, 1, 2):
        r['w4_v%d_us' % v] = round(t(lambda: S.wino4_conv(x, u4, stats=acc, variant=v)), 1)
    r['wt2_us'] = round(t(lambda: S.wino_weights(w, u, ut)), 1)
    r['wt4_us'] = round(t(lambda: S.wino4_u(w)), 1)
    dy = torch.randn(N, H, H, K, device='cuda')
    dw = torch.empty(K, 9 * C, device='cuda')
    tw = {c[2]: t(lambda: S.wino_wgrad(dy, x, dw, splits=c[2])) for c in S._wino_wgrad_cands(N, H, H, K, C)}
    if tw:
        sb = min(tw, key=tw.get)
        r['wg2_us'], r['wg2_splits'] = round(tw[sb], 1), sb
    for v in (0, 1, 2):
        tw = {c[2]: t(lambda: S.wino4_wgrad(dy, x, dw, splits=c[2], variant=v))
              for c in S._wino4_wgrad_cands(N, H, H, K, C) if c[1] == v}
        if tw:
            sb = min(tw, key=tw.get)
            r['wg4_v%d_us' % v], r['wg4_v%d_splits' % v] = round(tw[sb], 1), sb
    fl = 2.0 * N * H * H * K * 9 * C
    best2 = min(r['w2_v%d_us' % v] for v in range(6))
    best4 = min(r['w4_v%d_us' % v] for v in range(3))
    r['speedup_4_over_2'] = round(best2 / best4, 3)
    r['w4_direct_equiv_tflops'] = round(fl / best4 / 1e6, 1)
    # accuracy on the first 8 images
    xs = x[:8].contiguous()
    ref = TF.conv2d(xs.double().permute(0, 3, 1, 2), w.view(K, 3, 3, C).double().permute(0, 3, 1, 2),
                    padding=1).permute(0, 2, 3, 1)
    for name, y in (('w2', S.wino_conv(xs, u)), ('w4', S.wino4_conv(xs, u4))):
        r[name + '_rel_err'] = float(((y.double() - ref).norm() / ref.norm()).item())
    res.append(r)
    print(json.dumps(r), flush=True)
if len(sys.argv) > 1:
    with open(sys.argv[1], 'w') as f:
        for r in res:
            f.write(json.dumps(r) + '\n')
