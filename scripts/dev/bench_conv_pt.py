"""Deep-layer fp32 3x3 convs (VGG-small, batch 256): fused Winograd kernels (F(2x2) v0-v5, F(4x4) v0-v1)
vs the pre-transformed F(4x4) path (input transform + 36-group sgemm + output transform), forward with
BN statistics; microseconds, best config each.  usage: python scripts/dev/bench_conv_pt.py [out.jsonl]"""
import json
import sys

sys.path.insert(0, '.')
import torch  # noqa: E402

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
for (N, H, C, K) in [(256, 8, 128, 256), (256, 8, 256, 256), (256, 4, 256, 512), (256, 4, 512, 512)]:
    x = torch.randn(N, H, H, C, device='cuda')
    w = torch.randn(K, 9 * C, device='cuda') * (1.0 / (9 * C)) ** 0.5
    u = torch.empty(16, K, C, device='cuda')
    ut = torch.empty(16, C, K, device='cuda')
    S.wino_weights(w, u, ut)
    u4 = S.wino4_u(w)
    acc = torch.zeros((S.bn_slots(K), 2, K), dtype=torch.float64, device='cuda')
    r = dict(N=N, H=H, C=C, K=K)
    f2 = {v: t(lambda: S.wino_conv(x, u, stats=acc, variant=v)) for v in range(6)}
    f4 = {v: t(lambda: S.wino4_conv(x, u4, stats=acc, variant=v)) for v in range(2)}
    pt = {c: t(lambda: S.wino4_conv_pt(x, u4, stats=acc, tile=c[1], nst=c[2])) for c in S.WINO4_PT_CFGS}
    r['fused_best_us'] = round(min(list(f2.values()) + list(f4.values())), 1)
    r['pt_best_us'] = round(min(pt.values()), 1)
    r['pt_cfg'] = list(min(pt, key=pt.get))
    r['pt_all'] = {str(list(k)): round(v, 1) for k, v in pt.items()}
    print(json.dumps(r), flush=True)
    res.append(r)
if len(sys.argv) > 1:
    with open(sys.argv[1], 'w') as f:
        for r in res:
            f.write(json.dumps(r) + '\n')
