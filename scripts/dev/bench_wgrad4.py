"""F(4x4,3x3) weight-gradient variants on the VGG-small layer shapes (batch 256): best split per
variant, microseconds including the split-K slab reduction.
usage: python scripts/dev/bench_wgrad4.py [out.jsonl]"""
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
for (N, H, C, K) in [(256, 32, 8, 64), (256, 32, 64, 64), (256, 16, 64, 128), (256, 16, 128, 128),
                     (256, 8, 128, 256), (256, 8, 256, 256), (256, 4, 256, 512), (256, 4, 512, 512)]:
    x = torch.randn(N, H, H, C, device='cuda')
    dy = torch.randn(N, H, H, K, device='cuda')
    dw = torch.empty(K, 9 * C, device='cuda')
    r = dict(N=N, H=H, C=C, K=K)
    for v in (0, 1):
        tw = {c[2]: t(lambda: S.wino4_wgrad(dy, x, dw, splits=c[2], variant=v))
              for c in S._wino4_wgrad_cands(N, H, H, K, C) if c[1] == v}
        if tw:
            sb = min(tw, key=tw.get)
            r['v%d_us' % v], r['v%d_splits' % v] = round(tw[sb], 1), sb
            r['v%d_all' % v] = {s: round(u, 1) for s, u in sorted(tw.items())}
    tp = {(c[1], c[2]): t(lambda: S.wino4_wgrad_pt(dy, x, dw, tile=c[1], nst=c[2]))
          for c in S._wino4_pt_cands(N, H, H, K, C)}
    if tp:
        cb = min(tp, key=tp.get)
        r['pt_us'], r['pt_cfg'] = round(tp[cb], 1), list(cb)
    fl = 2.0 * N * H * H * K * 9 * C
    r['direct_equiv_tflops_best'] = round(fl / min([r.get('v%d_us' % v, 1e9) for v in (0, 1)] +
                                                  [r.get('pt_us', 1e9)]) / 1e6, 1)
    print(json.dumps(r), flush=True)
    res.append(r)
if len(sys.argv) > 1:
    with open(sys.argv[1], 'w') as f:
        for r in res:
            f.write(json.dumps(r) + '\n')
