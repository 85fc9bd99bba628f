"""Normalise-on-load diagnosis: record every conv / BN call of one fp32 engine step with the fusion on and
off and print the first call whose inputs or outputs diverge."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from rafiki_amd.engine.convnet import ConvNetEngine  # noqa: E402
from rafiki_amd.ops import f32 as S  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def run(on):
    S.BN_ON_LOAD = on
    rec = []
    names = ['conv_fwd', 'conv_wgrad', 'conv_dgrad', 'conv_dgrad_t', 'bn_fwd', 'bn_finalize', 'bn_bwd']
    names = [n for n in names if hasattr(S, n)]
    orig = {n: getattr(S, n) for n in names}

    def wrap(n):
        def f(*a, **k):
            r = orig[n](*a, **k)
            torch.cuda.synchronize()
            ins = [t.clone() for t in a if isinstance(t, torch.Tensor)]
            outs = [t.clone() for t in (r if isinstance(r, tuple) else (r,)) if isinstance(t, torch.Tensor)]
            rec.append((n, ins, outs, {kk: v for kk, v in k.items() if kk in ('pro', 'xpro')}))
            return r
        return f
    for n in names:
        setattr(S, n, wrap(n))
    try:
        e = ConvNetEngine(num_classes=10, in_channels=3, image_size=16, cfg=(32, 32, 'M', 64, 64, 'M'),
                          fc_dims=(32,), device='cuda', seed=3, lr=0.05)
        g = torch.Generator().manual_seed(0)
        x = torch.zeros(e.input_shape(32))
        x[..., :3] = torch.randn(32, 16, 16, 3, generator=g)
        y = torch.randint(0, 10, (32,), generator=g, dtype=torch.int32).cuda()
        rec.clear()
        e.forward_backward(x.cuda(), y)
        torch.cuda.synchronize()
        first = list(rec)
        rec.clear()
        e.flat.grads.zero_() if hasattr(e.flat, 'grads') else None
        e.forward_backward(x.cuda(), y)
        torch.cuda.synchronize()
        return first, list(rec)
    finally:
        for n in names:
            setattr(S, n, orig[n])


on1, on2 = run(True)
off1, off2 = run(False)
for tag, A, B in (('step1', on1, off1),):
    print('==', tag, len(A), len(B))
    j = 0
    for i, (n, ins, outs, kw) in enumerate(A):
        if n == 'bn_finalize':
            continue
        while j < len(B) and B[j][0] != n and not (n == 'bn_finalize'):
            j += 1
        if j >= len(B):
            break
        nb, insb, outsb, _ = B[j]
        j += 1
        din = [rel(a, b) for a, b in zip(ins, insb) if a.shape == b.shape and a.is_floating_point()]
        dout = [rel(a, b) for a, b in zip(outs, outsb) if a.shape == b.shape and a.is_floating_point()]
        print(i, n, list(kw), 'in', ['%.1e' % d for d in din], 'out', ['%.1e' % d for d in dout])
        if n == 'bn_bwd' and dout and dout[0] > 1e-4:
            a, b = outs[0].double(), outsb[0].double()
            big = ((a - b).abs() > 1e-3 * b.abs().max()).nonzero()
            print('   differing elements', big.shape[0], big[:8].tolist())
            yy = ins[1].double()
            for idx in big[:4].tolist():
                nn, hh, ww, cc = idx
                h0, w0 = hh // 2 * 2, ww // 2 * 2
                print('   window', yy[nn, h0:h0 + 2, w0:w0 + 2, cc].flatten().tolist(),
                      'on-engine y', ins[1][nn, h0:h0 + 2, w0:w0 + 2, cc].flatten().tolist(),
                      'off-engine y', insb[1][nn, h0:h0 + 2, w0:w0 + 2, cc].flatten().tolist())
