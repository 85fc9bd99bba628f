"""Diagnostic: per-layer conv outputs / BN statistics of the fp32 engine's forward, with each conv's
tuned kernel, against an fp64 conv of the same fp32 input (full-width VGG-small, batch 32)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as TF  # noqa: E402

from rafiki_amd.engine.convnet import ConvNetEngine  # noqa: E402
from rafiki_amd.ops import f32 as S  # noqa: E402

orig = S.conv_fwd
rec = []


def wrapped(x, w, **kw):
    y = orig(x, w, **kw)
    acc = kw.get('stats_acc')
    torch.cuda.synchronize()
    rec.append((x.detach().clone(), w.detach().clone(), y.detach().clone(),
                None if acc is None else acc.sum(0).detach().clone()))
    return y


S.conv_fwd = wrapped
eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=32, cfg=(64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512,
                                                                       512, 'M'), fc_dims=(512,), device='cuda',
                    seed=3, lr=0.05, dtype='fp32')
g = torch.Generator().manual_seed(1)
B = 32
x = torch.zeros(B, 32, 32, 8)
x[..., :3] = torch.randn(B, 32, 32, 3, generator=g)
y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
for it in range(2):
    rec.clear()
    eng.forward_backward(x.cuda(), y.cuda())
    torch.cuda.synchronize()
    print('pass', it)
    for li, (xi, wi, yi, st) in enumerate(rec):
        Co = wi.shape[0]
        ref = TF.conv2d(xi.double().permute(0, 3, 1, 2), wi.double().reshape(Co, 3, 3, -1).permute(0, 3, 1, 2),
                        padding=1).permute(0, 2, 3, 1)
        e = ((yi.double() - ref).norm() / ref.norm()).item()
        r = ref.reshape(-1, Co)
        es = ((st[0] - r.sum(0)).norm() / r.sum(0).norm()).item() if st is not None else -1
        es2 = ((st[1] - (r * r).sum(0)).norm() / (r * r).sum(0).norm()).item() if st is not None else -1
        mx = ((yi.double() - ref).abs().max() / ref.abs().max()).item()
        print('  L{} y err {:.2e} max {:.2e} stats {:.2e} {:.2e} x>=0 {}'.format(li, e, mx, es, es2,
                                                                                 bool((xi >= 0).all())))
