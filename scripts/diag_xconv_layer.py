"""Diagnostic: which forward layer's xconv moves the top-layer gradients (RAFIKI_XCONV=fwd, xconv
candidates offered on one (map size, Cin) at a time; autotune forced to pick xconv there)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ['RAFIKI_XCONV'] = 'fwd'
os.environ['RAFIKI_TUNE_CACHE'] = 'off'
import torch  # noqa: E402

from rafiki_amd.engine.convnet import ConvNetEngine  # noqa: E402
from rafiki_amd.ops import f32 as S, autotune  # noqa: E402

target = tuple(int(v) for v in sys.argv[1].split(','))   # (H, Cin)
orig = S._xconv_cands


def only(H, W, C, N, M, force=False):
    return orig(H, W, C, N, M, force) if (H, C) == target else []


S._xconv_cands = only
orig_pick = S._pick


def pick(key, cands, run, protect=()):
    x = [c for c in cands if c[0] <= S.XCONV]
    if x:   # force the xconv candidate where offered
        return x[0]
    return orig_pick(key, cands, run, protect)


S._pick = pick


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=32, cfg=(64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512,
                                                                       512, 'M'), fc_dims=(512,), device='cuda',
                    seed=3, lr=0.05, dtype='fp32')
g = torch.Generator().manual_seed(1)
B = 32
x = torch.zeros(B, 32, 32, 8)
x[..., :3] = torch.randn(B, 32, 32, 3, generator=g)
y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
x, y = x.cuda(), y.cuda()
eng.forward_backward(x, y)
torch.cuda.synchronize()
fl = eng.flat
params = {n: fl.w(n).detach().double().cpu().clone().requires_grad_(True) for n in fl.names()}
loss, _ = eng.reference_loss(x.double().cpu(), y.cpu(), params, training=True)
grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
out = {n: rel(fl.g(n), gr) for n, gr in zip(fl.names(), grads) if n in ('conv7.w', 'conv7.beta', 'conv6.gamma',
                                                                         'conv4.gamma', 'fc0.w')}
print('xconv at', target, {k: '%.2e' % v for k, v in out.items()})
