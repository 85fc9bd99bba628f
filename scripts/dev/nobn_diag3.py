"""Stem weight gradient inside the no-BN engine (WINO off, 48x48, cin_p 4): every wgrad candidate run on the
engine's own dy / x into the engine's gradient slot, against fp64 autograd (diagnostic)."""
import sys
import torch
sys.path.insert(0, '.')
from rafiki_amd.engine.convnet import ConvNetEngine
from rafiki_amd.ops import f32 as S

S.WINO = False
DEV = 'cuda'


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def batch(B, hw, seed, c):
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(B, hw, hw, c)
    x[..., :3] = torch.randn(B, hw, hw, 3, generator=g)
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
    return x.to(DEV), y.to(DEV)


# the test's sequence: a 32x32 engine first, then the 48x48 one, each trained two steps
e32 = ConvNetEngine(num_classes=10, in_channels=3, image_size=32, cfg=(16, 16, 'M', 32, 32, 'M', 64, 'M'),
                    fc_dims=(64,), device=DEV, seed=3, lr=1e-3, dtype='fp32', bn=False, optimizer='adam',
                    weight_decay=0.0)
for i in range(2):
    e32.train_step(*batch(32, 32, 20 + i, e32.cin_p))
cfg = (16, 'M', 32, 'M', 32, 'M', 64, 'M', 64, 'M')
eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=48, cfg=cfg, fc_dims=(64,), device=DEV,
                    seed=3, lr=1e-3, dtype='fp32', bn=False, optimizer='adam', weight_decay=0.0)
TRAIN = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for i in range(TRAIN):
    eng.train_step(*batch(16, 48, 20 + i, eng.cin_p))
eng.reset_metrics()
x, y = batch(16, 48, 9, eng.cin_p)
cap = {}
orig_wgrad = S.conv_wgrad


def spy(dy, xx, **kw):
    if dy.shape[-1] == 16 and xx.shape[-1] == eng.cin_p:
        cap['dy'], cap['x'], cap['out'] = dy.clone(), xx.clone(), kw.get('out')
    return orig_wgrad(dy, xx, **kw)


S.conv_wgrad = spy
for rep in range(3):
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    fl = eng.flat
    params = {n: fl.w(n).detach().double().cpu().clone().requires_grad_(True) for n in fl.names()}
    loss, _ = eng.reference_loss(x.double().cpu(), y.cpu(), params, training=True)
    grads = dict(zip(fl.names(), torch.autograd.grad(loss, [params[n] for n in fl.names()])))
    print('rep', rep, 'conv0.w', rel(fl.g('conv0.w'), grads['conv0.w']), 'conv0.b', rel(fl.g('conv0.b'), grads['conv0.b']),
          'out ptr % 16:', cap['out'].data_ptr() % 16, flush=True)
# the reference stem gradient from the captured dy (checks dy itself)
dy, xx = cap['dy'], cap['x']
ref = torch.nn.grad.conv2d_weight(xx.double().cpu().permute(0, 3, 1, 2), (16, eng.cin_p, 3, 3),
                                  dy.double().cpu().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1).reshape(16, -1)
print('dy-based ref vs autograd', rel(ref, grads['conv0.w'].reshape(16, -1)), flush=True)
from rafiki_amd.ops import autotune as A
print('picks', {k: v for k, v in A.snapshot().items() if str(k[0]) == 'sw' and 36864 in k}, flush=True)
cands = {}


def grab(key, c, run, protect=()):
    cands['list'], cands['run'] = list(c), run
    return c[0]


S._pick = grab
orig_wgrad(dy, xx, out=cap['out'])
for c in cands['list']:
    cap['out'].zero_()
    cands['run'](c)
    torch.cuda.synchronize()
    print('cand', c, rel(cap['out'], ref), flush=True)
