"""Stem weight-gradient error at 48x48 with WINO off: BN vs no-BN, picked configs (diagnostic)."""
import sys
import torch
sys.path.insert(0, '.')
from rafiki_amd.engine.convnet import ConvNetEngine
from rafiki_amd.ops import autotune as A
from rafiki_amd.ops import f32 as S

S.WINO = False
DEV = 'cuda'


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


for bn in (True, False):
    cfg = (16, 'M', 32, 'M', 32, 'M', 64, 'M', 64, 'M')
    eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=48, cfg=cfg, fc_dims=(64,), device=DEV,
                        seed=3, lr=1e-3, dtype='fp32', bn=bn, optimizer='adam', weight_decay=0.0)
    g = torch.Generator().manual_seed(9)
    x = torch.zeros(16, 48, 48, eng.cin_p)
    x[..., :3] = torch.randn(16, 48, 48, 3, generator=g)
    y = torch.randint(0, 10, (16,), generator=g, dtype=torch.int32)
    x, y = x.to(DEV), y.to(DEV)
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    fl = eng.flat
    params = {n: fl.w(n).detach().double().cpu().clone().requires_grad_(True) for n in fl.names()}
    loss, _ = eng.reference_loss(x.double().cpu(), y.cpu(), params, training=True)
    grads = dict(zip(fl.names(), torch.autograd.grad(loss, [params[n] for n in fl.names()])))
    e = rel(fl.g('conv0.w'), grads['conv0.w'])
    # per input channel / tap error of the stem gradient
    gw = fl.g('conv0.w').double().cpu().view(16, 3, 3, -1)
    rw = grads['conv0.w'].view(16, 3, 3, -1)
    per_c = [rel(gw[..., c], rw[..., c]) if rw[..., c].norm() > 0 else float(gw[..., c].norm()) for c in range(gw.shape[-1])]
    per_t = [[round(rel(gw[:, i, j], rw[:, i, j]), 7) for j in range(3)] for i in range(3)]
    picks = {k: v for k, v in A.snapshot().items() if str(k[0]) == 'sw'}
    print(dict(bn=bn, conv0_w=e, per_channel=per_c, per_tap=per_t, sw_picks=picks), flush=True)
