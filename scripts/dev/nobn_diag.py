"""Per-parameter gradient error of the bn=False engine vs fp64 autograd (diagnostic)."""
import sys
import torch
sys.path.insert(0, '.')
from rafiki_amd.engine.convnet import ConvNetEngine
from rafiki_amd.ops import f32 as S

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


for wino in (False, True):
    S.WINO = wino
    for image_size, cfg, B, steps in ((32, (16, 16, 'M', 32, 32, 'M', 64, 'M'), 32, 0),
                                      (32, (16, 16, 'M', 32, 32, 'M', 64, 'M'), 32, 2),
                                      (48, (16, 'M', 32, 'M', 32, 'M', 64, 'M', 64, 'M'), 16, 2)):
        eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=image_size, cfg=cfg, fc_dims=(64,), device=DEV,
                            seed=3, lr=1e-3, dtype='fp32', bn=False, optimizer='adam', weight_decay=0.0)
        c = eng.cin_p
        for i in range(steps):
            x, y = batch(B, image_size, 20 + i, c)
            eng.train_step(x, y)
        x, y = batch(B, image_size, 9, c)
        eng.reset_metrics()
        eng.forward_backward(x, y)
        torch.cuda.synchronize()
        fl = eng.flat
        params = {n: fl.w(n).detach().double().cpu().clone().requires_grad_(True) for n in fl.names()}
        loss, _ = eng.reference_loss(x.double().cpu(), y.cpu(), params, training=True)
        grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
        errs = {n: round(rel(fl.g(n), g), 7) for n, g in zip(fl.names(), grads) if g.norm() > 0}
        print(dict(wino=wino, hw=image_size, steps=steps, loss=(eng.loss_sum.item() / B, loss.item()), errs=errs),
              flush=True)
