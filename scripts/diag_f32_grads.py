"""Per-parameter gradient error of the fp32 engine (full-width VGG-small, batch 32) vs fp64 autograd,
next to PyTorch fp32's own error, plus the autotune choice of every conv (diagnostic for the
candidate families: RAFIKI_X6 / RAFIKI_XCONV / RAFIKI_PT_MAX_HW)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rafiki_amd.engine.convnet import ConvNetEngine  # noqa: E402
from rafiki_amd.ops import autotune  # noqa: E402


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


def ref_grads(dt):
    params = {n: fl.w(n).detach().to(dt).cpu().clone().requires_grad_(True) for n in fl.names()}
    loss, _ = eng.reference_loss(x.to(dt).cpu(), y.cpu(), params, training=True)
    return loss, torch.autograd.grad(loss, [params[n] for n in fl.names()])


loss, grads = ref_grads(torch.float64)
_, grads32 = ref_grads(torch.float32)
tag = 'X6={} XCONV={} PT={}'.format(os.environ.get('RAFIKI_X6', '1'), os.environ.get('RAFIKI_XCONV', '1'),
                                     os.environ.get('RAFIKI_PT_MAX_HW', '-'))
print(tag, 'loss', eng.loss_sum.item() / B, loss.item())
for n, gr, g32 in zip(fl.names(), grads, grads32):
    if gr.norm() == 0:
        continue
    print('  {:12s} engine {:.2e}  torch32 {:.2e}'.format(n, rel(fl.g(n), gr), rel(g32, gr)))
for k, v in sorted(autotune.snapshot().items(), key=lambda kv: str(kv[0])) if hasattr(autotune, 'snapshot') else []:
    if k[0] in ('sf', 'sd', 'sw'):
        print('  tune', k[:4], v)
