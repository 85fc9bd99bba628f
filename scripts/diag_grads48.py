import sys; sys.path.insert(0, '.')
import torch
sys.path.insert(0, 'tests')
from test_engine_gpu import _engine, _batch
for hw, cfg in [(48, (16, 'M', 32, 'M', 32, 'M', 64, 'M', 64, 'M')), (32, (16, 'M', 32, 'M', 32, 'M', 64, 'M', 64, 'M'))]:
    eng = _engine(image_size=hw, cfg=cfg, fc_dims=(64,))
    x, y = _batch(32, hw=hw, seed=7)
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    fl = eng.flat
    params = {n: fl.w(n).detach().clone().requires_grad_(True) for n in fl.names()}
    loss, _ = eng.reference_loss(x, y, params, training=True, emulate_bf16=True)
    grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
    print(hw, 'loss', eng.loss_sum.item() / 32, loss.item())
    for n, g in zip(fl.names(), grads):
        got = fl.g(n)
        fro = ((got - g).norm() / g.norm().clamp_min(1e-12)).item()
        cos = torch.nn.functional.cosine_similarity(got.flatten(), g.flatten(), 0).item()
        print('  %-10s fro %.4f cos %.5f' % (n, fro, cos))
