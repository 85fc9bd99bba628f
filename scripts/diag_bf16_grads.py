"""bf16 engine gradients vs the bf16-emulating fp32 oracle, per parameter (relative Frobenius).
Run under different RAFIKI_* fusion switches to localise a discrepancy."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rafiki_amd.engine.convnet import ConvNetEngine  # noqa: E402


def main():
    eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=16, cfg=(16, 'M', 32, 32, 'M'), fc_dims=(32,),
                        device='cuda', seed=3, lr=0.05, dtype='bf16')
    g = torch.Generator().manual_seed(0)
    x = torch.zeros(64, 16, 16, 8)
    x[..., :3] = torch.randn(64, 16, 16, 3, generator=g)
    y = torch.randint(0, 10, (64,), generator=g, dtype=torch.int32)
    x, y = x.bfloat16().cuda(), y.cuda()
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    fl = eng.flat
    params = {n: fl.w(n).detach().clone().requires_grad_(True) for n in fl.names()}
    loss, _ = eng.reference_loss(x, y, params, training=True, emulate_bf16=True)
    grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
    tag = ' '.join('{}={}'.format(k, v) for k, v in sorted(os.environ.items()) if k.startswith('RAFIKI_'))
    out = []
    for n, gr in zip(fl.names(), grads):
        out.append('{}:{:.4f}'.format(n, ((fl.g(n) - gr).norm() / gr.norm().clamp_min(1e-12)).item()))
    print('[{}]'.format(tag), ' '.join(out), flush=True)


if __name__ == '__main__':
    main()
