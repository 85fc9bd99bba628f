"""Per-parameter gradient error of the GPU engine vs the fp32 PyTorch reference (diagnostic)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from rafiki_amd.engine.convnet import ConvNetEngine

for cfg, hw in [((16, 'M', 32, 32, 'M'), 16), ((64, 'M', 128, 'M'), 16)]:
    eng = ConvNetEngine(num_classes=10, in_channels=3, image_size=hw, cfg=cfg, fc_dims=(32,), device='cuda', seed=3)
    g = torch.Generator().manual_seed(0)
    B = 64
    x = torch.zeros(B, hw, hw, 8); x[..., :3] = torch.randn(B, hw, hw, 3, generator=g)
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
    x, y = x.bfloat16().cuda(), y.cuda()
    eng.forward_backward(x, y); torch.cuda.synchronize()
    fl = eng.flat
    params = {n: fl.w(n).detach().clone().requires_grad_(True) for n in fl.names()}
    loss, _ = eng.reference_loss(x, y, params, training=True, emulate_bf16=('--bf16' in sys.argv))
    grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
    print(cfg, 'loss gpu', eng.loss_sum.item() / B, 'ref', loss.item())
    for n, gr in zip(fl.names(), grads):
        got = fl.g(n)
        mx = ((got - gr).abs().max() / gr.abs().max().clamp_min(1e-9)).item()
        fro = ((got - gr).norm() / gr.norm().clamp_min(1e-12)).item()
        cos = torch.nn.functional.cosine_similarity(got.flatten(), gr.flatten(), 0).item()
        print('  {:12s} max-rel {:.4f} fro-rel {:.4f} cos {:.5f} |g| {:.3e}'.format(n, mx, fro, cos, gr.norm().item()))
