"""Diagnose the flat-input (MLP) engine on GPU: gradient check vs the fp32 reference + short training."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from rafiki_amd.engine.convnet import ConvNetEngine

for ibn in (False, True):
    for opt in ('sgd', 'adam'):
        eng = ConvNetEngine(num_classes=10, in_channels=1, image_size=28, cfg=(), fc_dims=(128, 128), device='cuda',
                            seed=0, optimizer=opt, lr=0.01, input_bn=ibn, weight_decay=0.0)
        g = torch.Generator().manual_seed(0)
        imgs = torch.randint(0, 256, (128, 28, 28), dtype=torch.uint8, generator=g)
        y = torch.randint(0, 10, (128,), dtype=torch.int32, generator=g).cuda()
        x = eng.prepare_inputs(imgs)
        eng.forward_backward(x, y)
        torch.cuda.synchronize()
        fl = eng.flat
        params = {n: fl.w(n).detach().clone().requires_grad_(True) for n in fl.names()}
        loss, _ = eng.reference_loss(x.float() if x.dtype != torch.bfloat16 else x, y, params, training=True,
                                     emulate_bf16=True)
        grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
        print('input_bn', ibn, opt, 'loss eng %.4f ref %.4f' % (eng.loss_sum.item() / 128, loss.item()))
        for n, gr in zip(fl.names(), grads):
            got = fl.g(n)
            cos = torch.nn.functional.cosine_similarity(got.flatten(), gr.flatten(), 0).item()
            fro = ((got - gr).norm() / gr.norm().clamp_min(1e-12)).item()
            print('   %-14s cos %.4f fro %.4f' % (n, cos, fro))
        # training on a fixed batch must drive the loss down
        eng.reset_metrics()
        for it in range(60):
            eng.reset_metrics()
            eng.train_step(x, y)
        print('   loss after 60 steps %.4f' % (eng.loss_sum.item() / 128))
