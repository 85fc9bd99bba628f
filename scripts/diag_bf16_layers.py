"""Layer-by-layer bf16 engine vs bf16-emulating oracle: forward activations and conv-output
gradients per block (localises the bf16 gradient residual)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as TF  # noqa: E402

from rafiki_amd.engine import convnet as CN  # noqa: E402
from rafiki_amd.ops import functional as F  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    eng = CN.ConvNetEngine(num_classes=10, in_channels=3, image_size=16, cfg=(16, 'M', 32, 32, 'M'), fc_dims=(32,),
                           device='cuda', seed=3, lr=0.05, dtype='bf16')
    g = torch.Generator().manual_seed(0)
    x = torch.zeros(64, 16, 16, 8)
    x[..., :3] = torch.randn(64, 16, 16, 3, generator=g)
    y = torch.randint(0, 10, (64,), generator=g, dtype=torch.int32)
    x, y = x.bfloat16().cuda(), y.cuda()
    cap = {'wgrad_dy': [], 'wgrad_x': [], 'bn_in_d': [], 'conv_y': [], 'act': []}
    orig_wg, orig_bb, orig_cf, orig_ba = F.conv_wgrad, F.bn_bwd_acc, F.conv_fwd, F.bn_act_fwd_acc

    def wg(dy, xx, **kw):
        cap['wgrad_dy'].append(dy.clone())
        cap['wgrad_x'].append(xx.clone())
        return orig_wg(dy, xx, **kw)

    def bb(d, yy, *a, **kw):
        cap['bn_in_d'].append(d.clone())
        return orig_bb(d, yy, *a, **kw)

    def cf(h, w, **kw):
        out = orig_cf(h, w, **kw)
        cap['conv_y'].append(out[0].clone())
        return out

    def ba(*a, **kw):
        out = orig_ba(*a, **kw)
        cap['act'].append(out[0].clone())
        return out
    F.conv_wgrad, F.bn_bwd_acc, F.conv_fwd, F.bn_act_fwd_acc = wg, bb, cf, ba
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    F.conv_wgrad, F.bn_bwd_acc, F.conv_fwd, F.bn_act_fwd_acc = orig_wg, orig_bb, orig_cf, orig_ba
    # oracle with hooks
    fl = eng.flat
    P = {n: fl.w(n).detach().clone().requires_grad_(True) for n in fl.names()}
    ys, hs, gys, ghs = [], [], {}, {}
    orig_conv, orig_bn, orig_pool = TF.conv2d, TF.batch_norm, TF.max_pool2d
    idx = {'c': 0}

    def conv_hook(*a, **kw):
        out = orig_conv(*a, **kw)
        i = len(ys)
        ys.append(out)
        out.register_hook(lambda gr, i=i: gys.__setitem__(i, gr.clone()))
        return out
    pools, gpools = [], {}

    def pool_hook(*a, **kw):
        out = orig_pool(*a, **kw)
        i = len(pools)
        pools.append(out)
        out.register_hook(lambda gr, i=i: gpools.__setitem__(i, gr.clone()))
        return out
    TF.conv2d, TF.max_pool2d = conv_hook, pool_hook
    loss, _ = eng.reference_loss(x, y, P, training=True, emulate_bf16=True)
    TF.conv2d, TF.max_pool2d = orig_conv, orig_pool
    loss.backward()
    nb = len(eng.blocks)
    print('loss engine {:.6f} oracle {:.6f}'.format(eng.loss_sum.item() / 64, loss.item()))
    for bi in range(nb):
        ye = cap['conv_y'][bi].float().permute(0, 3, 1, 2)
        print('block', bi, 'conv out y: rel', round(rel(ye, ys[bi].detach().bfloat16().float()), 5))
    # backward: engine wgrad dy order is last block first
    for k, bi in enumerate(range(nb - 1, -1, -1)):
        de = cap['wgrad_dy'][k].float().permute(0, 3, 1, 2)
        do = gys[bi]
        print('block', bi, 'grad wrt conv output: rel', round(rel(de, do), 5),
              ' | grad into block output (pre-BN-bwd): engine norm', round(cap['bn_in_d'][k].float().norm().item(), 4))
        if bi == nb - 1:
            dd = cap['bn_in_d'][k].float().permute(0, 3, 1, 2)
            print('        grad into pooled block output: rel', round(rel(dd, gpools[len(pools) - 1]), 5))
            # BN(+ReLU+pool) backward in float64 from the ENGINE's own inputs (its y, its d, batch stats of y)
            yb = cap['conv_y'][bi].double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
            gam = eng.flat.w(eng.blocks[bi][0] + '.gamma').double().cpu()
            bet = eng.flat.w(eng.blocks[bi][0] + '.beta').double().cpu()
            hh = orig_pool(torch.relu(TF.batch_norm(yb, None, None, gam, bet, training=True, eps=eng.bn_eps)), 2)
            (gy64,) = torch.autograd.grad(hh, yb, dd.double().cpu())
            print('        engine dz vs fp64 BN-backward of the engine inputs: rel', round(rel(de, gy64), 5),
                  '| oracle dz vs the same:', round(rel(do, gy64), 5))
        xe = cap['wgrad_x'][k].float()
        print('        wgrad input act rel vs engine-forward act', round(rel(xe, cap['act'][bi - 1] if bi > 0 else x), 5)
              if bi > 0 else '')


if __name__ == '__main__':
    main()
