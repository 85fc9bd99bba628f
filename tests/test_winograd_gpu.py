"""Fused Winograd F(2x2,3x3) fp32 conv (csrc/kernels/winograd.hip; variants 2 / 3 are the small-wave-tile
kernels of csrc/kernels/winograd4.hip) vs fp64 PyTorch references.

F(2x2,3x3) adds a few fp32 roundings in the input / output transforms (values up to 4x the inputs),
measured ~1e-7 relative; the gate is the same 1e-5 relative Frobenius error as the direct kernels."""
import math

import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = 'cuda'
VARIANTS = [0, 1, 2, 3, 4, 5]   # 2-5: winograd4.hip's 16x16-wave-tile kernels (5: two-stage pipelined)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).float()


def _conv_ref(x_nhwc, w_ohwi):
    return TF.conv2d(x_nhwc.double().permute(0, 3, 1, 2), w_ohwi.double().permute(0, 3, 1, 2),
                     padding=1).permute(0, 2, 3, 1)


def _u(w):
    from rafiki_amd.ops import f32 as S
    Cout, Cin = w.shape[0], w.shape[-1]
    u = torch.empty((16, Cout, Cin), device=DEV)
    ut = torch.empty((16, Cin, Cout), device=DEV)
    S.wino_weights(w.to(DEV).reshape(Cout, -1).contiguous(), u, ut)
    return u, ut


@pytest.mark.parametrize("N,H,W,Cin,Cout", [
    (2, 8, 8, 16, 32), (3, 6, 10, 24, 40), (4, 32, 32, 64, 64), (8, 4, 4, 512, 512), (2, 2, 2, 8, 72),
    (5, 16, 16, 128, 128), (1, 12, 20, 8, 8)])
@pytest.mark.parametrize("variant", VARIANTS)
def test_wino_fwd_and_stats(N, H, W, Cin, Cout, variant):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=1)
    w = _rand(Cout, 3, 3, Cin, seed=2, scale=1.0 / math.sqrt(9 * Cin))
    u, _ = _u(w)
    acc = torch.zeros((S.bn_slots(Cout), 2, Cout), dtype=torch.float64, device=DEV)
    y = S.wino_conv(x.to(DEV), u, stats=acc, variant=variant)
    torch.cuda.synchronize()
    ref = _conv_ref(x, w)
    assert rel(y, ref) < 1e-5
    s = acc.sum(0).cpu()
    r = ref.reshape(-1, Cout)
    assert rel(s[0], r.sum(0)) < 1e-5 and rel(s[1], (r * r).sum(0)) < 1e-5


def test_wino_bias_relu():
    from rafiki_amd.ops import f32 as S
    x = _rand(3, 8, 8, 32, seed=3)
    w = _rand(48, 3, 3, 32, seed=4, scale=0.1)
    b = _rand(48, seed=5)
    u, _ = _u(w)
    y = S.wino_conv(x.to(DEV), u, bias=b.to(DEV), relu=True)
    torch.cuda.synchronize()
    assert rel(y, torch.relu(_conv_ref(x, w) + b.double())) < 1e-5


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(4, 8, 8, 64, 128), (2, 16, 16, 64, 64), (8, 4, 4, 512, 256),
                                            (2, 6, 6, 24, 16)])
@pytest.mark.parametrize("variant", VARIANTS)
def test_wino_dgrad_from_transposed_set(N, H, W, Cin, Cout, variant):
    """dx = conv(dy, flip(w)^T) from the ut set (transpose of u with positions 0 <-> 3 swapped)."""
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=6)
    w = _rand(Cout, 3, 3, Cin, seed=7, scale=0.1)
    dy = _rand(N, H, W, Cout, seed=8)
    _, ut = _u(w)
    dx = S.wino_conv(dy.to(DEV), ut, variant=variant)
    torch.cuda.synchronize()
    xd = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    out = TF.conv2d(xd, w.double().permute(0, 3, 1, 2), padding=1)
    (gx,) = torch.autograd.grad(out, xd, dy.double().permute(0, 3, 1, 2))
    assert rel(dx, gx.permute(0, 2, 3, 1)) < 1e-5


@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("H", [8, 4])
def test_wino_dgrad_bn_epilogues_match_direct(pool, variant, H):
    """The BNB / BNP epilogues (ReLU mask / pool routing + BN-backward sums of the layer below) give
    the same dx and sums as the direct kernel's."""
    from rafiki_amd.ops import f32 as S
    N, W, Cin, Cout = 4, H, 64, 128
    Hy, Wy = (2 * H, 2 * W) if pool else (H, W)
    y = _rand(N, Hy, Wy, Cin, seed=17) + 0.2
    gamma, beta = torch.ones(Cin) * 1.3, _rand(Cin, seed=18) * 0.1
    acc = torch.zeros((S.bn_slots(Cin), 2, Cin), dtype=torch.float64, device=DEV)
    S.col_stats(y.to(DEV).view(-1, Cin), acc)
    _, coeffs = S.bn_fwd(y.to(DEV), acc, N * Hy * Wy, gamma.to(DEV), beta.to(DEV), 1e-5, pool=pool, act=1)
    w = _rand(Cout, 3, 3, Cin, seed=19, scale=0.05)
    arena = w.reshape(-1).to(DEV).contiguous()
    wt = S.SConvWT(arena, [arena.view(Cout, 3, 3, Cin)])
    wt.refresh()
    _, ut = _u(w)
    dyo = _rand(N, H, W, Cout, seed=20).to(DEV)
    acc_w, acc_d = torch.zeros_like(acc), torch.zeros_like(acc)
    key = 'bnp' if pool else 'bnb'
    d_w = S.wino_conv(dyo, ut, variant=variant, **{key: (y.to(DEV), coeffs, acc_w)})
    d_d = S.conv_dgrad(dyo, wt.view(0), **{key: (y.to(DEV), coeffs, acc_d)})
    torch.cuda.synchronize()
    assert rel(d_w, d_d) < 1e-5
    assert rel(acc_w.sum(0), acc_d.sum(0)) < 1e-5


def test_wino_weights_arena_refresh():
    from rafiki_amd.ops import f32 as S
    shapes = [(64, 32), (16, 64), (40, 24)]
    arena = torch.zeros(sum(co * 9 * ci for co, ci in shapes) + 7, device=DEV)
    ws, off = [], 3
    for k, (co, ci) in enumerate(shapes):
        w = arena[off:off + co * 9 * ci].view(co, 9 * ci)
        w.copy_(_rand(co, 9 * ci, seed=21 + k))
        ws.append(w)
        off += co * 9 * ci
    ww = S.WinoWeights(arena, ws)
    ww.refresh()
    for l, w in enumerate(ws):
        u, ut = _u(w.view(w.shape[0], 3, 3, -1).cpu())
        assert torch.equal(ww.u(l), u) and torch.equal(ww.ut(l), ut)


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(4, 8, 8, 64, 128), (2, 32, 32, 64, 64), (16, 4, 4, 256, 512),
                                            (3, 6, 10, 24, 40), (2, 2, 2, 16, 16)])
@pytest.mark.parametrize("splits", [1, 2, 5])
def test_wino_wgrad(N, H, W, Cin, Cout, splits):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=30)
    dy = _rand(N, H, W, Cout, seed=31)
    nt = N * (H // 2) * (W // 2)
    tps = -(-(-(-nt // splits)) // 8) * 8
    s_eff = -(-nt // tps)
    dw = torch.empty(Cout, 9 * Cin, device=DEV)
    S.wino_wgrad(dy.to(DEV), x.to(DEV), dw, splits=s_eff)
    prev = _rand(Cout, 9 * Cin, seed=32).to(DEV)
    acc = prev.clone()
    S.wino_wgrad(dy.to(DEV), x.to(DEV), acc, splits=s_eff, accumulate=True)
    torch.cuda.synchronize()
    wd = torch.zeros(Cout, Cin, 3, 3, dtype=torch.float64, requires_grad=True)
    out = TF.conv2d(x.double().permute(0, 3, 1, 2), wd, padding=1)
    (gw,) = torch.autograd.grad(out, wd, dy.double().permute(0, 3, 1, 2))
    ref = gw.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)
    assert rel(dw, ref) < 1e-5
    assert rel(acc, ref + prev.double().cpu()) < 1e-5


@pytest.mark.parametrize("shared", [True, False])
@pytest.mark.parametrize("variant", VARIANTS)
def test_wino_conv_grouped(shared, variant):
    """k convs in one grid (the serving ensemble's layers) == k separate convs."""
    from rafiki_amd.ops import f32 as S
    G, Nb, H, Cin, Cout = 3, 5, 8, 32, 48
    x = (_rand(Nb, H, H, Cin, seed=40) if shared else _rand(G, Nb, H, H, Cin, seed=40)).to(DEV)
    w = [_rand(Cout, 3, 3, Cin, seed=41 + g, scale=0.1) for g in range(G)]
    u = torch.stack([_u(wg)[0] for wg in w]).contiguous()
    b = _rand(G, Cout, seed=45).to(DEV)
    y = S.wino_conv_grp(x, u, bias=b, relu=True, variant=variant)
    torch.cuda.synchronize()
    for g in range(G):
        xg = x if shared else x[g]
        ref = torch.relu(_conv_ref(xg.cpu(), w[g]) + b[g].double().cpu())
        assert rel(y[g], ref) < 1e-5
