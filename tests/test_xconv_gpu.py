"""Halo-tiled X6 3x3 conv (csrc/kernels/xconv.hip) against fp64 PyTorch references of the same fp32
inputs: forward (+ BN statistics in the epilogue), data gradient through the flipped transposed
weight planes (plain, FLAG_BNB and FLAG_BNP epilogues), every item shape on every map size it takes.
Gate: relative Frobenius error <= 1e-5 (the sgemm fp32 tests' gate; measured ~1e-7)."""
import math

import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).float()


SHAPES = [(4, 32, 64, 64), (2, 16, 64, 128), (4, 8, 128, 256), (8, 4, 256, 512), (16, 4, 64, 64), (8, 8, 32, 64)]


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("N,H,Cin,Cout", SHAPES)
def test_xconv_forward_and_stats(N, H, Cin, Cout, cfg):
    from rafiki_amd.ops import f32 as S
    if (S.XCONV - cfg, 0, 1) not in S._xconv_cands(H, H, Cin, Cout, N * H * H, force=True):
        pytest.skip('item shape does not tile this problem')
    x = _rand(N, H, H, Cin, seed=1)
    w = _rand(Cout, 3, 3, Cin, seed=2, scale=1.0 / math.sqrt(9 * Cin))
    ref = TF.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    wd = w.to(DEV)
    planes = S.xconv_planes(wd)
    acc = torch.zeros((S.bn_slots(Cout), 2, Cout), dtype=torch.float64, device=DEV)
    y = S.xconv(x.to(DEV), planes, cfg=cfg, stats=acc)
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-5
    s = acc.sum(0).cpu()
    r = ref.reshape(-1, Cout)
    assert rel(s[0], r.sum(0)) < 1e-5 and rel(s[1], (r * r).sum(0)) < 1e-5


@pytest.mark.parametrize("N,H,Cin,Cout", [(4, 16, 64, 128), (8, 4, 512, 256), (2, 32, 64, 64)])
def test_xconv_dgrad(N, H, Cin, Cout):
    from rafiki_amd.ops import f32 as S
    w = _rand(Cout, 3, 3, Cin, seed=3, scale=0.1)
    dy = _rand(N, H, H, Cout, seed=4)
    xd = torch.zeros(N, Cin, H, H, dtype=torch.float64, requires_grad=True)
    yd = TF.conv2d(xd, w.double().permute(0, 3, 1, 2), padding=1)
    (ref,) = torch.autograd.grad(yd, xd, dy.double().permute(0, 3, 1, 2))
    ref = ref.permute(0, 2, 3, 1)
    planes = S.xconv_planes(w.to(DEV), dgrad=True)
    assert planes.shape == (3, 9, Cin, Cout)
    dx = S.xconv(dy.to(DEV), planes, cfg=3)
    torch.cuda.synchronize()
    assert rel(dx, ref) < 1e-5


def test_xconv_dgrad_bn_epilogues():
    """FLAG_BNB (input block BN+ReLU) and FLAG_BNP (BN+ReLU+2x2 max-pool) through the X6 conv agree with
    the same epilogues on the f32 implicit GEMM (sgemm.hip) to fp32 round-off."""
    from rafiki_amd.ops import f32 as S
    N, H, Cin, Cout = 4, 8, 64, 128
    w = _rand(Cout, 3, 3, Cin, seed=5, scale=0.1).to(DEV)
    dy = _rand(N, H, H, Cout, seed=6).to(DEV)
    planes = S.xconv_planes(w, dgrad=True)
    arena = w.reshape(-1).contiguous()
    wt = S.SConvWT(arena, [arena.view(Cout, 3, 3, Cin)])
    wt.refresh()
    coeffs = torch.stack([torch.zeros(Cin), torch.ones(Cin), _rand(Cin, seed=7), _rand(Cin, seed=8)]).to(DEV)
    for mode, yshape in (('bnb', (N, H, H, Cin)), ('bnp', (N, 2 * H, 2 * H, Cin))):
        y = _rand(*yshape, seed=9).to(DEV)
        a1 = torch.zeros((S.bn_slots(Cin), 2, Cin), dtype=torch.float64, device=DEV)
        a2 = torch.zeros_like(a1)
        d1 = S.xconv(dy, planes, cfg=3, **{mode: (y, coeffs, a1)})
        S._PIN_BAK = S._PIN
        S._PIN = (3, 2)
        try:
            d2 = S.conv_dgrad(dy, wt.view(0), **{mode: (y, coeffs, a2)})
        finally:
            S._PIN = S._PIN_BAK
        torch.cuda.synchronize()
        assert rel(d1, d2) < 1e-5, mode
        assert rel(a1.sum(0), a2.sum(0)) < 1e-5, mode


@pytest.mark.parametrize("mode", ["fwd", "bnb", "bnp"])
def test_xconv_writes_only_its_outputs(mode):
    """Canaries around the output and the fp64 statistic slots: nothing outside them changes."""
    from rafiki_amd.ops import f32 as S
    N, H, Cin, Cout = 8, 8, 64, 128
    g = torch.Generator().manual_seed(11)
    if mode == 'fwd':
        x = torch.randn(N, H, H, Cin, generator=g).to(DEV)
        planes = S.xconv_planes((torch.randn(Cout, 3, 3, Cin, generator=g) * 0.05).to(DEV))
        No = Cout
    else:
        x = torch.randn(N, H, H, Cout, generator=g).to(DEV)
        planes = S.xconv_planes((torch.randn(Cout, 3, 3, Cin, generator=g) * 0.05).to(DEV), dgrad=True)
        No = Cin
    n_out = N * H * H * No
    big = torch.full((n_out + 2 * 4096,), 7.0, device=DEV)
    out = big[4096:4096 + n_out].view(N, H, H, No)
    SL = S.bn_slots(No)
    sbig = torch.full((SL * 2 * No + 2 * 512,), 3.0, dtype=torch.float64, device=DEV)
    stats = sbig[512:512 + SL * 2 * No].view(SL, 2, No)
    stats.zero_()
    for cfg in [c[0] for c in S._xconv_cands(H, H, x.shape[-1], No, N * H * H, force=True)]:
        if mode == 'fwd':
            S.xconv(x, planes, cfg=S.XCONV - cfg, out=out, stats=stats)
        else:
            coeffs = torch.stack([torch.zeros(No), torch.ones(No), torch.randn(No, generator=g),
                                  torch.randn(No, generator=g)]).to(DEV)
            ys = (N, H, H, No) if mode == 'bnb' else (N, 2 * H, 2 * H, No)
            y = torch.randn(*ys, generator=g).to(DEV)
            S.xconv(x, planes, cfg=S.XCONV - cfg, out=out, **{mode: (y, coeffs, stats)})
        torch.cuda.synchronize()
        assert bool((big[:4096] == 7.0).all()) and bool((big[4096 + n_out:] == 7.0).all()), cfg
        assert bool((sbig[:512] == 3.0).all()) and bool((sbig[512 + SL * 2 * No:] == 3.0).all()), cfg
