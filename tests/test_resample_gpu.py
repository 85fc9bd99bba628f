"""Stride-2 gather convolutions (the PG-GAN up / down convs: S2, its adjoint S2T, weight gradient
S2W) and the 2x resampling kernels vs PyTorch fp64 references (conv2d / conv_transpose2d with the
4x4 stride-2 weights, nearest upsample, avg-pool).  Gate: relative Frobenius error <= 1e-5."""
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


def _w4(W, Co, Ci):   # [Co, 16*Ci] tap-major -> torch [Co, Ci, 4, 4]
    return W.reshape(Co, 4, 4, Ci).permute(0, 3, 1, 2)


SHAPES = [(2, 8, 8, 32, 64), (3, 4, 4, 512, 512), (1, 16, 16, 24, 40), (2, 12, 12, 64, 16), (5, 2, 2, 128, 256)]


@pytest.mark.parametrize("N,H,W,Ci,Co", SHAPES)
def test_s2_conv_forward(N, H, W, Ci, Co):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Ci, seed=1)
    Wt = _rand(Co, 16 * Ci, seed=2, scale=0.05)
    b = _rand(Co, seed=3, scale=0.1)
    ref = TF.conv2d(x.double().permute(0, 3, 1, 2), _w4(Wt.double(), Co, Ci), b.double(), stride=2, padding=1)
    ref = TF.leaky_relu(ref, 0.2).permute(0, 2, 3, 1)
    y = S.s2_conv(x.to(DEV), Wt.to(DEV), bias=b.to(DEV), act=S.ACT_LRELU, slope=0.2)
    assert y.shape == (N, H // 2, W // 2, Co)
    assert rel(y, ref) < 1e-5


@pytest.mark.parametrize("N,H,W,Ci,Co", SHAPES)
def test_s2t_conv_is_the_adjoint(N, H, W, Ci, Co):
    from rafiki_amd.ops import f32 as S
    z = _rand(N, H // 2, W // 2, Co, seed=4)
    Wt = _rand(Co, 16 * Ci, seed=5, scale=0.05)
    ref = TF.conv_transpose2d(z.double().permute(0, 3, 1, 2), _w4(Wt.double(), Co, Ci), stride=2, padding=1)
    ref = ref.permute(0, 2, 3, 1)
    y = S.s2t_conv(z.to(DEV), Wt.to(DEV))
    assert y.shape == (N, H, W, Ci)
    assert rel(y, ref) < 1e-5
    b = _rand(Ci, seed=6)
    yb = S.s2t_conv(z.to(DEV), Wt.to(DEV), bias=b.to(DEV), act=S.ACT_LRELU, slope=0.2)
    assert rel(yb, TF.leaky_relu(ref + b.double(), 0.2)) < 1e-5


@pytest.mark.parametrize("N,H,W,Ci,Co", SHAPES)
def test_s2_wgrad(N, H, W, Ci, Co):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Ci, seed=7)
    g = _rand(N, H // 2, W // 2, Co, seed=8)
    Wt = torch.zeros(Co, Ci, 4, 4, dtype=torch.float64, requires_grad=True)
    y = TF.conv2d(x.double().permute(0, 3, 1, 2), Wt, stride=2, padding=1)
    (ref,) = torch.autograd.grad((y * g.double().permute(0, 3, 1, 2)).sum(), Wt)
    ref = ref.permute(0, 2, 3, 1).reshape(Co, 16 * Ci)
    dW = S.s2_wgrad(x.to(DEV), g.to(DEV))
    assert rel(dW, ref) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_resample2x(dt):
    from rafiki_amd.ops import f32 as S
    x = _rand(3, 6, 10, 12, seed=9).to(dt)
    up = S.upscale2x(x.to(DEV), scale=0.5)
    ref_up = x.double().repeat_interleave(2, 1).repeat_interleave(2, 2) * 0.5
    assert up.dtype == dt and rel(up, ref_up) < (1e-6 if dt == torch.float32 else 1e-2)
    dn = S.downscale2x(x.to(DEV))
    ref_dn = TF.avg_pool2d(x.double().permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    assert rel(dn, ref_dn) < (1e-6 if dt == torch.float32 else 1e-2)
