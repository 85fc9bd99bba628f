"""The X6 K loop of sgemm.hip (fp32 operands split into three bf16 pieces, six
v_mfma_f32_32x32x16_bf16 per 16-deep chunk) against fp64 PyTorch references of the same fp32
inputs, side by side with the v_mfma_f32_32x32x2_f32 loop of the same tile: the split must be as
accurate as the native fp32 matrix instruction (relative Frobenius error within 2x of it, and
< 1e-5), on every operand mode (conv gathers, K-inner / K-outer dense, split-K slabs,
table-driven resampling gathers, grouped launches)."""
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


def _both(run, ref):
    """run(tile) -> output tensor; returns (err f32 loop, err X6 loop) for tiles 0..3."""
    from rafiki_amd.ops import f32 as S
    out = []
    for t in (0, 3, 8, 9, 10):   # 8-10: the 1- / 2-wave tiles
        e32 = rel(run(t), ref)
        e6 = rel(run(t + S.X6), ref)
        out.append((t, e32, e6))
    return out


def _check(errs):
    for t, e32, e6 in errs:
        assert e6 < 1e-5 and e6 <= 2.0 * e32 + 2e-8, (t, e32, e6)


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(4, 8, 8, 64, 128), (2, 16, 16, 32, 64), (3, 6, 6, 12, 24)])
def test_x6_conv_fwd(N, H, W, Cin, Cout):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=1)
    w = _rand(Cout, 3, 3, Cin, seed=2, scale=1.0 / math.sqrt(9 * Cin))
    ref = TF.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    xd, wd = x.to(DEV), w.to(DEV)
    M, K = N * H * W, 9 * Cin

    def run(tile):
        y = torch.empty(N, H, W, Cout, device=DEV)
        S.sgemm(S.KIND_CONV, xd, wd, y, M, Cout, K, Cin, K, Cout, tile=tile, nst=2, H=H, W=W, C=Cin, taps=9)
        torch.cuda.synchronize()
        return y
    _check(_both(run, ref))


@pytest.mark.parametrize("splits", [1, 4])
def test_x6_conv_wgrad(splits):
    from rafiki_amd.ops import f32 as S
    N, H, W, Cin, Cout = 4, 16, 16, 64, 64
    x = _rand(N, H, W, Cin, seed=3)
    dy = _rand(N, H, W, Cout, seed=4)
    xd = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    wd = torch.zeros(Cout, Cin, 3, 3, dtype=torch.float64, requires_grad=True)
    y = TF.conv2d(xd, wd, padding=1)
    (gw,) = torch.autograd.grad(y, wd, dy.double().permute(0, 3, 1, 2))
    ref = gw.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)
    X, D = x.to(DEV), dy.to(DEV)
    M, Nn, K = Cout, 9 * Cin, N * H * W

    def run(tile):
        out = torch.empty(M, Nn, device=DEV)
        if splits == 1:
            S.sgemm(S.KIND_WGRAD, D, X, out, M, Nn, K, Cout, Cin, Nn, tile=tile, nst=2, H=H, W=W, C=Cin, taps=9)
        else:
            slab = torch.empty(splits, M, Nn, device=DEV)
            S.sgemm(S.KIND_WGRAD, D, X, slab, M, Nn, K, Cout, Cin, Nn, tile=tile, nst=2, splits=splits,
                    slab_stride=M * Nn, H=H, W=W, C=Cin, taps=9)
            S.reduce_slabs(slab, out)
        torch.cuda.synchronize()
        return out
    _check(_both(run, ref))


@pytest.mark.parametrize("kind", ["dense", "dx", "dw"])
def test_x6_dense(kind):
    from rafiki_amd.ops import f32 as S
    M, N, K = 200, 96, 520
    if kind == "dense":    # A [M][K] . B [N][K]^T
        A, B = _rand(M, K, seed=5), _rand(N, K, seed=6)
        ref = A.double() @ B.double().t()
        args = (S.KIND_DENSE, M, N, K, K, K, N)
    elif kind == "dx":     # A [M][K] . B [K][N]
        A, B = _rand(M, K, seed=7), _rand(K, N, seed=8)
        ref = A.double() @ B.double()
        args = (S.KIND_DENSE_DX, M, N, K, K, N, N)
    else:                  # A [K][M]^T . B [K][N]
        A, B = _rand(K, M, seed=9), _rand(K, N, seed=10)
        ref = A.double().t() @ B.double()
        args = (S.KIND_DENSE_DW, M, N, K, M, N, N)
    Ad, Bd = A.to(DEV), B.to(DEV)

    def run(tile):
        out = torch.empty(M, N, device=DEV)
        S.sgemm(args[0], Ad, Bd, out, *args[1:], tile=tile, nst=2)
        torch.cuda.synchronize()
        return out
    _check(_both(run, ref))


def test_x6_large_k_accumulation():
    """K = 9 x 512 (VGG-small's deepest conv): the accumulation error dominates both loops alike."""
    from rafiki_amd.ops import f32 as S
    M, N, K = 256, 128, 4608
    A, B = _rand(M, K, seed=11), _rand(N, K, seed=12)
    ref = A.double() @ B.double().t()
    Ad, Bd = A.to(DEV), B.to(DEV)

    def run(tile):
        out = torch.empty(M, N, device=DEV)
        S.sgemm(S.KIND_DENSE, Ad, Bd, out, M, N, K, K, K, N, tile=tile, nst=2)
        torch.cuda.synchronize()
        return out
    _check(_both(run, ref))


def test_x6_wide_dynamic_range():
    """Operands spanning 2^-40 .. 2^40 per element: the pieces keep fp32's exponent range."""
    from rafiki_amd.ops import f32 as S
    M, N, K = 128, 64, 256
    g = torch.Generator().manual_seed(13)
    A = torch.randn(M, K, generator=g) * torch.exp2(torch.randint(-40, 40, (M, K), generator=g).float())
    B = torch.randn(N, K, generator=g)
    ref = A.double() @ B.double().t()
    Ad, Bd = A.to(DEV), B.to(DEV)

    def run(tile):
        out = torch.empty(M, N, device=DEV)
        S.sgemm(S.KIND_DENSE, Ad, Bd, out, M, N, K, K, K, N, tile=tile, nst=2)
        torch.cuda.synchronize()
        return out
    _check(_both(run, ref))


def test_x6_resampling_gather(monkeypatch):
    """The PG-GAN stride-2 4x4 conv (table-driven gather, kind 6) on both K loops."""
    from rafiki_amd.ops import f32 as S
    Nb, H, Ci, Co = 4, 16, 32, 64
    x = _rand(Nb, H, H, Ci, seed=14)
    Wt = _rand(Co, 4, 4, Ci, seed=15, scale=0.1)
    w4 = Wt.double().permute(0, 3, 1, 2)
    ref = TF.conv2d(x.double().permute(0, 3, 1, 2), w4, stride=2, padding=1).permute(0, 2, 3, 1)
    xd, wd = x.to(DEV), Wt.reshape(Co, 16 * Ci).to(DEV)

    def run(tile):
        monkeypatch.setattr(S, '_pick', lambda key, cands, run, protect=(): (tile, 2, 1))   # force the K loop
        y = S.s2_conv(xd, wd)
        torch.cuda.synchronize()
        return y
    _check(_both(run, ref))
