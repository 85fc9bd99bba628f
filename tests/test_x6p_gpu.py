"""Pre-split X6 GEMMs (csrc/kernels/x6p.hip) and their plane producers (winograd4.hip) vs fp64 PyTorch.

The X6 products are fp32-accurate (the three bf16 pieces represent every operand to 2^-26 and the dropped
piece products are below 2^-25 of |xy|), so the plain GEMM is gated at the fp32 GEMM's own error scale
(2e-6 relative Frobenius against fp64) and the Winograd paths at test_winograd4_gpu.py's 3e-5 (F(4x4)'s
transform round-off, which is the same with either GEMM)."""
import math

import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = 'cuda'
TOL = 3e-5


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).float()


def test_split_planes_sum_back_exactly():
    from rafiki_amd.ops import f32 as S
    x = torch.cat([_rand(64, 96, seed=1), _rand(64, 96, seed=2) * 1e-20, _rand(64, 96, seed=3) * 1e20])
    p = S.x6p_split(x.to(DEV)).cpu()
    assert p.shape == (3, 192, 96) and p.dtype == torch.bfloat16
    back = p[0].double() + p[1].double() + p[2].double()
    err = ((back - x.double()).abs() / x.double().abs().clamp_min(1e-38)).max().item()
    assert err < 2 ** -23, err


@pytest.mark.parametrize("G,M,N,K", [(1, 256, 256, 256), (3, 100, 72, 64), (4, 256, 512, 512), (2, 33, 130, 96),
                                     (5, 1, 64, 32)])
@pytest.mark.parametrize("tile", range(13))
@pytest.mark.parametrize("nst", [2, 3])
def test_x6p_gemm_vs_fp64(G, M, N, K, tile, nst):
    from rafiki_amd.ops import f32 as S
    if nst == 3 and tile not in S.XP_NST3:
        pytest.skip('8-wave tiles ring two stages only')
    a = _rand(G, M, K, seed=10 + tile)
    b = _rand(G, N, K, seed=20 + nst)
    ap = torch.stack([S.x6p_split(a[g].to(DEV)) for g in range(G)]).contiguous()
    bp = torch.stack([S.x6p_split(b[g].to(DEV)) for g in range(G)]).contiguous()
    out = torch.full((G, M, N), float('nan'), device=DEV)
    S.x6p_gemm(ap, bp, out, M, N, K, groups=G, tile=tile, nst=nst)
    prev = _rand(G, M, N, seed=30).to(DEV)
    acc = prev.clone()
    S.x6p_gemm(ap, bp, acc, M, N, K, groups=G, tile=tile, nst=nst, accumulate=True)
    torch.cuda.synchronize()
    ref = torch.einsum('gmk,gnk->gmn', a.double(), b.double())
    assert rel(out, ref) < 2e-6
    assert rel(acc, ref + prev.double().cpu()) < 2e-6


@pytest.mark.parametrize("splits", [2, 3, 4])
@pytest.mark.parametrize("tile", [0, 3, 7, 9, 12])
def test_x6p_gemm_split_k_slabs(splits, tile):
    from rafiki_amd.ops import f32 as S
    G, M, N, K = 3, 96, 160, 224
    a = _rand(G, M, K, seed=3)
    b = _rand(G, N, K, seed=4)
    ap = torch.stack([S.x6p_split(a[g].to(DEV)) for g in range(G)]).contiguous()
    bp = torch.stack([S.x6p_split(b[g].to(DEV)) for g in range(G)]).contiguous()
    s = S.x6p_splits(K, splits)
    out = torch.full((s, G, M, N), float('nan'), device=DEV)
    S.x6p_gemm(ap, bp, out, M, N, K, groups=G, tile=tile, nst=2, splits=s)
    torch.cuda.synchronize()
    ref = torch.einsum('gmk,gnk->gmn', a.double(), b.double())
    assert rel(out.sum(0), ref) < 2e-6


def test_x6p_gemm_rejects_bad_k():
    from rafiki_amd.ops import _lib
    from rafiki_amd.ops import f32 as S
    a = torch.zeros((3, 64, 40), dtype=torch.bfloat16, device=DEV)
    out = torch.zeros((64, 64), device=DEV)
    with pytest.raises(_lib.KernelError):
        S.x6p_gemm(a, a, out, 64, 64, 40)


def _w2(w):
    return w.to(DEV).reshape(w.shape[0], -1).contiguous()


def _planes(w, dgrad=False):
    from rafiki_amd.ops import _lib
    from rafiki_amd.ops import f32 as S
    Co, Ci = w.shape[0], w.numel() // (9 * w.shape[0])
    out = torch.empty((36, 3, Ci, Co) if dgrad else (36, 3, Co, Ci), dtype=torch.bfloat16, device=DEV)
    _lib.call("rk_x6p_w4_weights", S._p(_w2(w)), None if dgrad else S._p(out), S._p(out) if dgrad else None,
              Co, Ci, S._s())
    return out


def test_weight_planes_match_fp32_sets():
    from rafiki_amd.ops import f32 as S
    w = _rand(96, 3, 3, 64, seed=5, scale=0.1)
    for dgrad in (False, True):
        p = _planes(w, dgrad).double()
        ref = (S.wino4_ut(_w2(w)) if dgrad else S.wino4_u(_w2(w))).double()
        assert rel(p[:, 0] + p[:, 1] + p[:, 2], ref) < 1e-7


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(8, 4, 4, 512, 512), (3, 8, 8, 256, 96), (16, 8, 8, 64, 128),
                                            (2, 16, 16, 32, 64), (1, 4, 4, 64, 64)])
@pytest.mark.parametrize("tile,splits", [(0, 1), (3, 1), (4, 1), (0, 2), (7, 4), (9, 1), (10, 2)])
def test_wino4_conv_pt_planes_fwd_stats_bias_relu(N, H, W, Cin, Cout, tile, splits):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=50)
    w = _rand(Cout, 3, 3, Cin, seed=51, scale=1.0 / math.sqrt(9 * Cin))
    up = _planes(w)
    acc = torch.zeros((S.bn_slots(Cout), 2, Cout), dtype=torch.float64, device=DEV)
    y = S.wino4_conv_pt(x.to(DEV), up, stats=acc, tile=tile, nst=2, splits=splits)
    b = _rand(Cout, seed=52)
    yb = S.wino4_conv_pt(x.to(DEV), up, bias=b.to(DEV), relu=True, tile=tile, nst=3 if tile in S.XP_NST3 else 2,
                         splits=splits)
    torch.cuda.synchronize()
    ref = TF.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert rel(y, ref) < TOL
    s = acc.sum(0).cpu()
    r = ref.reshape(-1, Cout)
    assert rel(s[0], r.sum(0)) < TOL and rel(s[1], (r * r).sum(0)) < TOL
    assert rel(yb, torch.relu(ref + b.double())) < TOL


@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("H", [8, 4])
def test_wino4_conv_pt_planes_bn_epilogues(pool, H):
    """BNB / BNP data-gradient epilogues of the plane path == the fused kernel's."""
    from rafiki_amd.ops import f32 as S
    N, W, Cin, Cout = 4, H, 64, 128
    Hy, Wy = (2 * H, 2 * W) if pool else (H, W)
    y = _rand(N, Hy, Wy, Cin, seed=57) + 0.2
    gamma, beta = torch.ones(Cin) * 1.3, _rand(Cin, seed=58) * 0.1
    acc = torch.zeros((S.bn_slots(Cin), 2, Cin), dtype=torch.float64, device=DEV)
    S.col_stats(y.to(DEV).view(-1, Cin), acc)
    _, coeffs = S.bn_fwd(y.to(DEV), acc, N * Hy * Wy, gamma.to(DEV), beta.to(DEV), 1e-5, pool=pool, act=1)
    w = _rand(Cout, 3, 3, Cin, seed=59, scale=0.05)
    ut = S.wino4_ut(_w2(w))
    utp = _planes(w, dgrad=True)
    dyo = _rand(N, H, W, Cout, seed=60).to(DEV)
    acc_f, acc_p = torch.zeros_like(acc), torch.zeros_like(acc)
    key = 'bnp' if pool else 'bnb'
    d_f = S.wino4_conv(dyo, ut, **{key: (y.to(DEV), coeffs, acc_f)})
    d_p = S.wino4_conv_pt(dyo, utp, **{key: (y.to(DEV), coeffs, acc_p)}, tile=0, splits=2)
    torch.cuda.synchronize()
    assert rel(d_p, d_f) < TOL
    assert rel(acc_p.sum(0), acc_f.sum(0)) < TOL


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(16, 8, 8, 64, 128), (32, 4, 4, 256, 128), (8, 16, 16, 32, 64),
                                            (64, 4, 4, 40, 36)])
@pytest.mark.parametrize("tile,splits", [(0, 1), (3, 1), (5, 1), (8, 2), (0, 4), (11, 1), (9, 4)])
def test_wino4_wgrad_pt_planes(N, H, W, Cin, Cout, tile, splits):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=40)
    dy = _rand(N, H, W, Cout, seed=41)
    dw = torch.empty(Cout, 9 * Cin, device=DEV)
    S.wino4_wgrad_pt(dy.to(DEV), x.to(DEV), dw, tile=tile, nst=2, planes=True, splits=splits)
    prev = _rand(Cout, 9 * Cin, seed=42).to(DEV)
    acc = prev.clone()
    S.wino4_wgrad_pt(dy.to(DEV), x.to(DEV), acc, accumulate=True, tile=tile, nst=3 if tile in S.XP_NST3 else 2, planes=True,
                     splits=splits)
    torch.cuda.synchronize()
    wd = torch.zeros(Cout, Cin, 3, 3, dtype=torch.float64, requires_grad=True)
    out = TF.conv2d(x.double().permute(0, 3, 1, 2), wd, padding=1)
    (gw,) = torch.autograd.grad(out, wd, dy.double().permute(0, 3, 1, 2))
    ref = gw.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)
    assert rel(dw, ref) < TOL
    assert rel(acc, ref + prev.double().cpu()) < TOL


def test_conv_fwd_tuner_offers_and_runs_plane_path():
    """The autotuned conv offers the plane candidates and every one of them runs and agrees."""
    from rafiki_amd.ops import f32 as S
    N, H, Cin, Cout = 16, 8, 128, 256
    x = _rand(N, H, H, Cin, seed=70).to(DEV)
    w = _rand(Cout, 3, 3, Cin, seed=71, scale=0.05)
    up = _planes(w)
    ref = S.conv_fwd(x, _w2(w))
    for cfg in S.WINO4_PTX_CFGS:
        y = torch.full_like(ref, float('nan'))
        S.wino4_conv_pt(x, up, out=y, tile=cfg[1] // 4, nst=cfg[1] % 4, splits=cfg[2])
        assert rel(y, ref) < TOL, cfg


@pytest.mark.parametrize("N,H,Cin,Cout", [(8, 4, 520, 512), (4, 8, 256, 128), (2, 32, 64, 64)])
def test_wino4_conv_pt_lrelu_epilogue(N, H, Cin, Cout, monkeypatch):
    """bias + leaky-ReLU epilogue of the pre-transformed F(4x4) output transform (PG-GAN D convs): the fp32-U
    path and, where K % 32 == 0, the X6 plane path, against fp64; and every tuner candidate of conv_fwd with
    act = leaky ReLU (the direct GEMMs and the PT paths) agrees."""
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, H, Cin, seed=80)
    w = _rand(Cout, 3, 3, Cin, seed=81, scale=1.0 / math.sqrt(9 * Cin))
    b = _rand(Cout, seed=82)
    ref = TF.leaky_relu(TF.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), padding=1)
                        .permute(0, 2, 3, 1) + b.double(), 0.2)
    xd, bd = x.to(DEV), b.to(DEV)
    y = S.wino4_conv_pt(xd, S.wino4_u(_w2(w)), bias=bd, lrelu=0.2, tile=0, nst=2)
    assert rel(y, ref) < TOL
    if Cin % 32 == 0:
        yp = S.wino4_conv_pt(xd, S.wino4_u4p(_w2(w)), bias=bd, lrelu=0.2, tile=0, nst=2)
        assert rel(yp, ref) < TOL
        assert rel(S.wino4_u4p(_w2(w), dgrad=True).double().sum(1), S.wino4_ut(_w2(w)).double()) < 1e-7
    seen = {}

    def grab(key, cands, run, protect=()):
        seen['cands'], seen['run'] = list(cands), run
        return cands[0]
    monkeypatch.setattr(S, '_pick', grab)
    yy = torch.full((N, H, H, Cout), float('nan'), device=DEV)
    S.conv_fwd(xd, _w2(w), bias=bd, act=S.ACT_LRELU, slope=0.2, out=yy, wino4=lambda: S.wino4_u(_w2(w)),
               wino4p=lambda: S.wino4_u4p(_w2(w)))
    pt = [c for c in seen['cands'] if c[0] in (S.WINO4_PT, S.WINO4_PTX)]
    assert any(c[0] == S.WINO4_PT for c in pt) and (Cin % 32 or any(c[0] == S.WINO4_PTX for c in pt))
    for cfg in pt[:3] + pt[-2:] + [seen['cands'][0]]:
        yy.fill_(float('nan'))
        seen['run'](cfg)
        torch.cuda.synchronize()
        assert rel(yy, ref) < TOL, cfg
