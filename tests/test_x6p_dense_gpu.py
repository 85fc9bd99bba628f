"""Pre-split X6 dense candidates (ops/f32.py XPD_CFGS: x6p_split / x6p_split_t planes + the x6p GEMM, the
epilogue in sreduce_epi / reduce_slabs) against fp64 PyTorch on the same fp32 inputs: forward with bias and
leaky ReLU, data gradient with a ReLU gate, weight gradient over an unaligned batch (the K padding of the
transposing split) with and without accumulation, unsplit and split-K."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).float().to(DEV)


def _force(monkeypatch, key, cfg):
    from rafiki_amd.ops import autotune
    from rafiki_amd.ops import f32 as S
    monkeypatch.setattr(S, 'XPD_MIN_MACS', 0)
    monkeypatch.setitem(autotune._cache, key, cfg)


def _cfgs():
    from rafiki_amd.ops import f32 as S
    return [c for c in S.XPD_CFGS if c[1] in (0 * 4 + 2, 3 * 4 + 3, 7 * 4 + 2) and c[2] in (1, 4)]


@pytest.mark.parametrize('k', range(6))
def test_x6p_split_t_planes_sum_to_transpose(k):
    from rafiki_amd.ops import f32 as S
    rows, cols = [(100, 70), (64, 64), (1, 5), (33, 129), (512, 96), (200, 8)][k]
    x = _rand(rows, cols, seed=k)
    p = S.x6p_split_t(x)
    assert p.shape == (3, cols, (rows + 31) // 32 * 32)
    s = p[0].double() + p[1].double() + p[2].double()
    assert torch.equal(s[:, rows:].cpu(), torch.zeros_like(s[:, rows:]).cpu())
    assert (s[:, :rows].cpu() - x.double().t().cpu()).abs().max().item() <= 2 ** -24 * x.abs().max().item()


@pytest.mark.parametrize('ci', range(3))
def test_linear_x6p_forward(monkeypatch, ci):
    from rafiki_amd.ops import f32 as S
    cfg = _cfgs()[ci]
    M, K, N = 96, 256, 160
    x, w, b = _rand(M, K, seed=1), _rand(N, K, seed=2, scale=K ** -0.5), _rand(N, seed=3, scale=0.1)
    _force(monkeypatch, ('sl', M, N, K, S.ACT_LRELU, True, 1.0, 'xp'), cfg)
    y = S.linear(x, w, b, act=S.ACT_LRELU, slope=0.2)
    ref = torch.nn.functional.leaky_relu(x.double() @ w.double().t() + b.double(), 0.2)
    assert rel(y, ref) < 2e-6, (cfg, rel(y, ref))


@pytest.mark.parametrize('ci', range(3))
def test_linear_dx_x6p_gated(monkeypatch, ci):
    from rafiki_amd.ops import f32 as S
    cfg = _cfgs()[ci]
    M, Nout, Nin = 72, 128, 200
    dy, w, gate = _rand(M, Nout, seed=4), _rand(Nout, Nin, seed=5), _rand(M, Nin, seed=6)
    _force(monkeypatch, ('sx', M, Nin, Nout, True, 'xp'), cfg)
    dx = S.linear_dx(dy, w, gate=gate)
    ref = (dy.double() @ w.double()) * (gate.double() > 0)
    assert rel(dx, ref) < 2e-6, (cfg, rel(dx, ref))


@pytest.mark.parametrize('ci', range(3))
@pytest.mark.parametrize('acc', [False, True])
def test_linear_dw_x6p_unaligned_batch(monkeypatch, ci, acc):
    from rafiki_amd.ops import f32 as S
    cfg = _cfgs()[ci]
    M, Nout, Nin = 100, 96, 136
    dy, x = _rand(M, Nout, seed=7), _rand(M, Nin, seed=8)
    out = _rand(Nout, Nin, seed=9)
    before = out.clone()
    _force(monkeypatch, ('sdw', M, Nout, Nin, acc, 'xp'), cfg)
    S.linear_dw(dy, x, out=out, accumulate=acc)
    ref = dy.double().t() @ x.double() + (before.double() if acc else 0)
    assert rel(out, ref) < 2e-6, (cfg, acc, rel(out, ref))
