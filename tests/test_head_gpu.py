"""Fused classifier head (csrc/kernels/head.hip) vs fp64 PyTorch: output layer + softmax cross-entropy +
d(logits) + gated d(hidden) (rk_head_fwd_bwd) and the output weight / bias and hidden bias gradients
(rk_head_dw), fp32 gated at 1e-5 relative Frobenius error."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("B,D,NC,ncls,gated", [(256, 512, 16, 10, True), (37, 96, 8, 5, True),
                                               (64, 2048, 32, 20, False), (5, 32, 16, 16, True)])
def test_head_matches_fp64(B, D, NC, ncls, gated):
    from rafiki_amd.ops import f32 as S
    g = torch.Generator().manual_seed(B + D)
    z = torch.randn(B, D, generator=g)
    if gated:
        z = torch.relu(z)
    w = torch.randn(NC, D, generator=g) * D ** -0.5
    w[ncls:] = 0.0
    b = torch.randn(NC, generator=g) * 0.1
    b[ncls:] = 0.0
    y = torch.randint(0, ncls, (B,), generator=g, dtype=torch.int32)
    dlog = torch.full((B, NC), float('nan'), device=DEV)
    dz = torch.full((B, D), float('nan'), device=DEV)
    loss = torch.zeros(1, device=DEV)
    corr = torch.zeros(1, dtype=torch.int32, device=DEV)
    seen = torch.zeros(1, dtype=torch.int32, device=DEV)
    zd, wd, bd = z.to(DEV), w.to(DEV), b.to(DEV)
    S.head_fwd_bwd(zd, wd, bd, y.to(DEV), ncls, dlogits=dlog, dz=dz, gated=gated, loss_sum=loss, correct=corr,
                   counted=seen)
    dw = torch.full((NC, D), float('nan'), device=DEV)
    db = torch.full((NC,), float('nan'), device=DEV)
    dbh = torch.full((D,), float('nan'), device=DEV)
    S.head_dw(zd, dlog, dz, dw=dw, db=db, dbh=dbh)
    torch.cuda.synchronize()
    # fp64 reference
    z64 = z.double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    b64 = b.double().requires_grad_(True)
    logits = (z64 @ w64.t() + b64)[:, :ncls]
    lo = TF.cross_entropy(logits, y.long())
    gz, gw, gb = torch.autograd.grad(lo, [z64, w64, b64])
    if gated:
        gz = gz * (z.double() > 0)
    ref_dlog = torch.zeros(B, NC, dtype=torch.float64)
    ref_dlog[:, :ncls] = (torch.softmax(logits.detach(), 1) - TF.one_hot(y.long(), ncls)) / B
    assert rel(dlog, ref_dlog) < 1e-5
    assert rel(dz, gz) < 1e-5
    assert rel(dw, gw) < 1e-5 and rel(db, gb) < 1e-5
    assert rel(dbh, gz.sum(0)) < 1e-5
    assert abs(loss.item() / B - lo.item()) < 1e-5 * max(1.0, lo.item())
    assert corr.item() == int((logits.argmax(1) == y.long()).sum()) and seen.item() == B
