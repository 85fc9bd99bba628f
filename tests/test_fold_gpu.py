"""Split-K / column-sum fold over more than 16 slabs (loss_optim.hip fold_rows_kernel, one block-cooperative
pass): against an fp64 sum of the same fp32 slabs, with scale / accumulate, run-to-run bitwise identical,
and equal within fp32 round-off to the two-pass rows_reduce + reduce_slabs path it replaces."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.mark.parametrize("S,n", [(17, 256), (40, 1000), (128, 4 * 4608), (384, 512), (300, 12), (33, 260),
                                 (128, 36864)])
@pytest.mark.parametrize("acc", [False, True])
def test_fold_rows_vs_fp64(S, n, acc, monkeypatch):
    from rafiki_amd.ops import functional as F
    g = torch.Generator().manual_seed(S * 7 + n)
    slab = torch.randn(S, n, generator=g).to(DEV)
    base = torch.randn(n, generator=g).to(DEV)
    got = F.reduce_slabs(slab, base.clone(), accumulate=acc, scale=0.37)
    again = F.reduce_slabs(slab, base.clone(), accumulate=acc, scale=0.37)
    monkeypatch.setattr(F, 'FOLD_ROWS', False)
    two = F.reduce_slabs(slab, base.clone(), accumulate=acc, scale=0.37)
    torch.cuda.synchronize()
    ref = slab.double().sum(0) * 0.37 + (base.double() if acc else 0)
    tol = 4 * S * 2 ** -24 * slab.abs().max().item()
    assert (got.double() - ref).abs().max().item() <= tol
    assert (two.double() - ref).abs().max().item() <= tol
    assert torch.equal(got, again)
