"""Multi-segment optimizer / zeroing / finite-check launches (loss_optim.hip adam_multi_kernel, zero_multi,
nonfinite_multi): one launch over a set of arena ranges gives bit-identical results to one launch per range
(the PG-GAN live ranges, per-layer equalized-LR multipliers), and leaves everything outside the ranges alone."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _flat():
    from rafiki_amd.engine.flat import FlatParams, init_const
    f = FlatParams(torch.device(DEV))
    for i, n in enumerate((70000, 33, 4096, 517, 123457, 8)):
        f.add('p{}'.format(i), (n,), init_const(0.5 + 0.1 * i), decay=i % 2 == 0, lr_mult=1.0 + 0.37 * i)
    f.build()
    g = torch.Generator().manual_seed(0)
    f.master.copy_(torch.randn(f.master.shape, generator=g).to(DEV))
    f.grad.copy_(torch.randn(f.grad.shape, generator=g).to(DEV))
    return f


def test_adam_multi_matches_per_segment_launches():
    from rafiki_amd.engine.flat import FlatAdam
    from rafiki_amd.ops import functional as F
    out = []
    for multi in (False, True):
        f = _flat()
        opt = FlatAdam(f, 1e-3, betas=(0.0, 0.99), eps=1e-8, weight_decay=1e-4)
        opt.skip_flag = torch.zeros(1, dtype=torch.int32, device=DEV)
        specs = {s.name: s for s in f.specs}
        live = f.ranges_of(['p0', 'p1', 'p4', 'p5'])
        if not multi:   # the per-segment path: hide the table builder
            opt._seg_tables = {}
            orig = F.seg_table_ok
            F.seg_table_ok = lambda segs: False
        try:
            for _ in range(3):
                opt.step(live=live)
        finally:
            if not multi:
                F.seg_table_ok = orig
        torch.cuda.synchronize()
        assert (multi and opt.__dict__.get('_seg_tables')) or not multi
        out.append((f.master.clone(), opt.m.clone(), opt.v.clone(), specs))
    (w0, m0, v0, sp), (w1, m1, v1, _) = out
    assert torch.equal(w0, w1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    # the ranges left out are untouched (p2, p3: zero moments)
    for n in ('p2', 'p3'):
        a, b = sp[n].offset, sp[n].offset + sp[n].numel
        assert torch.count_nonzero(m1[a:b]) == 0


def test_zero_and_nonfinite_multi():
    from rafiki_amd.ops import functional as F
    f = _flat()
    live = f.ranges_of(['p0', 'p1', 'p4'])
    tab = F.SegTable(f.device, live)
    before = f.grad.clone()
    F.zero_multi(f.grad, tab)
    mask = torch.zeros_like(f.grad, dtype=torch.bool)
    for a, b in live:
        mask[a:b] = True
    torch.cuda.synchronize()
    assert torch.count_nonzero(f.grad[mask]) == 0 and torch.equal(f.grad[~mask], before[~mask])
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    F.nonfinite_multi(f.grad, tab, flag)
    assert int(flag.item()) == 0
    a, b = live[-1]
    f.grad[b - 1] = float('nan')     # the last element of the last range
    F.nonfinite_multi(f.grad, tab, flag)
    assert int(flag.item()) == 1
    flag.zero_()
    f.grad[b - 1] = 0.0
    s2 = f.specs[2]
    f.grad[s2.offset] = float('inf')  # outside the ranges: not seen
    F.nonfinite_multi(f.grad, tab, flag)
    assert int(flag.item()) == 0


def test_lerp_multi_matches_lerp():
    """lerp_multi_kernel: the Gs EMA over chunk-table ranges, bit-identical to lerp_ on those ranges (fp32
    and the bf16 copy), everything outside untouched."""
    from rafiki_amd.ops import functional as F
    f = _flat()
    g = torch.Generator().manual_seed(3)
    dst = torch.randn(f.master.shape, generator=g).to(DEV)
    live = f.ranges_of(['p0', 'p1', 'p4'])
    tab = F.SegTable(f.device, live)
    a, ab = dst.clone(), torch.zeros(dst.shape, dtype=torch.bfloat16, device=DEV)
    b, bb = dst.clone(), ab.clone()
    F.lerp_multi(a, f.master, 0.99, tab, dst_bf16=ab)
    for lo, hi in live:
        F.lerp_(b[lo:hi], f.master[lo:hi], 0.99, dst_bf16=bb[lo:hi])
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(ab, bb)


def test_pg_gan_trimmed_gs_ema_bit_identical():
    """PgGan._update_Gs at lod 3 (only the G ranges Adam stepped, one multi-segment launch) == the whole-arena
    EMA, bit for bit: outside those ranges G - Gs is exactly zero.  A restored state falls back to the full
    EMA (its Gs may differ from G anywhere)."""
    from rafiki_amd.models.pg_gan import PgGan
    from rafiki_amd.ops import functional as F
    from rafiki_amd.parallel.context import TrialContext, use_context
    with use_context(TrialContext(device=torch.device(DEV))):
        m = PgGan(D_repeats=1, minibatch_base=16)
        m._build([1, 32, 32], 0)
    nets = m.nets
    m.set_lod_live(3.0)
    rng = nets.G.ranges_of(sorted(nets.gs_moved))
    assert sum(b - a for a, b in rng) < nets.G.master.numel() // 2
    gen = torch.Generator().manual_seed(5)
    for _ in range(3):
        for a, b in m._live[id(nets.G)]:      # what Adam changes at this LOD
            nets.G.master[a:b] += 1e-3 * torch.randn(b - a, generator=gen).to(DEV)
        ref = nets.Gs_master.clone()
        F.lerp_(ref, nets.G.master, 0.99)     # the whole-arena EMA
        m._update_Gs(0.99)
        torch.cuda.synchronize()
        assert torch.equal(nets.Gs_master, ref)
    assert any(k[1] == 'Gs' for k in m._seg_tables) or len(rng) == 1
    nets.load_state(nets.state())
    assert nets.gs_moved is None


def test_pg_gan_fused_flag_and_counter_bitwise(monkeypatch):
    """The finite-check flag zeroed by the gradient-zeroing launch, the Adam step counter advanced by the
    finite-check launch and the random stream's counter by the Adam launch (PgGan._zero_grad / _finite_guard /
    _apply) give the same weights, bit for bit, as the per-range launches with their own zeroing and counter
    kernels; every counter advances once per step."""
    from rafiki_amd.engine.flat import FlatAdam
    from rafiki_amd.models.pg_gan import PgGan, TrialRng
    from rafiki_amd.ops import functional as F
    from rafiki_amd.parallel.context import TrialContext, use_context
    out = []
    for multi in (True, False):
        monkeypatch.setattr(F, 'MULTISEG', multi)
        with use_context(TrialContext(device=torch.device(DEV))):
            m = PgGan(D_repeats=1, minibatch_base=16)
            m._build([1, 32, 32], 0)
        nets = m.nets
        G_opt = FlatAdam(nets.G, 1e-3, betas=(0.0, 0.99))
        D_opt = FlatAdam(nets.D, 1e-3, betas=(0.0, 0.99))
        for o in (G_opt, D_opt):
            o.skip_flag = torch.zeros(1, dtype=torch.int32, device=DEV)
        rng = TrialRng(torch.device(DEV), 0)
        level = torch.randint(0, 256, (64, 1, 4, 4), dtype=torch.uint8, generator=torch.Generator().manual_seed(1))
        acc = torch.zeros(6, device=DEV)
        m.set_lod_live(3.0)
        for _ in range(3):
            m.train_round(3.0, 16, level.to(DEV), torch.zeros((64, 0), device=DEV), rng, G_opt, D_opt, acc)
        torch.cuda.synchronize()
        assert int(G_opt.t.item()) == 3 and int(D_opt.t.item()) == 3
        assert int(rng.step.item()) == 6     # advanced once per optimizer step (by the Adam launch when fused)
        assert int(G_opt.skip_flag.item()) == 0 and int(D_opt.skip_flag.item()) == 0
        out.append((nets.G.master.clone(), nets.D.master.clone(), nets.Gs_master.clone()))
    (g1, d1, s1), (g0, d0, s0) = out
    assert torch.equal(g1, g0) and torch.equal(d1, d0) and torch.equal(s1, s0)
