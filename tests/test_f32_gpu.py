"""fp32 kernel path (sgemm.hip: v_mfma_f32_32x32x2_f32; bnf.hip) vs PyTorch references computed in
fp64 from the same fp32 inputs — no bf16 anywhere.  Gate: relative Frobenius error <= 1e-5 per op
(fp32 accumulation over K <= 4608 measures ~1e-7), <= 1e-4 for whole-network gradients."""
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


def _conv_ref(x_nhwc, w_ohwi, taps):
    x = x_nhwc.double().permute(0, 3, 1, 2)
    w = w_ohwi.double().permute(0, 3, 1, 2)
    return TF.conv2d(x, w, padding=1 if taps == 9 else 0).permute(0, 2, 3, 1)


@pytest.mark.parametrize("N,H,W,Cin,Cout,taps", [
    (4, 8, 8, 64, 128, 9), (2, 32, 32, 4, 64, 9), (3, 6, 6, 12, 24, 9), (2, 16, 16, 128, 64, 1),
    (8, 4, 4, 256, 512, 9), (2, 12, 12, 64, 64, 9)])
def test_conv_fwd_and_stats(N, H, W, Cin, Cout, taps):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=1)
    w = _rand(Cout, 3 if taps == 9 else 1, 3 if taps == 9 else 1, Cin, seed=2, scale=1.0 / math.sqrt(Cin * taps))
    acc = torch.zeros((S.bn_slots(Cout), 2, Cout), dtype=torch.float64, device=DEV)
    y = S.conv_fwd(x.to(DEV), w.to(DEV), taps=taps, stats_acc=acc)
    torch.cuda.synchronize()
    ref = _conv_ref(x, w, taps)
    assert rel(y, ref) < 1e-5
    s = acc.sum(0).cpu()
    r = ref.reshape(-1, Cout)
    assert rel(s[0], r.sum(0)) < 1e-5 and rel(s[1], (r * r).sum(0)) < 1e-5


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(4, 8, 8, 64, 128), (2, 16, 16, 64, 64), (8, 4, 4, 512, 256),
                                            (2, 6, 6, 24, 16)])
def test_conv_dgrad_via_transposed_weights(N, H, W, Cin, Cout):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=3)
    w = _rand(Cout, 3, 3, Cin, seed=4, scale=0.1)
    dy = _rand(N, H, W, Cout, seed=5)
    arena = w.reshape(-1).to(DEV).contiguous()
    wt = S.SConvWT(arena, [arena.view(Cout, 3, 3, Cin)])
    wt.refresh()
    dx = S.conv_dgrad(dy.to(DEV), wt.view(0))
    torch.cuda.synchronize()
    xd = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    out = TF.conv2d(xd, w.double().permute(0, 3, 1, 2), padding=1)
    (gx,) = torch.autograd.grad(out, xd, dy.double().permute(0, 3, 1, 2))
    assert rel(dx, gx.permute(0, 2, 3, 1)) < 1e-5


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(4, 8, 8, 64, 128), (2, 32, 32, 4, 64), (16, 4, 4, 256, 512),
                                            (3, 6, 6, 12, 24)])
def test_conv_wgrad(N, H, W, Cin, Cout):
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, W, Cin, seed=6)
    dy = _rand(N, H, W, Cout, seed=7)
    dw = S.conv_wgrad(dy.to(DEV), x.to(DEV))
    torch.cuda.synchronize()
    wd = torch.zeros(Cout, Cin, 3, 3, dtype=torch.float64, requires_grad=True)
    out = TF.conv2d(x.double().permute(0, 3, 1, 2), wd, padding=1)
    (gw,) = torch.autograd.grad(out, wd, dy.double().permute(0, 3, 1, 2))
    assert rel(dw.view(Cout, 3, 3, Cin), gw.permute(0, 2, 3, 1)) < 1e-5


@pytest.mark.parametrize("M,K,N,act", [(256, 2048, 512, 1), (64, 1024, 16, 0), (37, 100, 44, 1), (512, 512, 512, 2)])
def test_dense_fwd_dx_dw(M, K, N, act):
    from rafiki_amd.ops import f32 as S
    x = _rand(M, K, seed=8)
    w = _rand(N, K, seed=9, scale=1.0 / math.sqrt(K))
    b = _rand(N, seed=10)
    y = S.linear(x.to(DEV), w.to(DEV), b.to(DEV), act=act)
    ref = x.double() @ w.double().t() + b.double()
    ref = torch.relu(ref) if act == 1 else TF.leaky_relu(ref, 0.2) if act == 2 else ref
    dy = _rand(M, N, seed=11)
    gate = _rand(M, K, seed=12)
    dx = S.linear_dx(dy.to(DEV), w.to(DEV), gate=gate.to(DEV))
    dw = S.linear_dw(dy.to(DEV), x.to(DEV))
    db = torch.empty(N, device=DEV)
    S.colsum(dy.to(DEV), db)
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-5
    rdx = (dy.double() @ w.double()) * (gate > 0).double()
    assert rel(dx, rdx) < 1e-5
    assert rel(dw, dy.double().t() @ x.double()) < 1e-5
    assert rel(db, dy.double().sum(0)) < 1e-5


def _bn_ref(y, gamma, beta, eps, pool, act):
    y = y.double().permute(0, 3, 1, 2).requires_grad_(True)
    g = gamma.double().requires_grad_(True)
    b = beta.double().requires_grad_(True)
    z = TF.batch_norm(y, None, None, g, b, training=True, eps=eps)
    z = torch.relu(z) if act == 1 else z
    if pool:
        z = TF.max_pool2d(z, 2)
    return y, g, b, z


@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("C", [64, 512])
def test_bn_fwd_bwd(pool, C):
    from rafiki_amd.ops import f32 as S
    N, H, W = 8, 8, 8
    yv = _rand(N, H, W, C, seed=13, scale=2.0) + 0.5
    gamma, beta = _rand(C, seed=14) * 0.5 + 1.0, _rand(C, seed=15) * 0.1
    acc = torch.zeros((S.bn_slots(C), 2, C), dtype=torch.float64, device=DEV)
    S.col_stats(yv.to(DEV).view(-1, C), acc)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    out, coeffs = S.bn_fwd(yv.to(DEV), acc, N * H * W, gamma.to(DEV), beta.to(DEV), 1e-5, rm, rv, 0.1, pool=pool,
                           act=1)
    ys, gs, bs, ref = _bn_ref(yv, gamma, beta, 1e-5, pool, 1)
    assert rel(out, ref.permute(0, 2, 3, 1)) < 1e-5
    var = yv.double().reshape(-1, C).var(0, unbiased=True)
    assert rel(rv, 0.9 + 0.1 * var) < 1e-5
    dout = _rand(*out.shape, seed=16)
    accb = torch.zeros_like(acc)
    dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    dy = S.bn_bwd(dout.to(DEV), yv.to(DEV), coeffs, gamma.to(DEV), accb, pool=pool, act=1, dgamma=dg, dbeta=db)
    torch.cuda.synchronize()
    gy, gg, gb = torch.autograd.grad(ref, [ys, gs, bs], dout.double().permute(0, 3, 1, 2))
    assert rel(dy, gy.permute(0, 2, 3, 1)) < 1e-5
    assert rel(dg, gg) < 1e-5 and rel(db, gb) < 1e-5


@pytest.mark.parametrize("pool", [False, True])
def test_dgrad_epilogue_bn_fusion(pool):
    """conv_dgrad(bnb=/bnp=...) forms the input layer's BN-backward sums in its epilogue: the apply pass
    then must reproduce the unfused bn_bwd exactly (up to fp32 summation order)."""
    from rafiki_amd.ops import f32 as S
    N, H, W, Cin, Cout = 4, 8, 8, 64, 128
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
    dyo = _rand(N, H, W, Cout, seed=20).to(DEV)
    acc_f = torch.zeros_like(acc)
    kw = {'bnp': (y.to(DEV), coeffs, acc_f)} if pool else {'bnb': (y.to(DEV), coeffs, acc_f)}
    d_fused = S.conv_dgrad(dyo, wt.view(0), **kw)
    dy_fused = S.bn_bwd(d_fused, y.to(DEV), coeffs, gamma.to(DEV), acc_f, pool=pool, act=1, reduced=True)
    d_plain = S.conv_dgrad(dyo, wt.view(0))
    acc_p = torch.zeros_like(acc)
    dy_plain = S.bn_bwd(d_plain, y.to(DEV), coeffs, gamma.to(DEV), acc_p, pool=pool, act=1)
    torch.cuda.synchronize()
    assert rel(acc_f.sum(0), acc_p.sum(0)) < 1e-5
    assert rel(dy_fused, dy_plain) < 1e-5


def _engine(**kw):
    from rafiki_amd.engine.convnet import ConvNetEngine
    args = dict(num_classes=10, in_channels=3, image_size=16, cfg=(16, 'M', 32, 32, 'M'), fc_dims=(32,),
                device=DEV, seed=3, lr=0.05, dtype='fp32')
    args.update(kw)
    return ConvNetEngine(**args)


def _batch(B, hw=16, seed=0, c=None):
    if c is None:   # the fp32 engine's input padding: 8 channels with the Winograd stem, else 4
        from rafiki_amd.ops import f32 as S
        c = 8 if S.WINO else 4
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(B, hw, hw, c)
    x[..., :3] = torch.randn(B, hw, hw, 3, generator=g)
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
    return x.to(DEV), y.to(DEV)


def _grad_check(eng, x, y, tol):
    """Engine gradients vs fp64 autograd of the same network.  Gate per parameter: rel <= tol, or — for
    deep nets where a handful of ReLU-sign / max-pool-tie decisions sit within fp32 rounding of the
    boundary and flip (measured: PyTorch's own CPU fp32 is 3.1e-3 off fp64 on VGG-small conv0.w at
    batch 32) — no worse than 2x PyTorch fp32's own error vs fp64 (+1e-5)."""
    eng.forward_backward(x, y)
    torch.cuda.synchronize()
    fl = eng.flat

    def ref_grads(dt):
        params = {n: fl.w(n).detach().to(dt).cpu().clone().requires_grad_(True) for n in fl.names()}
        loss, _ = eng.reference_loss(x.to(dt).cpu(), y.cpu(), params, training=True)
        return loss, torch.autograd.grad(loss, [params[n] for n in fl.names()])
    loss, grads = ref_grads(torch.float64)
    _, grads32 = ref_grads(torch.float32)
    assert abs(eng.loss_sum.item() / x.shape[0] - loss.item()) < 1e-5 * max(1.0, loss.item())
    worst = 0.0
    for n, g, g32 in zip(fl.names(), grads, grads32):
        if g.norm() == 0:
            continue
        e, e32 = rel(fl.g(n), g), rel(g32, g)
        worst = max(worst, e)
        assert e < max(tol, 2.0 * e32 + 1e-5), (n, e, e32)
    return worst


def test_engine_grads_match_fp64_reference():
    """Whole VGG-style step (conv+BN+ReLU+pool, FC, softmax-CE) in fp32 vs fp64 autograd: <= 1e-4."""
    eng = _engine()
    x, y = _batch(64)
    _grad_check(eng, x, y, 1e-4)


@pytest.mark.parametrize("wino", [False, True])
def test_engine_grads_vgg_small_full_width(wino, monkeypatch):
    """Direct convs: 1e-4 (or 2x torch fp32).  With the fused Winograd convs as autotune candidates
    the conv outputs are as accurate (scripts/dev/wino_error.py: 2.6e-7..7.4e-7 vs fp64, direct
    4.2e-7..5.9e-7) but round differently from torch, so a ReLU-boundary sign in the 4x4 layers can
    flip where torch's does not — one flipped element moves a BN dgamma by ~1e-4 relative: gate 1e-3."""
    from rafiki_amd.ops import f32 as S
    monkeypatch.setattr(S, 'WINO', wino)
    eng = _engine(image_size=32, cfg=(64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512, 512, 'M'), fc_dims=(512,))
    x, y = _batch(32, hw=32, seed=1)
    _grad_check(eng, x, y, 1e-3 if wino else 1e-4)


def test_engine_grads_non_pow2_and_odd_pool():
    """48x48 -> 3x3 -> 1x1 (reciprocal gathers, odd pooling: the unfused BN-backward path) and a 36x36
    VGG-small layout whose 9x9 -> 4x4 pool must not take the pooled dgrad fusion."""
    eng = _engine(image_size=48, cfg=(16, 'M', 32, 'M', 32, 'M', 64, 'M', 64, 'M'), fc_dims=(64,))
    x, y = _batch(32, hw=48, seed=7)
    _grad_check(eng, x, y, 1e-4)
    eng = _engine(image_size=36, cfg=(16, 'M', 32, 'M', 32, 'M', 64, 'M'), fc_dims=(32,))
    x, y = _batch(16, hw=36, seed=8)
    _grad_check(eng, x, y, 1e-4)


@pytest.mark.parametrize("wino", [False, True])
def test_engine_no_bn_grads_match_fp64_reference(wino, monkeypatch):
    """bn=False (Keras VGG16's conv3x3 + bias + ReLU blocks, TfVgg16.py:115-130): the fp32 step against
    fp64 autograd, after two steps so the biases are non-zero.  32x32 maps (Winograd paths, pooled and
    pool-free blocks, the dgrad's BNB / BNP epilogues with the constant coefficients) and 48x48 -> 3x3 ->
    1x1 (reciprocal gathers, odd pooling)."""
    from rafiki_amd.ops import f32 as S
    monkeypatch.setattr(S, 'WINO', wino)
    for image_size, cfg, B in ((32, (16, 16, 'M', 32, 32, 'M', 64, 'M'), 32),
                               (48, (16, 'M', 32, 'M', 32, 'M', 64, 'M', 64, 'M'), 16)):
        eng = _engine(image_size=image_size, cfg=cfg, fc_dims=(64,), bn=False, optimizer='adam', lr=1e-3,
                      weight_decay=0.0)
        assert not any(n.endswith(('.gamma', '.beta')) for n in eng.flat.names())
        for i in range(2):
            x, y = _batch(B, hw=image_size, seed=20 + i)
            eng.train_step(x, y)
        assert all(eng.flat.w(b[0] + '.b').abs().sum().item() > 0 for b in eng.blocks)
        eng.reset_metrics()
        # (seed 9 on the 48x48 net with the direct stem puts one stem max-pool window within fp32 rounding of
        # a tie, whose flipped argmax moves conv0.w's gradient by 1.8e-3 while every other gradient and the
        # stem's dy sum stay at 1e-7: scripts/dev/nobn_diag3.py; seed 11 has no such window)
        x, y = _batch(B, hw=image_size, seed=11)
        _grad_check(eng, x, y, 1e-3 if wino else 1e-4)


def test_engine_no_bn_eval_and_grouped_match_reference():
    """bn=False inference: the per-model eval forward (conv without bias + the bias as the folded shift)
    and the grouped ensemble network both match fp64 PyTorch."""
    from rafiki_amd.engine.convnet import GroupedConvNets
    engs = [_engine(image_size=16, bn=False, seed=s) for s in (3, 4)]
    x, y = _batch(64, seed=5)
    for e in engs:
        for _ in range(2):
            e.train_step(x, y)
        e.prepare_eval()
    refs = []
    for e in engs:
        probs = e.forward_eval_graphed(x)
        _, ref_logits = e.reference_loss(x.double().cpu(), None, training=False,
                                         params={n: e.flat.w(n).double().cpu() for n in e.flat.names()})
        refs.append(torch.softmax(ref_logits, 1))
        assert (probs.double().cpu() - refs[-1]).abs().max().item() < 1e-5
    grp = GroupedConvNets(engs)
    out = torch.empty((2, x.shape[0], 10), dtype=torch.float32, device=DEV)
    grp.forward_into(x, out)
    for g in range(2):
        assert (out[g].double().cpu() - refs[g]).abs().max().item() < 1e-5


def test_mlp_input_bn_grads():
    eng = _engine(cfg=(), fc_dims=(64, 64), input_bn=True, optimizer='adam', lr=1e-3, in_channels=1, image_size=28)
    g = torch.Generator().manual_seed(2)
    x = torch.randn(64, eng.feat_dim, generator=g).to(DEV)
    y = torch.randint(0, 10, (64,), generator=g, dtype=torch.int32).to(DEV)
    _grad_check(eng, x, y, 1e-4)


def test_graph_replay_matches_eager_fp32():
    e1, e2 = _engine(), _engine()
    e2.capture(32)
    for i in range(3):
        x, y = _batch(32, seed=i)
        e1.train_step(x, y)
        e2.step_graph(x, y)
    torch.cuda.synchronize()
    assert torch.allclose(e1.flat.master, e2.flat.master, rtol=1e-6, atol=1e-7)
    assert torch.allclose(e1.running, e2.running, rtol=1e-5, atol=1e-7)


def test_scheduled_graph_fp32():
    e1, e2 = _engine(), _engine()
    data, labels = _batch(96, seed=7)
    steps, B = 4, 32
    idx = torch.randint(0, 96, (steps, B), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
    e2.capture_scheduled(data, labels, steps, B)
    e2.set_schedule(idx)
    for i in range(steps):
        e1.train_step(data[idx[i]].contiguous(), labels[idx[i]].contiguous())
        e2.replay()
    torch.cuda.synchronize()
    assert int(e2._ctr.item()) == steps
    assert torch.allclose(e1.flat.master, e2.flat.master, rtol=1e-5, atol=1e-6)


def test_eval_forward_matches_reference():
    eng = _engine()
    x, y = _batch(128, seed=5)
    for _ in range(3):
        eng.train_step(x, y)
    eng.prepare_eval()
    probs = eng.forward_eval_graphed(x)
    _, ref_logits = eng.reference_loss(x.double().cpu(), None, training=False,
                                       params={n: eng.flat.w(n).double().cpu() for n in eng.flat.names()})
    ref = torch.softmax(ref_logits, 1)
    assert (probs.double().cpu() - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("N,H,Cin,Cout,splits", [(1, 4, 512, 512, 16), (2, 2, 256, 512, 8), (1, 8, 128, 256, 4)])
def test_conv_fwd_split_k_small_batch(N, H, Cin, Cout, splits):
    """Inference-sized convs (tiny M, K = 9 x Cin): split-K slabs + the bias/ReLU combine == fp64 conv."""
    from rafiki_amd.ops import f32 as S
    x = _rand(N, H, H, Cin, seed=1).to(DEV)
    w = _rand(Cout, 3, 3, Cin, seed=2, scale=0.05).to(DEV)
    b = _rand(Cout, seed=3, scale=0.1).to(DEV)
    ref = torch.relu(_conv_ref(x.cpu().double(), w.cpu().double(), 9) + b.cpu().double())
    M, K = N * H * H, 9 * Cin
    slab = torch.empty(splits, M, Cout, device=DEV)
    S.sgemm(S.KIND_CONV, x, w, slab, M, Cout, K, Cin, K, Cout, tile=3, nst=2, splits=splits, slab_stride=M * Cout,
            H=H, W=H, C=Cin, taps=9)
    out = torch.empty(N, H, H, Cout, device=DEV)
    S.sreduce_epi(slab, M, Cout, out.view(M, Cout), bias=b, act=S.ACT_RELU)
    assert rel(out.double(), ref) < 1e-5
    y = S.conv_fwd(x, w, bias=b, act=S.ACT_RELU)   # whatever config the autotuner keeps
    assert rel(y.double(), ref) < 1e-5


def test_host_tensor_is_refused_before_launch():
    from rafiki_amd.ops import f32 as S
    with pytest.raises(ValueError, match='host tensor'):
        S.conv_fwd(torch.zeros(1, 4, 4, 32), torch.zeros(32, 3, 3, 32, device=DEV))


def test_prepare_inputs_nhwc_pack():
    eng = _engine(image_size=16)
    imgs = torch.randint(0, 256, (5, 16, 16, 3), dtype=torch.uint8)
    got = eng.prepare_inputs(imgs.to(DEV)).cpu()
    ref = torch.zeros(5, 16, 16, eng.cin_p)
    ref[..., :3] = imgs.float() / 127.5 - 1.0
    assert torch.allclose(got, ref, atol=1e-6)
    got_host = eng.prepare_inputs(imgs.numpy()).cpu()
    assert torch.allclose(got_host, ref, atol=1e-6)


@pytest.mark.parametrize("shared", [True, False])
def test_grouped_conv_linear_bn_match_per_group(shared):
    """rk_sgemm_grp / rk_bnf_eval_grp: k same-shape problems in one launch == k separate launches."""
    from rafiki_amd.ops import f32 as S
    G, Nb, H, Cin, Cout = 3, 2, 8, 32, 64
    x = (_rand(Nb, H, H, Cin, seed=1) if shared else _rand(G, Nb, H, H, Cin, seed=1)).to(DEV)
    W = _rand(G, Cout, 9 * Cin, seed=2, scale=0.05).to(DEV)
    b = _rand(G, Cout, seed=3, scale=0.1).to(DEV)
    y = S.conv_fwd_grp(x, W, bias=b, act=S.ACT_RELU)
    for g in range(G):
        ref = S.conv_fwd(x if shared else x[g].contiguous(), W[g].contiguous(), bias=b[g].contiguous(), act=S.ACT_RELU)
        assert rel(y[g], ref) < 1e-6
    sc, sh = _rand(G, Cout, seed=4).to(DEV), _rand(G, Cout, seed=5).to(DEV)
    z = S.bn_eval_grp(y, sc, sh, pool=True)
    for g in range(G):
        assert rel(z[g], S.bn_eval(y[g].contiguous(), sc[g].contiguous(), sh[g].contiguous(), pool=True)) < 1e-6
    M, K, N = 5, 256, 40
    xa = (_rand(M, K, seed=6) if shared else _rand(G, M, K, seed=6)).to(DEV)
    wl, bl = _rand(G, N, K, seed=7, scale=0.05).to(DEV), _rand(G, N, seed=8).to(DEV)
    o = S.linear_grp(xa, wl, bl, act=S.ACT_RELU)
    for g in range(G):
        ref = torch.relu((xa if shared else xa[g]).double().cpu() @ wl[g].double().cpu().t() + bl[g].double().cpu())
        assert rel(o[g], ref) < 1e-5


@pytest.mark.parametrize("R,C,ld", [(8192, 512, 512), (8192 + 37, 520, 520), (4099, 12, 16), (300, 3, 3),
                                    (65536, 64, 64), (777, 1000, 1004), (5, 256, 256)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_colsum_vectorised_and_scalar_paths(R, C, ld, accumulate):
    """bnf.hip column sums (bias gradients): the float4 kernel (C % 4 == 0, 16-B rows, row chunks + slab
    fold) and the scalar one, strided rows, accumulate — vs fp64."""
    from rafiki_amd.ops import f32 as S
    g = torch.Generator().manual_seed(R + C)
    full = torch.randn(R, ld, generator=g).to(DEV)
    x = full[:, :C]
    base = torch.randn(C, generator=g).to(DEV)
    out = base.clone() if accumulate else torch.empty(C, device=DEV)
    S.colsum(x, out, accumulate=accumulate)
    ref = x.double().sum(0) + (base.double() if accumulate else 0)
    assert rel(out, ref) < 1e-6


@pytest.mark.parametrize("shape", [(512, 4, 4, 512), (64, 8, 8, 256), (37, 3, 5, 12), (9, 7, 7, 3)])
def test_lrelu_gate_colsum_vectorised(shape):
    from rafiki_amd.ops import f32 as S
    g = torch.Generator().manual_seed(sum(shape))
    gy = torch.randn(*shape, generator=g).to(DEV)
    y = torch.randn(*shape, generator=g).to(DEV)
    ref = torch.where(y > 0, gy, gy * 0.2)
    out, cs = S.lrelu_gate_colsum(gy, y, 0.2)
    assert torch.equal(out, ref)
    assert rel(cs, ref.reshape(-1, shape[-1]).double().sum(0)) < 1e-6
    acc = torch.ones(shape[-1], device=DEV)
    _, acc2 = S.lrelu_gate_colsum(gy, y, 0.2, acc=acc)
    assert rel(acc2, ref.reshape(-1, shape[-1]).double().sum(0) + 1) < 1e-6


def test_grouped_ensemble_with_folded_bn_matches_reference():
    """BN engines: the grouped ensemble folds every block's eval BN into its conv (weights x scale, shift
    as the bias, ReLU epilogue; pooled blocks with the 2x2 max-pool written by the fused kernel's
    epilogue) — vs fp64 PyTorch eval and each engine's own (unfolded) eval forward."""
    from rafiki_amd.engine.convnet import GroupedConvNets
    engs = [_engine(image_size=16, cfg=(16, 16, 'M', 32, 32, 'M'), seed=s) for s in (3, 4, 5)]
    x, y = _batch(64, seed=6)
    for e in engs:
        for _ in range(3):
            e.train_step(x, y)
        e.prepare_eval()
    grp = GroupedConvNets(engs)
    assert grp.folded == [True, True, True, True]   # the pooled blocks through the pooled epilogue
    out = torch.empty((3, x.shape[0], 10), dtype=torch.float32, device=DEV)
    grp.forward_into(x, out)
    small = torch.empty((3, 4, 10), dtype=torch.float32, device=DEV)
    grp.forward_into(x[:4].contiguous(), small)   # below POOL_EPILOGUE_MIN_PIXELS: conv + ReLU / max pass
    assert 4 * 16 * 16 < grp.POOL_EPILOGUE_MIN_PIXELS <= 64 * 8 * 8
    assert (small - out[:, :4]).abs().max().item() < 1e-5
    for g, e in enumerate(engs):
        own = e.forward_eval(x)
        _, ref_logits = e.reference_loss(x.double().cpu(), None, training=False,
                                         params={n: e.flat.w(n).double().cpu() for n in e.flat.names()})
        ref = torch.softmax(ref_logits, 1)
        assert (out[g].double().cpu() - ref).abs().max().item() < 1e-5
        assert (out[g] - own).abs().max().item() < 1e-5


@pytest.mark.parametrize("H,Cin,Cout", [(16, 16, 32), (8, 64, 64), (4, 128, 96), (12, 24, 40)])
@pytest.mark.parametrize("kind,variant", [('w4', 0), ('w4', 1), ('w4', 2), ('w2', 2), ('w2', 3), ('w2', 4),
                                          ('w2', 5)])
def test_grouped_winograd_pooled_epilogue(H, Cin, Cout, kind, variant):
    """rk_wino4_conv_grp / rk_wino2s_conv_grp with WF_POOL: maxpool2(relu(conv + bias)) from the epilogue
    == the same kernel unpooled then pooled by PyTorch (bitwise), and vs fp64."""
    from rafiki_amd.ops import f32 as S
    if kind == 'w4' and H % 4:
        pytest.skip('F(4x4) maps in multiples of 4')
    G, Nb = 3, 5
    g = torch.Generator().manual_seed(H * 1000 + Cin)
    x = torch.randn(G, Nb, H, H, Cin, generator=g).to(DEV)
    w = (torch.randn(G, Cout, 3, 3, Cin, generator=g) / math.sqrt(9 * Cin)).to(DEV)
    b = (torch.randn(G, Cout, generator=g) * 0.1).to(DEV)
    fn = S.wino4_u if kind == 'w4' else S.wino_u
    u = torch.stack([fn(w[k].reshape(Cout, -1).contiguous()) for k in range(G)]).contiguous()
    conv = S.wino4_conv_grp if kind == 'w4' else S.wino_conv_grp
    full = conv(x, u, bias=b, relu=True, variant=variant)
    pooled = conv(x, u, bias=b, relu=True, variant=variant, pool=True)
    torch.cuda.synchronize()
    ref = TF.max_pool2d(full.reshape(G * Nb, H, H, Cout).permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    assert torch.equal(pooled.reshape(G * Nb, H // 2, H // 2, Cout), ref)
    r64 = torch.stack([TF.conv2d(x[k].double().permute(0, 3, 1, 2), w[k].double().permute(0, 3, 1, 2),
                                 b[k].double(), padding=1) for k in range(G)])
    r64 = TF.max_pool2d(torch.relu(r64).reshape(G * Nb, Cout, H, H), 2).permute(0, 2, 3, 1)
    assert rel(pooled.reshape(G * Nb, H // 2, H // 2, Cout), r64) < 3e-5


@pytest.mark.parametrize("H,Cin,Cout,shared", [(16, 16, 32, False), (8, 64, 64, True), (12, 24, 40, False),
                                               (32, 8, 16, True)])
def test_conv_fwd_grp_pooled_entry_vs_fp64(H, Cin, Cout, shared):
    """the public pooled entry (conv_fwd_grp(pool=True), whichever fused candidate the tuner
    picks) vs fp64 conv2d + bias + ReLU + max_pool2d at a tight tolerance, including odd map borders
    (H=12: 3 F(4x4) tiles per side, pool windows straddling no tile edge) and a batch shared by the groups."""
    from rafiki_amd.ops import f32 as S
    G, Nb = 3, 4
    g = torch.Generator().manual_seed(H * 100 + Cin + int(shared))
    x = torch.randn(*((Nb, H, H, Cin) if shared else (G, Nb, H, H, Cin)), generator=g).to(DEV)
    w = (torch.randn(G, Cout, 3, 3, Cin, generator=g) / math.sqrt(9 * Cin)).to(DEV)
    b = (torch.randn(G, Cout, generator=g) * 0.1).to(DEV)
    W = w.reshape(G, Cout, 9 * Cin).contiguous()
    u2 = torch.stack([S.wino_u(W[k]) for k in range(G)]).contiguous()
    u4 = torch.stack([S.wino4_u(W[k]) for k in range(G)]).contiguous() if H % 4 == 0 else None
    assert S.conv_fwd_grp_pool_ok(H, H, Cin, u2, u4)
    got = S.conv_fwd_grp(x, W, bias=b, act=S.ACT_RELU, wino=u2, wino4=u4, pool=True)
    torch.cuda.synchronize()
    assert got.shape == (G, Nb, H // 2, H // 2, Cout)
    xs = [x if shared else x[k] for k in range(G)]
    r64 = torch.stack([TF.max_pool2d(torch.relu(TF.conv2d(xs[k].double().permute(0, 3, 1, 2),
                                                          w[k].double().permute(0, 3, 1, 2), b[k].double(),
                                                          padding=1)), 2).permute(0, 2, 3, 1) for k in range(G)])
    assert rel(got, r64) < 3e-5
    # per-row check too: an error confined to a few pooled pixels (a wrong window at a border) shows here
    err = (got.double().cpu() - r64.cpu()).abs().amax(-1)
    assert err.max().item() < 1e-4 * max(1.0, r64.abs().max().item()), err.max().item()
