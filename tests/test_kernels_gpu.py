"""Numerics of every hand-written gfx950 kernel against a plain PyTorch fp32 reference of the same op.

Inputs are rounded to bf16 first, so the reference sees exactly the kernel's operands; the only
differences left are fp32 accumulation order and the bf16 rounding of outputs.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.fixture(scope="module")
def fn():
    from rafiki_amd.ops import _lib, functional
    _lib.lib()  # loud failure if the native library is missing
    return functional


def _nhwc_to_nchw(x):
    return x.permute(0, 3, 1, 2)


def _w_to_oihw(w):  # [Cout, 3, 3, Cin] -> [Cout, Cin, 3, 3]
    return w.permute(0, 3, 1, 2)


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(4, 8, 8, 64, 64), (2, 16, 16, 8, 64), (3, 4, 4, 128, 256),
                                            (2, 32, 32, 64, 128), (5, 2, 2, 512, 512)])
def test_conv_fwd(fn, N, H, W, Cin, Cout):
    torch.manual_seed(0)
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    w = (torch.randn(Cout, 3, 3, Cin, device=DEV) / (3 * Cin ** 0.5)).bfloat16()
    y, stats = fn.conv_fwd(x, w, want_stats=True)
    ref = F.conv2d(_nhwc_to_nchw(x.float()), _w_to_oihw(w.float()), padding=1).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 1e-2
    s = stats.sum(0)
    assert torch.allclose(s[0], ref.reshape(-1, Cout).sum(0), rtol=1e-3, atol=1e-2 * N * H * W ** 0.5)
    assert torch.allclose(s[1], (ref ** 2).reshape(-1, Cout).sum(0), rtol=2e-3, atol=1e-1)


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(4, 8, 8, 64, 64), (3, 4, 4, 128, 256), (2, 16, 16, 64, 128)])
def test_conv_dgrad(fn, N, H, W, Cin, Cout):
    torch.manual_seed(1)
    dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    w = (torch.randn(Cout, 3, 3, Cin, device=DEV) / (3 * Cin ** 0.5)).bfloat16()
    dx = fn.conv_dgrad(dy, w)
    ref = torch.nn.grad.conv2d_input((N, Cin, H, W), _w_to_oihw(w.float()), _nhwc_to_nchw(dy.float()),
                                     padding=1).permute(0, 2, 3, 1)
    assert rel_err(dx, ref) < 1e-2


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(4, 8, 8, 64, 64), (2, 16, 16, 8, 64), (3, 4, 4, 128, 256),
                                            (8, 32, 32, 64, 64)])
def test_conv_wgrad(fn, N, H, W, Cin, Cout):
    torch.manual_seed(2)
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    dw = fn.conv_wgrad(dy, x)
    ref = torch.nn.grad.conv2d_weight(_nhwc_to_nchw(x.float()), (Cout, Cin, 3, 3), _nhwc_to_nchw(dy.float()),
                                      padding=1).permute(0, 2, 3, 1).reshape(Cout, -1)
    assert rel_err(dw, ref) < 5e-3


@pytest.mark.parametrize("M,K,N", [(256, 2048, 512), (37, 64, 16), (128, 1024, 104), (300, 512, 10 + 6)])
def test_dense_fwd_bwd(fn, M, K, N):
    torch.manual_seed(3)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=DEV)
    y = fn.linear(x, w, b, act=fn.ACT_RELU)
    ref = torch.relu(x.float() @ w.float().t() + b)
    assert rel_err(y, ref) < 1e-2
    y32 = fn.linear(x, w, out_dtype=torch.float32)
    assert rel_err(y32, x.float() @ w.float().t()) < 1e-3
    dy = torch.randn(M, N, device=DEV).bfloat16()
    dx = fn.linear_dx(dy, w)
    assert rel_err(dx, dy.float() @ w.float()) < 1e-2
    gate = torch.randn(M, K, device=DEV).bfloat16()
    dxg = fn.linear_dx(dy, w, gate=gate)
    assert rel_err(dxg, (dy.float() @ w.float()) * (gate.float() > 0)) < 1e-2
    dw = fn.linear_dw(dy, x)
    assert rel_err(dw, dy.float().t() @ x.float()) < 5e-3


@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("N,H,W,C", [(4, 8, 8, 64), (2, 4, 4, 512), (3, 16, 16, 128), (4, 3, 3, 64), (2, 6, 6, 32)])
def test_bn_relu_pool_fwd_bwd(fn, N, H, W, C, pool):
    torch.manual_seed(4)
    y = (torch.randn(N, H, W, C, device=DEV) * 2 + 0.5).bfloat16()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    part = fn.channel_stats(y.view(-1, C))
    coeffs = fn.bn_finalize_fwd(part, N * H * W, gamma, beta, 1e-5, rm, rv, 0.1)
    out = fn.bn_act_fwd(y, coeffs[2], coeffs[3], pool=pool, act=fn.ACT_RELU)
    # reference
    yr = y.float().permute(0, 3, 1, 2).requires_grad_(True)
    g_ = gamma.clone().requires_grad_(True)
    b_ = beta.clone().requires_grad_(True)
    rm2, rv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    z = F.batch_norm(yr, rm2, rv2, g_, b_, training=True, momentum=0.1, eps=1e-5)
    a = torch.relu(z)
    if pool:
        a = F.max_pool2d(a, 2)
    ref = a.permute(0, 2, 3, 1)
    assert rel_err(out, ref) < 1e-2
    assert torch.allclose(rm, rm2, atol=1e-3) and torch.allclose(rv, rv2, rtol=1e-3, atol=1e-3)
    dout = torch.randn_like(ref).bfloat16()
    ref.backward(dout.float())
    dgamma = torch.zeros(C, device=DEV)
    dbeta = torch.zeros(C, device=DEV)
    dy = fn.bn_bwd(dout.contiguous(), y, coeffs, gamma, pool=pool, act=fn.ACT_RELU, dgamma=dgamma, dbeta=dbeta)
    assert rel_err(dy, yr.grad.permute(0, 2, 3, 1)) < 2e-2
    assert rel_err(dgamma, g_.grad) < 1e-2
    assert rel_err(dbeta, b_.grad) < 1e-2


def test_softmax_xent(fn):
    torch.manual_seed(5)
    B, ncls, ld = 300, 10, 16
    logits = torch.randn(B, ld, device=DEV) * 3
    labels = torch.randint(0, ncls, (B,), device=DEV, dtype=torch.int32)
    dl = torch.empty(B, ld, device=DEV, dtype=torch.bfloat16)
    loss = torch.zeros(1, device=DEV)
    correct = torch.zeros(1, device=DEV, dtype=torch.int32)
    probs = torch.empty(B, ncls, device=DEV)
    fn.softmax_xent(logits, labels, ncls, dlogits=dl, probs=probs, loss_sum=loss, correct=correct)
    lr = logits[:, :ncls].clone().requires_grad_(True)
    ref = F.cross_entropy(lr, labels.long())
    ref.backward()
    assert abs(loss.item() / B - ref.item()) < 1e-4
    assert rel_err(dl[:, :ncls], lr.grad) < 1e-2
    assert dl[:, ncls:].float().abs().max().item() == 0
    assert correct.item() == (lr.argmax(1) == labels).sum().item()
    assert torch.allclose(probs, torch.softmax(logits[:, :ncls], 1), atol=1e-5)


def test_optimizers(fn):
    torch.manual_seed(6)
    n = 4096 + 8
    w = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    wb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    p = torch.nn.Parameter(w.clone())
    opt = torch.optim.SGD([p], lr=0.1, momentum=0.9, weight_decay=5e-4, nesterov=True)
    for _ in range(3):
        p.grad = g.clone()
        opt.step()
        fn.sgd_step(w, g, m, wb=wb, lr=0.1, momentum=0.9, weight_decay=5e-4, nesterov=True)
    assert torch.allclose(w, p.detach(), atol=1e-5)
    assert torch.equal(wb, w.bfloat16())
    w2 = torch.randn(n, device=DEV)
    p2 = torch.nn.Parameter(w2.clone())
    opt2 = torch.optim.Adam([p2], lr=1e-3, betas=(0.0, 0.99), eps=1e-8)
    m2, v2 = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for step in range(1, 4):
        p2.grad = g.clone()
        opt2.step()
        fn.adam_step(w2, g, m2, v2, lr=1e-3, beta1=0.0, beta2=0.99, eps=1e-8, step=step)
    assert torch.allclose(w2, p2.detach(), atol=1e-6)


def test_misc(fn):
    torch.manual_seed(7)
    probs = torch.rand(4, 33, 10, device=DEV)
    assert torch.allclose(fn.ensemble_mean(probs), probs.mean(0), atol=1e-6)
    a, b = torch.randn(1000, device=DEV), torch.randn(1000, device=DEV)
    ref = b + (a - b) * 0.99
    fn.lerp_(a, b, 0.99)
    assert torch.allclose(a, ref, atol=1e-6)
    flag = torch.zeros(1, device=DEV, dtype=torch.int32)
    fn.nonfinite_flag(a, flag)
    assert flag.item() == 0
    a[17] = float("nan")
    fn.nonfinite_flag(a, flag)
    assert flag.item() == 1
    x = torch.randn(77, 24, device=DEV).bfloat16()
    out = torch.empty(24, device=DEV)
    fn.colsum(x, out)
    assert torch.allclose(out, x.float().sum(0), atol=1e-3)
    img = torch.randint(0, 255, (3, 3, 8, 8), device=DEV, dtype=torch.uint8)
    packed = fn.pack_nhwc(img, 8, 1 / 255.0, 0.0)
    assert torch.allclose(packed[..., :3].float(), (img.float() / 255).permute(0, 2, 3, 1), atol=4e-3)
    assert packed[..., 3:].abs().max().item() == 0


@pytest.mark.parametrize("N,H,W,Cin,Cout,bn_bit,grid", [(2, 32, 32, 64, 64, 0, 0), (2, 16, 16, 128, 128, 1, 0),
                                                        (3, 8, 8, 256, 64, 0, 7), (2, 32, 32, 128, 256, 1, 5),
                                                        (4, 8, 8, 512, 128, 0, 0), (2, 16, 16, 64, 128, 0, 3),
                                                        (8, 4, 4, 256, 512, 0, 0), (16, 4, 4, 512, 256, 1, 3),
                                                        (24, 4, 4, 64, 128, 0, 2)])
def test_hconv_fwd_dgrad(fn, N, H, W, Cin, Cout, bn_bit, grid):
    """Halo-tiled conv (forward with BN-stats epilogue, and data-gradient) vs PyTorch fp32."""
    torch.manual_seed(11)
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    w = (torch.randn(Cout, 3, 3, Cin, device=DEV) / (3 * Cin ** 0.5)).bfloat16()
    M, K = N * H * W, 9 * Cin
    y = torch.empty(N, H, W, Cout, device=DEV, dtype=torch.bfloat16)
    bm = 64 if W == 8 else 128
    stats = torch.zeros(M // bm * 2, 2, Cout, device=DEV)
    fn.hconv(0, x, w, y, M, Cout, K, K, H, W, Cin, stats=stats, flags=fn.FLAG_STATS, bn_bit=bn_bit, grid=grid)
    ref = F.conv2d(_nhwc_to_nchw(x.float()), _w_to_oihw(w.float()), padding=1).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 1e-2
    s = stats.sum(0)
    assert torch.allclose(s[0], ref.reshape(-1, Cout).sum(0), rtol=2e-2, atol=0.5)
    # data-gradient: dx = conv_transpose(dy, w)
    dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    dx = torch.empty(N, H, W, Cin, device=DEV, dtype=torch.bfloat16)
    fn.hconv(1, dy, w.reshape(Cout, -1), dx, M, Cin, 9 * Cout, 9 * Cin, H, W, Cout, bn_bit=bn_bit if Cin % 128 == 0
             else 0, grid=grid)
    xr = _nhwc_to_nchw(x.float()).requires_grad_(True)
    F.conv2d(xr, _w_to_oihw(w.float()), padding=1).backward(_nhwc_to_nchw(dy.float()))
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("N,H,W,Cin,Cout,S", [(2, 32, 32, 64, 64, 3), (2, 16, 16, 128, 128, 4), (4, 8, 8, 256, 64, 5),
                                              (1, 16, 16, 64, 128, 1), (3, 32, 32, 64, 128, 64),
                                              (16, 4, 4, 256, 128, 2), (8, 4, 4, 64, 64, 3)])
def test_hconv_wgrad(fn, N, H, W, Cin, Cout, S):
    """Halo-tiled weight gradient (slabs + reduce) vs PyTorch fp32 (incl. more slabs than items)."""
    torch.manual_seed(12)
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    slab = torch.full((S, Cout, 9 * Cin), float('nan'), device=DEV)
    fn.hconv_wgrad(dy, x, slab, S)
    out = torch.empty(Cout, 9 * Cin, device=DEV)
    fn.reduce_slabs(slab, out)
    w = torch.zeros(Cout, Cin, 3, 3, device=DEV, requires_grad=True)
    F.conv2d(_nhwc_to_nchw(x.float()), w, padding=1).backward(_nhwc_to_nchw(dy.float()))
    ref = w.grad.permute(0, 2, 3, 1).reshape(Cout, -1)
    assert rel_err(out, ref) < 2e-3


@pytest.mark.parametrize("N,H,Cin,Cout,pool", [(4, 16, 64, 64, True), (2, 8, 128, 256, False), (3, 7, 64, 128, True),
                                               (2, 4, 256, 512, True)])
def test_bn_atomic_accumulator_path(fn, N, H, Cin, Cout, pool):
    """conv_fwd(stats_acc) + fused finalize/apply (fwd) and atomic reduce + fused apply (bwd) agree with
    the deterministic partial-row path."""
    torch.manual_seed(13)
    x = torch.randn(N, H, H, Cin, device=DEV).bfloat16()
    w = (torch.randn(Cout, 9 * Cin, device=DEV) / (3 * Cin ** 0.5)).bfloat16()
    gamma = torch.rand(Cout, device=DEV) + 0.5
    beta = torch.randn(Cout, device=DEV) * 0.1
    y1, st = fn.conv_fwd(x, w, want_stats=True)
    rm1, rv1 = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    c1 = fn.bn_finalize_fwd(st, N * H * H, gamma, beta, 1e-5, rm1, rv1, 0.1)
    o1 = fn.bn_act_fwd(y1, c1[2], c1[3], pool=pool)
    acc = fn.bn_acc_buffer(Cout, DEV)
    y2, _ = fn.conv_fwd(x, w, stats_acc=acc)
    assert rel_err(y2, y1) < 1e-2  # the two stats modes may tune to different (split-K) configs
    rm2, rv2 = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    o2, c2 = fn.bn_act_fwd_acc(y2, acc, N * H * H, gamma, beta, 1e-5, rm2, rv2, 0.1, pool=pool)
    assert torch.allclose(c1, c2, rtol=1e-4, atol=1e-5)
    assert torch.allclose(rm1, rm2, rtol=1e-4, atol=1e-6) and torch.allclose(rv1, rv2, rtol=1e-4, atol=1e-6)
    assert rel_err(o2, o1) < 1e-2
    dout = torch.randn_like(o1)
    g1, b1 = torch.zeros(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    g2, b2 = torch.zeros(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    d1 = fn.bn_bwd(dout, y1, c1, gamma, pool=pool, dgamma=g1, dbeta=b1)
    bacc = fn.bn_acc_buffer(Cout, DEV)
    d2 = fn.bn_bwd_acc(dout, y2, c2, gamma, bacc, pool=pool, dgamma=g2, dbeta=b2)
    assert rel_err(g2, g1) < 1e-4 and rel_err(b2, b1) < 1e-4
    assert rel_err(d2, d1) < 1e-2


@pytest.mark.parametrize("stages", [64, 32])
@pytest.mark.parametrize("N,H,W,Cin,Cout", [(16, 4, 4, 512, 512), (4, 8, 8, 256, 128), (3, 4, 4, 64, 128),
                                            (5, 2, 2, 64, 64)])
def test_wave_ksplit_tile_all_kinds(fn, stages, N, H, W, Cin, Cout):
    """64x64 wave-K-split kernel (tile shape 4): conv fwd with fp64-atomic stats, dgrad with the
    ReLU-gate epilogue, split-K wgrad (odd K-tile counts per split), dense fwd/dX/dW vs fp32."""
    torch.manual_seed(14)
    tile = fn.KS_TILE | stages
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    w = (torch.randn(Cout, 9 * Cin, device=DEV) / (3 * Cin ** 0.5)).bfloat16()
    M, K = N * H * W, 9 * Cin
    # conv forward + SATOM statistics
    y = torch.empty(N, H, W, Cout, device=DEV, dtype=torch.bfloat16)
    acc = fn.bn_acc_buffer(Cout, DEV)
    flags = fn.FLAG_STATS | fn.FLAG_SATOM | ((acc.shape[0] - 1) << 12)
    fn.igemm(fn.KIND_CONV_FWD, 0, x, w, y, M, Cout, K, Cin, K, Cout, stats=acc, H=H, W=W, C=Cin, taps=9,
             flags=flags, tile=tile)
    ref = F.conv2d(_nhwc_to_nchw(x.float()), _w_to_oihw(w.float().reshape(Cout, 3, 3, Cin)),
                   padding=1).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 1e-2
    s = acc.sum(0).float()
    assert torch.allclose(s[0], ref.reshape(-1, Cout).sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)
    assert torch.allclose(s[1], (ref ** 2).reshape(-1, Cout).sum(0), rtol=2e-3, atol=1e-1)
    # data gradient with a ReLU gate
    dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    gate = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    dx = torch.empty(N, H, W, Cin, device=DEV, dtype=torch.bfloat16)
    fn.igemm(fn.KIND_CONV_DGRAD, 0, dy, w, dx, M, Cin, 9 * Cout, Cout, 9 * Cin, Cin, gate=gate, H=H, W=W, C=Cout,
             taps=9, Cb=Cout, flags=fn.FLAG_GATE, tile=tile)
    xr = _nhwc_to_nchw(x.float()).requires_grad_(True)
    F.conv2d(xr, _w_to_oihw(w.float().reshape(Cout, 3, 3, Cin)), padding=1).backward(_nhwc_to_nchw(dy.float()))
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1) * (gate.float() > 0)) < 1e-2
    # weight gradient, split-K slabs (3 splits: uneven, odd K-tile counts)
    splits = 3
    slab = torch.full((splits, Cout, K), float('nan'), device=DEV)
    kt = (M + 63) // 64
    per = (kt + splits - 1) // splits
    s_eff = (kt + per - 1) // per
    fn.igemm(fn.KIND_CONV_WGRAD, 1, dy, x, slab, Cout, K, M, Cout, 0, K, H=H, W=W, C=Cin, taps=9, splits=s_eff,
             slab_stride=Cout * K, tile=tile)
    dw = slab[:s_eff].sum(0)
    wr = torch.zeros(Cout, Cin, 3, 3, device=DEV, requires_grad=True)
    F.conv2d(_nhwc_to_nchw(x.float()), wr, padding=1).backward(_nhwc_to_nchw(dy.float()))
    assert rel_err(dw, wr.grad.permute(0, 2, 3, 1).reshape(Cout, -1)) < 5e-3
    # dense forward (bias + ReLU), dX and dW on flattened operands
    a = x.reshape(M, Cin)
    wd = (torch.randn(Cout, Cin, device=DEV) / Cin ** 0.5).bfloat16()
    b = torch.randn(Cout, device=DEV)
    yd = torch.empty(M, Cout, device=DEV, dtype=torch.bfloat16)
    fn.igemm(fn.KIND_DENSE, 0, a, wd, yd, M, Cout, Cin, Cin, Cin, Cout, bias=b, flags=fn.FLAG_BIAS | fn.FLAG_RELU,
             tile=tile)
    assert rel_err(yd, torch.relu(a.float() @ wd.float().t() + b)) < 1e-2
    dyd = dy.reshape(M, Cout)
    dxd = torch.empty(M, Cin, device=DEV, dtype=torch.bfloat16)
    fn.igemm(fn.KIND_DENSE_DX, 0, dyd, wd, dxd, M, Cin, Cout, Cout, Cin, Cin, tile=tile)
    assert rel_err(dxd, dyd.float() @ wd.float()) < 1e-2
    dwd = torch.empty(Cout, Cin, device=DEV)
    fn.igemm(fn.KIND_DENSE_DW, 1, dyd, a, dwd, Cout, Cin, M, Cout, Cin, Cin, splits=1, tile=tile)
    assert rel_err(dwd, dyd.float().t() @ a.float()) < 5e-3


def test_wave_ksplit_refuses_partial_row_stats(fn):
    x = torch.randn(2, 4, 4, 64, device=DEV).bfloat16()
    w = torch.randn(64, 9 * 64, device=DEV).bfloat16()
    y = torch.empty(2, 4, 4, 64, device=DEV, dtype=torch.bfloat16)
    stats = torch.zeros(4, 2, 64, device=DEV)
    with pytest.raises(Exception):
        fn.igemm(fn.KIND_CONV_FWD, 0, x, w, y, 32, 64, 576, 64, 576, 64, stats=stats, H=4, W=4, C=64, taps=9,
                 flags=fn.FLAG_STATS, tile=fn.KS_TILE | 64)


@pytest.mark.parametrize("tile,S", [(64, 2), (65, 3), (66, 4), (0, 2)])
@pytest.mark.parametrize("N,H,W,Cin,Cout", [(16, 4, 4, 512, 512), (4, 8, 8, 256, 128), (3, 4, 4, 64, 64)])
def test_conv_split_k_slab_epilogue(fn, tile, S, N, H, W, Cin, Cout):
    """Split-K conv forward / data-gradient into fp32 slabs + rk_slab_epi: forward statistics (mode 1),
    the BN-backward mask and sums (mode 2, FLAG_BNB semantics) and a ReLU gate (mode 3) vs fp32."""
    torch.manual_seed(15)
    x = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    w = (torch.randn(Cout, 9 * Cin, device=DEV) / (3 * Cin ** 0.5)).bfloat16()
    M, K = N * H * W, 9 * Cin
    kt = (K + 63) // 64
    per = (kt + S - 1) // S
    s_eff = (kt + per - 1) // per
    slab = torch.full((s_eff, M, Cout), float('nan'), device=DEV)
    fn.igemm(fn.KIND_CONV_FWD, 1, x, w, slab, M, Cout, K, Cin, K, Cout, H=H, W=W, C=Cin, taps=9, splits=s_eff,
             slab_stride=M * Cout, tile=tile)
    y = torch.empty(N, H, W, Cout, device=DEV, dtype=torch.bfloat16)
    acc = fn.bn_acc_buffer(Cout, DEV)
    fn.slab_epi(slab, s_eff, M, Cout, y, mode=1, acc=acc)
    ref = F.conv2d(_nhwc_to_nchw(x.float()), _w_to_oihw(w.float().reshape(Cout, 3, 3, Cin)),
                   padding=1).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 1e-2
    st = acc.sum(0).float()
    assert torch.allclose(st[0], ref.reshape(-1, Cout).sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)
    assert torch.allclose(st[1], (ref ** 2).reshape(-1, Cout).sum(0), rtol=2e-3, atol=1e-1)
    # data gradient: split-K slabs, then BNB (mode 2) and gate (mode 3) combines
    dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
    kt = (9 * Cout + 63) // 64
    per = (kt + S - 1) // S
    s_eff = (kt + per - 1) // per
    slab = torch.full((s_eff, M, Cin), float('nan'), device=DEV)
    fn.igemm(fn.KIND_CONV_DGRAD, 1, dy, w, slab, M, Cin, 9 * Cout, Cout, 9 * Cin, Cin, H=H, W=W, C=Cout, taps=9,
             Cb=Cout, splits=s_eff, slab_stride=M * Cin, tile=tile)
    xr = _nhwc_to_nchw(x.float()).requires_grad_(True)
    F.conv2d(xr, _w_to_oihw(w.float().reshape(Cout, 3, 3, Cin)), padding=1).backward(_nhwc_to_nchw(dy.float()))
    dref = xr.grad.permute(0, 2, 3, 1)
    yb = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
    scale = torch.rand(Cin, device=DEV) + 0.5
    shift = torch.randn(Cin, device=DEV) * 0.1
    dx = torch.empty(N, H, W, Cin, device=DEV, dtype=torch.bfloat16)
    bacc = fn.bn_acc_buffer(Cin, DEV)
    fn.slab_epi(slab, s_eff, M, Cin, dx, mode=2, gate=yb, scale=scale, shift=shift, acc=bacc)
    mask = (yb.float() * scale + shift) > 0
    dz = dref * mask
    assert rel_err(dx, dz) < 1e-2
    sb = bacc.sum(0).float()
    assert torch.allclose(sb[0], dz.reshape(-1, Cin).sum(0), rtol=1e-2, atol=1e-1)
    assert torch.allclose(sb[1], (dz * yb.float()).reshape(-1, Cin).sum(0), rtol=1e-2, atol=1e-1)
    fn.slab_epi(slab, s_eff, M, Cin, dx, mode=3, gate=yb)
    assert rel_err(dx, dref * (yb.float() > 0)) < 1e-2


def test_conv_wt_transposed_dgrad(fn):
    """ConvWT (one launch for several layers) + conv_dgrad_t (forward kernels on the flipped/transposed
    weights) vs the PyTorch fp32 data gradient, plain, with a ReLU gate and with the BNB epilogue."""
    torch.manual_seed(16)
    shapes = [(16, 4, 4, 512, 512), (8, 8, 8, 128, 256), (2, 32, 32, 64, 64), (3, 16, 16, 64, 128), (2, 6, 6, 64, 64)]
    ws = [(torch.randn(co, 9 * ci, device=DEV) / (3 * ci ** 0.5)).bfloat16() for (_, _, _, ci, co) in shapes]
    arena = torch.zeros(sum((w.numel() + 63) // 64 * 64 for w in ws) + 64, device=DEV, dtype=torch.bfloat16)
    views, off = [], 0
    for w in ws:
        v = arena[off:off + w.numel()].view_as(w)
        v.copy_(w)
        views.append(v)
        off += (w.numel() + 63) // 64 * 64
    wt = fn.ConvWT(arena, views)
    wt.refresh()
    for l, (N, H, W, Cin, Cout) in enumerate(shapes):
        w4 = ws[l].float().reshape(Cout, 3, 3, Cin)
        ref_t = w4.flip(1).flip(2).permute(3, 1, 2, 0).reshape(Cin, 9 * Cout)
        assert torch.equal(wt.view(l).float(), ref_t)
        dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
        xr = torch.zeros(N, Cin, H, W, device=DEV, requires_grad=True)
        F.conv2d(xr, _w_to_oihw(w4), padding=1).backward(_nhwc_to_nchw(dy.float()))
        dref = xr.grad.permute(0, 2, 3, 1)
        assert rel_err(fn.conv_dgrad_t(dy, wt.view(l)), dref) < 1e-2
        gate = torch.randn(N, H, W, Cin, device=DEV).bfloat16()
        assert rel_err(fn.conv_dgrad_t(dy, wt.view(l), gate=gate), dref * (gate.float() > 0)) < 1e-2
        scale = torch.rand(Cin, device=DEV) + 0.5
        coeffs = torch.stack([torch.zeros(Cin, device=DEV), torch.ones(Cin, device=DEV), scale,
                              torch.randn(Cin, device=DEV) * 0.1])
        bacc = fn.bn_acc_buffer(Cin, DEV)
        dz = fn.conv_dgrad_t(dy, wt.view(l), bn_y=gate, bn_coeffs=coeffs, bn_acc=bacc)
        dz_ref = dref * ((gate.float() * coeffs[2] + coeffs[3]) > 0)
        assert rel_err(dz, dz_ref) < 1e-2
        sb = bacc.sum(0).float()
        assert torch.allclose(sb[0], dz_ref.reshape(-1, Cin).sum(0), rtol=1e-2, atol=2e-1)


def test_conv_wt_dgrad_bn_pool_sums(fn):
    """conv_dgrad_t(bn_pool_y=...) (FLAG_BNP): the output is the unchanged pooled data gradient and the
    fp64 slots hold the BN-backward sums (sum dz, sum dz*y) of the BN+ReLU+2x2-max-pool layer below,
    dz routed to the window's first maximum — vs torch max_pool2d indices in fp32."""
    torch.manual_seed(17)
    shapes = [(16, 4, 4, 512, 512), (8, 8, 8, 128, 256), (2, 16, 16, 64, 128)]
    ws = [(torch.randn(co, 9 * ci, device=DEV) / (3 * ci ** 0.5)).bfloat16() for (_, _, _, ci, co) in shapes]
    arena = torch.zeros(sum((w.numel() + 63) // 64 * 64 for w in ws) + 64, device=DEV, dtype=torch.bfloat16)
    views, off = [], 0
    for w in ws:
        v = arena[off:off + w.numel()].view_as(w)
        v.copy_(w)
        views.append(v)
        off += (w.numel() + 63) // 64 * 64
    wt = fn.ConvWT(arena, views)
    wt.refresh()
    for l, (N, H, W, Cin, Cout) in enumerate(shapes):
        w4 = ws[l].float().reshape(Cout, 3, 3, Cin)
        dy = torch.randn(N, H, W, Cout, device=DEV).bfloat16()
        xr = torch.zeros(N, Cin, H, W, device=DEV, requires_grad=True)
        F.conv2d(xr, _w_to_oihw(w4), padding=1).backward(_nhwc_to_nchw(dy.float()))
        dref = xr.grad.permute(0, 2, 3, 1)
        y = torch.randn(N, 2 * H, 2 * W, Cin, device=DEV).bfloat16()
        scale = torch.rand(Cin, device=DEV) + 0.5
        coeffs = torch.stack([torch.zeros(Cin, device=DEV), torch.ones(Cin, device=DEV), scale,
                              torch.randn(Cin, device=DEV) * 0.1])
        bacc = fn.bn_acc_buffer(Cin, DEV)
        d = fn.conv_dgrad_t(dy, wt.view(l), bn_pool_y=y, bn_coeffs=coeffs, bn_acc=bacc)
        assert rel_err(d, dref) < 1e-2
        z = y.float() * coeffs[2] + coeffs[3]
        _, idx = F.max_pool2d(_nhwc_to_nchw(z.relu()), 2, return_indices=True)
        # route the kernel's own (bf16) pooled gradient so only the sums are compared
        routed = F.max_unpool2d(_nhwc_to_nchw(d.float()), idx, 2).permute(0, 2, 3, 1)
        dz = routed * (z > 0)
        sb = bacc.sum(0).float()
        s0, s1 = dz.reshape(-1, Cin).sum(0), (dz * y.float()).reshape(-1, Cin).sum(0)
        assert torch.allclose(sb[0], s0, rtol=1e-2, atol=2e-1)
        assert torch.allclose(sb[1], s1, rtol=1e-2, atol=2e-1)
