"""Twice-differentiable autograd wrappers over the gfx950 conv / dense kernels.

WGAN-GP (pg_gans.py:1305-1315) differentiates the discriminator's input-gradient with respect to
the discriminator's weights, so every backward here is itself expressed through these Functions
(SURVEY §7.4 (1)): the three GEMMs of a layer close under differentiation

    y  = conv(x, w)        dx = dgrad(dy, w)      dw = wgrad(x, dy)
    d(dgrad)/d(dy) = conv(., w)     d(dgrad)/d(w) = wgrad(., dy)
    d(wgrad)/d(x)  = dgrad(dy, .)   d(wgrad)/d(dy) = conv(x, .)

and the same for dense (x @ w.T, dy @ w, dy.T @ x).  Conventions: activations are NHWC / [M, K] in
the tensor's own precision — fp32 (the reference's, ``ops.f32``: v_mfma_f32_32x32x2_f32) or bf16
(opt-in, ``ops.functional``: bf16 MFMA with fp32 masters ``w`` and a bf16 shadow ``wb`` the fused
optimizer keeps in sync; ``wb=None`` casts on the fly); weight gradients are fp32 either way.

The PG-GAN resampling convolutions (pg_gans.py:1032-1067) in fp32 are the stride-2 gather family
(``S2Fn`` / ``S2TFn`` / ``S2WFn``, itself closed under differentiation): conv3x3 + 2x2 box downscale
is one 4x4 stride-2 gather conv with box-summed weights, upscale2d + conv3x3 is its adjoint with
box-summed flipped weights — 1/2.25 of the full-resolution MACs and no 2x tensor.  The weight
transforms are tiny differentiable torch ops, so the gradient reaches the 3x3 parameters.

On CPU tensors every op falls back to plain fp32 PyTorch (F.conv2d / matmul), which torch already
differentiates twice — that path is the numerics oracle for the GPU tests.  On a GPU tensor the
native library is mandatory (a missing extension raises, it never silently falls back).
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.nn.functional as TF

from . import _lib
from . import f32 as S
from . import functional as F

BF16 = torch.bfloat16
F32 = torch.float32


def _bf(t: Optional[torch.Tensor]):
    if t is None:
        return None
    return t.detach().to(BF16).contiguous() if t.dtype != BF16 else t.detach().contiguous()


def _wshadow(w, wb):
    return wb if wb is not None else _bf(w)


def _needed(ctx, i):
    """Input i needs a gradient in THIS backward: autograd.grad(..., inputs=[images]) (the WGAN-GP
    input gradient) must not pay for weight gradients it then drops."""
    if not ctx.needs_input_grad[i]:
        return False
    try:
        fn = ctx.next_functions[i][0]
        return fn is None or bool(torch._C._will_engine_execute_node(fn))
    except Exception:
        return True


def _bias_grad(gy):
    """sum of gy over all but the channel axis, fp32.  Outside a create_graph backward the result
    is never differentiated, so it comes from the fused column-sum kernels instead of a reduction."""
    Cc = gy.shape[-1]
    if not torch.is_grad_enabled() and gy.is_cuda and gy.is_contiguous():
        out = torch.empty(Cc, device=gy.device, dtype=torch.float32)
        if gy.dtype == BF16:
            return F.colsum(gy.reshape(-1, Cc), out)
        if gy.dtype == F32:
            return S.colsum(gy.reshape(-1, Cc), out)
    return gy.float().reshape(-1, Cc).sum(0)


def _as(t, dt):
    return t.to(dt).contiguous()


def _act(slope):
    return F.ACT_NONE if slope is None else F.ACT_LRELU


def _k(taps):
    return 3 if taps == 9 else 1


# ------------------------------------------------------------------------------- CPU reference
def _conv_ref(x, w, b, taps):
    Cout = w.shape[0]
    Cin = w.numel() // (Cout * taps)
    k = _k(taps)
    wt = w.reshape(Cout, k, k, Cin).permute(0, 3, 1, 2)
    y = TF.conv2d(x.permute(0, 3, 1, 2), wt.to(x.dtype), None if b is None else b.to(x.dtype), padding=k // 2)
    return y.permute(0, 2, 3, 1)


def upscale2d(x, factor=2):
    """Nearest-neighbour upscale of NHWC (pg_gans.py:1042-1050); native kernel on GPU."""
    if factor == 1:
        return x
    if x.is_cuda and x.shape[-1] % 4 == 0 and factor & (factor - 1) == 0:
        while factor > 1:
            x = Up2Fn.apply(x, 1.0)
            factor //= 2
        return x
    N, h, w, C = x.shape
    return x[:, :, None, :, None, :].expand(N, h, factor, w, factor, C).reshape(N, h * factor, w * factor, C)


def downscale2d(x, factor=2):
    """Box-filter downscale of NHWC (pg_gans.py:1062-1067), accumulated in fp32; native kernel on GPU."""
    if factor == 1:
        return x
    N, H, W, C = x.shape
    if x.is_cuda and factor == 2 and C % 4 == 0 and H % 2 == 0 and W % 2 == 0:
        return Down2Fn.apply(x, 0.25)
    y = x.reshape(N, H // factor, factor, W // factor, factor, C).float().mean((2, 4))
    return y.to(x.dtype)


def sumpool2(x):
    N, H, W, C = x.shape
    return x.reshape(N, H // 2, 2, W // 2, 2, C).float().sum((2, 4)).to(x.dtype)


# ------------------------------------------------------------------------------------- conv
@contextlib.contextmanager
def accumulate_weight_grads_in_place(params):
    """Within this context a plain ``loss.backward()`` (no create_graph) accumulates the fp32 conv / dense
    weight and bias gradients of the leaves in ``params`` straight into each leaf's persistent ``.grad``
    buffer (the flat gradient arena) and returns None for them, skipping autograd's gradient sums and
    AccumulateGrad adds — a parameter is used several times per WGAN-GP step (real/fake, mixed, the
    penalty's double backward).  Only for ``.backward()`` into ``.grad`` (not autograd.grad).

    The opt-in is a mark on the leaves themselves, not thread-local state: autograd runs a CUDA
    backward on its own device thread, which never sees the caller's thread-locals."""
    leaves = [p for p in params if isinstance(p, torch.Tensor)]
    prev = [getattr(p, '_rk_direct', False) for p in leaves]
    for p in leaves:
        p._rk_direct = True
    try:
        yield
    finally:
        for p, v in zip(leaves, prev):
            p._rk_direct = v


_WT = {'on': 0, 'cache': {}}


@contextlib.contextmanager
def cached_weight_transforms(params):
    """Within this context the derived forms of the conv weights in ``params`` (Winograd U sets, their X6
    planes, the data-gradient transposes) are computed once and reused by every conv / dgrad that reads the
    same weight — a WGAN-GP step reads each discriminator weight in 4-6 convs.  The weights must not
    change inside the context (wrap forward + backward, not the optimizer step).  Only leaves marked here
    are cached (persistent arena storage: their addresses never name another tensor); the marks and the
    cache are process-global because the backward runs on autograd's device thread."""
    leaves = [p for p in params if isinstance(p, torch.Tensor)]
    prev = [getattr(p, '_rk_wcache', False) for p in leaves]
    for p in leaves:
        p._rk_wcache = True
    _WT['on'] += 1
    try:
        yield
    finally:
        _WT['on'] -= 1
        if _WT['on'] == 0:
            _WT['cache'].clear()
        for p, v in zip(leaves, prev):
            p._rk_wcache = v


def _wt(kind, w, fn):
    """``fn`` (a producer of a derived form of weight ``w``), cached by (kind, address, shape) when ``w`` is
    (a reinterpreting view of) a leaf marked by ``cached_weight_transforms``; else ``fn`` itself."""
    if not _WT['on']:
        return fn
    leaf = w if w.is_leaf else getattr(w, '_base', None)
    if leaf is None or not getattr(leaf, '_rk_wcache', False) or not w.is_contiguous():
        return fn
    key = (kind, w.data_ptr(), tuple(w.shape))

    def get():
        t = _WT['cache'].get(key)
        if t is None:
            t = _WT['cache'][key] = fn()
        return t
    return get


# Observer of in-place gradient writes: GRAD_WATCH[0](leaf) is called right before a backward enqueues a
# contribution into a leaf's persistent .grad buffer (parallel/grad_bucket.py places each bucket's
# all-reduce event after the bucket's last contribution).  Process-global: the backward of a CUDA graph
# runs on autograd's device thread.
GRAD_WATCH = [None]


def _param_grad_buffer(w):
    """The persistent fp32 gradient buffer of a parameter (the leaf's .grad, or the viewed leaf's, in
    the parameter's shape), for a leaf marked by ``accumulate_weight_grads_in_place`` and outside a
    create_graph backward; None otherwise (the caller returns the gradient to autograd)."""
    if w is None or torch.is_grad_enabled() or w.dtype != F32 or not w.is_cuda:
        return None
    leaf = w if w.is_leaf else getattr(w, '_base', None)
    if leaf is None or not leaf.is_leaf or not leaf.requires_grad or not getattr(leaf, '_rk_direct', False):
        return None
    g = leaf.grad
    if g is None or g.dtype != F32 or not g.is_contiguous() or g.numel() != w.numel() or leaf.numel() != w.numel():
        return None
    # a reinterpreting view only (reshape of the whole contiguous leaf), never a transpose
    if not (w.is_contiguous() and leaf.is_contiguous() and w.data_ptr() == leaf.data_ptr()):
        return None
    watch = GRAD_WATCH[0]
    if watch is not None:
        watch(leaf)
    return g.view(w.shape)


def _bias_grad_into(gy, b):
    """Bias gradient of ``gy`` for parameter ``b``: accumulated in place into b's .grad buffer when
    ``_param_grad_buffer`` allows it (returns None), else returned for autograd."""
    buf = _param_grad_buffer(b)
    if buf is not None and gy.dtype in (F32, BF16) and gy.is_cuda:
        Cc = gy.shape[-1]
        g2 = gy.contiguous().reshape(-1, Cc)
        (S.colsum if gy.dtype == F32 else F.colsum)(g2, buf, accumulate=True)
        return None
    return _bias_grad(gy)


def _gate_colsum(ctx, gy, y, b):
    """(gated gy, bias gradient or None): the leaky-ReLU gate and the bias column sum in one pass over
    gy (outside a create_graph backward); the sum goes straight into b's .grad when allowed."""
    buf = _param_grad_buffer(b)
    if buf is not None:
        g, _ = S.lrelu_gate_colsum(gy, y.contiguous(), float(ctx.slope), acc=buf)
        return g, None
    return S.lrelu_gate_colsum(gy, y.contiguous(), float(ctx.slope))


class LReluGateFn(torch.autograd.Function):
    """g = gy * (y > 0 ? 1 : slope) on the native kernel; linear in gy, so its derivative is the same
    gate (WGAN-GP double backward).  The mask is piecewise constant: no gradient flows into y."""

    @staticmethod
    def forward(ctx, gy, y, slope):
        ctx.save_for_backward(y)
        ctx.slope = slope
        return S.lrelu_gate(gy.contiguous(), y.detach().contiguous(), slope)

    @staticmethod
    def backward(ctx, gg):
        (y,) = ctx.saved_tensors
        return LReluGateFn.apply(gg, y, ctx.slope), None, None


def _lrelu_gate(gy, y, slope):
    """gy * lrelu'(.) with the mask read from the activation OUTPUT y (same sign as its input);
    linear in gy, so it differentiates again (WGAN-GP double backward).  The mask is piecewise
    constant, so y is detached: no (zero) gradient is routed back into y's producer."""
    if gy.is_cuda and gy.dtype == F32 and y.dtype == F32 and gy.shape[-1] % 4 == 0:
        return LReluGateFn.apply(gy, y, float(slope))
    return torch.ops.aten.leaky_relu_backward(gy, y.detach(), slope, True)


class ConvFn(torch.autograd.Function):
    """y = act(conv_{taps}(x, w) + b)   (x NHWC bf16, w fp32 [Cout, taps*Cin] tap-major); act is
    leaky ReLU(slope) fused into the GEMM epilogue when ``slope`` is given, else the identity."""

    @staticmethod
    def forward(ctx, x, w, b, wb, taps, slope):
        x = x.contiguous()
        bd = None if b is None else b.detach().float().contiguous()
        if x.dtype == F32:
            wd = w.detach().contiguous()
            # 3x3: the fused Winograd kernels (weights transformed inside the candidate) compete in the tuner
            y = S.conv_fwd(x, wd, taps=taps, bias=bd, act=_act(slope), slope=0.2 if slope is None else slope,
                           wino=_wt('u2', w, lambda: S.wino_u(wd)) if taps == 9 else None,
                           wino4=_wt('u4', w, lambda: S.wino4_u(wd)) if taps == 9 else None,
                           wino4p=_wt('u4p', w, lambda: S.wino4_u4p(wd)) if taps == 9 else None)
        else:
            y = F.conv_fwd(x, _wshadow(w, wb), taps=taps, bias=bd, act=_act(slope),
                           slope=0.2 if slope is None else slope)
        ctx.dt = x.dtype
        if slope is None:
            ctx.save_for_backward(x, w)
        else:
            ctx.save_for_backward(x, w, y)
        ctx.wb, ctx.taps, ctx.has_b, ctx.slope = wb, taps, b is not None, slope
        ctx.b = b   # the bias leaf: its .grad takes the bias gradient in place (_param_grad_buffer)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors[:2]
        gb, b_done = None, False
        if ctx.slope is not None:
            y = ctx.saved_tensors[2]
            if (ctx.has_b and _needed(ctx, 2) and not torch.is_grad_enabled() and gy.is_cuda
                    and gy.dtype == F32 and y.dtype == F32 and gy.is_contiguous()):
                # outside a create_graph backward: gate + bias gradient in one pass over gy
                gy, gb = _gate_colsum(ctx, gy, y, ctx.b)
                b_done = True
            else:
                gy = _lrelu_gate(gy, y, ctx.slope)
        gy = _as(gy, ctx.dt)
        gx = gw = None
        if _needed(ctx, 0):
            gx = ConvDgradFn.apply(gy, w, ctx.wb, ctx.taps)
        if _needed(ctx, 1):
            buf = _param_grad_buffer(w) if x.dtype == F32 else None
            if buf is not None:
                S.conv_wgrad(gy.contiguous(), x.contiguous(), taps=ctx.taps, out=buf.view(buf.shape[0], -1),
                             accumulate=True)
            else:
                gw = ConvWgradFn.apply(x, gy, ctx.taps)
        if ctx.has_b and _needed(ctx, 2) and not b_done:
            gb = _bias_grad_into(gy, ctx.b)
        return gx, gw, gb, None, None, None


class ConvDgradFn(torch.autograd.Function):
    """dx = dgrad(dy, w)  (the transposed conv, tap-flipped gather of the forward weights)."""

    @staticmethod
    def forward(ctx, gy, w, wb, taps):
        gy = gy.contiguous()
        if gy.dtype == F32:
            wd = w.detach().contiguous()
            dx = S.conv_dgrad(gy, _wt('wt%d' % taps, w, lambda: S.conv_wt(wd, taps)), taps=taps,
                              cin=wd.numel() // (taps * wd.shape[0]),
                              wino=_wt('ut2', w, lambda: S.wino_ut(wd)) if taps == 9 else None,
                              wino4=_wt('ut4', w, lambda: S.wino4_ut(wd)) if taps == 9 else None,
                              wino4p=_wt('ut4p', w, lambda: S.wino4_u4p(wd, dgrad=True)) if taps == 9 else None)
        else:
            dx = F.conv_dgrad(gy, _wshadow(w, wb), taps=taps)
        ctx.save_for_backward(gy, w)
        ctx.wb, ctx.taps, ctx.dt = wb, taps, gy.dtype
        return dx

    @staticmethod
    def backward(ctx, ggx):
        gy, w = ctx.saved_tensors
        ggx = _as(ggx, ctx.dt)
        g_gy = g_w = None
        if _needed(ctx, 0):
            g_gy = ConvFn.apply(ggx, w, None, ctx.wb, ctx.taps, None)
        if _needed(ctx, 1):
            # the WGAN-GP penalty's second-order weight gradient: straight into the .grad arena when the
            # outer backward allows it (no autograd sum / AccumulateGrad add kernels)
            buf = _param_grad_buffer(w) if gy.dtype == F32 and ggx.dtype == F32 else None
            if buf is not None:
                S.conv_wgrad(gy.contiguous(), ggx.contiguous(), taps=ctx.taps, out=buf.view(buf.shape[0], -1),
                             accumulate=True)
            else:
                g_w = ConvWgradFn.apply(ggx, gy, ctx.taps)
        return g_gy, g_w, None, None


class ConvWgradFn(torch.autograd.Function):
    """dw (fp32) = wgrad(x, dy)."""

    @staticmethod
    def forward(ctx, x, gy, taps):
        x, gy = x.contiguous(), gy.contiguous()
        dw = S.conv_wgrad(gy, x, taps=taps) if x.dtype == F32 else F.conv_wgrad(gy, x, taps=taps)
        ctx.save_for_backward(x, gy)
        ctx.taps = taps
        return dw

    @staticmethod
    def backward(ctx, ggw):
        x, gy = ctx.saved_tensors
        ggw = ggw.contiguous()
        g_x = g_gy = None
        if _needed(ctx, 0):
            g_x = ConvDgradFn.apply(gy, ggw, None, ctx.taps)
        if _needed(ctx, 1):
            g_gy = ConvFn.apply(x, ggw, None, None, ctx.taps, None)
        return g_x, g_gy, None


def conv2d(x, w, b=None, *, taps=9, wb=None, lrelu=None):
    """NHWC conv, stride 1, SAME padding (3x3 when taps == 9, 1x1 when taps == 1); ``lrelu`` = slope
    of a fused leaky-ReLU epilogue."""
    if x.device.type != 'cuda':
        y = _conv_ref(x, w, b, taps)
        return y if lrelu is None else leaky_relu(y, lrelu)
    return ConvFn.apply(x, w, b, wb, taps, None if lrelu is None else float(lrelu))


class UpConvFn(torch.autograd.Function):
    """y = conv3x3(upscale2d(x), w) + b with the upscale fused into the conv gather (forward only;
    the backward runs on the 2x grid and sum-pools, built from the differentiable Functions)."""

    @staticmethod
    def forward(ctx, x, w, b, wb):
        x = x.contiguous()
        y = F.conv_up(x, _wshadow(w, wb), bias=None if b is None else b.detach().float().contiguous())
        ctx.save_for_backward(x, w)
        ctx.wb, ctx.has_b = wb, b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.to(BF16).contiguous()
        gx = gw = gb = None
        if _needed(ctx, 0):
            gx = sumpool2(ConvDgradFn.apply(gy, w, ctx.wb, 9))
        if _needed(ctx, 1):
            gw = ConvWgradFn.apply(upscale2d(x).contiguous(), gy, 9)
        if ctx.has_b and _needed(ctx, 2):
            gb = _bias_grad(gy)
        return gx, gw, gb, None


def _box4(w3):
    """[Co, 3, 3, Ci] -> [Co, 4, 4, Ci]: sum of the four 1-pixel shifts of the zero-padded kernel
    (the reference's fused-resample weights, pg_gans.py:1035-1036 / 1055-1056)."""
    wp = TF.pad(w3, (0, 0, 1, 1, 1, 1))
    return wp[:, 1:, 1:] + wp[:, :-1, 1:] + wp[:, 1:, :-1] + wp[:, :-1, :-1]


def _box_launch(mode, src, co, cin):
    """rk_box_weights (resample.hip): mode 0 down [Co,9Ci]->[Co,16Ci] (x1/4), 1 its adjoint, 2 up (flipped,
    transposed) [Co,9Ci]->[Ci,16Co], 3 its adjoint."""
    src = src.contiguous()
    shape = {0: (co, 16 * cin), 1: (co, 9 * cin), 2: (cin, 16 * co), 3: (co, 9 * cin)}[mode]
    out = torch.empty(shape, device=src.device, dtype=torch.float32)
    _lib.call("rk_box_weights", int(mode), S._p(src), S._p(out), co, cin, 0.25 if mode < 2 else 1.0, S._s())
    return out


class BoxWeightsFn(torch.autograd.Function):
    """The resampling convs' 4x4 box-filter weights of a 3x3 kernel (linear in w) on one native kernel,
    backward = the adjoint kernel (itself differentiable: WGAN-GP's double backward goes through it)."""

    @staticmethod
    def forward(ctx, w, co, cin, mode):
        ctx.co, ctx.cin, ctx.mode = co, cin, mode
        return _box_launch(mode, w, co, cin)

    @staticmethod
    def backward(ctx, g):
        return BoxWeightsAdjFn.apply(g, ctx.co, ctx.cin, ctx.mode), None, None, None


class BoxWeightsAdjFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, co, cin, mode):
        ctx.co, ctx.cin, ctx.mode = co, cin, mode
        return _box_launch(mode + 1, g, co, cin)

    @staticmethod
    def backward(ctx, gg):
        return BoxWeightsFn.apply(gg, ctx.co, ctx.cin, ctx.mode), None, None, None


def down_weights(w, cin):
    """3x3 weights [Cout, 9*Cin] -> S2 weights [Cout, 16*Cin] of conv3x3 + 2x2 box downscale (one native
    kernel forward, its adjoint backward: no pad + four shifted adds + scale, no vendor GEMM)."""
    co = w.shape[0]
    if w.device.type != 'cuda' or w.dtype != F32:
        return (_box4(w.reshape(co, 3, 3, cin)) * 0.25).reshape(co, 16 * cin)
    return BoxWeightsFn.apply(w.reshape(co, 9 * cin), co, cin, 0)


def up_weights(w, cin):
    """3x3 weights [Cout, 9*Cin] -> S2 weights [Cin, 16*Cout] whose adjoint S2T is upscale2d + conv3x3 (the
    tap flip and the transpose folded into the same native kernel)."""
    co = w.shape[0]
    if w.device.type != 'cuda' or w.dtype != F32:
        return _box4(w.reshape(co, 3, 3, cin).flip(1, 2)).permute(3, 1, 2, 0).reshape(cin, 16 * co)
    return BoxWeightsFn.apply(w.reshape(co, 9 * cin), co, cin, 2)


def resample_via_winograd(full_hw: int, channels: int) -> bool:
    """Resampling conv by Winograd at full resolution instead of the direct stride-2 / transposed conv?

    The fused stride-2 forms (S2: 4x4 taps at the low resolution, S2T: 4 parity groups of 2x2 taps) do
    16 / 4 MACs per low-res / full-res output and channel pair; conv3x3 at full resolution by F(4x4,3x3)
    does 2.25 per full-res pixel — 1.8x fewer MFMA cycles for the down conv, 1.8x fewer for the up conv
    — at the price of one full-resolution activation round trip (upscale / box-filter pass).  On the
    32x32x512 PG-GAN layers the resampling convs are a third of the lod-0 step
    (profiles/pg_gan_lod0_f32_kernels_r3_direct.txt).  In round 3 the Winograd route lost end to end
    (lod 0: 73.0 vs 71.3 ms per D+G round, profiles/pg_gan_bench_r3e.jsonl); with the pre-split X6 plane
    GEMMs, the leaky-ReLU output-transform epilogue and the native leaky ReLU after the box filter it wins
    (40.2 vs 46.3 ms, profiles/pg_gan_resample_ab_r4.jsonl), so it is the default.
    RAFIKI_PGGAN_RESAMPLE = wino (default) | direct | auto (Winograd on maps >= 16 with >= 64 channels)."""
    mode = os.environ.get('RAFIKI_PGGAN_RESAMPLE', 'wino')
    if mode == 'wino':
        return S.WINO and S.WINO4 and full_hw % 4 == 0 and channels % 8 == 0
    if mode == 'auto':
        return S.WINO and S.WINO4 and full_hw >= 16 and full_hw % 4 == 0 and channels >= 64 and channels % 8 == 0
    return False


def upscale_conv2d(x, w, b=None, *, wb=None, lrelu=None):
    """conv3x3(upscale2d(x), w) + b (pg_gans.py:1032-1039)."""
    if x.device.type != 'cuda':
        y = _conv_ref(upscale2d(x), w, b, 9)
        return y if lrelu is None else leaky_relu(y, lrelu)
    if x.dtype == F32:
        if resample_via_winograd(2 * x.shape[1], x.shape[-1]):
            # upscale (native kernel) then the Winograd-capable 3x3 conv with bias + leaky ReLU epilogue
            return conv2d(upscale2d(x.contiguous()), w, b, lrelu=lrelu)
        return S2TFn.apply(x.contiguous(), up_weights(w, x.shape[-1]), b, None if lrelu is None else float(lrelu))
    y = UpConvFn.apply(x, w, b, wb)
    return y if lrelu is None else leaky_relu(y, lrelu)


def conv2d_downscale2d(x, w, b=None, *, wb=None, lrelu=None):
    """conv3x3 then 2x2 box downscale (+b) == the reference's fused 4x4 stride-2 conv (pg_gans.py:1053-1059)."""
    if x.device.type == 'cuda' and x.dtype == F32:
        if resample_via_winograd(x.shape[1], x.shape[-1]):
            # Winograd conv at full resolution (+bias in its epilogue: the box filter commutes with it),
            # the native box-filter downscale, then the leaky ReLU on the quarter-size map
            y = downscale2d(conv2d(x.contiguous(), w, b))
            return y if lrelu is None else leaky_relu(y, lrelu)
        return S2Fn.apply(x.contiguous(), down_weights(w, x.shape[-1]), b, None if lrelu is None else float(lrelu))
    y = downscale2d(conv2d(x, w, b, taps=9, wb=wb))
    return y if lrelu is None else leaky_relu(y, lrelu)


# ------------------------------------------------------------------ stride-2 gather family (fp32)
class S2Fn(torch.autograd.Function):
    """y = act(S2(x, W) + b): 4x4 taps at -1..2, stride 2 (ops.f32.s2_conv)."""

    @staticmethod
    def forward(ctx, x, W, b, slope):
        y = S.s2_conv(x, W.detach().contiguous(), bias=None if b is None else b.detach().float().contiguous(),
                      act=_act(slope), slope=0.2 if slope is None else slope)
        ctx.save_for_backward(*((x, W) if slope is None else (x, W, y)))
        ctx.has_b, ctx.slope, ctx.b = b is not None, slope, b
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W = ctx.saved_tensors[:2]
        if ctx.slope is not None:
            gy = _lrelu_gate(gy, ctx.saved_tensors[2], ctx.slope)
        gy = _as(gy, F32)
        gx = gW = gb = None
        if _needed(ctx, 0):
            gx = S2TFn.apply(gy, W, None, None)
        if _needed(ctx, 1):
            gW = S2WFn.apply(x, gy)
        if ctx.has_b and _needed(ctx, 2):
            gb = _bias_grad_into(gy, ctx.b)
        return gx, gW, gb, None


class S2TFn(torch.autograd.Function):
    """y = act(S2T(z, W) + b): the adjoint of S2 (the 2x transposed conv, ops.f32.s2t_conv)."""

    @staticmethod
    def forward(ctx, z, W, b, slope):
        y = S.s2t_conv(z, W.detach().contiguous(), bias=None if b is None else b.detach().float().contiguous(),
                       act=_act(slope), slope=0.2 if slope is None else slope)
        ctx.save_for_backward(*((z, W) if slope is None else (z, W, y)))
        ctx.has_b, ctx.slope, ctx.b = b is not None, slope, b
        return y

    @staticmethod
    def backward(ctx, gy):
        z, W = ctx.saved_tensors[:2]
        if ctx.slope is not None:
            gy = _lrelu_gate(gy, ctx.saved_tensors[2], ctx.slope)
        gy = _as(gy, F32)
        gz = gW = gb = None
        if _needed(ctx, 0):
            gz = S2Fn.apply(gy, W, None, None)
        if _needed(ctx, 1):
            gW = S2WFn.apply(gy, z)
        if ctx.has_b and _needed(ctx, 2):
            gb = _bias_grad_into(gy, ctx.b)
        return gz, gW, gb, None


class S2WFn(torch.autograd.Function):
    """dW = S2W(x, g) (ops.f32.s2_wgrad); its own gradients are S2T(g, .) and S2(x, .)."""

    @staticmethod
    def forward(ctx, x, g):
        x, g = x.contiguous(), g.contiguous()
        ctx.save_for_backward(x, g)
        return S.s2_wgrad(x, g)

    @staticmethod
    def backward(ctx, ggW):
        x, g = ctx.saved_tensors
        ggW = _as(ggW, F32)
        gx = gg = None
        if _needed(ctx, 0):
            gx = S2TFn.apply(g, ggW, None, None)
        if _needed(ctx, 1):
            gg = S2Fn.apply(x, ggW, None, None)
        return gx, gg


# --------------------------------------------------------------------------- 2x resampling
class Up2Fn(torch.autograd.Function):
    """y = s * upscale2d(x) on the native kernel; its adjoint is s * 2x2 sum-pool (Down2Fn)."""

    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return S.upscale2x(x.contiguous(), scale=s)

    @staticmethod
    def backward(ctx, g):
        return Down2Fn.apply(g.contiguous(), ctx.s), None


class Down2Fn(torch.autograd.Function):
    """y = s * (2x2 sum of x) on the native kernel (s = 0.25: downscale2d); adjoint s * upscale2d."""

    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return S.downscale2x(x.contiguous(), scale=s)

    @staticmethod
    def backward(ctx, g):
        return Up2Fn.apply(g.contiguous(), ctx.s), None


# ------------------------------------------------------------------------------------ dense
class DenseFn(torch.autograd.Function):
    """y = act(x @ w.T + b)   (x [M, K] bf16, w fp32 [N, K]; act as in ConvFn)."""

    @staticmethod
    def forward(ctx, x, w, b, wb, slope):
        x = x.contiguous()
        bd = None if b is None else b.detach().float().contiguous()
        if x.dtype == F32:
            y = S.linear(x, w.detach().contiguous(), bd, act=_act(slope), slope=0.2 if slope is None else slope)
        else:
            y = F.linear(x, _wshadow(w, wb), bd, act=_act(slope), slope=0.2 if slope is None else slope)
        ctx.dt = x.dtype
        if slope is None:
            ctx.save_for_backward(x, w)
        else:
            ctx.save_for_backward(x, w, y)
        ctx.wb, ctx.has_b, ctx.slope, ctx.b = wb, b is not None, slope, b
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors[:2]
        gb, b_done = None, False
        if ctx.slope is not None:
            y = ctx.saved_tensors[2]
            if (ctx.has_b and _needed(ctx, 2) and not torch.is_grad_enabled() and gy.is_cuda
                    and gy.dtype == F32 and y.dtype == F32 and gy.is_contiguous()):
                # outside a create_graph backward: gate + bias gradient in one pass over gy
                gy, gb = _gate_colsum(ctx, gy, y, ctx.b)
                b_done = True
            else:
                gy = _lrelu_gate(gy, y, ctx.slope)
        gy = _as(gy, ctx.dt)
        gx = gw = None
        if _needed(ctx, 0):
            gx = DenseDxFn.apply(gy, w, ctx.wb)
        if _needed(ctx, 1):
            buf = _param_grad_buffer(w) if x.dtype == F32 else None
            if buf is not None:
                S.linear_dw(gy.contiguous(), x.contiguous(), out=buf, accumulate=True)
            else:
                gw = DenseDwFn.apply(x, gy)
        if ctx.has_b and _needed(ctx, 2) and not b_done:
            gb = _bias_grad_into(gy, ctx.b)
        return gx, gw, gb, None, None


class DenseDxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gy, w, wb):
        gy = gy.contiguous()
        if gy.dtype == F32:
            dx = S.linear_dx(gy, w.detach().contiguous())
        else:
            dx = F.linear_dx(gy, _wshadow(w, wb))
        ctx.save_for_backward(gy, w)
        ctx.wb, ctx.dt = wb, gy.dtype
        return dx

    @staticmethod
    def backward(ctx, ggx):
        gy, w = ctx.saved_tensors
        ggx = _as(ggx, ctx.dt)
        g_gy = g_w = None
        if _needed(ctx, 0):
            g_gy = DenseFn.apply(ggx, w, None, ctx.wb, None)
        if _needed(ctx, 1):
            buf = _param_grad_buffer(w) if gy.dtype == F32 and ggx.dtype == F32 else None
            if buf is not None:
                S.linear_dw(gy.contiguous(), ggx.contiguous(), out=buf, accumulate=True)
            else:
                g_w = DenseDwFn.apply(ggx, gy)
        return g_gy, g_w, None


class DenseDwFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gy):
        x, gy = x.contiguous(), gy.contiguous()
        dw = S.linear_dw(gy, x) if x.dtype == F32 else F.linear_dw(gy, x)
        ctx.save_for_backward(x, gy)
        return dw

    @staticmethod
    def backward(ctx, ggw):
        x, gy = ctx.saved_tensors
        ggw = ggw.contiguous()
        g_x = g_gy = None
        if _needed(ctx, 0):
            g_x = DenseDxFn.apply(gy, ggw, None)
        if _needed(ctx, 1):
            g_gy = DenseFn.apply(x, ggw, None, None, None)
        return g_x, g_gy


def dense(x, w, b=None, *, wb=None, lrelu=None):
    if x.device.type != 'cuda':
        y = TF.linear(x, w.to(x.dtype), None if b is None else b.to(x.dtype))
        return y if lrelu is None else leaky_relu(y, lrelu)
    return DenseFn.apply(x, w, b, wb, None if lrelu is None else float(lrelu))


# ---------------------------------------------------------------------------- elementwise glue
class LReluFn(torch.autograd.Function):
    """y = max(x, slope x) on the native gate kernel (lrelu_gate(x, x) = x (x > 0 ? 1 : slope)); backward is
    the gate read from y (LReluGateFn), itself differentiable, so WGAN-GP's double backward goes through."""

    @staticmethod
    def forward(ctx, x, slope):
        y = S.lrelu_gate(x, x, slope)
        ctx.save_for_backward(y)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        return _lrelu_gate(gy.contiguous(), y, ctx.slope), None


def leaky_relu(x, slope=0.2):
    """max(x*a, x) (pg_gans.py:987-990); twice differentiable (native kernels on fp32 GPU tensors)."""
    if x.is_cuda and x.dtype == F32 and x.is_contiguous() and x.numel() % 4 == 0:
        return LReluFn.apply(x, float(slope))
    return TF.leaky_relu(x, slope)


def pixel_norm(x, eps=1e-8):
    """x * rsqrt(mean_c(x^2) + eps) over the channel (last) axis, fp32 accumulation (pg_gans.py:993-995)."""
    xf = x.float()
    return (xf * torch.rsqrt(xf.square().mean(-1, keepdim=True) + eps)).to(x.dtype)


class LReluPixelNormFn(torch.autograd.Function):
    """z = pixel_norm(leaky_relu(x + b)) in one fused HIP pass (the generator's per-layer epilogue,
    pg_gans.py:853-869).  Generator-side only, so once-differentiable: WGAN-GP differentiates the
    discriminator twice, never the generator."""

    @staticmethod
    def forward(ctx, x, b, slope, eps):
        x = x.contiguous()
        bd = None if b is None else b.detach().float().contiguous()
        z = F.lrelu_pixelnorm(x, bd, slope=slope, eps=eps)
        ctx.save_for_backward(x)
        ctx.bd, ctx.slope, ctx.eps, ctx.has_b, ctx.b = bd, slope, eps, b is not None, b
        return z

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gz):
        (x,) = ctx.saved_tensors
        gx = F.lrelu_pixelnorm(x, ctx.bd, slope=ctx.slope, eps=ctx.eps, dz=gz)
        gb = None
        if ctx.has_b and ctx.needs_input_grad[1]:
            gb = _bias_grad_into(gx, ctx.b)
        return (gx if ctx.needs_input_grad[0] else None), gb, None, None


def lrelu_pixel_norm(x, b=None, slope=0.2, eps=1e-8):
    """pixel_norm(leaky_relu(x + b)); fused HIP kernel on GPU, torch composite on CPU."""
    if x.device.type != 'cuda':
        return pixel_norm(leaky_relu(x if b is None else x + b.to(x.dtype), slope), eps)
    return LReluPixelNormFn.apply(x, b, float(slope), float(eps))


class MbstdFn(torch.autograd.Function):
    """Minibatch-stddev feature (pg_gans.py:1070-1082) on the fused HIP kernels; its backward is
    MbstdBwdFn so the WGAN-GP penalty can differentiate through it once more."""

    @staticmethod
    def forward(ctx, x, group, segs, cp):
        ctx.save_for_backward(x)
        ctx.group, ctx.segs = group, segs
        return F.mbstd(0, x, group=group, segs=segs, cp=cp)

    @staticmethod
    def backward(ctx, gout):
        (x,) = ctx.saved_tensors
        return MbstdBwdFn.apply(gout, x, ctx.group, ctx.segs), None, None, None


class MbstdBwdFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gout, x, group, segs):
        gout = _as(gout, x.dtype)
        ctx.save_for_backward(gout, x)
        ctx.group, ctx.segs = group, segs
        return F.mbstd(1, x, gout, group=group, segs=segs)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, ggx):
        gout, x = ctx.saved_tensors
        g_x, gg_out = F.mbstd(2, x, ggx, gout, group=ctx.group, segs=ctx.segs)
        return (gg_out if ctx.needs_input_grad[0] else None), (g_x if ctx.needs_input_grad[1] else None), None, None


def minibatch_stddev(x, group_size=4, pad_to=8, segs=1):
    """Append the group-stddev feature map (pg_gans.py:1070-1082) and zero-pad the channel count
    to a multiple of ``pad_to`` so the following conv can run on the MFMA path (512+1 -> 520).
    ``segs`` > 1: x is that many independent minibatches stacked (grouping stays inside each)."""
    N, H, W, C = x.shape
    g = min(group_size, N // segs)
    if x.device.type == 'cuda' and x.dtype in (BF16, F32) and g <= 8 and (N // segs) % g == 0:
        return MbstdFn.apply(x, g, segs, C + 1 + (-(C + 1)) % pad_to)
    if segs > 1:
        return torch.cat([minibatch_stddev(t, group_size, pad_to) for t in x.chunk(segs)], 0)
    g = min(group_size, N)
    y = x.float().reshape(g, -1, H, W, C)
    y = y - y.mean(0, keepdim=True)
    y = (y.square().mean(0) + 1e-8).sqrt()
    y = y.mean((1, 2, 3))  # [N/g]
    y = y.reshape(1, -1, 1, 1, 1).expand(g, -1, H, W, 1).reshape(N, H, W, 1).to(x.dtype)
    extra = (-(C + 1)) % pad_to
    parts = [x, y]
    if extra:
        parts.append(x.new_zeros((N, H, W, extra)))
    return torch.cat(parts, -1)
