"""fp32 tensor ops over the gfx950 kernels (``csrc/kernels/sgemm.hip`` + ``bnf.hip``) — the
reference-precision training path.  Every GEMM runs on v_mfma_f32_32x32x2_f32 (exact fp32 products,
fp32 accumulation); activations, gradients and BatchNorm are fp32.  The reference trains in fp32
everywhere (pg_gans.py:830,914; Keras defaults in TfFeedForward.py / TfVgg16.py).

Layouts (all device tensors contiguous):
  * activations  : NHWC fp32 ``[N, H, W, C]`` with C % 4 == 0 (the stem pads RGB to 4 channels)
  * conv weights : fp32 ``[Cout, kh, kw, Cin]`` (GEMM B operand ``[N][K]``, K = taps*Cin)
  * dense weights: fp32 ``[out, in]``

Every function launches on the current HIP stream and allocates only through the torch caching
allocator, so whole steps capture into one hipGraph.  Tile shape / LDS-ring depth / split-K are
picked per layer shape by the autotuner (``rafiki_amd.ops.autotune``) outside capture.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import _lib, autotune
from .functional import ACT_LRELU, ACT_NONE, ACT_RELU, bn_slots, cdiv  # noqa: F401

KIND_CONV, KIND_WGRAD, KIND_DENSE, KIND_DENSE_DX, KIND_DENSE_DW = 0, 2, 3, 4, 5
F_RELU, F_BIAS, F_STATS, F_GATE, F_ACCUM, F_LRELU, F_BNB, F_BNP = 1, 2, 4, 8, 16, 32, 512, 1024
# block tiles (see rk_sgemm): 0-3 four-wave 2x2, 4 256x64 (4x1 waves), 5 256x128 / 6 128x256 (8 waves),
# 7 64x256 (1x4).  Tiles 4-7 exist for the conv kinds with C % 32 == 0 and the weight gradient.
TILES = [(128, 128), (128, 64), (64, 128), (64, 64), (256, 64), (256, 128), (128, 256), (64, 256),
         (64, 64), (128, 64), (64, 128)]   # 8-10: 1- / 2-wave tiles of 64x64 wave tiles (X6 candidates)
_NST3 = (0, 1, 2, 3, 4, 7)   # 3-stage rings: 4-wave tiles only (sgemm.hip s_launch)
_FEW_WAVE = (8, 9, 10)
NUM_CU = 256
# tile code + X6: the split-bf16 K loop of rk_sgemm (fp32-accurate products on the bf16 MFMA: every
# fp32 operand value = three bf16 pieces, six v_mfma_f32_32x32x16_bf16 per 16-deep chunk; see
# sgemm.hip).  RAFIKI_X6=0 keeps every GEMM on v_mfma_f32_32x32x2_f32.
X6 = 16
USE_X6 = os.environ.get('RAFIKI_X6', '1') != '0'


def tile_dims(t: int):
    """(BM, BN) of a tile code (X6 codes included)."""
    return TILES[t & 15]




def _p(t: Optional[torch.Tensor]):
    """Device pointer of a kernel operand; a host tensor here would be an illegal GPU access."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError('host tensor {} {} passed to a gfx950 kernel'.format(tuple(t.shape), t.dtype))
    return t.data_ptr()


def _nbytes(t):
    return t.untyped_storage().nbytes() - t.storage_offset() * t.element_size()


def _s():
    return torch.cuda.current_stream().cuda_stream


def _check(t, name):
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError('{}: contiguous fp32 tensor required (got {} contiguous={})'.format(
            name, t.dtype, t.is_contiguous()))


def sgemm(kind, A, B, out, M, N, K, lda, ldb, ldc, *, tile=0, nst=2, splits=1, slab_stride=0, bias=None,
          stats=None, gate=None, H=1, W=1, C=4, taps=1, flags=0, alpha=1.0, slope=0.2):
    slot_mask = 0
    if stats is not None:
        assert stats.dtype == torch.float64 and stats.is_contiguous()
        slot_mask = stats.shape[0] - 1
    _lib.call("rk_sgemm", int(kind), int(tile), int(nst), _p(A), _p(B), _p(out), _p(bias), _p(stats), int(slot_mask),
              _p(gate), int(M), int(N), int(K), int(lda), int(ldb), int(ldc), int(H), int(W), int(C), int(taps),
              int(splits), int(slab_stride), int(flags), float(alpha), float(slope), _nbytes(A), _nbytes(B), _s())
    return out


# ------------------------------------------------------------------------------ config selection
def pick_tile(M: int, N: int) -> int:
    """Largest tile that still puts >= one block on every CU (else the tile with most blocks)."""
    best, best_blocks = 3, -1
    for t, (bm, bn) in enumerate(TILES[:4]):
        blocks = cdiv(M, bm) * cdiv(N, bn)
        waste = (cdiv(M, bm) * bm * cdiv(N, bn) * bn) / float(M * N)
        if waste > 1.3 and t != 3:
            continue
        if blocks >= NUM_CU:
            return t
        if blocks > best_blocks:
            best, best_blocks = t, blocks
    return best


def _cands(M, N, splittable=False, K=0, big=False):
    """(tile, nst, splits) configs: the heuristic first, then every tile x ring depth (``big``: also the
    256-wide tiles), plus split-K variants for grids that leave the chip idle."""
    t0 = pick_tile(M, N)
    out = [(t0, 2, 1)]
    tiles = range(8 if big else 4)
    for t in tiles:
        bm, bn = TILES[t]
        if t >= 4 and (cdiv(M, bm) * bm * cdiv(N, bn) * bn) / float(M * N) > 1.3:
            continue  # the big tiles only where they do not mostly compute padding
        for nst in ((2, 3) if t in _NST3 else (2,)):
            c = (t, nst, 1)
            if c not in out:
                out.append(c)
    if splittable:
        kt = cdiv(K, 32)
        for t in tiles:
            bm, bn = TILES[t]
            if t >= 4 and (cdiv(M, bm) * bm * cdiv(N, bn) * bn) / float(M * N) > 1.3:
                continue
            blocks = cdiv(M, bm) * cdiv(N, bn)
            for s in (2, 4, 8, 16, 32, 64, 128, 256):
                if s > kt // 2 or blocks * s > 8 * NUM_CU or s * M * N * 4 > (512 << 20):
                    continue
                if blocks * s < NUM_CU // 2:
                    continue
                s_eff = cdiv(kt, cdiv(kt, s))
                for nst in ((2, 3) if t in _NST3 else (2,)):
                    c = (t, nst, s_eff)
                    if c not in out:
                        out.append(c)
    if USE_X6:
        x6 = [(t + X6, nst, s) for (t, nst, s) in out if t < 4 or t >= 4]
        # the few-wave 64x64-wave-tile shapes, X6 only (their point is the split VALU per MFMA)
        for t in _FEW_WAVE:
            bm, bn = TILES[t]
            if (cdiv(M, bm) * bm * cdiv(N, bn) * bn) / float(M * N) > 1.3:
                continue
            x6.append((t + X6, 2, 1))
        out += x6
    return out


def _pick(key, cands, run, protect=()):
    """The tuned config for ``key``.  ``protect``: tensors the op accumulates into — a tuning sweep runs
    every candidate several times, so their contents are saved first and restored afterwards."""
    if not autotune.ENABLED:
        return cands[0]
    if protect and not autotune._valid(autotune.lookup(key), cands) and autotune.can_tune():
        saved = [t.clone() for t in protect]
        cfg = autotune.tune(key, cands, run)
        for t, v in zip(protect, saved):
            t.copy_(v)
        return cfg
    return autotune.tune(key, cands, run)


def _slots_flags(acc):
    return 0 if acc is None else acc.shape[0] - 1


# ------------------------------------------------------------------------------------------ conv
def conv_fwd(x: torch.Tensor, w: torch.Tensor, *, taps: int = 9, stats_acc=None, bias=None, act=ACT_NONE,
             slope=0.2, out=None, wino=None, wino4=None, wino4p=None, wino4b=None, pro=None):
    """y = conv3x3(x, w) (stride 1, pad 1; taps=1: 1x1) [+bias][act]; with ``stats_acc`` (zeroed fp64
    [SL][2][Cout]) the per-channel (sum y, sum y^2) BatchNorm statistics ride in the epilogue.
    ``wino``: the layer's Winograd weights (WinoWeights.u), or a callable producing them (run only
    when a Winograd candidate runs, so the tuner times transform + conv) -> the fused F(2x2,3x3)
    kernels are more autotune candidates; ``wino4`` likewise for the F(4x4,3x3) kernels (WinoWeights.u4),
    ``wino4p`` the X6 weight planes (WinoWeights 'u4p') of the pre-split pre-transformed F(4x4) path.
    ``pro``: normalise-on-load — x is the pre-BN output y of the previous conv, pro = its coeffs
    (bn_finalize): every candidate loads relu(y * scale + shift) (the F(4x4) kernels with blocked weights
    and the pre-transformed paths; see bn_on_load_ok)."""
    _check(x, 'conv_fwd x')
    Nb, H, W, Cin = x.shape
    Cout = w.shape[0]
    M, K = Nb * H * W, taps * Cin
    assert w.numel() == Cout * K, (w.shape, taps, Cin)
    if out is None:
        out = torch.empty((Nb, H, W, Cout), device=x.device, dtype=torch.float32)
    flags = (F_STATS if stats_acc is not None else 0) | (F_BIAS if bias is not None else 0)
    flags |= F_RELU if act == ACT_RELU else F_LRELU if act == ACT_LRELU else 0

    use_w = wino is not None and taps == 9 and wino_ok(H, W, Cin) and act in (ACT_NONE, ACT_RELU)
    use_w4 = wino4 is not None and taps == 9 and wino4_ok(H, W, Cin) and act in (ACT_NONE, ACT_RELU)
    use_w4b = wino4b is not None and taps == 9 and wino4_ok(H, W, Cin) and act in (ACT_NONE, ACT_RELU)
    # the pre-transformed paths also carry a leaky-ReLU epilogue (no statistics with it): PG-GAN's D convs
    act_pt = act in (ACT_NONE, ACT_RELU) or (act == ACT_LRELU and stats_acc is None)
    use_pt = (wino4 is not None and taps == 9 and wino4_ok(H, W, Cin) and act_pt and wino4_pt_ok(H, W, Cin, Cout))
    use_ptx = wino4p is not None and taps == 9 and wino4_ptx_ok(H, W, Cin, Cout) and act_pt
    lrelu = slope if act == ACT_LRELU else None

    def run(cfg):
        tile, nst, s = cfg
        if tile == WINO4_PTX:
            wino4_conv_pt(x, wino4p() if callable(wino4p) else wino4p, out=out, bias=bias, stats=stats_acc,
                          relu=act == ACT_RELU, tile=nst // 4, nst=nst % 4, splits=s, lrelu=lrelu, pro=pro)
            return
        if tile == WINO4_PT:
            wino4_conv_pt(x, wino4() if callable(wino4) else wino4, out=out, bias=bias, stats=stats_acc,
                          relu=act == ACT_RELU, tile=nst, nst=s, lrelu=lrelu, pro=pro)
            return
        if cfg in WINO4_CFGS:
            wino4_conv(x, wino4() if callable(wino4) else wino4, out=out, bias=bias, stats=stats_acc,
                       relu=act == ACT_RELU, variant=_wino4_variant(cfg))
            return
        if cfg in WINO4B_CFGS:
            wino4_conv(x, wino4b() if callable(wino4b) else wino4b, out=out, bias=bias, stats=stats_acc,
                       relu=act == ACT_RELU, variant=_WINO4B_VARIANT[cfg[0]], n_out=Cout, pro=pro)
            return
        if cfg in WINO_CFGS:
            wino_conv(x, wino() if callable(wino) else wino, out=out, bias=bias, stats=stats_acc,
                      relu=act == ACT_RELU, variant=_wino_variant(cfg))
            return
        if s == 1:
            sgemm(KIND_CONV, x, w, out, M, Cout, K, Cin, K, Cout, tile=tile, nst=nst, bias=bias, stats=stats_acc,
                  H=H, W=W, C=Cin, taps=taps, flags=flags, slope=slope)
            return
        # small-M deep layers (inference at small batch: 4x4 maps, K = 9 x 512): split-K slabs + one
        # combine that applies bias / activation
        slab = torch.empty((s, M, Cout), device=x.device, dtype=torch.float32)
        sgemm(KIND_CONV, x, w, slab, M, Cout, K, Cin, K, Cout, tile=tile, nst=nst, splits=s, slab_stride=M * Cout,
              H=H, W=W, C=Cin, taps=taps)
        sreduce_epi(slab, M, Cout, out.view(M, Cout), bias=bias, act=act, slope=slope)
    if pro is not None:   # only the kernels that normalise on load are candidates
        assert bias is None and act == ACT_NONE and pro.shape == (4, Cin)
        use_w = use_w4 = False
        cands = []
    else:
        cands = _cands(M, Cout, splittable=stats_acc is None and Cout % 4 == 0, K=K, big=Cin % 32 == 0)
    if use_w:
        cands.extend(WINO_CFGS)
    if use_w4:
        cands.extend(WINO4_CFGS)
    if use_w4b:
        cands.extend(WINO4B_CFGS)
    if use_pt:
        cands.extend(WINO4_PT_CFGS)
    if use_ptx:
        cands.extend(WINO4_PTX_CFGS)
    if not cands:
        raise ValueError('conv_fwd(pro=...): no normalise-on-load kernel for this shape (see bn_on_load_ok)')
    cfg = _pick(('sf', M, Cout, K, H, W, Cin, taps, flags, 'lazy' if callable(wino) else use_w,
                 'lazy' if callable(wino4) else use_w4, use_pt, 'lazy' if callable(wino4p) else use_ptx)
                + (('b', 'lazy' if callable(wino4b) else True),) * use_w4b + (('pro',) if pro is not None else ()),
                cands, run)
    if stats_acc is not None and autotune.can_tune():
        stats_acc.zero_()  # tuning runs accumulated into it
    run(cfg)
    return out


def conv_dgrad(dy: torch.Tensor, wt, *, taps: int = 9, out=None, gate=None, bnb=None, bnp=None,
               wino=None, wino4=None, cin=None, wino4p=None, wino4b=None):
    """dx = data gradient of a 3x3 conv as conv3x3(dy, wt) with wt = SConvWT.view() [Cin][taps*Cout].
    Epilogue options: ``gate`` (ReLU mask of the input activation), ``bnb = (y, coeffs, acc)`` (the input
    is BN+ReLU(y): mask + BN-backward sums into acc), ``bnp = (y, coeffs, acc)`` (the input is
    maxpool(BN+ReLU(y)), y at 2x resolution: routing + sums; dx stays the pooled gradient)."""
    _check(dy, 'conv_dgrad dy')
    Nb, H, W, Cout = dy.shape
    # wt / wino may be callables (weights prepared per call, inside the timed candidate): then ``cin``
    Cin = cin if callable(wt) else wt.shape[0]
    M, K = Nb * H * W, taps * Cout
    assert callable(wt) or wt.numel() == Cin * K
    if out is None:
        out = torch.empty((Nb, H, W, Cin), device=dy.device, dtype=torch.float32)
    flags, bias, stats = 0, None, None
    if bnb is not None:
        y, coeffs, stats = bnb
        assert y.shape == out.shape and stats.dtype == torch.float64 and stats.shape[-1] == Cin
        gate, bias, flags = y, coeffs[2:4].reshape(-1), F_BNB
    elif bnp is not None:
        y, coeffs, stats = bnp
        assert y.shape == (Nb, 2 * H, 2 * W, Cin) and stats.dtype == torch.float64
        assert not (H & (H - 1)) and not (W & (W - 1)), 'pooled BN fusion needs power-of-two maps'
        gate, bias, flags = y, coeffs[2:4].reshape(-1), F_BNP
    elif gate is not None:
        flags = F_GATE
    # ``wino``: the layer's Winograd data-gradient weights (WinoWeights.ut), one more candidate
    use_w = wino is not None and taps == 9 and wino_ok(H, W, Cout) and not (flags & F_GATE)
    use_w4 = wino4 is not None and taps == 9 and wino4_ok(H, W, Cout) and not (flags & F_GATE)
    use_w4b = wino4b is not None and taps == 9 and wino4_ok(H, W, Cout) and not (flags & F_GATE)

    use_pt = use_w4 and wino4_pt_ok(H, W, Cout, Cin)
    # ``wino4p``: the X6 planes of the data-gradient set (WinoWeights 'ut4p'): the pre-split PT path
    use_ptx = wino4p is not None and taps == 9 and wino4_ptx_ok(H, W, Cout, Cin) and not (flags & F_GATE)

    def run(cfg):
        if cfg[0] == WINO4_PTX:
            wino4_conv_pt(dy, wino4p() if callable(wino4p) else wino4p, out=out, bnb=bnb, bnp=bnp, tile=cfg[1] // 4,
                          nst=cfg[1] % 4, splits=cfg[2])
            return
        if cfg[0] == WINO4_PT:
            wino4_conv_pt(dy, wino4() if callable(wino4) else wino4, out=out, bnb=bnb, bnp=bnp, tile=cfg[1],
                          nst=cfg[2])
            return
        if cfg in WINO4_CFGS:
            wino4_conv(dy, wino4() if callable(wino4) else wino4, out=out, bnb=bnb, bnp=bnp,
                       variant=_wino4_variant(cfg))
            return
        if cfg in WINO4B_CFGS:
            wino4_conv(dy, wino4b() if callable(wino4b) else wino4b, out=out, bnb=bnb, bnp=bnp,
                       variant=_WINO4B_VARIANT[cfg[0]], n_out=Cin)
            return
        if cfg in WINO_CFGS:
            wino_conv(dy, wino() if callable(wino) else wino, out=out, bnb=bnb, bnp=bnp, variant=_wino_variant(cfg))
            return
        sgemm(KIND_CONV, dy, wt() if callable(wt) else wt, out, M, Cin, K, Cout, K, Cin, tile=cfg[0], nst=cfg[1], bias=bias, stats=stats,
              gate=gate, H=H, W=W, C=Cout, taps=taps, flags=flags)
    cands = _cands(M, Cin, big=Cout % 32 == 0)
    if use_w:
        cands.extend(WINO_CFGS)
    if use_w4:
        cands.extend(WINO4_CFGS)
    if use_w4b:
        cands.extend(WINO4B_CFGS)
    if use_pt:
        cands.extend(WINO4_PT_CFGS)
    if use_ptx:
        cands.extend(WINO4_PTX_CFGS)
    cfg = _pick(('sd', M, Cin, K, H, W, Cout, taps, flags, 'lazy' if callable(wino) else use_w,
                 'lazy' if callable(wino4) else use_w4, use_pt, 'lazy' if callable(wino4p) else use_ptx)
                + (('b', 'lazy' if callable(wino4b) else True),) * use_w4b, cands, run)
    if stats is not None and autotune.can_tune():
        stats.zero_()
    run(cfg)
    return out


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, *, taps: int = 9, out=None, accumulate=False, xpro=None):
    """dW[co][tap][ci] (fp32 [Cout][taps*Cin]) = sum over pixels of dy[p][co] * x[shift_tap(p)][ci].
    ``xpro``: x is the pre-BN output of its producer and xpro that BN's coeffs (bn_finalize): the F(4x4)
    kernels normalise + ReLU it on load (the only candidates then; see bn_on_load_ok)."""
    _check(dy, 'conv_wgrad dy')
    _check(x, 'conv_wgrad x')
    Nb, H, W, Cout = dy.shape
    Cin = x.shape[-1]
    M, N, K = Cout, taps * Cin, Nb * H * W
    if out is None:
        out = torch.empty((Cout, N), device=dy.device, dtype=torch.float32)

    def run(cfg):
        tile, nst, s = cfg
        if tile == WINO_WGRAD:
            wino_wgrad(dy, x, out, splits=s, accumulate=accumulate)
            return
        if tile == WINO4_WGRAD:
            wino4_wgrad(dy, x, out, splits=s, accumulate=accumulate, variant=nst, xpro=xpro)
            return
        if tile == WINO4_WGRAD_PT:
            wino4_wgrad_pt(dy, x, out, accumulate=accumulate, tile=nst, nst=s, xpro=xpro)
            return
        if tile == WINO4_WGRAD_PTX:
            wino4_wgrad_pt(dy, x, out, accumulate=accumulate, tile=nst // 4, nst=nst % 4, planes=True, splits=s)
            return
        if s == 1:
            sgemm(KIND_WGRAD, dy, x, out, M, N, K, Cout, Cin, N, tile=tile, nst=nst, H=H, W=W, C=Cin, taps=taps,
                  flags=F_ACCUM if accumulate else 0)
            return
        slab = torch.empty((s, M, N), device=dy.device, dtype=torch.float32)
        sgemm(KIND_WGRAD, dy, x, slab, M, N, K, Cout, Cin, N, tile=tile, nst=nst, splits=s, slab_stride=M * N,
              H=H, W=W, C=Cin, taps=taps)
        reduce_slabs(slab, out, accumulate=accumulate)
    cands = _cands(M, N, splittable=True, K=K, big=True)
    # the split-K configs fill the chip: lead with the best-filling heuristic one
    split = [c for c in cands if c[2] > 1]
    if split:
        cands = [max(split, key=lambda c: min(cdiv(M, tile_dims(c[0])[0]) * cdiv(N, tile_dims(c[0])[1]) * c[2],
                                              2 * NUM_CU))] + cands
    wcands = _wino_wgrad_cands(Nb, H, W, Cout, Cin) if taps == 9 else []
    w4cands = _wino4_wgrad_cands(Nb, H, W, Cout, Cin) if taps == 9 else []
    ptcands = _wino4_pt_cands(Nb, H, W, Cout, Cin) if taps == 9 else []
    ptxcands = _wino4_ptx_wgrad_cands(Nb, H, W, Cout, Cin) if taps == 9 else []
    if xpro is not None:
        assert taps == 9 and xpro.shape == (4, Cin)
        cands, wcands, ptxcands = w4cands + ptcands, [], []
        if not cands:
            raise ValueError('conv_wgrad(xpro=...): no normalise-on-load kernel for this shape (see bn_on_load_ok)')
    else:
        cands += wcands + w4cands + ptcands + ptxcands
    cfg = _pick(('sw', M, N, K, H, W, Cin, taps, bool(accumulate), bool(wcands), bool(w4cands), bool(ptcands),
                 bool(ptxcands)) + (('pro',) if xpro is not None else ()), cands, run,
                protect=(out,) if accumulate else ())
    run(cfg)
    return out


class SConvWT:
    """Flipped, transposed fp32 copies wt[ci][taps-1-t][co] = w[co][t][ci] of several conv weights living
    in one fp32 arena, refreshed by ONE rk_swt launch per step; with them the data gradient is a forward
    conv of dy on the forward kernels (``conv_dgrad``)."""

    def __init__(self, arena: torch.Tensor, weights, taps: int = 9):
        self.arena = arena
        meta, desc, self._views, off = [], [], [], 0
        for l, w in enumerate(weights):
            Cout = w.shape[0]
            Cin = w.numel() // (taps * Cout)
            so = (w.data_ptr() - arena.data_ptr()) // 4
            meta.append([so, off, Cout, Cin, taps])
            for t in range(taps):
                for co0 in range(0, Cout, 32):
                    for ci0 in range(0, Cin, 32):
                        desc.append([l, t, co0, ci0])
            self._views.append((off, Cin, Cout))
            off += (Cin * taps * Cout + 63) // 64 * 64
        dev = arena.device
        self.taps = taps
        self.buf = torch.zeros(max(off, 64), dtype=torch.float32, device=dev)
        self.meta = torch.tensor(meta, dtype=torch.int64, device=dev)
        self.desc = torch.tensor(desc, dtype=torch.int32, device=dev)

    _fresh = False

    def refresh(self):
        _lib.call("rk_swt", _p(self.arena), _p(self.buf), _p(self.desc), self.desc.shape[0], _p(self.meta), _s())
        self._fresh = True

    def begin_step(self):
        """The weights change every step: the next lazy() read refreshes (one launch) first."""
        self._fresh = False

    def lazy(self, l: int):
        """Callable view for conv_dgrad's direct candidates: the refresh launch runs only in steps whose
        tuned data gradients use the direct kernel (Winograd ones read WinoWeights instead)."""
        def get():
            if not self._fresh:
                self.refresh()
            return self.view(l)
        return get

    def view(self, l: int) -> torch.Tensor:
        off, Cin, Cout = self._views[l]
        return self.buf[off:off + Cin * self.taps * Cout].view(Cin, self.taps * Cout)


# -------------------------------------------------------------------- Winograd F(2x2, 3x3) convs
WF_RELU, WF_BIAS, WF_STATS, WF_LRELU, WF_BNB, WF_BNP, WF_POOL = 1, 2, 4, 8, 512, 1024, 2048
WINO = os.environ.get('RAFIKI_WINOGRAD', '1') != '0'
# autotune candidates that run rk_wino_conv: 4-wave 64x32 tiles (variant 0) / 8-wave 64x64 (variant 1),
# and the 16x16-wave-tile kernels of winograd4.hip: 4-wave 32x32 (variant 2), 2-wave 16x32 (variant 3),
# 8-wave 64x32 (variant 4)
# software-pipelined (two LDS stage) variants: the F(2x2) 8-wave one wins the 4x4-map layers and is a
# candidate; the F(4x4) ones (one wave per SIMD) measured 1.3-1.5x slower than the single-stage kernels on
# every VGG-small layer (profiles/winograd_variants_r2e.jsonl) and are not offered to the tuner (kept
# callable as variant 2 of rk_wino4_conv / rk_wino4_wgrad_v, exercised by tests/test_winograd4_gpu.py)
WINO_CFGS = ((-1, 0, 1), (-2, 0, 1), (-8, 0, 1), (-9, 0, 1), (-10, 0, 1), (-12, 0, 1))
_WINO_VARIANT = {-1: 0, -2: 1, -8: 2, -9: 3, -10: 4, -12: 5}   # -12: 8-wave 64x32, two-stage pipelined


def _wino_variant(cfg):
    return _WINO_VARIANT[cfg[0]]


def wino_ok(H: int, W: int, C: int) -> bool:
    """Shapes the fused Winograd kernel takes: stride-1 3x3, even maps, C % 8 == 0."""
    return WINO and H % 2 == 0 and W % 2 == 0 and C % 8 == 0 and C > 0


def wino_weights(w: torch.Tensor, u: torch.Tensor, ut: Optional[torch.Tensor] = None):
    """u [16][Cout][Cin] = G g G^T of w [Cout][9*Cin]; ut [16][Cin][Cout]: the data-gradient set."""
    Cout = w.shape[0]
    Cin = w.numel() // (9 * Cout)
    assert u.numel() == 16 * Cout * Cin and (ut is None or ut.numel() == 16 * Cout * Cin)
    _lib.call("rk_wino_weights", _p(w), _p(u), _p(ut), Cout, Cin, _s())
    return u, ut


def wino_u(w: torch.Tensor) -> torch.Tensor:
    """Forward Winograd weights [16][Cout][Cin] of one conv weight [Cout, 3, 3, Cin] (fresh buffer)."""
    Cout = w.shape[0]
    u = torch.empty((16, Cout, w.numel() // (9 * Cout)), device=w.device, dtype=torch.float32)
    _lib.call("rk_wino_weights", _p(w), _p(u), None, Cout, u.shape[2], _s())
    return u


def wino_ut(w: torch.Tensor) -> torch.Tensor:
    """Data-gradient Winograd weights [16][Cin][Cout] of one conv weight [Cout, 3, 3, Cin]."""
    Cout = w.shape[0]
    Cin = w.numel() // (9 * Cout)
    u = torch.empty((16, Cout, Cin), device=w.device, dtype=torch.float32)
    ut = torch.empty((16, Cin, Cout), device=w.device, dtype=torch.float32)
    _lib.call("rk_wino_weights", _p(w), _p(u), _p(ut), Cout, Cin, _s())
    return ut


def wino_conv(x: torch.Tensor, u: torch.Tensor, *, out=None, bias=None, stats=None, relu=False, bnb=None, bnp=None,
              variant=0):
    """y = conv3x3(x, w) (stride 1, pad 1) from u = wino_weights(w): x [Nb, H, W, C] fp32 NHWC.
    ``stats``: fp64 BN slots (sum y, sum y^2); ``bnb`` / ``bnp`` = (y, coeffs, acc) as in conv_dgrad."""
    _check(x, 'wino_conv x')
    Nb, H, W, C = x.shape
    N = u.shape[1]
    assert u.shape == (16, N, C) and u.is_contiguous(), (u.shape, x.shape)
    if out is None:
        out = torch.empty((Nb, H, W, N), device=x.device, dtype=torch.float32)
    assert out.shape == (Nb, H, W, N) and out.is_contiguous()
    flags, gate = 0, None
    if bias is not None:
        flags |= WF_BIAS
    if relu:
        flags |= WF_RELU
    if stats is not None:
        flags |= WF_STATS
    if bnb is not None:
        gate, coeffs, stats = bnb
        assert gate.shape == out.shape
        bias, flags = coeffs[2:4].reshape(-1), WF_BNB
    elif bnp is not None:
        gate, coeffs, stats = bnp
        assert gate.shape == (Nb, 2 * H, 2 * W, N)
        bias, flags = coeffs[2:4].reshape(-1), WF_BNP
    if stats is not None:
        assert stats.dtype == torch.float64 and stats.is_contiguous() and stats.shape[-1] == N
    if variant >= 2:   # the small-wave-tile F(2x2) kernels (csrc/kernels/winograd4.hip): small grids
        _lib.call("rk_wino2s_conv_grp", _p(x), _p(u), _p(out), _p(bias), _p(stats), _slots_flags(stats), _p(gate),
                  Nb, H, W, C, N, flags, int(variant) - 2, 1, 0, 0, 0, 0, _s())
        return out
    _lib.call("rk_wino_conv", _p(x), _p(u), _p(out), _p(bias), _p(stats), _slots_flags(stats), _p(gate),
              Nb, H, W, C, N, flags, int(variant), _s())
    return out


# ----------------------------------------------------------------- Winograd F(4x4, 3x3) forward
# autotune candidates that run rk_wino4_conv: 8-wave 64 tiles x 32 channels (variant 0) / 4-wave 32 x 32
# (variant 1) / 4-wave 32 x 32 over two LDS stages, software-pipelined (variant 2)
WINO4_CFGS = ((-5, 0, 1), (-6, 0, 1))
_WINO4_VARIANT = {-5: 0, -6: 1, -11: 2}


def _wino4_variant(cfg):
    return _WINO4_VARIANT[cfg[0]]
WINO4 = os.environ.get('RAFIKI_WINOGRAD4', '1') != '0'


def wino4_ok(H: int, W: int, C: int) -> bool:
    """Shapes the fused F(4x4,3x3) kernel takes: stride-1 3x3, maps in multiples of 4, C % 8 == 0."""
    return WINO and WINO4 and H % 4 == 0 and W % 4 == 0 and C % 8 == 0 and C > 0


# normalise-on-load (the non-pooled BN + ReLU blocks of the fp32 engine): RAFIKI_BN_ON_LOAD=0 materialises
# every BN output instead
BN_ON_LOAD = os.environ.get('RAFIKI_BN_ON_LOAD', '1') != '0'


def bn_on_load_ok(Nb: int, H: int, W: int, Cin: int, Cout: int) -> bool:
    """Whether a 3x3 conv of Cin -> Cout channels on [Nb, H, W] can take its input as the previous conv's
    pre-BN output (conv_fwd(pro=...) with blocked F(4x4) weights, conv_wgrad(xpro=...))."""
    # Cin <= 512: the fused forward stages the 2 x Cin coefficients in 4 KiB of LDS (W4_PRO_MAXC)
    return (BN_ON_LOAD and wino4_ok(H, W, Cin) and Cin % 4 == 0 and Cin <= 512
            and bool(_wino4_wgrad_cands(Nb, H, W, Cout, Cin) or _wino4_pt_cands(Nb, H, W, Cout, Cin)))


def wino4_u(w: torch.Tensor) -> torch.Tensor:
    """Forward F(4x4) weights [36][Cout][Cin] of one conv weight [Cout, 3, 3, Cin] (fresh buffer)."""
    Cout = w.shape[0]
    Cin = w.numel() // (9 * Cout)
    u = torch.empty((36, Cout, Cin), device=w.device, dtype=torch.float32)
    _lib.call("rk_wino4_weights", _p(w), _p(u), None, Cout, Cin, _s())
    return u


def wino4_ut(w: torch.Tensor) -> torch.Tensor:
    """Data-gradient F(4x4) weights [36][Cin][Cout] (flipped, transposed filters) of w [Cout, 3, 3, Cin]."""
    Cout = w.shape[0]
    Cin = w.numel() // (9 * Cout)
    ut = torch.empty((36, Cin, Cout), device=w.device, dtype=torch.float32)
    _lib.call("rk_wino4_weights", _p(w), None, _p(ut), Cout, Cin, _s())
    return ut


# blocked-weight variants of the fused F(4x4) kernel (weights as the kernel's LDS stage image, one contiguous
# 36-KiB block per 32 output channels x 8 input channels: rk_wino4b_weights / WinoWeights 'u4b' / 'ut4b'):
# variant 3 = variant 0's 8-wave tile, 4 = variant 1's 4-wave tile, 5 = warp-specialised (4 compute + 4 loader
# waves over two LDS stages)
WINO4B_CFGS = ((-17, 0, 1), (-18, 0, 1), (-19, 0, 1))
_WINO4B_VARIANT = {-17: 3, -18: 4, -19: 5}


def wino4b_numel(N: int, C: int) -> int:
    """Floats of a blocked F(4x4) set with N output rows (padded to 32) and C input columns."""
    return 36 * cdiv(N, 32) * 32 * C


def wino4b_u(w: torch.Tensor, dgrad: bool = False) -> torch.Tensor:
    """Blocked F(4x4) set (forward, or the data-gradient one) of one conv weight [Cout, 3, 3, Cin]."""
    Cout = w.shape[0]
    Cin = w.numel() // (9 * Cout)
    n = wino4b_numel(Cin, Cout) if dgrad else wino4b_numel(Cout, Cin)
    ub = torch.zeros(n, device=w.device, dtype=torch.float32)
    _lib.call("rk_wino4b_weights", _p(w), None if dgrad else _p(ub), _p(ub) if dgrad else None, Cout, Cin, _s())
    return ub


def wino4_conv(x: torch.Tensor, u: torch.Tensor, *, out=None, bias=None, stats=None, relu=False, bnb=None, bnp=None,
               variant=0, n_out=None, pro=None):
    """y = conv3x3(x, w) (stride 1, pad 1) by F(4x4,3x3) from u = wino4_u(w); options as wino_conv.
    Variants 3 / 4 take the blocked set (wino4b_u / WinoWeights 'u4b'), flat, with ``n_out`` channels.
    ``pro``: normalise-on-load — x is the pre-BN output of the previous conv and pro its BN coeffs [4][C]
    (bn_finalize): the kernel loads relu(x * scale + shift) (blocked variants 3-5, no bias / activation)."""
    _check(x, 'wino4_conv x')
    Nb, H, W, C = x.shape
    if variant >= 3:
        N = int(n_out)
        assert u.dim() == 1 and u.numel() == wino4b_numel(N, C) and u.is_contiguous(), (u.shape, N, C)
    else:
        N = u.shape[1]
        assert u.shape == (36, N, C) and u.is_contiguous(), (u.shape, x.shape)
    if out is None:
        out = torch.empty((Nb, H, W, N), device=x.device, dtype=torch.float32)
    assert out.shape == (Nb, H, W, N) and out.is_contiguous()
    flags, gate = 0, None
    if bias is not None:
        flags |= WF_BIAS
    if relu:
        flags |= WF_RELU
    if stats is not None:
        flags |= WF_STATS
    if bnb is not None:
        gate, coeffs, stats = bnb
        assert gate.shape == out.shape
        bias, flags = coeffs[2:4].reshape(-1), WF_BNB
    elif bnp is not None:
        gate, coeffs, stats = bnp
        assert gate.shape == (Nb, 2 * H, 2 * W, N)
        bias, flags = coeffs[2:4].reshape(-1), WF_BNP
    if stats is not None:
        assert stats.dtype == torch.float64 and stats.is_contiguous() and stats.shape[-1] == N
    if pro is not None:
        assert variant >= 3 and flags in (0, WF_STATS) and pro.shape == (4, C) and pro.is_contiguous()
        _lib.call("rk_wino4_conv_pro", _p(x), _p(u), _p(out), None, _p(stats), _slots_flags(stats), None,
                  Nb, H, W, C, N, flags, int(variant), _p(pro[2]), _s())
        return out
    _lib.call("rk_wino4_conv", _p(x), _p(u), _p(out), _p(bias), _p(stats), _slots_flags(stats), _p(gate),
              Nb, H, W, C, N, flags, int(variant), _s())
    return out


WINO4_PT = -14   # pre-transformed F(4x4) conv: cfg = (-14, sgemm tile, sgemm nst)


# largest map the pre-transformed paths are offered on: 8 with the f32 GEMM (they lost on 16x16 maps,
# profiles/wgrad4_variants_r3.jsonl); with the X6 GEMM loop their batched GEMM is 1.1-1.3x faster, so the
# tuner also weighs them on 16x16 and 32x32 maps
PT_MAX_HW = int(os.environ.get('RAFIKI_PT_MAX_HW', '32' if USE_X6 else '8'))


def wino4_pt_ok(H, W, C, N):
    """Deep maps (<= 8x8), where the fused kernels re-transform each input window once per output-channel
    block: there the transform-once + grouped-GEMM path is a tuner candidate."""
    return (WINO and WINO4 and H % 4 == 0 and W % 4 == 0 and H <= PT_MAX_HW and W <= PT_MAX_HW and C % 4 == 0
            and C >= 32
            and N >= 32)


WINO4_PT_CFGS = tuple((WINO4_PT, t + x, n) for x in ((0, X6) if USE_X6 else (0,)) for t in (0, 1, 2, 3)
                      for n in ((2, 3) if t in _NST3 else (2,))) + \
    (tuple((WINO4_PT, t + X6, 2) for t in _FEW_WAVE) if USE_X6 else ())


def wino4_conv_pt(x: torch.Tensor, u: torch.Tensor, *, out=None, bias=None, stats=None, relu=False, bnb=None,
                  bnp=None, tile=0, nst=2, splits=1, lrelu=None, pro=None):
    """wino4_conv through position-major buffers: V = B^T x B [36][T][C] (one launch), Y'[q] = V[q] u[q]^T
    as one 36-group sgemm, then A^T Y' A with the same epilogues (bias / ReLU / BN statistics / BNB / BNP;
    ``lrelu`` = slope: bias + leaky ReLU, the PG-GAN discriminator's conv epilogue).
    With bf16 X6 planes u [36][3][N][C] (WinoWeights 'u4p' / 'ut4p') the input transform writes V as planes
    too and the GEMM is the pre-split X6 one (x6p_gemm; ``tile`` / ``nst`` are its configs)."""
    _check(x, 'wino4_conv_pt x')
    Nb, H, W, C = x.shape
    planes = u.dtype == torch.bfloat16   # u4p / ut4p X6 planes [36][3][N][C]
    N = u.shape[-2]
    assert u.shape == ((36, 3, N, C) if planes else (36, N, C)) and u.is_contiguous() and H % 4 == 0 and W % 4 == 0, \
        (u.shape, x.shape)
    if out is None:
        out = torch.empty((Nb, H, W, N), device=x.device, dtype=torch.float32)
    assert out.shape == (Nb, H, W, N) and out.is_contiguous()
    flags, gate = 0, None
    if bias is not None:
        flags |= WF_BIAS
    if relu:
        flags |= WF_RELU
    if lrelu is not None:
        assert not relu and stats is None and bnb is None and bnp is None
        flags |= WF_LRELU
    if stats is not None:
        flags |= WF_STATS
    if bnb is not None:
        gate, coeffs, stats = bnb
        assert gate.shape == out.shape
        bias, flags = coeffs[2:4].reshape(-1).contiguous(), WF_BNB
    elif bnp is not None:
        gate, coeffs, stats = bnp
        assert gate.shape == (Nb, 2 * H, 2 * W, N)
        bias, flags = coeffs[2:4].reshape(-1).contiguous(), WF_BNP
    if stats is not None:
        assert stats.dtype == torch.float64 and stats.is_contiguous() and stats.shape[-1] == N
    T = Nb * (H // 4) * (W // 4)
    if pro is not None:   # normalise-on-load in the input transform (pro = the producer's BN coeffs [4][C])
        assert pro.shape == (4, C) and pro.is_contiguous()
    if planes:   # pre-split X6: V planes [36][3][T][C] once, then the plane GEMM (no split in the K loop)
        splits = x6p_splits(C, splits)
        # Y' tile-major [T][36][N]: the output transform reads each tile's 36 positions as one run
        yt = torch.empty((splits, T, 36, N), device=x.device, dtype=torch.float32)
        v = torch.empty((36, 3, T, C), device=x.device, dtype=torch.bfloat16)
        if pro is None:
            _lib.call("rk_x6p_w4_input", _p(x), _p(v), Nb, H, W, C, _s())
        else:
            _lib.call("rk_x6p_w4_input_pro", _p(x), _p(v), Nb, H, W, C, _p(pro[2]), _s())
        x6p_gemm(v, u, yt, T, N, C, groups=36, tile=tile, nst=nst, splits=splits, row_major_groups=True)
    else:
        splits = 1
        yt = torch.empty((36, T, N), device=x.device, dtype=torch.float32)
        v = torch.empty((36, T, C), device=x.device, dtype=torch.float32)
        if pro is None:
            _lib.call("rk_wino4_pt_input", _p(x), _p(v), Nb, H, W, C, _s())
        else:
            _lib.call("rk_wino4_pt_input_pro", _p(x), _p(v), Nb, H, W, C, _p(pro[2]), _s())
        sgemm_grp(KIND_DENSE, v, u, yt, T, N, C, C, C, N, 36, T * C, N * C, T * N, tile=tile, nst=nst)
    _lib.call("rk_wino4_pt_conv_out", _p(yt), _p(out), _p(bias), _p(stats), _slots_flags(stats), _p(gate),
              Nb, H, W, N, flags, splits, 36 * T * N, int(planes), float(0.0 if lrelu is None else lrelu), _s())
    return out


def wino4_conv_grp(x, u, *, out=None, bias=None, relu=False, variant=0, pool=False):
    """k F(4x4) convs in one grid: x [G, Nb, H, W, C] (or shared [Nb, H, W, C]), u [G, 36, N, C].
    ``pool`` (with bias + relu): the 2x2 max-pool from the epilogue, out [G, Nb, H/2, W/2, N]."""
    G, _, N, C = u.shape
    shared = x.dim() == 4
    Nb, H, W, Cx = x.shape[-4:]
    assert Cx == C and (shared or x.shape[0] == G) and u.is_contiguous() and x.is_contiguous()
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    if out is None:
        out = torch.empty((G, Nb, Ho, Wo, N), device=x.device, dtype=torch.float32)
    assert out.shape == (G, Nb, Ho, Wo, N) and out.is_contiguous()
    M = Nb * H * W
    flags = (WF_BIAS if bias is not None else 0) | (WF_RELU if relu else 0)
    if pool:
        assert bias is not None and relu
        flags |= WF_POOL
    _lib.call("rk_wino4_conv_grp", _p(x), _p(u), _p(out), _p(bias), None, 0, None, Nb, H, W, C, N, flags,
              int(variant), G, 0 if shared else M * C, 36 * N * C, Nb * Ho * Wo * N, N if bias is not None else 0,
              _s())
    return out


WINO4_WGRAD = -7  # autotune tile id of the F(4x4) weight gradient (cfg = (-7, 0, splits))


def _wino4_wgrad_cands(Nb, H, W, Cout, Cin):
    """Split-K choices of rk_wino4_wgrad_v (variant 0: 32 co x 32 ci blocks, 1: 64 co x 32 ci, 2: 32 x 32
    software-pipelined over two LDS stages): 128..4096
    blocks, >= 4 chunks of 8 tiles per block, slabs <= 256 MiB.  cfg = (WINO4_WGRAD, variant, splits)."""
    if not (WINO and WINO4 and H % 4 == 0 and W % 4 == 0 and Cin >= 8 and Cout >= 16):
        return []
    nt = Nb * (H // 4) * (W // 4)
    if nt >= (1 << 22) or 4 * Nb * H * W * max(Cin, Cout) >= 0x7fffffff:
        return []
    out = []
    for v, bco in ((0, 32), (1, 64)):   # 2 (software-pipelined) measured 1.2-1.3x slower, wino4_variants_r5
        if v == 1 and Cout < 64:
            continue
        base = cdiv(Cout, bco) * cdiv(Cin, 32)
        for s in (1, 2, 4, 8, 16, 32, 64, 128, 256):
            tps = cdiv(cdiv(nt, s), 8) * 8
            s_eff = cdiv(nt, tps)
            if tps < 32 or base * s_eff > 4096 or (s_eff > 1 and s_eff * 9 * Cout * Cin * 4 > (256 << 20)):
                continue
            if base * s_eff < 128 and s != 1:
                continue
            c = (WINO4_WGRAD, v, s_eff)
            if c not in out:
                out.append(c)
    return out


def wino4_wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, *, splits=1, accumulate=False, variant=0,
                xpro=None):
    """out [Cout][9*Cin] (+)= weight gradient of a 3x3 stride-1 conv by F(4x4,3x3); splits > 1: per-split
    slabs summed by reduce_slabs.  ``xpro``: x is pre-BN, normalised + ReLU'd on load (variants 0 / 1)."""
    _check(dy, 'wino4_wgrad dy')
    _check(x, 'wino4_wgrad x')
    Nb, H, W, Cout = dy.shape
    Cin = x.shape[-1]
    assert x.shape[:3] == dy.shape[:3] and out.numel() == Cout * 9 * Cin and out.is_contiguous()
    if xpro is not None:
        assert xpro.shape == (4, Cin) and xpro.is_contiguous() and variant in (0, 1)
        fn, tail = "rk_wino4_wgrad_pro", (_p(xpro[2]), _s())
    else:
        fn, tail = "rk_wino4_wgrad_v", (_s(),)
    if splits == 1:
        _lib.call(fn, _p(dy), _p(x), _p(out), Nb, H, W, Cout, Cin, 1, int(bool(accumulate)), int(variant), *tail)
        return out
    slab = torch.empty((splits, Cout, 9 * Cin), device=dy.device, dtype=torch.float32)
    _lib.call(fn, _p(dy), _p(x), _p(slab), Nb, H, W, Cout, Cin, int(splits), 0, int(variant), *tail)
    reduce_slabs(slab, out.view(Cout, 9 * Cin), accumulate=accumulate)
    return out


WINO4_WGRAD_PT = -13  # pre-transformed F(4x4) weight gradient: cfg = (-13, sgemm tile, sgemm nst)


def _wino4_pt_cands(Nb, H, W, Cout, Cin):
    """The pre-transformed F(4x4) weight gradient (transform once, 36 GEMMs as one split-K sgemm) on
    maps of <= 8x8, where the fused kernels' redundant per-block transforms dominate (VGG-small batch
    256: 8x8x256x256 84.8 vs 101.7 us, 4x4x512x512 76.4 vs 96.3; it loses on 16x16 maps,
    profiles/wgrad4_variants_r3.jsonl)."""
    if not (WINO and WINO4 and H % 4 == 0 and W % 4 == 0 and H <= PT_MAX_HW and W <= PT_MAX_HW and Cin % 4 == 0
            and Cout % 4 == 0 and Cin >= 32 and Cout >= 32):
        return []
    T = Nb * (H // 4) * (W // 4)
    if T % 32 or 36 * T * max(Cin, Cout) * 4 >= (1 << 31) or 36 * Cout * Cin * 4 > (512 << 20):
        return []
    return [(WINO4_WGRAD_PT, t + x, n) for x in ((0, X6) if USE_X6 else (0,)) for t in (0, 1, 2, 3)
            for n in ((2, 3) if t in _NST3 else (2,))] + \
        ([(WINO4_WGRAD_PT, t + X6, 2) for t in _FEW_WAVE] if USE_X6 else [])


def wino4_wgrad_pt(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, *, accumulate=False, tile=0, nst=2,
                   planes=False, splits=1, xpro=None):
    """out [Cout][9*Cin] (+)= the F(4x4,3x3) weight gradient through position-major transformed buffers:
    M [36][T][Cout], V [36][T][Cin] (one transform launch each), dU[q] = M[q]^T V[q] as ONE sgemm with
    36 K-splits (slab q = dU[q]), then dW = G^T dU G.  ``planes``: the operands as X6 planes transposed to
    K-inner ([36][3][C][T]) and the 36 GEMMs as one grouped pre-split X6 launch (x6p_gemm configs)."""
    _check(dy, 'wino4_wgrad_pt dy')
    _check(x, 'wino4_wgrad_pt x')
    Nb, H, W, Cout = dy.shape
    Cin = x.shape[-1]
    T = Nb * (H // 4) * (W // 4)
    assert H % 4 == 0 and W % 4 == 0 and T % 32 == 0 and x.shape[:3] == dy.shape[:3], (dy.shape, x.shape)
    assert out.numel() == Cout * 9 * Cin and out.is_contiguous()
    assert xpro is None or (not planes and xpro.shape == (4, Cin) and xpro.is_contiguous())
    if planes:   # pre-split X6: M^T / V^T planes [36][3][C][T] (K = tiles inner), 36-group plane GEMM
        splits = x6p_splits(T, splits)
        du = torch.empty((splits, 36, Cout, Cin), device=dy.device, dtype=torch.float32)
        m = torch.empty((36, 3, Cout, T), device=dy.device, dtype=torch.bfloat16)
        v = torch.empty((36, 3, Cin, T), device=dy.device, dtype=torch.bfloat16)
        _lib.call("rk_x6p_w4_wgrad_transform", _p(dy), _p(x), _p(m), _p(v), Nb, H, W, Cout, Cin, _s())
        x6p_gemm(m, v, du, Cout, Cin, T, groups=36, tile=tile, nst=nst, splits=splits)
    else:
        splits = 1
        du = torch.empty((36, Cout, Cin), device=dy.device, dtype=torch.float32)
        m = torch.empty((36 * T, Cout), device=dy.device, dtype=torch.float32)
        v = torch.empty((36 * T, Cin), device=dy.device, dtype=torch.float32)
        if xpro is None:
            _lib.call("rk_wino4_pt_transform", _p(dy), _p(x), _p(m), _p(v), Nb, H, W, Cout, Cin, _s())
        else:
            _lib.call("rk_wino4_pt_transform_pro", _p(dy), _p(x), _p(m), _p(v), Nb, H, W, Cout, Cin, _p(xpro[2]),
                      _s())
        sgemm(KIND_DENSE_DW, m, v, du, Cout, Cin, 36 * T, Cout, Cin, Cin, tile=tile, nst=nst, splits=36,
              slab_stride=Cout * Cin)
    _lib.call("rk_wino4_pt_output", _p(du), _p(out), Cout, Cin, int(bool(accumulate)), splits, 36 * Cout * Cin, _s())
    return out


# ---------------------------------------------------------------- pre-split X6 GEMMs (x6p.hip)
# The X6 products with the operands split into bf16 planes ONCE by their producers (the Winograd
# transforms) instead of after every LDS read inside the K loop: the pre-transformed F(4x4) paths on
# planes are autotune candidates next to their fp32-operand sgemm forms.  RAFIKI_X6P=0 turns them off.
USE_X6P = USE_X6 and os.environ.get('RAFIKI_X6P', '1') != '0'
# tiles 9-12: warp-specialised (2x2 compute waves + 4 loader waves that alone issue the LDS-DMA pieces)
XP_TILES = ((128, 128), (128, 64), (64, 128), (64, 64), (64, 64), (128, 64), (64, 128), (256, 128), (128, 256),
            (128, 128), (128, 64), (64, 128), (64, 64))
XP_NST3 = (0, 1, 2, 3, 4, 5, 6, 9, 10, 11, 12)   # tiles 7-8 (8 waves, 72 KiB per stage) ring 2 stages only
# (tile, nst, splits) of the x6p GEMM: every tile x ring depth unsplit; the big tiles also with 2 / 4 K-splits
# (the 4x4-map GEMMs have T = 256 rows: 288 blocks of 128x128 for 256 CUs; the slabs are summed by the
# output transforms that read Y' / dU anyway)
_XP_CFGS = tuple((t, n, 1) for t in range(len(XP_TILES)) for n in ((2, 3) if t in XP_NST3 else (2,))) + \
    tuple((t, 2, s) for t in (0, 1, 2, 7, 8) for s in (2, 4)) + tuple((t, 3, s) for t in (9, 10, 11) for s in (2, 4))
WINO4_PTX = -15         # conv / data gradient: cfg = (-15, x6p code, splits), code = tile * 4 + nst
WINO4_WGRAD_PTX = -16   # weight gradient: likewise
WINO4_PTX_CFGS = tuple((WINO4_PTX, 4 * t + n, s) for t, n, s in _XP_CFGS) if USE_X6P else ()


def x6p_split(src: torch.Tensor, out=None) -> torch.Tensor:
    """bf16 X6 planes [3][rows][cols] (hi, mid, lo; x = hi + mid + lo) of an fp32 [rows][cols] matrix."""
    _check(src, 'x6p_split src')
    rows, cols = src.shape
    if out is None:
        out = torch.empty((3, rows, cols), dtype=torch.bfloat16, device=src.device)
    _lib.call("rk_x6p_split", _p(src), _p(out), rows, cols, cols, cols, rows * cols, _s())
    return out


def x6p_split_t(src: torch.Tensor, ldd: Optional[int] = None, out=None) -> torch.Tensor:
    """bf16 X6 planes [3][cols][ldd] of the TRANSPOSE of an fp32 [rows][cols] matrix (row stride any), the
    plane columns rows .. ldd-1 zero (ldd: rows rounded up to 32, the x6p GEMM's K granularity)."""
    rows, cols = src.shape
    assert src.dtype == torch.float32 and src.stride(1) == 1, (src.dtype, src.stride())
    ldd = ldd or cdiv(rows, 32) * 32
    if out is None:
        out = torch.empty((3, cols, ldd), dtype=torch.bfloat16, device=src.device)
    _lib.call("rk_x6p_split_t", _p(src), _p(out), rows, cols, src.stride(0), ldd, cols * ldd, _s())
    return out


def x6p_gemm(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, M: int, N: int, K: int, *, groups: int = 1,
             tile: int = 0, nst: int = 2, accumulate: bool = False, splits: int = 1,
             row_major_groups: bool = False) -> torch.Tensor:
    """out[g] (+)= A[g] . B[g]^T for g < groups: A bf16 planes [G][3][M][K], B [G][3][N][K] (contiguous),
    out fp32 [G][M][N] (``row_major_groups``: [M][G][N]); K % 32 == 0.  splits > 1: out is [splits][...] raw
    split-K partial sums."""
    assert A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16 and A.is_contiguous() and B.is_contiguous()
    assert A.numel() == groups * 3 * M * K and B.numel() == groups * 3 * N * K
    assert out.numel() == splits * groups * M * N and not (accumulate and splits > 1)
    ldc, gsc = (groups * N, N) if row_major_groups else (N, M * N)
    _lib.call("rk_x6p_gemm", int(tile), int(nst), _p(A), _p(B), _p(out), M, N, K, K, K, ldc, M * K, N * K, 3 * M * K,
              3 * N * K, gsc, int(groups), int(bool(accumulate)), int(splits), groups * M * N, _nbytes(A),
              _nbytes(B), _s())
    return out


def x6p_splits(K: int, s: int) -> int:
    """The effective split count of ``s`` requested splits over K (every split gets >= one 32-deep K-tile)."""
    nk = K // 32
    per = cdiv(nk, max(1, s))
    return cdiv(nk, per)


def wino4_u4p(w: torch.Tensor, dgrad: bool = False) -> torch.Tensor:
    """X6 planes of the F(4x4) weights of one conv weight [Cout, 3, 3, Cin] (fresh buffer): forward set
    [36][3][Cout][Cin] (WinoWeights 'u4p'), ``dgrad``: the data-gradient set [36][3][Cin][Cout] ('ut4p')."""
    Cout = w.shape[0]
    Cin = w.numel() // (9 * Cout)
    out = torch.empty((36, 3, Cin, Cout) if dgrad else (36, 3, Cout, Cin), device=w.device, dtype=torch.bfloat16)
    _lib.call("rk_x6p_w4_weights", _p(w), None if dgrad else _p(out), _p(out) if dgrad else None, Cout, Cin, _s())
    return out


def wino4_ptx_ok(H, W, C, N):
    """Shapes the plane path of the pre-transformed F(4x4) conv takes (K = C channels, % 32)."""
    return USE_X6P and wino4_pt_ok(H, W, C, N) and C % 32 == 0


def _wino4_ptx_wgrad_cands(Nb, H, W, Cout, Cin):
    """The plane path of the pre-transformed F(4x4) weight gradient: K = T tiles (% 32)."""
    if not (USE_X6P and _wino4_pt_cands(Nb, H, W, Cout, Cin)):
        return []
    T = Nb * (H // 4) * (W // 4)
    if T % 32 or 108 * T * max(Cin, Cout) >= (1 << 31):
        return []
    return [(WINO4_WGRAD_PTX, 4 * t + n, x6p_splits(T, s)) for t, n, s in _XP_CFGS]


WINO_WGRAD = -3   # autotune tile id of the Winograd weight gradient (cfg = (-3, 0, splits))


def _wino_wgrad_cands(Nb, H, W, Cout, Cin):
    """Split-K choices of rk_wino_wgrad that fill the chip: 128..4096 blocks, >= 8 chunks of 8 tiles per
    block, slabs <= 256 MiB."""
    if not (WINO and H % 2 == 0 and W % 2 == 0 and Cin >= 8 and Cout >= 16):
        return []
    nt = Nb * (H // 2) * (W // 2)
    if nt >= (1 << 22) or 4 * Nb * H * W * max(Cin, Cout) >= 0x7fffffff:
        return []
    base = cdiv(Cout, 64) * cdiv(Cin, 64)
    out = []
    for s in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512):
        tps = cdiv(cdiv(nt, s), 8) * 8
        s_eff = cdiv(nt, tps)
        if tps < 64 or base * s_eff > 4096 or (s_eff > 1 and s_eff * 9 * Cout * Cin * 4 > (256 << 20)):
            continue
        if base * s_eff < 128 and s != 1:
            continue
        c = (WINO_WGRAD, 0, s_eff)
        if c not in out:
            out.append(c)
    return out


def wino_wgrad(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, *, splits=1, accumulate=False):
    """out [Cout][9*Cin] (+)= weight gradient of a 3x3 stride-1 conv by F(2x2,3x3); splits > 1: per-split
    slabs summed by reduce_slabs."""
    _check(dy, 'wino_wgrad dy')
    _check(x, 'wino_wgrad x')
    Nb, H, W, Cout = dy.shape
    Cin = x.shape[-1]
    assert x.shape[:3] == dy.shape[:3] and out.numel() == Cout * 9 * Cin and out.is_contiguous()
    if splits == 1:
        _lib.call("rk_wino_wgrad", _p(dy), _p(x), _p(out), Nb, H, W, Cout, Cin, 1, int(bool(accumulate)), _s())
        return out
    slab = torch.empty((splits, Cout, 9 * Cin), device=dy.device, dtype=torch.float32)
    _lib.call("rk_wino_wgrad", _p(dy), _p(x), _p(slab), Nb, H, W, Cout, Cin, int(splits), 0, _s())
    reduce_slabs(slab, out.view(Cout, 9 * Cin), accumulate=accumulate)
    return out


def wino_conv_grp(x, u, *, out=None, bias=None, relu=False, variant=0, pool=False):
    """k Winograd convs in one grid: x [G, Nb, H, W, C] (or [Nb, H, W, C] shared), u [G, 16, N, C],
    bias [G, N] -> out [G, Nb, H, W, N].  ``pool`` (with bias + relu, variants >= 2): the 2x2 max-pool of
    the output from the epilogue, out [G, Nb, H/2, W/2, N]."""
    G, _, N, C = u.shape
    shared = x.dim() == 4
    Nb, H, W, Cx = x.shape[-4:]
    assert Cx == C and (shared or x.shape[0] == G) and u.is_contiguous() and x.is_contiguous()
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    if out is None:
        out = torch.empty((G, Nb, Ho, Wo, N), device=x.device, dtype=torch.float32)
    assert out.shape == (G, Nb, Ho, Wo, N) and out.is_contiguous()
    M = Nb * H * W
    flags = (WF_BIAS if bias is not None else 0) | (WF_RELU if relu else 0)
    if pool:
        assert bias is not None and relu and variant >= 2 and H % 2 == 0 and W % 2 == 0
        flags |= WF_POOL
    name, v = ("rk_wino2s_conv_grp", int(variant) - 2) if variant >= 2 else ("rk_wino_conv_grp", int(variant))
    _lib.call(name, _p(x), _p(u), _p(out), _p(bias), None, 0, None, Nb, H, W, C, N, flags,
              v, G, 0 if shared else M * C, 16 * N * C, Nb * Ho * Wo * N, N if bias is not None else 0, _s())
    return out


class WinoWeights:
    """Winograd-domain weights of several 3x3 convs whose fp32 weights live in one arena: per layer the
    F(2x2) sets u2 [16][Cout][Cin] (forward) and ut2 [16][Cin][Cout] (data gradient, ``dgrad=True``)
    and, for maps in multiples of 4 (``f4``), the F(4x4) sets u4 [36][Cout][Cin] / ut4 [36][Cin][Cout].

    ``refresh()`` transforms every LIVE set in at most two launches per weight update.  The convs take
    the sets through ``lazy(kind, l)`` callables, which the autotuned conv calls only when a Winograd
    candidate of that kind runs: a set that is not fresh this step is transformed on demand (always
    correct), and ``end_step()`` narrows the live sets to the ones the tuned convs actually used, so a
    step pays only for the transforms it needs (outside graph capture; the captured step replays the
    narrowed refresh)."""

    KINDS = ('u2', 'ut2', 'u4', 'ut4', 'u4p', 'ut4p', 'u4b', 'ut4b')

    def __init__(self, arena: torch.Tensor, weights, dgrad=True, f4=None, hw=None):
        """hw[l]: the layer's map size (F(4x4) sets only where it is a multiple of 4; None: every layer)."""
        self.arena = arena
        self.weights = list(weights)
        self.dgrad = dgrad
        f4 = WINO4 if f4 is None else f4
        self._layers, self._sets, off = [], {}, 0
        for l, w in enumerate(self.weights):
            Cout = w.shape[0]
            Cin = w.numel() // (9 * Cout)
            so = (w.data_ptr() - arena.data_ptr()) // 4
            assert 0 <= so and so + w.numel() <= arena.numel() and w.is_contiguous()
            self._layers.append((so, Cout, Cin))
            kinds = ['u2'] + (['ut2'] if dgrad else [])
            if f4 and (hw is None or hw[l] % 4 == 0):
                kinds += ['u4'] + (['ut4'] if dgrad else [])
                # X6 planes (bf16 [36][3][..], 54 floats per weight) where the pre-split PT path takes the shape
                if hw is None or wino4_ptx_ok(hw[l], hw[l], Cin, Cout):
                    kinds.append('u4p')
                if dgrad and (hw is None or wino4_ptx_ok(hw[l], hw[l], Cout, Cin)):
                    kinds.append('ut4p')
                # blocked sets of the UB fused kernels (input columns in multiples of 8)
                if Cin % 8 == 0:
                    kinds.append('u4b')
                if dgrad and Cout % 8 == 0:
                    kinds.append('ut4b')
            for k in kinds:
                if k == 'u4b':
                    n = wino4b_numel(Cout, Cin)
                elif k == 'ut4b':
                    n = wino4b_numel(Cin, Cout)
                else:
                    n = 54 * Cout * Cin if k.endswith('p') else (16 if k.endswith('2') else 36) * Cout * Cin
                self._sets[(k, l)] = (off, n)
                off += n
        dev = arena.device
        self.buf = torch.zeros(max(off, 1), dtype=torch.float32, device=dev)
        self._tables = {}
        self.live = frozenset(self._sets)
        self._fresh = set()
        self._used = set()
        self._prepare(self.live)

    # ---- transform tables: one (desc, meta) pair per kernel family for a set of live sets
    def _prepare(self, live):
        if live in self._tables:
            return self._tables[live]
        out = []
        for fam, (ka, kb) in (('2', ('u2', 'ut2')), ('4', ('u4', 'ut4')), ('p', ('u4p', 'ut4p')), ('b', ('u4b', 'ut4b'))):
            scale = 2 if fam == 'p' else 1   # plane sets: offsets in bf16 elements
            meta, desc, idx = [], [], {}
            for l, (so, Cout, Cin) in enumerate(self._layers):
                u = self._sets.get((ka, l)) if (ka, l) in live else None
                ut = self._sets.get((kb, l)) if (kb, l) in live else None
                if u is None and ut is None:
                    continue
                idx[l] = len(meta)
                meta.append([so, scale * u[0] if u else -1, scale * ut[0] if ut else -1, Cout, Cin])
                for co0 in range(0, Cout, 32):
                    for ci0 in range(0, Cin, 32):
                        desc.append([idx[l], co0, ci0, 0])
            if desc:
                dev = self.arena.device
                out.append((fam, torch.tensor(desc, dtype=torch.int32, device=dev).reshape(-1),
                            torch.tensor(meta, dtype=torch.int64, device=dev).reshape(-1), len(desc)))
        self._tables[live] = out
        # every family in one table for the single-launch refresh (rk_wino_weights_all): meta rows
        # concatenated, each block's desc row = (meta row, co0, ci0, family)
        fam_id = {'2': 0, '4': 1, 'p': 2, 'b': 3}
        adesc, ameta, base = [], [], 0
        for fam, desc, meta, nb in out:
            d = desc.view(-1, 4).cpu().clone()
            d[:, 0] += base
            d[:, 3] = fam_id[fam]
            adesc.append(d)
            ameta.append(meta.view(-1, 5).cpu())
            base += ameta[-1].shape[0]
        if adesc:
            dev = self.arena.device
            self._tables[('all', live)] = (torch.cat(adesc).to(dev).reshape(-1), torch.cat(ameta).to(dev).reshape(-1),
                                           sum(int(t.shape[0]) for t in adesc))
        return out

    def refresh(self):
        """Every live set of every family in ONE launch (rk_wino_weights_all)."""
        self._prepare(self.live)
        allt = self._tables.get(('all', self.live))
        if allt is not None:
            desc, meta, nb = allt
            _lib.call("rk_wino_weights_all", _p(self.arena), _p(self.buf), _p(desc), nb, _p(meta), _s())
        self._fresh = set(self.live)

    def end_step(self):
        """Narrow the live sets to the ones this step's convs used (no-op inside graph capture)."""
        used, self._used = frozenset(self._used), set()
        if not used or used == self.live:
            return
        try:
            capturing = torch.cuda.is_current_stream_capturing()
        except Exception:
            capturing = False
        if not capturing:
            self._prepare(used)
            self.live = used

    def _view(self, kind, l):
        off, n = self._sets[(kind, l)]
        _, Cout, Cin = self._layers[l]
        if kind in ('u4b', 'ut4b'):
            return self.buf[off:off + n]
        if kind.endswith('p'):
            flat = self.buf[off:off + n].view(torch.bfloat16)
            return flat.view((36, 3, Cout, Cin) if kind == 'u4p' else (36, 3, Cin, Cout))
        pos = 16 if kind.endswith('2') else 36
        shape = (pos, Cout, Cin) if kind.startswith('u') and not kind.startswith('ut') else (pos, Cin, Cout)
        return self.buf[off:off + n].view(shape)

    def _ensure(self, kind, l):
        if (kind, l) not in self._fresh:   # not refreshed this step: transform this layer's set now
            so, Cout, Cin = self._layers[l]
            w = self.arena[so:so + 9 * Cout * Cin]
            v = self._view(kind, l)
            name = "rk_wino_weights" if kind.endswith('2') else "rk_wino4_weights"
            if kind.endswith('p'):
                name = "rk_x6p_w4_weights"
            if kind.endswith('b'):
                name = "rk_wino4b_weights"
            if kind.startswith('ut'):
                _lib.call(name, _p(w), None, _p(v), Cout, Cin, _s())
            else:
                _lib.call(name, _p(w), _p(v), None, Cout, Cin, _s())
            self._fresh.add((kind, l))
        self._used.add((kind, l))
        return self._view(kind, l)

    def has(self, kind, l):
        return (kind, l) in self._sets

    def lazy(self, kind, l):
        """Callable returning the fresh set (or None when the layer has no such set)."""
        if (kind, l) not in self._sets:
            return None
        return lambda: self._ensure(kind, l)

    def u(self, l):
        return self._view('u2', l)

    def ut(self, l):
        assert self.dgrad
        return self._view('ut2', l)

    def u4(self, l):
        return self._view('u4', l) if ('u4', l) in self._sets else None

    def ut4(self, l):
        return self._view('ut4', l) if ('ut4', l) in self._sets else None

    def u4p(self, l):
        return self._view('u4p', l) if ('u4p', l) in self._sets else None


# ----------------------------------------------------------------------------------------- dense
# Pre-split X6 dense candidates (cfg = (XP_DENSE, x6p tile * 4 + nst, splits)): both operands split into bf16
# planes by one pass each (x6p_split / x6p_split_t, inside the timed candidate), then the x6p GEMM — its K
# loop is LDS reads + MFMAs only, where the sgemm X6 loop re-splits every fragment after its LDS read and runs
# VALU-bound (the PG-GAN dense layers: 512 x 8192 at mb 512, profiles/pg_gan_lod3_f32_kernels_r5.txt); the
# bias / activation / gate epilogue and the split-K combine ride in sreduce_epi / reduce_slabs
XP_DENSE = -21
XPD_MIN_MACS = 1 << 28   # GEMM size below which the split passes cannot pay (VGG / MLP heads, tiny layers)
XPD_CFGS = tuple((XP_DENSE, 4 * t + n, s) for t in (0, 1, 2, 3) for n in (2, 3) for s in (1, 2, 4)) + \
    tuple((XP_DENSE, 4 * t + 2, s) for t in (7, 8) for s in (1, 2, 4)) if USE_X6P else ()


def _xpd(cfg):
    return cfg[0] == XP_DENSE


def _xp_gemm_into(A, B, M, N, K, code, s, out=None, accumulate=False):
    """x6p GEMM of planes A [3][M][K] . B [3][N][K]^T: into ``out`` (s == 1) or a fresh [s][M][N] slab."""
    s = x6p_splits(K, s)
    if s == 1 and out is not None:
        x6p_gemm(A, B, out, M, N, K, tile=code // 4, nst=code % 4, accumulate=accumulate)
        return out, 1
    slab = torch.empty((s, M, N), device=A.device, dtype=torch.float32)
    x6p_gemm(A, B, slab, M, N, K, tile=code // 4, nst=code % 4, splits=s)
    return slab, s


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, *, act=ACT_NONE, slope=0.2, out=None, alpha=1.0):
    """out = act(alpha * x @ w.T + bias), fp32; small-M layers autotune split-K + a fused combine."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), device=x.device, dtype=torch.float32)
    flags = (F_BIAS if bias is not None else 0) | (F_RELU if act == ACT_RELU else F_LRELU if act == ACT_LRELU else 0)

    def run(cfg):
        tile, nst, s = cfg
        if _xpd(cfg):
            slab, _ = _xp_gemm_into(x6p_split(x), x6p_split(w), M, N, K, nst, s)
            sreduce_epi(slab, M, N, out, bias=bias, act=act, slope=slope, alpha=alpha)
            return
        if s == 1:
            sgemm(KIND_DENSE, x, w, out, M, N, K, x.stride(0), w.stride(0), out.stride(0), tile=tile, nst=nst,
                  bias=bias, flags=flags, slope=slope, alpha=alpha)
            return
        slab = torch.empty((s, M, N), device=x.device, dtype=torch.float32)
        sgemm(KIND_DENSE, x, w, slab, M, N, K, x.stride(0), w.stride(0), N, tile=tile, nst=nst, splits=s,
              slab_stride=M * N)
        sreduce_epi(slab, M, N, out, bias=bias, act=act, slope=slope, alpha=alpha)
    cands = _cands(M, N, splittable=N % 4 == 0 and out.stride(0) % 4 == 0, K=K)
    xp = K % 32 == 0 and x.is_contiguous() and w.is_contiguous() and M * N * K >= XPD_MIN_MACS
    if xp:
        cands = cands + list(XPD_CFGS)
    run(_pick(('sl', M, N, K, act, bias is not None, float(alpha)) + (('xp',) if xp else ()), cands, run))
    return out


def linear_dx(dy: torch.Tensor, w: torch.Tensor, *, gate=None, out=None):
    """dx[M][in] = dy[M][out] @ w[out][in], optionally gated (dx = 0 where gate <= 0)."""
    M, Nout = dy.shape
    Nin = w.shape[1]
    if out is None:
        out = torch.empty((M, Nin), device=dy.device, dtype=torch.float32)

    def run(cfg):
        tile, nst, s = cfg
        if _xpd(cfg):
            slab, _ = _xp_gemm_into(x6p_split(dy), x6p_split_t(w), M, Nin, Nout, nst, s)
            sreduce_epi(slab, M, Nin, out, gate=gate)
            return
        if s == 1:
            sgemm(KIND_DENSE_DX, dy, w, out, M, Nin, Nout, dy.stride(0), w.stride(0), out.stride(0), tile=tile,
                  nst=nst, gate=gate, flags=F_GATE if gate is not None else 0)
            return
        slab = torch.empty((s, M, Nin), device=dy.device, dtype=torch.float32)
        sgemm(KIND_DENSE_DX, dy, w, slab, M, Nin, Nout, dy.stride(0), w.stride(0), Nin, tile=tile, nst=nst,
              splits=s, slab_stride=M * Nin)
        sreduce_epi(slab, M, Nin, out, gate=gate)
    cands = _cands(M, Nin, splittable=Nin % 4 == 0, K=Nout)
    xp = Nout % 32 == 0 and dy.is_contiguous() and w.is_contiguous() and M * Nin * Nout >= XPD_MIN_MACS
    if xp:
        cands = cands + list(XPD_CFGS)
    run(_pick(('sx', M, Nin, Nout, gate is not None) + (('xp',) if xp else ()), cands, run))
    return out


def linear_dw(dy: torch.Tensor, x: torch.Tensor, *, out=None, accumulate=False):
    """dw[out][in] = dy[M][out]^T @ x[M][in] (fp32)."""
    M, Nout = dy.shape
    Nin = x.shape[1]
    if out is None:
        out = torch.empty((Nout, Nin), device=dy.device, dtype=torch.float32)

    def run(cfg):
        tile, nst, s = cfg
        if _xpd(cfg):
            Mp = cdiv(M, 32) * 32
            res, k = _xp_gemm_into(x6p_split_t(dy, Mp), x6p_split_t(x, Mp), Nout, Nin, Mp, nst, s,
                                   out=out if out.is_contiguous() else None, accumulate=accumulate)
            if k > 1 or res is not out:
                reduce_slabs(res, out, accumulate=accumulate)
            return
        if s == 1:
            sgemm(KIND_DENSE_DW, dy, x, out, Nout, Nin, M, dy.stride(0), x.stride(0), Nin, tile=tile, nst=nst,
                  flags=F_ACCUM if accumulate else 0)
            return
        slab = torch.empty((s, Nout, Nin), device=dy.device, dtype=torch.float32)
        sgemm(KIND_DENSE_DW, dy, x, slab, Nout, Nin, M, dy.stride(0), x.stride(0), Nin, tile=tile, nst=nst,
              splits=s, slab_stride=Nout * Nin)
        reduce_slabs(slab, out, accumulate=accumulate)
    cands = _cands(Nout, Nin, splittable=True, K=M)
    xp = Nout * Nin * M >= XPD_MIN_MACS
    if xp:
        cands = cands + list(XPD_CFGS)
    run(_pick(('sdw', M, Nout, Nin, bool(accumulate)) + (('xp',) if xp else ()), cands, run,
              protect=(out,) if accumulate else ()))
    return out


def sreduce_epi(slab, M, N, out, *, bias=None, act=ACT_NONE, slope=0.2, alpha=1.0, gate=None, bias_rows=0):
    """out = act(alpha * sum_s slab[s] + bias) (gated); bias_rows > 0: row block g uses bias[g]."""
    _lib.call("rk_sreduce_epi", _p(slab), slab.shape[0], int(M), int(N), _p(bias), int(act), float(slope),
              float(alpha), _p(gate), 0 if gate is None else gate.stride(0), _p(out), out.stride(0), int(bias_rows),
              _s())
    return out


def reduce_slabs(slab, out, *, accumulate=False, scale=1.0):
    from .functional import reduce_slabs as _rs
    return _rs(slab, out, accumulate=accumulate, scale=scale)


def lrelu_gate(gy: torch.Tensor, y: torch.Tensor, slope: float, out=None):
    """gy * (y > 0 ? 1 : slope) (fp32, contiguous, same shape)."""
    _check(gy, 'lrelu_gate gy')
    _check(y, 'lrelu_gate y')
    assert gy.shape == y.shape
    if out is None:
        out = torch.empty_like(gy)
    _lib.call("rk_lrelu_gate_f32", _p(gy), _p(y), _p(out), gy.numel(), float(slope), _s())
    return out


def lrelu_gate_colsum(gy: torch.Tensor, y: torch.Tensor, slope: float, acc=None):
    """(g, colsum(g)) with g = lrelu_gate(gy, y, slope) in one pass; gy / y [..., C] fp32.  ``acc`` (fp32
    [C]): the column sum is added into it instead (returns (g, acc))."""
    _check(gy, 'lrelu_gate_colsum gy')
    _check(y, 'lrelu_gate_colsum y')
    assert gy.shape == y.shape
    Cc = gy.shape[-1]
    R = gy.numel() // Cc
    g = torch.empty_like(gy)
    chunks = _colsum_chunks(R, Cc) if Cc % 4 == 0 else 1
    part = torch.empty((chunks, Cc), device=gy.device, dtype=torch.float32)
    _lib.call("rk_lrelu_gate_colsum_f32", _p(gy), _p(y), _p(g), R, Cc, float(slope), _p(part), chunks, _s())
    if acc is not None:
        assert acc.shape == (Cc,) and acc.dtype == torch.float32 and acc.is_contiguous()
        if Cc % 4:   # odd width (the slab fold takes whole float4s)
            return g, acc.add_(part.sum(0))
        return g, reduce_slabs(part, acc, accumulate=True)
    if chunks == 1:
        return g, part[0]
    out = torch.empty(Cc, device=gy.device, dtype=torch.float32)
    return g, reduce_slabs(part, out)


def _colsum_chunks(R, Cc):
    """Row chunks of the column-sum kernels: ~2 blocks per CU over the column blocks (256 columns per
    block on the vectorised path, C % 4 == 0; 64 otherwise), >= 64 rows per chunk."""
    cols = min(Cc // 4, 64) * 4 if Cc % 4 == 0 else 64
    return max(1, min(cdiv(R, 64), cdiv(2 * NUM_CU, cdiv(Cc, cols))))


def colsum(x2d, out, *, accumulate=False):
    """out[c] (+)= sum_r x2d[r, c] (fp32).  Tall inputs split the rows over ~2 blocks per CU, then fold
    the partial rows with reduce_slabs."""
    R, Cc = x2d.shape
    chunks = _colsum_chunks(R, Cc)
    if chunks == 1:
        _lib.call("rk_colsum_f32", _p(x2d), R, Cc, x2d.stride(0), _p(out), int(accumulate), 1, _s())
        return out
    part = torch.empty((chunks, Cc), device=x2d.device, dtype=torch.float32)
    _lib.call("rk_colsum_f32", _p(x2d), R, Cc, x2d.stride(0), _p(part), 0, chunks, _s())
    if Cc % 4:   # the slab fold takes whole float4s; an odd width (not on the engines' padded paths) folds here
        s = part.sum(0)
        return out.add_(s) if accumulate else out.copy_(s)
    return reduce_slabs(part, out, accumulate=accumulate)


# -------------------------------------------------------------------------------------- batchnorm
def bn_fwd(y, acc, count, gamma, beta, eps, running_mean=None, running_var=None, momentum=0.1, *, pool=False,
           act=ACT_RELU, slope=0.2, coeffs=None, out=None):
    """Train-mode BN (+act, +2x2 max-pool) from the fp64 slot sums ``acc`` [SL][2][C]; writes coeffs
    [4][C] = mean, rstd, scale, shift (for backward).  Returns (out, coeffs)."""
    Nb, H, W, C = y.shape
    if coeffs is None:
        coeffs = torch.empty((4, C), device=y.device, dtype=torch.float32)
    if out is None:
        shape = (Nb, H // 2, W // 2, C) if pool else (Nb, H, W, C)
        out = torch.empty(shape, device=y.device, dtype=torch.float32)
    _lib.call("rk_bnf_fwd", _p(y), _p(acc), acc.shape[0], float(count), _p(gamma), _p(beta), float(eps),
              _p(running_mean), _p(running_var), float(momentum), None, None, _p(coeffs), _p(out), Nb, H, W, C,
              int(pool), int(act), float(slope), _s())
    return out, coeffs


def bn_finalize(y, acc, count, gamma, beta, eps, running_mean=None, running_var=None, momentum=0.1, *, coeffs=None):
    """The coefficient half of bn_fwd (one block): coeffs [4][C] = mean, rstd, scale, shift and the
    running-statistics update, no output pass — the consumer conv normalises + ReLUs y on its loads
    (conv_fwd(pro=coeffs), conv_wgrad(xpro=coeffs))."""
    Nb, H, W, C = y.shape
    if coeffs is None:
        coeffs = torch.empty((4, C), device=y.device, dtype=torch.float32)
    _lib.call("rk_bnf_fwd", _p(y), _p(acc), acc.shape[0], float(count), _p(gamma), _p(beta), float(eps),
              _p(running_mean), _p(running_var), float(momentum), None, None, _p(coeffs), None, Nb, H, W, C,
              0, int(ACT_RELU), 0.2, _s())
    return coeffs


def bn_eval(y, scale, shift, *, pool=False, act=ACT_RELU, slope=0.2, out=None):
    Nb, H, W, C = y.shape
    if out is None:
        shape = (Nb, H // 2, W // 2, C) if pool else (Nb, H, W, C)
        out = torch.empty(shape, device=y.device, dtype=torch.float32)
    _lib.call("rk_bnf_fwd", _p(y), None, 0, 1.0, None, None, 0.0, None, None, 0.0, _p(scale), _p(shift), None, _p(out),
              Nb, H, W, C, int(pool), int(act), float(slope), _s())
    return out


def col_stats(a2d, acc, b2d=None):
    """fp64 slot 0 of ``acc`` += per-column (sum a, sum a*b) (b = a when None)."""
    R, C = a2d.shape
    _lib.call("rk_bnf_colstats", _p(a2d), _p(b2d), R, C, _p(acc), _s())
    return acc


_BWD_BLOCKS = 1024   # grid cap of the BN-backward reduce (8 passes of pixel rows per block)


def bn_bwd(dout, y, coeffs, gamma, acc, *, pool=False, act=ACT_RELU, slope=0.2, dgamma=None, dbeta=None, dy=None,
           accumulate=False, reduced=False, count=None):
    """Backward of out = pool?(act(BN(y))).  ``acc``: zeroed fp64 [SL][2][C] for (sum dz, sum dz*y);
    ``reduced``: the producer of dout already accumulated them (conv_dgrad(bnb=/bnp=...)).
    ``count`` (default the pixel count): ``inf`` with unit coefficients drops the normalisation terms
    (dy = the act mask / pool routing of dout; ``dbeta`` = sum dz, a bias gradient)."""
    Nb, H, W, C = y.shape
    s = _s()
    if not reduced:
        if C <= 1024 and not (C & (C - 1)):
            npix = dout.numel() // C
            # 8 passes of 256 / (C / 4) pixel rows per block (2 passes: 4x the slot atomics, measured slower)
            blocks = max(1, min(_BWD_BLOCKS, cdiv(npix, max(1, 256 // (C // 4)) * 8)))
            _lib.call("rk_bnf_bwd_reduce", _p(dout), _p(y), _p(coeffs), _p(acc), acc.shape[0], blocks, Nb, H, W, C,
                      int(pool), int(act), float(slope), s)
        elif not pool and act == ACT_NONE:
            col_stats(dout.reshape(-1, C), acc, y.reshape(-1, C))
        else:
            raise ValueError('bn_bwd: unsupported channel count {} for pool/act'.format(C))
    if dy is None:
        dy = torch.empty_like(y)
    _lib.call("rk_bnf_bwd_apply", _p(dout), _p(y), _p(coeffs), _p(acc), acc.shape[0],
              float(Nb * H * W) if count is None else float(count), _p(gamma),
              _p(dgamma), _p(dbeta), int(accumulate), _p(dy), Nb, H, W, C, int(pool), int(act), float(slope), s)
    return dy


# ----------------------------------------------------------------------------------- loss / misc
def softmax_xent(logits, labels, ncls, *, dlogits=None, probs=None, loss_sum=None, correct=None, counted=None,
                 ignore_index=-100, grad_scale=None):
    B = logits.shape[0]
    if grad_scale is None:
        grad_scale = 1.0 / max(1, B)
    if dlogits is not None:
        _check(dlogits, 'softmax_xent dlogits')
    _lib.call("rk_softmax_xent_f32", _p(logits), logits.stride(0), _p(labels), B, ncls, ignore_index,
              float(grad_scale), _p(dlogits), 0 if dlogits is None else dlogits.stride(0), _p(probs), _p(loss_sum),
              _p(correct), _p(counted), _s())


HEAD_NC = (8, 16, 32)


def head_ok(ncls_p: int, D: int) -> bool:
    """Shapes the fused classifier head (csrc/kernels/head.hip) takes."""
    return ncls_p in HEAD_NC and D % 32 == 0 and D > 0


def head_fwd_bwd(z, w, bias, labels, ncls, *, dlogits, dz, gated, loss_sum=None, correct=None, counted=None,
                 grad_scale=None):
    """Output layer + softmax cross-entropy + its data gradient in one launch: z [B][D] -> dlogits [B][NC]
    ((softmax - onehot) * grad_scale), dz [B][D] = dlogits W (gated by z > 0 when ``gated``)."""
    _check(z, 'head z')
    B, D = z.shape
    NC = w.shape[0]
    assert w.shape == (NC, D) and dlogits.shape == (B, NC) and dz.shape == (B, D)
    _lib.call("rk_head_fwd_bwd", _p(z), B, D, _p(w), _p(bias), NC, _p(labels), int(ncls),
              float(1.0 / max(1, B) if grad_scale is None else grad_scale), _p(dlogits), _p(dz), int(bool(gated)),
              _p(loss_sum), _p(correct), _p(counted), _s())


def head_dw(z, dlogits, dz, *, dw, db=None, dbh=None):
    """dw [NC][D] = dlogits^T z, db = colsum(dlogits), dbh = colsum(dz) (the hidden layer's bias gradient)."""
    B, D = z.shape
    NC = dlogits.shape[1]
    _lib.call("rk_head_dw", _p(z), _p(dlogits), _p(dz), B, D, NC, _p(dw), _p(db), _p(dbh), _s())


def pack_nhwc(images, cpad=4, scale=1.0, shift=0.0, out=None, nhwc=False, idx=None):
    """uint8/float32 NCHW (``nhwc``: NHWC) -> fp32 NHWC with channels padded to ``cpad``, x*scale+shift.
    ``idx`` (int32 [n], device): pack images[idx] (the minibatch gather in the same pass)."""
    if nhwc:
        Nb, H, W, Cc = images.shape
    else:
        Nb, Cc, H, W = images.shape
    nsrc = Nb
    if idx is not None:
        assert idx.dtype == torch.int32 and idx.is_cuda and idx.dim() == 1
        idx = idx.contiguous()
        Nb = idx.numel()
    if out is None:
        out = torch.empty((Nb, H, W, cpad), device=images.device, dtype=torch.float32)
    is_u8 = 1 if images.dtype == torch.uint8 else 0
    if not is_u8 and images.dtype != torch.float32:
        images = images.float()
    _lib.call("rk_pack_nhwc_f32", _p(images.contiguous()), is_u8 | (2 if nhwc else 0), Nb, Cc, H, W, cpad,
              float(scale), float(shift), _p(out), _p(idx), nsrc, _s())
    return out


# ------------------------------------------------------------------- stride-2 gather convolutions
# The PG-GAN resampling convs as one family closed under differentiation:
#   S2(x, W)  : y[o]  = sum_t W[t] x[2o + d_t]       (4x4 taps d_t in {-1..2}^2, stride 2)
#   S2T(z, W) : x'[p] = sum_{o,t: 2o + d_t = p} W[t]^T z[o]    (its adjoint: the 2x transposed conv)
#   S2W(x, g) : dW[t] = sum_o g[o] x[2o + d_t]^T   (weight gradient)
# with W [Co][16][Ci] (tap t = 4(dy+1) + dx+1).  conv3x3 + 2x2 box downscale (_conv2d_downscale2d,
# pg_gans.py:1053-1059) is S2 with box-summed weights; upscale2d + conv3x3 (_upscale2d_conv2d,
# pg_gans.py:1032-1039) is S2T with box-summed flipped weights — both at 1/2.25 of the MACs of the
# full-resolution conv and without any materialised 2x tensor.
def _tap_word(vals):
    w = 0
    for t, v in enumerate(vals):
        w |= (int(v) + 1 & 3) << (2 * t)
    return w


def _par_d(r, u):
    return (0 if u == 0 else 2) if r == 0 else (1 if u == 0 else -1)


_S2_TPY = _tap_word([t // 4 - 1 for t in range(16)])
_S2_TPX = _tap_word([t % 4 - 1 for t in range(16)])
# S2T parity group g = 2 ry + rx, tap t4 = 2u + v: source offset (r - d) / 2 of the matching S2 tap
_S2T_TPY = [_tap_word([(g >> 1) - _par_d(g >> 1, t4 >> 1) >> 1 for t4 in range(4)]) for g in range(4)]
_S2T_TPX = [_tap_word([(g & 1) - _par_d(g & 1, t4 & 1) >> 1 for t4 in range(4)]) for g in range(4)]
_S2T_OYX = sum(((g >> 1) | ((g & 1) << 1)) << (2 * g) for g in range(4))


def _u32x4(vals):
    import ctypes
    v = list(vals) + [0] * (4 - len(vals))
    return (ctypes.c_uint * 4)(*v)


def sgemm_g(kind, A, B, out, M, N, K, lda, ldb, ldc, H, W, C, Ho, Wo, stride, ntaps, tpy, tpx, *, groups=1, oyx=0,
            os_=1, gstride_b=0, tile=0, nst=2, splits=1, slab_stride=0, bias=None, flags=0, alpha=1.0, slope=0.2):
    _lib.call("rk_sgemm_g", int(kind), int(tile), int(nst), _p(A), _p(B), _p(out), _p(bias), int(M), int(N), int(K),
              int(lda), int(ldb), int(ldc), int(H), int(W), int(C), int(Ho), int(Wo), int(stride), int(ntaps),
              int(groups), _u32x4(tpy), _u32x4(tpx), int(oyx), int(os_), int(gstride_b), int(splits),
              int(slab_stride), int(flags), float(alpha), float(slope), _nbytes(A), _nbytes(B), _s())
    return out


def _act_flags(bias, act):
    return (F_BIAS if bias is not None else 0) | (F_RELU if act == ACT_RELU else F_LRELU if act == ACT_LRELU else 0)


def s2_conv(x, W, *, bias=None, act=ACT_NONE, slope=0.2, out=None):
    """S2: x [N, H, W, Ci] -> [N, H/2, W/2, Co] with W [Co, 16*Ci] (+bias, act)."""
    _check(x, 's2_conv x')
    Nb, H, Wd, Ci = x.shape
    Co = W.shape[0]
    assert W.numel() == Co * 16 * Ci and H % 2 == 0 and Wd % 2 == 0, (W.shape, x.shape)
    Ho, Wo = H // 2, Wd // 2
    M, K = Nb * Ho * Wo, 16 * Ci
    if out is None:
        out = torch.empty((Nb, Ho, Wo, Co), device=x.device, dtype=torch.float32)
    flags = _act_flags(bias, act)

    def run(cfg):
        tile, nst, s = cfg
        geo = (H, Wd, Ci, Ho, Wo, 2, 16, [_S2_TPY], [_S2_TPX])
        if s == 1:
            sgemm_g(6, x, W, out, M, Co, K, Ci, K, Co, *geo, tile=tile, nst=nst, bias=bias, flags=flags, slope=slope)
            return
        slab = torch.empty((s, M, Co), device=x.device, dtype=torch.float32)
        sgemm_g(6, x, W, slab, M, Co, K, Ci, K, Co, *geo, tile=tile, nst=nst, splits=s, slab_stride=M * Co)
        sreduce_epi(slab, M, Co, out.view(M, Co), bias=bias, act=act, slope=slope)
    run(_pick(('s2f', M, Co, K, H, Wd, Ci, flags), _cands(M, Co, splittable=Co % 4 == 0, K=K), run))
    return out


def s2t_weights(W, Co, Ci):
    """W [Co, 16*Ci] -> the 4 parity groups' [Ci][4 taps * Co] B operands of S2T."""
    out = torch.empty((4, Ci, 4 * Co), device=W.device, dtype=torch.float32)
    _lib.call("rk_s2t_weights", _p(W), _p(out), int(Co), int(Ci), _s())
    return out


def s2t_conv(z, W, *, bias=None, act=ACT_NONE, slope=0.2, out=None, wr=None):
    """S2T: z [N, h, w, Co] -> [N, 2h, 2w, Ci] (the adjoint of S2 with the same W [Co, 16*Ci]):
    four output-parity GEMMs of 4 taps each in ONE launch (grid = 4 parity groups x tiles)."""
    _check(z, 's2t_conv z')
    Nb, h, w, Co = z.shape
    Ci = W.numel() // (16 * Co)
    assert W.numel() == Co * 16 * Ci
    if wr is None:
        wr = s2t_weights(W, Co, Ci)
    M, K = Nb * h * w, 4 * Co
    if out is None:
        out = torch.empty((Nb, 2 * h, 2 * w, Ci), device=z.device, dtype=torch.float32)
    flags = _act_flags(bias, act)
    geo = (h, w, Co, h, w, 1, 4, _S2T_TPY, _S2T_TPX)
    kw = dict(groups=4, oyx=_S2T_OYX, os_=2, gstride_b=Ci * K)

    def run(cfg):
        tile, nst, s = cfg
        if s == 1:
            sgemm_g(6, z, wr, out, M, Ci, K, Co, K, Ci, *geo, tile=tile, nst=nst, bias=bias, flags=flags, slope=slope,
                    **kw)
            return
        slab = torch.empty((s, 4 * M, Ci), device=z.device, dtype=torch.float32)
        sgemm_g(6, z, wr, slab, M, Ci, K, Co, K, Ci, *geo, tile=tile, nst=nst, splits=s, slab_stride=4 * M * Ci, **kw)
        sreduce_epi(slab, 4 * M, Ci, out.view(4 * M, Ci), bias=bias, act=act, slope=slope)
    run(_pick(('s2t', M, Ci, K, h, w, Co, flags), _cands(M, Ci, splittable=Ci % 4 == 0, K=K), run))
    return out


def s2_wgrad(x, g, *, out=None):
    """S2W: dW [Co, 16*Ci] = sum_o g[o] (x) x[2o + d_t]; x [N, H, W, Ci], g [N, H/2, W/2, Co]."""
    _check(x, 's2_wgrad x')
    _check(g, 's2_wgrad g')
    Nb, H, Wd, Ci = x.shape
    Co = g.shape[-1]
    Ho, Wo = H // 2, Wd // 2
    assert g.shape == (Nb, Ho, Wo, Co), (g.shape, x.shape)
    M, N, K = Co, 16 * Ci, Nb * Ho * Wo
    if out is None:
        out = torch.empty((Co, N), device=x.device, dtype=torch.float32)
    geo = (H, Wd, Ci, Ho, Wo, 2, 16, [_S2_TPY], [_S2_TPX])

    def run(cfg):
        tile, nst, s = cfg
        if s == 1:
            sgemm_g(7, g, x, out, M, N, K, Co, Ci, N, *geo, tile=tile, nst=nst)
            return
        slab = torch.empty((s, M, N), device=x.device, dtype=torch.float32)
        sgemm_g(7, g, x, slab, M, N, K, Co, Ci, N, *geo, tile=tile, nst=nst, splits=s, slab_stride=M * N)
        reduce_slabs(slab, out)
    cands = _cands(M, N, splittable=True, K=K)
    split = [c for c in cands if c[2] > 1]
    if split:
        cands = [max(split, key=lambda c: min(cdiv(M, tile_dims(c[0])[0]) * cdiv(N, tile_dims(c[0])[1]) * c[2],
                                              2 * NUM_CU))] + cands
    run(_pick(('s2w', M, N, K, H, Wd, Ci), cands, run))
    return out


# ------------------------------------------------------------------------------------ resampling
def upscale2x(x, scale=1.0, out=None):
    """nearest 2x upscale of NHWC fp32 / bf16 (times ``scale``)."""
    Nb, H, W, Cc = x.shape
    if out is None:
        out = torch.empty((Nb, 2 * H, 2 * W, Cc), device=x.device, dtype=x.dtype)
    _lib.call("rk_resample2x", 0, int(x.dtype == torch.bfloat16), _p(x.contiguous()), _p(out), Nb, H, W, Cc,
              float(scale), _s())
    return out


def downscale2x(x, scale=0.25, out=None):
    """``scale`` x 2x2 sum of NHWC fp32 / bf16 (0.25: the box-filter downscale2d)."""
    Nb, H, W, Cc = x.shape
    if out is None:
        out = torch.empty((Nb, H // 2, W // 2, Cc), device=x.device, dtype=x.dtype)
    _lib.call("rk_resample2x", 1, int(x.dtype == torch.bfloat16), _p(x.contiguous()), _p(out), Nb, H, W, Cc,
              float(scale), _s())
    return out


def conv_wt(w, taps=9):
    """w [Cout, taps*Cin] -> [Cin, taps*Cout] flipped transposed weights: conv_dgrad(dy, conv_wt(w)) is the
    data gradient of conv_fwd(x, w) (one LDS-tiled transpose launch; the autograd path's per-call
    equivalent of SConvWT)."""
    Cout = w.shape[0]
    Cin = w.numel() // (taps * Cout)
    out = torch.empty((Cin, taps * Cout), device=w.device, dtype=torch.float32)
    _lib.call("rk_wflip_t", _p(w.contiguous()), _p(out), int(Cout), int(Cin), int(taps), _s())
    return out


# ------------------------------------------------------------------------------ grouped GEMMs
# k same-shape problems per launch (rk_sgemm_grp): the k models of an inference ensemble run each layer
# as ONE kernel (k x the workgroups of one model: small-batch layers fill the chip, launches / k).
def sgemm_grp(kind, A, B, out, M, N, K, lda, ldb, ldc, groups, gstride_a, gstride_b, gstride_o, gstride_bias=0, *,
              tile=0, nst=2, splits=1, slab_stride=0, bias=None, flags=0, alpha=1.0, slope=0.2, H=1, W=1, C=4,
              taps=1):
    _lib.call("rk_sgemm_grp", int(kind), int(tile), int(nst), _p(A), _p(B), _p(out), _p(bias), int(M), int(N), int(K),
              int(lda), int(ldb), int(ldc), int(H), int(W), int(C), int(taps), int(splits), int(slab_stride),
              int(flags), float(alpha), float(slope), _nbytes(A), _nbytes(B), int(groups), int(gstride_a),
              int(gstride_b), int(gstride_o), int(gstride_bias), _s())
    return out


def _grp_run(kind, A, B, out, M, N, K, lda, ldb, G, gsa, key, *, bias=None, act=ACT_NONE, slope=0.2, geo=None,
             extra=None):
    """Autotuned grouped launch: out [G, M, N]; split-K slabs [s, G*M, N] combined by sreduce_epi with
    per-group bias.  ``extra(cfg)``: runs the WINO_CFGS candidates (grouped Winograd convs)."""
    flags = _act_flags(bias, act)
    geo = geo or {}

    def run(cfg):
        tile, nst, s = cfg
        if cfg in WINO_CFGS or cfg in WINO4_CFGS:
            extra(cfg)
            return
        if s == 1:
            sgemm_grp(kind, A, B, out, M, N, K, lda, ldb, N, G, gsa, N * K, M * N, N, tile=tile, nst=nst,
                      bias=bias, flags=flags, slope=slope, **geo)
            return
        slab = torch.empty((s, G * M, N), device=out.device, dtype=torch.float32)
        sgemm_grp(kind, A, B, slab, M, N, K, lda, ldb, N, G, gsa, N * K, M * N, 0, tile=tile, nst=nst, splits=s,
                  slab_stride=G * M * N, **geo)
        sreduce_epi(slab, G * M, N, out.view(G * M, N), bias=bias, act=act, slope=slope, bias_rows=M)
    cands = [c for c in _cands(M * G, N, splittable=N % 4 == 0, K=K) if (c[0] & 15) < 4 or (c[0] & 15) in _FEW_WAVE]
    if extra is not None:
        cands.extend(getattr(extra, 'cfgs', WINO_CFGS))
    run(_pick(key, cands, run))
    return out


def conv_fwd_grp_pool_ok(H, W, Cin, wino, wino4):
    """conv_fwd_grp(pool=True) has a fused candidate for this shape (F(4x4) or the small-tile F(2x2))."""
    return ((wino4 is not None and wino4_ok(H, W, Cin))
            or (wino is not None and wino_ok(H, W, Cin) and any(_wino_variant(c) >= 2 for c in WINO_CFGS)))


def conv_fwd_grp(x, W, *, bias=None, act=ACT_NONE, slope=0.2, out=None, wino=None, wino4=None, pool=False):
    """k convs in one launch: x [G, Nb, H, W, Cin] (or [Nb, H, W, Cin] shared by every group),
    W [G, Cout, taps*Cin], bias [G, Cout] -> [G, Nb, H, W, Cout] (3x3 stride-1 or 1x1).
    ``wino``: stacked Winograd weights [G, 16, Cout, Cin] -> grouped fused F(2x2,3x3) candidates;
    ``wino4``: [G, 36, Cout, Cin] -> grouped F(4x4,3x3) candidates.  ``pool`` (bias + ReLU): the 2x2
    max-pool written by the fused kernels' epilogue -> [G, Nb, H/2, W/2, Cout] (only they are candidates;
    see conv_fwd_grp_pool_ok)."""
    G, Cout, K = W.shape
    shared = x.dim() == 4
    Nb, H, Wd, Cin = x.shape[-4:]
    taps = K // Cin
    assert taps in (1, 9) and K == taps * Cin and (shared or x.shape[0] == G), (x.shape, W.shape)
    _check(x, 'conv_fwd_grp x')
    M = Nb * H * Wd
    if pool:
        return _conv_fwd_grp_pooled(x, W, bias, act, out, wino, wino4)
    if out is None:
        out = torch.empty((G, Nb, H, Wd, Cout), device=x.device, dtype=torch.float32)
    extra = None
    w2 = wino is not None and taps == 9 and wino_ok(H, Wd, Cin) and act in (ACT_NONE, ACT_RELU)
    w4 = wino4 is not None and taps == 9 and wino4_ok(H, Wd, Cin) and act in (ACT_NONE, ACT_RELU)
    if w2 or w4:
        assert not w2 or (wino.shape == (G, 16, Cout, Cin) and wino.is_contiguous())
        assert not w4 or (wino4.shape == (G, 36, Cout, Cin) and wino4.is_contiguous())

        def extra(cfg):
            if cfg in WINO4_CFGS:
                wino4_conv_grp(x, wino4, out=out, bias=bias, relu=act == ACT_RELU, variant=_wino4_variant(cfg))
            else:
                wino_conv_grp(x, wino, out=out, bias=bias, relu=act == ACT_RELU, variant=_wino_variant(cfg))
        extra.cfgs = (WINO_CFGS if w2 else ()) + (WINO4_CFGS if w4 else ())
    return _grp_run(0, x, W, out, M, Cout, K, Cin, K, G, 0 if shared else M * Cin,
                    ('sfg', G, M, Cout, K, H, Wd, Cin, shared, bias is not None, act, w2, w4), bias=bias,
                    act=act, slope=slope, geo=dict(H=H, W=Wd, C=Cin, taps=taps), extra=extra)


def _conv_fwd_grp_pooled(x, W, bias, act, out, wino, wino4):
    G, Cout, K = W.shape
    Nb, H, Wd, Cin = x.shape[-4:]
    assert bias is not None and act == ACT_RELU and K == 9 * Cin and H % 2 == 0 and Wd % 2 == 0
    if out is None:
        out = torch.empty((G, Nb, H // 2, Wd // 2, Cout), device=x.device, dtype=torch.float32)
    w4 = wino4 is not None and wino4_ok(H, Wd, Cin)
    w2 = wino is not None and wino_ok(H, Wd, Cin)
    cands = ([c for c in WINO4_CFGS] if w4 else []) + ([c for c in WINO_CFGS if _wino_variant(c) >= 2] if w2 else [])
    if not cands:
        raise ValueError('conv_fwd_grp(pool=True): no fused candidate (see conv_fwd_grp_pool_ok)')

    def run(cfg):
        if cfg in WINO4_CFGS:
            wino4_conv_grp(x, wino4, out=out, bias=bias, relu=True, variant=_wino4_variant(cfg), pool=True)
        else:
            wino_conv_grp(x, wino, out=out, bias=bias, relu=True, variant=_wino_variant(cfg), pool=True)
    run(_pick(('sfgp', G, Nb * H * Wd, Cout, K, H, Wd, Cin, x.dim() == 4, w2, w4), cands, run))
    return out


def linear_grp(x, w, bias=None, *, act=ACT_NONE, slope=0.2, out=None):
    """k dense layers in one launch: x [G, M, K] (or [M, K] shared), w [G, N, K], bias [G, N] -> [G, M, N]."""
    G, N, K = w.shape
    shared = x.dim() == 2
    M = x.shape[-2]
    _check(x, 'linear_grp x')
    if out is None:
        out = torch.empty((G, M, N), device=x.device, dtype=torch.float32)
    return _grp_run(3, x, w, out, M, N, K, K, K, G, 0 if shared else M * K,
                    ('slg', G, M, N, K, shared, bias is not None, act), bias=bias, act=act, slope=slope)


def bn_eval_grp(y, scale, shift, *, pool=False, act=ACT_RELU, slope=0.2, out=None):
    """eval BN(+act, +2x2 max-pool) of G stacked batches y [G, Nb, H, W, C] with per-group scale / shift [G, C]."""
    G, Nb, H, W, C = y.shape
    if out is None:
        out = torch.empty((G, Nb, H // 2 if pool else H, W // 2 if pool else W, C), device=y.device,
                          dtype=torch.float32)
    _lib.call("rk_bnf_eval_grp", _p(y), _p(scale.contiguous()), _p(shift.contiguous()), _p(out), G, Nb, H, W, C,
              int(pool), int(act), float(slope), _s())
    return out
