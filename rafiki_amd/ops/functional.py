"""Tensor-level wrappers over the gfx950 kernels (no autograd; see ``rafiki_amd.ops.autograd``).

Layout conventions (all device tensors contiguous):
  * activations  : NHWC bf16 ``[N, H, W, C]`` with C % 8 == 0 (the stem pads RGB to 8 channels)
  * conv weights : bf16 ``[Cout, kh, kw, Cin]`` (= GEMM B operand ``[N][K]``, K = 9*Cin)
  * dense weights: bf16 ``[out, in]``
  * grads of weights and all optimizer state: fp32

Every function launches on ``torch.cuda.current_stream()`` and allocates only through the torch
caching allocator, so whole training steps can be captured into a hipGraph.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import _lib, autotune

KIND_CONV_FWD, KIND_CONV_DGRAD, KIND_CONV_WGRAD, KIND_DENSE, KIND_DENSE_DX, KIND_DENSE_DW, KIND_CONV_UP = range(7)
FLAG_RELU, FLAG_BIAS, FLAG_STATS, FLAG_GATE, FLAG_ACCUM, FLAG_LRELU = 1, 2, 4, 8, 16, 32
FLAG_SATOM = 256
FLAG_BNB = 512
FLAG_BNP = 1024  # dgrad into a BN+ReLU+maxpool layer: its BN-backward sums in the epilogue
# BatchNorm statistics as fp64 atomic sums in a few slots (conv epilogue / bwd reduce) consumed by
# fused finalize+apply kernels: 2 launches per BN layer and direction instead of 4 / 3 (summation order
# varies run to run in the last bits of the fp64 sums; the partial-row path remains for channel counts
# the slot kernels do not take)
BN_ATOMIC = True
ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2
# shape 4: 64x64 wave-K-split kernel (igemm_ks_kernel, LDS-DMA rings only): each wave owns the whole
# tile for a quarter of every K-tile pair — half the LDS reads per MFMA of shape 3 (small-M layers)
TILES = [(128, 128), (128, 64), (64, 128), (64, 64), (64, 64)]
KS_TILE = 4
_KS_VARIANTS = (64, 32)  # 2-stage (64 KiB LDS, 2 blocks/CU) and 3-stage (96 KiB) rings
NUM_CU = 256
# Kernel variant bits OR'ed into the tile code (see rk_igemm): 0 register-staged, 16 register ring,
# 32 LDS-DMA 3-stage ring, 64 LDS-DMA 2-stage, 128 LDS-DMA 4-stage (chosen per shape by the tuner).


def _p(t: Optional[torch.Tensor]):
    """Device pointer of a kernel operand; a host tensor here would be an illegal GPU access."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError('host tensor {} {} passed to a gfx950 kernel'.format(tuple(t.shape), t.dtype))
    return t.data_ptr()


def _nbytes(t):
    """Bytes addressable from t.data_ptr() to the end of its storage (buffer-descriptor extent)."""
    return t.untyped_storage().nbytes() - t.storage_offset() * t.element_size()


def _s():
    return torch.cuda.current_stream().cuda_stream


def cdiv(a: int, b: int) -> int:
    return (a + b - 1) // b


def pick_tile(M: int, N: int) -> int:
    """Largest tile that still gives >= 2 blocks per CU without padding waste > 30%."""
    best, best_blocks = 3, -1
    for t, (bm, bn) in enumerate(TILES[:4]):
        blocks = cdiv(M, bm) * cdiv(N, bn)
        waste = (cdiv(M, bm) * bm * cdiv(N, bn) * bn) / float(M * N)
        if waste > 1.3 and t != 3:
            continue
        if blocks >= 2 * NUM_CU:
            return t
        if blocks > best_blocks:
            best, best_blocks = t, blocks
    return best


def pick_splits(M: int, N: int, K: int, tile: int, target_blocks: int = 2 * NUM_CU, min_ktiles: int = 4) -> int:
    bm, bn = TILES[tile & 15]
    tiles = cdiv(M, bm) * cdiv(N, bn)
    ktiles = cdiv(K, 64)
    s = max(1, min(cdiv(target_blocks, tiles), ktiles // min_ktiles))
    # make every split non-empty
    per = cdiv(ktiles, s)
    return cdiv(ktiles, per)


# Staging variants the tuner tries.  The 3/4-stage LDS-DMA rings (32/128) win some isolated timings
# but lose inside the training step (less occupancy when neighbouring kernels share L2), so they are not
# offered (the kernels keep them: tile codes | 32 / | 128).
_VARIANTS = (0, 64)


def _tile_candidates(M, N, fixed_bm=None, ks=True):
    """Heuristic pick first (used when tuning is impossible), then every shape x staging variant.
    ks=False leaves out the wave-K-split shape (it cannot write per-wave partial statistics rows)."""
    first = pick_tile(M, N)
    if fixed_bm is not None:  # stats partial-row count depends on BM: keep BM fixed for stats outputs
        shapes = [t for t in range(4) if TILES[t][0] == fixed_bm]
    else:
        shapes = list(range(4))
    out = [(first,)]
    for t in shapes:
        for v in _VARIANTS:
            c = (t | v,)
            if c not in out:
                out.append(c)
    if ks and KS and fixed_bm in (None, 64):
        out += [(KS_TILE | v,) for v in _KS_VARIANTS]
    return out


def _split_candidates(M, N, K):
    t0 = pick_tile(M, N)
    s_h = pick_splits(M, N, K, t0)
    first = (t0, s_h)
    out = [first]
    kt = cdiv(K, 64)
    for t in range(5 if KS else 4):
        blocks = cdiv(M, TILES[t][0]) * cdiv(N, TILES[t][1])
        for v in ((0, 64, 128) if t != KS_TILE else _KS_VARIANTS):
            for s in (1, 2, 4, 8, 16, 32, 64, 128, 256):
                if s > kt or (s == 1 and kt > 64) or s * M * N * 4 > (256 << 20):
                    continue
                # keep the grid between ~1/2 and ~8 waves of the chip: fewer blocks idle CUs, more only
                # add slab traffic (prunes ~2/3 of the space; tuning time matters for short trials)
                if not (NUM_CU // 2 <= blocks * s <= 8 * NUM_CU) and s != s_h and not (s == 1 and blocks >= NUM_CU // 2):
                    continue
                per = cdiv(kt, s)
                s_eff = cdiv(kt, per)
                c = (t | v, s_eff)
                if c not in out:
                    out.append(c)
    return out


def _tuned(key, candidates, run):
    from . import autotune
    if not autotune.ENABLED:
        return candidates[0]
    return autotune.tune(key, candidates, run)


def igemm(kind, epi, A, B, out, M, N, K, lda=0, ldb=0, ldc=0, *, bias=None, stats=None, gate=None, H=1, W=1,
          C=8, taps=1, Cb=1, splits=1, slab_stride=0, flags=0, alpha=1.0, slope=0.2, tile=None):
    if tile is None:
        tile = pick_tile(M, N)
    _lib.call("rk_igemm", kind, epi, tile, _p(A), _p(B), _p(out), _p(bias), _p(stats), _p(gate), M, N, K, lda, ldb,
              ldc, H, W, C, taps, Cb, splits, slab_stride, flags, alpha, slope, _nbytes(A), _nbytes(B), _s())
    return out


# ------------------------------------------------------------------------------------------ conv
def stats_rows(M: int, N: int, tile: Optional[int] = None) -> int:
    t = pick_tile(M, N) if tile is None else tile
    return cdiv(M, TILES[t & 15][0]) * 2


# Halo-tiled 3x3 conv (rk_hconv): one LDS patch per (item, 64-channel chunk) serves all 9 taps.
# Candidates are ('h', bn_bit, grid): grid 0 = one item per block, else a persistent grid.
HCONV = True
KS = True


def _hconv_bm(W: int) -> int:
    return 64 if W == 8 else 128


def _hconv_candidates(M, N, H, W, C, taps):
    if not HCONV or taps != 9 or W not in (4, 8, 16, 32) or H & (H - 1):
        return []
    if (W == 4 and (H != 4 or M % _hconv_bm(W))) or (W != 4 and (H * W) % _hconv_bm(W)):
        return []  # W = 4: items of 8 whole 4x4 images
    if C < 64 or C & (C - 1) or N % 64:
        return []
    out = []
    for bn_bit in ((0, 1) if N % 128 == 0 else (0,)):
        items = (M // _hconv_bm(W)) * (N // (128 if bn_bit else 64))
        per_cu = 1 if bn_bit else 2  # LDS-resident blocks per CU
        for g in (0, NUM_CU * per_cu):
            if g and g >= items:
                continue
            out.append(('h', bn_bit, g))
    return out


def _cfg_bm(cfg, W: int) -> int:
    return _hconv_bm(W) if cfg[0] == 'h' else TILES[cfg[0] & 15][0]


def hconv(dgrad, A, B, out, M, N, K, ldb, H, W, C, *, bias=None, stats=None, gate=None, flags=0, alpha=1.0,
          slope=0.2, bn_bit=0, grid=0):
    _lib.call("rk_hconv", int(dgrad), int(bn_bit), _p(A), _p(B), _p(out), _p(bias), _p(stats), _p(gate), M, N, K,
              ldb, H, W, C, flags, float(alpha), float(slope), _nbytes(A), _nbytes(B), int(grid), _s())
    return out


def slab_epi(slab, S, M, N, out, *, mode=0, gate=None, scale=None, shift=None, acc=None):
    """bf16 out[M][N] = sum of S fp32 split-K slabs, plus BN statistics into ``acc`` (mode 1), the
    BN-backward ReLU mask and sums (mode 2, as FLAG_BNB) or a ReLU-backward gate (mode 3)."""
    slmask = acc.shape[0] - 1 if acc is not None else 0
    _lib.call("rk_slab_epi", _p(slab), int(S), int(M), int(N), int(mode), _p(gate), _p(scale), _p(shift), _p(acc),
              int(slmask), _p(out), _s())
    return out


# Split-K conv forward / data-gradient: ('k', tile, S) = S fp32 slabs from the igemm + one rk_slab_epi
# combine.  Offered only where a big tile shape (fewer L2->LDS re-reads of both operands) has too few
# output tiles to fill the chip on its own: the VGG 4x4 / 8x8 layers (M = 4096 / 16384 at batch 256).
CONV_SPLIT = True


def _conv_split_candidates(M, N, K, H, W, C):
    if not CONV_SPLIT or N % 4 or N > 1024 or 256 % (N // 4) or C & (C - 1) or H & (H - 1) or W & (W - 1):
        return []
    kt = cdiv(K, 64)
    out = []
    for t in (0, 1, 2):
        blocks = cdiv(M, TILES[t][0]) * cdiv(N, TILES[t][1])
        if blocks >= 2 * NUM_CU:
            continue
        for s in (2, 3, 4):
            if s > kt // 4 or blocks * s > 4 * NUM_CU:
                continue
            per = cdiv(kt, s)
            c = ('k', t | 64, cdiv(kt, per))
            if c not in out:
                out.append(c)
    return out


_BWD_RED_CAP = 2048


def bn_slots(C: int) -> int:
    """Atomic-accumulator slots for C channels (fewer adders per address; the consumers read
    slots*2*C doubles per block, kept at 8 KiB)."""
    return max(1, min(8, 512 // C))


def bn_acc_buffer(C: int, device) -> torch.Tensor:
    return torch.zeros((bn_slots(C), 2, C), device=device, dtype=torch.float64)


def conv_fwd(x: torch.Tensor, w: torch.Tensor, *, taps: int = 9, bias=None, want_stats=False, act=ACT_NONE,
             slope=0.2, out=None, stats_acc=None):
    """y = conv3x3(x, w) (stride 1, pad 1) [+bias][act]; optional per-channel partial stats."""
    Nb, H, W, Cin = x.shape
    Cout = w.shape[0]
    M, K = Nb * H * W, taps * Cin
    assert w.numel() == Cout * K, (w.shape, taps, Cin)
    if out is None:
        out = torch.empty((Nb, H, W, Cout), device=x.device, dtype=torch.bfloat16)
    stats = None
    flags = 0
    if stats_acc is not None:  # fp64 atomic sums into a zeroed [SL][2][Cout] table
        assert stats_acc.dtype == torch.float64 and stats_acc.shape[-1] == Cout
        stats = stats_acc
        flags |= FLAG_STATS | FLAG_SATOM | ((stats_acc.shape[0] - 1) << 12)
    elif want_stats:
        stats = _bn_rows_buffer(M, Cout, x.device)
        flags |= FLAG_STATS
    if bias is not None:
        flags |= FLAG_BIAS
    if act == ACT_RELU:
        flags |= FLAG_RELU
    elif act == ACT_LRELU:
        flags |= FLAG_LRELU
    def run(cfg):
        if cfg[0] == 'h':
            hconv(0, x, w, out, M, Cout, K, K, H, W, Cin, bias=bias, stats=stats, flags=flags, slope=slope,
                  bn_bit=cfg[1], grid=cfg[2])
        elif cfg[0] == 'k':
            slab = torch.empty((cfg[2], M, Cout), device=x.device, dtype=torch.float32)
            igemm(KIND_CONV_FWD, 1, x, w, slab, M, Cout, K, Cin, K, Cout, H=H, W=W, C=Cin, taps=taps,
                  splits=cfg[2], slab_stride=M * Cout, tile=cfg[1])
            slab_epi(slab, cfg[2], M, Cout, out, mode=1 if stats_acc is not None else 0, acc=stats_acc)
        else:
            igemm(KIND_CONV_FWD, 0, x, w, out, M, Cout, K, Cin, K, Cout, bias=bias, stats=stats, H=H, W=W, C=Cin,
                  taps=taps, flags=flags, slope=slope, tile=cfg[0])
    mode = 'acc' if stats_acc is not None else bool(want_stats)
    partial_rows = want_stats and stats_acc is None
    split_ok = bias is None and act == ACT_NONE and not partial_rows
    cfg = _tuned(('cf', M, Cout, K, H, W, Cin, taps, mode),
                 _tile_candidates(M, Cout, ks=not partial_rows)
                 + _hconv_candidates(M, Cout, H, W, Cin, taps)
                 + (_conv_split_candidates(M, Cout, K, H, W, Cin) if split_ok else []), run)
    if stats_acc is not None and autotune.can_tune():
        stats_acc.zero_()  # tuning runs accumulated into it
    run(cfg)
    if stats_acc is not None:
        return out, stats_acc
    return (out, stats[:cdiv(M, _cfg_bm(cfg, W)) * 2]) if want_stats else out


def conv_up(x: torch.Tensor, w: torch.Tensor, *, bias=None, act=ACT_NONE, slope=0.2, out=None):
    """y = conv3x3(upscale2d_nearest(x)) [+bias][act] without materialising the 2x input: the gather
    reads input pixel ((h+dy)>>1, (w+dx)>>1) directly (PG-GAN ``_upscale2d_conv2d``, pg_gans.py:1032-1039)."""
    Nb, h, w_, Cin = x.shape
    H, W = 2 * h, 2 * w_
    Cout = w.shape[0]
    M, K = Nb * H * W, 9 * Cin
    assert w.numel() == Cout * K, (w.shape, Cin)
    if out is None:
        out = torch.empty((Nb, H, W, Cout), device=x.device, dtype=torch.bfloat16)
    flags = (FLAG_BIAS if bias is not None else 0) | (FLAG_RELU if act == ACT_RELU else 0) | (
        FLAG_LRELU if act == ACT_LRELU else 0)

    def run(cfg):
        igemm(KIND_CONV_UP, 0, x, w, out, M, Cout, K, Cin, K, Cout, bias=bias, H=H, W=W, C=Cin, taps=9,
              flags=flags, slope=slope, tile=cfg[0])
    run(_tuned(('cu', M, Cout, K, H, W, Cin), [c for c in _tile_candidates(M, Cout) if c[0] < 32], run))
    return out


def _bn_rows_buffer(M, C, device):
    # sized for the smallest BM (64); the tuned tile's BM decides how many rows are written
    return torch.empty((cdiv(M, 64) * 2, 2, C), device=device, dtype=torch.float32)


def conv_dgrad(dy: torch.Tensor, w: torch.Tensor, *, taps: int = 9, out=None, gate=None, bn_y=None,
               bn_coeffs=None, bn_acc=None):
    """dx = dgrad(dy, w).  With ``bn_y``/``bn_coeffs``/``bn_acc`` (the input layer's BN input,
    its [4][C] coefficients and its zeroed fp64 backward slot table) the epilogue applies that
    layer's ReLU mask and accumulates BN backward's (sum dz, sum dz*y), so bn_bwd_acc(...,
    reduced=True) skips its reduction pass (FLAG_BNB)."""
    Nb, H, W, Cout = dy.shape
    Cin = w.numel() // (Cout * taps)
    M, K = Nb * H * W, taps * Cout
    if out is None:
        out = torch.empty((Nb, H, W, Cin), device=dy.device, dtype=torch.bfloat16)
    flags, bias, stats = (FLAG_GATE if gate is not None else 0), None, None
    if bn_y is not None:
        assert bn_y.shape == out.shape and bn_acc.dtype == torch.float64 and bn_acc.shape[-1] == Cin
        gate, bias, stats = bn_y, bn_coeffs[2], bn_acc
        flags = FLAG_BNB | FLAG_SATOM | ((bn_acc.shape[0] - 1) << 12)

    def run(cfg):
        if cfg[0] == 'h':
            hconv(1, dy, w, out, M, Cin, K, taps * Cin, H, W, Cout, gate=gate, bias=bias, stats=stats, flags=flags,
                  bn_bit=cfg[1], grid=cfg[2])
        elif cfg[0] == 'k':
            slab = torch.empty((cfg[2], M, Cin), device=dy.device, dtype=torch.float32)
            igemm(KIND_CONV_DGRAD, 1, dy, w, slab, M, Cin, K, Cout, taps * Cin, Cin, H=H, W=W, C=Cout, taps=taps,
                  Cb=Cout, splits=cfg[2], slab_stride=M * Cin, tile=cfg[1])
            if bn_y is not None:
                slab_epi(slab, cfg[2], M, Cin, out, mode=2, gate=bn_y, scale=bn_coeffs[2], shift=bn_coeffs[3],
                         acc=bn_acc)
            else:
                slab_epi(slab, cfg[2], M, Cin, out, mode=3 if gate is not None else 0, gate=gate)
        else:
            igemm(KIND_CONV_DGRAD, 0, dy, w, out, M, Cin, K, Cout, taps * Cin, Cin, gate=gate, bias=bias,
                  stats=stats, H=H, W=W, C=Cout, taps=taps, Cb=Cout, flags=flags, tile=cfg[0])
    cfg = _tuned(('cd', M, Cin, K, H, W, Cout, taps),
                 _tile_candidates(M, Cin) + _hconv_candidates(M, Cin, H, W, Cout, taps)
                 + _conv_split_candidates(M, Cin, K, H, W, Cout), run)
    if bn_acc is not None and autotune.can_tune():
        bn_acc.zero_()  # tuning runs accumulated into it
    run(cfg)
    return out


class ConvWT:
    """Flipped, transposed bf16 copies wt[ci][8-t][co] = w[co][t][ci] of several 3x3 conv weights that
    live in one bf16 arena, refreshed by ONE rk_conv_wt launch per training step.  With them the data
    gradient is a forward conv of dy (``conv_dgrad_t``) on the forward kernels."""

    def __init__(self, arena: torch.Tensor, weights):
        """arena: contiguous bf16 tensor; weights: list of bf16 views into it, shaped [Cout, 9*Cin]
        (or [Cout, 3, 3, Cin])."""
        self.arena = arena
        meta, desc, self._views, off = [], [], [], 0
        for l, w in enumerate(weights):
            Cout = w.shape[0]
            Cin = w.numel() // (9 * Cout)
            so = (w.data_ptr() - arena.data_ptr()) // 2
            assert so % 8 == 0 and Cin % 8 == 0 and Cout % 8 == 0, (so, Cin, Cout)
            meta.append([so, off, Cout, Cin])
            for t in range(9):
                for co0 in range(0, Cout, 64):
                    for ci0 in range(0, Cin, 64):
                        desc.append([l, t, co0, ci0])
            self._views.append((off, Cin, Cout))
            off += (Cin * 9 * Cout + 63) // 64 * 64
        dev = arena.device
        self.buf = torch.zeros(max(off, 64), dtype=torch.bfloat16, device=dev)
        self.meta = torch.tensor(meta, dtype=torch.int64, device=dev)
        self.desc = torch.tensor(desc, dtype=torch.int32, device=dev)

    def refresh(self):
        _lib.call("rk_conv_wt", _p(self.arena), _p(self.buf), _p(self.desc), self.desc.shape[0], _p(self.meta), _s())

    def view(self, l: int) -> torch.Tensor:
        off, Cin, Cout = self._views[l]
        return self.buf[off:off + Cin * 9 * Cout].view(Cin, 9 * Cout)


def conv_dgrad_t(dy: torch.Tensor, wt: torch.Tensor, *, out=None, gate=None, bn_y=None, bn_coeffs=None,
                 bn_acc=None, bn_pool_y=None):
    """dx = dgrad(dy, w) computed as conv3x3(dy, wt) with wt = ConvWT.view(...) [Cin][9*Cout]: the forward
    kernels (halo-tiled / implicit GEMM / split-K) with the data-gradient epilogues of conv_dgrad
    (ReLU gate, or FLAG_BNB: the input layer's BN+ReLU mask and BN-backward sums)."""
    Nb, H, W, Cout = dy.shape
    Cin = wt.shape[0]
    M, K = Nb * H * W, 9 * Cout
    assert wt.numel() == Cin * K
    if out is None:
        out = torch.empty((Nb, H, W, Cin), device=dy.device, dtype=torch.bfloat16)
    flags, bias, stats = (FLAG_GATE if gate is not None else 0), None, None
    if bn_y is not None:
        assert bn_y.shape == out.shape and bn_acc.dtype == torch.float64 and bn_acc.shape[-1] == Cin
        gate, bias, stats = bn_y, bn_coeffs[2], bn_acc
        flags = FLAG_BNB | FLAG_SATOM | ((bn_acc.shape[0] - 1) << 12)
    elif bn_pool_y is not None:
        assert bn_pool_y.shape == (Nb, 2 * H, 2 * W, Cin) and bn_acc.dtype == torch.float64
        assert not (H & (H - 1)) and not (W & (W - 1)), 'FLAG_BNP needs power-of-two geometry'
        gate, bias, stats = bn_pool_y, bn_coeffs[2], bn_acc
        flags = FLAG_BNP | FLAG_SATOM | ((bn_acc.shape[0] - 1) << 12)

    def run(cfg):
        if cfg[0] == 'h':
            hconv(0, dy, wt, out, M, Cin, K, K, H, W, Cout, gate=gate, bias=bias, stats=stats, flags=flags,
                  bn_bit=cfg[1], grid=cfg[2])
        elif cfg[0] == 'k':
            slab = torch.empty((cfg[2], M, Cin), device=dy.device, dtype=torch.float32)
            igemm(KIND_CONV_FWD, 1, dy, wt, slab, M, Cin, K, Cout, K, Cin, H=H, W=W, C=Cout, taps=9,
                  splits=cfg[2], slab_stride=M * Cin, tile=cfg[1])
            if bn_y is not None:
                slab_epi(slab, cfg[2], M, Cin, out, mode=2, gate=bn_y, scale=bn_coeffs[2], shift=bn_coeffs[3],
                         acc=bn_acc)
            else:
                slab_epi(slab, cfg[2], M, Cin, out, mode=3 if gate is not None else 0, gate=gate)
        else:
            igemm(KIND_CONV_FWD, 0, dy, wt, out, M, Cin, K, Cout, K, Cin, gate=gate, bias=bias, stats=stats, H=H,
                  W=W, C=Cout, taps=9, flags=flags, tile=cfg[0])
    mode = 'bnb' if bn_y is not None else 'bnp' if bn_pool_y is not None else bool(gate is not None)
    cfg = _tuned(('cdT', M, Cin, K, H, W, Cout, mode),
                 _tile_candidates(M, Cin) + _hconv_candidates(M, Cin, H, W, Cout, 9)
                 + (_conv_split_candidates(M, Cin, K, H, W, Cout) if bn_pool_y is None else []), run)
    if bn_acc is not None and autotune.can_tune():
        bn_acc.zero_()  # tuning runs accumulated into it
    run(cfg)
    return out


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, *, taps: int = 9, out=None, accumulate=False, splits=None):
    """dW[co][tap][ci] (fp32) = sum over pixels of dy[p][co] * x[shift_tap(p)][ci]."""
    Nb, H, W, Cout = dy.shape
    Cin = x.shape[-1]
    M, N, K = Cout, taps * Cin, Nb * H * W
    if out is None:
        out = torch.empty((Cout, N), device=dy.device, dtype=torch.float32)
    def run(cfg):
        if cfg[0] == 'hw':
            s = cfg[1]
            slab = torch.empty((s, M, N), device=dy.device, dtype=torch.float32)
            hconv_wgrad(dy, x, slab, s)
            reduce_slabs(slab, out, accumulate=accumulate)
            return
        tile, s = cfg
        if s == 1:
            igemm(KIND_CONV_WGRAD, 1, dy, x, out, M, N, K, Cout, 0, N, H=H, W=W, C=Cin, taps=taps, splits=1,
                  flags=FLAG_ACCUM if accumulate else 0, tile=tile)
            return
        slab = torch.empty((s, M, N), device=dy.device, dtype=torch.float32)
        igemm(KIND_CONV_WGRAD, 1, dy, x, slab, M, N, K, Cout, 0, N, H=H, W=W, C=Cin, taps=taps, splits=s,
              slab_stride=M * N, tile=tile)
        reduce_slabs(slab, out, accumulate=accumulate)
    if splits is not None:
        t0 = pick_tile(M, N)
        run((t0, splits))
        return out
    cands = _split_candidates(M, N, K) + _hconv_wgrad_candidates(Nb, H, W, Cin, Cout, taps)
    run(_tuned(('cw', M, N, K, H, W, Cin, taps, bool(accumulate)), cands, run) if not accumulate else cands[0])
    return out


def _hconv_wgrad_candidates(Nb, H, W, Cin, Cout, taps):
    if not HCONV or taps != 9 or W not in (4, 8, 16, 32) or H & (H - 1) or Cin < 64 or Cin & (Cin - 1) or Cout % 64:
        return []
    P = 64 if W == 8 else 128
    if (W == 4 and (H != 4 or (Nb * 16) % P)) or (W != 4 and (H * W) % P):
        return []  # W = 4: items of 8 whole 4x4 images
    items = Nb * H * W // P
    tiles = (Cout // 64) * (Cin // 64)
    out = []
    for blocks in (NUM_CU // 2, NUM_CU, 2 * NUM_CU):
        s = max(1, min(items, blocks // tiles))
        c = ('hw', s)
        if c not in out and s * Cout * 9 * Cin * 4 <= (256 << 20):
            out.append(c)
    return out


def hconv_wgrad(dy, x, slab, S):
    """Halo-tiled weight gradient into fp32 slabs [S][Cout][9*Cin] (sum them with reduce_slabs)."""
    Nb, H, W, Cout = dy.shape
    Cin = x.shape[-1]
    _lib.call("rk_hconv_wgrad", _p(dy), _p(x), _p(slab), Nb, H, W, Cin, Cout, int(S), _nbytes(dy), _nbytes(x), _s())
    return slab


# ----------------------------------------------------------------------------------------- dense
def linear(x: torch.Tensor, w: torch.Tensor, bias=None, *, act=ACT_NONE, slope=0.2, out_dtype=torch.bfloat16,
           out=None, alpha=1.0):
    """out = act(alpha * x @ w.T + bias).  Small-M layers (few output tiles) are autotuned between the
    direct bf16 epilogue and split-K into fp32 slabs + one fused combine/epilogue kernel."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), device=x.device, dtype=out_dtype)
    flags = (FLAG_BIAS if bias is not None else 0) | (FLAG_RELU if act == ACT_RELU else 0) | (
        FLAG_LRELU if act == ACT_LRELU else 0)
    epi = 0 if out.dtype == torch.bfloat16 else 1
    if epi == 1 and act != ACT_NONE:
        raise ValueError("fp32 dense output supports no fused activation")

    def run(cfg):
        tile, s = cfg
        if s == 1:
            igemm(KIND_DENSE, epi, x, w, out, M, N, K, x.stride(0), w.stride(0), out.stride(0), bias=bias,
                  flags=flags, slope=slope, alpha=alpha, tile=tile)
            return
        slab = torch.empty((s, M, N), device=x.device, dtype=torch.float32)
        igemm(KIND_DENSE, 1, x, w, slab, M, N, K, x.stride(0), w.stride(0), N, splits=s, slab_stride=M * N,
              tile=tile)
        _lib.call("rk_reduce_slabs_epi", _p(slab), s, M, N, _p(bias), act, float(slope), float(alpha),
                  _p(out) if epi == 0 else None, _p(out) if epi == 1 else None, out.stride(0), _s())
    t0 = pick_tile(M, N)
    cands = [(t0, 1)]
    if N % 4 == 0 and out.stride(0) % 4 == 0 and cdiv(M, 64) * cdiv(N, 64) < NUM_CU and K >= 512:
        cands += [c for c in _split_candidates(M, N, K) if c[1] > 1 and c[1] <= 16]
    run(_tuned(('dn', M, N, K, epi, act, bias is not None), cands, run) if len(cands) > 1 else cands[0])
    return out


def linear_dx(dy: torch.Tensor, w: torch.Tensor, *, gate=None, out=None):
    """dx[M][in] = dy[M][out] @ w[out][in]; optional ReLU-backward gate (dx = 0 where gate <= 0)."""
    M, Nout = dy.shape
    Nin = w.shape[1]
    if out is None:
        out = torch.empty((M, Nin), device=dy.device, dtype=torch.bfloat16)
    igemm(KIND_DENSE_DX, 0, dy, w, out, M, Nin, Nout, dy.stride(0), w.stride(0), out.stride(0), gate=gate,
          flags=FLAG_GATE if gate is not None else 0)
    return out


def linear_dw(dy: torch.Tensor, x: torch.Tensor, *, out=None, accumulate=False):
    """dw[out][in] (fp32) = dy[M][out]^T @ x[M][in]."""
    M, Nout = dy.shape
    Nin = x.shape[1]
    if out is None:
        out = torch.empty((Nout, Nin), device=dy.device, dtype=torch.float32)
    tile = pick_tile(Nout, Nin)
    s = pick_splits(Nout, Nin, M, tile)
    if s == 1:
        igemm(KIND_DENSE_DW, 1, dy, x, out, Nout, Nin, M, dy.stride(0), x.stride(0), Nin, splits=1,
              flags=FLAG_ACCUM if accumulate else 0, tile=tile)
        return out
    slab = torch.empty((s, Nout, Nin), device=dy.device, dtype=torch.float32)
    igemm(KIND_DENSE_DW, 1, dy, x, slab, Nout, Nin, M, dy.stride(0), x.stride(0), Nin, splits=s,
          slab_stride=Nout * Nin, tile=tile)
    reduce_slabs(slab, out, accumulate=accumulate)
    return out


# -------------------------------------------------------------------------------------- batchnorm
def bn_partial_rows(P: int, C: int) -> int:
    return _lib.lib().rk_bn_partial_rows(P, C)


def channel_stats(x2d: torch.Tensor):
    P, C = x2d.shape
    rows = bn_partial_rows(P, C)
    part = torch.empty((rows, 2, C), device=x2d.device, dtype=torch.float32)
    _lib.call("rk_channel_stats", _p(x2d), _p(part), P, C, rows, _s())
    return part


def rows_reduce(x2d: torch.Tensor, groups: int) -> torch.Tensor:
    """[R][W] fp32 -> [groups][W] partial sums (parallel stage 1 of a long row reduction)."""
    R = x2d.shape[0]
    W = x2d.numel() // R
    out = torch.empty((groups,) + tuple(x2d.shape[1:]), device=x2d.device, dtype=torch.float32)
    _lib.call("rk_rows_reduce", _p(x2d), R, W, groups, _p(out), _s())
    return out


def _shrink_rows(part: torch.Tensor, max_rows: int = 512) -> torch.Tensor:
    """Cut a [R][2][C] partial-stat table to <= max_rows rows with a parallel pass (~32 rows/block);
    the finalize kernels read up to ~512 rows in one pass (16 row lanes x 2 chains)."""
    R = part.shape[0]
    if R <= max_rows:
        return part
    return rows_reduce(part, min(max_rows, cdiv(R, 32)))


def bn_finalize_fwd(part, count, gamma, beta, eps, running_mean=None, running_var=None, momentum=0.1, outs=None):
    part = _shrink_rows(part)
    R, _, C = part.shape
    if outs is None:
        outs = torch.empty((4, C), device=part.device, dtype=torch.float32)
    mean, rstd, scale, shift = outs[0], outs[1], outs[2], outs[3]
    _lib.call("rk_bn_finalize_fwd", _p(part), R, C, float(count), _p(gamma), _p(beta), float(eps), _p(running_mean),
              _p(running_var), float(momentum), _p(mean), _p(rstd), _p(scale), _p(shift), _s())
    return outs


def bn_act_fwd_acc(y, acc, count, gamma, beta, eps, running_mean=None, running_var=None, momentum=0.1, *,
                   coeffs=None, pool=False, act=ACT_RELU, slope=0.2, out=None):
    """Fused BN finalize + apply from fp64 slot sums ``acc`` [SL][2][C] (conv_fwd(stats_acc=...)).
    Writes ``coeffs`` [4][C] = mean, rstd, scale, shift (for backward) and returns out."""
    Nb, H, W, C = y.shape
    if coeffs is None:
        coeffs = torch.empty((4, C), device=y.device, dtype=torch.float32)
    if out is None:
        shape = (Nb, H // 2, W // 2, C) if pool else (Nb, H, W, C)
        out = torch.empty(shape, device=y.device, dtype=torch.bfloat16)
    _lib.call("rk_bn_act_fwd_acc", _p(y), _p(acc), acc.shape[0], float(count), _p(gamma), _p(beta), float(eps),
              _p(running_mean), _p(running_var), float(momentum), _p(coeffs), _p(out), Nb, H, W, C, int(pool), act,
              float(slope), _s())
    return out, coeffs


def bn_bwd_acc(dout, y, coeffs, gamma, acc, *, pool=False, act=ACT_RELU, slope=0.2, dgamma=None, dbeta=None,
               dy=None, accumulate=False, reduced=False):
    """bn_bwd with the reduction accumulated atomically into the zeroed fp64 table ``acc`` [SL][2][C]
    and the finalize fused into the apply kernel (2 launches instead of 3).  ``reduced``: the
    producer of ``dout`` already accumulated the sums (conv_dgrad(bn_y=...)), apply only."""
    Nb, H, W, C = y.shape
    P_out = dout.numel() // C
    # no finalize reads these rows any more: size the grid for streaming only (4 pixels per lane)
    pl = 256 // min(C // 8, 256)
    rows = max(1, min(_BWD_RED_CAP, cdiv(P_out, pl * 4)))
    s = _s()
    if not reduced:
        _lib.call("rk_bn_bwd_reduce_acc", _p(dout), _p(y), _p(coeffs[2]), _p(coeffs[3]), _p(acc), acc.shape[0],
                  rows, Nb, H, W, C, int(pool), act, float(slope), s)
    coef = torch.empty((3, C), device=y.device, dtype=torch.float32)
    if dy is None:
        dy = torch.empty_like(y)
    _lib.call("rk_bn_bwd_apply_acc", _p(dout), _p(y), _p(coeffs), _p(acc), acc.shape[0], float(Nb * H * W),
              _p(gamma), _p(dgamma), _p(dbeta), _p(coef), int(accumulate), _p(dy), Nb, H, W, C, int(pool), act,
              float(slope), s)
    return dy


def bn_eval_coeffs(gamma, beta, running_mean, running_var, eps, outs=None):
    C = running_mean.numel()
    if outs is None:
        outs = torch.empty((4, C), device=running_mean.device, dtype=torch.float32)
    _lib.call("rk_bn_eval_coeffs", C, _p(gamma), _p(beta), _p(running_mean), _p(running_var), float(eps),
              _p(outs[2]), _p(outs[3]), _s())
    return outs


def bn_act_fwd(y, scale, shift, *, pool=False, act=ACT_RELU, slope=0.2, out=None):
    Nb, H, W, C = y.shape
    if out is None:
        shape = (Nb, H // 2, W // 2, C) if pool else (Nb, H, W, C)
        out = torch.empty(shape, device=y.device, dtype=torch.bfloat16)
    _lib.call("rk_bn_act_fwd", _p(y), _p(scale), _p(shift), _p(out), Nb, H, W, C, int(pool), act, float(slope), _s())
    return out


def bn_bwd(dout, y, coeffs, gamma, *, pool=False, act=ACT_RELU, slope=0.2, dgamma=None, dbeta=None, dy=None,
           accumulate=False, part=None):
    """Backward of out = pool(act(bn(y))).  coeffs = [mean, rstd, scale, shift] rows from forward.
    ``part``: precomputed (sum dz, sum dz*y) partial rows [R][2][C] — skips the reduce pass.

    Measured alternative (MI355X, VGG-small): folding this reduction into the data-gradient GEMM
    epilogue (reading y there) made the step 5% slower — +22 VGPRs in every igemm variant plus the
    y-load latency exposed at each block's tail cost more than the separate streaming pass."""
    Nb, H, W, C = y.shape
    mean, rstd, scale, shift = coeffs[0], coeffs[1], coeffs[2], coeffs[3]
    s = _s()
    if part is not None:
        part = _shrink_rows(part)
        rows = part.shape[0]
    else:
        P_out = dout.numel() // C
        rows = _lib.lib().rk_bn_bwd_rows(P_out, C)
        part = torch.empty((rows, 2, C), device=y.device, dtype=torch.float32)
        _lib.call("rk_bn_bwd_reduce", _p(dout), _p(y), _p(scale), _p(shift), _p(part), rows, Nb, H, W, C, int(pool),
                  act, float(slope), s)
    coef = torch.empty((3, C), device=y.device, dtype=torch.float32)
    _lib.call("rk_bn_finalize_bwd", _p(part), rows, C, float(Nb * H * W), _p(gamma), _p(mean), _p(rstd), _p(dgamma),
              _p(dbeta), _p(coef), int(accumulate), s)
    if dy is None:
        dy = torch.empty_like(y)
    _lib.call("rk_bn_bwd_apply", _p(dout), _p(y), _p(scale), _p(shift), _p(coef), _p(dy), Nb, H, W, C, int(pool), act,
              float(slope), s)
    return dy


# ----------------------------------------------------------------------------------- loss / optim
def softmax_xent(logits, labels, ncls, *, dlogits=None, probs=None, loss_sum=None, correct=None, counted=None,
                 ignore_index=-100, grad_scale=None):
    B = logits.shape[0]
    if grad_scale is None:
        grad_scale = 1.0 / max(1, B)
    _lib.call("rk_softmax_xent", _p(logits), logits.stride(0), _p(labels), B, ncls, ignore_index, float(grad_scale),
              _p(dlogits), 0 if dlogits is None else dlogits.stride(0), _p(probs), _p(loss_sum), _p(correct),
              _p(counted), _s())


def sgd_step(w, g, mom=None, *, wb=None, lr, momentum=0.0, weight_decay=0.0, nesterov=False, grad_scale=1.0,
             lr_tensor=None, decay_end=None, bump=None):
    """Fused SGD over a flat range; ``weight_decay`` applies to elements [0, decay_end) (default: all).
    ``bump``: int32 device counter incremented once by the launch (graph-step counters)."""
    n = w.numel()
    _lib.call("rk_sgd_step", _p(w), _p(wb), _p(g), _p(mom), n, float(lr), float(momentum),
              float(weight_decay), int(nesterov), float(grad_scale), _p(lr_tensor), n if decay_end is None else
              int(decay_end), _p(bump), _s())


def adam_step(w, g, m, v, *, wb=None, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, decoupled=False,
              step=1, grad_scale=1.0, skip_flag=None, step_tensor=None):
    """Adam/AdamW.  ``step_tensor`` (device int32, already incremented) overrides ``step`` so the
    bias corrections stay right under hipGraph replay."""
    c1 = 1.0 / (1.0 - beta1 ** step) if beta1 > 0 else 1.0
    c2 = 1.0 / (1.0 - beta2 ** step)
    _lib.call("rk_adam_step", _p(w), _p(wb), _p(g), _p(m), _p(v), w.numel(), float(lr), float(beta1), float(beta2),
              1.0 - float(beta1), 1.0 - float(beta2), float(eps), float(weight_decay), int(decoupled), float(c1),
              float(c2), float(grad_scale), _p(skip_flag), _p(step_tensor), _s())


# ---- multi-segment updates (one launch over a set of arena ranges; loss_optim.hip adam_multi_kernel)
SEG_CHUNK = 16384   # elements per block


class SegTable:
    """The device chunk table [nblk][3] (segment, begin, end) of arena ranges segs [(a, b)] (+ per-segment
    Adam parameters [nseg][4] = lr, eps, wd, 0), built once on the host.  Tables are device tensors that a
    captured graph reads by address, so callers cache them for as long as the graphs live."""

    def __init__(self, device, segs, params=None):
        rows = []
        for i, (a, b) in enumerate(segs):
            assert a % 4 == 0 and b % 4 == 0 and b > a, (a, b)
            for c in range(a, b, SEG_CHUNK):
                rows.append((i, c, min(b, c + SEG_CHUNK)))
        self.nblk = len(rows)
        self.blk = torch.tensor(rows, dtype=torch.int64).to(device)
        self.params = None if params is None else torch.tensor(params, dtype=torch.float32).to(device)


MULTISEG = os.environ.get('RAFIKI_MULTISEG', '1') != '0'


def seg_table_ok(segs) -> bool:
    """Multi-segment launches apply (RAFIKI_MULTISEG=0: one launch per range): 16-B aligned bounds."""
    return MULTISEG and bool(segs) and all(a % 4 == 0 and b % 4 == 0 and b > a for a, b in segs)


def adam_multi(w, g, m, v, table: SegTable, *, wb=None, beta1, beta2, decoupled=False, grad_scale=1.0,
               skip_flag=None, step_tensor, bump=None):
    """Adam over every segment of ``table`` (per-segment lr / eps / wd in table.params) in one launch; same
    arithmetic per element as adam_step.  ``bump``: an int32 counter the launch also advances (always)."""
    _lib.call("rk_adam_multi", _p(w), _p(wb), _p(g), _p(m), _p(v), _p(table.blk), table.nblk, _p(table.params),
              float(beta1), float(beta2), 1.0 - float(beta1), 1.0 - float(beta2), int(decoupled), float(grad_scale),
              _p(skip_flag), _p(step_tensor), _p(bump), _s())


def zero_multi(t, table: SegTable, flag=None):
    """Zero ``t`` over the table's ranges (and the int32 ``flag``) in one launch."""
    _lib.call("rk_zero_multi", _p(t), _p(table.blk), table.nblk, _p(flag), _s())


def lerp_multi(dst, src, t, table: SegTable, dst_bf16=None):
    """lerp_ (dst <- src + (dst - src) * t, + the bf16 copy) over the segments of ``table`` only."""
    _lib.call("rk_lerp_multi", _p(dst), _p(src), _p(dst_bf16), _p(table.blk), table.nblk, float(t), _s())


def nonfinite_multi(x, table: SegTable, flag, bump=None):
    """flag |= any non-finite element over the table's ranges; ``bump``: an int32 step counter the same launch
    advances (for the optimizer launch that follows)."""
    _lib.call("rk_nonfinite_multi", _p(x), _p(table.blk), table.nblk, _p(flag), _p(bump), _s())


def _capturing() -> bool:
    try:
        return torch.cuda.is_current_stream_capturing()
    except Exception:
        return False


def add_int_(t, v=1):
    _lib.call("rk_add_int", _p(t), int(v), _s())


def lerp_(dst, src, t, dst_bf16=None):
    _lib.call("rk_lerp", _p(dst), _p(src), _p(dst_bf16), dst.numel(), float(t), _s())


def zero_(t):
    """t.zero_() on the native kernel (4-byte dtypes, contiguous, 16-B aligned): keeps the per-step
    gradient-arena and flag resets out of PyTorch's fill kernels inside captured training graphs."""
    if (t.is_cuda and t.is_contiguous() and t.element_size() == 4 and t.data_ptr() % 16 == 0):
        _lib.call("rk_zero32", _p(t), t.numel(), _s())
        return t
    return t.zero_()


def nonfinite_flag(x, flag):
    _lib.call("rk_nonfinite", _p(x), x.numel(), _p(flag), _s())


# more than 16 slabs: one block-cooperative pass (rk_fold_rows) instead of rows_reduce + reduce_slabs
FOLD_ROWS = os.environ.get('RAFIKI_FOLD_ROWS', '1') != '0'


def reduce_slabs(slab, out, *, accumulate=False, scale=1.0):
    """out (+)= scale * sum_s slab[s] (slab [S][...] with out.numel() elements per slab)."""
    S = slab.shape[0]
    n = out.numel()
    if S > 16:
        if FOLD_ROWS and n % 4 == 0 and slab.is_contiguous() and out.is_contiguous():
            _lib.call("rk_fold_rows", _p(slab), S, n, _p(out), int(accumulate), float(scale), _s())
            return out
        slab = rows_reduce(slab, min(16, cdiv(S, 16)))
        S = slab.shape[0]
    _lib.call("rk_reduce_slabs", _p(slab), S, n, _p(out), int(accumulate), float(scale), _s())
    return out


def colsum(x2d, out, *, accumulate=False):
    """out[c] (+)= sum_r x2d[r, c] (bf16 in, fp32 out).  Tall inputs (R > 2048, C % 8 == 0) take the
    two-stage path: row chunks summed by ~2 blocks per CU, then folded by reduce_slabs."""
    R, Cc = x2d.shape
    ld = x2d.stride(0)
    if R > 2048 and Cc % 8 == 0 and ld % 8 == 0 and Cc % 4 == 0 and x2d.stride(1) == 1:
        chunks = max(1, min(cdiv(R, 64), cdiv(2 * NUM_CU, cdiv(Cc, 512))))
        part = torch.empty((chunks, Cc), device=x2d.device, dtype=torch.float32)
        _lib.call("rk_colsum_part", _p(x2d), R, Cc, ld, chunks, _p(part), _s())
        return reduce_slabs(part, out, accumulate=accumulate)
    _lib.call("rk_colsum", _p(x2d), R, Cc, ld, _p(out), int(accumulate), _s())
    return out


def mbstd(mode, x, a=None, b=None, *, group, segs=1, cp=None):
    """Minibatch-stddev kernels over NHWC bf16 or fp32 x [N, H, W, C] (see pggan.hip):
    mode 0 -> [N, H, W, cp] = [x, f, 0];  mode 1 -> gx from gout=a;  mode 2 -> (g_x, gg_out) from
    ggx=a and gout=b."""
    N, H, W, Cc = x.shape
    cp = cp or (a.shape[-1] if mode == 1 else b.shape[-1] if mode == 2 else Cc + 1)
    dt = x.dtype
    if dt not in (torch.bfloat16, torch.float32) or N % segs or (N // segs) % group:
        raise ValueError('mbstd: bf16 / fp32 input with N divisible by segs * group required')
    x = x.contiguous()
    a = None if a is None else a.to(dt).contiguous()
    b = None if b is None else b.to(dt).contiguous()
    out2 = None
    if mode == 0:
        out = torch.empty((N, H, W, cp), device=x.device, dtype=dt)
    else:
        out = torch.empty_like(x)
        if mode == 2:
            out2 = torch.empty((N, H, W, cp), device=x.device, dtype=dt)
    part = torch.empty((N // group) * 32, device=x.device, dtype=torch.float32)
    _lib.call("rk_mbstd" if dt == torch.bfloat16 else "rk_mbstd_f32", int(mode), _p(x), _p(a), _p(b), N, H * W, Cc,
              cp, int(group), int(segs), _p(out), _p(out2), _p(part), _s())
    return (out, out2) if mode == 2 else out


def ensemble_mean(probs, weights=None, out=None):
    """probs [W, Q, C] fp32 -> mean over W (optionally weighted)."""
    Wm = probs.shape[0]
    n = probs[0].numel()
    if out is None:
        out = torch.empty(probs.shape[1:], device=probs.device, dtype=torch.float32)
    _lib.call("rk_ensemble_mean", _p(probs), Wm, n, _p(weights), _p(out), _s())
    return out


def gather_batch(data, labels, sched, counter, out_x, out_y, *, zero=None, done=None, lr_table=None, lr_out=None):
    """out_x[b] = data[sched[*counter][b]], out_y likewise — device-side step counter (graph-safe).
    ``zero``: an fp64 tensor zeroed in the same launch; ``done`` (int32 [1], zero-initialised): the
    kernel also advances ``counter`` by one after every block has read it; ``lr_table``: lr_out[0] =
    lr_table[*counter] (a per-step learning-rate schedule inside the replayed graph)."""
    B = out_x.shape[0]
    row_bytes = data[0].numel() * data.element_size()
    if zero is not None:
        assert zero.dtype == torch.float64 and zero.is_contiguous()
    if sched.dim() != 2 or sched.shape[1] != B or sched.dtype != torch.int64:
        raise ValueError('sched must be int64 [steps, {}], got {} {}'.format(B, sched.dtype, tuple(sched.shape)))
    if lr_table is not None and lr_table.numel() < sched.shape[0]:
        raise ValueError('lr_table shorter than the schedule')
    _lib.call("rk_gather_batch", _p(data), row_bytes, _p(labels), _p(sched), _p(counter), B, _p(out_x), _p(out_y),
              _p(zero), 0 if zero is None else zero.numel(), _p(done), _p(lr_table), _p(lr_out), sched.shape[0],
              data.shape[0], _s())
    return out_x


def cast_bf16(src, dst):
    _lib.call("rk_cast_f32_bf16", _p(src), _p(dst), src.numel(), _s())
    return dst


def pack_nhwc(images, cpad=8, scale=1.0, shift=0.0, out=None):
    """uint8/float32 NCHW -> bf16 NHWC with channels padded to ``cpad``."""
    Nb, Cc, H, W = images.shape
    if out is None:
        out = torch.empty((Nb, H, W, cpad), device=images.device, dtype=torch.bfloat16)
    is_u8 = 1 if images.dtype == torch.uint8 else 0
    if not is_u8 and images.dtype != torch.float32:
        images = images.float()
    _lib.call("rk_pack_nhwc", _p(images), is_u8, Nb, Cc, H, W, cpad, float(scale), float(shift), _p(out), _s())
    return out


RNG_UNIFORM, RNG_NORMAL, RNG_RANDINT = 0, 1, 2


def philox_(out, dist, *, seed, stream_id, step=None, hi=0, a=0.0, b=1.0):
    """Fill ``out`` (fp32, or int32 for RNG_RANDINT) from the Philox4x32-10 stream
    (seed, stream_id, *step): uniform a + b*U[0,1), normal a + b*N(0,1), or randint [0, hi).
    ``step`` is a device int32 counter (graph-safe: bumping it draws new numbers per replay)."""
    want = torch.int32 if dist == RNG_RANDINT else torch.float32
    if out.dtype != want or not out.is_contiguous():
        raise ValueError('philox_: out must be contiguous %s' % want)
    _lib.call("rk_philox", _p(out), out.numel(), int(dist), int(hi), float(a), float(b),
              int(seed) & 0xFFFFFFFFFFFFFFFF, int(stream_id) & 0xFFFFFFFF, _p(step), _s())
    return out


def lrelu_pixelnorm(x, bias=None, *, slope=0.2, eps=1e-8, dz=None, out=None):
    """z = PN(lrelu(x + bias)) over the last (channel) dim of bf16 or fp32 NHWC rows; with ``dz`` the
    backward dL/dx instead (recomputes the activation from x)."""
    Cc = x.shape[-1]
    P = x.numel() // Cc
    dt = x.dtype
    if dt not in (torch.bfloat16, torch.float32) or Cc % 8 or Cc > 1024:
        raise ValueError('lrelu_pixelnorm: bf16 / fp32 rows with C % 8 == 0 and C <= 1024 required')
    x = x.contiguous()
    if dz is not None:
        dz = dz.to(dt).contiguous()
    if bias is not None:
        bias = bias.float().contiguous()
    if out is None:
        out = torch.empty_like(x)
    _lib.call("rk_lrelu_pixelnorm" if dt == torch.bfloat16 else "rk_lrelu_pixelnorm_f32", _p(x), _p(bias), _p(dz), P,
              Cc, float(slope), float(eps), _p(out), _s())
    return out


def pad8(n: int) -> int:
    return int(math.ceil(n / 8.0) * 8)
