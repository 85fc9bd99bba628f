"""Static-graph trainer for BN-ReLU conv nets (VGG-small and friends) on gfx950.

The whole training step — forward, backward, loss, optimizer — is a fixed sequence of hand-written
kernel launches over pre-planned buffers, captured once into a hipGraph (``torch.cuda.CUDAGraph``
is hipGraph on ROCm) and replayed per step.  There is no autograd tape and no per-step host work.

Precision: fp32 by default — the reference's precision (pg_gans.py:830,914; Keras fp32 in
TfVgg16.py:115-130 / TfFeedForward.py:141-164): every GEMM on v_mfma_f32_32x32x2_f32 with fp32
activations, gradients and BatchNorm (``rafiki_amd.ops.f32``: sgemm.hip + bnf.hip).  ``dtype='bf16'``
(or RAFIKI_DTYPE=bf16) opts into the bf16 MFMA engine (igemm.hip + bn.hip; fp32 master weights).

Per conv block (conv3x3 -> BatchNorm -> ReLU [-> maxpool2x2]) the step runs
  fwd : conv (BN (sum, sum^2) from the accumulators, fp64 slots) -> fused BN finalize + apply + ReLU
        (+pool)
  bwd : BN backward (reduce, or its sums already formed in the next layer's dgrad epilogue) + apply
        -> conv wgrad (split-K) -> conv dgrad as a forward conv of dy with flipped/transposed weights
        (epilogue: the input layer's ReLU mask / max-pool routing + BN-backward sums)
then one fused SGD/Adam pass over the flat parameter arena.

``bn=False`` builds conv3x3 + bias + ReLU blocks instead (Keras VGG16, TfVgg16.py:115-130, has no
BatchNorm): the conv epilogue adds the bias (and applies the ReLU when no max-pool follows); the same
backward kernels run with the constant coefficients (mean 0, rstd 1, scale 1, shift 0) and an
infinite count, which turns the BN-backward apply into the ReLU mask / max-pool routing alone and
its per-channel sum of dz into the bias gradient.

VGG-small (the BASELINE benchmark architecture; the reference's TfVgg16.py:115-130 is 48x48x3
VGG16 without BN — SURVEY §7.4 item 8 asks for an explicit definition):
  input 32x32x3 (zero-padded to 8 channels)
  [64, 64, M, 128, 128, M, 256, 256, M, 512, 512, M]  conv3x3(pad 1, no bias) + BN + ReLU, M = maxpool 2x2
  flatten 2x2x512 -> FC 512 + ReLU -> FC num_classes -> softmax cross-entropy
  = 5.75 M parameters, 0.43 GFLOP forward / image at 32x32 (~1.3 GFLOP / image / train step).

A pure-PyTorch fp32 reference of the same network (``reference_loss``) is the CPU execution path
and the numerics oracle for GPU tests.
"""
from __future__ import annotations

import math
import os
import warnings
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as TF

from ..ops import f32 as S
from ..ops import functional as F
from ..ops.graphs import capture as _capture, device_sync as _device_sync
from .flat import FlatAdam, FlatParams, FlatSGD, init_const, init_kaiming

VGG_SMALL_CFG = (64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512, 512, 'M')
DTYPES = ('fp32', 'bf16')


def default_dtype() -> str:
    """Compute dtype of the native engines: fp32 (the reference's precision) unless RAFIKI_DTYPE=bf16."""
    d = os.environ.get('RAFIKI_DTYPE', 'fp32').lower()
    d = {'float32': 'fp32', 'f32': 'fp32', 'bfloat16': 'bf16'}.get(d, d)
    if d not in DTYPES:
        raise ValueError('RAFIKI_DTYPE must be one of {}'.format(DTYPES))
    return d


def _pad8(n):
    return (n + 7) // 8 * 8


def _pad4(n):
    return (n + 3) // 4 * 4


def _is_pow2(n):
    return n > 0 and (n & (n - 1)) == 0


class _BF16Storage(torch.autograd.Function):
    """Identity whose forward value AND backward gradient are rounded to bf16 — models a tensor
    the engine stores in bf16 (the activation and its gradient both live in bf16 buffers)."""

    @staticmethod
    def forward(ctx, t):
        return t.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


class _BF16Grad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t):
        return t.clone()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


def _bf16_storage(t):
    return _BF16Storage.apply(t)


def _bf16_grad(t):
    return _BF16Grad.apply(t)


def _init_fc(fan_in, rows_real, cols_real, gain=math.sqrt(2.0)):
    """Kaiming-normal over the real [rows_real, cols_real] block; padded rows/cols stay zero forever
    (zero weights + zero bias -> zero activations -> zero gradients under SGD/Adam)."""
    std = gain / math.sqrt(max(1, fan_in))

    def f(t, g):
        t.zero_()
        t[:rows_real, :cols_real].normal_(0.0, std, generator=g)
    return f


class ConvNetEngine:
    def __init__(self, num_classes: int = 10, in_channels: int = 3, image_size: int = 32,
                 cfg: Sequence = VGG_SMALL_CFG, fc_dims: Sequence[int] = (512,), device='cuda', seed: int = 0,
                 bn_eps: float = 1e-5, bn_momentum: float = 0.1, optimizer: str = 'sgd', lr: float = 0.05,
                 momentum: float = 0.9, weight_decay: float = 5e-4, nesterov: bool = True,
                 betas=(0.9, 0.999), input_bn: bool = False, dtype: Optional[str] = None, bn: bool = True):
        self.device = torch.device(device)
        self.dtype = dtype or default_dtype()
        if self.dtype not in DTYPES:
            raise ValueError('dtype must be one of {}'.format(DTYPES))
        self.f32 = self.dtype == 'fp32'
        self.act_dtype = torch.float32 if self.f32 else torch.bfloat16
        self.num_classes, self.in_channels, self.image_size = num_classes, in_channels, image_size
        self.flat_input = not any(v != 'M' for v in cfg)
        # fp32 K-inner operands move 16-B = 4-channel chunks, bf16 ones 8-channel chunks; with the
        # Winograd kernels (C % 8 == 0) the fp32 stem is padded to 8 channels too, so the first conv
        # and its weight gradient get the fused Winograd candidates (zero channels, zero weights)
        self.cin_p = ((_pad8(in_channels) if S.WINO and not self.flat_input else _pad4(in_channels)) if self.f32
                      else _pad8(in_channels))
        self.ncls_p = _pad8(num_classes)
        self.bn_eps, self.bn_momentum = bn_eps, bn_momentum
        self.bn = bool(bn)
        if not self.bn and not self.f32:
            raise ValueError('bn=False (conv + bias + ReLU blocks) runs on the fp32 engine')
        self.input_bn = bool(input_bn)
        if self.input_bn and not self.flat_input:
            raise ValueError('input_bn is for fully-connected nets (no conv blocks)')
        # any image size: power-of-two maps use the shift-decoded (and LDS-DMA) gather, others the
        # reciprocal-decoded register-staged gather (VGG16 at 48x48: 48/24/12/6/3)
        flat = FlatParams(self.device, seed, compute_bf16=not self.f32)
        self.blocks = []  # (name, cin, cout, pool, H_in)
        cin, hw, i = self.cin_p, image_size, 0
        real_cin = in_channels
        for j, v in enumerate(cfg):
            if v == 'M':
                continue
            pool = j + 1 < len(cfg) and cfg[j + 1] == 'M'
            name = 'conv{}'.format(i)
            zero = slice(real_cin, None) if real_cin < cin else None
            flat.add(name + '.w', (v, 3, 3, cin), init_kaiming(9 * real_cin, zero_in_slice=zero))
            if self.bn:
                flat.add(name + '.gamma', (v,), init_const(1.0), decay=False)
                flat.add(name + '.beta', (v,), init_const(0.0), decay=False)
            else:
                flat.add(name + '.b', (v,), init_const(0.0), decay=False)
            self.blocks.append((name, cin, v, pool, hw))
            if pool:
                hw //= 2
            cin, real_cin, i = v, v, i + 1
        if hw < 1:
            raise ValueError('too many pooling stages for image_size {}'.format(image_size))
        self.feat_hw = hw
        if self.flat_input:
            self.in_dim = image_size * image_size * in_channels
            self.feat_dim = _pad4(self.in_dim) if self.f32 else _pad8(self.in_dim)
            real_in = self.in_dim
        else:
            self.feat_dim = hw * hw * cin
            real_in = self.feat_dim
        if self.input_bn:
            flat.add('in_bn.gamma', (self.feat_dim,), init_const(1.0), decay=False)
            flat.add('in_bn.beta', (self.feat_dim,), init_const(0.0), decay=False)
        self.fcs = []  # (name, d_in_padded, d_padded, d_real)
        d_in, d_in_real = self.feat_dim, real_in
        for k, d in enumerate(fc_dims):
            dp = _pad8(d)
            flat.add('fc{}.w'.format(k), (dp, d_in), _init_fc(d_in_real, d, d_in_real))
            flat.add('fc{}.b'.format(k), (dp,), init_const(0.0), decay=False)
            self.fcs.append(('fc{}'.format(k), d_in, dp, d))
            d_in, d_in_real = dp, d
        flat.add('out.w', (self.ncls_p, d_in), _init_fc(d_in_real, num_classes, d_in_real, gain=1.0))
        flat.add('out.b', (self.ncls_p,), init_const(0.0), decay=False)
        self.flat = flat.build()
        self.d_last = d_in
        self.d_last_real = d_in_real
        C = (sum(b[2] for b in self.blocks) if self.bn else 0) + (self.feat_dim if self.input_bn else 0)
        self.running = torch.zeros((2, C), dtype=torch.float32, device=self.device)
        self.running[1].fill_(1.0)
        self._roff = []
        off = 0
        for b in self.blocks:
            self._roff.append(off)
            off += b[2] if self.bn else 0
        self._in_roff = off
        # bn=False: per block the constant BN-backward coefficients [4][C] (mean 0, rstd 1, scale 1, shift 0)
        # and a unit gamma, built once (no allocation inside a captured step)
        self._nobn_coeffs = [] if self.bn else [
            torch.tensor([[0.0], [1.0], [1.0], [0.0]]).expand(4, b[2]).contiguous().to(self.device)
            for b in self.blocks]
        self._ones = None if self.bn else torch.ones(max([b[2] for b in self.blocks] or [1]), device=self.device)
        if optimizer == 'adam':
            self.opt = FlatAdam(self.flat, lr, betas=betas, weight_decay=weight_decay, decoupled=True)
        else:
            self.opt = FlatSGD(self.flat, lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov)
        self.loss_sum = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.correct = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.seen = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._graph = None
        self._graph_batch = None
        self._static_x = self._static_y = None
        self._eval_coeffs = None
        self._eval_graphs = {}

    # ------------------------------------------------------------------------------- helpers
    def running_stats(self, bi):
        if bi == 'in':
            o, c = self._in_roff, self.feat_dim
        else:
            o, c = self._roff[bi], self.blocks[bi][2]
        return self.running[0, o:o + c], self.running[1, o:o + c]

    def _block_coeffs(self, bi):
        """bn=False: the [4][C] constant coefficients of block ``bi``."""
        return self._nobn_coeffs[bi]

    def real_param_count(self) -> int:
        """Trainable parameters of the network as defined (channel / class padding excluded)."""
        n, real_cin = 0, self.in_channels
        for (_, cin, cout, _, _) in self.blocks:
            n += cout * 9 * real_cin + 2 * cout if self.bn else cout * 9 * real_cin + cout
            real_cin = cout
        d_in = self.in_dim if self.flat_input else self.feat_hw * self.feat_hw * real_cin
        if self.input_bn:
            n += 2 * d_in
        for (_, _, _, d) in self.fcs:
            n += d * d_in + d
            d_in = d
        return n + self.num_classes * d_in + self.num_classes

    def train_flops_per_image(self) -> float:
        """Model FLOPs of one training image as a direct computation: forward + data gradient +
        weight gradient of every layer, minus the stem's data gradient (never computed).  The
        Winograd kernels execute 4/9 of the 3x3 conv MACs counted here."""
        stem = 2.0 * self.blocks[0][4] ** 2 * self.blocks[0][2] * 9 * self.blocks[0][1] if self.blocks else 0.0
        return 3.0 * self.flops_per_image() - stem

    def flops_per_image(self) -> float:
        """Forward MACs*2 of the conv + FC layers (train step = 3x)."""
        fl = 0.0
        for (_, cin, cout, _, hw) in self.blocks:
            fl += 2.0 * hw * hw * cout * 9 * cin
        for (_, di, do, _) in self.fcs:
            fl += 2.0 * di * do
        fl += 2.0 * self.d_last * self.num_classes
        return fl

    # Weight gradients run in stream order.  Overlapping them on a side stream was measured slower on
    # VGG-small every time it was tried: bf16 1.161 -> 1.289 ms, fp32 2.27 -> 2.46 ms, and with the
    # round-4 kernels 5-6% (profiles/step_switches_ab_r4.txt): the concurrent GEMMs and split-K slab
    # traffic interfere, and the LDS-heavy Winograd kernels leave no room for a second workgroup.
    _acc_zeroed_by_prologue = False  # set while a scheduled step's gather kernel zeroes the BN tables
    # the dgrad epilogue forms the ReLU mask / max-pool routing and BN-backward sums of the layer below
    # (FLAG_BNB / FLAG_BNP), so its BN backward is a single apply pass
    fuse_bn_dgrad = True
    fuse_bn_pool = True
    # data gradients as forward convs of dy with flipped/transposed weights (F.ConvWT, one transpose
    # launch per step): the forward kernels' K-inner weight operand and tiles are the faster ones
    dgrad_wt = True
    # fp32 path: the classifier head (output layer, softmax-xent, its gradients) as two fused launches
    fused_head = True

    def reset_metrics(self):
        self.loss_sum.zero_()
        self.correct.zero_()
        self.seen.zero_()

    # ----------------------------------------------------------------------------- GPU train
    def _train_step_gpu(self, x, labels):
        self._fwd_bwd_gpu(x, labels)
        self.opt.step()

    def _fwd_bwd_gpu(self, x, labels):
        """x: [B, H, W, cin_p] NHWC (engine dtype), labels: [B] int32. Everything stays on-device."""
        if self.f32:
            return self._fwd_bwd_gpu_f32(x, labels)
        fl = self.flat
        B = x.shape[0]
        acts = [x]
        saved = []
        h = x
        accs = self._bn_accumulators() if self._use_bn_acc() else None
        if accs is not None and not self._acc_zeroed_by_prologue:
            self._bn_acc_flat.zero_()  # one memset node for every layer's fp64 statistic slots
        for bi, (name, cin, cout, pool, hw) in enumerate(self.blocks):
            rm, rv = self.running_stats(bi)
            if accs is not None:
                y, _ = F.conv_fwd(h, fl.wb(name + '.w'), stats_acc=accs[bi][0])
                h, coeffs = F.bn_act_fwd_acc(y, accs[bi][0], B * hw * hw, fl.w(name + '.gamma'), fl.w(name + '.beta'),
                                             self.bn_eps, rm, rv, self.bn_momentum, pool=pool, act=F.ACT_RELU)
            else:
                y, stats = F.conv_fwd(h, fl.wb(name + '.w'), want_stats=True)
                coeffs = F.bn_finalize_fwd(stats, B * hw * hw, fl.w(name + '.gamma'), fl.w(name + '.beta'),
                                           self.bn_eps, rm, rv, self.bn_momentum)
                h = F.bn_act_fwd(y, coeffs[2], coeffs[3], pool=pool, act=F.ACT_RELU)
            saved.append((y, coeffs))
            acts.append(h)
        in_saved = None
        if self.input_bn:
            raw = h.reshape(B, 1, 1, self.feat_dim)
            stats = F.channel_stats(raw.view(B, self.feat_dim))
            rm, rv = self.running_stats('in')
            coeffs = F.bn_finalize_fwd(stats, B, fl.w('in_bn.gamma'), fl.w('in_bn.beta'), self.bn_eps, rm, rv,
                                       self.bn_momentum)
            h = F.bn_act_fwd(raw, coeffs[2], coeffs[3], pool=False, act=F.ACT_NONE)
            in_saved = (raw, coeffs)
        feat = h.reshape(B, self.feat_dim)
        fc_in = [feat]
        z = feat
        for (name, di, do, _) in self.fcs:
            z = F.linear(z, fl.wb(name + '.w'), fl.w(name + '.b'), act=F.ACT_RELU)
            fc_in.append(z)
        logits = F.linear(z, fl.wb('out.w'), fl.w('out.b'), out_dtype=torch.float32)
        dlogits = torch.empty((B, self.ncls_p), dtype=torch.bfloat16, device=self.device)
        F.softmax_xent(logits, labels, self.num_classes, dlogits=dlogits, loss_sum=self.loss_sum,
                       correct=self.correct, counted=self.seen)
        # ---- backward
        F.linear_dw(dlogits, fc_in[-1], out=fl.g('out.w'))
        F.colsum(dlogits, fl.g('out.b'))
        d = dlogits
        wname = 'out'
        for k in range(len(self.fcs) - 1, -1, -1):
            name = self.fcs[k][0]
            d = F.linear_dx(d, fl.wb(wname + '.w'), gate=fc_in[k + 1])
            F.linear_dw(d, fc_in[k], out=fl.g(name + '.w'))
            F.colsum(d, fl.g(name + '.b'))
            wname = name
        if not self.blocks and not self.input_bn:
            return
        d = F.linear_dx(d, fl.wb(wname + '.w'))
        if self.input_bn:
            raw, coeffs = in_saved
            F.bn_bwd(d.view(B, 1, 1, self.feat_dim), raw, coeffs, fl.w('in_bn.gamma'), pool=False, act=F.ACT_NONE,
                     dgamma=fl.g('in_bn.gamma'), dbeta=fl.g('in_bn.beta'))
            return
        d = d.view(B, self.feat_hw, self.feat_hw, -1)
        reduced = False
        wt = self._conv_wt() if self.dgrad_wt else None
        if wt is not None:
            wt.refresh()  # one launch: flipped/transposed bf16 weights of every dgrad layer
        for bi in range(len(self.blocks) - 1, -1, -1):
            name, cin, cout, pool, hw = self.blocks[bi]
            y, coeffs = saved[bi]
            if accs is not None:
                dy = F.bn_bwd_acc(d, y, coeffs, fl.w(name + '.gamma'), accs[bi][1], pool=pool, act=F.ACT_RELU,
                                  dgamma=fl.g(name + '.gamma'), dbeta=fl.g(name + '.beta'), reduced=reduced)
            else:
                dy = F.bn_bwd(d, y, coeffs, fl.w(name + '.gamma'), pool=pool, act=F.ACT_RELU,
                              dgamma=fl.g(name + '.gamma'), dbeta=fl.g(name + '.beta'))
            F.conv_wgrad(dy, acts[bi], out=fl.g(name + '.w').view(cout, -1))
            if bi > 0:
                # into a pool-free BN+ReLU block: its ReLU mask and BN-backward sums ride in the
                # dgrad epilogue (FLAG_BNB), so its bn_bwd_acc is a single apply pass
                py, pco = saved[bi - 1]
                reduced = accs is not None and self.fuse_bn_dgrad and not self.blocks[bi - 1][3]
                # into a BN+ReLU+max-pool block (power-of-two geometry): its BN-backward sums ride in
                # the dgrad epilogue too (FLAG_BNP, argmax routing from the pre-BN output)
                pool_fused = (accs is not None and self.fuse_bn_dgrad and wt is not None and self.blocks[bi - 1][3]
                              and self.fuse_bn_pool and not (hw & (hw - 1)) and self.blocks[bi - 1][4] == 2 * hw)
                if wt is not None:
                    if reduced:
                        d = F.conv_dgrad_t(dy, wt.view(bi - 1), bn_y=py, bn_coeffs=pco, bn_acc=accs[bi - 1][1])
                    elif pool_fused:
                        d = F.conv_dgrad_t(dy, wt.view(bi - 1), bn_pool_y=py, bn_coeffs=pco,
                                           bn_acc=accs[bi - 1][1])
                        reduced = True
                    else:
                        d = F.conv_dgrad_t(dy, wt.view(bi - 1))
                elif reduced:
                    d = F.conv_dgrad(dy, fl.wb(name + '.w'), bn_y=py, bn_coeffs=pco, bn_acc=accs[bi - 1][1])
                else:
                    d = F.conv_dgrad(dy, fl.wb(name + '.w'))

    # ------------------------------------------------------------------------- fp32 train
    def _bn_on_load(self, bi, B, ww):
        """Block bi's BN + ReLU is applied by its consumer's loads (normalise-on-load): a non-pooled block
        followed by another conv block whose F(4x4) kernels (blocked weights) take pre-BN input."""
        if ww is None or bi + 1 >= len(self.blocks):
            return False
        name, cin, cout, pool, hw = self.blocks[bi]
        nxt = self.blocks[bi + 1]
        return (not pool and nxt[1] == cout and nxt[4] == hw and ww.lazy('u4b', bi + 1) is not None
                and S.bn_on_load_ok(B, hw, hw, cout, nxt[2]))

    def _fwd_bwd_gpu_f32(self, x, labels):
        """The fp32 step: x [B, H, W, cin_p] fp32 NHWC, labels [B] int32; every GEMM on the f32 MFMA."""
        fl = self.flat
        B = x.shape[0]
        accs = self._bn_accumulators()
        if not self._acc_zeroed_by_prologue:
            self._bn_acc_flat.zero_()  # one memset node for every layer's fp64 statistic slots
        ww = self._wino_train()
        if ww is not None:
            ww.refresh()   # one launch per family: the live Winograd-domain weight sets of every block
        acts, saved, h = [x], [], x
        pros, hpro = [None], None   # normalise-on-load: the BN coeffs acts[bi] still needs applied (or None)
        for bi, (name, cin, cout, pool, hw) in enumerate(self.blocks):
            wk = dict(wino=ww.lazy('u2', bi) if ww is not None else None,
                      wino4=ww.lazy('u4', bi) if ww is not None else None,
                      wino4p=ww.lazy('u4p', bi) if ww is not None else None,
                      wino4b=ww.lazy('u4b', bi) if ww is not None else None)
            if not self.bn:
                # conv + bias (+ ReLU in the epilogue when no pool follows; the saved post-ReLU output
                # gives the same mask); a pooled block runs ReLU + max-pool in the eval-BN kernel
                c = self._block_coeffs(bi)
                y = S.conv_fwd(h, fl.w(name + '.w'), bias=fl.w(name + '.b'),
                               act=F.ACT_NONE if pool else F.ACT_RELU, **wk)
                h = S.bn_eval(y, c[2], c[3], pool=True, act=F.ACT_RELU) if pool else y
                saved.append((y, c))
                acts.append(h)
                continue
            rm, rv = self.running_stats(bi)
            y = S.conv_fwd(h, fl.w(name + '.w'), stats_acc=accs[bi][0], pro=hpro, **wk)
            if self._bn_on_load(bi, B, ww):
                # BN + ReLU never materialised: the next conv's forward and weight-gradient kernels apply
                # scale / shift + ReLU to y as they load it (bn_finalize = the coefficient half, one block)
                coeffs = S.bn_finalize(y, accs[bi][0], B * hw * hw, fl.w(name + '.gamma'), fl.w(name + '.beta'),
                                       self.bn_eps, rm, rv, self.bn_momentum)
                h, hpro = y, coeffs
            else:
                h, coeffs = S.bn_fwd(y, accs[bi][0], B * hw * hw, fl.w(name + '.gamma'), fl.w(name + '.beta'),
                                     self.bn_eps, rm, rv, self.bn_momentum, pool=pool, act=F.ACT_RELU)
                hpro = None
            saved.append((y, coeffs))
            acts.append(h)
            pros.append(hpro)
        in_saved = None
        if self.input_bn:
            raw = h.reshape(B, 1, 1, self.feat_dim)
            acc_f, acc_b = accs[-1]
            S.col_stats(raw.view(B, self.feat_dim), acc_f)
            rm, rv = self.running_stats('in')
            h, coeffs = S.bn_fwd(raw, acc_f, B, fl.w('in_bn.gamma'), fl.w('in_bn.beta'), self.bn_eps, rm, rv,
                                 self.bn_momentum, pool=False, act=F.ACT_NONE)
            in_saved = (raw, coeffs)
        feat = h.reshape(B, self.feat_dim)
        fc_in = [feat]
        z = feat
        for (name, di, do, _) in self.fcs:
            z = S.linear(z, fl.w(name + '.w'), fl.w(name + '.b'), act=F.ACT_RELU)
            fc_in.append(z)
        dlogits = torch.empty((B, self.ncls_p), dtype=torch.float32, device=self.device)
        k_top = len(self.fcs) - 1
        if self.fused_head and S.head_ok(self.ncls_p, self.d_last):
            # output layer + softmax-xent + d(hidden) in one launch, the output weight / bias and the top
            # hidden layer's bias gradients in a second (csrc/kernels/head.hip)
            gated = k_top >= 0
            dz = torch.empty((B, self.d_last), dtype=torch.float32, device=self.device)
            S.head_fwd_bwd(z, fl.w('out.w'), fl.w('out.b'), labels, self.num_classes, dlogits=dlogits, dz=dz,
                           gated=gated, loss_sum=self.loss_sum, correct=self.correct, counted=self.seen)
            S.head_dw(z, dlogits, dz, dw=fl.g('out.w'), db=fl.g('out.b'),
                      dbh=fl.g(self.fcs[k_top][0] + '.b') if gated else None)
            d = dz
            if gated:
                S.linear_dw(d, fc_in[k_top], out=fl.g(self.fcs[k_top][0] + '.w'))
                wname, k_top = self.fcs[k_top][0], k_top - 1
            else:
                wname = None   # dz is already the gradient of the flattened features
        else:
            logits = S.linear(z, fl.w('out.w'), fl.w('out.b'))
            S.softmax_xent(logits, labels, self.num_classes, dlogits=dlogits, loss_sum=self.loss_sum,
                           correct=self.correct, counted=self.seen)
            # ---- backward
            S.linear_dw(dlogits, fc_in[-1], out=fl.g('out.w'))
            S.colsum(dlogits, fl.g('out.b'))
            d, wname = dlogits, 'out'
        for k in range(k_top, -1, -1):
            name = self.fcs[k][0]
            d = S.linear_dx(d, fl.w(wname + '.w'), gate=fc_in[k + 1])
            S.linear_dw(d, fc_in[k], out=fl.g(name + '.w'))
            S.colsum(d, fl.g(name + '.b'))
            wname = name
        if not self.blocks and not self.input_bn:
            return
        if wname is not None:
            d = S.linear_dx(d, fl.w(wname + '.w'))
        if self.input_bn:
            raw, coeffs = in_saved
            S.bn_bwd(d.view(B, 1, 1, self.feat_dim), raw, coeffs, fl.w('in_bn.gamma'), accs[-1][1], pool=False,
                     act=F.ACT_NONE, dgamma=fl.g('in_bn.gamma'), dbeta=fl.g('in_bn.beta'))
            return
        d = d.view(B, self.feat_hw, self.feat_hw, -1)
        wt = self._conv_wt()
        if wt is not None:
            # flipped/transposed fp32 weights of every dgrad layer, refreshed (one launch) on first use
            wt.begin_step()
        reduced = False
        for bi in range(len(self.blocks) - 1, -1, -1):
            name, cin, cout, pool, hw = self.blocks[bi]
            y, coeffs = saved[bi]
            if self.bn:
                dy = S.bn_bwd(d, y, coeffs, fl.w(name + '.gamma'), accs[bi][1], pool=pool, act=F.ACT_RELU,
                              dgamma=fl.g(name + '.gamma'), dbeta=fl.g(name + '.beta'), reduced=reduced)
            else:   # ReLU mask / pool routing only; sum dz -> the bias gradient
                dy = S.bn_bwd(d, y, coeffs, self._ones[:cout], accs[bi][1], pool=pool, act=F.ACT_RELU,
                              dbeta=fl.g(name + '.b'), reduced=reduced, count=float('inf'))
            S.conv_wgrad(dy, acts[bi], out=fl.g(name + '.w').view(cout, -1),
                         xpro=pros[bi] if self.bn else None)
            if bi == 0:
                break
            py, pco = saved[bi - 1]
            pname, pcin, pcout, ppool, phw = self.blocks[bi - 1]
            wu = ww.lazy('ut2', bi) if ww is not None else None
            wu4 = ww.lazy('ut4', bi) if ww is not None else None
            wu4p = ww.lazy('ut4p', bi) if ww is not None else None
            wu4b = ww.lazy('ut4b', bi) if ww is not None else None
            wl = wt.lazy(bi - 1)
            dk = dict(wino=wu, wino4=wu4, cin=cin, wino4p=wu4p, wino4b=wu4b)
            if not ppool:
                # the input block is BN+ReLU: its mask and BN-backward sums ride in this dgrad's epilogue
                d = S.conv_dgrad(dy, wl, bnb=(py, pco, accs[bi - 1][1]), **dk)
                reduced = True
            elif phw == 2 * hw and not (hw & (hw - 1)):
                # BN+ReLU+max-pool input (even power-of-two geometry): pool routing + sums in the epilogue
                d = S.conv_dgrad(dy, wl, bnp=(py, pco, accs[bi - 1][1]), **dk)
                reduced = True
            else:
                d = S.conv_dgrad(dy, wl, **dk)
                reduced = False
        if ww is not None:
            ww.end_step()   # only the Winograd sets the tuned convs use are transformed from now on

    def _wino_train(self):
        """WinoWeights over blocks 1.. (fp32 path): the fused F(2x2,3x3) and F(4x4,3x3) kernels become
        autotune candidates of every forward / data-gradient conv they fit (RAFIKI_WINOGRAD=0 turns
        both off, RAFIKI_WINOGRAD4=0 the F(4x4) ones)."""
        if not (self.f32 and S.WINO and self.blocks and self.device.type == 'cuda'):
            return None
        ww = getattr(self, '_ww', None)
        if ww is None:
            fl = self.flat
            ww = self._ww = S.WinoWeights(fl.master, [fl.w(b[0] + '.w') for b in self.blocks],
                                          hw=[b[4] for b in self.blocks])
        return ww

    def _conv_wt(self):
        """ConvWT over the weights of blocks 1.. (block 0 has no data gradient), built once."""
        wt = getattr(self, '_wt', None)
        if wt is None and len(self.blocks) > 1 and self.f32:
            fl = self.flat
            wt = self._wt = S.SConvWT(fl.master, [fl.w(b[0] + '.w') for b in self.blocks[1:]])
        if wt is None and len(self.blocks) > 1:
            fl = self.flat
            ws = [fl.wb(b[0] + '.w') for b in self.blocks[1:]]
            if all(w.shape[0] % 8 == 0 and (w.numel() // (9 * w.shape[0])) % 8 == 0 for w in ws):
                wt = self._wt = F.ConvWT(fl.bf16, ws)
        return wt

    def _use_bn_acc(self) -> bool:
        if self.f32:
            return True
        return F.BN_ATOMIC and all(b[2] <= 1024 and b[2] % 8 == 0 for b in self.blocks)

    def _bn_accumulators(self):
        """Per conv block (and, fp32 path, the input BN): (forward, backward) fp64 slot tables
        [SL][2][C], views of one flat buffer so a single memset per step zeroes them all."""
        accs = getattr(self, '_bn_accs', None)
        if accs is None:
            chans = [b[2] for b in self.blocks] + ([self.feat_dim] if self.input_bn and self.f32 else [])
            sizes = [F.bn_slots(c) * 2 * c for c in chans]
            flat = torch.zeros(2 * sum(sizes), dtype=torch.float64, device=self.device)
            accs, off = [], 0
            for c, n in zip(chans, sizes):
                shape = (F.bn_slots(c), 2, c)
                accs.append((flat[off:off + n].view(shape), flat[off + n:off + 2 * n].view(shape)))
                off += 2 * n
            self._bn_acc_flat, self._bn_accs = flat, accs
        return accs

    # ------------------------------------------------------------------------ reference path
    def reference_loss(self, x_nhwc: torch.Tensor, labels: torch.Tensor, params: Optional[dict] = None,
                       training=True, update_running=False, emulate_bf16=False):
        """Pure PyTorch fp32 forward of the same network (NCHW internally). Returns (loss, logits).

        ``emulate_bf16`` rounds (straight-through) at exactly the points where the GPU engine stores
        bf16: weights, conv outputs, block outputs and FC hidden activations — the tight oracle for
        the kernel path (max-pool argmax routing then agrees with the kernels' bf16 values)."""
        fl = self.flat
        P = params if params is not None else {n: fl.w(n) for n in fl.names()}
        ste = (lambda t: t + (t.bfloat16().float() - t).detach())
        # emulate_bf16='fwd': round the stored forward values only (gradients stay fp32) — the second
        # placement of the same bf16 storage, used to measure the oracle's own rounding noise floor
        rnd = ste if emulate_bf16 == 'fwd' else _bf16_storage if emulate_bf16 else (lambda t: t)
        rndw = ste if emulate_bf16 else (lambda t: t)
        # fp64 inputs keep fp64 (the fp32 kernels' numerics oracle); everything else runs in fp32
        up = (lambda t: t) if x_nhwc.dtype == torch.float64 else (lambda t: t.float())
        h = up(x_nhwc).permute(0, 3, 1, 2) if x_nhwc.dim() == 4 else up(x_nhwc)
        for bi, (name, cin, cout, pool, hw) in enumerate(self.blocks):
            w = rndw(P[name + '.w']).permute(0, 3, 1, 2)
            if not self.bn:
                h = torch.relu(TF.conv2d(h, w, P[name + '.b'], padding=1))
                h = rnd(TF.max_pool2d(h, 2) if pool else h)
                continue
            h = rnd(TF.conv2d(h, w, padding=1))
            rm, rv = self.running_stats(bi)
            if not update_running:
                rm, rv = rm.to(h), rv.to(h)
            if training:
                h = TF.batch_norm(h, rm if update_running else None, rv if update_running else None,
                                  P[name + '.gamma'], P[name + '.beta'], training=True,
                                  momentum=self.bn_momentum, eps=self.bn_eps)
            else:
                h = TF.batch_norm(h, rm, rv, P[name + '.gamma'], P[name + '.beta'], training=False,
                                  eps=self.bn_eps)
            h = torch.relu(h)
            if pool:
                h = TF.max_pool2d(h, 2)
            h = rnd(h)
        if self.flat_input:
            h = up(x_nhwc).reshape(x_nhwc.shape[0], -1)
            if self.input_bn:
                rm, rv = self.running_stats('in')
                if not update_running:
                    rm, rv = rm.to(h), rv.to(h)
                if training:
                    h = TF.batch_norm(h, rm if update_running else None, rv if update_running else None,
                                      P['in_bn.gamma'], P['in_bn.beta'], training=True, momentum=self.bn_momentum,
                                      eps=self.bn_eps)
                else:
                    h = TF.batch_norm(h, rm, rv, P['in_bn.gamma'], P['in_bn.beta'], training=False, eps=self.bn_eps)
                h = rnd(h)
        else:
            h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)
        for (name, di, do, _) in self.fcs:
            h = rnd(torch.relu(h @ rndw(P[name + '.w']).t() + P[name + '.b']))
        logits = (h @ rndw(P['out.w']).t() + P['out.b'])[:, :self.num_classes]
        logits = _bf16_grad(logits) if emulate_bf16 and emulate_bf16 != 'fwd' else logits
        loss = TF.cross_entropy(logits, labels.long()) if labels is not None else None
        return loss, logits

    def _train_step_cpu(self, x, labels):
        self._fwd_bwd_cpu(x, labels)
        self.opt.step()

    def _fwd_bwd_cpu(self, x, labels):
        fl = self.flat
        params = {n: fl.w(n).detach().clone().requires_grad_(True) for n in fl.names()}
        loss, logits = self.reference_loss(x, labels, params, training=True, update_running=True)
        grads = torch.autograd.grad(loss, [params[n] for n in fl.names()])
        for n, g in zip(fl.names(), grads):
            fl.g(n).copy_(g)
        with torch.no_grad():
            self.loss_sum += loss.detach() * x.shape[0]
            self.correct += (logits.argmax(1) == labels.long()).sum().to(torch.int32)
            self.seen += x.shape[0]

    # --------------------------------------------------------------------------- public API
    def forward_backward(self, x, labels):
        """Fill the flat grad buffer (no optimizer step)."""
        if self.device.type == 'cuda':
            self._fwd_bwd_gpu(x, labels)
        else:
            self._fwd_bwd_cpu(x, labels)

    def train_step(self, x, labels):
        if self.device.type == 'cuda':
            self._train_step_gpu(x, labels)
        else:
            self._train_step_cpu(x, labels)

    def capture(self, batch_size: int, warmup: int = 2):
        """Capture one training step on static input buffers into a hipGraph."""
        if self.device.type != 'cuda':
            return None
        self._static_x = torch.zeros(self.input_shape(batch_size), dtype=self.act_dtype, device=self.device)
        self._static_y = torch.zeros((batch_size,), dtype=torch.int32, device=self.device)
        # warm the allocator / library outside capture; these steps use zero inputs and are
        # undone by restoring the parameter state afterwards.
        snap = [self.flat.master.clone(), self.running.clone()]
        opt_state = [t.clone() for t in self._opt_tensors()]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._train_step_gpu(self._static_x, self._static_y)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with _capture(g):
            self._train_step_gpu(self._static_x, self._static_y)
        _device_sync(self.device)
        self.flat.master.copy_(snap[0])
        self.flat.sync_bf16()
        self.running.copy_(snap[1])
        for t, v in zip(self._opt_tensors(), opt_state):
            t.copy_(v)
        self.reset_metrics()
        self._graph, self._graph_batch = g, batch_size
        return g

    def capture_scheduled(self, data, labels, max_steps: int, batch_size: int, warmup: int = 2):
        """Capture gather + train step + counter increment into ONE hipGraph: every replay trains on
        rows ``sched[ctr]`` of the device-resident dataset and advances ``ctr`` on the device, so a
        training loop is just ``set_schedule(idx); for _: replay()`` — no per-step copies."""
        if self.device.type != 'cuda':
            raise RuntimeError('capture_scheduled needs a GPU')
        self._data, self._labels = data, labels
        self._sched = torch.zeros((max_steps, batch_size), dtype=torch.int64, device=self.device)
        self._ctr = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._static_x = torch.zeros(self.input_shape(batch_size), dtype=self.act_dtype, device=self.device)
        self._static_y = torch.zeros((batch_size,), dtype=torch.int32, device=self.device)

        self._done = torch.zeros(1, dtype=torch.int32, device=self.device)
        # per-step LR multipliers read by the prologue into the optimizer's device scalar (SGD)
        self._lr_table = torch.ones(max_steps, dtype=torch.float32, device=self.device)
        lr_out = getattr(self.opt, 'lr_scale', None)
        accs = self._bn_accumulators() if self._use_bn_acc() else None

        # the step counter advances inside the step's last kernel (SGD) or, for other optimizers, in
        # the prologue once every gather block has read it
        opt_bumps = isinstance(self.opt, FlatSGD)

        def body():
            # one prologue launch: gather + zero the BN slot tables (+ counter)
            F.gather_batch(self._data, self._labels, self._sched, self._ctr, self._static_x, self._static_y,
                           zero=self._bn_acc_flat if accs is not None else None,
                           done=None if opt_bumps else self._done,
                           lr_table=self._lr_table if lr_out is not None else None, lr_out=lr_out)
            self._acc_zeroed_by_prologue = accs is not None
            if opt_bumps:
                self.opt.bump = self._ctr
            try:
                self._train_step_gpu(self._static_x, self._static_y)
            finally:
                self._acc_zeroed_by_prologue = False
                if opt_bumps:
                    self.opt.bump = None

        snap = [self.flat.master.clone(), self.running.clone()]
        opt_state = [t.clone() for t in self._opt_tensors()]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                body()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with _capture(g):
            body()
        _device_sync(self.device)
        self.flat.master.copy_(snap[0])
        self.flat.sync_bf16()
        self.running.copy_(snap[1])
        for t, v in zip(self._opt_tensors(), opt_state):
            t.copy_(v)
        self._ctr.zero_()
        self.reset_metrics()
        self._sched_graph = g
        return g

    def set_schedule(self, idx, start: int = 0, lr_scales=None):
        """idx: [steps, B] row indices (device) -> schedule buffer; the next replay uses row ``start``.
        ``lr_scales`` [steps] (optional): the optimizer's LR multiplier of each step."""
        self._sched[:idx.shape[0]].copy_(idx)
        self._ctr.fill_(start)
        if lr_scales is not None:
            self._lr_table[:len(lr_scales)].copy_(torch.as_tensor(lr_scales, dtype=torch.float32))

    def replay(self):
        self._sched_graph.replay()

    def _opt_tensors(self):
        o = self.opt
        if isinstance(o, FlatAdam):
            return [o.m, o.v, o.t]
        return [o.mom] if o.mom is not None else []

    def step_graph(self, x, labels):
        """Copy a batch into the static buffers and replay the captured step."""
        self._static_x.copy_(x)
        self._static_y.copy_(labels)
        self._graph.replay()

    # ------------------------------------------------------------------------------ inputs
    def input_shape(self, batch):
        if self.flat_input:
            return (batch, self.feat_dim)
        return (batch, self.image_size, self.image_size, self.cin_p)

    def prepare_inputs(self, images, scale=1.0 / 127.5, shift=-1.0):
        """uint8 images [N, H, W] or [N, H, W, C] (host numpy / torch) -> device tensor in this engine's
        input layout (bf16 NHWC with channels padded to 8, or flat [N, D] padded to 8).  The
        normalisation (x*scale+shift) and packing run in one gfx950 kernel on the GPU."""
        if isinstance(images, np.ndarray) and not images.flags.writeable:
            with warnings.catch_warnings():   # shared read-only dataset cache arrays: only read here
                warnings.simplefilter('ignore', UserWarning)
                t = torch.as_tensor(images)
        else:
            t = torch.as_tensor(images)
        if t.dim() == 3:
            t = t.unsqueeze(-1)
        N = t.shape[0]
        if self.device.type != 'cuda':
            x = t.float() * scale + shift
            if self.flat_input:
                out = torch.zeros((N, self.feat_dim))
                out[:, :self.in_dim] = x.reshape(N, -1)
                return out
            out = torch.zeros((N, self.image_size, self.image_size, self.cin_p))
            out[..., :x.shape[-1]] = x
            return out
        t = t.to(self.device, non_blocking=True)
        pack = S.pack_nhwc if self.f32 else F.pack_nhwc
        if self.flat_input:
            nchw = t.reshape(N, -1, 1, 1)
            return pack(nchw.contiguous(), self.feat_dim, scale, shift).view(N, self.feat_dim)
        if self.f32:   # the fp32 pack kernel reads NHWC directly (no transposing copy)
            return S.pack_nhwc(t.contiguous(), self.cin_p, scale, shift, nhwc=True)
        nchw = t.permute(0, 3, 1, 2).contiguous()
        return pack(nchw, self.cin_p, scale, shift)

    # ------------------------------------------------------------------------------ inference
    def prepare_eval(self):
        """Fold BN running stats into per-channel scale/shift (inference coefficients)."""
        fl = self.flat
        coeffs = []
        items = [(bi, b[0]) for bi, b in enumerate(self.blocks)]
        if self.input_bn:
            items.append(('in', 'in_bn'))
        for bi, name in items:
            if bi != 'in' and not self.bn:   # conv bias as the shift (the eval conv runs without bias)
                b = fl.w(name + '.b').detach()
                coeffs.append(torch.stack([torch.zeros_like(b), torch.ones_like(b), torch.ones_like(b), b.clone()]))
                continue
            rm, rv = self.running_stats(bi)
            if self.device.type == 'cuda':
                c = F.bn_eval_coeffs(fl.w(name + '.gamma'), fl.w(name + '.beta'), rm, rv, self.bn_eps)
            else:
                r = torch.rsqrt(rv + self.bn_eps)
                sc = fl.w(name + '.gamma') * r
                c = torch.stack([rm, r, sc, fl.w(name + '.beta') - rm * sc])
            coeffs.append(c)
        self._eval_coeffs = coeffs
        from ..ops.graphs import quiesced
        with quiesced():
            self._eval_graphs = {}
        self._eval_wino = None
        if self.f32 and S.WINO and self.blocks and self.device.type == 'cuda':
            self._eval_wino = S.WinoWeights(fl.master, [fl.w(b[0] + '.w') for b in self.blocks], dgrad=False,
                                            hw=[b[4] for b in self.blocks])
            self._eval_wino.refresh()
        return coeffs

    @torch.no_grad()
    def _forward_eval_gpu_f32(self, x, out_probs):
        fl = self.flat
        h = x
        B = x.shape[0]
        ew = getattr(self, '_eval_wino', None)
        for bi, (name, cin, cout, pool, hw) in enumerate(self.blocks):
            y = S.conv_fwd(h, fl.w(name + '.w'), wino=ew.u(bi) if ew is not None else None,
                           wino4=ew.u4(bi) if ew is not None else None, wino4p=ew.u4p(bi) if ew is not None else None)
            c = self._eval_coeffs[bi]
            h = S.bn_eval(y, c[2], c[3], pool=pool, act=F.ACT_RELU)
        if self.input_bn:
            c = self._eval_coeffs[-1]
            h = S.bn_eval(h.reshape(B, 1, 1, self.feat_dim), c[2], c[3], pool=False, act=F.ACT_NONE)
        z = h.reshape(B, self.feat_dim)
        for (name, di, do, _) in self.fcs:
            z = S.linear(z, fl.w(name + '.w'), fl.w(name + '.b'), act=F.ACT_RELU)
        logits = S.linear(z, fl.w('out.w'), fl.w('out.b'))
        S.softmax_xent(logits, None, self.num_classes, probs=out_probs)
        return out_probs

    @torch.no_grad()
    def _forward_eval_gpu(self, x, out_probs):
        if self.f32:
            return self._forward_eval_gpu_f32(x, out_probs)
        fl = self.flat
        h = x
        B = x.shape[0]
        for bi, (name, cin, cout, pool, hw) in enumerate(self.blocks):
            y = F.conv_fwd(h, fl.wb(name + '.w'))
            c = self._eval_coeffs[bi]
            h = F.bn_act_fwd(y, c[2], c[3], pool=pool, act=F.ACT_RELU)
        if self.input_bn:
            c = self._eval_coeffs[-1]
            h = F.bn_act_fwd(h.reshape(B, 1, 1, self.feat_dim), c[2], c[3], pool=False, act=F.ACT_NONE)
        z = h.reshape(B, self.feat_dim)
        for (name, di, do, _) in self.fcs:
            z = F.linear(z, fl.wb(name + '.w'), fl.w(name + '.b'), act=F.ACT_RELU)
        logits = F.linear(z, fl.wb('out.w'), fl.w('out.b'), out_dtype=torch.float32)
        F.softmax_xent(logits, None, self.num_classes, probs=out_probs)
        return out_probs

    @torch.no_grad()
    def forward_eval(self, x, out_probs=None):
        """x: engine input layout -> probabilities [B, num_classes] fp32."""
        if self.device.type != 'cuda':
            _, logits = self.reference_loss(x, None, training=False)
            return torch.softmax(logits.float(), 1)
        if self._eval_coeffs is None:
            self.prepare_eval()
        if out_probs is None:
            out_probs = torch.empty((x.shape[0], self.num_classes), dtype=torch.float32, device=self.device)
        return self._forward_eval_gpu(x, out_probs)

    EVAL_BUCKETS = (1, 8, 32, 64, 128, 256, 512)

    @torch.no_grad()
    def forward_eval_graphed(self, x):
        """Inference through hipGraph-captured forwards, one per batch-size bucket (captured lazily,
        reused for every later request of that bucket).  Returns a view [B, num_classes]."""
        if self.device.type != 'cuda':
            return self.forward_eval(x)
        if self._eval_coeffs is None:
            self.prepare_eval()
        B = x.shape[0]
        bucket = next((b for b in self.EVAL_BUCKETS if b >= B), None)
        if bucket is None:  # larger than the biggest bucket: chunk it (each chunk's result is a view
            # of the bucket's static output buffer, so copy it out before the next replay reuses it)
            outs = [self.forward_eval_graphed(x[i:i + self.EVAL_BUCKETS[-1]]).clone() for i in
                    range(0, B, self.EVAL_BUCKETS[-1])]
            return torch.cat(outs)
        ent = self._eval_graphs.get(bucket)
        if ent is None:
            sx = torch.zeros(self.input_shape(bucket), dtype=self.act_dtype, device=self.device)
            so = torch.empty((bucket, self.num_classes), dtype=torch.float32, device=self.device)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._forward_eval_gpu(sx, so)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with _capture(g):
                self._forward_eval_gpu(sx, so)
            ent = self._eval_graphs[bucket] = (g, sx, so)
        g, sx, so = ent
        sx[:B].copy_(x)
        if B < bucket:
            sx[B:].zero_()
        g.replay()
        return so[:B]

    def resident_bytes(self):
        ew = getattr(self, '_eval_wino', None)
        extra = ew.buf.numel() * 4 if ew is not None else 0
        return self.flat.total * (4 + (0 if self.f32 else 2) + 4) + self.running.numel() * 4 + extra

    def release_training(self):
        """Drop what only training needs — the captured step graphs (and with them their private
        activation pools), static batch buffers, the step schedule and the optimizer state — so a
        finished trial can stay resident in HBM for serving at its inference footprint."""
        from ..ops.graphs import quiesced
        with quiesced():
            for a in ('_graph', '_sched_graph', '_static_x', '_static_y', '_sched', '_ctr', '_ww', '_wt'):
                if hasattr(self, a):
                    setattr(self, a, None)
            self.opt = None

    # ---------------------------------------------------------------------------- state I/O
    def state_dict(self):
        d = self.flat.state_dict()
        d['__running__'] = self.running.detach().cpu().numpy().copy()
        return d

    def load_state_dict(self, d):
        self.flat.load_state_dict(d)
        if '__running__' in d:
            self.running.copy_(torch.as_tensor(d['__running__']))
        self._eval_coeffs = None


class GroupedConvNets:
    """k trained fp32 ConvNetEngines of ONE architecture evaluated as a single network: every layer
    of all k models is one grouped kernel (ops.f32 *_grp) over weights stacked [k, ...] at build
    time, so an ensemble forward costs the launches of one model with k x the work per launch (the
    small-batch serving latency of k models ~ that of one).  The request batch is packed once and
    shared by every group's first layer.  Inference only (BN folded into scale / shift)."""

    POOL_EPILOGUE_MIN_PIXELS = 2048   # batch x map pixels from which a pooled block uses the pooled epilogue

    @staticmethod
    def arch_key(eng):
        if not isinstance(eng, ConvNetEngine) or not eng.f32 or eng.input_bn or eng.flat_input:
            return None
        return (tuple(eng.blocks), tuple(eng.fcs), eng.num_classes, eng.ncls_p, eng.cin_p, eng.image_size,
                eng.feat_dim, str(eng.device), eng.bn)

    def __init__(self, engines):
        keys = {self.arch_key(e) for e in engines}
        if len(keys) != 1 or None in keys:
            raise ValueError('GroupedConvNets needs fp32 conv engines of one architecture')
        self.engines = list(engines)
        e0 = self.engines[0]
        self.k, self.proto = len(engines), e0
        self.device = e0.device
        self.refresh()

    @torch.no_grad()
    def refresh(self):
        """(Re)stack the current weights and folded BN coefficients of the k engines."""
        e0 = self.proto
        for e in self.engines:
            if e._eval_coeffs is None:
                e.prepare_eval()

        def stack(fn):
            return torch.stack([fn(e) for e in self.engines]).contiguous()
        self.conv_w = [stack(lambda e, n=name: e.flat.w(n + '.w').reshape(e.flat.w(n + '.w').shape[0], -1))
                       for (name, _, _, _, _) in e0.blocks]
        self.scale = [stack(lambda e, i=bi: e._eval_coeffs[i][2]) for bi in range(len(e0.blocks))]
        self.shift = [stack(lambda e, i=bi: e._eval_coeffs[i][3]) for bi in range(len(e0.blocks))]
        # the eval BN folded into the conv (weights x scale per output channel, shift as the bias, ReLU in
        # the conv epilogue): no separate BN pass over the activation.  A pooled block folds too when a
        # fused Winograd kernel takes its shape (its epilogue writes the 2x2 max-pool); otherwise it keeps
        # its one BN + ReLU + 2x2 max pass
        self.folded = [not b[3] for b in e0.blocks]
        # Winograd-domain weights [k, 16, Cout, Cin] of the 3x3 layers the fused kernel takes
        self.conv_u = [None] * len(e0.blocks)
        self.conv_u4 = [None] * len(e0.blocks)   # F(4x4) sets [k, 36, Cout, Cin] (maps in multiples of 4)
        if S.WINO and self.device.type == 'cuda':
            for bi, (name, cin, cout, pool, hw) in enumerate(e0.blocks):
                w = self.conv_w[bi]
                if w.shape[2] % 9 == 0 and (w.shape[2] // 9) % 8 == 0 and hw % 2 == 0:
                    self.conv_u[bi] = torch.stack([S.wino_u(w[g]) for g in range(self.k)]).contiguous()
                    if S.WINO4 and hw % 4 == 0:
                        self.conv_u4[bi] = torch.stack([S.wino4_u(w[g]) for g in range(self.k)]).contiguous()
        # (the Winograd sets above are rebuilt from the folded weights below)
        for bi, (name, cin, cout, pool, hw) in enumerate(e0.blocks):
            if pool and self.device.type == 'cuda' and S.conv_fwd_grp_pool_ok(hw, hw, cin, self.conv_u[bi],
                                                                             self.conv_u4[bi]):
                self.folded[bi] = True
                self._unit = getattr(self, '_unit', {})
                self._unit[cout] = (torch.ones((self.k, cout), device=self.device),
                                    torch.zeros((self.k, cout), device=self.device))
            if not self.folded[bi]:
                continue
            w = self.conv_w[bi] = (self.conv_w[bi] * self.scale[bi].unsqueeze(-1)).contiguous()
            if self.conv_u[bi] is not None:
                self.conv_u[bi] = torch.stack([S.wino_u(w[g]) for g in range(self.k)]).contiguous()
            if self.conv_u4[bi] is not None:
                self.conv_u4[bi] = torch.stack([S.wino4_u(w[g]) for g in range(self.k)]).contiguous()
        self.fc_w = [stack(lambda e, n=name: e.flat.w(n + '.w')) for (name, _, _, _) in e0.fcs]
        self.fc_b = [stack(lambda e, n=name: e.flat.w(n + '.b')) for (name, _, _, _) in e0.fcs]
        self.out_w = stack(lambda e: e.flat.w('out.w'))
        self.out_b = stack(lambda e: e.flat.w('out.b'))

    @torch.no_grad()
    def forward_into(self, x, out_probs):
        """x: the engines' input layout [B, H, W, cin_p] fp32 (shared); out_probs [k, B, num_classes]."""
        e0, k = self.proto, self.k
        B = x.shape[0]
        h = x
        for bi, (name, cin, cout, pool, hw) in enumerate(e0.blocks):
            if self.folded[bi] and pool and B * hw * hw < self.POOL_EPILOGUE_MIN_PIXELS:
                # small batches: the unrestricted conv candidates + one ReLU / max pass beat the pooled epilogue
                # (batch 1: 0.23 vs 0.29 ms for the four-model forward)
                y = S.conv_fwd_grp(h, self.conv_w[bi], bias=self.shift[bi], wino=self.conv_u[bi],
                                   wino4=self.conv_u4[bi])
                one, zero = self._unit[cout]
                h = S.bn_eval_grp(y, one, zero, pool=True, act=F.ACT_RELU)
                continue
            if self.folded[bi]:
                h = S.conv_fwd_grp(h, self.conv_w[bi], bias=self.shift[bi], act=F.ACT_RELU, wino=self.conv_u[bi],
                                   wino4=self.conv_u4[bi], pool=pool)
                continue
            y = S.conv_fwd_grp(h, self.conv_w[bi], wino=self.conv_u[bi], wino4=self.conv_u4[bi])
            h = S.bn_eval_grp(y, self.scale[bi], self.shift[bi], pool=pool, act=F.ACT_RELU)
        z = h.reshape(k, B, e0.feat_dim)
        for i in range(len(e0.fcs)):
            z = S.linear_grp(z, self.fc_w[i], self.fc_b[i], act=F.ACT_RELU)
        logits = S.linear_grp(z, self.out_w, self.out_b)
        S.softmax_xent(logits.view(k * B, -1), None, e0.num_classes, probs=out_probs.view(k * B, -1))
        return out_probs
