"""Flat parameter arena + fused optimizers.

All trainable parameters of a model live in ONE fp32 master buffer (plus, for the opt-in bf16
compute path, a bf16 compute copy) and an fp32 gradient buffer of the same layout.  Consequences, all deliberate for MI355X:
  * the optimizer is one streaming kernel over the whole model (multi-tensor for free, §2.4 K9),
    and it writes the bf16 copy the next forward reads — no separate cast pass;
  * data-parallel gradient all-reduce is a handful of large contiguous RCCL buckets over the flat
    grad buffer (``rafiki_amd.parallel.grad_bucket``) instead of one call per tensor
    (pg_gans.py:1164-1171 does one NCCL all-sum per variable);
  * a trial's full state is three tensors: cheap to snapshot into the per-GPU HBM param cache.

Parameters with weight decay are laid out first so decay / no-decay are two contiguous ranges.
Offsets are aligned to 64 elements (256-B fp32 / 128-B bf16 lines).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import torch

from ..ops import functional as F

ALIGN = 64


@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    init: Callable[[torch.Tensor, torch.Generator], None]
    decay: bool = True
    offset: int = 0
    lr_mult: float = 1.0  # per-parameter LR multiplier (PG-GAN equalized learning rate)

    @property
    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n


def _align(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


def init_normal(std):
    def f(t, g):
        t.normal_(0.0, std, generator=g)
    return f


def init_const(v):
    def f(t, g):
        t.fill_(v)
    return f


def init_kaiming(fan_in, gain=math.sqrt(2.0), zero_in_slice=None):
    std = gain / math.sqrt(max(1, fan_in))

    def f(t, g):
        t.normal_(0.0, std, generator=g)
        if zero_in_slice is not None:
            t[..., zero_in_slice] = 0.0
    return f


class FlatParams:
    def __init__(self, device, seed: int = 0, compute_bf16: bool = True):
        self.device = torch.device(device)
        self.seed = seed
        self.compute_bf16 = bool(compute_bf16)  # fp32 engines read the master weights directly
        self.specs: List[ParamSpec] = []
        self._by_name: Dict[str, ParamSpec] = {}
        self.master = self.bf16 = self.grad = None
        self.total = 0
        self.decay_end = 0

    def add(self, name, shape, init, decay=True, lr_mult=1.0):
        spec = ParamSpec(name, tuple(int(s) for s in shape), init, decay, lr_mult=float(lr_mult))
        self.specs.append(spec)
        self._by_name[name] = spec
        return spec

    def build(self):
        ordered = [s for s in self.specs if s.decay] + [s for s in self.specs if not s.decay]
        off = 0
        for s in ordered:
            s.offset = off
            off += _align(s.numel)
            if s.decay:
                self.decay_end = off
        self.total = _align(max(off, ALIGN))
        dev = self.device
        self.master = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=dev)
        g = torch.Generator(device='cpu')
        g.manual_seed(self.seed)
        host = torch.zeros(self.total, dtype=torch.float32)
        for s in ordered:
            t = torch.empty(s.shape, dtype=torch.float32)
            s.init(t, g)
            host[s.offset:s.offset + s.numel] = t.reshape(-1)
        self.master.copy_(host)
        self.bf16 = self.master.to(torch.bfloat16) if self.compute_bf16 else None
        return self

    # views
    def _view(self, buf, name):
        s = self._by_name[name]
        return buf[s.offset:s.offset + s.numel].view(s.shape)

    def w(self, name):
        return self._view(self.master, name)

    def wb(self, name):
        if self.bf16 is None:
            raise RuntimeError('fp32 arena has no bf16 compute copy')
        return self._view(self.bf16, name)

    def g(self, name):
        return self._view(self.grad, name)

    def names(self):
        return [s.name for s in self.specs]

    def segments(self, weight_decay: float = 0.0):
        """Contiguous arena ranges [(a, b, wd, lr_mult)] of equal decay and LR multiplier."""
        segs = []
        for s in sorted(self.specs, key=lambda s: s.offset):
            wd = weight_decay if s.decay else 0.0
            a, b = s.offset, s.offset + _align(s.numel)
            if segs and segs[-1][2] == wd and segs[-1][3] == s.lr_mult and segs[-1][1] == a:
                segs[-1] = (segs[-1][0], b, wd, s.lr_mult)
            else:
                segs.append((a, b, wd, s.lr_mult))
        if segs:
            segs[-1] = (segs[-1][0], self.total, segs[-1][2], segs[-1][3])
        return segs

    def param_ranges(self):
        return [(s.offset, s.numel) for s in self.specs]

    def ranges_of(self, names):
        """Merged contiguous arena ranges [(a, b)] (aligned extents) of the named parameters."""
        rs = sorted((self._by_name[n].offset, self._by_name[n].offset + _align(self._by_name[n].numel)) for n in names)
        out = []
        for a, b in rs:
            if out and out[-1][1] == a:
                out[-1] = (out[-1][0], b)
            else:
                out.append((a, b))
        return out

    def num_params(self):
        return sum(s.numel for s in self.specs)

    def sync_bf16(self):
        if self.bf16 is not None:
            self.bf16.copy_(self.master)

    def state_dict(self):
        """{name: float32 numpy array} — picklable, device-independent."""
        return {s.name: self.w(s.name).detach().float().cpu().numpy().copy() for s in self.specs}

    def load_state_dict(self, d):
        for s in self.specs:
            if s.name not in d:
                continue
            v = torch.as_tensor(d[s.name], dtype=torch.float32)
            if v.numel() != math.prod(s.shape) and v.dim() == len(s.shape) and \
                    tuple(v.shape[:-1]) == tuple(s.shape[:-1]):
                # a conv stem saved with another input-channel padding (4 vs 8 fp32 channels,
                # RAFIKI_WINOGRAD on/off, or a bf16 save): the padding channels are zero either way
                out = torch.zeros(s.shape, dtype=torch.float32)
                c = min(v.shape[-1], s.shape[-1])
                if v.shape[-1] > c and bool(v[..., c:].any()):
                    raise ValueError('{}: cannot drop non-zero input channels {}..{}'.format(s.name, c, v.shape[-1]))
                out[..., :c] = v[..., :c]
                v = out
            self.w(s.name).copy_(v.reshape(s.shape))
        self.sync_bf16()


class FlatSGD:
    """SGD (+momentum, +nesterov, decoupled-range weight decay) over a FlatParams arena."""

    def __init__(self, flat: FlatParams, lr, momentum=0.9, weight_decay=5e-4, nesterov=True):
        self.flat, self.lr, self.momentum, self.wd, self.nesterov = flat, float(lr), float(momentum), float(
            weight_decay), bool(nesterov)
        self.mom = torch.zeros_like(flat.master) if momentum > 0 else None
        # device-side LR multiplier: schedules change it without re-capturing the graph
        self.lr_scale = torch.ones(1, dtype=torch.float32, device=flat.device)
        self.bump: Optional[torch.Tensor] = None  # int32 device counter the step kernel advances

    def step(self):
        f = self.flat
        if f.device.type == 'cuda':
            # one launch: decayed parameters come first in the arena, wd applies below decay_end
            F.sgd_step(f.master, f.grad, self.mom, wb=f.bf16, lr=self.lr, momentum=self.momentum,
                       weight_decay=self.wd, nesterov=self.nesterov, lr_tensor=self.lr_scale,
                       decay_end=f.decay_end, bump=self.bump)
            return
        # CPU reference path (same math as sgd_kernel)
        lr = self.lr * float(self.lr_scale.item())
        wd = torch.zeros_like(f.master)
        wd[:f.decay_end] = self.wd
        g = f.grad + wd * f.master
        if self.mom is not None:
            self.mom.mul_(self.momentum).add_(g)
            d = g + self.momentum * self.mom if self.nesterov else self.mom
        else:
            d = g
        f.master.sub_(lr * d)
        f.sync_bf16()

    def set_lr_scale(self, s):
        self.lr_scale.fill_(float(s))


class FlatAdam:
    """Adam / AdamW over a FlatParams arena; step counter lives on the device (graph-safe)."""

    def __init__(self, flat: FlatParams, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False):
        self.flat, self.lr, self.b1, self.b2, self.eps = flat, float(lr), float(betas[0]), float(betas[1]), float(eps)
        self.wd, self.decoupled = float(weight_decay), bool(decoupled)
        self.m = torch.zeros_like(flat.master)
        self.v = torch.zeros_like(flat.master)
        self.t = torch.zeros(1, dtype=torch.int32, device=flat.device)
        self.skip_flag: Optional[torch.Tensor] = None

    def reset_state(self):
        self.m.zero_()
        self.v.zero_()
        self.t.zero_()

    def step(self, live=None, bumped=False, bump=None):
        """``live``: arena ranges [(a, b)] to update (None: the whole arena).  Only exact for ranges
        left out whose gradient AND first moment are zero (an untouched parameter with beta1 = 0, or
        one never touched since reset_state): Adam then leaves the weight unchanged.  ``bumped``: the
        device step counter was already advanced for this step (by the finite-check launch).  ``bump``:
        another int32 device counter to advance in the same launch when the step runs as one
        multi-segment launch; returns True when it did (the caller advances it otherwise)."""
        f = self.flat
        # Equalized LR (pg_gans.py:1006-1013) is applied by re-parameterisation: the arena holds the
        # EFFECTIVE weights c*w, stepped with lr*c and eps*c — algebraically identical to Adam on w.
        segs = f.segments(self.wd)
        if live is not None:
            segs = [(max(a, c), min(b, d), wd, mult) for a, b, wd, mult in segs for c, d in live
                    if min(b, d) > max(a, c)]
        if f.device.type == 'cuda':
            if not bumped:
                F.add_int_(self.t, 1)
            if live is not None and len(segs) > 1 and F.seg_table_ok([(a, b) for a, b, _, _ in segs]):
                # every live segment in one launch (per-segment lr / eps / wd from a cached device table)
                key = (tuple(segs), self.lr, self.eps)
                tabs = self.__dict__.setdefault('_seg_tables', {})
                tab = tabs.get(key)
                if tab is None and not F._capturing():
                    tab = tabs[key] = F.SegTable(f.device, [(a, b) for a, b, _, _ in segs],
                                                 [(self.lr * mult, self.eps * mult, wd, 0.0) for _, _, wd, mult in segs])
                if tab is not None:
                    F.adam_multi(f.master, f.grad, self.m, self.v, tab, wb=f.bf16, beta1=self.b1, beta2=self.b2,
                                 decoupled=self.decoupled, step_tensor=self.t, skip_flag=self.skip_flag, bump=bump)
                    return bump is not None
            for a, b, wd, mult in segs:
                if b > a:
                    F.adam_step(f.master[a:b], f.grad[a:b], self.m[a:b], self.v[a:b],
                                wb=None if f.bf16 is None else f.bf16[a:b],
                                lr=self.lr * mult, beta1=self.b1, beta2=self.b2, eps=self.eps * mult,
                                weight_decay=wd, decoupled=self.decoupled, step_tensor=self.t,
                                skip_flag=self.skip_flag)
            return
        if self.skip_flag is not None and int(self.skip_flag.item()) != 0:
            return
        self.t += 1
        t = int(self.t.item())
        c1 = 1.0 / (1.0 - self.b1 ** t) if self.b1 > 0 else 1.0
        c2 = 1.0 / (1.0 - self.b2 ** t)
        for a, b, wd, mult in segs:
            w, gr, m, v = f.master[a:b], f.grad[a:b], self.m[a:b], self.v[a:b]
            g = gr if self.decoupled else gr + wd * w
            m.mul_(self.b1).add_((1 - self.b1) * g)
            v.mul_(self.b2).add_((1 - self.b2) * g * g)
            upd = (m * c1) / ((v * c2).sqrt() + self.eps * mult)
            if self.decoupled:
                upd = upd + wd * w
            w.sub_(self.lr * mult * upd)
        f.sync_bf16()
