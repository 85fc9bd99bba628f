"""Bucketed gradient all-reduce over a flat fp32 gradient arena (overlapped with an eager backward).

Replaces the reference's per-variable ``tf.contrib.nccl.all_sum`` (pg_gans.py:1164-1171: ~25 calls
per network per step, several of them on tiny bias tensors) with a handful of large RCCL
all-reduces over contiguous slices of the FlatParams gradient buffer:

* buckets are contiguous ranges of the arena in REVERSE parameter order (backward produces the
  last layers' gradients first), each ~``bucket_mb`` MiB.  On xGMI a ring all-reduce is bound by
  one 153 GB/s link per hop, so a 16-32 MiB bucket amortises the ~10-20 us launch/latency to <5%
  while still giving several buckets to overlap with the remaining backward;
* a ``register_post_accumulate_grad_hook`` per parameter counts arrivals; when a bucket is
  complete its all-reduce is launched asynchronously (``async_op=True``) on RCCL's internal
  stream, overlapping the rest of the backward;
* ``finish()`` launches whatever did not fire (parameters outside the active graph, e.g. PG-GAN
  blocks above the current level of detail, still hold zeros and must be reduced to keep the
  replicas identical) and waits, then applies the 1/world mean (pg_gans.py:1175-1179);
* ``traced(grads_fn, tag)`` is the form for CAPTURED data-parallel rounds (GraphedRounds'
  segments): while the gradient segment runs (eagerly, the first time a round shape is seen) every
  gradient contribution is observed (ops.autograd.GRAD_WATCH for the in-place weight-gradient
  writes, the post-accumulate hooks for autograd's), and the reduce segment that follows the
  segment's replays all-reduces only the buckets that received any — PG-GAN blocks above the
  current level of detail hold zero gradient on every rank, so their sum is zero and they are not
  reduced at all (two thirds of the arena at the reference schedule's 4x4 LOD).  Starting each
  bucket's reduce while the replay still runs the earlier layers' backward would need an event
  recorded inside the capture that a stream outside the graph can wait on; HIP refuses external
  event records during stream capture (hipErrorInvalidValue, ROCm 7.2; torch refuses
  Event(external=True) on ROCm), and an internal event does not order the other stream, so the
  reduce runs between the replays.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops import autograd as _ag


class FlatGradAllReduce:
    def __init__(self, grad: torch.Tensor, param_ranges: Sequence[Tuple[int, int]], params: Sequence[torch.Tensor],
                 world_size: int, group=None, bucket_mb: Optional[float] = None, overlap: bool = True,
                 force: bool = False):
        """grad: flat fp32 buffer; param_ranges[i] = (offset, numel) of params[i] inside it.
        bucket_mb: default NodeConfig.grad_bucket_mb (RAFIKI_GRAD_BUCKET_MB).  force: issue the
        collectives even for a 1-rank group (single-GPU rehearsal of the DP path)."""
        if bucket_mb is None:
            from ..config import NodeConfig
            bucket_mb = NodeConfig().grad_bucket_mb
        self.bucket_mb = float(bucket_mb)
        self.grad = grad
        self.world = int(world_size)
        self.group = group
        self.force = bool(force)
        self.overlap = overlap and (self.world > 1 or self.force)
        cap = max(1, int(bucket_mb * (1 << 20)) // 4)
        order = sorted(range(len(param_ranges)), key=lambda i: -param_ranges[i][0])  # reverse arena order
        self.buckets: List[Tuple[int, int]] = []
        self.bucket_of: List[int] = [0] * len(param_ranges)
        self.bucket_size: List[int] = []
        lo = hi = None
        count = 0
        for i in order:
            off, n = param_ranges[i]
            if hi is None:
                lo, hi, count = off, off + n, 0
            elif (hi - min(lo, off)) > cap:
                self.buckets.append((lo, hi))
                self.bucket_size.append(count)
                lo, hi, count = off, off + n, 0
            lo = min(lo, off)
            hi = max(hi, off + n)
            self.bucket_of[i] = len(self.buckets)
            count += 1
        if hi is not None:
            self.buckets.append((lo, hi))
            self.bucket_size.append(count)
        # close gaps: buckets cover the arena exactly (alignment padding included) so finish() reduces
        # everything once
        total = grad.numel()
        bounds = sorted(self.buckets)
        fixed = []
        prev = 0
        for a, b in bounds:
            fixed.append((prev, b))
            prev = b
        if fixed:
            fixed[-1] = (fixed[-1][0], total)
        remap = {old: new for old, new in zip(bounds, fixed)}
        self.buckets = [remap[b] for b in self.buckets]
        self._pending = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._works = []
        self._hooks = []
        self._idx = {id(p): i for i, p in enumerate(params)}
        self._note = None        # the gradient-contribution observer of a traced segment (traced())
        self._plans = {}
        self._side = None
        if self.overlap:
            for i, p in enumerate(params):
                if p.requires_grad:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))

    def _make_hook(self, i):
        def hook(p):
            note = self._note
            if note is not None:
                note(p)
            if not self.active:
                return
            b = self.bucket_of[i]
            self._pending[b] += 1
            if self._pending[b] == self.bucket_size[b] and not self._launched[b]:
                self._launch(b)
        return hook

    active = False

    def begin(self):
        """Call before the backward whose gradients should be reduced."""
        self._pending = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._works = []
        self.active = self.overlap

    def _launch(self, b):
        a, e = self.buckets[b]
        self._launched[b] = True
        self._works.append(dist.all_reduce(self.grad[a:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def finish(self, average: bool = True):
        self.active = False
        if self.world <= 1 and not self.force:
            return
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        for w in self._works:
            w.wait()
        self._works = []
        if average:
            self.grad.mul_(1.0 / self.world)

    def allreduce_now(self):
        """Launch every bucket's all-reduce (sum) and make the current stream wait for them — the eager
        collective segment between two captured segments of a data-parallel round (the 1/world mean is
        ``scale()``, the first op of the next captured segment)."""
        if self.world <= 1 and not self.force:
            return
        works = [dist.all_reduce(self.grad[a:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                 for a, e in self.buckets]
        for w in works:
            w.wait()

    # ------------------------------------------------------------ traced reduce of a captured segment
    def traced(self, grads_fn, tag):
        """(grads, reduce) callables for a data-parallel round's segments: ``grads`` runs ``grads_fn``
        recording which buckets its gradient contributions land in; ``reduce`` all-reduces (sum) those
        buckets, in the order the backward completed them, and makes the current stream wait for
        them.  ``tag`` names the segment across rounds (its graph key and position): a replayed
        segment keeps the buckets traced when it first ran."""
        plan = self._plans.get(tag)
        if plan is None:
            plan = self._plans[tag] = {'last': None}
        return (lambda: self._watched(plan, grads_fn)), (lambda: self._reduce_plan(plan))

    def clear_plans(self):
        self._plans.clear()

    def _watched(self, plan, fn):
        seq = []

        def note(leaf):
            i = self._idx.get(id(leaf))
            if i is not None:
                seq.append(self.bucket_of[i])

        prev = _ag.GRAD_WATCH[0]
        _ag.GRAD_WATCH[0] = note
        self._note = note
        try:
            fn()
        finally:
            _ag.GRAD_WATCH[0] = prev
            self._note = None
        traced = {}
        for pos, b in enumerate(seq):
            traced[b] = pos
        if traced or plan['last'] is None:
            plan['last'] = traced

    def _reduce_plan(self, plan):
        if self.world <= 1 and not self.force:
            return
        last = plan['last'] or {}
        works = []
        for b in sorted(last, key=last.get):   # buckets in the order the backward completed them
            a, e = self.buckets[b]
            works.append(dist.all_reduce(self.grad[a:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        for w in works:
            w.wait()

    def scale(self):
        """grad *= 1/world (the all-reduce mean, pg_gans.py:1175-1179)."""
        if self.world > 1:
            self.grad.mul_(1.0 / self.world)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def broadcast_flat(t: torch.Tensor, src: int = 0, group=None, world_size: int = 1):
    """Make a replicated flat buffer identical on every rank (initial weights)."""
    if world_size > 1:
        dist.broadcast(t, src=src, group=group)
