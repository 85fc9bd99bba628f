"""Bucketed gradient all-reduce over a flat fp32 gradient arena, overlapped with the backward.

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
  segments).  The first time a round shape runs (eagerly), every gradient contribution of the
  segment is observed in order (ops.autograd.GRAD_WATCH for the in-place weight-gradient writes,
  the post-accumulate hooks for autograd's) and becomes the segment's PLAN: the sequence of buckets
  the contributions land in.  Buckets that receive none are never reduced: PG-GAN blocks above the
  current level of detail hold zero gradient on every rank, so their sum is zero (two thirds of the
  arena at the reference schedule's 4x4 LOD).  From then on each bucket's all-reduce starts as soon
  as its last contribution is enqueued, while the rest of the backward still runs:
    - eager rounds launch it from the observer, at the next contribution after the bucket's last;
    - captured rounds CUT the capture there (``ops.graphs.SplitCapture``): the gradient segment
      becomes a sequence of graphs, and each bucket's all-reduce is launched on RCCL's stream
      between the replay of the graph that finished the bucket and the replay of the next one, so
      the reduce overlaps the later layers' backward on the GPU (pg_gans.py:1164-1171 starts each
      per-variable nccl all_sum as soon as its gradient exists).  No collective is ever inside a
      capture, and no event crosses a graph boundary (HIP refuses external event records during
      capture: ``profiles/graph_external_events_r5.txt``).
  The reduce segment that follows waits for every launched bucket (the current stream waits on
  RCCL's), so the mean + optimizer graph starts only after all of them.  Every rank must launch the
  same buckets in the same order: the first reduce of each plan compares a digest of it across the
  group and raises on a mismatch instead of hanging in mismatched collectives.
"""
from __future__ import annotations

import zlib
from typing import Dict, List, Optional, Sequence, Tuple

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

    # ------------------------------------------------------------ traced, overlapped gradient segments
    def traced(self, grads_fn, tag):
        """(grads, reduce) for a data-parallel round's segments: ``grads`` (a ``BucketedGrads``: callable
        eagerly, or captured as a graph sequence) runs ``grads_fn`` and starts each bucket's all-reduce
        once the bucket is complete; ``reduce`` launches whatever has not started (the whole plan on the
        tracing run) and makes the current stream wait for all of them.  ``tag`` names the segment
        across rounds (its graph key and position): a replayed segment keeps the plan traced when it
        first ran."""
        plan = self._plans.get(tag)
        if plan is None:
            plan = self._plans[tag] = {'seq': None, 'cuts': {}, 'tail': [], 'order': [], 'checked': False}
        seg = BucketedGrads(self, plan, grads_fn)
        return seg, seg.reduce

    def clear_plans(self):
        self._plans.clear()

    def _launch_slice(self, b, works):
        a, e = self.buckets[b]
        works.append(dist.all_reduce(self.grad[a:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def _check_plan(self, plan):
        """Every rank must reduce the same buckets in the same order (a rank-dependent branch or a stale
        plan would otherwise mismatch the collectives and hang): all_gather (count, crc32 of the order)."""
        order = plan['order']
        crc = zlib.crc32(','.join(str(b) for b in order).encode())
        mine = torch.tensor([len(order), crc], dtype=torch.int64, device=self.grad.device)
        world = dist.get_world_size(self.group)
        outs = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(outs, mine, group=self.group)
        got = [tuple(int(v) for v in o.tolist()) for o in outs]
        if any(g != got[0] for g in got):
            raise RuntimeError('data-parallel gradient buckets differ across ranks (count, crc32 per rank): '
                               '{}'.format(got))
        plan['checked'] = True

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


class BucketedGrads:
    """One data-parallel gradient segment (forward + backward of a D or G step) whose bucket
    all-reduces overlap its own backward; see the module docstring.  Made by
    ``FlatGradAllReduce.traced``; run eagerly by calling it, or captured with ``capture(pool)`` and
    replayed with ``replay(parts)`` (GraphedRounds.run_segments)."""

    def __init__(self, ar: FlatGradAllReduce, plan: dict, fn):
        self.ar, self.plan, self.fn = ar, plan, fn
        self.pre = []            # compute run before ``fn`` in the same (first) graph: a merged prelude
        self.works = []
        self.launched = set()

    @property
    def live(self) -> bool:
        return self.ar.world > 1 or self.ar.force

    def _body(self):
        for f in self.pre:
            f()
        self.fn()

    def _observe(self, on_cut):
        """Run the segment with an observer over its gradient contributions; ``on_cut(b)`` is called at
        the first contribution after bucket b's last one (the plan's cut points), before it."""
        ar, plan = self.ar, self.plan
        seq: List[int] = []
        cuts = plan['cuts'] if plan['seq'] is not None else {}

        def note(leaf):
            i = ar._idx.get(id(leaf))
            if i is None:
                return
            b = cuts.get(len(seq))
            if b is not None:
                on_cut(b)
            seq.append(ar.bucket_of[i])

        prev = _ag.GRAD_WATCH[0]
        _ag.GRAD_WATCH[0] = note
        ar._note = note
        try:
            self._body()
        finally:
            _ag.GRAD_WATCH[0] = prev
            ar._note = None
        return seq

    def _set_plan(self, seq):
        last: Dict[int, int] = {}
        for pos, b in enumerate(seq):
            last[b] = pos
        order = sorted(last, key=last.get)   # buckets in the order the backward completed them
        n = len(seq)
        self.plan.update(seq=list(seq), order=order, tail=[b for b in order if last[b] == n - 1],
                         cuts={last[b] + 1: b for b in order if last[b] + 1 < n})

    def _verify(self, seq):
        if seq != self.plan['seq']:
            raise RuntimeError('data-parallel gradient segment changed since it was traced ({} contributions, '
                               'traced {}): its bucket reduces would start early'.format(len(seq),
                                                                                        len(self.plan['seq'])))

    def _launch(self, b):
        if b not in self.launched:
            self.launched.add(b)
            self.ar._launch_slice(b, self.works)

    def __call__(self):
        """Eager run: trace the plan on the first run; later runs launch each bucket at its cut."""
        self.works, self.launched = [], set()
        if self.plan['seq'] is None or not self.live:
            seq = self._observe(lambda b: None)
            if self.plan['seq'] is None and (seq or not self.live):
                self._set_plan(seq)
            return
        seq = self._observe(self._launch)
        self._verify(seq)
        for b in self.plan['tail']:
            self._launch(b)

    def capture(self, pool):
        """Capture the segment as a graph sequence cut at the plan's points; returns the parts
        [(graph, bucket to launch after it or None)] (the last part's mark is the tail list)."""
        from ..ops.graphs import SplitCapture
        sc = SplitCapture(pool)
        if not self.live or self.plan['seq'] is None:
            with sc.region():
                self._observe(lambda b: None)
            return sc.parts
        with sc.region():
            sc.tail_mark = list(self.plan['tail'])
            seq = self._observe(lambda b: sc.cut(b))
        self._verify(seq)
        return sc.parts

    def replay(self, parts):
        self.works, self.launched = [], set()
        for g, mark in parts:
            g.replay()
            if not self.live or mark is None:
                continue
            for b in (mark if isinstance(mark, list) else [mark]):
                self._launch(b)

    def reduce(self):
        """The reduce segment: launch what has not started (the tracing run's buckets), then make the
        current stream wait for every bucket of the round."""
        if not self.live:
            return
        if not self.plan['checked'] and self.ar.world > 1:
            self._check_plan_once()
        for b in self.plan['order']:
            self._launch(b)
        for w in self.works:
            w.wait()
        self.works, self.launched = [], set()

    def _check_plan_once(self):
        self.ar._check_plan(self.plan)
