"""Bucketed gradient all-reduce over a flat fp32 gradient arena, overlapped with the backward.

Replaces the reference's per-variable ``tf.contrib.nccl.all_sum`` (pg_gans.py:1164-1171: ~25 calls
per network per step, several of them on tiny bias tensors) with a handful of large RCCL
all-reduces over contiguous slices of the FlatParams gradient buffer:

* buckets are contiguous ranges of the arena in REVERSE parameter order (backward produces the
  last layers' gradients first), each ~``bucket_mb`` MiB.  On xGMI a ring all-reduce is bound by
  one 153 GB/s link per hop, so a 16-32 MiB bucket amortises the ~10-20 us launch/latency to <5%
  while still giving several buckets to overlap with the remaining backward; PG-GAN
  runs 4 MiB (models/pg_gan.py grad_bucket_mb): one 3x3x512x512 conv per bucket, so the untouched
  blocks above the current LOD are skipped exactly and the first reduces start early — the measured
  per-rank rounds and the traced completion points put that ahead of 16-32 MiB at N = 2-8
  (profiles/pggan_comm_model_r6.json);
* a ``register_post_accumulate_grad_hook`` per parameter counts arrivals; when a bucket is
  complete its all-reduce is launched asynchronously (``async_op=True``) on RCCL's internal
  stream, overlapping the rest of the backward;
* ``finish()`` launches whatever did not fire (parameters outside the active graph, e.g. PG-GAN
  blocks above the current level of detail, still hold zeros and must be reduced to keep the
  replicas identical) and waits, then applies the 1/world mean (pg_gans.py:1175-1179);
* ``traced(grads_fn, tag)`` is the form for CAPTURED data-parallel rounds (GraphedRounds'
  segments).  The first eager runs of a round shape observe every gradient contribution of the
  segment (ops.autograd.GRAD_WATCH for the in-place weight-gradient writes, the post-accumulate hooks
  for autograd's) and record the segment's PLAN: how many contributions each bucket receives.
  Buckets that receive none are never reduced: PG-GAN blocks above the current level of detail hold
  zero gradient on every rank, so their sum is zero (two thirds of the arena at the reference
  schedule's 4x4 LOD).  From then on each bucket's all-reduce starts as soon as it is complete, while
  the rest of the backward still runs:
    - eager rounds launch it from the observer, at the first contribution after the bucket's last;
    - captured rounds CUT the capture there (``ops.graphs.SplitCapture``): the gradient segment
      becomes a sequence of graphs, and each bucket's all-reduce is launched on RCCL's stream
      between the replay of the graph that completed the bucket and the replay of the next one, so
      the reduce overlaps the later layers' backward on the GPU (pg_gans.py:1164-1171 starts each
      per-variable nccl all_sum as soon as its gradient exists).  No collective is ever inside a
      capture, and no event crosses a graph boundary (HIP refuses external event records during
      capture: ``profiles/graph_external_events_r5.txt``).
  Every rank reduces the live buckets in ONE order: rank 0's completion order of its last tracing
  run, broadcast (``_agree_order``), a bucket as soon as it and every bucket before it in that order
  are complete — so the order the collectives are issued in never depends on a rank's own autograd
  order, which a per-rank autotuner pick can change (ascending bucket order would not do: WGAN-GP's
  double backward completes the output layers' buckets last, leaving nothing to overlap).  The reduce segment that follows waits for every launched
  bucket (the current stream waits on RCCL's), so the mean + optimizer graph starts after all of
  them.  The first reduce of each plan compares a digest of it across the group and raises on a
  mismatch instead of hanging in mismatched collectives.
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
            plan = self._plans[tag] = {'count': None, 'order': [], 'traces': 0, 'ready': False}
        seg = BucketedGrads(self, plan, grads_fn)
        return seg, seg.reduce

    def clear_plans(self):
        self._plans.clear()

    def _launch_slice(self, b, works):
        a, e = self.buckets[b]
        works.append(dist.all_reduce(self.grad[a:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def _check_plan(self, plan):
        """Every rank must reduce the same buckets (a rank-dependent branch would otherwise mismatch the
        collectives and hang): all_gather (live buckets, crc32 of (bucket, contributions)) and compare."""
        live = sorted(plan['count'] or {})
        crc = zlib.crc32(','.join('{}:{}'.format(b, plan['count'][b]) for b in live).encode())
        mine = torch.tensor([len(live), crc], dtype=torch.int64, device=self.grad.device)
        world = dist.get_world_size(self.group)
        outs = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(outs, mine, group=self.group)
        got = [tuple(int(v) for v in o.tolist()) for o in outs]
        if any(g != got[0] for g in got):
            raise RuntimeError('data-parallel gradient buckets differ across ranks (count, crc32 per rank): '
                               '{}'.format(got))

    def _agree_order(self, order):
        """Rank 0's bucket completion order, the same list on every rank (the order collectives are issued in)."""
        t = torch.full((len(self.buckets) + 1,), -1, dtype=torch.int64, device=self.grad.device)
        t[0] = len(order)
        if order:
            t[1:1 + len(order)] = torch.tensor(order, dtype=torch.int64)
        dist.broadcast(t, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0, group=self.group)
        v = t.tolist()
        return [int(b) for b in v[1:1 + int(v[0])]]

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
    replayed with ``replay(parts)`` (GraphedRounds.run_segments).

    The plan is the number of gradient contributions each live bucket receives (``count``) and the ORDER the
    buckets are reduced in, traced on the first TRACES eager runs (the first one also autotunes, and a
    tuned pick may reorder the backward).  The order is rank 0's completion order of the last tracing run,
    broadcast, so every rank issues the collectives in the same order whatever its own autograd order (a
    per-rank tuner pick can change it; the WGAN-GP double backward completes the output layers' buckets
    last, so bucket index order would leave nothing to overlap).  A bucket becomes ready at the first
    contribution after its count is reached (its last write is enqueued by then) once every bucket
    before it in the order is ready.  Tracing runs reduce everything after the backward, in bucket order."""

    TRACES = 2

    def __init__(self, ar: FlatGradAllReduce, plan: dict, fn):
        self.ar, self.plan, self.fn = ar, plan, fn
        self.pre = []            # compute run before ``fn`` in the same (first) graph: a merged prelude
        self.works = []
        self.launched = set()
        self._traced = False     # this round's gradient pass was a tracing run (its reduce finalises)

    @property
    def live(self) -> bool:
        return self.ar.world > 1 or self.ar.force

    @property
    def planned(self) -> bool:
        return self.plan['ready']

    def _body(self):
        for f in self.pre:
            f()
        self.fn()

    def _observe(self, on_ready, extra=None):
        """Run the segment with an observer over its gradient contributions.  Planned: ``on_ready(bs)`` is
        called with the buckets that just became ready (in order), before the contribution that found
        them so; returns (per-bucket contribution counts, buckets not yet ready at the end)."""
        ar, plan = self.ar, self.plan
        planned = self.planned
        order = plan['order'] if planned else []
        count = plan['count'] if planned else {}
        seen: Dict[int, int] = {}
        nxt = [0]

        def note(leaf):
            i = ar._idx.get(id(leaf))
            if i is None:
                return
            if planned:
                ready = []
                while nxt[0] < len(order) and seen.get(order[nxt[0]], 0) == count[order[nxt[0]]]:
                    ready.append(order[nxt[0]])
                    nxt[0] += 1
                if ready:
                    on_ready(ready)
            b = ar.bucket_of[i]
            if planned and b in order[:nxt[0]]:
                raise RuntimeError('data-parallel bucket {} received a gradient after its all-reduce was '
                                   'started (the segment changed since it was traced: contribution {} of a '
                                   'traced {}, leaf {})'.format(b, seen.get(b, 0) + 1, count.get(b),
                                                               tuple(leaf.shape)))
            seen[b] = seen.get(b, 0) + 1
            if extra is not None:
                extra(leaf)

        prev = _ag.GRAD_WATCH[0]
        _ag.GRAD_WATCH[0] = note
        ar._note = note
        try:
            self._body()
        finally:
            _ag.GRAD_WATCH[0] = prev
            ar._note = None
        if planned and seen != count:
            raise RuntimeError('data-parallel gradient segment changed since it was traced: contributions per '
                               'bucket {} vs traced {}'.format(seen, count))
        return seen, order[nxt[0]:]

    def _trace(self):
        ar = self.ar
        last: Dict[int, int] = {}
        pos = [0]

        def note(leaf):   # the order the backward completes the buckets in (position of the last contribution)
            i = ar._idx.get(id(leaf))
            if i is not None:
                last[ar.bucket_of[i]] = pos[0]
                pos[0] += 1
        seen, _ = self._observe(None, extra=note)
        if seen or self.plan['count'] is None:
            # 'at': where in the pass each bucket completed (fraction of the contributions; the comm model)
            self.plan.update(count=dict(seen), order=sorted(seen, key=lambda b: last[b]),
                             at={b: (last[b] + 1) / max(1, pos[0]) for b in last})
        self.plan['traces'] += 1
        self._traced = True

    def _launch(self, b):
        if b not in self.launched:
            self.launched.add(b)
            self.ar._launch_slice(b, self.works)

    def _launch_all(self, bs):
        for b in bs:
            self._launch(b)

    def __call__(self):
        """Eager run: trace until the plan is settled; then launch each bucket as it becomes ready."""
        self.works, self.launched = [], set()
        self._traced = False
        if not self.planned or not self.live:
            self._trace()
            return
        _, tail = self._observe(self._launch_all)
        self._launch_all(tail)

    def capture(self, pool):
        """Capture the segment as a graph sequence cut where buckets become ready; returns the parts
        [(graph, buckets to launch after it)]."""
        from ..ops.graphs import SplitCapture
        if not self.planned:
            raise RuntimeError('BucketedGrads.capture before the plan is traced ({} eager runs needed)'.format(
                self.TRACES))
        sc = SplitCapture(pool)
        with sc.region():
            _, tail = self._observe(lambda bs: sc.cut(list(bs)) if self.live else None)
            sc.tail_mark = list(tail) if self.live else None
        return sc.parts

    def replay(self, parts):
        self.works, self.launched = [], set()
        for g, mark in parts:
            g.replay()
            if self.live and mark:
                self._launch_all(mark)

    def reduce(self):
        """The reduce segment: after a tracing run, check the plan across the ranks and reduce every live
        bucket in bucket order (and, after the last tracing run, agree on rank 0's completion order); then
        make the current stream wait for every bucket of the round."""
        if not self.live:
            return
        if self._traced:
            self._traced = False
            if self.ar.world > 1:
                self.ar._check_plan(self.plan)
            self._launch_all(sorted(self.plan['count'] or {}))
            if self.plan['traces'] >= self.TRACES and not self.plan['ready']:
                if self.ar.world > 1:
                    self.plan['order'] = self.ar._agree_order(self.plan['order'])
                self.plan['ready'] = True
        self._launch_all(self.plan['order'])   # none left on a planned round: each started when ready
        for w in self.works:
            w.wait()
        self.works, self.launched = [], set()
