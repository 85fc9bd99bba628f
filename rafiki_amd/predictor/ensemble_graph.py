"""One hipGraph per batch bucket for a whole top-k ensemble.

The reference answers a query by pushing it through Redis to one inference-worker container per
model and polling for the k answers (rafiki/predictor/predictor.py:31-74, worker/inference.py:
31-93).  Here the k resident models of one replica are captured together: per bucket B the graph
holds

    pinned host uint8 [B, ...]  --H2D-->  device input (one per input signature)
      -> for every model, on its own captured stream branch: pack/normalise kernel + eval forward
         (conv + folded-BN + ReLU/pool ... + softmax) into slot i of a [k, B, C] buffer
      -> gfx950 weighted ensemble-mean kernel -> [B, C]  --D2H-->  pinned host output

so a request costs one host memcpy into the pinned buffer, ONE graph launch and one stream sync —
independent of k and of the model depth (at batch 1 the per-model graphs + stack + ensemble of the
previous design were launch-bound at ~0.9 ms for 4 fp32 models).  Models of one architecture are
evaluated as ONE grouped network (engine.convnet.GroupedConvNets: every layer of all of them is a
single grouped kernel), so the graph holds the launches of one model, not k; other models get their
own captured stream branch.  Buckets are captured lazily on first use; a replica's graphs are
serialised by a lock (each replica owns its models, buffers and stream, so replicas run concurrently).
"""
from __future__ import annotations

import os
import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops.graphs import LOCK as _GRAPH_LOCK
from ..ops.graphs import capture as _capture

# batch buckets: above 64 the ensemble's graph time grows about linearly with the bucket, so the steps are
# at most 1.5x (a 84-query batch of 256 closed-loop JSON clients ran the 128 graph: 66 % of it useful,
# bench.py ensemble_http_json_sweep)
BUCKETS = (1, 8, 16, 32, 64, 96, 128, 192, 256, 384, 512)


def supports(models: Sequence[object]) -> bool:
    """True when every model can be captured in the shared graph: native device models with an
    input signature, a capture-safe ``forward_into`` and one common class count, all on one GPU."""
    if not models:
        return False
    devs, ncls = set(), set()
    for m in models:
        if not all(callable(getattr(m, a, None)) for a in ('forward_into', 'input_signature', 'prepare_serving')):
            return False
        d = getattr(m, 'device', None)
        if d is None or torch.device(d).type != 'cuda':
            return False
        devs.add(torch.device(d))
        ncls.add(int(getattr(m, 'num_classes', -1)))
    return len(devs) == 1 and len(ncls) == 1 and -1 not in ncls


class _Entry:
    __slots__ = ('graph', 'h_in', 'd_in', 'slots', 'out', 'h_out', 'bucket', 'host')


def _plan_groups(models):
    """[(member indices, GroupedConvNets or None)]: same-architecture native fp32 engines share one
    grouped network; everything else runs alone."""
    from ..engine.convnet import GroupedConvNets
    by = OrderedDict()
    for i, m in enumerate(models):
        fn = getattr(m, 'serving_engine', None)
        eng = fn() if callable(fn) else None
        key = GroupedConvNets.arch_key(eng) if eng is not None else None
        if key is None or os.environ.get('RAFIKI_ENSEMBLE_GROUPED', '1') == '0':
            key = ('single', i)
        by.setdefault(key, []).append(i)
    plan = []
    for key, idx in by.items():
        grouped = None
        if len(idx) > 1 and key[0] != 'single':
            grouped = GroupedConvNets([models[i].serving_engine() for i in idx])
        plan.append((idx, grouped))
    return plan


class EnsembleGraphs:
    def __init__(self, models: Sequence[object], weights: Optional[Sequence[float]] = None):
        for m in models:
            m.prepare_serving()
        plan = _plan_groups(list(models))
        order = [i for idx, _ in plan for i in idx]   # slot order: group members contiguous
        self.models = [models[i] for i in order]
        if weights is not None:
            weights = [weights[i] for i in order]
        self.plan, pos = [], 0
        for idx, grouped in plan:
            self.plan.append((pos, pos + len(idx), grouped))
            pos += len(idx)
        self.device = torch.device(getattr(self.models[0], 'device'))
        self.num_classes = int(self.models[0].num_classes)
        self.sigs: List[Tuple] = []
        for m in self.models:
            s = m.input_signature()
            if s not in self.sigs:
                self.sigs.append(s)
        self.weights = None if weights is None else torch.tensor(list(weights), dtype=torch.float32,
                                                                   device=self.device)
        self.lock = threading.Lock()
        self.stream = torch.cuda.Stream(device=self.device)
        self._branches = [torch.cuda.Stream(device=self.device) for _ in self.plan]
        self._graphs: Dict[Tuple[int, object], _Entry] = {}
        self._shapes: Dict[Tuple, Tuple] = {}
        self._stage = self._stage_out = None
        self.replays = 0

    # ------------------------------------------------------------------ capture
    def _body(self, e: _Entry):
        from ..ops import functional as F
        main = torch.cuda.current_stream(self.device)
        if e.host:
            for s in self.sigs:
                e.d_in[s].copy_(e.h_in[s], non_blocking=True)
        for (lo, hi, grouped), br in zip(self.plan, self._branches):
            br.wait_stream(main)
            with torch.cuda.stream(br):
                m = self.models[lo]
                xin = e.d_in[m.input_signature()]
                if grouped is not None:
                    grouped.forward_into(grouped.proto.prepare_inputs(xin), e.slots[lo:hi])
                else:
                    m.forward_into(xin, e.slots[lo])
        for br in self._branches:
            main.wait_stream(br)
        F.ensemble_mean(e.slots, self.weights, out=e.out)
        if e.host:
            e.h_out.copy_(e.out, non_blocking=True)

    def _entry(self, bucket: int, host) -> _Entry:
        """host: False (device in/out), True (own pinned buffers) or ('stage', slot) (the staging slot's)."""
        e = self._graphs.get((bucket, host))
        if e is not None:
            return e
        # warm-up (autotuning, allocator growth, device syncs) and capture of a new bucket are
        # serialised process-wide: another replica's thread may be capturing at the same moment
        with _GRAPH_LOCK:
            return self._build_entry(bucket, host)

    def _build_entry(self, bucket: int, host) -> _Entry:
        e = _Entry()
        e.bucket, e.host = bucket, bool(host)
        if isinstance(host, tuple):   # a staging slot: views of its shared max-bucket pinned buffers
            e.h_in = {self.sigs[0]: self._stage[host[1]][:bucket]}
        else:
            e.h_in = {s: torch.zeros((bucket,) + self._shapes[s], dtype=torch.uint8).pin_memory()
                      for s in self.sigs} if host else None
        e.d_in = {s: torch.zeros((bucket,) + self._shapes[s], dtype=torch.uint8, device=self.device)
                  for s in self.sigs}
        e.slots = torch.zeros((len(self.models), bucket, self.num_classes), dtype=torch.float32, device=self.device)
        e.out = torch.zeros((bucket, self.num_classes), dtype=torch.float32, device=self.device)
        if isinstance(host, tuple):
            e.h_out = self._stage_out[host[1]][:bucket]
        else:
            e.h_out = torch.zeros((bucket, self.num_classes), dtype=torch.float32).pin_memory() if host else None
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            self._body(e)          # eager warm-up: autotunes every GEMM shape, sizes the allocator
        self.stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with _capture(g, stream=self.stream):
            self._body(e)
        e.graph = g
        self._graphs[(bucket, host)] = e
        return e

    def _check(self, arrays):
        for s, a in arrays.items():
            if s not in self.sigs:
                raise KeyError('no model of this ensemble takes input {}'.format(s))
            shp = tuple(a.shape[1:])
            if self._shapes.setdefault(s, shp) != shp:
                raise ValueError('input shape {} does not match {} for {}'.format(shp, self._shapes[s], s))

    # ------------------------------------------------------------------ run
    def run_host(self, images: Dict[Tuple, np.ndarray]) -> np.ndarray:
        """{signature: uint8 numpy [B, ...]} -> ensemble probabilities numpy [B, C] (float32):
        pinned staging copy, ONE graph launch (H2D, k forwards, ensemble, D2H), one stream sync."""
        B = len(next(iter(images.values())))
        if B == 0:
            return np.zeros((0, self.num_classes), np.float32)
        if B > BUCKETS[-1]:
            step = BUCKETS[-1]
            return np.concatenate([self.run_host({s: a[i:i + step] for s, a in images.items()})
                                   for i in range(0, B, step)])
        bucket = next(b for b in BUCKETS if b >= B)
        with self.lock:
            self._check(images)
            e = self._entry(bucket, True)
            for s, a in images.items():
                e.h_in[s][:B].copy_(torch.from_numpy(np.ascontiguousarray(a)))
            with torch.cuda.stream(self.stream):
                e.graph.replay()
            self.stream.synchronize()
            self.replays += 1
            return e.h_out[:B].numpy().copy()

    def run_device(self, inputs: Dict[Tuple, torch.Tensor]) -> torch.Tensor:
        """{signature: device uint8 [B, ...]} -> device probabilities [B, C] (a fresh tensor, ordered
        after the caller's current stream; no host sync)."""
        B = next(iter(inputs.values())).shape[0]
        if B > BUCKETS[-1]:
            step = BUCKETS[-1]
            return torch.cat([self.run_device({s: t[i:i + step] for s, t in inputs.items()})
                              for i in range(0, B, step)])
        bucket = next(b for b in BUCKETS if b >= B)
        cur = torch.cuda.current_stream(self.device)
        with self.lock:
            self._check(inputs)
            e = self._entry(bucket, False)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                for s, t in inputs.items():
                    e.d_in[s][:B].copy_(t, non_blocking=True)
                e.graph.replay()
                res = e.out[:B].clone()
            cur.wait_stream(self.stream)
            res.record_stream(cur)
            self.replays += 1
            return res

    # ------------------------------------------------------------------ double-buffered host path
    def staging(self, shape: Tuple[int, ...]):
        """Two pinned uint8 staging slots [BUCKETS[-1], *shape] (returned as flat numpy views) with their
        pinned fp32 outputs, for a single-signature ensemble (None otherwise).  The native front end
        decodes batch n+1 into one slot while the graph of batch n replays from the other: per bucket
        and slot one graph whose H2D reads the slot and whose D2H writes the slot's output."""
        if len(self.sigs) != 1:
            return None
        shape = tuple(int(v) for v in shape)
        with self.lock:
            if self._shapes.setdefault(self.sigs[0], shape) != shape:
                return None
            if self._stage is None:
                n = BUCKETS[-1]
                self._stage = [torch.zeros((n,) + shape, dtype=torch.uint8).pin_memory() for _ in range(2)]
                self._stage_out = [torch.zeros((n, self.num_classes), dtype=torch.float32).pin_memory()
                                   for _ in range(2)]
        return [t.numpy().reshape(-1) for t in self._stage]

    def warm_staged(self):
        """Capture every bucket's graph for both staging slots now (a lazy first capture inside the serving
        loop stalls every queued query for its warm-up + capture: the p99 spikes of a server that meets new
        batch sizes under load)."""
        if self._stage is None:
            raise RuntimeError('staging() first')
        with self.lock:
            for slot in (0, 1):
                for b in BUCKETS:
                    self._entry(b, ('stage', slot))
        torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def launch_staged(self, slot: int, B: int):
        """Replay the graph of staging slot ``slot`` for its first B images (B <= BUCKETS[-1]); returns an
        event the caller waits on before reading ``staged_out(slot)[:B]``.  No host sync here."""
        if not 0 < B <= BUCKETS[-1]:
            raise ValueError('staged batch of {} images'.format(B))
        bucket = next(b for b in BUCKETS if b >= B)
        with self.lock:
            e = self._entry(bucket, ('stage', slot))
            with torch.cuda.stream(self.stream):
                e.graph.replay()
            ev = torch.cuda.Event()
            ev.record(self.stream)
            self.replays += 1
        return ev

    def staged_out(self, slot: int) -> np.ndarray:
        return self._stage_out[slot].numpy()

