"""Asynchronous knob/score exchange for trial-parallel HPO: ONE advisor on rank 0, payloads over RCCL.

Reference: every trial round-trips through the advisor service over HTTP —
``POST /advisors/<id>/propose`` before training and ``/feedback`` after
(rafiki/worker/train.py:83-115, :189-196; client.py:603-641).  SURVEY §2.5 C3 / §7.2 step 7 move that
exchange onto the GPU interconnect with asynchronous rounds.

Protocol (one node, one process per GPU):

* a dedicated control process group (``control_group``) so the exchange never interleaves with a
  model's gradient collectives on the default group;
* rank r != 0 finishing a trial pushes its rank onto a FIFO in the rendezvous TCPStore (a doorbell:
  ``queue_push`` / blocking ``queue_pop``, no polling), then point-to-point ``send``s one packed
  fp64 row ``[op, has_prev, score, ok, secs, *prev_knob_row]`` to rank 0 and, for ``op=request``,
  ``recv``s the reply ``[valid, *next_knob_row]`` (``op=report`` feeds a score only, ``op=finish``
  feeds the last score and leaves).  Both rows travel over the backend of the group — RCCL over
  xGMI on the GPU node (gloo on CPU tests);
* rank 0 runs a server thread that pops doorbells in arrival order, receives the row, feeds the
  score into its single GP-EI advisor and proposes the next knob set with every in-flight trial as
  a constant-liar pending point, then sends it back.  Rank 0's own trials call the same handler
  in-process.  One posterior, one proposer: no per-rank GP refits;
* the trial budget stays an atomic claim in the SQLite store (the durable record and the budget
  authority): a rank claims a trial BEFORE asking for its knobs and sends ``finish`` once a claim
  fails.

GPU hygiene: the server thread issues its RCCL ops on its own HIP stream and under
``ops.graphs.LOCK``, so it never launches work while another thread of rank 0 is capturing a
hipGraph; RCCL recv kernels are only posted once the doorbell says the matching send is coming,
so no receive sits spinning on a CU during a trial.
"""
from __future__ import annotations

import datetime
import logging
import math
import os
import sys
import threading
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import dist as D

logger = logging.getLogger(__name__)

_GROUPS: Dict[tuple, object] = {}
_HDR = 5   # op, has_prev, score, ok, secs
OP_FINISH, OP_REQUEST, OP_REPORT = 0, 1, 2


def control_group(info: D.DistInfo):
    """All-ranks process group reserved for control traffic (created once per process; collective)."""
    key = (info.world_size, info.backend)
    if key not in _GROUPS:
        _GROUPS[key] = dist.new_group(ranks=list(range(info.world_size)), backend=info.backend)
    return _GROUPS[key]


def _store(timeout_s: float):
    from torch.distributed import distributed_c10d as c10d
    s = c10d._get_default_store().clone()
    s.set_timeout(datetime.timedelta(seconds=timeout_s))
    return s


class _Channel:
    """Point-to-point rows between rank 0 and one peer on the control group."""

    def __init__(self, info: D.DistInfo, group):
        self.info, self.group = info, group
        self.dev = D.comm_device(info)
        self.stream = torch.cuda.Stream(self.dev) if self.dev.type == 'cuda' else None

    def _ctx(self):
        import contextlib
        if self.stream is None:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.stream)

    def send(self, row: List[float], peer: int):
        with self._ctx():
            t = torch.tensor(row, dtype=torch.float64, device=self.dev)
            dist.send(t, dst=peer, group=self.group)
            if self.stream is not None:
                self.stream.synchronize()

    def recv(self, n: int, peer: int) -> List[float]:
        with self._ctx():
            t = torch.empty(n, dtype=torch.float64, device=self.dev)
            dist.recv(t, src=peer, group=self.group)
            return t.cpu().tolist()

    def recv_bounded(self, n: int, peer: int, lock, timeout_s: float) -> List[float]:
        """Rank 0's receive of a row whose doorbell has rung: the receive is POSTED under ``lock``
        (a launch: never while another thread captures a graph) and waited for outside it, up to
        ``timeout_s`` — a peer that died between its doorbell and its send leaves a TimeoutError,
        not a server thread blocked forever while holding the capture lock."""
        with lock:
            with self._ctx():
                t = torch.empty(n, dtype=torch.float64, device=self.dev)
                work = dist.irecv(t, src=peer, group=self.group)
        msg = 'knob exchange: rank {} rang its doorbell but sent no row within {:.0f} s'.format(peer, timeout_s)
        if self.dev.type != 'cuda':
            # gloo: a receive completes only inside wait(), which takes the deadline itself
            try:
                work.wait(timeout=datetime.timedelta(seconds=timeout_s))
            except RuntimeError as e:
                raise TimeoutError(msg) from e
        else:
            # RCCL: poll the completion event.  Each poll is an event query on the GPU, so it runs
            # under ``lock`` (never mid-capture of another thread); the deadline check and the sleep
            # between polls stay outside it, so a capture waits at most one poll.
            deadline = time.monotonic() + timeout_s
            while True:
                with lock:
                    done = work.is_completed()
                if done:
                    break
                if time.monotonic() > deadline:
                    raise TimeoutError(msg)
                time.sleep(0.0002)
        with lock:   # the stream sync and the D2H copy are GPU calls too
            if self.stream is not None:
                self.stream.synchronize()
            return t.cpu().tolist()


class KnobExchange:
    """Rank 0: the advisor + server thread.  Other ranks: a thin client.  Same API on every rank:

        ex = KnobExchange(info, knob_config, advisor_factory, tag)
        knobs = ex.request(prev=None)            # after claiming a trial
        knobs = ex.request(prev=(knobs, score, ok, secs))
        ex.report(prev)                          # a score without asking for knobs (resumed trials)
        ex.finish(prev)                          # once a claim fails
        ex.close()                               # rank 0: waits for every peer's finish
    """

    def __init__(self, info: D.DistInfo, knob_config, advisor_factory, tag: str,
                 history: Optional[List[tuple]] = None, store_timeout_s: float = 600.0):
        self.info = info
        self.knob_config = knob_config
        self.names = sorted(knob_config)
        # a fresh nonce per incarnation: a restarted worker group never pops a dead one's doorbells
        nonce = D.broadcast_object(info, '{:x}'.format(time.time_ns()) if info.is_main else None)
        self.tag = 'rafiki/knobx/{}/{}'.format(tag, nonce)
        self.stats = {'requests': 0, 'remote_requests': 0, 'proposals': 0, 'stale_served': 0, 'serve_s': 0.0,
                      'wait_s': 0.0}
        self.advisor = None
        self._threads = []
        self._error = None
        self._broken = False
        # rank 0: how long a doorbell may precede its row (the peer's send follows its push at once)
        self.recv_timeout_s = float(os.environ.get('RAFIKI_EXCHANGE_RECV_TIMEOUT_S', '120'))
        if info.world_size > 1:
            self.group = control_group(info)
            self.chan = _Channel(info, self.group)
            self.store = _store(store_timeout_s)
            # the server thread blocks in queue_pop on ``store``; a TCPStore client serialises its
            # requests, so rank 0's own doorbell pushes need a connection of their own
            self._push_store = _store(store_timeout_s)
        if info.is_main:
            self.advisor = advisor_factory()
            for knobs, score in history or []:
                self.advisor.feedback(knobs, score)
            self._cv = threading.Condition()
            self._hv = 0                                   # history version: +1 per scored trial
            self._ahead: Dict[int, tuple] = {}             # rank -> (knobs, hv when proposed)
            self._running: Dict[int, dict] = {}            # rank -> knobs of its in-flight trial
            self._active = set(range(info.world_size))     # ranks that have not finished
            self._closed = False
            # the advisor thread computes GP fits in Python/numpy; a short GIL switch interval keeps
            # the trial thread's host work (launches, DB writes) from queueing behind them
            self._switch = sys.getswitchinterval()
            sys.setswitchinterval(min(self._switch, 0.0005))
            # ONE advisor thread: it serves remote requests and, between them, keeps a proposal
            # ready per rank (a single thread, so GP fits never fight the server for the GIL)
            self._spawn(self._serve if info.world_size > 1 else self._ahead_loop, 'rafiki-knob-advisor')

    def _spawn(self, fn, name):
        def run():
            try:
                fn()
            except BaseException as e:   # surfaced by close()
                self._error = e
                logger.error('%s failed: %r', name, e)
        t = threading.Thread(target=run, name=name, daemon=True)
        t.start()
        self._threads.append(t)

    # ------------------------------------------------------------------------------ encoding
    def _row(self, knobs: Optional[dict]) -> List[float]:
        if knobs is None:
            return [0.0] * len(self.names)
        return D.pack_knobs(self.knob_config, [knobs])[0].tolist()

    def _knobs(self, row: List[float]) -> dict:
        return D.unpack_knobs(self.knob_config, torch.tensor([row], dtype=torch.float64))[0]

    # ------------------------------------------------------------------------------ rank 0
    def _ahead_work(self):
        """The next rank to (re)propose for, or None: ranks without a ready proposal first, then
        ranks whose ready proposal predates the newest score."""
        active = sorted(self._active)
        for r in active:
            if r not in self._ahead:
                return r
        # refresh a ready proposal once it lags several new scores (a refresh per score would keep
        # the advisor thread, and so the GIL, busy all the time on short trials)
        lag = max(1, (len(active) + 1) // 2)
        for r in active:
            if self._ahead[r][1] + lag <= self._hv:
                return r
        return None

    def _propose_one(self, r, hv, old):
        """One GP-EI proposal for rank ``r`` with every in-flight trial and every other ready
        proposal as constant-liar pending points; installed unless superseded meanwhile."""
        knobs = self.advisor.propose()
        with self._cv:
            self.stats['proposals'] += 1
            cur = self._ahead.get(r)
            if r not in self._active:
                self.advisor.feedback(knobs, None)          # rank left: withdraw it
            elif cur is not None and cur is not old and cur[1] >= hv:
                self.advisor.feedback(knobs, None)          # superseded while computing
            else:
                if cur is not None:
                    self.advisor.feedback(cur[0], None)     # replace the stale one
                self._ahead[r] = (knobs, hv)
            self._cv.notify_all()
            return knobs

    def _ahead_loop(self):
        """world_size 1: keep the next proposal ready while the trial trains."""
        while True:
            with self._cv:
                while not self._closed and self._ahead_work() is None:
                    self._cv.wait()
                if self._closed:
                    return
                r = self._ahead_work()
                hv, old = self._hv, self._ahead.get(r)
            self._propose_one(r, hv, old)

    def _handle(self, rank: int, op: int, prev) -> Optional[dict]:
        """Feed ``prev = (knobs, score, ok, secs)`` (or None); for a request, hand out ``rank``'s ready
        proposal (computed inline if none is ready); on finish, retire the rank."""
        with self._cv:
            self.stats['requests'] += 1
            if prev is not None:
                knobs, score, ok, _secs = prev
                given = self._running.pop(rank, None)
                scored = ok and math.isfinite(score)
                self.advisor.feedback(given if given is not None else knobs, float(score) if scored else None)
                if scored:
                    self._hv += 1
            if op == OP_FINISH:
                self._active.discard(rank)
                old = self._ahead.pop(rank, None)
                if old is not None:
                    self.advisor.feedback(old[0], None)
            if op != OP_REQUEST:
                self._cv.notify_all()
                return None
            ready = self._ahead.pop(rank, None)
            if ready is not None:
                self.stats['stale_served'] += int(ready[1] < self._hv)
                self._running[rank] = ready[0]
                self._cv.notify_all()
                return ready[0]
        t0 = time.perf_counter()
        knobs = self.advisor.propose()
        with self._cv:
            self.stats['proposals'] += 1
            self.stats['wait_s'] += time.perf_counter() - t0
            self._running[rank] = knobs
            self._cv.notify_all()
        return knobs

    def _kick(self):
        """Wake the advisor thread after a local request/score (world_size > 1: it sleeps in the
        doorbell queue)."""
        if self.info.world_size > 1:
            self._push_store.queue_push(self.tag + '/q', '-1')

    def _serve(self):
        """Remote requests in doorbell order; between them, proposals for ranks that need one."""
        from ..ops import graphs
        if self.chan.dev.type == 'cuda':
            torch.cuda.set_device(self.chan.dev)
        done = set()
        ahead_failed = False
        qkey = self.tag + '/q'
        while len(done) < self.info.world_size - 1:
            with self._cv:
                r = self._ahead_work()
                hv, old = self._hv, self._ahead.get(r)
            if r is not None and not ahead_failed and self.store.queue_len(qkey) == 0:
                try:
                    self._propose_one(r, hv, old)
                except Exception as e:   # advisor failure: stop proposing ahead; requests get refusals
                    logger.error('knob exchange: proposal for rank %d failed: %r', r, e)
                    self._error = self._error or e
                    ahead_failed = True
                continue
            try:
                peer = int(self.store.queue_pop(qkey, block=True))
            except dist.DistStoreError:
                continue   # store timeout while every peer trains: keep waiting
            if peer < 0:
                continue   # a local kick: re-check the proposal work
            t0 = time.perf_counter()
            try:
                row = self.chan.recv_bounded(_HDR + len(self.names), peer, graphs.LOCK, self.recv_timeout_s)
            except TimeoutError as e:
                # the control group now holds a receive that will never complete: stop serving (rank 0's
                # own requests raise from here on, so the worker exits and the launcher ends the group)
                logger.error('%s', e)
                with self._cv:
                    self._error = self._error or e
                    self._broken = True
                    self._active.clear()
                    self._cv.notify_all()
                return
            op, has_prev, score, ok, secs = row[:_HDR]
            op = int(op)
            prev = (self._knobs(row[_HDR:]), score, ok > 0, secs) if has_prev > 0 else None
            try:
                knobs, valid = self._handle(peer, op, prev), 1.0
            except Exception as e:   # advisor failure: the peer still gets a (refusing) reply, never a hang
                logger.error('knob exchange: request of rank %d failed: %r', peer, e)
                self._error = self._error or e
                knobs, valid = None, 0.0
            if op == OP_REQUEST:
                with graphs.LOCK:
                    self.chan.send([valid] + self._row(knobs), peer)
            elif op == OP_FINISH:
                done.add(peer)
            with self._cv:
                self.stats['remote_requests'] += 1
                self.stats['serve_s'] += time.perf_counter() - t0
        self._ahead_loop()   # only rank 0 is left: keep serving its proposals until close()

    # ------------------------------------------------------------------------------ all ranks
    def _remote(self, op: int, prev) -> Optional[dict]:
        hdr = [float(op), 0.0, 0.0, 0.0, 0.0]
        kn = None
        if prev is not None:
            kn, score, ok, secs = prev
            hdr[1:] = [1.0, float(score) if ok else float('nan'), 1.0 if ok else 0.0, float(secs)]
        self.store.queue_push(self.tag + '/q', str(self.info.rank))
        self.chan.send(hdr + self._row(kn), 0)
        if op != OP_REQUEST:
            return None
        rep = self.chan.recv(1 + len(self.names), 0)
        if rep[0] <= 0:
            raise RuntimeError('knob exchange: rank 0 could not propose knobs (advisor failed)')
        return self._knobs(rep[1:])

    def _check_broken(self):
        if self._broken:
            raise RuntimeError('knob exchange is down (a peer stopped mid-exchange)') from self._error

    def request(self, prev=None) -> dict:
        if self.info.is_main:
            self._check_broken()
            knobs = self._handle(0, OP_REQUEST, prev)
            self._kick()
            return knobs
        return self._remote(OP_REQUEST, prev)

    def report(self, prev):
        if self.info.is_main:
            self._handle(0, OP_REPORT, prev)
            self._kick()
        else:
            self._remote(OP_REPORT, prev)

    def finish(self, prev=None):
        if self.info.is_main:
            self._handle(0, OP_FINISH, prev)
        else:
            self._remote(OP_FINISH, prev)

    def close(self):
        """Rank 0: wait until every peer has finished, then stop the helper threads."""
        if not self.info.is_main:
            return
        with self._cv:
            while self._active and self._threads and self._threads[0].is_alive():
                self._cv.wait(0.05)      # the server retires each peer on its finish
            self._closed = True
            self._cv.notify_all()
        for t in self._threads:
            t.join()
        self._threads = []
        sys.setswitchinterval(self._switch)
        if self._error is not None:
            raise RuntimeError('knob exchange failed') from self._error
