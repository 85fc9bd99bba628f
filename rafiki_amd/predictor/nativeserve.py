"""Native HTTP front end of the predictor (``csrc/runtime/httpfront.cpp``): the default predictor server.

Same wire contract as ``server.create_app`` and ``fastserve`` (reference rafiki/predictor/app.py:23-30):
``POST /predict {"query": q} -> {"prediction": p}``, ``POST /predict_batch``, ``POST /predict_batch_npy``,
``GET /``, ``/stats``, ``/metrics``.

Division of labour:

* C++ I/O threads (epoll) own every socket: HTTP/1.1 keep-alive parsing, JSON image queries decoded
  straight to uint8, response formatting and writing.  No per-request Python.
* One Python batch thread per predictor replica, bound to that replica, loops on
  ``rt_http_next_batch`` (blocking in C++, GIL released): it receives every image request pending at
  that moment — single JSON queries and whole ``.npy`` batches — as ONE contiguous uint8 batch and
  hands the probabilities back with ``rt_http_complete``; C++ writes one ``{"prediction": [...]}``
  per JSON query and one ``.npy`` float32 array per npy request.  Queries that arrive while the GPU
  runs batch k become batch k+1 — no timer, no per-query futures.
* Double buffering: for a one-graph ensemble (``EnsembleGraphs.staging``) C++ decodes straight into
  one of two pinned staging slots; batch k+1 is collected into slot B and its graph queued right
  behind batch k's (slot A) before the thread waits for batch k and completes it.  Each replica has
  its own graphs, stream and slots, so R replicas take disjoint batches from the C++ queue and run
  concurrently.  Other predictors go through ``Predictor.predict_array``.
* Everything else (non-image queries, batch routes, stats) is a generic request answered by a
  small Python pool, exactly as ``fastserve`` answers it.
"""
from __future__ import annotations

import concurrent.futures
import ctypes
import io
import json
import logging
import math
import threading
import time
import traceback

import numpy as np

from .. import runtime

logger = logging.getLogger(__name__)

MAX_BODY = 256 << 20
# one image query on the C++ batch path (larger ones are routed to the generic Python path) and the most
# the batch buffer of a replica may grow to
MAX_QUERY = 1 << 20
MAX_BATCH_BUF = 64 << 20

_SIGS = {
    'rt_http_start': (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                                        ctypes.c_longlong, ctypes.c_int]),
    'rt_http_port': (ctypes.c_int, [ctypes.c_void_p]),
    'rt_http_next_batch': (ctypes.c_longlong, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'rt_http_complete': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_void_p, ctypes.c_longlong,
                                        ctypes.c_longlong]),
    'rt_http_fail': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_char_p]),
    'rt_http_next_request': (ctypes.c_longlong, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p,
                                                 ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    'rt_http_request_body': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_void_p]),
    'rt_http_respond': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_char_p,
                                       ctypes.c_char_p, ctypes.c_longlong]),
    'rt_http_stats': (None, [ctypes.c_void_p, ctypes.c_void_p]),
    'rt_http_shutdown': (None, [ctypes.c_void_p]),
    'rt_http_stop': (None, [ctypes.c_void_p]),
    'rt_http_set_max_query': (None, [ctypes.c_void_p, ctypes.c_longlong]),
}
_STAT_KEYS = ('requests', 'batches', 'batched_queries', 'generic_requests', 'errors', 'connections_accepted',
              'connections_open', 'queued_queries')


def _lib():
    h = runtime.lib()
    if h is None or getattr(h, 'rt_http_start', None) is None:
        return None
    if not getattr(h, '_http_bound', False):
        for name, (res, args) in _SIGS.items():
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
        h._http_bound = True
    return h


def available() -> bool:
    return _lib() is not None


def route(predictor, counters, method: str, path: str, body: bytes):
    """The Python-side routes (synchronous): -> (status, content type, payload bytes)."""
    if path == '/predict' and method == 'POST':
        arr = runtime.json_u8_array(body, 'query') if predictor._fast_path() else None
        if arr is not None:
            p = np.asarray(predictor.predict_array(arr[None]))[0]
            return 200, 'application/json', json.dumps({'prediction': p.tolist()}).encode()
        q = json.loads(body or b'{}')['query']
        p = predictor.predict([q])[0]
        return 200, 'application/json', json.dumps({'prediction': p.tolist() if hasattr(p, 'tolist') else p}).encode()
    if path == '/predict_batch' and method == 'POST':
        arr = runtime.json_u8_array(body, 'queries')
        if arr is not None:
            out = predictor.predict_array(arr)
            out = out.tolist() if hasattr(out, 'tolist') else out
        else:
            out = predictor.predict(json.loads(body or b'{}')['queries'])
        return 200, 'application/json', json.dumps({'predictions': out}).encode()
    if path == '/predict_batch_npy' and method == 'POST':
        arr = np.load(io.BytesIO(body), allow_pickle=False)
        probs = predictor.predict_array(arr)
        buf = io.BytesIO()
        np.save(buf, np.asarray(probs, dtype=np.float32), allow_pickle=False)
        return 200, 'application/octet-stream', buf.getvalue()
    if method == 'GET':
        if path == '/':
            return 200, 'text/html; charset=utf-8', b'Rafiki Predictor is up.'
        if path == '/stats':
            st = dict(predictor.stats, server=dict(counters), models=[n for n, _ in predictor.models],
                      resident_bytes=predictor.cache.used)
            return 200, 'application/json', json.dumps(st).encode()
        if path == '/metrics':
            lines = ['# TYPE rafiki_predictor_{} counter\nrafiki_predictor_{} {}'.format(k, k, v)
                     for k, v in counters.items()]
            return 200, 'text/plain; version=0.0.4', ('\n'.join(lines) + '\n').encode()
    known = ('/', '/predict', '/predict_batch', '/predict_batch_npy', '/stats', '/metrics')
    return (405 if path in known else 404), 'text/plain', b''


class NativePredictorServer:
    """Drop-in for ``FastPredictorServer``: ``start()`` / ``serve_forever()`` / ``shutdown()`` / ``port``."""

    TIMING_RING = 1 << 16

    def __init__(self, predictor, host='0.0.0.0', port=3003, max_batch=512, io_threads=4, generic_threads=4):
        self.predictor = predictor
        self.host, self.port = host, int(port)
        self.max_batch = int(max_batch)
        self.io_threads = int(io_threads)
        self.generic_threads = int(generic_threads)
        self.slots = max(1, len(getattr(predictor, 'replicas', [None])))
        self._h = None
        self._threads = []
        self._running = threading.Event()
        self._stopped = threading.Event()
        self._pool = None
        self._base = {'python_batches': 0, 'python_errors': 0}
        self._ready = []
        # per-batch timeline of the staged loop (ring of the last TIMING_RING batches): queries, then the
        # seconds from the batch leaving the C++ queue to its launch, to its graph finishing, and to its
        # responses being handed back (batch_timing() summarises; the p99 analysis of docs/serving.md)
        self._timing = np.zeros((self.TIMING_RING, 4), dtype=np.float64)
        self._timing_n = 0
        self.ready_timeout_s = 300.0

    # ------------------------------------------------------------------------------ stats
    @property
    def counters(self):
        out = dict(self._base)
        h = _lib()
        if self._h is not None and h is not None:
            buf = (ctypes.c_longlong * 8)()
            h.rt_http_stats(self._h, buf)
            out.update({k: int(v) for k, v in zip(_STAT_KEYS, buf)})
        return out

    def reset_timing(self):
        self._timing_n = 0

    def batch_timing(self) -> dict:
        """Percentiles (ms) of the staged batches since ``reset_timing``: ``launch`` = C++ queue -> graph
        launched, ``device`` = launch -> graph done (includes waiting behind the previous batch on the
        stream), ``complete`` = done -> responses handed to C++; plus the batch-size distribution."""
        n = min(self._timing_n, self.TIMING_RING)
        if n == 0:
            return {}
        t = self._timing[:n]
        out = {'batches': int(n), 'batch_queries_p50': float(np.percentile(t[:, 0], 50)),
               'batch_queries_max': float(t[:, 0].max())}
        for j, k in ((1, 'launch'), (2, 'device'), (3, 'complete')):
            for q in (50, 99):
                out['{}_p{}_ms'.format(k, q)] = round(float(np.percentile(t[:, j], q)) * 1e3, 3)
        tot = t[:, 1:].sum(1)
        out['total_p50_ms'] = round(float(np.percentile(tot, 50)) * 1e3, 3)
        out['total_p99_ms'] = round(float(np.percentile(tot, 99)) * 1e3, 3)
        return out

    # ------------------------------------------------------------------------------ loops
    def _batch_loop(self, idx=0):
        try:
            return self._batch_loop_body(idx)
        finally:
            self._ready[idx].set()

    def _batch_loop_body(self, idx):
        fn = getattr(self.predictor, 'staged_graphs', None)
        staged = None
        if callable(fn):
            try:
                staged = fn(idx)
            except Exception:
                logger.error('replica %d: no staged ensemble graphs:\n%s', idx, traceback.format_exc())
        if staged is not None:
            bufs = staged[1].staging(staged[2])
            if bufs is not None:
                try:
                    staged[1].warm_staged()   # every bucket x slot captured before the first query
                except Exception:
                    logger.error('replica %d: staged graphs failed:\n%s', idx, traceback.format_exc())
                    self._ready[idx].set()
                    return self._plain_loop()
                self._ready[idx].set()
                return self._staged_loop(staged[1], staged[2], bufs)
        self._ready[idx].set()
        return self._plain_loop()

    def _complete(self, bid, probs, n):
        h = _lib()
        try:
            probs = np.ascontiguousarray(np.asarray(probs), dtype=np.float32)
            if probs.ndim != 2 or probs.shape[0] < n:
                raise ValueError('predictor returned shape {} for {} queries'.format(probs.shape, n))
            h.rt_http_complete(self._h, bid, probs.ctypes.data, int(n), int(probs.shape[1]))
            self._base['python_batches'] += 1
        except Exception as e:
            self._fail(bid, e)

    def _fail(self, bid, e):
        self._base['python_errors'] += 1
        logger.error('predictor batch failed: %r', e)
        _lib().rt_http_fail(self._h, bid, '{}: {}'.format(type(e).__name__, e).encode('utf-8', 'replace'))

    def _staged_loop(self, g, img_shape, bufs):
        """Double-buffered loop over one replica's ensemble graphs: collect batch k+1 into the free
        staging slot and queue its replay before waiting for batch k."""
        h = _lib()
        cap = int(bufs[0].size)
        shape = (ctypes.c_longlong * 8)()
        nd = ctypes.c_int(0)
        bid = ctypes.c_ulonglong(0)
        pending = None   # (event, slot, batch id, images)
        slot = 0
        big = None       # fallback buffer for requests the staging slot cannot hold
        while self._running.is_set():
            launched = None
            taken = None   # a batch id handed out by rt_http_next_batch and not yet launched / completed
            try:
                n = h.rt_http_next_batch(self._h, 0 if pending else 100, bufs[slot].ctypes.data, cap, shape,
                                         ctypes.byref(nd), ctypes.byref(bid))
                if n == -1:
                    break
                if n == -3:   # larger than a staging slot: take it into the bounded fallback buffer
                    pending = self._finish_staged(g, pending)
                    if big is None:
                        big = np.empty(MAX_BATCH_BUF, dtype=np.uint8)
                    n = h.rt_http_next_batch(self._h, 0, big.ctypes.data, big.size, shape, ctypes.byref(nd),
                                             ctypes.byref(bid))
                    if n > 0:
                        taken = bid.value
                        q = tuple(int(shape[i]) for i in range(nd.value))
                        arr = big[:n * math.prod(q)].reshape((int(n),) + q)
                        taken = None
                        self._run_sync(bid.value, arr, n)
                    continue
                if n > 0:
                    taken = bid.value
                    t_take = time.perf_counter()
                    q = tuple(int(shape[i]) for i in range(nd.value))
                    if q == tuple(img_shape):
                        try:
                            launched = (g.launch_staged(slot, int(n)), slot, bid.value, int(n), t_take,
                                        time.perf_counter())
                        except Exception as e:
                            self._fail(bid.value, e)
                        taken = None
                        slot ^= 1
                    else:   # another image shape (resized by the models): the synchronous array path
                        pending = self._finish_staged(g, pending)
                        arr = bufs[slot][:n * math.prod(q)].reshape((int(n),) + q).copy()
                        taken = None
                        self._run_sync(bid.value, arr, n)
            except Exception as e:   # never let the replica's only batch thread die
                self._base['python_errors'] += 1
                logger.error('batch loop error:\n%s', traceback.format_exc())
                if taken is not None:   # the clients of a taken batch get an error reply, not a hang
                    self._fail(taken, e)
            pending = self._finish_staged(g, pending)
            pending = launched
        self._finish_staged(g, pending)

    def _finish_staged(self, g, pending):
        """Wait for a launched staged batch and complete it; returns None (the new 'pending')."""
        if pending is None:
            return None
        ev, slot, bid, n, t_take, t_launch = pending
        try:
            ev.synchronize()
        except Exception as e:
            self._fail(bid, e)
            return None
        t_done = time.perf_counter()
        self.predictor.stats['queries'] = self.predictor.stats.get('queries', 0) + n
        self._complete(bid, g.staged_out(slot), n)
        i = self._timing_n % self.TIMING_RING
        self._timing[i] = (n, t_launch - t_take, t_done - t_launch, time.perf_counter() - t_done)
        self._timing_n += 1
        return None

    def _run_sync(self, bid, arr, n):
        try:
            probs = self.predictor.predict_array(arr)
        except Exception as e:
            self._fail(bid, e)
            return
        self._complete(bid, probs, n)

    def _plain_loop(self):
        h = _lib()
        cap = max(1, self.max_batch) * 32 * 32 * 3
        buf = np.empty(cap, dtype=np.uint8)
        shape = (ctypes.c_longlong * 8)()
        nd = ctypes.c_int(0)
        bid = ctypes.c_ulonglong(0)
        while self._running.is_set():
            taken = None
            try:
                n = h.rt_http_next_batch(self._h, 100, buf.ctypes.data, cap, shape, ctypes.byref(nd),
                                         ctypes.byref(bid))
                if n == 0:
                    continue
                if n == -1:
                    break
                if n == -3:   # the first request does not fit: grow to the bound (C++ keeps requests below it)
                    cap = max(cap, MAX_BATCH_BUF)
                    buf = np.empty(cap, dtype=np.uint8)
                    continue
                if n < 0:
                    continue
                taken = bid.value
                q = tuple(int(shape[i]) for i in range(nd.value))
                arr = buf[:n * int(math.prod(q))].reshape((int(n),) + q)
            except Exception as e:   # never let the replica's only batch thread die
                self._base['python_errors'] += 1
                logger.error('batch loop error:\n%s', traceback.format_exc())
                if taken is not None:
                    self._fail(taken, e)
                continue
            self._run_sync(bid.value, arr, n)

    def _serve_generic(self, rid, method, path, body):
        h = _lib()
        try:
            status, ctype, payload = route(self.predictor, self.counters, method, path, body)
        except Exception as e:
            self._base['python_errors'] += 1
            logger.error('predictor request failed:\n%s', traceback.format_exc())
            status, ctype, payload = 500, 'text/plain', '{}: {}'.format(type(e).__name__, e).encode()
        h.rt_http_respond(self._h, rid, status, ctype.encode(), payload, len(payload))

    def _generic_loop(self):
        h = _lib()
        rid = ctypes.c_ulonglong(0)
        method = ctypes.create_string_buffer(16)
        path = ctypes.create_string_buffer(2048)
        while self._running.is_set():
            n = h.rt_http_next_request(self._h, 100, ctypes.byref(rid), method, 16, path, 2048)
            if n == -1:
                continue
            if n < 0:
                break
            body = ctypes.create_string_buffer(int(n)) if n else None
            if n:
                h.rt_http_request_body(self._h, rid.value, body)
            data = body.raw[:n] if n else b''
            self._pool.submit(self._serve_generic, rid.value, method.value.decode('latin-1'),
                              path.value.decode('latin-1'), data)

    # ------------------------------------------------------------------------------ running
    def start(self):
        h = _lib()
        if h is None:
            raise RuntimeError('librafiki_runtime.so with the HTTP front end is not built')
        self._h = h.rt_http_start(self.host.encode(), self.port, self.io_threads, self.max_batch, MAX_BODY,
                                  1 if self.predictor._fast_path() else 0)
        if not self._h:
            raise OSError('cannot listen on {}:{}'.format(self.host, self.port))
        h.rt_http_set_max_query(self._h, MAX_QUERY)
        self.port = int(h.rt_http_port(self._h))
        self._running.set()
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=self.generic_threads,
                                                           thread_name_prefix='rafiki-http-py')
        self._ready = [threading.Event() for _ in range(self.slots)]
        for i in range(self.slots):
            t = threading.Thread(target=self._batch_loop, args=(i,), name='rafiki-http-batch-{}'.format(i),
                                 daemon=True)
            t.start()
            self._threads.append(t)
        t = threading.Thread(target=self._generic_loop, name='rafiki-http-generic', daemon=True)
        t.start()
        self._threads.append(t)
        # replicas' graphs captured (queries arriving meanwhile wait in the C++ queue): one shared deadline
        deadline = time.monotonic() + self.ready_timeout_s
        late = [i for i, e in enumerate(self._ready) if not e.wait(max(0.0, deadline - time.monotonic()))]
        if late:
            logger.warning('native predictor server: replica(s) %s not ready after %.0f s; serving anyway '
                           '(their batches queue until they are)', late, self.ready_timeout_s)
        self.not_ready = late
        return self

    def serve_forever(self):
        if self._h is None:
            self.start()
        try:
            while not self._stopped.wait(1.0):
                pass
        except KeyboardInterrupt:
            pass
        finally:
            self.shutdown()

    def shutdown(self):
        h = _lib()
        if self._h is None or h is None:
            return
        self._running.clear()
        h.rt_http_shutdown(self._h)
        for t in self._threads:
            t.join(5)
        self._threads = []
        if self._pool is not None:
            self._pool.shutdown(wait=True)
        h.rt_http_stop(self._h)
        self._h = None
        self._stopped.set()


def make_server(predictor, host, port, **kw):
    """The native front end when the runtime is built (RAFIKI_PREDICTOR_SERVER=fast picks asyncio)."""
    import os
    kind = os.environ.get('RAFIKI_PREDICTOR_SERVER', 'native')
    if kind == 'native' and available():
        return NativePredictorServer(predictor, host, port, **kw)
    from .fastserve import FastPredictorServer
    return FastPredictorServer(predictor, host, port)
