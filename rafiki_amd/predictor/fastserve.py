"""Event-loop HTTP front end of the predictor (the default predictor service server).

Same wire contract as ``server.create_app`` (reference rafiki/predictor/app.py:23-30):
``POST /predict {"query": q} -> {"prediction": p}``, ``POST /predict_batch``, the binary
``POST /predict_batch_npy`` and ``GET /``, ``/stats``, ``/metrics``.  Why not Flask: a threaded
WSGI server spends ~1 ms of GIL-bound Python per request before the model is even reached, which
capped single-query serving at ~1.1 k QPS.  Here one asyncio loop parses HTTP/1.1 keep-alive
requests (request line + Content-Length only), decodes image queries with the native JSON parser,
and batches by construction: every query that arrives while the GPU runs batch k becomes batch
k+1 (no timer), which is submitted as ONE uint8 array to ``Predictor.predict_array`` (one hipGraph
for the whole ensemble).  With R predictor replicas, up to R batches are in flight at once on R
executor threads (each request lands on the least-busy replica).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import io
import json
import logging
import threading
import time
import traceback

import numpy as np

logger = logging.getLogger(__name__)

_REASON = {200: b'OK', 400: b'Bad Request', 404: b'Not Found', 405: b'Method Not Allowed',
           413: b'Payload Too Large', 500: b'Internal Server Error'}
MAX_BODY = 256 << 20  # request bodies above this are refused (413) before any byte is buffered


class FastPredictorServer:
    def __init__(self, predictor, host='0.0.0.0', port=3003, max_batch=512):
        self.predictor = predictor
        self.host, self.port = host, int(port)
        self.max_batch = int(max_batch)
        self.slots = max(1, len(getattr(predictor, 'replicas', [None])))
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=self.slots, thread_name_prefix='rafiki-gpu')
        self._inflight = 0
        self._pending = []            # (array, future) of single queries waiting for the next batch
        self._wake = None
        self._loop = None
        self._server = None
        self._thread = None
        self._started = threading.Event()
        self.counters = {'requests': 0, 'batches': 0, 'batched_queries': 0, 'errors': 0}
        # single image queries are stacked into device batches only for ensembles of native image
        # models; anything else (POS tagging, image generation, remote workers) takes predict()
        self._stackable = bool(predictor._fast_path())
        self._lat_sum = 0.0

    # ----------------------------------------------------------------------------- batching
    async def _run_batch(self, take):
        loop = asyncio.get_running_loop()
        try:
            probs = await loop.run_in_executor(self._pool, self.predictor.predict_array,
                                               np.stack([a for a, _ in take]))
            probs = np.asarray(probs)
            for i, (_, fut) in enumerate(take):
                if not fut.done():
                    fut.set_result(probs[i])
        except Exception as e:  # every waiter of the batch gets the error
            for _, fut in take:
                if not fut.done():
                    fut.set_exception(e)
        finally:
            self.counters['batches'] += 1
            self.counters['batched_queries'] += len(take)
            self._inflight -= 1
            self._wake.set()

    async def _batch_loop(self):
        while True:
            await self._wake.wait()
            self._wake.clear()
            while self._pending and self._inflight < self.slots:
                # one shape per batch (queries of the same model input size stack)
                shape = self._pending[0][0].shape
                take, rest = [], []
                for item in self._pending:
                    (take if item[0].shape == shape and len(take) < self.max_batch else rest).append(item)
                self._pending = rest
                self._inflight += 1
                asyncio.ensure_future(self._run_batch(take))

    def _enqueue(self, arr):
        fut = self._loop.create_future()
        self._pending.append((arr, fut))
        self._wake.set()
        return fut

    # ------------------------------------------------------------------------------- routes
    async def _route(self, method, path, body):
        loop = asyncio.get_running_loop()
        from .. import runtime
        if path == '/predict' and method == b'POST':
            arr = runtime.json_u8_array(body, 'query') if self._stackable else None
            if arr is not None:
                p = await self._enqueue(arr)
                return 200, b'application/json', json.dumps({'prediction': p.tolist()}).encode()
            q = json.loads(body or b'{}')['query']
            out = await loop.run_in_executor(self._pool, self.predictor.predict, [q])
            p = out[0]
            return 200, b'application/json', json.dumps({'prediction': p.tolist() if hasattr(p, 'tolist') else p}).encode()
        if path == '/predict_batch' and method == b'POST':
            arr = runtime.json_u8_array(body, 'queries')
            if arr is not None:
                out = await loop.run_in_executor(self._pool, self.predictor.predict_array, arr)
                out = out.tolist() if hasattr(out, 'tolist') else out
            else:
                qs = json.loads(body or b'{}')['queries']
                out = await loop.run_in_executor(self._pool, self.predictor.predict, qs)
            return 200, b'application/json', json.dumps({'predictions': out}).encode()
        if path == '/predict_batch_npy' and method == b'POST':
            arr = np.load(io.BytesIO(body), allow_pickle=False)
            probs = await loop.run_in_executor(self._pool, self.predictor.predict_array, arr)
            buf = io.BytesIO()
            np.save(buf, np.asarray(probs, dtype=np.float32), allow_pickle=False)
            return 200, b'application/octet-stream', buf.getvalue()
        if method == b'GET':
            if path == '/':
                return 200, b'text/html; charset=utf-8', b'Rafiki Predictor is up.'
            if path == '/stats':
                st = dict(self.predictor.stats, server=dict(self.counters),
                          models=[n for n, _ in self.predictor.models],
                          resident_bytes=self.predictor.cache.used)
                return 200, b'application/json', json.dumps(st).encode()
            if path == '/metrics':
                lines = ['# TYPE rafiki_predictor_{} counter\nrafiki_predictor_{} {}'.format(k, k, v)
                         for k, v in self.counters.items()]
                lines.append('# TYPE rafiki_predictor_request_seconds_sum counter\n'
                             'rafiki_predictor_request_seconds_sum {:.6f}'.format(self._lat_sum))
                return 200, b'text/plain; version=0.0.4', ('\n'.join(lines) + '\n').encode()
        known = ('/', '/predict', '/predict_batch', '/predict_batch_npy', '/stats', '/metrics')
        return (405 if path in known else 404), b'text/plain', b''

    # --------------------------------------------------------------------------- connection
    async def _handle(self, reader, writer):
        try:
            while True:
                try:
                    head = await reader.readuntil(b'\r\n\r\n')
                except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, ConnectionError):
                    break
                t0 = time.perf_counter()
                lines = head.split(b'\r\n')
                parts = lines[0].split(b' ')
                if len(parts) < 3:
                    break
                method, target, version = parts[0], parts[1], parts[2]
                path = target.split(b'?', 1)[0].decode('latin-1')
                clen, keep, bad = 0, version == b'HTTP/1.1', None
                for ln in lines[1:]:
                    k, _, v = ln.partition(b':')
                    k = k.strip().lower()
                    if k == b'content-length':
                        v = v.strip()
                        if not v.isdigit():
                            bad = (400, b'bad Content-Length')
                        else:
                            clen = int(v)
                            if clen > MAX_BODY:
                                bad = (413, b'request body too large')
                    elif k == b'connection':
                        v = v.strip().lower()
                        keep = v == b'keep-alive' or (keep and v != b'close')
                if bad is not None:  # answer and drop the connection: the body is never read
                    self.counters['errors'] += 1
                    writer.write(b'HTTP/1.1 %d %s\r\nContent-Type: text/plain\r\nContent-Length: %d\r\n'
                                 b'Connection: close\r\n\r\n' % (bad[0], _REASON[bad[0]], len(bad[1])) + bad[1])
                    await writer.drain()
                    break
                body = await reader.readexactly(clen) if clen else b''
                self.counters['requests'] += 1
                try:
                    status, ctype, payload = await self._route(method, path, body)
                except Exception as e:
                    # the traceback stays in the server log; the client gets the error type + message
                    self.counters['errors'] += 1
                    logger.error('predictor request failed:\n%s', traceback.format_exc())
                    status, ctype, payload = 500, b'text/plain', '{}: {}'.format(type(e).__name__, e).encode()
                writer.write(b'HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %d\r\n%s\r\n' % (
                    status, _REASON.get(status, b'OK'), ctype, len(payload),
                    b'' if keep else b'Connection: close\r\n') + payload)
                await writer.drain()
                self._lat_sum += time.perf_counter() - t0
                if not keep:
                    break
        finally:
            try:
                writer.close()
            except Exception:
                pass

    # ------------------------------------------------------------------------------ running
    async def _main(self):
        self._loop = asyncio.get_running_loop()
        self._wake = asyncio.Event()
        batcher = asyncio.ensure_future(self._batch_loop())
        self._server = await asyncio.start_server(self._handle, self.host, self.port, backlog=1024,
                                                  limit=1 << 26)
        self.port = self._server.sockets[0].getsockname()[1]
        self._started.set()
        try:
            async with self._server:
                await self._server.serve_forever()
        finally:
            batcher.cancel()

    def serve_forever(self):
        try:
            asyncio.run(self._main())
        except asyncio.CancelledError:
            pass

    def start(self):
        """Serve from a background thread (tests / in-process services); returns once listening."""
        self._thread = threading.Thread(target=self.serve_forever, name='rafiki-fastserve', daemon=True)
        self._thread.start()
        if not self._started.wait(30):
            raise RuntimeError('predictor server did not start')
        return self

    def shutdown(self):
        if self._loop is not None and self._server is not None:
            try:
                # closing the server ends serve_forever, and asyncio.run may close the loop before
                # the cancel coroutine below is scheduled: either order is a clean shutdown
                self._loop.call_soon_threadsafe(self._server.close)
                coro = self._cancel_all()
                try:
                    asyncio.run_coroutine_threadsafe(coro, self._loop).result(5)
                except Exception:
                    coro.close()   # the loop ended first: nothing left to cancel
            except Exception:
                pass
        if self._thread is not None:
            self._thread.join(5)
        self._pool.shutdown(wait=False)

    async def _cancel_all(self):
        for t in asyncio.all_tasks():
            if t is not asyncio.current_task():
                t.cancel()
