"""Closed-loop HTTP load against a predictor front end: what BASELINE.json's "predictor ensemble QPS"
names — queries through ``POST /predict`` (reference rafiki/predictor/app.py:23-30, predictor.py:31-74),
not a device-only batch.

``http_load`` starts the native front end (``nativeserve``: C++ epoll server, JSON / .npy decoded in C++
into the batch queue) on a free local port over an existing ``Predictor`` and drives it from OUTSIDE the
server's process with the native generator ``_native/httpload`` (csrc/tools/httpload.cpp: keep-alive
connections, one request in flight each, microseconds of client cost per request): single-query JSON
bodies on ``/predict`` and uint8 ``.npy`` batches on ``/predict_batch_npy``.  Each phase reports QPS
(queries, not requests) and per-request p50 / p99 latency measured by the client.
"""
from __future__ import annotations

import io
import json
import os
import subprocess
import tempfile

import numpy as np

HTTPLOAD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), '_native', 'httpload')


def available() -> bool:
    return os.path.exists(HTTPLOAD) and os.access(HTTPLOAD, os.X_OK)


def run_httpload(port, path, body: bytes, connections, threads, seconds, per_request=1):
    with tempfile.NamedTemporaryFile(suffix='.body') as bf:
        bf.write(body)
        bf.flush()
        r = subprocess.run([HTTPLOAD, '127.0.0.1', str(port), path, bf.name, str(connections),
                            str(max(1, min(threads, connections))), str(seconds)],
                           capture_output=True, text=True, timeout=seconds + 60)
    if r.returncode != 0 or not r.stdout.strip():
        raise RuntimeError('httpload failed (rc {}): {}'.format(r.returncode, r.stderr[-400:]))
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return {'qps': round(d['qps'] * per_request, 1), 'requests_per_s': round(d['qps'], 1),
            'p50_ms': d['p50_ms'], 'p99_ms': d['p99_ms'], 'errors': d['errors'], 'connections': connections}


def http_load(pred, image_shape=(32, 32, 3), seconds=3.0, json_clients=64, npy_clients=8, npy_batch=128,
              seed=0, json_sweep=(), npy_sweep=(), sweep_seconds=2.0):
    """Serve ``pred`` on the native front end and measure it with httpload; returns a dict of phases.
    ``json_sweep`` / ``npy_sweep``: further client counts, each its own closed-loop phase (where the front end
    saturates against the device rate).  Every phase carries the server's own per-batch timeline
    (NativePredictorServer.batch_timing) next to the client's latencies."""
    from ..container.container_manager import free_port
    from .nativeserve import NativePredictorServer
    if not available():
        raise RuntimeError('httpload is not built (python -m rafiki_amd._build)')
    rng = np.random.default_rng(seed)
    one = rng.integers(0, 255, image_shape).tolist()   # (255 is the test stand-in predictor's poison value)
    batch = rng.integers(0, 255, (npy_batch,) + tuple(image_shape), dtype=np.uint8)
    buf = io.BytesIO()
    np.save(buf, batch, allow_pickle=False)
    port = free_port()
    srv = NativePredictorServer(pred, '127.0.0.1', port).start()
    try:
        warm = json.dumps({'query': one}).encode()
        run_httpload(port, '/predict', warm, 8, 2, 0.5)   # graphs / buckets warm before the timed phases
        npy = buf.getvalue()

        def phase(path, body, clients, secs, per_request=1):
            srv.reset_timing()
            c0 = srv.counters
            r = dict(run_httpload(port, path, body, clients, 4, secs, per_request=per_request), clients=clients)
            c1 = srv.counters
            nb = c1.get('batches', 0) - c0.get('batches', 0)
            r['mean_batch'] = round((c1.get('batched_queries', 0) - c0.get('batched_queries', 0)) / max(1, nb), 1)
            r['server_batches'] = srv.batch_timing()
            return r
        out = {'server': 'native', 'client': 'httpload (separate process, keep-alive, closed loop)',
               'json_single_query': phase('/predict', warm, json_clients, seconds),
               'npy_batch{}'.format(npy_batch): phase('/predict_batch_npy', npy, npy_clients, seconds,
                                                      per_request=npy_batch)}
        if json_sweep:
            out['json_sweep'] = [phase('/predict', warm, k, sweep_seconds) for k in json_sweep]
        if npy_sweep:
            out['npy_sweep'] = [phase('/predict_batch_npy', npy, k, sweep_seconds, per_request=npy_batch)
                                for k in npy_sweep]
        c = getattr(srv, 'counters', {})
        out['server_counters'] = {k: c[k] for k in ('requests', 'batches', 'batched_queries') if k in c}
        return out
    finally:
        srv.shutdown()
