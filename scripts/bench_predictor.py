"""Predictor ensemble QPS benchmark (BASELINE config #4: top-4 trained CNNs batched on 1 MI355X,
hipGraph forwards).

Four VGG-small models (random init, the BASELINE architecture; weights do not change the cost)
are loaded into one in-process ``Predictor`` on cuda:0.  Three measurements:

* ``device``: a uint8 query batch already in HBM -> 4 hipGraph-captured forwards on 4 HIP streams
  -> on-device ensemble mean; QPS per batch size (the serving ceiling of the GPU path);
* ``api``: ``Predictor.predict(list-of-lists queries)`` — the JSON-shaped path of POST
  /predict_batch: host decode, one pinned upload, ensemble, ``tolist()``;
* ``batcher``: C concurrent clients each calling ``predict_one`` (dynamic batcher, max_wait 2 ms)
  -> QPS and p50/p99 latency — the POST /predict path without HTTP.

Reference analogue: <=128 QPS per inference worker with a >=0.25 s latency floor
(Redis polling).  Prints one JSON line; ``--out`` also writes it to a file.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build_models(k, device, classes=10):
    from rafiki_amd.models.vgg_small import VggSmall
    models = []
    for i in range(k):
        m = VggSmall(epochs=1, learning_rate=0.05, momentum=0.9, weight_decay=5e-4, batch_size=128, width_mult=1.0,
                     image_size=32, seed=i)
        m.device = device
        m._build(classes, 3)
        m._engine.prepare_eval()
        models.append(('trial{}'.format(i), m))
    return models


def timed(fn, iters):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t


def _client_proc(url, kind, threads, seconds, q, payload):
    """Load generator process: ``threads`` keep-alive connections, each sending one request at a time.
    json1: pre-encoded single-query JSON bodies over a raw socket (the client must not be the
    bottleneck: requests + json.dumps of 3072 ints costs ~1 ms per call); npy: batch bodies."""
    import socket
    host, port = url.split('//')[1].split(':')
    port = int(port)
    if kind == 'json1':
        body = json.dumps({'query': payload}).encode()
        path, per = b'/predict', 1
    else:
        body, path, per = payload, b'/predict_batch_npy', 128
    req = b'POST %s HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n' % (path, len(body)) + body
    stop = threading.Event()
    counts = [0] * threads
    lats = [[] for _ in range(threads)]

    def worker(i):
        s = socket.create_connection((host, port))
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        buf = b''
        while not stop.is_set():
            t = time.perf_counter()
            s.sendall(req)
            while True:
                h = buf.find(b'\r\n\r\n')
                if h >= 0:
                    head = buf[:h].lower()
                    cl = int(head.split(b'content-length:')[1].split(b'\r\n')[0])
                    if len(buf) >= h + 4 + cl:
                        if not buf.startswith(b'HTTP/1.1 200'):
                            raise RuntimeError(buf[:200])
                        buf = buf[h + 4 + cl:]
                        break
                buf += s.recv(1 << 16)
            lats[i].append(time.perf_counter() - t)
            counts[i] += per
        s.close()
    ths = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for t in ths:
        t.start()
    time.sleep(seconds)
    stop.set()
    for t in ths:
        t.join()
    q.put((sum(counts), [x for lst in lats for x in lst]))


def http_bench(pred, rng, args, server='fast'):
    import io
    from rafiki_amd.container.container_manager import free_port
    port = free_port()
    if server == 'native':
        from rafiki_amd.predictor.nativeserve import NativePredictorServer
        srv = NativePredictorServer(pred, '127.0.0.1', port).start()
    elif server == 'fast':
        from rafiki_amd.predictor.fastserve import FastPredictorServer
        srv = FastPredictorServer(pred, '127.0.0.1', port).start()
    else:
        from werkzeug.serving import make_server
        from rafiki_amd.predictor.server import create_app
        srv = make_server('127.0.0.1', port, create_app(pred), threaded=True)
        threading.Thread(target=srv.serve_forever, daemon=True).start()
    url = 'http://127.0.0.1:{}'.format(port)
    out = {}
    one = rng.integers(0, 256, (32, 32, 3)).tolist()
    batch = rng.integers(0, 256, (128, 32, 32, 3), dtype=np.uint8)
    buf = io.BytesIO()
    np.save(buf, batch, allow_pickle=False)
    body = npy_body = buf.getvalue()

    httpload = os.path.join(ROOT, 'rafiki_amd', '_native', 'httpload')

    def run(kind, procs, threads, seconds=4.0):
        """Load from outside the server's process: the native closed-loop generator (csrc/tools/
        httpload.cpp, ~microseconds per request) when built, else Python client processes (a load
        generator sharing the server's GIL would measure itself)."""
        if os.path.exists(httpload):
            import subprocess
            import tempfile
            body = json.dumps({'query': one}).encode() if kind == 'json1' else npy_body
            with tempfile.NamedTemporaryFile(suffix='.body') as bf:
                bf.write(body)
                bf.flush()
                r = subprocess.run([httpload, '127.0.0.1', str(port), '/predict' if kind == 'json1' else
                                    '/predict_batch_npy', bf.name, str(procs * threads), str(min(4, procs)),
                                    str(seconds)], capture_output=True, text=True, timeout=seconds + 60)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            per = 1 if kind == 'json1' else 128
            return {'qps': round(d['qps'] * per, 1), 'p50_ms': d['p50_ms'], 'p99_ms': d['p99_ms'],
                    'errors': d['errors'], 'client': 'httpload'}
        import multiprocessing as mproc
        ctx = mproc.get_context('spawn')
        q = ctx.Queue()
        ps = [ctx.Process(target=_client_proc, args=(url, kind, threads, seconds, q, one if kind == 'json1' else body))
              for _ in range(procs)]
        for p in ps:
            p.start()
        got = [q.get(timeout=120) for _ in ps]
        for p in ps:
            p.join(30)
        lat = np.array([x for _, lst in got for x in lst]) * 1e3
        return {'qps': round(sum(n for n, _ in got) / seconds, 1),
                'p50_ms': round(float(np.percentile(lat, 50)), 3), 'p99_ms': round(float(np.percentile(lat, 99)), 3)}
    pred.start()
    out['json_single_query_64clients'] = run('json1', 8, 8)
    out['npy_batch128_8clients'] = run('npy', 4, 2)
    if server != 'flask':
        out['json_single_query_256clients'] = run('json1', 16, 16)
    if hasattr(srv, 'counters'):
        c = srv.counters
        out['server_counters'] = {k: c[k] for k in ('requests', 'batches', 'batched_queries') if k in c}
    srv.shutdown()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--models', type=int, default=4)
    ap.add_argument('--batches', default='1,8,32,128,512')
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--clients', type=int, default=64)
    ap.add_argument('--seconds', type=float, default=5.0)
    ap.add_argument('--replicas', type=int, default=1)
    ap.add_argument('--skip-http', action='store_true')
    ap.add_argument('--flask', action='store_true', help='also measure the Flask app')
    ap.add_argument('--skip-http-asyncio', action='store_true')
    ap.add_argument('--out', default='')
    args = ap.parse_args()
    from rafiki_amd.ops import _lib
    from rafiki_amd.predictor.predictor import Predictor
    _lib.lib()
    dev = torch.device('cuda', 0)
    models = build_models(args.models, dev)
    pred = Predictor(models, max_batch=512, max_wait_ms=2.0,
                     replicas=[build_models(args.models, dev) for _ in range(args.replicas - 1)])
    rng = np.random.default_rng(0)
    res = {'metric': 'predictor ensemble QPS (top-{} VGG-small 32x32x3, 1 GPU)'.format(args.models),
           'n_models': args.models, 'replicas': args.replicas, 'device': {}, 'api': {},
           'dtype': models[0][1]._meta.get('dtype'), 'data': 'synthetic, random-init',
           'ensemble_graph': os.environ.get('RAFIKI_ENSEMBLE_GRAPH', '1') != '0'}
    sig = models[0][1].input_signature()
    for b in [int(x) for x in args.batches.split(',')]:
        imgs = torch.from_numpy(rng.integers(0, 256, (b, 32, 32, 3), dtype=np.uint8)).to(dev)
        inputs = {sig: imgs}
        for _ in range(3):
            pred.predict_proba_device(inputs)
        dt = timed(lambda: pred.predict_proba_device(inputs), args.iters)
        res['device'][b] = {'qps': round(b * args.iters / dt, 1), 'ms_per_batch': round(1e3 * dt / args.iters, 3)}
        q = rng.integers(0, 256, (b, 32, 32, 3)).tolist()
        pred.predict(q)
        it = max(3, args.iters // 5)
        dt = timed(lambda: pred.predict(q), it)
        res['api'][b] = {'qps': round(b * it / dt, 1), 'ms_per_batch': round(1e3 * dt / it, 3)}
    # numpy batches straight into the device path (what POST /predict_batch_npy does)
    res['array'] = {}
    for b in (128, 512):
        arr = rng.integers(0, 256, (b, 32, 32, 3), dtype=np.uint8)
        pred.predict_array(arr)
        it = max(3, args.iters // 5)
        dt = timed(lambda: pred.predict_array(arr), it)
        res['array'][b] = {'qps': round(b * it / dt, 1), 'ms_per_batch': round(1e3 * dt / it, 3)}
    # real HTTP: the predictor's Flask app on a local port, concurrent clients
    if not args.skip_http:
        res['http_native'] = http_bench(pred, rng, args, 'native')
        if not args.skip_http_asyncio:
            res['http_asyncio'] = http_bench(pred, rng, args, 'fast')
        if args.flask:
            res['http_flask'] = http_bench(pred, rng, args, 'flask')
    # dynamic batcher under concurrent single-query clients
    pred.start()
    one = rng.integers(0, 256, (32, 32, 3)).tolist()
    for _ in range(20):
        pred.predict_one(one)
    lat, stop = [], threading.Event()
    lock = threading.Lock()

    def client():
        mine = []
        while not stop.is_set():
            t = time.perf_counter()
            pred.predict_one(one)
            mine.append(time.perf_counter() - t)
        with lock:
            lat.extend(mine)
    ths = [threading.Thread(target=client) for _ in range(args.clients)]
    q0, b0 = pred.stats['queries'], pred.stats['batches']
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    time.sleep(args.seconds)
    stop.set()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    nq = pred.stats['queries'] - q0
    pred.stop()
    lat_ms = np.array(lat) * 1e3
    res['batcher'] = {'clients': args.clients, 'qps': round(nq / el, 1), 'p50_ms': round(float(np.percentile(lat_ms, 50)), 2),
                      'p99_ms': round(float(np.percentile(lat_ms, 99)), 2),
                      'mean_batch': round(nq / max(1, pred.stats['batches'] - b0), 1)}
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, 'w') as f:
            f.write(line + '\n')


if __name__ == '__main__':
    main()
