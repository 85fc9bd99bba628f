"""The event-loop predictor front end (rafiki_amd.predictor.fastserve) against a numpy stand-in
predictor: wire contract of the reference predictor app (POST /predict {query} -> {prediction}),
keep-alive and Connection: close, batching of concurrent single queries, errors as HTTP 500."""
import io
import threading

import numpy as np
import pytest
import requests


class FakeCache:
    used = 0


class FakePredictor:
    def __init__(self):
        self.models = [('a', None), ('b', None)]
        self.stats = {'queries': 0}
        self.cache = FakeCache()
        self.batch_sizes = []
        self.lock = threading.Lock()

    def _fast_path(self):
        return True

    def _probs(self, arr):
        s = arr.reshape(len(arr), -1).astype(np.float64).sum(1)
        return np.stack([s % 7, s % 5, s % 3], 1).astype(np.float32)

    def predict_array(self, arr):
        arr = np.asarray(arr)
        if arr.reshape(len(arr), -1).max(initial=0) == 255:
            raise ValueError('poisoned query')
        with self.lock:
            self.batch_sizes.append(len(arr))
        return self._probs(arr)

    def predict(self, queries):
        return [self._probs(np.asarray([q], dtype=np.uint8))[0].tolist() for q in queries]


@pytest.fixture(params=['fast', 'native'])
def server(request):
    """Both front ends: asyncio (fastserve) and the C++ epoll server (nativeserve)."""
    fake = FakePredictor()
    if request.param == 'native':
        from rafiki_amd.predictor import nativeserve
        if not nativeserve.available():
            pytest.skip('librafiki_runtime.so not built')
        srv = nativeserve.NativePredictorServer(fake, '127.0.0.1', 0).start()
    else:
        from rafiki_amd.predictor.fastserve import FastPredictorServer
        srv = FastPredictorServer(fake, '127.0.0.1', 0).start()
    yield srv, fake, 'http://127.0.0.1:{}'.format(srv.port)
    srv.shutdown()


def test_single_and_batch_contract(server):
    srv, fake, url = server
    assert requests.get(url + '/').text == 'Rafiki Predictor is up.'
    q = np.arange(12, dtype=np.uint8).reshape(3, 4)
    r = requests.post(url + '/predict', json={'query': q.tolist()})
    assert r.status_code == 200 and r.json()['prediction'] == fake._probs(q[None])[0].tolist()
    qs = np.arange(24, dtype=np.uint8).reshape(2, 3, 4)
    r = requests.post(url + '/predict_batch', json={'queries': qs.tolist()})
    assert np.allclose(r.json()['predictions'], fake._probs(qs))
    buf = io.BytesIO()
    np.save(buf, qs, allow_pickle=False)
    r = requests.post(url + '/predict_batch_npy', data=buf.getvalue())
    assert np.allclose(np.load(io.BytesIO(r.content)), fake._probs(qs))
    # non-image query (e.g. POS tokens) goes through predict()
    r = requests.post(url + '/predict', json={'query': [[1, 2], [3, 4]]})
    assert r.status_code == 200
    assert requests.get(url + '/nope').status_code == 404
    assert requests.get(url + '/predict').status_code == 405
    assert requests.get(url + '/stats').json()['server']['requests'] >= 5
    assert 'rafiki_predictor_requests' in requests.get(url + '/metrics').text


def test_errors_are_500_and_connection_close(server):
    srv, fake, url = server
    bad = np.full((2, 2), 255, dtype=np.uint8).tolist()
    r = requests.post(url + '/predict', json={'query': bad})
    assert r.status_code == 500 and 'poisoned query' in r.text
    r = requests.post(url + '/predict', json={'query': [[1, 2]]}, headers={'Connection': 'close'})
    assert r.status_code == 200 and r.headers.get('Connection', '').lower() == 'close'


def test_concurrent_single_queries_are_batched(server):
    srv, fake, url = server
    rng = np.random.default_rng(0)
    qs = rng.integers(0, 200, (96, 4, 4), dtype=np.uint8)
    out = [None] * len(qs)

    def client(lo, hi):
        s = requests.Session()
        for i in range(lo, hi):
            out[i] = s.post(url + '/predict', json={'query': qs[i].tolist()}).json()['prediction']
    ts = [threading.Thread(target=client, args=(k * 12, (k + 1) * 12)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert np.allclose(np.asarray(out), fake._probs(qs))
    assert sum(fake.batch_sizes) == 96 and len(fake.batch_sizes) < 96   # stacked into batches


def test_bad_and_oversized_content_length(server):
    """Content-Length is validated before any body byte is buffered (400 / 413)."""
    import socket
    srv, fake, url = server
    for hdr, code in ((b'Content-Length: -5', b'400'), (b'Content-Length: abc', b'400'),
                      (b'Content-Length: 99999999999', b'413')):
        s = socket.create_connection(('127.0.0.1', srv.port), timeout=10)
        s.sendall(b'POST /predict HTTP/1.1\r\nHost: x\r\n' + hdr + b'\r\n\r\n')
        resp = s.recv(4096)
        s.close()
        assert resp.split(b' ')[1] == code, resp
    assert requests.get(url + '/').status_code == 200   # server still serving


def test_native_single_query_latency_with_idle_generic_thread():
    """An image query must wake a batch thread at once even while the generic thread waits on its own
    queue (one shared condition variable let notify_one wake the wrong waiter: ~100 ms stalls)."""
    import time
    from rafiki_amd.predictor import nativeserve
    if not nativeserve.available():
        pytest.skip('librafiki_runtime.so not built')
    fake = FakePredictor()
    srv = nativeserve.NativePredictorServer(fake, '127.0.0.1', 0).start()
    try:
        url = 'http://127.0.0.1:{}/predict'.format(srv.port)
        s = requests.Session()
        s.post(url, json={'query': [[1, 2], [3, 4]]}).raise_for_status()
        worst = 0.0
        for i in range(20):
            time.sleep(0.02)   # let every waiter go back to sleep
            t = time.perf_counter()
            r = s.post(url, json={'query': [[i, 2], [3, 4]]})
            worst = max(worst, time.perf_counter() - t)
            assert r.status_code == 200
        assert worst < 0.05, worst
    finally:
        srv.shutdown()


def test_native_oversized_query_takes_the_generic_path(monkeypatch):
    """A query larger than the batch path's per-query limit is served by the generic (Python) path
    instead of growing the replica's batch buffer without bound."""
    from rafiki_amd.predictor import nativeserve
    if not nativeserve.available():
        pytest.skip('librafiki_runtime.so not built')
    monkeypatch.setattr(nativeserve, 'MAX_QUERY', 64)
    fake = FakePredictor()
    srv = nativeserve.NativePredictorServer(fake, '127.0.0.1', 0).start()
    try:
        url = 'http://127.0.0.1:{}/predict'.format(srv.port)
        big = np.arange(100, dtype=np.uint8).reshape(10, 10).tolist()
        r = requests.post(url, json={'query': big})
        assert r.status_code == 200
        assert np.allclose(r.json()['prediction'], fake._probs(np.asarray([big], dtype=np.uint8))[0])
        c = srv.counters
        assert c['generic_requests'] == 1 and c['batched_queries'] == 0   # the generic path, not the batch path
        small = requests.post(url, json={'query': [[1, 2], [3, 4]]})
        assert small.status_code == 200 and srv.counters['batched_queries'] == 1
    finally:
        srv.shutdown()


def _npy(a):
    buf = io.BytesIO()
    np.save(buf, a, allow_pickle=False)
    return buf.getvalue()


def test_native_npy_batches_join_the_image_queue():
    """POST /predict_batch_npy with a uint8 body is decoded in C++ and batched with concurrent JSON
    queries of the same image shape (one predict_array call can serve both); the reply is an .npy
    float32 array.  Non-uint8 arrays and batches above max_batch take the generic Python path."""
    from rafiki_amd.predictor import nativeserve
    if not nativeserve.available():
        pytest.skip('librafiki_runtime.so not built')
    fake = FakePredictor()
    srv = nativeserve.NativePredictorServer(fake, '127.0.0.1', 0, max_batch=64).start()
    try:
        url = 'http://127.0.0.1:{}'.format(srv.port)
        rng = np.random.default_rng(1)
        qs = rng.integers(0, 200, (40, 3, 4), dtype=np.uint8)
        r = requests.post(url + '/predict_batch_npy', data=_npy(qs))
        assert r.status_code == 200 and r.headers['Content-Type'] == 'application/octet-stream'
        got = np.load(io.BytesIO(r.content), allow_pickle=False)
        assert got.dtype == np.float32 and np.array_equal(got, fake._probs(qs))
        assert srv.counters['batched_queries'] == 40 and srv.counters['generic_requests'] == 0
        # many npy batches and single JSON queries at once: every reply is its own slice
        out, errs = {}, []

        def npy_client(k):
            try:
                s = requests.Session()
                for j in range(4):
                    a = qs[(k + j) % 8 * 5:(k + j) % 8 * 5 + 5]
                    out[('n', k, j)] = (np.load(io.BytesIO(s.post(url + '/predict_batch_npy', data=_npy(a)).content)),
                                        fake._probs(a))
            except Exception as e:
                errs.append(e)

        def json_client(k):
            try:
                s = requests.Session()
                for j in range(6):
                    q = qs[(k * 6 + j) % 40]
                    out[('j', k, j)] = (np.asarray(s.post(url + '/predict', json={'query': q.tolist()}).json()
                                                   ['prediction']), fake._probs(q[None])[0])
            except Exception as e:
                errs.append(e)
        ts = [threading.Thread(target=npy_client, args=(k,)) for k in range(4)] + \
             [threading.Thread(target=json_client, args=(k,)) for k in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert not errs, errs
        assert len(out) == 4 * 4 + 4 * 6
        for got, want in out.values():
            assert np.allclose(got, want)
        g0 = srv.counters['generic_requests']
        # float32 npy: generic path (np.load + predict_array), same wire format
        r = requests.post(url + '/predict_batch_npy', data=_npy(qs[:3].astype(np.float32)))
        assert r.status_code == 200 and np.allclose(np.load(io.BytesIO(r.content)), fake._probs(qs[:3]))
        # above max_batch images: generic path
        big = rng.integers(0, 200, (70, 3, 4), dtype=np.uint8)
        r = requests.post(url + '/predict_batch_npy', data=_npy(big))
        assert r.status_code == 200 and np.allclose(np.load(io.BytesIO(r.content)), fake._probs(big))
        assert srv.counters['generic_requests'] == g0 + 2
        # a poisoned npy batch fails as a whole with 500, the server keeps serving
        bad = qs[:2].copy()
        bad[1, 0, 0] = 255
        assert requests.post(url + '/predict_batch_npy', data=_npy(bad)).status_code == 500
        assert requests.post(url + '/predict', json={'query': qs[0].tolist()}).status_code == 200
    finally:
        srv.shutdown()


def _raw_npy_header(shape_text):
    hd = "{'descr': '|u1', 'fortran_order': False, 'shape': %s, }" % shape_text
    total = (10 + len(hd) + 1 + 63) // 64 * 64
    hd = hd + ' ' * (total - 10 - len(hd) - 1) + '\n'
    return b'\x93NUMPY\x01\x00' + bytes([len(hd) & 255, len(hd) >> 8]) + hd.encode('latin-1')


def test_native_npy_overflowing_shape_is_rejected_and_server_keeps_serving():
    """A .npy header whose dims multiply past int64 (and an empty data section) must not be accepted as
    a batch: the C++ decoder rejects it (checked before every multiply), the request is answered with
    an error, and later queries are still served (the replica's batch thread is alive)."""
    from rafiki_amd.predictor import nativeserve
    if not nativeserve.available():
        pytest.skip('librafiki_runtime.so not built')
    fake = FakePredictor()
    srv = nativeserve.NativePredictorServer(fake, '127.0.0.1', 0, max_batch=64).start()
    try:
        url = 'http://127.0.0.1:{}'.format(srv.port)
        for shape in ('(1, %d, %d)' % (2 ** 40, 2 ** 24), '(%d, %d, %d)' % (2 ** 40, 2 ** 40, 2 ** 40),
                      '(0, 3, 4)', '(2, 3, 4)'):
            r = requests.post(url + '/predict_batch_npy', data=_raw_npy_header(shape), timeout=30)
            assert r.status_code in (400, 500), (shape, r.status_code)
        q = np.arange(12, dtype=np.uint8).reshape(3, 4)
        r = requests.post(url + '/predict', json={'query': q.tolist()}, timeout=30)
        assert r.status_code == 200 and np.allclose(r.json()['prediction'], fake._probs(q[None])[0])
        r = requests.post(url + '/predict_batch_npy', data=_npy(q[None].repeat(5, 0)), timeout=30)
        assert r.status_code == 200 and np.load(io.BytesIO(r.content)).shape == (5, 3)
    finally:
        srv.shutdown()


def test_loadgen_measures_the_native_front_end():
    """bench.py's HTTP phase (predictor/loadgen.py): the native server over a predictor, driven by the
    separate httpload process — JSON single queries and .npy batches, QPS in queries, no errors."""
    from rafiki_amd.predictor import loadgen, nativeserve
    if not (nativeserve.available() and loadgen.available()):
        pytest.skip('native runtime / httpload not built')
    fake = FakePredictor()
    out = loadgen.http_load(fake, image_shape=(3, 4), seconds=0.5, json_clients=8, npy_clients=2, npy_batch=16)
    js, nb = out['json_single_query'], out['npy_batch16']
    assert js['errors'] == 0 and nb['errors'] == 0 and js['qps'] > 0 and nb['qps'] > 0
    assert nb['qps'] == pytest.approx(16 * nb['requests_per_s'], rel=1e-3)
    assert js['p99_ms'] >= js['p50_ms'] > 0
    assert out['server_counters']['batched_queries'] > 0
