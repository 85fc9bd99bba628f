"""Predictor replicas and the resident (in-HBM) model store, on CPU with stand-in models."""
import threading
import time

import numpy as np
import torch

from rafiki_amd.constants import TaskType


class SlowModel:
    """predict() sleeps so concurrent requests overlap; records which thread served it."""

    def __init__(self, bias):
        self.bias = bias
        self.calls = 0
        self.lock = threading.Lock()

    def predict(self, queries):
        with self.lock:
            self.calls += 1
        time.sleep(0.02)
        return [[float(q[0]) + self.bias, 1.0] for q in queries]


def _predictor(replicas=2):
    from rafiki_amd.predictor.predictor import Predictor
    sets = [[('a', SlowModel(0.0)), ('b', SlowModel(1.0))] for _ in range(replicas)]
    return Predictor(sets[0], task=TaskType.IMAGE_CLASSIFICATION, replicas=sets[1:]), sets


def test_requests_spread_over_replicas_and_ensemble_is_correct():
    p, sets = _predictor(2)
    out = {}

    def worker(k):
        out[k] = p.predict([[k], [k + 0.5]])
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for k, v in out.items():
        assert np.allclose(v, [[k + 0.5, 1.0], [k + 1.0, 1.0]])
    served = [r.served for r in p.replicas]
    assert sum(served) == 8 and min(served) >= 2, served
    assert all(m.calls > 0 for s in sets for _, m in s)


def test_batcher_runs_one_consumer_per_replica():
    p, _ = _predictor(3)
    p.max_wait_s, p.max_batch = 0.0, 4
    p.start()
    try:
        assert len(p._threads) == 3
        futs = [p.submit([i]) for i in range(30)]
        res = [f.result(timeout=10) for f in futs]
        assert np.allclose([r[0] for r in res], [i + 0.5 for i in range(30)])
        assert sum(1 for r in p.replicas if r.served) >= 2
    finally:
        p.stop()


def test_replicas_must_hold_the_same_trials():
    import pytest
    from rafiki_amd.predictor.predictor import Predictor
    with pytest.raises(ValueError):
        Predictor([('a', SlowModel(0))], replicas=[[('b', SlowModel(0))]])


class FakeResident:
    def __init__(self, nbytes):
        self.device = torch.device('cuda', 0)
        self.nbytes = nbytes
        self.released = self.destroyed = False

    def resident_bytes(self):
        return self.nbytes

    def release_training(self):
        self.released = True

    def destroy(self):
        self.destroyed = True


def test_resident_store_keeps_best_models_within_budget():
    from rafiki_amd.predictor.resident import ResidentStore
    st = ResidentStore(budget_bytes=100)
    a, b, c, d = FakeResident(40), FakeResident(40), FakeResident(40), FakeResident(200)
    assert st.offer('a', a, 0.5) and a.released
    assert st.offer('b', b, 0.7)
    assert st.offer('c', c, 0.9)          # evicts the worst (a)
    assert a.destroyed and 'a' not in st and 'b' in st and 'c' in st
    assert not st.offer('x', FakeResident(40), 0.1)   # never evicts a better model
    assert not st.offer('d', d, 1.0)      # larger than the whole budget
    assert st.take('c') is c and st.take('c') is None
    assert st.hits == 1 and st.misses == 1
    cpu_model = FakeResident(10)
    cpu_model.device = torch.device('cpu')
    assert not st.offer('cpu', cpu_model, 1.0)        # host models are not held
    st.clear()
    assert b.destroyed and st.used == 0
