"""Query/prediction queues between the predictor and inference workers — the reference's Redis
``Cache`` (rafiki/cache/cache.py:10-81) with the same methods, on node-local shared memory.

* per inference worker: a query queue ``rkq_<worker>`` and a prediction queue ``rkp_<worker>``
  (native shared-memory rings, csrc/runtime/mq.cpp); messages are JSON ``{id, query}`` /
  ``{id, prediction}`` like the reference's;
* the set of running workers of an inference job is a small registry file under the workdir
  (replacing ``SADD/SREM/SMEMBERS INFERENCE_WORKERS_<job>``);
* ``pop_prediction_of_worker(worker, query_id)`` drains the worker's prediction queue into a local
  map and returns the wanted one — atomic per message, so no prediction is ever dropped (reference
  bug: ``LTRIM key i+1 i`` emptied the whole list).
"""
from __future__ import annotations

import json
import os
import threading
from typing import Dict, List, Optional

from .mq import MessageQueue


def _qname(kind, worker_id):
    return 'rk{}_{}'.format(kind, ''.join(c for c in str(worker_id) if c.isalnum())[:48])


MISSING = object()  # "no prediction yet" (a worker may legitimately answer None for a failed query)


class Cache:
    def __init__(self, workdir: Optional[str] = None, capacity: int = 64 << 20):
        from ..config import get_config
        self.workdir = workdir or get_config().workdir
        self.capacity = capacity
        self._queues: Dict[str, MessageQueue] = {}
        self._preds: Dict[str, Dict[str, object]] = {}
        self._lock = threading.Lock()

    # ------------------------------------------------------------- workers of inference job
    def _reg_path(self, inference_job_id):
        d = os.path.join(self.workdir, 'cache')
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, 'inference_workers_{}.json'.format(inference_job_id))

    def _update_reg(self, inference_job_id, fn):
        import fcntl
        path = self._reg_path(inference_job_id)
        with open(path + '.lock', 'a') as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                cur = json.load(open(path)) if os.path.exists(path) else []
            except ValueError:
                cur = []
            new = fn(cur)
            tmp = path + '.tmp'
            with open(tmp, 'w') as f:
                json.dump(new, f)
            os.replace(tmp, path)
            fcntl.flock(lk, fcntl.LOCK_UN)
        return new

    def add_worker_of_inference_job(self, worker_id, inference_job_id):
        self._update_reg(inference_job_id, lambda c: c if worker_id in c else c + [worker_id])

    def delete_worker_of_inference_job(self, worker_id, inference_job_id):
        self._update_reg(inference_job_id, lambda c: [w for w in c if w != worker_id])

    def get_workers_of_inference_job(self, inference_job_id) -> List[str]:
        path = self._reg_path(inference_job_id)
        try:
            with open(path) as f:
                return list(json.load(f))
        except (OSError, ValueError):
            return []

    # ------------------------------------------------------------------------- queues
    def _q(self, kind, worker_id) -> MessageQueue:
        name = _qname(kind, worker_id)
        with self._lock:
            q = self._queues.get(name)
            if q is None:
                q = self._queues[name] = MessageQueue(name, self.capacity, create=True)
            return q

    def add_query_of_worker(self, worker_id, query_id, query):
        return self._q('q', worker_id).push(json.dumps({'id': query_id, 'query': query}).encode())

    def add_queries_of_worker(self, worker_id, items):
        """Batched form: one message carrying [(query_id, query), ...]."""
        return self._q('q', worker_id).push(json.dumps({'batch': [[i, q] for i, q in items]}).encode())

    def pop_queries_of_worker(self, worker_id, batch_size, timeout_ms=250):
        """-> (query_ids, queries); waits up to timeout_ms for the first message only."""
        q = self._q('q', worker_id)
        ids, queries = [], []
        first = True
        while len(ids) < batch_size:
            m = q.pop(timeout_ms if first else 0)
            first = False
            if m is None:
                break
            d = json.loads(m)
            if 'batch' in d:
                for i, x in d['batch']:
                    ids.append(i)
                    queries.append(x)
            else:
                ids.append(d['id'])
                queries.append(d['query'])
        return ids, queries

    def add_prediction_of_worker(self, worker_id, query_id, prediction):
        return self._q('p', worker_id).push(json.dumps({'id': query_id, 'prediction': prediction}).encode())

    def add_predictions_of_worker(self, worker_id, items):
        return self._q('p', worker_id).push(json.dumps({'batch': [[i, p] for i, p in items]}).encode())

    def pop_prediction_of_worker(self, worker_id, query_id, timeout_ms=0):
        """-> the prediction, or ``MISSING`` if it has not arrived within timeout_ms."""
        q = self._q('p', worker_id)
        got = self._preds.setdefault(worker_id, {})
        if query_id in got:
            return got.pop(query_id)
        wait = timeout_ms
        while True:
            m = q.pop(wait)
            if m is None:
                return MISSING
            wait = 0
            d = json.loads(m)
            for i, p in (d['batch'] if 'batch' in d else [[d['id'], d['prediction']]]):
                got[i] = p
            if query_id in got:
                return got.pop(query_id)

    def clear_worker(self, worker_id):
        for kind in ('q', 'p'):
            name = _qname(kind, worker_id)
            with self._lock:
                q = self._queues.pop(name, None)
            if q is None:
                q = MessageQueue(name, self.capacity, create=True)
            q.close()
            q.unlink()
        self._preds.pop(worker_id, None)
