"""Predictor: top-k trained models resident on ONE GPU, dynamic batching, on-device ensembling.

Reference parity: rafiki/predictor/predictor.py (``Predictor.predict`` :31-74) + inference
workers (worker/inference.py:31-93) + Redis queues (cache/cache.py).  The reference fans every
query out through Redis lists to one container per model and polls for answers every 0.25 s
(≥0.25-0.5 s latency floor, ≤128 QPS per worker).  Here:
  * all top-k models live in this process on one MI355X (288 GB HBM holds thousands of such
    models); ``ParamCache`` accounts their bytes;
  * requests go through a lock-free-ish in-process queue into a dynamic batcher (up to
    ``max_batch`` queries or ``max_wait_ms``), replacing Redis + polling;
  * models exposing ``predict_proba(queries) -> Tensor[Q, C]`` (the native zoo: hipGraph-captured
    bucketed forwards) run on their own HIP streams and are ensembled by the gfx950
    ensemble-mean kernel; any other BaseModel falls back to ``predict()`` + host ensembling;
  * every request has a timeout (reference bug (g)); a model that fails is dropped from that
    batch's ensemble (partial-ensemble fallback) instead of hanging the request.
"""
from __future__ import annotations

import logging
import os
import pickle
import queue
import threading
import time
import traceback
from concurrent.futures import Future
from typing import List, Optional, Tuple

from .. import config
from ..constants import TaskType
from .ensemble import ensemble_predictions, ensemble_probabilities

logger = logging.getLogger(__name__)


class ParamCache:
    """Byte-budgeted registry of resident models (LRU eviction beyond the budget)."""

    def __init__(self, budget_bytes: float):
        self.budget = float(budget_bytes)
        self._items = {}
        self._order = []
        self._lock = threading.Lock()

    @staticmethod
    def model_bytes(model) -> int:
        fn = getattr(model, 'resident_bytes', None)
        return int(fn()) if callable(fn) else 0

    def put(self, key, model):
        with self._lock:
            self._items[key] = (model, self.model_bytes(model))
            if key in self._order:
                self._order.remove(key)
            self._order.append(key)
            evicted = []
            while self.used > self.budget and len(self._order) > 1:
                k = self._order.pop(0)
                evicted.append(self._items.pop(k)[0])
            return evicted

    def get(self, key):
        with self._lock:
            v = self._items.get(key)
            return None if v is None else v[0]

    @property
    def used(self):
        return sum(b for _, b in self._items.values())

    def keys(self):
        return list(self._order)


class RemoteWorkerModel:
    """Proxy for a model served by an ``InferenceWorker`` process (``workers`` serving mode)."""

    def __init__(self, worker_id, cache):
        self.worker_id = worker_id
        self.cache = cache

    def submit(self, ids, queries):
        self.cache.add_queries_of_worker(self.worker_id, list(zip(ids, queries)))

    def collect(self, ids, deadline):
        from ..cache.cache import MISSING
        out = []
        for i in ids:
            while True:
                left_ms = int((deadline - time.perf_counter()) * 1000)
                p = self.cache.pop_prediction_of_worker(self.worker_id, i, timeout_ms=max(0, min(left_ms, 200)))
                if p is not MISSING or left_ms <= 0:
                    break
            if p is MISSING:
                raise TimeoutError('worker {} did not answer in time'.format(self.worker_id))
            out.append(p)
        return out


class Predictor:
    def __init__(self, models: Optional[List[Tuple[str, object]]] = None, task=TaskType.IMAGE_CLASSIFICATION,
                 max_batch: int = 256, max_wait_ms: float = 2.0, timeout_s: float = None,
                 weights: Optional[List[float]] = None):
        self.task = task
        self.models = list(models or [])
        self.max_batch = max_batch
        self.max_wait_s = max_wait_ms / 1000.0
        self.timeout_s = timeout_s or config.PREDICTOR_TIMEOUT_S
        self.weights = weights
        self.cache = ParamCache(config.get_config().node.param_cache_gb * 1e9)
        for name, m in self.models:
            self.cache.put(name, m)
        self._q: "queue.Queue" = queue.Queue()
        self._thread = None
        self._stop = threading.Event()
        self._streams = None
        self.stats = {'batches': 0, 'queries': 0, 'errors': 0}

    # ------------------------------------------------------------------ loading from the DB
    @classmethod
    def from_inference_job(cls, inference_job_id, db=None, **kw):
        if os.environ.get('RAFIKI_INFERENCE_MODE', 'local') == 'workers':
            return cls.from_inference_workers(inference_job_id, db=db, **kw)
        from ..db.database import Database
        from ..model.model import load_model_class
        db = db or Database()
        ij = db.get_inference_job(inference_job_id)
        tj = db.get_train_job(ij.train_job_id)
        models = []
        for w in db.get_workers_of_inference_job(inference_job_id):
            trial = db.get_trial(w.trial_id)
            sub = db.get_sub_train_job(trial.sub_train_job_id)
            mrec = db.get_model(sub.model_id)
            clazz = load_model_class(mrec.model_file_bytes, mrec.model_class)
            inst = clazz(**(trial.knobs or {}))
            with open(trial.params_file_path, 'rb') as f:
                inst.load_parameters(pickle.loads(f.read()))
            models.append((trial.id, inst))
        return cls(models, task=tj.task, **kw)

    @classmethod
    def from_inference_workers(cls, inference_job_id, db=None, cache=None, **kw):
        from ..cache import Cache
        from ..db.database import Database
        db = db or Database()
        ij = db.get_inference_job(inference_job_id)
        tj = db.get_train_job(ij.train_job_id)
        cache = cache or Cache()
        models = [(w.trial_id, RemoteWorkerModel(w.service_id, cache))
                  for w in db.get_workers_of_inference_job(inference_job_id)]
        return cls(models, task=tj.task, **kw)

    # ------------------------------------------------------------------------- inference
    def _fast_path(self):
        return self.task == TaskType.IMAGE_CLASSIFICATION and self.models and all(
            callable(getattr(m, 'predict_proba', None)) for _, m in self.models)

    def predict(self, queries):
        """Synchronous batched prediction over the whole ensemble."""
        if not queries:
            return []
        if self.models and all(isinstance(m, RemoteWorkerModel) for _, m in self.models):
            return self._predict_remote(queries)
        if self._fast_path():
            try:
                return self._predict_fast(queries)
            except Exception:
                logger.error('fast path failed, falling back:\n%s', traceback.format_exc())
        preds, ok = [], []
        for name, m in self.models:
            try:
                preds.append(m.predict(queries))
                ok.append(name)
            except Exception:
                self.stats['errors'] += 1
                logger.error('model %s failed:\n%s', name, traceback.format_exc())
        if not preds:
            raise RuntimeError('every model of the ensemble failed')
        return ensemble_predictions(preds, self.task)

    def predict_array(self, arr):
        """Ensemble probabilities for a numpy batch (images already decoded): skips the per-query
        list handling of ``predict``; native models take the uint8 batch straight to the device."""
        if self._fast_path():
            import numpy as np
            import torch
            dev = None
            for _, m in self.models:
                d = getattr(m, 'device', None)
                if d is not None and torch.device(d).type == 'cuda':
                    dev = torch.device(d)
                    break
            if dev is not None and all(callable(getattr(m, 'input_signature', None)) for _, m in self.models):
                inputs = {}
                for _, m in self.models:
                    sig = m.input_signature()
                    if sig not in inputs:
                        imgs = np.ascontiguousarray(m.queries_to_images(arr))
                        inputs[sig] = torch.from_numpy(imgs).pin_memory().to(dev, non_blocking=True)
                self.stats['queries'] += len(arr)
                return self.predict_proba_device(inputs).cpu().numpy()
        return self.predict(arr.tolist())

    def _predict_remote(self, queries):
        """Fan the batch out to every worker first, then gather (workers run concurrently); a worker
        that misses the deadline is dropped from this batch's ensemble (partial-ensemble fallback)."""
        import uuid
        base = uuid.uuid4().hex[:12]
        ids = ['{}-{}'.format(base, i) for i in range(len(queries))]
        for _, m in self.models:
            m.submit(ids, queries)
        deadline = time.perf_counter() + self.timeout_s
        preds = []
        for name, m in self.models:
            try:
                p = m.collect(ids, deadline)
                if any(x is None for x in p):
                    raise RuntimeError('worker {} failed to predict'.format(name))
                preds.append(p)
            except Exception:
                self.stats['errors'] += 1
                logger.error('remote model %s dropped from ensemble:\n%s', name, traceback.format_exc())
        if not preds:
            raise RuntimeError('every model of the ensemble failed')
        return ensemble_predictions(preds, self.task)

    def _predict_fast(self, queries):
        return self.predict_proba(queries).cpu().tolist()

    def predict_proba(self, queries):
        """Ensemble probabilities [Q, C] as a tensor (on the GPU when the models are).

        Queries are decoded to uint8 once per distinct model input signature and uploaded once
        (pinned, non-blocking); every model then runs its hipGraph-captured bucketed forward on its
        own HIP stream, and the gfx950 ensemble-mean kernel reduces the [models, Q, C] stack."""
        import numpy as np
        import torch
        dev = None
        for name, m in self.models:
            d = getattr(m, 'device', None)
            if d is not None and torch.device(d).type == 'cuda':
                dev = torch.device(d)
                break
        if dev is None:
            probs = [m.predict_proba(queries) for _, m in self.models]
            return ensemble_probabilities(torch.stack([p.float().cpu() for p in probs]))
        inputs = {}
        for _, m in self.models:
            sig_fn = getattr(m, 'input_signature', None)
            sig = sig_fn() if callable(sig_fn) else None
            if sig is not None and sig not in inputs:
                arr = np.ascontiguousarray(m.queries_to_images(queries))
                host = torch.from_numpy(arr).pin_memory()
                inputs[sig] = host.to(dev, non_blocking=True)
        return self.predict_proba_device(inputs, queries)

    def predict_proba_device(self, inputs, queries=None):
        """inputs: {input_signature: device uint8 batch}.  Models without a signature get ``queries``."""
        import torch
        dev = next(iter(inputs.values())).device if inputs else torch.device('cuda')
        if self._streams is None or len(self._streams) != len(self.models):
            self._streams = [torch.cuda.Stream(device=dev) for _ in self.models]
        main = torch.cuda.current_stream(dev)
        outs = []
        for (name, m), s in zip(self.models, self._streams):
            s.wait_stream(main)
            with torch.cuda.stream(s):
                sig_fn = getattr(m, 'input_signature', None)
                sig = sig_fn() if callable(sig_fn) else None
                if sig is not None and sig in inputs:
                    p = m.predict_proba_images(inputs[sig])
                else:
                    p = m.predict_proba(queries)
                outs.append(p)
        for s in self._streams:
            main.wait_stream(s)
        for p in outs:
            p.record_stream(main)
        stacked = torch.stack(outs)
        w = None
        if self.weights is not None:
            w = torch.tensor(self.weights, dtype=torch.float32, device=dev)
        return ensemble_probabilities(stacked, w)

    # ------------------------------------------------------------------- dynamic batching
    def start(self):
        if self._thread is None:
            self._stop.clear()
            self._thread = threading.Thread(target=self._batch_loop, name='rafiki-batcher', daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    def submit(self, query) -> Future:
        fut = Future()
        self._q.put((query, fut))
        if self._thread is None:
            self.start()
        return fut

    def predict_one(self, query):
        return self.submit(query).result(timeout=self.timeout_s)

    def _batch_loop(self):
        while not self._stop.is_set():
            try:
                first = self._q.get(timeout=0.05)
            except queue.Empty:
                continue
            batch = [first]
            deadline = time.perf_counter() + self.max_wait_s
            while len(batch) < self.max_batch:
                rem = deadline - time.perf_counter()
                try:
                    batch.append(self._q.get(timeout=max(0.0, rem)) if rem > 0 else self._q.get_nowait())
                except queue.Empty:
                    break
            queries = [q for q, _ in batch]
            try:
                preds = self.predict(queries)
                for (_, fut), p in zip(batch, preds):
                    fut.set_result(p)
            except Exception as e:
                for _, fut in batch:
                    fut.set_exception(e)
            self.stats['batches'] += 1
            self.stats['queries'] += len(batch)
