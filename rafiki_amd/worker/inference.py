"""InferenceWorker: one trial's model behind a shared-memory query queue (reference
rafiki/worker/inference.py:19-105).

Used by the optional ``workers`` serving mode (``RAFIKI_INFERENCE_MODE=workers``): each top-k
trial gets its own worker process — on its own GPU when the node has free ones — and the predictor
fans query batches out through ``Cache`` (csrc/runtime/mq.cpp rings instead of Redis).  The
default mode keeps every model inside the predictor process on one GPU (no IPC at all); this mode
scales serving past one GPU and isolates model code in separate processes, like the reference.

Loop: pop up to ``batch_size`` queries (blocking <= poll_ms for the first; no fixed 0.25 s sleep,
reference inference.py:65), ``model.predict``, push the predictions as one message.
"""
from __future__ import annotations

import logging
import pickle
import threading
import traceback

from .. import config
from ..cache import Cache
from ..model.model import load_model_class
from ..parallel.context import TrialContext, default_device, use_context

logger = logging.getLogger(__name__)


class InferenceWorker:
    def __init__(self, service_id, db=None, cache: Cache = None, batch_size: int = None, poll_ms: int = 50):
        from ..db.database import Database
        self._service_id = service_id
        self._db = db or Database()
        self._cache = cache or Cache()
        self._batch_size = int(batch_size or max(config.INFERENCE_WORKER_PREDICT_BATCH_SIZE, 256))
        self._poll_ms = poll_ms
        self._stop = threading.Event()
        self._model = None
        self._inference_job_id = None
        self.served = 0

    def load(self):
        w = self._db.get_inference_job_worker(self._service_id)
        if w is None:
            raise RuntimeError('no inference job worker for service {}'.format(self._service_id))
        self._inference_job_id = w.inference_job_id
        trial = self._db.get_trial(w.trial_id)
        sub = self._db.get_sub_train_job(trial.sub_train_job_id)
        mrec = self._db.get_model(sub.model_id)
        clazz = load_model_class(mrec.model_file_bytes, mrec.model_class)
        with use_context(TrialContext(device=default_device())):
            self._model = clazz(**(trial.knobs or {}))
            with open(trial.params_file_path, 'rb') as f:
                self._model.load_parameters(pickle.loads(f.read()))
        return self

    def start(self):
        if self._model is None:
            self.load()
        self._cache.add_worker_of_inference_job(self._service_id, self._inference_job_id)
        logger.info('inference worker %s serving job %s', self._service_id, self._inference_job_id)
        while not self._stop.is_set():
            ids, queries = self._cache.pop_queries_of_worker(self._service_id, self._batch_size, self._poll_ms)
            if not ids:
                continue
            try:
                with use_context(TrialContext(device=default_device())):
                    preds = self._model.predict(queries)
            except Exception:
                logger.error('predict failed:\n%s', traceback.format_exc())
                preds = [None] * len(ids)
            self._cache.add_predictions_of_worker(self._service_id, list(zip(ids, preds)))
            self.served += len(ids)

    def stop(self):
        self._stop.set()
        if self._inference_job_id is not None:
            try:
                self._cache.delete_worker_of_inference_job(self._service_id, self._inference_job_id)
            except Exception:
                pass
        if self._model is not None:
            try:
                self._model.destroy()
            except Exception:
                pass
