"""In-HBM trainer -> predictor model handoff.

The reference moves a finished trial to serving through the filesystem: the train worker pickles
the parameters to the shared params dir (rafiki/worker/train.py:178-183) and every inference
worker unpickles them again (rafiki/worker/inference.py:78-93).  When the trainer and the
predictor share a process (inline services, bench.py, notebooks), the trained model is already
resident in HBM: the train worker ``offer``s it here after writing its params file (which stays
the durable copy), and ``Predictor.from_inference_job`` ``take``s it instead of re-reading and
re-uploading the weights.

The store keeps the best-scoring models that fit the byte budget (``NodeConfig.param_cache_gb``):
only top-k trials are ever served, so a lower-scoring offer never evicts a better model, and an
evicted model is destroyed (its HBM returned).  Models that cannot be shared this way (host-only
models, models without ``resident_bytes``) are never held.
"""
from __future__ import annotations

import logging
import os
import threading
from typing import Dict, Optional, Tuple

logger = logging.getLogger(__name__)


def _destroy(model):
    from ..ops.graphs import quiesced
    with quiesced():
        try:
            model.destroy()
        except Exception:
            pass


class ResidentStore:
    def __init__(self, budget_bytes: Optional[float] = None):
        if budget_bytes is None:
            from ..config import NodeConfig
            budget_bytes = NodeConfig().param_cache_gb * 1e9
        self.budget = float(budget_bytes)
        self._items: Dict[str, Tuple[object, float, int]] = {}   # trial id -> (model, score, bytes)
        self._lock = threading.Lock()
        self.hits = 0
        self.misses = 0

    @staticmethod
    def eligible(model) -> bool:
        if os.environ.get('RAFIKI_RESIDENT_HANDOFF', '1') == '0':
            return False
        fn = getattr(model, 'resident_bytes', None)
        dev = getattr(model, 'device', None)
        return callable(fn) and dev is not None and getattr(dev, 'type', str(dev)) == 'cuda'

    @property
    def used(self) -> int:
        return sum(b for _, _, b in self._items.values())

    def offer(self, trial_id: str, model, score: float) -> bool:
        """Hold ``model`` (the store takes ownership) if it is among the best that fit the budget.
        Returns False when it is not kept — the caller then destroys it as usual."""
        if not self.eligible(model):
            return False
        nbytes = int(model.resident_bytes())
        if nbytes > self.budget:
            return False
        release = getattr(model, 'release_training', None)
        evicted = []
        with self._lock:
            ranked = sorted(self._items.items(), key=lambda kv: kv[1][1])   # worst score first
            free = self.budget - self.used
            victims = []
            for tid, (_, sc, b) in ranked:
                if free >= nbytes:
                    break
                if sc >= score:
                    return False       # would have to evict a better model
                victims.append(tid)
                free += b
            if free < nbytes:
                return False
            for tid in victims:
                evicted.append(self._items.pop(tid)[0])
            if callable(release):
                release()
            self._items[trial_id] = (model, float(score), nbytes)
        for m in evicted:
            _destroy(m)
        logger.info('trial %s resident for serving (%.1f MB, %d held)', trial_id, nbytes / 1e6, len(self._items))
        return True

    def take(self, trial_id: str):
        """The resident model of ``trial_id`` (ownership passes to the caller), or None."""
        with self._lock:
            ent = self._items.pop(trial_id, None)
        if ent is None:
            self.misses += 1
            return None
        self.hits += 1
        return ent[0]

    def __contains__(self, trial_id):
        return trial_id in self._items

    def clear(self):
        with self._lock:
            items, self._items = list(self._items.values()), {}
        for m, _, _ in items:
            _destroy(m)


STORE = ResidentStore()
