"""Ensembling of per-model predictions (reference rafiki/predictor/ensemble.py:6-33).

IMAGE_CLASSIFICATION: mean of class-probability vectors over models; other tasks: the first
model's predictions.  ``ensemble_probabilities`` is the on-device path used by the predictor for
native models (one fused kernel over a [models, queries, classes] tensor).
"""
from __future__ import annotations

from collections.abc import Iterable

import numpy as np

from ..constants import TaskType


def ensemble_predictions(predictions_list, task):
    if len(predictions_list) == 0 or len(predictions_list[0]) == 0:
        return []
    if task == TaskType.IMAGE_CLASSIFICATION:
        arr = np.asarray(predictions_list, dtype=np.float64)  # [models, queries, classes]
        preds = arr.mean(axis=0)
    else:
        preds = predictions_list[0]
    return _simplify(preds)


def _simplify(preds):
    if isinstance(preds, np.ndarray):
        return preds.tolist()
    if isinstance(preds, Iterable) and not isinstance(preds, (str, bytes, dict)):
        return [p.tolist() if isinstance(p, np.ndarray) else p for p in preds]
    return preds


def ensemble_probabilities(probs, weights=None):
    """probs: torch [models, Q, C] (on GPU -> gfx950 ensemble-mean kernel) -> [Q, C]."""
    import torch
    if probs.is_cuda:
        from ..ops import functional as F
        return F.ensemble_mean(probs.float().contiguous(), weights)
    if weights is None:
        return probs.float().mean(0)
    w = weights.float().reshape(-1, 1, 1)
    return (probs.float() * w).sum(0) / w.sum()
