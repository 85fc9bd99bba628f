"""Per-process trial execution context: which device a model trains on and, for data-parallel
trials, the process group it shares with the other ranks of its worker group.

Models read it through ``rafiki_amd.parallel.context.current()`` instead of probing
``CUDA_VISIBLE_DEVICES`` (the reference's pg_gans crashes when it is unset).
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field
from typing import Optional

import torch

from .dist import DistInfo


@dataclass
class TrialContext:
    device: torch.device = field(default_factory=lambda: torch.device('cpu'))
    dist: DistInfo = field(default_factory=DistInfo)
    data_parallel: bool = False  # True: this trial is trained jointly by every rank of the group
    trial_id: Optional[str] = None
    checkpoint: Optional[object] = None  # utils.checkpoint.TrialCheckpoint when the worker supports resume

    @property
    def is_gpu(self):
        return self.device.type == 'cuda'

    @property
    def world_size(self):
        return self.dist.world_size if self.data_parallel else 1

    @property
    def rank(self):
        return self.dist.rank if self.data_parallel else 0


_local = threading.local()


def default_device() -> torch.device:
    if os.environ.get('RAFIKI_CPU_ONLY') == '1':
        return torch.device('cpu')
    try:
        if torch.cuda.is_available():
            return torch.device('cuda', int(os.environ.get('LOCAL_RANK', '0')) % max(1, torch.cuda.device_count()))
    except Exception:
        pass
    return torch.device('cpu')


def current() -> TrialContext:
    ctx = getattr(_local, 'ctx', None)
    if ctx is None:
        ctx = TrialContext(device=default_device())
        _local.ctx = ctx
    return ctx


def set_current(ctx: TrialContext):
    _local.ctx = ctx


class use_context:
    def __init__(self, ctx: TrialContext):
        self.ctx = ctx

    def __enter__(self):
        self.prev = getattr(_local, 'ctx', None)
        _local.ctx = self.ctx
        return self.ctx

    def __exit__(self, *exc):
        _local.ctx = self.prev
        return False
