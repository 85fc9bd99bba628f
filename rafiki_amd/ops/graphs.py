"""Process-wide hipGraph capture discipline.

Several threads of one process can drive the same GPU: the predictor's batcher and its HTTP
handlers, in-process (inline) train workers, the autotuner.  A capture in the default *global*
mode makes every other thread's capture-unsafe call (synchronize, event sync, allocator growth)
fail — and a failed capture can abort the process.  Every capture in rafiki_amd therefore goes
through ``capture()``: ``thread_local`` error mode (only the capturing thread is checked) and one
process-wide re-entrant lock, so two captures (and autotuning sweeps, which time captured graphs)
never interleave.
"""
from __future__ import annotations

import contextlib
import threading

import torch

LOCK = threading.RLock()


@contextlib.contextmanager
def capture(graph: "torch.cuda.CUDAGraph", pool=None, stream=None):
    with LOCK:
        with torch.cuda.graph(graph, pool=pool, stream=stream, capture_error_mode='thread_local'):
            yield
