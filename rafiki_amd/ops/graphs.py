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
import gc
import threading

import torch

LOCK = threading.RLock()


@contextlib.contextmanager
def quiesced():
    """Hold while dropping the last reference to captured graphs (engine teardown, trainer ->
    predictor handoff): a graph's destructor frees its exec and private memory pool, which must not
    run while another thread of this process is capturing."""
    with LOCK:
        yield


def device_sync(device=None):
    """``torch.cuda.synchronize`` that never overlaps another thread's capture.  On ROCm a device-wide
    synchronize walks every stream of the device, including one that another thread is capturing
    into, and that invalidates the capture whatever its error mode (measured: an inline trainer's
    end-of-loop synchronize failed with hipErrorStreamCaptureUnsupported and the concurrent trainer's
    capture died in its next launch).  Captures hold LOCK for their whole duration, so taking it
    here serialises the two."""
    with LOCK:
        torch.cuda.synchronize(device)


_depth = [0, False]   # [nesting depth of capture() in this process, gc enabled before the outermost]


@contextlib.contextmanager
def capture(graph: "torch.cuda.CUDAGraph", pool=None, stream=None):
    # Python's cyclic GC must not run while a capture is open: a collection can destroy an unreachable
    # CUDAGraph / event whose destructor calls into HIP, which is illegal on a capturing thread, and a
    # C++ destructor cannot report the error (the process aborts).  torch.cuda.graph collects once
    # before the capture begins; further collections wait until the outermost capture has ended.
    with LOCK:
        if _depth[0] == 0:
            _depth[1] = gc.isenabled()
            gc.disable()
        _depth[0] += 1
        try:
            with torch.cuda.graph(graph, pool=pool, stream=stream, capture_error_mode='thread_local'):
                yield
        finally:
            _depth[0] -= 1
            if _depth[0] == 0 and _depth[1]:
                gc.enable()


