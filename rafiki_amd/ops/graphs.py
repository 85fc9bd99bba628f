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


class SplitCapture:
    """One capture region recorded as a SEQUENCE of graphs on one stream and one memory pool.

    ``cut(mark)`` ends the current graph and begins the next one where the stream's work stands; the
    caller replays the graphs in order and may enqueue other work between them (the data-parallel
    gradient segments start each bucket's all-reduce after the graph that finished the bucket, so the
    reduce runs on RCCL's stream while the next graph replays the rest of the backward).  Cuts are
    made from inside a backward, i.e. on autograd's device thread, whose current stream is the
    capture stream there; so the graphs are captured in ``relaxed`` mode (a graph may end on another
    thread than the one that began it).  LOCK is held and the cyclic GC is off for the whole region,
    as in ``capture``; the graphs share ``pool`` and are replayed in capture order, so memory reuse
    across them is stream-ordered exactly as inside one graph."""

    def __init__(self, pool=None):
        self.pool = pool if pool is not None else torch.cuda.graph_pool_handle()
        self.parts = []            # [(graph, mark)]
        self.tail_mark = None      # the mark of the last graph (set before the region ends)
        self._cur = None
        self._stream = None

    def _begin(self):
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self.pool, capture_error_mode='relaxed')
        self._cur = g

    def cut(self, mark=None):
        """End the current graph (its replay is followed by ``mark``'s work) and begin the next."""
        assert torch.cuda.current_stream() == self._stream, 'SplitCapture.cut off the capture stream'
        self._cur.capture_end()
        self.parts.append((self._cur, mark))
        self._begin()

    @contextlib.contextmanager
    def region(self):
        with LOCK:
            if _depth[0] == 0:
                _depth[1] = gc.isenabled()
                gc.disable()
            _depth[0] += 1
            try:
                torch.cuda.synchronize()
                self._stream = torch.cuda.Stream()
                with torch.cuda.stream(self._stream):
                    self._begin()
                    try:
                        yield self
                    finally:
                        self._cur.capture_end()
                        self.parts.append((self._cur, self.tail_mark))
                        self._cur = None
            finally:
                _depth[0] -= 1
                if _depth[0] == 0 and _depth[1]:
                    gc.enable()

