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



_HIP = {}


def _hip():
    """The HIP runtime library this process already uses (the copy torch loaded, found in the process
    map, so no second runtime instance is ever opened)."""
    if 'lib' not in _HIP:
        import ctypes
        path = None
        try:
            with open('/proc/self/maps') as f:
                for line in f:
                    if 'libamdhip64.so' in line:
                        path = line.split()[-1]
                        break
        except OSError:
            pass
        lib = ctypes.CDLL(path or 'libamdhip64.so')
        vp, u32 = ctypes.c_void_p, ctypes.c_uint
        lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), u32]
        lib.hipEventRecordWithFlags.argtypes = [vp, vp, u32]
        lib.hipStreamWaitEvent.argtypes = [vp, vp, u32]
        lib.hipEventDestroy.argtypes = [vp]
        for fn in (lib.hipEventCreateWithFlags, lib.hipEventRecordWithFlags, lib.hipStreamWaitEvent,
                   lib.hipEventDestroy):
            fn.restype = ctypes.c_int
        _HIP['lib'] = lib
    return _HIP['lib']


class HipExternalEvent:
    """A HIP event recorded with the external flag: inside a stream capture it becomes an event-record
    node of the graph, so a stream outside the graph can wait on that point of every replay
    (hipStreamWaitEvent after the replay is enqueued).  torch.cuda.Event(external=True) is refused on
    ROCm builds of torch, so this calls the runtime directly; ``external_events_ok`` verifies the
    ordering on the device before anything relies on it."""
    DISABLE_TIMING, RECORD_EXTERNAL = 0x2, 0x1

    def __init__(self):
        import ctypes
        self._h = ctypes.c_void_p()
        rc = _hip().hipEventCreateWithFlags(ctypes.byref(self._h), self.DISABLE_TIMING)
        if rc != 0:
            raise RuntimeError('hipEventCreateWithFlags failed: {}'.format(rc))

    def record(self, stream=None):
        st = stream if stream is not None else torch.cuda.current_stream()
        rc = _hip().hipEventRecordWithFlags(self._h, st.cuda_stream, self.RECORD_EXTERNAL)
        if rc != 0:
            raise RuntimeError('hipEventRecordWithFlags(external) failed: {}'.format(rc))

    def wait_on(self, stream):
        rc = _hip().hipStreamWaitEvent(stream.cuda_stream, self._h, 0)
        if rc != 0:
            raise RuntimeError('hipStreamWaitEvent failed: {}'.format(rc))

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value:
            try:
                _hip().hipEventDestroy(h)
            except Exception:
                pass


_EXT_EVENTS = {}


def external_events_ok(device=None) -> bool:
    """Whether an external event recorded inside a captured graph orders work that another stream
    issues after the replay (``side.wait_event(ev)``) behind the graph's work before the event — what
    FlatGradAllReduce.overlapped relies on.  Checked once per process and device with a sentinel: the
    graph copies a 64 MiB source (refilled with a new value before every replay) and records the
    event; a side stream waiting on it must read the new value, every time.  False (the reduce then
    runs after the whole segment) if the runtime lacks the feature or the check fails."""
    dev = torch.device('cuda', torch.cuda.current_device()) if device is None else torch.device(device)
    key = dev.index
    if key in _EXT_EVENTS:
        return _EXT_EVENTS[key]
    ok = False
    try:
        with LOCK:
            n = 16 << 20
            src = torch.zeros(n, device=dev)
            dst = torch.zeros(n, device=dev)
            tail = torch.zeros(n, device=dev)
            seen = torch.zeros(8, device=dev)
            ev = HipExternalEvent()
            side = torch.cuda.Stream(device=dev)
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(dev)
            with capture(g):
                dst.copy_(src)
                ev.record()
                tail.copy_(dst)          # more graph work after the event
                tail.copy_(src)
            ok = True
            for k in range(1, 9):
                src.fill_(float(k))
                g.replay()
                ev.wait_on(side)
                with torch.cuda.stream(side):
                    seen[k - 1:k].copy_(dst[n - 1:n])
                torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            ok = bool((seen == torch.arange(1, 9, device=dev, dtype=seen.dtype)).all())
            del g
    except Exception:
        ok = False
    _EXT_EVENTS[key] = ok
    return ok
