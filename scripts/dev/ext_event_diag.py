"""Diagnose external graph events: does side.wait_event(ev) after g.replay() wait for the graph's work
before the event?  Prints one JSON line per variant."""
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def run(external, n=16 << 20, sync_mode='wait_stream'):
    dev = torch.device('cuda', 0)
    src = torch.zeros(n, device=dev)
    dst = torch.zeros(n, device=dev)
    tail = torch.zeros(n, device=dev)
    seen = torch.zeros(8, device=dev)
    ev = torch.cuda.Event(external=external)
    side = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, capture_error_mode='thread_local'):
        dst.copy_(src)
        ev.record()
        tail.copy_(dst)
        tail.copy_(src)
    for k in range(1, 9):
        src.fill_(float(k))
        g.replay()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            seen[k - 1:k].copy_(dst[n - 1:n])
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    return seen.cpu().tolist()


for ext in (True, False):
    try:
        print(json.dumps({'external': ext, 'seen': run(ext)}), flush=True)
    except Exception as e:
        print(json.dumps({'external': ext, 'error': repr(e), 'tb': traceback.format_exc()[-800:]}), flush=True)


class HipExternalEvent:
    """hipEventRecordWithFlags(external) through the runtime torch loaded (torch refuses
    Event(external=True) on ROCm)."""

    def __init__(self):
        import ctypes
        path = None
        with open('/proc/self/maps') as f:
            for line in f:
                if 'libamdhip64.so' in line:
                    path = line.split()[-1]
                    break
        self.lib = lib = ctypes.CDLL(path or 'libamdhip64.so')
        vp, u32 = ctypes.c_void_p, ctypes.c_uint
        lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), u32]
        lib.hipEventRecordWithFlags.argtypes = [vp, vp, u32]
        lib.hipStreamWaitEvent.argtypes = [vp, vp, u32]
        self.h = vp()
        assert lib.hipEventCreateWithFlags(ctypes.byref(self.h), 2) == 0

    def record(self):
        rc = self.lib.hipEventRecordWithFlags(self.h, torch.cuda.current_stream().cuda_stream, 1)
        if rc != 0:
            raise RuntimeError('hipEventRecordWithFlags(external) failed: {}'.format(rc))

    def wait_on(self, stream):
        assert self.lib.hipStreamWaitEvent(stream.cuda_stream, self.h, 0) == 0


def run_hip(n=16 << 20):
    from rafiki_amd.ops.graphs import capture
    dev = torch.device('cuda', 0)
    src = torch.zeros(n, device=dev)
    dst = torch.zeros(n, device=dev)
    tail = torch.zeros(n, device=dev)
    seen = torch.zeros(8, device=dev)
    ev = HipExternalEvent()
    side = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with capture(g):
        dst.copy_(src)
        ev.record()
        for _ in range(4):
            tail.copy_(dst)
            tail.copy_(src)
    for k in range(1, 9):
        src.fill_(float(k))
        g.replay()
        ev.wait_on(side)
        with torch.cuda.stream(side):
            seen[k - 1:k].copy_(dst[n - 1:n])
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    return seen.cpu().tolist()


try:
    print(json.dumps({'hip_external': True, 'seen': run_hip()}), flush=True)
except Exception as e:
    print(json.dumps({'hip_external': True, 'error': repr(e), 'tb': traceback.format_exc()[-800:]}), flush=True)
