"""CPU tests of the capture discipline in ops/graphs.py: Python's cyclic GC is
off inside every capture (nested too), restored afterwards — also when the capture raises — and left
off if it was off on entry; graph teardown (``quiesced``) waits for an open capture."""
import contextlib
import gc
import threading
import time

import pytest
import torch

from rafiki_amd.ops import graphs


@pytest.fixture
def fake_graph(monkeypatch):
    seen = []

    @contextlib.contextmanager
    def fake(graph, pool=None, stream=None, capture_error_mode='global'):
        seen.append(capture_error_mode)
        yield

    monkeypatch.setattr(torch.cuda, 'graph', fake)
    was = gc.isenabled()
    gc.enable()
    yield seen
    (gc.enable if was else gc.disable)()


def test_gc_off_inside_and_restored(fake_graph):
    with graphs.capture(object()):
        assert not gc.isenabled()
    assert gc.isenabled()
    assert fake_graph == ['thread_local']


def test_nested_capture_restores_only_at_outermost(fake_graph):
    with graphs.capture(object()):
        with graphs.capture(object()):
            assert not gc.isenabled()
        assert not gc.isenabled()   # still inside the outer capture
    assert gc.isenabled()


def test_exception_inside_capture_restores_gc(fake_graph):
    with pytest.raises(RuntimeError):
        with graphs.capture(object()):
            raise RuntimeError('capture failed')
    assert gc.isenabled()
    assert graphs._depth[0] == 0
    with pytest.raises(ValueError):   # an exception in a nested capture too
        with graphs.capture(object()):
            with graphs.capture(object()):
                raise ValueError('inner')
    assert gc.isenabled() and graphs._depth[0] == 0


def test_gc_disabled_on_entry_stays_disabled(fake_graph):
    gc.disable()
    with graphs.capture(object()):
        assert not gc.isenabled()
    assert not gc.isenabled()


def test_quiesced_waits_for_an_open_capture(fake_graph):
    order = []
    entered = threading.Event()

    def capturer():
        with graphs.capture(object()):
            entered.set()
            time.sleep(0.2)
            order.append('capture-end')

    t = threading.Thread(target=capturer)
    t.start()
    entered.wait(5)
    with graphs.quiesced():
        order.append('teardown')
    t.join()
    assert order == ['capture-end', 'teardown']


def test_device_sync_waits_for_an_open_capture(fake_graph, monkeypatch):
    """A device-wide synchronize invalidates another thread's open capture on ROCm, so the
    trainers' synchronize goes through graphs.device_sync, which waits for the capture to end."""
    order = []
    entered = threading.Event()
    monkeypatch.setattr(torch.cuda, 'synchronize', lambda device=None: order.append('sync'))

    def capturer():
        with graphs.capture(object()):
            entered.set()
            time.sleep(0.2)
            order.append('capture-end')

    t = threading.Thread(target=capturer)
    t.start()
    entered.wait(5)
    graphs.device_sync()
    t.join()
    assert order == ['capture-end', 'sync']
