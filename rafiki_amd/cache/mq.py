"""Python handle over the native shared-memory message queue (csrc/runtime/mq.cpp).

Without the native runtime (a CPU dev box that could not build it) an in-process fallback with the
same semantics is used; it only connects threads of one process.
"""
from __future__ import annotations

import ctypes
import queue
import threading
from typing import Optional

from .. import runtime

_local_queues = {}
_local_lock = threading.Lock()


class MessageQueue:
    def __init__(self, name: str, capacity: int = 64 << 20, create: bool = True):
        self.name = name
        h = runtime.lib()
        self._lib = h
        self._buf = ctypes.create_string_buffer(1 << 16)
        if h is not None:
            self._h = h.rt_mq_open(name.encode(), int(capacity), int(create))
            if not self._h:
                raise OSError('cannot open shared-memory queue {}'.format(name))
        else:
            with _local_lock:
                self._q = _local_queues.setdefault(name, queue.Queue())

    @property
    def native(self):
        return self._lib is not None

    def push(self, data: bytes, timeout_ms: int = 5000) -> bool:
        if self._lib is None:
            self._q.put(bytes(data))
            return True
        rc = self._lib.rt_mq_push(self._h, data, len(data), int(timeout_ms))
        if rc == -2:
            raise ValueError('message of {} bytes exceeds queue {} capacity'.format(len(data), self.name))
        return rc == 0

    def pop(self, timeout_ms: int = 0) -> Optional[bytes]:
        if self._lib is None:
            try:
                return self._q.get(timeout=timeout_ms / 1000.0) if timeout_ms > 0 else self._q.get_nowait()
            except queue.Empty:
                return None
        while True:
            n = self._lib.rt_mq_pop(self._h, self._buf, len(self._buf), int(timeout_ms))
            if n >= 0:
                return self._buf.raw[:n]
            if n == -1:
                return None
            if n <= -16:  # buffer too small: grow and retry (the message stayed queued)
                self._buf = ctypes.create_string_buffer(int(-n - 16) * 2)
                continue
            raise OSError('queue {} error {}'.format(self.name, n))

    def size(self) -> int:
        if self._lib is None:
            return self._q.qsize()
        return int(self._lib.rt_mq_size(self._h))

    def close(self):
        if self._lib is not None and self._h:
            self._lib.rt_mq_close(self._h)
            self._h = None

    def unlink(self):
        if self._lib is not None:
            self._lib.rt_mq_unlink(self.name.encode())
        else:
            with _local_lock:
                _local_queues.pop(self.name, None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
