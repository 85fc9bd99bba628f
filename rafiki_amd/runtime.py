"""ctypes bindings of the host C++ runtime (``rafiki_amd/_native/librafiki_runtime.so``).

The runtime is optional on CPU-only dev boxes (pure-Python fallbacks exist for every entry point);
``available()`` reports whether it was built.
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path

_LIB_PATH = Path(__file__).resolve().parent / "_native" / "librafiki_runtime.so"
_lock = threading.Lock()
_lib = None
_tried = False

_SIGS = {
    "rt_crc32c": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_longlong]),
    "rt_masked_crc32c": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_longlong]),
    "rt_tfrecord_info": (ctypes.c_longlong, [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]),
    "rt_tfrecord_decode_images": (ctypes.c_longlong,
                                  [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong,
                                   ctypes.c_int]),
    "rt_json_u8_array": (ctypes.c_longlong, [ctypes.c_char_p, ctypes.c_longlong, ctypes.c_char_p, ctypes.c_void_p,
                                            ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p]),
    "rt_mq_open": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_longlong, ctypes.c_int]),
    "rt_mq_close": (None, [ctypes.c_void_p]),
    "rt_mq_unlink": (ctypes.c_int, [ctypes.c_char_p]),
    "rt_mq_push": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_longlong, ctypes.c_int]),
    "rt_mq_pop": (ctypes.c_longlong, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int]),
    "rt_mq_size": (ctypes.c_longlong, [ctypes.c_void_p]),
}


def lib():
    global _lib, _tried
    with _lock:
        if _lib is None and not _tried:
            _tried = True
            if _LIB_PATH.exists():
                h = ctypes.CDLL(str(_LIB_PATH))
                for name, (res, args) in _SIGS.items():
                    fn = getattr(h, name, None)
                    if fn is None:
                        continue
                    fn.restype, fn.argtypes = res, args
                _lib = h
        return _lib


def available() -> bool:
    return lib() is not None


def reset():
    """Forget a cached handle (after a rebuild in the same process)."""
    global _lib, _tried
    with _lock:
        _lib, _tried = None, False


def json_u8_array(body: bytes, key: str, max_elems: int = 1 << 26):
    """Parse ``body[key]`` as a rectangular uint8 integer array with the native parser.
    Returns a numpy array, or None when the runtime is missing or the value is not such an array."""
    h = lib()
    if h is None:
        return None
    import numpy as np
    cap = min(max_elems, len(body))  # every element takes >= 1 byte of JSON
    out = np.empty(cap, dtype=np.uint8)
    shape = (ctypes.c_longlong * 8)()
    nd = ctypes.c_int(0)
    n = h.rt_json_u8_array(body, len(body), key.encode(), out.ctypes.data, cap, shape, ctypes.byref(nd))
    if n < 0:
        return None
    return out[:n].reshape([int(shape[i]) for i in range(nd.value)])


# ------------------------------------------------------------------- nested lists -> uint8 (GIL held)
_PYLIST = Path(__file__).resolve().parent / "_native" / "librafiki_pylist.so"
_py = None


def _pylib():
    global _py
    if _py is None and _PYLIST.exists():
        h = ctypes.PyDLL(str(_PYLIST))
        h.rk_pylist_shape.restype, h.rk_pylist_shape.argtypes = ctypes.c_int, [ctypes.py_object, ctypes.c_void_p]
        h.rk_pylist_u8.restype = ctypes.c_int
        h.rk_pylist_u8.argtypes = [ctypes.py_object, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        _py = h
    return _py


def pylist_u8(obj, max_elems: int = 1 << 26):
    """A rectangular nest of Python lists / tuples of ints or floats -> uint8 numpy array (clipped to
    [0, 255], floats truncated) by the native walker; None when the library is missing or the nest
    is ragged / non-numeric (callers then fall back to numpy).

    The shape comes from the first-element chain before the walk proves the nest rectangular, so
    the allocation is capped (``max_elems`` bytes): a small adversarial query whose first children
    are long and the rest empty cannot request a huge buffer."""
    h = _pylib()
    if h is None or not isinstance(obj, (list, tuple)):
        return None
    import numpy as np
    shape = (ctypes.c_longlong * 8)()
    nd = h.rk_pylist_shape(obj, shape)
    if nd < 0:
        return None
    dims = [int(shape[i]) for i in range(nd)]
    total = 1
    for d in dims:
        total *= d
        if total > max_elems:
            return None
    try:
        out = np.empty(dims, dtype=np.uint8)
    except (MemoryError, ValueError):
        return None
    if out.size and h.rk_pylist_u8(obj, shape, nd, out.ctypes.data) != 0:
        return None
    return out
