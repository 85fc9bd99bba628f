// Nested Python sequences of numbers -> a contiguous uint8 buffer, with the GIL held (loaded through
// ctypes.PyDLL).  The in-process predictor receives image queries as nested lists (the reference's
// query format, docs/src/user/tasks.rst:33-37); numpy's generic converter walks them at ~100 ns per
// element, this at a few ns: ints clip to [0, 255], floats clip then truncate toward zero (the same
// result as np.clip(np.asarray(q), 0, 255).astype(np.uint8)).
#include <Python.h>
#include <stdint.h>

namespace {

constexpr int MAX_DIMS = 8;

// shape of the first element chain; -1 if the leaf is not a number
int probe(PyObject* o, int64_t* shape) {
  int nd = 0;
  while (PyList_Check(o) || PyTuple_Check(o)) {
    if (nd >= MAX_DIMS) return -1;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(o);
    shape[nd++] = n;
    if (n == 0) return nd;
    o = PySequence_Fast_GET_ITEM(o, 0);
  }
  return (PyLong_Check(o) || PyFloat_Check(o)) ? nd : -1;
}

inline bool leaf(PyObject* o, uint8_t* dst) {
  if (PyLong_Check(o)) {
    int overflow = 0;
    const long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
    *dst = overflow > 0 ? 255 : overflow < 0 ? 0 : (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    return true;
  }
  if (PyFloat_Check(o)) {
    const double v = PyFloat_AS_DOUBLE(o);
    *dst = (uint8_t)(v != v ? 0.0 : v < 0.0 ? 0.0 : v > 255.0 ? 255.0 : v);   // NaN -> 0
    return true;
  }
  return false;
}

// fill in row-major order; false on a ragged / non-numeric input
bool fill(PyObject* o, const int64_t* shape, int d, int nd, uint8_t*& dst) {
  if (d == nd) return leaf(o, dst++);
  if (!(PyList_Check(o) || PyTuple_Check(o))) return false;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(o);
  if (n != shape[d]) return false;
  PyObject** items = PySequence_Fast_ITEMS(o);
  if (d + 1 == nd) {
    for (Py_ssize_t i = 0; i < n; ++i)
      if (!leaf(items[i], dst++)) return false;
    return true;
  }
  for (Py_ssize_t i = 0; i < n; ++i)
    if (!fill(items[i], shape, d + 1, nd, dst)) return false;
  return true;
}

}  // namespace

// shape query: returns ndim (>= 0) and writes shape[0..ndim), or -1 (not a rectangular numeric nest)
extern "C" int rk_pylist_shape(PyObject* obj, int64_t* shape) { return probe(obj, shape); }

// fill out (prod(shape) bytes) -> 0, or -1 on a ragged / non-numeric nest
extern "C" int rk_pylist_u8(PyObject* obj, const int64_t* shape, int ndim, uint8_t* out) {
  uint8_t* p = out;
  return fill(obj, shape, 0, ndim, p) ? 0 : -1;
}
