// Fast path for the predictor's JSON query bodies: find `"<key>":` in a JSON object and parse the
// value when it is a (nested, rectangular) array of integers 0..255 — an image query — straight
// into a uint8 buffer.  Python's json module spends ~1 us per pixel on these bodies (3072 ints per
// CIFAR-sized query); this runs at memory speed.  Anything else (strings, floats, ragged lists)
// returns -1 and the server falls back to the json module, so behaviour never changes.
#include <cstdint>
#include <cstring>

namespace {

const char* skip_ws(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  return p;
}

struct Parser {
  const char* p;
  const char* e;
  uint8_t* out;
  long long cap, n;
  long long shape[8];
  long long cnt[8];
  int ndim = -1;  // fixed by the first leaf

  // parse an array at depth d; returns false on anything that is not a rectangular int array
  bool array(int d) {
    if (d >= 8) return false;
    p = skip_ws(p, e);
    if (p >= e || *p != '[') return false;
    ++p;
    long long k = 0;
    p = skip_ws(p, e);
    if (p < e && *p == ']') return false;  // empty arrays: let the json module decide
    while (true) {
      p = skip_ws(p, e);
      if (p >= e) return false;
      if (*p == '[') {
        if (ndim >= 0 && d + 1 >= ndim) return false;
        if (!array(d + 1)) return false;
      } else {
        if (ndim < 0) ndim = d + 1;
        if (d + 1 != ndim) return false;
        if (*p < '0' || *p > '9') return false;
        unsigned v = 0;
        int digits = 0;
        while (p < e && *p >= '0' && *p <= '9') { v = v * 10 + (unsigned)(*p - '0'); ++p; if (++digits > 3) return false; }
        if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) return false;
        if (v > 255 || n >= cap) return false;
        out[n++] = (uint8_t)v;
      }
      ++k;
      p = skip_ws(p, e);
      if (p >= e) return false;
      if (*p == ',') { ++p; continue; }
      if (*p == ']') { ++p; break; }
      return false;
    }
    if (cnt[d] == 0) shape[d] = k;
    else if (shape[d] != k) return false;
    cnt[d]++;
    return true;
  }
};

}  // namespace

extern "C" long long rt_json_u8_array(const char* body, long long len, const char* key, uint8_t* out, long long cap,
                                      long long* shape, int* ndim) {
  const char* e = body + len;
  const size_t kl = strlen(key);
  // find "key" followed by ':'
  const char* p = body;
  while (true) {
    p = (const char*)memchr(p, '"', (size_t)(e - p));
    if (!p || e - p < (long long)kl + 2) return -1;
    if (!memcmp(p + 1, key, kl) && p[kl + 1] == '"') {
      const char* q = skip_ws(p + kl + 2, e);
      if (q < e && *q == ':') { p = q + 1; break; }
    }
    ++p;
  }
  Parser ps{p, e, out, cap, 0, {0}, {0}};
  if (!ps.array(0)) return -1;
  *ndim = ps.ndim;
  for (int i = 0; i < ps.ndim; ++i) shape[i] = ps.shape[i];
  return ps.n;
}
