// Host-side data runtime: TFRecord framing, CRC32C (SSE4.2 when present) and a zero-copy decoder
// of tf.train.Example image records into one contiguous uint8 batch.
//
// Replaces the reference's TF input pipeline for IMAGE_GENERATION datasets (pg_gans.py:380-527:
// tf.data.TFRecordDataset -> parse_single_example -> decode_raw).  A whole level of detail is
// decoded in one call straight into a caller-provided (pinned) buffer, which the model uploads to
// HBM once; no per-record Python work.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

namespace {

constexpr uint64_t kMaxRecord = 1ull << 30;  // a record never exceeds 1 GiB: reject hostile lengths

uint32_t g_table[256];
bool g_table_init = false;

void init_table() {
  if (g_table_init) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_table[i] = c;
  }
  g_table_init = true;
}

uint32_t crc_sw(const uint8_t* p, size_t n) {
  init_table();
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = g_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32 ^ 0xFFFFFFFFu;
}
#endif

uint32_t crc32c(const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  static const bool hw = __builtin_cpu_supports("sse4.2");
  if (hw) return crc_hw(p, n);
#endif
  return crc_sw(p, n);
}

uint32_t masked(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xA282EAD8u; }

bool read_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  int shift = 0;
  while (p < end && shift < 64) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) return true;
    shift += 7;
  }
  return false;
}

struct Field {
  uint32_t num;
  uint32_t wt;
  uint64_t v;          // varint value
  const uint8_t* ptr;  // length-delimited payload
  uint64_t len;
};

bool next_field(const uint8_t*& p, const uint8_t* end, Field& f) {
  if (p >= end) return false;
  uint64_t key;
  if (!read_varint(p, end, key)) return false;
  f.num = (uint32_t)(key >> 3);
  f.wt = (uint32_t)(key & 7);
  f.ptr = nullptr;
  f.len = 0;
  switch (f.wt) {
    case 0: return read_varint(p, end, f.v);
    case 1: if (end - p < 8) return false; f.ptr = p; f.len = 8; p += 8; return true;
    case 5: if (end - p < 4) return false; f.ptr = p; f.len = 4; p += 4; return true;
    case 2:
      if (!read_varint(p, end, f.len) || (uint64_t)(end - p) < f.len) return false;
      f.ptr = p;
      p += f.len;
      return true;
    default: return false;
  }
}

// Example{1: Features{1: map entry{1: key, 2: Feature{1: BytesList{1: bytes}, 3: Int64List{1: packed}}}}}
bool parse_image(const uint8_t* p, const uint8_t* end, int64_t shape[3], int& ndim, const uint8_t*& data,
                 uint64_t& dlen) {
  ndim = 0;
  data = nullptr;
  dlen = 0;
  Field ex;
  while (next_field(p, end, ex)) {
    if (ex.num != 1 || ex.wt != 2) continue;
    const uint8_t* q = ex.ptr;
    const uint8_t* qe = ex.ptr + ex.len;
    Field ent;
    while (next_field(q, qe, ent)) {
      if (ent.num != 1 || ent.wt != 2) continue;
      const uint8_t* r = ent.ptr;
      const uint8_t* re = ent.ptr + ent.len;
      Field kv;
      const uint8_t* key = nullptr;
      uint64_t klen = 0;
      const uint8_t* feat = nullptr;
      uint64_t flen = 0;
      while (next_field(r, re, kv)) {
        if (kv.num == 1 && kv.wt == 2) { key = kv.ptr; klen = kv.len; }
        if (kv.num == 2 && kv.wt == 2) { feat = kv.ptr; flen = kv.len; }
      }
      if (!key || !feat) continue;
      const bool is_shape = klen == 5 && !memcmp(key, "shape", 5);
      const bool is_data = klen == 4 && !memcmp(key, "data", 4);
      if (!is_shape && !is_data) continue;
      const uint8_t* s = feat;
      const uint8_t* se = feat + flen;
      Field kind;
      while (next_field(s, se, kind)) {
        if (kind.wt != 2) continue;
        const uint8_t* t = kind.ptr;
        const uint8_t* te = kind.ptr + kind.len;
        Field item;
        while (next_field(t, te, item)) {
          if (item.num != 1) continue;
          if (is_data && kind.num == 1 && item.wt == 2) { data = item.ptr; dlen = item.len; }
          if (is_shape && kind.num == 3) {
            if (item.wt == 0 && ndim < 3) {
              shape[ndim++] = (int64_t)item.v;
            } else if (item.wt == 2) {
              const uint8_t* u = item.ptr;
              const uint8_t* ue = item.ptr + item.len;
              uint64_t v;
              while (u < ue && ndim < 3 && read_varint(u, ue, v)) shape[ndim++] = (int64_t)v;
            }
          }
        }
      }
    }
  }
  return ndim == 3 && data != nullptr;
}

}  // namespace

extern "C" {

uint32_t rt_crc32c(const uint8_t* p, long long n) { return crc32c(p, (size_t)n); }
uint32_t rt_masked_crc32c(const uint8_t* p, long long n) { return masked(crc32c(p, (size_t)n)); }

// Count the records of a file and, if `shape` is non-null, report the [C, H, W] of the first one.
// Returns the record count, or a negative error (-1 open, -2 framing, -3 crc, -4 parse).
long long rt_tfrecord_info(const char* path, int verify, long long* shape) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  const long long fsize = ftell(f);
  fseek(f, 0, SEEK_SET);
  long long n = 0;
  std::vector<uint8_t> buf;
  uint8_t head[12];
  long long rc = 0;
  while (true) {
    const size_t got = fread(head, 1, 12, f);
    if (got == 0) break;
    if (got < 12) { rc = -2; break; }
    uint64_t len;
    memcpy(&len, head, 8);
    uint32_t lcrc;
    memcpy(&lcrc, head + 8, 4);
    if (verify && lcrc != masked(crc32c(head, 8))) { rc = -3; break; }
    if (len > kMaxRecord) { rc = -2; break; }
    const bool need = verify || (n == 0 && shape);
    if (need) {
      buf.resize(len + 4);
      if (fread(buf.data(), 1, len + 4, f) != len + 4) { rc = -2; break; }
      if (verify) {
        uint32_t pcrc;
        memcpy(&pcrc, buf.data() + len, 4);
        if (pcrc != masked(crc32c(buf.data(), len))) { rc = -3; break; }
      }
      if (n == 0 && shape) {
        int64_t s[3];
        int nd;
        const uint8_t* d;
        uint64_t dl;
        if (!parse_image(buf.data(), buf.data() + len, s, nd, d, dl)) { rc = -4; break; }
        shape[0] = s[0]; shape[1] = s[1]; shape[2] = s[2];
      }
    } else if ((long long)len + 4 > fsize - ftell(f) || fseek(f, (long)(len + 4), SEEK_CUR) != 0) {
      rc = -2;
      break;
    }
    ++n;
  }
  fclose(f);
  return rc < 0 ? rc : n;
}

// Decode up to `max_images` image records into `out` (each exactly `item_bytes` bytes, shapes must
// match).  Returns the number decoded or a negative error (as above, -5 shape mismatch).
long long rt_tfrecord_decode_images(const char* path, uint8_t* out, long long max_images, long long item_bytes,
                                    int verify) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  std::vector<uint8_t> buf;
  uint8_t head[12];
  long long n = 0, rc = 0;
  while (n < max_images) {
    const size_t got = fread(head, 1, 12, f);
    if (got == 0) break;
    if (got < 12) { rc = -2; break; }
    uint64_t len;
    memcpy(&len, head, 8);
    if (len > kMaxRecord) { rc = -2; break; }
    buf.resize(len + 4);
    if (fread(buf.data(), 1, len + 4, f) != len + 4) { rc = -2; break; }
    if (verify) {
      uint32_t lcrc, pcrc;
      memcpy(&lcrc, head + 8, 4);
      memcpy(&pcrc, buf.data() + len, 4);
      if (lcrc != masked(crc32c(head, 8)) || pcrc != masked(crc32c(buf.data(), len))) { rc = -3; break; }
    }
    int64_t s[3];
    int nd;
    const uint8_t* d;
    uint64_t dl;
    if (!parse_image(buf.data(), buf.data() + len, s, nd, d, dl)) { rc = -4; break; }
    if ((long long)dl != item_bytes || s[0] * s[1] * s[2] != item_bytes) { rc = -5; break; }
    memcpy(out + n * item_bytes, d, dl);
    ++n;
  }
  fclose(f);
  return rc < 0 ? rc : n;
}

}  // extern "C"
