// Host-side test driver for the C++ runtime, built with -fsanitize=address,undefined
// (sanitizer CI variant of the host code).  Writes a TFRecord file of image Examples,
// decodes it through the runtime, then fuzzes it (truncations, random byte flips, hostile length
// varints): every call must return a value or an error code — never crash or read out of bounds.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../runtime/tfrecord.cpp"

static void put_varint(std::vector<uint8_t>& b, uint64_t v) {
  while (v >= 0x80) { b.push_back((uint8_t)(v | 0x80)); v >>= 7; }
  b.push_back((uint8_t)v);
}
static void put_ld(std::vector<uint8_t>& b, int field, const std::vector<uint8_t>& payload) {
  put_varint(b, (uint64_t)(field << 3) | 2);
  put_varint(b, payload.size());
  b.insert(b.end(), payload.begin(), payload.end());
}
static std::vector<uint8_t> example(int c, int h, int w, uint8_t seed) {
  std::vector<uint8_t> shape_packed, int64list, feat_shape, data, byteslist, feat_data, e1, e2, features, ex;
  for (int v : {c, h, w}) put_varint(shape_packed, (uint64_t)v);
  put_ld(int64list, 1, shape_packed);
  put_ld(feat_shape, 3, int64list);
  for (int i = 0; i < c * h * w; ++i) data.push_back((uint8_t)(seed + i));
  put_ld(byteslist, 1, data);
  put_ld(feat_data, 1, byteslist);
  put_ld(e1, 1, std::vector<uint8_t>{'s', 'h', 'a', 'p', 'e'});
  put_ld(e1, 2, feat_shape);
  put_ld(e2, 1, std::vector<uint8_t>{'d', 'a', 't', 'a'});
  put_ld(e2, 2, feat_data);
  put_ld(features, 1, e1);
  put_ld(features, 1, e2);
  put_ld(ex, 1, features);
  return ex;
}
static void write_file(const std::string& path, const std::vector<uint8_t>& bytes) {
  FILE* f = fopen(path.c_str(), "wb");
  fwrite(bytes.data(), 1, bytes.size(), f);
  fclose(f);
}
static std::vector<uint8_t> record_file(int n, int c, int h, int w) {
  std::vector<uint8_t> out;
  for (int i = 0; i < n; ++i) {
    std::vector<uint8_t> p = example(c, h, w, (uint8_t)i);
    uint64_t len = p.size();
    uint8_t head[8];
    memcpy(head, &len, 8);
    const uint32_t lc = rt_masked_crc32c(head, 8), pc = rt_masked_crc32c(p.data(), (long long)p.size());
    out.insert(out.end(), head, head + 8);
    out.insert(out.end(), (const uint8_t*)&lc, (const uint8_t*)&lc + 4);
    out.insert(out.end(), p.begin(), p.end());
    out.insert(out.end(), (const uint8_t*)&pc, (const uint8_t*)&pc + 4);
  }
  return out;
}

#define CHECK(x) do { if (!(x)) { fprintf(stderr, "CHECK failed: %s (line %d)\n", #x, __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const std::string path = dir + "/rt_test.tfrecords";
  // crc32c known answer
  CHECK(rt_crc32c((const uint8_t*)"123456789", 9) == 0xE3069283u);
  // round trip
  const int N = 37, C = 3, H = 8, W = 8;
  std::vector<uint8_t> good = record_file(N, C, H, W);
  write_file(path, good);
  long long shape[3] = {0, 0, 0};
  CHECK(rt_tfrecord_info(path.c_str(), 1, shape) == N);
  CHECK(shape[0] == C && shape[1] == H && shape[2] == W);
  std::vector<uint8_t> out((size_t)N * C * H * W);
  CHECK(rt_tfrecord_decode_images(path.c_str(), out.data(), N, C * H * W, 1) == N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < C * H * W; ++j) CHECK(out[(size_t)i * C * H * W + j] == (uint8_t)(i + j));
  CHECK(rt_tfrecord_info((dir + "/does_not_exist").c_str(), 0, nullptr) == -1);
  // fuzz: truncations and byte flips; results must be sane, sanitizers must stay quiet
  std::mt19937 rng(1234);
  int errors = 0, oks = 0;
  for (int it = 0; it < 3000; ++it) {
    std::vector<uint8_t> bad = good;
    const int mode = it % 3;
    if (mode == 0) {
      bad.resize(rng() % bad.size());
    } else if (mode == 1) {
      for (int k = 0; k < 1 + (int)(rng() % 8); ++k) bad[rng() % bad.size()] ^= (uint8_t)(1u << (rng() % 8));
    } else {  // hostile record length
      const uint64_t huge = ((uint64_t)rng() << 32) | rng();
      memcpy(bad.data(), &huge, 8);
    }
    write_file(path, bad);
    const int verify = (int)(rng() % 2);
    const long long n = rt_tfrecord_info(path.c_str(), verify, shape);
    const long long m = rt_tfrecord_decode_images(path.c_str(), out.data(), N, C * H * W, verify);
    CHECK(n <= N && m <= N);
    (m < 0 || n < 0) ? ++errors : ++oks;
  }
  printf("runtime tests ok (fuzz: %d rejected, %d accepted)\n", errors, oks);
  remove(path.c_str());
  return 0;
}
