// Shared device helpers for the rafiki_amd gfx950 (MI355X / CDNA4) kernel library.
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC (channel-contiguous) bf16, so a 16-byte vector = 8 channels;
//   * GEMM-shaped work runs on v_mfma_f32_16x16x32_bf16 with fp32 accumulation;
//   * statistics / reductions accumulate in fp32 (fp64 in the tiny finalize kernels);
//   * every launcher is `extern "C"` and takes the HIP stream as an opaque pointer so the
//     Python side can hand in torch's current stream (graph-capture safe: no malloc/sync).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

#define RK_DEV __device__ __forceinline__

RK_DEV float bf2f(bf16 x) { return (float)x; }
RK_DEV bf16 f2bf(float x) { return (bf16)x; }

// 16-byte vector <-> 8 floats
RK_DEV void unpack8(const uint4 v, float (&f)[8]) {
  const bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)b[i];
}
RK_DEV uint4 pack8(const float (&f)[8]) {
  bf16x8 b;
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (bf16)f[i];
  return __builtin_bit_cast(uint4, b);
}

RK_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
RK_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks b and b+8 are dealt to the same XCD, so give each XCD a contiguous range of
// logical tile ids -> neighbouring tiles (which share operand panels) hit the same L2.
RK_DEV int xcd_remap(int orig, int nwg) {
  if (nwg <= 8) return orig;
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// x = hi + mid + lo: bf16 round-to-nearest of x, then of the residuals (x - hi and x - hi - mid are exact
// in fp32) — the operand pieces of the X6 (fp32-accurate split-bf16) GEMMs, written once by producers
RK_DEV void split3v(float x, bf16& h, bf16& m, bf16& l) {
  h = (bf16)x;
  const float r = x - (float)h;
  m = (bf16)r;
  l = (bf16)(r - (float)m);
}

static inline int rk_cdiv(int a, int b) { return (a + b - 1) / b; }
static inline int rk_log2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return ((1 << l) == v) ? l : -1;
}

enum RkStatus { RK_OK = 0, RK_EBADARG = -1, RK_EUNSUPPORTED = -2, RK_ELAUNCH = -3 };

#define RK_LAUNCH_CHECK() \
  do { if (hipGetLastError() != hipSuccess) return RK_ELAUNCH; } while (0)
