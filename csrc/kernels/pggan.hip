// PG-GAN side kernels for gfx950 (SURVEY.md §2.4 K11 pixel norm, K15 RNG).
//
//  * rk_philox: counter-based Philox4x32-10 generator (uniform / normal / integer range).  The
//    counter is (element quad, call-site stream id, device step counter), so a captured hipGraph
//    that bumps the step counter once per replay draws fresh numbers every replay with no host
//    involvement — the property the graphed PG-GAN D/G steps rely on (pg_gans.py:1278,1297,1306
//    draw latents / mixing factors / minibatch indices every step).
//  * rk_lrelu_pixelnorm(_bwd): the generator's per-layer epilogue
//    z = PN(lrelu(x + b)),  PN(y) = y * rsqrt(mean_c(y^2) + eps)   (pg_gans.py:987-995, 853-869)
//    fused into one pass over NHWC rows: one wave per pixel, the channel vector lives in registers
//    (C <= 1024: up to 2 x 8 bf16 per lane), so the reduction is a 64-lane shuffle tree and the
//    tensor is read once and written once.  The backward recomputes y and the norm from x:
//    dy = r*dz - (r^3/C) * y * sum(dz*y),  dx = dy * (y_pre >= 0 ? 1 : slope).
#include "common.h"

namespace {

struct U4 { uint32_t v[4]; };

RK_DEV U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    const uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += W0; k1 += W1;
  }
  U4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}

// [0, 1) with 24 random mantissa bits; (0, 1] variant for the Box-Muller log
RK_DEV float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
RK_DEV float u01_open(uint32_t x) { return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f); }

// dist 0: a + b*U[0,1) (fp32)   1: a + b*N(0,1) (fp32)   2: floor(U*hi) (int32)
__global__ __launch_bounds__(256) void philox_kernel(void* __restrict__ out, long long n, int dist, int hi, float a,
                                                     float b, uint32_t k0, uint32_t k1, uint32_t stream_id,
                                                     const int* __restrict__ step) {
  const uint32_t st = step ? (uint32_t)step[0] : 0u;
  const long long quads = (n + 3) >> 2;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < quads;
       q += (long long)gridDim.x * blockDim.x) {
    const U4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), stream_id, st, k0, k1);
    float f[4];
    if (dist == 1) {
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const float rad = sqrtf(-2.0f * __logf(u01_open(r.v[j])));
        float s, c;
        __sincosf(6.283185307179586f * u01(r.v[j + 1]), &s, &c);
        f[j] = rad * c;
        f[j + 1] = rad * s;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) f[j] = u01(r.v[j]);
    }
    const long long base = q << 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long i = base + j;
      if (i >= n) break;
      if (dist == 2) {
        int v = (int)(f[j] * (float)hi);
        ((int*)out)[i] = v < hi ? v : hi - 1;
      } else {
        ((float*)out)[i] = a + b * f[j];
      }
    }
  }
}

// One wave per row of C channels (C % 8 == 0, C <= 64 * 8 * NV).  bias: fp32 [C] or null.
template <int NV>
__global__ __launch_bounds__(256) void lrelu_pn_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ bias,
                                                           int P, int C, float slope, float eps,
                                                           bf16* __restrict__ z) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= P) return;
  const uint4* xr = (const uint4*)(x + (long long)row * C);
  const int nvec = C >> 3;
  float y[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c8 = lane + v * 64;
    if (c8 < nvec) {
      unpack8(xr[c8], y[v]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = y[v][j] + (bias ? bias[c8 * 8 + j] : 0.f);
        t = t >= 0.f ? t : t * slope;
        y[v][j] = t;
        ss += t * t;
      }
    }
  }
  const float r = rsqrtf(wave_sum(ss) / (float)C + eps);
  uint4* zr = (uint4*)(z + (long long)row * C);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c8 = lane + v * 64;
    if (c8 < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = y[v][j] * r;
      zr[c8] = pack8(o);
    }
  }
}

template <int NV>
__global__ __launch_bounds__(256) void lrelu_pn_bwd_kernel(const bf16* __restrict__ x, const float* __restrict__ bias,
                                                           const bf16* __restrict__ dz, int P, int C, float slope,
                                                           float eps, bf16* __restrict__ dx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= P) return;
  const uint4* xr = (const uint4*)(x + (long long)row * C);
  const uint4* dr = (const uint4*)(dz + (long long)row * C);
  const int nvec = C >> 3;
  float y[NV][8], g[NV][8];
  float ss = 0.f, sd = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c8 = lane + v * 64;
    if (c8 < nvec) {
      unpack8(xr[c8], y[v]);
      unpack8(dr[c8], g[v]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pre = y[v][j] + (bias ? bias[c8 * 8 + j] : 0.f);
        const float t = pre >= 0.f ? pre : pre * slope;
        y[v][j] = pre;   // keep the pre-activation; the activated value is recomputed below
        ss += t * t;
        sd += t * g[v][j];
      }
    }
  }
  ss = wave_sum(ss);
  sd = wave_sum(sd);
  const float r = rsqrtf(ss / (float)C + eps);
  const float k = r * r * r * sd / (float)C;
  uint4* xo = (uint4*)(dx + (long long)row * C);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c8 = lane + v * 64;
    if (c8 < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pre = y[v][j];
        const float t = pre >= 0.f ? pre : pre * slope;
        const float dy = r * g[v][j] - k * t;
        o[j] = pre >= 0.f ? dy : dy * slope;
      }
      xo[c8] = pack8(o);
    }
  }
}

int grid_for(long long work, int cap) {
  long long g = (work + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" int rk_philox(void* out, long long n, int dist, int hi, float a, float b, unsigned long long seed,
                         unsigned int stream_id, const int* step, void* stream) {
  if (n <= 0) return RK_OK;
  if (dist < 0 || dist > 2 || (dist == 2 && hi <= 0)) return RK_EBADARG;
  hipLaunchKernelGGL(philox_kernel, dim3(grid_for((n + 3) / 4, 2048)), dim3(256), 0, (hipStream_t)stream, out, n,
                     dist, hi, a, b, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)stream_id, step);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_lrelu_pixelnorm(const void* x, const float* bias, const void* dz, int P, int C, float slope,
                                  float eps, void* out, void* stream) {
  if (P <= 0) return RK_OK;
  if (C % 8 || C > 1024) return RK_EUNSUPPORTED;
  const dim3 grid(rk_cdiv(P, 4)), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (dz == nullptr) {
    if (C <= 512)
      hipLaunchKernelGGL(lrelu_pn_fwd_kernel<1>, grid, block, 0, s, (const bf16*)x, bias, P, C, slope, eps, (bf16*)out);
    else
      hipLaunchKernelGGL(lrelu_pn_fwd_kernel<2>, grid, block, 0, s, (const bf16*)x, bias, P, C, slope, eps, (bf16*)out);
  } else {
    if (C <= 512)
      hipLaunchKernelGGL(lrelu_pn_bwd_kernel<1>, grid, block, 0, s, (const bf16*)x, bias, (const bf16*)dz, P, C, slope,
                         eps, (bf16*)out);
    else
      hipLaunchKernelGGL(lrelu_pn_bwd_kernel<2>, grid, block, 0, s, (const bf16*)x, bias, (const bf16*)dz, P, C, slope,
                         eps, (bf16*)out);
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}
