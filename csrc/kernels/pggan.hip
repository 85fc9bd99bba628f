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
//  * rk_mbstd (K12, pg_gans.py:1070-1082): minibatch-stddev feature, its backward and the backward
//    of that backward (WGAN-GP differentiates the discriminator twice).  One block per stddev
//    group: the group's g samples are read together, the statistics never leave registers/LDS.
//    With n = N/g, sample i = k*n + j belongs to group j (tf.reshape(x, [g, -1, ...])); with
//    `segs` > 1 the batch is `segs` independent minibatches (grouping stays inside each), so
//    several D evaluations can share one batched forward.
//      s_pc = sqrt(var_k x_kpc + 1e-8),  f_j = mean_pc s_pc,  out = [x, f_j, 0-pad]
//      bwd:   gx_k = gout_k[:C] + G_j * (x_k - mu) / (g s P C),   G_j = sum_{k,p} gout_k[p, C]
//      bwd2:  gg_out = [ggx, H_j, 0],  H_j = sum_{k,pc} ggx_k (x_k - mu) / (g s P C)
//             g_x_k = G_j / (g P C s) * (ggx_k - mean(ggx) - u_k * mean(ggx * u)),  u = (x - mu) / s
#include "common.h"
#include "philox.h"

#include <algorithm>

namespace {


// 8 consecutive channels of a bf16 or fp32 NHWC row <-> 8 floats (the PG-GAN ops run in either
// precision: bf16 for the opt-in fast path, fp32 — the reference's precision — by default)
template <class T> RK_DEV void ld8(const T* p, float (&f)[8]);
template <> RK_DEV void ld8<bf16>(const bf16* p, float (&f)[8]) { unpack8(*(const uint4*)p, f); }
template <> RK_DEV void ld8<float>(const float* p, float (&f)[8]) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[i] = a[i]; f[4 + i] = b[i]; }
}
template <class T> RK_DEV void st8(T* p, const float (&f)[8]);
template <> RK_DEV void st8<bf16>(bf16* p, const float (&f)[8]) { *(uint4*)p = pack8(f); }
template <> RK_DEV void st8<float>(float* p, const float (&f)[8]) {
  *(f32x4*)p = f32x4{f[0], f[1], f[2], f[3]};
  *(f32x4*)(p + 4) = f32x4{f[4], f[5], f[6], f[7]};
}

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
template <int NV, class T>
__global__ __launch_bounds__(256) void lrelu_pn_fwd_kernel(const T* __restrict__ x, const float* __restrict__ bias,
                                                           int P, int C, float slope, float eps,
                                                           T* __restrict__ z) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= P) return;
  const T* xr = x + (long long)row * C;
  const int nvec = C >> 3;
  float y[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c8 = lane + v * 64;
    if (c8 < nvec) {
      ld8(xr + c8 * 8, y[v]);
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
  T* zr = z + (long long)row * C;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c8 = lane + v * 64;
    if (c8 < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = y[v][j] * r;
      st8(zr + c8 * 8, o);
    }
  }
}

template <int NV, class T>
__global__ __launch_bounds__(256) void lrelu_pn_bwd_kernel(const T* __restrict__ x, const float* __restrict__ bias,
                                                           const T* __restrict__ dz, int P, int C, float slope,
                                                           float eps, T* __restrict__ dx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= P) return;
  const T* xr = x + (long long)row * C;
  const T* dr = dz + (long long)row * C;
  const int nvec = C >> 3;
  float y[NV][8], g[NV][8];
  float ss = 0.f, sd = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c8 = lane + v * 64;
    if (c8 < nvec) {
      ld8(xr + c8 * 8, y[v]);
      ld8(dr + c8 * 8, g[v]);
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
  T* xo = dx + (long long)row * C;
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
      st8(xo + c8 * 8, o);
    }
  }
}

constexpr int MB_MAXG = 8;

// sample index of member k of group J (segs independent minibatches of N/segs samples each)
RK_DEV long long mb_sample(int J, int k, int N, int g, int segs) {
  const int ns = N / segs, n = ns / g;
  const int sg = J / n, j = J - sg * n;
  return (long long)sg * ns + (long long)k * n + j;
}

RK_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

// group statistics of one channel element: mean and 1/s over the g members
template <int G>
RK_DEV void mb_stats(const float (&xv)[G], int g, float& mu, float& rs) {
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < G; ++k) if (k < g) m += xv[k];
  m /= (float)g;
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < G; ++k) if (k < g) { const float d = xv[k] - m; v += d * d; }
  mu = m;
  rs = rsqrtf(v / (float)g + 1e-8f);
}

// mode 0: forward   out[N,P,Cp] = [x, f, 0]
// mode 1: backward  out[N,P,C]  = gx from gout [N,P,Cp]
// mode 2: backward of backward: out = g_x [N,P,C], out2 = gg_out [N,P,Cp]; a = ggx [N,P,C], b = gout
template <class T>
__global__ __launch_bounds__(256) void mbstd_kernel(int mode, const T* __restrict__ x, const T* __restrict__ a,
                                                    const T* __restrict__ b, int N, int P, int C, int Cp, int g,
                                                    int segs, T* __restrict__ out, T* __restrict__ out2) {
  __shared__ float red[4];
  const int J = blockIdx.x;
  const int PC = P * C;
  const float inv = 1.0f / ((float)g * (float)PC);
  long long smp[MB_MAXG];
#pragma unroll
  for (int k = 0; k < MB_MAXG; ++k) smp[k] = k < g ? mb_sample(J, k, N, g, segs) : 0;
  float red0 = 0.f;
  if (mode == 0) {
    for (int e = threadIdx.x; e < PC; e += blockDim.x) {
      float xv[MB_MAXG], mu, rs;
#pragma unroll
      for (int k = 0; k < MB_MAXG; ++k) xv[k] = k < g ? (float)x[smp[k] * PC + e] : 0.f;
      mb_stats<MB_MAXG>(xv, g, mu, rs);
      red0 += 1.0f / rs;   // s = sqrt(var + eps)
    }
    const float f = block_sum(red0, red) / (float)PC;
    for (int e = threadIdx.x; e < P * Cp; e += blockDim.x) {
      const int p = e / Cp, c = e - p * Cp;
#pragma unroll
      for (int k = 0; k < MB_MAXG; ++k) {
        if (k >= g) break;
        const float v = c < C ? (float)x[smp[k] * PC + (long long)p * C + c] : (c == C ? f : 0.f);
        out[smp[k] * P * Cp + e] = (T)v;
      }
    }
    return;
  }
  // G_j = sum over the group's extra-channel gradient (mode 1: gout = a; mode 2: gout = b)
  const T* gout = mode == 1 ? a : b;
  float gs = 0.f;
  for (int t = threadIdx.x; t < g * P; t += blockDim.x) {
    const int k = t / P, p = t - k * P;
    long long sk = 0;
#pragma unroll
    for (int q = 0; q < MB_MAXG; ++q) if (q == k) sk = smp[q];
    gs += (float)gout[(sk * P + p) * Cp + C];
  }
  const float Gj = block_sum(gs, red);
  if (mode == 1) {
    for (int e = threadIdx.x; e < PC; e += blockDim.x) {
      const int p = e / C, c = e - p * C;
      float xv[MB_MAXG], mu, rs;
#pragma unroll
      for (int k = 0; k < MB_MAXG; ++k) xv[k] = k < g ? (float)x[smp[k] * PC + e] : 0.f;
      mb_stats<MB_MAXG>(xv, g, mu, rs);
#pragma unroll
      for (int k = 0; k < MB_MAXG; ++k) {
        if (k >= g) break;
        const float go = (float)gout[(smp[k] * P + p) * Cp + c];
        out[smp[k] * PC + e] = (T)(go + Gj * (xv[k] - mu) * rs * inv);
      }
    }
    return;
  }
  // mode 2: g_x (gg_out comes from mbstd_h_kernel)
  for (int e = threadIdx.x; e < PC; e += blockDim.x) {
    float xv[MB_MAXG], mu, rs;
#pragma unroll
    for (int k = 0; k < MB_MAXG; ++k) xv[k] = k < g ? (float)x[smp[k] * PC + e] : 0.f;
    mb_stats<MB_MAXG>(xv, g, mu, rs);
    float m1 = 0.f, m2 = 0.f;
#pragma unroll
    for (int k = 0; k < MB_MAXG; ++k) {
      if (k >= g) break;
      const float gg = (float)a[smp[k] * PC + e];
      const float u = (xv[k] - mu) * rs;
      m1 += gg;
      m2 += gg * u;
    }
    const float kk = Gj * rs * inv;
    m1 /= (float)g;
    m2 /= (float)g;
#pragma unroll
    for (int k = 0; k < MB_MAXG; ++k) {
      if (k >= g) break;
      const float gg = (float)a[smp[k] * PC + e];
      const float u = (xv[k] - mu) * rs;
      out[smp[k] * PC + e] = (T)(kk * (gg - m1 - u * m2));
    }
  }
}

template <class T>
__global__ __launch_bounds__(256) void mbstd_h_kernel(const T* __restrict__ x, const T* __restrict__ a, int N,
                                                      int P, int C, int Cp, int g, int segs, T* __restrict__ out2) {
  __shared__ float red[4];
  const int J = blockIdx.x;
  const int PC = P * C;
  const float inv = 1.0f / ((float)g * (float)PC);
  long long smp[MB_MAXG];
#pragma unroll
  for (int k = 0; k < MB_MAXG; ++k) smp[k] = k < g ? mb_sample(J, k, N, g, segs) : 0;
  float hs = 0.f;
  for (int e = threadIdx.x; e < PC; e += blockDim.x) {
    float xv[MB_MAXG], mu, rs;
#pragma unroll
    for (int k = 0; k < MB_MAXG; ++k) xv[k] = k < g ? (float)x[smp[k] * PC + e] : 0.f;
    mb_stats<MB_MAXG>(xv, g, mu, rs);
#pragma unroll
    for (int k = 0; k < MB_MAXG; ++k) {
      if (k >= g) break;
      hs += (float)a[smp[k] * PC + e] * (xv[k] - mu) * rs;
    }
  }
  const float H = block_sum(hs, red) * inv;
  for (int e = threadIdx.x; e < P * Cp; e += blockDim.x) {
    const int p = e / Cp, c = e - p * Cp;
#pragma unroll
    for (int k = 0; k < MB_MAXG; ++k) {
      if (k >= g) break;
      const float v = c < C ? (float)a[smp[k] * PC + (long long)p * C + c] : (c == C ? H : 0.f);
      out2[smp[k] * P * Cp + e] = (T)v;
    }
  }
}

// ---- vectorised minibatch-stddev (C % 8 == 0): stage A reduces per-group partial sums over
// row chunks (grid groups x chunks, deterministic), stage B recomputes the per-channel group
// statistics and writes every member's output, one thread per (group, 8-channel vector).
// part[J][chunk][2]: mode 0 {sum s, -}; mode 1 {sum gout[.., C], -}; mode 2 {G sum, H sum}.
template <int G, class T>
RK_DEV void mb_load(const T* __restrict__ base, const long long (&smp)[G], long long stride, long long off,
                    int g, float (&v)[G][8]) {
#pragma unroll
  for (int k = 0; k < G; ++k)
    if (k < g) ld8(base + smp[k] * stride + off, v[k]);
}

template <int G>
RK_DEV void mb_vstats(const float (&xv)[G][8], int g, float (&mu)[8], float (&rs)[8]) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k) if (k < g) m += xv[k][c];
    m /= (float)g;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k) if (k < g) { const float d = xv[k][c] - m; v += d * d; }
    mu[c] = m;
    rs[c] = rsqrtf(v / (float)g + 1e-8f);
  }
}

// G: the compile-time group-size bound (4 for the usual group of 4: half the registers of G)
template <int G, class T>
__global__ __launch_bounds__(256) void mbstd_vec_a_kernel(int mode, const T* __restrict__ x,
                                                          const T* __restrict__ a, const T* __restrict__ gout,
                                                          int N, int P, int C, int Cp, int g, int segs, int chunks,
                                                          float* __restrict__ part) {
  __shared__ float red[4];
  const int J = blockIdx.x, ch = blockIdx.y;
  const int C8 = C >> 3, V = P * C8;
  long long smp[G];
#pragma unroll
  for (int k = 0; k < G; ++k) smp[k] = k < g ? mb_sample(J, k, N, g, segs) : 0;
  const int per = (V + chunks - 1) / chunks, v0 = ch * per, v1 = min(V, v0 + per);
  float s0 = 0.f, s1 = 0.f;
  if (mode != 1) {
    for (int v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
      float xv[G][8], mu[8], rs[8];
      mb_load<G>(x, smp, (long long)P * C, (long long)v * 8, g, xv);
      mb_vstats(xv, g, mu, rs);
      if (mode == 0) {
#pragma unroll
        for (int c = 0; c < 8; ++c) s0 += 1.0f / rs[c];
      } else {
        float av[G][8];
        mb_load<G>(a, smp, (long long)P * C, (long long)v * 8, g, av);
#pragma unroll
        for (int k = 0; k < G; ++k)
          if (k < g)
#pragma unroll
            for (int c = 0; c < 8; ++c) s1 += av[k][c] * (xv[k][c] - mu[c]) * rs[c];
      }
    }
  }
  if (mode != 0) {   // G_j: the extra channel of gout over this chunk's pixels, all members
    const int p0 = (int)(((long long)P * ch) / chunks), p1 = (int)(((long long)P * (ch + 1)) / chunks);
    for (int t = threadIdx.x; t < g * (p1 - p0); t += blockDim.x) {
      const int k = t / (p1 - p0), p = p0 + t - k * (p1 - p0);
      long long sk = 0;
#pragma unroll
      for (int q = 0; q < G; ++q) if (q == k) sk = smp[q];
      s0 += (float)gout[(sk * P + p) * Cp + C];
    }
  }
  s0 = block_sum(s0, red);
  s1 = block_sum(s1, red);
  if (threadIdx.x == 0) {
    part[((long long)J * chunks + ch) * 2] = s0;
    part[((long long)J * chunks + ch) * 2 + 1] = s1;
  }
}

template <int G, class T>
__global__ __launch_bounds__(256) void mbstd_vec_b_kernel(int mode, const T* __restrict__ x,
                                                          const T* __restrict__ a, const T* __restrict__ gout,
                                                          int N, int P, int C, int Cp, int g, int segs, int chunks,
                                                          const float* __restrict__ part, T* __restrict__ out,
                                                          T* __restrict__ out2) {
  const int C8 = C >> 3, V = P * C8;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int J = (int)(t / V), v = (int)(t - (long long)J * V);
  if (J >= N / g) return;
  long long smp[G];
#pragma unroll
  for (int k = 0; k < G; ++k) smp[k] = k < g ? mb_sample(J, k, N, g, segs) : 0;
  float S0 = 0.f, S1 = 0.f;
  for (int c = 0; c < chunks; ++c) {
    S0 += part[((long long)J * chunks + c) * 2];
    S1 += part[((long long)J * chunks + c) * 2 + 1];
  }
  const long long PC = (long long)P * C, PCp = (long long)P * Cp;
  const int p = v / C8, c8 = v - p * C8;
  const float inv = 1.0f / ((float)g * (float)PC);
  float xv[G][8], mu[8], rs[8];
  if (mode == 0) {
    mb_load<G>(x, smp, PC, (long long)v * 8, g, xv);
#pragma unroll
    for (int k = 0; k < G; ++k) {
      if (k >= g) break;
      st8(out + smp[k] * PCp + (long long)p * Cp + c8 * 8, xv[k]);
      if (c8 == 0) {                        // [f, 0 ...] over the padded tail C .. Cp-1 (8 per store)
        float f[8] = {S0 / (float)PC, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int t = C; t < Cp; t += 8, f[0] = 0.f) st8(out + smp[k] * PCp + (long long)p * Cp + t, f);
      }
    }
    return;
  }
  mb_load<G>(x, smp, PC, (long long)v * 8, g, xv);
  mb_vstats(xv, g, mu, rs);
  if (mode == 1) {
    float go[G][8];
    mb_load<G>(gout, smp, PCp, (long long)p * Cp + c8 * 8, g, go);
#pragma unroll
    for (int k = 0; k < G; ++k) {
      if (k >= g) break;
      float o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = go[k][c] + S0 * (xv[k][c] - mu[c]) * rs[c] * inv;
      st8(out + smp[k] * PC + (long long)v * 8, o);
    }
    return;
  }
  // mode 2: g_x -> out, gg_out -> out2
  float av[G][8];
  mb_load<G>(a, smp, PC, (long long)v * 8, g, av);
  float m1[8], m2[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k)
      if (k < g) { s1 += av[k][c]; s2 += av[k][c] * (xv[k][c] - mu[c]) * rs[c]; }
    m1[c] = s1 / (float)g;
    m2[c] = s2 / (float)g;
  }
#pragma unroll
  for (int k = 0; k < G; ++k) {
    if (k >= g) break;
    float o[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float u = (xv[k][c] - mu[c]) * rs[c];
      o[c] = S0 * rs[c] * inv * (av[k][c] - m1[c] - u * m2[c]);
    }
    st8(out + smp[k] * PC + (long long)v * 8, o);
    st8(out2 + smp[k] * PCp + (long long)p * Cp + c8 * 8, av[k]);
    if (c8 == 0) {
      float f[8] = {S1 * inv, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int t = C; t < Cp; t += 8, f[0] = 0.f) st8(out2 + smp[k] * PCp + (long long)p * Cp + t, f);
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

namespace {

template <class T>
int mbstd_launch(int mode, const void* x, const void* a, const void* b, int N, int P, int C, int Cp, int g, int segs,
                 void* out, void* out2, float* part, hipStream_t s) {
  if (g < 1 || g > MB_MAXG || segs < 1 || N % segs || (N / segs) % g || Cp <= C || mode < 0 || mode > 2)
    return RK_EBADARG;
  const dim3 grid(N / g), block(256);
  if (part && C % 8 == 0 && (Cp - C) % 8 == 0 && Cp - C <= 64) {   // the feature + zero tail in 8-wide stores
    const int groups = N / g;
    const int chunks = std::max(1, std::min(16, 1024 / groups));
    const T* gout = (const T*)(mode == 1 ? a : b);
    const long long threads = (long long)groups * P * (C / 8);
    if (g <= 4) {
      hipLaunchKernelGGL((mbstd_vec_a_kernel<4, T>), dim3(groups, chunks), block, 0, s, mode, (const T*)x,
                         (const T*)a, gout, N, P, C, Cp, g, segs, chunks, part);
      hipLaunchKernelGGL((mbstd_vec_b_kernel<4, T>), dim3((unsigned)((threads + 255) / 256)), block, 0, s, mode,
                         (const T*)x, (const T*)a, gout, N, P, C, Cp, g, segs, chunks, part, (T*)out, (T*)out2);
    } else {
      hipLaunchKernelGGL((mbstd_vec_a_kernel<MB_MAXG, T>), dim3(groups, chunks), block, 0, s, mode, (const T*)x,
                         (const T*)a, gout, N, P, C, Cp, g, segs, chunks, part);
      hipLaunchKernelGGL((mbstd_vec_b_kernel<MB_MAXG, T>), dim3((unsigned)((threads + 255) / 256)), block, 0, s,
                         mode, (const T*)x, (const T*)a, gout, N, P, C, Cp, g, segs, chunks, part, (T*)out,
                         (T*)out2);
    }
    RK_LAUNCH_CHECK();
    return RK_OK;
  }
  hipLaunchKernelGGL(mbstd_kernel<T>, grid, block, 0, s, mode, (const T*)x, (const T*)a, (const T*)b, N, P, C, Cp, g,
                     segs, (T*)out, (T*)out2);
  if (mode == 2)
    hipLaunchKernelGGL(mbstd_h_kernel<T>, grid, block, 0, s, (const T*)x, (const T*)a, N, P, C, Cp, g, segs, (T*)out2);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

template <class T>
int lrelu_pn_launch(const void* x, const float* bias, const void* dz, int P, int C, float slope, float eps, void* out,
                    hipStream_t s) {
  if (P <= 0) return RK_OK;
  if (C % 8 || C > 1024) return RK_EUNSUPPORTED;
  const dim3 grid(rk_cdiv(P, 4)), block(256);
  if (dz == nullptr) {
    if (C <= 512)
      hipLaunchKernelGGL((lrelu_pn_fwd_kernel<1, T>), grid, block, 0, s, (const T*)x, bias, P, C, slope, eps, (T*)out);
    else
      hipLaunchKernelGGL((lrelu_pn_fwd_kernel<2, T>), grid, block, 0, s, (const T*)x, bias, P, C, slope, eps, (T*)out);
  } else {
    if (C <= 512)
      hipLaunchKernelGGL((lrelu_pn_bwd_kernel<1, T>), grid, block, 0, s, (const T*)x, bias, (const T*)dz, P, C, slope,
                         eps, (T*)out);
    else
      hipLaunchKernelGGL((lrelu_pn_bwd_kernel<2, T>), grid, block, 0, s, (const T*)x, bias, (const T*)dz, P, C, slope,
                         eps, (T*)out);
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}

}  // namespace

// part: fp32 scratch of >= (N/g) * 16 * 2 floats (vectorised path, C % 8 == 0 and Cp == C + 8).
// rk_mbstd / rk_lrelu_pixelnorm: bf16 tensors; the _f32 entry points: fp32 tensors.
extern "C" int rk_mbstd(int mode, const void* x, const void* a, const void* b, int N, int P, int C, int Cp, int g,
                        int segs, void* out, void* out2, float* part, void* stream) {
  return mbstd_launch<bf16>(mode, x, a, b, N, P, C, Cp, g, segs, out, out2, part, (hipStream_t)stream);
}

extern "C" int rk_mbstd_f32(int mode, const void* x, const void* a, const void* b, int N, int P, int C, int Cp, int g,
                            int segs, void* out, void* out2, float* part, void* stream) {
  return mbstd_launch<float>(mode, x, a, b, N, P, C, Cp, g, segs, out, out2, part, (hipStream_t)stream);
}

extern "C" int rk_lrelu_pixelnorm(const void* x, const float* bias, const void* dz, int P, int C, float slope,
                                  float eps, void* out, void* stream) {
  return lrelu_pn_launch<bf16>(x, bias, dz, P, C, slope, eps, out, (hipStream_t)stream);
}

extern "C" int rk_lrelu_pixelnorm_f32(const void* x, const float* bias, const void* dz, int P, int C, float slope,
                                      float eps, void* out, void* stream) {
  return lrelu_pn_launch<float>(x, bias, dz, P, C, slope, eps, out, (hipStream_t)stream);
}

// ------------------------------------------------------------------------------ leaky-ReLU gate
// g = gy * (y > 0 ? 1 : slope): the gradient through a leaky ReLU read from its OUTPUT y (same sign as the
// input).  Linear in gy, so the autograd Function applies the same gate to differentiate it again
// (WGAN-GP double backward).  The _colsum form also reduces g over rows (the conv bias gradient) in
// the same pass: 64 channels per block, gridDim.y row chunks write partial sums to part + y * C.
namespace {

__global__ __launch_bounds__(256) void lrelu_gate_kernel(const float4* __restrict__ gy, const float4* __restrict__ y,
                                                         float4* __restrict__ out, long long n4, float slope) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 g = gy[i], v = y[i];
    out[i] = make_float4(v.x > 0.f ? g.x : g.x * slope, v.y > 0.f ? g.y : g.y * slope,
                         v.z > 0.f ? g.z : g.z * slope, v.w > 0.f ? g.w : g.w * slope);
  }
}

__global__ __launch_bounds__(256) void lrelu_gate_colsum_kernel(const float* __restrict__ gy, const float* __restrict__ y,
                                                                float* __restrict__ out, int R, int C, float slope,
                                                                float* __restrict__ part) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  const int per = (R + gridDim.y - 1) / gridDim.y, r0 = blockIdx.y * per, r1 = min(R, r0 + per);
  float s = 0.f;
  if (c < C)
    for (int r = r0 + q; r < r1; r += 4) {
      const long long i = (long long)r * C + c;
      const float g = y[i] > 0.f ? gy[i] : gy[i] * slope;
      out[i] = g;
      s += g;
    }
  red[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && c < C)
    part[(long long)blockIdx.y * C + c] = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

}  // namespace

extern "C" int rk_lrelu_gate_f32(const float* gy, const float* y, float* out, long long n, float slope, void* stream) {
  if (n <= 0 || (n & 3)) return RK_EUNSUPPORTED;
  const long long n4 = n / 4;
  const unsigned blocks = (unsigned)std::min<long long>((n4 + 255) / 256, 4096);
  hipLaunchKernelGGL(lrelu_gate_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4*)gy,
                     (const float4*)y, (float4*)out, n4, slope);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_lrelu_gate_colsum4_f32(const float* gy, const float* y, float* g, int R, int C, float slope,
                                         float* part, int chunks, void* stream);   // bnf.hip (vectorised)

extern "C" int rk_lrelu_gate_colsum_f32(const float* gy, const float* y, float* out, int R, int C, float slope,
                                        float* part, int chunks, void* stream) {
  if (R <= 0 || C <= 0 || chunks < 1) return RK_EBADARG;
  if (rk_lrelu_gate_colsum4_f32(gy, y, out, R, C, slope, part, chunks, stream) == RK_OK) return RK_OK;
  hipLaunchKernelGGL(lrelu_gate_colsum_kernel, dim3(rk_cdiv(C, 64), chunks), dim3(256), 0, (hipStream_t)stream, gy, y,
                     out, R, C, slope, part);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// ------------------------------------------------------------------------------ WGAN-GP loss head
// The D loss of _D_wgangp_acgan (pg_gans.py:1291-1315) without labels, per sample r < mb:
//   loss_r = fake_r - real_r + lam (|g_r| - t)^2 + eps real_r^2
// with real_r / fake_r = column 0 of the discriminator's raw output rows r / mb + r (ld floats apart) and
// g_r the penalty gradient row (P floats); the G loss (pg_gans.py:1276-1289) is loss_r = -s_r (P = 0).
// Two launches forward (one block per sample row: norm + per-row terms into rows[4][mb]; one block: the
// four means in a fixed order -> loss, acc += means) and one backward replace the ~30 small PyTorch
// kernels of the composed loss (slices, sub, lerp-free penalty chain, addcmul, mean and their backward).
namespace {

RK_DEV float block_sum256(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();   // red may still be read by a previous call
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void wgan_rows_kernel(const float* __restrict__ s, int ld, int mb,
                                                        const float* __restrict__ g, int P, float lam, float target,
                                                        float eps, float* __restrict__ rows) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  float ss = 0.f;
  if (P > 0) {
    const float* gr = g + (long long)r * P;
    if ((P & 3) == 0) {
      for (int i = threadIdx.x; i < P / 4; i += 256) {
        const f32x4 v = *(const f32x4*)(gr + 4 * i);
        ss += (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
      }
    } else {
      for (int i = threadIdx.x; i < P; i += 256) ss += gr[i] * gr[i];
    }
  }
  ss = block_sum256(ss, red);
  if (threadIdx.x == 0) {
    float loss, real = 0.f, fake = 0.f, n = 0.f;
    if (P > 0) {
      real = s[(long long)r * ld];
      fake = s[(long long)(mb + r) * ld];
      n = sqrtf(ss);
      const float d = n - target;
      loss = (fake - real) + lam * d * d + eps * real * real;
    } else {
      loss = -s[(long long)r * ld];
    }
    rows[r] = loss;
    rows[mb + r] = real;
    rows[2 * mb + r] = fake;
    rows[3 * mb + r] = n;
  }
}

__global__ __launch_bounds__(256) void wgan_final_kernel(const float* __restrict__ rows, int mb, int nstat,
                                                         float* __restrict__ loss, float* __restrict__ acc) {
  __shared__ float red[4];
  for (int k = 0; k < nstat; ++k) {
    float a = 0.f;
    for (int i = threadIdx.x; i < mb; i += 256) a += rows[k * mb + i];
    a = block_sum256(a, red) / (float)mb;
    if (threadIdx.x == 0) {
      if (k == 0) *loss = a;
      if (acc) acc[k] += a;
    }
  }
}

// ds: d loss / d s over the whole raw output (zeros off column 0); dg = go lam 2 (n - t) / n / mb * g
__global__ __launch_bounds__(256) void wgan_bwd_kernel(const float* __restrict__ gl, const float* __restrict__ s,
                                                       int ld, int mb, const float* __restrict__ g, int P, float lam,
                                                       float target, float eps, const float* __restrict__ rows,
                                                       float* __restrict__ ds, float* __restrict__ dg) {
  const int r = blockIdx.x;
  const float go = *gl / (float)mb;
  if (P > 0) {
    const float n = rows[3 * mb + r];
    const float c = go * lam * 2.f * (n - target) / fmaxf(n, 1e-30f);
    const float* gr = g + (long long)r * P;
    float* dr = dg + (long long)r * P;
    if ((P & 3) == 0) {
      for (int i = threadIdx.x; i < P / 4; i += 256) *(f32x4*)(dr + 4 * i) = *(const f32x4*)(gr + 4 * i) * c;
    } else {
      for (int i = threadIdx.x; i < P; i += 256) dr[i] = gr[i] * c;
    }
    for (int j = threadIdx.x; j < ld; j += 256) {
      const float real = s[(long long)r * ld];
      ds[(long long)r * ld + j] = j == 0 ? go * (2.f * eps * real - 1.f) : 0.f;
      ds[(long long)(mb + r) * ld + j] = j == 0 ? go : 0.f;
    }
  } else {
    for (int j = threadIdx.x; j < ld; j += 256) ds[(long long)r * ld + j] = j == 0 ? -go : 0.f;
  }
}

}  // namespace

namespace {

// The D step's inputs in one pass (pg_gans.py:1297-1306): rf = [reals; fakes] (one batched D evaluation) and
// mixed_r = reals_r + (fakes_r - reals_r) alpha_r (the penalty's interpolates), P floats per sample.
__global__ __launch_bounds__(256) void wgan_mix_kernel(const float* __restrict__ reals, const float* __restrict__ fakes,
                                                       const float* __restrict__ alpha, float* __restrict__ rf,
                                                       float* __restrict__ mixed, int mb, int P4) {
  const long long n4 = (long long)mb * P4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int r = (int)(i / P4);
    const f32x4 a = ((const f32x4*)reals)[i], b = ((const f32x4*)fakes)[i];
    ((f32x4*)rf)[i] = a;
    ((f32x4*)rf)[n4 + i] = b;
    ((f32x4*)mixed)[i] = a + (b - a) * alpha[r];
  }
}

}  // namespace

// P > 0: D loss (s has 2 mb rows: reals then fakes; g [mb][P]); P == 0: G loss (s has mb rows).
// rows: scratch [4][mb]; acc (optional): += the means (loss, real, fake, |g|) (nstat = 4) or loss (1).
extern "C" int rk_wgan_loss_fwd(const float* s, int ld, int mb, const float* g, int P, float lam, float target,
                                float eps, float* rows, float* loss, float* acc, void* stream) {
  if (mb <= 0 || ld <= 0 || P < 0 || (P > 0 && !g) || !rows || !loss) return RK_EBADARG;
  hipLaunchKernelGGL(wgan_rows_kernel, dim3(mb), dim3(256), 0, (hipStream_t)stream, s, ld, mb, g, P, lam, target, eps,
                     rows);
  RK_LAUNCH_CHECK();
  hipLaunchKernelGGL(wgan_final_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, rows, mb, P > 0 ? 4 : 1, loss,
                     acc);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wgan_mix(const float* reals, const float* fakes, const float* alpha, float* rf, float* mixed, int mb,
                           int P, void* stream) {
  if (mb <= 0 || P <= 0 || (P & 3)) return RK_EUNSUPPORTED;
  const long long n4 = (long long)mb * (P / 4);
  const unsigned blocks = (unsigned)std::min<long long>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(wgan_mix_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, reals, fakes, alpha, rf, mixed,
                     mb, P / 4);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wgan_loss_bwd(const float* gl, const float* s, int ld, int mb, const float* g, int P, float lam,
                                float target, float eps, const float* rows, float* ds, float* dg, void* stream) {
  if (mb <= 0 || ld <= 0 || P < 0 || (P > 0 && (!g || !dg)) || !ds || !gl) return RK_EBADARG;
  hipLaunchKernelGGL(wgan_bwd_kernel, dim3(mb), dim3(256), 0, (hipStream_t)stream, gl, s, ld, mb, g, P, lam, target,
                     eps, rows, ds, dg);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
