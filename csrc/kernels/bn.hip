// BatchNorm (+ReLU/LeakyReLU, +2x2 max-pool) forward/backward for NHWC bf16 activations on gfx950.
//
// Training-mode BN over a conv output y[P][C] (P = N*H*W pixels):
//   forward : per-channel (sum, sumsq) partials come from the conv epilogue (igemm FLAG_STATS) or
//             from rk_channel_stats; rk_bn_finalize_fwd reduces them in fp64 -> mean/rstd and the
//             folded affine (scale = gamma*rstd, shift = beta - mean*scale), updates running stats;
//             rk_bn_act_fwd applies scale/shift + activation (+ 2x2 max-pool) in one streaming pass.
//   backward: rk_bn_bwd_reduce recomputes z = y*scale+shift, routes the upstream gradient through
//             pool argmax and the activation mask, and reduces (sum dz, sum dz*xhat) per channel
//             into per-block partial rows (deterministic, no atomics); rk_bn_finalize_bwd turns
//             them into dgamma/dbeta and the per-channel coefficients of
//             dy = k1*dz + k2*y + k3; rk_bn_bwd_apply streams dy out.
// No normalised activation is ever stored: backward recomputes it from y (saves a full write and
// read of every activation per layer).
//
// Reference parity: Keras BatchNormalization in TfFeedForward.py:148-149, ReLU
// epilogues (K7), VGG max-pool (K10), pg_gans lrelu (pg_gans.py:987-990).
#include "common.h"

namespace {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2 };

RK_DEV float act_f(float z, int act, float slope) {
  if (act == ACT_RELU) return fmaxf(z, 0.f);
  if (act == ACT_LRELU) return z > 0.f ? z : z * slope;
  return z;
}
RK_DEV float act_d(float z, int act, float slope) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_LRELU) return z > 0.f ? 1.f : slope;
  return 1.f;
}

// ---- per-channel stats of an arbitrary [P][C] bf16 tensor (when no conv epilogue produced them)
__global__ __launch_bounds__(256) void channel_stats_kernel(const bf16* __restrict__ x, float* __restrict__ part,
                                                            int P, int C) {
  extern __shared__ float red[];  // [PL][2][C]
  const int CC = C >> 3;
  const int CCt = CC < 256 ? CC : 256;
  const int PL = 256 / CCt;
  const int tid = threadIdx.x;
  const int pl = tid / CCt, c0 = tid % CCt;
  if (pl < PL) {
    for (int cc = c0; cc < CC; cc += CCt) {
      float s[8] = {0}, ss[8] = {0};
      for (int pix = blockIdx.x * PL + pl; pix < P; pix += gridDim.x * PL) {
        float f[8];
        unpack8(*(const uint4*)(x + (long long)pix * C + cc * 8), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) { s[e] += f[e]; ss[e] += f[e] * f[e]; }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(pl * 2) * C + cc * 8 + e] = s[e];
        red[(pl * 2 + 1) * C + cc * 8 + e] = ss[e];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += 256) {
    float a = 0.f;
    for (int q = 0; q < PL; ++q) a += red[q * 2 * C + i];
    part[(long long)blockIdx.x * 2 * C + i] = a;
  }
}

// ---- finalize forward stats: partial rows [R][2][C] -> mean, rstd, scale, shift (+running) ---
__global__ __launch_bounds__(256) void bn_finalize_fwd_kernel(const float* __restrict__ part, int R, int C,
                                                              double count, const float* gamma,
                                                              const float* beta, float eps, float* run_mean,
                                                              float* run_var, float momentum, float* mean,
                                                              float* rstd, float* scale, float* shift) {
  __shared__ double rs[4][64], rss[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  double s = 0.0, ss = 0.0;
  if (c < C)
    for (int r = q; r < R; r += 4) {
      s += part[(long long)r * 2 * C + c];
      ss += part[(long long)r * 2 * C + C + c];
    }
  rs[q][threadIdx.x & 63] = s;
  rss[q][threadIdx.x & 63] = ss;
  __syncthreads();
  if (q == 0 && c < C) {
    s = rs[0][threadIdx.x] + rs[1][threadIdx.x] + rs[2][threadIdx.x] + rs[3][threadIdx.x];
    ss = rss[0][threadIdx.x] + rss[1][threadIdx.x] + rss[2][threadIdx.x] + rss[3][threadIdx.x];
    const double mu = s / count;
    double var = ss / count - mu * mu;
    if (var < 0.0) var = 0.0;
    const float r = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    mean[c] = (float)mu;
    rstd[c] = r;
    scale[c] = g * r;
    shift[c] = b - (float)mu * g * r;
    if (run_mean) {
      const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mu;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unbiased;
    }
  }
}

__global__ void bn_eval_coeffs_kernel(int C, const float* gamma, const float* beta, const float* run_mean,
                                      const float* run_var, float eps, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float r = rsqrtf(run_var[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * r;
  shift[c] = b - run_mean[c] * g * r;
}

// ---- apply: out = act(y*scale + shift) [maxpool 2x2] ----------------------------------------
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const bf16* __restrict__ y, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, bf16* __restrict__ out,
                                                         int N, int H, int W, int C, int pool, int act, float slope) {
  const int CC = C >> 3;
  const int Ho = pool ? H >> 1 : H, Wo = pool ? W >> 1 : W;
  const long long total = (long long)N * Ho * Wo * CC;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int cc = (int)(idx % CC);
    const long long pix = idx / CC;
    float sc[8], sh[8];
    *(f32x4*)&sc[0] = *(const f32x4*)(scale + cc * 8);
    *(f32x4*)&sc[4] = *(const f32x4*)(scale + cc * 8 + 4);
    *(f32x4*)&sh[0] = *(const f32x4*)(shift + cc * 8);
    *(f32x4*)&sh[4] = *(const f32x4*)(shift + cc * 8 + 4);
    float o[8];
    if (!pool) {
      float f[8];
      unpack8(*(const uint4*)(y + pix * C + cc * 8), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = act_f(f[e] * sc[e] + sh[e], act, slope);
    } else {
      const int wo = (int)(pix % Wo);
      const long long t = pix / Wo;
      const int ho = (int)(t % Ho);
      const int n = (int)(t / Ho);
      const long long base = (((long long)n * H + 2 * ho) * W + 2 * wo) * C + cc * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = -INFINITY;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float f[8];
        unpack8(*(const uint4*)(y + base + ((q >> 1) * W + (q & 1)) * (long long)C), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], act_f(f[e] * sc[e] + sh[e], act, slope));
      }
    }
    *(uint4*)(out + pix * C + cc * 8) = pack8(o);
  }
}

// dz for the 8 channels of one (pre-pool) pixel position q of an output pixel, given upstream g.
// Pool routing: gradient goes to the first maximal element of the window (torch max_pool2d rule).
struct BwdCtx {
  float sc[8], sh[8];
};

__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ y,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, float* __restrict__ part,
                                                            int N, int H, int W, int C, int pool, int act,
                                                            float slope) {
  extern __shared__ float red[];  // [PL][2][C]
  const int CC = C >> 3;
  const int CCt = CC < 256 ? CC : 256;
  const int PL = 256 / CCt;
  const int tid = threadIdx.x;
  const int pl = tid / CCt, c0 = tid % CCt;
  const int Ho = pool ? H >> 1 : H, Wo = pool ? W >> 1 : W;
  const long long Pout = (long long)N * Ho * Wo;
  if (pl < PL) {
    for (int cc = c0; cc < CC; cc += CCt) {
      float sc[8], sh[8], mu[8], rs[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sc[e] = scale[cc * 8 + e]; sh[e] = shift[cc * 8 + e];
        mu[e] = mean[cc * 8 + e]; rs[e] = rstd[cc * 8 + e];
      }
      float s1[8] = {0}, s2[8] = {0};
      for (long long pix = (long long)blockIdx.x * PL + pl; pix < Pout; pix += (long long)gridDim.x * PL) {
        float g[8];
        unpack8(*(const uint4*)(dout + pix * C + cc * 8), g);
        if (!pool) {
          float f[8];
          unpack8(*(const uint4*)(y + pix * C + cc * 8), f);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dz = g[e] * act_d(f[e] * sc[e] + sh[e], act, slope);
            s1[e] += dz;
            s2[e] += dz * (f[e] - mu[e]) * rs[e];
          }
        } else {
          const int wo = (int)(pix % Wo);
          const long long t = pix / Wo;
          const int ho = (int)(t % Ho);
          const int n = (int)(t / Ho);
          const long long base = (((long long)n * H + 2 * ho) * W + 2 * wo) * C + cc * 8;
          float f[4][8], best[8];
          int arg[8];
#pragma unroll
          for (int q = 0; q < 4; ++q) unpack8(*(const uint4*)(y + base + ((q >> 1) * W + (q & 1)) * (long long)C), f[q]);
#pragma unroll
          for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float a = act_f(f[q][e] * sc[e] + sh[e], act, slope);
              if (a > best[e]) { best[e] = a; arg[e] = q; }
            }
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float dz = (arg[e] == q) ? g[e] * act_d(f[q][e] * sc[e] + sh[e], act, slope) : 0.f;
              s1[e] += dz;
              s2[e] += dz * (f[q][e] - mu[e]) * rs[e];
            }
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(pl * 2) * C + cc * 8 + e] = s1[e];
        red[(pl * 2 + 1) * C + cc * 8 + e] = s2[e];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += 256) {
    float a = 0.f;
    for (int q = 0; q < PL; ++q) a += red[q * 2 * C + i];
    part[(long long)blockIdx.x * 2 * C + i] = a;
  }
}

// partial rows [R][2][C] of (sum dz, sum dz*xhat) -> dgamma, dbeta, coef[3][C]
__global__ __launch_bounds__(256) void bn_finalize_bwd_kernel(const float* __restrict__ part, int R, int C,
                                                              double count, const float* gamma,
                                                              const float* mean, const float* rstd,
                                                              float* dgamma, float* dbeta, float* coef,
                                                              int accumulate) {
  __shared__ double rs[4][64], rss[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  double s = 0.0, ss = 0.0;
  if (c < C)
    for (int r = q; r < R; r += 4) {
      s += part[(long long)r * 2 * C + c];
      ss += part[(long long)r * 2 * C + C + c];
    }
  rs[q][threadIdx.x & 63] = s;
  rss[q][threadIdx.x & 63] = ss;
  __syncthreads();
  if (q == 0 && c < C) {
    const double db = rs[0][threadIdx.x] + rs[1][threadIdx.x] + rs[2][threadIdx.x] + rs[3][threadIdx.x];
    const double dg = rss[0][threadIdx.x] + rss[1][threadIdx.x] + rss[2][threadIdx.x] + rss[3][threadIdx.x];
    if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)dg;
    if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)db;
    const double g = gamma ? gamma[c] : 1.0, r = rstd[c], mu = mean[c];
    const double k1 = g * r;
    const double k2 = -g * r * r * dg / count;
    const double k3 = -g * r * db / count - k2 * mu;
    coef[c] = (float)k1;
    coef[C + c] = (float)k2;
    coef[2 * C + c] = (float)k3;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ y,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ coef, bf16* __restrict__ dy,
                                                           int N, int H, int W, int C, int pool, int act, float slope) {
  const int CC = C >> 3;
  const int Ho = pool ? H >> 1 : H, Wo = pool ? W >> 1 : W;
  const long long total = (long long)N * Ho * Wo * CC;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int cc = (int)(idx % CC);
    const long long pix = idx / CC;
    float sc[8], sh[8], k1[8], k2[8], k3[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cc * 8 + e;
      sc[e] = scale[c]; sh[e] = shift[c];
      k1[e] = coef[c]; k2[e] = coef[C + c]; k3[e] = coef[2 * C + c];
    }
    float g[8];
    unpack8(*(const uint4*)(dout + pix * C + cc * 8), g);
    if (!pool) {
      float f[8], o[8];
      unpack8(*(const uint4*)(y + pix * C + cc * 8), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = g[e] * act_d(f[e] * sc[e] + sh[e], act, slope);
        o[e] = k1[e] * dz + k2[e] * f[e] + k3[e];
      }
      *(uint4*)(dy + pix * C + cc * 8) = pack8(o);
    } else {
      const int wo = (int)(pix % Wo);
      const long long t = pix / Wo;
      const int ho = (int)(t % Ho);
      const int n = (int)(t / Ho);
      const long long base = (((long long)n * H + 2 * ho) * W + 2 * wo) * C + cc * 8;
      float f[4][8], best[8];
      int arg[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) unpack8(*(const uint4*)(y + base + ((q >> 1) * W + (q & 1)) * (long long)C), f[q]);
#pragma unroll
      for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = act_f(f[q][e] * sc[e] + sh[e], act, slope);
          if (a > best[e]) { best[e] = a; arg[e] = q; }
        }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = (arg[e] == q) ? g[e] * act_d(f[q][e] * sc[e] + sh[e], act, slope) : 0.f;
          o[e] = k1[e] * dz + k2[e] * f[q][e] + k3[e];
        }
        *(uint4*)(dy + base + ((q >> 1) * W + (q & 1)) * (long long)C) = pack8(o);
      }
    }
  }
}

// odd H or W with 2x2 pooling (VGG16 at 48x48 pools 3x3 -> 1x1): the last row / column belongs to
// no window (floor mode, as Keras/torch), so its upstream gradient is zero but BN still couples it:
// dy = k2*y + k3 there.
__global__ __launch_bounds__(256) void bn_bwd_edge_kernel(const bf16* __restrict__ y, const float* __restrict__ coef,
                                                          bf16* __restrict__ dy, int N, int H, int W, int C) {
  const int CC = C >> 3;
  const int He = H & ~1, We = W & ~1;
  const long long total = (long long)N * H * W * CC;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int cc = (int)(idx % CC);
    const long long pix = idx / CC;
    const int w = (int)(pix % W), h = (int)((pix / W) % H);
    if (h < He && w < We) continue;
    float f[8], o[8];
    unpack8(*(const uint4*)(y + pix * C + cc * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = coef[C + cc * 8 + e] * f[e] + coef[2 * C + cc * 8 + e];
    *(uint4*)(dy + pix * C + cc * 8) = pack8(o);
  }
}

int grid_for(long long work, int per_block, int cap) {
  long long g = (work + per_block - 1) / per_block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

int red_lds_bytes(int C) {
  const int CC = C >> 3;
  const int CCt = CC < 256 ? CC : 256;
  const int PL = 256 / CCt;
  return PL * 2 * C * 4;
}

}  // namespace

// Number of partial rows the reduce kernels will produce for a given problem (host helper).
extern "C" int rk_bn_partial_rows(long long P, int C) {
  const int CC = C >> 3;
  const int CCt = CC < 256 ? CC : 256;
  const int PL = 256 / CCt;
  return grid_for(P, PL * 4, 1024);
}

extern "C" int rk_channel_stats(const void* x, float* part, long long P, int C, int rows, void* stream) {
  if (C % 8 || C > 8192) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(channel_stats_kernel, dim3(rows), dim3(256), red_lds_bytes(C), (hipStream_t)stream,
                     (const bf16*)x, part, (int)P, C);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_finalize_fwd(const float* part, int R, int C, double count, const float* gamma,
                                  const float* beta, float eps, float* run_mean, float* run_var, float momentum,
                                  float* mean, float* rstd, float* scale, float* shift, void* stream) {
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3(rk_cdiv(C, 64)), dim3(256), 0, (hipStream_t)stream, part, R, C,
                     count, gamma, beta, eps, run_mean, run_var, momentum, mean, rstd, scale, shift);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* run_mean,
                                 const float* run_var, float eps, float* scale, float* shift, void* stream) {
  hipLaunchKernelGGL(bn_eval_coeffs_kernel, dim3(rk_cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, C, gamma,
                     beta, run_mean, run_var, eps, scale, shift);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_act_fwd(const void* y, const float* scale, const float* shift, void* out, int N, int H, int W,
                             int C, int pool, int act, float slope, void* stream) {
  if (C % 8) return RK_EUNSUPPORTED;
  const long long work = (long long)N * (pool ? (H / 2) * (W / 2) : H * W) * (C / 8);
  hipLaunchKernelGGL(bn_act_fwd_kernel, dim3(grid_for(work, 256, 8192)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)y, scale, shift, (bf16*)out, N, H, W, C, pool, act, slope);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_bwd_reduce(const void* dout, const void* y, const float* scale, const float* shift,
                                const float* mean, const float* rstd, float* part, int rows, int N, int H, int W,
                                int C, int pool, int act, float slope, void* stream) {
  if (C % 8 || C > 8192) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(rows), dim3(256), red_lds_bytes(C), (hipStream_t)stream,
                     (const bf16*)dout, (const bf16*)y, scale, shift, mean, rstd, part, N, H, W, C, pool, act, slope);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_finalize_bwd(const float* part, int R, int C, double count, const float* gamma,
                                  const float* mean, const float* rstd, float* dgamma, float* dbeta, float* coef,
                                  int accumulate, void* stream) {
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3(rk_cdiv(C, 64)), dim3(256), 0, (hipStream_t)stream, part, R, C,
                     count, gamma, mean, rstd, dgamma, dbeta, coef, accumulate);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_bwd_apply(const void* dout, const void* y, const float* scale, const float* shift,
                               const float* coef, void* dy, int N, int H, int W, int C, int pool, int act,
                               float slope, void* stream) {
  if (C % 8) return RK_EUNSUPPORTED;
  const long long work = (long long)N * (pool ? (H / 2) * (W / 2) : H * W) * (C / 8);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(work, 256, 8192)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)dout, (const bf16*)y, scale, shift, coef, (bf16*)dy, N, H, W, C, pool, act, slope);
  RK_LAUNCH_CHECK();
  if (pool && ((H & 1) || (W & 1))) {
    hipLaunchKernelGGL(bn_bwd_edge_kernel, dim3(grid_for((long long)N * H * W * (C / 8), 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16*)y, coef, (bf16*)dy, N, H, W, C);
    RK_LAUNCH_CHECK();
  }
  return RK_OK;
}
