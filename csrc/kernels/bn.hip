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

// Sum rows rl, rl+16, ... of a [R][2][C] partial table for channel c (both stats), loads issued
// 8 rows at a time so a lane keeps 16 independent loads in flight (one latency per 8 rows).
RK_DEV void rows_sum2(const float* __restrict__ part, int R, int C, int c, int rl, double& s, double& q) {
  int r0 = rl;
  for (; r0 + 16 * 7 < R; r0 += 16 * 8) {  // full groups: no per-load predicate (guide §5 trap (c))
    float a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a[k] = part[(long long)(r0 + 16 * k) * 2 * C + c];
      b[k] = part[(long long)(r0 + 16 * k) * 2 * C + C + c];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) { s += a[k]; q += b[k]; }
  }
  for (; r0 < R; r0 += 16) {
    s += part[(long long)r0 * 2 * C + c];
    q += part[(long long)r0 * 2 * C + C + c];
  }
}

// ---- finalize forward stats: partial rows [R][2][C] -> mean, rstd, scale, shift (+running) ---
__global__ __launch_bounds__(256) void bn_finalize_fwd_kernel(const float* __restrict__ part, int R, int C,
                                                              double count, const float* gamma,
                                                              const float* beta, float eps, float* run_mean,
                                                              float* run_var, float momentum, float* mean,
                                                              float* rstd, float* scale, float* shift) {
  // 16 channels x 16 row lanes per block, two independent fp64 chains per lane, fixed order
  __shared__ double rs[16][16], rss[16][16];
  const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double s0 = 0.0, q0 = 0.0;
  if (c < C) rows_sum2(part, R, C, c, rl, s0, q0);
  rs[rl][cl] = s0;
  rss[rl][cl] = q0;
  __syncthreads();
  if (rl == 0 && c < C) {
    double s = 0.0, ss = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) { s += rs[q][cl]; ss += rss[q][cl]; }
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
// Per-channel coefficients come from global memory (after rk_bn_finalize_fwd) or from LDS (the
// fused-finalize variant below computes them in its prologue): the body is shared.
struct CoefLds {
  const float* sc;  // __shared__ arrays (inlined: the compiler sees the LDS address space)
  const float* sh;
  RK_DEV void load(int cc, float (&a)[8], float (&b)[8]) const {
    *(f32x4*)&a[0] = *(const f32x4*)(sc + cc * 8);
    *(f32x4*)&a[4] = *(const f32x4*)(sc + cc * 8 + 4);
    *(f32x4*)&b[0] = *(const f32x4*)(sh + cc * 8);
    *(f32x4*)&b[4] = *(const f32x4*)(sh + cc * 8 + 4);
  }
};
struct CoefPtr {
  const float* sc;
  const float* sh;
  RK_DEV void load(int cc, float (&a)[8], float (&b)[8]) const {
    *(f32x4*)&a[0] = *(const f32x4*)(sc + cc * 8);
    *(f32x4*)&a[4] = *(const f32x4*)(sc + cc * 8 + 4);
    *(f32x4*)&b[0] = *(const f32x4*)(sh + cc * 8);
    *(f32x4*)&b[4] = *(const f32x4*)(sh + cc * 8 + 4);
  }
};

template <int POOL, int ACT, class CS>
RK_DEV void bn_act_fwd_body(const CS& cs, const bf16* __restrict__ y, bf16* __restrict__ out, int N, int H, int W,
                            int C, float slope) {
  const int CC = C >> 3;
  const int Ho = POOL ? H >> 1 : H, Wo = POOL ? W >> 1 : W;
  const long long total = (long long)N * Ho * Wo * CC;
  // when the grid stride is a multiple of CC (every power-of-two C <= 2048) a thread's channel group
  // never changes: load its coefficients once
  const long long stride = (long long)gridDim.x * blockDim.x;
  const bool hoist = stride % CC == 0;
  float sc[8], sh[8];
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (hoist) {
    cs.load((int)(idx % CC), sc, sh);
    // U items per sweep with every load issued before any is consumed: a one-item grid-stride loop
    // keeps one 16-B load per lane in flight and runs at ~half the HBM rate on these sizes
    constexpr int U = POOL ? 2 : 4;
    constexpr int NL = POOL ? 4 : 1;
    const int cc = (int)(idx % CC);
    for (; idx + (U - 1) * stride < total; idx += U * stride) {
      uint4 v[U][NL];
      long long pixs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long pix = (idx + u * stride) / CC;
        pixs[u] = pix;
        if constexpr (!POOL) {
          v[u][0] = *(const uint4*)(y + pix * C + cc * 8);
        } else {
          const int wo = (int)(pix % Wo);
          const long long t = pix / Wo;
          const int ho = (int)(t % Ho);
          const int n = (int)(t / Ho);
          const long long base = (((long long)n * H + 2 * ho) * W + 2 * wo) * C + cc * 8;
#pragma unroll
          for (int q = 0; q < 4; ++q) v[u][q] = *(const uint4*)(y + base + ((q >> 1) * W + (q & 1)) * (long long)C);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float o[8];
        if constexpr (!POOL) {
          float f[8];
          unpack8(v[u][0], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = act_f(f[e] * sc[e] + sh[e], ACT, slope);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = -INFINITY;
#pragma unroll
          for (int q = 0; q < NL; ++q) {
            float f[8];
            unpack8(v[u][q], f);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], act_f(f[e] * sc[e] + sh[e], ACT, slope));
          }
        }
        *(uint4*)(out + pixs[u] * C + cc * 8) = pack8(o);
      }
    }
  }
  for (; idx < total; idx += stride) {
    const int cc = (int)(idx % CC);
    const long long pix = idx / CC;
    if (!hoist) cs.load(cc, sc, sh);
    float o[8];
    if constexpr (!POOL) {
      float f[8];
      unpack8(*(const uint4*)(y + pix * C + cc * 8), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = act_f(f[e] * sc[e] + sh[e], ACT, slope);
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
        for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], act_f(f[e] * sc[e] + sh[e], ACT, slope));
      }
    }
    *(uint4*)(out + pix * C + cc * 8) = pack8(o);
  }
}

template <int POOL, int ACT>
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const bf16* __restrict__ y, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, bf16* __restrict__ out,
                                                         int N, int H, int W, int C, float slope) {
  bn_act_fwd_body<POOL, ACT>(CoefPtr{scale, shift}, y, out, N, H, W, C, slope);
}

// ---- fused finalize + apply ---------------------------------------------------------------------
// Statistics arrive as fp64 sums in SL slots [SL][2][C] (atomically accumulated by the conv
// epilogue, igemm FLAG_SATOM): every block folds them into scale/shift in LDS (8 KiB of reads per
// block, the grid is capped at 1024 blocks), block 0 also publishes mean/rstd/scale/shift and
// updates the running statistics.  Replaces rows_reduce + bn_finalize_fwd (two launches).
constexpr int FUSED_MAX_C = 1024;

RK_DEV void acc_sums(const double* __restrict__ acc, int SL, int C, int c, double& a, double& b) {
  double va[8], vb[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {  // SL <= 8: all loads in flight at once
    va[s] = s < SL ? acc[(long long)(2 * s) * C + c] : 0.0;
    vb[s] = s < SL ? acc[(long long)(2 * s + 1) * C + c] : 0.0;
  }
  a = ((va[0] + va[1]) + (va[2] + va[3])) + ((va[4] + va[5]) + (va[6] + va[7]));
  b = ((vb[0] + vb[1]) + (vb[2] + vb[3])) + ((vb[4] + vb[5]) + (vb[6] + vb[7]));
}

template <int POOL, int ACT>
__global__ __launch_bounds__(256) void bn_act_fwd_acc_kernel(const bf16* __restrict__ y, const double* __restrict__ acc,
                                                             int SL, double count, const float* gamma,
                                                             const float* beta, float eps, float* run_mean,
                                                             float* run_var, float momentum, float* coeffs,
                                                             bf16* __restrict__ out, int N, int H, int W, int C,
                                                             float slope) {
  __shared__ __attribute__((aligned(16))) float s_sc[FUSED_MAX_C], s_sh[FUSED_MAX_C];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s, q;
    acc_sums(acc, SL, C, c, s, q);
    const double mu = s / count;
    double var = q / count - mu * mu;
    if (var < 0.0) var = 0.0;
    const float r = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    const float sc = g * r, sh = b - (float)mu * g * r;
    s_sc[c] = sc;
    s_sh[c] = sh;
    if (blockIdx.x == 0) {
      coeffs[c] = (float)mu;
      coeffs[C + c] = r;
      coeffs[2 * C + c] = sc;
      coeffs[3 * C + c] = sh;
      if (run_mean) {
        const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mu;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unbiased;
      }
    }
  }
  __syncthreads();
  bn_act_fwd_body<POOL, ACT>(CoefLds{s_sc, s_sh}, y, out, N, H, W, C, slope);
}

// ---- backward pass 1: per-block partial (sum dz, sum dz*y) ------------------------------------
// dz = d(act)/dz * (pool-routed upstream gradient), z = y*scale + shift recomputed from y.
// sum dz*xhat = rstd*(sum dz*y - mean*sum dz) is formed in the finalize kernel, so this streaming
// pass needs only scale/shift per channel (16 VGPRs) — the old form also held mean/rstd.
// Every thread owns 8 channels (one 16-B vector) of PL pixels/windows per sweep; U independent
// items are loaded before any is consumed so each wave keeps U*(1|4+1) 16-B loads in flight.
template <int POOL, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ y,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            float* __restrict__ part, int N, int H, int W, int C,
                                                            float slope, double* __restrict__ acc, int slmask) {
  extern __shared__ float red[];  // [PL][2][C]
  constexpr int U = POOL ? 2 : 4;
  const int CC = C >> 3;
  const int CCt = CC < 256 ? CC : 256;
  const int PL = 256 / CCt;
  const int tid = threadIdx.x;
  const int pl = tid / CCt, c0 = tid % CCt;
  const int Ho = POOL ? H >> 1 : H, Wo = POOL ? W >> 1 : W;
  const long long items = (long long)N * Ho * Wo;
  const long long stride = (long long)gridDim.x * PL;
  if (pl < PL) {
    for (int cc = c0; cc < CC; cc += CCt) {
      float sc[8], sh[8];
      *(f32x4*)&sc[0] = *(const f32x4*)(scale + cc * 8);
      *(f32x4*)&sc[4] = *(const f32x4*)(scale + cc * 8 + 4);
      *(f32x4*)&sh[0] = *(const f32x4*)(shift + cc * 8);
      *(f32x4*)&sh[4] = *(const f32x4*)(shift + cc * 8 + 4);
      float s1[8] = {0}, s2[8] = {0};
      long long i = (long long)blockIdx.x * PL + pl;
      auto base_of = [&](long long it) -> long long {
        if (!POOL) return it * C + cc * 8;
        const int wo = (int)(it % Wo);
        const long long t = it / Wo;
        const int ho = (int)(t % Ho);
        const int n = (int)(t / Ho);
        return (((long long)n * H + 2 * ho) * W + 2 * wo) * C + cc * 8;
      };
      auto consume = [&](const uint4 gv, const uint4 (&yv)[POOL ? 4 : 1]) {
        float g[8];
        unpack8(gv, g);
        if constexpr (!POOL) {
          float f[8];
          unpack8(yv[0], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dz = g[e] * act_d(f[e] * sc[e] + sh[e], ACT, slope);
            s1[e] += dz;
            s2[e] += dz * f[e];
          }
        } else {
          float f[4][8];
#pragma unroll
          for (int q = 0; q < 4; ++q) unpack8(yv[q], f[q]);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float best = -INFINITY, zb = 0.f, yb = 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // first maximal element of the window (torch rule)
              const float z = f[q][e] * sc[e] + sh[e];
              const float a = act_f(z, ACT, slope);
              if (a > best) { best = a; zb = z; yb = f[q][e]; }
            }
            const float dz = g[e] * act_d(zb, ACT, slope);
            s1[e] += dz;
            s2[e] += dz * yb;
          }
        }
      };
      for (; i + (U - 1) * stride < items; i += U * stride) {
        uint4 gv[U], yv[U][POOL ? 4 : 1];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long it = i + u * stride;
          gv[u] = *(const uint4*)(dout + it * C + cc * 8);
          const long long b = base_of(it);
          if constexpr (!POOL) {
            yv[u][0] = *(const uint4*)(y + b);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) yv[u][q] = *(const uint4*)(y + b + ((q >> 1) * W + (q & 1)) * (long long)C);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) consume(gv[u], yv[u]);
      }
      for (; i < items; i += stride) {
        uint4 yv[POOL ? 4 : 1];
        const uint4 gv = *(const uint4*)(dout + i * C + cc * 8);
        const long long b = base_of(i);
        if constexpr (!POOL) {
          yv[0] = *(const uint4*)(y + b);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) yv[q] = *(const uint4*)(y + b + ((q >> 1) * W + (q & 1)) * (long long)C);
        }
        consume(gv, yv);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(pl * 2) * C + cc * 8 + e] = s1[e];
        red[(pl * 2 + 1) * C + cc * 8 + e] = s2[e];
      }
    }
  }
  __syncthreads();
  // acc != null: add the block's row into fp64 slot (block & slmask) of [SL][2][C] (consumed by the
  // fused finalize of bn_bwd_apply_acc_kernel); else write partial row blockIdx of [R][2][C]
  double* dst = acc ? acc + (long long)(blockIdx.x & slmask) * 2 * C : nullptr;
  for (int i = tid; i < 2 * C; i += 256) {
    float a = 0.f;
    for (int q = 0; q < PL; ++q) a += red[q * 2 * C + i];
    if (dst) unsafeAtomicAdd(dst + i, (double)a);
    else part[(long long)blockIdx.x * 2 * C + i] = a;
  }
}

// ---- backward pass 2: partial rows [R][2][C] -> dgamma, dbeta, coef[3][C] ----------------------
// 16 channels x 16 row lanes per block, fp64 accumulation, fixed order (deterministic).
__global__ __launch_bounds__(256) void bn_finalize_bwd_kernel(const float* __restrict__ part, int R, int C,
                                                              double count, const float* gamma,
                                                              const float* mean, const float* rstd,
                                                              float* dgamma, float* dbeta, float* coef,
                                                              int accumulate) {
  __shared__ double r1[16][16], r2[16][16];
  const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double a0 = 0.0, b0 = 0.0;
  if (c < C) rows_sum2(part, R, C, c, rl, a0, b0);
  r1[rl][cl] = a0;
  r2[rl][cl] = b0;
  __syncthreads();
  if (rl == 0 && c < C) {
    double sdz = 0.0, sdzy = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) { sdz += r1[q][cl]; sdzy += r2[q][cl]; }
    const double g = gamma ? gamma[c] : 1.0, r = rstd[c], mu = mean[c];
    const double db = sdz;
    const double dg = r * (sdzy - mu * sdz);  // sum dz * xhat
    if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)dg;
    if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)db;
    const double k1 = g * r;
    const double k2 = -g * r * r * dg / count;
    const double k3 = -g * r * db / count - k2 * mu;
    coef[c] = (float)k1;
    coef[C + c] = (float)k2;
    coef[2 * C + c] = (float)k3;
  }
}

// ---- backward pass 3: dy = k1*dz + k2*y + k3 ---------------------------------------------------
struct BwdCoefPtr {
  const float* sc;
  const float* sh;
  const float* coef;  // [3][C]
  int C;
  RK_DEV void load(int cc, float (&a)[8], float (&b)[8], float (&k1)[8], float (&k2)[8], float (&k3)[8]) const {
    *(f32x4*)&a[0] = *(const f32x4*)(sc + cc * 8);
    *(f32x4*)&a[4] = *(const f32x4*)(sc + cc * 8 + 4);
    *(f32x4*)&b[0] = *(const f32x4*)(sh + cc * 8);
    *(f32x4*)&b[4] = *(const f32x4*)(sh + cc * 8 + 4);
    *(f32x4*)&k1[0] = *(const f32x4*)(coef + cc * 8);
    *(f32x4*)&k1[4] = *(const f32x4*)(coef + cc * 8 + 4);
    *(f32x4*)&k2[0] = *(const f32x4*)(coef + C + cc * 8);
    *(f32x4*)&k2[4] = *(const f32x4*)(coef + C + cc * 8 + 4);
    *(f32x4*)&k3[0] = *(const f32x4*)(coef + 2 * C + cc * 8);
    *(f32x4*)&k3[4] = *(const f32x4*)(coef + 2 * C + cc * 8 + 4);
  }
};
struct BwdCoefLds {
  const float* sc;  // __shared__
  const float* sh;
  const float* k;   // __shared__ [3][FUSED_MAX_C]
  RK_DEV void load(int cc, float (&a)[8], float (&b)[8], float (&k1)[8], float (&k2)[8], float (&k3)[8]) const {
    const float* src[5] = {sc, sh, k, k + FUSED_MAX_C, k + 2 * FUSED_MAX_C};
    float* dst[5] = {a, b, k1, k2, k3};
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      *(f32x4*)&dst[t][0] = *(const f32x4*)(src[t] + cc * 8);
      *(f32x4*)&dst[t][4] = *(const f32x4*)(src[t] + cc * 8 + 4);
    }
  }
};

template <int POOL, int ACT>
RK_DEV void bn_bwd_apply_item(const uint4 gv, const uint4 (&yv)[POOL ? 4 : 1], long long base, const float (&sc)[8],
                              const float (&sh)[8], const float (&k1)[8], const float (&k2)[8],
                              const float (&k3)[8], bf16* __restrict__ dy, int W, int C, float slope);

template <int POOL, int ACT, class CS>
RK_DEV void bn_bwd_apply_body(const CS& cs, const bf16* __restrict__ dout, const bf16* __restrict__ y,
                              bf16* __restrict__ dy, int N, int H, int W, int C, float slope) {
  const int CC = C >> 3;
  const int Ho = POOL ? H >> 1 : H, Wo = POOL ? W >> 1 : W;
  const long long total = (long long)N * Ho * Wo * CC;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const bool hoist = stride % CC == 0;  // see bn_act_fwd_body
  float sc[8], sh[8], k1[8], k2[8], k3[8];
  constexpr int NL = POOL ? 4 : 1;
  auto load_item = [&](long long pix, int cc, uint4& gv, uint4 (&yv)[NL]) -> long long {
    gv = *(const uint4*)(dout + pix * C + cc * 8);
    long long base;
    if constexpr (!POOL) {
      base = pix * C + cc * 8;
      yv[0] = *(const uint4*)(y + base);
    } else {
      const int wo = (int)(pix % Wo);
      const long long t = pix / Wo;
      const int ho = (int)(t % Ho);
      const int n = (int)(t / Ho);
      base = (((long long)n * H + 2 * ho) * W + 2 * wo) * C + cc * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) yv[q] = *(const uint4*)(y + base + ((q >> 1) * W + (q & 1)) * (long long)C);
    }
    return base;
  };
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (hoist) {
    cs.load((int)(idx % CC), sc, sh, k1, k2, k3);
    // U items per sweep, all loads issued before any is consumed (see bn_act_fwd_body)
    constexpr int U = POOL ? 2 : 4;
    const int cc = (int)(idx % CC);
    for (; idx + (U - 1) * stride < total; idx += U * stride) {
      uint4 gv[U], yv[U][NL];
      long long base[U];
#pragma unroll
      for (int u = 0; u < U; ++u) base[u] = load_item((idx + u * stride) / CC, cc, gv[u], yv[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) bn_bwd_apply_item<POOL, ACT>(gv[u], yv[u], base[u], sc, sh, k1, k2, k3, dy, W, C, slope);
    }
  }
  for (; idx < total; idx += stride) {
    const int cc = (int)(idx % CC);
    const long long pix = idx / CC;
    uint4 gv, yv[NL];
    const long long base = load_item(pix, cc, gv, yv);
    if (!hoist) cs.load(cc, sc, sh, k1, k2, k3);
    bn_bwd_apply_item<POOL, ACT>(gv, yv, base, sc, sh, k1, k2, k3, dy, W, C, slope);
  }
}

template <int POOL, int ACT>
RK_DEV void bn_bwd_apply_item(const uint4 gv, const uint4 (&yv)[POOL ? 4 : 1], long long base, const float (&sc)[8],
                              const float (&sh)[8], const float (&k1)[8], const float (&k2)[8],
                              const float (&k3)[8], bf16* __restrict__ dy, int W, int C, float slope) {
  {
    float g[8];
    unpack8(gv, g);
    if constexpr (!POOL) {
      float f[8], o[8];
      unpack8(yv[0], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = g[e] * act_d(f[e] * sc[e] + sh[e], ACT, slope);
        o[e] = k1[e] * dz + k2[e] * f[e] + k3[e];
      }
      *(uint4*)(dy + base) = pack8(o);
    } else {
      float f[4][8];
      int arg[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) unpack8(yv[q], f[q]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float best = -INFINITY;
        arg[e] = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float a = act_f(f[q][e] * sc[e] + sh[e], ACT, slope);
          if (a > best) { best = a; arg[e] = q; }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = (arg[e] == q) ? g[e] * act_d(f[q][e] * sc[e] + sh[e], ACT, slope) : 0.f;
          o[e] = k1[e] * dz + k2[e] * f[q][e] + k3[e];
        }
        *(uint4*)(dy + base + ((q >> 1) * W + (q & 1)) * (long long)C) = pack8(o);
      }
    }
  }
}

template <int POOL, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ y,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ coef, bf16* __restrict__ dy,
                                                           int N, int H, int W, int C, float slope) {
  bn_bwd_apply_body<POOL, ACT>(BwdCoefPtr{scale, shift, coef, C}, dout, y, dy, N, H, W, C, slope);
}

// Fused backward finalize + apply: (sum dz, sum dz*y) arrive as fp64 sums in SL slots
// (rk_bn_bwd_reduce with an accumulator); each block forms k1/k2/k3 in LDS, block 0 also writes
// dgamma/dbeta and coef (the odd-pool edge kernel reads it).  Replaces rk_bn_finalize_bwd.
template <int POOL, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_apply_acc_kernel(const bf16* __restrict__ dout,
                                                               const bf16* __restrict__ y,
                                                               const float* __restrict__ coeffs,
                                                               const double* __restrict__ acc, int SL, double count,
                                                               const float* gamma, float* dgamma, float* dbeta,
                                                               float* coef, int accumulate, bf16* __restrict__ dy,
                                                               int N, int H, int W, int C, float slope) {
  __shared__ __attribute__((aligned(16))) float s_sc[FUSED_MAX_C], s_sh[FUSED_MAX_C], s_k[3 * FUSED_MAX_C];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double sdz, sdzy;
    acc_sums(acc, SL, C, c, sdz, sdzy);
    const double mu = coeffs[c], r = coeffs[C + c];
    const double g = gamma ? gamma[c] : 1.0;
    const double db = sdz;
    const double dg = r * (sdzy - mu * sdz);  // sum dz * xhat
    const double k1 = g * r;
    const double k2 = -g * r * r * dg / count;
    const double k3 = -g * r * db / count - k2 * mu;
    s_sc[c] = coeffs[2 * C + c];
    s_sh[c] = coeffs[3 * C + c];
    s_k[c] = (float)k1;
    s_k[FUSED_MAX_C + c] = (float)k2;
    s_k[2 * FUSED_MAX_C + c] = (float)k3;
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)dg;
      if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)db;
      coef[c] = (float)k1;
      coef[C + c] = (float)k2;
      coef[2 * C + c] = (float)k3;
    }
  }
  __syncthreads();
  bn_bwd_apply_body<POOL, ACT>(BwdCoefLds{s_sc, s_sh, s_k}, dout, y, dy, N, H, W, C, slope);
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
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3(rk_cdiv(C, 16)), dim3(256), 0, (hipStream_t)stream, part, R, C,
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

#define RK_DISPATCH_POOL_ACT(POOLV, ACTV, ...)                                          \
  do {                                                                                 \
    if (POOLV) {                                                                       \
      if ((ACTV) == ACT_RELU) { constexpr int P_ = 1, A_ = ACT_RELU; __VA_ARGS__; }    \
      else if ((ACTV) == ACT_LRELU) { constexpr int P_ = 1, A_ = ACT_LRELU; __VA_ARGS__; } \
      else { constexpr int P_ = 1, A_ = ACT_NONE; __VA_ARGS__; }                       \
    } else {                                                                           \
      if ((ACTV) == ACT_RELU) { constexpr int P_ = 0, A_ = ACT_RELU; __VA_ARGS__; }    \
      else if ((ACTV) == ACT_LRELU) { constexpr int P_ = 0, A_ = ACT_LRELU; __VA_ARGS__; } \
      else { constexpr int P_ = 0, A_ = ACT_NONE; __VA_ARGS__; }                       \
    }                                                                                  \
  } while (0)

extern "C" int rk_bn_act_fwd(const void* y, const float* scale, const float* shift, void* out, int N, int H, int W,
                             int C, int pool, int act, float slope, void* stream) {
  if (C % 8) return RK_EUNSUPPORTED;
  const long long work = (long long)N * (pool ? (H / 2) * (W / 2) : H * W) * (C / 8);
  const dim3 grid(grid_for(work, 256, 8192));
  RK_DISPATCH_POOL_ACT(pool, act,
                       hipLaunchKernelGGL((bn_act_fwd_kernel<P_, A_>), grid, dim3(256), 0, (hipStream_t)stream,
                                          (const bf16*)y, scale, shift, (bf16*)out, N, H, W, C, slope));
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// Partial-row count for rk_bn_bwd_reduce: enough blocks to stream at full bandwidth (~4 per CU),
// few enough rows that the finalize reads them in one pass.
extern "C" int rk_bn_bwd_rows(long long items, int C) {
  const int CC = C >> 3;
  const int CCt = CC < 256 ? CC : 256;
  const int PL = 256 / CCt;
  return grid_for(items, PL * 8, 512);
}

extern "C" int rk_bn_bwd_reduce(const void* dout, const void* y, const float* scale, const float* shift,
                                float* part, int rows, int N, int H, int W, int C, int pool, int act, float slope,
                                void* stream) {
  if (C % 8 || C > 8192) return RK_EUNSUPPORTED;
  RK_DISPATCH_POOL_ACT(pool, act,
                       hipLaunchKernelGGL((bn_bwd_reduce_kernel<P_, A_>), dim3(rows), dim3(256), red_lds_bytes(C),
                                          (hipStream_t)stream, (const bf16*)dout, (const bf16*)y, scale, shift, part,
                                          N, H, W, C, slope, (double*)nullptr, 0));
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// Same reduction, accumulated atomically (fp64) into the SL-slot table acc [SL][2][C] (SL a power of
// two; the caller zeroes it) for rk_bn_bwd_apply_acc.
extern "C" int rk_bn_bwd_reduce_acc(const void* dout, const void* y, const float* scale, const float* shift,
                                    double* acc, int SL, int rows, int N, int H, int W, int C, int pool, int act,
                                    float slope, void* stream) {
  if (C % 8 || C > FUSED_MAX_C || SL <= 0 || SL > 8 || (SL & (SL - 1))) return RK_EUNSUPPORTED;
  RK_DISPATCH_POOL_ACT(pool, act,
                       hipLaunchKernelGGL((bn_bwd_reduce_kernel<P_, A_>), dim3(rows), dim3(256), red_lds_bytes(C),
                                          (hipStream_t)stream, (const bf16*)dout, (const bf16*)y, scale, shift,
                                          (float*)nullptr, N, H, W, C, slope, acc, SL - 1));
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_bwd_apply_acc(const void* dout, const void* y, const float* coeffs, const double* acc, int SL,
                                   double count, const float* gamma, float* dgamma, float* dbeta, float* coef,
                                   int accumulate, void* dy, int N, int H, int W, int C, int pool, int act,
                                   float slope, void* stream) {
  if (C % 8 || C > FUSED_MAX_C || SL <= 0 || SL > 8) return RK_EUNSUPPORTED;
  const long long work = (long long)N * (pool ? (H / 2) * (W / 2) : H * W) * (C / 8);
  const dim3 grid(grid_for(work, 256, 1024));
  RK_DISPATCH_POOL_ACT(pool, act,
                       hipLaunchKernelGGL((bn_bwd_apply_acc_kernel<P_, A_>), grid, dim3(256), 0, (hipStream_t)stream,
                                          (const bf16*)dout, (const bf16*)y, coeffs, acc, SL, count, gamma, dgamma,
                                          dbeta, coef, accumulate, (bf16*)dy, N, H, W, C, slope));
  RK_LAUNCH_CHECK();
  if (pool && ((H & 1) || (W & 1))) {
    hipLaunchKernelGGL(bn_bwd_edge_kernel, dim3(grid_for((long long)N * H * W * (C / 8), 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16*)y, (const float*)coef, (bf16*)dy, N, H, W, C);
    RK_LAUNCH_CHECK();
  }
  return RK_OK;
}

extern "C" int rk_bn_act_fwd_acc(const void* y, const double* acc, int SL, double count, const float* gamma,
                                 const float* beta, float eps, float* run_mean, float* run_var, float momentum,
                                 float* coeffs, void* out, int N, int H, int W, int C, int pool, int act, float slope,
                                 void* stream) {
  if (C % 8 || C > FUSED_MAX_C || SL <= 0 || SL > 8) return RK_EUNSUPPORTED;
  const long long work = (long long)N * (pool ? (H / 2) * (W / 2) : H * W) * (C / 8);
  const dim3 grid(grid_for(work, 256, 1024));
  RK_DISPATCH_POOL_ACT(pool, act,
                       hipLaunchKernelGGL((bn_act_fwd_acc_kernel<P_, A_>), grid, dim3(256), 0, (hipStream_t)stream,
                                          (const bf16*)y, acc, SL, count, gamma, beta, eps, run_mean, run_var,
                                          momentum, coeffs, (bf16*)out, N, H, W, C, slope));
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_finalize_bwd(const float* part, int R, int C, double count, const float* gamma,
                                  const float* mean, const float* rstd, float* dgamma, float* dbeta, float* coef,
                                  int accumulate, void* stream) {
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3(rk_cdiv(C, 16)), dim3(256), 0, (hipStream_t)stream, part, R, C,
                     count, gamma, mean, rstd, dgamma, dbeta, coef, accumulate);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bn_bwd_apply(const void* dout, const void* y, const float* scale, const float* shift,
                               const float* coef, void* dy, int N, int H, int W, int C, int pool, int act,
                               float slope, void* stream) {
  if (C % 8) return RK_EUNSUPPORTED;
  const long long work = (long long)N * (pool ? (H / 2) * (W / 2) : H * W) * (C / 8);
  const dim3 grid(grid_for(work, 256, 8192));
  RK_DISPATCH_POOL_ACT(pool, act,
                       hipLaunchKernelGGL((bn_bwd_apply_kernel<P_, A_>), grid, dim3(256), 0, (hipStream_t)stream,
                                          (const bf16*)dout, (const bf16*)y, scale, shift, coef, (bf16*)dy, N, H, W,
                                          C, slope));
  RK_LAUNCH_CHECK();
  if (pool && ((H & 1) || (W & 1))) {
    hipLaunchKernelGGL(bn_bwd_edge_kernel, dim3(grid_for((long long)N * H * W * (C / 8), 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16*)y, coef, (bf16*)dy, N, H, W, C);
    RK_LAUNCH_CHECK();
  }
  return RK_OK;
}
