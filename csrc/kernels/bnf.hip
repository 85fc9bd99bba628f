// fp32 BatchNorm (+ReLU / leaky-ReLU, + 2x2 max-pool) forward / backward and the small fp32 helper
// kernels of the fp32 training path (reference: Keras BatchNormalization
// in TfFeedForward.py:148-149 and the BN of the VGG-small benchmark net, all fp32).
//
// Statistics arrive as fp64 sums in a small slot table [SL][2][C] (written by the conv epilogue of
// sgemm.hip or by bnf_bwd_reduce), so every kernel here starts with a per-block fold of the slots into
// per-channel coefficients in LDS (SL*2*C doubles, <= 8 KiB) — finalize and apply are one launch.
// Activations are NHWC fp32, 4 channels per 16-byte vector; one thread owns one vector.
#include "common.h"
#include <algorithm>
#include <cstdint>

namespace {

RK_DEV int rk_log2_dev(int v) { return (v > 0 && (v & (v - 1)) == 0) ? 31 - __builtin_clz(v) : -1; }

// a / d for the launch-constant d (shift when d is a power of two: log2d >= 0); 32-bit index math
// (the launchers check that every element offset fits in an int)
RK_DEV int idiv(int a, int d, int log2d) { return log2d >= 0 ? a >> log2d : a / d; }

RK_DEV float act_f(float z, int act, float slope) {
  return act == 1 ? fmaxf(z, 0.f) : act == 2 ? (z > 0.f ? z : z * slope) : z;
}
RK_DEV float act_d(float z, int act, float slope) {
  return act == 1 ? (z > 0.f ? 1.f : 0.f) : act == 2 ? (z > 0.f ? 1.f : slope) : 1.f;
}

// y = conv output (pre-BN) [Nb,H,W,C]; out = pool?(act(y*scale+shift)).  Train mode: the batch
// statistics come from `slots`; block 0 writes coeffs [4][C] = mean, rstd, scale, shift and updates the
// running statistics (PyTorch semantics: unbiased variance in the running estimate).  Eval mode
// (slots == null): scale/shift given.  out == null (train mode, no pool): finalize only, one block —
// the next conv applies scale / shift + ReLU on its input loads (normalise-on-load, winograd4.hip).
template <bool POOL>
__global__ __launch_bounds__(256) void bnf_fwd_kernel(const float* __restrict__ y, const double* __restrict__ slots,
                                                      int SL, double count, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, float eps, float* rmean,
                                                      float* rvar, float mom, const float* __restrict__ scale_in,
                                                      const float* __restrict__ shift_in, float* __restrict__ coeffs,
                                                      float* __restrict__ out, int Nb, int H, int W, int C, int act,
                                                      float slope) {
  extern __shared__ float s_dyn[];  // [2][C]: scale, shift
  float* s_sc = s_dyn;
  float* s_sh = s_dyn + C;
  for (int c = threadIdx.x; c < C; c += 256) {
    float sc, sh;
    if (slots) {
      double s = 0.0, ss = 0.0;
      for (int l = 0; l < SL; ++l) {
        s += slots[(long long)l * 2 * C + c];
        ss += slots[(long long)l * 2 * C + C + c];
      }
      const double mean = s / count;
      const double var = fmax(ss / count - mean * mean, 0.0);
      const double rstd = 1.0 / sqrt(var + (double)eps);
      sc = (float)((double)gamma[c] * rstd);
      sh = (float)((double)beta[c] - mean * (double)gamma[c] * rstd);
      if (blockIdx.x == 0) {
        coeffs[c] = (float)mean;
        coeffs[C + c] = (float)rstd;
        coeffs[2 * C + c] = sc;
        coeffs[3 * C + c] = sh;
        if (rmean) {
          rmean[c] = (float)((1.0 - mom) * rmean[c] + mom * mean);
          rvar[c] = (float)((1.0 - mom) * rvar[c] + mom * var * count / fmax(count - 1.0, 1.0));
        }
      }
    } else {
      sc = scale_in[c];
      sh = shift_in[c];
    }
    s_sc[c] = sc;
    s_sh[c] = sh;
  }
  if (!out) return;   // finalize only: the consumers apply scale / shift + ReLU while loading y
  __syncthreads();
  const int G = C >> 2;
  const int Ho = POOL ? H >> 1 : H, Wo = POOL ? W >> 1 : W;
  const int lG = rk_log2_dev(G), lWo = rk_log2_dev(Wo), lHo = rk_log2_dev(Ho);
  const int total = Nb * Ho * Wo * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = idiv(i, G, lG);
    const int cg = i - pix * G;
    const int c = cg * 4;
    const f32x4 sc = *(const f32x4*)(s_sc + c), sh = *(const f32x4*)(s_sh + c);
    f32x4 o;
    if constexpr (!POOL) {
      const f32x4 v = *(const f32x4*)(y + pix * C + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = act_f(v[e] * sc[e] + sh[e], act, slope);
    } else {
      const int t = idiv(pix, Wo, lWo);
      const int wo = pix - t * Wo;
      const int n = idiv(t, Ho, lHo);
      const int ho = t - n * Ho;
      const int b0 = ((n * H + 2 * ho) * W + 2 * wo) * C + c;
      const f32x4 v0 = *(const f32x4*)(y + b0), v1 = *(const f32x4*)(y + b0 + C);
      const f32x4 v2 = *(const f32x4*)(y + b0 + W * C), v3 = *(const f32x4*)(y + b0 + W * C + C);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a0 = act_f(v0[e] * sc[e] + sh[e], act, slope), a1 = act_f(v1[e] * sc[e] + sh[e], act, slope);
        const float a2 = act_f(v2[e] * sc[e] + sh[e], act, slope), a3 = act_f(v3[e] * sc[e] + sh[e], act, slope);
        o[e] = fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
      }
    }
    *(f32x4*)(out + pix * C + c) = o;
  }
}

// gradient routing of one (window, channel): returns dz (at the routed position, 0 elsewhere) and
// the index (0..3) of the position that receives it — the first maximal act(z) (torch max_pool2d).
RK_DEV int route4(const float (&yq)[4], float sc, float sh, int act, float slope, float& zbest) {
  float best = -INFINITY;
  int qb = 0;
  zbest = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float z = yq[q] * sc + sh;
    const float a = act_f(z, act, slope);
    if (a > best) { best = a; qb = q; zbest = z; }
  }
  return qb;
}

// BN backward statistics: (sum dz, sum dz*y) per channel -> fp64 slots [SL][2][C]; dz = dL/d(bn out)
// recomputed from dout (the gradient of pool?(act(bn(y)))).  G = C/4 channel groups per row, 256/G rows
// per block pass.
template <bool POOL>
__global__ __launch_bounds__(256) void bnf_bwd_reduce_kernel(const float* __restrict__ dout,
                                                             const float* __restrict__ y,
                                                             const float* __restrict__ coeffs, double* slots,
                                                             int slot_mask, int Nb, int H, int W, int C, int act,
                                                             float slope) {
  __shared__ f32x4 red_s[256], red_ss[256];
  const int G = C >> 2, R = 256 / G;
  const int cg = threadIdx.x % G, r = threadIdx.x / G;
  const int c = cg * 4;
  const f32x4 sc = *(const f32x4*)(coeffs + 2 * C + c), sh = *(const f32x4*)(coeffs + 3 * C + c);
  const int Ho = POOL ? H >> 1 : H, Wo = POOL ? W >> 1 : W;
  const long long npix = (long long)Nb * Ho * Wo;
  f32x4 s = {0.f, 0.f, 0.f, 0.f}, ss = {0.f, 0.f, 0.f, 0.f};
  if (r < R) {
    for (long long p = (long long)blockIdx.x * R + r; p < npix; p += (long long)gridDim.x * R) {
      const f32x4 d = *(const f32x4*)(dout + p * C + c);
      if constexpr (!POOL) {
        const f32x4 v = *(const f32x4*)(y + p * C + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float dz = d[e] * act_d(v[e] * sc[e] + sh[e], act, slope);
          s[e] += dz;
          ss[e] += dz * v[e];
        }
      } else {
        const int wo = (int)(p % Wo);
        const long long t = p / Wo;
        const int ho = (int)(t % Ho);
        const long long n = t / Ho;
        const long long b0 = ((n * H + 2 * ho) * W + 2 * wo) * C + c;
        const long long offs[4] = {b0, b0 + C, b0 + (long long)W * C, b0 + (long long)W * C + C};
        f32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = *(const f32x4*)(y + offs[q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float yq[4] = {v[0][e], v[1][e], v[2][e], v[3][e]};
          float zb;
          const int qb = route4(yq, sc[e], sh[e], act, slope, zb);
          const float dz = d[e] * act_d(zb, act, slope);
          s[e] += dz;
          ss[e] += dz * yq[qb];
        }
      }
    }
  }
  red_s[threadIdx.x] = s;
  red_ss[threadIdx.x] = ss;
  __syncthreads();
  if (threadIdx.x < G) {
    f32x4 a = red_s[threadIdx.x], b = red_ss[threadIdx.x];
    for (int k = 1; k < R; ++k) {
      a += red_s[threadIdx.x + k * G];
      b += red_ss[threadIdx.x + k * G];
    }
    double* sl = slots + (long long)(blockIdx.x & slot_mask) * 2 * C;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      unsafeAtomicAdd(sl + c + e, (double)a[e]);
      unsafeAtomicAdd(sl + C + c + e, (double)b[e]);
    }
  }
}

// BN backward apply: dy = A*dz + B*y + Cc per channel, with (from the slot sums S0 = sum dz,
// S1 = sum dz*y, n = count): A = gamma*rstd, T = rstd*(S1 - mean*S0) (= sum dz*xhat),
// B = -A*rstd*T/n, Cc = -A*S0/n - B*mean.  Block 0 writes dgamma = T, dbeta = S0.
template <bool POOL>
__global__ __launch_bounds__(256) void bnf_bwd_apply_kernel(const float* __restrict__ dout, const float* __restrict__ y,
                                                            const float* __restrict__ coeffs,
                                                            const double* __restrict__ slots, int SL, double count,
                                                            const float* __restrict__ gamma, float* dgamma,
                                                            float* dbeta, int accumulate, float* __restrict__ dy,
                                                            int Nb, int H, int W, int C, int act, float slope) {
  extern __shared__ float s_dyn[];  // [3][C]: A, B, Cc
  float* kA = s_dyn;
  float* kB = s_dyn + C;
  float* kC = s_dyn + 2 * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    double s0 = 0.0, s1 = 0.0;
    for (int l = 0; l < SL; ++l) {
      s0 += slots[(long long)l * 2 * C + c];
      s1 += slots[(long long)l * 2 * C + C + c];
    }
    const double mean = coeffs[c], rstd = coeffs[C + c];
    const double T = rstd * (s1 - mean * s0);
    const double A = (double)gamma[c] * rstd;
    const double B = -A * rstd * T / count;
    kA[c] = (float)A;
    kB[c] = (float)B;
    kC[c] = (float)(-A * s0 / count - B * mean);
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] = (float)(accumulate ? dgamma[c] + T : T);
      if (dbeta) dbeta[c] = (float)(accumulate ? dbeta[c] + s0 : s0);
    }
  }
  __syncthreads();
  const int G = C >> 2;
  // pooled: one cell per 2x2 window of the ceil grid; with odd H / W the last row / column of cells
  // holds positions no (floor-mode) window covers: dz = 0 there, dy = B*y + Cc still has to be written
  const int Hc = POOL ? (H + 1) >> 1 : H, Wc = POOL ? (W + 1) >> 1 : W;
  const int Ho = POOL ? H >> 1 : H, Wo = POOL ? W >> 1 : W;
  const int lG = rk_log2_dev(G), lWc = rk_log2_dev(Wc), lHc = rk_log2_dev(Hc);
  const int total = Nb * Hc * Wc * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = idiv(i, G, lG);
    const int cg = i - pix * G;
    const int c = cg * 4;
    const f32x4 a = *(const f32x4*)(kA + c), b = *(const f32x4*)(kB + c), cc = *(const f32x4*)(kC + c);
    const f32x4 sc = *(const f32x4*)(coeffs + 2 * C + c), sh = *(const f32x4*)(coeffs + 3 * C + c);
    if constexpr (!POOL) {
      const f32x4 d = *(const f32x4*)(dout + pix * C + c);
      const f32x4 v = *(const f32x4*)(y + pix * C + c);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = a[e] * (d[e] * act_d(v[e] * sc[e] + sh[e], act, slope)) + b[e] * v[e] + cc[e];
      *(f32x4*)(dy + pix * C + c) = o;
    } else {
      const int t = idiv(pix, Wc, lWc);
      const int wc = pix - t * Wc;
      const int n = idiv(t, Hc, lHc);
      const int hc = t - n * Hc;
      const int b0 = ((n * H + 2 * hc) * W + 2 * wc) * C + c;
      const int offs[4] = {b0, b0 + C, b0 + W * C, b0 + W * C + C};
      if (hc < Ho && wc < Wo) {
        const f32x4 d = *(const f32x4*)(dout + ((n * Ho + hc) * Wo + wc) * C + c);
        f32x4 v[4], o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = *(const f32x4*)(y + offs[q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float yq[4] = {v[0][e], v[1][e], v[2][e], v[3][e]};
          float zb;
          const int qb = route4(yq, sc[e], sh[e], act, slope, zb);
          const float dzb = d[e] * act_d(zb, act, slope);
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q][e] = a[e] * (q == qb ? dzb : 0.f) + b[e] * yq[q] + cc[e];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) *(f32x4*)(dy + offs[q]) = o[q];
      } else {  // uncovered border positions of an odd map
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (2 * hc + (q >> 1) >= H || 2 * wc + (q & 1) >= W) continue;
          const f32x4 v = *(const f32x4*)(y + offs[q]);
          *(f32x4*)(dy + offs[q]) = b * v + cc;
        }
      }
    }
  }
}

// Per-column (sum a, sum a*b) of fp32 [R][C] matrices (b = a when null) -> fp64 slot 0 of [SL][2][C]:
// the statistics of a BatchNorm over features (the MLP's input BN, TfFeedForward.py:148-149) in
// forward (a = b = x) and backward (a = dout, b = x) — columns may exceed the conv kernels' 1024.
__global__ __launch_bounds__(256) void bnf_colstats_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           int R, int C, int rows_per, double* slots) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= C) return;
  const int r0 = blockIdx.y * rows_per, r1 = min(R, r0 + rows_per);
  f32x4 s = {0.f, 0.f, 0.f, 0.f}, ss = {0.f, 0.f, 0.f, 0.f};
  for (int r = r0; r < r1; ++r) {
    const f32x4 va = *(const f32x4*)(a + (long long)r * C + c);
    const f32x4 vb = b ? *(const f32x4*)(b + (long long)r * C + c) : va;
    s += va;
    ss += va * vb;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    unsafeAtomicAdd(slots + c + e, (double)s[e]);
    unsafeAtomicAdd(slots + C + c + e, (double)ss[e]);
  }
}

// Flipped, transposed fp32 weights for the data gradient: dst[ci][t][co] = src[co][8-t][ci]
// (taps = 9; taps = 1: dst[ci][co] = src[co][ci]), several layers per launch.  One block per
// (layer, tap, 32-co tile, 32-ci tile) descriptor; LDS transpose so both sides are coalesced.
__global__ __launch_bounds__(256) void swt_kernel(const float* __restrict__ arena, float* __restrict__ dst,
                                                  const int4* __restrict__ desc, const long long* __restrict__ meta) {
  __shared__ float tile[32][33];
  const int4 d = desc[blockIdx.x];
  const int l = d.x, t = d.y, co0 = d.z, ci0 = d.w;
  const long long so = meta[l * 5 + 0], doff = meta[l * 5 + 1];
  const int Cout = (int)meta[l * 5 + 2], Cin = (int)meta[l * 5 + 3], taps = (int)meta[l * 5 + 4];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const int ts = taps - 1 - t;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int co = co0 + ty + 8 * k, ci = ci0 + tx;
    float v = 0.f;
    if (co < Cout && ci < Cin) v = arena[so + ((long long)co * taps + ts) * Cin + ci];
    tile[ty + 8 * k][tx] = v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ci = ci0 + ty + 8 * k, co = co0 + tx;
    if (co < Cout && ci < Cin) dst[doff + ((long long)ci * taps + t) * Cout + co] = tile[tx][ty + 8 * k];
  }
}

// out[c] (+)= sum_r x[r][c] for an fp32 [R][C] matrix (bias gradients); 64 columns per block.
// gridDim.y > 1: block row-chunk y writes its partial sums to out + y * C (combined by the caller).
__global__ __launch_bounds__(256) void colsum_f32_kernel(const float* __restrict__ x, int R, int C, int ld,
                                                         float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  const int per = (R + gridDim.y - 1) / gridDim.y, r0 = blockIdx.y * per, r1 = min(R, r0 + per);
  out += (long long)blockIdx.y * C;
  float s = 0.f;
  if (c < C)
    for (int r = r0 + q; r < r1; r += 4) s += x[(long long)r * ld + c];
  red[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && c < C) {
    const float v = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    out[c] = accumulate ? out[c] + v : v;
  }
}

// colsum_f32_kernel for C % 4 == 0 (16-B aligned rows): a block covers CB <= 64 float4 columns x 256 / CB
// row lanes, each lane four independent row streams in flight (the scalar kernel above keeps one 4-B load
// per lane in flight: 0.2 TB/s on PG-GAN's bias gradients).  GATE: the column sums of
// g = lrelu_gate(gy = x, y) while writing g (pggan.hip's fused leaky-ReLU backward + bias gradient).
template <bool GATE>
__global__ __launch_bounds__(256) void colsum4_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                      float* __restrict__ g, int R, int C, int ld, float slope,
                                                      float* __restrict__ out, int accumulate, int CB) {
  __shared__ f32x4 red[256];
  const int t = threadIdx.x, RL = 256 / CB;
  const int cl = t % CB, rl = t / CB;
  const int C4 = C >> 2, c4 = blockIdx.x * CB + cl;
  const int per = (R + gridDim.y - 1) / gridDim.y, r0 = blockIdx.y * per, r1 = min(R, r0 + per);
  out += (long long)blockIdx.y * C;
  auto ld4 = [&](int r) -> f32x4 {
    const long long i = (long long)r * ld + 4 * c4;
    f32x4 v = *(const f32x4*)(x + i);
    if constexpr (GATE) {
      const f32x4 yv = *(const f32x4*)(y + i);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = yv[e] > 0.f ? v[e] : v[e] * slope;
      *(f32x4*)(g + i) = v;
    }
    return v;
  };
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
  if (c4 < C4 && rl < RL) {
    int r = r0 + rl;
    for (; r + 3 * RL < r1; r += 4 * RL) {
      a0 += ld4(r);
      a1 += ld4(r + RL);
      a2 += ld4(r + 2 * RL);
      a3 += ld4(r + 3 * RL);
    }
    for (; r < r1; r += RL) a0 += ld4(r);
  }
  red[t] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (t < CB && c4 < C4) {
    f32x4 v = red[t];
    for (int k = 1; k < RL; ++k) v += red[t + k * CB];
    if (accumulate) v += *(const f32x4*)(out + 4 * c4);
    *(f32x4*)(out + 4 * c4) = v;
  }
}

// split-K combine with the dense epilogue, fp32: out[m][n] = gate?(act(alpha * sum_s slab[s] + bias));
// gate [M][ldg]: zero where gate <= 0 (ReLU backward of the layer input).
__global__ __launch_bounds__(256) void sreduce_epi_kernel(const float* __restrict__ slab, int S, int M, int N,
                                                          const float* __restrict__ bias, int act, float slope,
                                                          float alpha, const float* __restrict__ gate, int ldg,
                                                          float* __restrict__ out, int ldc, int brows) {
  const long long n4 = (long long)M * N / 4;
  const long long sn = (long long)M * N;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    f32x4 a = ((const f32x4*)slab)[i];
    int s0 = 1;
    for (; s0 + 3 < S; s0 += 4) {
      f32x4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ((const f32x4*)(slab + (s0 + k) * sn))[i];
      a += (v[0] + v[1]) + (v[2] + v[3]);
    }
    for (; s0 < S; ++s0) a += ((const f32x4*)(slab + s0 * sn))[i];
    const long long e0 = i * 4;
    const int m = (int)(e0 / N), n = (int)(e0 - (long long)m * N);
    a *= alpha;
    if (bias) a += *(const f32x4*)(bias + (brows ? (long long)(m / brows) * N : 0) + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] = act_f(a[e], act, slope);
    if (gate) {
      const f32x4 g = *(const f32x4*)(gate + (long long)m * ldg + n);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = g[e] > 0.f ? a[e] : 0.f;
    }
    *(f32x4*)(out + (long long)m * ldc + n) = a;
  }
}

// uint8/float NCHW images -> fp32 NHWC with channels zero-padded to Cp: out = in * scale + shift
// flags bit 0: uint8 source (else fp32), bit 1: source already NHWC (else NCHW)
__global__ __launch_bounds__(256) void pack_nhwc_f32_kernel(const void* __restrict__ src, int flags, int N, int C,
                                                            int H, int W, int Cp, float scale, float shift,
                                                            float* __restrict__ dst, const int* __restrict__ idx,
                                                            int nsrc) {
  const bool is_u8 = flags & 1, nhwc = flags & 2;
  const long long total = (long long)N * H * W * Cp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % Cp);
    const long long pix = i / Cp;
    const int w = (int)(pix % W);
    const long long t = pix / W;
    const int h = (int)(t % H);
    const long long n = t / H;
    float v = 0.f;
    if (c < C) {
      // idx: output image n is source image idx[n] (the minibatch gather folded in; out-of-range -> 0)
      long long ns = n;
      if (idx) {
        ns = idx[n];
        if ((unsigned long long)ns >= (unsigned long long)nsrc) ns = 0;
      }
      const long long sp = (ns * H + h) * W + w;
      const long long si = nhwc ? sp * C + c : ((ns * C + c) * H + h) * W + w;
      v = (is_u8 ? (float)((const unsigned char*)src)[si] : ((const float*)src)[si]) * scale + shift;
    }
    dst[i] = v;
  }
}

int grid_cap(long long work, int cap) {
  long long g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : g > cap ? cap : g);
}

// eval BN(+act, +2x2 max-pool) of G stacked batches: y [G*Nb, H, W, C], scale / shift [G][C]
template <bool POOL>
__global__ __launch_bounds__(256) void bnf_eval_grp_kernel(const float* __restrict__ y, const float* __restrict__ scale,
                                                           const float* __restrict__ shift, float* __restrict__ out,
                                                           int GN, int Nb, int H, int W, int C, int act, float slope) {
  const int Cg = C >> 2;
  const int Ho = POOL ? H >> 1 : H, Wo = POOL ? W >> 1 : W;
  const long long total = (long long)GN * Ho * Wo * Cg;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cg = (int)(i % Cg);
    const long long pix = i / Cg;
    const int c = cg * 4;
    const long long n = pix / ((long long)Ho * Wo);
    const long long co = (n / Nb) * C + c;
    const f32x4 sc = *(const f32x4*)(scale + co), sh = *(const f32x4*)(shift + co);
    f32x4 o;
    if constexpr (!POOL) {
      const f32x4 v = *(const f32x4*)(y + pix * C + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = act_f(v[e] * sc[e] + sh[e], act, slope);
    } else {
      const long long r = pix - n * Ho * Wo;
      const int ho = (int)(r / Wo), wo = (int)(r - (long long)ho * Wo);
      const long long b0 = ((n * H + 2 * ho) * W + 2 * wo) * C + c;
      const f32x4 v0 = *(const f32x4*)(y + b0), v1 = *(const f32x4*)(y + b0 + C);
      const f32x4 v2 = *(const f32x4*)(y + b0 + (long long)W * C), v3 = *(const f32x4*)(y + b0 + (long long)W * C + C);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a0 = act_f(v0[e] * sc[e] + sh[e], act, slope), a1 = act_f(v1[e] * sc[e] + sh[e], act, slope);
        const float a2 = act_f(v2[e] * sc[e] + sh[e], act, slope), a3 = act_f(v3[e] * sc[e] + sh[e], act, slope);
        o[e] = fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
      }
    }
    *(f32x4*)(out + pix * C + c) = o;
  }
}

bool bn_shape_ok(int C) { return C >= 4 && C <= 1024 && (C & (C - 1)) == 0; }
constexpr int BN_MAX_C = 8192;  // per-channel coefficient arrays live in dynamic LDS

}  // namespace

extern "C" int rk_bnf_fwd(const float* y, const double* slots, int SL, double count, const float* gamma,
                          const float* beta, float eps, float* rmean, float* rvar, float mom, const float* scale,
                          const float* shift, float* coeffs, float* out, int Nb, int H, int W, int C, int pool, int act,
                          float slope, void* stream) {
  if (C % 4 || C > BN_MAX_C || (pool && (H < 2 || W < 2))) return RK_EUNSUPPORTED;
  if (slots && (!gamma || !beta || !coeffs)) return RK_EBADARG;
  if (!slots && (!scale || !shift)) return RK_EBADARG;
  if (!out && (!slots || pool)) return RK_EBADARG;   // out == null: train-mode finalize only (one block)
  const long long work = (long long)Nb * (pool ? H / 2 : H) * (pool ? W / 2 : W) * (C / 4);
  if ((long long)Nb * H * W * C >= (1ll << 31)) return RK_EUNSUPPORTED;   // 32-bit element offsets
  const dim3 grid(out ? grid_cap(work, 2048) : 1);
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = 2 * (size_t)C * sizeof(float);
  if (pool)
    hipLaunchKernelGGL(bnf_fwd_kernel<true>, grid, dim3(256), lds, st, y, slots, SL, count, gamma, beta, eps, rmean,
                       rvar, mom, scale, shift, coeffs, out, Nb, H, W, C, act, slope);
  else
    hipLaunchKernelGGL(bnf_fwd_kernel<false>, grid, dim3(256), lds, st, y, slots, SL, count, gamma, beta, eps, rmean,
                       rvar, mom, scale, shift, coeffs, out, Nb, H, W, C, act, slope);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bnf_bwd_reduce(const float* dout, const float* y, const float* coeffs, double* slots, int SL,
                                 int blocks, int Nb, int H, int W, int C, int pool, int act, float slope,
                                 void* stream) {
  if (!bn_shape_ok(C) || (SL & (SL - 1)) || blocks <= 0 || (pool && (H < 2 || W < 2))) return RK_EUNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  if (pool)
    hipLaunchKernelGGL(bnf_bwd_reduce_kernel<true>, dim3(blocks), dim3(256), 0, st, dout, y, coeffs, slots, SL - 1, Nb,
                       H, W, C, act, slope);
  else
    hipLaunchKernelGGL(bnf_bwd_reduce_kernel<false>, dim3(blocks), dim3(256), 0, st, dout, y, coeffs, slots, SL - 1, Nb,
                       H, W, C, act, slope);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bnf_bwd_apply(const float* dout, const float* y, const float* coeffs, const double* slots, int SL,
                                double count, const float* gamma, float* dgamma, float* dbeta, int accumulate,
                                float* dy, int Nb, int H, int W, int C, int pool, int act, float slope, void* stream) {
  if (C % 4 || C > BN_MAX_C || (pool && (H < 2 || W < 2))) return RK_EUNSUPPORTED;
  const long long work = (long long)Nb * (pool ? (H + 1) / 2 : H) * (pool ? (W + 1) / 2 : W) * (C / 4);
  if ((long long)Nb * H * W * C >= (1ll << 31)) return RK_EUNSUPPORTED;   // 32-bit element offsets
  const dim3 grid(grid_cap(work, 2048));
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = 3 * (size_t)C * sizeof(float);
  if (pool)
    hipLaunchKernelGGL(bnf_bwd_apply_kernel<true>, grid, dim3(256), lds, st, dout, y, coeffs, slots, SL, count, gamma,
                       dgamma, dbeta, accumulate, dy, Nb, H, W, C, act, slope);
  else
    hipLaunchKernelGGL(bnf_bwd_apply_kernel<false>, grid, dim3(256), lds, st, dout, y, coeffs, slots, SL, count, gamma,
                       dgamma, dbeta, accumulate, dy, Nb, H, W, C, act, slope);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bnf_colstats(const float* a, const float* b, int R, int C, double* slots, void* stream) {
  if (C % 4 || R <= 0) return RK_EUNSUPPORTED;
  const int rows_per = 64;
  const dim3 grid(rk_cdiv(C / 4, 256), rk_cdiv(R, rows_per));
  hipLaunchKernelGGL(bnf_colstats_kernel, grid, dim3(256), 0, (hipStream_t)stream, a, b, R, C, rows_per, slots);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_swt(const float* arena, float* dst, const int* desc, int nblocks, const long long* meta,
                      void* stream) {
  if (nblocks <= 0) return RK_OK;
  hipLaunchKernelGGL(swt_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, arena, dst, (const int4*)desc,
                     meta);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// chunks > 1: out is [chunks][C] partial sums (accumulate must be 0)
// the leaky-ReLU backward + its column sums (C % 4 == 0, 16-B aligned): g = gy where y > 0, slope * gy
// elsewhere; part [chunks][C] per-chunk column sums of g
extern "C" int rk_lrelu_gate_colsum4_f32(const float* gy, const float* y, float* g, int R, int C, float slope,
                                         float* part, int chunks, void* stream) {
  if (R <= 0 || C <= 0 || chunks < 1) return RK_EBADARG;
  if (C % 4 || ((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(g) |
                 reinterpret_cast<uintptr_t>(part)) & 15))
    return RK_EUNSUPPORTED;
  const int CB = std::min(C / 4, 64);
  hipLaunchKernelGGL(colsum4_kernel<true>, dim3(rk_cdiv(C / 4, CB), chunks), dim3(256), 0, (hipStream_t)stream, gy, y,
                     g, R, C, C, slope, part, 0, CB);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_colsum_f32(const float* x, int R, int C, int ld, float* out, int accumulate, int chunks,
                             void* stream) {
  if (chunks < 1 || (chunks > 1 && accumulate)) return RK_EBADARG;
  if (C % 4 == 0 && ld % 4 == 0 && !(reinterpret_cast<uintptr_t>(x) & 15) && !(reinterpret_cast<uintptr_t>(out) & 15)) {
    const int CB = std::min(C / 4, 64);
    hipLaunchKernelGGL(colsum4_kernel<false>, dim3(rk_cdiv(C / 4, CB), chunks), dim3(256), 0, (hipStream_t)stream, x,
                       nullptr, nullptr, R, C, ld, 0.f, out, accumulate, CB);
    RK_LAUNCH_CHECK();
    return RK_OK;
  }
  hipLaunchKernelGGL(colsum_f32_kernel, dim3(rk_cdiv(C, 64), chunks), dim3(256), 0, (hipStream_t)stream, x, R, C, ld,
                     out, accumulate);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// brows > 0: rows [g*brows, (g+1)*brows) take bias + g*N (grouped GEMM slabs)
extern "C" int rk_sreduce_epi(const float* slab, int S, int M, int N, const float* bias, int act, float slope,
                              float alpha, const float* gate, int ldg, float* out, int ldc, int brows, void* stream) {
  if (N % 4 || ldc % 4 || (gate && ldg % 4) || brows < 0) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(sreduce_epi_kernel, dim3(grid_cap((long long)M * N / 4, 2048)), dim3(256), 0,
                     (hipStream_t)stream, slab, S, M, N, bias, act, slope, alpha, gate, ldg, out, ldc, brows);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// idx (optional, N int32 rows of a source holding nsrc images): out[n] = pack(src[idx[n]])
extern "C" int rk_pack_nhwc_f32(const void* src, int flags, int N, int C, int H, int W, int Cp, float scale,
                                float shift, float* out, const int* idx, int nsrc, void* stream) {
  if (idx && nsrc <= 0) return RK_EBADARG;
  hipLaunchKernelGGL(pack_nhwc_f32_kernel, dim3(grid_cap((long long)N * H * W * Cp, 4096)), dim3(256), 0,
                     (hipStream_t)stream, src, flags, N, C, H, W, Cp, scale, shift, out, idx, nsrc);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_bnf_eval_grp(const float* y, const float* scale, const float* shift, float* out, int G, int Nb,
                               int H, int W, int C, int pool, int act, float slope, void* stream) {
  if (C % 4 || G < 1 || Nb < 1 || (pool && (H < 2 || W < 2))) return RK_EUNSUPPORTED;
  const long long work = (long long)G * Nb * (pool ? H / 2 : H) * (pool ? W / 2 : W) * (C / 4);
  if (pool)
    hipLaunchKernelGGL(bnf_eval_grp_kernel<true>, dim3(grid_cap(work, 2048)), dim3(256), 0, (hipStream_t)stream, y,
                       scale, shift, out, G * Nb, Nb, H, W, C, act, slope);
  else
    hipLaunchKernelGGL(bnf_eval_grp_kernel<false>, dim3(grid_cap(work, 2048)), dim3(256), 0, (hipStream_t)stream, y,
                       scale, shift, out, G * Nb, Nb, H, W, C, act, slope);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
