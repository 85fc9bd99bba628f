// Persistent bidirectional LSTM recurrence for gfx950 (reference
// examples/models/pos_tagging/PyBiLstm.py:249-268, nn.LSTM(bidirectional=True) on a padded batch).
//
// The input projection x @ W_ih^T + b for every timestep is one plain GEMM done outside (it has no
// time dependence).  What remains is T strictly sequential steps of a tiny GEMM + cell update —
// per-step kernel launches would be pure launch latency, so ONE launch runs the whole sequence:
//   * a workgroup owns (direction d, 16 batch rows); rows never interact, so no grid-wide sync;
//   * 4 waves split the hidden units: wave w owns units [w*HP/4, (w+1)*HP/4) of ALL FOUR gates, so
//     one lane's v_mfma_f32_16x16x32_bf16 outputs hold i, f, g, o of the same (row, unit) and the
//     cell update is lane-local (c lives in registers for the whole sequence);
//   * the recurrent weights never leave VGPRs: each lane loads its W_hh^T fragments once
//     (HP = 128: 32 x 16 B per lane), the per-step operand is h_{t-1} (bf16) from a
//     double-buffered LDS tile, so a step costs one barrier;
//   * the next step's input-projection row is prefetched into registers before this step's MFMAs.
// Backward (BPTT) runs the same structure in reverse time: dgates = f(dh, dc, saved gates, c),
// dh_rec = dgates @ W_hh with W_hh fragments held in VGPRs; dgates go to global for the
// weight-gradient GEMMs (plain GEMMs, done outside).
//
// Layouts (HP = padded hidden, 64 or 128; gate blocks [i | f | g | o] of HP each, like nn.LSTM):
//   gin   fp32 [T][B][2][4HP]   input projection incl. both biases
//   whh   bf16 [2][4HP][HP]
//   hout  fp32 [T][B][2][HP]   (padded units stay exactly 0)
//   gsave fp32 [T][B][2][4HP]  activated gates (i, f, g, o)     csave fp32 [T][B][2][HP]
//   dhout fp32 [T][B][2][HP]   upstream gradient of hout        dgin  fp32 [T][B][2][4HP]
#include "common.h"

namespace {

constexpr int LROWS = 16;

RK_DEV float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }
RK_DEV float tanh_f(float x) {
  const float e = __expf(-2.0f * fabsf(x));
  const float t = (1.0f - e) / (1.0f + e);
  return x < 0.f ? -t : t;
}

template <int HP>
__global__ __launch_bounds__(256) void lstm_fwd_kernel(const float* __restrict__ gin, const bf16* __restrict__ whh,
                                                       int T, int B, float* __restrict__ hout,
                                                       float* __restrict__ gsave, float* __restrict__ csave) {
  constexpr int UB = HP / 64;      // 16-unit blocks per wave
  constexpr int KS = HP / 32;      // K-steps of the recurrent GEMM
  constexpr int G4 = 4 * HP;
  constexpr int LD = HP + 8;       // padded LDS row (bf16): 16-B reads of 16 rows hit distinct banks
  __shared__ __attribute__((aligned(16))) bf16 hs[2][LROWS][LD];
  const int d = blockIdx.y, r0 = blockIdx.x * LROWS;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, kq = lane >> 4;
  // recurrent weights: b[q][ub][ks] = W_hh[q*HP + unit][ks*32 + 8*kq .. +8]
  bf16x8 bw[4][UB][KS];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      const int unit = w * (HP / 4) + ub * 16 + col;
      const bf16* row = whh + ((long long)d * G4 + q * HP + unit) * HP;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) bw[q][ub][ks] = *(const bf16x8*)(row + ks * 32 + 8 * kq);
    }
  for (int i = threadIdx.x; i < LROWS * LD; i += 256) (&hs[0][0][0])[i] = (bf16)0.f;
  float c[UB][4];
#pragma unroll
  for (int ub = 0; ub < UB; ++ub)
#pragma unroll
    for (int i = 0; i < 4; ++i) c[ub][i] = 0.f;
  // rows this lane owns in the MFMA output: kq*4 + i
  auto gin_at = [&](int t, int row, int q, int unit) -> float {
    const int b = r0 + row;
    return b < B ? gin[(((long long)t * B + b) * 2 + d) * G4 + q * HP + unit] : 0.f;
  };
  float pre[4][UB][4];
  const int t_first = d == 0 ? 0 : T - 1;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int ub = 0; ub < UB; ++ub)
#pragma unroll
      for (int i = 0; i < 4; ++i) pre[q][ub][i] = gin_at(t_first, kq * 4 + i, q, w * (HP / 4) + ub * 16 + col);
  __syncthreads();
  int cur = 0;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    f32x4 acc[4][UB];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ub = 0; ub < UB; ++ub) acc[q][ub] = f32x4{pre[q][ub][0], pre[q][ub][1], pre[q][ub][2], pre[q][ub][3]};
    // prefetch the next step's projection while the MFMAs run
    if (s + 1 < T) {
      const int tn = d == 0 ? t + 1 : t - 1;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int ub = 0; ub < UB; ++ub)
#pragma unroll
          for (int i = 0; i < 4; ++i) pre[q][ub][i] = gin_at(tn, kq * 4 + i, q, w * (HP / 4) + ub * 16 + col);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 a = *(const bf16x8*)&hs[cur][col][ks * 32 + 8 * kq];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int ub = 0; ub < UB; ++ub) acc[q][ub] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[q][ub][ks], acc[q][ub], 0, 0, 0);
    }
    // lane owns D[row kq*4+i][unit]: i, f, g, o of the same cell
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      const int unit = w * (HP / 4) + ub * 16 + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = kq * 4 + i, b = r0 + row;
        const float ig = sigm(acc[0][ub][i]), fg = sigm(acc[1][ub][i]);
        const float gg = tanh_f(acc[2][ub][i]), og = sigm(acc[3][ub][i]);
        const float cn = b < B ? fg * c[ub][i] + ig * gg : 0.f;
        const float h = og * tanh_f(cn);
        c[ub][i] = cn;
        hs[cur ^ 1][row][unit] = (bf16)(b < B ? h : 0.f);
        if (b < B) {
          const long long o = ((long long)t * B + b) * 2 + d;
          hout[o * HP + unit] = h;
          csave[o * HP + unit] = cn;
          float* gp = gsave + o * G4 + unit;
          gp[0] = ig; gp[HP] = fg; gp[2 * HP] = gg; gp[3 * HP] = og;
        }
      }
    }
    __syncthreads();
    cur ^= 1;
  }
}

template <int HP>
__global__ __launch_bounds__(256) void lstm_bwd_kernel(const bf16* __restrict__ whh, int T, int B,
                                                       const float* __restrict__ dhout,
                                                       const float* __restrict__ gsave,
                                                       const float* __restrict__ csave, float* __restrict__ dgin) {
  constexpr int UB = HP / 64;
  constexpr int G4 = 4 * HP;
  constexpr int KS = G4 / 32;      // K-steps of dh_rec = dgates @ W_hh (K = 4HP)
  constexpr int LD = G4 + 8;
  __shared__ __attribute__((aligned(16))) bf16 gs[2][LROWS][LD];
  const int d = blockIdx.y, r0 = blockIdx.x * LROWS;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, kq = lane >> 4;
  // b[ub][ks][j] = W_hh[ks*32 + 8*kq + j][unit]  (column gather, once)
  bf16x8 bw[UB][KS];
#pragma unroll
  for (int ub = 0; ub < UB; ++ub) {
    const int unit = w * (HP / 4) + ub * 16 + col;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = whh[((long long)d * G4 + ks * 32 + 8 * kq + j) * HP + unit];
      bw[ub][ks] = v;
    }
  }
  float dc[UB][4];
  f32x4 dhr[UB];
#pragma unroll
  for (int ub = 0; ub < UB; ++ub) {
    dhr[ub] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) dc[ub][i] = 0.f;
  }
  int cur = 0;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;            // reverse of the forward order
    const int tp = d == 0 ? t - 1 : t + 1;           // the forward's previous step
    const bool has_prev = d == 0 ? t > 0 : t < T - 1;
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      const int unit = w * (HP / 4) + ub * 16 + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = kq * 4 + i, b = r0 + row;
        float dai = 0.f, daf = 0.f, dag = 0.f, dao = 0.f;
        if (b < B) {
          const long long o = ((long long)t * B + b) * 2 + d;
          const float* gp = gsave + o * G4 + unit;
          const float ig = gp[0], fg = gp[HP], gg = gp[2 * HP], og = gp[3 * HP];
          const float ct = csave[o * HP + unit];
          const float cp = has_prev ? csave[(((long long)tp * B + b) * 2 + d) * HP + unit] : 0.f;
          const float dh = dhout[o * HP + unit] + dhr[ub][i];
          const float th = tanh_f(ct);
          const float dct = dc[ub][i] + dh * og * (1.f - th * th);
          dao = dh * th * og * (1.f - og);
          dai = dct * gg * ig * (1.f - ig);
          dag = dct * ig * (1.f - gg * gg);
          daf = dct * cp * fg * (1.f - fg);
          dc[ub][i] = dct * fg;
          float* dp = dgin + o * G4 + unit;
          dp[0] = dai; dp[HP] = daf; dp[2 * HP] = dag; dp[3 * HP] = dao;
        }
        gs[cur][row][unit] = (bf16)dai;
        gs[cur][row][HP + unit] = (bf16)daf;
        gs[cur][row][2 * HP + unit] = (bf16)dag;
        gs[cur][row][3 * HP + unit] = (bf16)dao;
      }
    }
    __syncthreads();
    // dh_rec[row][unit] = sum_k dgates[row][k] * W_hh[k][unit]
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) dhr[ub] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 a = *(const bf16x8*)&gs[cur][col][ks * 32 + 8 * kq];
#pragma unroll
      for (int ub = 0; ub < UB; ++ub) dhr[ub] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[ub][ks], dhr[ub], 0, 0, 0);
    }
    cur ^= 1;   // the other buffer is free: everyone passed this step's barrier after reading it
  }
}

// ---------------------------------------------------------------------------- fp32 recurrence
// The same structure on v_mfma_f32_16x16x4_f32 (exact fp32, the reference's precision): lane group
// kq = lane >> 4 supplies k in [kq*KQ, (kq+1)*KQ) (a permuted K order, so both operands stream as
// float4), the C/D map equals the bf16 form's, so the lane-local cell update is unchanged.  W_hh is
// fp32: register-resident for HP = 64 (64 VGPRs), re-read from L2 every step for HP = 128.
template <int HP>
__global__ __launch_bounds__(256) void lstm_fwd32_kernel(const float* __restrict__ gin, const float* __restrict__ whh,
                                                         int T, int B, float* __restrict__ hout,
                                                         float* __restrict__ gsave, float* __restrict__ csave) {
  constexpr int UB = HP / 64;
  constexpr int KQ = HP / 4;       // k per lane group
  constexpr int G4 = 4 * HP;
  constexpr int LD = HP + 4;
  constexpr bool RES = HP <= 64;   // weights in registers
  __shared__ __attribute__((aligned(16))) float hs[2][LROWS][LD];
  const int d = blockIdx.y, r0 = blockIdx.x * LROWS;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const float* wd = whh + (long long)d * G4 * HP;
  f32x4 wres[RES ? 4 : 1][RES ? UB : 1][RES ? KQ / 4 : 1];
  if constexpr (RES) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ub = 0; ub < UB; ++ub)
#pragma unroll
        for (int k4 = 0; k4 < KQ / 4; ++k4)
          wres[q][ub][k4] = *(const f32x4*)(wd + (long long)(q * HP + w * (HP / 4) + ub * 16 + col) * HP + kq * KQ + 4 * k4);
  }
  for (int i = threadIdx.x; i < LROWS * LD; i += 256) (&hs[0][0][0])[i] = 0.f;
  float c[UB][4];
#pragma unroll
  for (int ub = 0; ub < UB; ++ub)
#pragma unroll
    for (int i = 0; i < 4; ++i) c[ub][i] = 0.f;
  auto gin_at = [&](int t, int row, int q, int unit) -> float {
    const int b = r0 + row;
    return b < B ? gin[(((long long)t * B + b) * 2 + d) * G4 + q * HP + unit] : 0.f;
  };
  float pre[4][UB][4];
  const int t_first = d == 0 ? 0 : T - 1;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int ub = 0; ub < UB; ++ub)
#pragma unroll
      for (int i = 0; i < 4; ++i) pre[q][ub][i] = gin_at(t_first, kq * 4 + i, q, w * (HP / 4) + ub * 16 + col);
  __syncthreads();
  int cur = 0;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    f32x4 acc[4][UB];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int ub = 0; ub < UB; ++ub) acc[q][ub] = f32x4{pre[q][ub][0], pre[q][ub][1], pre[q][ub][2], pre[q][ub][3]};
    if (s + 1 < T) {
      const int tn = d == 0 ? t + 1 : t - 1;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int ub = 0; ub < UB; ++ub)
#pragma unroll
          for (int i = 0; i < 4; ++i) pre[q][ub][i] = gin_at(tn, kq * 4 + i, q, w * (HP / 4) + ub * 16 + col);
    }
#pragma unroll
    for (int k4 = 0; k4 < KQ / 4; ++k4) {   // fully unrolled: the register-resident weights stay in VGPRs
      const f32x4 a = *(const f32x4*)&hs[cur][col][kq * KQ + 4 * k4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int ub = 0; ub < UB; ++ub) {
          f32x4 bv;
          if constexpr (RES) bv = wres[q][ub][k4];
          else bv = *(const f32x4*)(wd + (long long)(q * HP + w * (HP / 4) + ub * 16 + col) * HP + kq * KQ + 4 * k4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[q][ub] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], bv[e], acc[q][ub], 0, 0, 0);
        }
    }
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      const int unit = w * (HP / 4) + ub * 16 + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = kq * 4 + i, b = r0 + row;
        const float ig = sigm(acc[0][ub][i]), fg = sigm(acc[1][ub][i]);
        const float gg = tanh_f(acc[2][ub][i]), og = sigm(acc[3][ub][i]);
        const float cn = b < B ? fg * c[ub][i] + ig * gg : 0.f;
        const float h = og * tanh_f(cn);
        c[ub][i] = cn;
        hs[cur ^ 1][row][unit] = b < B ? h : 0.f;
        if (b < B) {
          const long long o = ((long long)t * B + b) * 2 + d;
          hout[o * HP + unit] = h;
          csave[o * HP + unit] = cn;
          float* gp = gsave + o * G4 + unit;
          gp[0] = ig; gp[HP] = fg; gp[2 * HP] = gg; gp[3 * HP] = og;
        }
      }
    }
    __syncthreads();
    cur ^= 1;
  }
}

// BPTT in fp32: dh_rec = dgates [16 x 4HP] . W_hh [4HP x HP], read from W_hh^T [2][HP][4HP] (float4 along k);
// two accumulator sets per unit block hide the 40-cycle dependent MFMA latency.
template <int HP>
__global__ __launch_bounds__(256) void lstm_bwd32_kernel(const float* __restrict__ whhT, int T, int B,
                                                         const float* __restrict__ dhout,
                                                         const float* __restrict__ gsave,
                                                         const float* __restrict__ csave, float* __restrict__ dgin) {
  constexpr int UB = HP / 64;
  constexpr int G4 = 4 * HP;
  constexpr int KQ = G4 / 4;       // k per lane group (= HP)
  constexpr int LD = G4 + 4;
  __shared__ __attribute__((aligned(16))) float gs[2][LROWS][LD];
  const int d = blockIdx.y, r0 = blockIdx.x * LROWS;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const float* wt = whhT + (long long)d * HP * G4;
  float dc[UB][4];
  f32x4 dhr[UB];
#pragma unroll
  for (int ub = 0; ub < UB; ++ub) {
    dhr[ub] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) dc[ub][i] = 0.f;
  }
  int cur = 0;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    const int tp = d == 0 ? t - 1 : t + 1;
    const bool has_prev = d == 0 ? t > 0 : t < T - 1;
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      const int unit = w * (HP / 4) + ub * 16 + col;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = kq * 4 + i, b = r0 + row;
        float dai = 0.f, daf = 0.f, dag = 0.f, dao = 0.f;
        if (b < B) {
          const long long o = ((long long)t * B + b) * 2 + d;
          const float* gp = gsave + o * G4 + unit;
          const float ig = gp[0], fg = gp[HP], gg = gp[2 * HP], og = gp[3 * HP];
          const float ct = csave[o * HP + unit];
          const float cp = has_prev ? csave[(((long long)tp * B + b) * 2 + d) * HP + unit] : 0.f;
          const float dh = dhout[o * HP + unit] + dhr[ub][i];
          const float th = tanh_f(ct);
          const float dct = dc[ub][i] + dh * og * (1.f - th * th);
          dao = dh * th * og * (1.f - og);
          dai = dct * gg * ig * (1.f - ig);
          dag = dct * ig * (1.f - gg * gg);
          daf = dct * cp * fg * (1.f - fg);
          dc[ub][i] = dct * fg;
          float* dp = dgin + o * G4 + unit;
          dp[0] = dai; dp[HP] = daf; dp[2 * HP] = dag; dp[3 * HP] = dao;
        }
        gs[cur][row][unit] = dai;
        gs[cur][row][HP + unit] = daf;
        gs[cur][row][2 * HP + unit] = dag;
        gs[cur][row][3 * HP + unit] = dao;
      }
    }
    __syncthreads();
    f32x4 acc[2][UB];
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) acc[0][ub] = acc[1][ub] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int k4 = 0; k4 < KQ / 4; ++k4) {
      const f32x4 a = *(const f32x4*)&gs[cur][col][kq * KQ + 4 * k4];
#pragma unroll
      for (int ub = 0; ub < UB; ++ub) {
        const int unit = w * (HP / 4) + ub * 16 + col;
        const f32x4 bv = *(const f32x4*)(wt + (long long)unit * G4 + kq * KQ + 4 * k4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[e & 1][ub] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], bv[e], acc[e & 1][ub], 0, 0, 0);
      }
    }
#pragma unroll
    for (int ub = 0; ub < UB; ++ub) dhr[ub] = acc[0][ub] + acc[1][ub];
    cur ^= 1;
  }
}

}  // namespace

// fp32 entry points: whh fp32 [2][4HP][HP] (forward), whhT fp32 [2][HP][4HP] (backward)
extern "C" int rk_lstm_fwd32(const float* gin, const float* whh, int T, int B, int HP, float* hout, float* gsave,
                             float* csave, void* stream) {
  if (T <= 0 || B <= 0) return RK_OK;
  const dim3 grid(rk_cdiv(B, LROWS), 2), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (HP == 64)
    hipLaunchKernelGGL(lstm_fwd32_kernel<64>, grid, block, 0, s, gin, whh, T, B, hout, gsave, csave);
  else if (HP == 128)
    hipLaunchKernelGGL(lstm_fwd32_kernel<128>, grid, block, 0, s, gin, whh, T, B, hout, gsave, csave);
  else
    return RK_EUNSUPPORTED;
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_lstm_bwd32(const float* whhT, int T, int B, int HP, const float* dhout, const float* gsave,
                             const float* csave, float* dgin, void* stream) {
  if (T <= 0 || B <= 0) return RK_OK;
  const dim3 grid(rk_cdiv(B, LROWS), 2), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (HP == 64)
    hipLaunchKernelGGL(lstm_bwd32_kernel<64>, grid, block, 0, s, whhT, T, B, dhout, gsave, csave, dgin);
  else if (HP == 128)
    hipLaunchKernelGGL(lstm_bwd32_kernel<128>, grid, block, 0, s, whhT, T, B, dhout, gsave, csave, dgin);
  else
    return RK_EUNSUPPORTED;
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_lstm_fwd(const float* gin, const void* whh, int T, int B, int HP, float* hout, float* gsave,
                           float* csave, void* stream) {
  if (T <= 0 || B <= 0) return RK_OK;
  const dim3 grid(rk_cdiv(B, LROWS), 2), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (HP == 64)
    hipLaunchKernelGGL(lstm_fwd_kernel<64>, grid, block, 0, s, gin, (const bf16*)whh, T, B, hout, gsave, csave);
  else if (HP == 128)
    hipLaunchKernelGGL(lstm_fwd_kernel<128>, grid, block, 0, s, gin, (const bf16*)whh, T, B, hout, gsave, csave);
  else
    return RK_EUNSUPPORTED;
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_lstm_bwd(const void* whh, int T, int B, int HP, const float* dhout, const float* gsave,
                           const float* csave, float* dgin, void* stream) {
  if (T <= 0 || B <= 0) return RK_OK;
  const dim3 grid(rk_cdiv(B, LROWS), 2), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (HP == 64)
    hipLaunchKernelGGL(lstm_bwd_kernel<64>, grid, block, 0, s, (const bf16*)whh, T, B, dhout, gsave, csave, dgin);
  else if (HP == 128)
    hipLaunchKernelGGL(lstm_bwd_kernel<128>, grid, block, 0, s, (const bf16*)whh, T, B, dhout, gsave, csave, dgin);
  else
    return RK_EUNSUPPORTED;
  RK_LAUNCH_CHECK();
  return RK_OK;
}
