// Shared core of the fp32 GEMM kernels (sgemm.hip: implicit-GEMM convs / dense; x6p.hip: pre-split X6
// GEMMs): parameter block, flag bits, geometry decoders, the X6 split-bf16 product helpers and the
// 32x32-accumulator epilogue (bias / activation / BN statistics / BNB / BNP fusions / split-K slabs).
// Included inside each translation unit's anonymous namespace.
#pragma once
#include "common.h"


constexpr int SBK = 32;  // fp32 elements per K-tile: 128-B LDS rows
constexpr unsigned SOOB = 0x80000000u;

// SM_KIN_CONVF: SM_KIN_CONV with C % 32 == 0, so a 32-deep K-tile never straddles a tap and the
// tap / channel offset of every DMA is wave-uniform (~4 VALU per DMA instead of ~20)
// SM_KIN_CONVG / SM_KOUT_CONVG: table-driven gathers for the PG-GAN resampling convs — rows over an
// Ho x Wo output grid, source pixel stride*(i, j) + (dy_t, dx_t) of an H x W input, up to 16 taps
// per parity group (see rk_sgemm_g)
enum SMode { SM_KIN_DENSE = 0, SM_KIN_CONV = 1, SM_KOUT_DENSE = 2, SM_KOUT_CONV = 3, SM_KIN_CONVF = 4,
             SM_KIN_CONVG = 5, SM_KOUT_CONVG = 6 };
enum SFlags { SF_RELU = 1, SF_BIAS = 2, SF_STATS = 4, SF_GATE = 8, SF_ACCUM = 16, SF_LRELU = 32,
              SF_BNB = 512, SF_BNP = 1024 };

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((address_space(3))) void lds_void;

struct SgParams {
  const float* A;
  const float* B;
  float* out;
  const float* bias;    // [N] bias; FLAG_BNB/BNP: BN scale [N] then shift [N] of the gated layer
  double* stats;        // fp64 slot table [slotMask+1][2][N]
  const float* gate;    // ReLU gate [M][ldc] (SF_GATE) or the gated layer's BN input y (BNB / BNP)
  int M, N, K;
  int lda, ldb, ldc;
  int H, W, C, taps;    // geometry of the gathered (conv) operand; BNP: H, W = pooled resolution
  int log2H, log2W, log2C;
  float invC, invH, invW;
  int ktPer;            // K-tiles per split (gridDim.z splits)
  long long slabStride; // floats between split-K slabs
  int flags, slotMask;
  float alpha, slope;
  unsigned long long bytesA, bytesB;
  // table-driven gathers (SM_KIN_CONVG / SM_KOUT_CONVG); H, W above = the INPUT map
  int Ho, Wo, log2Ho, log2Wo;  // row grid (output pixels of the gather)
  float invHo, invWo;
  int stride, ntaps, groups, os;
  unsigned tpy[4], tpx[4];     // per group, tap t: offset = ((word >> 2t) & 3) - 1  (in -1 .. 2)
  unsigned oyx;                // per group g: output parity (bits 2g: oy, 2g+1: ox) when os == 2
  long long gstrideB;          // floats between the groups' B operands
  // grouped GEMMs (rk_sgemm_grp: k same-shape problems in one launch, e.g. the k models of an
  // inference ensemble): per-group operand / output / bias offsets in floats
  long long gstrideA, gstrideO, gstrideBias;
};

RK_DEV __amdgpu_buffer_rsrc_t s_rsrc(const void* base, unsigned long long bytes) {
  const unsigned nrec = bytes >= 0x80000000ull ? 0x80000000u : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nrec, 0x00020000);
}

RK_DEV int s_tap_dy(int t) { return ((t * 11) >> 5) - 1; }
RK_DEV int s_tap_dx(int t) { return t - 3 * ((t * 11) >> 5) - 1; }

// channel -> tap (power-of-two C by shift, else an fp32 reciprocal, exact below 2^22)
RK_DEV int s_cdiv(int k, const SgParams& p) {
  return p.log2C >= 0 ? (k >> p.log2C) : (int)(((float)k + 0.5f) * p.invC);
}
// pixel -> (n, i, j) of an N x Ho x Wo grid
RK_DEV void s_nhw(int k, const SgParams& p, int& n, int& i, int& j) {
  int q;
  if (p.log2Wo >= 0) {
    q = k >> p.log2Wo;
    j = k & (p.Wo - 1);
  } else {
    q = (int)(((float)k + 0.5f) * p.invWo);
    j = k - q * p.Wo;
  }
  if (p.log2Ho >= 0) {
    n = q >> p.log2Ho;
    i = q & (p.Ho - 1);
  } else {
    n = (int)(((float)q + 0.5f) * p.invHo);
    i = q - n * p.Ho;
  }
}
RK_DEV int s_tapoff(unsigned word, int t) { return (int)((word >> (2 * t)) & 3u) - 1; }

// pixel -> (h, w) of an H x W map
RK_DEV void s_hw(int k, int H, int W, int log2H, int log2W, float invH, float invW, int& h, int& w) {
  if (log2H >= 0 && log2W >= 0) {
    w = k & (W - 1);
    h = (k >> log2W) & (H - 1);
  } else {
    const int q = (int)(((float)k + 0.5f) * invW);
    w = k - q * W;
    const int n = (int)(((float)q + 0.5f) * invH);
    h = q - n * H;
  }
}

// x = hi + mid + lo for 8 fp32 values (two 4-value fragments): bf16 round-to-nearest of x, then of
// the residuals (x - hi and x - hi - mid are exact in fp32).  Written pairwise so every step is one packed
// instruction per two values — v_cvt_pk_bf16_f32 rounds a pair, the pair's fp32 values come back with one
// shift and one mask, v_pk_add_f32 forms both residuals: 36 VALU per 8 values (the per-element form
// compiled to 44)
typedef __attribute__((ext_vector_type(2))) float x6_f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 x6_bf16x2;
typedef __attribute__((ext_vector_type(4))) unsigned x6_u32x4;
RK_DEV x6_f32x2 x6_unpack(unsigned w) {
  return (x6_f32x2){__builtin_bit_cast(float, w << 16), __builtin_bit_cast(float, w & 0xffff0000u)};
}
RK_DEV void split3(const f32x4& v0, const f32x4& v1, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
  unsigned hw[4], mw[4], lw[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const x6_f32x2 x = p < 2 ? (x6_f32x2){v0[2 * p], v0[2 * p + 1]} : (x6_f32x2){v1[2 * p - 4], v1[2 * p - 3]};
    const unsigned h = __builtin_bit_cast(unsigned, __builtin_convertvector(x, x6_bf16x2));
    const x6_f32x2 r = x - x6_unpack(h);
    const unsigned m = __builtin_bit_cast(unsigned, __builtin_convertvector(r, x6_bf16x2));
    lw[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(r - x6_unpack(m), x6_bf16x2));
    hw[p] = h;
    mw[p] = m;
  }
  hi = __builtin_bit_cast(bf16x8, (x6_u32x4){hw[0], hw[1], hw[2], hw[3]});
  mid = __builtin_bit_cast(bf16x8, (x6_u32x4){mw[0], mw[1], mw[2], mw[3]});
  lo = __builtin_bit_cast(bf16x8, (x6_u32x4){lw[0], lw[1], lw[2], lw[3]});
}

RK_DEV f32x16 mfma6(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh, const bf16x8& bm,
                    const bf16x8& bl, f32x16 c) {
  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
}

template <int N>
RK_DEV void s_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

RK_DEV void s_barrier_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// accumulator register r of a 32x32 block: row (r&3) + 8(r>>2) + 4h, column lane&31
RK_DEV int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// PA / PB: the A (rows) / B (columns) fragments were read interleaved (frag_pair)
template <int MI, int NI, bool PA, bool PB, bool OMAP = false>
RK_DEV void s_epilogue(const SgParams& p, f32x16 (&acc)[MI][NI], int mbase, int nbase, int lane, int split,
                       int grp, float* outp, const float* biasp) {
  const int fl = p.flags;
  const int h = lane >> 5;
  float* C = outp + (long long)split * p.slabStride;
  const bool want_sums = fl & (SF_STATS | SF_BNB | SF_BNP);
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int n = PB ? nbase + 2 * (lane & 31) + ni : nbase + ni * 32 + (lane & 31);
    const bool nok = n < p.N;
    float b = 0.f, sh = 0.f;
    if ((fl & (SF_BIAS | SF_BNB | SF_BNP)) && nok) b = biasp[n];
    if ((fl & (SF_BNB | SF_BNP)) && nok) sh = biasp[p.N + n];
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = PA ? mbase + 2 * acc_row(r, h) + mi : mbase + mi * 32 + acc_row(r, h);
        if (!(nok && m < p.M)) continue;
        float v = acc[mi][ni][r] * p.alpha;
        long long row = m;
        if constexpr (OMAP) {   // parity group: row (n, i, j) of the Ho x Wo grid -> pixel (2i+oy, 2j+ox)
          if (p.os == 2) {
            int b, i, j;
            s_nhw(m, p, b, i, j);
            const int oy = (p.oyx >> (2 * grp)) & 1, ox = (p.oyx >> (2 * grp + 1)) & 1;
            row = ((long long)b * 2 * p.Ho + 2 * i + oy) * (2 * p.Wo) + 2 * j + ox;
          }
        }
        const long long idx = row * p.ldc + n;
        if (fl & SF_BIAS) v += b;
        if (fl & SF_STATS) {
          s += v;
          ss += v * v;
        }
        if (fl & SF_RELU) v = fmaxf(v, 0.f);
        else if (fl & SF_LRELU) v = v > 0.f ? v : v * p.slope;
        if (fl & SF_GATE) v = p.gate[idx] > 0.f ? v : 0.f;
        if (fl & SF_BNB) {
          const float yv = p.gate[idx];
          v = yv * b + sh > 0.f ? v : 0.f;
          s += v;
          ss += v * yv;
        }
        if (fl & SF_BNP) {
          // m = pooled pixel (img, ho, wo) of an H x W map; its window sits at 2H x 2W
          int ho, wo;
          s_hw(m, p.H, p.W, p.log2H, p.log2W, p.invH, p.invW, ho, wo);
          const long long img = (long long)(m - (ho * p.W + wo)) / ((long long)p.H * p.W);
          const long long W2 = 2LL * p.W;
          const long long b0 = ((img * 2 * p.H + 2 * ho) * W2 + 2 * wo) * p.ldc + n;
          const float y4[4] = {p.gate[b0], p.gate[b0 + p.ldc], p.gate[b0 + W2 * p.ldc], p.gate[b0 + W2 * p.ldc + p.ldc]};
          float best = -INFINITY, zb = 0.f, yb = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // first maximal relu(z) of the window (torch max_pool2d rule)
            const float z = y4[q] * b + sh;
            const float a = fmaxf(z, 0.f);
            if (a > best) { best = a; zb = z; yb = y4[q]; }
          }
          const float dz = zb > 0.f ? v : 0.f;
          s += dz;
          ss += dz * yb;
        }
        if (fl & SF_ACCUM) v += C[idx];
        C[idx] = v;
      }
    }
    if (want_sums) {
      s += __shfl_xor(s, 32, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (nok) {
        double* slot = p.stats + (long long)(blockIdx.x & p.slotMask) * 2 * p.N;
        unsafeAtomicAdd(slot + (h ? p.N : 0) + n, (double)(h ? ss : s));
      }
    }
  }
}
