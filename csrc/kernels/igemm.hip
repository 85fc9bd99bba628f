// MFMA implicit-GEMM engine for gfx950: 3x3/1x1 convolutions (forward, data-grad, weight-grad)
// and dense GEMMs, all on v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
//
// Why one engine: every hot op of the image-classification path is
// a GEMM whose operands are either "K-inner" (the reduction index is contiguous in memory: NHWC
// activations gathered per tap, [N][K] weights) or "K-outer" (the reduction index is the row:
// weight-grad reductions over pixels, dX = dY·W).  K-inner tiles are staged row-major into a
// XOR-swizzled LDS image and read with ds_read_b128; K-outer tiles are staged as they sit in
// memory (coalesced 16-B loads along the non-reduction dim) and transposed for free on the LDS
// read with ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10).  So conv wgrad and dense
// dW/dX need no explicit transpose pass, and dgrad reads the forward weights directly with the
// tap flip folded into the gather.
//
// Block = 256 threads = 4 waves (2x2), tile BMxBN, BK = 64; register-staged double-buffered LDS
// with the async-STAGE split (issue global loads for tile t+1 before the MFMAs of tile t, write
// LDS after them; one barrier per K-tile).  The MFMA is issued as D = B·A so each lane owns 4
// consecutive output channels of one output pixel: the epilogue writes 8-byte (bf16) / 16-byte
// (fp32) vectors straight into the NHWC / [M][N] result, and BatchNorm statistics come out of
// the accumulators with four lane shuffles (no extra pass over y).
//
// Reference parity: replaces the TF/cuDNN conv + dense ops of examples/models/image_classification
// (TfVgg16.py:115-130, TfFeedForward.py:141-164) and pg_gans `_conv2d`/`_dense`
// (pg_gans.py:998-1029).  Numerics: fp32 accumulate of bf16 products (tests compare against a
// PyTorch fp32 reference of the same op).
#include "common.h"
#include <cstdlib>

namespace {

constexpr int BK = 64;

enum OpMode {
  OP_DENSE_KIN = 0,   // X[i][k], row stride ld                      (weights, dense A)
  OP_CONV_KIN = 1,    // NHWC gather, tap shift +(kh-1,kw-1)         (conv forward A)
  OP_CONVT_KIN = 2,   // NHWC gather, tap shift -(kh-1,kw-1)         (conv data-grad A)
  OP_DENSE_KOUT = 3,  // X[k][i], row stride ld                      (dY in wgrad, W in dX)
  OP_CONV_KOUT = 4,   // rows = pixels, cols = (tap, c) gathered     (conv weight-grad B)
  OP_WTAP_KOUT = 5,   // rows = (tap, co), cols = c of W[co][tap][c] (conv data-grad B)
  OP_CONVUP_KIN = 6,  // NHWC gather from a 2x nearest-upscaled input (fused upscale2d + conv3x3)
};
enum EpiMode { EPI_BF16 = 0, EPI_F32 = 1 };
// FLAG_SATOM (with FLAG_STATS): add the per-wave (sum, sumsq) into fp64 slots [SL][2][N] at p.stats
// with device-scope atomics instead of writing partial rows; slot = blockIdx & ((flags >> 12) & 15).
// FLAG_BNB (data-gradient into a BatchNorm+ReLU layer): out = v * [y*scale + shift > 0] with y read
// through `gate` and scale/shift = bias[0:N] / bias[N:2N]; the per-channel sums (sum dz,
// sum dz*y) that BN backward needs go to the fp64 slot table `stats` (with FLAG_SATOM), so that
// layer's separate reduction pass disappears.
enum Flags { FLAG_RELU = 1, FLAG_BIAS = 2, FLAG_STATS = 4, FLAG_GATE = 8, FLAG_ACCUM = 16,
             FLAG_LRELU = 32, FLAG_SATOM = 256, FLAG_BNB = 512, FLAG_BNP = 1024 };
// FLAG_BNP (data-gradient into a BatchNorm+ReLU+2x2-max-pool layer): the output is that layer's
// pooled gradient (stored unchanged); its BN-backward sums are formed here: per output element the
// window's first maximal act(y*scale+shift) (y read through `gate` at the 2Hx2W input resolution,
// power-of-two geometry) routes the gradient, (sum dz, sum dz*y) -> fp64 slots (with FLAG_SATOM).

struct IgemmParams {
  const bf16* A;
  const bf16* B;
  void* out;
  const float* bias;    // [N]
  float* stats;         // [tilesM*2][2][N] per-wave partial (sum, sumsq) of the fp32 outputs
  const bf16* gate;     // [M][ldc]: out = gate > 0 ? out : 0 (ReLU backward fused in epilogue)
  int M, N, K;
  int lda, ldb, ldc;
  int H, W, C, taps;    // geometry of the gathered NHWC activation
  int log2H, log2W, log2C, log2Cb;  // log2Cb: channel count of the tap-major weight rows (dgrad)
  int P;                // rows of a pixel-indexed K-outer operand
  int ktPer;            // K-tiles per split (gridDim.z splits)
  long long slabStride; // elements between split-K slabs
  int flags;
  float alpha;          // output scale
  float slope;          // leaky-relu slope
  unsigned long long bytesA, bytesB;  // operand extents for the buffer descriptors (< 2 GiB)
  float invC, invH, invW;             // reciprocals for non-power-of-two channel / spatial extents
};

// channel arithmetic of the gathered activation: shifts when C is a power of two (every VGG /
// PG-GAN layer but one), multiply / reciprocal otherwise (the PG-GAN discriminator's 4x4 conv sees
// 512 + 1 minibatch-stddev channels, padded to 520).  The branch is on a kernel argument (uniform).
RK_DEV int ch_div(int k, const IgemmParams& p) {
  return p.log2C >= 0 ? (k >> p.log2C) : (int)(((float)k + 0.5f) * p.invC);
}
RK_DEV int ch_mod(int k, int q, const IgemmParams& p) { return p.log2C >= 0 ? (k & (p.C - 1)) : k - q * p.C; }
RK_DEV unsigned ch_mul(unsigned v, const IgemmParams& p) { return p.log2C >= 0 ? (v << p.log2C) : v * (unsigned)p.C; }
// pixel index -> (n, h, w).  Power-of-two maps use shifts; others (VGG16 at 48x48: 48/24/12/6/3) an
// fp32 reciprocal, exact for pixel indices < 2^22 (checked on the host).
RK_DEV void pix_nhw(int k, const IgemmParams& p, int& n, int& h, int& w) {
  if (p.log2H >= 0 && p.log2W >= 0) {
    w = k & (p.W - 1); h = (k >> p.log2W) & (p.H - 1); n = k >> (p.log2W + p.log2H);
  } else {
    const int q = (int)(((float)k + 0.5f) * p.invW);
    w = k - q * p.W;
    n = (int)(((float)q + 0.5f) * p.invH);
    h = q - n * p.H;
  }
}

// ---- LDS images --------------------------------------------------------------------------------
// K-inner [T][BK] bf16, 128-byte rows, 16-B chunk c of row i lives at chunk (c ^ ((i>>1)&7)):
// the 16 lanes of each ds_read_b128 lane group hit 16 distinct bank slots.
RK_DEV int kin_off(int i, int c) { return i * 128 + ((c ^ ((i >> 1) & 7)) << 4); }

// K-outer [BK][T] bf16, T/8 chunks per row; XOR the chunk with a row hash (guide T10 form (b)).
template <int R>
RK_DEV int kout_off(int k, int ch) {
  if constexpr (R == 16) return k * 256 + ((ch ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 4);
  else return k * 128 + ((ch ^ (((k & 3) << 1) | ((k >> 2) & 1))) << 4);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// Operand staging goes through buffer loads: a 128-bit descriptor (built from kernel arguments,
// so wave-uniform) + a 32-bit byte offset per lane.  Out-of-range offsets (conv halo, tile
// edges, K tail) are set to OOB and the hardware range check returns zeros — no zero-fill select
// on the loaded data (that made hipcc wait vmcnt right after every load, serialising global
// latency into each K-tile) and no 64-bit address arithmetic.  Per-row tap validity for the conv
// gather is a 9-bit mask computed once per thread, so a K-tile costs ~3 VALU per staged chunk.
constexpr unsigned OOB = 0x80000000u;

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

RK_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned long long bytes) {
  const unsigned nrec = bytes >= 0x80000000ull ? 0x80000000u : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nrec, 0x00020000);
}

RK_DEV uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// tap t of a 3x3 kernel -> (dy, dx) in {-1,0,1}^2 (times the gather sign s)
RK_DEV int tap_dy(int t) { return ((t * 11) >> 5) - 1; }
RK_DEV int tap_dx(int t) { return t - 3 * ((t * 11) >> 5) - 1; }

template <int MODE, int T>
struct Operand {
  static constexpr bool KIN = (MODE == OP_DENSE_KIN || MODE == OP_CONV_KIN || MODE == OP_CONVT_KIN ||
                               MODE == OP_CONVUP_KIN);
  static constexpr int CH = T * BK / 8 / 256;  // 16-B chunks per thread per K-tile
  static constexpr int R = T / 8;              // chunks per K-outer row
  static constexpr int KROWS_PER_PASS = 256 / R;

  __amdgpu_buffer_rsrc_t rsrc;
  int ldsoff[CH];
  // K-inner state
  unsigned rowoff[CH];  // byte offset of the row (pixel / matrix row)
  unsigned tapmask[CH]; // conv: bit t = tap t in bounds for this row; dense: 1 if row valid
  int cchunk;
  // K-outer state
  int krow0;
  unsigned coloff;
  bool colok;
  int dh, dw;  // fixed tap shift (conv K-outer)

  RK_DEV void init(const IgemmParams& p, const bf16* ptr, unsigned long long bytes, int ld, int tile0, int extent,
                   int tid) {
    rsrc = make_rsrc(ptr, bytes);
    if constexpr (KIN) {
      cchunk = tid & 7;
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int r = (tid >> 3) + 32 * i;
        ldsoff[i] = kin_off(r, cchunk);
        const int gi = tile0 + r;
        const bool ok = gi < extent;
        if constexpr (MODE == OP_DENSE_KIN) {
          rowoff[i] = (unsigned)gi * (unsigned)ld * 2u;
          tapmask[i] = ok ? 1u : 0u;
        } else {
          int n, h, w;
          pix_nhw(gi, p, n, h, w);
          if constexpr (MODE == OP_CONVUP_KIN) {
            // output pixel (n, h, w) reads input pixel (n, (h+dy)>>1, (w+dx)>>1) of the H/2 x W/2 map
            const unsigned ip = ((unsigned)n * (unsigned)(p.H >> 1) + (unsigned)(h >> 1)) * (unsigned)(p.W >> 1) +
                                (unsigned)(w >> 1);
            rowoff[i] = ch_mul(ip, p) * 2u;
          } else {
            rowoff[i] = ch_mul((unsigned)gi, p) * 2u;
          }
          unsigned m = 0;
          if (p.taps == 1) {
            m = 1u;
          } else {
#pragma unroll
            for (int t = 0; t < 9; ++t) {
              int dy = tap_dy(t), dx = tap_dx(t);
              if constexpr (MODE == OP_CONVT_KIN) { dy = -dy; dx = -dx; }
              const bool in = (unsigned)(h + dy) < (unsigned)p.H && (unsigned)(w + dx) < (unsigned)p.W;
              m |= (in ? 1u : 0u) << t;
            }
          }
          if constexpr (MODE == OP_CONVUP_KIN) m |= ((unsigned)(h & 1) << 16) | ((unsigned)(w & 1) << 17);
          tapmask[i] = ok ? m : 0u;
        }
      }
    } else {
      const int ch = tid % R;
      krow0 = tid / R;
#pragma unroll
      for (int i = 0; i < CH; ++i) ldsoff[i] = kout_off<R>(krow0 + KROWS_PER_PASS * i, ch);
      const int col = tile0 + ch * 8;
      colok = col < extent;
      dh = dw = 0;
      if constexpr (MODE == OP_CONV_KOUT) {
        const int tap = ch_div(col, p);
        colok = colok && tap < p.taps;
        if (p.taps == 9) { dh = tap_dy(tap); dw = tap_dx(tap); }
        coloff = (unsigned)ch_mod(col, tap, p) * 2u;
      } else {
        coloff = (unsigned)col * 2u;
      }
    }
  }

  RK_DEV void load(const IgemmParams& p, int kt, int K, int ld, uint4 (&r)[CH]) const {
    if constexpr (MODE == OP_DENSE_KIN) {
      const int k = kt * BK + cchunk * 8;
      const bool kok = k < K;
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const bool ok = kok && tapmask[i];
        r[i] = bload(rsrc, ok ? rowoff[i] + (unsigned)k * 2u : OOB);
      }
    } else if constexpr (MODE == OP_CONV_KIN || MODE == OP_CONVT_KIN) {
      const int k = kt * BK + cchunk * 8;
      const int tap = ch_div(k, p);  // >= taps -> no mask bit -> zero
      const int ci = ch_mod(k, tap, p);
      int dy = 0, dx = 0;
      if (p.taps == 9) {
        dy = tap_dy(tap);
        dx = tap_dx(tap);
        if constexpr (MODE == OP_CONVT_KIN) { dy = -dy; dx = -dx; }
      }
      const int delta = ((int)ch_mul((unsigned)(dy * p.W + dx), p) + ci) * 2;
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const bool ok = (tapmask[i] >> tap) & 1u;
        r[i] = bload(rsrc, ok ? (unsigned)((int)rowoff[i] + delta) : OOB);
      }
    } else if constexpr (MODE == OP_CONVUP_KIN) {
      const int k = kt * BK + cchunk * 8;
      const int tap = ch_div(k, p);
      const int ci = ch_mod(k, tap, p);
      const int dy = tap_dy(tap), dx = tap_dx(tap);
      const int Wi = p.W >> 1;
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const unsigned m = tapmask[i];
        const bool ok = (m >> tap) & 1u;
        const int dyi = ((int)((m >> 16) & 1u) + dy) >> 1;  // floor((parity + d) / 2)
        const int dxi = ((int)((m >> 17) & 1u) + dx) >> 1;
        const int delta = ((int)ch_mul((unsigned)(dyi * Wi + dxi), p) + ci) * 2;
        r[i] = bload(rsrc, ok ? (unsigned)((int)rowoff[i] + delta) : OOB);
      }
    } else if constexpr (MODE == OP_DENSE_KOUT) {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int k = kt * BK + krow0 + KROWS_PER_PASS * i;
        const bool ok = colok && k < K;
        r[i] = bload(rsrc, ok ? coloff + (unsigned)k * (unsigned)ld * 2u : OOB);
      }
    } else if constexpr (MODE == OP_CONV_KOUT) {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int k = kt * BK + krow0 + KROWS_PER_PASS * i;  // pixel index
        int n, h, w;
        pix_nhw(k, p, n, h, w);
        const bool ok = colok && k < K && (unsigned)(h + dh) < (unsigned)p.H && (unsigned)(w + dw) < (unsigned)p.W;
        r[i] = bload(rsrc, ok ? ch_mul((unsigned)(k + dh * p.W + dw), p) * 2u + coloff : OOB);
      }
    } else {  // OP_WTAP_KOUT: row k = tap*Cout + co  ->  W[co][tap][c]
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int k = kt * BK + krow0 + KROWS_PER_PASS * i;
        const int tap = k >> p.log2Cb, co = k & ((1 << p.log2Cb) - 1);
        const bool ok = colok && k < K;
        r[i] = bload(rsrc, ok ? ((unsigned)co * (unsigned)ld + (unsigned)tap * (unsigned)p.N) * 2u + coloff : OOB);
      }
    }
  }

  RK_DEV void store(char* lds, const uint4 (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) *(uint4*)(lds + ldsoff[i]) = r[i];
  }

  // Fragment of 16 rows (tile-local r0..r0+15) x 32 k (kb..kb+31) for mfma_f32_16x16x32_bf16:
  // lane l holds X[r0 + (l&15)][kb + 8(l>>4) + j], j = 0..7.
  static RK_DEV bf16x8 frag(const char* lds, int r0, int kb, int lane) {
    if constexpr (KIN) {
      const int i = r0 + (lane & 15);
      const int c = (kb >> 3) + (lane >> 4);
      return *(const bf16x8*)(lds + kin_off(i, c));
    } else {
      const int g = lane >> 4, ii = lane & 15, q = ii >> 2, pp = ii & 3;
      const int ch = (r0 >> 3) + (pp >> 1);
      const int k0 = kb + 8 * g + q;
      const int a0 = kout_off<R>(k0, ch) + 8 * (pp & 1);
      const int a1 = kout_off<R>(k0 + 4, ch) + 8 * (pp & 1);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + a0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + a1));
      const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo), h4 = __builtin_bit_cast(bf16x4, hi);
      bf16x8 f;
      f[0] = l4[0]; f[1] = l4[1]; f[2] = l4[2]; f[3] = l4[3];
      f[4] = h4[0]; f[5] = h4[1]; f[6] = h4[2]; f[7] = h4[3];
      return f;
    }
  }
};

// ================================================================================================
// LDS-DMA variant: operands go global -> LDS directly (buffer_load_dwordx4 ... lds), no VGPR
// staging and no ds_write pass.  The LDS image is lane-linear per wave-instruction (1 KiB), so each
// lane's SOURCE address is chosen by inverting the XOR swizzle: the bytes that land in LDS slot s
// are exactly the chunk kin_off/kout_off would have put there, and the frag() readers are unchanged
// (cdna_hip_programming.md §5.4 rule 21: swizzle the source, keep the destination linear).
// Out-of-range lanes (conv halo, tile edges, K tail) DMA zeros via the descriptor range check.
// NST = 3: a ring of three K-tile stages, two tiles in flight, ONE raw s_barrier per K-tile and a
// counted vmcnt (never __syncthreads(), whose implicit vmcnt(0) would drain the ring).
// ================================================================================================
typedef __attribute__((address_space(3))) void lds_void;

template <int MODE, int T>
struct DmaOperand {
  static constexpr bool KIN = Operand<MODE, T>::KIN;
  static constexpr int R = T / 8;           // 16-B slots per K-outer row / per K-inner tile column
  static constexpr int NI = T / 32;         // wave-instructions (1 KiB each) per wave per K-tile
  __amdgpu_buffer_rsrc_t rsrc;
  // per (lane, instruction) state, fixed across K-tiles
  unsigned base[NI];   // K-inner: row byte offset (+ chunk for dense); K-outer: column byte offset
  unsigned vmask[NI];  // K-inner conv: tap mask; dense: row-valid; K-outer: column-valid
  int sub[NI];         // K-inner: logical chunk c; K-outer: k-row within the tile
  int dh[NI], dw[NI];  // K-outer conv: tap shift of this lane's column
  // Fast path (uniform flag): when a 64-wide K-tile never straddles a tap / image-row boundary the
  // tile-dependent part of every address is wave-uniform (scalar ALU), so each DMA costs ~3 VALU
  // instead of ~15 (integer multiplies, branches).  fbase[q] folds the lane-constant part in.
  bool fast;
  unsigned fbase[NI];
  int fh[NI];          // CONV_KOUT: (k-row's image-row offset + tap dh) of this lane

  RK_DEV void init(const IgemmParams& p, const bf16* ptr, unsigned long long bytes, int ld, int tile0, int extent,
                   int wid, int lane) {
    rsrc = make_rsrc(ptr, bytes);
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int j = wid * NI + q;        // wave-instruction index within the operand tile
      const int slot = j * 64 + lane;    // 16-B slot this lane's bytes land in
      if constexpr (KIN) {
        const int i = slot >> 3;                       // tile row
        const int c = (slot & 7) ^ ((i >> 1) & 7);     // logical chunk stored at this slot
        sub[q] = c;
        const int gi = tile0 + i;
        const bool ok = gi < extent;
        if constexpr (MODE == OP_DENSE_KIN) {
          base[q] = (unsigned)gi * (unsigned)ld * 2u + (unsigned)c * 16u;
          vmask[q] = ok ? 1u : 0u;
        } else {
          const int h = (gi >> p.log2W) & (p.H - 1), w = gi & (p.W - 1);
          base[q] = ((unsigned)gi << p.log2C) * 2u;
          unsigned m = 1u;
          if (p.taps == 9) {
            m = 0u;
#pragma unroll
            for (int t = 0; t < 9; ++t) {
              int dy = tap_dy(t), dx = tap_dx(t);
              if constexpr (MODE == OP_CONVT_KIN) { dy = -dy; dx = -dx; }
              m |= (((unsigned)(h + dy) < (unsigned)p.H && (unsigned)(w + dx) < (unsigned)p.W) ? 1u : 0u) << t;
            }
          }
          vmask[q] = ok ? m : 0u;
        }
        dh[q] = dw[q] = 0;
      } else {
        const int krow = slot / R;
        int f;
        if constexpr (R == 16) f = ((krow & 3) << 2) | ((krow >> 2) & 3);
        else f = ((krow & 3) << 1) | ((krow >> 2) & 1);
        const int ch = (slot % R) ^ f;
        sub[q] = krow;
        const int col = tile0 + ch * 8;
        bool ok = col < extent;
        dh[q] = dw[q] = 0;
        if constexpr (MODE == OP_CONV_KOUT) {
          const int tap = col >> p.log2C;
          ok = ok && tap < p.taps;
          if (p.taps == 9) { dh[q] = tap_dy(tap); dw[q] = tap_dx(tap); }
          base[q] = (unsigned)(col & (p.C - 1)) * 2u;
        } else {
          base[q] = (unsigned)col * 2u;
        }
        vmask[q] = ok ? 1u : 0u;
      }
    }
    // ---- fast-path preconditions (uniform) and lane constants
    const bool k64 = (p.K & (BK - 1)) == 0;
    if constexpr (MODE == OP_DENSE_KIN) {
      fast = k64;
#pragma unroll
      for (int q = 0; q < NI; ++q) fbase[q] = vmask[q] ? base[q] : OOB;
    } else if constexpr (MODE == OP_CONV_KIN || MODE == OP_CONVT_KIN) {
      fast = p.log2C >= 6;  // C % 64 == 0: one tap per K-tile
#pragma unroll
      for (int q = 0; q < NI; ++q) fbase[q] = base[q] + (unsigned)sub[q] * 16u;
    } else if constexpr (MODE == OP_DENSE_KOUT) {
      fast = k64;
#pragma unroll
      for (int q = 0; q < NI; ++q) fbase[q] = vmask[q] ? base[q] + (unsigned)sub[q] * (unsigned)ld * 2u : OOB;
    } else if constexpr (MODE == OP_WTAP_KOUT) {
      fast = k64 && p.log2Cb >= 6;
#pragma unroll
      for (int q = 0; q < NI; ++q) fbase[q] = vmask[q] ? base[q] + (unsigned)sub[q] * (unsigned)ld * 2u : OOB;
    } else {  // OP_CONV_KOUT: pixel rows; a 64-pixel tile = 64/W whole image rows of one image
      fast = k64 && p.log2W >= 0 && p.log2H >= 0 && p.W <= BK && p.log2C >= 0 && (p.H * p.W) % BK == 0;
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const int wl = sub[q] & (p.W - 1);
        const bool wok = (unsigned)(wl + dw[q]) < (unsigned)p.W;
        fh[q] = (sub[q] >> (p.log2W > 0 ? p.log2W : 0)) + dh[q];
        fbase[q] = (vmask[q] && wok) ? base[q] + ((unsigned)(sub[q] + dh[q] * p.W + dw[q]) << p.log2C) * 2u : OOB;
      }
    }
  }

  // byte offset (or OOB) of this lane's chunk for instruction q of K-tile kt
  RK_DEV unsigned offset(const IgemmParams& p, int q, int kt, int K, int ld) const {
    if constexpr (MODE == OP_DENSE_KIN) {
      const int k = kt * BK + sub[q] * 8;
      return (vmask[q] && k < K) ? base[q] + (unsigned)(kt * BK) * 2u : OOB;
    } else if constexpr (MODE == OP_CONV_KIN || MODE == OP_CONVT_KIN) {
      const int k = kt * BK + sub[q] * 8;
      const int tap = k >> p.log2C, ci = k & (p.C - 1);
      int dy = 0, dx = 0;
      if (p.taps == 9) {
        dy = tap_dy(tap);
        dx = tap_dx(tap);
        if constexpr (MODE == OP_CONVT_KIN) { dy = -dy; dx = -dx; }
      }
      const bool ok = (vmask[q] >> tap) & 1u;
      return ok ? (unsigned)((int)base[q] + ((((dy * p.W + dx) << p.log2C) + ci) * 2)) : OOB;
    } else if constexpr (MODE == OP_DENSE_KOUT) {
      const int k = kt * BK + sub[q];
      return (vmask[q] && k < K) ? base[q] + (unsigned)k * (unsigned)ld * 2u : OOB;
    } else if constexpr (MODE == OP_CONV_KOUT) {
      const int k = kt * BK + sub[q];
      const int h = (k >> p.log2W) & (p.H - 1), w = k & (p.W - 1);
      const bool ok = vmask[q] && k < K && (unsigned)(h + dh[q]) < (unsigned)p.H &&
                      (unsigned)(w + dw[q]) < (unsigned)p.W;
      return ok ? (((unsigned)(k + dh[q] * p.W + dw[q])) << p.log2C) * 2u + base[q] : OOB;
    } else {  // OP_WTAP_KOUT
      const int k = kt * BK + sub[q];
      const int tap = k >> p.log2Cb, co = k & ((1 << p.log2Cb) - 1);
      return (vmask[q] && k < K) ? ((unsigned)co * (unsigned)ld + (unsigned)tap * (unsigned)p.N) * 2u + base[q]
                                 : OOB;
    }
  }

  RK_DEV void issue(const IgemmParams& p, char* lds_tile, int kt, int K, int ld, int wid) const {
    if (fast) {
      unsigned off[NI];
      const int k0 = kt * BK;  // wave-uniform below: scalar ALU
      if constexpr (MODE == OP_DENSE_KIN) {
#pragma unroll
        for (int q = 0; q < NI; ++q) off[q] = fbase[q] == OOB ? OOB : fbase[q] + (unsigned)k0 * 2u;
      } else if constexpr (MODE == OP_CONV_KIN || MODE == OP_CONVT_KIN) {
        const int tap = k0 >> p.log2C, ci0 = k0 & (p.C - 1);
        int dy = 0, dx = 0;
        if (p.taps == 9) {
          dy = tap_dy(tap);
          dx = tap_dx(tap);
          if constexpr (MODE == OP_CONVT_KIN) { dy = -dy; dx = -dx; }
        }
        const int delta = ((((dy * p.W + dx) << p.log2C) + ci0) * 2);
#pragma unroll
        for (int q = 0; q < NI; ++q) off[q] = ((vmask[q] >> tap) & 1u) ? (unsigned)((int)fbase[q] + delta) : OOB;
      } else if constexpr (MODE == OP_DENSE_KOUT) {
        const unsigned delta = (unsigned)k0 * (unsigned)ld * 2u;
#pragma unroll
        for (int q = 0; q < NI; ++q) off[q] = fbase[q] == OOB ? OOB : fbase[q] + delta;
      } else if constexpr (MODE == OP_WTAP_KOUT) {
        const int tap = k0 >> p.log2Cb, co0 = k0 & ((1 << p.log2Cb) - 1);
        const unsigned delta = ((unsigned)co0 * (unsigned)ld + (unsigned)tap * (unsigned)p.N) * 2u;
#pragma unroll
        for (int q = 0; q < NI; ++q) off[q] = fbase[q] == OOB ? OOB : fbase[q] + delta;
      } else {  // OP_CONV_KOUT
        const int h0 = (k0 >> p.log2W) & (p.H - 1);
        const unsigned delta = ((unsigned)k0 << p.log2C) * 2u;
#pragma unroll
        for (int q = 0; q < NI; ++q)
          off[q] = (fbase[q] != OOB && (unsigned)(h0 + fh[q]) < (unsigned)p.H) ? fbase[q] + delta : OOB;
      }
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        char* dst = lds_tile + (wid * NI + q) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)dst, 16, (int)off[q], 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      char* dst = lds_tile + (wid * NI + q) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)dst, 16, (int)offset(p, q, kt, K, ld), 0, 0, 0);
    }
  }
};

template <int N>
RK_DEV void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

RK_DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Sum over each 16-lane row of the wave with DPP lane permutes folded into the adds (no LDS
// round trip, unlike __shfl_xor's ds_bpermute): quad xor 1, quad xor 2, half-row mirror, row mirror.
RK_DEV float dpp_sum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

// BF16 tile epilogue shared by every kernel: lane owns out[m][n..n+3] of each (i, j) fragment.
// The flag set FL is a template argument: with runtime flags hipcc if-converts every optional step
// (activation, gate, statistics) into always-executed VALU + selects (~190 extra VALU per tile).
// tile_epilogue dispatches the common sets to specialised copies; FL = -1 is the runtime-flag
// fallback for any other combination.  GUARD: partial tiles (m >= M or n >= N lanes skip).
template <int MI, int NI, int FL, bool GUARD>
RK_DEV void tile_epi(const IgemmParams& p, f32x4 (&acc)[MI][NI], int mrow, int ncol, int mt, int wm, int lane) {
  const int fl = FL < 0 ? p.flags : FL;
  const bool ST = fl & FLAG_STATS, BI = fl & FLAG_BIAS, RE = fl & FLAG_RELU, LR = fl & FLAG_LRELU,
             GA = fl & FLAG_GATE, BB = fl & FLAG_BNB, BP = fl & FLAG_BNP;
  bf16* C = (bf16*)p.out;
  float s[NI][4], ss[NI][4];
#pragma unroll
  for (int j = 0; j < NI; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s[j][e] = ss[j][e] = 0.f;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int n = ncol + j * 16;
    const bool nok = !GUARD || n < p.N;
    f32x4 b = {0.f, 0.f, 0.f, 0.f}, sh = {0.f, 0.f, 0.f, 0.f};
    if ((BI || BB || BP) && nok) b = *(const f32x4*)(p.bias + n);
    if ((BB || BP) && nok) sh = *(const f32x4*)(p.bias + p.N + n);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = mrow + i * 16;
      if (GUARD && !(nok && m < p.M)) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = BI ? acc[i][j][e] * p.alpha + b[e] : acc[i][j][e] * p.alpha;
        if (ST) {
          s[j][e] += v[e];
          ss[j][e] += v[e] * v[e];
        }
        if (RE) v[e] = fmaxf(v[e], 0.f);
        else if (LR) v[e] = v[e] > 0.f ? v[e] : v[e] * p.slope;
      }
      if (GA) {
        const bf16x4 g = *(const bf16x4*)(p.gate + (long long)m * p.ldc + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (float)g[e] > 0.f ? v[e] : 0.f;
      }
      if (BB) {
        const bf16x4 g = *(const bf16x4*)(p.gate + (long long)m * p.ldc + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float yv = (float)g[e];
          // the sums see the bf16 value that is stored and that the BN-backward apply reads
          v[e] = yv * b[e] + sh[e] > 0.f ? (float)(bf16)v[e] : 0.f;
          s[j][e] += v[e];
          ss[j][e] += v[e] * yv;
        }
      }
      if (BP) {
        const int wo = m & (p.W - 1), t = m >> p.log2W, ho = t & (p.H - 1), nimg = t >> p.log2H;
        const long long row = 2LL * p.W * p.ldc;
        const long long b0 = (((long long)nimg * 2 * p.H + 2 * ho) * (2LL * p.W) + 2 * wo) * p.ldc + n;
        bf16x4 g4[4];
        g4[0] = *(const bf16x4*)(p.gate + b0);
        g4[1] = *(const bf16x4*)(p.gate + b0 + p.ldc);
        g4[2] = *(const bf16x4*)(p.gate + b0 + row);
        g4[3] = *(const bf16x4*)(p.gate + b0 + row + p.ldc);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float best = -INFINITY, zb = 0.f, yb = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // first maximal element of the window (torch rule)
            const float yv = (float)g4[q][e];
            const float z = yv * b[e] + sh[e];
            const float a = fmaxf(z, 0.f);
            if (a > best) { best = a; zb = z; yb = yv; }
          }
          v[e] = (float)(bf16)v[e];   // as stored (the pooled gradient the apply pass reads)
          const float dz = zb > 0.f ? v[e] : 0.f;
          s[j][e] += dz;
          ss[j][e] += dz * yb;
        }
      }
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
      *(bf16x4*)(C + (long long)m * p.ldc + n) = o;
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (ST || BB || BP) {
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[j][e] = dpp_sum16(s[j][e]);
        ss[j][e] = dpp_sum16(ss[j][e]);
      }
    if (fl & FLAG_SATOM) {
      // every lane of a 16-lane row holds the row's 8*NI sums: lane l adds value l (+16k)
      double* accd = (double*)p.stats + (long long)(blockIdx.x & ((p.flags >> 12) & 15)) * 2 * p.N;
      const int l16 = lane & 15;
#pragma unroll
      for (int k = 0; k < NI / 2; ++k) {
        const int v = l16 + 16 * k;
        const int kind = v / (4 * NI), r = v - kind * 4 * NI, jsel = r >> 2, esel = r & 3;
        float val = 0.f;
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (j == jsel && e == esel) val = kind ? ss[j][e] : s[j][e];
        const int n = ncol + jsel * 16 + esel;
        if (!GUARD || n < p.N) unsafeAtomicAdd(accd + kind * p.N + n, (double)val);
      }
    } else if ((lane & 15) == 0) {
      float* row = p.stats + (long long)(mt * 2 + wm) * 2 * p.N;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = ncol + j * 16;
        if (GUARD && n >= p.N) continue;
        *(f32x4*)(row + n) = f32x4{s[j][0], s[j][1], s[j][2], s[j][3]};
        *(f32x4*)(row + p.N + n) = f32x4{ss[j][0], ss[j][1], ss[j][2], ss[j][3]};
      }
    }
  }
}

template <int MI, int NI, bool GUARD>
RK_DEV void tile_epilogue(const IgemmParams& p, f32x4 (&acc)[MI][NI], int mrow, int ncol, int mt, int wm,
                          int lane) {
  constexpr int S_ = FLAG_STATS, B_ = FLAG_BIAS, R_ = FLAG_RELU, L_ = FLAG_LRELU, G_ = FLAG_GATE, A_ = FLAG_SATOM;
  switch (p.flags & (S_ | B_ | R_ | L_ | G_ | A_ | FLAG_BNB | FLAG_BNP)) {
    case 0: return tile_epi<MI, NI, 0, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    case S_: return tile_epi<MI, NI, S_, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    case S_ | A_: return tile_epi<MI, NI, S_ | A_, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    case G_: return tile_epi<MI, NI, G_, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    case B_: return tile_epi<MI, NI, B_, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    case B_ | R_: return tile_epi<MI, NI, B_ | R_, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    case B_ | L_: return tile_epi<MI, NI, B_ | L_, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    case FLAG_BNB | A_: return tile_epi<MI, NI, FLAG_BNB | A_, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    case FLAG_BNP | A_: return tile_epi<MI, NI, FLAG_BNP | A_, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
    default: return tile_epi<MI, NI, -1, GUARD>(p, acc, mrow, ncol, mt, wm, lane);
  }
}

template <int BM, int BN, int AM, int BMODE, int EPI, int NST>
__global__ __launch_bounds__(256) void igemm_dma_kernel(const IgemmParams p) {
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, SB = A_BYTES + B_BYTES;
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NI = WN / 16;
  constexpr int L = DmaOperand<AM, BM>::NI + DmaOperand<BMODE, BN>::NI;  // DMA instr / wave / K-tile
  __shared__ __attribute__((aligned(16))) char smem[NST * SB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int tilesN = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / tilesN, nt = bid - mt * tilesN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kTiles = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.ktPer;
  const int kt1 = min(kTiles, kt0 + p.ktPer);

  DmaOperand<AM, BM> opA;
  DmaOperand<BMODE, BN> opB;
  opA.init(p, p.A, p.bytesA, p.lda, m0, p.M, wid, lane);
  opB.init(p, p.B, p.bytesB, p.ldb, n0, p.N, wid, lane);

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt, int stage) {
    char* st = smem + stage * SB;
    opA.issue(p, st, kt, p.K, p.lda, wid);
    opB.issue(p, st + A_BYTES, kt, p.K, p.ldb, wid);
  };
  auto compute = [&](const char* la) {
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = Operand<AM, BM>::frag(la, wm * WM + i * 16, ks * 32, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = Operand<BMODE, BN>::frag(lb, wn * WN + j * 16, ks * 32, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (NST == 2) {
    if (kt0 < kt1) issue(kt0, 0);
    if (kt0 + 1 < kt1) issue(kt0 + 1, 1);
    int stage = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      if (kt + 1 < kt1) wait_vmcnt<L>();   // this wave's DMAs of tile kt landed (kt+1 may fly)
      else wait_vmcnt<0>();
      raw_barrier();                       // ... and every other wave's
      compute(smem + stage * SB);
      raw_barrier();                       // everyone is done reading this stage
      if (kt + 2 < kt1) issue(kt + 2, stage);
      stage ^= 1;
    }
  } else {
    // NST-stage ring, NST-1 tiles in flight: at tile kt, wait for it, one barrier, then refill the
    // stage tile kt-1 used (every wave is past computing it) with tile kt+NST-1, then compute kt
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
      if (kt0 + t < kt1) issue(kt0 + t, t);
    int stage = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const int ahead = kt1 - 1 - kt;      // tiles after kt already issued (capped below)
      if (ahead >= NST - 2) wait_vmcnt<L * (NST - 2)>();
      else if (NST >= 4 && ahead == 2) wait_vmcnt<L * 2>();
      else if (ahead == 1) wait_vmcnt<L>();
      else wait_vmcnt<0>();
      raw_barrier();
      if (kt + NST - 1 < kt1) issue(kt + NST - 1, stage == 0 ? NST - 1 : stage - 1);
      compute(smem + stage * SB);
      stage = stage == NST - 1 ? 0 : stage + 1;
    }
  }
  wait_vmcnt<0>();

  // ---- epilogue: lane owns out[m][n..n+3] of every (i, j) fragment --------------------------
  const int mrow = m0 + wm * WM + (lane & 15);
  const int ncol = n0 + wn * WN + 4 * (lane >> 4);
  if constexpr (EPI == EPI_BF16) {
    tile_epilogue<MI, NI, true>(p, acc, mrow, ncol, mt, wm, lane);
  } else {
    float* C = (float*)p.out + (long long)blockIdx.z * p.slabStride;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = ncol + j * 16;
      if (n >= p.N) continue;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = mrow + i * 16;
        if (m >= p.M) continue;
        f32x4 v = acc[i][j] * p.alpha;
        if (p.flags & FLAG_BIAS) v += *(const f32x4*)(p.bias + n);
        float* dst = C + (long long)m * p.ldc + n;
        if (p.flags & FLAG_ACCUM) v += *(const f32x4*)dst;
        *(f32x4*)dst = v;
      }
    }
  }
}

// ================================================================================================
// Wave-K-split 64x64 tile (tile shape 4).  The 2x2 wave grid above gives each wave a 32x32 quarter:
// 8 fragment reads (ds_read) per 8 MFMAs, and with the DMA writes that is ~1.5x the LDS bandwidth
// a CU has at full MFMA rate — the wall the small-M layers hit (VGG 4x4 / 8x8 convs: M = 4096 /
// 16384, where 64x64 is the only tile that fills 256 CUs without split-K slabs).  Here every wave
// owns the WHOLE 64x64 output tile for one 32-wide k-slice of each PAIR of K-tiles (4 slices per
// ring stage, one per wave): 8 fragment reads per 16 MFMAs.  The four partial tiles meet in LDS at
// the end and wave w runs the epilogue for rows 16w..16w+15 (fp64-atomic statistics only: the
// per-wave partial-row layout of FLAG_STATS without FLAG_SATOM is refused on the host).
// Ring: NST stages of two K-tiles, NST-1 pairs in flight, one raw barrier per pair.  An odd K-tile
// count leaves the last pair half-filled (waves 2-3 skip it); while that pair is in flight the
// counted waits fall back to vmcnt(0), since it carries fewer DMAs than the count assumes.
// ================================================================================================
template <int AM, int BMODE, int EPI, int NST>
__global__ __launch_bounds__(256) void igemm_ks_kernel(const IgemmParams p) {
  constexpr int BM = 64, BN = 64, MI = 4, NI = 4;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, TB = A_BYTES + B_BYTES, SB = 2 * TB;
  constexpr int L2 = 2 * (DmaOperand<AM, BM>::NI + DmaOperand<BMODE, BN>::NI);  // DMA instr / wave / pair
  constexpr int SMEM = NST * SB > 4 * MI * NI * 64 * 16 ? NST * SB : 4 * MI * NI * 64 * 16;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wid >> 1, ks = wid & 1;  // K-tile of the pair, 32-wide slice of that tile
  const int tilesN = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / tilesN, nt = bid - mt * tilesN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kTiles = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.ktPer;
  const int kt1 = min(kTiles, kt0 + p.ktPer);
  const int nPairs = kt1 > kt0 ? (kt1 - kt0 + 1) >> 1 : 0;
  const bool oddTail = ((kt1 - kt0) & 1) != 0;

  DmaOperand<AM, BM> opA;
  DmaOperand<BMODE, BN> opB;
  opA.init(p, p.A, p.bytesA, p.lda, m0, p.M, wid, lane);
  opB.init(p, p.B, p.bytesB, p.ldb, n0, p.N, wid, lane);

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int pr, int stage) {
    char* st = smem + stage * SB;
    const int kt = kt0 + 2 * pr;
    opA.issue(p, st, kt, p.K, p.lda, wid);
    opB.issue(p, st + A_BYTES, kt, p.K, p.ldb, wid);
    if (kt + 1 < kt1) {
      opA.issue(p, st + TB, kt + 1, p.K, p.lda, wid);
      opB.issue(p, st + TB + A_BYTES, kt + 1, p.K, p.ldb, wid);
    }
  };
  auto compute = [&](const char* sp) {
    const char* la = sp + half * TB;
    const char* lb = la + A_BYTES;
    bf16x8 af[MI], bfr[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = Operand<AM, BM>::frag(la, i * 16, ks * 32, lane);
#pragma unroll
    for (int j = 0; j < NI; ++j) bfr[j] = Operand<BMODE, BN>::frag(lb, j * 16, ks * 32, lane);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };

#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nPairs) issue(t, t);
  int stage = 0;
  for (int pr = 0; pr < nPairs; ++pr) {
    const int ahead = nPairs - 1 - pr;  // pairs after pr already issued (capped at NST-2 below)
    if (oddTail && ahead >= 1 && ahead <= NST - 2) wait_vmcnt<0>();
    else if (ahead >= NST - 2) wait_vmcnt<L2 * (NST - 2)>();
    else if (NST >= 4 && ahead == 2) wait_vmcnt<L2 * 2>();
    else if (ahead == 1) wait_vmcnt<L2>();
    else wait_vmcnt<0>();
    raw_barrier();
    if (pr + NST - 1 < nPairs) issue(pr + NST - 1, stage == 0 ? NST - 1 : stage - 1);
    if (half == 0 || kt0 + 2 * pr + 1 < kt1) compute(smem + stage * SB);
    stage = stage == NST - 1 ? 0 : stage + 1;
  }
  wait_vmcnt<0>();
  raw_barrier();  // every wave is done with the ring: reuse it for the cross-wave reduction

  // partial tile of wave w, fragment (i, j) -> red[i][w][j][lane]; wave w then sums row-block i = w
  f32x4* red = (f32x4*)smem;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) red[((i * 4 + wid) * NI + j) * 64 + lane] = acc[i][j];
  __syncthreads();
  f32x4 r[1][NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    f32x4 v = red[((wid * 4 + 0) * NI + j) * 64 + lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) v += red[((wid * 4 + w) * NI + j) * 64 + lane];
    r[0][j] = v;
  }

  const int mrow = m0 + wid * 16 + (lane & 15);
  const int ncol = n0 + 4 * (lane >> 4);
  if constexpr (EPI == EPI_BF16) {
    tile_epilogue<1, NI, true>(p, r, mrow, ncol, mt, 0, lane);
  } else {
    float* C = (float*)p.out + (long long)blockIdx.z * p.slabStride;
    if (mrow < p.M) {
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = ncol + j * 16;
        if (n >= p.N) continue;
        f32x4 v = r[0][j] * p.alpha;
        if (p.flags & FLAG_BIAS) v += *(const f32x4*)(p.bias + n);
        float* dst = C + (long long)mrow * p.ldc + n;
        if (p.flags & FLAG_ACCUM) v += *(const f32x4*)dst;
        *(f32x4*)dst = v;
      }
    }
  }
}

template <int BM, int BN, int AM, int BMODE, int EPI, int PF>
__global__ __launch_bounds__(256) void igemm_kernel(const IgemmParams p) {
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NI = WN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tilesN = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / tilesN, nt = bid - mt * tilesN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kTiles = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.ktPer;
  const int kt1 = min(kTiles, kt0 + p.ktPer);

  Operand<AM, BM> opA;
  Operand<BMODE, BN> opB;
  opA.init(p, p.A, p.bytesA, p.lda, m0, p.M, tid);
  opB.init(p, p.B, p.bytesB, p.ldb, n0, p.N, tid);

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const char* la) {
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = Operand<AM, BM>::frag(la, wm * WM + i * 16, ks * 32, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = Operand<BMODE, BN>::frag(lb, wn * WN + j * 16, ks * 32, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };
  constexpr int SB = A_BYTES + B_BYTES;  // one LDS stage
  uint4 ra0[Operand<AM, BM>::CH], rb0[Operand<BMODE, BN>::CH];
  if constexpr (PF == 1) {
    // one K-tile in flight: issue t+1 before computing t, write it to LDS after
    if (kt0 < kt1) {
      opA.load(p, kt0, p.K, p.lda, ra0);
      opB.load(p, kt0, p.K, p.ldb, rb0);
      opA.store(smem, ra0);
      opB.store(smem + A_BYTES, rb0);
    }
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int cur = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) {
        opA.load(p, kt + 1, p.K, p.lda, ra0);
        opB.load(p, kt + 1, p.K, p.ldb, rb0);
      }
      compute(smem + cur * SB);
      if (more) {
        opA.store(smem + (cur ^ 1) * SB, ra0);
        opB.store(smem + (cur ^ 1) * SB + A_BYTES, rb0);
      }
      __syncthreads();
    }
  } else {
    // two K-tiles in flight through two register sets (static indices: the loop is unrolled by 2):
    // at the top of step t, LDS stage t&1 holds tile t and register set (t+1)&1 holds tile t+1.
    uint4 ra1[Operand<AM, BM>::CH], rb1[Operand<BMODE, BN>::CH];
    if (kt0 < kt1) {
      opA.load(p, kt0, p.K, p.lda, ra0);
      opB.load(p, kt0, p.K, p.ldb, rb0);
      if (kt0 + 1 < kt1) {
        opA.load(p, kt0 + 1, p.K, p.lda, ra1);
        opB.load(p, kt0 + 1, p.K, p.ldb, rb1);
      }
      opA.store(smem, ra0);
      opB.store(smem + A_BYTES, rb0);
    }
    __syncthreads();
    for (int kt = kt0; kt < kt1; kt += 2) {
      // even step: compute stage 0, prefetch kt+2 into set 0, publish set 1 (kt+1) to stage 1
      if (kt + 2 < kt1) {
        opA.load(p, kt + 2, p.K, p.lda, ra0);
        opB.load(p, kt + 2, p.K, p.ldb, rb0);
      }
      compute(smem);
      if (kt + 1 < kt1) {
        opA.store(smem + SB, ra1);
        opB.store(smem + SB + A_BYTES, rb1);
      }
      __syncthreads();
      if (kt + 1 >= kt1) break;
      // odd step: compute stage 1, prefetch kt+3 into set 1, publish set 0 (kt+2) to stage 0
      if (kt + 3 < kt1) {
        opA.load(p, kt + 3, p.K, p.lda, ra1);
        opB.load(p, kt + 3, p.K, p.ldb, rb1);
      }
      compute(smem + SB);
      if (kt + 2 < kt1) {
        opA.store(smem, ra0);
        opB.store(smem + A_BYTES, rb0);
      }
      __syncthreads();
    }
  }

  // ---- epilogue: lane owns out[m][n..n+3] of every (i, j) fragment --------------------------
  const int mrow = m0 + wm * WM + (lane & 15);
  const int ncol = n0 + wn * WN + 4 * (lane >> 4);
  if constexpr (EPI == EPI_BF16) {
    tile_epilogue<MI, NI, true>(p, acc, mrow, ncol, mt, wm, lane);
  } else {
    float* C = (float*)p.out + (long long)blockIdx.z * p.slabStride;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = ncol + j * 16;
      if (n >= p.N) continue;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = mrow + i * 16;
        if (m >= p.M) continue;
        f32x4 v = acc[i][j] * p.alpha;
        if (p.flags & FLAG_BIAS) v += *(const f32x4*)(p.bias + n);
        float* dst = C + (long long)m * p.ldc + n;
        if (p.flags & FLAG_ACCUM) v += *(const f32x4*)dst;
        *(f32x4*)dst = v;
      }
    }
  }
}

template <int BM, int BN, int AM, int BMODE, int EPI>
int launch_tile(const IgemmParams& p, int splits, int pf, hipStream_t st) {
  const int tiles = rk_cdiv(p.M, BM) * rk_cdiv(p.N, BN);
  dim3 grid(tiles, 1, splits);
  if (pf == 5)
    hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, AM, BMODE, EPI, 4>), grid, dim3(256), 0, st, p);
  else if (pf == 3)
    hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, AM, BMODE, EPI, 3>), grid, dim3(256), 0, st, p);
  else if (pf == 4)
    hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, AM, BMODE, EPI, 2>), grid, dim3(256), 0, st, p);
  else if (pf == 2)
    hipLaunchKernelGGL((igemm_kernel<BM, BN, AM, BMODE, EPI, 2>), grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((igemm_kernel<BM, BN, AM, BMODE, EPI, 1>), grid, dim3(256), 0, st, p);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

template <int AM, int BMODE, int EPI>
int launch_modes(int tile, const IgemmParams& p, int splits, hipStream_t st) {
  // tile code: bits 0-3 tile shape; 16 = register ring (2 tiles in flight); 32 = LDS-DMA 3-stage
  // ring; 64 = LDS-DMA 2-stage; 128 = LDS-DMA 4-stage
  const int pf = (tile & 128) ? 5 : (tile & 32) ? 3 : (tile & 64) ? 4 : (tile & 16) ? 2 : 1;
  switch (tile & 15) {
    case 0: return launch_tile<128, 128, AM, BMODE, EPI>(p, splits, pf, st);
    case 1: return launch_tile<128, 64, AM, BMODE, EPI>(p, splits, pf, st);
    case 2: return launch_tile<64, 128, AM, BMODE, EPI>(p, splits, pf, st);
    case 3: return launch_tile<64, 64, AM, BMODE, EPI>(p, splits, pf, st);
    case 4: {  // 64x64 wave-K-split (LDS-DMA only; fp64-atomic statistics only)
      if (pf != 3 && pf != 4) return RK_EUNSUPPORTED;
      if ((p.flags & FLAG_STATS) && !(p.flags & FLAG_SATOM)) return RK_EUNSUPPORTED;
      dim3 grid(rk_cdiv(p.M, 64) * rk_cdiv(p.N, 64), 1, splits);
      if (pf == 3) hipLaunchKernelGGL((igemm_ks_kernel<AM, BMODE, EPI, 3>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((igemm_ks_kernel<AM, BMODE, EPI, 2>), grid, dim3(256), 0, st, p);
      RK_LAUNCH_CHECK();
      return RK_OK;
    }
  }
  return RK_EBADARG;
}

// ================================================================================================
// Halo-tiled 3x3 convolution (forward and data-gradient), persistent over work items.
//
// The implicit GEMM above gathers the activation once per tap: every input pixel crosses the
// L2->LDS path 9 times, which is what bounds the 32x32 / 16x16 VGG layers (~450 TB/s-class L2
// traffic for ~20 % MFMA utilisation).  Here a work item is BM output pixels = TH whole rows of one
// image (BM = TH*W) x BN output channels; per 64-channel input chunk the block DMAs ONE
// (TH+2) x (W+2) halo patch into LDS and runs all 9 taps out of it — the tap is just a constant
// shift of the patch pixel each lane reads (shift = dy*(W+2)+dx, negated for the data-gradient).
// B (weights) streams per (tap, chunk) K-tile through a 3-stage LDS-DMA ring exactly as in
// igemm_dma_kernel (same K-inner / K-outer LDS images and fragment readers).  Patches are double
// buffered: the patch of the next phase (next chunk or next item) is in flight during the 9 taps
// of the current one, so the pipeline never drains between items.  One raw barrier per tap.
// Patch image: pixel pp = 128-byte row (64 channels), 16-B chunk c stored at c ^ (pp&7) — the one
// XOR that keeps ds_read_b128 conflict-free (4 LDS cycles) for ANY start pixel, which the tap shift
// makes arbitrary (the GEMM image's (i>>1)&7 averages 7 cycles here); the
// DMA writes lane-linear, so each lane's SOURCE is the chunk that belongs in its slot, and slots
// outside the image (halo at the border, padding) read zeros through the buffer range check.
// ================================================================================================
// (a device function, not a builtin call inside the kernel's lambdas: hipcc then silently drops the
// host-side launch stub of the kernel template — undefined __device_stub__ at load time)
RK_DEV void dma16(__amdgpu_buffer_rsrc_t r, char* dst, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, off, 0, 0, 0);
}

RK_DEV bf16x8 patch_frag(const char* patch, int pp, int kb, int lane) {
  const int c = (kb >> 3) + (lane >> 4);
  return *(const bf16x8*)(patch + pp * 128 + ((c ^ (pp & 7)) << 4));
}

// IH > 0: whole-image items for small images (VGG 4x4 layers): an item is BM / (IH*W) images, the
// patch stacks one (IH+2) x (W+2) halo image per image, so the tap shift stays a constant offset.
template <int BM, int BN, int W, int BMODE, int FLIP, int IH = 0>
__global__ __launch_bounds__(256, BN == 64 && IH == 0 ? 2 : 1) void hconv_kernel(const IgemmParams p,
                                                                                const int per_block) {
  constexpr int TH = IH ? IH : BM / W;         // output rows per item (per image when IH > 0)
  constexpr int IMG = IH ? BM / (IH * W) : 1;  // images per item
  constexpr int PC = W + 2, PIMG = (TH + 2) * PC, NPP = IMG * PIMG;
  constexpr int LP = (NPP * 8 + 255) / 256;    // patch DMA instructions per wave
  constexpr int P_BYTES = LP * 4 * 1024;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int LB = BN / 32;                  // B DMA instructions per wave per K-tile
  constexpr int R = BN / 8;                    // K-outer B: 16-B slots per k-row
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NI = WN / 16;
  constexpr int LOG2W = W == 4 ? 2 : W == 8 ? 3 : W == 16 ? 4 : 5;
  static_assert(BM % W == 0 && LP + LB <= 63 && (IH == 0 || BM % (IH * W) == 0), "tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * P_BYTES + 3 * B_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int log2C = p.log2C;
  const int NCC = p.C >> 6;
  const int tilesN = p.N / BN;
  const int nItems = (p.M / BM) * tilesN;
  const int tilesPerImg = (p.H * W) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int item0 = bid * per_block;
  const int item1 = min(nItems, item0 + per_block);
  if (item0 >= item1) return;
  const int nPhases = (item1 - item0) * NCC;
  const int S = nPhases * 9;

  const __amdgpu_buffer_rsrc_t rA = make_rsrc(p.A, p.bytesA);
  const __amdgpu_buffer_rsrc_t rB = make_rsrc(p.B, p.bytesB);

  // ---- patch DMA lane constants
  int prel[LP], prow[LP];
#pragma unroll
  for (int q = 0; q < LP; ++q) {
    const int slot = (wid * LP + q) * 64 + lane;
    const int pp = slot >> 3;
    const int c = (slot & 7) ^ (pp & 7);
    const int img = pp / PIMG, rem = pp - img * PIMG;
    const int pr = rem / PC, pcol = rem - pr * PC;
    const bool ok = pp < NPP && pcol >= 1 && pcol <= W && (IH == 0 || (pr >= 1 && pr <= TH));
    prel[q] = ((((img * TH + pr - 1) * W + (pcol - 1)) << log2C) << 1) + c * 16;
    prow[q] = ok ? pr : -1000;
  }
  // ---- B DMA lane constants (tile-independent part of the source offset)
  unsigned boff[LB];
#pragma unroll
  for (int q = 0; q < LB; ++q) {
    const int slot = (wid * LB + q) * 64 + lane;
    if constexpr (BMODE == OP_DENSE_KIN) {  // forward: B[n][k], k contiguous, row length ldb
      const int i = slot >> 3;
      const int c = (slot & 7) ^ ((i >> 1) & 7);
      boff[q] = ((unsigned)i * (unsigned)p.ldb + (unsigned)c * 8u) * 2u;
    } else {  // data-gradient: row k = tap*C + co of W[co][tap][n]
      const int krow = slot / R;
      int f;
      if constexpr (R == 16) f = ((krow & 3) << 2) | ((krow >> 2) & 3);
      else f = ((krow & 3) << 1) | ((krow >> 2) & 1);
      const int ch = (slot % R) ^ f;
      boff[q] = ((unsigned)krow * (unsigned)p.ldb + (unsigned)ch * 8u) * 2u;
    }
  }
  // ---- A fragment rows: patch pixel of each lane's output pixel (before the tap shift)
  int ppb[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int ml = wm * WM + i * 16 + (lane & 15);
    const int img = ml / (TH * W), rem = ml - img * (TH * W);
    ppb[i] = img * PIMG + ((rem >> LOG2W) + 1) * PC + (rem & (W - 1)) + 1;
  }

  // phase = (item, 64-channel chunk): state of the current and the next phase, advanced once per
  // phase on the scalar unit (no per-tap integer division)
  struct Phase { int cc, mt, nt; };
  auto advance = [&](Phase q) {
    if (++q.cc == NCC) {
      q.cc = 0;
      if (++q.nt == tilesN) { q.nt = 0; ++q.mt; }
    }
    return q;
  };
  // B K-tile (phase q, tap t) source = bbase(q) + t * bstep
  const unsigned bstep = BMODE == OP_DENSE_KIN ? (unsigned)p.C * 2u : (unsigned)p.N * 2u;
  auto bbase = [&](const Phase& q) -> unsigned {
    if constexpr (BMODE == OP_DENSE_KIN)
      return ((unsigned)(q.nt * BN) * (unsigned)p.ldb + (unsigned)(q.cc * 64)) * 2u;
    else
      return ((unsigned)(q.cc * 64) * (unsigned)p.ldb + (unsigned)(q.nt * BN)) * 2u;
  };
  auto issue_patch = [&](const Phase& q, int buf) {
    const int r0 = IH ? 0 : (q.mt & (tilesPerImg - 1)) * TH;  // tilesPerImg = H*W/BM: a power of two
    const int base = (((q.mt * BM) << log2C) << 1) + q.cc * 128;
    char* dst = smem + buf * P_BYTES + wid * LP * 1024;
#pragma unroll
    for (int j = 0; j < LP; ++j) {
      const bool in = (unsigned)(r0 - 1 + prow[j]) < (unsigned)p.H;
      dma16(rA, dst + j * 1024, in ? base + prel[j] : (int)OOB);
    }
  };
  auto issue_b = [&](unsigned src, int stage) {
    char* dst = smem + 2 * P_BYTES + stage * B_BYTES + wid * LB * 1024;
#pragma unroll
    for (int j = 0; j < LB; ++j) dma16(rB, dst + j * 1024, (int)(boff[j] + src));
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Phase cur{0, item0 / tilesN, item0 % tilesN};
  Phase nxt = advance(cur);
  unsigned bcur = bbase(cur), bnxt = bbase(nxt);
  issue_patch(cur, 0);
  issue_b(bcur, 0);
  if (S > 1) issue_b(bcur + bstep, 1);
  for (int ph = 0; ph < nPhases; ++ph) {
    const bool last = ph == nPhases - 1;
    const char* pt = smem + (ph & 1) * P_BYTES;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      // loads issued after B(s): B(s+1), plus the next patch when it went out at tap 0 of this phase
      if (last && tap == 8) wait_vmcnt<0>();
      else if ((tap == 1 || tap == 2) && !last) wait_vmcnt<LB + LP>();
      else wait_vmcnt<LB>();
      raw_barrier();
      if (tap + 2 < 9) issue_b(bcur + (unsigned)(tap + 2) * bstep, (tap + 2) % 3);
      else if (!last) issue_b(bnxt + (unsigned)(tap - 7) * bstep, (tap + 2) % 3);
      if (tap == 0 && !last) issue_patch(nxt, (ph + 1) & 1);
      const char* lb = smem + 2 * P_BYTES + (tap % 3) * B_BYTES;
      const int shift = FLIP ? -(tap_dy(tap) * PC + tap_dx(tap)) : (tap_dy(tap) * PC + tap_dx(tap));
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[MI], bfr[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) af[i] = patch_frag(pt, ppb[i] + shift, ks * 32, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j) bfr[j] = Operand<BMODE, BN>::frag(lb, wn * WN + j * 16, ks * 32, lane);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
    if (cur.cc == NCC - 1)  // last chunk of this item: write it out
      tile_epilogue<MI, NI, false>(p, acc, cur.mt * BM + wm * WM + (lane & 15), cur.nt * BN + wn * WN + 4 * (lane >> 4),
                             cur.mt, wm, lane);
    cur = nxt;
    nxt = advance(nxt);
    bcur = bnxt;
    bnxt = bbase(nxt);
  }
}

template <int BM, int BN, int W, int IH = 0>
int launch_hconv_w(bool dgrad, const IgemmParams& p, int grid, hipStream_t st) {
  const int items = (p.M / BM) * (p.N / BN);
  if (grid <= 0 || grid > items) grid = items;
  const int per = rk_cdiv(items, grid);
  grid = rk_cdiv(items, per);
  if (dgrad)
    hipLaunchKernelGGL((hconv_kernel<BM, BN, W, OP_WTAP_KOUT, 1, IH>), dim3(grid), dim3(256), 0, st, p, per);
  else
    hipLaunchKernelGGL((hconv_kernel<BM, BN, W, OP_DENSE_KIN, 0, IH>), dim3(grid), dim3(256), 0, st, p, per);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

template <int BN>
int launch_hconv_bn(bool dgrad, const IgemmParams& p, int grid, hipStream_t st) {
  switch (p.W) {
    case 4: return launch_hconv_w<128, BN, 4, 4>(dgrad, p, grid, st);  // 8 whole 4x4 images per item
    case 8: return launch_hconv_w<64, BN, 8>(dgrad, p, grid, st);
    case 16: return launch_hconv_w<128, BN, 16>(dgrad, p, grid, st);
    case 32: return launch_hconv_w<128, BN, 32>(dgrad, p, grid, st);
  }
  return RK_EUNSUPPORTED;
}

// ================================================================================================
// Halo-tiled 3x3 weight gradient, dW[co][tap][ci] = sum_p dy[p][co] * x[p + tap][ci].
//
// A block owns a (64 co x 64 ci x 9 taps) output tile and a contiguous run of pixel items (TH whole
// image rows = 128 pixels; 64 at W = 8).  Per item it DMAs the dy tile [pixels][64 co] and ONE
// halo patch of x [(TH+2)(W+2) pixels][64 ci] into LDS and runs all 9 taps out of that patch.  Wave
// w owns ci 16w..16w+15 for all 64 co and 9 taps: 36 accumulators (144 AGPRs); per 32-pixel
// K-block a wave reads 4 dy fragments (shared by the 9 taps) + 9 x fragments for 36 MFMAs.  Both
// operands are K-outer (pixels are the reduction index), read with ds_read_b64_tr_b16; the tap
// shift makes the first patch row of a read arbitrary, so the image uses the XOR
// chunk ^ 2*(((row>>1)&1) | ((row>>3)&1)<<1), conflict-free for every start row (the two 4-row
// blocks of a 32-lane half are 8 rows apart).  Items are double buffered.  Each block writes its
// fp32 partial tile into slab blockIdx % S of [S][Cout][9*Cin]; rk_reduce_slabs sums the slabs.
// ================================================================================================
RK_DEV int wtr_off(int k, int ch) {
  return k * 128 + ((ch ^ ((((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1)) << 4);
}

// 16 (M or N) x 32 (K) MFMA operand from a K-outer [rows = K][64 cols] image (wtr_off): K rows
// kb0..kb0+7 of lane group g start at image row rowbase (consecutive), columns c0..c0+15.
// hrow: patch-row distance of K rows 4..7 from rows 0..3 (4 = consecutive; W + 2 for 4-wide images,
// whose 8 consecutive pixels span two patch rows).
RK_DEV bf16x8 wtr_frag(const char* lds, int rowbase, int c0, int lane, int hrow = 4) {
  const int ii = lane & 15, q = ii >> 2, pp = ii & 3;
  const int ch = (c0 >> 3) + (pp >> 1);
  const int a0 = wtr_off(rowbase + q, ch) + 8 * (pp & 1);
  const int a1 = wtr_off(rowbase + q + hrow, ch) + 8 * (pp & 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + a1));
  const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo), h4 = __builtin_bit_cast(bf16x4, hi);
  bf16x8 f;
  f[0] = l4[0]; f[1] = l4[1]; f[2] = l4[2]; f[3] = l4[3];
  f[4] = h4[0]; f[5] = h4[1]; f[6] = h4[2]; f[7] = h4[3];
  return f;
}

// W = 4: an item is 8 whole 4x4 images, their halo patches stacked (as hconv_kernel's IH > 0).
template <int W>
__global__ __launch_bounds__(256, 1) void hconv_wgrad_kernel(const IgemmParams p, const int S, const int per_block) {
  constexpr int P = W == 8 ? 64 : 128;         // pixels per item
  constexpr int IH = W == 4 ? 4 : 0;           // whole-image items of IH rows
  constexpr int TH = IH ? IH : P / W, PC = W + 2, PIMG = (TH + 2) * PC, NPP = (IH ? P / ((IH ? IH : 1) * W) : 1) * PIMG;
  constexpr int HI = W == 4 ? PC : 4;          // patch-row distance of a lane group's pixels 4..7
  constexpr int LP = (NPP * 8 + 255) / 256;    // patch DMA instructions per wave
  constexpr int LY = P / 32;                   // dy-tile DMA instructions per wave
  constexpr int P_BYTES = LP * 4 * 1024, Y_BYTES = P * 128, SB = P_BYTES + Y_BYTES;
  constexpr int LOG2W = W == 4 ? 2 : W == 8 ? 3 : W == 16 ? 4 : 5;
  constexpr int KB = P / 32;
  __shared__ __attribute__((aligned(16))) char smem[2 * SB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int log2C = p.log2C;                   // Cin (x channels)
  const int Cout = p.M;
  const int tilesCi = p.C >> 6;
  const int tile = blockIdx.x / S, sl = blockIdx.x - tile * S;
  const int cot = tile / tilesCi, cit = tile - cot * tilesCi;
  const int co0 = cot * 64, ci0 = cit * 64;
  const int nItems = p.K / P;                  // K = pixels
  const int item0 = sl * per_block;
  const int item1 = min(nItems, item0 + per_block);
  const int tilesPerImg = (p.H * W) / P;

  const __amdgpu_buffer_rsrc_t rX = make_rsrc(p.B, p.bytesB);   // x  [pixels][Cin]
  const __amdgpu_buffer_rsrc_t rY = make_rsrc(p.A, p.bytesA);   // dy [pixels][Cout]

  int prel[LP], prow[LP];
#pragma unroll
  for (int q = 0; q < LP; ++q) {
    const int slot = (wid * LP + q) * 64 + lane;
    const int pp = slot >> 3;
    const int c = (slot & 7) ^ ((((pp >> 1) & 1) | (((pp >> 3) & 1) << 1)) << 1);
    const int img = pp / PIMG, rem = pp - img * PIMG;
    const int pr = rem / PC, pcol = rem - pr * PC;
    const bool ok = pp < NPP && pcol >= 1 && pcol <= W && (IH == 0 || (pr >= 1 && pr <= TH));
    prel[q] = ((((img * TH + pr - 1) * W + (pcol - 1)) << log2C) << 1) + c * 16;
    prow[q] = ok ? pr : -1000;
  }
  unsigned yoff[LY];
#pragma unroll
  for (int q = 0; q < LY; ++q) {
    const int slot = (wid * LY + q) * 64 + lane;
    const int krow = slot >> 3;
    const int c = (slot & 7) ^ ((((krow >> 1) & 1) | (((krow >> 3) & 1) << 1)) << 1);
    yoff[q] = ((unsigned)krow * (unsigned)Cout + (unsigned)c * 8u) * 2u;
  }
  // first patch row of each lane group's 8 pixels in K-block kb (before the tap shift)
  int prb[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int k = kb * 32 + 8 * (lane >> 4);
    const int img = k / (TH * W), rem = k - img * (TH * W);
    prb[kb] = img * PIMG + ((rem >> LOG2W) + 1) * PC + (rem & (W - 1)) + 1;
  }

  auto issue = [&](int it, int buf) {
    const int r0 = IH ? 0 : (it & (tilesPerImg - 1)) * TH;  // tilesPerImg is a power of two
    const int pbase = (((it * P) << log2C) << 1) + ci0 * 2;
    char* dst = smem + buf * SB;
#pragma unroll
    for (int q = 0; q < LP; ++q) {
      const bool in = (unsigned)(r0 - 1 + prow[q]) < (unsigned)p.H;
      dma16(rX, dst + (wid * LP + q) * 1024, in ? pbase + prel[q] : (int)OOB);
    }
    const unsigned ybase = ((unsigned)(it * P) * (unsigned)Cout + (unsigned)co0) * 2u;
#pragma unroll
    for (int q = 0; q < LY; ++q) dma16(rY, dst + P_BYTES + (wid * LY + q) * 1024, (int)(ybase + yoff[q]));
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (item0 < item1) issue(item0, 0);
  for (int it = item0; it < item1; ++it) {
    const int buf = (it - item0) & 1;
    wait_vmcnt<0>();
    raw_barrier();
    if (it + 1 < item1) issue(it + 1, buf ^ 1);
    const char* pt = smem + buf * SB;
    const char* yt = pt + P_BYTES;
    // one wave per SIMD: nothing else hides LDS latency, so the 13 fragments of K-block kb+1 are
    // read while the 36 MFMAs of kb run (register double buffer) instead of one tap at a time
    bf16x8 af[2][4], bt[2][9];
    auto load_frags = [&](int kb, bf16x8 (&a)[4], bf16x8 (&b)[9]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = wtr_frag(yt, kb * 32 + 8 * (lane >> 4), 16 * i, lane);
#pragma unroll
      for (int t = 0; t < 9; ++t) b[t] = wtr_frag(pt, prb[kb] + tap_dy(t) * PC + tap_dx(t), 16 * wid, lane, HI);
    };
    load_frags(0, af[0], bt[0]);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      if (kb + 1 < KB) load_frags(kb + 1, af[(kb + 1) & 1], bt[(kb + 1) & 1]);
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bt[kb & 1][t], af[kb & 1][i], acc[i][t], 0, 0, 0);
    }
  }
  // partial tile -> slab sl: lane owns dW[co0 + 16i + (lane&15)][t][ci0 + 16 wid + 4(lane>>4) .. +3]
  float* out = (float*)p.out + (long long)sl * p.slabStride;
  const int N = p.N;  // 9 * Cin
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + 16 * i + (lane & 15);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int n = (t << log2C) + ci0 + 16 * wid + 4 * (lane >> 4);
      *(f32x4*)(out + (long long)co * N + n) = acc[i][t];
    }
  }
}

}  // namespace

// kind: 0 conv-fwd, 1 conv-dgrad, 2 conv-wgrad, 3 dense (A·Bᵀ), 4 dense dX (A·B), 5 dense dW (Aᵀ·B),
//       6 fused nearest-upscale(2x) + conv3x3 forward (PG-GAN _upscale2d_conv2d)
// epi: 0 bf16 out, 1 fp32 out (split-K slabs when splits > 1)
// tile: 0 128x128, 1 128x64, 2 64x128, 3 64x64; | 16 = two K-tiles in flight (register ring)
extern "C" int rk_igemm(int kind, int epi, int tile, const void* A, const void* B, void* C,
                        const float* bias, float* stats, const void* gate, int M, int N, int K,
                        int lda, int ldb, int ldc, int H, int W, int Cch, int taps, int Cb,
                        int splits, long long slabStride, int flags, float alpha, float slope,
                        long long bytesA, long long bytesB, void* stream) {
  if (bytesA <= 0 || bytesB <= 0 || bytesA >= (1ll << 31) || bytesB >= (1ll << 31)) return RK_EUNSUPPORTED;
  if (M <= 0 || N <= 0 || K <= 0 || splits <= 0) return RK_EBADARG;
  // K-inner A operands (every kind but the two K-outer x K-outer reductions) need K % 8 == 0
  if (N % 4 != 0 || (kind != 2 && kind != 5 && K % 8 != 0)) return RK_EUNSUPPORTED;
  if (taps != 1 && taps != 9) return RK_EBADARG;
  IgemmParams p{};
  p.A = (const bf16*)A; p.B = (const bf16*)B; p.out = C; p.bias = bias; p.stats = stats;
  p.gate = (const bf16*)gate;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.H = H; p.W = W; p.C = Cch; p.taps = taps;
  p.log2H = rk_log2(H); p.log2W = rk_log2(W); p.log2C = rk_log2(Cch); p.log2Cb = rk_log2(Cb);
  p.P = M;
  const int kTiles = rk_cdiv(K, BK);
  p.ktPer = rk_cdiv(kTiles, splits);
  p.slabStride = slabStride;
  p.flags = flags; p.alpha = alpha; p.slope = slope;
  p.bytesA = (unsigned long long)bytesA; p.bytesB = (unsigned long long)bytesB;
  hipStream_t st = (hipStream_t)stream;
  const bool conv = kind <= 2 || kind == 6;
  p.invC = 1.0f / (float)Cch; p.invH = 1.0f / (float)H; p.invW = 1.0f / (float)W;
  if (conv && (Cch % 8 != 0 || Cch < 8 || H <= 0 || W <= 0)) return RK_EUNSUPPORTED;
  if (conv && (p.log2H < 0 || p.log2W < 0) && (long long)(kind == 2 ? K : M) + (long long)W * (H + 2) >= (1ll << 22))
    return RK_EUNSUPPORTED;  // reciprocal pixel decode is exact below 2^22
  // the LDS-DMA operands use shift-only index arithmetic: other extents run register-staged
  if (conv && (p.log2C < 0 || p.log2H < 0 || p.log2W < 0)) tile &= 15 | 16;
  if (epi == 0 && splits != 1) return RK_EBADARG;
  if ((flags & FLAG_BNP) && (epi != 0 || p.log2H < 0 || p.log2W < 0 || !gate || !bias || !(flags & FLAG_SATOM)))
    return RK_EUNSUPPORTED;
  switch (kind) {
    // conv forward / data-gradient with epi 1: split-K fp32 slabs for the small-M layers (4x4 / 8x8
    // VGG convs), combined by rk_slab_epi (bf16 out + BN statistics / BN-backward gate)
    case 0: return epi == 0 ? launch_modes<OP_CONV_KIN, OP_DENSE_KIN, EPI_BF16>(tile, p, splits, st)
                            : launch_modes<OP_CONV_KIN, OP_DENSE_KIN, EPI_F32>(tile, p, splits, st);
    case 1: if (p.log2Cb < 0) return RK_EUNSUPPORTED;
      return epi == 0 ? launch_modes<OP_CONVT_KIN, OP_WTAP_KOUT, EPI_BF16>(tile, p, splits, st)
                      : launch_modes<OP_CONVT_KIN, OP_WTAP_KOUT, EPI_F32>(tile, p, splits, st);
    case 2: if (epi != 1) return RK_EBADARG;
      return launch_modes<OP_DENSE_KOUT, OP_CONV_KOUT, EPI_F32>(tile, p, splits, st);
    case 3: return epi == 0 ? launch_modes<OP_DENSE_KIN, OP_DENSE_KIN, EPI_BF16>(tile, p, splits, st)
                            : launch_modes<OP_DENSE_KIN, OP_DENSE_KIN, EPI_F32>(tile, p, splits, st);
    case 4: return epi == 0 ? launch_modes<OP_DENSE_KIN, OP_DENSE_KOUT, EPI_BF16>(tile, p, splits, st)
                            : launch_modes<OP_DENSE_KIN, OP_DENSE_KOUT, EPI_F32>(tile, p, splits, st);
    case 5: if (epi != 1) return RK_EBADARG;
      return launch_modes<OP_DENSE_KOUT, OP_DENSE_KOUT, EPI_F32>(tile, p, splits, st);
    case 6: if (epi != 0 || (H & 1) || (W & 1)) return RK_EBADARG;  // H, W = OUTPUT (2x) resolution
      return launch_modes<OP_CONVUP_KIN, OP_DENSE_KIN, EPI_BF16>(tile & (15 | 16), p, splits, st);
  }
  return RK_EBADARG;
}

// Halo-tiled 3x3 conv (see hconv_kernel).  dgrad = 0: y = conv(x, w) with w [N][9][C] (ldb = 9C);
// dgrad = 1: dx = conv^T(dy, w) with w [C][9][N] (ldb = 9N), C = channels of the input (dy).
// tile bit 0: BN = 128 (else 64).  grid <= 0: one item per block; otherwise the persistent grid
// size (items are dealt in contiguous runs).  Returns RK_EUNSUPPORTED outside the covered shapes
// (W in {8,16,32}, H a power of two with H*W a multiple of BM, C a power of two >= 64, N % BN == 0).
extern "C" int rk_hconv(int dgrad, int tile, const void* A, const void* B, void* C, const float* bias, float* stats,
                        const void* gate, int M, int N, int K, int ldb, int H, int W, int Cch, int flags, float alpha,
                        float slope, long long bytesA, long long bytesB, int grid, void* stream) {
  if (bytesA <= 0 || bytesB <= 0 || bytesA >= (1ll << 31) || bytesB >= (1ll << 31)) return RK_EUNSUPPORTED;
  const int BN = (tile & 1) ? 128 : 64;
  const int BM = W == 8 ? 64 : 128;
  if (W != 4 && W != 8 && W != 16 && W != 32) return RK_EUNSUPPORTED;
  if (W == 4) {  // whole-image items: 8 images of 4x4
    if (H != 4 || M <= 0 || M % BM != 0) return RK_EUNSUPPORTED;
  } else if (rk_log2(H) < 0 || (H * W) % BM != 0 || M <= 0 || M % (H * W) != 0) {
    return RK_EUNSUPPORTED;
  }
  if (rk_log2(Cch) < 6 || N <= 0 || N % BN != 0 || K != 9 * Cch) return RK_EUNSUPPORTED;
  if (ldb != (dgrad ? 9 * N : K)) return RK_EBADARG;
  if ((flags & FLAG_BNP) && (!gate || !bias || !(flags & FLAG_SATOM))) return RK_EUNSUPPORTED;
  IgemmParams p{};
  p.A = (const bf16*)A; p.B = (const bf16*)B; p.out = C; p.bias = bias; p.stats = stats;
  p.gate = (const bf16*)gate;
  p.M = M; p.N = N; p.K = K; p.lda = Cch; p.ldb = ldb; p.ldc = N;
  p.H = H; p.W = W; p.C = Cch; p.taps = 9;
  p.log2H = rk_log2(H); p.log2W = rk_log2(W); p.log2C = rk_log2(Cch); p.log2Cb = p.log2C;
  p.flags = flags; p.alpha = alpha; p.slope = slope;
  p.bytesA = (unsigned long long)bytesA; p.bytesB = (unsigned long long)bytesB;
  hipStream_t st = (hipStream_t)stream;
  return BN == 128 ? launch_hconv_bn<128>(dgrad != 0, p, grid, st) : launch_hconv_bn<64>(dgrad != 0, p, grid, st);
}

// Halo-tiled 3x3 weight gradient (see hconv_wgrad_kernel) into fp32 slabs [S][Cout][9*Cin]:
// dy [pixels][Cout], x [pixels][Cin] (NHWC, pixels = Nb*H*W).  Every slab element is written
// (blocks of slab s cover all tiles); sum the slabs with rk_reduce_slabs.  S = blocks per tile.
extern "C" int rk_hconv_wgrad(const void* dy, const void* x, float* slab, int Nb, int H, int W, int Cin, int Cout,
                              int S, long long bytesY, long long bytesX, void* stream) {
  if (bytesY <= 0 || bytesX <= 0 || bytesY >= (1ll << 31) || bytesX >= (1ll << 31)) return RK_EUNSUPPORTED;
  if (W != 4 && W != 8 && W != 16 && W != 32) return RK_EUNSUPPORTED;
  const int P = W == 8 ? 64 : 128;
  if (W == 4) {  // whole-image items: 8 images of 4x4
    if (H != 4 || Nb <= 0 || (Nb * 16) % P != 0) return RK_EUNSUPPORTED;
  } else if (rk_log2(H) < 0 || (H * W) % P != 0 || Nb <= 0) {
    return RK_EUNSUPPORTED;
  }
  if (rk_log2(Cin) < 6 || Cout % 64 != 0 || S <= 0) return RK_EUNSUPPORTED;
  IgemmParams p{};
  p.A = (const bf16*)dy; p.B = (const bf16*)x; p.out = slab;
  p.M = Cout; p.N = 9 * Cin; p.K = Nb * H * W;
  p.H = H; p.W = W; p.C = Cin; p.taps = 9;
  p.log2H = rk_log2(H); p.log2W = rk_log2(W); p.log2C = rk_log2(Cin);
  p.slabStride = (long long)Cout * 9 * Cin;
  p.bytesA = (unsigned long long)bytesY; p.bytesB = (unsigned long long)bytesX;
  const int items = p.K / P;
  const int per = rk_cdiv(items, S);
  const int tiles = (Cout / 64) * (Cin / 64);
  // S is fixed (the caller sized the slab array); blocks past the last item write zero tiles
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(tiles * S);
  switch (W) {
    case 4: hipLaunchKernelGGL((hconv_wgrad_kernel<4>), grid, dim3(256), 0, st, p, S, per); break;
    case 8: hipLaunchKernelGGL((hconv_wgrad_kernel<8>), grid, dim3(256), 0, st, p, S, per); break;
    case 16: hipLaunchKernelGGL((hconv_wgrad_kernel<16>), grid, dim3(256), 0, st, p, S, per); break;
    default: hipLaunchKernelGGL((hconv_wgrad_kernel<32>), grid, dim3(256), 0, st, p, S, per); break;
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}
