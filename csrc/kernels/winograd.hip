// Winograd F(2x2, 3x3) fp32 convolution for gfx950: stride 1, pad 1, NHWC, even H and W, C % 8 == 0.
//
// A 3x3 conv needs 9 MACs per output pixel and channel pair; F(2x2,3x3) needs 16 per 2x2 output tile,
// i.e. 4 — 2.25x fewer v_mfma_f32_16x16x4_f32 cycles on exactly the same fp32 data type (all
// transforms are fp32 adds / halvings).  The whole transform-GEMM-transform chain is fused in one
// kernel, so the 4x larger transformed tensors never touch HBM:
//   * weights: U = G g G^T, [16][Cout][Cin] (channel-contiguous), transformed once per weight
//     update by rk_wino_weights, which also emits the flipped / transposed set of the data gradient
//     (dgrad = forward conv of dy with flip(w)^T, whose transform is a transpose of U with the
//     Winograd positions 0 <-> 3 swapped in both dimensions, since G J = P G);
//   * block tile = 64 output tiles (2x2 px each: 256 pixels) x 32 output channels on 4 waves (one
//     48 KiB LDS stage, two workgroups per CU) or x 64 channels on 8 waves (2-stage 128 KiB ring),
//     picked per layer by the autotuner; the K loop walks Cin in chunks of 8: every thread loads its
//     (tile, channel) 4x4 input windows (raw buffer loads at fixed offsets,
//     zeros outside the image via the buffer range check), applies B^T d B in registers and writes
//     the 16 transformed values to LDS, and 4 float4 of U; the next chunk's global loads are in
//     flight while the current chunk's MFMAs run; LDS column pairs are XOR-swizzled per row so
//     the 64-bit fragment reads are bank-conflict-free;
//   * wave (wm, wn) owns tiles 16 wm .. 16 wm + 15 and channels 32 wn .. 32 wn + 31 for ALL 16
//     Winograd positions (32 16x16 accumulators, 128 fp32 registers), so the output transform
//     A^T M A is lane-local — no cross-wave reduction — and each lane ends up holding whole 2x2
//     output tiles of one channel;
//   * K order inside a chunk is permuted (lane group q supplies channels 2q, 2q+1 over the two MFMA
//     steps) so A and B fragments are single ds_read_b64s of contiguous LDS;
//   * epilogues as in the direct kernels (csrc/kernels/sgemm.hip): bias, ReLU, BN statistics
//     (fp64 slot atomics), and for the data gradient FLAG_BNB / FLAG_BNP (ReLU mask + BN-backward
//     sums of the BN+ReLU(+2x2 max-pool) layer below).
#include <type_traits>
#include "common.h"

namespace {

#include "wino_wt.h"

constexpr int WT = 64;    // output tiles per block
constexpr int WKC = 8;    // input channels per K chunk
enum { WF_RELU = 1, WF_BIAS = 2, WF_STATS = 4, WF_BNB = 512, WF_BNP = 1024 };

typedef __attribute__((ext_vector_type(2))) float f32x2;

struct WgParams {
  const float* x;       // NHWC [Nb][H][W][C]
  const float* u;       // [16][N][C]
  float* y;             // NHWC [Nb][H][W][N]
  const float* bias;    // [N] bias; BNB / BNP: BN scale [N] then shift [N] of the gated layer
  double* stats;        // fp64 slots [slotMask+1][2][N]
  const float* gate;    // BNB: BN input y of the gated layer [Nb][H][W][N]; BNP: at [Nb][2H][2W][N]
  int Nb, H, W, C, N;
  int TW, THW, ntiles, ncb, slotMask, flags;
  unsigned long long xbytes, ubytes, ybytes;
  // grouped launches (the k models of a serving ensemble): group g of gridDim = groups x bpg blocks
  // reads x + g*gx (gx = 0: shared input), u + g*gu and writes y + g*gy, bias + g*gbias
  int bpg;
  long long gx, gu, gy, gbias;
};

constexpr unsigned WOOB = 0x80000000u;

// LDS rows hold 8 channels (4 column pairs); row r stores column pair c at c ^ ((r >> 2) & 3): the 16
// rows x one pair of a ds_read2st64_b64 lane group (banks mod 32) and the 16 rows x two pairs of a
// ds_read_b64 group (banks mod 64) then hit distinct banks
RK_DEV int w_swz(int row) { return ((row >> 2) & 3) << 1; }
// the weight gradient's column swizzle (winograd4.hip swzw: stores conflict-free under the (a/4) mod 32
// banking of ds_write2st64_b32, 16-row fragment reads under that of ds_read2st64_b64; row bit 4 swaps the
// two columns of a pair, undone in registers by the reading wave)
RK_DEV int w_swzw(int row) { return (((row >> 2) & 1) << 1) | (((row >> 3) & 1) << 2) | ((row >> 4) & 1); }

RK_DEV __amdgpu_buffer_rsrc_t w_rsrc(const float* base, unsigned long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)(unsigned)bytes, 0x00020000);
}

// tile t -> (image, 2x2 tile origin)
RK_DEV void w_tile(const WgParams& p, int t, int& n, int& oy, int& ox) {
  n = t / p.THW;
  const int r = t - n * p.THW;
  const int ty = r / p.TW;
  oy = 2 * ty;
  ox = 2 * (r - ty * p.TW);
}

// NWN = 1: 4 waves, 64 tiles x 32 channels, one 48 KiB LDS stage, two workgroups per CU (small
// grids, overlapping epilogues); NWN = 2: 8 waves, 64 x 64, a 2-stage 128 KiB ring (one barrier per
// chunk, V loaded once for 64 channels).  The autotuner picks per layer.
template <int NWN>
__global__ __launch_bounds__(256 * NWN, 3 - NWN) void wino_fwd_kernel(const WgParams p) {
  constexpr int NT = 256 * NWN;            // threads
  constexpr int BNC = 32 * NWN;            // output channels per block
  constexpr int NSTG = NWN == 2 ? 2 : 1;   // LDS stages
  constexpr int IT = 2 / NWN;              // input windows per thread and chunk
  __shared__ __attribute__((aligned(16))) float Vs[NSTG][16][WT][WKC];
  __shared__ __attribute__((aligned(16))) float Us[NSTG][16][BNC][WKC];
  const int tid = threadIdx.x, lane = tid & 63, wm = (tid >> 6) & 3, wn = tid >> 8;
  const int b0 = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = b0 / p.bpg, b = b0 - grp * p.bpg;
  const int cb = b % p.ncb, tb = b / p.ncb;
  const int tbase = tb * WT, cbase = cb * BNC;
  const float* const gxp = p.x + grp * p.gx;
  const float* const gup = p.u + grp * p.gu;
  float* const gyp = p.y + grp * p.gy;
  const float* const gbp = p.bias ? p.bias + grp * p.gbias : nullptr;

  // loader role per thread and chunk: the (tile, channel) 4x4 input windows of tiles lt + NT/8 * h
  // and 4 float4 of U, as raw buffer loads whose byte offsets are fixed for the whole K loop (the
  // chunk advances the descriptors' base in SGPRs); window pixels outside the image carry an
  // offset past the buffer -> zeros
  const int lt = tid >> 3, lc = tid & 7;
  // per window: byte offset of its centre pixel (1, 1) and a 16-bit in-image mask; pixel (a, bb)
  // sits at a wave-uniform delta from the centre
  unsigned vb[IT], vm[IT];
#pragma unroll
  for (int h = 0; h < IT; ++h) {
    int ln, loy, lox;
    w_tile(p, tbase + lt + NT / 8 * h, ln, loy, lox);
    const bool lok = tbase + lt + NT / 8 * h < p.ntiles;
    vb[h] = lok ? (unsigned)((((ln * p.H + loy) * p.W + lox) * p.C + lc) * 4) : 0u;
    vm[h] = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int yy = loy - 1 + a, xx = lox - 1 + bb;
        if (lok && yy >= 0 && yy < p.H && xx >= 0 && xx < p.W) vm[h] |= 1u << (a * 4 + bb);
      }
  }
  unsigned uo[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int f = tid + NT * k;             // float4 index in [16][BNC][2]
    const int pos = f / (2 * BNC), co = (f >> 1) & (BNC - 1), half = f & 1;
    uo[k] = cbase + co < p.N ? (unsigned)(((pos * p.N + cbase + co) * p.C + half * 4) * 4) : WOOB;
  }

  float raw[IT][16];
  f32x4 ur[4];
  auto load = [&](int c0) {
    const __amdgpu_buffer_rsrc_t xr = w_rsrc(gxp + c0, p.xbytes - 4ull * c0);
    const __amdgpu_buffer_rsrc_t urs = w_rsrc(gup + c0, p.ubytes - 4ull * c0);
#pragma unroll
    for (int h = 0; h < IT; ++h)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int d = (((i >> 2) - 1) * p.W + (i & 3) - 1) * p.C * 4;
        const unsigned off = ((vm[h] >> i) & 1u) ? vb[h] + (unsigned)d : WOOB;
        raw[h][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)off, 0, 0));
      }
#pragma unroll
    for (int k = 0; k < 4; ++k) ur[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(urs, (int)uo[k], 0, 0));
  };
  auto store = [&](int st) {
#pragma unroll
    for (int h = 0; h < IT; ++h) {
      const int row = lt + NT / 8 * h, c = lc ^ w_swz(row);
      float t[16];
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {     // B^T d: rows
        t[0 * 4 + bb] = raw[h][0 * 4 + bb] - raw[h][2 * 4 + bb];
        t[1 * 4 + bb] = raw[h][1 * 4 + bb] + raw[h][2 * 4 + bb];
        t[2 * 4 + bb] = raw[h][2 * 4 + bb] - raw[h][1 * 4 + bb];
        t[3 * 4 + bb] = raw[h][1 * 4 + bb] - raw[h][3 * 4 + bb];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {        // (B^T d) B: columns
        Vs[st][a * 4 + 0][row][c] = t[a * 4 + 0] - t[a * 4 + 2];
        Vs[st][a * 4 + 1][row][c] = t[a * 4 + 1] + t[a * 4 + 2];
        Vs[st][a * 4 + 2][row][c] = t[a * 4 + 2] - t[a * 4 + 1];
        Vs[st][a * 4 + 3][row][c] = t[a * 4 + 1] - t[a * 4 + 3];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int f = tid + NT * k, pos = f / (2 * BNC), co = (f >> 1) & (BNC - 1), c0 = (f & 1) * 4, sw = w_swz(co);
      *(f32x2*)&Us[st][pos][co][c0 ^ sw] = f32x2{ur[k][0], ur[k][1]};
      *(f32x2*)&Us[st][pos][co][(c0 + 2) ^ sw] = f32x2{ur[k][2], ur[k][3]};
    }
  };

  f32x4 acc[16][2];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q][0] = acc[q][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = p.C / WKC;
  load(0);
  store(0);
  __syncthreads();
  const int ar = wm * 16 + (lane & 15), br = wn * 32 + (lane & 15);
  const int ka = (2 * (lane >> 4)) ^ w_swz(ar), kb = (2 * (lane >> 4)) ^ w_swz(br);
  for (int c = 0; c < nch; ++c) {
    const int st = NSTG == 2 ? (c & 1) : 0;
    if (c + 1 < nch) load((c + 1) * WKC);
    // two positions at a time: 4 independent MFMAs between dependent ones (32-cycle issue, ~40 latency)
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      f32x2 a[2], bv[2][2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        a[e] = *(const f32x2*)&Vs[st][q + e][ar][ka];
        bv[e][0] = *(const f32x2*)&Us[st][q + e][br][kb];
        bv[e][1] = *(const f32x2*)&Us[st][q + e][br + 16][kb];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int nb = 0; nb < 2; ++nb)
            acc[q + e][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e][s], bv[e][nb][s], acc[q + e][nb], 0, 0, 0);
    }
    if constexpr (NSTG == 2) {             // the other stage is free: one barrier per chunk
      if (c + 1 < nch) store(st ^ 1);
    } else if (c + 1 < nch) {              // one stage: wait for every wave's reads first
      __syncthreads();
      store(0);
    }
    __syncthreads();
  }

  // ---- output transform + epilogue: lane owns channels n0, n0 + 16 of 4 consecutive tiles; 32-bit
  // element indices (the host checks the sizes), one tile decode per lane
  const int fl = p.flags;
  const bool sums = fl & (WF_STATS | WF_BNB | WF_BNP);
  int nn[2];
  bool nok[2];
  float bs[2], sh[2], s[2], ss[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    nn[nb] = cbase + wn * 32 + nb * 16 + (lane & 15);
    nok[nb] = nn[nb] < p.N;
    bs[nb] = ((fl & (WF_BIAS | WF_BNB | WF_BNP)) && nok[nb]) ? gbp[nn[nb]] : 0.f;
    sh[nb] = ((fl & (WF_BNB | WF_BNP)) && nok[nb]) ? gbp[p.N + nn[nb]] : 0.f;
    s[nb] = ss[nb] = 0.f;
  }
  const int t0 = tbase + wm * 16 + (lane >> 4) * 4;
  int im, oy, ox;
  w_tile(p, t0, im, oy, ox);
  const __amdgpu_buffer_rsrc_t yr = w_rsrc(gyp, p.ybytes);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool tok = t0 + r < p.ntiles;
    const int pix = (im * p.H + oy) * p.W + ox;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      float tt[4][2];
#pragma unroll
      for (int a = 0; a < 4; ++a) {        // M A: columns
        const f32x4 m0 = acc[a * 4 + 0][nb], m1 = acc[a * 4 + 1][nb], m2 = acc[a * 4 + 2][nb], m3 = acc[a * 4 + 3][nb];
        tt[a][0] = m0[r] + m1[r] + m2[r];
        tt[a][1] = m1[r] - m2[r] - m3[r];
      }
      if (!(tok && nok[nb])) continue;
      const int n = nn[nb];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          // A^T (M A): rows
          float v = i == 0 ? tt[0][j] + tt[1][j] + tt[2][j] : tt[1][j] - tt[2][j] - tt[3][j];
          const int idx = (pix + i * p.W + j) * p.N + n;
          if (fl & WF_BIAS) v += bs[nb];
          if (fl & WF_STATS) {
            s[nb] += v;
            ss[nb] += v * v;
          }
          if (fl & WF_RELU) v = fmaxf(v, 0.f);
          if (fl & WF_BNB) {
            const float g = p.gate[idx];
            v = g * bs[nb] + sh[nb] > 0.f ? v : 0.f;
            s[nb] += v;
            ss[nb] += v * g;
          }
          if (fl & WF_BNP) {
            // pooled pixel (im, oy+i, ox+j) of an H x W map; its 2x2 window sits at 2H x 2W
            const int W2 = 2 * p.W;
            const int b0 = ((im * 2 * p.H + 2 * (oy + i)) * W2 + 2 * (ox + j)) * p.N + n;
            const float y4[4] = {p.gate[b0], p.gate[b0 + p.N], p.gate[b0 + W2 * p.N], p.gate[b0 + W2 * p.N + p.N]};
            float best = -INFINITY, zb = 0.f, yb = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {  // first maximal relu(z) of the window (torch max_pool2d rule)
              const float z = y4[e] * bs[nb] + sh[nb];
              const float av = fmaxf(z, 0.f);
              if (av > best) { best = av; zb = z; yb = y4[e]; }
            }
            const float dz = zb > 0.f ? v : 0.f;
            s[nb] += dz;
            ss[nb] += dz * yb;
          }
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), yr, idx * 4, 0, 0);
        }
    }
    ox += 2;                               // next tile: (im, oy, ox) in row-major tile order
    if (ox >= p.W) {
      ox = 0;
      oy += 2;
      if (oy >= p.H) {
        oy = 0;
        ++im;
      }
    }
  }
  if (sums) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      float a = s[nb], b2 = ss[nb];
      a += __shfl_xor(a, 16, 64);
      b2 += __shfl_xor(b2, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b2 += __shfl_xor(b2, 32, 64);
      if (nok[nb] && lane < 32) {
        double* slot = p.stats + (long long)(blockIdx.x & p.slotMask) * 2 * p.N;
        unsafeAtomicAdd(slot + (lane >= 16 ? p.N : 0) + nn[nb], (double)(lane >= 16 ? b2 : a));
      }
    }
  }
}

// ------------------------------------------------------------------------- weight gradient
// dW = sum over 2x2 output tiles of G^T [ (A dY A^T) (.) (B^T d B) ] G: per Winograd position a GEMM
// dU[pos][co][ci] = sum_t Mdy[pos][t][co] * V[pos][t][ci] with the reduction over tiles, 2.25x fewer
// MFMA cycles than the direct weight gradient.  Block = 8 waves, 64 co x 64 ci x 16 positions
// (wave (wm, wn): 16 co x 32 ci); the tile range is split over gridDim (split-K) and each block
// applies G^T . G in registers, so it writes plain dW taps [Co][9][Ci] (slab per split, summed by
// rk_reduce_slabs).  Every thread transforms one (tile, co) 2x2 output-gradient patch and one
// (tile, ci) 4x4 input window per chunk of 8 tiles.
struct WwParams {
  const float* dy;      // NHWC [Nb][H][W][Co]
  const float* x;       // NHWC [Nb][H][W][Ci]
  float* out;           // [splits][Co][9][Ci]
  int Nb, H, W, Co, Ci;
  int TW, THW, ntiles, tps, nco, nci, accumulate;
  float invTW, invTHW;
  unsigned long long dybytes, xbytes;
  long long slab;       // floats per split
};

__global__ __launch_bounds__(512, 1) void wino_wgrad_kernel(const WwParams p) {
  __shared__ __attribute__((aligned(16))) float Ms[2][16][64][WKC];   // [stage][pos][co][tile]
  __shared__ __attribute__((aligned(16))) float Vs[2][16][64][WKC];   // [stage][pos][ci][tile]
  const int tid = threadIdx.x, lane = tid & 63, wm = (tid >> 6) & 3, wn = tid >> 8;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int per = p.nco * p.nci;
  const int split = b / per, r0 = b - split * per;
  const int co0 = (r0 / p.nci) * 64, ci0 = (r0 % p.nci) * 64;
  const int t_begin = split * p.tps;
  const int t_end = min(t_begin + p.tps, p.ntiles);
  const int nch = (t_end - t_begin + WKC - 1) / WKC;
  // tile within the chunk, channel within the block: a wave covers 2 tiles x 32 consecutive channels, so
  // each buffer load moves two whole 128-B lines (the F(4x4) weight gradient measured 1.19-1.29x from the
  // same remap, profiles/wino4_wgrad_remap_r5.jsonl); LDS stores conflict-free under w_swzw
  const int tt = (tid >> 5) & 7, ch = (tid & 31) + 32 * (tid >> 8);
  const bool cok = co0 + ch < p.Co, iok = ci0 + ch < p.Ci;
  const __amdgpu_buffer_rsrc_t dyr = w_rsrc(p.dy, p.dybytes), xr = w_rsrc(p.x, p.xbytes);

  float gy[4], raw[16];
  auto load = [&](int c) {
    const int t = t_begin + c * WKC + tt;
    // branch-free validity: (tile in range) x (channel in range) x (window row / column in image)
    const unsigned okm = (t < t_end ? 1u : 0u);
    // tile -> (n, oy, ox) by fp32 reciprocals (exact below 2^22 tiles)
    const int n = (int)(((float)t + 0.5f) * p.invTHW);
    const int rr = t - n * p.THW;
    const int ty = (int)(((float)rr + 0.5f) * p.invTW);
    const int oy = 2 * ty, ox = 2 * (rr - ty * p.TW);
    const int pix = (n * p.H + oy) * p.W + ox;
    const unsigned gm = okm & (cok ? 1u : 0u);
    const unsigned ob = (unsigned)((pix * p.Co + co0 + ch) * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // invalid -> bit 31 set: past any buffer (a select here makes hipcc branch around the loads)
      const unsigned off = (ob + (unsigned)((((i >> 1) * p.W) + (i & 1)) * p.Co * 4)) | ((gm ^ 1u) << 31);
      gy[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dyr, (int)off, 0, 0));
    }
    // rows / columns 1, 2 of a window are always inside an even-sized map; 0 and 3 at the borders
    const unsigned xm = okm & (iok ? 1u : 0u);
    const unsigned rm = (xm * 6u) | ((oy > 0 ? xm : 0u) << 0) | ((oy + 2 < p.H ? xm : 0u) << 3);
    const unsigned cm = 6u | ((ox > 0 ? 1u : 0u) << 0) | ((ox + 2 < p.W ? 1u : 0u) << 3);
    const unsigned xb = (unsigned)((pix * p.Ci + ci0 + ch) * 4);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int a = i >> 2, bb = i & 3;
      const unsigned in = (rm >> a) & (cm >> bb) & 1u;
      const unsigned off = (xb + (unsigned)((((a - 1) * p.W) + bb - 1) * p.Ci * 4)) | ((in ^ 1u) << 31);
      raw[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)off, 0, 0));
    }
  };
  auto store = [&](int st) {
    const int c = tt ^ w_swzw(ch);
    // A dY A^T (4x4 from 2x2): rows (y0, y0 + y1, y0 - y1, -y1), then the same on columns
    float rw[4][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      rw[0][j] = gy[j];
      rw[1][j] = gy[j] + gy[2 + j];
      rw[2][j] = gy[j] - gy[2 + j];
      rw[3][j] = -gy[2 + j];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      Ms[st][a * 4 + 0][ch][c] = rw[a][0];
      Ms[st][a * 4 + 1][ch][c] = rw[a][0] + rw[a][1];
      Ms[st][a * 4 + 2][ch][c] = rw[a][0] - rw[a][1];
      Ms[st][a * 4 + 3][ch][c] = -rw[a][1];
    }
    float t[16];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {       // B^T d: rows
      t[0 * 4 + bb] = raw[0 * 4 + bb] - raw[2 * 4 + bb];
      t[1 * 4 + bb] = raw[1 * 4 + bb] + raw[2 * 4 + bb];
      t[2 * 4 + bb] = raw[2 * 4 + bb] - raw[1 * 4 + bb];
      t[3 * 4 + bb] = raw[1 * 4 + bb] - raw[3 * 4 + bb];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {          // (B^T d) B: columns
      Vs[st][a * 4 + 0][ch][c] = t[a * 4 + 0] - t[a * 4 + 2];
      Vs[st][a * 4 + 1][ch][c] = t[a * 4 + 1] + t[a * 4 + 2];
      Vs[st][a * 4 + 2][ch][c] = t[a * 4 + 2] - t[a * 4 + 1];
      Vs[st][a * 4 + 3][ch][c] = t[a * 4 + 1] - t[a * 4 + 3];
    }
  };

  f32x4 acc[16][2];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q][0] = acc[q][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nch > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  const int ar = wm * 16 + (lane & 15), br = wn * 32 + (lane & 15);
  const int ka = (2 * (lane >> 4)) ^ (w_swzw(ar) & 6), kb = (2 * (lane >> 4)) ^ (w_swzw(br) & 6);
  const int kb16 = (2 * (lane >> 4)) ^ (w_swzw(br + 16) & 6);
  // pair swap of the B fragment relative to A: row bit 4 of ar is wm's (wave-uniform), of br / br + 16 it is
  // 0 / 1, so the rows br swap when wm is odd and the rows br + 16 when it is even
  const bool swodd = (wm & 1) != 0;
  auto mfma = [&](int st, auto swc) __attribute__((always_inline)) {
    constexpr int SWO = decltype(swc)::value;   // rows br (nb 0) swap iff SWO, rows br + 16 iff !SWO
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
      f32x2 a[2], bv[2][2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        a[e] = *(const f32x2*)&Ms[st][q + e][ar][ka];
        bv[e][0] = *(const f32x2*)&Vs[st][q + e][br][kb];
        bv[e][1] = *(const f32x2*)&Vs[st][q + e][br + 16][kb16];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int nb = 0; nb < 2; ++nb)
            acc[q + e][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e][s], bv[e][nb][s ^ nb ^ SWO], acc[q + e][nb],
                                                                0, 0, 0);
    }
  };
  auto chunks = [&](auto swc) __attribute__((always_inline)) {   // per SWO, chosen once per wave
    for (int c = 0; c < nch; ++c) {
      const int st = c & 1;
      if (c + 1 < nch) load(c + 1);
      mfma(st, swc);
      if (c + 1 < nch) store(st ^ 1);
      __syncthreads();
    }
  };
  if (swodd)
    chunks(std::integral_constant<int, 1>{});
  else
    chunks(std::integral_constant<int, 0>{});

  // G^T dU G per (co, ci) in registers -> the 9 taps
  float* outp = p.out + (long long)split * p.slab;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int ci = ci0 + wn * 32 + nb * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + wm * 16 + (lane >> 4) * 4 + r;
      float tq[3][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {        // rows: G^T X
        const float x0 = acc[0 * 4 + q][nb][r], x1 = acc[1 * 4 + q][nb][r];
        const float x2 = acc[2 * 4 + q][nb][r], x3 = acc[3 * 4 + q][nb][r];
        tq[0][q] = x0 + 0.5f * (x1 + x2);
        tq[1][q] = 0.5f * (x1 - x2);
        tq[2][q] = 0.5f * (x1 + x2) + x3;
      }
      if (co >= p.Co || ci >= p.Ci) continue;
      float* o = outp + (long long)co * 9 * p.Ci + ci;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {     // columns: (G^T X) G
        float v[3];
        v[0] = tq[ky][0] + 0.5f * (tq[ky][1] + tq[ky][2]);
        v[1] = 0.5f * (tq[ky][1] - tq[ky][2]);
        v[2] = 0.5f * (tq[ky][1] + tq[ky][2]) + tq[ky][3];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          float* d = o + (ky * 3 + kx) * p.Ci;
          *d = p.accumulate ? *d + v[kx] : v[kx];
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void wino_wt_kernel(const float* __restrict__ w, float* __restrict__ u,
                                                      float* __restrict__ ut, int Co, int Ci) {
  __shared__ float g[32][9][33];
  wt_block(w, u, ut, Co, Ci, blockIdx.y * 32, blockIdx.x * 32, g);
}

// every layer of a network in one launch: desc[block] = (layer, co0, ci0, -); meta[layer] = (weight
// offset in the arena, u offset or -1, ut offset or -1, Co, Ci) in floats
__global__ __launch_bounds__(256) void wino_wt_multi_kernel(const float* __restrict__ arena, float* __restrict__ dst,
                                                            const int4* __restrict__ desc,
                                                            const long long* __restrict__ meta) {
  __shared__ float g[32][9][33];
  const int4 d = desc[blockIdx.x];
  const long long* m = meta + 5 * d.x;
  wt_block(arena + m[0], m[1] >= 0 ? dst + m[1] : nullptr, m[2] >= 0 ? dst + m[2] : nullptr, (int)m[3], (int)m[4],
           d.y, d.z, g);
}

}  // namespace

// dW [Co][9][Ci] (splits == 1, optionally accumulated) or per-split slabs [splits][Co][9][Ci] of the
// weight gradient of a 3x3 stride-1 pad-1 conv, by F(2x2,3x3); tiles_per_split % 8 == 0
extern "C" int rk_wino_wgrad(const float* dy, const float* x, float* out, int Nb, int H, int W, int Co, int Ci,
                             int splits, int accumulate, void* stream) {
  if (Nb <= 0 || H <= 0 || W <= 0 || (H & 1) || (W & 1) || Co <= 0 || Ci <= 0 || splits <= 0) return RK_EBADARG;
  if (splits > 1 && accumulate) return RK_EBADARG;
  WwParams p;
  p.dy = dy; p.x = x; p.out = out;
  p.Nb = Nb; p.H = H; p.W = W; p.Co = Co; p.Ci = Ci;
  p.TW = W / 2;
  p.THW = (H / 2) * (W / 2);
  const long long nt = (long long)Nb * p.THW;
  if (nt >= (1LL << 22)) return RK_EUNSUPPORTED;    // fp32-reciprocal tile decode
  p.ntiles = (int)nt;
  p.tps = ((p.ntiles + splits - 1) / splits + WKC - 1) / WKC * WKC;
  p.nco = rk_cdiv(Co, 64);
  p.nci = rk_cdiv(Ci, 64);
  p.accumulate = accumulate;
  p.invTW = 1.0f / (float)p.TW;
  p.invTHW = 1.0f / (float)p.THW;
  p.dybytes = 4ull * Nb * H * W * Co;
  p.xbytes = 4ull * Nb * H * W * Ci;
  if (p.dybytes >= 0x7fffffffull || p.xbytes >= 0x7fffffffull) return RK_EUNSUPPORTED;
  p.slab = 9LL * Co * Ci;
  const int used = rk_cdiv(p.ntiles, p.tps);        // splits that own tiles (the rest would be empty)
  if (used != splits) return RK_EBADARG;
  const long long blocks = (long long)splits * p.nco * p.nci;
  hipLaunchKernelGGL(wino_wgrad_kernel, dim3((unsigned)blocks), dim3(512), 0, (hipStream_t)stream, p);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// Winograd-domain weights of a 3x3 conv w [Co][9][Ci]: u (nullable) [16][Co][Ci], ut (nullable) [16][Ci][Co]
extern "C" int rk_wino_weights(const float* w, float* u, float* ut, int Co, int Ci, void* stream) {
  if (Co <= 0 || Ci <= 0 || (!u && !ut)) return RK_EBADARG;
  const dim3 grid(rk_cdiv(Ci, 32), rk_cdiv(Co, 32));
  hipLaunchKernelGGL(wino_wt_kernel, grid, dim3(256), 0, (hipStream_t)stream, w, u, ut, Co, Ci);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wino_weights_multi(const float* arena, float* dst, const int* desc, int nblocks, const long long* meta,
                                     void* stream) {
  if (nblocks <= 0) return RK_OK;
  hipLaunchKernelGGL(wino_wt_multi_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, arena, dst,
                     (const int4*)desc, meta);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// y = conv3x3(x, w) via F(2x2,3x3) with u = rk_wino_weights(w); flags WF_* (BNB/BNP: ``gate`` and the
// scale/shift pair in ``bias``; BNP: H x W is the pooled map and gate is at 2H x 2W).  groups > 1:
// k independent convs in one grid (x / u / y / bias strided by gx / gu / gy / gbias floats; gx = 0
// shares x), plain or bias / ReLU epilogues only.
extern "C" int rk_wino_conv_grp(const float* x, const float* u, float* y, const float* bias, double* stats,
                                int slotMask, const float* gate, int Nb, int H, int W, int C, int N, int flags,
                                int variant, int groups, long long gx, long long gu, long long gy, long long gbias,
                                void* stream) {
  if (variant != 0 && variant != 1) return RK_EBADARG;
  if (flags & 2048) return RK_EUNSUPPORTED;   // WF_POOL: the winograd4.hip launcher's pooled epilogue only
  const int BNC = variant ? 64 : 32;
  if (Nb <= 0 || (H & 1) || (W & 1) || H <= 0 || W <= 0 || C <= 0 || (C % WKC) || N <= 0 || groups <= 0)
    return RK_EBADARG;
  if ((flags & (WF_STATS | WF_BNB | WF_BNP)) && !stats) return RK_EBADARG;
  if ((flags & (WF_BNB | WF_BNP)) && (!gate || !bias)) return RK_EBADARG;
  if ((flags & WF_BIAS) && !bias) return RK_EBADARG;
  if (groups > 1 && (flags & (WF_STATS | WF_BNB | WF_BNP))) return RK_EUNSUPPORTED;
  WgParams p;
  p.x = x; p.u = u; p.y = y; p.bias = bias; p.stats = stats; p.gate = gate;
  p.Nb = Nb; p.H = H; p.W = W; p.C = C; p.N = N;
  p.TW = W / 2;
  p.THW = (H / 2) * (W / 2);
  const long long nt = (long long)Nb * p.THW;
  if (nt >= (1LL << 30)) return RK_EBADARG;
  p.ntiles = (int)nt;
  p.ncb = rk_cdiv(N, BNC);
  // raw-buffer byte offsets are 32-bit with 0x80000000 as the out-of-range marker
  p.xbytes = 4ull * Nb * H * W * C;
  p.ubytes = 64ull * N * C;
  p.ybytes = 4ull * Nb * H * W * N;
  const unsigned long long gbytes = (flags & WF_BNP) ? 4 * p.ybytes : p.ybytes;
  if (p.xbytes >= 0x7fffffffull || p.ubytes >= 0x7fffffffull || gbytes >= 0x7fffffffull) return RK_EUNSUPPORTED;
  p.slotMask = slotMask;
  p.flags = flags;
  p.gx = gx; p.gu = gu; p.gy = gy; p.gbias = gbias;
  const long long bpg = (long long)rk_cdiv(p.ntiles, WT) * p.ncb;
  const long long blocks = bpg * groups;
  if (blocks >= (1LL << 31)) return RK_EBADARG;
  p.bpg = (int)bpg;
  if (variant)
    hipLaunchKernelGGL(wino_fwd_kernel<2>, dim3((unsigned)blocks), dim3(512), 0, (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL(wino_fwd_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wino_conv(const float* x, const float* u, float* y, const float* bias, double* stats, int slotMask,
                            const float* gate, int Nb, int H, int W, int C, int N, int flags, int variant,
                            void* stream) {
  return rk_wino_conv_grp(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, variant, 1, 0, 0, 0, 0,
                          stream);
}
