// Winograd F(4x4, 3x3) fp32 convolution for gfx950: stride 1, pad 1, NHWC, H and W multiples of 4,
// C % 8 == 0.
//
// F(4x4,3x3) multiplies 36 transformed values per 4x4 output tile: 2.25 MACs per output pixel and
// channel pair against 9 for the direct conv and 4 for F(2x2,3x3) (csrc/kernels/winograd.hip), so
// 1.78x fewer v_mfma_f32_16x16x4_f32 cycles than the F(2x2) kernel on the same fp32 data; the 6x6
// input windows overlap less (2.25 loads per output against 4).  The transforms use the
// interpolation points 0, +-1, +-2 (Lavin & Gray): B^T d B, G g G^T and A^T M A, all fp32; their
// larger coefficients cost about one decimal digit of accuracy against F(2x2) (measured in
// profiles/winograd_error_r2.jsonl, still at fp32 round-off scale).
//
//   * weights: U = G g G^T [36][Cout][Cin] for the forward conv and, for the data gradient (a forward
//     conv of dy with the flipped, transposed filters), UT = G flip(g) G^T [36][Cin][Cout] — computed
//     directly (the F(2x2) position-swap identity has no F(4x4) counterpart: G J is not a row
//     permutation of G), all layers of a network in one launch;
//   * block tile = 16 WM tiles (4x4 px each) x 16 WN output channels on WM x WN waves; each wave owns
//     16 tiles x 16 channels for ALL 36 positions (36 16x16 accumulators, 144 fp32 registers), so the
//     output transform is lane-local and every lane ends up with whole 4x4 output tiles of one
//     channel; per position one 64-bit A read and one 64-bit B read feed two MFMAs;
//   * K loop over Cin in chunks of 8 channels through one LDS stage: every thread loads the 6x6 window
//     of one (tile, channel) (raw buffer loads at fixed offsets, zeros outside the image via an
//     out-of-range offset), transforms it in registers and writes 36 values; the next chunk's global
//     loads are in flight while the current chunk's MFMAs run; XOR-swizzled column pairs keep the
//     fragment reads bank-conflict-free (the same layout as the F(2x2) kernel);
//   * epilogues identical to the F(2x2) kernel: bias, ReLU, BN statistics (fp64 slot atomics) and
//     the data-gradient FLAG_BNB / FLAG_BNP fusions; grouped launches for the serving ensemble;
//   * blocked weights (UB): the per-step weight transform can also write U as the byte image of the
//     kernel's LDS stage, one contiguous [36][32 co][8 ci] block (36 KiB, column swizzle applied) per
//     (32-channel output block, 8-channel input chunk).  The weight loads then move 16 B per lane and
//     1 KiB per wave-instruction over whole cache lines, instead of 8 B per lane scattered over a
//     32-B segment of each (position, channel) row — those loads cost about as much time as the
//     MFMAs on the 32x32 layers (profiles/wino4_load_breakdown_r5.jsonl).
#include <type_traits>
#include "common.h"
#include <cstdlib>

namespace {

#include "wino_wt.h"

constexpr int KC = 8;     // input channels per K chunk
enum { WF_RELU = 1, WF_BIAS = 2, WF_STATS = 4, WF_LRELU = 8, WF_BNB = 512, WF_BNP = 1024, WF_POOL = 2048 };
// WF_POOL (fused forward, with exactly WF_BIAS | WF_RELU): the 2x2 max-pool of relu(conv + bias) written
// from the epilogue, y [Nb, H/2, W/2, N] — the serving network's pooled blocks with their eval BN folded
// into the weights / bias (each 2x2 window lies inside one output tile)
constexpr int WF_POOLED = WF_BIAS | WF_RELU | WF_POOL;

typedef __attribute__((ext_vector_type(2))) float f32x2;

struct W4Params {
  const float* x;       // NHWC [Nb][H][W][C]
  const float* u;       // [36][N][C]
  float* y;             // NHWC [Nb][H][W][N]
  const float* bias;    // [N] bias; BNB / BNP: BN scale [N] then shift [N] of the gated layer
  double* stats;        // fp64 slots [slotMask+1][2][N]
  const float* gate;    // BNB: BN input of the gated layer [Nb][H][W][N]; BNP: at [Nb][2H][2W][N]
  int Nb, H, W, C, N;
  int TW, THW, ntiles, ncb, slotMask, flags;
  unsigned long long xbytes, ubytes, ybytes;
  int bpg;
  long long gx, gu, gy, gbias;
  // normalise-on-load: the input is the pre-BN output y of the previous conv; scale [C] then shift [C] of its
  // BatchNorm, applied with the ReLU to every in-image element as it is loaded (null: x is used as is)
  const float* pro;
};

constexpr unsigned OOB = 0x80000000u;
constexpr int W4_PRO_MAXC = 512;   // normalise-on-load: input channels whose BN coefficients are staged in LDS

RK_DEV int swz(int row) { return ((row >> 2) & 3) << 1; }
// the weight-gradient kernels' column swizzle (tile column t of channel row r is stored at t ^ swzw(r)).
// The compiler pairs the stores into ds_write2st64_b32 and the fragment reads into ds_read2st64_b64, both
// banked (a/4) mod 32 (MI355X_MICROARCH.md §LDS): a store wave-half writes 32 consecutive rows of one
// tile, so the 8 rows of a bank group (equal r mod 4) need 8 different columns -> swzw is a bijection of
// row bits 2-4; a 16-lane read group takes 16 consecutive rows x one column pair, so the 4 rows of a bank
// group need 4 different pairs -> bits 2 and 3 land on the pair bits (2, 4).  Bit 4 lands on bit 0: it
// swaps the two columns of a pair, which is uniform over a wave's 16-row fragment (rows w*16 + 0..15), so a
// wave whose A and B fragments differ in it swaps its B pair in registers (wswap).  Round 5's swz (bits
// 2-3) left the stores 2-way (21.8 % of the LDS cycles, profiles/vgg_small_f32_step_pmc_r5.txt); a swizzle
// on bits 3-4 priced for 64 banks made both 2-way (49.5 %, the first round-6 build).
RK_DEV int swzw(int row) { return (((row >> 2) & 1) << 1) | (((row >> 3) & 1) << 2) | ((row >> 4) & 1); }
// the pair-aligned column offset of a fragment read of row r (the pair-swap bit dropped)
RK_DEV int swzp(int row) { return swzw(row) & 6; }

RK_DEV __amdgpu_buffer_rsrc_t rsrc(const float* base, unsigned long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)(unsigned)bytes, 0x00020000);
}

// B^T d of a 6-vector (interpolation points 0, 1, -1, 2, -2, inf)
RK_DEV void bt6(float d0, float d1, float d2, float d3, float d4, float d5, float (&t)[6]) {
  t[0] = 4.f * d0 - 5.f * d2 + d4;
  t[1] = d3 + d4 - 4.f * (d1 + d2);
  t[2] = d4 - d3 + 4.f * (d1 - d2);
  t[3] = d4 - d2 + 2.f * (d3 - d1);
  t[4] = d4 - d2 - 2.f * (d3 - d1);
  t[5] = 4.f * d1 - 5.f * d3 + d5;
}

// A^T m of a 6-vector -> 4 outputs
RK_DEV void at6(float m0, float m1, float m2, float m3, float m4, float m5, float (&o)[4]) {
  const float s12 = m1 + m2, d12 = m1 - m2, s34 = m3 + m4, d34 = m3 - m4;
  o[0] = m0 + s12 + s34;
  o[1] = d12 + 2.f * d34;
  o[2] = s12 + 4.f * s34;
  o[3] = d12 + 8.f * d34 + m5;
}

// F(2x2,3x3) counterparts (interpolation points 0, 1, -1, inf): B^T d of a 4-vector, A^T m -> 2 outputs
RK_DEV void bt4(float d0, float d1, float d2, float d3, float (&t)[4]) {
  t[0] = d0 - d2;
  t[1] = d1 + d2;
  t[2] = d2 - d1;
  t[3] = d1 - d3;
}
RK_DEV void at4(float m0, float m1, float m2, float m3, float (&o)[2]) {
  o[0] = m0 + m1 + m2;
  o[1] = m1 - m2 - m3;
}

// B^T / A^T of one window line (A = MO + 2 values, stride-strided in r) for output tile size MO
template <int MO>
RK_DEV void bt_line(const float* r, int stride, float (&o)[MO + 2]) {
  if constexpr (MO == 4)
    bt6(r[0], r[stride], r[2 * stride], r[3 * stride], r[4 * stride], r[5 * stride], o);
  else
    bt4(r[0], r[stride], r[2 * stride], r[3 * stride], o);
}
template <int MO>
RK_DEV void at_line(const float (&m)[MO + 2], float (&o)[MO]) {
  if constexpr (MO == 4)
    at6(m[0], m[1], m[2], m[3], m[4], m[5], o);
  else
    at4(m[0], m[1], m[2], m[3], o);
}

template <int MO>
RK_DEV void w_tile_of(const W4Params& p, int t, int& n, int& oy, int& ox) {
  n = t / p.THW;
  const int r = t - n * p.THW;
  const int ty = r / p.TW;
  oy = MO * ty;
  ox = MO * (r - ty * p.TW);
}
RK_DEV void w4_tile(const W4Params& p, int t, int& n, int& oy, int& ox) { w_tile_of<4>(p, t, n, oy, ox); }

// MO = 4: F(4x4,3x3), u [36][N][C]; MO = 2: F(2x2,3x3) on the same small-wave-tile layout (16 tiles x 16
// channels per wave, 16 accumulators), u [16][N][C] — the variant for small grids (deep 8x8 / 4x4 maps)
// FL >= 0: the epilogue flags as a compile-time constant (branch-free per-element epilogue for the
// combinations the engine uses); FL = -1 reads p.flags
// NS = 2: two LDS stages and two register sets — the transform of chunk c+1 (loaded during chunk c-1)
// is written to one stage while the MFMAs of chunk c read the other, in the same wave (software
// pipelining; one barrier per chunk; chunks past Cin load zeros, so the body is branch-free)
// WS: warp-specialised — WM x WN compute waves (MFMAs + epilogue) and as many loader waves (global loads,
// input transform, LDS writes) over two LDS stages: the loaders fill chunk c+1 while the compute waves run
// chunk c, one barrier per chunk; every SIMD holds one wave of each role, so the transform's VALU and the
// loads issue beside the other wave's MFMAs instead of in a phase of their own (NS = 2, blocked weights)
// PRO: normalise-on-load (p.pro = the producer's BN scale / shift; compile-time, so the kernels without it
// keep their register allocation)
template <int MO, int WM, int WN, int MINW, int FL, int NS = 1, bool UB = false, bool WS = false, bool PRO = false>
__global__ __launch_bounds__(64 * WM * WN * (WS ? 2 : 1), MINW) void wino_gfwd_kernel(const W4Params p) {
  constexpr int A = MO + 2;                // window / transformed tile side
  constexpr int P = A * A;                 // Winograd positions
  constexpr int NT = 64 * WM * WN;         // threads of one role (WS: compute and loader waves each)
  constexpr int T = 16 * WM;               // tiles per block
  constexpr int BNC = 16 * WN;             // output channels per block
  constexpr int IT = T * KC / NT;          // input windows per thread and chunk
  constexpr int UL = P * BNC * 4 / NT;    // f32x2 weight loads per thread and chunk
  // UB: 16-B units of one blocked weight chunk, per thread (the last round masked when NT does not divide)
  constexpr int UNITS = P * BNC * KC / 4;
  constexpr int UBL = (UNITS + NT - 1) / NT;
  constexpr int ULR = UB ? 1 : UL, UBR = UB ? UBL : 1;   // register arrays of the two weight paths
  static_assert(IT >= 1 && IT * NT == T * KC && UL * NT == P * BNC * 4, "tile shape");
  static_assert(!UB || (MO == 4 && BNC == 32), "blocked weights: F(4x4), 32-channel output blocks");
  static_assert(!WS || (NS == 2 && UB), "warp-specialised: two stages, blocked weights");
  __shared__ __attribute__((aligned(16))) float Vs[NS][P][T][KC];
  __shared__ __attribute__((aligned(16))) float Us[NS][P][BNC][KC];
  // PRO: the producer's BN scale [0, C) and shift [W4_PRO_MAXC, +C), staged once (4 KiB): read per chunk
  // from LDS at transform time instead of riding in registers across the MFMA phase
  __shared__ float Ps[PRO ? 2 * W4_PRO_MAXC : 1];
  if constexpr (PRO) {
    for (int i = threadIdx.x; i < 2 * p.C; i += (int)blockDim.x)
      Ps[i < p.C ? i : W4_PRO_MAXC + i - p.C] = p.pro[i];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool compute = !WS || wave < WM * WN;
  // tid: the thread's index within its role (WS loaders count from 0 too)
  const int tid = (WS && !compute) ? (int)threadIdx.x - NT : (int)threadIdx.x;
  const int wm = wave % WM, wn = (wave / WM) % WN;
  const int b0 = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = b0 / p.bpg, b = b0 - grp * p.bpg;
  const int cb = b % p.ncb, tb = b / p.ncb;
  const int tbase = tb * T, cbase = cb * BNC;
  const float* const gxp = p.x + grp * p.gx;
  const float* const gup = p.u + grp * p.gu;
  float* const gyp = p.y + grp * p.gy;
  const float* const gbp = p.bias ? p.bias + grp * p.gbias : nullptr;

  // loader role: windows (tile lt + NT/8 h, channel lc); byte offset of the tile origin pixel and the
  // in-image row / column masks of the A x A window (rows oy-1 .. oy+A-2)
  const int lt = tid >> 3, lc = tid & 7;
  unsigned vb[IT], rmk[IT], cmk[IT];
#pragma unroll
  for (int h = 0; h < IT; ++h) {
    int ln, loy, lox;
    const int t = tbase + lt + NT / 8 * h;
    w_tile_of<MO>(p, t, ln, loy, lox);
    const bool lok = t < p.ntiles;
    vb[h] = lok ? (unsigned)((((ln * p.H + loy) * p.W + lox) * p.C + lc) * 4) : 0u;
    rmk[h] = cmk[h] = 0;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      if (lok && loy - 1 + a >= 0 && loy - 1 + a < p.H) rmk[h] |= 1u << a;
      if (lox - 1 + a >= 0 && lox - 1 + a < p.W) cmk[h] |= 1u << a;
    }
  }
  // weight loads: thread tid covers (co, column pair) of positions pos0 + k * UPK, k < UL — one vector
  // offset, the position stride rides in the scalar offset
  constexpr int UPK = NT / (4 * BNC);
  static_assert(UPK * 4 * BNC == NT, "weight loader shape");
  const int uco = (tid >> 2) & (BNC - 1), upr = tid & 3, upos = tid / (4 * BNC);
  const unsigned ub_off = cbase + uco < p.N ? (unsigned)(((upos * p.N + cbase + uco) * p.C + 2 * upr) * 4) : OOB;
  const int ustride = __builtin_amdgcn_readfirstlane(UPK * p.N * p.C * 4);

  // UB: the block's weight chunks are consecutive 36-KiB images: chunk c of output block cb at
  // ((cb * nch + c) * UNITS) units of 16 B
  const int nchunk = p.C / KC;
  auto load = [&](int c0, float (&raw)[IT][P], f32x2 (&ur)[ULR], f32x4 (&ub)[UBR]) {
    // a chunk past Cin (the pipelined tail) reads zeros: empty buffer ranges
    const bool live = c0 < p.C;
    const __amdgpu_buffer_rsrc_t xr = rsrc(gxp + c0, live ? p.xbytes - 4ull * c0 : 0ull);
#pragma unroll
    for (int h = 0; h < IT; ++h) {
      // opaque copies: the window offsets are rebuilt per chunk from 3 registers instead of being
      // hoisted out of the K loop into P live registers.  One vector offset per window row and edge
      // column (interior columns are always inside the map); the column step rides in the scalar
      // offset, so a load costs no vector ALU
      unsigned b = vb[h], rm = rmk[h], cm = cmk[h];
      asm volatile("" : "+v"(b), "+v"(rm), "+v"(cm));
      const unsigned cl = cm & 1u, cr = (cm >> (A - 1)) & 1u;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const unsigned r = b + (unsigned)((a - 1) * p.W * p.C * 4);   // pixel (oy - 1 + a, ox)
        const unsigned rok = (rm >> a) & 1u;
        const unsigned mid = r | ((rok ^ 1u) << 31);
        const unsigned lft = (r - (unsigned)(p.C * 4)) | (((rok & cl) ^ 1u) << 31);
        const unsigned rgt = r | (((rok & cr) ^ 1u) << 31);
#pragma unroll
        for (int bb = 0; bb < A; ++bb) {
          const unsigned off = bb == 0 ? lft : bb == A - 1 ? rgt : mid;
          const int so = __builtin_amdgcn_readfirstlane(bb == 0 ? 0 : (bb - 1) * p.C * 4);   // keep it in an SGPR
          raw[h][a * A + bb] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)off, so, 0));
        }
      }
    }
    if constexpr (UB) {
      const __amdgpu_buffer_rsrc_t urs = rsrc(gup + (long long)(cb * nchunk + c0 / KC) * (UNITS * 4),
                                              live ? (unsigned long long)UNITS * 16 : 0ull);
#pragma unroll
      for (int k = 0; k < UBL; ++k) {
        const unsigned off = (tid + NT * k < UNITS) ? (unsigned)((tid + NT * k) * 16) : OOB;
        ub[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(urs, (int)off, 0, 0));
      }
    } else {
      const __amdgpu_buffer_rsrc_t urs = rsrc(gup + c0, live ? p.ubytes - 4ull * c0 : 0ull);
#pragma unroll
      for (int k = 0; k < UL; ++k)
        ur[k] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(urs, (int)ub_off,
                                                                             __builtin_amdgcn_readfirstlane(k * ustride), 0));
    }
  };
  // c0: the chunk's first input channel (PRO: its BN coefficients; chunks past C stay zero)
  auto store = [&](int st, float (&raw)[IT][P], const f32x2 (&ur)[ULR], const f32x4 (&ub)[UBR], int c0) {
    float psc = 0.f, psh = 0.f;
    if constexpr (PRO) {
      const bool ok = c0 + lc < p.C;
      psc = Ps[ok ? c0 + lc : 0];
      psh = Ps[W4_PRO_MAXC + (ok ? c0 + lc : 0)];
      psc = ok ? psc : 0.f;
      psh = ok ? psh : 0.f;
    }
#pragma unroll
    for (int h = 0; h < IT; ++h) {
      const int row = lt + NT / 8 * h, c = lc ^ swz(row);
      float* const r = raw[h];
      if constexpr (PRO) {
        // BN + ReLU of the producer on the in-image elements; the padding (loaded as 0) must stay 0, so its
        // shift is 0: only the edge rows / columns of a window can leave the map (H, W multiples of 4), and
        // a tile past the end has no row in it
        const unsigned rm = rmk[h], cm = cmk[h];
        const float shT = rm ? psh : 0.f;
        const float shTop = (rm & 1u) ? shT : 0.f, shBot = ((rm >> (A - 1)) & 1u) ? shT : 0.f;
        const bool lin = cm & 1u, rin = (cm >> (A - 1)) & 1u;
#pragma unroll
        for (int a = 0; a < A; ++a) {
          const float shA = a == 0 ? shTop : a == A - 1 ? shBot : shT;
          const float shL = lin ? shA : 0.f, shR = rin ? shA : 0.f;
#pragma unroll
          for (int bb = 0; bb < A; ++bb)
            r[a * A + bb] = fmaxf(fmaf(r[a * A + bb], psc, bb == 0 ? shL : bb == A - 1 ? shR : shA), 0.f);
        }
      }
#pragma unroll
      for (int bb = 0; bb < A; ++bb) {     // B^T d along rows, in place
        float o[A];
        bt_line<MO>(r + bb, A, o);
#pragma unroll
        for (int a = 0; a < A; ++a) r[a * A + bb] = o[a];
      }
#pragma unroll
      for (int a = 0; a < A; ++a) {        // (B^T d) B along columns, straight to LDS
        float o[A];
        bt_line<MO>(r + a * A, 1, o);
#pragma unroll
        for (int bb = 0; bb < A; ++bb) Vs[st][a * A + bb][row][c] = o[bb];
      }
    }
    if constexpr (UB) {   // the global image is the LDS image: a straight 16-B copy
      float* const us = &Us[st][0][0][0];
#pragma unroll
      for (int k = 0; k < UBL; ++k)
        if (tid + NT * k < UNITS) *(f32x4*)(us + 4 * (tid + NT * k)) = ub[k];
    } else {
#pragma unroll
      for (int k = 0; k < UL; ++k) *(f32x2*)&Us[st][upos + UPK * k][uco][(2 * upr) ^ swz(uco)] = ur[k];
    }
  };

  const int nch = p.C / KC;
  if constexpr (WS) {
    // loader waves (their own branch, so the compute waves' accumulators are not live here): chunk 0, then
    // per barrier the next chunk's transform + LDS writes, its successor's loads already in flight.  The
    // compute waves pass the same nch + 1 barriers.
    if (!compute) {
      float rL[IT][P];
      f32x2 uL[ULR];
      f32x4 bL[UBR];
      load(0, rL, uL, bL);
      store(0, rL, uL, bL, 0);
      if (nch > 1) load(KC, rL, uL, bL);
      __syncthreads();
      for (int c = 0; c < nch; ++c) {
        if (c + 1 < nch) {
          store((c + 1) & 1, rL, uL, bL, (c + 1) * KC);  // chunk c + 1 (its loads were issued one chunk ago)
          if (c + 2 < nch) load((c + 2) * KC, rL, uL, bL);
        }
        __syncthreads();
      }
      return;
    }
    __syncthreads();                       // chunk 0 is in stage 0
  }

  f32x4 acc[P];
#pragma unroll
  for (int q = 0; q < P; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ar = wm * 16 + (lane & 15), br = wn * 16 + (lane & 15);
  const int ka = (2 * (lane >> 4)) ^ swz(ar), kb = (2 * (lane >> 4)) ^ swz(br);
  auto mfma = [&](int st) {
    if constexpr (WS) {
      // one compute wave per SIMD: the next group's fragments are read while this group's MFMAs run
      f32x2 a[2][4], bv[2][4];
      auto rd = [&](int q, int buf) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[buf][e] = *(const f32x2*)&Vs[st][q + e][ar][ka];
          bv[buf][e] = *(const f32x2*)&Us[st][q + e][br][kb];
        }
      };
      rd(0, 0);
#pragma unroll
      for (int g = 0; g < P / 4; ++g) {
        if (g + 1 < P / 4) rd(4 * (g + 1), (g + 1) & 1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc[4 * g + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g & 1][e][s], bv[g & 1][e][s], acc[4 * g + e], 0,
                                                                  0, 0);
      }
      return;
    }
    // four positions at a time: 4 independent MFMAs between dependent ones
#pragma unroll
    for (int q = 0; q < P; q += 4) {
      f32x2 a[4], bv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = *(const f32x2*)&Vs[st][q + e][ar][ka];
        bv[e] = *(const f32x2*)&Us[st][q + e][br][kb];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[q + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e][s], bv[e][s], acc[q + e], 0, 0, 0);
    }
  };
  float rA[IT][P];
  f32x2 uA[ULR];
  f32x4 bA[UBR];
  if constexpr (WS) {
    for (int c = 0; c < nch; ++c) {        // compute waves: chunk c, then the barrier that publishes c + 1
      mfma(c & 1);
      __syncthreads();
    }
  } else if constexpr (NS == 1) {
    load(0, rA, uA, bA);
    store(0, rA, uA, bA, 0);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) load((c + 1) * KC, rA, uA, bA);
      mfma(0);
      if (c + 1 < nch) {
        __syncthreads();                   // every wave is done reading the stage
        store(0, rA, uA, bA, (c + 1) * KC);
      }
      __syncthreads();
    }
  } else {
    float rB[IT][P];
    f32x2 uB[ULR];
    f32x4 bB[UBR];
    load(0, rA, uA, bA);
    load(KC, rB, uB, bB);
    store(0, rA, uA, bA, 0);
    __syncthreads();
    for (int c = 0; c < nch; c += 2) {
      load((c + 2) * KC, rA, uA, bA);
      mfma(0);                             // chunk c
      store(1, rB, uB, bB, (c + 1) * KC);  // chunk c + 1, in the MFMAs' shadow
      __syncthreads();
      load((c + 3) * KC, rB, uB, bB);
      mfma(1);                             // chunk c + 1 (zeros past the end)
      store(0, rA, uA, bA, (c + 2) * KC);  // chunk c + 2
      __syncthreads();
    }
  }

  // ---- output transform + epilogue: lane owns channel n of 4 consecutive tiles
  const int fl = FL >= 0 ? FL : p.flags;
  const bool sums = fl & (WF_STATS | WF_BNB | WF_BNP);
  const int n = cbase + wn * 16 + (lane & 15);
  const bool nok = n < p.N;
  const float bs = ((fl & (WF_BIAS | WF_BNB | WF_BNP)) && nok) ? gbp[n] : 0.f;
  const float sh = ((fl & (WF_BNB | WF_BNP)) && nok) ? gbp[p.N + n] : 0.f;
  float s = 0.f, ss = 0.f;
  const int t0 = tbase + wm * 16 + (lane >> 4) * 4;
  int im, oy, ox;
  w_tile_of<MO>(p, t0, im, oy, ox);
  const __amdgpu_buffer_rsrc_t yr = rsrc(gyp, p.ybytes);
  // BNB (compile-time): the gate values of two tiles are requested at a time, ahead of their use (tiles
  // 0-1 before the loop, 2-3 while tile 1 is transformed) instead of a dependent load per element
  constexpr bool GPRE = FL == WF_BNB;
  float gpre[GPRE ? 4 : 1][GPRE ? MO * MO : 1];
  int gim = im, goy = oy, gox = ox;
  auto gate_fetch = [&](int r) {           // tile t0 + r; (gim, goy, gox) walks the tiles in order
    const __amdgpu_buffer_rsrc_t gr = rsrc(p.gate, p.ybytes);
    const unsigned bad = (t0 + r < p.ntiles && nok) ? 0u : 1u;
    const unsigned gb = (unsigned)((((gim * p.H + goy) * p.W + gox) * p.N + n) * 4);
#pragma unroll
    for (int i = 0; i < MO; ++i) {
      const unsigned off = (gb + (unsigned)(i * p.W * p.N * 4)) | (bad << 31);
#pragma unroll
      for (int j = 0; j < MO; ++j)
        gpre[r][i * MO + j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
            gr, (int)off, __builtin_amdgcn_readfirstlane(j * p.N * 4), 0));
    }
    gox += MO;
    if (gox >= p.W) {
      gox = 0;
      goy += MO;
      if (goy >= p.H) {
        goy = 0;
        ++gim;
      }
    }
  };
  if constexpr (GPRE) {
    gate_fetch(0);
    gate_fetch(1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if constexpr (GPRE) {
      if (r == 1) {
        gate_fetch(2);
        gate_fetch(3);
      }
    }
    const bool tok = t0 + r < p.ntiles;
    float tt[A][MO];
#pragma unroll
    for (int a = 0; a < A; ++a) {          // M A: along columns
      float m[A];
#pragma unroll
      for (int bb = 0; bb < A; ++bb) m[bb] = acc[a * A + bb][r];
      at_line<MO>(m, tt[a]);
    }
    if (tok && nok) {
      const int pix = (im * p.H + oy) * p.W + ox;
      [[maybe_unused]] float pm[MO / 2];   // FL == WF_POOLED: row-pair maxima of the current column pair
#pragma unroll
      for (int j = 0; j < MO; ++j) {
        float m[A], o[MO];                 // A^T (M A): along rows
#pragma unroll
        for (int a = 0; a < A; ++a) m[a] = tt[a][j];
        at_line<MO>(m, o);
        if constexpr (FL == WF_POOLED) {
#pragma unroll
          for (int k = 0; k < MO / 2; ++k) {
            const float mx = fmaxf(fmaxf(o[2 * k] + bs, 0.f), fmaxf(o[2 * k + 1] + bs, 0.f));
            pm[k] = (j & 1) ? fmaxf(pm[k], mx) : mx;
          }
          if (j & 1) {
            const int H2 = p.H >> 1, W2 = p.W >> 1;
#pragma unroll
            for (int k = 0; k < MO / 2; ++k) {
              const int pidx = ((im * H2 + (oy >> 1) + k) * W2 + (ox >> 1) + (j >> 1)) * p.N + n;
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, pm[k]), yr, pidx * 4, 0, 0);
            }
          }
          continue;
        }
#pragma unroll
        for (int i = 0; i < MO; ++i) {
          float v = o[i];
          const int idx = (pix + i * p.W + j) * p.N + n;
          if (fl & WF_BIAS) v += bs;
          if (fl & WF_STATS) {
            s += v;
            ss += v * v;
          }
          if (fl & WF_RELU) v = fmaxf(v, 0.f);
          if (fl & WF_BNB) {
            float g;
            if constexpr (GPRE) g = gpre[r][i * MO + j];
            else g = p.gate[idx];
            v = g * bs + sh > 0.f ? v : 0.f;
            s += v;
            ss += v * g;
          }
          if (fl & WF_BNP) {
            const int W2 = 2 * p.W;
            const int q0 = ((im * 2 * p.H + 2 * (oy + i)) * W2 + 2 * (ox + j)) * p.N + n;
            const float y4[4] = {p.gate[q0], p.gate[q0 + p.N], p.gate[q0 + W2 * p.N], p.gate[q0 + W2 * p.N + p.N]};
            float best = -INFINITY, zb = 0.f, yb = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {  // first maximal relu(z) of the window (torch max_pool2d rule)
              const float z = y4[e] * bs + sh;
              const float av = fmaxf(z, 0.f);
              if (av > best) { best = av; zb = z; yb = y4[e]; }
            }
            const float dz = zb > 0.f ? v : 0.f;
            s += dz;
            ss += dz * yb;
          }
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), yr, idx * 4, 0, 0);
        }
      }
    }
    ox += MO;                              // next tile in row-major tile order
    if (ox >= p.W) {
      ox = 0;
      oy += MO;
      if (oy >= p.H) {
        oy = 0;
        ++im;
      }
    }
  }
  if (sums) {
    s += __shfl_xor(s, 16, 64);
    ss += __shfl_xor(ss, 16, 64);
    s += __shfl_xor(s, 32, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (nok && lane < 32) {
      double* slot = p.stats + (long long)(blockIdx.x & p.slotMask) * 2 * p.N;
      unsafeAtomicAdd(slot + (lane >= 16 ? p.N : 0) + n, (double)(lane >= 16 ? ss : s));
    }
  }
}

// ------------------------------------------------------------------------------ weight gradient
// dW = sum over 4x4 output tiles of G^T [ (A dY A^T) (.) (B^T d B) ] G: per Winograd position a GEMM
// dU[pos][co][ci] = sum_t M[pos][t][co] * V[pos][t][ci] reduced over tiles (K), 1.78x fewer MFMA cycles
// than the F(2x2) weight gradient.  Block = WM x WN waves, 16 WM co x 16 WN ci x 36 positions (wave:
// 16 co x 16 ci); the tile range is split over gridDim (split-K); each block applies G^T . G in
// registers and writes plain dW taps [Co][9][Ci] (a slab per split, summed by rk_reduce_slabs).  Per
// chunk of 8 tiles every thread transforms (tile, co) 4x4 output-gradient patches and (tile, ci) 6x6
// input windows.
struct W4wParams {
  const float* dy;      // NHWC [Nb][H][W][Co]
  const float* x;       // NHWC [Nb][H][W][Ci]
  float* out;           // [splits][Co][9][Ci]
  int Nb, H, W, Co, Ci;
  int TW, THW, ntiles, tps, nco, nci, accumulate;
  float invTW, invTHW;
  unsigned long long dybytes, xbytes;
  long long slab;       // floats per split
  const float* xpro;    // normalise-on-load of x (BN scale [Ci], shift [Ci] + ReLU of its producer) or null
};

// A y of a 4-vector -> 6 values (the adjoint of A^T)
RK_DEV void a6(float y0, float y1, float y2, float y3, float (&m)[6]) {
  const float e = y0 + y2, o = y1 + y3, e4 = y0 + 4.f * y2, o8 = 2.f * y1 + 8.f * y3;
  m[0] = y0;
  m[1] = e + o;
  m[2] = e - o;
  m[3] = e4 + o8;
  m[4] = e4 - o8;
  m[5] = y3;
}

// G^T x of a 6-vector -> 3 values (the adjoint of G)
RK_DEV void gt6(float x0, float x1, float x2, float x3, float x4, float x5, float (&g)[3]) {
  const float s12 = x1 + x2, s34 = x3 + x4;
  g[0] = 0.25f * x0 - s12 * (1.f / 6.f) + s34 * (1.f / 24.f);
  g[1] = (x2 - x1) * (1.f / 6.f) + (x3 - x4) * (1.f / 12.f);
  g[2] = (s34 - s12) * (1.f / 6.f) + x5;
}

template <int WM, int WN, int MINW>
__global__ __launch_bounds__(64 * WM * WN, MINW) void wino4_wgrad_kernel(const W4wParams p) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BCO = 16 * WM, BCI = 16 * WN;
  // dy patches / x windows per thread and chunk; with fewer items than threads (the 64 co x 32 ci
  // block) only the first waves take that role
  constexpr bool YALL = BCO * KC >= NT, XALL = BCI * KC >= NT;
  constexpr int PY = YALL ? BCO * KC / NT : 1;
  constexpr int PX = XALL ? BCI * KC / NT : 1;
  static_assert((YALL ? PY * NT == BCO * KC : (BCO * KC) % 64 == 0) &&
                (XALL ? PX * NT == BCI * KC : (BCI * KC) % 64 == 0), "wgrad tile shape");
  __shared__ __attribute__((aligned(16))) float Ms[36][BCO][KC];   // [pos][co][tile]
  __shared__ __attribute__((aligned(16))) float Vs[36][BCI][KC];   // [pos][ci][tile]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int per = p.nco * p.nci;
  const int split = b / per, r0 = b - split * per;
  const int co0 = (r0 / p.nci) * BCO, ci0 = (r0 % p.nci) * BCI;
  const int t_begin = split * p.tps;
  const int t_end = min(t_begin + p.tps, p.ntiles);
  const int nch = (t_end - t_begin + KC - 1) / KC;
  // (tile, channel) item of the thread: a wave covers 2 tiles x 32 consecutive channels, so every buffer
  // load of dy / x moves two whole 128-B lines (lanes = 8 tiles x 8 channels touched 8 lines for 32 B
  // each, 4x the cache-line traffic through the texture path for the same bytes).  The LDS stores and the
  // fragment reads are bank-conflict-free under the column swizzle swzw.
  static_assert(PY == 1 && PX == 1, "one dy patch and at most one x window per thread and chunk");
  const int tt = (tid >> 5) & 7, ch = (tid & 31) + 32 * (tid >> 8);
  const __amdgpu_buffer_rsrc_t dyr = rsrc(p.dy, p.dybytes), xr = rsrc(p.x, p.xbytes);

  float gy[PY][16], raw[PX][36];
  unsigned xv[PX];                          // in-image rows (bits 0-5) / columns (bits 8-13) of each x window
  float xpc[PX][2];                         // normalise-on-load coefficients of the thread's input channel
  auto load = [&](int c) __attribute__((always_inline)) {
    const int t = t_begin + c * KC + tt;
    const unsigned okm = t < t_end ? 1u : 0u;
    const int n = (int)(((float)t + 0.5f) * p.invTHW);   // exact below 2^22 tiles
    const int rr = t - n * p.THW;
    const int ty = (int)(((float)rr + 0.5f) * p.invTW);
    const int oy = 4 * ty, ox = 4 * (rr - ty * p.TW);
    const int pix = (n * p.H + oy) * p.W + ox;
    const bool yact = YALL || threadIdx.x < BCO * KC, xact = XALL || threadIdx.x < BCI * KC;
#pragma unroll
    for (int h = 0; h < PY && yact; ++h) {
      const int co = co0 + ch + NT / 8 * h;
      const unsigned bad = (okm & (co < p.Co ? 1u : 0u)) ^ 1u;
      const unsigned ob = (unsigned)((pix * p.Co + co) * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {        // the 4x4 patch lies inside the map (H, W multiples of 4)
        const unsigned off = (ob + (unsigned)(i * p.W * p.Co * 4)) | (bad << 31);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          gy[h][i * 4 + j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
              dyr, (int)off, __builtin_amdgcn_readfirstlane(j * p.Co * 4), 0));
      }
    }
    // window rows / columns 1..4 are inside the map; row / column 0 and 5 only away from the border
    const unsigned rm = 30u | (oy > 0 ? 1u : 0u) | (oy + 4 < p.H ? 32u : 0u);
    const unsigned cm = 30u | (ox > 0 ? 1u : 0u) | (ox + 4 < p.W ? 32u : 0u);
#pragma unroll
    for (int h = 0; h < PX && xact; ++h) {
      const int ci = ci0 + ch + NT / 8 * h;
      const unsigned xm = okm & (ci < p.Ci ? 1u : 0u);
      const unsigned xb = (unsigned)((pix * p.Ci + ci) * 4);
      const unsigned cl = cm & 1u, cr = (cm >> 5) & 1u;
      if (p.xpro) {
        xv[h] = (xm ? (rm & 63u) : 0u) | ((cm & 63u) << 8);
        xpc[h][0] = ci < p.Ci ? p.xpro[ci] : 0.f;
        xpc[h][1] = ci < p.Ci ? p.xpro[p.Ci + ci] : 0.f;
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) {        // row / edge-column vector offsets, column step in soffset
        const unsigned r = xb + (unsigned)((a - 1) * p.W * p.Ci * 4);
        const unsigned rok = xm & (rm >> a) & 1u;
        const unsigned mid = r | ((rok ^ 1u) << 31);
        const unsigned lft = (r - (unsigned)(p.Ci * 4)) | (((rok & cl) ^ 1u) << 31);
        const unsigned rgt = r | (((rok & cr) ^ 1u) << 31);
#pragma unroll
        for (int bb = 0; bb < 6; ++bb) {
          const unsigned off = bb == 0 ? lft : bb == 5 ? rgt : mid;
          const int so = __builtin_amdgcn_readfirstlane(bb == 0 ? 0 : (bb - 1) * p.Ci * 4);
          raw[h][a * 6 + bb] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)off, so, 0));
        }
      }
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
    const bool yact = YALL || threadIdx.x < BCO * KC, xact = XALL || threadIdx.x < BCI * KC;
#pragma unroll
    for (int h = 0; h < PY && yact; ++h) {
      const int row = ch + NT / 8 * h, c = tt ^ swzw(row);
      float m[6][4];                       // A dY: along rows
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float o[6];
        a6(gy[h][j], gy[h][4 + j], gy[h][8 + j], gy[h][12 + j], o);
#pragma unroll
        for (int a = 0; a < 6; ++a) m[a][j] = o[a];
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) {        // (A dY) A^T: along columns
        float o[6];
        a6(m[a][0], m[a][1], m[a][2], m[a][3], o);
#pragma unroll
        for (int bb = 0; bb < 6; ++bb) Ms[a * 6 + bb][row][c] = o[bb];
      }
    }
#pragma unroll
    for (int h = 0; h < PX && xact; ++h) {
      const int row = ch + NT / 8 * h, c = tt ^ swzw(row);
      float* const r = raw[h];
      if (p.xpro) {                         // BN + ReLU of x's producer on the in-image elements
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
          for (int bb = 0; bb < 6; ++bb) {
            const bool in = (xv[h] >> a) & (xv[h] >> (8 + bb)) & 1u;
            r[a * 6 + bb] = in ? fmaxf(fmaf(r[a * 6 + bb], xpc[h][0], xpc[h][1]), 0.f) : 0.f;
          }
      }
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) {
        float o[6];
        bt6(r[bb], r[6 + bb], r[12 + bb], r[18 + bb], r[24 + bb], r[30 + bb], o);
#pragma unroll
        for (int a = 0; a < 6; ++a) r[a * 6 + bb] = o[a];
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        float o[6];
        bt6(r[a * 6 + 0], r[a * 6 + 1], r[a * 6 + 2], r[a * 6 + 3], r[a * 6 + 4], r[a * 6 + 5], o);
#pragma unroll
        for (int bb = 0; bb < 6; ++bb) Vs[a * 6 + bb][row][c] = o[bb];
      }
    }
  };

  f32x4 acc[36];
#pragma unroll
  for (int q = 0; q < 36; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nch > 0) {
    load(0);
    store();
  }
  __syncthreads();
  const int ar = wm * 16 + (lane & 15), br = wn * 16 + (lane & 15);
  const int ka = (2 * (lane >> 4)) ^ swzp(ar), kb = (2 * (lane >> 4)) ^ swzp(br);
  const bool wswap = ((swzw(ar) ^ swzw(br)) & 1) != 0;   // wave-uniform (row bit 4 = wm / wn parity)
  // the chunk's MFMAs; SW (= wswap, wave-uniform) pairs A's column s with B's column s ^ 1
  auto mfma = [&](auto swc) __attribute__((always_inline)) {
    constexpr int SW = decltype(swc)::value;
#pragma unroll
    for (int q = 0; q < 36; q += 4) {
      f32x2 a[4], bv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = *(const f32x2*)&Ms[q + e][ar][ka];
        bv[e] = *(const f32x2*)&Vs[q + e][br][kb];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[q + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e][s], bv[e][s ^ SW], acc[q + e], 0, 0, 0);
    }
  };
  // the chunk loop is instantiated per SW and chosen once per wave (a choice per chunk costs registers)
  auto chunks = [&](auto swc) __attribute__((always_inline)) {
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) load(c + 1);
      mfma(swc);
      if (c + 1 < nch) {
        __syncthreads();
        store();
      }
      __syncthreads();
    }
  };
  if (wswap)
    chunks(std::integral_constant<int, 1>{});
  else
    chunks(std::integral_constant<int, 0>{});

  // G^T dU G per (co, ci) in registers -> the 9 taps
  float* outp = p.out + (long long)split * p.slab;
  const int ci = ci0 + wn * 16 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = co0 + wm * 16 + (lane >> 4) * 4 + r;
    float tq[3][6];
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) {       // rows: G^T X
      float g[3];
      gt6(acc[0 * 6 + bb][r], acc[1 * 6 + bb][r], acc[2 * 6 + bb][r], acc[3 * 6 + bb][r], acc[4 * 6 + bb][r],
          acc[5 * 6 + bb][r], g);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) tq[ky][bb] = g[ky];
    }
    if (co >= p.Co || ci >= p.Ci) continue;
    float* o = outp + (long long)co * 9 * p.Ci + ci;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {       // columns: (G^T X) G
      float v[3];
      gt6(tq[ky][0], tq[ky][1], tq[ky][2], tq[ky][3], tq[ky][4], tq[ky][5], v);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float* d = o + (ky * 3 + kx) * p.Ci;
        *d = p.accumulate ? *d + v[kx] : v[kx];
      }
    }
  }
}

// Software-pipelined weight gradient: 32 co x 32 ci blocks of 4 waves with TWO LDS stages (147 KiB, one
// block and one wave per SIMD, accumulators in AGPRs).  While the MFMAs of chunk c read one stage, the
// same wave transforms chunk c+1 (loaded during chunk c-1) into the other, so the transform VALU and
// LDS writes issue in the shadow of the 32-cycle MFMAs instead of in a phase of their own; one barrier
// per chunk.  Chunks past the end load zeros (out-of-range offsets), so the body is branch-free.
// (A warp-specialised form — 4 MFMA waves plus 4 loader waves transforming chunk c+1 into the other
// stage, 512 threads — measured 35-60% slower on every VGG-small layer, profiles/wino4_variants_r5.jsonl.)
__global__ __launch_bounds__(256, 1) void wino4_wgrad_pipe_kernel(const W4wParams p) {
  constexpr int BCO = 32, BCI = 32;
  __shared__ __attribute__((aligned(16))) float Ms[2][36][BCO][KC];
  __shared__ __attribute__((aligned(16))) float Vs[2][36][BCI][KC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tid = (int)threadIdx.x;
  const int wm = wave & 1, wn = (wave >> 1) & 1;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int per = p.nco * p.nci;
  const int split = b / per, r0 = b - split * per;
  const int co0 = (r0 / p.nci) * BCO, ci0 = (r0 % p.nci) * BCI;
  const int t_begin = split * p.tps;
  const int t_end = min(t_begin + p.tps, p.ntiles);
  const int nch = (t_end - t_begin + KC - 1) / KC;
  const int tt = (tid >> 5) & 7, ch = tid & 31;   // a wave: 2 tiles x 32 channels (whole 128-B lines)
  const __amdgpu_buffer_rsrc_t dyr = rsrc(p.dy, p.dybytes), xr = rsrc(p.x, p.xbytes);
  const int co = co0 + ch, ci = ci0 + ch;

  auto load = [&](int c, float (&gy)[16], float (&raw)[36]) {
    const int t = t_begin + c * KC + tt;
    const unsigned okm = t < t_end ? 1u : 0u;
    const int tq = t < t_end ? t : t_begin;            // decode a valid tile; masks zero the data
    const int n = (int)(((float)tq + 0.5f) * p.invTHW);
    const int rr = tq - n * p.THW;
    const int ty = (int)(((float)rr + 0.5f) * p.invTW);
    const int oy = 4 * ty, ox = 4 * (rr - ty * p.TW);
    const int pix = (n * p.H + oy) * p.W + ox;
    const unsigned bad = (okm & (co < p.Co ? 1u : 0u)) ^ 1u;
    const unsigned ob = (unsigned)((pix * p.Co + co) * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned off = (ob + (unsigned)(i * p.W * p.Co * 4)) | (bad << 31);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        gy[i * 4 + j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
            dyr, (int)off, __builtin_amdgcn_readfirstlane(j * p.Co * 4), 0));
    }
    const unsigned rm = 30u | (oy > 0 ? 1u : 0u) | (oy + 4 < p.H ? 32u : 0u);
    const unsigned cm = 30u | (ox > 0 ? 1u : 0u) | (ox + 4 < p.W ? 32u : 0u);
    const unsigned xm = okm & (ci < p.Ci ? 1u : 0u);
    const unsigned xb = (unsigned)((pix * p.Ci + ci) * 4);
    const unsigned cl = cm & 1u, cr = (cm >> 5) & 1u;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const unsigned r = xb + (unsigned)((a - 1) * p.W * p.Ci * 4);
      const unsigned rok = xm & (rm >> a) & 1u;
      const unsigned mid = r | ((rok ^ 1u) << 31);
      const unsigned lft = (r - (unsigned)(p.Ci * 4)) | (((rok & cl) ^ 1u) << 31);
      const unsigned rgt = r | (((rok & cr) ^ 1u) << 31);
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) {
        const unsigned off = bb == 0 ? lft : bb == 5 ? rgt : mid;
        const int so = __builtin_amdgcn_readfirstlane(bb == 0 ? 0 : (bb - 1) * p.Ci * 4);
        raw[a * 6 + bb] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (int)off, so, 0));
      }
    }
  };
  const int srow = ch, scol = tt ^ swzw(ch);
  auto store = [&](int st, const float (&gy)[16], float (&raw)[36]) {
    float m[6][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[6];
      a6(gy[j], gy[4 + j], gy[8 + j], gy[12 + j], o);
#pragma unroll
      for (int a = 0; a < 6; ++a) m[a][j] = o[a];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      float o[6];
      a6(m[a][0], m[a][1], m[a][2], m[a][3], o);
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) Ms[st][a * 6 + bb][srow][scol] = o[bb];
    }
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) {
      float o[6];
      bt6(raw[bb], raw[6 + bb], raw[12 + bb], raw[18 + bb], raw[24 + bb], raw[30 + bb], o);
#pragma unroll
      for (int a = 0; a < 6; ++a) raw[a * 6 + bb] = o[a];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      float o[6];
      bt6(raw[a * 6 + 0], raw[a * 6 + 1], raw[a * 6 + 2], raw[a * 6 + 3], raw[a * 6 + 4], raw[a * 6 + 5], o);
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) Vs[st][a * 6 + bb][srow][scol] = o[bb];
    }
  };

  f32x4 acc[36];
#pragma unroll
  for (int q = 0; q < 36; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ar = wm * 16 + (lane & 15), br = wn * 16 + (lane & 15);
  const int ka = (2 * (lane >> 4)) ^ swzp(ar), kb = (2 * (lane >> 4)) ^ swzp(br);
  const bool wswap = ((swzw(ar) ^ swzw(br)) & 1) != 0;   // wave-uniform (row bit 4 = wm / wn parity)
  auto mfma_sw = [&](int st, auto swc) __attribute__((always_inline)) {
    constexpr int SW = decltype(swc)::value;
#pragma unroll
    for (int q = 0; q < 36; q += 4) {
      f32x2 a[4], bv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = *(const f32x2*)&Ms[st][q + e][ar][ka];
        bv[e] = *(const f32x2*)&Vs[st][q + e][br][kb];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[q + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e][s], bv[e][s ^ SW], acc[q + e], 0, 0, 0);
    }
  };

  {
    float gA[16], rA[36], gB[16], rB[36];
    if (nch > 0) {
      load(0, gA, rA);
      load(1, gB, rB);
      store(0, gA, rA);
      __syncthreads();
      auto chunks = [&](auto swc) __attribute__((always_inline)) {   // per SW, chosen once per wave
        for (int c = 0; c < nch; c += 2) {
          load(c + 2, gA, rA);
          mfma_sw(0, swc);                 // chunk c
          store(1, gB, rB);                // chunk c + 1, in the MFMAs' shadow
          __syncthreads();
          load(c + 3, gB, rB);
          mfma_sw(1, swc);                 // chunk c + 1 (zeros past the end)
          store(0, gA, rA);                // chunk c + 2
          __syncthreads();
        }
      };
      if (wswap)
        chunks(std::integral_constant<int, 1>{});
      else
        chunks(std::integral_constant<int, 0>{});
    }
  }

  float* outp = p.out + (long long)split * p.slab;
  const int oci = ci0 + wn * 16 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int oco = co0 + wm * 16 + (lane >> 4) * 4 + r;
    float tq[3][6];
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) {
      float g[3];
      gt6(acc[0 * 6 + bb][r], acc[1 * 6 + bb][r], acc[2 * 6 + bb][r], acc[3 * 6 + bb][r], acc[4 * 6 + bb][r],
          acc[5 * 6 + bb][r], g);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) tq[ky][bb] = g[ky];
    }
    if (oco >= p.Co || oci >= p.Ci) continue;
    float* o = outp + (long long)oco * 9 * p.Ci + oci;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      float v[3];
      gt6(tq[ky][0], tq[ky][1], tq[ky][2], tq[ky][3], tq[ky][4], tq[ky][5], v);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float* d = o + (ky * 3 + kx) * p.Ci;
        *d = p.accumulate ? *d + v[kx] : v[kx];
      }
    }
  }
}

// ------------------------------------------------------------------------------ weight transform
__global__ __launch_bounds__(256) void wino4_wt_kernel(const float* __restrict__ w, float* __restrict__ u,
                                                       float* __restrict__ ut, int Co, int Ci) {
  __shared__ float g[32][9][33];
  w4_block(w, u, ut, Co, Ci, blockIdx.y * 32, blockIdx.x * 32, g);
}

// every layer in one launch: desc[block] = (layer, co0, ci0, -); meta[layer] = (weight offset in the
// arena, u offset or -1, ut offset or -1, Co, Ci) in floats
__global__ __launch_bounds__(256) void wino4_wt_multi_kernel(const float* __restrict__ arena, float* __restrict__ dst,
                                                             const int4* __restrict__ desc,
                                                             const long long* __restrict__ meta) {
  __shared__ float g[32][9][33];
  const int4 d = desc[blockIdx.x];
  const long long* m = meta + 5 * d.x;
  w4_block(arena + m[0], m[1] >= 0 ? dst + m[1] : nullptr, m[2] >= 0 ? dst + m[2] : nullptr, (int)m[3], (int)m[4],
           d.y, d.z, g);
}

// the X6 planes of every layer in one launch: as wino4_wt_multi_kernel, offsets in bf16 elements of dst
__global__ __launch_bounds__(256) void x6p_wt_multi_kernel(const float* __restrict__ arena, bf16* __restrict__ dst,
                                                           const int4* __restrict__ desc,
                                                           const long long* __restrict__ meta) {
  __shared__ float g[32][9][33];
  const int4 d = desc[blockIdx.x];
  const long long* m = meta + 5 * d.x;
  w4_block<true>(arena + m[0], m[1] >= 0 ? dst + m[1] : nullptr, m[2] >= 0 ? dst + m[2] : nullptr, (int)m[3],
                 (int)m[4], d.y, d.z, g);
}

// element (pos, r, c) of a set with R output rows and C input columns (C % 8 == 0) in the blocked layout of
// the fused forward kernel's weight stage: [R / 32 rounded up][C / 8][36][32][8], column swizzled
RK_DEV long long w4b_index(int pos, int r, int c, int C) {
  const int rb = r >> 5, rr = r & 31, ch = c >> 3, lc = c & 7;
  return ((((long long)rb * (C >> 3) + ch) * 36 + pos) * 32 + rr) * 8 + (lc ^ swz(rr));
}

// one 32 co x 32 ci block of filters -> the blocked forward set ub (rows co, columns ci) and / or the blocked
// data-gradient set utb (rows ci, columns co, flipped filters); either may be null
RK_DEV void w4b_block(const float* __restrict__ w, float* __restrict__ ub, float* __restrict__ utb, int Co, int Ci,
                      int co0, int ci0, float (&g)[32][9][33]) {
  float st[36];
#pragma unroll
  for (int k = 0; k < 36; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int ci = i & 31, t = (i >> 5) % 9, co = i / (9 * 32);
    st[k] = (co0 + co < Co && ci0 + ci < Ci) ? w[((long long)(co0 + co) * 9 + t) * Ci + ci0 + ci] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 36; ++k) {
    const int i = threadIdx.x + 256 * k;
    g[i / (9 * 32)][(i >> 5) % 9][i & 31] = st[k];
  }
  __syncthreads();
  if (ub != nullptr)
    for (int i = threadIdx.x; i < 1024; i += 256) {
      const int ci = i & 31, co = i >> 5;
      if (co0 + co >= Co || ci0 + ci >= Ci) continue;
      float gg[9], U[36];
#pragma unroll
      for (int t = 0; t < 9; ++t) gg[t] = g[co][t][ci];
      w4_transform(gg, U);
#pragma unroll
      for (int q = 0; q < 36; ++q) ub[w4b_index(q, co0 + co, ci0 + ci, Ci)] = U[q];
    }
  if (utb != nullptr)
    for (int i = threadIdx.x; i < 1024; i += 256) {
      const int co = i & 31, ci = i >> 5;
      if (co0 + co >= Co || ci0 + ci >= Ci) continue;
      float gg[9], U[36];
#pragma unroll
      for (int t = 0; t < 9; ++t) gg[t] = g[co][8 - t][ci];
      w4_transform(gg, U);
#pragma unroll
      for (int q = 0; q < 36; ++q) utb[w4b_index(q, ci0 + ci, co0 + co, Co)] = U[q];
    }
}

__global__ __launch_bounds__(256) void w4b_wt_kernel(const float* __restrict__ w, float* __restrict__ ub,
                                                     float* __restrict__ utb, int Co, int Ci) {
  __shared__ float g[32][9][33];
  w4b_block(w, ub, utb, Co, Ci, blockIdx.y * 32, blockIdx.x * 32, g);
}

__global__ __launch_bounds__(256) void wt_all_kernel(const float* __restrict__ arena, float* __restrict__ dst,
                                                     const int4* __restrict__ desc, const long long* __restrict__ meta) {
  __shared__ float g[32][9][33];
  const int4 d = desc[blockIdx.x];
  const long long* m = meta + 5 * d.x;
  const float* w = arena + m[0];
  if (d.w == 0) {
    wt_block(w, m[1] >= 0 ? dst + m[1] : nullptr, m[2] >= 0 ? dst + m[2] : nullptr, (int)m[3], (int)m[4], d.y, d.z, g);
  } else if (d.w == 1) {
    w4_block<false>(w, m[1] >= 0 ? dst + m[1] : nullptr, m[2] >= 0 ? dst + m[2] : nullptr, (int)m[3], (int)m[4], d.y,
                    d.z, g);
  } else if (d.w == 2) {
    bf16* db = (bf16*)dst;
    w4_block<true>(w, m[1] >= 0 ? db + m[1] : nullptr, m[2] >= 0 ? db + m[2] : nullptr, (int)m[3], (int)m[4], d.y,
                   d.z, g);
  } else {
    w4b_block(w, m[1] >= 0 ? dst + m[1] : nullptr, m[2] >= 0 ? dst + m[2] : nullptr, (int)m[3], (int)m[4], d.y, d.z, g);
  }
}

__global__ __launch_bounds__(256) void x6p_wt_kernel(const float* __restrict__ w, bf16* __restrict__ u,
                                                     bf16* __restrict__ ut, int Co, int Ci) {
  __shared__ float g[32][9][33];
  w4_block<true>(w, u, ut, Co, Ci, blockIdx.y * 32, blockIdx.x * 32, g);
}


}  // namespace

// u [36][Co][Ci] (nullable) / ut [36][Ci][Co] (nullable) of a 3x3 conv weight w [Co][9][Ci]
extern "C" int rk_wino4_weights(const float* w, float* u, float* ut, int Co, int Ci, void* stream) {
  if (Co <= 0 || Ci <= 0 || (!u && !ut)) return RK_EBADARG;
  const dim3 grid(rk_cdiv(Ci, 32), rk_cdiv(Co, 32));
  hipLaunchKernelGGL(wino4_wt_kernel, grid, dim3(256), 0, (hipStream_t)stream, w, u, ut, Co, Ci);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// Every live Winograd weight set of a network, all families, in ONE launch: desc[block] = (meta row, co0,
// ci0, family), family 0 F(2x2) fp32 sets, 1 F(4x4) fp32 sets, 2 F(4x4) X6 bf16 planes, 3 blocked F(4x4) fp32
// sets of the UB fused kernels; meta rows as the
// per-family kernels' (offsets in floats of dst, bf16 elements of dst for family 2).  Replaces three
// launches, two of them a few dozen latency-bound blocks (profiles/vgg_small_f32_step_kernels_r4*).
extern "C" int rk_wino_weights_all(const float* arena, float* dst, const int* desc, int nblocks,
                                   const long long* meta, void* stream);

// X6 planes u [36][3][Co][Ci] (nullable) / ut [36][3][Ci][Co] (nullable), bf16, of w [Co][9][Ci]
extern "C" int rk_x6p_w4_weights(const float* w, void* u, void* ut, int Co, int Ci, void* stream) {
  if (Co <= 0 || Ci <= 0 || (!u && !ut)) return RK_EBADARG;
  if (108ll * Co * Ci >= (1ll << 31)) return RK_EUNSUPPORTED;
  const dim3 grid(rk_cdiv(Ci, 32), rk_cdiv(Co, 32));
  hipLaunchKernelGGL(x6p_wt_kernel, grid, dim3(256), 0, (hipStream_t)stream, w, (bf16*)u, (bf16*)ut, Co, Ci);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// blocked forward / data-gradient sets (either nullable) of w [Co][9][Ci] for the UB fused kernels:
// ub holds ceil(Co / 32) * 32 * Ci * 36 floats, utb ceil(Ci / 32) * 32 * Co * 36 (zero padding rows stay
// as the caller initialised them); Ci % 8 == 0 for ub, Co % 8 == 0 for utb
extern "C" int rk_wino4b_weights(const float* w, float* ub, float* utb, int Co, int Ci, void* stream) {
  if (Co <= 0 || Ci <= 0 || (!ub && !utb) || (ub && Ci % 8) || (utb && Co % 8)) return RK_EBADARG;
  const dim3 grid(rk_cdiv(Ci, 32), rk_cdiv(Co, 32));
  hipLaunchKernelGGL(w4b_wt_kernel, grid, dim3(256), 0, (hipStream_t)stream, w, ub, utb, Co, Ci);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_x6p_w4_weights_multi(const float* arena, void* dst, const int* desc, int nblocks,
                                       const long long* meta, void* stream) {
  if (nblocks <= 0) return RK_OK;
  hipLaunchKernelGGL(x6p_wt_multi_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, arena, (bf16*)dst,
                     (const int4*)desc, meta);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wino_weights_all(const float* arena, float* dst, const int* desc, int nblocks,
                                   const long long* meta, void* stream) {
  if (nblocks <= 0) return RK_OK;
  hipLaunchKernelGGL(wt_all_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, arena, dst, (const int4*)desc,
                     meta);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wino4_weights_multi(const float* arena, float* dst, const int* desc, int nblocks,
                                      const long long* meta, void* stream) {
  if (nblocks <= 0) return RK_OK;
  hipLaunchKernelGGL(wino4_wt_multi_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, arena, dst,
                     (const int4*)desc, meta);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

namespace {
// shared launcher of the small-wave-tile Winograd forward kernels: MO = 4 (u [36][N][C], H, W multiples
// of 4) or MO = 2 (u [16][N][C], even H, W); T tiles x BNC channels per block of NT threads
// PRO: normalise-on-load instantiations (flags 0 / WF_STATS only: the conv after a BN + ReLU block)
template <int MO, int WM, int WN, int MINW, int NS = 1, bool UB = false, bool WS = false, bool PRO = false>
int launch_gfwd(const float* x, const float* u, float* y, const float* bias, double* stats, int slotMask,
                const float* gate, int Nb, int H, int W, int C, int N, int flags, int groups, long long gx,
                long long gu, long long gy, long long gbias, void* stream, const float* pro = nullptr) {
  constexpr int T = 16 * WM, BNC = 16 * WN, P = (MO + 2) * (MO + 2);
  if (Nb <= 0 || H <= 0 || W <= 0 || (H % MO) || (W % MO) || C <= 0 || (C % KC) || N <= 0 || groups <= 0)
    return RK_EBADARG;
  if ((flags & (WF_STATS | WF_BNB | WF_BNP)) && !stats) return RK_EBADARG;
  if ((flags & (WF_BNB | WF_BNP)) && (!gate || !bias)) return RK_EBADARG;
  if ((flags & WF_BIAS) && !bias) return RK_EBADARG;
  if (groups > 1 && (flags & (WF_STATS | WF_BNB | WF_BNP))) return RK_EUNSUPPORTED;
  if (PRO != (pro != nullptr)) return RK_EBADARG;
  if ((flags & WF_POOL) && (flags != WF_POOLED || PRO || (H & 1) || (W & 1))) return RK_EUNSUPPORTED;
  if (PRO && (groups > 1 || (flags & ~WF_STATS) || C > W4_PRO_MAXC)) return RK_EUNSUPPORTED;
  W4Params p;
  p.x = x; p.u = u; p.y = y; p.bias = bias; p.stats = stats; p.gate = gate;
  p.pro = pro;
  p.Nb = Nb; p.H = H; p.W = W; p.C = C; p.N = N;
  p.TW = W / MO;
  p.THW = (H / MO) * (W / MO);
  const long long nt = (long long)Nb * p.THW;
  if (nt >= (1LL << 30)) return RK_EBADARG;
  p.ntiles = (int)nt;
  p.ncb = rk_cdiv(N, BNC);
  p.xbytes = 4ull * Nb * H * W * C;
  p.ubytes = UB ? 4ull * P * rk_cdiv(N, 32) * 32 * C : 4ull * P * N * C;
  p.ybytes = (flags & WF_POOL) ? 4ull * Nb * (H / 2) * (W / 2) * N : 4ull * Nb * H * W * N;
  const unsigned long long gbytes = (flags & WF_BNP) ? 4 * p.ybytes : p.ybytes;
  if (p.xbytes >= 0x7fffffffull || p.ubytes >= 0x7fffffffull || gbytes >= 0x7fffffffull) return RK_EUNSUPPORTED;
  p.slotMask = slotMask;
  p.flags = flags;
  p.gx = gx; p.gu = gu; p.gy = gy; p.gbias = gbias;
  const long long bpg = (long long)rk_cdiv(p.ntiles, T) * p.ncb;
  const long long blocks = bpg * groups;
  if (blocks >= (1LL << 31)) return RK_EBADARG;
  p.bpg = (int)bpg;
  const dim3 grid((unsigned)blocks), block(64 * WM * WN * (WS ? 2 : 1));
  const hipStream_t st = (hipStream_t)stream;
  if constexpr (PRO) {
    if (flags == WF_STATS)
      hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, WF_STATS, NS, UB, WS, true>), grid, block, 0, st, p);
    else
      hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, 0, NS, UB, WS, true>), grid, block, 0, st, p);
    RK_LAUNCH_CHECK();
    return RK_OK;
  }
  switch (flags) {
    case 0: hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, 0, NS, UB, WS>), grid, block, 0, st, p); break;
    case WF_STATS:
      hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, WF_STATS, NS, UB, WS>), grid, block, 0, st, p);
      break;
    case WF_BNB: hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, WF_BNB, NS, UB, WS>), grid, block, 0, st, p); break;
    case WF_BNP: hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, WF_BNP, NS, UB, WS>), grid, block, 0, st, p); break;
    case WF_BIAS | WF_RELU:
      hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, WF_BIAS | WF_RELU, NS, UB, WS>), grid, block, 0, st, p);
      break;
    case WF_POOLED:
      hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, WF_POOLED, NS, UB, WS>), grid, block, 0, st, p);
      break;
    default: hipLaunchKernelGGL((wino_gfwd_kernel<MO, WM, WN, MINW, -1, NS, UB, WS>), grid, block, 0, st, p); break;
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}
}  // namespace

// y = conv3x3(x, w) via F(4x4,3x3) with u = rk_wino4_weights(w); flags / grouping as rk_wino_conv_grp.
// variant 0: 8 waves, 64 tiles x 32 channels (1 block per CU); 1: 4 waves, 32 x 32 (2 per CU)
static int wino4_conv_dispatch(const float* x, const float* u, float* y, const float* bias, double* stats,
                               int slotMask, const float* gate, int Nb, int H, int W, int C, int N, int flags,
                               int variant, int groups, long long gx, long long gu, long long gy, long long gbias,
                               void* stream, const float* pro) {
  if (pro) {   // normalise-on-load: the blocked-weight tiles only (the training path's weight sets)
    if (variant == 3)
      return launch_gfwd<4, 4, 2, 1, 1, true, false, true>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N,
                                                           flags, groups, gx, gu, gy, gbias, stream, pro);
    if (variant == 4)
      return launch_gfwd<4, 2, 2, 2, 1, true, false, true>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N,
                                                           flags, groups, gx, gu, gy, gbias, stream, pro);
    if (variant == 5)
      return launch_gfwd<4, 2, 2, 1, 2, true, true, true>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N,
                                                          flags, groups, gx, gu, gy, gbias, stream, pro);
    return RK_EUNSUPPORTED;
  }
  if (variant == 0)
    return launch_gfwd<4, 4, 2, 1>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx, gu, gy,
                                   gbias, stream);
  if (variant == 1)
    return launch_gfwd<4, 2, 2, 2>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx, gu, gy,
                                   gbias, stream);
  if (variant == 2)   // 4 waves, 32 x 32, two LDS stages (147 KiB), software-pipelined
    return launch_gfwd<4, 2, 2, 1, 2>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx, gu,
                                      gy, gbias, stream);
  // blocked weights (rk_wino4b_weights layout): variant 3 = variant 0's tile, 4 = variant 1's
  if (variant == 3)
    return launch_gfwd<4, 4, 2, 1, 1, true>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx,
                                            gu, gy, gbias, stream);
  if (variant == 4)
    return launch_gfwd<4, 2, 2, 2, 1, true>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx,
                                            gu, gy, gbias, stream);
  // 5: warp-specialised 32 x 32 (4 compute + 4 loader waves, two stages, 147 KiB), blocked weights
  if (variant == 5)
    return launch_gfwd<4, 2, 2, 1, 2, true, true>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups,
                                                  gx, gu, gy, gbias, stream);
  return RK_EBADARG;
}

extern "C" int rk_wino4_conv_grp(const float* x, const float* u, float* y, const float* bias, double* stats,
                                 int slotMask, const float* gate, int Nb, int H, int W, int C, int N, int flags,
                                 int variant, int groups, long long gx, long long gu, long long gy, long long gbias,
                                 void* stream) {
  return wino4_conv_dispatch(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, variant, groups, gx, gu,
                             gy, gbias, stream, nullptr);
}

// normalise-on-load: x is the pre-BN output of the previous conv and pro = its BN scale [C], shift [C]; every
// in-image input element is loaded as relu(x * scale + shift) (the consumer of a materialised BN + ReLU pass)
extern "C" int rk_wino4_conv_pro(const float* x, const float* u, float* y, const float* bias, double* stats,
                                 int slotMask, const float* gate, int Nb, int H, int W, int C, int N, int flags,
                                 int variant, const float* pro, void* stream) {
  if (!pro) return RK_EBADARG;
  return wino4_conv_dispatch(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, variant, 1, 0, 0, 0, 0,
                             stream, pro);
}

// F(2x2,3x3) with u = rk_wino_weights(w) [16][N][C] on small wave tiles (many blocks for small grids):
// variant 0: 4 waves, 32 tiles x 32 channels (32 KiB LDS, 3 blocks per CU); 1: 2 waves, 16 x 32
extern "C" int rk_wino2s_conv_grp(const float* x, const float* u, float* y, const float* bias, double* stats,
                                  int slotMask, const float* gate, int Nb, int H, int W, int C, int N, int flags,
                                  int variant, int groups, long long gx, long long gu, long long gy, long long gbias,
                                  void* stream) {
  if (variant == 0)
    return launch_gfwd<2, 2, 2, 3>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx, gu, gy,
                                   gbias, stream);
  if (variant == 1)
    return launch_gfwd<2, 1, 2, 3>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx, gu, gy,
                                   gbias, stream);
  if (variant == 2)   // 8 waves, 64 tiles x 32 channels (48 KiB LDS)
    return launch_gfwd<2, 4, 2, 2>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx, gu, gy,
                                   gbias, stream);
  if (variant == 3)   // 8 waves, 64 x 32, two LDS stages (96 KiB), software-pipelined
    return launch_gfwd<2, 4, 2, 1, 2>(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, groups, gx, gu,
                                      gy, gbias, stream);
  return RK_EBADARG;
}

extern "C" int rk_wino4_conv(const float* x, const float* u, float* y, const float* bias, double* stats, int slotMask,
                             const float* gate, int Nb, int H, int W, int C, int N, int flags, int variant,
                             void* stream) {
  return rk_wino4_conv_grp(x, u, y, bias, stats, slotMask, gate, Nb, H, W, C, N, flags, variant, 1, 0, 0, 0, 0,
                           stream);
}

// dW [Co][9][Ci] (splits == 1, optionally accumulated) or per-split slabs [splits][Co][9][Ci] of the
// weight gradient of a 3x3 stride-1 pad-1 conv by F(4x4,3x3); H, W multiples of 4; tiles_per_split % 8 == 0
// variant 0: 4 waves, 32 co x 32 ci blocks (two per CU); 1: 8 waves, 64 co x 32 ci (a quarter less
// transform work and LDS writes per MFMA); 2: 32 x 32, two LDS stages, transform in the MFMA shadow.
// (A position-split variant — each wave 9 of the 36 positions for a whole 32x32 tile on 32x32x2 MFMAs,
// half the LDS reads per MFMA cycle — measured 5-8% SLOWER than variant 1 on every VGG-small layer,
// profiles/wgrad4_variants_r3.jsonl, and was removed: the LDS-write / transform phase bounds it.)
static int wino4_wgrad_dispatch(const float* dy, const float* x, float* out, int Nb, int H, int W, int Co, int Ci,
                                int splits, int accumulate, int variant, void* stream, const float* xpro) {
  if (Nb <= 0 || H <= 0 || W <= 0 || (H & 3) || (W & 3) || Co <= 0 || Ci <= 0 || splits <= 0) return RK_EBADARG;
  if (splits > 1 && accumulate) return RK_EBADARG;
  if (variant < 0 || variant > 2) return RK_EBADARG;
  if (xpro && variant == 2) return RK_EUNSUPPORTED;
  const int BCO = variant == 1 ? 64 : 32, BCI = 32;
  W4wParams p;
  p.dy = dy; p.x = x; p.out = out;
  p.xpro = xpro;
  p.Nb = Nb; p.H = H; p.W = W; p.Co = Co; p.Ci = Ci;
  p.TW = W / 4;
  p.THW = (H / 4) * (W / 4);
  const long long nt = (long long)Nb * p.THW;
  if (nt >= (1LL << 22)) return RK_EUNSUPPORTED;    // fp32-reciprocal tile decode
  p.ntiles = (int)nt;
  p.tps = ((p.ntiles + splits - 1) / splits + KC - 1) / KC * KC;
  p.nco = rk_cdiv(Co, BCO);
  p.nci = rk_cdiv(Ci, BCI);
  p.accumulate = accumulate;
  p.invTW = 1.0f / (float)p.TW;
  p.invTHW = 1.0f / (float)p.THW;
  p.dybytes = 4ull * Nb * H * W * Co;
  p.xbytes = 4ull * Nb * H * W * Ci;
  if (p.dybytes >= 0x7fffffffull || p.xbytes >= 0x7fffffffull) return RK_EUNSUPPORTED;
  p.slab = 9LL * Co * Ci;
  const int used = rk_cdiv(p.ntiles, p.tps);
  if (used != splits) return RK_EBADARG;
  const long long blocks = (long long)splits * p.nco * p.nci;
  if (variant == 2)
    hipLaunchKernelGGL(wino4_wgrad_pipe_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p);
  else if (variant == 1)
    hipLaunchKernelGGL((wino4_wgrad_kernel<4, 2, 1>), dim3((unsigned)blocks), dim3(512), 0, (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL((wino4_wgrad_kernel<2, 2, 2>), dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wino4_wgrad_v(const float* dy, const float* x, float* out, int Nb, int H, int W, int Co, int Ci,
                                int splits, int accumulate, int variant, void* stream) {
  return wino4_wgrad_dispatch(dy, x, out, Nb, H, W, Co, Ci, splits, accumulate, variant, stream, nullptr);
}

// normalise-on-load: x is the pre-BN output of its producer, xpro = that BN's scale [Ci], shift [Ci] (+ ReLU)
extern "C" int rk_wino4_wgrad_pro(const float* dy, const float* x, float* out, int Nb, int H, int W, int Co, int Ci,
                                  int splits, int accumulate, int variant, const float* xpro, void* stream) {
  if (!xpro) return RK_EBADARG;
  return wino4_wgrad_dispatch(dy, x, out, Nb, H, W, Co, Ci, splits, accumulate, variant, stream, xpro);
}

extern "C" int rk_wino4_wgrad(const float* dy, const float* x, float* out, int Nb, int H, int W, int Co, int Ci,
                              int splits, int accumulate, void* stream) {
  return rk_wino4_wgrad_v(dy, x, out, Nb, H, W, Co, Ci, splits, accumulate, 0, stream);
}


// ------------------------------------------------------------- pre-transformed weight gradient (deep layers)
// dW by F(4x4,3x3) as three launches: transform every 4x4 dy patch (M = A dY A^T) and every 6x6 x
// window (V = B^T x B) ONCE into position-major buffers M [36][T][Co], V [36][T][Ci]; the 36 GEMMs
// dU[q] = M[q]^T V[q] run as ONE split-K launch of the tuned sgemm (kind 5, splits = 36, slab q = dU[q]);
// then dW = G^T dU G.  In the fused kernels each (co, ci) block re-transforms its whole dy / x range,
// i.e. every x window Co/32 times — on the 8x8 / 4x4 maps (T = 1024 / 256 tiles, 256-512 channels) that
// redundant transform work dominates, and here it is done once.
namespace {

// one thread per (tile, 4-channel group): float4 loads / stores (coalesced across the channel groups of
// a tile), 32-bit index math (the launchers check T * C < 2^31); the transforms run componentwise
__global__ __launch_bounds__(256) void w4pt_dy_kernel(const float* __restrict__ dy, float* __restrict__ m, int H,
                                                      int W, int C, int TW, int THW, int total4, int T) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const int C4 = C >> 2;
  const int c4 = i % C4, t = i / C4;
  const int n = t / THW, r = t - n * THW, ty = r / TW;
  const int oy = 4 * ty, ox = 4 * (r - ty * TW);
  const float* src = dy + ((n * H + oy) * W + ox) * C + 4 * c4;
  f32x4 g[16];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) g[a * 4 + b] = *(const f32x4*)(src + (a * W + b) * C);
  f32x4 res[36];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float mm[6][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[6];
      a6(g[j][e], g[4 + j][e], g[8 + j][e], g[12 + j][e], o);
#pragma unroll
      for (int a = 0; a < 6; ++a) mm[a][j] = o[a];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      float o[6];
      a6(mm[a][0], mm[a][1], mm[a][2], mm[a][3], o);
#pragma unroll
      for (int b = 0; b < 6; ++b) res[a * 6 + b][e] = o[b];
    }
  }
  float* dst = m + t * C + 4 * c4;
  const int ps = T * C;
#pragma unroll
  for (int q = 0; q < 36; ++q) *(f32x4*)(dst + q * ps) = res[q];
}

// PL: bf16 X6 planes v [36][3][T][C] (hi, mid, lo) instead of fp32 v [36][T][C]
// pro (nullable): normalise-on-load — x is the pre-BN output of its producer; relu(x * scale + shift) with
// scale = pro[0 .. C), shift = pro[C .. 2C) on every in-image element (the padding stays 0)
// VW channels per thread (4 or 2: half the 144 window registers, twice the resident waves)
template <bool PL = false, int VW = 4>
__global__ __launch_bounds__(256) void w4pt_x_kernel(const float* __restrict__ x, void* __restrict__ v, int H,
                                                     int W, int C, int TW, int THW, int total4, int T,
                                                     const float* __restrict__ pro) {
  typedef __attribute__((ext_vector_type(VW))) float fvec;
  typedef __attribute__((ext_vector_type(VW))) __bf16 bvec;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;            // total4: T * C / VW items
  const int CV = C / VW;
  const int cv = i % CV, t = i / CV;
  const int n = t / THW, r = t - n * THW, ty = r / TW;
  const int oy = 4 * ty - 1, ox = 4 * (r - ty * TW) - 1;
  fvec psc, psh;
#pragma unroll
  for (int e = 0; e < VW; ++e) psc[e] = 1.f, psh[e] = 0.f;
  if (pro) {
    psc = *(const fvec*)(pro + VW * cv);
    psh = *(const fvec*)(pro + C + VW * cv);
  }
  fvec d[36];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int yy = oy + a, xx = ox + b;
      const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      fvec val;
      if (in) {
        val = *(const fvec*)(x + ((n * H + yy) * W + xx) * C + VW * cv);
      } else {
#pragma unroll
        for (int e = 0; e < VW; ++e) val[e] = 0.f;
      }
      if (pro && in) {
#pragma unroll
        for (int e = 0; e < VW; ++e) val[e] = fmaxf(fmaf(val[e], psc[e], psh[e]), 0.f);
      }
      d[a * 6 + b] = val;
    }
#pragma unroll
  for (int b = 0; b < 6; ++b)
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      float o[6];
      bt6(d[b][e], d[6 + b][e], d[12 + b][e], d[18 + b][e], d[24 + b][e], d[30 + b][e], o);
#pragma unroll
      for (int a = 0; a < 6; ++a) d[a * 6 + b][e] = o[a];
    }
  const int ps = T * C;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    fvec o4[6];
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      float o[6];
      bt6(d[a * 6 + 0][e], d[a * 6 + 1][e], d[a * 6 + 2][e], d[a * 6 + 3][e], d[a * 6 + 4][e], d[a * 6 + 5][e], o);
#pragma unroll
      for (int b = 0; b < 6; ++b) o4[b][e] = o[b];
    }
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      if constexpr (PL) {
        bvec h4, m4, l4;
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          bf16 hh, mm, ll;
          split3v(o4[b][e], hh, mm, ll);
          h4[e] = hh;
          m4[e] = mm;
          l4[e] = ll;
        }
        bvec* dst = (bvec*)((bf16*)v + (long long)(a * 6 + b) * 3 * ps + t * C + VW * cv);
        dst[0] = h4;
        dst[ps / VW] = m4;
        dst[2 * (ps / VW)] = l4;
      } else {
        *(fvec*)((float*)v + (long long)(a * 6 + b) * ps + t * C + VW * cv) = o4[b];
      }
    }
  }
}

// Weight-gradient operands for the pre-split X6 GEMM (x6p.hip), K-inner over the tiles: M^T planes
// [36][3][Co][T] of dy (A dY A^T per 4x4 patch) and V^T planes [36][3][Ci][T] of x (B^T d B per 6x6
// window).  One thread per (tile, 4-channel group), tiles fastest, so every bf16 store of a wave writes
// 64 consecutive tiles of one (position, plane, channel) row.
// LDS-staged form (T % 32 == 0, C % 8 == 0): one wave per 32 tiles x 8 channels.  Lane (tile tl, 4-channel
// group g) transforms its window, splits the 36 x 4 values and writes them as bf16 into an LDS image of 12
// positions at a time [12][3][8][32 tiles]; the wave then stores 16-B pieces of those 288 (position, plane,
// channel) rows of 32 tiles — 54 vector stores per lane instead of 432 two-byte ones (the T-fastest kernels
// were store-issue bound: 29.7 / 22.5 us for the 8x8x256 layer, profiles/vgg_small_f32_step_kernels_r4*).
// Three 18-KiB rounds instead of one 54-KiB image: 8 waves per CU can be resident instead of 2.
template <bool DY>
__global__ __launch_bounds__(64) void w4pt_planesT_kernel(const float* __restrict__ src, bf16* __restrict__ dst,
                                                          int H, int W, int C, int TW, int THW, int T) {
  constexpr int QG = 12;                   // positions per LDS round
  __shared__ __attribute__((aligned(16))) bf16 sm[QG * 3 * 8 * 32];
  const int lane = threadIdx.x;
  const int g = lane & 1, tl = lane >> 1;
  const int t = blockIdx.x * 32 + tl, c0 = blockIdx.y * 8 + 4 * g;
  const int n = t / THW, r = t - n * THW, ty = r / TW;
  f32x4 res[36];
  if (DY) {
    const int oy = 4 * ty, ox = 4 * (r - ty * TW);
    const float* sp = src + ((n * H + oy) * W + ox) * C + c0;
    f32x4 gy[16];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) gy[a * 4 + b] = *(const f32x4*)(sp + (a * W + b) * C);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float mm[6][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float o[6];
        a6(gy[j][e], gy[4 + j][e], gy[8 + j][e], gy[12 + j][e], o);
#pragma unroll
        for (int a = 0; a < 6; ++a) mm[a][j] = o[a];
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        float o[6];
        a6(mm[a][0], mm[a][1], mm[a][2], mm[a][3], o);
#pragma unroll
        for (int b = 0; b < 6; ++b) res[a * 6 + b][e] = o[b];
      }
    }
  } else {
    const int oy = 4 * ty - 1, ox = 4 * (r - ty * TW) - 1;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const int yy = oy + a, xx = ox + b;
        res[a * 6 + b] = ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
                             ? *(const f32x4*)(src + ((n * H + yy) * W + xx) * C + c0)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int b = 0; b < 6; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float o[6];
        bt6(res[b][e], res[6 + b][e], res[12 + b][e], res[18 + b][e], res[24 + b][e], res[30 + b][e], o);
#pragma unroll
        for (int a = 0; a < 6; ++a) res[a * 6 + b][e] = o[a];
      }
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float o[6];
        bt6(res[a * 6][e], res[a * 6 + 1][e], res[a * 6 + 2][e], res[a * 6 + 3][e], res[a * 6 + 4][e],
            res[a * 6 + 5][e], o);
#pragma unroll
        for (int b = 0; b < 6; ++b) res[a * 6 + b][e] = o[b];
      }
  }
  const uint4* sv = (const uint4*)sm;
  const int tbase = blockIdx.x * 32, cbase = blockIdx.y * 8;
#pragma unroll
  for (int q0 = 0; q0 < 36; q0 += QG) {
    if (q0) __syncthreads();                 // the previous round's rows are stored
#pragma unroll
    for (int qq = 0; qq < QG; ++qq)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bf16 hh, mi, lo;
        split3v(res[q0 + qq][e], hh, mi, lo);
        const int row = (qq * 3) * 8 + 4 * g + e;   // (q, plane 0, channel) of this round
        sm[row * 32 + tl] = hh;
        sm[(row + 8) * 32 + tl] = mi;
        sm[(row + 16) * 32 + tl] = lo;
      }
    __syncthreads();
    // 288 rows x 64 B = 1152 pieces of 16 B; row (q, p, c) -> dst[((q * 3 + p) * C + cbase + c) * T + tbase ..]
    for (int i = lane; i < QG * 3 * 8 * 4; i += 64) {
      const int row = i >> 2, piece = i & 3;
      const int qp = q0 * 3 + (row >> 3), c = row & 7;
      bf16* d = dst + ((long long)qp * C + cbase + c) * T + tbase + piece * 8;
      *(uint4*)d = sv[i];
    }
  }
}

RK_DEV void store_planes_t(bf16* dst, int q, int c, int C, int T, int t, float v) {
  bf16 h, m, l;
  split3v(v, h, m, l);
  bf16* d = dst + ((long long)q * 3 * C + c) * T + t;
  const long long ps = (long long)C * T;
  d[0] = h;
  d[ps] = m;
  d[2 * ps] = l;
}

__global__ __launch_bounds__(256) void w4pt_dyT_kernel(const float* __restrict__ dy, bf16* __restrict__ m, int H,
                                                       int W, int C, int TW, int THW, int total4, int T) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const int t = i % T, c4 = i / T;
  const int n = t / THW, r = t - n * THW, ty = r / TW;
  const int oy = 4 * ty, ox = 4 * (r - ty * TW);
  const float* src = dy + ((n * H + oy) * W + ox) * C + 4 * c4;
  f32x4 g[16];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) g[a * 4 + b] = *(const f32x4*)(src + (a * W + b) * C);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float mm[6][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[6];
      a6(g[j][e], g[4 + j][e], g[8 + j][e], g[12 + j][e], o);
#pragma unroll
      for (int a = 0; a < 6; ++a) mm[a][j] = o[a];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      float o[6];
      a6(mm[a][0], mm[a][1], mm[a][2], mm[a][3], o);
#pragma unroll
      for (int b = 0; b < 6; ++b) store_planes_t(m, a * 6 + b, 4 * c4 + e, C, T, t, o[b]);
    }
  }
}

__global__ __launch_bounds__(256) void w4pt_xT_kernel(const float* __restrict__ x, bf16* __restrict__ v, int H,
                                                      int W, int C, int TW, int THW, int total4, int T) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const int t = i % T, c4 = i / T;
  const int n = t / THW, r = t - n * THW, ty = r / TW;
  const int oy = 4 * ty - 1, ox = 4 * (r - ty * TW) - 1;
  f32x4 d[36];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int yy = oy + a, xx = ox + b;
      d[a * 6 + b] = ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
                         ? *(const f32x4*)(x + ((n * H + yy) * W + xx) * C + 4 * c4)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
  for (int b = 0; b < 6; ++b)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float o[6];
      bt6(d[b][e], d[6 + b][e], d[12 + b][e], d[18 + b][e], d[24 + b][e], d[30 + b][e], o);
#pragma unroll
      for (int a = 0; a < 6; ++a) d[a * 6 + b][e] = o[a];
    }
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float o[6];
      bt6(d[a * 6 + 0][e], d[a * 6 + 1][e], d[a * 6 + 2][e], d[a * 6 + 3][e], d[a * 6 + 4][e], d[a * 6 + 5][e], o);
#pragma unroll
      for (int b = 0; b < 6; ++b) store_planes_t(v, a * 6 + b, 4 * c4 + e, C, T, t, o[b]);
    }
}

// dU [36][Co][Ci] -> dW [Co][9][Ci] (+= with accumulate); one thread per (co, 4-channel group)
// VW = 2 channels per thread (72 accumulator registers; the 4-channel form needed all 256 VGPRs, one wave
// per SIMD, and ran latency-bound on the PG-GAN lod-3 weight gradients)
__global__ __launch_bounds__(256) void w4pt_out_kernel(const float* __restrict__ du, float* __restrict__ out, int Co,
                                                       int Ci, int accumulate, int nslab, long long slab) {
  typedef __attribute__((ext_vector_type(2))) float fv2;
  const int i = blockIdx.x * 256 + threadIdx.x;   // 2-channel group index in [Co][Ci/2]
  const int plane = Co * Ci;
  if (i * 2 >= plane) return;
  const int C2 = Ci >> 1;
  const int co = i / C2, ci = 2 * (i - co * C2);
  const float* src = du + co * Ci + ci;
  fv2 u[36];
#pragma unroll
  for (int q = 0; q < 36; ++q) u[q] = *(const fv2*)(src + q * plane);
  for (int k = 1; k < nslab; ++k)   // split-K partial slabs of the GEMM
#pragma unroll
    for (int q = 0; q < 36; ++q) u[q] += *(const fv2*)(src + k * slab + q * plane);
  float* o = out + co * 9 * Ci + ci;
  fv2 w[9];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    float tq[3][6];
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      float g[3];
      gt6(u[b][e], u[6 + b][e], u[12 + b][e], u[18 + b][e], u[24 + b][e], u[30 + b][e], g);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) tq[ky][b] = g[ky];
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      float v[3];
      gt6(tq[ky][0], tq[ky][1], tq[ky][2], tq[ky][3], tq[ky][4], tq[ky][5], v);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) w[ky * 3 + kx][e] = v[kx];
    }
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    fv2* d = (fv2*)(o + k * Ci);
    *d = accumulate ? *d + w[k] : w[k];
  }
}

}  // namespace

// M [36][T][Co] and V [36][T][Ci] (T = Nb * H/4 * W/4 tiles) of dy / x (NHWC, H and W multiples of 4)
static int wino4_pt_transform(const float* dy, const float* x, float* m, float* v, int Nb, int H, int W, int Co,
                              int Ci, void* stream, const float* xpro) {
  if (Nb <= 0 || H <= 0 || W <= 0 || (H & 3) || (W & 3) || Co <= 0 || Ci <= 0) return RK_EBADARG;
  if ((Co & 3) || (Ci & 3)) return RK_EUNSUPPORTED;
  const int TW = W / 4, THW = (H / 4) * (W / 4);
  const long long T = (long long)Nb * THW;
  if (36 * T * Co >= (1ll << 31) || 36 * T * Ci >= (1ll << 31)) return RK_EUNSUPPORTED;
  const long long ty = T * Co / 4, tx = T * Ci / 4;
  hipLaunchKernelGGL(w4pt_dy_kernel, dim3((unsigned)((ty + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dy, m, H,
                     W, Co, TW, THW, (int)ty, (int)T);
  RK_LAUNCH_CHECK();
  hipLaunchKernelGGL(w4pt_x_kernel<false>, dim3((unsigned)((tx + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                     v, H, W, Ci, TW, THW, (int)tx, (int)T, xpro);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wino4_pt_transform(const float* dy, const float* x, float* m, float* v, int Nb, int H, int W,
                                     int Co, int Ci, void* stream) {
  return wino4_pt_transform(dy, x, m, v, Nb, H, W, Co, Ci, stream, nullptr);
}

// the same with x normalised on load (xpro: its producer's BN scale [Ci], shift [Ci], + ReLU)
extern "C" int rk_wino4_pt_transform_pro(const float* dy, const float* x, float* m, float* v, int Nb, int H, int W,
                                         int Co, int Ci, const float* xpro, void* stream) {
  if (!xpro) return RK_EBADARG;
  return wino4_pt_transform(dy, x, m, v, Nb, H, W, Co, Ci, stream, xpro);
}

// du: nslab slabs of [36][Co][Ci], slab floats apart (split-K partial sums), summed here
extern "C" int rk_wino4_pt_output(const float* du, float* out, int Co, int Ci, int accumulate, int nslab,
                                  long long slab, void* stream) {
  if (Co <= 0 || Ci <= 0 || nslab <= 0 || (nslab > 1 && slab < 36ll * Co * Ci)) return RK_EBADARG;
  if ((Ci & 3) || 36ll * Co * Ci >= (1ll << 31)) return RK_EUNSUPPORTED;
  const long long g2 = (long long)Co * Ci / 2;
  hipLaunchKernelGGL(w4pt_out_kernel, dim3((unsigned)((g2 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, du,
                     out, Co, Ci, accumulate, nslab, slab);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// ---------------------------------------------------------- pre-transformed F(4x4) conv (deep layers)
// y = conv3x3(x, w) as V = B^T x B once per 6x6 window (rk_wino4_pt_transform's x half, [36][T][C]),
// Y'[q] = V[q] U[q]^T as ONE 36-group sgemm (u = wino4_u(w) [36][N][C], kind 3), then this output
// transform A^T Y' A per 4x4 tile with the fused kernels' epilogues (bias, ReLU, BN statistics, BNB /
// BNP data-gradient gating).  On the 8x8 / 4x4 maps the fused kernels re-transform every input window
// once per output-channel block; here each window is transformed once and the GEMMs run at sgemm speed.
namespace {

__global__ __launch_bounds__(256) void w4pt_conv_out_kernel(const float* __restrict__ yt, float* __restrict__ y,
                                                            const float* __restrict__ bp, double* stats, int slotMask,
                                                            const float* __restrict__ gate, int Nb, int H, int W,
                                                            int N, int TW, int THW, int T, int flags, int nslab,
                                                            long long slab, long long qs, long long ts, float slope) {
  constexpr int TPB = 4;                   // tiles per block: one per 64-thread group (>= 2 blocks per CU
                                           // on the 4x4 x 512 maps: T x N / 256 blocks)
  __shared__ float red[2][4][64];
  const int nblk = (N + 63) / 64;
  const int nb = blockIdx.x % nblk, tb = blockIdx.x / nblk;
  const int lane = threadIdx.x & 63, tg = threadIdx.x >> 6;
  const int n = nb * 64 + lane;
  const bool nok = n < N;
  const float bs = ((flags & (WF_BIAS | WF_BNB | WF_BNP)) && nok) ? bp[n] : 0.f;
  const float sh = ((flags & (WF_BNB | WF_BNP)) && nok) ? bp[N + n] : 0.f;
  float s = 0.f, ss = 0.f;
  {
    const int t = tb * TPB + tg;
    if (t < T && nok) {
    float m[36];
#pragma unroll
    for (int q = 0; q < 36; ++q) m[q] = yt[q * qs + (long long)t * ts + n];
    for (int k = 1; k < nslab; ++k)   // split-K partial slabs of the GEMM
#pragma unroll
      for (int q = 0; q < 36; ++q) m[q] += yt[k * slab + q * qs + (long long)t * ts + n];
    float tt[6][4];
#pragma unroll
    for (int a = 0; a < 6; ++a) {          // M A: along columns
      float o[4];
      at6(m[a * 6 + 0], m[a * 6 + 1], m[a * 6 + 2], m[a * 6 + 3], m[a * 6 + 4], m[a * 6 + 5], o);
#pragma unroll
      for (int j = 0; j < 4; ++j) tt[a][j] = o[j];
    }
    const int im = t / THW, rr = t - im * THW, ty = rr / TW;
    const int oy = 4 * ty, ox = 4 * (rr - ty * TW);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[4];
      at6(tt[0][j], tt[1][j], tt[2][j], tt[3][j], tt[4][j], tt[5][j], o);   // A^T (M A): along rows
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = o[i];
        const long long idx = (((long long)im * H + oy + i) * W + ox + j) * N + n;
        if (flags & WF_BIAS) v += bs;
        if (flags & WF_STATS) {
          s += v;
          ss += v * v;
        }
        if (flags & WF_RELU) v = fmaxf(v, 0.f);
        if (flags & WF_LRELU) v = v > 0.f ? v : v * slope;
        if (flags & WF_BNB) {
          const float g = gate[idx];
          v = g * bs + sh > 0.f ? v : 0.f;
          s += v;
          ss += v * g;
        }
        if (flags & WF_BNP) {
          const long long W2 = 2LL * W;
          const long long q0 = (((long long)im * 2 * H + 2 * (oy + i)) * W2 + 2 * (ox + j)) * N + n;
          const float y4[4] = {gate[q0], gate[q0 + N], gate[q0 + W2 * N], gate[q0 + W2 * N + N]};
          float best = -INFINITY, zb = 0.f, yb = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {    // first maximal relu(z) of the window (torch max_pool2d rule)
            const float z = y4[e] * bs + sh;
            const float av = fmaxf(z, 0.f);
            if (av > best) { best = av; zb = z; yb = y4[e]; }
          }
          const float dz = zb > 0.f ? v : 0.f;
          s += dz;
          ss += dz * yb;
        }
        y[idx] = v;
      }
    }
    }
  }
  if (flags & (WF_STATS | WF_BNB | WF_BNP)) {
    red[0][tg][lane] = s;
    red[1][tg][lane] = ss;
    __syncthreads();
    if (tg == 0 && nok) {
      const float a = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
      const float b = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
      double* slot = stats + (long long)(blockIdx.x & slotMask) * 2 * N;
      unsafeAtomicAdd(slot + n, (double)a);
      unsafeAtomicAdd(slot + N + n, (double)b);
    }
  }
}

// The same with VW-channel vectors (VW = 2: 8-B, 4: 16-B accesses; the scalar kernel's 4-B accesses ran at
// ~3.2 TB/s): one thread per (tile, VW channels) — 36 vector loads of Y', 16 vector stores, vector gate
// loads; a 64-thread block = 64 / (64 / VW) tiles x 64 channels, many blocks even on the 4x4 maps.
template <int VW>
__global__ __launch_bounds__(64) void w4pt_conv_outv_kernel(const float* __restrict__ yt, float* __restrict__ y,
                                                            const float* __restrict__ bp, double* stats, int slotMask,
                                                            const float* __restrict__ gate, int Nb, int H, int W,
                                                            int N, int TW, int THW, int T, int flags, int nslab,
                                                            long long slab, long long qs, long long ts,
                                                            float slope) {
  constexpr int LPT = 64 / VW, TPB = 64 / LPT;   // lanes per tile, tiles per block
  typedef __attribute__((ext_vector_type(VW))) float fv;
  __shared__ float red[2][TPB][64];
  const int nblk = (N + 63) / 64;
  const int nb = blockIdx.x % nblk, tb = blockIdx.x / nblk;
  const int qd = threadIdx.x % LPT, tg = threadIdx.x / LPT;
  const int n = nb * 64 + VW * qd;
  const bool nok = n < N;
  fv bs = {}, sh = {};
  if ((flags & (WF_BIAS | WF_BNB | WF_BNP)) && nok) bs = *(const fv*)(bp + n);
  if ((flags & (WF_BNB | WF_BNP)) && nok) sh = *(const fv*)(bp + N + n);
  fv s = {}, ss = {};
  const int t = tb * TPB + tg;
  if (t < T && nok) {
    fv m[36];
    const float* src = yt + (long long)t * ts + n;
#pragma unroll
    for (int q = 0; q < 36; ++q) m[q] = *(const fv*)(src + q * qs);
    for (int k = 1; k < nslab; ++k)   // split-K partial slabs of the GEMM
#pragma unroll
      for (int q = 0; q < 36; ++q) m[q] += *(const fv*)(src + k * slab + q * qs);
    const int im = t / THW, rr = t - im * THW, ty = rr / TW;
    const int oy = 4 * ty, ox = 4 * (rr - ty * TW);
    fv res[4][4];
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      float tt[6][4];
#pragma unroll
      for (int a = 0; a < 6; ++a) {          // M A: along columns
        float o[4];
        at6(m[a * 6 + 0][e], m[a * 6 + 1][e], m[a * 6 + 2][e], m[a * 6 + 3][e], m[a * 6 + 4][e], m[a * 6 + 5][e], o);
#pragma unroll
        for (int j = 0; j < 4; ++j) tt[a][j] = o[j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float o[4];
        at6(tt[0][j], tt[1][j], tt[2][j], tt[3][j], tt[4][j], tt[5][j], o);   // A^T (M A): along rows
#pragma unroll
        for (int i = 0; i < 4; ++i) res[i][j][e] = o[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fv v = res[i][j];
        const long long idx = (((long long)im * H + oy + i) * W + ox + j) * N + n;
        if (flags & WF_BIAS) v += bs;
        if (flags & WF_STATS) {
          s += v;
          ss += v * v;
        }
        if (flags & WF_RELU) {
#pragma unroll
          for (int e = 0; e < VW; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (flags & WF_LRELU) {
#pragma unroll
          for (int e = 0; e < VW; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * slope;
        }
        if (flags & WF_BNB) {
          const fv g = *(const fv*)(gate + idx);
#pragma unroll
          for (int e = 0; e < VW; ++e) {
            v[e] = g[e] * bs[e] + sh[e] > 0.f ? v[e] : 0.f;
            s[e] += v[e];
            ss[e] += v[e] * g[e];
          }
        }
        if (flags & WF_BNP) {
          const long long W2 = 2LL * W;
          const long long q0 = (((long long)im * 2 * H + 2 * (oy + i)) * W2 + 2 * (ox + j)) * N + n;
          const fv y4[4] = {*(const fv*)(gate + q0), *(const fv*)(gate + q0 + N), *(const fv*)(gate + q0 + W2 * N),
                            *(const fv*)(gate + q0 + W2 * N + N)};
#pragma unroll
          for (int e = 0; e < VW; ++e) {
            float best = -INFINITY, zb = 0.f, yb = 0.f;
#pragma unroll
            for (int w4 = 0; w4 < 4; ++w4) {   // first maximal relu(z) of the window (torch max_pool2d rule)
              const float z = y4[w4][e] * bs[e] + sh[e];
              const float av = fmaxf(z, 0.f);
              if (av > best) { best = av; zb = z; yb = y4[w4][e]; }
            }
            const float dz = zb > 0.f ? v[e] : 0.f;
            s[e] += dz;
            ss[e] += dz * yb;
          }
        }
        *(fv*)(y + idx) = v;
      }
  }
  if (flags & (WF_STATS | WF_BNB | WF_BNP)) {
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      red[0][tg][VW * qd + e] = s[e];
      red[1][tg][VW * qd + e] = ss[e];
    }
    __syncthreads();
    const int c = threadIdx.x;   // 64 threads: one channel of the block's 64 each
    if (nb * 64 + c < N) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int r = 0; r < TPB; ++r) {
        a += red[0][r][c];
        b += red[1][r][c];
      }
      double* slot = stats + (long long)(blockIdx.x & slotMask) * 2 * N;
      unsafeAtomicAdd(slot + nb * 64 + c, (double)a);
      unsafeAtomicAdd(slot + N + nb * 64 + c, (double)b);
    }
  }
}

}  // namespace

// yt: nslab slabs of [36][T][N], slab floats apart (split-K partial sums of the GEMM), summed here
// slope: the leaky-ReLU slope of WF_LRELU (bias, then max(v, slope v); no statistics with it)
// tmajor: Y' is tile-major [T][36][N] (the plane GEMM writes it so: each tile's 36 positions in one 36N-float
// run instead of 36 runs a T x N plane apart), else position-major [36][T][N]
extern "C" int rk_wino4_pt_conv_out(const float* yt, float* y, const float* bias, double* stats, int slotMask,
                                    const float* gate, int Nb, int H, int W, int N, int flags, int nslab,
                                    long long slab, int tmajor, float slope, void* stream) {
  if (Nb <= 0 || H <= 0 || W <= 0 || (H & 3) || (W & 3) || N <= 0 || nslab <= 0) return RK_EBADARG;
  if ((flags & WF_LRELU) && (flags & (WF_RELU | WF_STATS | WF_BNB | WF_BNP))) return RK_EBADARG;
  if ((flags & (WF_STATS | WF_BNB | WF_BNP)) && !stats) return RK_EBADARG;
  if ((flags & (WF_BNB | WF_BNP)) && (!gate || !bias)) return RK_EBADARG;
  if ((flags & WF_BIAS) && !bias) return RK_EBADARG;
  const int TW = W / 4, THW = (H / 4) * (W / 4);
  const long long T = (long long)Nb * THW;
  if (T * N >= (1LL << 31)) return RK_EUNSUPPORTED;
  const long long blocks = ((N + 63) / 64) * ((T + 3) / 4);
  if (nslab > 1 && slab < 36 * T * N) return RK_EBADARG;
  const long long qs = tmajor ? N : T * N, ts = tmajor ? 36LL * N : N;
  // vector width 2 (8-B accesses, 2 tiles x 64 channels per block) by default; RAFIKI_PT_OUT_VW=4 selects the
  // 16-B form: -4 us per VGG-small step but +45 us per PG-GAN lod-3 round and +0.23 ms at lod 0 on the same
  // box (profiles/pt_out_vw_ab_r6.txt)
  static const int vw = [] {
    const char* e = std::getenv("RAFIKI_PT_OUT_VW");
    return e && std::atoi(e) == 4 ? 4 : 2;
  }();
  if (N % vw == 0) {
    const long long blocksv = ((N + 63) / 64) * ((T + vw - 1) / vw);   // vw tiles x 64 channels per block
    if (vw == 4)
      hipLaunchKernelGGL(w4pt_conv_outv_kernel<4>, dim3((unsigned)blocksv), dim3(64), 0, (hipStream_t)stream, yt, y,
                         bias, stats, slotMask, gate, Nb, H, W, N, TW, THW, (int)T, flags, nslab, slab, qs, ts, slope);
    else
      hipLaunchKernelGGL(w4pt_conv_outv_kernel<2>, dim3((unsigned)blocksv), dim3(64), 0, (hipStream_t)stream, yt, y,
                         bias, stats, slotMask, gate, Nb, H, W, N, TW, THW, (int)T, flags, nslab, slab, qs, ts, slope);
    RK_LAUNCH_CHECK();
    return RK_OK;
  }
  hipLaunchKernelGGL(w4pt_conv_out_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, yt, y, bias,
                     stats, slotMask, gate, Nb, H, W, N, TW, THW, (int)T, flags, nslab, slab, qs, ts, slope);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// V = B^T x B of every 6x6 window: [36][T][C] (the x half of rk_wino4_pt_transform)
extern "C" int rk_wino4_pt_input_pro(const float* x, float* v, int Nb, int H, int W, int C, const float* pro,
                                     void* stream) {
  if (Nb <= 0 || H <= 0 || W <= 0 || (H & 3) || (W & 3) || C <= 0) return RK_EBADARG;
  if (C & 3) return RK_EUNSUPPORTED;
  const int TW = W / 4, THW = (H / 4) * (W / 4);
  const long long T = (long long)Nb * THW;
  if (36 * T * C >= (1ll << 31)) return RK_EUNSUPPORTED;
  const long long tx = T * C / 4;
  hipLaunchKernelGGL(w4pt_x_kernel<false>, dim3((unsigned)((tx + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                     v, H, W, C, TW, THW, (int)tx, (int)T, pro);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_wino4_pt_input(const float* x, float* v, int Nb, int H, int W, int C, void* stream) {
  return rk_wino4_pt_input_pro(x, v, Nb, H, W, C, nullptr, stream);
}

// V planes [36][3][T][C] (bf16 hi, mid, lo of B^T x B) for the pre-split X6 GEMM (x6p.hip); pro as above
extern "C" int rk_x6p_w4_input_pro(const float* x, void* v, int Nb, int H, int W, int C, const float* pro,
                                   void* stream) {
  if (Nb <= 0 || H <= 0 || W <= 0 || (H & 3) || (W & 3) || C <= 0) return RK_EBADARG;
  if (C & 3) return RK_EUNSUPPORTED;
  const int TW = W / 4, THW = (H / 4) * (W / 4);
  const long long T = (long long)Nb * THW;
  if (108 * T * C >= (1ll << 31) || (long long)Nb * H * W * C >= (1ll << 31)) return RK_EUNSUPPORTED;
  // 4 channels per thread by default; RAFIKI_PT_X_VW=2: 2 channels (83 instead of 159 VGPRs, 5 waves per SIMD
  // instead of 3) — +6 us per VGG-small step, -0.1 ms per PG-GAN lod-0 round (profiles/pt_x_vw_ab_r6.txt)
  static const int vw = [] {
    const char* e = std::getenv("RAFIKI_PT_X_VW");
    return e && std::atoi(e) == 2 ? 2 : 4;
  }();
  const long long tx = T * C / vw;
  if (vw == 4)
    hipLaunchKernelGGL((w4pt_x_kernel<true, 4>), dim3((unsigned)((tx + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, x, v, H, W, C, TW, THW, (int)tx, (int)T, pro);
  else
    hipLaunchKernelGGL((w4pt_x_kernel<true, 2>), dim3((unsigned)((tx + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, x, v, H, W, C, TW, THW, (int)tx, (int)T, pro);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_x6p_w4_input(const float* x, void* v, int Nb, int H, int W, int C, void* stream) {
  return rk_x6p_w4_input_pro(x, v, Nb, H, W, C, nullptr, stream);
}

// M^T planes [36][3][Co][T] of dy and V^T planes [36][3][Ci][T] of x (bf16), the weight-gradient operands
// of the pre-split X6 GEMM: dU[q] = M^T[q] (V^T[q])^T, K = T tiles
extern "C" int rk_x6p_w4_wgrad_transform(const float* dy, const float* x, void* mt, void* vt, int Nb, int H, int W,
                                         int Co, int Ci, void* stream) {
  if (Nb <= 0 || H <= 0 || W <= 0 || (H & 3) || (W & 3) || Co <= 0 || Ci <= 0) return RK_EBADARG;
  if ((Co & 3) || (Ci & 3)) return RK_EUNSUPPORTED;
  const int TW = W / 4, THW = (H / 4) * (W / 4);
  const long long T = (long long)Nb * THW;
  if (108 * T * Co >= (1ll << 31) || 108 * T * Ci >= (1ll << 31)) return RK_EUNSUPPORTED;
  if ((long long)Nb * H * W * (Co > Ci ? Co : Ci) >= (1ll << 31)) return RK_EUNSUPPORTED;
  if (T % 32 == 0 && Co % 8 == 0 && Ci % 8 == 0) {
    hipLaunchKernelGGL(w4pt_planesT_kernel<true>, dim3((unsigned)(T / 32), Co / 8), dim3(64), 0, (hipStream_t)stream,
                       dy, (bf16*)mt, H, W, Co, TW, THW, (int)T);
    RK_LAUNCH_CHECK();
    hipLaunchKernelGGL(w4pt_planesT_kernel<false>, dim3((unsigned)(T / 32), Ci / 8), dim3(64), 0, (hipStream_t)stream,
                       x, (bf16*)vt, H, W, Ci, TW, THW, (int)T);
    RK_LAUNCH_CHECK();
    return RK_OK;
  }
  const long long ty = T * Co / 4, tx = T * Ci / 4;
  hipLaunchKernelGGL(w4pt_dyT_kernel, dim3((unsigned)((ty + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dy,
                     (bf16*)mt, H, W, Co, TW, THW, (int)ty, (int)T);
  RK_LAUNCH_CHECK();
  hipLaunchKernelGGL(w4pt_xT_kernel, dim3((unsigned)((tx + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                     (bf16*)vt, H, W, Ci, TW, THW, (int)tx, (int)T);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
