// fp32 implicit-GEMM engine for gfx950: 3x3/1x1 convolutions (forward, data-grad as a forward conv
// of dy with flipped/transposed weights, weight-grad) and dense GEMMs on v_mfma_f32_32x32x2_f32 —
// exact fp32 products with fp32 accumulation (bit-equal to an fmaf chain), i.e. the reference's own
// precision (pg_gans.py:830,914 dtype='float32'; Keras fp32 in TfFeedForward.py:141-164 and
// TfVgg16.py:115-130).  No bf16 anywhere on this path.
//
// Design for the f32 MFMA rate (64 FLOP/clk/SIMD, 1/16 of bf16): the arithmetic, not the memory
// system, is the bound, so a block owns a large tile and keeps every SIMD issuing MFMAs:
//   * 4 or 8 waves (2x2, 4x1, 1x4, 4x2, 2x4); wave tile (32*MI) x (32*NI), MI, NI in {1,2} -> block
//     tiles 64x64 .. 256x128 (up to 64 fp32 accumulator registers per lane), BK = 32 fp32 (128-B
//     LDS rows); the big tiles cut the L2 / Infinity-Cache bytes per FLOP (a 64x64 tile needs
//     16 B/clk/CU of operands at the f32 MFMA rate — the measured bound of the small tiles);
//   * operands go global -> LDS by buffer_load_dwordx4 ... lds (no VGPR staging, no ds_write):
//     "K-inner" operands (reduction index contiguous: NHWC activations gathered per 3x3 tap, [N][K]
//     weights) land as XOR-swizzled [T][32] rows read with ds_read_b128; "K-outer" operands
//     (reduction over rows: dY / X in the weight gradients, W in dense dX) land as [32][T] rows read
//     with ds_read_b32 (32 consecutive dwords per half-wave: conflict-free);
//   * the K order inside a 8-deep group is permuted so one ds_read_b128 feeds 4 MFMAs: lane half h
//     supplies k = 8g + 4h + e at MFMA step e, for both operands;
//   * an NST-stage LDS ring (2: 64 KiB at 128x128, 2 blocks/CU; 3: one block/CU, two tiles in
//     flight) with ONE raw s_barrier per K-tile and a counted vmcnt;
//   * out-of-range lanes (conv halo, tile edges, K tail) DMA zeros through the buffer range check;
//   * the accumulator layout puts one output channel per lane and 16 pixels in registers, so BN
//     statistics are 16 in-register adds + one lane swap, and stores are 2 x 128-B rows per
//     instruction.
// X6 = true (tile code + 16): the same kernel with the products on the bf16 matrix cores at fp32
// accuracy.  Every fp32 fragment value is split after its LDS read into three bf16 pieces,
// x = hi + mid + lo (each the round-to-nearest bf16 of the remaining residual; the subtractions are
// exact), and a 16-deep k chunk takes SIX v_mfma_f32_32x32x16_bf16 — hi*hi, hi*mid, mid*hi, hi*lo,
// lo*hi, mid*mid — into the same fp32 accumulators.  The dropped terms (mid*lo, lo*mid, lo*lo) are
// below 2^-25 of |x*y| and the pieces represent x to 2^-26, so every product is fp32-accurate
// (below the unit roundoff of the fp32 accumulation that follows, which is unchanged): at the bf16
// MFMA rate (16x the f32 one) six products cost 6/16 of the v_mfma_f32_32x32x2_f32 cycles.  The
// error against fp64 is measured in tests/test_x6_gpu.py and profiles/ (equal to the f32 MFMA's).
// Epilogues (runtime flags: the epilogue runs once per tile after K/32 x 4096 MFMA cycles, so its
// VALU is noise): bias, ReLU / leaky-ReLU, ReLU gate (dense dX), BN statistics (fp64 atomic slots),
// FLAG_BNB / FLAG_BNP (data-gradient into a BN+ReLU [+2x2 max-pool] layer: mask + BN-backward sums),
// split-K fp32 slabs, accumulate.
#include "common.h"
#include <cstdlib>

namespace {

#include "sgemm_core.h"

// One operand tile of T rows (K-inner) or T columns (K-outer) per K-tile; T*128 bytes = T/8 DMA
// wave-instructions, T/(8*NW) per wave of an NW-wave workgroup.
template <int MODE, int T, int NW>
struct SOperand {
  static constexpr bool KIN = MODE == SM_KIN_DENSE || MODE == SM_KIN_CONV || MODE == SM_KIN_CONVF ||
                              MODE == SM_KIN_CONVG;
  static constexpr int NQ = T / (8 * NW);
  static_assert(NQ >= 1 && NQ * 8 * NW == T, "operand tile must split evenly over the waves");
  static constexpr int RS = T / 4;  // 16-B slots per K-outer row
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned base[NQ];
  unsigned mask[NQ];
  int sub[NQ];
  int dyx[NQ];  // K-outer conv: (dy, dx) packed as dy*W + dx
  int dy[NQ], dx[NQ];
  unsigned tpy, tpx;  // table-driven gathers: this group's tap offsets

  RK_DEV void init(const SgParams& p, const float* ptr, unsigned long long bytes, int ld, int tile0, int extent,
                   int wid, int lane, int grp = 0) {
    rsrc = s_rsrc(ptr, bytes);
    tpy = tpx = 0u;
    if constexpr (MODE == SM_KIN_CONVG || MODE == SM_KOUT_CONVG) {
      tpy = p.tpy[grp];
      tpx = p.tpx[grp];
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int slot = (wid * NQ + q) * 64 + lane;
      dy[q] = dx[q] = dyx[q] = 0;
      if constexpr (KIN) {
        const int i = slot >> 3;
        const int c = (slot & 7) ^ ((i >> 1) & 7);  // logical 16-B chunk stored at this slot
        sub[q] = c;
        const int gi = tile0 + i;
        const bool ok = gi < extent;
        if constexpr (MODE == SM_KIN_DENSE) {
          base[q] = (unsigned)gi * (unsigned)ld * 4u;
          mask[q] = ok ? 1u : 0u;
        } else if constexpr (MODE == SM_KIN_CONVG) {
          int n, i, j;
          s_nhw(gi, p, n, i, j);
          const int si = p.stride * i, sj = p.stride * j;
          base[q] = (unsigned)(((n * p.H + si) * p.W + sj) * p.C) * 4u;
          unsigned m = 0u;
          for (int t = 0; t < p.ntaps; ++t)
            m |= (((unsigned)(si + s_tapoff(tpy, t)) < (unsigned)p.H && (unsigned)(sj + s_tapoff(tpx, t)) < (unsigned)p.W)
                      ? 1u : 0u) << t;
          mask[q] = ok ? m : 0u;
        } else {
          int h, w;
          s_hw(gi, p.H, p.W, p.log2H, p.log2W, p.invH, p.invW, h, w);
          base[q] = (unsigned)gi * (unsigned)p.C * 4u;
          if constexpr (MODE == SM_KIN_CONVF) base[q] += (unsigned)c * 16u;
          unsigned m = 1u;
          if (p.taps == 9) {
            m = 0u;
#pragma unroll
            for (int t = 0; t < 9; ++t)
              m |= (((unsigned)(h + s_tap_dy(t)) < (unsigned)p.H && (unsigned)(w + s_tap_dx(t)) < (unsigned)p.W) ? 1u : 0u)
                   << t;
          }
          mask[q] = ok ? m : 0u;
        }
      } else {
        const int krow = slot / RS;
        const int col = tile0 + 4 * (slot % RS);
        sub[q] = krow;
        bool ok = col < extent;
        if constexpr (MODE == SM_KOUT_DENSE) {
          base[q] = (unsigned)col * 4u;
        } else if constexpr (MODE == SM_KOUT_CONVG) {  // column = (tap, channel), tap from the table
          const int tap = s_cdiv(col, p);
          const int ci = col - tap * p.C;
          ok = ok && tap < p.ntaps;
          const int tt = tap < p.ntaps ? tap : 0;
          dy[q] = s_tapoff(tpy, tt);
          dx[q] = s_tapoff(tpx, tt);
          base[q] = (unsigned)ci * 4u;
        } else {  // SM_KOUT_CONV: column = (tap, channel) of the gathered activation
          const int tap = s_cdiv(col, p);
          const int ci = col - tap * p.C;
          ok = ok && tap < p.taps;
          if (p.taps == 9) {
            dy[q] = s_tap_dy(tap);
            dx[q] = s_tap_dx(tap);
          }
          dyx[q] = dy[q] * p.W + dx[q];
          base[q] = (unsigned)ci * 4u;
        }
        mask[q] = ok ? 1u : 0u;
      }
    }
  }

  // byte offset (or SOOB) of this lane's 16-B chunk for instruction q of K-tile kt.  Branch-free
  // (selects; reciprocal decodes, exact below 2^22), so the DMA issue code is straight-line and the
  // scheduler can interleave it with the MFMA stream.
  // (invalid lanes get bit 31 OR'ed in: >= 2 GiB, past every descriptor's range -> zeros)
  RK_DEV unsigned offset(const SgParams& p, int q, int kt, int K, int ld) const {
    if constexpr (MODE == SM_KIN_DENSE) {
      const int k = kt * SBK + 4 * sub[q];
      const bool ok = mask[q] && k < K;
      return (base[q] + (unsigned)k * 4u) | ((unsigned)!ok << 31);
    } else if constexpr (MODE == SM_KIN_CONVF) {
      const int k0 = kt * SBK;  // wave-uniform: one tap per K-tile
      const int tap = (int)(((float)k0 + 0.5f) * p.invC);
      const int ci0 = k0 - tap * p.C;
      const int d = p.taps == 9 ? s_tap_dy(tap) * p.W + s_tap_dx(tap) : 0;
      const bool ok = k0 < K && ((mask[q] >> tap) & 1u);
      return (unsigned)((int)base[q] + (d * p.C + ci0) * 4) | ((unsigned)!ok << 31);
    } else if constexpr (MODE == SM_KIN_CONV) {
      const int k = kt * SBK + 4 * sub[q];
      const int tap = (int)(((float)k + 0.5f) * p.invC);
      const int ci = k - tap * p.C;
      const int d = p.taps == 9 ? s_tap_dy(tap) * p.W + s_tap_dx(tap) : 0;
      const bool ok = k < K && ((mask[q] >> tap) & 1u);
      return (unsigned)((int)base[q] + (d * p.C + ci) * 4) | ((unsigned)!ok << 31);
    } else if constexpr (MODE == SM_KIN_CONVG) {
      const int k = kt * SBK + 4 * sub[q];
      const int tap = s_cdiv(k, p);
      const int ci = k - tap * p.C;
      const int tt = tap & 15;
      const int d = s_tapoff(tpy, tt) * p.W + s_tapoff(tpx, tt);
      const bool ok = k < K && ((mask[q] >> tt) & 1u);
      return (unsigned)((int)base[q] + (d * p.C + ci) * 4) | ((unsigned)!ok << 31);
    } else if constexpr (MODE == SM_KOUT_DENSE) {
      const int k = kt * SBK + sub[q];
      const bool ok = mask[q] && k < K;
      return (base[q] + (unsigned)k * (unsigned)ld * 4u) | ((unsigned)!ok << 31);
    } else if constexpr (MODE == SM_KOUT_CONVG) {  // row k = output pixel (n, i, j) of the Ho x Wo grid
      const int k = kt * SBK + sub[q];
      int n, i, j;
      s_nhw(k, p, n, i, j);
      const int si = p.stride * i + dy[q], sj = p.stride * j + dx[q];
      const bool ok = mask[q] && k < K && (unsigned)si < (unsigned)p.H && (unsigned)sj < (unsigned)p.W;
      return (unsigned)(((n * p.H + si) * p.W + sj) * p.C * 4 + (int)base[q]) | ((unsigned)!ok << 31);
    } else {  // SM_KOUT_CONV: row k = pixel, column chunk = 4 channels of one tap
      const int k = kt * SBK + sub[q];
      const int qq = (int)(((float)k + 0.5f) * p.invW);
      const int w = k - qq * p.W;
      const int n = (int)(((float)qq + 0.5f) * p.invH);
      const int h = qq - n * p.H;
      const bool ok = mask[q] && k < K && (unsigned)(h + dy[q]) < (unsigned)p.H && (unsigned)(w + dx[q]) < (unsigned)p.W;
      return ((unsigned)(k + dyx[q]) * (unsigned)p.C * 4u + base[q]) | ((unsigned)!ok << 31);
    }
  }

  // live = false: every lane DMAs zeros (keeps the issue code branch-free at the end of the K loop)
  RK_DEV void issue(const SgParams& p, char* tile, int kt, int K, int ld, int wid, bool live = true) const {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      char* dst = tile + (wid * NQ + q) * 1024;
      const unsigned off = offset(p, q, kt, K, ld) | ((unsigned)!live << 31);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)dst, 16, (int)off, 0, 0, 0);
    }
  }

  // fragment of 32 rows starting at r0 for k-group g: element e is k = 8g + 4h + e (h = lane >> 5)
  RK_DEV f32x4 frag(const char* tile, int r0, int g, int lane) const {
    const int h = lane >> 5;
    if constexpr (KIN) {
      const int r = r0 + (lane & 31);
      return *(const f32x4*)(tile + r * 128 + ((((2 * g + h) ^ ((r >> 1) & 7))) << 4));
    } else {
      const float* t = (const float*)tile + (8 * g + 4 * h) * T + r0 + (lane & 31);
      return f32x4{t[0], t[T], t[2 * T], t[3 * T]};
    }
  }

  // K-outer, two 32-row blocks at once with INTERLEAVED rows (block b, lane row r <-> tile row
  // r0 + 2r + b): one ds_read_b64 per k feeds both blocks, halving the LDS read instructions of the
  // weight-gradient operands.  The epilogue maps the rows back (s_epilogue PA / PB).
  RK_DEV void frag_pair(const char* tile, int r0, int g, int lane, f32x4& f0, f32x4& f1) const {
    const int h = lane >> 5;
    const float* t = (const float*)tile + (8 * g + 4 * h) * T + r0 + 2 * (lane & 31);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float2 v = *(const float2*)(t + e * T);
      f0[e] = v.x;
      f1[e] = v.y;
    }
  }
};

// fragment loads of one operand for one k-group: MI (or NI) 32-row blocks of the wave's slab
template <class OP, int NB>
RK_DEV void load_frags(const OP& op, const char* tile, int r0, int g, int lane, f32x4 (&f)[NB]) {
  if constexpr (!OP::KIN && NB == 2) {
    op.frag_pair(tile, r0, g, lane, f[0], f[1]);
  } else {
#pragma unroll
    for (int i = 0; i < NB; ++i) f[i] = op.frag(tile, r0 + i * 32, g, lane);
  }
}

// Scheduling pattern of one 8-deep k-group (NMF MFMAs): one MFMA, the NR LDS reads of the next
// group's fragments, then ND (MFMA, DMA) pairs, then the remaining MFMAs.
template <int NMF, int NR, int ND>
RK_DEV void s_group_sched() {
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  if constexpr (NR > 0) __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
  if constexpr (ND > 0) {
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      if (d + 1 < NMF) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
  }
  if constexpr (NMF - 1 - ND > 0) __builtin_amdgcn_sched_group_barrier(0x008, NMF - 1 - ND, 0);
  __builtin_amdgcn_sched_group_barrier(0x002, 256, 0);  // leftover VALU after the MFMAs
}

// Workgroup = WGM x WGN waves, each owning (32*MI) x (32*NI) outputs: block tile BM x BN.
template <int WGM, int WGN, int MI, int NI, int AM, int BMD, int NST, bool GRP = false, bool X6 = false>
__global__ __launch_bounds__(64 * WGM * WGN) void sgemm_kernel(const SgParams p) {
  constexpr bool GR = GRP || AM == SM_KIN_CONVG;  // grid = groups x splits x tiles
  constexpr int NW = WGM * WGN;
  constexpr int WMT = 32 * MI, WNT = 32 * NI;  // wave tile
  constexpr int BM = WGM * WMT, BN = WGN * WNT;
  constexpr int ABYTES = BM * 128, SB = (BM + BN) * 128;
  constexpr int L = (BM + BN) / (8 * NW);  // DMA wave-instructions per wave per K-tile
  __shared__ __attribute__((aligned(16))) char smem[NST * SB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid - (wid / WGN) * WGN;
  const int tilesN = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tilesN;
  // 1-D grid of tiles x splits; the XCD-aware remap deals each XCD a contiguous range of logical ids
  // ordered (split, tile), so the tiles that share a split's K range (the same dY / X pixel rows of a
  // weight gradient) run on one XCD and hit one L2
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  int grp = 0, rem = lin;
  if constexpr (GR) {
    const int per = (int)(gridDim.x / p.groups);
    grp = lin / per;
    rem = lin - grp * per;
  }
  const int split = rem / tiles;
  const int bid = rem - split * tiles;
  const int mt = bid / tilesN, nt = bid - mt * tilesN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk = (p.K + SBK - 1) / SBK;
  const int kt0 = split * p.ktPer;
  const int kt1 = min(nk, kt0 + p.ktPer);

  SOperand<AM, BM, NW> A;
  SOperand<BMD, BN, NW> B;
  if constexpr (GRP)
    A.init(p, p.A + grp * p.gstrideA, p.bytesA - (unsigned long long)(grp * p.gstrideA) * 4ull, p.lda, m0, p.M,
           wid, lane, grp);
  else
    A.init(p, p.A, p.bytesA, p.lda, m0, p.M, wid, lane, grp);
  if constexpr (GR)
    B.init(p, p.B + grp * p.gstrideB, p.bytesB - (unsigned long long)(grp * p.gstrideB) * 4ull, p.ldb, n0, p.N,
           wid, lane);
  else
    B.init(p, p.B, p.bytesB, p.ldb, n0, p.N, wid, lane);

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int kt, int st) {
    char* t = smem + st * SB;
    A.issue(p, t, kt, p.K, p.lda, wid);
    B.issue(p, t + ABYTES, kt, p.K, p.ldb, wid);
  };

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (kt0 + s < kt1) issue(kt0 + s, s);

  int st = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    // tile kt has landed once only the younger tiles' DMAs are outstanding
    if constexpr (NST == 3) {
      if (kt + 1 < kt1) s_wait_vmcnt<L>();
      else s_wait_vmcnt<0>();
    } else {
      s_wait_vmcnt<0>();
    }
    s_barrier_lds();  // every wave's DMA for tile kt is in LDS; done with tile kt-1
    const char* As = smem + st * SB;
    const char* Bs = As + ABYTES;
    const bool more = kt + NST - 1 < kt1;
    char* nxt = smem + (st == 0 ? NST - 1 : st - 1) * SB;  // stage of tile kt + NST - 1
    // Fragments are double-buffered in registers (group g+1 is read from LDS while group g's MFMAs
    // run) and the next tile's DMAs go out among the first group's MFMAs; the schedule is
    // pinned with sched_group_barrier (left alone, hipcc sinks the reads behind the MFMAs they should
    // overlap and clusters the DMA issue in front of them).
    constexpr int NMF = 4 * MI * NI;
    // LDS read instructions per group
    constexpr int RA = A.KIN ? MI : (MI == 2 ? 4 : 4 * MI), RB = B.KIN ? NI : (NI == 2 ? 4 : 4 * NI);
    constexpr int DA = BM / (8 * NW), DB = BN / (8 * NW);              // DMA instructions per wave
    if constexpr (X6) {
      // two 16-deep chunks per K-tile; chunk c = k-groups 2c, 2c+1: lane half h supplies
      // k = 16c + {4h..4h+3, 8+4h..8+4h+3} of A and B alike (the MFMA sums over matched k-slots)
#pragma unroll
      for (int c = 0; c < SBK / 16; ++c) {
        f32x4 a0[MI], a1[MI], b0[NI], b1[NI];
        load_frags(A, As, wm * WMT, 2 * c, lane, a0);
        load_frags(A, As, wm * WMT, 2 * c + 1, lane, a1);
        load_frags(B, Bs, wn * WNT, 2 * c, lane, b0);
        load_frags(B, Bs, wn * WNT, 2 * c + 1, lane, b1);
        if (c == 0) {
          A.issue(p, nxt, kt + NST - 1, p.K, p.lda, wid, more);
          B.issue(p, nxt + ABYTES, kt + NST - 1, p.K, p.ldb, wid, more);
        }
        bf16x8 ah[MI], am[MI], al[MI], bh[NI], bm[NI], bl[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) split3(a0[i], a1[i], ah[i], am[i], al[i]);
#pragma unroll
        for (int j = 0; j < NI; ++j) split3(b0[j], b1[j], bh[j], bm[j], bl[j]);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = mfma6(ah[i], am[i], al[i], bh[j], bm[j], bl[j], acc[i][j]);
      }
      st = st + 1 == NST ? 0 : st + 1;
      continue;
    }
    f32x4 a[2][MI], b[2][NI];
    load_frags(A, As, wm * WMT, 0, lane, a[0]);
    load_frags(B, Bs, wn * WNT, 0, lane, b[0]);
#pragma unroll
    for (int g = 0; g < SBK / 8; ++g) {
      const int cur = g & 1;
      if (g + 1 < SBK / 8) {
        load_frags(A, As, wm * WMT, g + 1, lane, a[cur ^ 1]);
        load_frags(B, Bs, wn * WNT, g + 1, lane, b[cur ^ 1]);
      }
      // the reads above may not sink below this group's MFMAs (that would collapse the two fragment
      // register sets into one and expose the LDS latency at every group boundary)
      __builtin_amdgcn_sched_barrier(0);
      // unconditional (zeros past the end: that stage is never read again) — no branch splits the
      // scheduling region
      // the next tile's DMAs go out in the first group, so they have (NST-1) whole K-tiles of MFMAs
      // to land (a 64x64 tile's K-tile is only 16 MFMAs = ~1k cycles per wave)
      if (g == 0) {
        A.issue(p, nxt, kt + NST - 1, p.K, p.lda, wid, more);
        B.issue(p, nxt + ABYTES, kt + NST - 1, p.K, p.ldb, wid, more);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cur][i][e], b[cur][j][e], acc[i][j], 0, 0, 0);
      // group schedule: MFMAs with one DMA (and its address VALU) after each of the first few
      if (g == 0) s_group_sched<NMF, 0, DA + DB>();
      __builtin_amdgcn_sched_barrier(0);
    }
    st = st + 1 == NST ? 0 : st + 1;
  }
  s_wait_vmcnt<0>();  // the trailing zero-DMAs land before the workgroup's LDS is released
  s_epilogue<MI, NI, !SOperand<AM, BM, NW>::KIN && MI == 2, !SOperand<BMD, BN, NW>::KIN && NI == 2,
             AM == SM_KIN_CONVG>(p, acc, m0 + wm * WMT, n0 + wn * WNT, lane, split, grp,
                                 GRP ? p.out + grp * p.gstrideO : p.out,
                                 GRP && p.bias ? p.bias + grp * p.gstrideBias : p.bias);
}

template <int WGM, int WGN, int MI, int NI, int AM, int BMD, bool GRP = false>
int s_launch(const SgParams& p, int nst, int splits, hipStream_t st, bool x6) {
  constexpr int BM = WGM * 32 * MI, BN = WGN * 32 * NI;
  const int tiles = rk_cdiv(p.M, BM) * rk_cdiv(p.N, BN);
  dim3 grid(tiles * splits * ((GRP || AM == SM_KIN_CONVG) ? p.groups : 1));
  if (nst == 3) {
    if constexpr (WGM * WGN == 4) {  // 3-stage rings only for the 4-wave tiles (8-wave ones fill LDS at 2)
      if (x6)
        hipLaunchKernelGGL((sgemm_kernel<WGM, WGN, MI, NI, AM, BMD, 3, GRP, true>), grid, dim3(64 * WGM * WGN), 0, st, p);
      else
        hipLaunchKernelGGL((sgemm_kernel<WGM, WGN, MI, NI, AM, BMD, 3, GRP>), grid, dim3(64 * WGM * WGN), 0, st, p);
    } else {
      return RK_EUNSUPPORTED;
    }
  } else if (x6) {
    hipLaunchKernelGGL((sgemm_kernel<WGM, WGN, MI, NI, AM, BMD, 2, GRP, true>), grid, dim3(64 * WGM * WGN), 0, st, p);
  } else {
    hipLaunchKernelGGL((sgemm_kernel<WGM, WGN, MI, NI, AM, BMD, 2, GRP>), grid, dim3(64 * WGM * WGN), 0, st, p);
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// tile codes (block tile, waves): 0 128x128 (2x2), 1 128x64 (2x2), 2 64x128 (2x2), 3 64x64 (2x2),
// 4 256x64 (4x1), 5 256x128 (4x2, 512 threads), 6 128x256 (2x4, 512 threads), 7 64x256 (1x4).
// BIG = false instantiates only tiles 0-3 (dense layers, the general conv gather).
template <int AM, int BMD, bool BIG, bool GRP = false>
int s_launch_tile(int tile, const SgParams& p, int nst, int splits, hipStream_t st) {
  const bool x6 = tile >= 16;  // tile code + 16: the split-bf16 (X6) K loop
  switch (tile & 15) {
    case 0: return s_launch<2, 2, 2, 2, AM, BMD, GRP>(p, nst, splits, st, x6);
    case 1: return s_launch<2, 2, 2, 1, AM, BMD, GRP>(p, nst, splits, st, x6);
    case 2: return s_launch<2, 2, 1, 2, AM, BMD, GRP>(p, nst, splits, st, x6);
    case 3: return s_launch<2, 2, 1, 1, AM, BMD, GRP>(p, nst, splits, st, x6);
    // few-wave tiles with 64 x 64 wave tiles (twice the MFMAs per split fragment of the 2x2-wave
    // tiles: the X6 loop's split VALU per MFMA halves) for small grids of many groups
    case 8: return s_launch<1, 1, 2, 2, AM, BMD, GRP>(p, nst, splits, st, x6);
    case 9: return s_launch<2, 1, 2, 2, AM, BMD, GRP>(p, nst, splits, st, x6);
    case 10: return s_launch<1, 2, 2, 2, AM, BMD, GRP>(p, nst, splits, st, x6);
  }
  if constexpr (BIG) {
    switch (tile & 15) {
      case 4: return s_launch<4, 1, 2, 2, AM, BMD>(p, nst, splits, st, x6);
      case 5: return s_launch<4, 2, 2, 2, AM, BMD>(p, nst, splits, st, x6);
      case 6: return s_launch<2, 4, 2, 2, AM, BMD>(p, nst, splits, st, x6);
      case 7: return s_launch<1, 4, 2, 2, AM, BMD>(p, nst, splits, st, x6);
    }
  }
  return RK_EUNSUPPORTED;
}

}  // namespace

// fp32 implicit GEMM.  kind: 0 conv forward (A = NHWC activation gathered per tap [M = pixels][K = taps*C],
// B = weights [N][K]; the data gradient is kind 0 on dy with rk_swt-transposed weights), 2 conv weight
// gradient (A = dy [K = pixels][M = Cout] K-outer, B = x gathered [K = pixels][N = taps*C]),
// 3 dense A·Bᵀ (A [M][K], B [N][K]), 4 dense dX A·B (A [M][K], B [K][N]), 5 dense dW Aᵀ·B
// (A [K][M], B [K][N]).  tile: 0 128x128, 1 128x64, 2 64x128, 3 64x64 (2x2 waves), 8 64x64 (1 wave),
// 9 128x64 (2x1), 10 64x128 (1x2); +16: the X6 split-bf16 K loop.
// nst: LDS ring stages (2, 3).
// splits > 1: fp32 slabs out + split * slabStride (combine with rk_reduce_slabs / rk_sreduce_epi).
// flags: SF_* above; stats = fp64 slots [slotMask+1][2][N] (zeroed by the caller).
extern "C" int rk_sgemm(int kind, int tile, int nst, const float* A, const float* B, float* C, const float* bias,
                        double* stats, int slotMask, const float* gate, int M, int N, int K, int lda, int ldb,
                        int ldc, int H, int W, int Cch, int taps, int splits, long long slabStride, int flags,
                        float alpha, float slope, long long bytesA, long long bytesB, void* stream) {
  if (bytesA <= 0 || bytesB <= 0 || bytesA >= (1ll << 31) || bytesB >= (1ll << 31)) return RK_EUNSUPPORTED;
  if (M <= 0 || N <= 0 || K <= 0 || splits <= 0 || (nst != 2 && nst != 3) || tile < 0 || (tile & 15) > 10 ||
      tile > 26)
    return RK_EBADARG;
  if (taps != 1 && taps != 9) return RK_EBADARG;
  const bool conv = kind == 0 || kind == 2;
  // 16-B chunks: K-inner operands need K % 4 == 0 (and 16-B aligned rows); K-outer ones need the
  // non-reduction extent % 4 == 0
  if (kind == 0 || kind == 3 || kind == 4) {
    if (K % 4 || lda % 4) return RK_EUNSUPPORTED;
  }
  if ((kind == 0 || kind == 3) && ldb % 4) return RK_EUNSUPPORTED;
  if ((kind == 4 || kind == 5 || kind == 2) && (N % 4 || ldb % 4)) return RK_EUNSUPPORTED;
  if ((kind == 5 || kind == 2) && (M % 4 || lda % 4)) return RK_EUNSUPPORTED;
  if (conv && (Cch % 4 || Cch <= 0 || H <= 0 || W <= 0)) return RK_EUNSUPPORTED;
  if (splits > 1 && (flags & (SF_BIAS | SF_RELU | SF_LRELU | SF_GATE | SF_STATS | SF_BNB | SF_BNP)))
    return RK_EBADARG;  // split-K writes raw partial slabs
  SgParams p{};
  p.A = A; p.B = B; p.out = C; p.bias = bias; p.stats = stats; p.gate = gate;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.H = H; p.W = W; p.C = Cch; p.taps = taps;
  p.log2H = rk_log2(H); p.log2W = rk_log2(W); p.log2C = rk_log2(Cch);
  p.invC = 1.0f / (float)Cch; p.invH = 1.0f / (float)H; p.invW = 1.0f / (float)W;
  // reciprocal decodes are exact below 2^22 (pixel indices, tap*C column indices)
  if (conv && (p.log2H < 0 || p.log2W < 0) && (long long)(kind == 2 ? K : M) + (long long)W * (H + 2) >= (1ll << 22))
    return RK_EUNSUPPORTED;
  if ((flags & SF_BNP) && (p.log2H < 0 || p.log2W < 0 || !gate || !bias || !stats)) return RK_EUNSUPPORTED;
  if ((flags & (SF_STATS | SF_BNB)) && !stats) return RK_EBADARG;
  p.ktPer = rk_cdiv(rk_cdiv(K, SBK), splits);
  p.slabStride = splits > 1 ? slabStride : 0;
  p.flags = flags; p.slotMask = slotMask; p.alpha = alpha; p.slope = slope;
  p.bytesA = (unsigned long long)bytesA; p.bytesB = (unsigned long long)bytesB;
  p.groups = 1;
  p.Ho = H; p.Wo = W; p.log2Ho = p.log2H; p.log2Wo = p.log2W; p.invHo = p.invH; p.invWo = p.invW;
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case 0:
      if (Cch % SBK == 0) return s_launch_tile<SM_KIN_CONVF, SM_KIN_DENSE, true>(tile, p, nst, splits, st);
      return s_launch_tile<SM_KIN_CONV, SM_KIN_DENSE, false>(tile, p, nst, splits, st);
    case 2: return s_launch_tile<SM_KOUT_DENSE, SM_KOUT_CONV, true>(tile, p, nst, splits, st);
    case 3: return s_launch_tile<SM_KIN_DENSE, SM_KIN_DENSE, false>(tile, p, nst, splits, st);
    case 4: return s_launch_tile<SM_KIN_DENSE, SM_KOUT_DENSE, false>(tile, p, nst, splits, st);
    case 5: return s_launch_tile<SM_KOUT_DENSE, SM_KOUT_DENSE, false>(tile, p, nst, splits, st);
  }
  return RK_EBADARG;
}

// Table-driven gathers (the PG-GAN resampling convolutions).
// kind 6 — forward: out[row][n] = sum_{t, c} B_g[n][t*C + c] * A[src_t(row)][c] over `groups` parity
//   groups (grid groups x splits x tiles); rows = pixels (b, i, j) of the Ho x Wo grid, source pixel
//   (stride*i + dy_t, stride*j + dx_t) of the H x W input (zero outside), B_g = B + g * gstrideB
//   ([N][ntaps*C]).  os == 2: group g writes output pixel (2i + oy_g, 2j + ox_g) of a 2Ho x 2Wo map.
// kind 7 — weight gradient: out[m][t*C + c] = sum_rows A[row][m] * X[src_t(row)][c] (A = dY [rows][M],
//   X = the gathered input), one group.
// tpy / tpx: per group, 2-bit tap offsets (value + 1); oyx: per group 2 bits (oy, ox).
extern "C" int rk_sgemm_g(int kind, int tile, int nst, const float* A, const float* B, float* C, const float* bias,
                          int M, int N, int K, int lda, int ldb, int ldc, int H, int W, int Cch, int Ho, int Wo,
                          int stride, int ntaps, int groups, const unsigned* tpy, const unsigned* tpx, unsigned oyx,
                          int os, long long gstrideB, int splits, long long slabStride, int flags, float alpha,
                          float slope, long long bytesA, long long bytesB, void* stream) {
  if (kind != 6 && kind != 7) return RK_EBADARG;
  if (bytesA <= 0 || bytesB <= 0 || bytesA >= (1ll << 31) || bytesB >= (1ll << 31)) return RK_EUNSUPPORTED;
  if (M <= 0 || N <= 0 || K <= 0 || splits <= 0 || (nst != 2 && nst != 3) || tile < 0 ||
      ((tile & 15) > 3 && (tile & 15) < 8) || (tile & 15) > 10 || tile > 26)
    return RK_EBADARG;
  if (ntaps < 1 || ntaps > 16 || groups < 1 || groups > 4 || (stride != 1 && stride != 2) || (os != 1 && os != 2))
    return RK_EBADARG;
  if (kind == 7 && groups != 1) return RK_EBADARG;
  if (Cch % 4 || Cch <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return RK_EUNSUPPORTED;
  if ((kind == 6 ? K : N) != ntaps * Cch) return RK_EBADARG;
  if (kind == 6 && (lda % 4 || ldb % 4)) return RK_EUNSUPPORTED;
  if (kind == 7 && (N % 4 || M % 4 || lda % 4)) return RK_EUNSUPPORTED;
  if (splits > 1 && (flags & (SF_BIAS | SF_RELU | SF_LRELU | SF_GATE | SF_STATS | SF_BNB | SF_BNP))) return RK_EBADARG;
  if (flags & (SF_GATE | SF_STATS | SF_BNB | SF_BNP)) return RK_EUNSUPPORTED;
  // reciprocal decodes are exact below 2^22
  const long long rows = kind == 6 ? M : K;
  if (rows + (long long)W * (H + 2) >= (1ll << 22) || (long long)ntaps * Cch >= (1ll << 22)) return RK_EUNSUPPORTED;
  SgParams p{};
  p.A = A; p.B = B; p.out = C; p.bias = bias;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.H = H; p.W = W; p.C = Cch; p.taps = ntaps;
  p.log2H = rk_log2(H); p.log2W = rk_log2(W); p.log2C = rk_log2(Cch);
  p.invC = 1.0f / (float)Cch; p.invH = 1.0f / (float)H; p.invW = 1.0f / (float)W;
  p.Ho = Ho; p.Wo = Wo; p.log2Ho = rk_log2(Ho); p.log2Wo = rk_log2(Wo);
  p.invHo = 1.0f / (float)Ho; p.invWo = 1.0f / (float)Wo;
  p.stride = stride; p.ntaps = ntaps; p.groups = groups; p.os = os; p.oyx = oyx; p.gstrideB = gstrideB;
  for (int g = 0; g < 4; ++g) {
    p.tpy[g] = g < groups ? tpy[g] : 0u;
    p.tpx[g] = g < groups ? tpx[g] : 0u;
  }
  p.ktPer = rk_cdiv(rk_cdiv(K, SBK), splits);
  p.slabStride = splits > 1 ? slabStride : 0;
  p.flags = flags; p.alpha = alpha; p.slope = slope;
  p.bytesA = (unsigned long long)bytesA; p.bytesB = (unsigned long long)bytesB;
  hipStream_t st = (hipStream_t)stream;
  if (kind == 6) return s_launch_tile<SM_KIN_CONVG, SM_KIN_DENSE, false>(tile, p, nst, splits, st);
  return s_launch_tile<SM_KOUT_DENSE, SM_KOUT_CONVG, false>(tile, p, nst, splits, st);
}

// Grouped GEMMs: `groups` same-shape problems in ONE launch (grid groups x splits x tiles) — the k models
// of an inference ensemble run each layer as one kernel.  Group g reads A + g*gstrideA (0: a shared
// input, e.g. the request batch), B + g*gstrideB, writes out + g*gstrideO and uses bias + g*gstrideBias.
// kind 0 (conv forward) and 3 (dense A.B^T); flags: bias / ReLU / leaky-ReLU (no statistics).
// bytesA / bytesB cover every group's operand.
extern "C" int rk_sgemm_grp(int kind, int tile, int nst, const float* A, const float* B, float* C, const float* bias,
                            int M, int N, int K, int lda, int ldb, int ldc, int H, int W, int Cch, int taps, int splits,
                            long long slabStride, int flags, float alpha, float slope, long long bytesA,
                            long long bytesB, int groups, long long gstrideA, long long gstrideB, long long gstrideO,
                            long long gstrideBias, void* stream) {
  if (kind != 0 && kind != 3) return RK_EBADARG;
  if (bytesA <= 0 || bytesB <= 0 || bytesA >= (1ll << 31) || bytesB >= (1ll << 31)) return RK_EUNSUPPORTED;
  if (M <= 0 || N <= 0 || K <= 0 || splits <= 0 || (nst != 2 && nst != 3) || tile < 0 ||
      ((tile & 15) > 3 && (tile & 15) < 8) || (tile & 15) > 10 || tile > 26)
    return RK_EBADARG;
  if (groups < 1 || gstrideA < 0 || gstrideB < 0 || gstrideO < 0 || gstrideBias < 0) return RK_EBADARG;
  if (taps != 1 && taps != 9) return RK_EBADARG;
  if (K % 4 || lda % 4 || ldb % 4) return RK_EUNSUPPORTED;
  if (kind == 0 && (Cch % 4 || Cch <= 0 || H <= 0 || W <= 0)) return RK_EUNSUPPORTED;
  if (flags & ~(SF_BIAS | SF_RELU | SF_LRELU)) return RK_EUNSUPPORTED;
  if (splits > 1 && flags) return RK_EBADARG;
  SgParams p{};
  p.A = A; p.B = B; p.out = C; p.bias = bias;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.H = H; p.W = W; p.C = Cch; p.taps = taps;
  p.log2H = rk_log2(H); p.log2W = rk_log2(W); p.log2C = rk_log2(Cch);
  p.invC = 1.0f / (float)Cch; p.invH = 1.0f / (float)H; p.invW = 1.0f / (float)W;
  if (kind == 0 && (p.log2H < 0 || p.log2W < 0) && (long long)M + (long long)W * (H + 2) >= (1ll << 22))
    return RK_EUNSUPPORTED;
  p.ktPer = rk_cdiv(rk_cdiv(K, SBK), splits);
  p.slabStride = splits > 1 ? slabStride : 0;
  p.flags = flags; p.alpha = alpha; p.slope = slope;
  p.bytesA = (unsigned long long)bytesA; p.bytesB = (unsigned long long)bytesB;
  p.groups = groups; p.gstrideA = gstrideA; p.gstrideB = gstrideB; p.gstrideO = gstrideO; p.gstrideBias = gstrideBias;
  p.Ho = H; p.Wo = W; p.log2Ho = p.log2H; p.log2Wo = p.log2W; p.invHo = p.invH; p.invWo = p.invW;
  hipStream_t st = (hipStream_t)stream;
  if (kind == 3) return s_launch_tile<SM_KIN_DENSE, SM_KIN_DENSE, false, true>(tile, p, nst, splits, st);
  if (Cch % SBK == 0) return s_launch_tile<SM_KIN_CONVF, SM_KIN_DENSE, false, true>(tile, p, nst, splits, st);
  return s_launch_tile<SM_KIN_CONV, SM_KIN_DENSE, false, true>(tile, p, nst, splits, st);
}
