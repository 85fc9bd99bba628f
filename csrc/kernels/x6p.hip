// Pre-split X6 GEMMs for gfx950: C[g] = A[g] · B[g]^T (+ C[g]) with both operands ALREADY split into
// three bf16 planes, x = hi + mid + lo (split3v: each piece the round-to-nearest bf16 of the remaining
// residual), written once by their producers — the Winograd transforms of the pre-transformed F(4x4)
// convolutions (winograd4.hip: input windows, weights, weight-gradient patches) — instead of being
// re-split from fp32 after every LDS fragment read.  In the sgemm X6 loop (sgemm.hip) that split is
// ~90 VALU per 16-deep chunk and 32x32 block pair against 6 MFMAs: the loop ran VALU-bound at 21%
// MfmaUtil (profiles/vgg_small_f32_step_pmc_r3k.txt).  Here the K loop is LDS reads + MFMAs only:
// per 16-deep chunk a wave reads 3 (planes) x MI + 3 x NI bf16x8 fragments and issues 6 MI NI
// v_mfma_f32_32x32x16_bf16 — hi·hi, hi·mid, mid·hi, hi·lo, lo·hi, mid·mid (mfma6, small terms first) —
// into fp32 accumulators: products exact to below fp32's unit roundoff, 6/16 of the f32 MFMA cycles.
//
// Operands are K-inner (K contiguous), plane-major per group: A planes at A + g*gsA + p*psA, rows of
// lda bf16 ([M][K] each); B likewise ([N][K]).  K % 32 == 0 (one 32-deep K-tile = a 64-B row per plane).
//   * global -> LDS by buffer_load_dword x4 ... lds (no VGPR staging): one wave-instruction moves 16
//     plane rows of one K-tile (1 KiB); the 16-B chunks of a 64-B row are XOR-swizzled by (row >> 2) & 3,
//     which makes the ds_read_b128 fragment reads conflict-free for its 16-lane groups;
//   * NST-stage LDS ring (2 or 3), one barrier per K-tile, counted vmcnt; the next tile's DMAs issue
//     among the first chunk's MFMAs;
//   * out-of-range rows (M / N edges) DMA zeros through the buffer range check; the epilogue masks them;
//   * block = WGM x WGN waves, wave tile (32 MI) x (32 NI); the grid is groups x tiles with the
//     XCD-aware remap (a group's tiles share their A / B panels in one XCD's L2).
#include "common.h"
#include <cstdlib>
#include <utility>

namespace {

#include "sgemm_core.h"

constexpr int XBK = 32;   // K granularity: K % 32 == 0; a K-tile is KT = 32 or 64 deep (64- or 128-B plane rows)

struct XpParams {
  const bf16* A;
  const bf16* B;
  float* C;
  int M, N, K;
  int lda, ldb, ldc;            // elements
  long long psA, psB;           // plane strides (elements)
  long long gsA, gsB, gsC;      // group strides (elements)
  int groups, flags;            // flags: 1 = accumulate into C
  int splits, ktPer;            // split-K: split s covers K-tiles [s ktPer, (s+1) ktPer), writes slab s
  long long slabStride;         // elements between split-K slabs of C
  unsigned long long bytesA, bytesB;
};

// chunk position of logical 16-B chunk c of LDS row r: conflict-free ds_read_b128 for the 16-lane groups of
// 32 consecutive rows (64-B rows: 4 chunks, 128-B rows: 8)
template <int KT>
RK_DEV int xswz(int r) { return KT == 32 ? (r >> 2) & 3 : (r >> 1) & 7; }

// One operand: T rows x 3 planes x KT k per K-tile; one DMA wave-instruction moves 1 KiB = 1024 / (2 KT)
// plane rows (16 or 8: whole 64- / 128-B pieces of the row), 3 T 2 KT / 1024 instructions per K-tile.
template <int T, int NW, int KT>
struct XOp {
  static constexpr int RB = 2 * KT;          // bytes per plane row per K-tile
  static constexpr int RPI = 1024 / RB;      // rows per DMA wave-instruction
  static constexpr int PI = T / RPI;         // wave-instructions per plane
  static constexpr int NQ = 3 * PI / NW;     // per wave
  static constexpr int CPR = RB / 16;        // 16-B chunks per row
  static_assert(NQ >= 1 && NQ * NW == 3 * PI, "operand tile must split evenly over the waves");
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned off[NQ];

  RK_DEV void init(const bf16* base, unsigned long long bytes, int ld, long long ps, int row0, int extent, int wid,
                   int lane) {
    rsrc = s_rsrc(base, bytes);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = wid * NQ + q;
      const int plane = idx / PI;
      const int r = (idx - plane * PI) * RPI + lane / CPR;   // LDS slot lane*16 B: row r, position lane % CPR
      const int c = (lane % CPR) ^ xswz<KT>(r);              // logical chunk stored at that position
      const int gr = row0 + r;
      off[q] = gr < extent ? (unsigned)((plane * ps + (long long)gr * ld + c * 8) * 2) : SOOB;
    }
  }

  // live = false: zeros (keeps the issue code branch-free at the end of the K loop)
  RK_DEV void issue(char* tile, int kt, int wid, bool live) const {
#pragma unroll
    for (int q = 0; q < NQ; ++q) issue_q(tile, kt, wid, live, q);
  }
  // one DMA wave-instruction (1 KiB) of this wave's share
  RK_DEV void issue_q(char* tile, int kt, int wid, bool live, int q) const {
    const unsigned o = (off[q] + (unsigned)kt * (unsigned)RB) | ((unsigned)!live << 31);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(tile + (wid * NQ + q) * 1024), 16, (int)o, 0, 0, 0);
  }

  // plane p, rows r0 .. r0+31, 16-deep chunk cc of the K-tile: lane (r, h) holds k = 16 cc + 8 h + j
  RK_DEV bf16x8 frag(const char* tile, int p, int r0, int cc, int lane) const {
    const int r = r0 + (lane & 31);
    const int c = 2 * cc + (lane >> 5);
    return *(const bf16x8*)(tile + p * (T * RB) + r * RB + ((c ^ xswz<KT>(r)) << 4));
  }
};

// Schedule of one 16-deep chunk: NM MFMAs; the NR LDS reads of the next chunk's fragments go out one per
// MFMA from the first; the NV DMA pieces of a later K-tile are spread evenly among the MFMAs (an LDS-DMA
// wave-instruction costs ~60 issue cycles, two MFMA slots: issued in a cluster in front of the MFMAs they
// left the matrix core idle for L x 60 cycles per K-tile)
template <class F, int... I>
RK_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
RK_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int NM, int NR, int NV>
RK_DEV void xp_sched() {
  static_assert(NR <= NM, "one fragment read per MFMA slot");
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (m < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    if ((m + 1) * NV / NM > m * NV / NM) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
  }
}

// Epilogue of one wave tile: register r of 32x32 block (i, j) is row acc_row(r, h), column lane & 31.  Buffer
// stores with one VGPR offset per store (no 64-bit address math or per-element branches): rows >= M fall past
// the group slab's range and are dropped by the buffer range check; columns >= N get an out-of-range offset.
template <int MI, int NI>
RK_DEV void xp_store(const XpParams& p, f32x16 (&acc)[MI][NI], int grp, int split, int mw, int nw, int lane) {
  float* C = p.C + grp * p.gsC + split * p.slabStride;
  const __amdgpu_buffer_rsrc_t rs = s_rsrc(C, (unsigned long long)p.M * p.ldc * 4);
  const int h = lane >> 5;
  const bool acc_in = p.flags & 1;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int n = nw + j * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const unsigned base = n < p.N ? (unsigned)(((mw + i * 32 + 4 * h) * p.ldc + n) * 4) : SOOB;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const unsigned o = base + (unsigned)(((r & 3) + 8 * (r >> 2)) * p.ldc * 4);
        float v = acc[i][j][r];
        if (acc_in) v += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)o, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, (int)o, 0, 0);
      }
    }
  }
}

template <int WGM, int WGN, int MI, int NI, int NST, int KT>
__global__ __launch_bounds__(64 * WGM * WGN) void x6p_gemm_kernel(const XpParams p) {
  constexpr int NW = WGM * WGN;
  constexpr int BM = WGM * 32 * MI, BN = WGN * 32 * NI;
  constexpr int ABYTES = 3 * BM * 2 * KT, SB = 3 * (BM + BN) * 2 * KT;
  constexpr int L = XOp<BM, NW, KT>::NQ + XOp<BN, NW, KT>::NQ;   // DMA wave-instructions per wave per K-tile
  __shared__ __attribute__((aligned(16))) char smem[NST * SB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid - (wid / WGN) * WGN;
  const int tilesN = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tilesN;
  // grid = groups x splits x tiles; the XCD-aware remap gives each XCD a contiguous range of (group, split)
  // tile sets, so the tiles sharing one group's A / B panels run on one XCD and hit one L2
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int gs = lin / tiles, bid = lin - gs * tiles;
  const int grp = gs / p.splits, split = gs - grp * p.splits;
  const int mt = bid / tilesN, nt = bid - mt * tilesN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kt0 = split * p.ktPer;
  const int nk = min(p.K / KT - kt0, p.ktPer);   // K-tiles of this split (>= 1: the launcher checks)

  XOp<BM, NW, KT> A;
  XOp<BN, NW, KT> B;
  const unsigned long long ka = 2ull * (unsigned long long)kt0 * KT;   // the split's first K-tile, bytes
  A.init(p.A + grp * p.gsA + kt0 * KT, p.bytesA - 2ull * (unsigned long long)(grp * p.gsA) - ka, p.lda, p.psA,
         m0, p.M, wid, lane);
  B.init(p.B + grp * p.gsB + kt0 * KT, p.bytesB - 2ull * (unsigned long long)(grp * p.gsB) - ka, p.ldb, p.psB,
         n0, p.N, wid, lane);

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) {
    if (s < nk) {
      A.issue(smem + s * SB, s, wid, true);
      B.issue(smem + s * SB + ABYTES, s, wid, true);
    }
  }

  constexpr int NC = KT / 16;                 // 16-deep chunks per K-tile
  constexpr int LA = XOp<BM, NW, KT>::NQ;
  constexpr int NM = 6 * MI * NI;             // MFMAs per chunk
  constexpr int NR = 3 * (MI + NI);           // fragment reads per chunk
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt has landed once only the younger tiles' DMAs are outstanding
    if constexpr (NST == 3) {
      if (kt + 1 < nk) s_wait_vmcnt<L>();
      else s_wait_vmcnt<0>();
    } else {
      s_wait_vmcnt<0>();
    }
    s_barrier_lds();   // every wave's DMA for tile kt is in LDS; every wave is done with tile kt-1
    const char* As = smem + st * SB;
    const char* Bs = As + ABYTES;
    const bool more = kt + NST - 1 < nk;
    char* nxt = smem + (st == 0 ? NST - 1 : st - 1) * SB;   // stage of tile kt + NST - 1
    // fragments double-buffered in registers: chunk c+1's are read while chunk c's MFMAs run; the DMA
    // pieces of tile kt + NST - 1 are spread over the tile's chunks and interleaved with the MFMAs
    bf16x8 fa[2][3][MI], fb[2][3][NI];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[0][pl][i] = A.frag(As, pl, wm * 32 * MI + i * 32, 0, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[0][pl][j] = B.frag(Bs, pl, wn * 32 * NI + j * 32, 0, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for<NC>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      constexpr int cur = c & 1, nx = cur ^ 1;
      if constexpr (c + 1 < NC) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
          for (int i = 0; i < MI; ++i) fa[nx][pl][i] = A.frag(As, pl, wm * 32 * MI + i * 32, c + 1, lane);
#pragma unroll
          for (int j = 0; j < NI; ++j) fb[nx][pl][j] = B.frag(Bs, pl, wn * 32 * NI + j * 32, c + 1, lane);
        }
      }
#pragma unroll
      for (int q = L * c / NC; q < L * (c + 1) / NC; ++q) {
        if (q < LA) A.issue_q(nxt, kt + NST - 1, wid, more, q);
        else B.issue_q(nxt + ABYTES, kt + NST - 1, wid, more, q - LA);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = mfma6(fa[cur][0][i], fa[cur][1][i], fa[cur][2][i], fb[cur][0][j], fb[cur][1][j],
                            fb[cur][2][j], acc[i][j]);
      xp_sched<NM, (c + 1 < NC ? NR : 0), L * (c + 1) / NC - L * c / NC>();
      __builtin_amdgcn_sched_barrier(0);
    });
    st = st + 1 == NST ? 0 : st + 1;
  }
  s_wait_vmcnt<0>();   // the trailing zero-DMAs land before the workgroup's LDS is released

  xp_store<MI, NI>(p, acc, grp, split, m0 + wm * 32 * MI, n0 + wn * 32 * NI, lane);
}

// Warp-specialised variant: 2 x 2 compute waves (wave tile 32 MI x 32 NI) that only read fragments and
// issue MFMAs, plus 4 loader waves that only issue the LDS-DMA pieces.  An LDS-DMA wave-instruction costs
// its issuing wave ~60-185 cycles; issued by the compute waves (x6p_gemm_kernel) those cycles come out of
// the MFMA stream (every tile shape measured at 25-30 % of the X6 peak).  Here a loader wave on each SIMD
// issues while the compute wave beside it keeps the matrix core busy.  Per K-tile: loaders wait for
// their pieces of tile kt, one workgroup barrier (tile kt landed; every compute wave is done with tile
// kt-1), then the loaders issue tile kt+NST-1 into the freed stage while the compute waves consume kt.
template <int MI, int NI, int NST, int KT>
__global__ __launch_bounds__(512) void x6p_ws_kernel(const XpParams p) {
  constexpr int BM = 64 * MI, BN = 64 * NI;
  constexpr int ABYTES = 3 * BM * 2 * KT, SB = 3 * (BM + BN) * 2 * KT;
  using OA = XOp<BM, 4, KT>;
  using OB = XOp<BN, 4, KT>;
  constexpr int L = OA::NQ + OB::NQ;   // DMA pieces per loader wave per K-tile
  static_assert(L <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[NST * SB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = wv >= 4;
  const int wid = loader ? wv - 4 : wv;
  const int wm = wid >> 1, wn = wid & 1;
  const int tilesN = (p.N + BN - 1) / BN;
  const int tiles = ((p.M + BM - 1) / BM) * tilesN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int gs = lin / tiles, bid = lin - gs * tiles;
  const int grp = gs / p.splits, split = gs - grp * p.splits;
  const int mt = bid / tilesN, nt = bid - mt * tilesN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kt0 = split * p.ktPer;
  const int nk = min(p.K / KT - kt0, p.ktPer);

  if (loader) {
    OA A;
    OB B;
    const unsigned long long ka = 2ull * (unsigned long long)kt0 * KT;
    A.init(p.A + grp * p.gsA + kt0 * KT, p.bytesA - 2ull * (unsigned long long)(grp * p.gsA) - ka, p.lda, p.psA, m0,
           p.M, wid, lane);
    B.init(p.B + grp * p.gsB + kt0 * KT, p.bytesB - 2ull * (unsigned long long)(grp * p.gsB) - ka, p.ldb, p.psB, n0,
           p.N, wid, lane);
#pragma unroll
    for (int s = 0; s < NST - 1; ++s) {
      if (s < nk) {
        A.issue(smem + s * SB, s, wid, true);
        B.issue(smem + s * SB + ABYTES, s, wid, true);
      }
    }
    int st = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if constexpr (NST == 3) {
        if (kt + 1 < nk) s_wait_vmcnt<L>();
        else s_wait_vmcnt<0>();
      } else {
        s_wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + NST - 1 < nk) {
        char* nxt = smem + (st == 0 ? NST - 1 : st - 1) * SB;
        A.issue(nxt, kt + NST - 1, wid, true);
        B.issue(nxt + ABYTES, kt + NST - 1, wid, true);
      }
      st = st + 1 == NST ? 0 : st + 1;
    }
    return;
  }

  OA A;   // fragment addressing only (the compute waves issue no DMA)
  OB B;
  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  constexpr int NC = KT / 16;
  constexpr int NM = 6 * MI * NI;
  constexpr int NR = 3 * (MI + NI);
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    s_barrier_lds();   // tile kt is in LDS; every compute wave is done reading tile kt-1
    const char* As = smem + st * SB;
    const char* Bs = As + ABYTES;
    bf16x8 fa[2][3][MI], fb[2][3][NI];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[0][pl][i] = A.frag(As, pl, wm * 32 * MI + i * 32, 0, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[0][pl][j] = B.frag(Bs, pl, wn * 32 * NI + j * 32, 0, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for<NC>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      constexpr int cur = c & 1, nx = cur ^ 1;
      if constexpr (c + 1 < NC) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
          for (int i = 0; i < MI; ++i) fa[nx][pl][i] = A.frag(As, pl, wm * 32 * MI + i * 32, c + 1, lane);
#pragma unroll
          for (int j = 0; j < NI; ++j) fb[nx][pl][j] = B.frag(Bs, pl, wn * 32 * NI + j * 32, c + 1, lane);
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = mfma6(fa[cur][0][i], fa[cur][1][i], fa[cur][2][i], fb[cur][0][j], fb[cur][1][j], fb[cur][2][j],
                            acc[i][j]);
      xp_sched<NM, (c + 1 < NC ? NR : 0), 0>();
      __builtin_amdgcn_sched_barrier(0);
    });
    st = st + 1 == NST ? 0 : st + 1;
  }

  xp_store<MI, NI>(p, acc, grp, split, m0 + wm * 32 * MI, n0 + wn * 32 * NI, lane);
}

template <int MI, int NI, int KT>
int ws_launch(const XpParams& p, int nst, hipStream_t st) {
  constexpr int BM = 64 * MI, BN = 64 * NI;
  constexpr int SB = 3 * (BM + BN) * 2 * KT;
  const long long blocks = (long long)rk_cdiv(p.M, BM) * rk_cdiv(p.N, BN) * p.groups * p.splits;
  if (blocks >= (1ll << 31)) return RK_EUNSUPPORTED;
  const dim3 grid((unsigned)blocks), block(512);
  if (nst == 3) {
    if constexpr (3 * SB <= 163840)
      hipLaunchKernelGGL((x6p_ws_kernel<MI, NI, 3, KT>), grid, block, 0, st, p);
    else
      return RK_EUNSUPPORTED;
  } else {
    if constexpr (2 * SB <= 163840)
      hipLaunchKernelGGL((x6p_ws_kernel<MI, NI, 2, KT>), grid, block, 0, st, p);
    else
      return RK_EUNSUPPORTED;
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}

template <int MI, int NI>
int ws_launch_kt(const XpParams& p, int nst, int kt, hipStream_t st) {
  return kt == 64 ? ws_launch<MI, NI, 64>(p, nst, st) : ws_launch<MI, NI, 32>(p, nst, st);
}

template <int WGM, int WGN, int MI, int NI, int KT>
int xp_launch(const XpParams& p, int nst, hipStream_t st) {
  constexpr int BM = WGM * 32 * MI, BN = WGN * 32 * NI;
  constexpr int SB = 3 * (BM + BN) * 2 * KT;
  const long long blocks = (long long)rk_cdiv(p.M, BM) * rk_cdiv(p.N, BN) * p.groups * p.splits;
  if (blocks >= (1ll << 31)) return RK_EUNSUPPORTED;
  const dim3 grid((unsigned)blocks), block(64 * WGM * WGN);
  if (nst == 3) {
    if constexpr (3 * SB <= 163840)
      hipLaunchKernelGGL((x6p_gemm_kernel<WGM, WGN, MI, NI, 3, KT>), grid, block, 0, st, p);
    else
      return RK_EUNSUPPORTED;
  } else {
    if constexpr (2 * SB <= 163840)
      hipLaunchKernelGGL((x6p_gemm_kernel<WGM, WGN, MI, NI, 2, KT>), grid, block, 0, st, p);
    else
      return RK_EUNSUPPORTED;
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}

template <int WGM, int WGN, int MI, int NI>
int xp_launch_kt(const XpParams& p, int nst, int kt, hipStream_t st) {
  return kt == 64 ? xp_launch<WGM, WGN, MI, NI, 64>(p, nst, st) : xp_launch<WGM, WGN, MI, NI, 32>(p, nst, st);
}

// fp32 [rows][ld_src] -> three bf16 planes [3][rows][ld_dst] (columns >= cols are left untouched)
__global__ __launch_bounds__(256) void x6p_split_kernel(const float* __restrict__ src, bf16* __restrict__ dst,
                                                        int rows, int cols, int lds, int ldd, long long ps) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)rows * cols) return;
  const int r = (int)(i / cols), c = (int)(i - (long long)r * cols);
  bf16 h, m, l;
  split3v(src[(long long)r * lds + c], h, m, l);
  const long long o = (long long)r * ldd + c;
  dst[o] = h;
  dst[o + ps] = m;
  dst[o + 2 * ps] = l;
}

// fp32 src [rows][lds] -> three bf16 planes [3][cols][ldd] of its TRANSPOSE (plane stride ps): the K-inner
// operand of a GEMM that reduces over src's rows (the dense weight gradient dW = dY^T X reduces over the
// batch; the dense data gradient dX = dY W takes W^T).  The plane columns rows .. ldd-1 (the K padding to a
// 32-deep K-tile) are written as zeros.  64 x 64 tiles through LDS; each thread stores 4 consecutive plane
// elements per plane (8-B stores).
__global__ __launch_bounds__(256) void x6p_split_t_kernel(const float* __restrict__ src, bf16* __restrict__ dst,
                                                          int rows, int cols, int lds, int ldd, long long ps) {
  __shared__ float t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  const int lc = (tid & 15) * 4, lr = tid >> 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r0 + lr + 16 * k;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + lc + e;
      t[lr + 16 * k][lc + e] = (r < rows && c < cols) ? src[(long long)r * lds + c] : 0.f;
    }
  }
  __syncthreads();
  const int sr = (tid & 15) * 4, sc = tid >> 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + sc + 16 * k, r = r0 + sr;
    if (c >= cols || r >= ldd) continue;
    bf16 h[4], m[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) split3v(t[sr + e][sc + 16 * k], h[e], m[e], l[e]);
    const long long o = (long long)c * ldd + r;
    if (r + 3 < ldd) {   // ldd % 4 == 0: an aligned 8-B store per plane
      typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
      u16x4 vh, vm, vl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        vh[e] = __builtin_bit_cast(unsigned short, h[e]);
        vm[e] = __builtin_bit_cast(unsigned short, m[e]);
        vl[e] = __builtin_bit_cast(unsigned short, l[e]);
      }
      *(u16x4*)(dst + o) = vh;
      *(u16x4*)(dst + o + ps) = vm;
      *(u16x4*)(dst + o + 2 * ps) = vl;
    } else {
      for (int e = 0; e < 4 && r + e < ldd; ++e) {
        dst[o + e] = h[e];
        dst[o + e + ps] = m[e];
        dst[o + e + 2 * ps] = l[e];
      }
    }
  }
}

}  // namespace

// C[g] (+)= A[g] · B[g]^T for g < groups, A[g] planes [3][M][lda] (plane stride psA), B[g] planes
// [3][N][ldb]; fp32 C[g] [M][ldc].  tile: 0 128x128 (2x2 waves), 1 128x64, 2 64x128, 3 64x64 (2x2 waves),
// 4 64x64 (1 wave), 5 128x64 (2x1), 6 64x128 (1x2), 7 256x128 (4x2), 8 128x256 (2x4), 9-12 the
// warp-specialised 128x128, 128x64, 64x128, 64x64 (2x2 compute + 4 loader waves); nst: LDS ring stages
// (2, 3 where the LDS fits); tile + 16: 64-deep K-tiles (K % 64 == 0); flags 1: accumulate.  splits > 1: split-K, slab s of the output at
// C + s * slabStride (raw partial sums; the consumers add the slabs).
extern "C" int rk_x6p_gemm(int tile, int nst, const void* A, const void* B, float* C, int M, int N, int K, int lda,
                           int ldb, int ldc, long long psA, long long psB, long long gsA, long long gsB, long long gsC,
                           int groups, int flags, int splits, long long slabStride, long long bytesA, long long bytesB,
                           void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || groups <= 0 || (nst != 2 && nst != 3) || tile < 0 || (tile & 15) > 12 ||
      tile >= 32 || splits <= 0)
    return RK_EBADARG;
  if (splits > 1 && ((flags & 1) || slabStride < (long long)groups * gsC || slabStride < (long long)M * ldc))
    return RK_EBADARG;   // split-K writes raw partial slabs
  const int kt = (tile >> 4) ? 64 : 32;   // tile + 16: 64-deep K-tiles (128-B plane rows)
  tile &= 15;
  if (K % kt || lda % 8 || ldb % 8 || lda < K || ldb < K) return RK_EUNSUPPORTED;
  if (psA < (long long)M * lda || psB < (long long)N * ldb || bytesA <= 0 || bytesB <= 0) return RK_EBADARG;
  if ((long long)M * ldc * 4 >= (1ll << 31) || ldc < N) return RK_EUNSUPPORTED;   // 32-bit epilogue offsets
  // every in-group byte offset must stay below the 2 GiB buffer range
  if ((2 * psA + (long long)M * lda) * 2 >= (1ll << 31) || (2 * psB + (long long)N * ldb) * 2 >= (1ll << 31))
    return RK_EUNSUPPORTED;
  // gsA / gsB == 0: one operand shared by every group (broadcast)
  // group outputs: group-major (gsC >= M ldc) or row-interleaved (gsC >= N, ldc >= groups gsC, e.g. [M][G][N])
  if (groups > 1 && ((gsA && gsA < 3 * psA) || (gsB && gsB < 3 * psB) ||
                     (gsC < (long long)M * ldc && (gsC < N || ldc < (long long)groups * gsC))))
    return RK_EBADARG;
  if (2 * (gsA * (groups - 1) + 3 * psA) > bytesA || 2 * (gsB * (groups - 1) + 3 * psB) > bytesB) return RK_EBADARG;
  XpParams p;
  p.A = (const bf16*)A; p.B = (const bf16*)B; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.psA = psA; p.psB = psB; p.gsA = gsA; p.gsB = gsB; p.gsC = gsC;
  p.groups = groups; p.flags = flags;
  const int nk = K / kt;
  p.ktPer = rk_cdiv(nk, splits);
  p.splits = rk_cdiv(nk, p.ktPer);   // every split gets >= 1 K-tile
  if (p.splits != splits) return RK_EBADARG;
  p.slabStride = splits > 1 ? slabStride : 0;
  p.bytesA = (unsigned long long)bytesA; p.bytesB = (unsigned long long)bytesB;
  const hipStream_t st = (hipStream_t)stream;
  switch (tile) {
    case 0: return xp_launch_kt<2, 2, 2, 2>(p, nst, kt, st);
    case 1: return xp_launch_kt<2, 2, 2, 1>(p, nst, kt, st);
    case 2: return xp_launch_kt<2, 2, 1, 2>(p, nst, kt, st);
    case 3: return xp_launch_kt<2, 2, 1, 1>(p, nst, kt, st);
    case 4: return xp_launch_kt<1, 1, 2, 2>(p, nst, kt, st);
    case 5: return xp_launch_kt<2, 1, 2, 2>(p, nst, kt, st);
    case 6: return xp_launch_kt<1, 2, 2, 2>(p, nst, kt, st);
    // 8-wave tiles of 64x64 wave tiles (two waves per SIMD): NST 2 only (73.7 KiB per stage)
    case 7: return xp_launch_kt<4, 2, 2, 2>(p, nst, kt, st);
    case 8: return xp_launch_kt<2, 4, 2, 2>(p, nst, kt, st);
    // warp-specialised (4 compute + 4 loader waves): 9 128x128, 10 128x64, 11 64x128, 12 64x64
    case 9: return ws_launch_kt<2, 2>(p, nst, kt, st);
    case 10: return ws_launch_kt<2, 1>(p, nst, kt, st);
    case 11: return ws_launch_kt<1, 2>(p, nst, kt, st);
    case 12: return ws_launch_kt<1, 1>(p, nst, kt, st);
  }
  return RK_EBADARG;
}

// planes [3][rows][ldd] (plane stride ps) of an fp32 [rows][lds] matrix
extern "C" int rk_x6p_split(const float* src, void* dst, int rows, int cols, int lds, int ldd, long long ps,
                            void* stream) {
  if (rows <= 0 || cols <= 0 || lds < cols || ldd < cols || ps < (long long)rows * ldd) return RK_EBADARG;
  const long long n = (long long)rows * cols;
  hipLaunchKernelGGL(x6p_split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, src,
                     (bf16*)dst, rows, cols, lds, ldd, ps);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// planes [3][cols][ldd] (plane stride ps) of the transpose of an fp32 [rows][lds] matrix; plane columns
// rows .. ldd-1 zero; ldd % 4 == 0
extern "C" int rk_x6p_split_t(const float* src, void* dst, int rows, int cols, int lds, int ldd, long long ps,
                              void* stream) {
  if (rows <= 0 || cols <= 0 || lds < cols || ldd < rows || (ldd & 3) || ps < (long long)cols * ldd)
    return RK_EBADARG;
  const dim3 grid((unsigned)rk_cdiv(cols, 64), (unsigned)rk_cdiv(ldd, 64));
  hipLaunchKernelGGL(x6p_split_t_kernel, grid, dim3(256), 0, (hipStream_t)stream, src, (bf16*)dst, rows, cols, lds,
                     ldd, ps);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
