// Halo-tiled 3x3 convolution (stride 1, pad 1, NHWC fp32) with fp32-accurate products on the bf16
// matrix cores — the X6 scheme of sgemm_core.h: every fp32 operand value is three bf16 pieces
// (hi + mid + lo, round-to-nearest residuals) and a 16-deep k chunk is six
// v_mfma_f32_32x32x16_bf16 (hi*hi, hi*mid, mid*hi, hi*lo, lo*hi, mid*mid) into fp32 accumulators.
//
// Why a second conv kernel next to the implicit GEMM of sgemm.hip: that one gathers the activation
// once per tap, so every input pixel crosses L2 -> LDS nine times; once the products run at the bf16
// rate (6/16 of the f32 MFMA cycles) that gather traffic, not the matrix core, bounds it
// (profiles/x6_layers_r3.jsonl: 1.0-1.3x over the f32 loop).  Here a block owns BM output pixels
// (TH whole rows of one image, or IMG whole small images) x BN output channels; per 32-channel
// input chunk it DMAs ONE (TH+2) x (W+2) halo patch of fp32 activations into LDS and runs all nine
// taps out of it (the tap is a constant shift of the patch pixel a lane reads).  The weights are
// split ONCE per weight update by xconv_wt_kernel into bf16 planes [3][9][N][K] (K permuted inside
// each 16-group so a lane's eight k values are one 16-byte read) and stream per (tap, chunk) through
// a 3-stage LDS-DMA ring; the activation patch is split once per block and chunk (register-staged:
// loaded during the previous chunk's nine taps, split and written at the chunk boundary), so the
// tap loop is ds_read_b128 + MFMA only.  One barrier per tap.
//
// The data gradient is the same kernel on dy with the flipped, transposed weight planes (xconv_wt
// writes both sets), so the BN-backward epilogues (FLAG_BNB / FLAG_BNP) of sgemm_core.h apply as is.
// Reference parity: the fp32 conv2d of the reference's Keras / TF models (TfVgg16.py:115-130,
// pg_gans.py:998-1029 `conv2d`), same precision.
#include "common.h"

namespace {

#include "sgemm_core.h"

constexpr int XKC = 32;  // input channels per chunk (one 64-byte row per pixel and plane)
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

RK_DEV void x_dma16(__amdgpu_buffer_rsrc_t r, char* dst, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, off, 0, 0, 0);
}

template <int N>
RK_DEV void x_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

RK_DEV void x_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// IH > 0: an item is IMG whole IH x W images (small maps); IH == 0: TH = BM / W rows of one image
//
// LDS images (every ds_read_b128 conflict-free for the four 16-lane groups of that instruction,
// MI355X_MICROARCH.md §LDS, whatever the tap shift of the start pixel):
//   patch: 3 bf16 planes x NPP pixels x 64 B (32 channels); 16-B piece q of pixel pp (channels
//          {16(q>>1) + 4(q&1) .. +3} U {16(q>>1) + 8 + 4(q&1) .. +3}: a lane's eight k values) stored at
//          q ^ ((pp >> 2) & 3);
//   B:     3 planes x BN rows x 64 B, piece q of row n at q ^ ((n >> 2) & 3).
// The patch is split into its planes ONCE per block and chunk: its fp32 chunk is loaded into registers
// during the nine taps of the previous chunk and written (split, ds_write_b64) at the chunk boundary.
template <int BM, int BN, int WGM, int W, int IH>
__global__ __launch_bounds__(256, 1) void xconv_kernel(const SgParams p) {
  constexpr int TH = IH ? IH : BM / W;
  constexpr int IMG = IH ? BM / ((IH ? IH : 1) * W) : 1;
  constexpr int PC = W + 2, PIMG = (TH + 2) * PC, NPP = IMG * PIMG;
  constexpr int LQ = (NPP * 8 + 255) / 256;   // 16-B patch loads per thread (4 fp32 channels each)
  constexpr int PLANE = NPP * 64;             // bytes per patch plane
  constexpr int P_BYTES = 3 * PLANE;
  constexpr int B_BYTES = 3 * BN * 64;        // 3 planes x BN rows x 32 bf16
  constexpr int LB = 3 * BN / 64;             // B DMA instructions per wave per tap
  constexpr int WGN = 4 / WGM;                // 4 waves: WGM x WGN
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 32, NI = WN / 32;
  static_assert(MI >= 1 && NI >= 1 && BM % W == 0 && (IH == 0 || BM % (IH * W) == 0), "tile");
  static_assert(LB * 256 == 3 * BN * 4, "B tile must split evenly over the waves");
  static_assert(2 * LB + LQ <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[P_BYTES + 3 * B_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid - (wid / WGN) * WGN;
  const int C = p.C, N = p.N, K = p.K;   // K = C (reduction channels of one tap)
  const int NCC = C / XKC;
  const int tilesN = N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / tilesN, nt = bid - mt * tilesN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HW = p.H * W;
  const int img0 = m0 / HW;
  const int r0 = IH ? 0 : (m0 - img0 * HW) / W;

  const __amdgpu_buffer_rsrc_t rA = s_rsrc(p.A, p.bytesA);
  const __amdgpu_buffer_rsrc_t rB = s_rsrc(p.B, p.bytesB);

  // ---- patch load slots: thread t, load q -> slot t + 256 q = (pixel, 4-channel chunk c); source byte
  // offset of chunk 0 (or SOOB) and the LDS byte offset (plane 0) of its 8-byte half-piece
  unsigned poff[LQ];
  int pdst[LQ];
#pragma unroll
  for (int q = 0; q < LQ; ++q) {
    const int slot = tid + 256 * q;
    const int pp = slot >> 3, c = slot & 7;
    const int img = pp / PIMG, rem = pp - img * PIMG;
    const int pr = rem / PC, pc = rem - pr * PC;
    const int row = r0 - 1 + pr;
    const bool ok = pp < NPP && pc >= 1 && pc <= W && (unsigned)row < (unsigned)p.H && (IH == 0 || (pr >= 1 && pr <= TH));
    poff[q] = ok ? (unsigned)((((img0 + img) * p.H + row) * W + pc - 1) * C) * 4u + (unsigned)c * 16u : SOOB;
    const int piece = 2 * (c >> 2) + (c & 1), half = (c >> 1) & 1;
    pdst[q] = pp < NPP ? pp * 64 + ((piece ^ ((pp >> 2) & 3)) << 4) + half * 8 : -1;
  }
  // ---- B DMA lane constants: planes [3][9][N][K] bf16, rows n0.., 64-byte k-chunk pieces
  unsigned boff[LB];
#pragma unroll
  for (int q = 0; q < LB; ++q) {
    const int slot = (wid * LB + q) * 64 + lane;
    const int pl = slot / (BN * 4), rem = slot - pl * (BN * 4);
    const int n = rem >> 2;
    const int pc = (rem & 3) ^ ((n >> 2) & 3);
    boff[q] = ((unsigned)(pl * 9) * (unsigned)N * (unsigned)K + (unsigned)(n0 + n) * (unsigned)K) * 2u + (unsigned)pc * 16u;
  }
  const unsigned tstep = (unsigned)N * (unsigned)K * 2u;  // bytes between taps of one plane
  // ---- A fragment rows: patch pixel of each lane's output pixel (before the tap shift)
  int ppb[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int ml = wm * WM + i * 32 + (lane & 31);
    const int img = ml / (TH * W), rem = ml - img * (TH * W);
    ppb[i] = img * PIMG + (rem / W + 1) * PC + (rem % W) + 1;
  }

  u32x4 pv[LQ];
  auto load_patch = [&](int cc) {
#pragma unroll
    for (int q = 0; q < LQ; ++q)
      pv[q] = __builtin_amdgcn_raw_buffer_load_b128(rA, (int)(poff[q] == SOOB ? SOOB : poff[q] + (unsigned)cc * 128u), 0, 0);
  };
  auto write_patch = [&]() {   // split the registers' fp32 chunk into the three bf16 planes
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
      if (pdst[q] < 0) continue;
      const f32x4 v = __builtin_bit_cast(f32x4, pv[q]);
      bf16x4 ph, pm, pl;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16 a = (bf16)v[e];
        const float r = v[e] - (float)a;
        const bf16 b = (bf16)r;
        ph[e] = a;
        pm[e] = b;
        pl[e] = (bf16)(r - (float)b);
      }
      *(bf16x4*)(smem + pdst[q]) = ph;
      *(bf16x4*)(smem + PLANE + pdst[q]) = pm;
      *(bf16x4*)(smem + 2 * PLANE + pdst[q]) = pl;
    }
  };
  auto issue_b = [&](int s, int stage) {  // step s = cc * 9 + tap
    const int cc = s / 9, tap = s - cc * 9;
    const unsigned src = (unsigned)tap * tstep + (unsigned)cc * 64u;
    char* dst = smem + P_BYTES + stage * B_BYTES + wid * LB * 1024;
#pragma unroll
    for (int j = 0; j < LB; ++j) x_dma16(rB, dst + j * 1024, (int)(boff[j] + src));
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int S = NCC * 9;
  load_patch(0);
  issue_b(0, 0);
  issue_b(1, 1);
  x_wait_vmcnt<2 * LB>();
  write_patch();
  for (int cc = 0; cc < NCC; ++cc) {
    const bool last = cc == NCC - 1;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int s = cc * 9 + tap;
      // loads issued after B(s): B(s+1), plus the next patch when it went out at tap 0 of this chunk
      if (last && tap == 8) x_wait_vmcnt<0>();
      else if ((tap == 1 || tap == 2) && !last) x_wait_vmcnt<LB + LQ>();
      else x_wait_vmcnt<LB>();
      x_barrier();
      if (s + 2 < S) issue_b(s + 2, (s + 2) % 3);
      if (tap == 0 && !last) load_patch(cc + 1);
      const char* lb = smem + P_BYTES + (s % 3) * B_BYTES;
      const int shift = ((tap * 11) >> 5) * PC + (tap - 3 * ((tap * 11) >> 5)) - PC - 1;  // (dy, dx) in -1..1
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 ah[MI], am[MI], al[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int pp = ppb[i] + shift;
          const int o = pp * 64 + (((2 * ks + h) ^ ((pp >> 2) & 3)) << 4);
          ah[i] = *(const bf16x8*)(smem + o);
          am[i] = *(const bf16x8*)(smem + PLANE + o);
          al[i] = *(const bf16x8*)(smem + 2 * PLANE + o);
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int n = wn * WN + j * 32 + (lane & 31);
          const int o = n * 64 + (((2 * ks + h) ^ ((n >> 2) & 3)) << 4);
          const bf16x8 bh = *(const bf16x8*)(lb + o);
          const bf16x8 bm = *(const bf16x8*)(lb + BN * 64 + o);
          const bf16x8 bl = *(const bf16x8*)(lb + 2 * BN * 64 + o);
#pragma unroll
          for (int i = 0; i < MI; ++i) acc[i][j] = mfma6(ah[i], am[i], al[i], bh, bm, bl, acc[i][j]);
        }
      }
    }
    if (!last) {
      // the next chunk's patch: loaded before B(s+1), B(s+2) of taps 7, 8; every wave is done with
      // this chunk's patch once it passes the barrier
      x_wait_vmcnt<2 * LB>();
      x_barrier();
      write_patch();
    }
  }
  s_epilogue<MI, NI, false, false>(p, acc, m0 + wm * WM, n0 + wn * WN, lane, 0, 0, p.out, p.bias);
}

template <int BM, int BN, int WGM, int W>
int x_launch_w(const SgParams& p, hipStream_t st) {
  const int items = (p.M / BM) * (p.N / BN);
  if (BM >= p.H * W) {
    if (BM % (p.H * W)) return RK_EUNSUPPORTED;
    switch (p.H) {  // whole images per item
      case 4: if constexpr (BM % (4 * W) == 0) { hipLaunchKernelGGL((xconv_kernel<BM, BN, WGM, W, 4>), dim3(items), dim3(256), 0, st, p); break; } return RK_EUNSUPPORTED;
      case 8: if constexpr (BM % (8 * W) == 0) { hipLaunchKernelGGL((xconv_kernel<BM, BN, WGM, W, 8>), dim3(items), dim3(256), 0, st, p); break; } return RK_EUNSUPPORTED;
      case 16: if constexpr (BM % (16 * W) == 0) { hipLaunchKernelGGL((xconv_kernel<BM, BN, WGM, W, 16>), dim3(items), dim3(256), 0, st, p); break; } return RK_EUNSUPPORTED;
      default: return RK_EUNSUPPORTED;
    }
  } else {
    if (p.H % (BM / W)) return RK_EUNSUPPORTED;
    hipLaunchKernelGGL((xconv_kernel<BM, BN, WGM, W, 0>), dim3(items), dim3(256), 0, st, p);
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}

template <int BM, int BN, int WGM = 2>
int x_launch(const SgParams& p, hipStream_t st) {
  switch (p.W) {
    case 4:  // 16 whole 4x4 images per 256-pixel item: the patch registers would spill
      if constexpr (BM <= 128) return x_launch_w<BM, BN, WGM, 4>(p, st);
      return RK_EUNSUPPORTED;
    case 8: return x_launch_w<BM, BN, WGM, 8>(p, st);
    case 16: return x_launch_w<BM, BN, WGM, 16>(p, st);
    case 32: return x_launch_w<BM, BN, WGM, 32>(p, st);
  }
  return RK_EUNSUPPORTED;
}

// ---- weight planes: one 32 (co) x 32 (ci) block of a [Co][9][Ci] fp32 weight -> the forward planes
// [3][9][Co][Ci] and / or the data-gradient planes [3][9][Ci][Co] (taps flipped), bf16, the k index
// permuted inside each 16-group (stored position 8h + j <-> channel j < 4 ? 4h + j : 8 + 4h + j - 4)
RK_DEV int x_kperm(int s) {
  const int g = s & ~15, hh = (s >> 3) & 1, j = s & 7;
  return g + (j < 4 ? 4 * hh + j : 8 + 4 * hh + j - 4);
}

RK_DEV void x_piece3(float x, bf16& a, bf16& b, bf16& c) {
  a = (bf16)x;
  const float r = x - (float)a;
  b = (bf16)r;
  c = (bf16)(r - (float)b);
}

RK_DEV void xwt_block(const float* __restrict__ w, bf16* __restrict__ fw, bf16* __restrict__ dg, int Co, int Ci, int co0,
                      int ci0, float (&g)[9][32][33]) {
  const int tid = threadIdx.x;
  for (int e = tid; e < 9 * 32 * 32; e += 256) {
    const int t = e >> 10, r = e & 1023, co = r >> 5, ci = r & 31;
    g[t][co][ci] = w[((long long)(co0 + co) * 9 + t) * Ci + ci0 + ci];
  }
  __syncthreads();
  // 16-byte units: (tap, row, 8-group) -> 3 planes each
  for (int u = tid; u < 9 * 32 * 4; u += 256) {
    const int t = u >> 7, r = (u >> 2) & 31, g8 = u & 3;
    bf16x8 ph, pm, pl;
    if (fw) {   // forward: row = co, k = ci
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bf16 a, b, c;
        x_piece3(g[t][r][x_kperm(g8 * 8 + j)], a, b, c);
        ph[j] = a; pm[j] = b; pl[j] = c;
      }
      const long long base = ((long long)t * Co + co0 + r) * Ci + ci0 + g8 * 8;
      const long long ps = 9LL * Co * Ci;
      *(bf16x8*)(fw + base) = ph;
      *(bf16x8*)(fw + ps + base) = pm;
      *(bf16x8*)(fw + 2 * ps + base) = pl;
    }
    if (dg) {   // data gradient: row = ci, k = co, tap 8 - t
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bf16 a, b, c;
        x_piece3(g[8 - t][x_kperm(g8 * 8 + j)][r], a, b, c);
        ph[j] = a; pm[j] = b; pl[j] = c;
      }
      const long long base = ((long long)t * Ci + ci0 + r) * Co + co0 + g8 * 8;
      const long long ps = 9LL * Co * Ci;
      *(bf16x8*)(dg + base) = ph;
      *(bf16x8*)(dg + ps + base) = pm;
      *(bf16x8*)(dg + 2 * ps + base) = pl;
    }
  }
}

__global__ __launch_bounds__(256) void xconv_wt_kernel(const float* __restrict__ w, bf16* fw, bf16* dg, int Co, int Ci) {
  __shared__ float g[9][32][33];
  const int nb = Ci / 32;
  xwt_block(w, fw, dg, Co, Ci, (blockIdx.x / nb) * 32, (blockIdx.x % nb) * 32, g);
}

// every layer in one launch: desc[block] = (layer, co0, ci0, -); meta[layer] = (weight offset in the
// arena, forward-plane offset or -1, data-gradient-plane offset or -1, Co, Ci); offsets in floats
__global__ __launch_bounds__(256) void xconv_wt_multi_kernel(const float* __restrict__ arena, float* __restrict__ dst,
                                                             const int4* __restrict__ desc,
                                                             const long long* __restrict__ meta) {
  __shared__ float g[9][32][33];
  const int4 d = desc[blockIdx.x];
  const long long* m = meta + 5 * d.x;
  xwt_block(arena + m[0], m[1] >= 0 ? (bf16*)(dst + m[1]) : nullptr, m[2] >= 0 ? (bf16*)(dst + m[2]) : nullptr,
            (int)m[3], (int)m[4], d.y, d.z, g);
}

}  // namespace

// y = conv3x3(x, w) (stride 1, pad 1): x [Nb][H][W][C] fp32 NHWC, wp = the bf16 planes [3][9][N][C] of
// rk_xconv_weights (forward set: N = Cout; data-gradient set of the transposed conv: N = Cin, C = Cout),
// out [Nb][H][W][N] fp32.  cfg 0-3: bit 0 64-pixel items (else 128), bit 1 64-channel items (else 128),
// 2 x 2 waves; cfg 4: 256 x 64 items on 4 x 1 waves (a wave = 64 px x 64 channels: 4x less weight
// traffic per FLOP than 64 x 64 items, the B ring three 1.5k-cycle steps deep).
// flags: SF_BIAS / SF_RELU / SF_LRELU / SF_STATS (fp64 slots [slotMask+1][2][N]) / SF_BNB / SF_BNP
// (gate = the gated layer's pre-BN input, bias = its BN scale [N] then shift [N]) / SF_ACCUM.
// Square maps of 4, 8, 16 or 32; C % 32 == 0; N % (item channels) == 0.
extern "C" int rk_xconv(int cfg, const float* x, const void* wp, float* out, const float* bias, double* stats,
                        int slotMask, const float* gate, int Nb, int H, int W, int C, int N, int flags,
                        long long bytesA, long long bytesB, void* stream) {
  if (bytesA <= 0 || bytesB <= 0 || bytesA >= (1ll << 31) || bytesB >= (1ll << 31)) return RK_EUNSUPPORTED;
  if (Nb <= 0 || C <= 0 || N <= 0 || cfg < 0 || cfg > 4) return RK_EBADARG;
  if (H != W || (W != 4 && W != 8 && W != 16 && W != 32) || C % XKC) return RK_EUNSUPPORTED;
  const int BM = cfg == 4 ? 256 : (cfg & 1) ? 64 : 128, BN = cfg == 4 ? 64 : (cfg & 2) ? 64 : 128;
  const long long M = (long long)Nb * H * W;
  if (M % BM || N % BN || M >= (1ll << 30)) return RK_EUNSUPPORTED;
  if (flags & ~(SF_BIAS | SF_RELU | SF_LRELU | SF_STATS | SF_BNB | SF_BNP | SF_ACCUM)) return RK_EUNSUPPORTED;
  if ((flags & (SF_STATS | SF_BNB | SF_BNP)) && !stats) return RK_EBADARG;
  if ((flags & (SF_BNB | SF_BNP)) && (!gate || !bias)) return RK_EBADARG;
  if ((long long)27 * N * C * 2 > bytesB) return RK_EBADARG;
  SgParams p{};
  p.A = x; p.B = (const float*)wp; p.out = out; p.bias = bias; p.stats = stats; p.gate = gate;
  p.M = (int)M; p.N = N; p.K = C; p.lda = C; p.ldb = C; p.ldc = N;
  p.H = H; p.W = W; p.C = C; p.taps = 9;
  p.log2H = rk_log2(H); p.log2W = rk_log2(W); p.log2C = rk_log2(C);
  p.invC = 1.0f / (float)C; p.invH = 1.0f / (float)H; p.invW = 1.0f / (float)W;
  p.flags = flags; p.slotMask = slotMask; p.alpha = 1.0f; p.slope = 0.2f;
  p.bytesA = (unsigned long long)bytesA; p.bytesB = (unsigned long long)bytesB;
  p.groups = 1;
  p.Ho = H; p.Wo = W; p.log2Ho = p.log2H; p.log2Wo = p.log2W; p.invHo = p.invH; p.invWo = p.invW;
  hipStream_t st = (hipStream_t)stream;
  switch (cfg) {
    case 0: return x_launch<128, 128>(p, st);
    case 1: return x_launch<64, 128>(p, st);
    case 2: return x_launch<128, 64>(p, st);
    case 3: return x_launch<64, 64>(p, st);
    case 4: return x_launch<256, 64, 4>(p, st);   // 4 x 1 waves of 64 px x 64 channels
  }
  return RK_EBADARG;
}

// forward planes fw [3][9][Co][Ci] and / or data-gradient planes dg [3][9][Ci][Co] (bf16) of w [Co][9][Ci]
extern "C" int rk_xconv_weights(const float* w, void* fw, void* dg, int Co, int Ci, void* stream) {
  if (Co % 32 || Ci % 32 || Co <= 0 || Ci <= 0) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(xconv_wt_kernel, dim3((Co / 32) * (Ci / 32)), dim3(256), 0, (hipStream_t)stream, w, (bf16*)fw,
                     (bf16*)dg, Co, Ci);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_xconv_weights_multi(const float* arena, float* dst, const int* desc, int nblocks,
                                      const long long* meta, void* stream) {
  if (nblocks <= 0) return RK_OK;
  hipLaunchKernelGGL(xconv_wt_multi_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, arena, dst,
                     (const int4*)desc, meta);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
