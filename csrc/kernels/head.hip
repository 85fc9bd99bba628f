// Classifier head of the fp32 conv-net engines on gfx950, fused: the tiny output layer (D -> NC <= 32
// classes), softmax cross-entropy and everything the backward needs from it, in two launches instead of
// six (the output GEMM, softmax-xent, the output weight / bias gradients, the gated data gradient into
// the hidden layer and that layer's bias gradient; profiles/vgg_small_f32_step_kernels_r4*: 66 us of
// latency-bound launches for 0.01 GFLOP).  fp32 FMAs throughout (the reference's precision); every sum
// runs in a fixed order, so the results are deterministic (only loss_sum / correct / counted use atomics,
// as rk_softmax_xent does).
//
//   head_fwd_bwd (one wave per row b):  logits = z W^T + bias; log-softmax; loss / #correct;
//     dlogits = (softmax - onehot(y)) * grad_scale over the ncls real classes (0 in the padding);
//     dz = (dlogits W) gated by z > 0 (the hidden layer's ReLU; ungated without a gate)
//   head_dw (one block per 8 columns k):  dW[c][k] = sum_b dlogits[b][c] z[b][k], db[c] = sum_b dlogits[b][c]
//     and, for the hidden layer, dbh[k] = sum_b dz[b][k] (its bias gradient)
// Reference: TfFeedForward.py / TfVgg16.py Dense(softmax) + categorical cross-entropy.
#include "common.h"

namespace {

template <int NC>
__global__ __launch_bounds__(256) void head_fwd_bwd_kernel(const float* __restrict__ z, int D,
                                                           const float* __restrict__ w, const float* __restrict__ bias,
                                                           const int* __restrict__ labels, int B, int ncls,
                                                           float grad_scale, float* __restrict__ dlogits,
                                                           float* __restrict__ dz, int gated, float* loss_sum,
                                                           int* correct, int* counted) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float* zr = z + (long long)row * D;
  float part[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) part[c] = 0.f;
  for (int k = 4 * lane; k < D; k += 256) {
    const f32x4 zv = *(const f32x4*)(zr + k);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const f32x4 wv = *(const f32x4*)(w + (long long)c * D + k);
      part[c] += zv[0] * wv[0] + zv[1] * wv[1] + zv[2] * wv[2] + zv[3] * wv[3];
    }
  }
  float logit[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) logit[c] = wave_sum(part[c]) + (bias ? bias[c] : 0.f);
  // log-softmax over the real classes (every lane holds every logit)
  float mx = -INFINITY;
  int amax = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < ncls && logit[c] > mx) { mx = logit[c]; amax = c; }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < ncls) se += __expf(logit[c] - mx);
  const float lse = mx + __logf(se);
  const int y = labels[row];
  const bool valid = y >= 0 && y < ncls;
  float g[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c)
    g[c] = (valid && c < ncls) ? (__expf(logit[c] - lse) - (c == y ? 1.f : 0.f)) * grad_scale : 0.f;
  if (lane < NC) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) v = lane == c ? g[c] : v;
    dlogits[(long long)row * NC + lane] = v;
  }
  if (lane == 0 && valid) {
    float ly = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) ly = c == y ? logit[c] : ly;
    if (loss_sum) atomicAdd(loss_sum, lse - ly);
    if (correct) atomicAdd(correct, amax == y ? 1 : 0);
    if (counted) atomicAdd(counted, 1);
  }
  // dz = dlogits . W, gated by the hidden layer's ReLU output
  float* dzr = dz + (long long)row * D;
  for (int k = 4 * lane; k < D; k += 256) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c) acc += g[c] * *(const f32x4*)(w + (long long)c * D + k);
    if (gated) {
      const f32x4 zv = *(const f32x4*)(zr + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = zv[e] > 0.f ? acc[e] : 0.f;
    }
    *(f32x4*)(dzr + k) = acc;
  }
}

// 256 threads = 32 row groups x 8 columns (D / 8 blocks: 64 at D = 512, so the 32-step row loop of the
// 32-column form — 16 blocks, 18 us in profiles/vgg_small_f32_step_kernels_r6.txt — becomes 8 steps over
// four times the CUs); rows b = rg, rg + 32, ... ; the 32 partial sums per output are combined through LDS
// in a fixed order
template <int NC>
__global__ __launch_bounds__(256) void head_dw_kernel(const float* __restrict__ z, const float* __restrict__ dlogits,
                                                      const float* __restrict__ dz, int B, int D,
                                                      float* __restrict__ dw, float* __restrict__ db,
                                                      float* __restrict__ dbh) {
  constexpr int CB = 8, RG = 256 / CB;
  __shared__ float red[RG][NC + 1][CB];
  __shared__ float dbr[RG][NC];
  const int kk = threadIdx.x % CB, rg = threadIdx.x / CB;
  const int k = blockIdx.x * CB + kk;
  const bool dbl = blockIdx.x == 0 && kk == 0 && db;   // block 0 also sums dlogits' columns (the bias gradient)
  float acc[NC], dba[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = dba[c] = 0.f;
  float hs = 0.f;
  for (int b = rg; b < B; b += RG) {
    const float zv = z[(long long)b * D + k];
    const float* gr = dlogits + (long long)b * NC;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float g = gr[c];
      acc[c] += g * zv;
      dba[c] += g;
    }
    if (dbh) hs += dz[(long long)b * D + k];
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) red[rg][c][kk] = acc[c];
  red[rg][NC][kk] = hs;
  if (dbl) {
#pragma unroll
    for (int c = 0; c < NC; ++c) dbr[rg][c] = dba[c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (NC + 1) * CB; i += 256) {
    const int c = i / CB, col = i % CB;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < RG; ++r) s += red[r][c][col];
    const int kc = blockIdx.x * CB + col;
    if (c < NC) dw[(long long)c * D + kc] = s;
    else if (dbh) dbh[kc] = s;
  }
  if (blockIdx.x == 0 && db && threadIdx.x < NC) {   // the row-group partials of the bias gradient, in order
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < RG; ++r) s += dbr[r][threadIdx.x];
    db[threadIdx.x] = s;
  }
}

}  // namespace

// z [B][D] (D % 4 == 0), w [NC][D], bias [NC] (nullable), labels [B] int32 -> dlogits [B][NC], dz [B][D]
// (gated by z > 0 when `gated`); loss / correct / counted accumulate (nullable).  NC in {8, 16, 32}.
extern "C" int rk_head_fwd_bwd(const float* z, int B, int D, const float* w, const float* bias, int NC,
                               const int* labels, int ncls, float grad_scale, float* dlogits, float* dz, int gated,
                               float* loss_sum, int* correct, int* counted, void* stream) {
  if (B <= 0 || D <= 0 || (D & 3) || ncls <= 0 || ncls > NC || !labels || !dlogits || !dz) return RK_EBADARG;
  const dim3 grid(rk_cdiv(B, 4)), block(256);
  const hipStream_t st = (hipStream_t)stream;
  switch (NC) {
    case 8: hipLaunchKernelGGL(head_fwd_bwd_kernel<8>, grid, block, 0, st, z, D, w, bias, labels, B, ncls, grad_scale,
                               dlogits, dz, gated, loss_sum, correct, counted); break;
    case 16: hipLaunchKernelGGL(head_fwd_bwd_kernel<16>, grid, block, 0, st, z, D, w, bias, labels, B, ncls,
                                grad_scale, dlogits, dz, gated, loss_sum, correct, counted); break;
    case 32: hipLaunchKernelGGL(head_fwd_bwd_kernel<32>, grid, block, 0, st, z, D, w, bias, labels, B, ncls,
                                grad_scale, dlogits, dz, gated, loss_sum, correct, counted); break;
    default: return RK_EUNSUPPORTED;
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// dw [NC][D] = dlogits^T z, db [NC] = column sums of dlogits (nullable), dbh [D] = column sums of dz
// (nullable: the hidden layer's bias gradient); D % 8 == 0.
extern "C" int rk_head_dw(const float* z, const float* dlogits, const float* dz, int B, int D, int NC, float* dw,
                          float* db, float* dbh, void* stream) {
  if (B <= 0 || D <= 0 || (D & 7) || !dw || (dbh && !dz)) return RK_EBADARG;
  const dim3 grid(D / 8), block(256);
  const hipStream_t st = (hipStream_t)stream;
  switch (NC) {
    case 8: hipLaunchKernelGGL(head_dw_kernel<8>, grid, block, 0, st, z, dlogits, dz, B, D, dw, db, dbh); break;
    case 16: hipLaunchKernelGGL(head_dw_kernel<16>, grid, block, 0, st, z, dlogits, dz, B, D, dw, db, dbh); break;
    case 32: hipLaunchKernelGGL(head_dw_kernel<32>, grid, block, 0, st, z, dlogits, dz, B, D, dw, db, dbh); break;
    default: return RK_EUNSUPPORTED;
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}
