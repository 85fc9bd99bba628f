// Loss, optimizer and small streaming kernels for gfx950.
//
//  * rk_softmax_xent: fused log-softmax + NLL forward and d(logits) backward in one pass, one wave
//    per row (64-lane shuffles), optional ignore-index, optional probability output for predict.
//    Loss and #correct are reduced with a single atomic per wave into device scalars so the whole
//    training step stays on the GPU (graph-capturable, no host sync per step).
//  * rk_sgd_step / rk_adam_step: multi-tensor optimizer over ONE flat parameter buffer — fp32
//    master weights, fp32 grads and state, plus the bf16 compute copy written in the same pass
//    (so the next forward never needs a separate cast kernel).  16-byte vectors, grid-stride.
//  * rk_lerp (Gs EMA, pg_gans.py:730-740), rk_nonfinite_count (pg_gans.py:1180-1191),
//    rk_reduce_slabs (split-K combine), rk_colsum (bias grads), rk_ensemble_mean (predictor).
#include "common.h"

namespace {

template <typename DT>  // d(logits) storage: bf16 (bf16 engine) or float (fp32 engine)
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ logits, int ldl,
                                                           const int* __restrict__ labels, int B, int ncls,
                                                           int ignore_index, float grad_scale,
                                                           DT* __restrict__ dlogits, int ldd,
                                                           float* __restrict__ probs, float* loss_sum,
                                                           int* correct, int* counted,
                                                           const float* __restrict__ scale_ptr) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float* lr = logits + (long long)row * ldl;
  float mx = -INFINITY;
  int amax = 0;
  for (int c = lane; c < ncls; c += 64) {
    const float v = lr[c];
    if (v > mx) { mx = v; amax = c; }
  }
  // wave argmax (first index of the max)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(amax, o, 64);
    if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
  }
  float se = 0.f;
  for (int c = lane; c < ncls; c += 64) se += __expf(lr[c] - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const int y = labels ? labels[row] : -1;
  const bool valid = labels && y != ignore_index && y >= 0 && y < ncls;
  // scale_ptr: a device factor on the gradient and the loss (the tagger's 1 / #valid tokens of a batch,
  // written with the batch, so a replayed graph takes each batch's mean)
  const float sc = scale_ptr ? scale_ptr[0] : 1.f;
  grad_scale *= sc;
  if (dlogits) {
    DT* dr = dlogits + (long long)row * ldd;
    for (int c = lane; c < ldd; c += 64) {
      float g = 0.f;
      if (valid && c < ncls) g = (__expf(lr[c] - lse) - (c == y ? 1.f : 0.f)) * grad_scale;
      dr[c] = (DT)g;
    }
  }
  if (probs) {
    float* pr = probs + (long long)row * ncls;
    for (int c = lane; c < ncls; c += 64) pr[c] = __expf(lr[c] - lse);
  }
  if (lane == 0 && valid) {
    if (loss_sum) atomicAdd(loss_sum, (lse - lr[y]) * sc);
    if (correct) atomicAdd(correct, amax == y ? 1 : 0);
    if (counted) atomicAdd(counted, 1);
  }
}

// One launch over the whole arena: weight decay applies to elements [0, decay_end) (the arena puts
// decayed parameters first).  bump: a device step counter advanced once (the last kernel of a
// scheduled training step owns it, so no separate increment launch is needed).
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ w, bf16* __restrict__ wb,
                                                  const float* __restrict__ g, float* __restrict__ mom, long long n,
                                                  float lr, float momentum, float wd, int nesterov, float gscale,
                                                  const float* lr_ptr, long long decay_end, int* bump) {
  if (bump && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(bump, 1);
  const float lrv = lr_ptr ? lr_ptr[0] * lr : lr;
  const long long n4 = n >> 2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 wv = ((const f32x4*)w)[i];
    f32x4 gv = ((const f32x4*)g)[i] * gscale + (4 * i < decay_end ? wd : 0.f) * wv;
    f32x4 d = gv;
    if (mom) {
      f32x4 m = ((const f32x4*)mom)[i] * momentum + gv;
      ((f32x4*)mom)[i] = m;
      d = nesterov ? gv + momentum * m : m;
    }
    wv -= lrv * d;
    ((f32x4*)w)[i] = wv;
    if (wb) {
      bf16x4 o;
      o[0] = (bf16)wv[0]; o[1] = (bf16)wv[1]; o[2] = (bf16)wv[2]; o[3] = (bf16)wv[3];
      ((bf16x4*)wb)[i] = o;
    }
  }
}

// omb1 / omb2: 1 - beta as computed on the host in double (torch's Adam adds (1 - beta) * g the same
// way); forming 1 - b2 from the fp32 b2 here would cancel to 1.3e-5 relative error at b2 = 0.999
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ w, bf16* __restrict__ wb,
                                                   const float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, long long n, float lr, float b1, float b2,
                                                   float omb1, float omb2, float eps, float wd, int decoupled,
                                                   float c1, float c2, float gscale, const int* skip,
                                                   const int* step_ptr) {
  if (skip && skip[0] != 0) return;  // non-finite gradients: skip the update (pg_gans.py:1180-1191)
  if (step_ptr) {  // device-side step counter: bias corrections survive hipGraph replay (in double:
                   // 1 - beta^t cancels at small t)
    const int t = step_ptr[0];
    c1 = omb1 < 1.f ? (float)(1.0 / (1.0 - pow(1.0 - (double)omb1, t))) : 1.f;
    c2 = (float)(1.0 / (1.0 - pow(1.0 - (double)omb2, t)));
  }
  const long long n4 = n >> 2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 wv = ((const f32x4*)w)[i];
    f32x4 gv = ((const f32x4*)g)[i] * gscale;
    if (!decoupled) gv += wd * wv;
    f32x4 mv = ((const f32x4*)m)[i] * b1 + omb1 * gv;
    f32x4 vv = ((const f32x4*)v)[i] * b2 + omb2 * gv * gv;
    ((f32x4*)m)[i] = mv;
    ((f32x4*)v)[i] = vv;
    f32x4 upd;
#pragma unroll
    for (int e = 0; e < 4; ++e) upd[e] = (mv[e] * c1) / (sqrtf(vv[e] * c2) + eps);
    if (decoupled) upd += wd * wv;
    wv -= lr * upd;
    ((f32x4*)w)[i] = wv;
    if (wb) {
      bf16x4 o;
      o[0] = (bf16)wv[0]; o[1] = (bf16)wv[1]; o[2] = (bf16)wv[2]; o[3] = (bf16)wv[3];
      ((bf16x4*)wb)[i] = o;
    }
  }
}

// Multi-segment forms (one launch over a LOD's live arena ranges instead of one per range: at the PG-GAN
// reference schedule's 4x4 LOD the live set is 3-4 ranges per arena, several of them a few hundred
// elements, and Adam splits further by the per-layer equalized-LR multiplier — 11 Adam, 9 zeroing and 7
// finite-check launches per round, profiles/pg_gan_lod3_f32_kernels_r5.txt).  blk [nblk][3] int64 =
// (segment, first element, end element) of each block's chunk, built on the host once per live set;
// every bound a multiple of 4 (16-B vectors).
__global__ __launch_bounds__(256) void adam_multi_kernel(float* __restrict__ w, bf16* __restrict__ wb,
                                                         const float* __restrict__ g, float* __restrict__ m,
                                                         float* __restrict__ v, const long long* __restrict__ blk,
                                                         const float* __restrict__ segp, float b1, float b2,
                                                         float omb1, float omb2, int decoupled, float gscale,
                                                         const int* skip, const int* step_ptr, int* bump) {
  // bump (nullable): another int32 step counter (the trial's random stream) advanced by block 0 whether or not
  // the update is skipped, read by later launches only
  if (bump && blockIdx.x == 0 && threadIdx.x == 0) *bump += 1;
  if (skip && skip[0] != 0) return;
  const int t = step_ptr[0];
  const float c1 = omb1 < 1.f ? (float)(1.0 / (1.0 - pow(1.0 - (double)omb1, t))) : 1.f;
  const float c2 = (float)(1.0 / (1.0 - pow(1.0 - (double)omb2, t)));
  const long long* e = blk + 3 * (long long)blockIdx.x;
  const int sg = (int)e[0];
  const float lr = segp[4 * sg], eps = segp[4 * sg + 1], wd = segp[4 * sg + 2];
  for (long long i = (e[1] >> 2) + threadIdx.x; i < (e[2] >> 2); i += 256) {
    f32x4 wv = ((const f32x4*)w)[i];
    f32x4 gv = ((const f32x4*)g)[i] * gscale;
    if (!decoupled) gv += wd * wv;
    f32x4 mv = ((const f32x4*)m)[i] * b1 + omb1 * gv;
    f32x4 vv = ((const f32x4*)v)[i] * b2 + omb2 * gv * gv;
    ((f32x4*)m)[i] = mv;
    ((f32x4*)v)[i] = vv;
    f32x4 upd;
#pragma unroll
    for (int q = 0; q < 4; ++q) upd[q] = (mv[q] * c1) / (sqrtf(vv[q] * c2) + eps);
    if (decoupled) upd += wd * wv;
    wv -= lr * upd;
    ((f32x4*)w)[i] = wv;
    if (wb) {
      bf16x4 o;
      o[0] = (bf16)wv[0]; o[1] = (bf16)wv[1]; o[2] = (bf16)wv[2]; o[3] = (bf16)wv[3];
      ((bf16x4*)wb)[i] = o;
    }
  }
}

// flag (nullable): also zeroed (the step's finite-check flag, so the check needs no launch of its own)
__global__ __launch_bounds__(256) void zero_multi_kernel(unsigned* __restrict__ dst, const long long* __restrict__ blk,
                                                         int* __restrict__ flag) {
  if (flag && blockIdx.x == 0 && threadIdx.x == 0) *flag = 0;
  const long long* e = blk + 3 * (long long)blockIdx.x;
  for (long long i = (e[1] >> 2) + threadIdx.x; i < (e[2] >> 2); i += 256) ((uint4*)dst)[i] = make_uint4(0u, 0u, 0u, 0u);
}

// bump (nullable): block 0 also advances this int32 step counter (the optimizer's, read by the next launch)
__global__ __launch_bounds__(256) void nonfinite_multi_kernel(const float* __restrict__ x,
                                                              const long long* __restrict__ blk, int* flag,
                                                              int* __restrict__ bump) {
  if (bump && blockIdx.x == 0 && threadIdx.x == 0) *bump += 1;
  const long long* e = blk + 3 * (long long)blockIdx.x;
  int bad = 0;
  for (long long i = (e[1] >> 2) + threadIdx.x; i < (e[2] >> 2); i += 256) {
    const f32x4 q = ((const f32x4*)x)[i];
    bad |= !isfinite(q[0]) | !isfinite(q[1]) | !isfinite(q[2]) | !isfinite(q[3]);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ __launch_bounds__(256) void lerp_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                   bf16* __restrict__ dstb, long long n, float t) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    // dst <- src + (dst - src) * t   (tf lerp(a=src, b=dst, t): Gs = lerp(G, Gs, beta))
    const float s = src[i];
    const float r = s + (dst[i] - s) * t;
    dst[i] = r;
    if (dstb) dstb[i] = (bf16)r;
  }
}

// lerp_kernel over the chunk table's ranges (16-B aligned): the same per-element arithmetic, 16-B vectors
__global__ __launch_bounds__(256) void lerp_multi_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                         bf16* __restrict__ dstb, const long long* __restrict__ blk,
                                                         float t) {
  const long long* e = blk + 3 * (long long)blockIdx.x;
  for (long long i = (e[1] >> 2) + threadIdx.x; i < (e[2] >> 2); i += 256) {
    const f32x4 s = ((const f32x4*)src)[i], d = ((const f32x4*)dst)[i];
    f32x4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = s[k] + (d[k] - s[k]) * t;
    ((f32x4*)dst)[i] = r;
    if (dstb) {
      bf16x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (bf16)r[k];
      ((bf16x4*)dstb)[i] = o;
    }
  }
}

// dst[0 .. n) = 0 for any 4-byte element type: 16-B vector stores, a scalar tail
__global__ __launch_bounds__(256) void zero32_kernel(unsigned* __restrict__ dst, long long n) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    ((uint4*)dst)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (long long i = 4 * n4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = 0u;
}

__global__ __launch_bounds__(256) void nonfinite_kernel(const float* __restrict__ x, long long n, int* flag) {
  int bad = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ __launch_bounds__(256) void reduce_slabs_kernel(const float* __restrict__ slab, int S, long long n,
                                                           float* __restrict__ out, int accumulate, float scale) {
  const long long n4 = n >> 2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 a = ((const f32x4*)slab)[i];
    int s0 = 1;
    for (; s0 + 3 < S; s0 += 4) {  // 4 independent slab loads in flight, fixed summation order
      f32x4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ((const f32x4*)(slab + (s0 + k) * n))[i];
#pragma unroll
      for (int k = 0; k < 4; ++k) a += v[k];
    }
    for (; s0 < S; ++s0) a += ((const f32x4*)(slab + s0 * n))[i];
    a *= scale;
    if (accumulate) a += ((const f32x4*)out)[i];
    ((f32x4*)out)[i] = a;
  }
}

// split-K combine with the dense epilogue: out[M][N] (bf16 or fp32, row stride ldc) =
// act(alpha * sum_s slab[s] + bias).  Lets a small-M dense layer (fc at batch 256: 32 output tiles)
// spread K over the chip and still write the bf16 activation the next layer reads.
__global__ __launch_bounds__(256) void reduce_slabs_epi_kernel(const float* __restrict__ slab, int S, int M, int N,
                                                               const float* __restrict__ bias, int act, float slope,
                                                               float alpha, bf16* __restrict__ outb,
                                                               float* __restrict__ outf, int ldc) {
  const long long n4 = (long long)M * N / 4;
  const long long sn = (long long)M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 a = ((const f32x4*)slab)[i];
    int s0 = 1;
    for (; s0 + 3 < S; s0 += 4) {
      f32x4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ((const f32x4*)(slab + (s0 + k) * sn))[i];
#pragma unroll
      for (int k = 0; k < 4; ++k) a += v[k];
    }
    for (; s0 < S; ++s0) a += ((const f32x4*)(slab + s0 * sn))[i];
    const long long e0 = i * 4;
    const int m = (int)(e0 / N), n = (int)(e0 - (long long)m * N);
    a *= alpha;
    if (bias) a += *(const f32x4*)(bias + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (act == 1) a[e] = fmaxf(a[e], 0.f);
      else if (act == 2) a[e] = a[e] > 0.f ? a[e] : a[e] * slope;
    }
    if (outb) {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)a[e];
      *(bf16x4*)(outb + (long long)m * ldc + n) = o;
    } else {
      *(f32x4*)(outf + (long long)m * ldc + n) = a;
    }
  }
}

// Minibatch gather inside the captured training graph: out_x[b] = data[idx[step][b]] (rows of
// row_vec 16-B vectors), out_y[b] = labels[idx[step][b]], where step = *counter is read on the
// device — the replayed graph walks a precomputed index schedule with no per-step host copies.
// Step prologue of a scheduled training graph, one launch: gather minibatch rows sched[*counter],
// zero the step's fp64 BatchNorm slot tables (`zero`, zero_n doubles) and, with `done`, advance the
// device step counter once every block has read it (the last block to arrive bumps it) — replaces a
// memset node and a separate counter-increment kernel (~4 us of dispatch each).
__global__ __launch_bounds__(256) void gather_batch_kernel(const uint4* __restrict__ data, long long row_vec,
                                                           const int* __restrict__ labels,
                                                           const long long* __restrict__ sched,
                                                           int* __restrict__ counter, int B,
                                                           uint4* __restrict__ out, int* __restrict__ out_y,
                                                           double* __restrict__ zero, long long zero_n,
                                                           int* __restrict__ done, const float* __restrict__ lr_table,
                                                           float* __restrict__ lr_out, int nsteps, long long nrows) {
  // the schedule holds nsteps rows: a counter past it wraps around (warm-up runs, extra replays) instead
  // of reading beyond the buffers; row indices outside the dataset read row 0
  const long long step = (long long)((unsigned)*counter % (unsigned)nsteps);
  // the step's learning-rate multiplier from a per-step table (a schedule inside the replayed graph)
  if (lr_table && blockIdx.x == 0 && threadIdx.x == 0) *lr_out = lr_table[step];
  const long long total = (long long)B * row_vec;
  const long long gstride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gstride) {
    const int b = (int)(i / row_vec);
    const long long c = i - (long long)b * row_vec;
    long long src = sched[step * B + b];
    if ((unsigned long long)src >= (unsigned long long)nrows) src = 0;
    out[i] = data[src * row_vec + c];
    if (c == 0 && out_y) out_y[b] = labels[src];
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < zero_n; i += gstride) zero[i] = 0.0;
  if (done) {
    __syncthreads();  // this block's reads of *counter are done (every thread used the value)
    if (threadIdx.x == 0 && atomicAdd(done, 1) == (int)gridDim.x - 1) {
      *done = 0;
      atomicAdd(counter, 1);
    }
  }
}

// Stage-1 parallel row reduction: in [R][W] fp32 -> out [G][W], block (x, g) sums its slice of rows
// for 256 consecutive columns (coalesced).  Turns the serial "sum thousands of partial rows" tails
// of BN finalize / split-K combine into a chip-wide pass; stage 2 then reads only G rows.
__global__ __launch_bounds__(256) void rows_reduce_kernel(const float* __restrict__ in, int R, long long W,
                                                          float* __restrict__ out) {
  const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
  if (c >= W) return;
  const int G = gridDim.y, g = blockIdx.y;
  const int per = (R + G - 1) / G;
  const int r0 = g * per, r1 = min(R, r0 + per);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int r = r0;
  for (; r + 3 < r1; r += 4) {
    a0 += in[(long long)r * W + c];
    a1 += in[(long long)(r + 1) * W + c];
    a2 += in[(long long)(r + 2) * W + c];
    a3 += in[(long long)(r + 3) * W + c];
  }
  for (; r < r1; ++r) a0 += in[(long long)r * W + c];
  out[(long long)g * W + c] = (a0 + a1) + (a2 + a3);
}

// out (+)= scale * sum_r in[r] for in [R][n], R > 16, in ONE pass (replaces rows_reduce + reduce_slabs): a
// block owns 64 columns (16 float4 lanes) x 16 row lanes; row lane l sums rows l, l + 16, ... (two chains),
// then lane 0 of each column folds the 16 lane sums in order — deterministic, no cross-block dependence.
__global__ __launch_bounds__(256) void fold_rows_kernel(const float* __restrict__ in, int R, long long n,
                                                        float* __restrict__ out, int accumulate, float scale) {
  const int q = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const long long c = (long long)blockIdx.x * 64 + 4 * q;
  __shared__ f32x4 red[16][16];
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  if (c < n) {
    int r = rl;
    for (; r + 16 < R; r += 32) {
      a += *(const f32x4*)(in + (long long)r * n + c);
      b += *(const f32x4*)(in + (long long)(r + 16) * n + c);
    }
    if (r < R) a += *(const f32x4*)(in + (long long)r * n + c);
  }
  red[rl][q] = a + b;
  __syncthreads();
  if (rl == 0 && c < n) {
    f32x4 s = red[0][q];
#pragma unroll
    for (int k = 1; k < 16; ++k) s += red[k][q];
    s *= scale;
    if (accumulate) s += *(const f32x4*)(out + c);
    *(f32x4*)(out + c) = s;
  }
}

// column sums of a bf16 [R][C] matrix into fp32 out[C] (bias gradients)
__global__ __launch_bounds__(256) void colsum_kernel(const bf16* __restrict__ x, int R, int C, int ld,
                                                     float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  __shared__ float red[4][64];
  float s = 0.f;
  if (c < C)
  {
    int r0 = q;
    for (; r0 + 4 * 7 < R; r0 += 4 * 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (float)x[(long long)(r0 + 4 * k) * ld + c];
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; r0 < R; r0 += 4) s += (float)x[(long long)r0 * ld + c];
  }
  red[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && c < C) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    out[c] = accumulate ? out[c] + t : t;
  }
}

// mean over models: probs [Wm][Q*C] -> out [Q*C]   (predictor/ensemble.py:10-14 on device)
__global__ __launch_bounds__(256) void ensemble_mean_kernel(const float* __restrict__ probs, int Wm, long long n,
                                                            const float* __restrict__ weights, float* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float a = 0.f, ws = 0.f;
    for (int w = 0; w < Wm; ++w) {
      const float wt = weights ? weights[w] : 1.f;
      a += wt * probs[w * n + i];
      ws += wt;
    }
    out[i] = a / ws;
  }
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ src, bf16* __restrict__ dst,
                                                            long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = (bf16)src[i];
}

// uint8/float NCHW images -> bf16 NHWC with channels zero-padded to Cp (input staging, K19):
// out = (in * scale + shift)
__global__ __launch_bounds__(256) void pack_nhwc_kernel(const void* __restrict__ src, int is_u8, int N, int C, int H,
                                                        int W, int Cp, float scale, float shift,
                                                        bf16* __restrict__ dst) {
  const long long total = (long long)N * H * W * Cp;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const long long pix = i / Cp;
    const int w = (int)(pix % W);
    const long long t = pix / W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float v = 0.f;
    if (c < C) {
      const long long si = (((long long)n * C + c) * H + h) * W + w;
      const float raw = is_u8 ? (float)((const unsigned char*)src)[si] : ((const float*)src)[si];
      v = raw * scale + shift;
    }
    dst[i] = (bf16)v;
  }
}

// Column sums of a tall bf16 matrix in two deterministic stages: block (x, y) sums 512 columns
// (8 per lane, 16-byte loads) over row chunk y into part[y][C]; rk_reduce_slabs folds the chunks.
__global__ __launch_bounds__(256) void colsum_part_kernel(const bf16* __restrict__ x, int R, int C, int ld,
                                                          int rows_per, float* __restrict__ part) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int r0 = blockIdx.y * rows_per, r1 = min(R, r0 + rows_per);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
    for (int r = r0 + q; r < r1; r += 4) {
      float f[8];
      unpack8(*(const uint4*)(x + (long long)r * ld + c0), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[q][lane * 8 + j] = s[j];
  __syncthreads();
  for (int t = threadIdx.x; t < 512; t += 256) {
    const int c = blockIdx.x * 512 + t;
    if (c < C) part[(long long)blockIdx.y * C + c] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
  }
}

__global__ void add_int_kernel(int* p, int v) { if (threadIdx.x == 0) p[0] += v; }

int grid_for(long long work, int cap) {
  long long g = (work + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" int rk_softmax_xent(const float* logits, int ldl, const int* labels, int B, int ncls, int ignore_index,
                               float grad_scale, void* dlogits, int ldd, float* probs, float* loss_sum, int* correct,
                               int* counted, void* stream) {
  if (B <= 0) return RK_OK;
  hipLaunchKernelGGL(softmax_xent_kernel<bf16>, dim3(rk_cdiv(B, 4)), dim3(256), 0, (hipStream_t)stream, logits, ldl,
                     labels, B, ncls, ignore_index, grad_scale, (bf16*)dlogits, ldd, probs, loss_sum, correct, counted,
                     nullptr);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// same with fp32 d(logits) (fp32 training path)
extern "C" int rk_softmax_xent_f32(const float* logits, int ldl, const int* labels, int B, int ncls, int ignore_index,
                                   float grad_scale, float* dlogits, int ldd, float* probs, float* loss_sum,
                                   int* correct, int* counted, void* stream) {
  if (B <= 0) return RK_OK;
  hipLaunchKernelGGL(softmax_xent_kernel<float>, dim3(rk_cdiv(B, 4)), dim3(256), 0, (hipStream_t)stream, logits, ldl,
                     labels, B, ncls, ignore_index, grad_scale, dlogits, ldd, probs, loss_sum, correct, counted,
                     nullptr);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// fp32 d(logits) with a device scale factor: gradient and loss both times *scale (mean over a
// data-dependent count, e.g. the non-ignored tokens of a tagger batch)
extern "C" int rk_softmax_xent_f32s(const float* logits, int ldl, const int* labels, int B, int ncls,
                                    int ignore_index, const float* scale, float* dlogits, int ldd, float* loss_sum,
                                    void* stream) {
  if (B <= 0) return RK_OK;
  hipLaunchKernelGGL(softmax_xent_kernel<float>, dim3(rk_cdiv(B, 4)), dim3(256), 0, (hipStream_t)stream, logits, ldl,
                     labels, B, ncls, ignore_index, 1.0f, dlogits, ldd, nullptr, loss_sum, nullptr, nullptr, scale);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_sgd_step(float* w, void* wb, const float* g, float* mom, long long n, float lr, float momentum,
                           float wd, int nesterov, float gscale, const float* lr_ptr, long long decay_end, int* bump,
                           void* stream) {
  if (n % 4 || decay_end % 4) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n / 4, 4096)), dim3(256), 0, (hipStream_t)stream, w, (bf16*)wb, g, mom,
                     n, lr, momentum, wd, nesterov, gscale, lr_ptr, decay_end, bump);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_adam_step(float* w, void* wb, const float* g, float* m, float* v, long long n, float lr, float b1,
                            float b2, float omb1, float omb2, float eps, float wd, int decoupled, float c1, float c2,
                            float gscale, const int* skip, const int* step_ptr, void* stream) {
  if (n % 4) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4, 4096)), dim3(256), 0, (hipStream_t)stream, w, (bf16*)wb, g, m,
                     v, n, lr, b1, b2, omb1, omb2, eps, wd, decoupled, c1, c2, gscale, skip, step_ptr);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_lerp(float* dst, const float* src, void* dstb, long long n, float t, void* stream) {
  hipLaunchKernelGGL(lerp_kernel, dim3(grid_for(n, 4096)), dim3(256), 0, (hipStream_t)stream, dst, src, (bf16*)dstb,
                     n, t);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// zero n 4-byte elements (16-B aligned base: a torch allocation or an offset multiple of 4 elements)
extern "C" int rk_zero32(void* dst, long long n, void* stream) {
  if (n < 0 || (n > 0 && !dst)) return RK_EBADARG;
  if (n == 0) return RK_OK;
  if (((unsigned long long)dst) & 15) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(zero32_kernel, dim3(grid_for((n + 3) / 4, 2048)), dim3(256), 0, (hipStream_t)stream,
                     (unsigned*)dst, n);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_nonfinite(const float* x, long long n, int* flag, void* stream) {
  hipLaunchKernelGGL(nonfinite_kernel, dim3(grid_for(n, 2048)), dim3(256), 0, (hipStream_t)stream, x, n, flag);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_reduce_slabs(const float* slab, int S, long long n, float* out, int accumulate, float scale,
                               void* stream) {
  if (n % 4) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(grid_for(n / 4, 4096)), dim3(256), 0, (hipStream_t)stream, slab, S, n,
                     out, accumulate, scale);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_reduce_slabs_epi(const float* slab, int S, int M, int N, const float* bias, int act, float slope,
                                   float alpha, void* outb, float* outf, int ldc, void* stream) {
  if (N % 4 || ldc % 4) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(reduce_slabs_epi_kernel, dim3(grid_for((long long)M * N / 4, 4096)), dim3(256), 0,
                     (hipStream_t)stream, slab, S, M, N, bias, act, slope, alpha, (bf16*)outb, outf, ldc);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// ---- split-K combine for conv forward / data-gradient ----------------------------------------
// out[m][n] (bf16) = sum_s slab[s][m][n] with the igemm tile epilogue's BatchNorm options, so the
// small-M convs (VGG 4x4 / 8x8 layers: 64-128 output tiles of 128x128) can split K over the chip:
//   mode 0 plain; mode 1 forward statistics (sum v, sum v^2) -> fp64 slot table acc [SL][2][N];
//   mode 2 FLAG_BNB data-gradient: v *= [y*scale + shift > 0], (sum v, sum v*y) -> acc;
//   mode 3 ReLU-backward gate: v *= [gate > 0].
// A block sweeps whole rows: N/4 threads per row (4 fixed channels each), 256/(N/4) rows per sweep,
// so a thread's channel sums stay in registers; one LDS fold per block, then one fp64 atomic per
// (kind, channel) per block into slot blockIdx & slmask (the grid is capped to bound atomics).
__global__ __launch_bounds__(256) void slab_epi_kernel(const float* __restrict__ slab, int S, int M, int N, int mode,
                                                       const bf16* __restrict__ gate, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, double* __restrict__ acc,
                                                       int slmask, bf16* __restrict__ out) {
  __shared__ float red[2][1024];
  const int tpr = N >> 2, rpb = 256 / tpr;
  const int tid = threadIdx.x, c4 = tid % tpr, r0 = tid / tpr;
  const long long sn = (long long)M * N;
  float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sh = {0.f, 0.f, 0.f, 0.f};
  if (mode == 2) {
    sc = *(const f32x4*)(scale + 4 * c4);
    sh = *(const f32x4*)(shift + 4 * c4);
  }
  // rows of one sweep: U rows per thread with every slab (and gate) load issued before any add —
  // the grid is capped (atomics), so each thread walks many rows and a one-row loop is latency-bound
  constexpr int U = 8;
  const int step = gridDim.x * rpb;
  for (int m0 = blockIdx.x * rpb + r0; m0 < M; m0 += U * step) {
    f32x4 av[U];
    bf16x4 gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * step;
      const long long i = (long long)(m < M ? m : m0) * N + 4 * c4;
      av[u] = *(const f32x4*)(slab + i);
      if (mode >= 2) gv[u] = *(const bf16x4*)(gate + i);
    }
    for (int s1 = 1; s1 < S; ++s1) {  // fixed summation order per element
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = m0 + u * step;
        v[u] = *(const f32x4*)(slab + s1 * sn + (long long)(m < M ? m : m0) * N + 4 * c4);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) av[u] += v[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * step;
      if (m >= M) break;
      const long long i = (long long)m * N + 4 * c4;
      f32x4 a = av[u];
      if (mode >= 2) {
        const bf16x4 g = gv[u];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float yv = (float)g[e];
          if (mode == 3) {
            a[e] = yv > 0.f ? a[e] : 0.f;
          } else {
            a[e] = yv * sc[e] + sh[e] > 0.f ? a[e] : 0.f;
            s[e] += a[e];
            q[e] += a[e] * yv;
          }
        }
      } else if (mode == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[e] += a[e];
          q[e] += a[e] * a[e];
        }
      }
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)a[e];
      *(bf16x4*)(out + i) = o;
    }
  }
  if (mode == 1 || mode == 2) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[0][r0 * N + 4 * c4 + e] = s[e];
      red[1][r0 * N + 4 * c4 + e] = q[e];
    }
    __syncthreads();
    double* dst = acc + (long long)(blockIdx.x & slmask) * 2 * N;
    for (int c = tid; c < 2 * N; c += 256) {
      const int k = c >= N ? 1 : 0, ch = c - k * N;
      float v = 0.f;
      for (int r = 0; r < rpb; ++r) v += red[k][r * N + ch];
      unsafeAtomicAdd(dst + (long long)k * N + ch, (double)v);
    }
  }
}

extern "C" int rk_slab_epi(const float* slab, int S, int M, int N, int mode, const void* gate, const float* scale,
                           const float* shift, double* acc, int slmask, void* out, void* stream) {
  if (S <= 0 || M <= 0 || N % 4 || N > 1024 || 256 % (N / 4) || mode < 0 || mode > 3) return RK_EUNSUPPORTED;
  if ((mode == 1 || mode == 2) && !acc) return RK_EBADARG;
  if (mode >= 2 && !gate) return RK_EBADARG;
  if (mode == 2 && (!scale || !shift)) return RK_EBADARG;
  const int rpb = 256 / (N / 4);
  // with statistics every block adds 2N fp64 values into at most 8 slots: same-address atomics from
  // many blocks serialise at the memory side (measured 17 us at 256 blocks for a 4 MB output), so
  // the statistics modes run fewer, wider blocks
  const int cap = (mode == 1 || mode == 2) ? 64 : 256;
  const int blocks = min((M + rpb - 1) / rpb, cap);
  hipLaunchKernelGGL(slab_epi_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, slab, S, M, N, mode,
                     (const bf16*)gate, scale, shift, acc, slmask, (bf16*)out);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// ---- flipped, transposed conv weights for the data gradient ------------------------------------
// wt[ci][8 - t][co] = w[co][t][ci] for every listed 3x3 layer in ONE launch: the data gradient is then
// a FORWARD conv of dy with wt, so it runs on the forward kernels, whose weight operand is K-inner
// (one ds_read_b128 per MFMA fragment; the K-outer dgrad operand needs two transposing reads) and
// whose tuned tiles are the faster ones.  A block moves one 64 co x 64 ci tile of one tap through LDS
// (coalesced 128-B rows both ways).  desc[b] = {layer, tap, co0, ci0}; meta[l] = {src, dst, Cout, Cin}
// (element offsets into the two bf16 arenas).
__global__ __launch_bounds__(256) void conv_wt_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                      const int* __restrict__ desc, const long long* __restrict__ meta) {
  __shared__ bf16 tile[64][64 + 8];
  const int4 d = ((const int4*)desc)[blockIdx.x];
  const int layer = d.x, tap = d.y, co0 = d.z, ci0 = d.w;
  const long long so = meta[4 * layer], dso = meta[4 * layer + 1];
  const int Cout = (int)meta[4 * layer + 2], Cin = (int)meta[4 * layer + 3];
  const int tid = threadIdx.x;
  // load: row r = co (64 rows), 64 ci per row as 8 x 16-B vectors
  for (int v = tid; v < 64 * 8; v += 256) {
    const int r = v >> 3, c8 = (v & 7) * 8;
    const int co = co0 + r, ci = ci0 + c8;
    if (co < Cout && ci < Cin) {
      const bf16* s = src + so + ((long long)co * 9 + tap) * Cin + ci;
      if (ci + 8 <= Cin) {
        const bf16x8 x = *(const bf16x8*)s;
#pragma unroll
        for (int e = 0; e < 8; ++e) tile[r][c8 + e] = x[e];
      } else {
        for (int e = 0; e < Cin - ci; ++e) tile[r][c8 + e] = s[e];
      }
    }
  }
  __syncthreads();
  // store: row = ci, 64 co contiguous
  for (int v = tid; v < 64 * 8; v += 256) {
    const int r = v >> 3, c8 = (v & 7) * 8;
    const int ci = ci0 + r, co = co0 + c8;
    if (ci < Cin && co < Cout) {
      bf16* t = dst + dso + ((long long)ci * 9 + (8 - tap)) * Cout + co;
      if (co + 8 <= Cout) {
        bf16x8 x;
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = tile[c8 + e][r];
        *(bf16x8*)t = x;
      } else {
        for (int e = 0; e < Cout - co; ++e) t[e] = tile[c8 + e][r];
      }
    }
  }
}

extern "C" int rk_conv_wt(const void* src, void* dst, const int* desc, int nblocks, const long long* meta,
                          void* stream) {
  if (nblocks <= 0) return RK_EBADARG;
  hipLaunchKernelGGL(conv_wt_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, (const bf16*)src, (bf16*)dst,
                     desc, meta);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// lr_table (nullable): *lr_out = lr_table[*counter] (the optimizer kernel later in the step reads lr_out)
// sched [nsteps][B] row indices into data [nrows][row_bytes]; lr_table [nsteps]
extern "C" int rk_gather_batch(const void* data, long long row_bytes, const int* labels, const long long* sched,
                               int* counter, int B, void* out, int* out_y, double* zero, long long zero_n, int* done,
                               const float* lr_table, float* lr_out, int nsteps, long long nrows, void* stream) {
  if (row_bytes % 16 || zero_n < 0 || (zero_n && !zero) || (lr_table && !lr_out)) return RK_EUNSUPPORTED;
  if (nsteps <= 0 || nrows <= 0) return RK_EBADARG;
  const long long rv = row_bytes / 16;
  hipLaunchKernelGGL(gather_batch_kernel, dim3(grid_for((long long)B * rv, 2048)), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)data, rv, labels, sched, counter, B, (uint4*)out, out_y, zero, zero_n, done,
                     lr_table, lr_out, nsteps, nrows);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_colsum(const void* x, int R, int C, int ld, float* out, int accumulate, void* stream) {
  hipLaunchKernelGGL(colsum_kernel, dim3(rk_cdiv(C, 64)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, R, C, ld,
                     out, accumulate);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_colsum_part(const void* x, int R, int C, int ld, int chunks, float* part, void* stream) {
  if (C % 8 || ld % 8 || chunks < 1 || chunks > 65535) return RK_EUNSUPPORTED;
  const int rows_per = rk_cdiv(R, chunks);
  hipLaunchKernelGGL(colsum_part_kernel, dim3(rk_cdiv(C, 512), chunks), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, R, C, ld, rows_per, part);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_ensemble_mean(const float* probs, int Wm, long long n, const float* weights, float* out,
                                void* stream) {
  hipLaunchKernelGGL(ensemble_mean_kernel, dim3(grid_for(n, 2048)), dim3(256), 0, (hipStream_t)stream, probs, Wm, n,
                     weights, out);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_cast_f32_bf16(const float* src, void* dst, long long n, void* stream) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n, 4096)), dim3(256), 0, (hipStream_t)stream, src, (bf16*)dst,
                     n);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_pack_nhwc(const void* src, int is_u8, int N, int C, int H, int W, int Cp, float scale, float shift,
                            void* dst, void* stream) {
  hipLaunchKernelGGL(pack_nhwc_kernel, dim3(grid_for((long long)N * H * W * Cp, 8192)), dim3(256), 0,
                     (hipStream_t)stream, src, is_u8, N, C, H, W, Cp, scale, shift, (bf16*)dst);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_add_int(int* p, int v, void* stream) {
  hipLaunchKernelGGL(add_int_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, p, v);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_rows_reduce(const float* in, int R, long long W, int G, float* out, void* stream) {
  if (G <= 0 || G > 65535) return RK_EBADARG;
  dim3 grid((unsigned)((W + 255) / 256), (unsigned)G);
  hipLaunchKernelGGL(rows_reduce_kernel, grid, dim3(256), 0, (hipStream_t)stream, in, R, W, out);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_fold_rows(const float* in, int R, long long n, float* out, int accumulate, float scale,
                            void* stream) {
  if (R <= 0 || n <= 0) return RK_EBADARG;
  if (n % 4) return RK_EUNSUPPORTED;
  const long long blocks = (n + 63) / 64;
  if (blocks > 0x7fffffffLL) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(fold_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, in, R, n, out,
                     accumulate, scale);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// the multi-segment launches: nblk blocks over the chunk table blk (see adam_multi_kernel)
extern "C" int rk_adam_multi(float* w, void* wb, const float* g, float* m, float* v, const long long* blk, int nblk,
                             const float* segp, float b1, float b2, float omb1, float omb2, int decoupled, float gscale,
                             const int* skip, const int* step_ptr, int* bump, void* stream) {
  if (nblk <= 0 || !blk || !segp || !step_ptr) return RK_EBADARG;
  if ((((unsigned long long)w) | ((unsigned long long)g) | ((unsigned long long)m) | ((unsigned long long)v)) & 15)
    return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, w, (bf16*)wb, g, m, v,
                     blk, segp, b1, b2, omb1, omb2, decoupled, gscale, skip, step_ptr, bump);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_zero_multi(void* dst, const long long* blk, int nblk, int* flag, void* stream) {
  if (nblk <= 0 || !blk || !dst) return RK_EBADARG;
  if (((unsigned long long)dst) & 15) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(zero_multi_kernel, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, (unsigned*)dst, blk,
                     flag);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_lerp_multi(float* dst, const float* src, void* dstb, const long long* blk, int nblk, float t,
                             void* stream) {
  if (nblk <= 0 || !blk || !dst || !src) return RK_EBADARG;
  if ((((unsigned long long)dst) | ((unsigned long long)src) | ((unsigned long long)dstb)) & 15) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(lerp_multi_kernel, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, dst, src, (bf16*)dstb,
                     blk, t);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

extern "C" int rk_nonfinite_multi(const float* x, const long long* blk, int nblk, int* flag, int* bump,
                                  void* stream) {
  if (nblk <= 0 || !blk || !x || !flag) return RK_EBADARG;
  if (((unsigned long long)x) & 15) return RK_EUNSUPPORTED;
  hipLaunchKernelGGL(nonfinite_multi_kernel, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, x, blk, flag,
                     bump);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
