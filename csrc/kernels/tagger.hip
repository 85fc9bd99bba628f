// Kernels of the native BiLSTM tagger training step (PyBiLstm; reference
// examples/models/pos_tagging/PyBiLstm.py:185-235 train loop, :249-268 Embedding -> Dropout -> BiLSTM ->
// Linear).  With these, the whole step (engine/tagger.py) runs on in-tree kernels: the GEMMs on sgemm.hip,
// the recurrence on lstm.hip, cross-entropy and Adam on loss_optim.hip, and here
//
//   * rk_tag_embed_fwd: embedding gather fused with the dropout mask — one thread per 16-B vector of a
//     row; the keep decision of element i is Philox4x32-10 at counter (i / 4, stream id, device step),
//     so a replayed graph draws a fresh mask every step; the 0 / (1 / (1 - p)) multipliers are kept for
//     the backward (n x E floats, cheaper than recomputing Philox there);
//   * rk_tag_embed_bwd: dW[v] = sum of dropout-masked dy rows of the tokens with id v, in ascending token
//     order.  The host already holds the batch's ids, so it sorts them (numpy stable argsort, overlapped
//     with the previous step on the GPU) and uploads (perm, run ids, run starts) with the batch; one wave
//     per run sums its rows in order: bit-reproducible, no device sort, no float atomics.  Rows no token
//     touches keep the zeros of the gradient arena's memset; the padding id's run is listed as id -1
//     and skipped (torch's padding_idx semantics);
//   * rk_tag_transpose: W_hh [2][4HP][HP] -> [2][HP][4HP] for the BPTT kernel, once per step (the weights
//     change every step), 32 x 32 LDS tiles;
//   * rk_tag_add: out = a + b (or a copy): the combined LSTM bias b_ih + b_hh of the input projection,
//     and the bias gradient written to both parameters (nn.LSTM keeps two bias vectors, each with the
//     same gradient; Adam treats them as separate parameters, so both are kept).
#include "common.h"
#include "philox.h"

namespace {

__global__ __launch_bounds__(256) void tag_embed_fwd_kernel(const int* __restrict__ ids, const float* __restrict__ w,
                                                            float* __restrict__ out, float* __restrict__ mask, int n,
                                                            int E4, int V, float p, float inv_keep, uint32_t k0,
                                                            uint32_t k1, uint32_t sid, const int* __restrict__ step) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n * E4) return;
  const int tok = (int)(i / E4), c = (int)(i - (long long)tok * E4);
  int id = ids[tok];
  id = id < 0 || id >= V ? 0 : id;   // out-of-range ids read the (zero) padding row
  f32x4 v = ((const f32x4*)w)[(long long)id * E4 + c];
  if (mask) {
    const uint32_t st = step ? (uint32_t)step[0] : 0u;
    const U4 r = philox4x32_10((uint32_t)i, (uint32_t)(i >> 32), sid, st, k0, k1);
    f32x4 m;
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e] = u01(r.v[e]) >= p ? inv_keep : 0.f;
    v *= m;
    ((f32x4*)mask)[i] = m;
  }
  ((f32x4*)out)[i] = v;
}

// one wave per run u < nruns[0]: dw[uniq[u]][:] = sum_{k = start[u]}^{start[u+1]-1} dy[perm[k]][:] * mask
__global__ __launch_bounds__(256) void tag_embed_bwd_kernel(const int* __restrict__ perm, const int* __restrict__ uniq,
                                                            const int* __restrict__ start, const int* __restrict__ nruns,
                                                            const float* __restrict__ dy,
                                                            const float* __restrict__ mask, float* __restrict__ dw,
                                                            int maxruns, int E, int V) {
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (u >= maxruns || u >= nruns[0]) return;
  const long long v = uniq[u];
  if (v < 0 || v >= V) return;       // the padding id's run (and, like the forward's clamp, any id out of range)
  const int k0 = start[u], k1 = start[u + 1];
  for (int c = lane; c < E; c += 64) {
    float s = 0.f;
    for (int k = k0; k < k1; ++k) {
      const long long o = (long long)perm[k] * E + c;
      s += mask ? dy[o] * mask[o] : dy[o];
    }
    dw[v * E + c] = s;
  }
}

// dst[g][c][r] = src[g][r][c]
__global__ __launch_bounds__(256) void tag_transpose_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                            int R, int C) {
  __shared__ float t[32][33];
  const int g = blockIdx.z, r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const float* s = src + (long long)g * R * C;
  float* d = dst + (long long)g * R * C;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
#pragma unroll
  for (int k = 0; k < 32; k += 8)
    if (r0 + ty + k < R && c0 + tx < C) t[ty + k][tx] = s[(long long)(r0 + ty + k) * C + c0 + tx];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8)
    if (c0 + ty + k < C && r0 + tx < R) d[(long long)(c0 + ty + k) * R + r0 + tx] = t[tx][ty + k];
}

__global__ __launch_bounds__(256) void tag_add_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                      float* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = b ? a[i] + b[i] : a[i];
}

}  // namespace

// out [n][E] = W[ids] (* dropout multipliers, written to mask, when p > 0); E % 4 == 0, V rows of W
extern "C" int rk_tag_embed_fwd(const int* ids, const float* w, float* out, float* mask, int n, int E, int V, float p,
                                unsigned long long seed, int stream_id, const int* step, void* stream) {
  if (n <= 0) return RK_OK;
  if (E <= 0 || (E & 3) || V <= 0 || p < 0.f || p >= 1.f) return RK_EBADARG;
  if (p > 0.f && !mask) return RK_EBADARG;
  const long long t = (long long)n * (E / 4);
  hipLaunchKernelGGL(tag_embed_fwd_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ids,
                     w, out, p > 0.f ? mask : nullptr, n, E / 4, V, p, 1.0f / (1.0f - p), (uint32_t)seed,
                     (uint32_t)(seed >> 32), (uint32_t)stream_id, step);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// dW rows of the runs (uniq, start [maxruns + 1], nruns on the device); mask nullable (no dropout)
extern "C" int rk_tag_embed_bwd(const int* perm, const int* uniq, const int* start, const int* nruns, const float* dy,
                                const float* mask, float* dw, int maxruns, int E, int V, void* stream) {
  if (maxruns <= 0) return RK_OK;
  if (E <= 0 || V <= 0) return RK_EBADARG;
  hipLaunchKernelGGL(tag_embed_bwd_kernel, dim3((unsigned)((maxruns + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     perm, uniq, start, nruns, dy, mask, dw, maxruns, E, V);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// G matrices [R][C] -> [C][R]
extern "C" int rk_tag_transpose(const float* src, float* dst, int G, int R, int C, void* stream) {
  if (G <= 0 || R <= 0 || C <= 0) return RK_EBADARG;
  hipLaunchKernelGGL(tag_transpose_kernel, dim3((unsigned)rk_cdiv(C, 32), (unsigned)rk_cdiv(R, 32), (unsigned)G),
                     dim3(256), 0, (hipStream_t)stream, src, dst, R, C);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// out = a + b (b null: out = a)
extern "C" int rk_tag_add(const float* a, const float* b, float* out, long long n, void* stream) {
  if (n <= 0) return RK_OK;
  hipLaunchKernelGGL(tag_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a, b, out,
                     n);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
