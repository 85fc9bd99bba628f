// Embedding lookup and its deterministic gradient for gfx950 (the PyBiLstm tagger's word embedding,
// reference examples/models/pos_tagging/PyBiLstm.py:249-268 ``nn.Embedding(V, E, padding_idx=0)``).
//
//  * rk_embedding_fwd: out[i][:] = W[ids[i]][:] — one thread per 16-B vector of a row (the padding row's
//    weights stay zero by construction, so it is gathered like any other);
//  * rk_embedding_bwd: dW[v][:] = sum over tokens i with ids[i] == v of dy[i][:], in ascending token
//    order (bit-reproducible, unlike an atomic scatter-add): a stable radix sort of (id, token) pairs
//    (rocPRIM through hipCUB), then one wave per run of equal ids sums that run's dy rows in order and
//    writes the row; rows no token touches are zeroed by the same launch; the padding row gets no
//    gradient (torch's padding_idx semantics).
#include "common.h"
#include <hipcub/hipcub.hpp>

namespace {

__global__ __launch_bounds__(256) void embedding_fwd_kernel(const long long* __restrict__ ids,
                                                            const float* __restrict__ w, float* __restrict__ out,
                                                            int n, int E4, int V) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n * E4) return;
  const int tok = (int)(i / E4), c = (int)(i - (long long)tok * E4);
  long long id = ids[tok];
  id = id < 0 || id >= V ? 0 : id;   // an out-of-range id reads row 0 (the padding row) instead of past W
  ((f32x4*)out)[i] = ((const f32x4*)w)[id * E4 + c];
}

__global__ __launch_bounds__(256) void iota_kernel(int* __restrict__ v, const long long* __restrict__ ids,
                                                   int* __restrict__ keys, int n, int V) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  v[i] = i;
  const long long id = ids[i];
  keys[i] = id < 0 || id >= V ? 0 : (int)id;   // as the forward: out-of-range ids are row 0
}

// zero every row no token touches: rows v with no entry in the sorted ids (binary search), padding row too
__global__ __launch_bounds__(256) void embedding_zero_kernel(const int* __restrict__ skeys, int n, float* __restrict__ dw,
                                                             int V, int E4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)V * E4) return;
  const int v = (int)(i / E4);
  int lo = 0, hi = n;   // first sorted key >= v
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (skeys[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  if (lo == n || skeys[lo] != v) ((f32x4*)dw)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// one wave per sorted position: the first position of each run sums the run in ascending token order
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const int* __restrict__ skeys, const int* __restrict__ perm,
                                                            const float* __restrict__ dy, float* __restrict__ dw,
                                                            int n, int E, int padding_idx) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= n) return;
  const int v = skeys[j];
  if (j > 0 && skeys[j - 1] == v) return;   // not the start of a run
  int end = j + 1;
  while (end < n && skeys[end] == v) ++end;
  for (int c = lane; c < E; c += 64) {
    float s = 0.f;
    if (v != padding_idx)
      for (int k = j; k < end; ++k) s += dy[(long long)perm[k] * E + c];
    dw[(long long)v * E + c] = s;
  }
}

}  // namespace

// out [n][E] = W[ids] (E % 4 == 0, V rows of W)
extern "C" int rk_embedding_fwd(const long long* ids, const float* w, float* out, int n, int E, int V, void* stream) {
  if (n <= 0) return RK_OK;
  if (E <= 0 || (E & 3)) return RK_EUNSUPPORTED;
  const long long t = (long long)n * (E / 4);
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ids,
                     w, out, n, E / 4, V);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// workspace bytes rk_embedding_bwd needs for n tokens
extern "C" long long rk_embedding_bwd_ws(int n) {
  size_t tmp = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const int*)nullptr, (int*)nullptr, (const int*)nullptr,
                                     (int*)nullptr, n);
  return (long long)(tmp + 4ull * n * sizeof(int) + 256);
}

// dW [V][E] = scatter-sum of dy [n][E] by ids (every row written; padding_idx's row zero; -1: none)
extern "C" int rk_embedding_bwd(const long long* ids, const float* dy, float* dw, int n, int V, int E, int padding_idx,
                                void* ws, long long ws_bytes, void* stream) {
  if (n <= 0 || V <= 0 || E <= 0 || (E & 3)) return RK_EBADARG;
  if (ws_bytes < rk_embedding_bwd_ws(n)) return RK_EBADARG;
  hipStream_t st = (hipStream_t)stream;
  int* keys = (int*)ws;
  int* vals = keys + n;
  int* skeys = vals + n;
  int* perm = skeys + n;
  void* tmp = (void*)(((uintptr_t)(perm + n) + 255) & ~(uintptr_t)255);
  size_t tmp_bytes = (size_t)(ws_bytes - ((char*)tmp - (char*)ws));
  hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, st, vals, ids, keys, n, V);
  RK_LAUNCH_CHECK();
  int bits = 1;
  while (bits < 31 && (1 << bits) < V) ++bits;
  if (hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, skeys, vals, perm, n, 0, bits, st) != hipSuccess)
    return RK_ELAUNCH;
  const long long z = (long long)V * (E / 4);
  hipLaunchKernelGGL(embedding_zero_kernel, dim3((unsigned)((z + 255) / 256)), dim3(256), 0, st, skeys, n, dw, V,
                     E / 4);
  RK_LAUNCH_CHECK();
  hipLaunchKernelGGL(embedding_bwd_kernel, dim3((n + 3) / 4), dim3(256), 0, st, skeys, perm, dy, dw, n, E,
                     padding_idx);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
