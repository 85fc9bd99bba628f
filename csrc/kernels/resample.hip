// PG-GAN resampling kernels for gfx950 (reference pg_gans.py:1042-1067).
//
//  * rk_resample2x: nearest 2x upscale (upscale2d) and 2x2 box downscale (downscale2d = 0.25 x the
//    2x2 sum) of NHWC maps, fp32 or bf16, 16-B vectors of channels per thread.  They are each other's
//    adjoints up to the scale (d upscale = sum-pool, d downscale = 0.25 x upscale), so the autograd
//    layer differentiates them any number of times with these two kernels.
//  * rk_s2t_weights: the transposed-conv weight layout of the stride-2 gather convolutions (the
//    4x4 / stride-2 down-conv and its adjoint, the 2x up-conv): out[g][ci][t4][co] =
//    W[co][tap(g, t4)][ci] for the 4 output parities g, 4 taps each — LDS-tiled 32 x 32 transposes.
#include "common.h"

namespace {

template <class T> struct V4;
template <> struct V4<float> {
  typedef f32x4 vec;
  static RK_DEV void ld(const float* p, float (&f)[4]) {
    const f32x4 v = *(const f32x4*)p;
    f[0] = v[0]; f[1] = v[1]; f[2] = v[2]; f[3] = v[3];
  }
  static RK_DEV void st(float* p, const float (&f)[4]) { *(f32x4*)p = f32x4{f[0], f[1], f[2], f[3]}; }
};
template <> struct V4<bf16> {
  static RK_DEV void ld(const bf16* p, float (&f)[4]) {
    const bf16x4 v = *(const bf16x4*)p;
    f[0] = (float)v[0]; f[1] = (float)v[1]; f[2] = (float)v[2]; f[3] = (float)v[3];
  }
  static RK_DEV void st(bf16* p, const float (&f)[4]) {
    *(bf16x4*)p = bf16x4{(bf16)f[0], (bf16)f[1], (bf16)f[2], (bf16)f[3]};
  }
};

// up: dst [N, 2h, 2w, C] = scale * src[N, h, w, C] (nearest); one thread per destination 4-vector
template <class T>
__global__ __launch_bounds__(256) void up2_kernel(const T* __restrict__ src, T* __restrict__ dst, int N, int h, int w,
                                                  int C, float scale) {
  const int C4 = C >> 2;
  const long long total = (long long)N * 4 * h * w * C4;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    const long long pix = e / C4;
    const int X = (int)(pix % (2 * w));
    const long long t = pix / (2 * w);
    const int Y = (int)(t % (2 * h));
    const long long n = t / (2 * h);
    float f[4];
    V4<T>::ld(src + (((n * h + (Y >> 1)) * w + (X >> 1)) * C + c4 * 4), f);
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] *= scale;
    V4<T>::st(dst + pix * C + c4 * 4, f);
  }
}

// down: dst [N, H/2, W/2, C] = scale * (2x2 sum of src [N, H, W, C])
template <class T>
__global__ __launch_bounds__(256) void down2_kernel(const T* __restrict__ src, T* __restrict__ dst, int N, int H, int W,
                                                    int C, float scale) {
  const int C4 = C >> 2, h = H >> 1, w = W >> 1;
  const long long total = (long long)N * h * w * C4;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int c4 = (int)(e % C4);
    const long long pix = e / C4;
    const int x = (int)(pix % w);
    const long long t = pix / w;
    const int y = (int)(t % h);
    const long long n = t / h;
    const T* s0 = src + (((n * H + 2 * y) * W + 2 * x) * C + c4 * 4);
    float a[4], b[4], c[4], d[4], o[4];
    V4<T>::ld(s0, a);
    V4<T>::ld(s0 + C, b);
    V4<T>::ld(s0 + (long long)W * C, c);
    V4<T>::ld(s0 + (long long)W * C + C, d);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = ((a[i] + b[i]) + (c[i] + d[i])) * scale;
    V4<T>::st(dst + pix * C + c4 * 4, o);
  }
}

// tap offsets of the stride-2 gather: 4x4 taps t = 4a + b at (a - 1, b - 1); output parity r takes
// the taps with (r - d) even, source offset s = (r - d) / 2: r = 0 -> d in {0, 2}, r = 1 -> d in {-1, 1}
RK_DEV int par_d(int r, int u) { return r == 0 ? (u == 0 ? 0 : 2) : (u == 0 ? 1 : -1); }

// out[g][ci][t4][co] = W[co][tap][ci], g = 2 ry + rx, t4 = 2u + v, tap = 4 (d(ry,u)+1) + d(rx,v)+1.
// grid (ceil(Ci/32), ceil(Co/32), 16 = g x t4), block 256 (32 x 8)
__global__ __launch_bounds__(256) void s2t_weights_kernel(const float* __restrict__ W, float* __restrict__ out,
                                                          int Co, int Ci) {
  __shared__ float tile[32][33];
  const int ci0 = blockIdx.x * 32, co0 = blockIdx.y * 32;
  const int g = blockIdx.z >> 2, t4 = blockIdx.z & 3;
  const int ry = g >> 1, rx = g & 1, u = t4 >> 1, v = t4 & 1;
  const int tap = 4 * (par_d(ry, u) + 1) + par_d(rx, v) + 1;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {   // read rows co, contiguous ci
    const int co = co0 + r, ci = ci0 + tx;
    tile[r][tx] = (co < Co && ci < Ci) ? W[((long long)co * 16 + tap) * Ci + ci] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {   // write rows ci, contiguous co
    const int ci = ci0 + r, co = co0 + tx;
    if (ci < Ci && co < Co) out[(((long long)g * Ci + ci) * 4 + t4) * Co + co] = tile[tx][r];
  }
}

// data-gradient weights of a taps-tap conv: out[ci][taps-1-t][co] = w[co][t][ci] (dgrad = forward conv
// of dy with these).  grid (ceil(Ci/32), ceil(Co/32), taps), block 256
__global__ __launch_bounds__(256) void wflip_t_kernel(const float* __restrict__ w, float* __restrict__ out, int Co,
                                                      int Ci, int taps) {
  __shared__ float tile[32][33];
  const int ci0 = blockIdx.x * 32, co0 = blockIdx.y * 32, t = blockIdx.z;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int co = co0 + r, ci = ci0 + tx;
    tile[r][tx] = (co < Co && ci < Ci) ? w[((long long)co * taps + t) * Ci + ci] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int ci = ci0 + r, co = co0 + tx;
    if (ci < Ci && co < Co) out[((long long)ci * taps + (taps - 1 - t)) * Co + co] = tile[tx][r];
  }
}

int grid_n(long long work, int cap) {
  long long g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : g > cap ? cap : g);
}

template <class T>
int resample_launch(int mode, const void* src, void* dst, int N, int H, int W, int C, float scale, hipStream_t s) {
  if (C % 4 || N <= 0 || H <= 0 || W <= 0) return RK_EUNSUPPORTED;
  if (mode == 0) {
    hipLaunchKernelGGL(up2_kernel<T>, dim3(grid_n((long long)N * 4 * H * W * (C / 4), 8192)), dim3(256), 0, s,
                       (const T*)src, (T*)dst, N, H, W, C, scale);
  } else if (mode == 1) {
    if (H % 2 || W % 2) return RK_EUNSUPPORTED;
    hipLaunchKernelGGL(down2_kernel<T>, dim3(grid_n((long long)N * (H / 2) * (W / 2) * (C / 4), 8192)), dim3(256), 0,
                       s, (const T*)src, (T*)dst, N, H, W, C, scale);
  } else {
    return RK_EBADARG;
  }
  RK_LAUNCH_CHECK();
  return RK_OK;
}

}  // namespace

// mode 0: dst = scale * upscale2x(src), src [N, H, W, C];  mode 1: dst = scale * sumpool2x2(src), src [N, H, W, C]
// is_bf16: element type (else fp32)
extern "C" int rk_resample2x(int mode, int is_bf16, const void* src, void* dst, int N, int H, int W, int C, float scale,
                             void* stream) {
  if (is_bf16) return resample_launch<bf16>(mode, src, dst, N, H, W, C, scale, (hipStream_t)stream);
  return resample_launch<float>(mode, src, dst, N, H, W, C, scale, (hipStream_t)stream);
}

// W [Co][16][Ci] fp32 -> out [4][Ci][4][Co]
extern "C" int rk_s2t_weights(const float* W, float* out, int Co, int Ci, void* stream) {
  if (Co <= 0 || Ci <= 0) return RK_EBADARG;
  hipLaunchKernelGGL(s2t_weights_kernel, dim3(rk_cdiv(Ci, 32), rk_cdiv(Co, 32), 16), dim3(256), 0, (hipStream_t)stream,
                     W, out, Co, Ci);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// w [Co][taps][Ci] fp32 -> out [Ci][taps][Co] with the taps reversed (conv data-gradient weights)
extern "C" int rk_wflip_t(const float* w, float* out, int Co, int Ci, int taps, void* stream) {
  if (Co <= 0 || Ci <= 0 || taps <= 0) return RK_EBADARG;
  hipLaunchKernelGGL(wflip_t_kernel, dim3(rk_cdiv(Ci, 32), rk_cdiv(Co, 32), taps), dim3(256), 0, (hipStream_t)stream,
                     w, out, Co, Ci, taps);
  RK_LAUNCH_CHECK();
  return RK_OK;
}

// ---- box-filter weights of the fused resampling convs (pg_gans.py:1035-1036 / 1055-1056) and their adjoints
// The 4x4 kernel W4[a][b] = s * sum of w3[ky][kx] over ky in {a-1, a}, kx in {b-1, b} (the four 1-pixel shifts
// of the zero-padded 3x3 kernel; flip: of the 180-degree-rotated kernel).  One thread per (co, ci):
//   mode 0: down  w [Co][9][Ci]  -> W4 [Co][16][Ci]          (s = 1/4)
//   mode 1: adjoint of mode 0: g4 [Co][16][Ci] -> g3 [Co][9][Ci]
//   mode 2: up    w [Co][9][Ci]  -> W4^T [Ci][16][Co], flipped (s = 1)
//   mode 3: adjoint of mode 2: g4 [Ci][16][Co] -> g3 [Co][9][Ci]
namespace {
__global__ __launch_bounds__(256) void box_weights_kernel(int mode, const float* __restrict__ src,
                                                         float* __restrict__ dst, int Co, int Ci, float s) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)Co * Ci) return;
  // modes 2 / 3 index the transposed [Ci][16][Co] layout with co fastest (coalesced on that side)
  const bool tr = mode >= 2;
  const int co = tr ? (int)(i % Co) : (int)(i / Ci);
  const int ci = tr ? (int)(i / Co) : (int)(i % Ci);
  const bool flip = mode >= 2;
  if (mode == 0 || mode == 2) {
    float g[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) g[q] = src[((long long)co * 9 + q) * Ci + ci];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float v = 0.f;
#pragma unroll
        for (int ky = a - 1; ky <= a; ++ky)
#pragma unroll
          for (int kx = b - 1; kx <= b; ++kx)
            if (ky >= 0 && ky < 3 && kx >= 0 && kx < 3) v += g[flip ? 8 - (ky * 3 + kx) : ky * 3 + kx];
        const int t = a * 4 + b;
        dst[tr ? ((long long)ci * 16 + t) * Co + co : ((long long)co * 16 + t) * Ci + ci] = s * v;
      }
  } else {
    float g4[16];
#pragma unroll
    for (int t = 0; t < 16; ++t)
      g4[t] = src[tr ? ((long long)ci * 16 + t) * Co + co : ((long long)co * 16 + t) * Ci + ci];
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const int qq = flip ? 8 - q : q;   // the 3x3 tap this output is, before the flip
      const int ky = qq / 3, kx = qq % 3;
      float v = 0.f;
#pragma unroll
      for (int a = ky; a <= ky + 1; ++a)
#pragma unroll
        for (int b = kx; b <= kx + 1; ++b) v += g4[a * 4 + b];
      dst[((long long)co * 9 + q) * Ci + ci] = s * v;
    }
  }
}
}  // namespace

extern "C" int rk_box_weights(int mode, const float* src, float* dst, int Co, int Ci, float scale, void* stream) {
  if (mode < 0 || mode > 3 || Co <= 0 || Ci <= 0 || !src || !dst) return RK_EBADARG;
  const long long n = (long long)Co * Ci;
  hipLaunchKernelGGL(box_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, mode,
                     src, dst, Co, Ci, scale);
  RK_LAUNCH_CHECK();
  return RK_OK;
}
