// Winograd weight transforms shared by winograd.hip (F(2x2,3x3)) and winograd4.hip (F(4x4,3x3) and its X6
// bf16 planes): one 32 co x 32 ci block of 3x3 filters per 256-thread workgroup, staged through LDS so the
// [pos][Co][Ci] (forward) and [pos][Ci][Co] (data-gradient) layouts are both written coalesced.
// Included inside each translation unit's anonymous namespace.
#pragma once
#include "common.h"

// U = G g G^T of every (co, ci) 3x3 filter g = w[co][ky*3+kx][ci]: u[pos][co][ci]; optionally the
// data-gradient set ut[pos][ci][co] = U[p(pos)][co][ci] with p swapping positions 0 and 3 per axis.
// Block = 32 co x 32 ci filters staged through LDS (coalesced both ways).
RK_DEV void w_transform(const float (&g)[9], float (&U)[16]) {
  float t[4][3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const float g0 = g[kx], g1 = g[3 + kx], g2 = g[6 + kx];
    t[0][kx] = g0;
    t[1][kx] = 0.5f * (g0 + g1 + g2);
    t[2][kx] = 0.5f * (g0 - g1 + g2);
    t[3][kx] = g2;
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    U[a * 4 + 0] = t[a][0];
    U[a * 4 + 1] = 0.5f * (t[a][0] + t[a][1] + t[a][2]);
    U[a * 4 + 2] = 0.5f * (t[a][0] - t[a][1] + t[a][2]);
    U[a * 4 + 3] = t[a][2];
  }
}

// one 32 co x 32 ci block of filters: LDS-staged so both output layouts are written coalesced
RK_DEV void wt_block(const float* __restrict__ w, float* __restrict__ u, float* __restrict__ ut, int Co, int Ci,
                     int co0, int ci0, float (&g)[32][9][33]) {
  float st[36];   // all loads in flight before the first LDS store
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
  if (u != nullptr)
    for (int i = threadIdx.x; i < 1024; i += 256) {
      const int ci = i & 31, co = i >> 5;
      if (co0 + co >= Co || ci0 + ci >= Ci) continue;
      float gg[9], U[16];
#pragma unroll
      for (int t = 0; t < 9; ++t) gg[t] = g[co][t][ci];
      w_transform(gg, U);
#pragma unroll
      for (int q = 0; q < 16; ++q) u[((long long)q * Co + co0 + co) * Ci + ci0 + ci] = U[q];
    }
  if (ut == nullptr) return;
  for (int i = threadIdx.x; i < 1024; i += 256) {
    const int co = i & 31, ci = i >> 5;
    if (co0 + co >= Co || ci0 + ci >= Ci) continue;
    float gg[9], U[16];
#pragma unroll
    for (int t = 0; t < 9; ++t) gg[t] = g[co][t][ci];
    w_transform(gg, U);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int a = q >> 2, bq = q & 3;
      const int pa = a == 0 ? 3 : a == 3 ? 0 : a, pb = bq == 0 ? 3 : bq == 3 ? 0 : bq;
      ut[((long long)q * Ci + ci0 + ci) * Co + co0 + co] = U[pa * 4 + pb];
    }
  }
}

// G g of a 3-vector -> 6 values
RK_DEV void g6(float g0, float g1, float g2, float (&u)[6]) {
  const float s = g0 + g2;
  u[0] = 0.25f * g0;
  u[1] = -(s + g1) * (1.f / 6.f);
  u[2] = -(s - g1) * (1.f / 6.f);
  u[3] = g0 * (1.f / 24.f) + g1 * (1.f / 12.f) + g2 * (1.f / 6.f);
  u[4] = g0 * (1.f / 24.f) - g1 * (1.f / 12.f) + g2 * (1.f / 6.f);
  u[5] = g2;
}

// U = G g G^T (36 values) of a 3x3 filter g[ky*3+kx]
RK_DEV void w4_transform(const float (&g)[9], float (&U)[36]) {
  float t[6][3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    float o[6];
    g6(g[kx], g[3 + kx], g[6 + kx], o);
#pragma unroll
    for (int a = 0; a < 6; ++a) t[a][kx] = o[a];
  }
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float o[6];
    g6(t[a][0], t[a][1], t[a][2], o);
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) U[a * 6 + bb] = o[bb];
  }
}

// one 32 co x 32 ci block of filters, LDS-staged so both layouts are written coalesced:
// u [36][Co][Ci] of w, ut [36][Ci][Co] of the flipped filters (either may be null).  PL: the X6 planes
// instead, bf16 u [36][3][Co][Ci] / ut [36][3][Ci][Co] (hi, mid, lo of every value; x6p.hip)
template <bool PL = false>
RK_DEV void w4_block(const float* __restrict__ w, void* __restrict__ u, void* __restrict__ ut, int Co, int Ci,
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
  auto put = [&](void* dst, long long q, long long rows, long long r, long long cols, long long c, float v) {
    if constexpr (PL) {
      bf16* d = (bf16*)dst + (q * 3 * rows + r) * cols + c;
      bf16 h, m, l;
      split3v(v, h, m, l);
      d[0] = h;
      d[rows * cols] = m;
      d[2 * rows * cols] = l;
    } else {
      ((float*)dst)[(q * rows + r) * cols + c] = v;
    }
  };
  if (u != nullptr)
    for (int i = threadIdx.x; i < 1024; i += 256) {
      const int ci = i & 31, co = i >> 5;
      if (co0 + co >= Co || ci0 + ci >= Ci) continue;
      float gg[9], U[36];
#pragma unroll
      for (int t = 0; t < 9; ++t) gg[t] = g[co][t][ci];
      w4_transform(gg, U);
#pragma unroll
      for (int q = 0; q < 36; ++q) put(u, q, Co, co0 + co, Ci, ci0 + ci, U[q]);
    }
  if (ut != nullptr)
    for (int i = threadIdx.x; i < 1024; i += 256) {
      const int co = i & 31, ci = i >> 5;
      if (co0 + co >= Co || ci0 + ci >= Ci) continue;
      float gg[9], U[36];
#pragma unroll
      for (int t = 0; t < 9; ++t) gg[t] = g[co][8 - t][ci];
      w4_transform(gg, U);
#pragma unroll
      for (int q = 0; q < 36; ++q) put(ut, q, Ci, ci0 + ci, Co, co0 + co, U[q]);
    }
}

