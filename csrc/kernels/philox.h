// Counter-based Philox4x32-10 (Salmon et al., SC'11): 10 rounds of two 32x32->64 multiplies per
// 128-bit counter.  Shared by the PG-GAN generator draws (pggan.hip) and the tagger's dropout masks
// (tagger.hip); callers build the counter from (element quad, call-site stream id, device step
// counter), so a replayed hipGraph that bumps the step counter draws fresh numbers every replay.
#pragma once
#include "common.h"

struct U4 { uint32_t v[4]; };

RK_DEV U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    const uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += W0; k1 += W1;
  }
  U4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}

// [0, 1) with 24 random mantissa bits; (0, 1] variant for the Box-Muller log
RK_DEV float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
RK_DEV float u01_open(uint32_t x) { return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f); }
