// ed_scalar.cuh -- scalars mod the ed25519 group order L = 2^252 + c:
//   sc_reduce512  ScReduce (go1.14 edwards25519): a 64-byte little-endian
//                 integer (the SHA-512 digest) reduced mod L, by Barrett
//                 reduction (HAC 14.42, base 2^32, k = 8, mu = floor(2^512/L))
//   sc_minimal    ScMinimal: s < L (crypto/ed25519 Verify's malleability check)
// Host-compilable.  Words are little-endian u32.
#pragma once
#include <stdint.h>
#include "ed_sha512.cuh"     // GV_DEV / GV_EDC

namespace gv {
namespace ed {

#ifndef GV_ED_CONSTS_INCLUDED
#define GV_ED_CONSTS_INCLUDED
typedef uint32_t u32;
#include "ed_consts.inc"
#endif

// r = x mod L, x = 16 words (< 2^512); r < L in 8 words.
GV_DEV void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  // q1 = floor(x / b^7) = x[7..15];  q3 = floor(q1 * mu / b^9)
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const uint64_t t = (uint64_t)x[7 + i] * kEdMu[j] + q2[i + j] + c;
      q2[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    q2[i + 9] = (uint32_t)c;
  }
  // r2 = q3 * L mod b^9
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i + j >= 9) break;
      const uint64_t t = (uint64_t)q2[9 + i] * kEdL[j] + r2[i + j] + c;
      r2[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    if (i + 8 < 9) r2[i + 8] += (uint32_t)c;
  }
  // r = x mod b^9 - r2 (mod b^9): 0 <= r < 3L
  uint32_t t[9];
  uint64_t bw = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t d = (uint64_t)x[i] - r2[i] - bw;
    t[i] = (uint32_t)d;
    bw = (d >> 32) & 1u;
  }
  // at most two subtractions of L
#pragma unroll
  for (int rep = 0; rep < 2; ++rep) {
    uint32_t u[9];
    uint64_t b2 = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const uint64_t d = (uint64_t)t[i] - (i < 8 ? kEdL[i] : 0u) - b2;
      u[i] = (uint32_t)d;
      b2 = (d >> 32) & 1u;
    }
    const bool ge = b2 == 0;             // t >= L
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = ge ? u[i] : t[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = t[i];
}

// ScMinimal: s < L
GV_DEV bool sc_minimal(const uint32_t s[8]) {
  uint64_t b = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)s[i] - kEdL[i] - b;
    b = (d >> 32) & 1u;
  }
  return b != 0;                         // s - L borrows
}

}  // namespace ed
}  // namespace gv
