// secp_modinv.cuh -- s^-1 mod n by Bernstein-Yang divsteps (safegcd), for the
// latency kernel's scalar chain (gv_lat.hip).
//
// Why: the Fermat chain s^(n-2) is 253 squarings + 74 products, every one
// dependent on the previous -- on a lone wave that is the longest serial
// chain of the small-batch kernel (tools/lat_trace.py: 202 us of scalar work
// against 148 us for the pubkey square root + tables).  Divsteps decide each
// step from the low bit of g and the sign of delta only, so 30 steps at a time
// run on the low 32 bits of f and g, exactly, and the accumulated 2x2 matrix
// (entries <= 2^30) is applied once to the full-width values: ~25 rounds of
// (30 cheap steps + 4 x 9 signed mads) instead of 327 dependent 9-limb
// products.  The inputs are public signature data, so the loop may stop as
// soon as every lane's g is zero.
//
// divstep(delta, f, g) (Bernstein & Yang, "Fast constant-time gcd computation
// and modular inversion", 2019):
//   delta > 0 and g odd:  (1 - delta, g, (g - f) / 2)
//   g odd:                (1 + delta, f, (g + f) / 2)
//   else:                 (1 + delta, f, g / 2)
// from (1, n, s): g reaches 0 within 741 steps for 256-bit inputs and then
// f = +-1.  With d, e tracked so that f == d*s and g == e*s (mod n), the
// inverse is +-d.
//
// Numbers are "signed-30": 9 limbs, value = sum v[i] * 2^(30 i), limbs 0..7 in
// [0, 2^30), limb 8 a signed int32.
#pragma once
#include <stdint.h>
#ifndef GV_DEV
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GV_DEV __device__ __forceinline__
#else
#define GV_DEV static inline
#endif
#endif

namespace gv {

struct s30 { int32_t v[9]; };

#define S30_M 0x3FFFFFFF
// n (secp256k1 group order) in signed-30 limbs, and n^-1 mod 2^30
#define S30_N_INV 0x2A774EC1u
GV_DEV int32_t s30_n(int i) {
  const int32_t t[9] = {271991105, 1061780019, 881460155, 733428139, 1073741498,
                        1073741823, 1073741823, 1073741823, 65535};
  return t[i];
}

GV_DEV void s30_from_words(s30& r, const uint32_t w[8]) {     // 0 <= value < 2^256
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = 30 * i, k = b >> 5, s = b & 31;
    uint64_t x = (uint64_t)w[k] >> s;
    if (k + 1 < 8) x |= (uint64_t)w[k + 1] << (32 - s);
    r.v[i] = (int32_t)(x & S30_M);
  }
}

GV_DEV void s30_to_words(uint32_t w[8], const s30& a) {       // 0 <= value < 2^256
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int b = 32 * k, i = b / 30, s = b % 30;
    uint64_t x = (uint64_t)(uint32_t)a.v[i] >> s;
    if (i + 1 < 9) x |= (uint64_t)(uint32_t)a.v[i + 1] << (30 - s);
    if (i + 2 < 9 && 60 - s < 64) x |= (uint64_t)(uint32_t)a.v[i + 2] << (60 - s);
    w[k] = (uint32_t)x;
  }
}

// 30 divsteps on the low 32 bits of f and g.  Returns delta; t = (u, v, q, r)
// with 2^30 f' = u f + v g and 2^30 g' = q f + r g (|u| + |v| <= 2^30).
GV_DEV int32_t s30_divsteps(int32_t delta, uint32_t f, uint32_t g, int32_t t[4]) {
  int32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll 6
  for (int i = 0; i < 30; ++i) {
    const uint32_t godd = g & 1u;
    const bool sw = (delta > 0) & (godd != 0u);
    const uint32_t f2 = sw ? g : f;
    uint32_t g2 = sw ? 0u - f : g;
    const int32_t u2 = sw ? q : u, v2 = sw ? r : v;
    int32_t q2 = sw ? -u : q, r2 = sw ? -v : r;
    delta = sw ? -delta : delta;
    const uint32_t m = 0u - godd;               // all ones when g is odd
    g2 += f2 & m;
    q2 += u2 & (int32_t)m;
    r2 += v2 & (int32_t)m;
    delta += 1;
    f = f2; g = g2 >> 1;
    u = u2 << 1; v = v2 << 1; q = q2; r = r2;
  }
  t[0] = u; t[1] = v; t[2] = q; t[3] = r;
  return delta;
}

// (f, g) <- (u f + v g, q f + r g) / 2^30  (exact division)
GV_DEV void s30_update_fg(s30& f, s30& g, const int32_t t[4]) {
  int64_t cf = (int64_t)t[0] * f.v[0] + (int64_t)t[1] * g.v[0];
  int64_t cg = (int64_t)t[2] * f.v[0] + (int64_t)t[3] * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cf += (int64_t)t[0] * f.v[i] + (int64_t)t[1] * g.v[i];
    cg += (int64_t)t[2] * f.v[i] + (int64_t)t[3] * g.v[i];
    f.v[i - 1] = (int32_t)((uint32_t)cf & S30_M);
    g.v[i - 1] = (int32_t)((uint32_t)cg & S30_M);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// a in (-n, 2n) -> [0, n)
GV_DEV void s30_normalize(s30& a) {
  const int32_t neg = a.v[8] >> 31;             // all ones when a < 0
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {                 // a += n if a < 0
    c += (int64_t)a.v[i] + (s30_n(i) & neg);
    a.v[i] = i < 8 ? (int32_t)((uint32_t)c & S30_M) : (int32_t)c;
    c >>= 30;
  }
  s30 t;
  c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {                 // t = a - n
    c += (int64_t)a.v[i] - s30_n(i);
    t.v[i] = i < 8 ? (int32_t)((uint32_t)c & S30_M) : (int32_t)c;
    c >>= 30;
  }
  const bool ge = t.v[8] >= 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) a.v[i] = ge ? t.v[i] : a.v[i];
}

// (d, e) <- (u d + v e, q d + r e) / 2^30 mod n, d, e in [0, n) -> [0, n)
GV_DEV void s30_update_de(s30& d, s30& e, const int32_t t[4]) {
  const int64_t d0 = (int64_t)t[0] * d.v[0] + (int64_t)t[1] * e.v[0];
  const int64_t e0 = (int64_t)t[2] * d.v[0] + (int64_t)t[3] * e.v[0];
  const int32_t md = (int32_t)(((0u - (uint32_t)d0) * S30_N_INV) & S30_M);   // clears the low 30 bits
  const int32_t me = (int32_t)(((0u - (uint32_t)e0) * S30_N_INV) & S30_M);
  int64_t cd = (d0 + (int64_t)md * s30_n(0)) >> 30;
  int64_t ce = (e0 + (int64_t)me * s30_n(0)) >> 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cd += (int64_t)t[0] * d.v[i] + (int64_t)t[1] * e.v[i] + (int64_t)md * s30_n(i);
    ce += (int64_t)t[2] * d.v[i] + (int64_t)t[3] * e.v[i] + (int64_t)me * s30_n(i);
    d.v[i - 1] = (int32_t)((uint32_t)cd & S30_M);
    e.v[i - 1] = (int32_t)((uint32_t)ce & S30_M);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
  s30_normalize(d);
  s30_normalize(e);
}

// w = x^-1 mod n for 0 < x < n (words, little-endian); x == 0 gives 0.
// `all_done` is the caller's wave-wide "every lane finished" test
// (device: a ballot; host: the lane's own flag).
template <class AllDone>
GV_DEV void s30_modinv(uint32_t w[8], const uint32_t x[8], AllDone all_done) {
  s30 f, g, d, e;
#pragma unroll
  for (int i = 0; i < 9; ++i) { f.v[i] = s30_n(i); d.v[i] = 0; e.v[i] = 0; }
  e.v[0] = 1;
  s30_from_words(g, x);
  int32_t delta = 1;
#pragma unroll 1
  for (int round = 0; round < 25; ++round) {    // 25 * 30 = 750 >= 741 steps
    int32_t gz = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) gz |= g.v[i];
    if (all_done(gz == 0)) break;
    int32_t t[4];
    delta = s30_divsteps(delta, (uint32_t)f.v[0] | ((uint32_t)f.v[1] << 30),
                         (uint32_t)g.v[0] | ((uint32_t)g.v[1] << 30), t);
    s30_update_fg(f, g, t);
    s30_update_de(d, e, t);
  }
  // f = +-1: the inverse is f * d
  if (f.v[8] < 0) {                             // d <- n - d (d == 0 only for x == 0)
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      c += (int64_t)s30_n(i) - d.v[i];
      d.v[i] = i < 8 ? (int32_t)((uint32_t)c & S30_M) : (int32_t)c;
      c >>= 30;
    }
    s30_normalize(d);
  }
  s30_to_words(w, d);
}

// ---------------------------------------------------------------------------
// Variable-time divsteps (the signature data is public): the "eta = -delta"
// form of Bernstein-Yang with the batching of libsecp256k1's var-time
// modinv32 (Wuille's safegcd implementation notes, "divsteps_var"): a run of
// zero low bits of g is ONE shift, and up to 8 low bits of g are cancelled at
// once by g += w f with w = -g / f (mod 2^k), k <= eta + 1 so that no swap
// falls inside the batch.  The same transition matrix as 30 single divsteps
// of that form (|u| + |v| <= 2^30), in ~1/4 of the instructions on a lone
// lane (the latency kernels' scalar chain).

// f^-1 mod 2^8 for odd f (Newton from f*f == 1 mod 8)
GV_DEV uint32_t s30_inv8(uint32_t f) {
  uint32_t x = f;
  x *= 2u - f * x;                              // mod 2^6
  x *= 2u - f * x;                              // mod 2^12
  return x;
}

GV_DEV int32_t s30_divsteps_var(int32_t eta, uint32_t f, uint32_t g, int32_t t[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t nfi = 0u - s30_inv8(f);              // -f^-1 mod 2^8
  int i = 30;
#pragma unroll 1
  for (;;) {
    const int zeros = __builtin_ctz(g | (0xFFFFFFFFu << i));   // sentinel: at most i
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {                              // (f, g) <- (g, -f)
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
      nfi = 0u - s30_inv8(f);
    }
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 255u;
    const uint32_t w = (g * nfi) & m;           // g + w f == 0 (mod 2^min(limit, 8))
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int32_t)u; t[1] = (int32_t)v; t[2] = (int32_t)q; t[3] = (int32_t)r;
  return eta;
}

// w = x^-1 mod n (0 < x < n; x == 0 gives 0), one lane, variable time.
// `done` counts rounds for the host tests.
template <class Count>
GV_DEV void s30_modinv_var(uint32_t w[8], const uint32_t x[8], Count count) {
  s30 f, g, d, e;
#pragma unroll
  for (int i = 0; i < 9; ++i) { f.v[i] = s30_n(i); d.v[i] = 0; e.v[i] = 0; }
  e.v[0] = 1;
  s30_from_words(g, x);
  int32_t eta = -1;
#pragma unroll 1
  for (int round = 0; round < 25; ++round) {    // eta form from -1: g == 0 within 590 divsteps
    int32_t gz = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) gz |= g.v[i];
    if (gz == 0) break;
    count();
    int32_t t[4];
    eta = s30_divsteps_var(eta, (uint32_t)f.v[0] | ((uint32_t)f.v[1] << 30),
                           (uint32_t)g.v[0] | ((uint32_t)g.v[1] << 30), t);
    s30_update_fg(f, g, t);
    s30_update_de(d, e, t);
  }
  if (f.v[8] < 0) {                             // f = -1: the inverse is -d
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      c += (int64_t)s30_n(i) - d.v[i];
      d.v[i] = i < 8 ? (int32_t)((uint32_t)c & S30_M) : (int32_t)c;
      c >>= 30;
    }
    s30_normalize(d);
  }
  s30_to_words(w, d);
}

}  // namespace gv
