// secp_sc29.cuh -- arithmetic modulo the group order n in radix 2^29 (9 limbs),
// Montgomery form with R = 2^261, one scalar per lane.
//
// Restates the scalar part of go1.14 crypto/ecdsa.verifyGeneric
// (w = s^-1 mod n, u1 = e*w mod n, u2 = r*w mod n) on the same column engine
// as the base field (secp_fe29.cuh): product scanning with the Montgomery
// reduction interleaved column by column -- column k sums a_i*b_(k-i) and
// m_i*n_(k-i) in one v_mad_u64_u32 chain (at most 18 terms < 2^58, so the
// 64-bit addend never overflows), m_k = (column * n') mod 2^29 clears the
// column's low 29 bits.  ~2x fewer instructions than the 8 x 32 CIOS product
// of secp_scalar.cuh as compiled by hipcc.
//
// Representation: limbs < 2^29, value < 2^258.  montmul of such inputs
// returns a value < n + 2^255 < 2n (so < 2^258 again); sc29_canon() reduces
// to [0, n).
#pragma once
#include "secp_fe29.cuh"

namespace gv {

struct sc29 { u32 n[9]; };

// n in radix 2^29, n' = -n^-1 mod 2^29, R^2 mod n (R = 2^261)
#define SC29_N0 0x10364141u
#define SC29_N1 0x1E92F466u
#define SC29_N2 0x12280EEFu
#define SC29_N3 0x1DB9CD5Eu
#define SC29_N4 0x1FFFEBAAu
#define SC29_NF 0x1FFFFFFFu   // limbs 5..7
#define SC29_N8 0x00FFFFFFu
#define SC29_NP 0x1588B13Fu

GV_DEV constexpr u32 sc29_r2(int i) {
  constexpr u32 t[9] = {0x09F6AB4Bu, 0x1F300D1Eu, 0x1C0BD5D8u, 0x0C8ADA8Cu, 0x11CEFA2Bu,
                        0x08B79A0Fu, 0x1E697F5Eu, 0x00E34DE2u, 0x009C7356u};
  return t[i];
}

// r = a * b / 2^261 mod n (partially reduced, < 2n).  SQR: b == a, cross
// terms doubled.  r may alias a or b.
template <bool SQR>
GV_DEV void sc29_montmulsqr(sc29& r, const sc29& a, const sc29& b) {
  u32 nk[7] = {SC29_N0, SC29_N1, SC29_N2, SC29_N3, SC29_N4, SC29_NF, SC29_N8};
  u32 np = SC29_NP;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(nk[0]), "+v"(nk[1]), "+v"(nk[2]), "+v"(nk[3]), "+v"(nk[4]), "+v"(nk[5]), "+v"(nk[6]));
#endif
#define SC29_NL(j) ((j) <= 4 ? nk[j] : (j) <= 7 ? nk[5] : nk[6])
  u32 d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = SQR ? (a.n[i] << 1) : 0u;
#define SC29_T(i, j) f29_mad(SQR ? ((i) == (j) ? a.n[i] : d[i]) : a.n[i], SQR ? a.n[j] : b.n[j], acc)
  u32 m[9];
  sc29 o;
  u64 acc = 0;
#pragma unroll
  for (int k = 0; k <= 16; ++k) {
    const int lo = k < 9 ? 0 : k - 8;
#pragma unroll
    for (int i = lo; i <= (SQR ? (k >> 1) : (k < 9 ? k : 8)); ++i) acc = SC29_T(i, k - i);
#pragma unroll
    for (int i = lo; i <= (k < 9 ? k - 1 : 8); ++i) acc = f29_mad(m[i], SC29_NL(k - i), acc);
    if (k < 9) {
      m[k] = ((u32)acc * np) & F29_M;
      acc = f29_mad(m[k], SC29_NL(0), acc);      // low 29 bits -> 0
    } else {
      o.n[k - 9] = (u32)acc & F29_M;
    }
    acc >>= 29;
  }
  o.n[8] = (u32)acc;
#undef SC29_T
#undef SC29_NL
  r = o;
}
GV_DEV void sc29_mul(sc29& r, const sc29& a, const sc29& b) { sc29_montmulsqr<false>(r, a, b); }
GV_DEV void sc29_sqr(sc29& r, const sc29& a) { sc29_montmulsqr<true>(r, a, a); }
GV_DEV void sc29_sqr_n(sc29& r, int k) {
#pragma unroll 1
  for (int i = 0; i < k; ++i) sc29_sqr(r, r);
}

// 8 x 32 words (value < 2^256) <-> limbs
GV_DEV void sc29_from_words(sc29& r, const u32 w[8]) {
  fe29 t;
  f29_from_words(t, w);
#pragma unroll
  for (int i = 0; i < 9; ++i) r.n[i] = t.n[i];
}
// canonical [0, n) of a value < 2n
GV_DEV void sc29_canon(sc29& r, const sc29& a) {
  const u32 nl[9] = {SC29_N0, SC29_N1, SC29_N2, SC29_N3, SC29_N4, SC29_NF, SC29_NF, SC29_NF, SC29_N8};
  u32 t[9];
  int br = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int x = (int)a.n[i] - (int)nl[i] - br;   // limbs < 2^29: no int overflow
    br = x < 0;
    t[i] = (u32)x & F29_M;
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) r.n[i] = br ? a.n[i] : t[i];
}
// canonical value as 8 x 32 words
GV_DEV void sc29_to_words(u32 w[8], const sc29& a) {
  sc29 c;
  sc29_canon(c, a);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int b = 32 * k, i = b / 29, s = b % 29;
    u64 x = ((u64)c.n[i] >> s);
    if (i + 1 < 9) x |= (u64)c.n[i + 1] << (29 - s);
    if (i + 2 < 9 && (58 - s) < 32) x |= (u64)c.n[i + 2] << (58 - s);
    w[k] = (u32)x;
  }
}

// x -> x * R mod n (Montgomery form, < 2n)
GV_DEV void sc29_to_mont(sc29& r, const sc29& a) {
  sc29 r2;
#pragma unroll
  for (int i = 0; i < 9; ++i) r2.n[i] = sc29_r2(i);
  sc29_mul(r, a, r2);
}

// r = x^(n-2) (Montgomery form in and out): x^-1 for x != 0 mod n
GV_DEV void sc29_inv(sc29& r, const sc29& x) {
  sc29 t[4], x2, acc;
  sc29_sqr(x2, x);
  t[0] = x;
#pragma unroll
  for (int k = 1; k < 4; ++k) sc29_mul(t[k], t[k - 1], x2);
#include "secp_sc29_inv.inc"
  r = acc;
}

}  // namespace gv
