// ed_fe29.cuh -- the ed25519 base field GF(2^255 - 19) in the same reduced
// radix as the secp256k1 layer (secp_fe29.cuh): 9 limbs of 29 bits, one
// element per lane, magnitude tracking, column products summed inside
// v_mad_u64_u32's 64-bit addend.  Only the fold differs:
//
//   2^261 = 2^6 * 2^255 == 2^6 * 19 = 1216   (mod p)
//
// so each high column folds back with ONE mad by 1216 (secp needs two).
// Magnitude rules are the secp layer's (every limb <= m * F29_B,
// F29_B = 2^29 + 2^18): mul needs mag(a) * mag(b) <= 6, sqr mag(a) <= 2,
// add/sub results <= 7, e29_norm input <= 7; mul/sqr/norm outputs are
// magnitude 1.  Checked by the host build's GV_F29_CHECK traps in
// tests/test_ed_fe29_host.py.
#pragma once
#include "secp_fe29.cuh"

namespace gv {
namespace ed {

#define E29_R 1216u        // 2^261 mod p
#define E29_RH 9728u       // 2^293 mod p = 1216 * 2^32 = 9728 * 2^29: limb 1
// E29_HICARRY: high columns of the products split as lo + 2^32 hi (1), or
// the classic 29-bit extraction (0; A/B)
#ifndef E29_HICARRY
#define E29_HICARRY 1
#endif

template <bool SQR>
GV_DEV void e29_mulsqr(fe29& r, const fe29& a, const fe29& b) {
  u32 kr = E29_R;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(kr));                 // keep the fold constant a mad operand
#endif
  u32 d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = SQR ? (a.n[i] << 1) : 0u;
#define E29_X(i, j) (SQR ? ((i) == (j) ? a.n[i] : d[i]) : a.n[i])
#define E29_Y(i, j) (SQR ? a.n[j] : b.n[j])
  u32 t[9];
  u64 acc = 0;
#if E29_HICARRY
  // high columns split as lo + 2^32 hi (secp_fe29x.cuh's GV_F29X_HICARRY):
  // t_k keeps all 32 bits (the fold multiplies it by 1216: < 2^43) and 8 hi
  // re-enters column k+1 by one mad instead of a mask and a 64-bit shift
  {
    u32 hi = 0, k8 = 8u;
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(k8));                       // keep "mad by 8" a mad
#endif
#pragma unroll
    for (int k = 9; k <= 16; ++k) {
      u64 col = 0;
#pragma unroll
      for (int i = k - 8; i <= f29_col_hi<SQR>(k); ++i) col = f29_mad(E29_X(i, k - i), E29_Y(i, k - i), col);
      if (k > 9) col = f29_mad(hi, k8, col);  // carry of column k-1 (weight 2^32 there)
      t[k - 9] = (u32)col;
      hi = (u32)(col >> 32);
    }
    F29_TRAP(hi >= (1u << 29), "e29 mul t17");
    t[8] = hi << 3;                           // limb 17
  }
#else
#pragma unroll
  for (int k = 9; k <= 16; ++k) {             // high columns 9..16, carry chained
#pragma unroll
    for (int i = k - 8; i <= f29_col_hi<SQR>(k); ++i) acc = f29_mad(E29_X(i, k - i), E29_Y(i, k - i), acc);
    t[k - 9] = (u32)acc & F29_M;
    acc >>= 29;
  }
  F29_TRAP((acc >> 32) != 0, "e29 mul t17");
  t[8] = (u32)acc;                            // limb 17
#endif
  fe29 o;
  acc = 0;
#pragma unroll
  for (int j = 0; j <= 8; ++j) {              // low columns + 1216 * (column j + 9)
#pragma unroll
    for (int i = 0; i <= f29_col_hi<SQR>(j); ++i) acc = f29_mad(E29_X(i, j - i), E29_Y(i, j - i), acc);
    acc = f29_mad(t[j], kr, acc);
    o.n[j] = (u32)acc & F29_M;
    acc >>= 29;
  }
#undef E29_X
#undef E29_Y
  // the carry out of column 8 has weight 2^261: fold it once more
  const u32 clo = (u32)acc, chi = (u32)(acc >> 32);
  u64 x = f29_mad(clo, kr, (u64)o.n[0]);
  o.n[0] = (u32)x & F29_M;
  x = (x >> 29) + o.n[1];
  x = f29_mad(chi, E29_RH, x);
  o.n[1] = (u32)x & F29_M;
  o.n[2] = f29_add32(o.n[2], (u32)(x >> 29));
  r = o;
}

// r = a * b (magnitude 1).  mag(a) * mag(b) <= 6.  r may alias a or b.
GV_DEV void e29_mul(fe29& r, const fe29& a, const fe29& b) { e29_mulsqr<false>(r, a, b); }
// r = a^2 (magnitude 1).  mag(a) <= 2.
GV_DEV void e29_sqr(fe29& r, const fe29& a) { e29_mulsqr<true>(r, a, a); }
// r = a^(2^k)
GV_DEV void e29_sqr_n(fe29& r, const fe29& a, int k) {
  e29_sqr(r, a);
  for (int i = 1; i < k; ++i) e29_sqr(r, r);
}

#include "ed_fe29_consts.inc"

// r = K_mb - b  (mag(b) <= mb; result magnitude mb + 1)
template <int MB>
GV_DEV void e29_neg(fe29& r, const fe29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    F29_TRAP(b.n[i] > e29_kneg(MB, i), "e29 neg");
    r.n[i] = e29_kneg(MB, i) - b.n[i];
  }
}
// r = a + K_mb - b  (magnitude mag(a) + mb + 1)
template <int MB>
GV_DEV void e29_sub(fe29& r, const fe29& a, const fe29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    F29_TRAP(b.n[i] > e29_kneg(MB, i), "e29 sub");
    r.n[i] = f29_add32(a.n[i], e29_kneg(MB, i) - b.n[i]);
  }
}
// Carry pass: magnitude <= 7 -> 1 (the carry out of limb 8 re-enters as 1216 c)
GV_DEV void e29_norm(fe29& r, const fe29& a) {
  u32 c = 0;
  fe29 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const u32 x = f29_add32(a.n[i], c);
    o.n[i] = x & F29_M;
    c = x >> 29;
  }
  o.n[0] += c * E29_R;
  r = o;
}

// Canonical value in [0, p) as 8 little-endian words.  Input magnitude <= 7.
GV_DEV void e29_to_words(u32 w[8], const fe29& a0) {
  fe29 a;
  e29_norm(a, a0);
  e29_norm(a, a);
  // full carry pass with bits >= 255 (limb 8 bits >= 23) folded as 19 each, twice
#pragma unroll
  for (int rep = 0; rep < 2; ++rep) {
    const u32 h = a.n[8] >> 23;
    a.n[8] &= 0x7FFFFFu;
    u32 x = a.n[0] + h * 19u, c;
    a.n[0] = x & F29_M; c = x >> 29;
#pragma unroll
    for (int i = 1; i < 9; ++i) { x = a.n[i] + c; a.n[i] = x & F29_M; c = x >> 29; }
  }
  // value < 2^255 with every limb < 2^29: pack
  u32 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int bb = 32 * k, i = bb / 29, s = bb % 29;
    u64 x = ((u64)a.n[i] >> s);
    if (i + 1 < 9) x |= (u64)a.n[i + 1] << (29 - s);
    if (i + 2 < 9 && (58 - s) < 32) x |= (u64)a.n[i + 2] << (58 - s);
    v[k] = (u32)x;
  }
  // subtract p once if v >= p:  v + 19 reaches bit 255 iff v >= p
  u32 t[8];
  u64 c = (u64)v[0] + 19u;
  t[0] = (u32)c; c >>= 32;
#pragma unroll
  for (int i = 1; i < 8; ++i) { c += v[i]; t[i] = (u32)c; c >>= 32; }
  const bool ge = (t[7] >> 31) != 0;
  t[7] &= 0x7FFFFFFFu;
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = ge ? t[i] : v[i];
}

// FeFromBytes: 8 little-endian words, bit 255 dropped, NOT reduced mod p
// (y >= p is accepted and simply computed with).  Magnitude 1.
GV_DEV void e29_from_words(fe29& r, const u32 w0[8]) {
  u32 w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = w0[i];
  w[7] &= 0x7FFFFFFFu;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int bb = 29 * i, k = bb / 32, s = bb % 32;
    u64 x = (u64)w[k] >> s;
    if (k + 1 < 8) x |= (u64)w[k + 1] << (32 - s);
    r.n[i] = (u32)x & F29_M;
  }
}

GV_DEV bool e29_is_zero(const fe29& a) {
  u32 w[8];
  e29_to_words(w, a);
  u32 z = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) z |= w[i];
  return z == 0;
}
// FeIsNegative: parity of the canonical value
GV_DEV u32 e29_is_negative(const fe29& a) {
  u32 w[8];
  e29_to_words(w, a);
  return w[0] & 1u;
}

GV_DEV void e29_set(fe29& r, u32 x) { f29_set_u32(r, x); }

// z^(2^250 - 1) and z^11 -- the shared prefix of the two exponentiations
// below (the standard 2^255 - 19 addition chain: 11 multiplications, 254
// squarings in total for either result).
GV_DEV void e29_pow_prefix(fe29& z250, fe29& z11, const fe29& z) {
  fe29 t0, t1, t2;
  e29_sqr(t0, z);                  // z^2
  e29_sqr_n(t1, t0, 2);            // z^8
  e29_mul(t1, z, t1);              // z^9
  e29_mul(z11, t0, t1);            // z^11
  e29_sqr(t0, z11);                // z^22
  e29_mul(t0, t1, t0);             // z^31 = z^(2^5 - 1)
  e29_sqr_n(t1, t0, 5);
  e29_mul(t0, t1, t0);             // 2^10 - 1
  e29_sqr_n(t1, t0, 10);
  e29_mul(t1, t1, t0);             // 2^20 - 1
  e29_sqr_n(t2, t1, 20);
  e29_mul(t1, t2, t1);             // 2^40 - 1
  e29_sqr_n(t1, t1, 10);
  e29_mul(t0, t1, t0);             // 2^50 - 1
  e29_sqr_n(t1, t0, 50);
  e29_mul(t1, t1, t0);             // 2^100 - 1
  e29_sqr_n(t2, t1, 100);
  e29_mul(t1, t2, t1);             // 2^200 - 1
  e29_sqr_n(t1, t1, 50);
  e29_mul(z250, t1, t0);           // 2^250 - 1
}
// r = z^(p - 2) = z^-1 (0 -> 0)
GV_DEV void e29_inv(fe29& r, const fe29& z) {
  fe29 z250, z11;
  e29_pow_prefix(z250, z11, z);
  e29_sqr_n(z250, z250, 5);        // 2^255 - 32
  e29_mul(r, z250, z11);           // 2^255 - 21
}
// r = z^((p - 5) / 8) = z^(2^252 - 3)
GV_DEV void e29_pow22523(fe29& r, const fe29& z) {
  fe29 z250, z11;
  e29_pow_prefix(z250, z11, z);
  e29_sqr_n(z250, z250, 2);        // 2^252 - 4
  e29_mul(r, z250, z);             // 2^252 - 3
}

}  // namespace ed
}  // namespace gv
