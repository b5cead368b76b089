// ed_group.cuh -- edwards25519 group arithmetic and the ed25519 verification
// core on the 9 x 29 field layer (ed_fe29.cuh).  Host-compilable: the same
// source runs in tests/test_ed_host.py (g++, overflow traps) and in the
// gfx950 kernels (ed_verify.hip).
//
// Restates (go1.14 crypto/ed25519 + internal/edwards25519, the code
// tendermint v0.33.4 PubKeyEd25519.VerifyBytes calls):
//   ge_frombytes   ExtendedGroupElement.FromBytes (y = bytes mod 2^255, no
//                  canonicality check; x from the (p-5)/8 power; sign fix-up)
//   ge_tobytes     ProjectiveGroupElement.ToBytes (canonical y | parity(x))
//   ed_verify_core Verify after the length / sig[63] & 224 checks:
//                  R' = [h](-A) + [s]B compared with sig[:32] as bytes.
// [h](-A) runs MSB-first over signed radix-16 digits of h with a per-lane
// table j(-A), j = 0..8 (cached form, in global scratch); [s]B is a fixed-base
// comb over signed radix-256 digits of s against a resident table of
// j * 256^w * B (w < 32, j <= 128, affine precomputed form), added after the
// last doubling.  The twisted-Edwards (a = -1) formulas used are complete on
// this curve, so small-order and mixed-order keys need no special cases.
#pragma once
#include "ed_fe29.cuh"
#include "ed_scalar.cuh"

namespace gv {
namespace ed {

struct ge_ext { fe29 X, Y, Z, T; };               // x = X/Z, y = Y/Z, xy = T/Z
struct ge_cached { fe29 ypx, ymx, z2, t2d; };     // (Y+X, Y-X, 2Z, 2dT), magnitude 1
struct ge_pre { fe29 ypx, ymx, xy2d; };           // (y+x, y-x, 2dxy), affine, magnitude 1

#define ED_CACHED_WORDS 36                        // 4 fe x 9 limbs
#define ED_PRE_WORDS 27                           // 3 fe x 9 limbs
#define ED_ATAB_ENTRIES 9                         // j(-A), j = 0..8 (entry 0 = the identity)
#define ED_ATAB_WORDS (ED_ATAB_ENTRIES * ED_CACHED_WORDS)
#define ED_BTAB_WINDOWS 32
#define ED_BTAB_ENTRIES 129                       // j = 0..128
#define ED_BTAB_WORDS (ED_BTAB_WINDOWS * ED_BTAB_ENTRIES * ED_PRE_WORDS)
// The radix-2^16 comb table of B (k_ed_keyed): j * 65536^w * B, w < 16,
// j = 0..2^15 -- 16 additions for [s]B instead of 32, 56.6 MB per device.
#define ED_BTAB16_WINDOWS 16
#define ED_BTAB16_ENTRIES 32769
#define ED_BTAB16_WORDS ((size_t)ED_BTAB16_WINDOWS * ED_BTAB16_ENTRIES * ED_PRE_WORDS)

GV_DEV void fe_const(fe29& r, const u32* c) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.n[i] = c[i];
}
GV_DEV void fe_select(fe29& r, bool c, const fe29& a, const fe29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.n[i] = c ? a.n[i] : b.n[i];
}

// r = norm(a + K_mb - b): subtraction fused into the carry pass, magnitude 1
template <int MB>
GV_DEV void e29_sub_norm(fe29& r, const fe29& a, const fe29& b) {
  u32 c = 0;
  fe29 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    F29_TRAP(b.n[i] > e29_kneg(MB, i), "e29 sub_norm");
    const u32 x = f29_add32(f29_add32(a.n[i], e29_kneg(MB, i) - b.n[i]), c);
    o.n[i] = x & F29_M;
    c = x >> 29;
  }
  o.n[0] += c * E29_R;
  r = o;
}
// r = norm(a + b)
GV_DEV void e29_add_norm(fe29& r, const fe29& a, const fe29& b) {
  fe29 t;
  f29_add(t, a, b);
  e29_norm(r, t);
}

GV_DEV void ge_identity(ge_ext& r) {
  f29_set_zero(r.X);
  e29_set(r.Y, 1);
  e29_set(r.Z, 1);
  f29_set_zero(r.T);
}

// r = 2p (ref10 ge_p2_dbl + p1p1 -> p3).  p: X, Y magnitude 1, Z <= 2.
// Every output magnitude 1.  T of p is not read; T of r is computed only
// when T_OUT (the next operation is an addition).
template <bool T_OUT>
GV_DEV void ge_dbl_t(ge_ext& r, const ge_ext& p) {
  fe29 xx, yy, b, a, aa, y1, z1, x1, t1;
  e29_sqr(xx, p.X);
  e29_sqr(yy, p.Y);
  e29_sqr(b, p.Z);
  f29_add(b, b, b);                   // 2 Z^2            (mag 2)
  f29_add(a, p.X, p.Y);               //                  (mag 2)
  e29_sqr(aa, a);                     // (X + Y)^2
  f29_add(y1, yy, xx);                // Y' = YY + XX     (mag 2)
  e29_sub<1>(z1, yy, xx);             // Z' = YY - XX     (mag 3)
  e29_sub_norm<2>(x1, aa, y1);        // X' = AA - Y'     (mag 1)
  e29_sub_norm<3>(t1, b, z1);         // T' = 2Z^2 - Z'   (mag 1)
  e29_mul(r.X, x1, t1);
  e29_mul(r.Y, y1, z1);
  e29_mul(r.Z, z1, t1);
  if (T_OUT) e29_mul(r.T, x1, y1);
}
GV_DEV void ge_dbl(ge_ext& r, const ge_ext& p) { ge_dbl_t<true>(r, p); }

// r = p + (neg ? -q : q) with q in cached form (ref10 ge_add / ge_sub).
// p magnitude 1; outputs magnitude 1.  r may alias p.
GV_DEV void ge_add_cached(ge_ext& r, const ge_ext& p, const ge_cached& q, bool neg) {
  fe29 ypx1, ymx1, qa, qb, a, b, c, d, x1, y1, dpc, dmc, z1, t1;
  f29_add(ypx1, p.Y, p.X);            // mag 2
  e29_sub<1>(ymx1, p.Y, p.X);         // mag 3
  fe_select(qa, neg, q.ymx, q.ypx);   // -q = (Y-X, Y+X, 2Z, -2dT)
  fe_select(qb, neg, q.ypx, q.ymx);
  e29_mul(a, ypx1, qa);
  e29_mul(b, ymx1, qb);
  e29_mul(c, q.t2d, p.T);
  e29_mul(d, p.Z, q.z2);
  e29_sub_norm<1>(x1, a, b);          // X' = A - B       (mag 1)
  f29_add(y1, a, b);                  // Y' = A + B       (mag 2)
  f29_add(dpc, d, c);                 //                  (mag 2)
  e29_sub_norm<1>(dmc, d, c);         //                  (mag 1)
  fe_select(z1, neg, dmc, dpc);       // Z' = D + C  (neg: D - C)
  fe_select(t1, neg, dpc, dmc);       // T' = D - C  (neg: D + C)
  e29_mul(r.X, x1, t1);
  e29_mul(r.Y, y1, z1);
  e29_mul(r.Z, z1, t1);
  e29_mul(r.T, x1, y1);
}

// r = p + (neg ? -q : q) with q affine precomputed (ref10 ge_madd / ge_msub).
GV_DEV void ge_add_pre(ge_ext& r, const ge_ext& p, const ge_pre& q, bool neg) {
  fe29 ypx1, ymx1, qa, qb, a, b, c, d, x1, y1, dpc, dmc, z1, t1;
  f29_add(ypx1, p.Y, p.X);
  e29_sub<1>(ymx1, p.Y, p.X);
  fe_select(qa, neg, q.ymx, q.ypx);
  fe_select(qb, neg, q.ypx, q.ymx);
  e29_mul(a, ypx1, qa);
  e29_mul(b, ymx1, qb);
  e29_mul(c, q.xy2d, p.T);
  f29_add(d, p.Z, p.Z);               // 2 Z1             (mag 2)
  e29_sub_norm<1>(x1, a, b);
  f29_add(y1, a, b);                  //                  (mag 2)
  f29_add(dpc, d, c);                 //                  (mag 3)
  e29_sub_norm<1>(dmc, d, c);         //                  (mag 1)
  fe_select(z1, neg, dmc, dpc);
  fe_select(t1, neg, dpc, dmc);
  e29_mul(r.X, x1, t1);               // 1 x 3
  e29_mul(r.Y, y1, z1);               // 2 x 3
  e29_mul(r.Z, z1, t1);               // 3 x 1
  e29_mul(r.T, x1, y1);
}

GV_DEV void ge_to_cached(ge_cached& r, const ge_ext& p) {
  fe29 d2;
  fe_const(d2, kEd2D);
  e29_add_norm(r.ypx, p.Y, p.X);
  e29_sub_norm<1>(r.ymx, p.Y, p.X);
  e29_add_norm(r.z2, p.Z, p.Z);
  e29_mul(r.t2d, p.T, d2);
}

// affine precomputed form (one inversion)
GV_DEV void ge_to_pre(ge_pre& r, const ge_ext& p) {
  fe29 zi, x, y, xy, d2;
  e29_inv(zi, p.Z);
  e29_mul(x, p.X, zi);
  e29_mul(y, p.Y, zi);
  fe_const(d2, kEd2D);
  e29_add_norm(r.ypx, y, x);
  e29_sub_norm<1>(r.ymx, y, x);
  e29_mul(xy, x, y);
  e29_mul(r.xy2d, xy, d2);
}

// ExtendedGroupElement.FromBytes on 8 little-endian words; false if the
// encoding is not a curve point.  r is always written (garbage on failure).
GV_DEV bool ge_frombytes(ge_ext& r, const u32 w[8]) {
  fe29 one, u, v, v3, vxx, chk, t, dd, sm1;
  e29_from_words(r.Y, w);
  e29_set(one, 1);
  e29_set(r.Z, 1);
  fe_const(dd, kEdD);
  e29_sqr(u, r.Y);                    // y^2
  e29_mul(v, u, dd);                  // d y^2
  e29_sub_norm<1>(u, u, one);         // u = y^2 - 1
  e29_add_norm(v, v, one);            // v = d y^2 + 1
  e29_sqr(v3, v);
  e29_mul(v3, v3, v);                 // v^3
  e29_sqr(t, v3);
  e29_mul(t, t, v);                   // v^7
  e29_mul(t, t, u);                   // u v^7
  e29_pow22523(t, t);                 // (u v^7)^((p-5)/8)
  e29_mul(t, t, v3);
  e29_mul(r.X, t, u);                 // x = u v^3 (u v^7)^((p-5)/8)
  e29_sqr(vxx, r.X);
  e29_mul(vxx, vxx, v);               // v x^2
  e29_sub<1>(chk, vxx, u);
  const bool root = e29_is_zero(chk);
  f29_add(chk, vxx, u);
  const bool neg_root = e29_is_zero(chk);
  fe_const(sm1, kEdSqrtM1);
  e29_mul(t, r.X, sm1);
  fe_select(r.X, root, r.X, t);       // v x^2 == -u: x *= sqrt(-1)
  const u32 want = w[7] >> 31;
  e29_neg<1>(t, r.X);
  fe_select(r.X, e29_is_negative(r.X) != want, t, r.X);
  e29_norm(r.X, r.X);
  e29_mul(r.T, r.X, r.Y);
  return root || neg_root;
}

// ToBytes: canonical y with bit 255 = parity of canonical x (one inversion)
GV_DEV void ge_tobytes(u32 w[8], const ge_ext& p) {
  fe29 zi, x, y;
  e29_inv(zi, p.Z);
  e29_mul(x, p.X, zi);
  e29_mul(y, p.Y, zi);
  u32 xw[8];
  e29_to_words(xw, x);
  e29_to_words(w, y);
  w[7] |= (xw[0] & 1u) << 31;
}

GV_DEV void ge_neg(ge_ext& r, const ge_ext& p) {
  e29_neg<1>(r.X, p.X);
  e29_norm(r.X, r.X);
  r.Y = p.Y;
  r.Z = p.Z;
  e29_neg<1>(r.T, p.T);
  e29_norm(r.T, r.T);
}

// ---- per-lane table j(-A), j = 1..8, cached form; word (e*36 + k) of lane
// at tab[(e*36 + k) * stride] (stride = lanes per launch: coalesced).
GV_DEV void atab_store(u32* tab, size_t stride, int e, const ge_cached& c) {
  const fe29* f[4] = {&c.ypx, &c.ymx, &c.z2, &c.t2d};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < 9; ++k) tab[(size_t)(e * ED_CACHED_WORDS + q * 9 + k) * stride] = f[q]->n[k];
}
GV_DEV void atab_load(ge_cached& c, const u32* tab, size_t stride, int e) {
  fe29* f[4] = {&c.ypx, &c.ymx, &c.z2, &c.t2d};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < 9; ++k) f[q]->n[k] = tab[(size_t)(e * ED_CACHED_WORDS + q * 9 + k) * stride];
}
GV_DEV void cached_identity(ge_cached& c) {
  e29_set(c.ypx, 1);
  e29_set(c.ymx, 1);
  e29_set(c.z2, 2);
  f29_set_zero(c.t2d);
}
GV_DEV void pre_load(ge_pre& q, const u32* btab, int w, int j) {
  const u32* e = btab + (size_t)(w * ED_BTAB_ENTRIES + j) * ED_PRE_WORDS;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    q.ypx.n[k] = e[k];
    q.ymx.n[k] = e[9 + k];
    q.xy2d.n[k] = e[18 + k];
  }
}

// Build the table of j(-A) (j = 0..8; entry 0 = the identity) for one lane.
GV_DEV void atab_build(u32* tab, size_t stride, const ge_ext& negA) {
  ge_cached c1, c;
  cached_identity(c);
  atab_store(tab, stride, 0, c);
  ge_to_cached(c1, negA);
  atab_store(tab, stride, 1, c1);
  ge_ext p2, acc;
  ge_dbl(p2, negA);
  ge_to_cached(c, p2);
  atab_store(tab, stride, 2, c);
  acc = p2;
  for (int j = 3; j <= 8; ++j) {
    ge_add_cached(acc, acc, c1, false);
    ge_to_cached(c, acc);
    atab_store(tab, stride, j, c);
  }
}

// Load one field element of 9 limbs, limb k at f[k * stride].
GV_DEV void fe_load(fe29& r, const u32* f, size_t stride) {
#pragma unroll
  for (int k = 0; k < 9; ++k) r.n[k] = f[(size_t)k * stride];
}

// r = p + (neg ? -q : q), q = entry e of this lane's table, its field
// elements loaded from memory right before use (the negation picks
// addresses, not values).  r may alias p.  T of r only when T_OUT.
template <bool T_OUT>
GV_DEV void ge_add_tab(ge_ext& r, const ge_ext& p, const u32* tab, size_t stride, int e, bool neg) {
  const u32* ent = tab + (size_t)(e * ED_CACHED_WORDS) * stride;
  const u32* qa = ent + (size_t)(neg ? 9 : 0) * stride;          // Y+X  (neg: Y-X)
  const u32* qb = ent + (size_t)(neg ? 0 : 9) * stride;
  fe29 t, q, a, b, x1, y1, dpc, dmc, z1, t1;
  f29_add(t, p.Y, p.X);
  fe_load(q, qa, stride);
  e29_mul(a, t, q);
  e29_sub<1>(t, p.Y, p.X);
  fe_load(q, qb, stride);
  e29_mul(b, t, q);
  e29_sub_norm<1>(x1, a, b);
  f29_add(y1, a, b);
  fe_load(q, ent + (size_t)27 * stride, stride);                  // 2dT
  e29_mul(a, q, p.T);
  fe_load(q, ent + (size_t)18 * stride, stride);                  // 2Z
  e29_mul(b, p.Z, q);
  f29_add(dpc, b, a);
  e29_sub_norm<1>(dmc, b, a);
  fe_select(z1, neg, dmc, dpc);
  fe_select(t1, neg, dpc, dmc);
  e29_mul(r.X, x1, t1);
  e29_mul(r.Y, y1, z1);
  e29_mul(r.Z, z1, t1);
  if (T_OUT) e29_mul(r.T, x1, y1);
}

// r = p + (neg ? -q : q), q = a comb-table entry (27 contiguous words).
GV_DEV void ge_add_pretab(ge_ext& r, const ge_ext& p, const u32* ent, bool neg) {
  fe29 t, q, a, b, x1, y1, dpc, dmc, z1, t1;
  f29_add(t, p.Y, p.X);
  fe_load(q, ent + (neg ? 9 : 0), 1);
  e29_mul(a, t, q);
  e29_sub<1>(t, p.Y, p.X);
  fe_load(q, ent + (neg ? 0 : 9), 1);
  e29_mul(b, t, q);
  e29_sub_norm<1>(x1, a, b);
  f29_add(y1, a, b);
  fe_load(q, ent + 18, 1);                                        // 2dxy
  e29_mul(a, q, p.T);
  f29_add(b, p.Z, p.Z);                                           // 2Z (mag 2)
  f29_add(dpc, b, a);                                             // mag 3
  e29_sub_norm<1>(dmc, b, a);
  fe_select(z1, neg, dmc, dpc);
  fe_select(t1, neg, dpc, dmc);
  e29_mul(r.X, x1, t1);
  e29_mul(r.Y, y1, z1);
  e29_mul(r.Z, z1, t1);
  e29_mul(r.T, x1, y1);
}

// Signed radix-16 recoding carries of h (< 2^253): bit i of the result = the
// carry OUT of digit i; digit i = nibble_i + carry_in_i - 16 carry_out_i in
// [-8, 8) (digit 63 = nibble_63 + carry_in_63 <= 2).
GV_DEV uint64_t sc_radix16_carries(const u32 h[8]) {
  uint64_t k = 0;
  u32 c = 0;
#pragma unroll
  for (int i = 0; i < 63; ++i) {
    const u32 nib = (h[i >> 3] >> (4 * (i & 7))) & 15u;
    c = (nib + c + 8u) >> 4;
    k |= (uint64_t)c << i;
  }
  return k;
}

// acc += [s]B from the radix-2^16 table: signed digits, LSB-first, digit w in
// (-2^15, 2^15] (a digit above 2^15 borrows 2^16 and carries one into the
// next window; s < 2^253 leaves no carry out of window 15).
GV_DEV void ed_add_sb16(ge_ext& acc, const u32 s[8], const u32* btab16) {
  int carry = 0;
#pragma unroll 1
  for (int w = 0; w < ED_BTAB16_WINDOWS; ++w) {
    int dgt = (int)((s[w >> 1] >> (16 * (w & 1))) & 0xFFFFu) + carry;
    carry = dgt > 32768 ? 1 : 0;
    dgt -= 65536 * carry;
    const int mag = dgt < 0 ? -dgt : dgt;
    ge_add_pretab(acc, acc, btab16 + (size_t)(w * ED_BTAB16_ENTRIES + mag) * ED_PRE_WORDS, dgt < 0);
  }
}

// R' = [h](-A) + [s]B and compare its encoding with rw (sig[:32] words).
// tab/stride: this lane's j(-A) table (already built); btab: the comb table;
// btab16 (may be null): the radix-2^16 comb table, then [s]B takes 16
// additions from it instead of 32 from btab.
GV_DEV bool ed_ladder_check(const u32 h[8], const u32 s[8], const u32* tab, size_t stride, const u32* btab,
                            const u32 rw[8], const u32* btab16 = nullptr) {
  // [h](-A): MSB-first, 4 doublings then one table add per digit
  uint64_t carries = sc_radix16_carries(h);
  u32 hs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) hs[i] = h[i];
  ge_ext acc;
  ge_identity(acc);
  for (int i = 63; i >= 0; --i) {
    if (i != 63) {
      ge_dbl_t<false>(acc, acc);
      ge_dbl_t<false>(acc, acc);
      ge_dbl_t<false>(acc, acc);
      ge_dbl_t<true>(acc, acc);
    }
    const int nib = (int)(hs[7] >> 28);
    const int cin = i > 0 ? (int)((carries >> (i - 1)) & 1u) : 0;
    const int cout = i < 63 ? (int)((carries >> i) & 1u) : 0;
    const int dgt = nib + cin - 16 * cout;
    // shift h left by one nibble so the next digit is on top
#pragma unroll
    for (int k = 7; k > 0; --k) hs[k] = (hs[k] << 4) | (hs[k - 1] >> 28);
    hs[0] <<= 4;
    const int mag = dgt < 0 ? -dgt : dgt;
    if (i) ge_add_tab<false>(acc, acc, tab, stride, mag, dgt < 0);   // a doubling follows
    else ge_add_tab<true>(acc, acc, tab, stride, mag, dgt < 0);      // the comb adds follow
  }
  // + [s]B: signed radix-256 digits, LSB-first, one precomputed add each
  // (or 16 radix-2^16 digits from btab16)
  if (btab16) {
    ed_add_sb16(acc, s, btab16);
  } else {
    u32 ss[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ss[i] = s[i];
    int carry = 0;
    for (int w = 0; w < ED_BTAB_WINDOWS; ++w) {
      int dgt = (int)(ss[0] & 0xFFu) + carry;
#pragma unroll
      for (int k = 0; k < 7; ++k) ss[k] = (ss[k] >> 8) | (ss[k + 1] << 24);
      ss[7] >>= 8;
      carry = dgt > 128 ? 1 : 0;
      dgt -= 256 * carry;
      const int mag = dgt < 0 ? -dgt : dgt;
      ge_add_pretab(acc, acc, btab + (size_t)(w * ED_BTAB_ENTRIES + mag) * ED_PRE_WORDS, dgt < 0);
    }
  }
  u32 ew[8];
  ge_tobytes(ew, acc);
  u32 diff = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) diff |= ew[i] ^ rw[i];
  return diff == 0;
}

}  // namespace ed
}  // namespace gv

namespace gv {
namespace ed {

// Comb table entry j * 256^w * B (affine precomputed form, 27 words).
GV_DEV void ed_btab_entry(u32 out[ED_PRE_WORDS], int w, int j) {
  ge_ext b;
  fe_const(b.X, kEdBx);
  fe_const(b.Y, kEdBy);
  e29_set(b.Z, 1);
  e29_mul(b.T, b.X, b.Y);
  for (int k = 0; k < 8 * w; ++k) ge_dbl(b, b);
  ge_cached cb;
  ge_to_cached(cb, b);
  ge_ext acc;
  ge_identity(acc);
  for (int bit = 7; bit >= 0; --bit) {
    ge_dbl(acc, acc);
    if ((j >> bit) & 1) ge_add_cached(acc, acc, cb, false);
  }
  ge_pre p;
  ge_to_pre(p, acc);
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    out[k] = p.ypx.n[k];
    out[9 + k] = p.ymx.n[k];
    out[18 + k] = p.xy2d.n[k];
  }
}

// Radix-2^16 comb table entry j * 65536^w * B (affine precomputed form).
GV_DEV void ed_btab16_entry(u32 out[ED_PRE_WORDS], int w, int j) {
  ge_ext b;
  fe_const(b.X, kEdBx);
  fe_const(b.Y, kEdBy);
  e29_set(b.Z, 1);
  e29_mul(b.T, b.X, b.Y);
  for (int k = 0; k < 16 * w; ++k) ge_dbl(b, b);
  ge_cached cb;
  ge_to_cached(cb, b);
  ge_ext acc;
  ge_identity(acc);
  for (int bit = 15; bit >= 0; --bit) {
    ge_dbl(acc, acc);
    if ((j >> bit) & 1) ge_add_cached(acc, acc, cb, false);
  }
  ge_pre p;
  ge_to_pre(p, acc);
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    out[k] = p.ypx.n[k];
    out[9 + k] = p.ymx.n[k];
    out[18 + k] = p.xy2d.n[k];
  }
}


// The per-item work before the ladder: h = SHA-512(R || A || M) mod L, the
// S checks (sig[63] & 224 == 0, ScMinimal), FromBytes(A) and the table
// j(-A).  Returns whether the item can still verify.
template <class Msg>
GV_DEV bool ed_prep_item(const u32 pw[8], const u32 sw[16], Msg msg, u32 len, u32* tab, size_t stride,
                         u32 h[8]) {
  u32 pre[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    pre[i] = sw[i];                     // R
    pre[8 + i] = pw[i];                 // A
  }
  u32 dig[16];
  sha512_pre64(dig, pre, msg, len);
  sc_reduce512(h, dig);                 // ScReduce
  const bool s_ok = (sw[15] >> 29) == 0 && sc_minimal(sw + 8);   // sig[63] & 224 == 0, ScMinimal
  ge_ext a, na;
  const bool a_ok = ge_frombytes(a, pw);
  ge_neg(na, a);
  atab_build(tab, stride, na);
  return s_ok && a_ok;
}

// One item of go1.14 crypto/ed25519 Verify (64-byte signature): pw = the 32
// key bytes as 8 little-endian words, sw = the signature as 16 words, msg(i)
// = message byte i.  tab/stride: this item's j(-A) scratch; btab: the comb
// table.  (The kernels run the two halves as two launches.)
template <class Msg>
GV_DEV bool ed_verify_item(const u32 pw[8], const u32 sw[16], Msg msg, u32 len, u32* tab, size_t stride,
                           const u32* btab) {
  u32 h[8];
  const bool pre_ok = ed_prep_item(pw, sw, msg, len, tab, stride, h);
  const bool r_ok = ed_ladder_check(h, sw + 8, tab, stride, btab, sw);
  return pre_ok && r_ok;
}

}  // namespace ed
}  // namespace gv
