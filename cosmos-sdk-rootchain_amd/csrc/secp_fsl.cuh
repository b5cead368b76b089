// secp_fsl.cuh -- limb-sliced GF(p) arithmetic for the latency kernels
// (gv_lat.hip): ONE field element per 16-lane DPP row, limb i of the 9 x 29
// representation (secp_fe29.cuh) in lane i of the row, lanes 9..15 zero.
//
// Why: a lone wave issues one instruction every ~4-6 cycles whatever the
// number of active lanes (tools/microbench/lat_ops.hip: f29_mul 876 cycles,
// a Jacobian doubling 5,715 on one lane).  The small-batch kernel is bound by
// that serial chain, so spreading each field operation over the nine limb
// lanes shortens it: a product is 9 broadcast / shifted DPP moves and 9 mads
// per lane (lane c sums column c), the reduction folds the high columns with
// per-lane constants, and additions are ONE instruction instead of nine.
//
// Product (lane c = column c, c = 0..15; column 16 = a8*b8 kept row-uniform):
//   col_c = sum_i a_i * b_(c-i)       a_i: row_newbcast:i,  b_(c-i): row_shr:i
// Reduction, 2^261 == 2^37 + 31264 (mod p):
//   R1  split every column into 29 + 29 + 6 bits, move the upper parts one and
//       two lanes up (columns 16..18 stay row-uniform);
//   F   lane c (0..8) += 31264 * w_(c+9) + 256 * w_(c+8) + K16 w16 + K17 w17 +
//       K18 w18 (K_j = 2^(29 j) mod p, as per-lane limb constants), in 64 bits;
//   R2  one carry pass, the carry out of limb 8 folded into limbs 0 and 1;
//   R3  one more carry step over limbs 0..7 (limb 8 keeps its bit).
// Bounds (N-form: every limb < 2^29 + 2^17, the output of every product and
// of fsl_norm):
//   mul(a, b) needs max_limb(a) * max_limb(b) < 2^60.8 (column sums of nine
//   products < 2^64): N x N, N x 4N, 2N x 2N, N x (4N + BIAS) all fit.
//   The F accumulator stays < 2^53; extras folded into it (mul_plus) are
//   64-bit values < 2^36.
//   BIAS (sub/neg) has limbs in [2^29 + 2^16, 2^30 + 2^16], == 0 (mod p), so
//   a - b = a + BIAS - b is non-negative for b in N-form.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "secp_fe29.cuh"

namespace gv {

// DPP moves (gfx950: row_newbcast / row_shr / row_shl on 16-lane rows).
// bound_ctrl: a lane whose source lies outside its row reads 0.
template <int I> GV_DEV u32 fsl_bc(u32 v) { return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + I, 0xF, 0xF, true); }
template <int I> GV_DEV u32 fsl_shr(u32 v) { return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + I, 0xF, 0xF, true); }
template <int I> GV_DEV u32 fsl_shl(u32 v) { return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + I, 0xF, 0xF, true); }

// Per-lane constants of the row layout (computed once per kernel).
struct fslk {
  u32 L;          // lane within the row
  u32 m29;        // 2^29 - 1 for limbs 0..8, 0 above
  u32 mw;         // all ones for limbs 0..8, 0 above
  u32 m29lo;      // 2^29 - 1 for limbs 0..7, all ones for limb 8, 0 above (R3)
  u32 k9, k8;     // fold of columns 9..15: 31264 (c - 9), 256 (c - 8)
  u32 k16, k17, k18;
  u32 kc;         // carry out of limb 8: 31264 into limb 0, 256 into limb 1
  u32 bias;       // BIAS limb
  u64 big8;       // BIG8 limb (== 0 mod p, limbs >= 8 * 2^29.01): 64-bit extras
};

GV_DEV fslk fsl_consts() {
  fslk k;
  const u32 L = __lane_id() & 15u;
  k.L = L;
  const bool lo = L <= 8u;
  k.m29 = lo ? F29_M : 0u;
  k.mw = lo ? 0xFFFFFFFFu : 0u;
  k.m29lo = L < 8u ? F29_M : (L == 8u ? 0xFFFFFFFFu : 0u);
  k.k9 = lo ? 31264u : 0u;
  k.k8 = (L >= 1u && L <= 8u) ? 256u : 0u;
  k.k16 = L == 7u ? 31264u : (L == 8u ? 256u : 0u);
  k.k17 = L == 0u ? 8003584u : (L == 1u ? 65536u : (L == 8u ? 31264u : 0u));
  k.k18 = L == 0u ? 440566784u : (L == 1u ? 16007169u : (L == 2u ? 65536u : 0u));
  k.kc = L == 0u ? 31264u : (L == 1u ? 256u : 0u);
  k.bias = !lo ? 0u : (L == 0u ? 0x3fff0bc0u : (L == 1u ? 0x3ffffdfeu : 0x3ffffffeu));
  k.big8 = !lo ? 0ull : (L == 0u ? 0x1fff85e00ull : (L == 1u ? 0x1ffffeff0ull : 0x1fffffff0ull));
  return k;
}

// FSL_BARRIER: an empty asm value barrier after every mad keeps the chains as
// written (the compiler otherwise may split a mad into a product and a 64-bit
// add); 0 lets the scheduler interleave independent products.
#ifndef FSL_BARRIER
#define FSL_BARRIER 0
#endif
GV_DEV u64 fsl_mad(u32 a, u32 b, u64 c) {
  u64 r = (u64)a * b + c;
#if FSL_BARRIER
  asm("" : "+v"(r));
#endif
  return r;
}

// The 64-bit product columns of a * b (+ a2 * b2), column 16 row-uniform.
template <bool TWO>
GV_DEV void fsl_cols(u64& v, u64& u, u32 a, u32 b, u32 a2, u32 b2) {
  u64 c0 = fsl_mad(fsl_bc<0>(a), b, 0), c1 = fsl_mad(fsl_bc<1>(a), fsl_shr<1>(b), 0);
  c0 = fsl_mad(fsl_bc<2>(a), fsl_shr<2>(b), c0);
  c1 = fsl_mad(fsl_bc<3>(a), fsl_shr<3>(b), c1);
  c0 = fsl_mad(fsl_bc<4>(a), fsl_shr<4>(b), c0);
  c1 = fsl_mad(fsl_bc<5>(a), fsl_shr<5>(b), c1);
  c0 = fsl_mad(fsl_bc<6>(a), fsl_shr<6>(b), c0);
  c1 = fsl_mad(fsl_bc<7>(a), fsl_shr<7>(b), c1);
  const u32 a8 = fsl_bc<8>(a);
  c0 = fsl_mad(a8, fsl_shr<8>(b), c0);
  u = (u64)a8 * fsl_bc<8>(b);
  if constexpr (TWO) {
    c1 = fsl_mad(fsl_bc<0>(a2), b2, c1);
    c0 = fsl_mad(fsl_bc<1>(a2), fsl_shr<1>(b2), c0);
    c1 = fsl_mad(fsl_bc<2>(a2), fsl_shr<2>(b2), c1);
    c0 = fsl_mad(fsl_bc<3>(a2), fsl_shr<3>(b2), c0);
    c1 = fsl_mad(fsl_bc<4>(a2), fsl_shr<4>(b2), c1);
    c0 = fsl_mad(fsl_bc<5>(a2), fsl_shr<5>(b2), c0);
    c1 = fsl_mad(fsl_bc<6>(a2), fsl_shr<6>(b2), c1);
    c0 = fsl_mad(fsl_bc<7>(a2), fsl_shr<7>(b2), c0);
    const u32 b8 = fsl_bc<8>(a2);
    c1 = fsl_mad(b8, fsl_shr<8>(b2), c1);
    u = fsl_mad(b8, fsl_bc<8>(b2), u);
  }
  v = c0 + c1;
}

// Columns -> N-form limbs, plus a 64-bit per-limb extra (== its value mod p
// is added; < 2^40) folded in before R2.
GV_DEV u32 fsl_reduce(u64 v, u64 u, u64 extra, const fslk& k) {
  // R1
  const u32 lo = (u32)v & F29_M;
  const u32 m = (u32)(v >> 29) & F29_M;
  const u32 h = (u32)(v >> 58);
  const u32 w = lo + fsl_shr<1>(m) + fsl_shr<2>(h);
  const u32 w16 = ((u32)u & F29_M) + fsl_bc<15>(m) + fsl_bc<14>(h);
  const u32 w17 = ((u32)(u >> 29) & F29_M) + fsl_bc<15>(h);
  const u32 w18 = (u32)(u >> 58);
  // F
  u64 t = (u64)(w & k.mw) + extra;
  t = fsl_mad(fsl_shl<9>(w), k.k9, t);
  t = fsl_mad(fsl_shl<8>(w), k.k8, t);
  t = fsl_mad(w16, k.k16, t);
  t = fsl_mad(w17, k.k17, t);
  t = fsl_mad(w18, k.k18, t);
  // R2: carries up one lane; limb 8's carry (lane 9) back into limbs 0, 1
  const u32 m2 = (u32)(t >> 29);
  u32 x = ((u32)t & k.m29) + fsl_shr<1>(m2);
  x = (x + __umul24(fsl_bc<9>(x), k.kc)) & k.mw;
  // R3: limbs 0..7 once more (limb 0 may be ~2^30.5 after the fold)
  const u32 c = (x & ~k.m29lo) >> 29;
  return (x & k.m29lo) + fsl_shr<1>(c);
}

GV_DEV u32 fsl_mul(u32 a, u32 b, const fslk& k) {
  u64 v, u;
  fsl_cols<false>(v, u, a, b, 0u, 0u);
  return fsl_reduce(v, u, 0ull, k);
}
GV_DEV u32 fsl_sqr(u32 a, const fslk& k) { return fsl_mul(a, a, k); }
// a * b + extra (extra: 64-bit per limb, e.g. BIG8 - 8 d)
GV_DEV u32 fsl_mul_plus(u32 a, u32 b, u64 extra, const fslk& k) {
  u64 v, u;
  fsl_cols<false>(v, u, a, b, 0u, 0u);
  return fsl_reduce(v, u, extra, k);
}
// a * b + c * d, one reduction
GV_DEV u32 fsl_mul2(u32 a, u32 b, u32 c, u32 d, const fslk& k) {
  u64 v, u;
  fsl_cols<true>(v, u, a, b, c, d);
  return fsl_reduce(v, u, 0ull, k);
}

// Carry pass: limbs < 2^32 -> N-form.
GV_DEV u32 fsl_norm(u32 x, const fslk& k) {
  const u32 c = x >> 29;
  x = (x & k.m29) + fsl_shr<1>(c);
  x = (x + __umul24(fsl_bc<9>(x), k.kc)) & k.mw;
  const u32 c2 = (x & ~k.m29lo) >> 29;
  return (x & k.m29lo) + fsl_shr<1>(c2);
}
// a - b for b in N-form (result < 2^31; not N-form)
GV_DEV u32 fsl_sub_raw(u32 a, u32 b, const fslk& k) { return a + k.bias - b; }
GV_DEV u32 fsl_sub(u32 a, u32 b, const fslk& k) { return fsl_norm(a + k.bias - b, k); }
GV_DEV u32 fsl_neg(u32 b, const fslk& k) { return fsl_norm(k.bias - b, k); }

// Row gather: the nine limbs of the row's element in every lane of the row.
GV_DEV void fsl_gather(fe29& r, u32 v) {
  r.n[0] = fsl_bc<0>(v); r.n[1] = fsl_bc<1>(v); r.n[2] = fsl_bc<2>(v);
  r.n[3] = fsl_bc<3>(v); r.n[4] = fsl_bc<4>(v); r.n[5] = fsl_bc<5>(v);
  r.n[6] = fsl_bc<6>(v); r.n[7] = fsl_bc<7>(v); r.n[8] = fsl_bc<8>(v);
}
// A lane-held fe29 (the same in every lane of the row) -> sliced.
GV_DEV u32 fsl_scatter(const fe29& a, const fslk& k) {
  u32 v = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) v = (k.L == (u32)i) ? a.n[i] : v;
  return v;
}
// Affine words (8 x 32, little-endian, uniform in the row) -> sliced.
GV_DEV u32 fsl_from_words(const u32 w[8], const fslk& k) {
  fe29 t;
  f29_from_words(t, w);
  return fsl_scatter(t, k);
}
// Limb L of a value stored as 8 little-endian words at p (lane-private load).
GV_DEV u32 fsl_load_words(const u32* p, const fslk& k) {
  const u32 bit = 29u * k.L, wi = bit >> 5, sh = bit & 31u;
  if (k.L > 8u) return 0u;
  const u32 lo = p[wi];
  const u32 hi = wi < 7u ? p[wi + 1] : 0u;
  return (u32)((((u64)hi << 32) | lo) >> sh) & F29_M;
}

// a == 0 (mod p) for limbs < 2^32 (row-uniform answer): the low-limb filter
// of f29_is_zero_fast, then the canonical test on the gathered element.
GV_DEV bool fsl_is_zero(u32 a) {
  const u32 z = fsl_bc<0>(a) & F29_M;
  const bool cand = (z == 0u) | (z >= F29_M + 1u - 977u * 256u);
  bool res = false;
  if (cand) {
    fe29 t;
    fsl_gather(t, a);
    res = f29_is_zero(t);
  }
  return res;
}

// ------------------------------------------------------------ rows of a wave
// The row-parallel kernels (k_verify_lat_sl4, k_ed_lat_unc) keep ONE point
// per wave, replicated in its four rows, and give each row a different
// product of the same round; every row then needs every row's result.
// The four rows' values of v, each in every row: r[i] = row i's v (three
// lane swaps, VALU only).
struct rows4 { u32 r[4]; };
GV_DEV rows4 rows_all(u32 v) {
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);     // {v0 v0 v2 v2}, {v1 v1 v3 v3}
  const auto e = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);   // v0, v2
  const auto o = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false);   // v1, v3
  rows4 r;
  r.r[0] = e[0]; r.r[1] = o[0]; r.r[2] = e[1]; r.r[3] = o[1];
  return r;
}

// Row r's operand of four: every candidate is materialised first (the empty
// asm keeps the compiler from sinking a candidate's arithmetic into a branch
// on the row), then one v_cndmask per step.
GV_DEV u32 rsel(u32 row, u32 a, u32 b, u32 c, u32 d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  u32 r = row == 1u ? b : a;
  r = row == 2u ? c : r;
  return row == 3u ? d : r;
}
GV_DEV u64 rsel64(u32 row, u64 a, u64 b, u64 c, u64 d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  u64 r = row == 1u ? b : a;
  r = row == 2u ? c : r;
  return row == 3u ? d : r;
}

// One-shot LDS flags between the waves of a block (a wave waits only for the
// producer it needs, instead of a block barrier).
GV_DEV void lds_flag_set(u32* f) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
GV_DEV void lds_flag_wait(u32* f) {
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) __builtin_amdgcn_s_sleep(2);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ------------------------------------------------------------ group law
// Jacobian point, one row: X, Y, Z sliced (N-form).
struct gjsl { u32 x, y, z; };

// r = 2a, 3M + 4S (gej29_double's formula):
//   B = Y^2, Z3 = 2Y Z, E = 3X^2, D = X B, C = B^2,
//   X3 = E^2 - 8D, Y3 = E (4D - X3) - 8C.
// Operand order: products sharing a first operand share its nine row
// broadcasts, products sharing a second operand its eight row shifts
// (Y: B, Z3; X: E, D; B: D, C; E: X3, Y3).
GV_DEV void gjsl_double(gjsl& r, const gjsl& a, const fslk& k) {
  const u32 B = fsl_sqr(a.y, k);
  const u32 z3 = fsl_mul(a.y, a.z << 1, k);                 // N x 2N
  const u32 E = fsl_mul(a.x, a.x * 3u, k);                  // N x 3N
  const u32 D = fsl_mul(a.x, B, k);
  const u32 C = fsl_mul(B, B, k);
  const u32 x3 = fsl_mul_plus(E, E, k.big8 - ((u64)D << 3), k);
  const u32 t = (D << 2) + k.bias - x3;                     // < 2^31.1
  r.y = fsl_mul_plus(E, t, k.big8 - ((u64)C << 3), k);     // N x (4N + BIAS)
  r.x = x3;
  r.z = z3;
}

// a += (x, y), affine on the curve scaled by az (gej29x_add_scaled's
// semantics): U2 = x az^2, S2 = y az^3, H = U2 - X1, R = S2 - Y1; H == 0:
// R == 0 -> doubling, else infinity.  a finite.  x N-form, y < 2^30.1.
GV_DEV void gjsl_add_scaled(gjsl& a, bool& inf, u32 x, u32 y, u32 az, const fslk& k) {
  const u32 z2 = fsl_sqr(az, k);
  const u32 h = fsl_mul_plus(x, z2, (u64)(k.bias - a.x), k);
  const u32 z3 = fsl_mul(z2, az, k);
  const u32 rr = fsl_mul_plus(y, z3, (u64)(k.bias - a.y), k);
  bool dbl = false;
  if (fsl_is_zero(h)) {
    dbl = fsl_is_zero(rr);
    if (!dbl) inf = true;                                   // a == -b
  } else {
    const u32 h2 = fsl_sqr(h, k);
    const u32 h3 = fsl_mul(h2, h, k);
    const u32 v = fsl_mul(a.x, h2, k);
    a.z = fsl_mul(a.z, h, k);
    a.x = fsl_mul_plus(rr, rr, k.big8 - (u64)h3 - ((u64)v << 1), k);   // R^2 - H^3 - 2V
    const u32 t = v + k.bias - a.x;                          // V - X3 < 2^31.1
    const u32 ny = k.bias - a.y;                             // -Y1 < 2^30.1
    a.y = fsl_mul2(rr, t, ny, h3, k);                        // R (V - X3) - Y1 H^3
  }
  if (dbl) gjsl_double(a, a, k);
}

// r = a + b, two Jacobian points of the row's curve (gej29_add_gej's formula
// and cases): either infinite -> the other; a == b -> 2a; a == -b -> infinity.
GV_DEV void gjsl_add_gej(gjsl& r, bool& rinf, const gjsl& a, bool ainf, const gjsl& b, bool binf,
                         const fslk& k) {
  if (ainf || binf) {
    r.x = ainf ? b.x : a.x;
    r.y = ainf ? b.y : a.y;
    r.z = ainf ? b.z : a.z;
    rinf = ainf && binf;
    return;
  }
  const u32 z1z1 = fsl_sqr(a.z, k), z2z2 = fsl_sqr(b.z, k);
  const u32 u1 = fsl_mul(a.x, z2z2, k), u2 = fsl_mul(b.x, z1z1, k);
  const u32 s1 = fsl_mul(a.y, fsl_mul(b.z, z2z2, k), k);
  const u32 s2 = fsl_mul(b.y, fsl_mul(a.z, z1z1, k), k);
  const u32 h = fsl_sub(u2, u1, k), rr = fsl_sub(s2, s1, k);
  bool inf = false, dbl = false;
  gjsl o = a;
  if (fsl_is_zero(h)) {
    dbl = fsl_is_zero(rr);
    inf = !dbl;
  } else {
    const u32 h2 = fsl_sqr(h, k);
    const u32 h3 = fsl_mul(h2, h, k);
    const u32 v = fsl_mul(u1, h2, k);
    o.z = fsl_mul(fsl_mul(a.z, b.z, k), h, k);
    o.x = fsl_mul_plus(rr, rr, k.big8 - (u64)h3 - ((u64)v << 1), k);
    const u32 t = v + k.bias - o.x;
    o.y = fsl_mul2(rr, t, k.bias - s1, h3, k);             // R (V - X3) - S1 H^3
  }
  if (dbl) gjsl_double(o, a, k);
  r = o;
  rinf = inf;
}

// ------------------------------------------------------- exponentiation
GV_DEV u32 fsl_sqr_n(u32 a, int n, const fslk& k) {
#pragma unroll 1
  for (int i = 0; i < n; ++i) a = fsl_sqr(a, k);
  return a;
}
// a^((p+1)/4): btcec decompressPoint's square-root candidate, the addition
// chain of f29_sqrt_candidate (secp_group29.cuh).
GV_DEV u32 fsl_sqrt_candidate(u32 a, const fslk& k) {
  const u32 x2 = fsl_mul(fsl_sqr(a, k), a, k);                 // 2^2 - 1
  const u32 x3 = fsl_mul(fsl_sqr(x2, k), a, k);                // 2^3 - 1
  const u32 x6 = fsl_mul(fsl_sqr_n(x3, 3, k), x3, k);
  const u32 x9 = fsl_mul(fsl_sqr_n(x6, 3, k), x3, k);
  const u32 x11 = fsl_mul(fsl_sqr_n(x9, 2, k), x2, k);
  const u32 x22 = fsl_mul(fsl_sqr_n(x11, 11, k), x11, k);
  const u32 x44 = fsl_mul(fsl_sqr_n(x22, 22, k), x22, k);
  const u32 x88 = fsl_mul(fsl_sqr_n(x44, 44, k), x44, k);
  const u32 x176 = fsl_mul(fsl_sqr_n(x88, 88, k), x88, k);
  const u32 x220 = fsl_mul(fsl_sqr_n(x176, 44, k), x44, k);
  const u32 x223 = fsl_mul(fsl_sqr_n(x220, 3, k), x3, k);
  u32 t = fsl_mul(fsl_sqr_n(x223, 23, k), x22, k);
  t = fsl_mul(fsl_sqr_n(t, 6, k), x2, k);
  return fsl_sqr_n(t, 2, k);
}

// canonical 8 x 32 words of the row's element (every lane of the row)
GV_DEV void fsl_to_words(u32 w[8], u32 a) {
  fe29 t;
  fsl_gather(t, a);
  f29_to_words(w, t);
}

}  // namespace gv
