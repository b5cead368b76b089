// secp_fe29x.cuh -- fused product engine for the 9 x 29 field layer
// (secp_fe29.cuh), used by the throughput ladder (k_ecmult).
//
// k_ecmult is VALU-issue bound (profiles/r02/pmc: ~95 % VALU busy, every
// VALU instruction ~one issue slot in this mix), so the lever is instructions
// per verify.  Two changes against f29_mulsqr, same arithmetic:
//
//  * High columns (weights 2^(29k), k = 9..16, folded later by 2^261): each
//    column's 64-bit sum is split as lo + 2^32 hi instead of (low 29 bits,
//    sum >> 29).  t_k = lo (a full 32-bit word; the fold multiplies it by
//    31264 and 256, products < 2^47) and hi re-enters column k+1 as 8 * hi
//    (weight 2^(29k+32) = 8 * 2^(29(k+1))) by one mad at the end of that
//    column's chain: 1 instruction per column instead of v_and + v_lshrrev_b64,
//    and the 8 high column chains are independent until their last mad.
//  * Extra terms: the reduction column j (weight 2^(29j)) can take
//    sum_e K_e * v_e[j] as further mads (f29x_plus), so "a*b - c", "a^2 - 8c"
//    etc. leave the chain already reduced: one mad per limb instead of a
//    separate carry pass (~4 instructions per limb).  A subtraction feeds
//    K_m - c (f29_neg) with a small multiplier.
//  * Squares take their operands explicitly: column terms a_i * dg_i on the
//    diagonal and a_i * cr_j (i < j) across, so 3a^2 is (dg, cr) = (3a, 6a)
//    and the caller's 2a can double as another product's operand.
//
// Bounds (host build: GV_F29_CHECK traps every wrapping mad / add; tests/
// test_fe29_host.py drives the extremes):
//   mul: mag(a) * mag(b) <= 6           -> column sums <= 54 B^2 < 2^63.8
//   sqr (dg, cr) = (a, 2a): mag(a) <= 2 (column 8: 9 m^2 B^2)
//   sqr (dg, cr) = (3a, 6a): mag(a) <= 1 (column 8: 27 B^2)
//   extras: sum_e K_e * v_e[j] < 2^40 per column
// Output: magnitude 1, like f29_mul.
#pragma once
#include "secp_fe29.cuh"

// GV_F29X_HICARRY: high columns split as lo + 2^32 hi, hi re-entering the next
// column by one mad (1), or the classic 29-bit extraction (0).
#ifndef GV_F29X_HICARRY
#define GV_F29X_HICARRY 1
#endif

// member functions: GV_DEV is "static inline" in host builds
#if defined(__HIPCC__)
#define GV_DEVM __device__ __forceinline__
#else
#define GV_DEVM inline
#endif

namespace gv {

// Small multipliers held in VGPRs behind a value barrier: left visible, the
// compiler strength-reduces "mad by 8" / "mad by 1" into 64-bit shift, mask
// and add sequences (3-4 instructions instead of one mad).
struct f29x_k {
  u32 one, eight;
  GV_DEVM u32 get(u32 K) const { return K == 1u ? one : K == 8u ? eight : K; }
};
// Column accumulator: F29X_NCH independent mad chains (terms dealt round
// robin, joined by one 64-bit add per extra chain).  1 in the throughput
// ladder (several waves per SIMD hide a mad's latency); 2 in the latency
// kernels, where one wave runs alone and a second chain fills the wait
// after each dependent mad.  The chain index is a compile-time constant
// after unrolling.
#ifndef F29X_NCH
#define F29X_NCH 1
#endif
struct f29x_acc {
  u64 c[F29X_NCH];
  int i;
  GV_DEVM void init(u64 v) {
    c[0] = v;
#pragma unroll
    for (int k = 1; k < F29X_NCH; ++k) c[k] = 0;
    i = 0;
  }
  GV_DEVM void mad(u32 x, u32 y) {
    c[i] = f29_mad(x, y, c[i]);
    i = (i + 1) % F29X_NCH;
  }
  GV_DEVM u64 sum() const {
    u64 s = c[0];
#pragma unroll
    for (int k = 1; k < F29X_NCH; ++k) s += c[k];
    return s;
  }
};

struct f29x_none {
  GV_DEVM void operator()(int, f29x_acc&, const f29x_k&) const {}
};
// column j += K * v[j]   (K = 1 or 8)
template <u32 K>
struct f29x_plus {
  const u32* v;
  GV_DEVM void operator()(int j, f29x_acc& a, const f29x_k& k) const { a.mad(v[j], k.get(K)); }
};
// column j += K1 * v[j] + K2 * w[j]
template <u32 K1, u32 K2>
struct f29x_plus2 {
  const u32* v;
  const u32* w;
  GV_DEVM void operator()(int j, f29x_acc& a, const f29x_k& k) const {
    a.mad(v[j], k.get(K1));
    a.mad(w[j], k.get(K2));
  }
};

// The reduction shared by the cores: high limbs t[0..8] (t[8] = limb 17) and
// the low columns' product terms (lowterms(j, acc)) -> r, magnitude 1.
template <class LOW, class EX>
GV_DEV void f29x_reduce(fe29& r, const u32 t[9], const LOW& lowterms, const EX& ex, u32 kr0, u32 kr1,
                        const f29x_k& kk) {
  fe29 o;
  u64 carry = 0;
#pragma unroll
  for (int j = 0; j <= 8; ++j) {
    f29x_acc A;
    A.init(carry);
    lowterms(j, A);
    A.mad(t[j], kr0);
    if (j >= 1) A.mad(t[j - 1], kr1);
    ex(j, A, kk);
    const u64 acc = A.sum();
    o.n[j] = (u32)acc & F29_M;
    carry = acc >> 29;
  }
  u64 acc = f29_mad(t[8], kr1, carry);        // 256 * limb 17 -> weight 2^261
  const u32 clo = (u32)acc, chi = (u32)(acc >> 32);
  u64 x = f29_mad(clo, kr0, (u64)o.n[0]);
  o.n[0] = (u32)x & F29_M;
  x = (x >> 29) + o.n[1];
  x = f29_mad(clo, kr1, x);
  x = f29_mad(chi, F29_RH1, x);
  o.n[1] = (u32)x & F29_M;
  o.n[2] = f29_add32(o.n[2], f29_add32((u32)(x >> 29), chi * F29_RH2));
  r = o;
}

// High columns k = 9..16 from hiterms(k, acc) -> t[0..8].
template <class HI>
GV_DEV void f29x_high(u32 t[9], const HI& hiterms, const f29x_k& kk) {
#if GV_F29X_HICARRY
  u32 hi = 0;
#pragma unroll
  for (int k = 9; k <= 16; ++k) {
    f29x_acc A;
    A.init(0);
    hiterms(k, A);
    if (k > 9) A.mad(hi, kk.eight);           // carry of column k-1 (weight 2^32 there)
    const u64 acc = A.sum();
    t[k - 9] = (u32)acc;
    hi = (u32)(acc >> 32);
  }
  F29_TRAP(hi >= (1u << 29), "x t17");
  t[8] = hi << 3;                             // limb 17
#else
  u64 carry = 0;                              // classic: 29-bit high limbs, carry chained
#pragma unroll
  for (int k = 9; k <= 16; ++k) {
    f29x_acc A;
    A.init(carry);
    hiterms(k, A);
    const u64 acc = A.sum();
    t[k - 9] = (u32)acc & F29_M;
    carry = acc >> 29;
  }
  F29_TRAP((carry >> 32) != 0, "x t17");
  t[8] = (u32)carry;                          // limb 17
#endif
}

#define F29X_CONSTS                                        \
  u32 kr0 = F29_R0, kr1 = F29_R1;                          \
  f29x_k kk{1u, 8u};                                       \
  F29X_BARRIER
#if defined(__HIP_DEVICE_COMPILE__)
#define F29X_BARRIER                                       \
  asm("" : "+v"(kr0), "+v"(kr1));                          \
  asm("" : "+v"(kk.one), "+v"(kk.eight));
#else
#define F29X_BARRIER
#endif

// SQR: r = sum_{i<=j} (i == j ? a_i dg_i : a_i cr_j) 2^(29(i+j)) mod p.
// !SQR: r = a * dg mod p (cr unused).  Then + the extra terms.  r may alias
// any input (written last).
template <bool SQR, class EX>
GV_DEV void f29x_core(fe29& r, const u32* a, const u32* dg, const u32* cr, const EX& ex) {
  F29X_CONSTS
  auto op = [&](int i, int j) -> u32 { return SQR ? (i == j ? dg[i] : cr[j]) : dg[j]; };
  u32 t[9];
  f29x_high(t, [&](int k, f29x_acc& A) {
#pragma unroll
    for (int i = k - 8; i <= (SQR ? (k >> 1) : 8); ++i) A.mad(a[i], op(i, k - i));
  }, kk);
  f29x_reduce(r, t, [&](int j, f29x_acc& A) {
#pragma unroll
    for (int i = 0; i <= (SQR ? (j >> 1) : j); ++i) A.mad(a[i], op(i, j - i));
  }, ex, kr0, kr1, kk);
}

// r = a * b + c * d (+ extras): both products summed in the same column
// chains, one reduction.  mag(a) mag(b) + mag(c) mag(d) <= 6.
template <class EX = f29x_none>
GV_DEV void f29x_mul2(fe29& r, const fe29& a, const fe29& b, const fe29& c, const fe29& d, const EX& ex = EX()) {
  F29X_CONSTS
  u32 t[9];
  f29x_high(t, [&](int k, f29x_acc& A) {
#pragma unroll
    for (int i = k - 8; i <= 8; ++i) A.mad(a.n[i], b.n[k - i]);
#pragma unroll
    for (int i = k - 8; i <= 8; ++i) A.mad(c.n[i], d.n[k - i]);
  }, kk);
  f29x_reduce(r, t, [&](int j, f29x_acc& A) {
#pragma unroll
    for (int i = 0; i <= j; ++i) A.mad(a.n[i], b.n[j - i]);
#pragma unroll
    for (int i = 0; i <= j; ++i) A.mad(c.n[i], d.n[j - i]);
  }, ex, kr0, kr1, kk);
}

// r = a * b (+ extras).  mag(a) * mag(b) <= 6.
template <class EX = f29x_none>
GV_DEV void f29x_mul(fe29& r, const fe29& a, const fe29& b, const EX& ex = EX()) {
  f29x_core<false>(r, a.n, b.n, b.n, ex);
}
// r = a^2 (+ extras) given d = 2a.  mag(a) <= 2.
template <class EX = f29x_none>
GV_DEV void f29x_sqr_d(fe29& r, const fe29& a, const fe29& d, const EX& ex = EX()) {
  f29x_core<true>(r, a.n, a.n, d.n, ex);
}
// r = 2a, no carries (limbs < 2^31)
GV_DEV void f29x_shl1(fe29& r, const fe29& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    F29_TRAP(a.n[i] >= 0x80000000u, "shl1");
    r.n[i] = a.n[i] << 1;
  }
}
template <class EX = f29x_none>
GV_DEV void f29x_sqr(fe29& r, const fe29& a, const EX& ex = EX()) {
  fe29 d;
  f29x_shl1(d, a);
  f29x_core<true>(r, a.n, a.n, d.n, ex);
}
// r = 3 a^2 (+ extras).  mag(a) <= 1.
template <class EX = f29x_none>
GV_DEV void f29x_sqr3(fe29& r, const fe29& a, const EX& ex = EX()) {
  fe29 a3, a6;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    a3.n[i] = f29_add32(a.n[i] << 1, a.n[i]);
    a6.n[i] = a3.n[i] << 1;
  }
  f29x_core<true>(r, a.n, a3.n, a6.n, ex);
}

}  // namespace gv
