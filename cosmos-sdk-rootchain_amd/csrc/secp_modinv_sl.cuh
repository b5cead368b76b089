// secp_modinv_sl.cuh -- s^-1 mod n for the sliced latency kernels: the
// variable-time divsteps of secp_modinv.cuh (s30_divsteps_var, row-uniform)
// with the four 9-limb state vectors f, g, d, e held ONE LIMB PER LANE of a
// 16-lane row (limb i in lane i, lanes 9..15 zero), so each round's matrix
// application is two or three signed mads per lane instead of a 9-limb
// serial carry chain.
//
// Per round (t = (u, v, q, r) from 30 divsteps, |u| + |v| <= 2^30):
//   f, g <- (u f + v g) / 2^30, (q f + r g) / 2^30       (exact division)
//   d, e <- (u d + v e + md n) / 2^30, (q d + r e + me n) / 2^30
// with md, me in [0, 2^30) clearing the low 30 bits (n^-1 mod 2^30).  The
// division is a shift down by one lane: new limb j = lo(c_(j+1)) + hi(c_j),
// lo = c mod 2^30, hi = c >> 30 (arithmetic); one parallel carry pass then
// keeps limbs 0..7 in [-4, 2^30 + 4) (signed, redundant; limb 8 signed).
// Bounds: |c| < 2^61; |d|, |e| grow by at most n per round (no per-round
// reduction): |d| < 26 n after 25 rounds, reduced once at the end.  Rounds
// after g == 0 leave f and d unchanged, so an undetected redundant zero only
// costs a round.
#pragma once
#include "secp_modinv.cuh"
#include "secp_fsl.cuh"

namespace gv {

GV_DEV int32_t msl_shl1(int32_t v) { return (int32_t)fsl_shl<1>((u32)v); }
GV_DEV int32_t msl_shr1(int32_t v) { return (int32_t)fsl_shr<1>((u32)v); }

// c (64-bit signed per limb, value divisible by 2^30) -> c / 2^30, one carry
// pass.  |c| < 2^61 -> |x| < 2^32 (64-bit), carries in [-4, 4].
GV_DEV int32_t msl_div30(int64_t c, u32 L) {
  const int32_t lo = (int32_t)((u32)c & S30_M);
  const int64_t x = (int64_t)msl_shl1(lo) + (c >> 30);       // limb j: lo_(j+1) + hi_j
  const int32_t keep = L < 8u ? (int32_t)((u32)x & S30_M) : (L == 8u ? (int32_t)x : 0);
  const int32_t carry = L < 8u ? (int32_t)(x >> 30) : 0;
  return keep + msl_shr1(carry);
}

// Serial exact value of a sliced signed-30 vector (row-uniform result):
// canonical limbs 0..7 in [0, 2^30), limb 8 signed.
GV_DEV void msl_gather_norm(s30& r, int32_t v) {
  int64_t c = 0;
  int32_t t[9];
  t[0] = (int32_t)fsl_bc<0>((u32)v); t[1] = (int32_t)fsl_bc<1>((u32)v); t[2] = (int32_t)fsl_bc<2>((u32)v);
  t[3] = (int32_t)fsl_bc<3>((u32)v); t[4] = (int32_t)fsl_bc<4>((u32)v); t[5] = (int32_t)fsl_bc<5>((u32)v);
  t[6] = (int32_t)fsl_bc<6>((u32)v); t[7] = (int32_t)fsl_bc<7>((u32)v); t[8] = (int32_t)fsl_bc<8>((u32)v);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    c += t[i];
    r.v[i] = i < 8 ? (int32_t)((uint32_t)c & S30_M) : (int32_t)c;
    c >>= 30;
  }
}

// a in (-64 n, 64 n) (canonical signed limbs) -> a mod n in [0, n)
GV_DEV void msl_reduce_n(s30& a) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {                              // a += 64 n  -> (0, 128 n)
    c += (int64_t)a.v[i] + ((int64_t)s30_n(i) << 6);
    a.v[i] = i < 8 ? (int32_t)((uint32_t)c & S30_M) : (int32_t)c;
    c >>= 30;
  }
#pragma unroll
  for (int s = 6; s >= 0; --s) {                             // greedy: subtract 2^s n when it fits
    s30 t;
    c = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      c += (int64_t)a.v[i] - ((int64_t)s30_n(i) << s);
      t.v[i] = i < 8 ? (int32_t)((uint32_t)c & S30_M) : (int32_t)c;
      c >>= 30;
    }
    const bool ge = t.v[8] >= 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) a.v[i] = ge ? t.v[i] : a.v[i];
  }
}

// w = x^-1 mod n (0 < x < n; x == 0 gives 0).  Every lane of the wave runs it
// with the same x (rows identical); every lane receives w.
GV_DEV void s30_modinv_sl(uint32_t w[8], const uint32_t x[8], const fslk& k) {
  const u32 L = k.L;
  s30 xs;
  s30_from_words(xs, x);
  int32_t nl = 0, g = 0, d = 0, e = L == 0u ? 1 : 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    nl = L == (u32)i ? s30_n(i) : nl;                        // limb L of n
    g = L == (u32)i ? xs.v[i] : g;
  }
  int32_t f = nl;
  int32_t eta = -1;
#pragma unroll 1
  for (int round = 0; round < 25; ++round) {                 // g == 0 within 590 divsteps (20 rounds)
    if (__ballot(g != 0) == 0ull) break;
    const u32 f0 = fsl_bc<0>((u32)f), f1 = fsl_bc<1>((u32)f);
    const u32 g0 = fsl_bc<0>((u32)g), g1 = fsl_bc<1>((u32)g);
    // the low words are the same in every lane: readfirstlane makes the
    // divsteps wave-uniform, so they compile to scalar (SALU) code
    const u32 flo = (u32)__builtin_amdgcn_readfirstlane((int)(f0 + (f1 << 30)));
    const u32 glo = (u32)__builtin_amdgcn_readfirstlane((int)(g0 + (g1 << 30)));
    int32_t t[4];
    eta = s30_divsteps_var(eta, flo, glo, t);
    const int64_t cf = (int64_t)t[0] * f + (int64_t)t[1] * g;
    const int64_t cg = (int64_t)t[2] * f + (int64_t)t[3] * g;
    f = msl_div30(cf, L);
    g = msl_div30(cg, L);
    const int32_t d0 = (int32_t)fsl_bc<0>((u32)d), e0 = (int32_t)fsl_bc<0>((u32)e);
    const int64_t cd0 = (int64_t)t[0] * d0 + (int64_t)t[1] * e0;
    const int64_t ce0 = (int64_t)t[2] * d0 + (int64_t)t[3] * e0;
    const int32_t md = (int32_t)(((0u - (uint32_t)cd0) * S30_N_INV) & S30_M);
    const int32_t me = (int32_t)(((0u - (uint32_t)ce0) * S30_N_INV) & S30_M);
    const int64_t cd = (int64_t)t[0] * d + (int64_t)t[1] * e + (int64_t)md * nl;
    const int64_t ce = (int64_t)t[2] * d + (int64_t)t[3] * e + (int64_t)me * nl;
    d = msl_div30(cd, L);
    e = msl_div30(ce, L);
  }
  s30 fs, ds;
  msl_gather_norm(fs, f);
  msl_gather_norm(ds, d);
  if (fs.v[8] < 0) {                                         // f = -1: the inverse is -d
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      c -= ds.v[i];
      ds.v[i] = i < 8 ? (int32_t)((uint32_t)c & S30_M) : (int32_t)c;
      c >>= 30;
    }
  }
  msl_reduce_n(ds);
  s30_to_words(w, ds);
}

}  // namespace gv
