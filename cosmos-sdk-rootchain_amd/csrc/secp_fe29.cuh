// secp_fe29.cuh -- secp256k1 base field in reduced radix 2^29: 9 limbs, one
// element per lane, with magnitude tracking (value = sum n[i] * 2^(29 i)).
//
// Why 9 x 29 on gfx950 (measured rates: profiles/r01/alu_rate_v4.jsonl):
//   * v_mad_u64_u32 (64-bit addend) issues in ~4.7 cycles per wave64, a
//     carry-propagating v_addc_co_u32 in 4, plain 32-bit VOP2 ops (and, shifts,
//     add/sub without carry) in 2.
//   * With 29-bit limbs a product column holds at most 9 products < 2^61
//     (inputs of magnitude <= 2, or one of them <= 6 against magnitude 1), so a
//     whole column is summed inside v_mad_u64_u32's 64-bit addend with NO
//     carry instruction: 81 mads per multiply (45 per square) instead of the
//     8 x 32 layout's 64 mads + 49 carry adds + column moves.
//   * The reduction folds the nine high limbs with 2^261 == 2^37 + 31264
//     (mod p) as two more mads per limb inside the same column chains.
//   * Additions and subtractions are limb-wise 2-cycle ops with no carries; a
//     carry pass ("weak normalisation") is inserted only where the magnitude
//     budget demands it.
//
// Magnitude m: every limb <= m * F29_B, F29_B = 2^29 + 2^18.  mul/sqr outputs
// and f29_norm outputs have magnitude 1.  Limits (checked by the host build's
// GV_F29_CHECK overflow traps and by tests/test_fe29_host.py):
//   mul(a, b):   mag(a) * mag(b) <= 6          sqr(a):  mag(a) <= 2
//   add/sub/neg: result magnitude <= 7 (limbs stay below 2^32)
//   f29_norm:    input magnitude <= 7
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

#if defined(GV_F29_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
#include <stdio.h>
#include <stdlib.h>
#define F29_TRAP(cond, what)                                   \
  do {                                                         \
    if (cond) { fprintf(stderr, "fe29 overflow: %s\n", what); abort(); } \
  } while (0)
#else
#define F29_TRAP(cond, what) do { } while (0)
#endif

namespace gv {

typedef uint32_t u32;
typedef uint64_t u64;

struct fe29 { u32 n[9]; };

#define F29_M 0x1FFFFFFFu
#define F29_R0 31264u      // 2^261 == 2^37 + 31264 (mod p): low part, limb 0
#define F29_R1 256u        // 2^37 = 256 * 2^29: limb 1
#define F29_RH1 250112u    // 2^293 == 2^69 + 31264 * 2^32: 31264 * 8 into limb 1
#define F29_RH2 2048u      // 2^69 = 2^11 * 2^58: limb 2

// a * b + c.  The empty asm is a value barrier: left to itself the compiler
// re-associates the column chains (each column summed from zero, then the
// carries added with extra 64-bit adds) and strength-reduces the fold
// constants into 64-bit shifts.
// F29_BARRIER 0 drops it (A/B builds).
#ifndef F29_BARRIER
#define F29_BARRIER 1
#endif
GV_DEV u64 f29_mad(u32 a, u32 b, u64 c) {
#if defined(__HIP_DEVICE_COMPILE__)
  u64 r = (u64)a * b + c;
#if F29_BARRIER
  asm("" : "+v"(r));              // value barrier: keeps the chain order
#endif
  return r;
#else
#if defined(GV_F29_CHECK)
  unsigned __int128 x = (unsigned __int128)a * b + c;
  F29_TRAP((x >> 64) != 0, "mad");
#endif
  return (u64)a * b + c;
#endif
}
GV_DEV u32 f29_add32(u32 a, u32 b) {
  F29_TRAP((u64)a + b > 0xFFFFFFFFull, "add32");
  return a + b;
}

// ---------------------------------------------------------------- products

// Product engine shared by mul and sqr.  Each column is ONE v_mad_u64_u32
// chain that starts from the previous column's carry; the column's low 29 bits
// are kept and the chain shifted by 29.  A mad consuming the previous mad's
// 64-bit result needs a wait state on gfx950 (hipcc inserts s_nop 0), but with
// several waves per SIMD those slots are filled by other waves: measured on
// MI355X (tools/microbench/fe29_rate.hip) one chain beats two interleaved
// chains joined by a 64-bit add.  Squares use doubled cross-term operands.
template <bool SQR>
GV_DEV int f29_col_hi(int k) { return SQR ? (k >> 1) : (k < 9 ? k : 8); }

// NCH = 1: one chain per column (throughput kernels).  NCH = 2: even and odd
// terms on two interleaved chains joined by one 64-bit add per column -- more
// instructions, but a single wave on a SIMD (the small-batch latency kernels)
// no longer waits on every mad's predecessor.
template <bool SQR, int NCH>
GV_DEV void f29_mulsqr(fe29& r, const fe29& a, const fe29& b) {
  u32 kr0 = F29_R0, kr1 = F29_R1;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(kr0), "+v"(kr1));     // keep the fold constants as mad operands
#endif
  u32 d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = SQR ? (a.n[i] << 1) : 0u;
#define F29_X(i, j) (SQR ? ((i) == (j) ? a.n[i] : d[i]) : a.n[i])
#define F29_Y(i, j) (SQR ? a.n[j] : b.n[j])
#define F29_TERM(x, y)                                   \
  do {                                                   \
    if (NCH == 2 && (idx & 1)) cb = f29_mad(x, y, cb);    \
    else ca = f29_mad(x, y, ca);                          \
    ++idx;                                               \
  } while (0)
  u32 t[9];
  u64 acc = 0;
#pragma unroll
  for (int k = 9; k <= 16; ++k) {             // high columns, carry chained
    u64 ca = acc, cb = 0;
    int idx = 0;
#pragma unroll
    for (int i = k - 8; i <= f29_col_hi<SQR>(k); ++i) F29_TERM(F29_X(i, k - i), F29_Y(i, k - i));
    acc = (NCH == 2 && idx > 1) ? ca + cb : ca;
    t[k - 9] = (u32)acc & F29_M;
    acc >>= 29;
  }
  F29_TRAP((acc >> 32) != 0, "mul t17");
  t[8] = (u32)acc;                            // limb 17
  fe29 o;
  acc = 0;                                    // the carry out of column 8 into 9 is
#pragma unroll                                // NOT added above: it re-enters below
  for (int j = 0; j <= 8; ++j) {              // as part of the 2^261 fold
    u64 ca = acc, cb = 0;
    int idx = 0;
#pragma unroll
    for (int i = 0; i <= f29_col_hi<SQR>(j); ++i) F29_TERM(F29_X(i, j - i), F29_Y(i, j - i));
    F29_TERM(t[j], kr0);
    if (j >= 1) F29_TERM(t[j - 1], kr1);
    acc = (NCH == 2 && idx > 1) ? ca + cb : ca;
    o.n[j] = (u32)acc & F29_M;
    acc >>= 29;
  }
#undef F29_TERM
#undef F29_X
#undef F29_Y
  acc = f29_mad(t[8], kr1, acc);              // 256 * limb 17 -> weight 2^261
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


// S independent products in lockstep (stream s: SQ[s] ? a[s]^2 : a[s]*b[s]),
// each stream exactly the column engine above (one chain per column), with
// the streams' terms interleaved: a wave running alone on a SIMD (the latency
// kernel) always has S independent mad chains in flight, while the
// throughput kernels issue the same instructions as S separate calls.
// r may alias a or b (outputs are written last).
#define F29M_X(s, i, j) (sq[s] ? ((i) == (j) ? a[s].n[i] : d[s][i]) : a[s].n[i])
#define F29M_Y(s, i, j) (sq[s] ? a[s].n[j] : b[s].n[j])
template <bool... SQ>
GV_DEV void f29_multi(fe29* r, const fe29* a, const fe29* b) {
  constexpr int S = sizeof...(SQ);
  constexpr bool sq[S] = {SQ...};
  u32 kr0 = F29_R0, kr1 = F29_R1;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(kr0), "+v"(kr1));
#endif
  u32 d[S][9];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int i = 0; i < 9; ++i) d[s][i] = sq[s] ? (a[s].n[i] << 1) : 0u;
  u32 t[S][9];
  u64 acc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) acc[s] = 0;
#pragma unroll
  for (int k = 9; k <= 16; ++k) {
#pragma unroll
    for (int q = 0; q < 9; ++q) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int i = k - 8 + q;
        if (i <= (sq[s] ? (k >> 1) : 8)) acc[s] = f29_mad(F29M_X(s, i, k - i), F29M_Y(s, i, k - i), acc[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      t[s][k - 9] = (u32)acc[s] & F29_M;
      acc[s] >>= 29;
    }
  }
  fe29 o[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    F29_TRAP((acc[s] >> 32) != 0, "multi t17");
    t[s][8] = (u32)acc[s];
    acc[s] = 0;
  }
#pragma unroll
  for (int j = 0; j <= 8; ++j) {
#pragma unroll
    for (int q = 0; q <= 8; ++q) {
#pragma unroll
      for (int s = 0; s < S; ++s)
        if (q <= (sq[s] ? (j >> 1) : j)) acc[s] = f29_mad(F29M_X(s, q, j - q), F29M_Y(s, q, j - q), acc[s]);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) acc[s] = f29_mad(t[s][j], kr0, acc[s]);
    if (j >= 1) {
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s] = f29_mad(t[s][j - 1], kr1, acc[s]);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      o[s].n[j] = (u32)acc[s] & F29_M;
      acc[s] >>= 29;
    }
  }
  u32 clo[S], chi[S];
  u64 x[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    acc[s] = f29_mad(t[s][8], kr1, acc[s]);
    clo[s] = (u32)acc[s];
    chi[s] = (u32)(acc[s] >> 32);
  }
#pragma unroll
  for (int s = 0; s < S; ++s) x[s] = f29_mad(clo[s], kr0, (u64)o[s].n[0]);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    o[s].n[0] = (u32)x[s] & F29_M;
    x[s] = (x[s] >> 29) + o[s].n[1];
  }
#pragma unroll
  for (int s = 0; s < S; ++s) x[s] = f29_mad(clo[s], kr1, x[s]);
#pragma unroll
  for (int s = 0; s < S; ++s) x[s] = f29_mad(chi[s], F29_RH1, x[s]);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    o[s].n[1] = (u32)x[s] & F29_M;
    o[s].n[2] = f29_add32(o[s].n[2], f29_add32((u32)(x[s] >> 29), chi[s] * F29_RH2));
  }
#pragma unroll
  for (int s = 0; s < S; ++s) r[s] = o[s];
}
#undef F29M_X
#undef F29M_Y

// ------------------------------------------------------------ linear ops
GV_DEV void f29_set_u32(fe29& r, u32 x) {
  r.n[0] = x & F29_M;
  r.n[1] = x >> 29;
#pragma unroll
  for (int i = 2; i < 9; ++i) r.n[i] = 0;
}
GV_DEV void f29_set_zero(fe29& r) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.n[i] = 0;
}

GV_DEV void f29_add(fe29& r, const fe29& a, const fe29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.n[i] = f29_add32(a.n[i], b.n[i]);
}

// r = a * k for a small k (magnitude * k), no carries
GV_DEV void f29_mul_int(fe29& r, const fe29& a, u32 k) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    F29_TRAP((u64)a.n[i] * k > 0xFFFFFFFFull, "mul_int");
    r.n[i] = a.n[i] * k;
  }
}

// Multiples of p with every limb >= m * F29_B (so K_m - b >= 0 limb-wise for
// mag(b) <= m) and < (m + 1) * F29_B: generated by tools/gen_fe29_consts.py.
#include "secp_fe29_consts.inc"

// r = K_mb - b  (mag(b) <= mb; result magnitude mb + 1)
template <int MB>
GV_DEV void f29_neg(fe29& r, const fe29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    F29_TRAP(b.n[i] > f29_kneg(MB, i), "neg");
    r.n[i] = f29_kneg(MB, i) - b.n[i];
  }
}

// r = a + K_mb - b  (magnitude mag(a) + mb + 1)
template <int MB>
GV_DEV void f29_sub(fe29& r, const fe29& a, const fe29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    F29_TRAP(b.n[i] > f29_kneg(MB, i), "sub");
    r.n[i] = f29_add32(a.n[i], f29_kneg(MB, i) - b.n[i]);
  }
}

// Carry pass: input magnitude <= 7 -> magnitude 1.  The carry out of limb 8
// (weight 2^261, <= 7) re-enters as 31264 c (limb 0) + 256 c (limb 1).
GV_DEV void f29_norm(fe29& r, const fe29& a) {
  u32 c = 0;
  fe29 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const u32 x = f29_add32(a.n[i], c);
    o.n[i] = x & F29_M;
    c = x >> 29;
  }
  o.n[0] += c * F29_R0;
  o.n[1] += c * F29_R1;
  r = o;
}

// r = norm(a + K_mb - b): the subtraction fused into the carry pass
// (mag(a) + MB + 1 <= 7) -> magnitude 1.
template <int MB>
GV_DEV void f29_sub_norm(fe29& r, const fe29& a, const fe29& b) {
  u32 c = 0;
  fe29 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    F29_TRAP(b.n[i] > f29_kneg(MB, i), "sub_norm");
    const u32 x = f29_add32(f29_add32(a.n[i], f29_kneg(MB, i) - b.n[i]), c);
    o.n[i] = x & F29_M;
    c = x >> 29;
  }
  o.n[0] += c * F29_R0;
  o.n[1] += c * F29_R1;
  r = o;
}

// r = norm(3 a), mag(a) <= 2 -> magnitude 1.
GV_DEV void f29_mul3_norm(fe29& r, const fe29& a) {
  u32 c = 0;
  fe29 o;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const u32 x = f29_add32(f29_add32(a.n[i], f29_add32(a.n[i], a.n[i])), c);
    o.n[i] = x & F29_M;
    c = x >> 29;
  }
  o.n[0] += c * F29_R0;
  o.n[1] += c * F29_R1;
  r = o;
}

// r = a * 2^S, carried (a magnitude 1 with every limb < 2^29 + 2^18, S <= 3):
// magnitude 1.  Limb i keeps the low 29 - S bits of a_i shifted up and takes
// the top S bits of a_(i-1).
template <int S>
GV_DEV void f29_shl_norm(fe29& r, const fe29& a) {
  fe29 o;
  u32 prev = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    o.n[i] = ((a.n[i] << S) & F29_M) + prev;
    prev = a.n[i] >> (29 - S);
  }
  o.n[0] += prev * F29_R0;
  o.n[1] += prev * F29_R1;
  r = o;
}

// ------------------------------------------------------- canonical form
// Canonical value in [0, p) as 8 x 32 little-endian words.  Input magnitude
// <= 7.
GV_DEV void f29_to_words(u32 w[8], const fe29& a0) {
  fe29 a;
  f29_norm(a, a0);
  f29_norm(a, a);                 // all limbs < 2^29: value < 2^261
  // fold bits >= 256 (limb 8 bits >= 24) twice: 2^256 == 2^32 + 977
#pragma unroll
  for (int rep = 0; rep < 2; ++rep) {
    const u32 h = a.n[8] >> 24;
    a.n[8] &= 0xFFFFFFu;
    u32 c;
    u32 x = a.n[0] + h * 977u;
    a.n[0] = x & F29_M; c = x >> 29;
    x = a.n[1] + (h << 3) + c;
    a.n[1] = x & F29_M; c = x >> 29;
#pragma unroll
    for (int i = 2; i < 9; ++i) { x = a.n[i] + c; a.n[i] = x & F29_M; c = x >> 29; }
  }
  // now value < 2^256: pack
  u32 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int b = 32 * k, i = b / 29, s = b % 29;
    u64 x = ((u64)a.n[i] >> s);
    if (i + 1 < 9) x |= (u64)a.n[i + 1] << (29 - s);
    if (i + 2 < 9 && (58 - s) < 32) x |= (u64)a.n[i + 2] << (58 - s);
    v[k] = (u32)x;
  }
  // subtract p once if v >= p: v + (2^32 + 977) carries out of 2^256 iff v >= p
  u32 t[8];
  u64 c = (u64)v[0] + 977u; t[0] = (u32)c; c >>= 32;
  c += (u64)v[1] + 1u; t[1] = (u32)c; c >>= 32;
#pragma unroll
  for (int i = 2; i < 8; ++i) { c += v[i]; t[i] = (u32)c; c >>= 32; }
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = c ? t[i] : v[i];
}

// 8 x 32 little-endian words (any value < 2^256) -> magnitude 1
GV_DEV void f29_from_words(fe29& r, const u32 w[8]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = 29 * i, k = b / 32, s = b % 32;
    u64 x = (u64)w[k] >> s;
    if (k + 1 < 8) x |= (u64)w[k + 1] << (32 - s);
    r.n[i] = (u32)x & F29_M;
  }
}

// a == 0 (mod p); input magnitude <= 7
GV_DEV bool f29_is_zero(const fe29& a) {
  u32 w[8];
  f29_to_words(w, a);
  u32 z = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) z |= w[i];
  return z == 0;
}

}  // namespace gv

#ifndef F29_NCH
#define F29_NCH 1
#endif
namespace gv {
// r = a * b mod p (magnitude 1).  mag(a) * mag(b) <= 6.  r may alias a or b.
// (The fused core of secp_fe29x.cuh is slower for plain products: k_prep
// 2.09 -> 2.20 ms per 1M in a same-box A/B, profiles/r02/ab_classic.)
GV_DEV void f29_mul(fe29& r, const fe29& a, const fe29& b) { f29_mulsqr<false, F29_NCH>(r, a, b); }
// r = a^2 mod p (magnitude 1).  mag(a) <= 2.  r may alias a.
GV_DEV void f29_sqr(fe29& r, const fe29& a) { f29_mulsqr<true, F29_NCH>(r, a, a); }
}  // namespace gv
