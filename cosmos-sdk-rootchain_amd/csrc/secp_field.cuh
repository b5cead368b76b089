// secp_field.cuh -- secp256k1 base-field arithmetic for gfx950 (CDNA4), one
// field element per lane, 8 x 32-bit little-endian limbs.
//
// p = 2^256 - 2^32 - 977.  Values are kept "weakly reduced": any 256-bit value
// congruent to the intended residue (i.e. in [0, 2^256)); fe_normalize() gives
// the canonical representative when a comparison needs it.
//
// Multiply, square, reduction, add and sub are hand-scheduled inline-asm
// blocks (see below).  Measured on MI355X, v_mad_u64_u32 issues at ~the same
// chip rate as plain 32-bit VALU ops (tools/microbench/alu_rate.hip), so
// instruction count, not multiply count, is what this layer minimises; every
// carry chain is kept back-to-back because hipcc pads a VCC read that is one
// instruction away from its writer with an s_nop.
//
// Reference semantics being accelerated: btcec/field.go (btcd v0.20.1-beta)
// via crypto/ecdsa.Verify; see SURVEY.md §2 "External: btcec".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gv {

typedef uint32_t u32;
typedef uint64_t u64;

#define GV_DEV __device__ __forceinline__

struct fe { u32 v[8]; };

// p limbs (little-endian)
#define GV_P0 0xFFFFFC2Fu
#define GV_P1 0xFFFFFFFEu

GV_DEV void fe_set_zero(fe& r) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = 0;
}
GV_DEV void fe_set_u32(fe& r, u32 x) { fe_set_zero(r); r.v[0] = x; }

// ---------------------------------------------------------------------------
// Hand-scheduled sequences (tools/gen_field_asm.py; validated on the CPU by an
// instruction-level model in tests/test_field_asm_model.py).  Scratch: v0..v3
// and VCC, declared clobbered.
//   mul: product scanning -- column k accumulates in a 64-bit pair with
//        v_mad_u64_u32; each mad's carry-out (VCC) is counted by v_addc_co_u32
//        into the high word of the next column's pair: 2 VALU ops per product.
//   sqr: the 28 cross products the same way, then one pass of v_alignbit
//        doubling and one carry chain adding the 8 diagonal squares.
//   reduce: t = L + H*2^256 == L + 977*H + (H << 32) as three back-to-back
//        carry chains, then two folds of the (at most 34-bit) top word.
#include "secp_field_asm.inc"

GV_DEV void mul_256x256(u32 t[16], const u32 a[8], const u32 b[8]) {
  GV_MUL512_ASM(t, a, b);
}

GV_DEV void sqr_256(u32 t[16], const u32 a[8]) {
  u32 c[16];
  u64 sq[8];
  GV_SQRX_ASM(c, a);
#pragma unroll
  for (int i = 0; i < 8; ++i) sq[i] = (u64)a[i] * a[i];
  GV_SQRF_ASM(t, c, sq);
}

// Reduce a 512-bit value modulo p to a weakly reduced 256-bit value.
GV_DEV void fe_reduce512(fe& r, const u32 t[16]) {
  u64 m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = (u64)t[8 + i] * 977u;
  u32 top, top2;
  GV_REDUCE_ASM(r.v, t, m, top, top2);
}

GV_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  u32 t[16];
  mul_256x256(t, a.v, b.v);
  fe_reduce512(r, t);
}
GV_DEV void fe_sqr(fe& r, const fe& a) {
  u32 t[16];
  sqr_256(t, a.v);
  fe_reduce512(r, t);
}

// r = a + b (mod p), weakly reduced: carry chain, then two folds of the carry
// (c * (2^32 + 977)); the second fold can only touch limbs 0..1.
GV_DEV void fe_add(fe& r, const fe& a, const fe& b) { GV_ADD_ASM(r.v, a.v, b.v); }

// r = a - b (mod p), weakly reduced: a borrow means the result wrapped to
// a - b + 2^256, so subtract 2^32 + 977 (== 2^256 - p), at most twice.
GV_DEV void fe_sub(fe& r, const fe& a, const fe& b) { GV_SUB_ASM(r.v, a.v, b.v); }

GV_DEV void fe_neg(fe& r, const fe& a) { fe z; fe_set_zero(z); fe_sub(r, z, a); }
GV_DEV void fe_dbl(fe& r, const fe& a) { GV_SHL1_ASM(r.v, a.v); }

// r = a * 2^S and r = a - b * 2^S (S = 1..3), r = 3a: limb shifts by
// v_alignbit and a single fold of the bits above 2^256 -- one sequence instead
// of S chained additions.  r must not alias the inputs' storage only as far as
// the asm's early-clobber outputs already guarantee (aliasing is fine in C).
template <int S> GV_DEV void fe_shl(fe& r, const fe& a) {
  static_assert(S >= 1 && S <= 3, "shift");
  if (S == 1) GV_SHL1_ASM(r.v, a.v);
  else if (S == 2) GV_SHL2_ASM(r.v, a.v);
  else GV_SHL3_ASM(r.v, a.v);
}
template <int S> GV_DEV void fe_sub_shl(fe& r, const fe& a, const fe& b) {
  static_assert(S >= 1 && S <= 3, "shift");
  if (S == 1) GV_SUBSHL1_ASM(r.v, a.v, b.v);
  else if (S == 2) GV_SUBSHL2_ASM(r.v, a.v, b.v);
  else GV_SUBSHL3_ASM(r.v, a.v, b.v);
}
GV_DEV void fe_mul3(fe& r, const fe& a) { GV_MUL3_ASM(r.v, a.v); }

// canonical representative in [0, p)
GV_DEV void fe_normalize(fe& r) {
  // t = r + (2^32 + 977); if that carries out, r >= p and r - p == t mod 2^256
  u32 t[8], c;
  t[0] = __builtin_addc(r.v[0], 977u, 0u, &c);
  t[1] = __builtin_addc(r.v[1], 1u, c, &c);
#pragma unroll
  for (int i = 2; i < 8; ++i) t[i] = __builtin_addc(r.v[i], 0u, c, &c);
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c ? t[i] : r.v[i];
}

GV_DEV bool fe_is_zero(const fe& a) {      // a == 0 (mod p)
  fe t = a; fe_normalize(t);
  u32 o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= t.v[i];
  return o == 0;
}
GV_DEV bool fe_equal(const fe& a, const fe& b) {
  fe d; fe_sub(d, a, b); return fe_is_zero(d);
}

// a^(2^k)
GV_DEV void fe_sqr_n(fe& r, const fe& a, int k) {
  r = a;
  for (int i = 0; i < k; ++i) fe_sqr(r, r);
}

// Shared prefix of the p-2 and (p+1)/4 addition chains: x223 = a^(2^223-1),
// plus the small blocks x2 = a^3, x22 = a^(2^22-1) used by both tails.
GV_DEV void fe_pow_prefix(fe& x2, fe& x22, fe& x223, const fe& a) {
  fe x3, x6, x9, x11, x44, x88, x176, x220, t;
  fe_sqr(x2, a); fe_mul(x2, x2, a);            // 2^2-1
  fe_sqr(x3, x2); fe_mul(x3, x3, a);           // 2^3-1
  fe_sqr_n(t, x3, 3); fe_mul(x6, t, x3);        // 2^6-1
  fe_sqr_n(t, x6, 3); fe_mul(x9, t, x3);        // 2^9-1
  fe_sqr_n(t, x9, 2); fe_mul(x11, t, x2);       // 2^11-1
  fe_sqr_n(t, x11, 11); fe_mul(x22, t, x11);    // 2^22-1
  fe_sqr_n(t, x22, 22); fe_mul(x44, t, x22);    // 2^44-1
  fe_sqr_n(t, x44, 44); fe_mul(x88, t, x44);    // 2^88-1
  fe_sqr_n(t, x88, 88); fe_mul(x176, t, x88);   // 2^176-1
  fe_sqr_n(t, x176, 44); fe_mul(x220, t, x44);  // 2^220-1
  fe_sqr_n(t, x220, 3); fe_mul(x223, t, x3);    // 2^223-1
}

// r = a^(p-2) = a^-1 (a != 0).  p-2 = (2^223-1)<<33 | 0 | (2^22-1)<<10 | 0000101101
GV_DEV void fe_inv(fe& r, const fe& a) {
  fe x2, x22, x223, t;
  fe_pow_prefix(x2, x22, x223, a);
  fe_sqr_n(t, x223, 23); fe_mul(t, t, x22);     // ...(2^223-1)<<23 + (2^22-1): bits 255..33 ones, bit 32 zero, bits 31..10 ones
  fe_sqr_n(t, t, 5); fe_mul(t, t, a);           // bits 9..5 = 00001
  fe_sqr_n(t, t, 3); fe_mul(t, t, x2);          // bits 4..2  = 011
  fe_sqr_n(t, t, 2); fe_mul(r, t, a);           // bits 1..0  = 01
}

// r = a^((p+1)/4); (p+1)/4 = (2^223-1)<<31 | 0 | (2^22-1)<<8 | 00001100
GV_DEV void fe_sqrt_candidate(fe& r, const fe& a) {
  fe x2, x22, x223, t;
  fe_pow_prefix(x2, x22, x223, a);
  fe_sqr_n(t, x223, 23); fe_mul(t, t, x22);     // bits 253..31 ones, bit 30 zero, 29..8 ones
  fe_sqr_n(t, t, 6); fe_mul(t, t, x2);          // bits 7..2 = 000011
  fe_sqr_n(r, t, 2);                            // bits 1..0 = 00
}

// big-endian 32-byte -> limbs
GV_DEV void fe_from_be_words(fe& r, const u32 w_be[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = w_be[7 - i];
}

}  // namespace gv
