// secp_field26.cuh -- secp256k1 base field in reduced radix: 10 limbs of 26
// bits (limb 9: 22 bits), one element per lane, with magnitude tracking.
//
// Why a second representation: on gfx950 a carry-propagating op
// (v_add_co/v_addc_co) issues at the same rate as v_mad_u64_u32, while plain
// 32-bit ops (and, shifts, adds) issue at twice that rate
// (profiles/r01/alu_rate_v2.jsonl).  With 26-bit limbs every column of a
// product is summed inside v_mad_u64_u32's 64-bit addend without any carry
// handling, and additions/subtractions are limb-wise plain adds.
//
// value = sum n[i] * 2^(26 i).  "Magnitude m": n[i] <= m * (2^26-1) for i < 9,
// n[9] <= m * (2^22-1).  Outputs of mul/sqr have magnitude 1.  Inputs of
// mul/sqr must have magnitude <= 16 (column sums then stay below 2^64).
// Linear ops add magnitudes; fe26_sub(a, b, mb) has magnitude ma + mb + 1.
// The magnitudes used by the group formulas are annotated at each call.
#pragma once
#include <stdint.h>
#ifndef GV_DEV
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GV_DEV __device__ __forceinline__
#else
#define GV_DEV static inline          // host build: tests/test_field26_host.py
#endif
#endif

namespace gv {

typedef uint32_t u32;
typedef uint64_t u64;

struct fe26 { u32 n[10]; };

#define GV_M26 0x3FFFFFFu
#define GV_M22 0x3FFFFFu

GV_DEV void fe26_set_u32(fe26& r, u32 x) {
  r.n[0] = x;
#pragma unroll
  for (int i = 1; i < 10; ++i) r.n[i] = 0;
}

// 8 x 32 little-endian words (any value < 2^256) -> 10 x 26, magnitude 1
GV_DEV void fe26_from_words(fe26& r, const u32 v[8]) {
  r.n[0] = v[0] & GV_M26;
  r.n[1] = ((v[0] >> 26) | (v[1] << 6)) & GV_M26;
  r.n[2] = ((v[1] >> 20) | (v[2] << 12)) & GV_M26;
  r.n[3] = ((v[2] >> 14) | (v[3] << 18)) & GV_M26;
  r.n[4] = ((v[3] >> 8) | (v[4] << 24)) & GV_M26;
  r.n[5] = (v[4] >> 2) & GV_M26;
  r.n[6] = ((v[4] >> 28) | (v[5] << 4)) & GV_M26;
  r.n[7] = ((v[5] >> 22) | (v[6] << 10)) & GV_M26;
  r.n[8] = ((v[6] >> 16) | (v[7] << 16)) & GV_M26;
  r.n[9] = v[7] >> 10;
}

// Carry-propagate to magnitude 1 (limbs 26/22 bits, limb 2 may hold +1).
// Input magnitude <= 32.
GV_DEV void fe26_normalize_weak(fe26& r) {
  u32 t = r.n[9] >> 22;
  r.n[9] &= GV_M22;
  u32 x = r.n[0] + t * 977u;
  u32 c;
  r.n[0] = x & GV_M26; c = x >> 26;
  x = r.n[1] + (t << 6) + c; r.n[1] = x & GV_M26; c = x >> 26;
#pragma unroll
  for (int i = 2; i < 9; ++i) { x = r.n[i] + c; r.n[i] = x & GV_M26; c = x >> 26; }
  r.n[9] += c;
}

// Canonical value in [0, p) as 8 x 32 little-endian words.  Magnitude <= 32.
GV_DEV void fe26_to_words(u32 v[8], const fe26& a0) {
  fe26 a = a0;
  fe26_normalize_weak(a);
  fe26_normalize_weak(a);   // now n[9] <= 2^22 - 1: value < 2^256
  u32* r = v;
  r[0] = a.n[0] | (a.n[1] << 26);
  r[1] = (a.n[1] >> 6) | (a.n[2] << 20);
  r[2] = (a.n[2] >> 12) | (a.n[3] << 14);
  r[3] = (a.n[3] >> 18) | (a.n[4] << 8);
  r[4] = (a.n[4] >> 24) | (a.n[5] << 2) | (a.n[6] << 28);
  r[5] = (a.n[6] >> 4) | (a.n[7] << 22);
  r[6] = (a.n[7] >> 10) | (a.n[8] << 16);
  r[7] = (a.n[8] >> 16) | (a.n[9] << 10);
  // subtract p once if r >= p:  r + (2^32 + 977) carries out of 2^256 iff r >= p
  u32 t[8];
  u64 c = (u64)r[0] + 977u; t[0] = (u32)c; c >>= 32;
  c += (u64)r[1] + 1u; t[1] = (u32)c; c >>= 32;
#pragma unroll
  for (int i = 2; i < 8; ++i) { c += r[i]; t[i] = (u32)c; c >>= 32; }
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = c ? t[i] : r[i];
}

// r = a * b mod p.  Inputs magnitude <= 16, output magnitude 1.
// Pass 1: 19 product columns, each summed in a 64-bit mad chain that starts
// from the previous column's carry; 26 low bits kept.  Pass 2: fold limbs
// 10..19 with 2^260 == 2^36 + 0x3D10 (mod p) and carry again.
GV_DEV void fe26_mul(fe26& r, const fe26& a, const fe26& b) {
  u32 t[20];
  u64 c = 0;
#pragma unroll
  for (int k = 0; k < 19; ++k) {
    u64 acc = c;
#pragma unroll
    for (int i = (k < 10 ? 0 : k - 9); i <= (k < 10 ? k : 9); ++i) acc += (u64)a.n[i] * b.n[k - i];
    t[k] = (u32)acc & GV_M26;
    c = acc >> 26;
  }
  t[19] = (u32)c;
  c = 0;
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    u64 acc = c + t[j];
    acc += (u64)t[j + 10] * 0x3D10u;
    if (j >= 1) acc += (u64)t[j + 9] << 10;
    if (j == 0) acc += (u64)t[19] * 0xF44000u;
    if (j == 1) acc += (u64)t[19] << 20;
    if (j < 9) { r.n[j] = (u32)acc & GV_M26; c = acc >> 26; }
    else       { r.n[9] = (u32)acc & GV_M22; c = acc >> 22; }
  }
  // c * 2^256 == c * (2^32 + 977)
  const u32 cc = (u32)c;
  u64 x = (u64)r.n[0] + (u64)cc * 977u;
  r.n[0] = (u32)x & GV_M26;
  u32 y = r.n[1] + (cc << 6) + (u32)(x >> 26);
  r.n[1] = y & GV_M26;
  r.n[2] += y >> 26;
}

GV_DEV void fe26_sqr(fe26& r, const fe26& a) {
  u32 d[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) d[i] = a.n[i] << 1;
  u32 t[20];
  u64 c = 0;
#pragma unroll
  for (int k = 0; k < 19; ++k) {
    u64 acc = c;
    const int lo = (k < 10 ? 0 : k - 9), hi = (k < 10 ? k : 9);
#pragma unroll
    for (int i = lo; i <= hi; ++i) {
      const int j = k - i;
      if (i < j) acc += (u64)d[i] * a.n[j];
      else if (i == j) acc += (u64)a.n[i] * a.n[i];
    }
    t[k] = (u32)acc & GV_M26;
    c = acc >> 26;
  }
  t[19] = (u32)c;
  c = 0;
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    u64 acc = c + t[j];
    acc += (u64)t[j + 10] * 0x3D10u;
    if (j >= 1) acc += (u64)t[j + 9] << 10;
    if (j == 0) acc += (u64)t[19] * 0xF44000u;
    if (j == 1) acc += (u64)t[19] << 20;
    if (j < 9) { r.n[j] = (u32)acc & GV_M26; c = acc >> 26; }
    else       { r.n[9] = (u32)acc & GV_M22; c = acc >> 22; }
  }
  const u32 cc = (u32)c;
  u64 x = (u64)r.n[0] + (u64)cc * 977u;
  r.n[0] = (u32)x & GV_M26;
  u32 y = r.n[1] + (cc << 6) + (u32)(x >> 26);
  r.n[1] = y & GV_M26;
  r.n[2] += y >> 26;
}

GV_DEV void fe26_add(fe26& r, const fe26& a, const fe26& b) {
#pragma unroll
  for (int i = 0; i < 10; ++i) r.n[i] = a.n[i] + b.n[i];
}

// r = a * k (small k; magnitude * k)
GV_DEV void fe26_mul_int(fe26& r, const fe26& a, u32 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) r.n[i] = a.n[i] * k;
}

// r = (mb + 1) * p - b  (b magnitude <= mb), magnitude mb + 1
GV_DEV void fe26_neg(fe26& r, const fe26& b, u32 mb) {
  const u32 k = mb + 1;
  r.n[0] = 0x3FFFC2Fu * k - b.n[0];
  r.n[1] = 0x3FFFFBFu * k - b.n[1];
#pragma unroll
  for (int i = 2; i < 9; ++i) r.n[i] = GV_M26 * k - b.n[i];
  r.n[9] = GV_M22 * k - b.n[9];
}

// r = a - b (b magnitude <= mb): magnitude ma + mb + 1
GV_DEV void fe26_sub(fe26& r, const fe26& a, const fe26& b, u32 mb) {
  const u32 k = mb + 1;
  r.n[0] = a.n[0] + (0x3FFFC2Fu * k - b.n[0]);
  r.n[1] = a.n[1] + (0x3FFFFBFu * k - b.n[1]);
#pragma unroll
  for (int i = 2; i < 9; ++i) r.n[i] = a.n[i] + (GV_M26 * k - b.n[i]);
  r.n[9] = a.n[9] + (GV_M22 * k - b.n[9]);
}

// a == 0 (mod p); a magnitude <= 32
GV_DEV bool fe26_is_zero(const fe26& a0) {
  fe26 a = a0;
  fe26_normalize_weak(a);
  // now a < 2^256 + small; zero iff a == 0 or a == p
  u32 z0 = 0, z1 = 0;
  z0 = a.n[0] | a.n[1] | a.n[2] | a.n[3] | a.n[4] | a.n[5] | a.n[6] | a.n[7] | a.n[8] | a.n[9];
  z1 = (a.n[0] ^ 0x3FFFC2Fu) | (a.n[1] ^ 0x3FFFFBFu) | (a.n[2] ^ GV_M26) | (a.n[3] ^ GV_M26) | (a.n[4] ^ GV_M26) |
       (a.n[5] ^ GV_M26) | (a.n[6] ^ GV_M26) | (a.n[7] ^ GV_M26) | (a.n[8] ^ GV_M26) | (a.n[9] ^ GV_M22);
  return z0 == 0 || z1 == 0;
}

}  // namespace gv
