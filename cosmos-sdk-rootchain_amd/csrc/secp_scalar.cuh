// secp_scalar.cuh -- arithmetic modulo the group order n on gfx950, one scalar
// per lane (8 x 32-bit limbs), plus the GLV split used by the double-scalar
// multiplication.
//
// Restates the scalar part of go1.14 crypto/ecdsa.verifyGeneric:
//   w = s^-1 mod n ; u1 = e*w mod n ; u2 = r*w mod n
// with the inversion batched across the wavefront (Montgomery's trick over the
// 64 lanes via DPP/permute prefix products: one Fermat inversion per wave).
#pragma once
#include "secp_field.cuh"

namespace gv {

__constant__ const u32 kN[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                                0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
__constant__ const u32 kHalfN[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                                    0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
// p - n (129 bits): R.x may equal r + n only when r < p - n
__constant__ const u32 kPminusN[8] = {0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u,
                                      0x00000001u, 0u, 0u, 0u};
// R^2 mod n (R = 2^256) for conversion into Montgomery form
__constant__ const u32 kR2modN[8] = {0x67D7D140u, 0x896CF214u, 0x0E7CF878u, 0x741496C2u,
                                     0x5BCD07C6u, 0xE697F5E4u, 0x81C69BC5u, 0x9D671CD5u};
#define GV_NPRIME 0x5588B13Fu   // -n^-1 mod 2^32

// GLV basis: a1 = b2 = A1, b1 = -B1, a2 = A2.
__constant__ const u32 kA1[4] = {0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
__constant__ const u32 kB1[4] = {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};
__constant__ const u32 kA2[5] = {0x9D44CFD8u, 0x57C1108Du, 0xA8E2F3F6u, 0x14CA50F7u, 0x00000001u};
// g1 = round(2^384 * A1 / n), g2 = round(2^384 * B1 / n)
__constant__ const u32 kG1[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u,
                                 0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
__constant__ const u32 kG2[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu,
                                 0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};

// a >= b (256-bit, little-endian limbs)
GV_DEV bool u256_geq(const u32 a[8], const u32* b) {
  u32 br = 0, d;
#pragma unroll
  for (int i = 0; i < 8; ++i) d = __builtin_subc(a[i], b[i], br, &br);
  (void)d;
  return br == 0;
}
GV_DEV bool u256_is_zero(const u32 a[8]) {
  u32 o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a[i];
  return o == 0;
}
// r = a - n if a >= n (a < 2n assumed)
GV_DEV void sc_reduce_once(u32 a[8]) {
  u32 t[8], br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = __builtin_subc(a[i], kN[i], br, &br);
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = br ? a[i] : t[i];
}

// Montgomery product r = a*b*2^-256 mod n (CIOS), inputs < n, output < n.
GV_DEV void sc_montmul(u32 r[8], const u32 a[8], const u32 b[8]) {
  u32 t[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u64 c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      c = (u64)a[i] * b[j] + t[j] + (c >> 32);
      t[j] = (u32)c;
    }
    c = (u64)t[8] + (c >> 32);
    t[8] = (u32)c;
    t[9] = (u32)(c >> 32);
    u32 m = t[0] * GV_NPRIME;
    c = (u64)m * kN[0] + t[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      c = (u64)m * kN[j] + t[j] + (c >> 32);
      t[j - 1] = (u32)c;
    }
    c = (u64)t[8] + (c >> 32);
    t[7] = (u32)c;
    t[8] = t[9] + (u32)(c >> 32);
  }
  // result < 2n: subtract n when t >= n
  u32 s[8], br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = __builtin_subc(t[i], kN[i], br, &br);
  bool ge = (t[8] != 0) || (br == 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = ge ? s[i] : t[i];
}

GV_DEV void sc_to_mont(u32 r[8], const u32 a[8]) {
  u32 r2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) r2[i] = kR2modN[i];
  sc_montmul(r, a, r2);
}

// r = a^(n-2) in the Montgomery domain (a = x*R -> r = x^-1 * R).
GV_DEV void sc_mont_inv(u32 r[8], const u32 a[8]) {
  // n - 2, most significant word first
  const u32 e[8] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFEu,
                    0xBAAEDCE6u, 0xAF48A03Bu, 0xBFD25E8Cu, 0xD036413Fu};
  u32 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = a[i];     // top bit of n-2 is 1
  for (int w = 0; w < 8; ++w) {
    u32 word = e[w];
    for (int b = (w == 0 ? 30 : 31); b >= 0; --b) {
      sc_montmul(acc, acc, acc);
      if ((word >> b) & 1u) sc_montmul(acc, acc, a);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = acc[i];
}

// ---- cross-lane helpers (wave64) ----
GV_DEV u32 lane_id() { return __lane_id(); }
GV_DEV u32 shfl_up_u32(u32 v, int d) { return (u32)__shfl_up((int)v, d, 64); }
GV_DEV u32 shfl_down_u32(u32 v, int d) { return (u32)__shfl_down((int)v, d, 64); }
GV_DEV u32 shfl_idx_u32(u32 v, int src) { return (u32)__shfl((int)v, src, 64); }

// Batch inversion across the wavefront: every lane holds a nonzero x (Montgomery
// form, < n); returns x^-1 (Montgomery form).  All 64 lanes must be active.
// Prefix/suffix products by Hillis-Steele scans (6 steps each) + one Fermat
// inversion shared by the wave: ~20 Montgomery products per lane instead of ~380.
GV_DEV void sc_batch_inv_wave(u32 inv[8], const u32 x[8]) {
  const u32 lane = lane_id();
  u32 pre[8], suf[8], t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { pre[i] = x[i]; suf[i] = x[i]; }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = shfl_up_u32(pre[i], d);
    u32 m[8];
    sc_montmul(m, pre, t);
#pragma unroll
    for (int i = 0; i < 8; ++i) pre[i] = (lane >= (u32)d) ? m[i] : pre[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = shfl_down_u32(suf[i], d);
    sc_montmul(m, suf, t);
#pragma unroll
    for (int i = 0; i < 8; ++i) suf[i] = (lane + (u32)d < 64u) ? m[i] : suf[i];
  }
  // total = pre[63]; every lane computes the same inversion
  u32 tot[8], tinv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) tot[i] = shfl_idx_u32(pre[i], 63);
  sc_mont_inv(tinv, tot);
  // exclusive prefix/suffix; Montgomery one = R mod n = 2^256 - n
  const u32 one_m[8] = {0x2FC9BEBFu, 0x402DA173u, 0x50B75FC4u, 0x45512319u, 1u, 0u, 0u, 0u};
  u32 pe[8], se[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u32 a = shfl_up_u32(pre[i], 1), b = shfl_down_u32(suf[i], 1);
    pe[i] = lane == 0 ? one_m[i] : a;
    se[i] = lane == 63 ? one_m[i] : b;
  }
  u32 m[8];
  sc_montmul(m, pe, se);
  sc_montmul(inv, m, tinv);
}

// ---- GLV split:  k == k1 + k2*lambda (mod n), |k1|,|k2| < 2^128 ----------
// c1 = round(k*g1 / 2^384), c2 = round(k*g2 / 2^384)
// k2 = c1*B1 - c2*A1 ; k1 = k - c1*A1 - c2*A2   (exact integers; the
// Babai bound keeps both below 2^128 in magnitude)
// Outputs: magnitudes (4 limbs) and sign flags (1 = negative).
GV_DEV void glv_round_shift384(u32 c[4], const u32 k[8], const u32* g) {
  u32 gg[8], t[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) gg[i] = g[i];
  mul_256x256(t, k, gg);
  // c = (t >> 384) + bit 383
  u32 rb = t[11] >> 31, cc;
  c[0] = __builtin_addc(t[12], rb, 0u, &cc);
  c[1] = __builtin_addc(t[13], 0u, cc, &cc);
  c[2] = __builtin_addc(t[14], 0u, cc, &cc);
  c[3] = __builtin_addc(t[15], 0u, cc, &cc);
}
// t(256, wrap) = a(4 limbs) * b(nb limbs), low 8 limbs
GV_DEV void mul_lo256(u32 r[8], const u32 a[4], const u32* b, int nb) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u64 c = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (j >= nb || i + j >= 8) continue;
      c = (u64)a[i] * b[j] + r[i + j] + (c >> 32);
      r[i + j] = (u32)c;
    }
    int k = i + nb;
    if (k < 8) r[k] = (u32)(c >> 32);
  }
}
GV_DEV void u256_sub_wrap(u32 r[8], const u32 a[8], const u32 b[8]) {
  u32 br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = __builtin_subc(a[i], b[i], br, &br);
}
// two's-complement 256-bit value -> (|v| low 4 limbs, sign)
GV_DEV void to_sign_mag128(u32 mag[4], u32& neg, const u32 v[8]) {
  neg = v[7] >> 31;
  u32 br = 0, t[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) t[i] = __builtin_subc(0u, v[i], br, &br);
#pragma unroll
  for (int i = 0; i < 4; ++i) mag[i] = neg ? t[i] : v[i];
}
GV_DEV void glv_split(u32 k1[4], u32& k1neg, u32 k2[4], u32& k2neg, const u32 k[8]) {
  u32 c1[4], c2[4];
  glv_round_shift384(c1, k, kG1);
  glv_round_shift384(c2, k, kG2);
  u32 a1[4], b1[4], a2[5];
#pragma unroll
  for (int i = 0; i < 4; ++i) { a1[i] = kA1[i]; b1[i] = kB1[i]; }
#pragma unroll
  for (int i = 0; i < 5; ++i) a2[i] = kA2[i];
  u32 p1[8], p2[8], v2[8], v1[8], tmp[8];
  mul_lo256(p1, c1, b1, 4);          // c1*B1
  mul_lo256(p2, c2, a1, 4);          // c2*A1
  u256_sub_wrap(v2, p1, p2);         // k2
  mul_lo256(p1, c1, a1, 4);          // c1*A1
  mul_lo256(p2, c2, a2, 5);          // c2*A2 (mod 2^256)
  u256_sub_wrap(tmp, k, p1);
  u256_sub_wrap(v1, tmp, p2);        // k1
  to_sign_mag128(k1, k1neg, v1);
  to_sign_mag128(k2, k2neg, v2);
}

// Signed fixed-window (Booth) digit of a 128-bit magnitude k at window `win`
// of width W: d = (bits [W*win-1 .. W*win+W-1]) recoded into [-2^(W-1), 2^(W-1)].
template <int W>
GV_DEV int booth_digit(const u32 k[4], int win) {
  const int p = W * win - 1;          // lowest bit position used (borrow bit)
  u32 v;
  if (p < 0) {
    v = (k[0] << 1) & ((1u << (W + 1)) - 1u);
  } else {
    const int limb = p >> 5, sh = p & 31;
    u32 lo = limb == 0 ? k[0] : limb == 1 ? k[1] : limb == 2 ? k[2] : limb == 3 ? k[3] : 0u;
    u32 hi = limb == 0 ? k[1] : limb == 1 ? k[2] : limb == 2 ? k[3] : 0u;
    u32 w = (u32)((((u64)hi << 32) | lo) >> sh);
    v = w & ((1u << (W + 1)) - 1u);
  }
  const int mag = (int)((v >> 1) & ((1u << (W - 1)) - 1u)) + (int)(v & 1u);
  return mag - (int)((v >> W) << (W - 1));
}

// The same recoding of a 256-bit k (8 words; win a compile-time constant
// after unrolling, so the limb selects fold away).  W <= 31.
template <int W>
GV_DEV int booth_digit8(const u32 k[8], int win) {
  const int p = W * win - 1;
  u32 v;
  if (p < 0) {
    v = (k[0] << 1) & ((1u << (W + 1)) - 1u);
  } else {
    const int limb = p >> 5, sh = p & 31;
    const u32 lo = limb < 8 ? k[limb] : 0u;
    const u32 hi = limb + 1 < 8 ? k[limb + 1] : 0u;
    v = (u32)((((u64)hi << 32) | lo) >> sh) & ((1u << (W + 1)) - 1u);
  }
  const int mag = (int)((v >> 1) & ((1u << (W - 1)) - 1u)) + (int)(v & 1u);
  return mag - (int)((v >> W) << (W - 1));
}

}  // namespace gv
