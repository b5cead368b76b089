// ed_fsl.cuh -- the limb-sliced field layer of the small-batch kernels
// (secp_fsl.cuh: one element per 16-lane DPP row, limb i of the 9 x 29 form in
// lane i) for GF(2^255 - 19), and the edwards25519 operations the sliced
// ed25519 verifier needs (ed_lat.hip).
//
// The product columns and the three reduction steps are secp_fsl.cuh's; only
// the per-lane fold constants differ (2^261 == 2^6 * 19 = 1216 mod p):
//   column c + 9 (c <= 6) -> limb c   x 1216        (k9)
//   column 16 -> limb 7 x 1216, column 17 -> limb 8 x 1216 (k16, k17)
//   column 18 -> limb 0 x 1216^2 = 1478656           (k18)
//   carry out of limb 8 -> limb 0 x 1216             (kc)
// so efsl_consts() fills the secp layer's fslk and fsl_mul / fsl_mul_plus /
// fsl_mul2 / fsl_norm / fsl_sqr_n run unchanged.  Bounds are the secp
// layer's: outputs in N-form (every limb < 2^29 + 2^17), products need
// max_limb(a) * max_limb(b) < 2^60.8.
//   BIAS = 128 p: limbs 2^30 - 2432, 2^30 - 2 (x 8); BIG8 = 8 BIAS.
#pragma once
#include "secp_fsl.cuh"
#include "ed_group.cuh"

namespace gv {
namespace ed {

GV_DEV fslk efsl_consts() {
  fslk k;
  const u32 L = __lane_id() & 15u;
  k.L = L;
  const bool lo = L <= 8u;
  k.m29 = lo ? F29_M : 0u;
  k.mw = lo ? 0xFFFFFFFFu : 0u;
  k.m29lo = L < 8u ? F29_M : (L == 8u ? 0xFFFFFFFFu : 0u);
  k.k9 = lo ? 1216u : 0u;                 // lanes 7, 8 read columns 16, 17 through shl:9 = 0 (out of row)
  k.k8 = 0u;
  k.k16 = L == 7u ? 1216u : 0u;
  k.k17 = L == 8u ? 1216u : 0u;
  k.k18 = L == 0u ? 1478656u : 0u;
  k.kc = L == 0u ? 1216u : 0u;
  k.bias = !lo ? 0u : (L == 0u ? 0x3ffff680u : 0x3ffffffeu);
  k.big8 = (u64)k.bias << 3;
  return k;
}

// 9-limb constant (one-lane layout) -> sliced
GV_DEV u32 efsl_const(const u32* c, const fslk& k) { return k.L < 9u ? c[k.L] : 0u; }
GV_DEV u32 efsl_small(u32 v, const fslk& k) { return k.L == 0u ? v : 0u; }
// canonical 8 x 32 words of the row's element (every lane of the row)
GV_DEV void efsl_to_words(u32 w[8], u32 a) {
  fe29 t;
  fsl_gather(t, a);
  e29_to_words(w, t);
}
GV_DEV bool efsl_is_zero(u32 a) {
  u32 w[8];
  efsl_to_words(w, a);
  u32 z = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) z |= w[i];
  return z == 0;
}
// FeFromBytes of 8 little-endian words (bit 255 dropped) -> sliced
GV_DEV u32 efsl_from_words(const u32 w[8], const fslk& k) {
  fe29 t;
  e29_from_words(t, w);
  return fsl_scatter(t, k);
}
// z^((p - 5) / 8) = z^(2^252 - 3): e29_pow22523's chain
GV_DEV u32 efsl_pow22523(u32 z, const fslk& k) {
  u32 t0 = fsl_sqr(z, k);                           // z^2
  u32 t1 = fsl_sqr_n(t0, 2, k);                     // z^8
  t1 = fsl_mul(z, t1, k);                           // z^9
  const u32 z11 = fsl_mul(t0, t1, k);
  t0 = fsl_sqr(z11, k);                             // z^22
  t0 = fsl_mul(t1, t0, k);                          // 2^5 - 1
  t1 = fsl_sqr_n(t0, 5, k);
  t0 = fsl_mul(t1, t0, k);                          // 2^10 - 1
  t1 = fsl_sqr_n(t0, 10, k);
  t1 = fsl_mul(t1, t0, k);                          // 2^20 - 1
  u32 t2 = fsl_sqr_n(t1, 20, k);
  t1 = fsl_mul(t2, t1, k);                          // 2^40 - 1
  t1 = fsl_sqr_n(t1, 10, k);
  t0 = fsl_mul(t1, t0, k);                          // 2^50 - 1
  t1 = fsl_sqr_n(t0, 50, k);
  t1 = fsl_mul(t1, t0, k);                          // 2^100 - 1
  t2 = fsl_sqr_n(t1, 100, k);
  t1 = fsl_mul(t2, t1, k);                          // 2^200 - 1
  t1 = fsl_sqr_n(t1, 50, k);
  t0 = fsl_mul(t1, t0, k);                          // 2^250 - 1
  t0 = fsl_sqr_n(t0, 2, k);                         // 2^252 - 4
  return fsl_mul(t0, z, k);                         // 2^252 - 3
}

// The point whose encoding is exactly these 32 bytes, if there is one:
// R' = [h](-A) + [s]B encodes (ToBytes: canonical y, parity of canonical x in
// bit 255) to rw iff R' == (x, y) for the (x, y) returned here, so the
// verifier compares projectively instead of inverting Z'.  No point encodes to
// bytes whose y is >= p, whose y has no x on the curve, or that set the sign
// bit of x = 0.
GV_DEV bool efsl_decode_strict(u32& x, u32& y, const u32 rw[8], const fslk& k) {
  bool canon_y = true;                              // y < p
  {
    bool top = (rw[7] & 0x7FFFFFFFu) == 0x7FFFFFFFu;
#pragma unroll
    for (int i = 1; i < 7; ++i) top = top && rw[i] == 0xFFFFFFFFu;
    canon_y = !(top && rw[0] >= 0xFFFFFFEDu);
  }
  const u32 sign = rw[7] >> 31;
  y = efsl_from_words(rw, k);
  const u32 one = efsl_small(1u, k);
  const u32 yy = fsl_sqr(y, k);
  const u32 u = fsl_norm(yy + k.bias - one, k);                 // y^2 - 1
  const u32 v = fsl_norm(fsl_mul(yy, efsl_const(kEdD, k), k) + one, k);   // d y^2 + 1
  const u32 v3 = fsl_mul(fsl_sqr(v, k), v, k);
  u32 t = fsl_mul(fsl_sqr(v3, k), v, k);                        // v^7
  t = fsl_mul(t, u, k);                                         // u v^7
  t = efsl_pow22523(t, k);
  t = fsl_mul(t, v3, k);
  x = fsl_mul(t, u, k);                                         // u v^3 (u v^7)^((p-5)/8)
  const u32 vxx = fsl_mul(fsl_sqr(x, k), v, k);
  const bool root = efsl_is_zero(vxx + k.bias - u);
  const bool neg_root = efsl_is_zero(vxx + u);
  if (!root) x = fsl_mul(x, efsl_const(kEdSqrtM1, k), k);
  u32 xw[8];
  efsl_to_words(xw, x);
  u32 xz = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) xz |= xw[i];
  if ((xw[0] & 1u) != sign) x = fsl_norm(k.bias - x, k);
  return canon_y && (root || neg_root) && !(xz == 0u && sign);
}

// ---------------------------------------------------------------- group law
// Extended coordinates (x = X/Z, y = Y/Z, xy = T/Z), one point per row.
struct gesl { u32 X, Y, Z, T; };

GV_DEV void gesl_identity(gesl& r, const fslk& k) {
  r.X = 0u;
  r.Y = efsl_small(1u, k);
  r.Z = efsl_small(1u, k);
  r.T = 0u;
}

// r = p + (neg ? -q : q), q in cached form (Y+X, Y-X, 2Z, 2dT), the
// complete a = -1 addition (ge_add_cached's formula).  qa / qb limbs <= 2N.
GV_DEV void gesl_add_cached(gesl& r, const gesl& p, u32 ypx, u32 ymx, u32 z2, u32 t2d, bool neg, const fslk& k) {
  const u32 qa = neg ? ymx : ypx, qb = neg ? ypx : ymx;
  const u32 a = fsl_mul(p.Y + p.X, qa, k);                      // 2N x 2N
  const u32 b = fsl_mul(p.Y + k.bias - p.X, qb, k);             // (N + BIAS) x 2N
  const u32 c = fsl_mul(t2d, p.T, k);
  const u32 d = fsl_mul(p.Z, z2, k);
  const u32 x1 = fsl_norm(a + k.bias - b, k);                   // A - B
  const u32 y1 = a + b;                                         // A + B      (2N)
  const u32 dpc = d + c;                                        //            (2N)
  const u32 dmc = fsl_norm(d + k.bias - c, k);
  const u32 z1 = neg ? dmc : dpc, t1 = neg ? dpc : dmc;
  r.X = fsl_mul(x1, t1, k);
  r.Y = fsl_mul(y1, z1, k);
  r.Z = fsl_mul(z1, t1, k);
  r.T = fsl_mul(x1, y1, k);
}

// r = p + (neg ? -q : q), q affine precomputed (y+x, y-x, 2dxy) (ge_add_pre).
GV_DEV void gesl_add_pre(gesl& r, const gesl& p, u32 ypx, u32 ymx, u32 xy2d, bool neg, const fslk& k) {
  const u32 qa = neg ? ymx : ypx, qb = neg ? ypx : ymx;
  const u32 a = fsl_mul(p.Y + p.X, qa, k);
  const u32 b = fsl_mul(p.Y + k.bias - p.X, qb, k);
  const u32 c = fsl_mul(xy2d, p.T, k);
  const u32 d = p.Z << 1;                                       // 2 Z1       (2N)
  const u32 x1 = fsl_norm(a + k.bias - b, k);
  const u32 y1 = a + b;                                         //            (2N)
  const u32 dpc = d + c;                                        //            (3N)
  const u32 dmc = fsl_norm(d + k.bias - c, k);
  const u32 z1 = neg ? dmc : dpc, t1 = neg ? dpc : dmc;
  r.X = fsl_mul(x1, t1, k);                                     // N x 3N
  r.Y = fsl_mul(y1, z1, k);                                     // 2N x 3N
  r.Z = fsl_mul(z1, t1, k);
  r.T = fsl_mul(x1, y1, k);
}

// r = p + q, both extended (q moved to cached form first).  d2 = 2d sliced.
GV_DEV void gesl_add(gesl& r, const gesl& p, const gesl& q, u32 d2, const fslk& k) {
  const u32 ypx = q.Y + q.X;                                    // 2N
  const u32 ymx = fsl_norm(q.Y + k.bias - q.X, k);
  const u32 z2 = q.Z << 1;                                      // 2N
  const u32 t2d = fsl_mul(q.T, d2, k);
  gesl_add_cached(r, p, ypx, ymx, z2, t2d, false, k);
}

// The row's point from the row of another lane group (shuffle by xor m).
GV_DEV gesl gesl_shfl_xor(const gesl& a, int m) {
  gesl o;
  o.X = (u32)__shfl_xor((int)a.X, m, 64);
  o.Y = (u32)__shfl_xor((int)a.Y, m, 64);
  o.Z = (u32)__shfl_xor((int)a.Z, m, 64);
  o.T = (u32)__shfl_xor((int)a.T, m, 64);
  return o;
}

}  // namespace ed
}  // namespace gv
