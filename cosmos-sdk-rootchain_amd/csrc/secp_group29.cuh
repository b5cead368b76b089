// secp_group29.cuh -- secp256k1 group law and exponentiation chains on the
// 9 x 29 field layer (secp_fe29.cuh), one point per lane.
//
// Same formulas and exceptional-case semantics as secp_group.cuh (the complete
// group law of btcec KoblitzCurve.Add / addJacobian / doubleJacobian, btcd
// v0.20.1-beta btcec/btcec.go: P == Q doubles, P == -Q gives infinity,
// infinity is the identity), restated with the magnitude budget of the 9 x 29
// layer annotated at every step (mag(x) after the step; mul needs
// mag(a) * mag(b) <= 6, sqr mag <= 2, linear results <= 7).
//
// Point invariant between operations: X and Y magnitude 1, Z magnitude <= 2.
#pragma once
#include "secp_fe29.cuh"

namespace gv {

struct gej29 { fe29 x, y, z; };

// GV_ILP: issue the independent field products of a formula in lockstep
// (f29_multi); same instruction count, more independent chains per wave.
#ifndef GV_ILP
#define GV_ILP 1
#endif

// a == 0 (mod p), any magnitude <= 7.  V = sum n_i 2^(29 i) < 2^264 is a
// multiple k*p (k < 256) only if V mod 2^29 = (-977 k) mod 2^29, i.e. the low
// limb (mod 2^29) is 0 or >= 2^29 - 977*256: every other lane answers "no"
// from that one test; the (rare) candidates take the canonical comparison.
GV_DEV bool f29_is_zero_fast(const fe29& a) {
  const u32 z = a.n[0] & F29_M;
  const bool cand = (z == 0u) | (z >= F29_M + 1u - 977u * 256u);
  bool res = false;
  if (cand) res = f29_is_zero(a);
  return res;
}

// a == b (mod p), canonical comparison (not on the ladder's hot path)
GV_DEV bool f29_equal(const fe29& a, const fe29& b) {
  u32 wa[8], wb[8];
  f29_to_words(wa, a);
  f29_to_words(wb, b);
  u32 d = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) d |= wa[i] ^ wb[i];
  return d == 0;
}

// r = 2a (a finite; secp256k1 has no point of order 2).  3M + 4S:
//   A = X^2, B = Y^2, C = B^2, D = X*B, E = 3A, F = E^2,
//   X3 = F - 8D, Y3 = E*(4D - X3) - 8C, Z3 = 2*Y*Z.
// GV_DBL25: 2M + 5S, the product X*B taken as ((X + B)^2 - A - C) / 2
// (a square is 45 + 9 multiplies against 81 for a product, for two extra
// linear steps).
// In: X 1, Y 1, Z <= 2.  Out: X 1, Y 1, Z 2.  r may alias a.
#ifndef GV_DBL25
#define GV_DBL25 0
#endif
GV_DEV void gej29_double(gej29& r, const gej29& a) {
  fe29 A, B, C, D, E, F, t, u;
#if GV_DBL25
  {
    fe29 o[3];
    const fe29 x[3] = {a.x, a.y, a.y}, y[3] = {a.x, a.y, a.z};
    f29_multi<true, true, false>(o, x, y);
    A = o[0]; B = o[1]; t = o[2];    // 1, 1, 1 (1 x 2)
  }
  f29_add(r.z, t, t);                // Z3 = 2YZ: 2      (a.y, a.z dead)
  f29_mul3_norm(E, A);               // E = 3A: 1
  f29_add(u, a.x, B);                // X + B: 2         (a.x dead)
  {
    fe29 o[3];
    const fe29 x[3] = {B, E, u};
    f29_multi<true, true, true>(o, x, x);
    C = o[0]; F = o[1]; D = o[2];    // B^2, E^2, (X + B)^2: 1
  }
  f29_sub<1>(D, D, A);               // 3
  f29_sub_norm<1>(D, D, C);          // 2XB: 1           (in 3 + 1 + 1)
  f29_shl_norm<1>(D, D);             // 4D: 1
#elif GV_ILP
  {                                  // {A, B, YZ} and {C, F, D}: independent triples in lockstep
    fe29 o[3];
    const fe29 x[3] = {a.x, a.y, a.y}, y[3] = {a.x, a.y, a.z};
    f29_multi<true, true, false>(o, x, y);
    A = o[0]; B = o[1]; t = o[2];    // 1, 1, 1 (1 x 2)
  }
  f29_add(r.z, t, t);                // Z3 = 2YZ: 2      (a.y, a.z dead)
  f29_mul3_norm(E, A);               // E = 3A: 1
  {
    fe29 o[3];
    const fe29 x[3] = {B, E, a.x}, y[3] = {B, E, B};
    f29_multi<true, true, false>(o, x, y);
    C = o[0]; F = o[1]; D = o[2];    // B^2, E^2, X*B: 1  (a.x dead)
  }
#else
  f29_sqr(A, a.x);                   // 1
  f29_sqr(B, a.y);                   // 1
  f29_mul(t, a.y, a.z);              // 1   (1 x 2)
  f29_add(r.z, t, t);                // Z3 = 2YZ: 2      (a.y, a.z dead)
  f29_sqr(C, B);                     // 1
  f29_mul(D, a.x, B);                // 1                (a.x dead)
  f29_mul3_norm(E, A);               // E = 3A: 1
  f29_sqr(F, E);                     // 1
#endif
#if !GV_DBL25
  f29_shl_norm<2>(D, D);             // 4D: 1
#endif
  f29_add(u, D, D);                  // 8D: 2
  f29_sub_norm<2>(r.x, F, u);        // X3 = F - 8D: 1   (in 1 + 2 + 1)
  f29_sub<1>(t, D, r.x);             // 4D - X3: 3
  f29_mul(t, E, t);                  // 1   (1 x 3)
  f29_shl_norm<3>(u, C);             // 8C: 1
  f29_sub_norm<1>(r.y, t, u);        // Y3: 1            (in 1 + 1 + 1)
}

// Shared tail of the mixed additions: a += (u2, s2) where u2, s2 (magnitude 1)
// are the added point scaled to a's Z.  Exceptional cases: H == 0 and R == 0
// (a == b) -> doubling; H == 0 and R != 0 (a == -b) -> infinity.  The doubling
// runs after the regular formula's (exec-masked) region so the two register
// sets are never live together.  In/out: point invariant.
GV_DEV void gej29_add_tail(gej29& a, bool& inf, const fe29& u2, const fe29& s2) {
  fe29 h, rr;
  f29_sub_norm<1>(h, u2, a.x);       // H = U2 - X1: 1
  f29_sub_norm<1>(rr, s2, a.y);      // R = S2 - Y1: 1
  const bool exc = f29_is_zero_fast(h);
  bool dbl = false;
  if (exc) {
    dbl = f29_is_zero(rr);
    if (!dbl) inf = true;            // a == -b
  } else {
    fe29 h2, h3, v, t, w;
#if GV_ILP
    {
      fe29 o[2];
      const fe29 x[2] = {h, rr};
      f29_multi<true, true>(o, x, x);
      h2 = o[0]; t = o[1];           // H^2, R^2: 1
    }
    {
      fe29 o[3];
      const fe29 x[3] = {h2, a.x, a.z}, y[3] = {h, h2, h};
      f29_multi<false, false, false>(o, x, y);
      h3 = o[0]; v = o[1]; a.z = o[2];   // H^3, V = X1*H^2, Z3 = Z1*H (2 x 1): 1
    }
#else
    f29_sqr(h2, h);                  // 1
    f29_mul(h3, h2, h);              // 1
    f29_mul(v, a.x, h2);             // V = X1*H^2: 1
    f29_mul(a.z, a.z, h);            // Z3 = Z1*H: 1    (2 x 1)
    f29_sqr(t, rr);                  // R^2: 1
#endif
    f29_add(w, v, v);                // 2V: 2
    f29_add(w, w, h3);               // H^3 + 2V: 3
    f29_sub_norm<3>(a.x, t, w);      // X3 = R^2 - H^3 - 2V: 1   (in 1 + 3 + 1)
    f29_sub<1>(t, v, a.x);           // V - X3: 3
#if GV_ILP
    {
      fe29 o[2];
      const fe29 x[2] = {rr, a.y}, y[2] = {t, h3};
      f29_multi<false, false>(o, x, y);
      t = o[0]; h3 = o[1];           // R(V - X3) (1 x 3), Y1*H^3: 1
    }
#else
    f29_mul(t, rr, t);               // 1   (1 x 3)
    f29_mul(h3, a.y, h3);            // Y1*H^3: 1
#endif
    f29_sub_norm<1>(a.y, t, h3);     // Y3 = R(V - X3) - Y1*H^3: 1
  }
  if (dbl) gej29_double(a, a);       // a == b: a + b = 2a (a untouched above)
}

// a += (x2, y2) affine on a's curve (magnitude <= 2 each; x2 * z2 needs
// mag(x2) <= 6, y2 * z3 mag(y2) <= 6).  a finite.
GV_DEV void gej29_add_ge(gej29& a, bool& inf, const fe29& x2, const fe29& y2) {
  fe29 z2, u2, s2;
  f29_sqr(z2, a.z);                  // 1   (Z <= 2)
  f29_mul(u2, x2, z2);
  f29_mul(z2, z2, a.z);              // Z^3: 1
  f29_mul(s2, y2, z2);
  gej29_add_tail(a, inf, u2, s2);
}

// r = a + b for two Jacobian points of the same curve (12M + 4S), complete:
// either infinite -> the other; a == b -> 2a; a == -b -> infinity.  In: point
// invariant; out: X, Y, Z magnitude 1.  r may alias a or b.
GV_DEV void gej29_add_gej(gej29& r, bool& rinf, const gej29& a, bool ainf, const gej29& b, bool binf) {
  if (ainf || binf) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {        // per-limb selects: no address-taken struct
      r.x.n[i] = ainf ? b.x.n[i] : a.x.n[i];
      r.y.n[i] = ainf ? b.y.n[i] : a.y.n[i];
      r.z.n[i] = ainf ? b.z.n[i] : a.z.n[i];
    }
    rinf = ainf && binf;
    return;
  }
  fe29 z1z1, z2z2, u1, u2, s1, s2, t, h, rr;
  f29_sqr(z1z1, a.z);
  f29_sqr(z2z2, b.z);
  f29_mul(u1, a.x, z2z2);
  f29_mul(u2, b.x, z1z1);
  f29_mul(t, b.z, z2z2);             // 2 x 1
  f29_mul(s1, a.y, t);
  f29_mul(t, a.z, z1z1);
  f29_mul(s2, b.y, t);
  f29_sub_norm<1>(h, u2, u1);        // 1
  f29_sub_norm<1>(rr, s2, s1);       // 1
  bool inf = false, dbl = false;
  gej29 o;
  if (f29_is_zero_fast(h)) {
    dbl = f29_is_zero(rr);
    inf = !dbl;
  } else {
    fe29 h2, h3, v, w;
    f29_sqr(h2, h);
    f29_mul(h3, h2, h);
    f29_mul(v, u1, h2);
    f29_mul(t, a.z, b.z);            // <= 2 x 2
    f29_mul(o.z, t, h);
    f29_sqr(t, rr);
    f29_add(w, v, v);                // 2
    f29_add(w, w, h3);               // 3
    f29_sub_norm<3>(o.x, t, w);      // X3 = R^2 - H^3 - 2V: 1
    f29_sub<1>(t, v, o.x);           // 3
    f29_mul(t, rr, t);
    f29_mul(h3, s1, h3);
    f29_sub_norm<1>(o.y, t, h3);     // Y3 = R(V - X3) - S1*H^3: 1
  }
  if (dbl) gej29_double(o, a);
  r = o;
  rinf = inf;
}

// ---------------------------------------------------- exponentiation chains
GV_DEV void f29_sqr_n(fe29& r, const fe29& a, int k) {
  r = a;
#pragma unroll 1
  for (int i = 0; i < k; ++i) f29_sqr(r, r);
}

// Shared prefix of the p-2 and (p+1)/4 addition chains (the same chain as
// secp_field.cuh fe_pow_prefix): x223 = a^(2^223-1), x2 = a^3, x22 =
// a^(2^22-1).  a magnitude <= 2.
GV_DEV void f29_pow_prefix(fe29& x2, fe29& x22, fe29& x223, const fe29& a) {
  fe29 x3, x6, x9, x11, x44, x88, x176, x220, t;
  f29_sqr(x2, a); f29_mul(x2, x2, a);            // 2^2-1
  f29_sqr(x3, x2); f29_mul(x3, x3, a);           // 2^3-1
  f29_sqr_n(t, x3, 3); f29_mul(x6, t, x3);       // 2^6-1
  f29_sqr_n(t, x6, 3); f29_mul(x9, t, x3);       // 2^9-1
  f29_sqr_n(t, x9, 2); f29_mul(x11, t, x2);      // 2^11-1
  f29_sqr_n(t, x11, 11); f29_mul(x22, t, x11);   // 2^22-1
  f29_sqr_n(t, x22, 22); f29_mul(x44, t, x22);   // 2^44-1
  f29_sqr_n(t, x44, 44); f29_mul(x88, t, x44);   // 2^88-1
  f29_sqr_n(t, x88, 88); f29_mul(x176, t, x88);  // 2^176-1
  f29_sqr_n(t, x176, 44); f29_mul(x220, t, x44); // 2^220-1
  f29_sqr_n(t, x220, 3); f29_mul(x223, t, x3);   // 2^223-1
}

// r = a^(p-2) = a^-1 (a != 0)
GV_DEV void f29_inv(fe29& r, const fe29& a) {
  fe29 x2, x22, x223, t;
  f29_pow_prefix(x2, x22, x223, a);
  f29_sqr_n(t, x223, 23); f29_mul(t, t, x22);
  f29_sqr_n(t, t, 5); f29_mul(t, t, a);
  f29_sqr_n(t, t, 3); f29_mul(t, t, x2);
  f29_sqr_n(t, t, 2); f29_mul(r, t, a);
}

// r = a^((p+1)/4), the square-root candidate (btcec decompressPoint's
// QPlus1Div4 exponentiation)
GV_DEV void f29_sqrt_candidate(fe29& r, const fe29& a) {
  fe29 x2, x22, x223, t;
  f29_pow_prefix(x2, x22, x223, a);
  f29_sqr_n(t, x223, 23); f29_mul(t, t, x22);
  f29_sqr_n(t, t, 6); f29_mul(t, t, x2);
  f29_sqr_n(r, t, 2);
}

}  // namespace gv
