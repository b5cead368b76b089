// secp_group29x.cuh -- the throughput ladder's group law on the fused product
// engine (secp_fe29x.cuh): same formulas, same exceptional-case semantics and
// same results as secp_group29.cuh (btcec KoblitzCurve.Add / doubleJacobian,
// btcd v0.20.1-beta btcec/btcec.go), with every subtraction, small multiple
// and doubling-by-operand folded into a product chain instead of a separate
// carry pass.  Magnitudes after each step in the comments.
//
// Point invariant between operations: X, Y, Z magnitude 1 (Z <= 2 accepted).
#pragma once
#include "secp_group29.cuh"
#include "secp_fe29x.cuh"

namespace gv {

// r = 2a (a finite), 3M + 4S:
//   B = Y^2, Z3 = (2Y) Z, E = 3X^2, D = X B, C = B^2,
//   X3 = E^2 - 8D, Y3 = E (4D - X3) - 8C.
// In: X 1, Y 1, Z <= 2.  Out: X, Y, Z 1.  r may alias a.
GV_DEV void gej29x_double(gej29& r, const gej29& a) {
  fe29 dy, B, E, D, C, nD, nC, t, d;
  f29x_shl1(dy, a.y);                          // 2Y: 2
  f29x_sqr_d(B, a.y, dy);                      // Y^2: 1
  f29x_mul(r.z, dy, a.z);                      // Z3 = 2YZ: 1   (2 x 2)
  f29x_sqr3(E, a.x);                           // 3X^2: 1
  f29x_mul(D, a.x, B);                         // XY^2: 1       (a.x dead)
  f29x_shl1(d, B);
  f29x_sqr_d(C, B, d);                         // Y^4: 1
  f29_neg<1>(nD, D);                           // -D: 2
  f29x_shl1(d, E);
  f29x_sqr_d(r.x, E, d, f29x_plus<8>{nD.n});   // X3 = E^2 - 8D: 1
#pragma unroll
  for (int i = 0; i < 9; ++i)                  // 4D - X3: 4 + 2 = 6
    t.n[i] = f29_add32(D.n[i] << 2, f29_kneg(1, i) - r.x.n[i]);
  f29_neg<1>(nC, C);                           // -C: 2
  f29x_mul(r.y, E, t, f29x_plus<8>{nC.n});     // Y3 = E(4D - X3) - 8C: 1  (1 x 6)
}

// a += (x, y) where (x, y) is affine on the curve whose points are scaled by
// az (az = a.z for a table entry of the accumulator's curve, a.z * zinv for
// a G entry): U2 = x az^2, S2 = y az^3, H = U2 - X1, R = S2 - Y1.
// H == 0: R == 0 -> doubling (a == b), else infinity (a == -b).  a finite.
// x magnitude 1, y <= 2, az <= 2.
GV_DEV void gej29x_add_scaled(gej29& a, bool& inf, const fe29& x, const fe29& y, const fe29& az) {
  fe29 z2, z3, h, rr, n;
  f29x_sqr(z2, az);                            // 1
  f29_neg<1>(n, a.x);                          // -X1: 2
  f29x_mul(h, x, z2, f29x_plus<1>{n.n});       // H = x az^2 - X1: 1
  f29x_mul(z3, z2, az);                        // 1
  f29_neg<1>(n, a.y);                          // -Y1: 2
  f29x_mul(rr, y, z3, f29x_plus<1>{n.n});      // R = y az^3 - Y1: 1  (2 x 1)
#if defined(GV_ISA_NOEXC)
  const bool exc = false;                      // tools/isa_ops.hip: main path only
#else
  const bool exc = f29_is_zero_fast(h);
#endif
  bool dbl = false;
  if (exc) {
    dbl = f29_is_zero(rr);
    if (!dbl) inf = true;                      // a == -b
  } else {
    fe29 d, h2, h3, v, w, yh;
    f29x_shl1(d, h);
    f29x_sqr_d(h2, h, d);                      // H^2: 1
    f29x_mul(h3, h2, h);                       // H^3: 1
    f29x_mul(v, a.x, h2);                      // V = X1 H^2: 1
    f29x_mul(a.z, a.z, h);                     // Z3 = Z1 H: 1   (2 x 1)
#pragma unroll
    for (int i = 0; i < 9; ++i)                // -(2V + H^3): K_3 - 3 -> 4
      w.n[i] = f29_kneg(3, i) - f29_add32(v.n[i] << 1, h3.n[i]);
    f29x_shl1(d, rr);
    f29x_sqr_d(a.x, rr, d, f29x_plus<1>{w.n}); // X3 = R^2 - H^3 - 2V: 1
    fe29 t;
    f29_sub<1>(t, v, a.x);                     // V - X3: 3
    f29_neg<1>(yh, a.y);                       // -Y1: 2
    f29x_mul2(a.y, rr, t, yh, h3);             // Y3 = R(V - X3) + (-Y1) H^3: 1  (1 x 3 + 2 x 1)
  }
  if (dbl) gej29x_double(a, a);                // a == b: 2a (a untouched above)
}

// ---------------------------------------------------- exponentiation chains
// The (p+1)/4 square-root chain of secp_group29.cuh (f29_pow_prefix /
// f29_sqrt_candidate: the same addition chain, the same result) on the fused
// products.  a magnitude <= 2.
GV_DEV void f29x_sqr_n(fe29& r, const fe29& a, int k) {
  r = a;
#pragma unroll 1
  for (int i = 0; i < k; ++i) f29x_sqr(r, r);
}
GV_DEV void f29x_sqrt_candidate(fe29& r, const fe29& a) {
  fe29 x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  f29x_sqr(x2, a); f29x_mul(x2, x2, a);            // 2^2-1
  f29x_sqr(x3, x2); f29x_mul(x3, x3, a);           // 2^3-1
  f29x_sqr_n(t, x3, 3); f29x_mul(x6, t, x3);       // 2^6-1
  f29x_sqr_n(t, x6, 3); f29x_mul(x9, t, x3);       // 2^9-1
  f29x_sqr_n(t, x9, 2); f29x_mul(x11, t, x2);      // 2^11-1
  f29x_sqr_n(t, x11, 11); f29x_mul(x22, t, x11);   // 2^22-1
  f29x_sqr_n(t, x22, 22); f29x_mul(x44, t, x22);   // 2^44-1
  f29x_sqr_n(t, x44, 44); f29x_mul(x88, t, x44);   // 2^88-1
  f29x_sqr_n(t, x88, 88); f29x_mul(x176, t, x88);  // 2^176-1
  f29x_sqr_n(t, x176, 44); f29x_mul(x220, t, x44); // 2^220-1
  f29x_sqr_n(t, x220, 3); f29x_mul(x223, t, x3);   // 2^223-1
  f29x_sqr_n(t, x223, 23); f29x_mul(t, t, x22);
  f29x_sqr_n(t, t, 6); f29x_mul(t, t, x2);
  f29x_sqr_n(r, t, 2);
}

}  // namespace gv
