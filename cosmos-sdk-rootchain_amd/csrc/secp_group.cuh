// secp_group.cuh -- secp256k1 group law in Jacobian coordinates, one point per
// lane.  Restates the complete group law of btcec KoblitzCurve.Add /
// addJacobian / doubleJacobian (btcd v0.20.1-beta btcec/btcec.go): P == Q
// doubles, P == -Q gives the point at infinity, infinity is the identity.
// The fast formulas below are incomplete; the exceptional cases are detected
// (H == 0 mod p) and routed to doubling / infinity, so results are identical.
//
// Infinity is carried as a per-lane bool next to the Jacobian point.
#pragma once
#include "secp_field.cuh"

namespace gv {

struct gej { fe x, y, z; };

// r = 2a (a finite; secp256k1 has no point of order 2 so the result is finite).
// For a = 0 with D = X*B in place of the (X+B)^2 - A - C trick: 3M + 4S, but
// only six linear steps (x3, x2, x4, one subtraction, two fused
// "minus 8 times") instead of fourteen chained additions/subtractions:
//   A = X^2, B = Y^2, C = B^2, D = X*B, E = 3A, F = E^2,
//   X3 = F - 8D, Y3 = E*(4D - X3) - 8C, Z3 = 2*Y*Z.
// r may alias a.
GV_DEV void gej_double(gej& r, const gej& a) {
  fe A, B, C, D, E, t;
  fe_sqr(A, a.x);
  fe_sqr(B, a.y);
  fe_mul(t, a.y, a.z);
  fe_shl<1>(r.z, t);              // Z3 = 2*Y*Z   (a.y, a.z dead from here)
  fe_sqr(C, B);
  fe_mul(D, a.x, B);              // (a.x dead from here)
  fe_mul3(E, A);
  fe_sqr(t, E);
  fe_sub_shl<3>(r.x, t, D);       // X3 = F - 8D
  fe_shl<2>(D, D);
  fe_sub(t, D, r.x);
  fe_mul(t, E, t);
  fe_sub_shl<3>(r.y, t, C);       // Y3 = E*(4D - X3) - 8C
}

// Shared tail of the mixed additions: given U2, S2 (the added point scaled to
// a's Z), finish a + b.  Exceptional cases: H == 0 and R == 0 (a == b) ->
// doubling; H == 0 and R != 0 (a == -b) -> infinity.  The doubling is done
// AFTER the regular formula's region (which is masked off for those lanes) so
// its temporaries never overlap the addition's live values: with exec-masked
// SIMT branches an inline doubling inside the add would hold both register
// sets at once.
GV_DEV void gej_add_tail(gej& a, bool& inf, const fe& u2, const fe& s2) {
  fe h, rr;
  fe_sub(h, u2, a.x);
  fe_sub(rr, s2, a.y);
  const bool exc = fe_is_zero(h);
  bool dbl = false;
  if (exc) {
    dbl = fe_is_zero(rr);
    if (!dbl) inf = true;         // a == -b
  } else {
    fe h2, h3, v, t;
    fe_sqr(h2, h);
    fe_mul(h3, h2, h);
    fe_mul(v, a.x, h2);             // V = X1*H^2
    fe_mul(a.z, a.z, h);            // Z3 = Z1*H
    fe_sqr(t, rr);
    fe_sub(t, t, h3);
    fe_sub_shl<1>(a.x, t, v);       // X3 = R^2 - H^3 - 2V
    fe_sub(t, v, a.x);
    fe_mul(t, rr, t);
    fe_mul(h3, a.y, h3);
    fe_sub(a.y, t, h3);             // Y3 = R(V - X3) - Y1*H^3
  }
  if (dbl) gej_double(a, a);        // a == b: a + b = 2a (a untouched above)
}

// a += (x2, y2) affine (same curve as a).  a finite.
GV_DEV void gej_add_ge(gej& a, bool& inf, const fe& x2, const fe& y2) {
  fe z2, u2, s2;
  fe_sqr(z2, a.z);
  fe_mul(u2, x2, z2);
  fe_mul(z2, z2, a.z);
  fe_mul(s2, y2, z2);
  gej_add_tail(a, inf, u2, s2);
}

// a += b where b is the Jacobian point (x2, y2, 1/zinv) -- i.e. an affine point
// of the real curve added to an accumulator that lives on the isomorphic curve
// scaled by zinv (effective-affine table trick).  a finite.
GV_DEV void gej_add_zinv(gej& a, bool& inf, const fe& x2, const fe& y2, const fe& zinv) {
  fe az, z2, u2, s2;
  fe_mul(az, a.z, zinv);
  fe_sqr(z2, az);
  fe_mul(u2, x2, z2);
  fe_mul(z2, z2, az);
  fe_mul(s2, y2, z2);
  gej_add_tail(a, inf, u2, s2);
}

}  // namespace gv
