// Host build of csrc/secp_fe29x.cuh + secp_group29x.cuh (the fused product
// engine and the throughput ladder's group law) with the fe29 overflow traps,
// for tests/test_fe29x_host.py (ctypes).  Any wrapping u64 mad or u32 limb add
// aborts the process.
#define GV_F29_CHECK 1
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_group29x.cuh"
#include <string.h>
using namespace gv;
static void ld(fe29& r, const u32* a) { memcpy(r.n, a, 36); }
static void st(u32* r, const fe29& a) { memcpy(r, a.n, 36); }
extern "C" {
// mode 0: a*b; 1: a*b + 1*c; 2: a*b + 8*c; 3: a*b + 1*c + 8*e
void f29xh_mul(const u32* a, const u32* b, const u32* c, const u32* e, int mode, u32* r) {
  fe29 x, y, z;
  ld(x, a); ld(y, b);
  switch (mode) {
    case 0: f29x_mul(z, x, y); break;
    case 1: f29x_mul(z, x, y, f29x_plus<1>{c}); break;
    case 2: f29x_mul(z, x, y, f29x_plus<8>{c}); break;
    default: f29x_mul(z, x, y, f29x_plus2<1, 8>{c, e}); break;
  }
  st(r, z);
}
// mode 0: a^2; 1: a^2 + 1*c; 2: a^2 + 8*c; 3: 3a^2; 4: 3a^2 + 8*c
void f29xh_sqr(const u32* a, const u32* c, int mode, u32* r) {
  fe29 x, z;
  ld(x, a);
  switch (mode) {
    case 0: f29x_sqr(z, x); break;
    case 1: f29x_sqr(z, x, f29x_plus<1>{c}); break;
    case 2: f29x_sqr(z, x, f29x_plus<8>{c}); break;
    case 3: f29x_sqr3(z, x); break;
    default: f29x_sqr3(z, x, f29x_plus<8>{c}); break;
  }
  st(r, z);
}
// a*b + c*d (+ 8*e when mode)
void f29xh_mul2(const u32* a, const u32* b, const u32* c, const u32* d, const u32* e, int mode, u32* r) {
  fe29 x, y, z, w, v, o;
  ld(x, a); ld(y, b); ld(z, c); ld(w, d); ld(v, e);
  if (mode) f29x_mul2(o, x, y, z, w, f29x_plus<8>{v.n});
  else f29x_mul2(o, x, y, z, w);
  st(r, o);
}
// in/out: X, Y, Z raw limbs (27 words)
void g29xh_double(const u32* in, u32* out) {
  gej29 p;
  memcpy(p.x.n, in, 36); memcpy(p.y.n, in + 9, 36); memcpy(p.z.n, in + 18, 36);
  gej29x_double(p, p);
  memcpy(out, p.x.n, 36); memcpy(out + 9, p.y.n, 36); memcpy(out + 18, p.z.n, 36);
}
// acc (27 words) += (x, y) scaled by az; returns inf flag (bit 0) after
int g29xh_add_scaled(const u32* in, const u32* x, const u32* y, const u32* az, u32* out) {
  gej29 p;
  fe29 X, Y, Z;
  memcpy(p.x.n, in, 36); memcpy(p.y.n, in + 9, 36); memcpy(p.z.n, in + 18, 36);
  ld(X, x); ld(Y, y); ld(Z, az);
  bool inf = false;
  gej29x_add_scaled(p, inf, X, Y, Z);
  memcpy(out, p.x.n, 36); memcpy(out + 9, p.y.n, 36); memcpy(out + 18, p.z.n, 36);
  return inf ? 1 : 0;
}
}
