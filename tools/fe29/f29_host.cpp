// Host build of csrc/secp_fe29.cuh (with overflow traps) for
// tests/test_fe29_host.py (ctypes).  Any u64 mad or u32 limb add that would
// wrap aborts the process, so a magnitude-budget violation fails the test.
#define GV_F29_CHECK 1
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_fe29.cuh"
#include <string.h>
using namespace gv;
static void ld(fe29& r, const u32* a) { memcpy(r.n, a, 36); }
static void st(u32* r, const fe29& a) { memcpy(r, a.n, 36); }
template <int MB> static void sub_t(fe29& z, const fe29& x, const fe29& y) { f29_sub<MB>(z, x, y); }
template <int MB> static void neg_t(fe29& z, const fe29& y) { f29_neg<MB>(z, y); }
extern "C" {
void f29h_mul(const u32* a, const u32* b, u32* r) { fe29 x, y, z; ld(x, a); ld(y, b); f29_mul(z, x, y); st(r, z); }
void f29h_sqr(const u32* a, u32* r) { fe29 x, z; ld(x, a); f29_sqr(z, x); st(r, z); }
void f29h_add(const u32* a, const u32* b, u32* r) { fe29 x, y, z; ld(x, a); ld(y, b); f29_add(z, x, y); st(r, z); }
int f29h_sub(const u32* a, const u32* b, int mb, u32* r) {
  fe29 x, y, z; ld(x, a); ld(y, b);
  switch (mb) {
    case 1: sub_t<1>(z, x, y); break; case 2: sub_t<2>(z, x, y); break; case 3: sub_t<3>(z, x, y); break;
    case 4: sub_t<4>(z, x, y); break; case 5: sub_t<5>(z, x, y); break; case 6: sub_t<6>(z, x, y); break;
    default: return -1;
  }
  st(r, z); return 0;
}
int f29h_neg(const u32* b, int mb, u32* r) {
  fe29 y, z; ld(y, b);
  switch (mb) {
    case 1: neg_t<1>(z, y); break; case 2: neg_t<2>(z, y); break; case 3: neg_t<3>(z, y); break;
    case 4: neg_t<4>(z, y); break; case 5: neg_t<5>(z, y); break; case 6: neg_t<6>(z, y); break;
    default: return -1;
  }
  st(r, z); return 0;
}
void f29h_norm(const u32* a, u32* r) { fe29 x; ld(x, a); f29_norm(x, x); st(r, x); }
int f29h_shl_norm(const u32* a, int s, u32* r) {
  fe29 x, z; ld(x, a);
  switch (s) {
    case 1: f29_shl_norm<1>(z, x); break; case 2: f29_shl_norm<2>(z, x); break;
    case 3: f29_shl_norm<3>(z, x); break; default: return -1;
  }
  st(r, z); return 0;
}
void f29h_to_words(const u32* a, u32* w) { fe29 x; ld(x, a); f29_to_words(w, x); }
void f29h_from_words(const u32* w, u32* r) { fe29 x; f29_from_words(x, w); st(r, x); }
int f29h_is_zero(const u32* a) { fe29 x; ld(x, a); return f29_is_zero(x); }
}
extern "C" {
// three independent products in lockstep: (a0^2, a1^2, a2*b2) -> r (27 words)
void f29h_multi(const u32* a, const u32* b, u32* r) {
  fe29 x[3], y[3], o[3];
  for (int s = 0; s < 3; ++s) { ld(x[s], a + 9 * s); ld(y[s], b + 9 * s); }
  f29_multi<true, true, false>(o, x, y);
  for (int s = 0; s < 3; ++s) st(r + 9 * s, o[s]);
}
}
