// Host build of the ed25519 kernel family's device code (csrc/ed_fe29.cuh,
// ed_sha512.cuh, ed_scalar.cuh, ed_group.cuh) with the overflow traps on, for
// tests/test_ed_host.py (ctypes): the exact source the gfx950 kernels run,
// checked against oracle/ed25519_ref.py on the CPU.
#define GV_F29_CHECK 1
#include "../../cosmos-sdk-rootchain_amd/csrc/ed_group.cuh"
#include <string.h>
#include <vector>
using namespace gv;
using namespace gv::ed;
static void ld(fe29& r, const u32* a) { memcpy(r.n, a, 36); }
static void st(u32* r, const fe29& a) { memcpy(r, a.n, 36); }
template <int MB> static void sub_t(fe29& z, const fe29& x, const fe29& y) { e29_sub<MB>(z, x, y); }
template <int MB> static void neg_t(fe29& z, const fe29& y) { e29_neg<MB>(z, y); }
extern "C" {
void edh_mul(const u32* a, const u32* b, u32* r) { fe29 x, y, z; ld(x, a); ld(y, b); e29_mul(z, x, y); st(r, z); }
void edh_sqr(const u32* a, u32* r) { fe29 x, z; ld(x, a); e29_sqr(z, x); st(r, z); }
int edh_sub(const u32* a, const u32* b, int mb, u32* r) {
  fe29 x, y, z; ld(x, a); ld(y, b);
  switch (mb) {
    case 1: sub_t<1>(z, x, y); break; case 2: sub_t<2>(z, x, y); break; case 3: sub_t<3>(z, x, y); break;
    case 4: sub_t<4>(z, x, y); break; case 5: sub_t<5>(z, x, y); break; case 6: sub_t<6>(z, x, y); break;
    default: return -1;
  }
  st(r, z); return 0;
}
int edh_neg(const u32* b, int mb, u32* r) {
  fe29 y, z; ld(y, b);
  switch (mb) {
    case 1: neg_t<1>(z, y); break; case 2: neg_t<2>(z, y); break; case 3: neg_t<3>(z, y); break;
    case 4: neg_t<4>(z, y); break; case 5: neg_t<5>(z, y); break; case 6: neg_t<6>(z, y); break;
    default: return -1;
  }
  st(r, z); return 0;
}
void edh_norm(const u32* a, u32* r) { fe29 x; ld(x, a); e29_norm(x, x); st(r, x); }
void edh_to_words(const u32* a, u32* w) { fe29 x; ld(x, a); e29_to_words(w, x); }
void edh_from_words(const u32* w, u32* r) { fe29 x; e29_from_words(x, w); st(r, x); }
void edh_inv(const u32* a, u32* r) { fe29 x, z; ld(x, a); e29_inv(z, x); st(r, z); }
void edh_pow22523(const u32* a, u32* r) { fe29 x, z; ld(x, a); e29_pow22523(z, x); st(r, z); }
void edh_sha512(const u32* pre, const uint8_t* msg, u32 len, u32* out) {
  sha512_pre64(out, pre, [&](u32 i) { return (u32)msg[i]; }, len);
}
void edh_sc_reduce(const u32* x, u32* r) { sc_reduce512(r, x); }
int edh_sc_minimal(const u32* s) { return sc_minimal(s); }
// decode: returns ok; xy = canonical x, y words (16)
int edh_frombytes(const u32* w, u32* xy) {
  ge_ext a;
  const bool ok = ge_frombytes(a, w);
  ge_tobytes(xy, a);                  // re-encode (canonical) into xy[0..8)
  u32 xw[8];
  fe29 zi, x;
  e29_inv(zi, a.Z);
  e29_mul(x, a.X, zi);
  e29_to_words(xw, x);
  memcpy(xy + 8, xw, 32);
  return ok;
}
void edh_btab_entry(int w, int j, u32* out) { ed_btab_entry(out, w, j); }
void edh_btab(u32* out) {
  for (int w = 0; w < ED_BTAB_WINDOWS; ++w)
    for (int j = 0; j < ED_BTAB_ENTRIES; ++j) ed_btab_entry(out + (size_t)(w * ED_BTAB_ENTRIES + j) * ED_PRE_WORDS, w, j);
}
int edh_verify(const u32* pw, const u32* sw, const uint8_t* msg, u32 len, const u32* btab) {
  std::vector<u32> tab(ED_ATAB_WORDS);
  return ed_verify_item(pw, sw, [&](u32 i) { return (u32)msg[i]; }, len, tab.data(), 1, btab);
}
}
