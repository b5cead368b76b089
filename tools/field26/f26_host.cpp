// Host build of tools/field26/secp_field26.cuh (the 10 x 26 prototype, not in the product tree) for tests/test_field26_host.py (ctypes).
#include "secp_field26.cuh"
#include <string.h>
using namespace gv;
static void ld(fe26& r, const u32* a) { memcpy(r.n, a, 40); }
static void st(u32* r, const fe26& a) { memcpy(r, a.n, 40); }
extern "C" {
void f26_mul(const u32* a, const u32* b, u32* r) { fe26 x, y, z; ld(x, a); ld(y, b); fe26_mul(z, x, y); st(r, z); }
void f26_sqr(const u32* a, u32* r) { fe26 x, z; ld(x, a); fe26_sqr(z, x); st(r, z); }
void f26_sub(const u32* a, const u32* b, u32 mb, u32* r) { fe26 x, y, z; ld(x, a); ld(y, b); fe26_sub(z, x, y, mb); st(r, z); }
void f26_neg(const u32* b, u32 mb, u32* r) { fe26 y, z; ld(y, b); fe26_neg(z, y, mb); st(r, z); }
void f26_norm(const u32* a, u32* r) { fe26 x; ld(x, a); fe26_normalize_weak(x); st(r, x); }
void f26_to_words(const u32* a, u32* w) { fe26 x; ld(x, a); fe26_to_words(w, x); }
void f26_from_words(const u32* w, u32* r) { fe26 x; fe26_from_words(x, w); st(r, x); }
int f26_is_zero(const u32* a) { fe26 x; ld(x, a); return fe26_is_zero(x); }
}
