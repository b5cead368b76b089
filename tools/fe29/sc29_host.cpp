// Host build of csrc/secp_sc29.cuh (with overflow traps) for
// tests/test_sc29_host.py (ctypes).
#define GV_F29_CHECK 1
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_sc29.cuh"
#include <string.h>
using namespace gv;
static void ld(sc29& r, const u32* a) { memcpy(r.n, a, 36); }
static void st(u32* r, const sc29& a) { memcpy(r, a.n, 36); }
extern "C" {
void sc29h_mul(const u32* a, const u32* b, u32* r) { sc29 x, y, z; ld(x, a); ld(y, b); sc29_mul(z, x, y); st(r, z); }
void sc29h_sqr(const u32* a, u32* r) { sc29 x, z; ld(x, a); sc29_sqr(z, x); st(r, z); }
void sc29h_inv(const u32* a, u32* r) { sc29 x, z; ld(x, a); sc29_inv(z, x); st(r, z); }
void sc29h_to_mont(const u32* a, u32* r) { sc29 x, z; ld(x, a); sc29_to_mont(z, x); st(r, z); }
void sc29h_to_words(const u32* a, u32* w) { sc29 x; ld(x, a); sc29_to_words(w, x); }
void sc29h_from_words(const u32* w, u32* r) { sc29 x; sc29_from_words(x, w); st(r, x); }
}
