// Host build of csrc/secp_modinv.cuh for tests/test_modinv_host.py (ctypes).
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_modinv.cuh"
using namespace gv;
extern "C" {
// w = x^-1 mod n; returns the number of rounds used
int mi_inv(const uint32_t* x, uint32_t* w) {
  int rounds = 0;
  s30_modinv(w, x, [&](bool done) { if (!done) ++rounds; return done; });
  return rounds;
}
// one 30-step batch on low words (for the matrix-bound check)
int32_t mi_divsteps(int32_t delta, uint32_t f, uint32_t g, int32_t* t) { return s30_divsteps(delta, f, g, t); }
// variable-time form (eta = -delta), the latency kernels' scalar inverse
int mi_inv_var(const uint32_t* x, uint32_t* w) {
  int rounds = 0;
  s30_modinv_var(w, x, [&]() { ++rounds; });
  return rounds;
}
int32_t mi_divsteps_var(int32_t eta, uint32_t f, uint32_t g, int32_t* t) { return s30_divsteps_var(eta, f, g, t); }
}
