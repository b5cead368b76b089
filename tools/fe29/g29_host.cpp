// Host build of csrc/secp_group29.cuh (with the fe29 overflow traps) for
// tests/test_fe29_host.py: the Jacobian doubling in each formula variant
// (GV_DBL25 / GV_ILP chosen on the compile line) against Python integers.
#define GV_F29_CHECK 1
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_group29.cuh"
#include <string.h>
using namespace gv;
extern "C" {
// in/out: X, Y, Z raw limbs (27 words)
void g29h_double(const u32* in, u32* out) {
  gej29 p;
  memcpy(p.x.n, in, 36); memcpy(p.y.n, in + 9, 36); memcpy(p.z.n, in + 18, 36);
  gej29_double(p, p);
  memcpy(out, p.x.n, 36); memcpy(out + 9, p.y.n, 36); memcpy(out + 18, p.z.n, 36);
}
}
