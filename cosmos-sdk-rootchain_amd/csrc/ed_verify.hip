// ed_verify.hip -- ed25519 VerifyBytes on gfx950: the
// multisig ed25519 sub-key leaves of x/auth/ante/sigverify.go:303-306 /
// :325-338 (tendermint v0.33.4 PubKeyEd25519.VerifyBytes -> go1.14
// crypto/ed25519 Verify), one signature per lane.
//
//   k_ed_btab    one-time: the resident comb table j * 256^w * B
//                (32 windows x 129 entries x 27 words = 436 KB, L2-resident)
//   k_ed_prep    per lane: SHA-512(R || A || M) mod L, the sig[63] & 224 and
//                ScMinimal checks, FromBytes(A), the per-lane table j(-A)
//                (global scratch, lane-major: each lane's entry is 144
//                contiguous bytes, so a data-dependent lookup touches only
//                its own lines -- the SoA layout made every lookup pull a
//                line per lane per limb: 84 KB of HBM fetch per verify)
//   k_ed_ladder  per lane: 252 doublings + 64 signed radix-16 table adds for
//                [h](-A), 32 comb adds for [s]B, one inversion to encode R',
//                a byte compare with sig[:32]; the accept bitmap by ballot.
//                A separate launch so it can run at 3 waves per SIMD (the
//                hash / decode stage needs ~240 VGPRs, the ladder ~168).
// The arithmetic lives in ed_group.cuh and is the same source the CPU tests
// compile (tests/test_ed_host.py).
#include <hip/hip_runtime.h>

#include "ed_group.cuh"
#include "gv_kernels.h"

#if defined(__HIP_DEVICE_COMPILE__) && defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "ed_verify.hip writes one 64-bit ballot word per wave64"
#endif

namespace gv {
namespace ed {

static_assert(ED_ATAB_WORDS == GV_ED_ATAB_WORDS, "per-lane table size");
static_assert(GV_ED_ROWS == ED_ATAB_WORDS + 9, "scratch rows");
static_assert(ED_BTAB_WORDS == GV_ED_BTAB_WORDS, "comb table size");
static_assert(ED_BTAB16_WORDS == GV_ED_BTAB16_WORDS, "radix-2^16 comb table size");

__global__ __launch_bounds__(256) void k_ed_btab(u32* btab) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= ED_BTAB_WINDOWS * ED_BTAB_ENTRIES) return;
  u32 out[ED_PRE_WORDS];
  ed_btab_entry(out, t / ED_BTAB_ENTRIES, t % ED_BTAB_ENTRIES);
#pragma unroll
  for (int k = 0; k < ED_PRE_WORDS; ++k) btab[(size_t)t * ED_PRE_WORDS + k] = out[k];
}

__global__ __launch_bounds__(256) void k_ed_btab16(u32* btab16) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= ED_BTAB16_WINDOWS * ED_BTAB16_ENTRIES) return;
  u32 out[ED_PRE_WORDS];
  ed_btab16_entry(out, t / ED_BTAB16_ENTRIES, t % ED_BTAB16_ENTRIES);
#pragma unroll
  for (int k = 0; k < ED_PRE_WORDS; ++k) btab16[(size_t)t * ED_PRE_WORDS + k] = out[k];
}

// Stage 1 (register-heavy hash / decode / table build; ~11 % of the work).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_ed_prep(gvk_ed b) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  if (g >= b.n) return;
  u32 pw[8], sw[16];
  const uint4* pp = (const uint4*)(b.pub32 + (size_t)g * 32);
  const uint4* sp = (const uint4*)(b.sig64 + (size_t)g * 64);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint4 v = pp[k];
    pw[4 * k] = v.x; pw[4 * k + 1] = v.y; pw[4 * k + 2] = v.z; pw[4 * k + 3] = v.w;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 v = sp[k];
    sw[4 * k] = v.x; sw[4 * k + 1] = v.y; sw[4 * k + 2] = v.z; sw[4 * k + 3] = v.w;
  }
  const uint8_t* m = b.msg_blob + b.msg_off[g];
  u32 h[8];
  u32* tab = b.atab + (size_t)g * ED_ATAB_WORDS;      // lane-major: this lane's 9 entries, 1,296 B
  const bool ok = ed_prep_item(pw, sw, [=](u32 i) { return (u32)m[i]; }, b.msg_len[g], tab, 1, h);
  u32* hrow = b.atab + (size_t)b.C * ED_ATAB_WORDS + g;  // h and the prep verdict: SoA rows
#pragma unroll
  for (int i = 0; i < 8; ++i) hrow[(size_t)i * b.C] = h[i];
  hrow[(size_t)8 * b.C] = ok ? 1u : 0u;
}

// Stage 2: [h](-A) + [s]B, encode, compare; 3 waves per SIMD.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_ed_ladder(gvk_ed b) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  bool ok = false;
  if (g < b.n) {
    const u32* tab = b.atab + (size_t)g * ED_ATAB_WORDS;
    const u32* hrow = b.atab + (size_t)b.C * ED_ATAB_WORDS + g;
    u32 h[8], sw[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = hrow[(size_t)i * b.C];
    const uint4* sp = (const uint4*)(b.sig64 + (size_t)g * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = sp[k];
      sw[4 * k] = v.x; sw[4 * k + 1] = v.y; sw[4 * k + 2] = v.z; sw[4 * k + 3] = v.w;
    }
    const bool pre_ok = hrow[(size_t)8 * b.C] != 0;
    ok = ed_ladder_check(h, sw + 8, tab, 1, b.btab, sw, b.btab16) && pre_ok;
  }
  const uint64_t mask = __ballot(ok);
  if ((threadIdx.x & 63) == 0 && g < b.n) b.bits[g >> 6] = mask;   // words up to ceil(n / 64) only
}

}  // namespace ed
}  // namespace gv

extern "C" hipError_t gvk_ed_btab(uint32_t* btab, hipStream_t st) {
  const int n = ED_BTAB_WINDOWS * ED_BTAB_ENTRIES;
  hipLaunchKernelGGL(gv::ed::k_ed_btab, dim3((n + 255) / 256), dim3(256), 0, st, btab);
  return hipGetLastError();
}

extern "C" hipError_t gvk_ed_btab16(uint32_t* btab16, hipStream_t st) {
  const int n = ED_BTAB16_WINDOWS * ED_BTAB16_ENTRIES;
  hipLaunchKernelGGL(gv::ed::k_ed_btab16, dim3((n + 255) / 256), dim3(256), 0, st, btab16);
  return hipGetLastError();
}

extern "C" hipError_t gvk_ed_verify(const gvk_ed* b, hipStream_t st) {
  hipLaunchKernelGGL(gv::ed::k_ed_prep, dim3(b->C / 256), dim3(256), 0, st, *b);
  hipLaunchKernelGGL(gv::ed::k_ed_ladder, dim3(b->C / 256), dim3(256), 0, st, *b);
  return hipGetLastError();
}
