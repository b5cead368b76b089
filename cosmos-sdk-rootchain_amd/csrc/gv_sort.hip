// gv_sort.hip -- key-ordered lanes for keyed throughput batches.
//
// A keyed batch (in-batch key grouping, gv_keys_load slots, a host slice's
// grouped keys) gives item i the key-arena slot kslot[i]; the reference's
// block order puts an account's signatures anywhere in the batch (C2: 65,536
// keys round-robin over 1M signatures), so the 64 lanes of a ladder wave
// gather their 66 table entries from 64 different keys' 5.4 KB tables and
// every gather misses L2.  Here the lanes are put in slot order first: a
// counting sort by slot (rank within the slot by atomic increment, exclusive
// scan of the slot counts, placement), then the signature / digest rows are
// unpacked straight from the AoS input of item perm[g] into lane g, and after
// the ladder the accept bits are gathered back to item order.  A wave then
// covers ~4 keys (C2), whose tables stay in L1 / L2 for its 16 lanes each.
// Every kernel here is hand-written (the slot-count scan included).
// Verdicts are a pure function of the item, so the order within a slot
// (atomic arrival order) does not matter.
#include <hip/hip_runtime.h>
#include "gv_kernels.h"

namespace gv {
typedef uint32_t u32;

// rank[g] = g's arrival order among the items of its (clamped) slot
__global__ __launch_bounds__(256) void k_slot_rank(u32 n, const u32* kslot, u32 kcount, u32* cnt, u32* rank) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const u32 sl = min(kslot[g], kcount);     // out-of-range slots share the last bucket
  rank[g] = atomicAdd(&cnt[sl], 1u);
}

// pos = off[slot] + rank (written over rank), perm[pos] = g, kslot_s[pos] = slot
__global__ __launch_bounds__(256) void k_slot_place(u32 n, const u32* kslot, u32 kcount, const u32* off, u32* rank,
                                                     u32* perm, u32* kslot_s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const u32 sl = kslot[g];
  const u32 pos = off[min(sl, kcount)] + rank[g];
  rank[g] = pos;
  perm[pos] = g;
  kslot_s[pos] = sl;
}

// ---- exclusive scan of the slot counts (hand-written, three launches): each
// 256-thread block scans 2,048 counts (8 per thread: a sequential prefix, a
// wave scan of the thread totals by lane shuffles, the four wave totals
// through LDS) and writes its total; one block scans the block totals
// (sequential carry over chunks of 2,048); every block adds its offset.
#define GV_SCAN_PER 8
#define GV_SCAN_BLK (256 * GV_SCAN_PER)

// exclusive scan of the 256 threads' values v in a block; returns the block total
__device__ __forceinline__ u32 block_excl_scan(u32 v, u32& excl) {
  __shared__ u32 wsum[4];
  const u32 lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  u32 inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u32 t = (u32)__shfl_up((int)inc, d, 64);
    if (lane >= (u32)d) inc += t;
  }
  if (lane == 63u) wsum[w] = inc;
  __syncthreads();
  u32 woff = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    woff += (u32)k < w ? wsum[k] : 0u;
    tot += wsum[k];
  }
  __syncthreads();                          // wsum reusable by a later call
  excl = woff + inc - v;
  return tot;
}

__global__ __launch_bounds__(256) void k_scan_local(u32 n, const u32* in, u32* out, u32* sums) {
  const u32 base = blockIdx.x * GV_SCAN_BLK + threadIdx.x * GV_SCAN_PER;
  u32 v[GV_SCAN_PER], t = 0;
#pragma unroll
  for (int k = 0; k < GV_SCAN_PER; ++k) {
    v[k] = base + k < n ? in[base + k] : 0u;
    t += v[k];
  }
  u32 excl;
  const u32 tot = block_excl_scan(t, excl);
#pragma unroll
  for (int k = 0; k < GV_SCAN_PER; ++k) {
    if (base + k < n) out[base + k] = excl;
    excl += v[k];
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// one block: sums[0..m) -> exclusive prefix sums, in place
__global__ __launch_bounds__(256) void k_scan_top(u32 m, u32* sums) {
  u32 carry = 0;
  for (u32 c0 = 0; c0 < m; c0 += GV_SCAN_BLK) {   // uniform loop: every thread reaches each barrier
    const u32 base = c0 + threadIdx.x * GV_SCAN_PER;
    u32 v[GV_SCAN_PER], t = 0;
#pragma unroll
    for (int k = 0; k < GV_SCAN_PER; ++k) {
      v[k] = base + k < m ? sums[base + k] : 0u;
      t += v[k];
    }
    u32 excl;
    const u32 tot = block_excl_scan(t, excl);
    excl += carry;
#pragma unroll
    for (int k = 0; k < GV_SCAN_PER; ++k) {
      if (base + k < m) sums[base + k] = excl;
      excl += v[k];
    }
    carry += tot;
  }
}

__global__ __launch_bounds__(256) void k_scan_add(u32 n, u32* out, const u32* sums) {
  const u32 off = sums[blockIdx.x];
  const u32 base = blockIdx.x * GV_SCAN_BLK + threadIdx.x;
#pragma unroll
  for (int k = 0; k < GV_SCAN_PER; ++k)
    if (base + k * 256u < n) out[base + k * 256u] += off;
}

// big-endian 32-bit word k (0 = most significant) of a 16-byte vector pair
__device__ __forceinline__ u32 be_word(const uint4* p, int k) {
  const uint4 v = p[k >> 2];
  const u32 w = (k & 3) == 0 ? v.x : (k & 3) == 1 ? v.y : (k & 3) == 2 ? v.z : v.w;
  return __builtin_bswap32(w);
}

// Lane g < n takes item perm[g]: r, s from its 64 signature bytes, e from its
// 32 digest bytes (dig32 null: the message path hashes into e itself), read
// as 16-byte vectors straight from the AoS input.  Lanes >= n: r = 0, s = 1.
__global__ __launch_bounds__(256) void k_unpack_perm(const uint8_t* sig64, const uint8_t* dig32, const u32* perm,
                                                      u32 n, u32 C, u32* r, u32* s, u32* e) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= C) return;
  if (g >= n) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      r[(size_t)i * C + g] = 0u;
      s[(size_t)i * C + g] = i == 0 ? 1u : 0u;
      if (dig32) e[(size_t)i * C + g] = 0u;
    }
    return;
  }
  const size_t src = perm[g];
  const uint4* ps = (const uint4*)(sig64 + src * 64u);
  // limb i (little-endian 32-bit limbs) = big-endian word 7 - i
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r[(size_t)i * C + g] = be_word(ps, 7 - i);
    s[(size_t)i * C + g] = be_word(ps + 2, 7 - i);
  }
  if (dig32) {
    const uint4* pd = (const uint4*)(dig32 + src * 32u);
#pragma unroll
    for (int i = 0; i < 8; ++i) e[(size_t)i * C + g] = be_word(pd, 7 - i);
  }
}

// Item i's verdict is bit pos[i] of the slot-ordered bitmap.
__global__ __launch_bounds__(256) void k_unsort_bits(u32 n, const u32* pos, const uint64_t* sbits, uint64_t* bits) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  bool ok = false;
  if (i < n) {
    const u32 p = pos[i];
    ok = (sbits[p >> 6] >> (p & 63u)) & 1ull;
  }
  const uint64_t mask = __ballot(ok);
  if ((threadIdx.x & 63u) == 0 && (i >> 6) < ((n + 63u) >> 6)) bits[i >> 6] = mask;
}

}  // namespace gv

extern "C" {

size_t gvk_sort_temp_bytes(uint32_t nbuckets) {
  return ((size_t)(nbuckets + GV_SCAN_BLK - 1) / GV_SCAN_BLK) * 4;   // one total per scan block
}

// exclusive prefix sums of n counts (temp: gvk_sort_temp_bytes(n))
static hipError_t excl_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* temp, hipStream_t st) {
  const uint32_t nblk = (n + GV_SCAN_BLK - 1) / GV_SCAN_BLK;
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(gv::k_scan_local, dim3(nblk), dim3(256), 0, st, n, in, out, temp);
  if (nblk > 1) {
    hipLaunchKernelGGL(gv::k_scan_top, dim3(1), dim3(256), 0, st, nblk, temp);
    hipLaunchKernelGGL(gv::k_scan_add, dim3(nblk), dim3(256), 0, st, n, out, (const uint32_t*)temp);
  }
  return hipGetLastError();
}

hipError_t gvk_sort_slots(const gvk_sort* so, uint32_t n, const uint32_t* kslot, uint32_t kcount, hipStream_t st) {
  const uint32_t nb = kcount + 1;
  const dim3 blk(256), grd((n + 255) / 256);
  hipError_t e = hipMemsetAsync(so->cnt, 0, (size_t)nb * 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gv::k_slot_rank, grd, blk, 0, st, n, kslot, kcount, so->cnt, so->pos);
  if (so->temp_bytes < gvk_sort_temp_bytes(nb)) return hipErrorInvalidValue;
  e = excl_scan((const uint32_t*)so->cnt, so->off, nb, (uint32_t*)so->temp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gv::k_slot_place, grd, blk, 0, st, n, kslot, kcount, (const uint32_t*)so->off, so->pos,
                     so->perm, so->kslot);
  return hipGetLastError();
}

hipError_t gvk_unpack_perm(const uint8_t* sig64, const uint8_t* dig32, const uint32_t* perm, uint32_t n, uint32_t C,
                           uint32_t* r, uint32_t* s, uint32_t* e, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_unpack_perm, dim3(C / 256), dim3(256), 0, st, sig64, dig32, perm, n, C, r, s, e);
  return hipGetLastError();
}

hipError_t gvk_unsort_bits(uint32_t n, const uint32_t* pos, const uint64_t* sbits, uint64_t* bits, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_unsort_bits, dim3((n + 255) / 256), dim3(256), 0, st, n, pos, sbits, bits);
  return hipGetLastError();
}

}  // extern "C"
