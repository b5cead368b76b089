// gv_runtime.cpp -- the C-ABI runtime of libgpuverify.so (include/gpuverify.h).
//
// Per device: two pipeline "sets" (device scratch for one batch chunk, a HIP
// stream, pinned host staging), a persistent worker thread and a small pool of
// staging threads.  A host batch is split into contiguous slices, one per
// device (no collective -- SURVEY.md §8e); each slice is cut into chunks that
// alternate between the two sets, so the staging memcpy + H2D copy of chunk
// c+1 overlaps the kernels of chunk c (§8e "one host thread + 2 HIP streams
// per GPU, double-buffered pinned staging").  Only the packed accept bitmap
// comes back.  Fail-closed: any HIP error returns GV_EHIP and the caller
// re-verifies on the CPU.
//
// Ordering: every use of a set's device scratch, on whichever stream, first
// waits for the previous use of that set (its `last` event) and then records
// `last` again -- so a gv_dev_* call on a caller stream and a later host-path
// or gv_dev_* call on another stream can never overwrite the inputs of kernels
// still in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <list>
#include <unordered_map>
#include <future>
#include <mutex>
#include <memory>
#include <sched.h>
#include <thread>
#include <vector>

#include "../../include/gpuverify.h"
#include "gv_kernels.h"
#include "gv_stage.h"
#include "gv_async.h"

namespace {

#define CK(call)                                  \
  do {                                            \
    hipError_t e_ = (call);                       \
    if (e_ != hipSuccess) return GV_EHIP;         \
  } while (0)

constexpr size_t kMaxItems = 0xFFFFFF00ull;       // per launch (u32 lane indices)
constexpr size_t kLaneWords = 8 + 1 + 8 + 8 + 8 + GV_DIGIT_ROWS + 8 + 1 + GV_QTAB_WORDS;

size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

// ------------------------------------------------------------ thread helpers
// Pool, Worker, par_copy*, host_cpus, run_sliced: gv_stage.h
using gvstage::CopySeg;
using gvstage::Pool;
using gvstage::Worker;
using gvstage::host_cpus;
using gvstage::par_copy;
using gvstage::par_copy_segs;
using gvstage::run_sliced;

// The grouped route's kg layouts (gv_kernels.h GV_KG_NGS), or 0 (off).
bool kg_layout_ok(int ng) {
  static const int kNGs[] = {GV_KG_NGS};
  if (ng == 0) return true;
  for (int v : kNGs)
    if (v == ng) return true;
  return false;
}

// ------------------------------------------------------------ device state
// Device scratch of one batch chunk of C lanes (C % 256 == 0): the staged
// inputs (one contiguous region so a host chunk is ONE H2D copy), the SoA
// working rows of the kernels, the accept bitmap.
struct Set {
  size_t cap = 0;
  uint8_t* scratch = nullptr;
  uint8_t* d_in = nullptr;                        // staged inputs, layout of in_layout()
  uint32_t *in_x = nullptr, *in_pfx = nullptr, *in_r = nullptr, *in_s = nullptr, *in_e = nullptr;
  uint32_t *digits = nullptr, *zq = nullptr, *flags = nullptr, *qtab = nullptr;
  uint64_t* bits = nullptr;
  uint8_t* d_blob = nullptr;                      // message path blob
  size_t blob_cap = 0;
  hipStream_t st = nullptr;                       // the set's own stream (host path; front priority)
  hipStream_t lad = nullptr;                      // host path: the chunk's ladder (ladder priority), so the
                                                  // next chunk's / batch's front kernels take CU slots first
  hipEvent_t lad_done = nullptr;
  hipEvent_t last = nullptr;                      // end of the last work using this set
  hipStream_t last_st = nullptr;
  hipEvent_t done = nullptr;                      // host path: chunk finished (bits on host)
  hipEvent_t h2d = nullptr;                       // host path: the chunk's H2D copies enqueued so far done
  hipEvent_t ecm_ready = nullptr;                 // pipelined device calls: front kernels done
  hipStream_t side = nullptr;                     // grouped keys: table builds beside k_scalar_inv
  hipEvent_t fork = nullptr, keys_done = nullptr;
  hipEvent_t grp_ready = nullptr;                 // slice grouping on this set: the keys' tables are built
  // in-batch key grouping: the per-batch key arena (tables of the batch's
  // distinct keys, key-arena layout) for up to gcap keys, and the count
  uint32_t *g_kqt = nullptr, *g_kzq = nullptr, *g_kok = nullptr, *g_kqt2 = nullptr, *g_kzq2 = nullptr;
  size_t gcap = 0;
  int g_ent = 0, g_ng = 0;                        // the arena's layout: words per group table, groups per key
  uint32_t* h_count = nullptr;                    // pinned: the distinct-key count read back
  // pinned host staging
  uint8_t* h_in = nullptr;
  size_t h_in_cap = 0;
  uint8_t* h_blob = nullptr;
  size_t h_blob_cap = 0;
  uint64_t* h_bits = nullptr;
  size_t h_bits_cap = 0;
  uint8_t* h_out8 = nullptr;                      // zero-copy small batches: verdict bytes, written by the kernel
  size_t h_out8_cap = 0;
  // chunk waiting to be harvested
  bool busy = false;
  bool zc = false;                                // the chunk ran zero-copy (verdicts in h_out8)
  size_t c0 = 0, cn = 0;
};

// Input region layout of a chunk of C lanes: [pub33 (or u32 slot)] [sig64]
// [dig32 | u64 off + u32 len], each part 256-byte aligned.
struct InLayout {
  size_t sig, third, len, total;
};
InLayout in_layout(size_t C, bool keyed, bool msgs) {
  InLayout L;
  L.sig = round_up(C * (keyed ? 4 : 33), 256);
  L.third = L.sig + C * 64;
  L.len = L.third + C * 8;                        // msgs only
  L.total = msgs ? L.len + C * 4 : L.third + C * 32;
  return L;
}

struct Dev {
  int id = 0;
  uint32_t* gtab = nullptr;
  Set set[2];
  Set gset[2];                                    // host slices: whole-slice key grouping (slice_group); the
                                                  // async lane alternates the two (a slice's grouping under the
                                                  // previous slice's chunks)
  hipEvent_t last_h2d = nullptr;                  // host slice: the previous chunk's H2D (h2d_serial)
  // key arena (gv_keys_load): Q table rows, table Z (8 rows of stride kcap), verdicts
  uint32_t *kqt = nullptr, *kzq = nullptr, *kok = nullptr;
  uint32_t *kqt2 = nullptr, *kzq2 = nullptr;      // the keyed latency schedule's group tables (2^35 Q, ...)
  uint32_t* glat = nullptr;                       // group tables of G / lambda G (k_gen_glat)
  uint32_t* gtab4 = nullptr;                      // k_ecmult_k4's tables of 2^35 G, 2^70 G, 2^100 G (+ lambda)
  uint32_t* gtab6 = nullptr;                      // k_ecmult_k6's full-scalar 24-bit-window tables of 2^(36 t) G (3.5 GiB)
  bool gtab6_failed = false;                      // its allocation failed once: keyed / grouped batches stay on k4
  uint32_t* gtabf = nullptr;                      // k_ecmult_k4<true>'s full-scalar G tables (GV_GF_WORDS, 6 GiB)
  bool gtabf_failed = false;                      // its allocation failed once: k4 keeps the GLV G tables
  bool gtab4_failed = false;                      // gtab4's allocation failed: keyed batches on the 125-doubling ladder
  size_t kcap = 0;
  // the resident kn arena (option "keys_k6"): per slot the GV_KN_ARENA_NG (11)
  // 32-entry group tables of 2^(12 g) Q on one Z (kqt6: group 0, kqt62: groups
  // 1.., kzq6: the Z, 8 rows of stride kcap; kzq62 holds the chain's parked
  // Zs), read by k_ecmult_kn and k_verify_lat16_kn
  uint32_t *kqt6 = nullptr, *kzq6 = nullptr, *kqt62 = nullptr, *kzq62 = nullptr;
  size_t keys6 = 0;                               // leading slots whose k6 tables are built
  // the resident arena's wide-window tables (option "keys_wide"): per slot
  // kw_ng (GV_KW_NG1 = 12: one 11-bit window per group, or GV_KW_NG2 = 6: two;
  // GV_KW_QW, gv_kernels.h) 1,024-entry group tables on one Z (kqtw: group 0, kqtw2:
  // groups 1.., kzqw: the Z, 8 rows of stride kcapw; kzqw2: the chain's parked
  // Zs), in an arena of their own (capacity kcapw) grown by doubling while the
  // HBM budget holds it; keysw leading slots built.  kw_full: the budget
  // refused a growth (no more wide-window builds until gv_keys_reset)
  uint32_t *kqtw = nullptr, *kzqw = nullptr, *kqtw2 = nullptr, *kzqw2 = nullptr;
  size_t kcapw = 0, keysw = 0;
  int kw_ng = 0;
  bool kw_full = false;
  // HBM held by the optional tables (G tables, key arenas) against ctx->hbm_budget
  size_t opt_bytes = 0;
  // ring of per-launch stage events for gv_stage_stats
  static constexpr int kRing = 256;
  hipEvent_t ring[kRing][6] = {};                // start, after unpack / s^-1 / prep, ladder start, ladder end
  int ring_next = 0, ring_count = 0, last = -1;
  // ed25519: the resident comb table and one scratch set
  uint32_t* edtab = nullptr;
  uint32_t* edtab16 = nullptr;                    // the radix-2^16 comb table of B (k_ed_keyed), built on first use
  bool edtab16_failed = false;
  struct Ed {
    size_t cap = 0;                               // lanes
    uint8_t* d_in = nullptr;                      // pub32 | sig64 | off u64 | len u32 (ed_layout)
    uint32_t* atab = nullptr;                     // GV_ED_ROWS rows of cap words
    uint64_t* bits = nullptr;
    uint8_t* d_blob = nullptr;
    size_t blob_cap = 0;
    uint8_t* h_in = nullptr;
    size_t h_in_cap = 0;
    uint8_t* h_blob = nullptr;
    size_t h_blob_cap = 0;
    uint8_t* h_bits = nullptr;
    size_t h_bits_cap = 0;
    hipEvent_t last = nullptr;                    // end of the last work using the scratch
    hipStream_t last_st = nullptr;
  } ed;
  // ed25519 key arena (gv_ed_keys_load): per slot the comb table of -A
  // (GV_EDK_WORDS), the raw key words (8), the FromBytes verdict
  uint32_t *ektab = nullptr, *ekpub = nullptr, *ekok = nullptr;
  size_t ekcap = 0;
  uint8_t* edl_h = nullptr;                       // small keyed ed25519 batches: pinned inputs + verdicts (zero-copy)
  size_t edl_h_cap = 0;
  // ed25519 in-batch key grouping: per-batch key arena (comb tables of -A), pinned count, stats
  uint32_t *edg_ktab = nullptr, *edg_kpub = nullptr, *edg_kok = nullptr;
  size_t edg_cap = 0;
  size_t edg_words = 0;                           // table words per key of edg_ktab (the comb radix in use)
  uint32_t* ed_h_count = nullptr;
  uint64_t ed_grouped_batches = 0, ed_grouped_keys = 0;
  // large keyed ed25519 batches, two buffers (chunk i on set[i % 2]'s stream):
  // pinned staging, device copy, slot-order sort scratch (words)
  uint8_t *edk_h[2] = {nullptr, nullptr}, *edk_d[2] = {nullptr, nullptr};
  size_t edk_h_cap[2] = {0, 0}, edk_d_cap[2] = {0, 0};
  uint32_t* edk_s[2] = {nullptr, nullptr};
  size_t edk_s_cap[2] = {0, 0};
  std::mutex mu;
  Pool* pool = nullptr;                           // staging memcpy threads of this device (owned)
  Worker* worker = nullptr;                       // slice runner (devices 1..n-1 of a context)
  // pipelined device-resident calls on the context stream (gv_dev_verify_*,
  // stream NULL): the front kernels of call k+1 run under call k's ladder
  hipStream_t lo_st[2] = {nullptr, nullptr};
  hipStream_t hi_st[2] = {nullptr, nullptr};      // the ladders of set 0 / set 1 (two_ladders), else hi_st[0]
  hipEvent_t hi_done[2] = {nullptr, nullptr};     // the last ladder enqueued on hi_st[j]
  hipEvent_t bits_ev[2] = {nullptr, nullptr};     // the bitmap write of the last pipelined call of set j
  hipEvent_t bits_wait = nullptr, bits_rec = nullptr;   // the pipelined call being launched (dev_run -> launch)
  hipEvent_t plain_done = nullptr;                // the last non-pipelined call on the context stream
  bool hi_used[2] = {false, false}, plain_used = false, bits_used = false;
  uint64_t grouped_batches = 0, grouped_keys = 0;  // in-batch key grouping taken (gv_group_stats)
  uint64_t routes[GV_ROUTES] = {};                // batches per schedule (gv_route_stats)
  int flip = 0;
  double last_slice_ms = 0;                       // host-buffer calls: this device's slice, wall time
  size_t last_slice_n = 0;
};

int ensure_cap(Set* s, size_t C) {
  if (C <= s->cap) return GV_OK;
  if (s->scratch) { (void)hipFree(s->scratch); s->scratch = nullptr; s->cap = 0; }
  const size_t in_bytes = in_layout(C, false, true).total + C * 32;
  const size_t bytes = in_bytes + C * kLaneWords * 4 + (C / 64) * 8 + 16 * 256;
  if (hipMalloc(&s->scratch, bytes) != hipSuccess) return GV_ENOMEM;
  uint8_t* p = s->scratch;
  auto take = [&](size_t nbytes) { uint8_t* r = p; p += round_up(nbytes, 256); return r; };
  s->d_in = take(in_bytes);
  s->in_x = (uint32_t*)take(C * 8 * 4);
  s->in_pfx = (uint32_t*)take(C * 4);
  s->in_r = (uint32_t*)take(C * 8 * 4);
  s->in_s = (uint32_t*)take(C * 8 * 4);
  s->in_e = (uint32_t*)take(C * 8 * 4);
  s->digits = (uint32_t*)take(C * GV_DIGIT_ROWS * 4);
  s->zq = (uint32_t*)take(C * 8 * 4);
  s->flags = (uint32_t*)take(C * 4);
  s->qtab = (uint32_t*)take(C * GV_QTAB_WORDS * 4);
  s->bits = (uint64_t*)take((C / 64) * 8);
  s->cap = C;
  return GV_OK;
}

int ensure_blob(Set* s, size_t bytes) {
  if (bytes <= s->blob_cap) return GV_OK;
  if (s->d_blob) (void)hipFree(s->d_blob);
  s->blob_cap = round_up(std::max<size_t>(bytes, 1), 1 << 20);
  if (hipMalloc(&s->d_blob, s->blob_cap) != hipSuccess) { s->blob_cap = 0; s->d_blob = nullptr; return GV_ENOMEM; }
  return GV_OK;
}

int ensure_pinned(uint8_t** p, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return GV_OK;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t want = round_up(std::max<size_t>(bytes, 4096), 1 << 20);
  if (hipHostMalloc((void**)p, want, hipHostMallocDefault) != hipSuccess) { *p = nullptr; return GV_ENOMEM; }
  *cap = want;
  return GV_OK;
}

// Order work on stream st after the previous use of set s (any stream).
int set_acquire(Set* s, hipStream_t st) {
  if (s->last_st && s->last_st != st) CK(hipStreamWaitEvent(st, s->last, 0));
  return GV_OK;
}
int set_release(Set* s, hipStream_t st) {
  CK(hipEventRecord(s->last, st));
  s->last_st = st;
  return GV_OK;
}

// Bytes per slot of the resident key arena: the k4 tables (Q table, the three
// group tables, their Zs, the verdict) and, with the k6 arena, its four
// 32-entry group tables and Zs.
size_t key_slot_bytes(bool k6) {
  size_t b = ((size_t)GV_KEY_WORDS * (1 + GV_KEY2_TABLES) + 8 * (1 + GV_KEY2_TABLES) + 1) * 4;
  if (k6) b += ((size_t)GV_K6_KEY_WORDS * GV_KN_ARENA_NG + 8 * GV_KN_ARENA_NG) * 4;
  return b;
}

// Grow the key arena to hold `need` slots, keeping the first `used` (row
// stride of the Z rows changes with the capacity).  Doubling, but not past
// key_cap (the callers' reset point: GV_KEY_CAP or the "key_cap" option) --
// past it the arena grows to exactly what is needed (a caller that never
// resets pays one copy per load, not a quadratic series of doublings).
// k6: the arena also holds the k6 group tables (allocated on the first k6
// load; *k6 is cleared when they do not fit the budget, the k4 tables stay).
int ensure_keys(Dev* d, size_t need, size_t used, hipStream_t st, size_t key_cap, size_t budget, bool* k6) {
  const bool want6 = k6 && *k6;
  if (need <= d->kcap && (!want6 || d->kqt6)) return GV_OK;
  size_t cap = d->kcap;
  if (need > d->kcap) {
    const size_t grow = d->kcap >= key_cap ? need : std::min<size_t>(2 * d->kcap, std::max<size_t>(need, key_cap));
    cap = round_up(std::max<size_t>({need, grow, 4096}), 256);
  }
  const bool has6 = d->kqt6 != nullptr;
  bool alloc6 = want6 || has6;
  // budget: the new arena beside the old one during the copy, plus the other
  // optional tables
  const size_t old_b = d->kcap * key_slot_bytes(has6);
  const size_t base_b = d->opt_bytes - std::min(d->opt_bytes, old_b);
  if (base_b + old_b + cap * key_slot_bytes(alloc6) > budget) {
    if (!alloc6 || has6 || base_b + old_b + cap * key_slot_bytes(false) > budget) return GV_ENOMEM;
    alloc6 = false;                             // no room for the k6 tables: k4 only
    *k6 = false;
    if (need <= d->kcap) return GV_OK;
  }
  uint32_t *qt = nullptr, *zq = nullptr, *ok = nullptr, *qt2 = nullptr, *zq2 = nullptr;
  uint32_t *qt6 = nullptr, *zq6 = nullptr, *qt62 = nullptr, *zq62 = nullptr;
  auto fail = [&]() {
    for (uint32_t* p : {qt, zq, ok, qt2, zq2, qt6, zq6, qt62, zq62}) if (p) (void)hipFree(p);
    (void)hipGetLastError();
    return GV_ENOMEM;
  };
  if (hipMalloc(&qt, cap * GV_KEY_WORDS * 4) != hipSuccess) return fail();
  if (hipMalloc(&zq, cap * 8 * 4) != hipSuccess) return fail();
  if (hipMalloc(&ok, cap * 4) != hipSuccess) return fail();
  if (hipMalloc(&qt2, cap * GV_KEY2_TABLES * GV_KEY_WORDS * 4) != hipSuccess) return fail();
  if (hipMalloc(&zq2, cap * GV_KEY2_TABLES * 8 * 4) != hipSuccess) return fail();
  if (alloc6) {
    if (hipMalloc(&qt6, cap * GV_K6_KEY_WORDS * 4) != hipSuccess) return fail();
    if (hipMalloc(&zq6, cap * 8 * 4) != hipSuccess) return fail();
    if (hipMalloc(&qt62, cap * (GV_KN_ARENA_NG - 1) * GV_K6_KEY_WORDS * 4) != hipSuccess) return fail();
    if (hipMalloc(&zq62, cap * (GV_KN_ARENA_NG - 1) * 8 * 4) != hipSuccess) return fail();
  }
  // the k6 tables of the slots below `used` exist only if the old arena had them
  const size_t used6 = d->kqt6 ? used : 0;
  if (used) {
    CK(hipMemcpyAsync(qt, d->kqt, used * GV_KEY_WORDS * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemcpyAsync(qt2, d->kqt2, used * GV_KEY2_TABLES * GV_KEY_WORDS * 4, hipMemcpyDeviceToDevice, st));
    for (int r = 0; r < 8; ++r)
      CK(hipMemcpyAsync(zq + r * cap, d->kzq + r * d->kcap, used * 4, hipMemcpyDeviceToDevice, st));
    for (int r = 0; r < GV_KEY2_TABLES * 8; ++r)
      CK(hipMemcpyAsync(zq2 + r * cap, d->kzq2 + r * d->kcap, used * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemcpyAsync(ok, d->kok, used * 4, hipMemcpyDeviceToDevice, st));
  }
  if (used6 && alloc6) {
    CK(hipMemcpyAsync(qt6, d->kqt6, used6 * GV_K6_KEY_WORDS * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemcpyAsync(qt62, d->kqt62, used6 * (GV_KN_ARENA_NG - 1) * GV_K6_KEY_WORDS * 4, hipMemcpyDeviceToDevice,
                      st));
    for (int r = 0; r < 8; ++r)
      CK(hipMemcpyAsync(zq6 + r * cap, d->kzq6 + r * d->kcap, used6 * 4, hipMemcpyDeviceToDevice, st));
    for (int r = 0; r < (GV_KN_ARENA_NG - 1) * 8; ++r)
      CK(hipMemcpyAsync(zq62 + r * cap, d->kzq62 + r * d->kcap, used6 * 4, hipMemcpyDeviceToDevice, st));
  }
  if (used) CK(hipStreamSynchronize(st));
  for (uint32_t* p : {d->kqt, d->kzq, d->kok, d->kqt2, d->kzq2, d->kqt6, d->kzq6, d->kqt62, d->kzq62})
    if (p) (void)hipFree(p);
  d->kqt = qt; d->kzq = zq; d->kok = ok; d->kqt2 = qt2; d->kzq2 = zq2;
  d->kqt6 = qt6; d->kzq6 = zq6; d->kqt62 = qt62; d->kzq62 = zq62;
  d->kcap = cap;
  d->opt_bytes = base_b + cap * key_slot_bytes(alloc6);
  return GV_OK;
}

// Bytes per slot of the wide-window tables of ng groups.
constexpr size_t key_wide_slot_bytes(int ng) { return ((size_t)GV_KW_KEY_WORDS * ng + 8 * (size_t)ng) * 4; }

// Grow the wide-window arena to `need` slots keeping the first `used` (doubling, not
// past key_cap, then exact -- as ensure_keys).  Returns false when the budget
// (the new arena beside the old one during the copy) does not hold it, when
// it would take device memory the k4 / k6 arena needs to grow to key_cap
// (plus 8 GiB of batch scratch: these tables are an optimisation and never
// make a later gv_keys_load or batch fail), or when an allocation fails: the
// arena is left as it was and batches keep the k6 tables.
// The layout is d->kw_ng's; cap1 bounds the one-window layout's capacity (a
// test hook, option "keys_wide1_cap").  ed_room: device memory the ed25519
// key arena still needs to reach its own cap (reserved the same way).
bool ensure_keys_wide(Dev* d, size_t need, size_t used, hipStream_t st, size_t key_cap, size_t budget,
                      size_t ed_room, size_t cap1 = SIZE_MAX) {
  if (need <= d->kcapw) return true;
  const size_t grow = d->kcapw >= key_cap ? need : std::min<size_t>(2 * d->kcapw, std::max<size_t>(need, key_cap));
  const size_t cap = round_up(std::max<size_t>({need, grow, 4096}), 256);
  const size_t slot_b = key_wide_slot_bytes(d->kw_ng);
  if (d->kw_ng == GV_KW_NG1 && cap > cap1) return false;
  if (d->opt_bytes + cap * slot_b > budget) return false;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return false;
  const size_t reserve =
      (key_cap > d->kcap ? key_cap - d->kcap : 0) * key_slot_bytes(true) + ed_room + (size_t(8) << 30);
  if (free_b < cap * slot_b + reserve) return false;
  const size_t ng1 = (size_t)d->kw_ng - 1;
  uint32_t *qt = nullptr, *zq = nullptr, *qt2 = nullptr, *zq2 = nullptr;
  if (hipMalloc(&qt, cap * GV_KW_KEY_WORDS * 4) != hipSuccess || hipMalloc(&zq, cap * 8 * 4) != hipSuccess ||
      hipMalloc(&qt2, cap * ng1 * GV_KW_KEY_WORDS * 4) != hipSuccess ||
      hipMalloc(&zq2, cap * ng1 * 8 * 4) != hipSuccess) {
    for (uint32_t* p : {qt, zq, qt2, zq2}) if (p) (void)hipFree(p);
    (void)hipGetLastError();
    return false;
  }
  used = std::min(used, d->keysw);                // the slots whose wide-window tables exist
  if (used) {
    bool ok = hipMemcpyAsync(qt, d->kqtw, used * GV_KW_KEY_WORDS * 4, hipMemcpyDeviceToDevice, st) == hipSuccess &&
              hipMemcpyAsync(qt2, d->kqtw2, used * ng1 * GV_KW_KEY_WORDS * 4, hipMemcpyDeviceToDevice, st) ==
                  hipSuccess;
    for (int r = 0; ok && r < 8; ++r)
      ok = hipMemcpyAsync(zq + r * cap, d->kzqw + r * d->kcapw, used * 4, hipMemcpyDeviceToDevice, st) == hipSuccess;
    for (size_t r = 0; ok && r < ng1 * 8; ++r)
      ok = hipMemcpyAsync(zq2 + r * cap, d->kzqw2 + r * d->kcapw, used * 4, hipMemcpyDeviceToDevice, st) ==
           hipSuccess;
    if (!ok || hipStreamSynchronize(st) != hipSuccess) {
      for (uint32_t* p : {qt, zq, qt2, zq2}) (void)hipFree(p);
      (void)hipGetLastError();
      return false;
    }
  }
  for (uint32_t* p : {d->kqtw, d->kzqw, d->kqtw2, d->kzqw2})
    if (p) (void)hipFree(p);
  d->opt_bytes = d->opt_bytes - std::min(d->opt_bytes, d->kcapw * slot_b) + cap * slot_b;
  d->kqtw = qt; d->kzqw = zq; d->kqtw2 = qt2; d->kzqw2 = zq2;
  d->kcapw = cap;
  return true;
}

// Drop the wide-window arena (its memory back to the device).
void free_keys_wide(Dev* d) {
  for (uint32_t** p : {&d->kqtw, &d->kzqw, &d->kqtw2, &d->kzqw2})
    if (*p) { (void)hipFree(*p); *p = nullptr; }
  d->opt_bytes -= std::min(d->opt_bytes, d->kcapw * key_wide_slot_bytes(d->kw_ng));
  d->kcapw = d->keysw = 0;
}

// ---- ed25519 scratch
struct EdLayout {
  size_t sig, off, len, total;
};
EdLayout ed_layout(size_t C) {                    // C % 256 == 0: every part 256-aligned
  EdLayout L;
  L.sig = C * 32;
  L.off = L.sig + C * 64;
  L.len = L.off + C * 8;
  L.total = L.len + C * 4;
  return L;
}

int ed_ensure(Dev* d, size_t C, hipStream_t st) {
  if (!d->edtab) {                                // one-time: the comb table, built on the device
    if (hipMalloc(&d->edtab, (size_t)GV_ED_BTAB_WORDS * 4) != hipSuccess) { d->edtab = nullptr; return GV_ENOMEM; }
    CK(gvk_ed_btab(d->edtab, st));
    CK(hipStreamSynchronize(st));
  }
  if (!d->ed.last) CK(hipEventCreateWithFlags(&d->ed.last, hipEventDisableTiming));
  if (C <= d->ed.cap) return GV_OK;
  if (d->ed.last_st) CK(hipEventSynchronize(d->ed.last));
  if (d->ed.d_in) (void)hipFree(d->ed.d_in);
  if (d->ed.atab) (void)hipFree(d->ed.atab);
  if (d->ed.bits) (void)hipFree(d->ed.bits);
  d->ed.d_in = nullptr; d->ed.atab = nullptr; d->ed.bits = nullptr; d->ed.cap = 0;
  if (hipMalloc(&d->ed.d_in, ed_layout(C).total) != hipSuccess ||
      hipMalloc(&d->ed.atab, C * (size_t)GV_ED_ROWS * 4) != hipSuccess ||
      hipMalloc(&d->ed.bits, C / 8) != hipSuccess)
    return GV_ENOMEM;
  d->ed.cap = C;
  return GV_OK;
}

// One k_ed_verify launch over n items (device pointers) on stream st.
// ed25519 in-batch key grouping (option "ed_group"): batches of at least
// `min` items with at most items / `div` (and `cap`) distinct keys build each
// key's comb table once (k_ed_keys into a per-batch arena) and verify on
// k_ed_keyed; else the throughput kernels.
struct EdGroupCfg {
  bool on;
  size_t min;
  int div;
  size_t cap;
  bool sorted;
  bool split_keys;   // k_ed_keys_chain + k_ed_keys_tab (the table adds off the serial chain)
  bool btab16;       // k_ed_keyed takes [s]B from the radix-2^16 table
  bool r64;          // the per-batch key tables are radix-64 combs (43 windows of 32 entries)
};

// The radix-2^16 comb table of B, built on the device on first use (56.6 MB);
// null when the option is off or its allocation failed (k_ed_keyed then adds
// [s]B from the radix-256 table: same verdicts).
const uint32_t* ed_btab16(Dev* d, bool on, hipStream_t st) {
  if (!on) return nullptr;
  if (!d->edtab16 && !d->edtab16_failed) {
    uint32_t* t = nullptr;
    if (hipMalloc(&t, GV_ED_BTAB16_WORDS * 4) != hipSuccess) {
      (void)hipGetLastError();
      d->edtab16_failed = true;
    } else if (gvk_ed_btab16(t, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
      (void)hipFree(t);
      (void)hipGetLastError();
      d->edtab16_failed = true;
    } else {
      d->edtab16 = t;
    }
  }
  return d->edtab16;
}

int ensure_edg(Dev* d, size_t need, size_t words) {
  if (need <= d->edg_cap && words == d->edg_words) return GV_OK;
  for (uint32_t** q : {&d->edg_ktab, &d->edg_kpub, &d->edg_kok})
    if (*q) { (void)hipFree(*q); *q = nullptr; }
  d->edg_cap = 0;
  d->edg_words = words;
  const size_t cap = round_up(std::max<size_t>(need, 1024), 1024);
  if (hipMalloc(&d->edg_ktab, cap * words * 4) != hipSuccess ||
      hipMalloc(&d->edg_kpub, cap * 8 * 4) != hipSuccess || hipMalloc(&d->edg_kok, cap * 4) != hipSuccess)
    return GV_ENOMEM;
  d->edg_cap = cap;
  return GV_OK;
}

// The grouped route on the device (scratch: the per-lane table region, which
// the keyed kernel does not use).  *taken = false: the batch has too many
// distinct keys (or no room) and the caller runs the throughput kernels.
int ed_grouped(Dev* d, size_t n, const uint8_t* pub, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
               const uint32_t* len, uint64_t* bits, hipStream_t st, const EdGroupCfg& gc, bool* taken) {
  *taken = false;
  const size_t C = round_up(n, 256);
  size_t T = 512;
  while (T < 2 * n) T <<= 1;
  const size_t capU = std::min(gc.cap, std::max<size_t>(n / (size_t)gc.div, 1));
  const size_t nb = capU + 1, tb = gvk_sort_temp_bytes((uint32_t)nb);
  uint32_t* q = d->ed.atab;
  uint32_t *table = q, *rep = table + T, *uid = rep + C, *slot = uid + C, *count = slot + C;
  uint8_t* kpub32 = (uint8_t*)(count + 64);
  uint32_t* sp = count + 64 + round_up(capU * 8, 64);
  gvk_sort so;
  so.pos = sp;
  so.perm = sp + C;
  so.kslot = sp + 2 * C;
  so.bits = nullptr;
  so.cnt = sp + 3 * C;
  so.off = so.cnt + round_up(nb, 64);
  so.temp = so.off + round_up(nb, 64);
  so.temp_bytes = tb;
  uint32_t* o8 = (uint32_t*)so.temp + round_up(tb / 4 + 1, 64);
  if ((size_t)(o8 + C / 4 - q) > C * (size_t)GV_ED_ROWS) return GV_OK;
  if (!d->ed_h_count && hipHostMalloc((void**)&d->ed_h_count, 64, hipHostMallocDefault) != hipSuccess) {
    d->ed_h_count = nullptr;
    return GV_ENOMEM;
  }
  CK(gvk_ed_group((uint32_t)n, pub, table, (uint32_t)T, rep, uid, count, (uint32_t)capU, kpub32, slot, st));
  CK(hipMemcpyAsync(d->ed_h_count, count, 4, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  const size_t U = *d->ed_h_count;
  if (U == 0 || U > capU || U * (size_t)gc.div > n) return GV_OK;
  uint32_t* wb = o8 + round_up(C / 4, 64);        // window-base scratch of the split key build
  if (!gc.split_keys || (size_t)(wb + U * 64 * 36 - q) > C * (size_t)GV_ED_ROWS) wb = nullptr;
  // radix-64 comb tables (43 additions per [h](-A) instead of 64) on the
  // split build; the one-lane build writes the radix-16 ones
  const int rb = gc.r64 && wb ? 6 : 4;
  int rc = ensure_edg(d, U, rb == 6 ? (size_t)GV_EDK64_WORDS : (size_t)GV_EDK_WORDS);
  if (rc) return rc == GV_ENOMEM ? GV_OK : rc;
  CK(gvk_ed_keys(kpub32, (uint32_t)U, 0u, d->edg_ktab, d->edg_kpub, d->edg_kok, wb, rb, st));
  if (gc.sorted) CK(gvk_sort_slots(&so, (uint32_t)n, slot, (uint32_t)U, st));
  gvk_edk b;
  memset(&b, 0, sizeof b);
  b.n = (uint32_t)n;
  b.perm = gc.sorted ? so.perm : nullptr;
  b.slot = slot;
  b.sig64 = sig;
  b.msg_blob = blob;
  b.msg_off = off;
  b.msg_len = len;
  b.ktab = d->edg_ktab;
  b.kpub = d->edg_kpub;
  b.kok = d->edg_kok;
  b.kcount = (uint32_t)U;
  b.btab = d->edtab;
  b.btab16 = ed_btab16(d, gc.btab16, st);
  b.rb = rb;
  b.out8 = (uint8_t*)o8;
  CK(gvk_ed_keyed(&b, st));
  CK(gvk_ed_pack_bits((uint32_t)n, (const uint8_t*)o8, bits, st));
  d->ed_grouped_batches++;
  d->ed_grouped_keys += U;
  *taken = true;
  return GV_OK;
}

int ed_launch(bool timed, Dev* d, size_t n, const uint8_t* pub, const uint8_t* sig, const uint8_t* blob,
              const uint64_t* off, const uint32_t* len, uint64_t* bits, hipStream_t st, const EdGroupCfg& gc) {
  const size_t C = round_up(n, 256);
  int rc = ed_ensure(d, C, st);
  if (rc) return rc;
  if (d->ed.last_st && d->ed.last_st != st) CK(hipStreamWaitEvent(st, d->ed.last, 0));
  gvk_ed b;
  memset(&b, 0, sizeof b);
  b.n = (uint32_t)n;
  b.C = (uint32_t)C;
  b.pub32 = pub; b.sig64 = sig;
  b.msg_blob = blob; b.msg_off = off; b.msg_len = len;
  b.atab = d->ed.atab;
  b.btab = d->edtab;
  b.btab16 = ed_btab16(d, gc.btab16, st);
  b.bits = bits;
  hipEvent_t* rs = nullptr;
  if (timed) {                                    // stages: (none) x 3 | the ed25519 kernel
    rs = d->ring[d->ring_next];
    for (int i = 0; i < 6; ++i)
      if (!rs[i]) CK(hipEventCreate(&rs[i]));
    for (int i = 0; i < 5; ++i) CK(hipEventRecord(rs[i], st));
  }
  bool grouped = false;
  if (gc.on && n >= gc.min && (rc = ed_grouped(d, n, pub, sig, blob, off, len, bits, st, gc, &grouped))) return rc;
  if (!grouped) CK(gvk_ed_verify(&b, st));
  if (rs) {
    CK(hipEventRecord(rs[5], st));
    d->last = d->ring_next;
    d->ring_next = (d->ring_next + 1) % Dev::kRing;
    d->ring_count = std::min(d->ring_count + 1, Dev::kRing);
  }
  CK(hipEventRecord(d->ed.last, st));
  d->ed.last_st = st;
  return GV_OK;
}

}  // namespace

struct AsyncState;                               // gv_submit_* / gv_wait (below)

struct gv_ctx {
  std::vector<Dev*> devs;
  AsyncState* async = nullptr;                    // created by the first gv_submit_*
  size_t max_batch = size_t(1) << 20;
  size_t lat_max = 8192;        // batches up to this size take a fused small-batch kernel (gv_lat.hip), larger ones the pipeline
  size_t lat_sl_max = 2048;     // ... and up to this size the limb-sliced one (one signature per block); between the two the
                                // four-lanes-per-signature kernel (0.50 ms flat to 8192): profiles/r02/lat_sliced/batch_curve*.json
  // keyed batches (the key arena): the sliced keyed kernel takes 4 waves per
  // signature and the 16-lanes-per-signature kernel beats the k4 pipeline to
  // ~14k (profiles/r02/lat_sliced/keyed_curve.json).  Setting lat_max /
  // lat_sl_max sets these too; lat_max_keyed / lat_sl_max_keyed only these.
  size_t lat_max_keyed = 14336;
  size_t lat_sl_max_keyed = 1536;
  size_t pipe_chunk = 262144;   // host path: first chunk of the two-set copy/compute pipeline (0 = max_batch;
                                // profiles/r03/hostpath_sweep.jsonl: 262144 x 4 steadiest on pageable input)
  int pipe_growth = 4;          // host path: each later chunk at most this times the one before
  int stage_pieces = 2;         // host path, pageable chunks of >= 65,536 items: staged in this many pieces, each
                                // piece's H2D behind its copy (1 = one copy then one H2D; GV_STAGE_PIECES):
                                // 121.4 / 129.4 / 126.2 / 126.8M/s at 1 / 2 / 4 / 8 (profiles/r04/hostpath/stage_pieces_ab.jsonl)
  size_t async_chunk = 262144;  // submitted batches staged through the library (pageable, messages): fixed chunks
  int async_growth = 1;         // of this size growing by async_growth (GV_ASYNC_CHUNK, GV_ASYNC_GROWTH;
                                // "async_chunk" / "async_growth"): the copy of one chunk overlaps the others
  bool async_whole = true;      // submitted batches read in place (the caller's pinned buffers): a slice behind
                                // one still in flight is ONE chunk (its H2D and front run under the previous
                                // ladder), a slice on an idle device takes the synchronous ramp (GV_ASYNC_WHOLE,
                                // "async_whole").  1M pinned batches: 4.6 ms each steady vs 5.2 ms in 262,144-item
                                // chunks (a 262,144-item ladder is 1,024 blocks = 1.33 rounds of the chip's 768
                                // resident ones, and the next one only starts as it drains); pageable batches in
                                // one chunk lose the copy overlap (143 vs 177M/s): profiles/r06/async/
  bool host_ladder_stream = false;  // host chunks' ladders on the set's low-priority ladder stream (chunk_ladder;
                                    // GV_HOST_LADDER_STREAM=1).  Measured off: async pinned 185 vs 157-167M/s,
                                    // sync pinned 158-160 vs 150-152M/s (profiles/r05/async_ab.jsonl)
  size_t lane_burst = 16;       // submitted batches: slices an async lane runs before it drains and releases the
                                // device lock (GV_LANE_BURST)
  bool lat_kw = true;           // keyed small batches on the wide arena's one-window tables (k_verify_lat16_kw)
                                // when every slot has them, else the kn tables (GV_LAT_KW, "lat_kw")
  bool h2d_serial = true;       // host slices: a chunk's H2D waits for the previous chunk's, so concurrent
                                // transfers do not share the link and delay the chunk the GPU needs first
                                // (GV_H2D_SERIAL)
  bool gfull_item = true;       // the per-item (pub33, ungrouped) route takes G on the unsplit u1 too: 11 G
                                // additions from the full-scalar tables instead of 14 (GV_GFULL_ITEM)
  bool inv_small = true;        // k_scalar_inv folds fewer signatures per lane below 2^19 items (gvk_inv_m);
                                // 0: GV_INV_M always (GV_INV_SMALL)
  size_t slice_plain_first = 0; // host path, slices to be grouped: this many items first on the per-item pipeline,
                                // submitted before the rest's keys are sent, grouped and tabulated (0 = off;
                                // GV_SLICE_PLAIN_FIRST)
  int stage_threads = 8;        // host path: staging threads per device, its slice's thread included (gv_open:
                                // gvstage::stage_pool_threads -- half the process's CPUs, affinity capped by
                                // the cgroup quota, split over the devices, 1..8 each)
  bool time_kernels = false;
  bool fault_inject = false;
  bool lat_zero_copy = true;    // host-buffer batches on the sliced kernels read the pinned staging buffer and write
                                // verdict bytes to pinned memory directly: no H2D, memset or D2H (GV_LAT_ZC=0: A/B)
  bool lat_sliced = true;       // small batches on k_verify_lat_sl / k_verify_lat16_sl (GV_LAT_SLICED=0: the one-lane-field kernels, A/B)
  size_t lat_rows_max = 512;     // pub33 small batches of at most this many: k_verify_lat_sl4 (rows of a wave on one accumulator, G from gtab6); 0: k_verify_lat_sl
  bool keyed_k4 = true;         // keyed batches on k_ecmult_k4 (GV_KEYED_K4=0: the 125-doubling ladder, A/B)
  bool gfull = true;            // k4 batches take G on the unsplit scalar: 11 25-bit windows instead of 14 20-bit
                                // GLV windows (k_ecmult_k4<true>, 6 GiB of tables; GV_GFULL=0: A/B)
  bool k6 = false;              // grouped batches on k_ecmult_k6: 6-bit Q windows on 32-entry key tables, the lambda
                                // frame, G on the unsplit u1 in 24-bit windows (GV_K6=1)
  int kg = 0;                   // grouped batches on k_ecmult_kn<5, kg>: k4's 16-entry 5-bit tables over kg groups
                                // (one of GV_KG_NGS; 0 = k_ecmult_k4), G after the last doubling from the 24-bit
                                // tables on the real curve (GV_KG, "kg"; takes precedence over k6).  Off: with
                                // the unsplit key chain k4 stays ahead -- 223 vs 215-218M/s for kg 4 (its
                                // ladder 2-3 % shorter, but at 126 VGPRs x 4 waves the next call's front kernels
                                // no longer co-reside), 7 / 9 groups cut the ladder 10-17 % and cost more in the
                                // front (217 / 210M/s; profiles/r06/ab/ab3, ab4)
  int keys_wide = 2;            // ... and wide-window tables while device memory holds them (GV_KEYS_WIDE): 2 = one
                                // GV_KW_QW-bit window per group (11: 12 groups of 1,024 entries, no doublings, 24 Q
                                // additions), moving to two per group (6 groups, 11 doublings) when that no longer fits;
                                // 1 = two per group; 0 = none
  size_t keys_wide1_cap = SIZE_MAX;   // test hook: the one-window layout's slot capacity ("keys_wide1_cap")
  bool keys_k6 = true;          // the resident arena (gv_keys_load) also holds k6 tables and its throughput batches
                                // run k_ecmult_k6: the table build is paid once per key, not per batch (GV_KEYS_K6)
  size_t key_cap = GV_KEY_CAP;  // the callers' key-arena reset point: growth doubles up to here ("key_cap", GV_KEY_CAP)
  size_t ed_key_cap = GV_ED_KEY_CAP;   // the same for the ed25519 arena ("ed_key_cap", GV_ED_KEY_CAP)
  size_t hbm_budget = SIZE_MAX; // bytes of optional device tables per device (G tables, key arenas; "hbm_budget_mb",
                                // GV_HBM_BUDGET_MB): a table past it is not built and batches take the schedule
                                // that needs less, with the same verdicts
  bool pipeline_dev = true;     // pipelined device-resident calls on the context stream (dev_run; GV_PIPELINE=0: A/B)
  bool two_ladders = true;      // ... whose ladders alternate two high-priority streams, so the next ladder starts in
                                // the current one's tail (bitmap writes kept in call order; GV_TWO_LADDERS=0: A/B)
  bool group_keys = true;       // pub33 throughput batches parse each distinct key once (group_keys; GV_GROUP_KEYS=0: A/B)
  bool keys_scratch = true;     // key tables: forward entries through coalesced scratch rows (GV_KEYS_SCRATCH=0: A/B)
  bool sort_keys = true;        // keyed k4 batches run their lanes in slot order (gv_sort.hip; GV_SORT_KEYS=0: A/B)
  size_t group_min = 16384;     // ... batches of at least this many items
  int group_div = 5;            // ... taking the keyed pipeline when distinct keys <= items / group_div (break-even ~4:
                                // a key build ~18 ns vs ~4 ns saved per item, profiles/r03/group_ab)
  size_t keys = 0;              // key-arena slots in use (same on every device)
  std::atomic<uint64_t> keys_gen{0};  // gv_keys_reset calls
  std::mutex keys_mu;
  // ed25519 key arena (gv_ed_keys_load), same on every device
  size_t ed_keys = 0;
  std::atomic<uint64_t> ed_keys_gen{0};
  std::mutex ed_keys_mu;
  std::vector<uint8_t> ed_kpub;  // the raw keys per slot (large keyed batches run the throughput kernels on them)
  bool ed_group = true;          // ed25519 throughput batches: in-batch key grouping + k_ed_keyed (GV_ED_GROUP=0: A/B)
  size_t ed_group_min = 196608;  // ... from this many items (the key build's chain is ~1 ms of one-lane chains whatever
                                 // the key count up to ~65k keys; the keyed kernel saves ~6.4 ns per item; host
                                 // chunks of 262,144 qualify)
  int ed_group_div = 16;         // ... with at most items / ed_group_div distinct keys
  size_t ed_group_cap = 16384;   // ... and at most this many (72 KB of comb table per key)
  bool ed_keys_split = true;     // ed25519 key tables: serial chain and table adds in two launches (GV_ED_KEYS_SPLIT=0: A/B)
  bool ed_btab16 = true;         // k_ed_keyed's [s]B from the radix-2^16 table: 16 additions instead of 32 (GV_ED_BTAB16)
  bool ed_group_r64 = true;      // grouped ed25519 key tables as radix-64 combs: 43 [h](-A) additions, not 64 (GV_ED_GROUP_R64)
  bool ed_keyed = true;          // keyed ed25519 batches past ed_lat_max on k_ed_keyed (GV_ED_KEYED=0: the throughput kernels)
  size_t ed_lat_max = 2048;      // keyed ed25519 batches up to this size take k_ed_lat_sl (one signature per block)
  size_t ed_unc_lat_max = 2048;  // uncached ed25519 host batches up to this size take k_ed_lat_unc (one signature per block)
};

namespace {

EdGroupCfg ed_group_cfg(const gv_ctx* ctx) {
  return EdGroupCfg{ctx->ed_group, ctx->ed_group_min, ctx->ed_group_div, ctx->ed_group_cap, ctx->sort_keys,
                    ctx->ed_keys_split, ctx->ed_btab16, ctx->ed_group_r64};
}

// Optional device tables (the G tables past the 64 MiB GLV pair, the key
// arenas) are allocated against the context's HBM budget (gv_set_option
// "hbm_budget_mb", env GV_HBM_BUDGET_MB; default: whatever hipMalloc grants).
// A table that does not fit is remembered as failed and the batches take the
// schedule that needs less (k6 -> k4 -> the 125-doubling keyed ladder; the
// full-scalar G tables -> the GLV G windows) with the same verdicts.
uint32_t* opt_alloc(gv_ctx* ctx, Dev* d, size_t bytes) {
  if (d->opt_bytes + bytes > ctx->hbm_budget) return nullptr;
  uint32_t* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  d->opt_bytes += bytes;
  return p;
}
void opt_free(Dev* d, uint32_t*& p, size_t bytes) {
  if (!p) return;
  (void)hipFree(p);
  p = nullptr;
  d->opt_bytes -= std::min(d->opt_bytes, bytes);
}
constexpr size_t kGtab4Bytes = (size_t)GV_KEY2_TABLES * 2 * GV_GTAB_N * 16 * 4;

// Build one G table set on stream st (set s is a scratch set with capacity >=
// 256: its flags rows hold the base points).  Enqueued only; the caller syncs.
template <class GEN>
int gen_table(Set* s, hipStream_t st, GEN&& gen) {
  int rc;
  if ((rc = ensure_cap(s, 256))) return rc;
  if ((rc = set_acquire(s, st))) return rc;
  if (gen(s->flags) != hipSuccess) return GV_EHIP;
  return set_release(s, st);
}

// The full-scalar G tables (GV_GF_WORDS, 6 GiB: k_ecmult_k4<true> and the
// per-item route's k_ecmult<false, true>), the 20-bit-window tables of 2^35 G,
// 2^70 G, 2^100 G and their lambda images (k_ecmult_k4, 192 MiB) and the k6
// ladder's full-scalar 24-bit-window tables (GV_K6_GTAB_WORDS, 3.5 GiB):
// built at gv_open on every device at once (gv_open: enqueue on each device,
// then one sync each; ~0.5 s), or on first use after an option switched a
// schedule on.  sync = false: enqueue only.
int ensure_gtabf(gv_ctx* ctx, Dev* d, Set* s, hipStream_t st, bool sync = true) {
  if (d->gtabf || !ctx->gfull || d->gtabf_failed) return GV_OK;
  uint32_t* tf = opt_alloc(ctx, d, GV_GF_WORDS * 4);
  if (!tf) { d->gtabf_failed = true; return GV_OK; }
  int rc = gen_table(s, st, [&](uint32_t* sc) { return gvk_gen_gtablef(tf, sc, st); });
  if (!rc && sync && hipStreamSynchronize(st) != hipSuccess) rc = GV_EHIP;
  if (rc) { opt_free(d, tf, GV_GF_WORDS * 4); return rc; }
  d->gtabf = tf;
  return GV_OK;
}

int ensure_gtab4(gv_ctx* ctx, Dev* d, Set* s, hipStream_t st, bool sync = true) {
  if (!ctx->keyed_k4) return GV_OK;
  if (!d->gtab4 && !d->gtab4_failed) {
    uint32_t* t4 = opt_alloc(ctx, d, kGtab4Bytes);
    if (!t4) {
      d->gtab4_failed = true;                   // keyed batches keep k_ecmult<true>
      return GV_OK;
    }
    int rc = gen_table(s, st, [&](uint32_t* sc) { return gvk_gen_gtable4(t4, sc, st); });
    if (!rc && sync && hipStreamSynchronize(st) != hipSuccess) rc = GV_EHIP;
    if (rc) { opt_free(d, t4, kGtab4Bytes); return rc; }
    d->gtab4 = t4;
  }
  return ensure_gtabf(ctx, d, s, st, sync);
}

// k_ecmult_k6's G tables.  A failure is remembered and keyed / grouped batches
// stay on k4.  `want`: the schedule is on (ctx->k6 for the grouped route,
// ctx->keys_k6 for the resident arena).
int ensure_gtab6(gv_ctx* ctx, Dev* d, Set* s, hipStream_t st, bool want, bool sync = true) {
  if (d->gtab6 || !want || d->gtab6_failed) return GV_OK;
  uint32_t* t6 = opt_alloc(ctx, d, GV_K6_GTAB_WORDS * 4);
  if (!t6) { d->gtab6_failed = true; return GV_OK; }
  int rc = gen_table(s, st, [&](uint32_t* sc) { return gvk_gen_gtable6(t6, sc, st); });
  if (!rc && sync && hipStreamSynchronize(st) != hipSuccess) rc = GV_EHIP;
  if (rc) { opt_free(d, t6, GV_K6_GTAB_WORDS * 4); return rc; }
  d->gtab6 = t6;
  return GV_OK;
}

// The set's per-batch key arena for in-batch grouping (cap keys; k6: 32-entry
// group tables), charged to the HBM budget like the other optional tables.
// ent: words per group table (GV_KEY_WORDS: 16 entries; GV_K6_KEY_WORDS: 32),
// ng: groups per key (4; the kg layouts GV_KG_NGS).
size_t group_arena_bytes(size_t cap, int ent, int ng) {
  return cap * ((size_t)ent * 4 * ng + 8 * 4 * ng + 4);
}
int ensure_group_arena(gv_ctx* ctx, Dev* d, Set* s, size_t cap, int ent, int ng) {
  if (cap <= s->gcap && ent == s->g_ent && ng == s->g_ng) return GV_OK;
  for (uint32_t** p : {&s->g_kqt, &s->g_kzq, &s->g_kok, &s->g_kqt2, &s->g_kzq2})
    if (*p) { (void)hipFree(*p); *p = nullptr; }
  if (s->gcap) d->opt_bytes -= std::min(d->opt_bytes, group_arena_bytes(s->gcap, s->g_ent, s->g_ng));
  s->gcap = 0;
  s->g_ent = ent;
  s->g_ng = ng;
  const size_t eb = (size_t)ent * 4;
  if (d->opt_bytes + group_arena_bytes(cap, ent, ng) > ctx->hbm_budget) return GV_ENOMEM;
  if (hipMalloc(&s->g_kqt, cap * eb) != hipSuccess || hipMalloc(&s->g_kzq, cap * 8 * 4) != hipSuccess ||
      hipMalloc(&s->g_kok, cap * 4) != hipSuccess ||
      hipMalloc(&s->g_kqt2, cap * (ng - 1) * eb) != hipSuccess ||
      hipMalloc(&s->g_kzq2, cap * (ng - 1) * 8 * 4) != hipSuccess) {
    (void)hipGetLastError();
    for (uint32_t** p : {&s->g_kqt, &s->g_kzq, &s->g_kok, &s->g_kqt2, &s->g_kzq2})
      if (*p) { (void)hipFree(*p); *p = nullptr; }
    return GV_ENOMEM;
  }
  s->gcap = cap;
  d->opt_bytes += group_arena_bytes(cap, ent, ng);
  return GV_OK;
}

// In-batch key grouping for a pub33 throughput batch of n items (b prepared
// for the pub33 pipeline, inputs on the device): the SoA rows are unpacked,
// the items grouped by key (k_dedupe*), and when the batch has at most
// n / group_div distinct keys their tables are built once into the set's
// batch arena and b is switched to the keyed pipeline with the key id as
// slot.  Scratch: the set's per-lane Q-table region (unused by the keyed
// pipeline; the pub33 pipeline rewrites it).  One 4-byte read-back (the
// distinct-key count) decides the route.
int group_keys(gv_ctx* ctx, Dev* d, Set* s, gvk_batch& b, size_t n, hipStream_t st, uint32_t** used_end = nullptr) {
  const size_t C = b.C;
  size_t T = 512;
  while (T < 2 * n) T <<= 1;
  const size_t capU = round_up(std::max<size_t>(C / ctx->group_div, 256), 256);
  uint32_t* q = s->qtab;
  uint32_t *rep = q, *uid = q + C, *kslot = q + 2 * C, *count = q + 3 * C, *table = q + 3 * C + 256;
  uint32_t* kx = table + T;
  uint32_t* kpfx = kx + 8 * capU;
  uint32_t* sc = kpfx + capU;                   // the key-table build's scratch rows (gvk_keys_scratch_words)
  const size_t used = (size_t)(sc - q), total = (size_t)GV_QTAB_WORDS * C;
  const size_t room = used < total ? total - used : 0;
  if (gvk_keys_scratch_words((uint32_t)capU, GV_LGRP, GV_QTAB_N, 0) > room) return GV_OK;   // no room: pub33
  const bool k6_room = gvk_keys_scratch_words((uint32_t)capU, 4, GV_K6_NT, 0) <= room;
  const int kgng = ctx->kg;                     // 0 or one of GV_KG_NGS
  const bool kg_room = kgng && gvk_keys_scratch_words((uint32_t)capU, kgng, GV_QTAB_N, 0) <= room;
  if (!s->h_count && hipHostMalloc((void**)&s->h_count, 64, hipHostMallocDefault) != hipSuccess) {
    s->h_count = nullptr;
    return GV_ENOMEM;
  }
  int rc = GV_OK;
  // the key rows only: the signature / digest rows follow in gvk_verify, in
  // item order or (keyed, key-ordered lanes) in slot order
  CK(gvk_unpack(b.pub33, nullptr, nullptr, (uint32_t)n, (uint32_t)C, b.in_x, b.in_pfx, b.in_r, b.in_s, b.in_e, st));
  b.unpacked = 2;
  CK(gvk_dedupe((uint32_t)n, (uint32_t)C, b.in_x, b.in_pfx, table, (uint32_t)T, rep, uid, count, kslot,
                (uint32_t)capU, (uint32_t)capU, kx, kpfx, st));
  CK(hipMemcpyAsync(s->h_count, count, 4, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  const size_t U = *s->h_count;
  if (U == 0 || U * ctx->group_div > n || U > capU) return GV_OK;   // many distinct keys: the pub33 pipeline
  // the layout: kg (5-bit windows over kgng groups) > k6 (6-bit, 4 groups) > k4,
  // each needing gtab6 (kg, k6) and its arena within the HBM budget
  if (((ctx->k6 && k6_room) || kg_room) && (rc = ensure_gtab6(ctx, d, s, st, true))) return rc;
  // the arena for the set's whole capacity when the budget holds it: a later,
  // larger chunk on this set does not regrow it (hipFree waits for the device)
  auto arena = [&](int ent, int ng) {
    const size_t capA = round_up(std::max<size_t>(s->cap / ctx->group_div, 256), 256);
    if (capA > capU && !(capA <= s->gcap && ent == s->g_ent && ng == s->g_ng)) {
      const int r = ensure_group_arena(ctx, d, s, capA, ent, ng);
      if (r != GV_ENOMEM) return r;
    }
    return ensure_group_arena(ctx, d, s, capU, ent, ng);
  };
  bool kg = kg_room && d->gtab6;
  if (kg && (rc = arena(GV_KEY_WORDS, kgng))) {
    if (rc != GV_ENOMEM) return rc;
    kg = false;                                 // no room for kgng groups
  }
  bool k6 = !kg && ctx->k6 && k6_room && d->gtab6;
  if (k6 && (rc = arena(GV_K6_KEY_WORDS, GV_LGRP))) {
    if (rc != GV_ENOMEM) return rc;
    k6 = false;                                 // no room for the 32-entry tables: k4
  }
  if (!kg && !k6 && (rc = ensure_gtab4(ctx, d, s, st))) return rc;
  if (!kg && !k6 && (rc = arena(GV_KEY_WORDS, GV_LGRP)))
    return rc == GV_ENOMEM ? GV_OK : rc;
  // the tables are built on the set's side stream while k_scalar_inv (which
  // does not read keys) runs on st: both are one wave per SIMD or so
  CK(hipEventRecord(s->fork, st));
  CK(hipStreamWaitEvent(s->side, s->fork, 0));
  // the forward pass's entries in coalesced scratch rows after the ratio and
  // E rows, when they fit (else through the tables themselves)
  const int nt = k6 ? GV_K6_NT : GV_QTAB_N, ng = kg ? kgng : GV_LGRP;
  const int with_qe = ctx->keys_scratch && gvk_keys_scratch_words((uint32_t)U, ng, nt, 1) <= room ? 1 : 0;
  if (kg)
    CK(gvk_keys_build_rows_kg((uint32_t)U, (uint32_t)capU, kx, kpfx, sc, with_qe, s->g_kqt, s->g_kzq,
                              (uint32_t)capU, s->g_kok, s->g_kqt2, s->g_kzq2, kgng, s->side));
  else if (k6)
    CK(gvk_keys_build_rows6((uint32_t)U, (uint32_t)capU, kx, kpfx, sc, with_qe, s->g_kqt, s->g_kzq, (uint32_t)capU,
                            s->g_kok, s->g_kqt2, s->g_kzq2, s->side));
  else
    CK(gvk_keys_build_rows((uint32_t)U, (uint32_t)capU, kx, kpfx, sc, with_qe, s->g_kqt, s->g_kzq, (uint32_t)capU,
                           s->g_kok, s->g_kqt2, s->g_kzq2, s->side));
  if (used_end) *used_end = sc + gvk_keys_scratch_words((uint32_t)U, ng, nt, with_qe);
  CK(hipEventRecord(s->keys_done, s->side));
  b.keys_ready = s->keys_done;
  b.pub33 = nullptr;
  b.kslot = kslot; b.kqt = s->g_kqt; b.kzq = s->g_kzq; b.kok = s->g_kok;
  b.kC = (uint32_t)capU; b.kcount = (uint32_t)U;
  b.kqt2 = s->g_kqt2; b.gtab4 = d->gtab4;       // null gtab4: the 125-doubling keyed ladder
  b.gtabf = ctx->gfull ? d->gtabf : nullptr;    // built by ensure_gtab4 above on first use
  b.k6 = kg ? kgng : k6 ? 4 : 0; b.gtab6 = d->gtab6;
  b.kqw = kg ? 2 : 0;
  d->grouped_batches++;
  d->grouped_keys += U;
  return GV_OK;
}

// Key-ordered lanes (gv_sort.hip) for a keyed k4 batch: scratch from word
// `base` of the set's Q-table region (unused by the keyed pipeline past the
// grouping rows); no room or the option off: item order.
void plan_sort(gv_ctx* ctx, Set* s, gvk_batch& b, uint32_t* base) {
  if (!ctx->sort_keys || !b.kslot || !(b.gtab4 || (b.k6 && b.gtab6))) return;
  const size_t C = b.C, nb = (size_t)b.kcount + 1;
  const size_t tb = gvk_sort_temp_bytes((uint32_t)nb);
  uint32_t* p = s->qtab + round_up((size_t)(base - s->qtab), 64);
  gvk_sort so;
  so.pos = p; p += C;
  so.perm = p; p += C;
  so.kslot = p; p += C;
  so.bits = (uint64_t*)p; p += C / 32;
  so.cnt = p; p += round_up(nb, 64);
  so.off = p; p += round_up(nb, 64);
  so.temp = p; p += round_up(tb / 4 + 1, 64);
  so.temp_bytes = tb;
  if ((size_t)(p - s->qtab) > (size_t)GV_QTAB_WORDS * C) return;
  b.srt = so;
}

// A key arena other than the device's gv_keys_load arena: a host slice's
// grouped keys (slice_group).  The launch stream waits on `ready` first.
struct KeyArena {
  const uint32_t *kqt, *kzq, *kok, *kqt2, *kzq2;
  uint32_t kC, kcount;
  const uint32_t* gtab4;
  const uint32_t* gtab6;
  int k6;                                       // k6 / kg group tables: the throughput pipeline only
  int kqw;                                      // 2: the kg layout (gvk_batch kqw)
  hipEvent_t ready;
};

// A chunk past the ramp's first size grows its set straight to a whole
// max_batch chunk (device scratch, pinned staging, the grouping arena): a
// regrowth costs tens of ms (hipFree waits for the device, pinning pages), so
// it happens once -- not again when a larger chunk, a queued whole slice or a
// host-buffer call follows device-resident calls of another size.
size_t grow_items(const gv_ctx* ctx, size_t C) {
  return ctx->pipe_chunk && C > ctx->pipe_chunk ? std::max(C, round_up(ctx->max_batch, 256)) : C;
}

// Launch the pipeline for n items whose inputs already sit on the device, on
// set s's scratch, stream st.  The caller holds d->mu.
// st_ecm (pipelined device-resident calls): the ladder runs there, after the
// front kernels on st; the set's scratch is released on st_ecm.
int launch(gv_ctx* ctx, Dev* d, Set* s, size_t n, const uint8_t* pub, const uint8_t* sig, const uint8_t* dig,
           const uint8_t* blob, const uint64_t* off, const uint32_t* len, uint64_t* bits_out,
           hipStream_t st, const uint32_t* kslot = nullptr, uint8_t* out8 = nullptr, hipStream_t st_ecm = nullptr,
           const KeyArena* ka = nullptr, bool no_group = false) {
  if (n == 0 || n > kMaxItems) return GV_EINVAL;
  const size_t C = round_up(n, 256);
  int rc = ensure_cap(s, grow_items(ctx, C));
  if (rc) return rc;
  if (kslot && !ka) {                           // the arena always exists for a keyed batch
    rc = ensure_keys(d, 1, ctx->keys, st, ctx->key_cap, ctx->hbm_budget, nullptr);
    if (rc) return rc;
  }
  rc = set_acquire(s, st);
  if (rc) return rc;
  gvk_batch b;
  memset(&b, 0, sizeof b);
  b.n = (uint32_t)n; b.C = (uint32_t)C;
  b.pub33 = pub; b.sig64 = sig; b.dig32 = dig;
  b.msg_blob = blob; b.msg_off = off; b.msg_len = len;
  b.gtab = d->gtab;
  b.gtabf = ctx->gfull ? d->gtabf : nullptr;
  b.in_x = s->in_x; b.in_pfx = s->in_pfx; b.in_r = s->in_r; b.in_s = s->in_s; b.in_e = s->in_e;
  b.digits = s->digits; b.zq = s->zq; b.flags = s->flags; b.qtab = s->qtab;
  b.bits = bits_out;
  b.inv_m = ctx->inv_small ? 0u : (uint32_t)GV_INV_M;
  const uint32_t* kzq2 = d->kzq2;
  if (kslot && ka) {                            // a host slice's grouped keys
    b.pub33 = nullptr;
    b.kslot = kslot; b.kqt = ka->kqt; b.kzq = ka->kzq; b.kok = ka->kok;
    b.kC = ka->kC; b.kcount = ka->kcount;
    b.kqt2 = ka->kqt2; b.gtab4 = ka->gtab4;
    b.k6 = ka->k6; b.kqw = ka->kqw; b.gtab6 = ka->gtab6;
    kzq2 = ka->kzq2;
    // the slots are on the device already (slice_group read the key count
    // back after k_dedupe_map); only k_prep on reads the tables, so the
    // chunk's unpack / sort / s^-1 overlap the slice's table build
    b.keys_ready = ka->ready;
  } else if (kslot) {
    b.pub33 = nullptr;
    b.kslot = kslot; b.kqt = d->kqt; b.kzq = d->kzq; b.kok = d->kok;
    b.kC = (uint32_t)d->kcap; b.kcount = (uint32_t)ctx->keys;
    b.kqt2 = d->kqt2; b.gtab4 = d->gtab4;       // null: the 125-doubling keyed ladder
  }
  hipEvent_t* rs = nullptr;
  if (ctx->time_kernels) {
    rs = d->ring[d->ring_next];
    for (int i = 0; i < 6; ++i)
      if (!rs[i]) CK(hipEventCreate(&rs[i]));
    CK(hipEventRecord(rs[0], st));
    for (int i = 0; i < 3; ++i) b.ev[i] = rs[i + 1];
    b.ev_ecm_start = rs[4];
    b.ev[3] = rs[5];
  }
  // k6 group tables (a grouped slice's chunks) are read by k_ecmult_k6 only:
  // such a chunk takes the pipeline whatever its size
  const bool small = n <= (kslot ? ctx->lat_max_keyed : ctx->lat_max) && !b.k6;
  const bool pipelined = st_ecm != nullptr && !small;
  // the resident arena's k6 tables (every slot in use has them): throughput
  // batches on k_ecmult_k6; the small-batch kernels keep the k4 tables
  if (kslot && !ka && !small && ctx->keys_wide && d->kqtw && d->kw_ng && d->gtab6 && d->keysw >= ctx->keys) {
    // the wide-window tables (their own arena: Z rows of stride kcapw)
    b.kqt = d->kqtw; b.kzq = d->kzqw; b.kqt2 = d->kqtw2; b.kC = (uint32_t)d->kcapw;
    b.k6 = d->kw_ng; b.kqw = 1; b.gtab6 = d->gtab6;
  } else if (kslot && !ka && !small && ctx->keys_k6 && d->kqt6 && d->gtab6 && d->keys6 >= ctx->keys) {
    b.kqt = d->kqt6; b.kzq = d->kzq6; b.kqt2 = d->kqt62;
    b.k6 = GV_KN_ARENA_NG; b.gtab6 = d->gtab6;
  }
  if (pipelined) {
    b.st_ecm = st_ecm;
    b.ecm_ready = s->ecm_ready;
    b.bits_wait = d->bits_wait;
    b.bits_done = d->bits_rec;
  }
  if (small) {
    // small batch: one fused kernel, several lanes per signature (gv_lat.hip)
    if (b.keys_ready) CK(hipStreamWaitEvent(st, b.keys_ready, 0));   // a host slice's tables
    gvk_lat lb;
    memset(&lb, 0, sizeof lb);
    lb.n = (uint32_t)n; lb.C = (uint32_t)C;
    lb.pub33 = pub; lb.sig64 = sig; lb.dig32 = dig;
    lb.msg_blob = blob; lb.msg_off = off; lb.msg_len = len;
    lb.gtab = d->gtab; lb.e_soa = s->in_e; lb.bits = bits_out;
    lb.ev[0] = b.ev[0];
    if (!kslot && n <= ctx->lat_rows_max) lb.gtab6 = d->gtab6;   // k_verify_lat_sl4 (null: not built)
    if (kslot) {
      lb.pub33 = nullptr;
      lb.kslot = kslot; lb.kqt = b.kqt; lb.kzq = b.kzq; lb.kok = b.kok; lb.kC = b.kC; lb.kcount = b.kcount;
    }
    const bool sliced = ctx->lat_sliced && n <= (kslot ? ctx->lat_sl_max_keyed : ctx->lat_sl_max);
    if (out8 && !sliced) return GV_EINVAL;      // byte verdicts: the sliced kernels only
    lb.out8 = out8;
    d->routes[kslot ? GV_ROUTE_LAT_KEYED : GV_ROUTE_LAT]++;
    if (kslot) {                                // keyed: 16 lanes per signature (group tables)
      lb.kqt2 = b.kqt2; lb.kzq2 = kzq2; lb.glat = d->glat;
      if (sliced && !ka && ctx->keys_wide && ctx->lat_kw && d->kqtw && d->kw_ng == GV_KW_NG1 && d->gtab6 &&
          d->keysw >= ctx->keys) {
        // every slot has its one-window wide tables: k_verify_lat16_kw (no
        // doublings; their own arena: Z rows of stride kcapw)
        lb.kqt = d->kqtw; lb.kzq = d->kzqw; lb.kqt2 = d->kqtw2; lb.kzq2 = nullptr; lb.kC = (uint32_t)d->kcapw;
        lb.gtab6 = d->gtab6; lb.kn = 2;
      } else if (sliced && !ka && ctx->keys_k6 && d->kqt6 && d->gtab6 && d->keys6 >= ctx->keys) {
        // every slot has its kn tables: k_verify_lat16_kn (6 doublings, G from the 24-bit tables)
        lb.kqt = d->kqt6; lb.kzq = d->kzq6; lb.kqt2 = d->kqt62; lb.kzq2 = nullptr;
        lb.gtab6 = d->gtab6; lb.kn = 1;
      }
      if (sliced) CK(gvk_verify_lat16_sl(&lb, st));
      else CK(gvk_verify_lat16(&lb, st));
    } else if (sliced) {
      CK(gvk_verify_lat_sl(&lb, st));
    } else {
      CK(gvk_verify_lat(&lb, st));
    }
    if (rs) {                                   // stages: SHA | fused kernel | (none) | (none)
      CK(hipEventRecord(rs[2], st));
      CK(hipEventRecord(rs[3], st));
      CK(hipEventRecord(rs[4], st));
      CK(hipEventRecord(rs[5], st));
    }
  } else {
    uint32_t* sort_base = s->qtab;                // keyed: the Q-table region is free
    if (!kslot && pub && ctx->group_keys && !no_group && n >= ctx->group_min) {
      rc = group_keys(ctx, d, s, b, n, st, &sort_base);
      if (rc) return rc;
    }
    if (!b.kslot) {                               // the per-item route: G on the unsplit u1 (gfull_item)
      if (ctx->gfull && ctx->gfull_item && (rc = ensure_gtabf(ctx, d, s, st))) return rc;
      b.gtabf = ctx->gfull && ctx->gfull_item ? d->gtabf : nullptr;
    }
    plan_sort(ctx, s, b, sort_base);
    d->routes[b.kqw == 2 && b.gtab6               ? GV_ROUTE_KG
              : b.kqw && b.gtab6 && b.k6 == GV_KW_NG2 ? GV_ROUTE_KW2
              : b.kqw && b.gtab6                ? GV_ROUTE_KW
              : b.k6 == GV_KN_ARENA_NG && b.gtab6 ? GV_ROUTE_KN
              : b.k6 && b.gtab6                ? GV_ROUTE_K6
              : b.kslot && b.gtab4 && b.gtabf ? GV_ROUTE_K4F
              : b.kslot && b.gtab4            ? GV_ROUTE_K4
              : b.kslot                       ? GV_ROUTE_KEYED125
              : b.gtabf                       ? GV_ROUTE_ITEMF
                                              : GV_ROUTE_PUB33]++;
    CK(gvk_verify(&b, st));
  }
  if (rs) {
    d->last = d->ring_next;
    d->ring_next = (d->ring_next + 1) % Dev::kRing;
    d->ring_count = std::min(d->ring_count + 1, Dev::kRing);
  }
  return set_release(s, pipelined ? st_ecm : st);
}

// Device-resident calls.  A caller stream: everything on it, in order.  The
// context stream (stream NULL): batches past the small-batch bound are
// PIPELINED -- consecutive calls alternate the two scratch sets, their front
// kernels (unpack, s^-1, prep) go to the set's low-priority stream and every
// ladder to ONE high-priority stream, so call k+1's front kernels fill call
// k's ladder tail (the last ~1 ms of a 7 ms ladder runs below full occupancy)
// while the ladders stay in call order (their d_bits writes too).  Small
// batches and the other calls on the context stream are ordered after every
// pipelined ladder (hi_done) and the next ladder after them (plain_done).
void order_after_pipeline(Dev* d, hipStream_t st) {
  for (int j = 0; j < 2; ++j)
    if (d->hi_used[j]) (void)hipStreamWaitEvent(st, d->hi_done[j], 0);
}
template <class F>
int dev_run(gv_ctx* ctx, Dev* d, void* stream, size_t n, bool keyed, F&& fn) {
  if (stream) {
    order_after_pipeline(d, (hipStream_t)stream);
    return fn(&d->set[0], (hipStream_t)stream, (hipStream_t) nullptr);
  }
  if (!ctx->pipeline_dev || n <= (keyed ? ctx->lat_max_keyed : ctx->lat_max)) {
    hipStream_t st = d->set[0].st;
    order_after_pipeline(d, st);
    const int rc = fn(&d->set[0], st, (hipStream_t) nullptr);
    if (rc) return rc;
    CK(hipEventRecord(d->plain_done, st));
    d->plain_used = true;
    return GV_OK;
  }
  const int j = d->flip;
  d->flip ^= 1;
  // two_ladders: set j's ladder on hi_st[j], so call k+1's ladder starts in
  // call k's tail (its front ran under call k's ladder); the bitmap writes
  // stay in call order through bits_ev.  Else one ladder stream.
  hipStream_t hs = d->hi_st[ctx->two_ladders ? j : 0];
  hipEvent_t& hd = d->hi_done[ctx->two_ladders ? j : 0];
  if (d->plain_used) CK(hipStreamWaitEvent(hs, d->plain_done, 0));
  d->bits_wait = (ctx->two_ladders && d->bits_used) ? d->bits_ev[j ^ 1] : nullptr;
  d->bits_rec = ctx->two_ladders ? d->bits_ev[j] : nullptr;
  const int rc = fn(&d->set[j], d->lo_st[j], hs);
  d->bits_wait = d->bits_rec = nullptr;
  if (rc) return rc;
  CK(hipEventRecord(hd, hs));
  d->hi_used[ctx->two_ladders ? j : 0] = true;
  d->bits_used = ctx->two_ladders;
  return GV_OK;
}

struct HostBatch {
  const uint8_t *pub33, *sig64, *dig32, *blob;
  const uint64_t* off;
  const uint32_t* len;
  const uint32_t* slots;
  uint8_t* out_ok;
  uint64_t* out_bits;
  bool pinned = false;          // digest inputs in pinned host memory (gv_host_alloc): no staging copy
  const uint32_t* d_slots = nullptr;   // slice grouping: per-item key ids on the device (offset lo)
  const KeyArena* ka = nullptr;        // ... and the arena they index
  size_t d_slots_lo = 0;
  bool plain = false;                  // the per-item pub33 pipeline, no in-batch grouping (a grouped
                                       // slice's first chunk, run while the slice's key tables build)
};

// Host memory the device can read directly (hipHostMalloc / gv_host_alloc /
// hipHostRegister), as opposed to pageable memory that must be staged.
bool is_pinned(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Harvest a finished chunk of set s into the caller's outputs.
int harvest(Dev* d, Set* s, const HostBatch& hb) {
  CK(hipEventSynchronize(s->done));
  const size_t c0 = s->c0, cn = s->cn, words = (cn + 63) / 64;
  if (s->zc) {                                  // zero-copy small batch: verdict bytes in h_out8
    if (hb.out_ok) {
      memcpy(hb.out_ok + c0, s->h_out8, cn);
    } else {                                    // c0 % 64 == 0
      for (size_t w = 0; w < words; ++w) {
        uint64_t v = 0;
        const size_t lim = std::min<size_t>(64, cn - 64 * w);
        for (size_t i = 0; i < lim; ++i) v |= (uint64_t)(s->h_out8[64 * w + i] & 1u) << i;
        hb.out_bits[c0 / 64 + w] = v;
      }
    }
    s->busy = false;
    return GV_OK;
  }
  if (hb.out_ok) {
    uint8_t* o = hb.out_ok + c0;
    const uint64_t* w = s->h_bits;
    // 8 verdict bytes per bitmap byte through a 256-entry table (lo % 64 == 0)
    static const std::array<uint64_t, 256> spread = [] {
      std::array<uint64_t, 256> t{};
      for (int v = 0; v < 256; ++v)
        for (int b = 0; b < 8; ++b) t[v] |= (uint64_t)((v >> b) & 1) << (8 * b);
      return t;
    }();
    auto unpack = [&](size_t lo, size_t hi) {
      const uint8_t* wb = (const uint8_t*)w;
      size_t i = lo;
      for (; i + 8 <= hi; i += 8) {
        const uint64_t v = spread[wb[i >> 3]];
        memcpy(o + i, &v, 8);
      }
      for (; i < hi; ++i) o[i] = (uint8_t)((w[i >> 6] >> (i & 63)) & 1u);
    };
    if (cn < (size_t(1) << 18)) unpack(0, cn);
    else {
      const int parts = d->pool->size();
      const size_t per = round_up((cn + parts - 1) / parts, 64);
      d->pool->run(parts, [&](int p) { unpack(std::min(cn, p * per), std::min(cn, (p + 1) * per)); });
    }
  } else {
    memcpy(hb.out_bits + c0 / 64, s->h_bits, words * 8);   // c0 % 64 == 0 (chunks are 256-aligned)
  }
  s->busy = false;
  return GV_OK;
}

// A host chunk's ladder runs on the set's ladder stream (below the front
// priority of the set streams), so the next chunk's front kernels -- and an
// asynchronously submitted batch's grouping and key tables -- take CU slots
// as this ladder's workgroups retire instead of queueing behind it (the
// device-resident pipeline's stream priorities, dev_run).  Small batches run
// one fused kernel on the set stream.
hipStream_t chunk_ladder(const gv_ctx* ctx, Set* s, size_t cn, bool keyed) {
  const size_t lmax = keyed ? ctx->lat_max_keyed : ctx->lat_max;
  return ctx->host_ladder_stream && cn > lmax ? s->lad : nullptr;
}
// The set stream continues after the chunk's ladder (the bitmap's D2H).
int ladder_join(Set* s) {
  if (s->last_st != s->lad) return GV_OK;       // the ladder ran on the set stream
  CK(hipEventRecord(s->lad_done, s->lad));
  CK(hipStreamWaitEvent(s->st, s->lad_done, 0));
  return GV_OK;
}

// Stage chunk [c0, c0 + cn) of a host batch into set s and enqueue H2D ->
// kernels -> D2H of the bitmap on the set's stream.
int submit(gv_ctx* ctx, Dev* d, Set* s, size_t c0, size_t cn, const HostBatch& hb) {
  const size_t C = round_up(cn, 256);
  const bool dslots = hb.d_slots != nullptr;    // slice grouping: slots already on the device
  const bool keyed = hb.slots != nullptr || dslots, msgs = hb.dig32 == nullptr;
  const uint32_t* dsl = dslots ? hb.d_slots + (c0 - hb.d_slots_lo) : nullptr;
  const size_t grow_c = grow_items(ctx, C);   // (device scratch and pinned staging)
  int rc = ensure_cap(s, grow_c);
  if (rc) return rc;
  const InLayout L = in_layout(C, keyed, msgs);
  size_t hb_bytes = 0;
  if ((rc = ensure_pinned((uint8_t**)&s->h_bits, &s->h_bits_cap, (C / 64) * 8))) return rc;
  uint8_t* h = nullptr;                           // the staging buffer (not for the caller's pinned buffers)
  uint64_t bmin = 0;
  // h2d_serial: this chunk's copies start after the previous chunk's
  auto h2d_begin = [&]() -> int {
    if (ctx->h2d_serial && d->last_h2d) CK(hipStreamWaitEvent(s->st, d->last_h2d, 0));
    return GV_OK;
  };
  auto h2d_end = [&]() -> int {
    CK(hipEventRecord(s->h2d, s->st));
    d->last_h2d = s->h2d;
    return GV_OK;
  };
  if (hb.pinned && !msgs) {                 // the caller's pinned buffers: read in place, no staging
    const uint8_t* kp = keyed ? (const uint8_t*)(hb.slots + c0) : hb.pub33 + c0 * 33;
    const uint8_t* sp = hb.sig64 + c0 * 64;
    const uint8_t* dp = hb.dig32 + c0 * 32;
    const size_t lmax = keyed ? ctx->lat_max_keyed : ctx->lat_max;
    const size_t slmax = keyed ? ctx->lat_sl_max_keyed : ctx->lat_sl_max;
    if (ctx->lat_zero_copy && ctx->lat_sliced && cn <= slmax && cn <= lmax && !dslots) {
      if ((rc = ensure_pinned(&s->h_out8, &s->h_out8_cap, cn))) return rc;
      rc = launch(ctx, d, s, cn, keyed ? nullptr : kp, sp, dp, nullptr, nullptr, nullptr, nullptr, s->st,
                  keyed ? (const uint32_t*)kp : nullptr, s->h_out8);
      if (rc) return rc;
      CK(hipEventRecord(s->done, s->st));
      s->busy = true;
      s->zc = true;
      s->c0 = c0;
      s->cn = cn;
      return GV_OK;
    }
    if ((rc = set_acquire(s, s->st)) || (rc = h2d_begin())) return rc;
    if (!dslots) CK(hipMemcpyAsync(s->d_in, kp, cn * (keyed ? 4 : 33), hipMemcpyHostToDevice, s->st));
    CK(hipMemcpyAsync(s->d_in + L.sig, sp, cn * 64, hipMemcpyHostToDevice, s->st));
    CK(hipMemcpyAsync(s->d_in + L.third, dp, cn * 32, hipMemcpyHostToDevice, s->st));
    if ((rc = h2d_end())) return rc;
    const uint8_t* din = s->d_in;
    rc = launch(ctx, d, s, cn, keyed ? nullptr : din, din + L.sig, din + L.third, nullptr, nullptr, nullptr, s->bits,
                s->st, dslots ? dsl : keyed ? (const uint32_t*)din : nullptr, nullptr, chunk_ladder(ctx, s, cn, keyed),
                hb.ka, hb.plain);
    if (rc || (rc = ladder_join(s))) return rc;
    CK(hipMemcpyAsync(s->h_bits, s->bits, ((cn + 63) / 64) * 8, hipMemcpyDeviceToHost, s->st));
    CK(hipEventRecord(s->done, s->st));
    if ((rc = set_release(s, s->st))) return rc;
    s->busy = true;
    s->zc = false;
    s->c0 = c0;
    s->cn = cn;
    return GV_OK;
  }
  // (grown: room for the largest layout, pub33 + digests, so a plain chunk
  // after keyed ones does not regrow it either)
  const size_t stage_bytes = grow_c > C ? in_layout(grow_c, false, false).total : L.total;
  if ((rc = ensure_pinned(&s->h_in, &s->h_in_cap, stage_bytes))) return rc;
  h = s->h_in;
  const size_t lmax0 = keyed ? ctx->lat_max_keyed : ctx->lat_max;
  const size_t slmax0 = keyed ? ctx->lat_sl_max_keyed : ctx->lat_sl_max;
  const bool zc_path = ctx->lat_zero_copy && ctx->lat_sliced && cn <= slmax0 && cn <= lmax0 && !dslots;
  bool sent = false;
  if (!msgs && !zc_path && ctx->stage_pieces > 1 && cn >= 65536) {
    // large pageable chunk: staged in pieces, each piece's H2D right behind
    // its copy, so the transfer of piece i overlaps the staging of piece i+1
    if ((rc = set_acquire(s, s->st)) || (rc = h2d_begin())) return rc;
    const size_t per = round_up((cn + ctx->stage_pieces - 1) / ctx->stage_pieces, 256);
    const size_t kb = keyed ? 4 : 33;
    for (size_t a = 0; a < cn; a += per) {
      const size_t m = std::min(per, cn - a);
      const CopySeg segs[3] = {CopySeg{h + L.sig + a * 64, hb.sig64 + (c0 + a) * 64, m * 64},
                               CopySeg{h + L.third + a * 32, hb.dig32 + (c0 + a) * 32, m * 32},
                               keyed ? CopySeg{h + a * 4, (const uint8_t*)(hb.slots + c0 + a), m * 4}
                                     : CopySeg{h + a * 33, hb.pub33 + (c0 + a) * 33, m * 33}};
      par_copy_segs(d->pool, segs, dslots ? 2 : 3);
      if (!dslots) CK(hipMemcpyAsync(s->d_in + a * kb, h + a * kb, m * kb, hipMemcpyHostToDevice, s->st));
      CK(hipMemcpyAsync(s->d_in + L.sig + a * 64, h + L.sig + a * 64, m * 64, hipMemcpyHostToDevice, s->st));
      CK(hipMemcpyAsync(s->d_in + L.third + a * 32, h + L.third + a * 32, m * 32, hipMemcpyHostToDevice, s->st));
    }
    if ((rc = h2d_end())) return rc;
    sent = true;
  } else if (!msgs) {                       // keys/slots, signatures, digests: one pool pass
    const CopySeg segs[3] = {CopySeg{h + L.sig, hb.sig64 + c0 * 64, cn * 64},
                             CopySeg{h + L.third, hb.dig32 + c0 * 32, cn * 32},
                             keyed ? CopySeg{h, (const uint8_t*)(hb.slots + c0), cn * 4}
                                   : CopySeg{h, hb.pub33 + c0 * 33, cn * 33}};
    par_copy_segs(d->pool, segs, dslots ? 2 : 3);
  } else {
    if (dslots) {
    } else if (keyed) par_copy(d->pool, h, hb.slots + c0, cn * 4);
    else par_copy(d->pool, h, hb.pub33 + c0 * 33, cn * 33);
    par_copy(d->pool, h + L.sig, hb.sig64 + c0 * 64, cn * 64);
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t i = c0; i < c0 + cn; ++i) {
      lo = std::min<uint64_t>(lo, hb.off[i]);
      hi = std::max<uint64_t>(hi, hb.off[i] + hb.len[i]);
    }
    if (lo > hi) lo = hi = 0;
    bmin = lo;
    hb_bytes = hi - lo;
    uint64_t* ro = (uint64_t*)(h + L.third);
    for (size_t i = 0; i < cn; ++i) ro[i] = hb.off[c0 + i] - bmin;
    memcpy(h + L.len, hb.len + c0, cn * 4);
    if ((rc = ensure_pinned(&s->h_blob, &s->h_blob_cap, std::max<size_t>(hb_bytes, 1)))) return rc;
    if ((rc = ensure_blob(s, hb_bytes))) return rc;
    par_copy(d->pool, s->h_blob, hb.blob + bmin, hb_bytes);
  }
  const size_t lmax = keyed ? ctx->lat_max_keyed : ctx->lat_max;
  const size_t slmax = keyed ? ctx->lat_sl_max_keyed : ctx->lat_sl_max;
  if (ctx->lat_zero_copy && ctx->lat_sliced && cn <= slmax && cn <= lmax && !dslots) {
    // zero-copy small batch: the kernel reads the pinned staging buffers
    // (messages too: its scalar wave hashes them) and writes one verdict byte
    // per item to pinned memory (no H2D / memset / D2H)
    if ((rc = ensure_pinned(&s->h_out8, &s->h_out8_cap, cn))) return rc;
    rc = launch(ctx, d, s, cn, keyed ? nullptr : h, h + L.sig, msgs ? nullptr : h + L.third,
                msgs ? s->h_blob : nullptr, msgs ? (const uint64_t*)(h + L.third) : nullptr,
                msgs ? (const uint32_t*)(h + L.len) : nullptr, nullptr, s->st,
                keyed ? (const uint32_t*)h : nullptr, s->h_out8);
    if (rc) return rc;
    CK(hipEventRecord(s->done, s->st));
    s->busy = true;
    s->zc = true;
    s->c0 = c0;
    s->cn = cn;
    return GV_OK;
  }
  if (!sent) {
    if ((rc = set_acquire(s, s->st)) || (rc = h2d_begin())) return rc;
    const size_t from = dslots ? L.sig : 0;   // device slots: no key region to send
    CK(hipMemcpyAsync(s->d_in + from, h + from, (msgs ? L.total : L.third + cn * 32) - from, hipMemcpyHostToDevice,
                      s->st));
    if (msgs && hb_bytes) CK(hipMemcpyAsync(s->d_blob, s->h_blob, hb_bytes, hipMemcpyHostToDevice, s->st));
    if ((rc = h2d_end())) return rc;
  } else if (msgs && hb_bytes) {
    CK(hipMemcpyAsync(s->d_blob, s->h_blob, hb_bytes, hipMemcpyHostToDevice, s->st));
  }
  const uint8_t* din = s->d_in;
  rc = launch(ctx, d, s, cn, keyed ? nullptr : din, din + L.sig, msgs ? nullptr : din + L.third,
              msgs ? s->d_blob : nullptr, msgs ? (const uint64_t*)(din + L.third) : nullptr,
              msgs ? (const uint32_t*)(din + L.len) : nullptr, s->bits, s->st,
              dslots ? dsl : keyed ? (const uint32_t*)din : nullptr, nullptr, chunk_ladder(ctx, s, cn, keyed), hb.ka,
              hb.plain);
  if (rc || (rc = ladder_join(s))) return rc;
  CK(hipMemcpyAsync(s->h_bits, s->bits, ((cn + 63) / 64) * 8, hipMemcpyDeviceToHost, s->st));
  CK(hipEventRecord(s->done, s->st));
  if ((rc = set_release(s, s->st))) return rc;
  s->busy = true;
  s->zc = false;
  s->c0 = c0;
  s->cn = cn;
  return GV_OK;
}

// Does a host slice repeat its keys enough for grouping?  Birthday count on a
// pseudo-random sample of m keys: at average multiplicity k the sample holds
// about m^2 (k - 1) / 2n repeated keys; take the route when a quarter of the
// count expected at k = group_div is there (a strided sample would miss
// round-robin key orders).
bool worth_grouping(const uint8_t* pub33, size_t n, int div) {
  const size_t m = std::min<size_t>(n, 4096);
  std::vector<uint64_t> h(m);
  uint64_t r = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < m; ++i) {
    r ^= r << 13; r ^= r >> 7; r ^= r << 17;
    const uint8_t* p = pub33 + (r % n) * 33;
    uint64_t v;
    memcpy(&v, p + 1, 8);
    h[i] = v ^ ((uint64_t)p[0] * 0xFF51AFD7ED558CCDull) ^ ((uint64_t)p[25] << 32 | p[32]);
  }
  std::sort(h.begin(), h.end());
  size_t dups = 0;
  for (size_t i = 1; i < m; ++i) dups += h[i] == h[i - 1];
  const double expect = (double)m * (double)m * (double)(div - 1) / (2.0 * (double)n);
  return (double)dups >= std::max(1.0, expect / 4);
}

// Whole-slice key grouping for a pub33 host slice [lo, lo + n): the slice's
// keys are sent once (pageable input staged in pieces, each piece's H2D right
// behind its copy), unpacked and grouped over the WHOLE slice -- so the key
// tables are built once per slice, not once per pipeline chunk -- and when
// the slice has few enough distinct keys the chunks then run keyed: only
// signatures and digests (or messages) travel per chunk, the slots stay on
// the device.  *ka is filled and *d_slots set when the route is taken.
int slice_group(gv_ctx* ctx, Dev* d, size_t lo, size_t n, const HostBatch& hb, KeyArena* ka,
                const uint32_t** d_slots, Set* g) {
  *d_slots = nullptr;
  if (!worth_grouping(hb.pub33 + lo * 33, n, ctx->group_div)) return GV_OK;
  const size_t C = round_up(n, 256);
  int rc = ensure_cap(g, grow_items(ctx, C));
  if (rc) return rc;
  if ((rc = set_acquire(g, g->st))) return rc;
  const uint8_t* src = hb.pub33 + lo * 33;
  if (hb.pinned) {
    CK(hipMemcpyAsync(g->d_in, src, n * 33, hipMemcpyHostToDevice, g->st));
  } else {
    if ((rc = ensure_pinned(&g->h_in, &g->h_in_cap, n * 33))) return rc;
    const size_t piece = round_up((n + 3) / 4, 256) * 33;
    for (size_t o = 0; o < n * 33; o += piece) {
      const size_t b = std::min(piece, n * 33 - o);
      par_copy(d->pool, g->h_in + o, src + o, b);
      CK(hipMemcpyAsync(g->d_in + o, g->h_in + o, b, hipMemcpyHostToDevice, g->st));
    }
  }
  gvk_batch b;
  memset(&b, 0, sizeof b);
  b.n = (uint32_t)n; b.C = (uint32_t)C;
  b.pub33 = g->d_in;
  b.in_x = g->in_x; b.in_pfx = g->in_pfx; b.in_r = g->in_r; b.in_s = g->in_s; b.in_e = g->in_e;
  if ((rc = group_keys(ctx, d, g, b, n, g->st))) return rc;
  if (!b.kslot) return set_release(g, g->st);   // many distinct keys after all: per-chunk pipeline
  CK(hipStreamWaitEvent(g->st, b.keys_ready, 0));
  CK(hipEventRecord(g->grp_ready, g->st));
  ka->kqt = b.kqt; ka->kzq = b.kzq; ka->kok = b.kok; ka->kqt2 = b.kqt2; ka->kzq2 = g->g_kzq2;
  ka->kC = b.kC; ka->kcount = b.kcount; ka->gtab4 = b.gtab4;
  ka->gtab6 = b.gtab6; ka->k6 = b.k6; ka->kqw = b.kqw;
  ka->ready = g->grp_ready;
  *d_slots = b.kslot;
  return GV_OK;   // the set stays acquired until run_slice releases it after the last chunk
}

std::vector<Worker*> workers(const gv_ctx* ctx) {
  std::vector<Worker*> w;
  for (Dev* d : ctx->devs) w.push_back(d->worker);
  return w;
}

// Chunk sizes of a host slice of `count` items.  Pipelined (past lat_max): a
// ramp -- pipe_chunk first, each later chunk at most pipe_growth times the one
// before -- so the first kernels start after a short staging copy and every
// later chunk is staged (pageable -> pinned copy, H2D) while the one before it
// computes.  Else equal chunks of at most max_batch.  Every chunk but the last
// is a multiple of 256 (harvest copies bitmap words).
std::vector<size_t> chunk_ramp(const gv_ctx* ctx, size_t count, bool pipelined, bool async = false) {
  std::vector<size_t> sz;
  if (pipelined) {
    const size_t first = async ? ctx->async_chunk : ctx->pipe_chunk;
    const size_t growth = async ? (size_t)ctx->async_growth : (size_t)ctx->pipe_growth;
    size_t c = std::min(first, ctx->max_batch), left = count;
    while (left) {
      const size_t take = std::min(left, c);
      sz.push_back(take);
      left -= take;
      c = std::min(ctx->max_batch, c * growth);
    }
    const size_t m = sz.size();             // a runt tail joins the chunk before it
    if (m >= 2 && 2 * sz[m - 1] < sz[m - 2] && sz[m - 1] + sz[m - 2] <= ctx->max_batch) {
      sz[m - 2] += sz[m - 1];
      sz.pop_back();
    }
  } else {
    const size_t nch = (count + ctx->max_batch - 1) / ctx->max_batch;
    const size_t chunk = std::min(ctx->max_batch, round_up((count + nch - 1) / nch, 256));
    for (size_t c0 = 0; c0 < count; c0 += chunk) sz.push_back(std::min(chunk, count - c0));
  }
  return sz;
}

// Verify items [lo, hi) of a host batch on one device: chunks alternate
// between the two sets so staging + H2D of one overlaps the kernels of the other.
int run_slice(gv_ctx* ctx, Dev* d, size_t lo, size_t hi, const HostBatch& hb) {
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  const size_t n = hi - lo;
  const auto t_begin = std::chrono::steady_clock::now();
  struct SliceTimer {
    Dev* d;
    size_t n;
    std::chrono::steady_clock::time_point t0;
    ~SliceTimer() {
      d->last_slice_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      d->last_slice_n = n;
    }
  } timer{d, n, t_begin};
  d->last_h2d = nullptr;                          // no earlier chunk of this slice
  const bool pipelined = n > (hb.slots ? ctx->lat_max_keyed : ctx->lat_max) && ctx->pipe_chunk;
  auto chunk_sizes = [&](size_t count) { return chunk_ramp(ctx, count, pipelined); };
  std::vector<size_t> sizes = chunk_sizes(n);
  int rc = GV_OK;
  // a pub33 slice big enough for the pipeline: group its keys once for all chunks
  const bool try_group = hb.pub33 && !hb.slots && ctx->group_keys && n >= ctx->group_min && sizes.size() > 1;
  // ... and with slice_plain_first, its first items run the per-item pub33
  // pipeline (their own key parse and Q tables), submitted BEFORE the
  // grouping: their H2D and kernels run while the rest of the slice's keys
  // are sent, grouped and tabulated, so the GPU has ladder work from the
  // start instead of waiting for the key tables
  HostBatch hp = hb;
  hp.plain = true;
  const size_t np = try_group && pipelined && ctx->slice_plain_first
                        ? std::min(round_up(ctx->slice_plain_first, 256), round_up(n / 4, 256)) : 0;
  int k = 0;
  if (np) {
    if ((rc = submit(ctx, d, &d->set[0], lo, np, hp))) return rc;
    k = 1;
  }
  HostBatch hg = hb;
  KeyArena ka;
  bool grouped = false;
  if (try_group) {
    const uint32_t* dsl = nullptr;
    rc = slice_group(ctx, d, lo + np, n - np, hb, &ka, &dsl, &d->gset[0]);
    if (rc == GV_OK && dsl) {
      grouped = true;
      hg.d_slots = dsl;
      hg.d_slots_lo = lo + np;
      hg.ka = &ka;
    }
  }
  const HostBatch& hr = grouped ? hg : hb;
  if (np) sizes = chunk_sizes(n - np);
  size_t c0 = lo + np;
  for (size_t i = 0; i < sizes.size() && rc == GV_OK; c0 += sizes[i], ++i, k ^= 1) {
    Set* s = &d->set[k];
    if (s->busy && (rc = harvest(d, s, hr))) break;
    rc = submit(ctx, d, s, c0, sizes[i], hr);
  }
  for (Set& s : d->set)                          // drain (also after an error)
    if (s.busy) {
      const int r2 = harvest(d, &s, hr);
      if (rc == GV_OK) rc = r2;
      s.busy = false;
    }
  if (grouped) {                                  // every chunk done: the slice's arena is free
    const int r2 = set_release(&d->gset[0], d->gset[0].st);
    if (rc == GV_OK) rc = r2;
  }
  return rc;
}

// ---- ed25519 host-buffer batches: chunks of at most ed_chunk items, staged
// through pinned memory on the device's first stream.
struct EdHost {
  const uint8_t* pub32;
  const uint8_t* sig64;
  const uint8_t* blob;
  const uint64_t* off;
  const uint32_t* len;
  uint8_t* out_ok;
};

int ed_slice(gv_ctx* ctx, Dev* d, size_t lo, size_t hi, const EdHost& hb) {
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  hipStream_t st = d->set[0].st;
  const size_t chunk = std::min<size_t>(ctx->max_batch, 262144);
  for (size_t c0 = lo; c0 < hi; c0 += chunk) {
    const size_t cn = std::min(chunk, hi - c0), C = round_up(cn, 256);
    int rc = ed_ensure(d, C, st);
    if (rc) return rc;
    const EdLayout L = ed_layout(C);
    if ((rc = ensure_pinned(&d->ed.h_in, &d->ed.h_in_cap, L.total))) return rc;
    if ((rc = ensure_pinned(&d->ed.h_bits, &d->ed.h_bits_cap, C / 8))) return rc;
    if (d->ed.last_st) CK(hipEventSynchronize(d->ed.last));      // the staging buffers are free
    uint8_t* h = d->ed.h_in;
    uint64_t lo_b = UINT64_MAX, hi_b = 0;
    for (size_t i = c0; i < c0 + cn; ++i) {
      lo_b = std::min<uint64_t>(lo_b, hb.off[i]);
      hi_b = std::max<uint64_t>(hi_b, hb.off[i] + hb.len[i]);
    }
    if (lo_b > hi_b) lo_b = hi_b = 0;
    const size_t nb = hi_b - lo_b;
    if ((rc = ensure_pinned(&d->ed.h_blob, &d->ed.h_blob_cap, nb))) return rc;
    if (nb > d->ed.blob_cap) {
      if (d->ed.d_blob) (void)hipFree(d->ed.d_blob);
      d->ed.blob_cap = round_up(nb, 1 << 20);
      if (hipMalloc(&d->ed.d_blob, d->ed.blob_cap) != hipSuccess) { d->ed.d_blob = nullptr; d->ed.blob_cap = 0; return GV_ENOMEM; }
    }
    if (!d->ed.d_blob) {
      d->ed.blob_cap = 1 << 20;
      if (hipMalloc(&d->ed.d_blob, d->ed.blob_cap) != hipSuccess) { d->ed.d_blob = nullptr; d->ed.blob_cap = 0; return GV_ENOMEM; }
    }
    const CopySeg segs[2] = {CopySeg{h, hb.pub32 + c0 * 32, cn * 32}, CopySeg{h + L.sig, hb.sig64 + c0 * 64, cn * 64}};
    par_copy_segs(d->pool, segs, 2);
    uint64_t* ro = (uint64_t*)(h + L.off);
    for (size_t i = 0; i < cn; ++i) ro[i] = hb.off[c0 + i] - lo_b;
    memcpy(h + L.len, hb.len + c0, cn * 4);
    if (nb) par_copy(d->pool, d->ed.h_blob, hb.blob + lo_b, nb);
    CK(hipMemcpyAsync(d->ed.d_in, h, L.total, hipMemcpyHostToDevice, st));
    if (nb) CK(hipMemcpyAsync(d->ed.d_blob, d->ed.h_blob, nb, hipMemcpyHostToDevice, st));
    const uint8_t* din = d->ed.d_in;
    rc = ed_launch(ctx->time_kernels, d, cn, din, din + L.sig, d->ed.d_blob, (const uint64_t*)(din + L.off),
                   (const uint32_t*)(din + L.len), d->ed.bits, st, ed_group_cfg(ctx));
    if (rc) return rc;
    CK(hipMemcpyAsync(d->ed.h_bits, d->ed.bits, ((cn + 63) / 64) * 8, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    const uint64_t* w = (const uint64_t*)d->ed.h_bits;
    for (size_t i = 0; i < cn; ++i) hb.out_ok[c0 + i] = (uint8_t)((w[i >> 6] >> (i & 63)) & 1u);
  }
  return GV_OK;
}

int run_ed_host(gv_ctx* ctx, size_t n, const EdHost& hb) {
  if (!ctx) return GV_EINVAL;
  if (ctx->fault_inject) return GV_EFAULT;
  if (n == 0) return GV_OK;
  if (!hb.pub32 || !hb.sig64 || !hb.off || !hb.len || !hb.out_ok) return GV_EINVAL;
  for (size_t i = 0; i < n; ++i)
    if (hb.len[i] && !hb.blob) return GV_EINVAL;
  return run_sliced(workers(ctx), n, 256,
                    [&](size_t k, size_t lo, size_t hi) { return ed_slice(ctx, ctx->devs[k], lo, hi, hb); });
}

int run_host(gv_ctx* ctx, size_t n, const HostBatch& hb_in) {
  if (!ctx) return GV_EINVAL;
  if (ctx->fault_inject) return GV_EFAULT;
  if (n == 0) return GV_OK;
  if ((!hb_in.pub33 && !hb_in.slots) || !hb_in.sig64 || (!hb_in.out_ok && !hb_in.out_bits)) return GV_EINVAL;
  if (!hb_in.dig32 && (!hb_in.blob || !hb_in.off || !hb_in.len)) return GV_EINVAL;
  HostBatch hb = hb_in;
  hb.pinned = hb.dig32 && is_pinned(hb.slots ? (const void*)hb.slots : hb.pub33) && is_pinned(hb.sig64) &&
              is_pinned(hb.dig32);
  // device 0's slice on the caller, devices 1.. on their persistent workers
  return run_sliced(workers(ctx), n, 256,
                    [&](size_t k, size_t lo, size_t hi) { return run_slice(ctx, ctx->devs[k], lo, hi, hb); });
}


}  // namespace

// ---- asynchronous host batches (gv_submit_* / gv_wait)
//
// One lane thread per device takes the device's slices of submitted batches
// in submission order and runs them as ONE stream of chunks over the two
// scratch sets: the next slice's staging, key grouping and key tables (on the
// other grouping set) are enqueued while the previous slice's last chunks
// still compute, so consecutive batches overlap the way pipelined
// device-resident calls do -- the synchronous entry points drain every slice
// before they return.  A batch is done when every device's slice has been
// harvested; gv_wait returns its result.  The lane holds the device lock from
// its first queued slice until its queue is empty and every chunk harvested.
// The queue, tickets and quiesce are gv_async.h (also driven by the CPU
// harness with fake devices); the lane body is lane_stream below.
struct AsyncState : gvasync::Lanes<HostBatch> {
  using gvasync::Lanes<HostBatch>::Lanes;
};
using AsyncSlice = gvasync::Slice<HostBatch>;

namespace {

struct ActiveSlice {
  AsyncSlice sl;
  HostBatch hr;                                   // what the chunks run (a grouped slice: device slots)
  KeyArena ka;
  Set* g = nullptr;                               // its grouping set (released after its last chunk)
  int inflight = 0;
  bool submitted = false;
  int rc = GV_OK;
};

void finish_slice(AsyncState* as, ActiveSlice& a) {
  if (a.g) {
    const int rc = set_release(a.g, a.g->st);
    if (rc && !a.rc) a.rc = rc;
  }
  as->finish(a.sl, a.rc);
}

// Runs device k's queued slices (d->mu held) until the queue is empty or
// lane_burst slices have run, then drains.
void lane_stream(gv_ctx* ctx, AsyncState* as, size_t k, Dev* d) {
  std::list<ActiveSlice> act;
  ActiveSlice* owner[2] = {nullptr, nullptr};
  int sk = 0, gflip = 0;
  d->last_h2d = nullptr;
  auto retire = [&](ActiveSlice* a) {
    finish_slice(as, *a);
    for (auto it = act.begin(); it != act.end(); ++it)
      if (&*it == a) { act.erase(it); break; }
  };
  auto harvest_set = [&](int j) {                 // the chunk in flight on set j
    Set* s = &d->set[j];
    if (!s->busy) return;
    ActiveSlice* a = owner[j];
    const int rc = harvest(d, s, a->hr);
    if (rc && !a->rc) a->rc = rc;
    owner[j] = nullptr;
    if (--a->inflight == 0 && a->submitted) retire(a);
  };
  auto drain = [&]() {                            // the older chunk first
    harvest_set(sk);
    harvest_set(sk ^ 1);
  };
  for (size_t taken = 0;; ++taken) {
    AsyncSlice sl;
    // after lane_burst slices the lane drains and lets go of d->mu (the
    // Lanes loop calls it again while the queue holds slices): a caller that
    // keeps the queue full cannot starve synchronous calls on this device
    if (taken >= ctx->lane_burst || !as->pop(k, sl)) break;
    const bool behind = !act.empty();             // an earlier slice's chunks still in flight
    act.emplace_back();
    ActiveSlice& a = act.back();
    a.sl = sl;
    a.hr = sl.job->hb;
    const size_t lo = sl.lo, n = sl.hi - sl.lo;
    const HostBatch& hb = sl.job->hb;
    const bool pipelined = n > (hb.slots ? ctx->lat_max_keyed : ctx->lat_max) && ctx->pipe_chunk;
    const bool in_place = hb.pinned;               // read from the caller's pinned buffers, no staging
    const std::vector<size_t> sizes = ctx->async_whole && in_place ? chunk_ramp(ctx, n, pipelined && !behind)
                                                                   : chunk_ramp(ctx, n, pipelined, true);
    const bool try_group = hb.pub33 && !hb.slots && ctx->group_keys && n >= ctx->group_min && sizes.size() > 1;
    if (try_group) {
      Set* g = &d->gset[gflip];
      gflip ^= 1;
      for (const ActiveSlice& o : act)            // an older slice still on this grouping set: drain it
        if (&o != &a && o.g == g) { drain(); break; }
      const uint32_t* dsl = nullptr;
      const int rc = slice_group(ctx, d, lo, n, hb, &a.ka, &dsl, g);
      if (rc) a.rc = rc;
      else if (dsl) {
        a.g = g;
        a.hr.d_slots = dsl;
        a.hr.d_slots_lo = lo;
        a.hr.ka = &a.ka;
      }
    }
    size_t c0 = lo;
    for (size_t i = 0; i < sizes.size() && a.rc == GV_OK; c0 += sizes[i], ++i) {
      harvest_set(sk);
      const int rc = submit(ctx, d, &d->set[sk], c0, sizes[i], a.hr);
      if (rc) { a.rc = rc; break; }
      owner[sk] = &a;
      ++a.inflight;
      sk ^= 1;
    }
    a.submitted = true;
    if (a.inflight == 0) retire(&a);
  }
  drain();
}

// Device k's lane body (gvasync::Lanes calls it when k's queue holds a slice).
void lane_run(gv_ctx* ctx, AsyncState* as, size_t k) {
  Dev* d = ctx->devs[k];
  std::lock_guard<std::mutex> dl(d->mu);
  if (hipSetDevice(d->id) != hipSuccess) {        // fail every queued slice of this device
    as->fail_queued(k, GV_EHIP);
    return;
  }
  lane_stream(ctx, as, k, d);
}

AsyncState* async_state(gv_ctx* ctx) {
  static std::mutex create_mu;
  std::lock_guard<std::mutex> lk(create_mu);
  if (!ctx->async) {
    // (a lane runs only for a submitted slice, i.e. after ctx->async is set)
    ctx->async = new AsyncState(ctx->devs.size(), [ctx](size_t k) { lane_run(ctx, ctx->async, k); });
  }
  return ctx->async;
}

// Held by gv_keys_load / gv_keys_reset (gvasync::Lanes::Quiesce): no
// submitted keyed batch reads a slot that moves, and no submission slips in.
struct AsyncQuiesce : gvasync::Lanes<HostBatch>::Quiesce {
  explicit AsyncQuiesce(gv_ctx* ctx) : Quiesce(ctx->async) {}
};

int submit_host(gv_ctx* ctx, size_t n, const HostBatch& hb_in, uint64_t* ticket) {
  if (!ctx || !ticket) return GV_EINVAL;
  *ticket = 0;
  if (ctx->fault_inject) return GV_EFAULT;
  if (n > 0) {
    if ((!hb_in.pub33 && !hb_in.slots) || !hb_in.sig64 || (!hb_in.out_ok && !hb_in.out_bits)) return GV_EINVAL;
    if (!hb_in.dig32 && (!hb_in.blob || !hb_in.off || !hb_in.len)) return GV_EINVAL;
  }
  HostBatch hb = hb_in;
  hb.pinned = hb_in.dig32 && is_pinned(hb_in.slots ? (const void*)hb_in.slots : hb_in.pub33) &&
              is_pinned(hb_in.sig64) && is_pinned(hb_in.dig32);
  *ticket = async_state(ctx)->submit(hb, n);
  return GV_OK;
}

}  // namespace

namespace {

void free_set(Set& s) {
  if (s.st) (void)hipStreamSynchronize(s.st);
  if (s.scratch) (void)hipFree(s.scratch);
  if (s.d_blob) (void)hipFree(s.d_blob);
  if (s.h_in) (void)hipHostFree(s.h_in);
  if (s.h_blob) (void)hipHostFree(s.h_blob);
  if (s.h_bits) (void)hipHostFree(s.h_bits);
  if (s.h_out8) (void)hipHostFree(s.h_out8);
  if (s.last) (void)hipEventDestroy(s.last);
  if (s.done) (void)hipEventDestroy(s.done);
  if (s.ecm_ready) (void)hipEventDestroy(s.ecm_ready);
  if (s.fork) (void)hipEventDestroy(s.fork);
  if (s.keys_done) (void)hipEventDestroy(s.keys_done);
  if (s.grp_ready) (void)hipEventDestroy(s.grp_ready);
  if (s.side) { (void)hipStreamSynchronize(s.side); (void)hipStreamDestroy(s.side); }
  for (uint32_t* p : {s.g_kqt, s.g_kzq, s.g_kok, s.g_kqt2, s.g_kzq2})
    if (p) (void)hipFree(p);
  if (s.h_count) (void)hipHostFree(s.h_count);
  if (s.lad) { (void)hipStreamSynchronize(s.lad); (void)hipStreamDestroy(s.lad); }
  if (s.lad_done) (void)hipEventDestroy(s.lad_done);
  if (s.st) (void)hipStreamDestroy(s.st);
}

bool parse_size_env(const char* name, size_t* out) {
  const char* v = getenv(name);
  if (!v) return false;
  const long long x = atoll(v);
  if (x < 256 || (unsigned long long)x > kMaxItems) return false;
  *out = round_up((size_t)x, 256);
  return true;
}

}  // namespace

extern "C" {


// gv_open's pre-sizing (GV_PRESIZE=1, off by default): both scratch sets of
// every device at a whole max_batch chunk, and their grouping arenas when the
// HBM budget holds them, allocated and written once, so a node's first large
// calls neither allocate nor first-touch them.  First 1M call 1.30 -> 1.26x
// steady (profiles/r06/first_call/presize_ab.jsonl): the rest is the first
// ladders themselves (4.51, 4.30, 4.17 then 4.0 ms), not allocation; off by
// default because the ~6 GB it holds per device would come out of the HBM
// budget that the resident key arena sizes itself from.
static int presize_devices(gv_ctx* ctx) {
  const size_t C = round_up(ctx->max_batch, 256);
  const size_t capU = round_up(std::max<size_t>(C / ctx->group_div, 256), 256);
  for (Dev* d : ctx->devs) {
    if (hipSetDevice(d->id) != hipSuccess) return GV_EHIP;
    for (Set& s : d->set) {
      int rc = ensure_cap(&s, C);
      if (rc) return rc;
      if (hipMemsetAsync(s.scratch, 0, s.d_in ? (size_t)((uint8_t*)(s.bits + C / 64) - s.scratch) : 0, s.st) !=
          hipSuccess)
        return GV_EHIP;
      rc = ensure_group_arena(ctx, d, &s, capU, GV_KEY_WORDS, GV_LGRP);
      if (rc == GV_OK) {
        for (uint32_t* p : {s.g_kqt, s.g_kqt2})
          if (hipMemsetAsync(p, 0, (size_t)capU * GV_KEY_WORDS * 4 * (p == s.g_kqt ? 1 : GV_LGRP - 1), s.st) !=
              hipSuccess)
            return GV_EHIP;
      } else if (rc != GV_ENOMEM) {
        return rc;
      }
    }
    for (Set& s : d->set)
      if (hipStreamSynchronize(s.st) != hipSuccess) return GV_EHIP;
  }
  return GV_OK;
}

int gv_open(const int* dev_ids, int n_dev, gv_ctx** out) {
  if (!out || n_dev < 0 || (n_dev > 0 && !dev_ids)) return GV_EINVAL;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return GV_ENODEV;
  std::vector<int> ids;
  if (n_dev == 0) for (int i = 0; i < count; ++i) ids.push_back(i);
  else for (int i = 0; i < n_dev; ++i) {
    if (dev_ids[i] < 0 || dev_ids[i] >= count) return GV_ENODEV;
    ids.push_back(dev_ids[i]);
  }
  for (int id : ids) {                          // the kernels are written for wave64
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, id) != hipSuccess || prop.warpSize != 64) return GV_ENODEV;
  }
  gv_ctx* ctx = new gv_ctx();
  parse_size_env("GV_MAX_BATCH", &ctx->max_batch);
  if (const char* k4 = getenv("GV_KEYED_K4")) ctx->keyed_k4 = strcmp(k4, "0") != 0;
  if (const char* k6 = getenv("GV_K6")) ctx->k6 = strcmp(k6, "0") != 0;
  if (const char* kg = getenv("GV_KG")) {
    const int v = atoi(kg);
    if (kg_layout_ok(v)) ctx->kg = v;
  }
  if (const char* gf = getenv("GV_GFULL")) ctx->gfull = strcmp(gf, "0") != 0;
  if (const char* tl = getenv("GV_TWO_LADDERS")) ctx->two_ladders = strcmp(tl, "0") != 0;
  if (const char* ks = getenv("GV_KEYS_SCRATCH")) ctx->keys_scratch = strcmp(ks, "0") != 0;
  if (const char* sk = getenv("GV_SORT_KEYS")) ctx->sort_keys = strcmp(sk, "0") != 0;
  if (const char* ek = getenv("GV_ED_KEYED")) ctx->ed_keyed = strcmp(ek, "0") != 0;
  if (const char* eg = getenv("GV_ED_GROUP")) ctx->ed_group = strcmp(eg, "0") != 0;
  if (const char* es = getenv("GV_ED_KEYS_SPLIT")) ctx->ed_keys_split = strcmp(es, "0") != 0;
  if (const char* eb = getenv("GV_ED_BTAB16")) ctx->ed_btab16 = strcmp(eb, "0") != 0;
  if (const char* er = getenv("GV_ED_GROUP_R64")) ctx->ed_group_r64 = strcmp(er, "0") != 0;
  if (const char* ls = getenv("GV_LAT_SLICED")) ctx->lat_sliced = strcmp(ls, "0") != 0;
  if (const char* lr = getenv("GV_LAT_ROWS_MAX")) ctx->lat_rows_max = (size_t)strtoull(lr, nullptr, 10);
  if (const char* zc = getenv("GV_LAT_ZC")) ctx->lat_zero_copy = strcmp(zc, "0") != 0;
  if (const char* pl = getenv("GV_PIPELINE")) ctx->pipeline_dev = strcmp(pl, "0") != 0;
  if (const char* gk = getenv("GV_GROUP_KEYS")) ctx->group_keys = strcmp(gk, "0") != 0;
  if (const char* sp = getenv("GV_STAGE_PIECES")) ctx->stage_pieces = std::max(1, atoi(sp));
  if (const char* pf = getenv("GV_SLICE_PLAIN_FIRST")) ctx->slice_plain_first = strtoull(pf, nullptr, 10);
  if (const char* is = getenv("GV_INV_SMALL")) ctx->inv_small = strcmp(is, "0") != 0;
  if (const char* gi = getenv("GV_GFULL_ITEM")) ctx->gfull_item = strcmp(gi, "0") != 0;
  if (const char* hs = getenv("GV_H2D_SERIAL")) ctx->h2d_serial = strcmp(hs, "0") != 0;
  if (const char* lk = getenv("GV_LAT_KW")) ctx->lat_kw = strcmp(lk, "0") != 0;
  if (const char* lb = getenv("GV_LANE_BURST")) ctx->lane_burst = (size_t)std::max(1, atoi(lb));
  if (const char* kk = getenv("GV_KEYS_K6")) ctx->keys_k6 = strcmp(kk, "0") != 0;
  if (const char* kk = getenv("GV_KEYS_WIDE")) {
    const int v = atoi(kk);
    if (v >= 0 && v <= 2) ctx->keys_wide = v;
  }
  if (const char* hl = getenv("GV_HOST_LADDER_STREAM")) ctx->host_ladder_stream = strcmp(hl, "0") != 0;
  parse_size_env("GV_ASYNC_CHUNK", &ctx->async_chunk);
  if (const char* ag = getenv("GV_ASYNC_GROWTH")) ctx->async_growth = std::max(1, std::min(64, atoi(ag)));
  if (const char* aw = getenv("GV_ASYNC_WHOLE")) ctx->async_whole = strcmp(aw, "0") != 0;
  if (const char* kc = getenv("GV_KEY_CAP")) {
    const long long v = atoll(kc);
    if (v >= 256 && (unsigned long long)v <= kMaxItems) ctx->key_cap = (size_t)v;
  }
  if (const char* kc = getenv("GV_ED_KEY_CAP")) {
    const long long v = atoll(kc);
    if (v >= 256 && (unsigned long long)v <= kMaxItems) ctx->ed_key_cap = (size_t)v;
  }
  if (const char* hb = getenv("GV_HBM_BUDGET_MB")) {
    const long long v = atoll(hb);
    if (v > 0) ctx->hbm_budget = (size_t)v << 20;
  }
  ctx->stage_threads = gvstage::stage_pool_threads(host_cpus(), (int)ids.size());
  for (size_t k = 0; k < ids.size(); ++k) {
    Dev* d = new Dev();
    d->id = ids[k];
    ctx->devs.push_back(d);
    d->pool = new Pool(ctx->stage_threads - 1);
    if (k > 0) d->worker = new Worker();
    bool ok = hipSetDevice(d->id) == hipSuccess;
    // Stream priorities of the pipelined device-resident calls (env
    // GV_LADDER_PRIO): "front" (default) -- the front kernels (unpack, key
    // grouping, the key-table build on the side stream, s^-1, prep) above the
    // ladders, so a slot a ladder workgroup frees goes to the next call's
    // front first and it is done before the current ladder drains; "ladder" --
    // the ladders above (the round-3 order: the front then runs in the ladder's
    // tail); "equal".
    int lo_prio = 0, hi_prio = 0;
    ok = ok && hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) == hipSuccess;
    int front_prio = hi_prio, ladder_prio = lo_prio;
    if (const char* lp = getenv("GV_LADDER_PRIO")) {
      if (!strcmp(lp, "ladder")) { front_prio = lo_prio; ladder_prio = hi_prio; }
      else if (!strcmp(lp, "equal")) front_prio = ladder_prio = lo_prio;
    }
    for (Set* sp : {&d->set[0], &d->set[1], &d->gset[0], &d->gset[1]})
      ok = ok && hipStreamCreateWithPriority(&sp->st, hipStreamNonBlocking, front_prio) == hipSuccess &&
           hipStreamCreateWithPriority(&sp->lad, hipStreamNonBlocking, ladder_prio) == hipSuccess &&
           hipEventCreateWithFlags(&sp->lad_done, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&sp->last, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&sp->done, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&sp->h2d, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&sp->ecm_ready, hipEventDisableTiming) == hipSuccess &&
           hipStreamCreateWithPriority(&sp->side, hipStreamNonBlocking, front_prio) == hipSuccess &&
           hipEventCreateWithFlags(&sp->fork, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&sp->keys_done, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&sp->grp_ready, hipEventDisableTiming) == hipSuccess;
    // pipelined device-resident calls: front kernels on two streams
    // (alternating sets), the ladders on two more (two_ladders)
    for (int j = 0; j < 2; ++j)
      ok = ok && hipStreamCreateWithPriority(&d->lo_st[j], hipStreamNonBlocking, front_prio) == hipSuccess;
    for (int j = 0; j < 2; ++j)
      ok = ok && hipStreamCreateWithPriority(&d->hi_st[j], hipStreamNonBlocking, ladder_prio) == hipSuccess &&
           hipEventCreateWithFlags(&d->hi_done[j], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&d->bits_ev[j], hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&d->plain_done, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipMalloc(&d->gtab, (size_t)2 * GV_GTAB_N * 16 * 4) == hipSuccess &&
         gvk_gen_gtable(d->gtab, d->set[0].st) == hipSuccess && hipStreamSynchronize(d->set[0].st) == hipSuccess;
    ok = ok && hipMalloc(&d->glat, (size_t)GV_GLAT_WORDS * 4) == hipSuccess &&
         gvk_gen_glat(d->glat, d->set[0].st) == hipSuccess && hipStreamSynchronize(d->set[0].st) == hipSuccess;
    if (!ok) { gv_close(ctx); return GV_EHIP; }
  }
  // The large G tables of the default schedules (full-scalar k4 / per-item,
  // k4's group tables, k6), enqueued on every device before waiting on any, so
  // a node's first block does not build them (~0.5 s per device, concurrent
  // across devices).  GV_EAGER_TABLES=0: built on first use instead.
  const char* eager = getenv("GV_EAGER_TABLES");
  if (!eager || strcmp(eager, "0") != 0) {
    for (Dev* d : ctx->devs) {
      if (hipSetDevice(d->id) != hipSuccess) { gv_close(ctx); return GV_EHIP; }
      Set* s = &d->set[0];
      int rc = ensure_gtab4(ctx, d, s, s->st, false);
      if (!rc) rc = ensure_gtab6(ctx, d, s, s->st, ctx->k6 || ctx->keys_k6, false);
      if (rc) { gv_close(ctx); return rc; }
    }
    for (Dev* d : ctx->devs)
      if (hipSetDevice(d->id) != hipSuccess || hipStreamSynchronize(d->set[0].st) != hipSuccess) {
        gv_close(ctx);
        return GV_EHIP;
      }
  }
  const char* presize = getenv("GV_PRESIZE");
  if (presize && strcmp(presize, "0") != 0) {
    const int rc = presize_devices(ctx);
    if (rc) { gv_close(ctx); return rc; }
  }
  *out = ctx;
  return GV_OK;
}

void gv_close(gv_ctx* ctx) {
  if (!ctx) return;
  if (AsyncState* as = ctx->async) {              // the lanes finish what is queued, then quit
    as->close();
    delete as;
    ctx->async = nullptr;
  }
  for (Dev* d : ctx->devs) {
    delete d->worker;
    (void)hipSetDevice(d->id);
    for (Set& s : d->set) free_set(s);
    for (Set& g : d->gset) free_set(g);
    if (d->gtab) (void)hipFree(d->gtab);
    if (d->glat) (void)hipFree(d->glat);
    if (d->gtab4) (void)hipFree(d->gtab4);
    if (d->gtab6) (void)hipFree(d->gtab6);
    if (d->gtabf) (void)hipFree(d->gtabf);
    for (uint32_t* p : {d->kqt, d->kzq, d->kok, d->kqt2, d->kzq2, d->kqt6, d->kzq6, d->kqt62, d->kzq62, d->kqtw,
                        d->kzqw, d->kqtw2, d->kzqw2})
      if (p) (void)hipFree(p);
    if (d->edtab) (void)hipFree(d->edtab);
    if (d->edtab16) (void)hipFree(d->edtab16);
    if (d->ed.d_in) (void)hipFree(d->ed.d_in);
    if (d->ed.atab) (void)hipFree(d->ed.atab);
    if (d->ed.bits) (void)hipFree(d->ed.bits);
    if (d->ed.d_blob) (void)hipFree(d->ed.d_blob);
    if (d->ed.h_in) (void)hipHostFree(d->ed.h_in);
    if (d->ed.h_blob) (void)hipHostFree(d->ed.h_blob);
    if (d->ed.h_bits) (void)hipHostFree(d->ed.h_bits);
    if (d->ed.last) (void)hipEventDestroy(d->ed.last);
    for (uint32_t* p : {d->ektab, d->ekpub, d->ekok}) if (p) (void)hipFree(p);
    if (d->edl_h) (void)hipHostFree(d->edl_h);
    for (uint32_t* q : {d->edg_ktab, d->edg_kpub, d->edg_kok}) if (q) (void)hipFree(q);
    if (d->ed_h_count) (void)hipHostFree(d->ed_h_count);
    for (int k = 0; k < 2; ++k) {
      if (d->edk_h[k]) (void)hipHostFree(d->edk_h[k]);
      if (d->edk_d[k]) (void)hipFree(d->edk_d[k]);
      if (d->edk_s[k]) (void)hipFree(d->edk_s[k]);
    }
    for (auto& rs : d->ring)
      for (auto e : rs) if (e) (void)hipEventDestroy(e);
    for (hipStream_t t : {d->lo_st[0], d->lo_st[1], d->hi_st[0], d->hi_st[1]})
      if (t) { (void)hipStreamSynchronize(t); (void)hipStreamDestroy(t); }
    for (hipEvent_t e : {d->hi_done[0], d->hi_done[1], d->bits_ev[0], d->bits_ev[1]})
      if (e) (void)hipEventDestroy(e);
    if (d->plain_done) (void)hipEventDestroy(d->plain_done);
    delete d->pool;
    delete d;
  }
  delete ctx;
}

int gv_num_devices(const gv_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int gv_verify_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                   const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                   uint8_t* out_ok) {
  return run_host(ctx, n, HostBatch{pub33, sig64, nullptr, msg_blob, msg_off, msg_len, nullptr, out_ok, nullptr});
}

int gv_verify_digests(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                      const uint8_t* dig32, uint8_t* out_ok) {
  if (!dig32 && n) return GV_EINVAL;
  return run_host(ctx, n, HostBatch{pub33, sig64, dig32, nullptr, nullptr, nullptr, nullptr, out_ok, nullptr});
}

int gv_verify_digests_bits(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                           const uint8_t* dig32, uint64_t* out_bits) {
  if (!dig32 && n) return GV_EINVAL;
  return run_host(ctx, n, HostBatch{pub33, sig64, dig32, nullptr, nullptr, nullptr, nullptr, nullptr, out_bits});
}

int gv_verify_msgs_bits(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                        const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                        uint64_t* out_bits) {
  return run_host(ctx, n, HostBatch{pub33, sig64, nullptr, msg_blob, msg_off, msg_len, nullptr, nullptr, out_bits});
}

static int dev_common(gv_ctx* ctx, int slot, size_t n, const void* pub, const void* sig, void* bits,
                      Dev** dout) {
  if (!ctx) return GV_EINVAL;
  if (ctx->fault_inject) return GV_EFAULT;
  if (slot < 0 || slot >= (int)ctx->devs.size()) return GV_ENODEV;
  if (n == 0) return GV_OK;
  if (!pub || !sig || !bits) return GV_EINVAL;
  if (((uintptr_t)pub & 3) || ((uintptr_t)sig & 3)) return GV_EINVAL;
  if (n > kMaxItems) return GV_EINVAL;
  *dout = ctx->devs[slot];
  return GV_OK;
}

int gv_submit_digests(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32,
                      uint8_t* out_ok, uint64_t* ticket) {
  if (n && !dig32) return GV_EINVAL;
  return submit_host(ctx, n, HostBatch{pub33, sig64, dig32, nullptr, nullptr, nullptr, nullptr, out_ok, nullptr},
                     ticket);
}

int gv_submit_digests_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64, const uint8_t* dig32,
                            uint8_t* out_ok, uint64_t* ticket) {
  if (n && (!slot || !dig32)) return GV_EINVAL;
  return submit_host(ctx, n, HostBatch{nullptr, sig64, dig32, nullptr, nullptr, nullptr, slot, out_ok, nullptr},
                     ticket);
}

int gv_submit_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* msg_blob,
                   const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* out_ok, uint64_t* ticket) {
  return submit_host(ctx, n, HostBatch{pub33, sig64, nullptr, msg_blob, msg_off, msg_len, nullptr, out_ok, nullptr},
                     ticket);
}

int gv_submit_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64, const uint8_t* msg_blob,
                         const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* out_ok, uint64_t* ticket) {
  if (n && !slot) return GV_EINVAL;
  return submit_host(ctx, n, HostBatch{nullptr, sig64, nullptr, msg_blob, msg_off, msg_len, slot, out_ok, nullptr},
                     ticket);
}

int gv_wait(gv_ctx* ctx, uint64_t ticket) {
  if (!ctx || !ctx->async) return GV_EINVAL;
  return ctx->async->wait(ticket, GV_EINVAL);
}

int gv_dev_verify_digests(gv_ctx* ctx, int dev_slot, size_t n, const void* d_pub33,
                          const void* d_sig64, const void* d_dig32, void* d_bits, void* stream) {
  Dev* d = nullptr;
  int rc = dev_common(ctx, dev_slot, n, d_pub33, d_sig64, d_bits, &d);
  if (rc || n == 0) return rc;
  if (!d_dig32 || ((uintptr_t)d_dig32 & 3)) return GV_EINVAL;
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  return dev_run(ctx, d, stream, n, false, [&](Set* s, hipStream_t st, hipStream_t se) {
    return launch(ctx, d, s, n, (const uint8_t*)d_pub33, (const uint8_t*)d_sig64, (const uint8_t*)d_dig32, nullptr,
                  nullptr, nullptr, (uint64_t*)d_bits, st, nullptr, nullptr, se);
  });
}

int gv_dev_verify_msgs(gv_ctx* ctx, int dev_slot, size_t n, const void* d_pub33, const void* d_sig64,
                       const void* d_msg_blob, const void* d_msg_off, const void* d_msg_len, void* d_bits,
                       void* stream) {
  Dev* d = nullptr;
  int rc = dev_common(ctx, dev_slot, n, d_pub33, d_sig64, d_bits, &d);
  if (rc || n == 0) return rc;
  if (!d_msg_blob || !d_msg_off || !d_msg_len) return GV_EINVAL;
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  return dev_run(ctx, d, stream, n, false, [&](Set* s, hipStream_t st, hipStream_t se) {
    return launch(ctx, d, s, n, (const uint8_t*)d_pub33, (const uint8_t*)d_sig64, nullptr,
                  (const uint8_t*)d_msg_blob, (const uint64_t*)d_msg_off, (const uint32_t*)d_msg_len,
                  (uint64_t*)d_bits, st, nullptr, nullptr, se);
  });
}

// ---- ed25519
namespace {
// Small uncached ed25519 batches on one device (k_ed_lat_unc, one signature
// per block): the kernel reads keys, signatures and messages from the pinned
// staging buffer and writes verdict bytes there (no H2D / D2H copies).
int ed_unc_small(gv_ctx* ctx, size_t n, const EdHost& hb) {
  Dev* d = ctx->devs[0];
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  hipStream_t st = d->set[0].st;
  int rc = ed_ensure(d, 256, st);                 // the resident comb table of B
  if (rc) return rc;
  uint64_t lo = UINT64_MAX, hi = 0;
  for (size_t i = 0; i < n; ++i) {
    lo = std::min<uint64_t>(lo, hb.off[i]);
    hi = std::max<uint64_t>(hi, hb.off[i] + hb.len[i]);
  }
  if (lo > hi) lo = hi = 0;
  const size_t o_sig = round_up(n * 32, 64), o_off = o_sig + n * 64, o_len = o_off + n * 8, o_out = o_len + n * 4,
               o_blob = round_up(o_out + n, 64), total = o_blob + (hi - lo);
  if ((rc = ensure_pinned(&d->edl_h, &d->edl_h_cap, total))) return rc;
  uint8_t* h = d->edl_h;
  memcpy(h, hb.pub32, n * 32);
  memcpy(h + o_sig, hb.sig64, n * 64);
  uint64_t* ro = (uint64_t*)(h + o_off);
  for (size_t i = 0; i < n; ++i) ro[i] = hb.off[i] - lo;
  memcpy(h + o_len, hb.len, n * 4);
  if (hi > lo) memcpy(h + o_blob, hb.blob + lo, hi - lo);
  gvk_edl b;
  memset(&b, 0, sizeof b);
  b.n = (uint32_t)n;
  b.pub32 = h;
  b.sig64 = h + o_sig;
  b.msg_blob = h + o_blob;
  b.msg_off = (const uint64_t*)(h + o_off);
  b.msg_len = (const uint32_t*)(h + o_len);
  b.btab = d->edtab;
  b.out8 = h + o_out;
  d->routes[GV_ROUTE_ED_LAT]++;
  CK(gvk_ed_lat_unc(&b, st));
  CK(hipStreamSynchronize(st));
  memcpy(hb.out_ok, h + o_out, n);
  return GV_OK;
}
}  // namespace

int gv_verify_ed25519_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub32, const uint8_t* sig64,
                           const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                           uint8_t* out_ok) {
  const EdHost hb{pub32, sig64, msg_blob, msg_off, msg_len, out_ok};
  if (ctx && !ctx->fault_inject && n && n <= ctx->ed_unc_lat_max && pub32 && sig64 && msg_off && msg_len && out_ok) {
    for (size_t i = 0; i < n; ++i)
      if (msg_len[i] && !msg_blob) return GV_EINVAL;
    return ed_unc_small(ctx, n, hb);
  }
  return run_ed_host(ctx, n, hb);
}

int gv_dev_verify_ed25519_msgs(gv_ctx* ctx, int dev_slot, size_t n, const void* d_pub32, const void* d_sig64,
                               const void* d_msg_blob, const void* d_msg_off, const void* d_msg_len, void* d_bits,
                               void* stream) {
  Dev* d = nullptr;
  int rc = dev_common(ctx, dev_slot, n, d_pub32, d_sig64, d_bits, &d);
  if (rc || n == 0) return rc;
  if (!d_msg_off || !d_msg_len || ((uintptr_t)d_pub32 & 15) || ((uintptr_t)d_sig64 & 15)) return GV_EINVAL;
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  hipStream_t st = stream ? (hipStream_t)stream : d->set[0].st;
  order_after_pipeline(d, st);
  return ed_launch(ctx->time_kernels, d, n, (const uint8_t*)d_pub32, (const uint8_t*)d_sig64, (const uint8_t*)d_msg_blob,
                   (const uint64_t*)d_msg_off, (const uint32_t*)d_msg_len, (uint64_t*)d_bits, st, ed_group_cfg(ctx));
}

// ---- key arena
namespace {
// The wide-window tables (layout d->kw_ng) of the n keys pub33 (host) into
// slots base.. of the wide arena, in chunks whose build scratch stays within
// what the k6 build's chunks take.  The caller holds d->mu.
int build_wide(gv_ctx* ctx, Dev* d, Set* s, hipStream_t st, const uint8_t* pub33, size_t n, size_t base) {
  const size_t stepw = std::min<size_t>(ctx->max_batch, std::max<size_t>(256, 32768 / (size_t)d->kw_ng / 256 * 256));
  int rc;
  for (size_t c0 = 0; c0 < n; c0 += stepw) {
    const size_t cn = std::min(stepw, n - c0);
    const size_t C = round_up(cn, 256);
    const int qew = ctx->keys_scratch ? 1 : 0;
    const size_t ww = gvk_keys_scratch_words((uint32_t)cn, d->kw_ng, GV_KW_NT, qew);
    const size_t Cs = std::max(C, round_up(ww / GV_QTAB_WORDS + 1, 256));
    if ((rc = ensure_cap(s, Cs))) return rc;
    if ((rc = set_acquire(s, st))) return rc;
    CK(hipMemcpyAsync(s->d_in, pub33 + c0 * 33, cn * 33, hipMemcpyHostToDevice, st));
    CK(gvk_keys_build_wide(s->d_in, (uint32_t)cn, (uint32_t)C, s->in_x, s->in_pfx, s->in_r, s->in_s, s->in_e, s->qtab,
                           qew, (uint32_t)(base + c0), d->kqtw, d->kzqw, (uint32_t)d->kcapw, d->kok, d->kqtw2,
                           d->kzqw2, d->kw_ng, st));
    if ((rc = set_release(s, st))) return rc;
    CK(hipStreamSynchronize(st));
  }
  return GV_OK;
}

// The compressed keys of slots 0..n-1 read back from the k4 tables (affine
// 1*Q of each slot); a slot whose key ParsePubKey rejected gets a prefix
// byte it rejects again (0x00), so a rebuild keeps its verdict.
int read_back_pub33(gv_ctx* ctx, Dev* d, hipStream_t st, size_t n, std::vector<uint8_t>& pub) {
  std::vector<uint32_t> slots(n);
  for (size_t i = 0; i < n; ++i) slots[i] = (uint32_t)i;
  std::vector<uint8_t> xy(n * 64), ok(n);
  uint8_t* buf = nullptr;
  const size_t sb = round_up(n * 4, 256), xb = round_up(n * 64, 256);
  if (hipMalloc(&buf, sb + xb + n) != hipSuccess) return GV_ENOMEM;
  int rc = GV_OK;
  if (hipMemcpyAsync(buf, slots.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
      gvk_keys_point((uint32_t)n, (const uint32_t*)buf, d->kqt, d->kzq, (uint32_t)d->kcap, d->kok, (uint32_t)n,
                     buf + sb, buf + sb + xb, st) != hipSuccess ||
      hipMemcpyAsync(xy.data(), buf + sb, n * 64, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(ok.data(), buf + sb + xb, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    rc = GV_EHIP;
  (void)hipFree(buf);
  if (rc) return rc;
  pub.assign(n * 33, 0);
  for (size_t i = 0; i < n; ++i) {
    uint8_t* p = &pub[i * 33];
    memcpy(p + 1, &xy[i * 64], 32);
    p[0] = ok[i] ? (uint8_t)(0x02 | (xy[i * 64 + 63] & 1)) : 0x00;
  }
  return GV_OK;
}
}  // namespace

int gv_keys_load(gv_ctx* ctx, size_t n, const uint8_t* pub33, uint32_t* slot_out) {
  if (!ctx) return GV_EINVAL;
  if (n == 0) return GV_OK;
  if (!pub33 || !slot_out) return GV_EINVAL;
  AsyncQuiesce q(ctx);                          // no submitted keyed batch reads slots that move
  std::lock_guard<std::mutex> kl(ctx->keys_mu);
  const size_t base = ctx->keys;
  if (base + n > kMaxItems) return GV_EINVAL;
  for (Dev* d : ctx->devs) {                    // every device holds every key
    std::lock_guard<std::mutex> lk(d->mu);
    CK(hipSetDevice(d->id));
    Set* s = &d->set[0];
    hipStream_t st = s->st;
    for (hipStream_t t : d->hi_st) CK(hipStreamSynchronize(t));   // no pipelined ladder reads an arena being grown
    if (base == 0) {                            // after gv_keys_reset the slots are rewritten from 0
      d->keys6 = d->keysw = 0;
      d->kw_full = false;
    }
    // the k6 tables too when their G tables exist (or can be built) and the
    // arena has room for them (else k4 only: the k4 route serves the slots)
    int rc = ensure_gtab4(ctx, d, s, st);
    if (!rc) rc = ensure_gtab6(ctx, d, s, st, ctx->keys_k6 || ctx->keys_wide);
    if (rc) return rc;
    bool k6 = ctx->keys_k6 && d->gtab6 && d->keys6 == base;
    if ((rc = ensure_keys(d, base + n, base, st, ctx->key_cap, ctx->hbm_budget, &k6))) return rc;
    // chunks: the k4 build takes max_batch keys at a time; the resident k6
    // tables have GV_KN_ARENA_NG groups of 32 entries (scratch rows per key
    // ~12x the k4 build's), so those chunks are smaller
    const size_t step = k6 ? std::min<size_t>(ctx->max_batch, 32768) : ctx->max_batch;
    for (size_t c0 = 0; c0 < n; c0 += step) {
      const size_t cn = std::min(step, n - c0);
      const size_t C = round_up(cn, 256);
      // scratch: the key-table build's rows (ratios, E, and when they fit the
      // forward-pass entries) from the start of the set's Q-table region
      const size_t w4 = gvk_keys_scratch_words((uint32_t)cn, GV_LGRP, GV_QTAB_N, 0);
      const size_t w6 = k6 ? gvk_keys_scratch_words((uint32_t)cn, GV_KN_ARENA_NG, GV_K6_NT, 1) : 0;
      const size_t Cs = std::max(C, round_up(std::max(w4, w6) / GV_QTAB_WORDS + 1, 256));
      if ((rc = ensure_cap(s, Cs))) return rc;
      if ((rc = set_acquire(s, st))) return rc;
      CK(hipMemcpyAsync(s->d_in, pub33 + c0 * 33, cn * 33, hipMemcpyHostToDevice, st));
      const size_t room = (size_t)GV_QTAB_WORDS * s->cap;
      const int qe4 = ctx->keys_scratch && gvk_keys_scratch_words((uint32_t)cn, GV_LGRP, GV_QTAB_N, 1) <= room;
      CK(gvk_keys_build(s->d_in, (uint32_t)cn, (uint32_t)C, s->in_x, s->in_pfx, s->in_r, s->in_s, s->in_e,
                        s->qtab, qe4, (uint32_t)(base + c0), d->kqt, d->kzq,
                        (uint32_t)d->kcap, d->kok, d->kqt2, d->kzq2, st));
      if (k6)
        CK(gvk_keys_build6(s->d_in, (uint32_t)cn, (uint32_t)C, s->in_x, s->in_pfx, s->in_r, s->in_s, s->in_e,
                           s->qtab, ctx->keys_scratch ? 1 : 0, (uint32_t)(base + c0), d->kqt6, d->kzq6,
                           (uint32_t)d->kcap, d->kok, d->kqt62, d->kzq62, st));
      if ((rc = set_release(s, st))) return rc;
      CK(hipStreamSynchronize(st));            // the caller's pub33 chunk is read by then
    }
    if (k6) d->keys6 = base + n;
    // the wide-window tables: while every earlier slot has them and memory
    // holds the grown arena (a refusal stops them until gv_keys_reset:
    // batches then take the k6 tables).  An arena started from slot 0 takes
    // the option's layout; one window per group (15 tables per key) moves the
    // whole arena to two per group (8 tables) when it no longer fits: the
    // loaded slots' keys are read back from the k4 tables and rebuilt.
    if (ctx->keys_wide && d->gtab6 && d->keysw == base && !d->kw_full) {
      const int want = ctx->keys_wide == 2 ? GV_KW_NG1 : GV_KW_NG2;
      if ((base == 0 || !d->kw_ng) && d->kw_ng != want) {
        free_keys_wide(d);
        d->kw_ng = want;
      }
      // the ed25519 arena's growth to ed_key_cap is reserved too (72 KB per key)
      const size_t ed_room = (ctx->ed_key_cap > d->ekcap ? ctx->ed_key_cap - d->ekcap : 0) *
                             ((size_t)GV_EDK_WORDS + 8 + 1) * 4;
      bool ok = ensure_keys_wide(d, base + n, base, st, ctx->key_cap, ctx->hbm_budget, ed_room,
                                 ctx->keys_wide1_cap);
      if (!ok && d->kw_ng == GV_KW_NG1) {
        // (a failed read-back only stops the wide tables: the k6 ones serve)
        std::vector<uint8_t> old_pub;
        const bool back = !base || read_back_pub33(ctx, d, st, base, old_pub) == GV_OK;
        free_keys_wide(d);
        d->kw_ng = GV_KW_NG2;
        ok = back && ensure_keys_wide(d, base + n, 0, st, ctx->key_cap, ctx->hbm_budget, ed_room);
        // a failed rebuild only stops the wide tables (the k6 / k4 ones serve
        // every slot): never a gv_keys_load error
        if (ok && base && build_wide(ctx, d, s, st, old_pub.data(), base, 0) != GV_OK) ok = false;
      }
      if (ok && build_wide(ctx, d, s, st, pub33, n, base) != GV_OK) ok = false;
      if (!ok) {
        (void)hipGetLastError();
        d->keysw = 0;                             // no slot's wide tables are trusted past a failed build
        d->kw_full = true;
      } else {
        d->keysw = base + n;
      }
    }
  }
  ctx->keys = base + n;
  for (size_t i = 0; i < n; ++i) slot_out[i] = (uint32_t)(base + i);
  return GV_OK;
}

int gv_keys_reset(gv_ctx* ctx) {
  if (!ctx) return GV_EINVAL;
  AsyncQuiesce q(ctx);
  std::lock_guard<std::mutex> kl(ctx->keys_mu);
  ctx->keys = 0;
  ctx->keys_gen.fetch_add(1);
  return GV_OK;
}

size_t gv_keys_count(const gv_ctx* ctx) { return ctx ? ctx->keys : 0; }

// ---- ed25519 key arena + small keyed batches (k_ed_keys, k_ed_lat_sl)
namespace {
// Growth doubles the arena but stops at the callers' reset point (ed_key_cap:
// GV_ED_KEY_CAP or the option) and past it grows to exactly what is needed:
// the transient peak of a growth -- old and new arena both allocated, 72 KB
// per key each -- stays within cap + the old arena.
int ensure_ed_keys(Dev* d, size_t need, size_t used, hipStream_t st, size_t cap_limit) {
  if (need <= d->ekcap) return GV_OK;
  const size_t grow = d->ekcap >= cap_limit ? need
                                            : std::min<size_t>(2 * d->ekcap, std::max<size_t>(need, cap_limit));
  const size_t cap = round_up(std::max<size_t>({need, grow, 256}), 256);
  uint32_t *t = nullptr, *p = nullptr, *o = nullptr;
  auto fail = [&]() {
    for (uint32_t* q : {t, p, o}) if (q) (void)hipFree(q);
    return GV_ENOMEM;
  };
  if (hipMalloc(&t, cap * (size_t)GV_EDK_WORDS * 4) != hipSuccess) return fail();
  if (hipMalloc(&p, cap * 8 * 4) != hipSuccess) return fail();
  if (hipMalloc(&o, cap * 4) != hipSuccess) return fail();
  if (used) {
    CK(hipMemcpyAsync(t, d->ektab, used * (size_t)GV_EDK_WORDS * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemcpyAsync(p, d->ekpub, used * 8 * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemcpyAsync(o, d->ekok, used * 4, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
  }
  for (uint32_t* q : {d->ektab, d->ekpub, d->ekok}) if (q) (void)hipFree(q);
  d->ektab = t; d->ekpub = p; d->ekok = o; d->ekcap = cap;
  return GV_OK;
}
}  // namespace

int gv_ed_keys_load(gv_ctx* ctx, size_t n, const uint8_t* pub32, uint32_t* slot_out) {
  if (!ctx) return GV_EINVAL;
  if (n == 0) return GV_OK;
  if (!pub32 || !slot_out) return GV_EINVAL;
  std::lock_guard<std::mutex> kl(ctx->ed_keys_mu);
  const size_t base = ctx->ed_keys;
  if (base + n > kMaxItems) return GV_EINVAL;
  for (Dev* d : ctx->devs) {                    // every device holds every key
    std::lock_guard<std::mutex> lk(d->mu);
    CK(hipSetDevice(d->id));
    hipStream_t st = d->set[0].st;
    int rc = ensure_ed_keys(d, base + n, base, st, ctx->ed_key_cap);
    if (rc) return rc;
    uint8_t* dp = nullptr;
    const size_t o_wb = round_up(n * 32, 256), wb_bytes = n * 64 * 36 * 4;
    const bool split = ctx->ed_keys_split && wb_bytes <= ((size_t)1 << 30);
    if (hipMalloc(&dp, o_wb + (split ? wb_bytes : 0)) != hipSuccess) return GV_ENOMEM;
    if (hipMemcpyAsync(dp, pub32, n * 32, hipMemcpyHostToDevice, st) != hipSuccess ||
        gvk_ed_keys(dp, (uint32_t)n, (uint32_t)base, d->ektab, d->ekpub, d->ekok,
                    split ? (uint32_t*)(dp + o_wb) : nullptr, 4, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      (void)hipFree(dp);
      return GV_EHIP;
    }
    (void)hipFree(dp);
  }
  ctx->ed_kpub.insert(ctx->ed_kpub.end(), pub32, pub32 + n * 32);
  ctx->ed_keys = base + n;
  for (size_t i = 0; i < n; ++i) slot_out[i] = (uint32_t)(base + i);
  return GV_OK;
}

int gv_ed_keys_reset(gv_ctx* ctx) {
  if (!ctx) return GV_EINVAL;
  std::lock_guard<std::mutex> kl(ctx->ed_keys_mu);
  ctx->ed_keys = 0;
  ctx->ed_kpub.clear();
  ctx->ed_keys_gen.fetch_add(1);
  return GV_OK;
}
size_t gv_ed_keys_count(const gv_ctx* ctx) { return ctx ? ctx->ed_keys : 0; }
uint64_t gv_ed_keys_generation(const gv_ctx* ctx) { return ctx ? ctx->ed_keys_gen.load() : 0; }

namespace {
struct EdKeyedHost {
  const uint32_t* slot;
  const uint8_t* sig64;
  const uint8_t* blob;
  const uint64_t* off;
  const uint32_t* len;
  uint8_t* out_ok;
};

int ensure_dev(uint8_t** p, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return GV_OK;
  if (*p) (void)hipFree(*p);
  *cap = 0;
  const size_t c = round_up(bytes, (size_t)1 << 20);
  if (hipMalloc((void**)p, c) != hipSuccess) { *p = nullptr; return GV_ENOMEM; }
  *cap = c;
  return GV_OK;
}

// Items [lo, hi) of a large keyed ed25519 batch on one device (k_ed_keyed):
// chunks alternate between two buffers / streams, so the host staging of
// chunk i + 1 (slots, signatures, offsets, messages into pinned memory) runs
// while chunk i copies and computes; lanes sorted by slot on the device.
int ed_keyed_slice(gv_ctx* ctx, Dev* d, size_t lo, size_t hi, const EdKeyedHost& hb, size_t kcount) {
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  int rc = ed_ensure(d, 256, d->set[0].st);       // the resident comb table of B
  if (rc) return rc;
  const size_t n = hi - lo;
  const size_t chunk = std::min<size_t>(ctx->max_batch, n > 131072 ? round_up((n + 3) / 4, 256) : n);
  const size_t nb = kcount + 1, tb = gvk_sort_temp_bytes((uint32_t)nb);
  struct Pending { size_t c0 = 0, cn = 0, o_out = 0; bool busy = false; } pend[2];
  auto finish = [&](int k) -> int {                // chunk on buffer k: wait, copy the verdicts out
    if (!pend[k].busy) return GV_OK;
    pend[k].busy = false;
    CK(hipStreamSynchronize(d->set[k].st));
    memcpy(hb.out_ok + pend[k].c0, d->edk_h[k] + pend[k].o_out, pend[k].cn);
    return GV_OK;
  };
  auto submit = [&](int k, size_t c0) -> int {
    int rc = finish(k);
    if (rc) return rc;
    hipStream_t st = d->set[k].st;
    const size_t cn = std::min(chunk, hi - c0);
    uint64_t lo_b = UINT64_MAX, hi_b = 0;
    for (size_t i = c0; i < c0 + cn; ++i) {
      lo_b = std::min<uint64_t>(lo_b, hb.off[i]);
      hi_b = std::max<uint64_t>(hi_b, hb.off[i] + hb.len[i]);
    }
    if (lo_b > hi_b) lo_b = hi_b = 0;
    const size_t o_sig = round_up(cn * 4, 256), o_off = o_sig + cn * 64, o_len = o_off + cn * 8,
                 o_out = o_len + cn * 4, o_blob = round_up(o_out + cn, 256), total = o_blob + (hi_b - lo_b);
    const size_t C = round_up(cn, 256), sw = 3 * C + 2 * round_up(nb, 64) + round_up(tb / 4 + 1, 64);
    if ((rc = ensure_pinned(&d->edk_h[k], &d->edk_h_cap[k], total))) return rc;
    if ((rc = ensure_dev(&d->edk_d[k], &d->edk_d_cap[k], total))) return rc;
    if ((rc = ensure_dev((uint8_t**)&d->edk_s[k], &d->edk_s_cap[k], sw * 4))) return rc;
    uint8_t* h = d->edk_h[k];
    const CopySeg segs[2] = {CopySeg{h, (const uint8_t*)(hb.slot + c0), cn * 4},
                             CopySeg{h + o_sig, hb.sig64 + c0 * 64, cn * 64}};
    par_copy_segs(d->pool, segs, 2);
    uint64_t* ro = (uint64_t*)(h + o_off);
    for (size_t i = 0; i < cn; ++i) ro[i] = hb.off[c0 + i] - lo_b;
    memcpy(h + o_len, hb.len + c0, cn * 4);
    if (hi_b > lo_b) par_copy(d->pool, h + o_blob, hb.blob + lo_b, hi_b - lo_b);
    uint8_t* dd = d->edk_d[k];
    CK(hipMemcpyAsync(dd, h, total, hipMemcpyHostToDevice, st));
    uint32_t* p = d->edk_s[k];
    gvk_sort so;
    so.pos = p; p += C;
    so.perm = p; p += C;
    so.kslot = p; p += C;
    so.bits = nullptr;
    so.cnt = p; p += round_up(nb, 64);
    so.off = p; p += round_up(nb, 64);
    so.temp = p;
    so.temp_bytes = tb;
    if (ctx->sort_keys) CK(gvk_sort_slots(&so, (uint32_t)cn, (const uint32_t*)dd, (uint32_t)kcount, st));
    gvk_edk b;
    memset(&b, 0, sizeof b);
    b.n = (uint32_t)cn;
    b.perm = ctx->sort_keys ? so.perm : nullptr;
    b.slot = (const uint32_t*)dd;
    b.sig64 = dd + o_sig;
    b.msg_blob = dd + o_blob;
    b.msg_off = (const uint64_t*)(dd + o_off);
    b.msg_len = (const uint32_t*)(dd + o_len);
    b.ktab = d->ektab;
    b.kpub = d->ekpub;
    b.kok = d->ekok;
    b.kcount = (uint32_t)kcount;
    b.btab = d->edtab;
    b.btab16 = ed_btab16(d, ctx->ed_btab16, st);
    b.out8 = dd + o_out;
    CK(gvk_ed_keyed(&b, st));
    CK(hipMemcpyAsync(h + o_out, dd + o_out, cn, hipMemcpyDeviceToHost, st));
    pend[k] = Pending{c0, cn, o_out, true};
    return GV_OK;
  };
  int k = 0;
  for (size_t c0 = lo; c0 < hi && rc == GV_OK; c0 += chunk, k ^= 1) rc = submit(k, c0);
  for (int j = 0; j < 2; ++j) {                   // drain, the older chunk first (also after an error)
    const int r2 = finish(k ^ j);
    if (rc == GV_OK) rc = r2;
  }
  if (rc) {
    (void)hipStreamSynchronize(d->set[0].st);
    (void)hipStreamSynchronize(d->set[1].st);
  }
  return rc;
}
}  // namespace

int gv_verify_ed25519_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                                 const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                                 uint8_t* out_ok) {
  if (!ctx) return GV_EINVAL;
  if (ctx->fault_inject) return GV_EFAULT;
  if (n == 0) return GV_OK;
  if (!slot || !sig64 || !msg_off || !msg_len || !out_ok) return GV_EINVAL;
  for (size_t i = 0; i < n; ++i)
    if (msg_len[i] && !msg_blob) return GV_EINVAL;
  // ed_keys_mu is held for the whole call, small batches included: a
  // concurrent gv_ed_keys_reset + load cannot move a slot between the lookup
  // of kcount and the kernel (the large-batch path always held it; lock order
  // ed_keys_mu -> d->mu, as in gv_ed_keys_load)
  std::lock_guard<std::mutex> kl(ctx->ed_keys_mu);
  const size_t kcount = ctx->ed_keys;
  {
    if (n > ctx->ed_lat_max && kcount && ctx->ed_keyed) {
      // large batches: one signature per lane against the key tables
      // (k_ed_keyed), split over the devices like run_ed_host
      const EdKeyedHost hb{slot, sig64, msg_blob, msg_off, msg_len, out_ok};
      return run_sliced(workers(ctx), n, 256, [&](size_t k, size_t lo, size_t hi) {
        return ed_keyed_slice(ctx, ctx->devs[k], lo, hi, hb, kcount);
      });
    }
    if (n > ctx->ed_lat_max || kcount == 0) {
      // large batches (ed_keyed 0): the throughput kernels over the slots' raw keys
      std::vector<uint8_t> pub(n * 32, 0);
      for (size_t i = 0; i < n; ++i)
        if (slot[i] < kcount) memcpy(&pub[i * 32], &ctx->ed_kpub[(size_t)slot[i] * 32], 32);
      int rc = kcount ? run_ed_host(ctx, n, EdHost{pub.data(), sig64, msg_blob, msg_off, msg_len, out_ok}) : GV_OK;
      if (rc) return rc;
      for (size_t i = 0; i < n; ++i)
        if (slot[i] >= kcount) out_ok[i] = 0;              // no key in that slot: never a valid signature
      return GV_OK;
    }
  }
  Dev* d = ctx->devs[0];
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  hipStream_t st = d->set[0].st;
  int rc = ed_ensure(d, 256, st);                 // the resident comb table of B
  if (rc) return rc;
  uint64_t lo = UINT64_MAX, hi = 0;
  for (size_t i = 0; i < n; ++i) {
    lo = std::min<uint64_t>(lo, msg_off[i]);
    hi = std::max<uint64_t>(hi, msg_off[i] + msg_len[i]);
  }
  if (lo > hi) lo = hi = 0;
  // zero-copy: the kernel reads the pinned inputs and writes verdict bytes
  const size_t o_sig = round_up(n * 4, 64), o_off = o_sig + n * 64, o_len = o_off + n * 8, o_out = o_len + n * 4,
               o_blob = round_up(o_out + n, 64), total = o_blob + (hi - lo);
  if ((rc = ensure_pinned(&d->edl_h, &d->edl_h_cap, total))) return rc;
  uint8_t* h = d->edl_h;
  memcpy(h, slot, n * 4);
  memcpy(h + o_sig, sig64, n * 64);
  uint64_t* ro = (uint64_t*)(h + o_off);
  for (size_t i = 0; i < n; ++i) ro[i] = msg_off[i] - lo;
  memcpy(h + o_len, msg_len, n * 4);
  if (hi > lo) memcpy(h + o_blob, msg_blob + lo, hi - lo);
  gvk_edl b;
  memset(&b, 0, sizeof b);
  b.n = (uint32_t)n;
  b.slot = (const uint32_t*)h;
  b.sig64 = h + o_sig;
  b.msg_blob = h + o_blob;
  b.msg_off = (const uint64_t*)(h + o_off);
  b.msg_len = (const uint32_t*)(h + o_len);
  b.ktab = d->ektab;
  b.kpub = d->ekpub;
  b.kok = d->ekok;
  b.kcount = (uint32_t)kcount;
  b.btab = d->edtab;
  b.out8 = h + o_out;
  CK(gvk_ed_lat(&b, st));
  CK(hipStreamSynchronize(st));
  memcpy(out_ok, h + o_out, n);
  return GV_OK;
}

int gv_host_alloc(gv_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out || bytes == 0) return GV_EINVAL;
  *out = nullptr;
  if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) { *out = nullptr; return GV_ENOMEM; }
  return GV_OK;
}
int gv_host_free(gv_ctx* ctx, void* p) {
  if (!ctx) return GV_EINVAL;
  if (p && hipHostFree(p) != hipSuccess) return GV_EHIP;
  return GV_OK;
}

int gv_route_stats(gv_ctx* ctx, int dev_slot, uint64_t out[GV_ROUTES]) {
  if (!ctx || !out || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  std::lock_guard<std::mutex> lk(d->mu);
  for (int i = 0; i < GV_ROUTES; ++i) out[i] = d->routes[i];
  return GV_OK;
}

int gv_group_stats(gv_ctx* ctx, int dev_slot, uint64_t* batches, uint64_t* keys) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  std::lock_guard<std::mutex> lk(d->mu);
  if (batches) *batches = d->grouped_batches + d->ed_grouped_batches;
  if (keys) *keys = d->grouped_keys + d->ed_grouped_keys;
  return GV_OK;
}

int gv_last_slices(gv_ctx* ctx, double* ms_out, size_t* n_out, int cap) {
  if (!ctx || cap < 0 || (cap > 0 && (!ms_out || !n_out))) return GV_EINVAL;
  const int m = std::min<int>(cap, (int)ctx->devs.size());
  for (int k = 0; k < m; ++k) {
    Dev* d = ctx->devs[k];
    std::lock_guard<std::mutex> lk(d->mu);
    ms_out[k] = d->last_slice_ms;
    n_out[k] = d->last_slice_n;
  }
  return m;
}
uint64_t gv_keys_generation(const gv_ctx* ctx) { return ctx ? ctx->keys_gen.load() : 0; }

int gv_keys_point(gv_ctx* ctx, size_t n, const uint32_t* slots, uint8_t* out_xy64, uint8_t* out_ok) {
  if (!ctx) return GV_EINVAL;
  if (n == 0) return GV_OK;
  if (!slots || !out_xy64 || !out_ok || n > kMaxItems) return GV_EINVAL;
  Dev* d = ctx->devs[0];
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  hipStream_t st = d->set[0].st;
  int rc = ensure_keys(d, 1, ctx->keys, st, ctx->key_cap, ctx->hbm_budget, nullptr);
  if (rc) return rc;
  uint8_t* buf = nullptr;
  const size_t sb = round_up(n * 4, 256), xb = round_up(n * 64, 256);
  if (hipMalloc(&buf, sb + xb + n) != hipSuccess) return GV_ENOMEM;
  if (hipMemcpyAsync(buf, slots, n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
      gvk_keys_point((uint32_t)n, (const uint32_t*)buf, d->kqt, d->kzq, (uint32_t)d->kcap, d->kok,
                     (uint32_t)ctx->keys, buf + sb, buf + sb + xb, st) != hipSuccess ||
      hipMemcpyAsync(out_xy64, buf + sb, n * 64, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(out_ok, buf + sb + xb, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    rc = GV_EHIP;
  (void)hipFree(buf);
  return rc;
}

int gv_verify_digests_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                            const uint8_t* dig32, uint8_t* out_ok) {
  if (n && (!slot || !dig32)) return GV_EINVAL;
  return run_host(ctx, n, HostBatch{nullptr, sig64, dig32, nullptr, nullptr, nullptr, slot, out_ok, nullptr});
}

int gv_verify_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                         const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                         uint8_t* out_ok) {
  if (n && !slot) return GV_EINVAL;
  return run_host(ctx, n, HostBatch{nullptr, sig64, nullptr, msg_blob, msg_off, msg_len, slot, out_ok, nullptr});
}

int gv_dev_verify_digests_keyed(gv_ctx* ctx, int dev_slot, size_t n, const void* d_slot, const void* d_sig64,
                                const void* d_dig32, void* d_bits, void* stream) {
  Dev* d = nullptr;
  int rc = dev_common(ctx, dev_slot, n, d_slot, d_sig64, d_bits, &d);
  if (rc || n == 0) return rc;
  if (!d_dig32 || ((uintptr_t)d_dig32 & 3)) return GV_EINVAL;
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  return dev_run(ctx, d, stream, n, true, [&](Set* s, hipStream_t st, hipStream_t se) {
    return launch(ctx, d, s, n, nullptr, (const uint8_t*)d_sig64, (const uint8_t*)d_dig32, nullptr, nullptr, nullptr,
                  (uint64_t*)d_bits, st, (const uint32_t*)d_slot, nullptr, se);
  });
}

int gv_get_option(gv_ctx* ctx, const char* key, long long* val) {
  if (!ctx || !key || !val) return GV_EINVAL;
  const struct {
    const char* k;
    long long v;
  } opts[] = {{"kg", ctx->kg},
              {"k6", ctx->k6},
              {"gfull", ctx->gfull},
              {"keys_k6", ctx->keys_k6},
              {"keys_wide", ctx->keys_wide},
              {"group_keys", ctx->group_keys},
              {"sort_keys", ctx->sort_keys},
              {"pipeline_dev", ctx->pipeline_dev},
              {"two_ladders", ctx->two_ladders},
              {"key_cap", (long long)ctx->key_cap},
              {"max_batch", (long long)ctx->max_batch},
              {"async_chunk", (long long)ctx->async_chunk},
              {"async_growth", ctx->async_growth},
              {"async_whole", ctx->async_whole},
              {"lat_kw", ctx->lat_kw},
              {"kw_qw", GV_KW_QW}};                  // read-only: the wide arena's window width (build)
  for (const auto& o : opts)
    if (!strcmp(key, o.k)) {
      *val = o.v;
      return GV_OK;
    }
  return GV_EINVAL;
}

int gv_set_option(gv_ctx* ctx, const char* key, long long val) {
  if (!ctx || !key) return GV_EINVAL;
  if (!strcmp(key, "lat_max") || !strcmp(key, "lat_max_keyed")) {
    if (val < 0 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    if (!strcmp(key, "lat_max")) ctx->lat_max = (size_t)val;
    ctx->lat_max_keyed = (size_t)val;
  } else if (!strcmp(key, "lat_sl_max") || !strcmp(key, "lat_sl_max_keyed")) {
    if (val < 0 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    if (!strcmp(key, "lat_sl_max")) ctx->lat_sl_max = (size_t)val;
    ctx->lat_sl_max_keyed = (size_t)val;
  } else if (!strcmp(key, "ed_unc_lat_max")) {
    if (val < 0 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    ctx->ed_unc_lat_max = (size_t)val;
  } else if (!strcmp(key, "ed_lat_max")) {
    if (val < 0 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    ctx->ed_lat_max = (size_t)val;
  } else if (!strcmp(key, "lat_zero_copy")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->lat_zero_copy = val != 0;
  } else if (!strcmp(key, "lat_sliced")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->lat_sliced = val != 0;
  } else if (!strcmp(key, "lat_rows_max")) {
    if (val < 0 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    ctx->lat_rows_max = (size_t)val;
  } else if (!strcmp(key, "max_batch")) {
    if (val < 256 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    ctx->max_batch = round_up((size_t)val, 256);
  } else if (!strcmp(key, "pipe_chunk")) {
    if (val != 0 && (val < 256 || (unsigned long long)val > kMaxItems)) return GV_EINVAL;
    ctx->pipe_chunk = val ? round_up((size_t)val, 256) : 0;
  } else if (!strcmp(key, "pipe_growth")) {
    if (val < 1 || val > 64) return GV_EINVAL;
    ctx->pipe_growth = (int)val;
  } else if (!strcmp(key, "stage_threads")) {
    if (val < 1 || val > 64) return GV_EINVAL;
    std::vector<std::unique_lock<std::mutex>> held;   // no device stages while its pool is replaced
    for (Dev* d : ctx->devs) held.emplace_back(d->mu);
    ctx->stage_threads = (int)val;
    for (Dev* d : ctx->devs) {
      delete d->pool;
      d->pool = new Pool((int)val - 1);
    }
  } else if (!strcmp(key, "stage_pieces")) {
    if (val < 1 || val > 64) return GV_EINVAL;
    ctx->stage_pieces = (int)val;
  } else if (!strcmp(key, "h2d_serial")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->h2d_serial = val != 0;
  } else if (!strcmp(key, "gfull_item")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->gfull_item = val != 0;
  } else if (!strcmp(key, "inv_small")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->inv_small = val != 0;
  } else if (!strcmp(key, "slice_plain_first")) {
    if (val < 0 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    ctx->slice_plain_first = (size_t)val;
  } else if (!strcmp(key, "group_keys")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->group_keys = val != 0;
  } else if (!strcmp(key, "group_min")) {
    if (val < 256 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    ctx->group_min = (size_t)val;
  } else if (!strcmp(key, "group_div")) {
    if (val < 2 || val > 1024) return GV_EINVAL;
    ctx->group_div = (int)val;
  } else if (!strcmp(key, "ed_btab16")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->ed_btab16 = val != 0;
  } else if (!strcmp(key, "ed_group_r64")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->ed_group_r64 = val != 0;
  } else if (!strcmp(key, "ed_keys_split")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->ed_keys_split = val != 0;
  } else if (!strcmp(key, "ed_group")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->ed_group = val != 0;
  } else if (!strcmp(key, "ed_group_min")) {
    if (val < 256 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    ctx->ed_group_min = (size_t)val;
  } else if (!strcmp(key, "ed_keyed")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->ed_keyed = val != 0;
  } else if (!strcmp(key, "keys_wide")) {
    // the layout of an arena started from slot 0 from now on (a running arena
    // keeps its layout until gv_keys_reset); 0 stops its use at once
    if (val < 0 || val > 2) return GV_EINVAL;
    std::vector<std::unique_lock<std::mutex>> held;
    for (Dev* d : ctx->devs) held.emplace_back(d->mu);
    for (Dev* d : ctx->devs) {
      CK(hipSetDevice(d->id));
      for (hipStream_t t : d->hi_st) CK(hipStreamSynchronize(t));
      d->bits_used = false;
    }
    ctx->keys_wide = (int)val;
  } else if (!strcmp(key, "kg")) {
    if (!kg_layout_ok((int)val)) return GV_EINVAL;
    std::vector<std::unique_lock<std::mutex>> held;
    for (Dev* d : ctx->devs) held.emplace_back(d->mu);
    for (Dev* d : ctx->devs) {
      CK(hipSetDevice(d->id));
      for (hipStream_t t : d->hi_st) CK(hipStreamSynchronize(t));
      d->bits_used = false;
    }
    ctx->kg = (int)val;
  } else if (!strcmp(key, "keys_wide1_cap")) {
    if (val < 0) return GV_EINVAL;
    ctx->keys_wide1_cap = val == 0 ? SIZE_MAX : (size_t)val;
  } else if (!strcmp(key, "two_ladders") || !strcmp(key, "gfull") || !strcmp(key, "k6") ||
             !strcmp(key, "keys_k6")) {
    // schedule switches: every device lock held across the drain and the
    // write, so no pipelined call launches on a mix of old and new state
    if (val != 0 && val != 1) return GV_EINVAL;
    std::vector<std::unique_lock<std::mutex>> held;
    for (Dev* d : ctx->devs) held.emplace_back(d->mu);
    for (Dev* d : ctx->devs) {
      CK(hipSetDevice(d->id));
      for (hipStream_t t : d->hi_st) CK(hipStreamSynchronize(t));
      d->bits_used = false;
    }
    bool& flag = !strcmp(key, "two_ladders") ? ctx->two_ladders : !strcmp(key, "gfull") ? ctx->gfull
                 : !strcmp(key, "k6") ? ctx->k6 : ctx->keys_k6;
    flag = val != 0;
  } else if (!strcmp(key, "async_chunk")) {
    if (val < 256 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    ctx->async_chunk = round_up((size_t)val, 256);
  } else if (!strcmp(key, "lat_kw")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->lat_kw = val != 0;
  } else if (!strcmp(key, "async_whole")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->async_whole = val != 0;
  } else if (!strcmp(key, "async_growth")) {
    if (val < 1 || val > 64) return GV_EINVAL;
    ctx->async_growth = (int)val;
  } else if (!strcmp(key, "host_ladder_stream")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->host_ladder_stream = val != 0;
  } else if (!strcmp(key, "key_cap") || !strcmp(key, "ed_key_cap")) {
    if (val < 256 || (unsigned long long)val > kMaxItems) return GV_EINVAL;
    (!strcmp(key, "key_cap") ? ctx->key_cap : ctx->ed_key_cap) = (size_t)val;
  } else if (!strcmp(key, "hbm_budget_mb")) {
    if (val < 0) return GV_EINVAL;
    ctx->hbm_budget = val == 0 ? SIZE_MAX : (size_t)val << 20;
  } else if (!strcmp(key, "sort_keys")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->sort_keys = val != 0;
  } else if (!strcmp(key, "pipeline_dev")) {
    if (val != 0 && val != 1) return GV_EINVAL;
    ctx->pipeline_dev = val != 0;
  } else if (!strcmp(key, "time_kernels")) {
    ctx->time_kernels = val != 0;
  } else if (!strcmp(key, "fault_inject")) {
    ctx->fault_inject = val != 0;
  } else {
    return GV_EINVAL;
  }
  return GV_OK;
}

// [unpack/sha, s^-1, prep, ladder] ms of one launch (ladder: its own start to end)
static int stage_ms(hipEvent_t* e, float ms[4]) {
  CK(hipEventSynchronize(e[5]));
  for (int i = 0; i < 3; ++i) CK(hipEventElapsedTime(&ms[i], e[i], e[i + 1]));
  CK(hipEventElapsedTime(&ms[3], e[4], e[5]));
  return GV_OK;
}

int gv_last_stage_ms(gv_ctx* ctx, int dev_slot, float* unpack_ms, float* prep_ms, float* ecmult_ms) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  if (!ctx->time_kernels) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  if (d->last < 0) return GV_EINVAL;
  CK(hipSetDevice(d->id));
  float ms[4];
  int rc = stage_ms(d->ring[d->last], ms);
  if (rc) return rc;
  if (unpack_ms) *unpack_ms = ms[0];
  if (prep_ms) *prep_ms = ms[1] + ms[2];
  if (ecmult_ms) *ecmult_ms = ms[3];
  return GV_OK;
}

int gv_stage_stats4(gv_ctx* ctx, int dev_slot, int* count, double ms_out[4]) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size() || !ms_out) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  double sum[4] = {0, 0, 0, 0};
  const int cnt = d->ring_count;
  for (int k = 0; k < cnt; ++k) {
    float ms[4];
    int rc = stage_ms(d->ring[(d->ring_next - 1 - k + Dev::kRing) % Dev::kRing], ms);
    if (rc) return rc;
    for (int i = 0; i < 4; ++i) sum[i] += ms[i];
  }
  d->ring_count = 0;
  if (count) *count = cnt;
  for (int i = 0; i < 4; ++i) ms_out[i] = cnt ? sum[i] / cnt : 0.0;
  return GV_OK;
}

int gv_stage_stats(gv_ctx* ctx, int dev_slot, int* count, double* unpack_ms, double* prep_ms,
                   double* ecmult_ms) {
  double ms[4];
  int rc = gv_stage_stats4(ctx, dev_slot, count, ms);
  if (rc) return rc;
  if (unpack_ms) *unpack_ms = ms[0];
  if (prep_ms) *prep_ms = ms[1] + ms[2];
  if (ecmult_ms) *ecmult_ms = ms[3];
  return GV_OK;
}

int gv_dev_alloc(gv_ctx* ctx, int dev_slot, size_t bytes, void** d_ptr) {
  if (!ctx || !d_ptr || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  *d_ptr = nullptr;
  CK(hipSetDevice(ctx->devs[dev_slot]->id));
  if (hipMalloc(d_ptr, std::max<size_t>(bytes, 1)) != hipSuccess) return GV_ENOMEM;
  return GV_OK;
}

int gv_dev_free(gv_ctx* ctx, int dev_slot, void* d_ptr) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  CK(hipSetDevice(ctx->devs[dev_slot]->id));
  if (d_ptr) CK(hipFree(d_ptr));
  return GV_OK;
}

int gv_dev_copy(gv_ctx* ctx, int dev_slot, void* dst, const void* src, size_t bytes, int kind) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  if (bytes == 0) return GV_OK;
  if (!dst || !src) return GV_EINVAL;
  hipMemcpyKind k;
  switch (kind) {
    case 1: k = hipMemcpyHostToDevice; break;
    case 2: k = hipMemcpyDeviceToHost; break;
    case 3: k = hipMemcpyDeviceToDevice; break;
    default: return GV_EINVAL;
  }
  Dev* d = ctx->devs[dev_slot];
  CK(hipSetDevice(d->id));
  for (hipStream_t t : {d->lo_st[0], d->lo_st[1], d->hi_st[0], d->hi_st[1]})   // after every pipelined call (synchronous copy)
    CK(hipStreamSynchronize(t));
  hipStream_t st = d->set[0].st;
  CK(hipMemcpyAsync(dst, src, bytes, k, st));
  CK(hipStreamSynchronize(st));
  return GV_OK;
}

int gv_dev_stream_create(gv_ctx* ctx, int dev_slot, void** stream_out) {
  if (!ctx || !stream_out || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  *stream_out = nullptr;
  CK(hipSetDevice(ctx->devs[dev_slot]->id));
  hipStream_t st = nullptr;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  *stream_out = (void*)st;
  return GV_OK;
}

int gv_dev_stream_sync(gv_ctx* ctx, int dev_slot, void* stream) {
  if (!ctx || !stream || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  CK(hipSetDevice(ctx->devs[dev_slot]->id));
  CK(hipStreamSynchronize((hipStream_t)stream));
  return GV_OK;
}

int gv_dev_stream_destroy(gv_ctx* ctx, int dev_slot, void* stream) {
  if (!ctx || !stream || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  CK(hipSetDevice(ctx->devs[dev_slot]->id));
  CK(hipStreamDestroy((hipStream_t)stream));
  return GV_OK;
}

int gv_dev_sync(gv_ctx* ctx, int dev_slot) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  CK(hipSetDevice(d->id));
  for (Set& s : d->set) CK(hipStreamSynchronize(s.st));
  for (hipStream_t t : {d->lo_st[0], d->lo_st[1], d->hi_st[0], d->hi_st[1]}) CK(hipStreamSynchronize(t));
  return GV_OK;
}

const char* gv_strerror(int code) {
  switch (code) {
    case GV_OK: return "ok";
    case GV_EINVAL: return "invalid argument";
    case GV_ENODEV: return "no usable HIP device";
    case GV_EHIP: return "HIP runtime error";
    case GV_ENOMEM: return "out of memory";
    case GV_EFAULT: return "injected fault";
    default: return "unknown error";
  }
}

#if GV_STAMP
// Diagnostic builds only (not in gpuverify.h): the k_ecmult wave stamps of
// the last launches on dev_slot (tools/ecmult_stamps.py).
int gv_diag_stamps(gv_ctx* ctx, int dev_slot, uint64_t* out, size_t n_u64) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size() || !out) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  CK(hipDeviceSynchronize());
  CK(gvk_stamps_read(out, n_u64));
  return GV_OK;
}
#endif

int gv_debug_op(gv_ctx* ctx, int dev_slot, int op, size_t n, const uint32_t* in, uint32_t* out) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size() || !in || !out) return GV_EINVAL;
  if (n == 0) return GV_OK;
  if (n > kMaxItems) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  hipStream_t st = d->set[0].st;
  const size_t npad = round_up(n, 256);
  uint32_t *din = nullptr, *dout = nullptr;
  CK(hipMalloc(&din, npad * 64));
  if (hipMalloc(&dout, npad * 64) != hipSuccess) { (void)hipFree(din); return GV_ENOMEM; }
  int rc = GV_OK;
  if (hipMemsetAsync(din, 0, npad * 64, st) != hipSuccess ||
      hipMemcpyAsync(din, in, n * 64, hipMemcpyHostToDevice, st) != hipSuccess ||
      gvk_debug(op, (uint32_t)n, din, dout, st) != hipSuccess ||
      hipMemcpyAsync(out, dout, n * 64, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    rc = GV_EHIP;
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}

}  // extern "C"
