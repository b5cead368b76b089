// gv_runtime.cpp -- the C-ABI runtime of libgpuverify.so (include/gpuverify.h).
//
// Owns per-device state (stream, LDS-source G table, scratch buffers sized for
// the largest batch seen), splits host batches across the context's devices
// (contiguous slices, one host thread per device, no collective -- SURVEY.md
// §8e), streams each slice through the HIP pipeline in max_batch chunks and
// gathers the accept bitmaps.  Fail-closed: any HIP error returns GV_EHIP and
// the caller re-verifies on the CPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/gpuverify.h"
#include "gv_kernels.h"

namespace {

#define CK(call)                                  \
  do {                                            \
    hipError_t e_ = (call);                       \
    if (e_ != hipSuccess) return GV_EHIP;         \
  } while (0)

constexpr size_t kLaneWords = 8 + 1 + 8 + 8 + 8 + GV_DIGIT_ROWS + 8 + 1 + GV_QTAB_WORDS;

struct Dev {
  int id = 0;
  hipStream_t st = nullptr;
  uint32_t* gtab = nullptr;
  size_t cap = 0;               // lanes of scratch (multiple of 256)
  uint8_t* scratch = nullptr;   // one allocation, carved below
  uint8_t *d_pub = nullptr, *d_sig = nullptr, *d_dig = nullptr;
  uint32_t *in_x, *in_pfx, *in_r, *in_s, *in_e, *digits, *zq, *flags, *qtab;
  uint64_t* bits = nullptr;
  uint8_t* d_blob = nullptr;
  size_t blob_cap = 0;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  size_t msg_cap = 0;
  uint64_t* h_bits = nullptr;   // pinned
  size_t h_bits_cap = 0;
  uint32_t* d_slot = nullptr;   // keyed host batches: slot column (part of scratch)
  // key arena (gv_keys_load): Q table rows, table Z (8 rows of stride kcap), verdicts
  uint32_t *kqt = nullptr, *kzq = nullptr, *kok = nullptr;
  size_t kcap = 0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // ring of per-launch stage events for gv_stage_stats
  static constexpr int kRing = 256;
  hipEvent_t ring[kRing][4] = {};
  int ring_next = 0, ring_count = 0, last = -1;
  std::mutex mu;
};

size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

int ensure_cap(Dev* d, size_t C) {
  if (C <= d->cap) return GV_OK;
  if (d->scratch) { (void)hipFree(d->scratch); d->scratch = nullptr; d->cap = 0; }
  const size_t bytes = C * (33 + 64 + 32) + C * kLaneWords * 4 + (C / 64) * 8 + C * 4 + 4096;
  if (hipMalloc(&d->scratch, bytes) != hipSuccess) return GV_ENOMEM;
  uint8_t* p = d->scratch;
  auto take = [&](size_t nbytes) { uint8_t* r = p; p += round_up(nbytes, 256); return r; };
  d->d_pub = take(C * 33);
  d->d_sig = take(C * 64);
  d->d_dig = take(C * 32);
  d->in_x = (uint32_t*)take(C * 8 * 4);
  d->in_pfx = (uint32_t*)take(C * 4);
  d->in_r = (uint32_t*)take(C * 8 * 4);
  d->in_s = (uint32_t*)take(C * 8 * 4);
  d->in_e = (uint32_t*)take(C * 8 * 4);
  d->digits = (uint32_t*)take(C * GV_DIGIT_ROWS * 4);
  d->zq = (uint32_t*)take(C * 8 * 4);
  d->flags = (uint32_t*)take(C * 4);
  d->qtab = (uint32_t*)take(C * GV_QTAB_WORDS * 4);
  d->bits = (uint64_t*)take((C / 64) * 8);
  d->d_slot = (uint32_t*)take(C * 4);
  d->cap = C;
  return GV_OK;
}

int ensure_msg(Dev* d, size_t blob_bytes, size_t C) {
  if (blob_bytes > d->blob_cap) {
    if (d->d_blob) (void)hipFree(d->d_blob);
    d->blob_cap = round_up(std::max<size_t>(blob_bytes, 1), 1 << 20);
    if (hipMalloc(&d->d_blob, d->blob_cap) != hipSuccess) { d->blob_cap = 0; d->d_blob = nullptr; return GV_ENOMEM; }
  }
  if (C > d->msg_cap) {
    if (d->d_off) (void)hipFree(d->d_off);
    if (d->d_len) (void)hipFree(d->d_len);
    d->d_off = nullptr; d->d_len = nullptr; d->msg_cap = 0;
    if (hipMalloc(&d->d_off, C * 8) != hipSuccess) return GV_ENOMEM;
    if (hipMalloc(&d->d_len, C * 4) != hipSuccess) return GV_ENOMEM;
    d->msg_cap = C;
  }
  return GV_OK;
}

// Grow the key arena to hold `need` slots, keeping the first `used` (row
// stride of kzq changes with the capacity).
int ensure_keys(Dev* d, size_t need, size_t used, hipStream_t st) {
  if (need <= d->kcap) return GV_OK;
  const size_t cap = round_up(std::max<size_t>({need, 2 * d->kcap, 4096}), 256);
  uint32_t *qt = nullptr, *zq = nullptr, *ok = nullptr;
  if (hipMalloc(&qt, cap * GV_KEY_WORDS * 4) != hipSuccess) return GV_ENOMEM;
  if (hipMalloc(&zq, cap * 8 * 4) != hipSuccess) { (void)hipFree(qt); return GV_ENOMEM; }
  if (hipMalloc(&ok, cap * 4) != hipSuccess) { (void)hipFree(qt); (void)hipFree(zq); return GV_ENOMEM; }
  if (used) {
    CK(hipMemcpyAsync(qt, d->kqt, used * GV_KEY_WORDS * 4, hipMemcpyDeviceToDevice, st));
    for (int r = 0; r < 8; ++r)
      CK(hipMemcpyAsync(zq + r * cap, d->kzq + r * d->kcap, used * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemcpyAsync(ok, d->kok, used * 4, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
  }
  if (d->kqt) (void)hipFree(d->kqt);
  if (d->kzq) (void)hipFree(d->kzq);
  if (d->kok) (void)hipFree(d->kok);
  d->kqt = qt; d->kzq = zq; d->kok = ok; d->kcap = cap;
  return GV_OK;
}

int ensure_hbits(Dev* d, size_t words) {
  if (words <= d->h_bits_cap) return GV_OK;
  if (d->h_bits) (void)hipHostFree(d->h_bits);
  d->h_bits = nullptr;
  if (hipHostMalloc(&d->h_bits, words * 8, hipHostMallocDefault) != hipSuccess) { d->h_bits_cap = 0; return GV_ENOMEM; }
  d->h_bits_cap = words;
  return GV_OK;
}

}  // namespace

struct gv_ctx {
  std::vector<Dev*> devs;
  size_t max_batch = size_t(1) << 20;
  size_t lat_max = 4096;        // batches up to this size take the fused latency kernel (gv_lat.hip)
  bool time_kernels = false;
  bool fault_inject = false;
  size_t keys = 0;              // key-arena slots in use (same on every device)
  std::mutex keys_mu;
};

namespace {

// Launch the pipeline for n items whose inputs already sit on the device.
int launch(gv_ctx* ctx, Dev* d, size_t n, const uint8_t* pub, const uint8_t* sig, const uint8_t* dig,
           const uint8_t* blob, const uint64_t* off, const uint32_t* len, uint64_t* bits_out,
           hipStream_t st, const uint32_t* kslot = nullptr) {
  const size_t C = round_up(std::max<size_t>(n, 1), 256);
  int rc = ensure_cap(d, C);
  if (rc) return rc;
  if (kslot) {                                  // the arena always exists for a keyed batch
    rc = ensure_keys(d, 1, ctx->keys, st);
    if (rc) return rc;
  }
  gvk_batch b;
  memset(&b, 0, sizeof b);
  b.n = (uint32_t)n; b.C = (uint32_t)C;
  b.pub33 = pub; b.sig64 = sig; b.dig32 = dig;
  b.msg_blob = blob; b.msg_off = off; b.msg_len = len;
  b.gtab = d->gtab;
  b.in_x = d->in_x; b.in_pfx = d->in_pfx; b.in_r = d->in_r; b.in_s = d->in_s; b.in_e = d->in_e;
  b.digits = d->digits; b.zq = d->zq; b.flags = d->flags; b.qtab = d->qtab;
  b.bits = bits_out;
  if (kslot) {
    b.pub33 = nullptr;
    b.kslot = kslot; b.kqt = d->kqt; b.kzq = d->kzq; b.kok = d->kok;
    b.kC = (uint32_t)d->kcap; b.kcount = (uint32_t)ctx->keys;
  }
  hipEvent_t* rs = nullptr;
  if (ctx->time_kernels) {
    rs = d->ring[d->ring_next];
    for (int i = 0; i < 4; ++i)
      if (!rs[i]) CK(hipEventCreate(&rs[i]));
    CK(hipEventRecord(rs[3], st));
    b.ev[0] = rs[0]; b.ev[1] = rs[1]; b.ev[2] = rs[2];
  }
  if (n <= ctx->lat_max) {
    // small batch: one fused kernel, several lanes per signature (gv_lat.hip)
    gvk_lat lb;
    memset(&lb, 0, sizeof lb);
    lb.n = (uint32_t)n; lb.C = (uint32_t)C;
    lb.pub33 = pub; lb.sig64 = sig; lb.dig32 = dig;
    lb.msg_blob = blob; lb.msg_off = off; lb.msg_len = len;
    lb.gtab = d->gtab; lb.e_soa = d->in_e; lb.bits = bits_out;
    lb.ev[0] = b.ev[0];
    if (kslot) {
      lb.pub33 = nullptr;
      lb.kslot = kslot; lb.kqt = b.kqt; lb.kzq = b.kzq; lb.kok = b.kok; lb.kC = b.kC; lb.kcount = b.kcount;
    }
    CK(gvk_verify_lat(&lb, st));
    if (rs) {                                   // stages: SHA | fused kernel | (none)
      CK(hipEventRecord(rs[1], st));
      CK(hipEventRecord(rs[2], st));
    }
  } else {
    CK(gvk_verify(&b, st));
  }
  if (rs) {
    // mirror the last launch into ev[] for gv_last_stage_ms
    d->last = d->ring_next;
    d->ring_next = (d->ring_next + 1) % Dev::kRing;
    d->ring_count = std::min(d->ring_count + 1, Dev::kRing);
  }
  return GV_OK;
}

// Verify items [lo, hi) of a host batch on one device.  out_ok or out_bits.
int run_slice(gv_ctx* ctx, Dev* d, size_t lo, size_t hi, const uint8_t* pub33, const uint8_t* sig64,
              const uint8_t* dig32, const uint8_t* blob, const uint64_t* off, const uint32_t* len,
              uint8_t* out_ok, uint64_t* out_bits, const uint32_t* slots) {
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  const size_t chunk = ctx->max_batch;
  std::vector<uint64_t> roff;
  for (size_t c0 = lo; c0 < hi; c0 += chunk) {
    const size_t cn = std::min(chunk, hi - c0);
    const size_t C = round_up(cn, 256);
    int rc = ensure_cap(d, C);
    if (rc) return rc;
    rc = ensure_hbits(d, C / 64);
    if (rc) return rc;
    if (slots) CK(hipMemcpyAsync(d->d_slot, slots + c0, cn * 4, hipMemcpyHostToDevice, d->st));
    else CK(hipMemcpyAsync(d->d_pub, pub33 + c0 * 33, cn * 33, hipMemcpyHostToDevice, d->st));
    CK(hipMemcpyAsync(d->d_sig, sig64 + c0 * 64, cn * 64, hipMemcpyHostToDevice, d->st));
    const uint8_t* ddig = nullptr;
    const uint8_t* dblob = nullptr;
    if (dig32) {
      CK(hipMemcpyAsync(d->d_dig, dig32 + c0 * 32, cn * 32, hipMemcpyHostToDevice, d->st));
      ddig = d->d_dig;
    } else {
      uint64_t bmin = UINT64_MAX, bmax = 0;
      for (size_t i = c0; i < c0 + cn; ++i) {
        bmin = std::min<uint64_t>(bmin, off[i]);
        bmax = std::max<uint64_t>(bmax, off[i] + len[i]);
      }
      if (cn == 0 || bmin > bmax) bmin = bmax = 0;
      rc = ensure_msg(d, bmax - bmin, C);
      if (rc) return rc;
      roff.resize(cn);
      for (size_t i = 0; i < cn; ++i) roff[i] = off[c0 + i] - bmin;
      if (bmax > bmin) CK(hipMemcpyAsync(d->d_blob, blob + bmin, bmax - bmin, hipMemcpyHostToDevice, d->st));
      CK(hipMemcpyAsync(d->d_off, roff.data(), cn * 8, hipMemcpyHostToDevice, d->st));
      CK(hipMemcpyAsync(d->d_len, len + c0, cn * 4, hipMemcpyHostToDevice, d->st));
      dblob = d->d_blob;
    }
    rc = launch(ctx, d, cn, d->d_pub, d->d_sig, ddig, dblob, dblob ? d->d_off : nullptr,
                dblob ? d->d_len : nullptr, d->bits, d->st, slots ? d->d_slot : nullptr);
    if (rc) return rc;
    const size_t words = (cn + 63) / 64;
    CK(hipMemcpyAsync(d->h_bits, d->bits, words * 8, hipMemcpyDeviceToHost, d->st));
    CK(hipStreamSynchronize(d->st));
    if (out_ok) {
      for (size_t i = 0; i < cn; ++i) out_ok[c0 + i] = (uint8_t)((d->h_bits[i >> 6] >> (i & 63)) & 1u);
    } else {
      // c0 is a multiple of 64 (slices and chunks are multiples of 256)
      memcpy(out_bits + c0 / 64, d->h_bits, words * 8);
    }
  }
  return GV_OK;
}

int run_host(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32,
             const uint8_t* blob, const uint64_t* off, const uint32_t* len, uint8_t* out_ok,
             uint64_t* out_bits, const uint32_t* slots = nullptr) {
  if (!ctx) return GV_EINVAL;
  if (ctx->fault_inject) return GV_EFAULT;
  if (n == 0) return GV_OK;
  if ((!pub33 && !slots) || !sig64 || (!out_ok && !out_bits)) return GV_EINVAL;
  if (!dig32 && (!blob || !off || !len)) return GV_EINVAL;
  const size_t nd = ctx->devs.size();
  const size_t per = round_up((n + nd - 1) / nd, 256);
  std::vector<int> rcs(nd, GV_OK);
  std::vector<std::thread> th;
  for (size_t k = 0; k < nd; ++k) {
    const size_t lo = std::min(n, k * per), hi = std::min(n, (k + 1) * per);
    if (lo >= hi) continue;
    auto job = [=, &rcs]() {
      rcs[k] = run_slice(ctx, ctx->devs[k], lo, hi, pub33, sig64, dig32, blob, off, len, out_ok, out_bits, slots);
    };
    if (nd == 1) job(); else th.emplace_back(job);
  }
  for (auto& t : th) t.join();
  for (int rc : rcs) if (rc) return rc;
  return GV_OK;
}

}  // namespace

extern "C" {

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
  gv_ctx* ctx = new gv_ctx();
  if (const char* mb = getenv("GV_MAX_BATCH")) {
    long long v = atoll(mb);
    if (v >= 256) ctx->max_batch = round_up((size_t)v, 256);
  }
  for (int id : ids) {
    Dev* d = new Dev();
    d->id = id;
    ctx->devs.push_back(d);
    if (hipSetDevice(id) != hipSuccess ||
        hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d->gtab, (size_t)2 * GV_GTAB_N * 16 * 4) != hipSuccess ||
        gvk_gen_gtable(d->gtab, d->st) != hipSuccess ||
        hipStreamSynchronize(d->st) != hipSuccess) {
      gv_close(ctx);
      return GV_EHIP;
    }
    for (auto& e : d->ev)
      if (hipEventCreate(&e) != hipSuccess) { gv_close(ctx); return GV_EHIP; }
  }
  *out = ctx;
  return GV_OK;
}

void gv_close(gv_ctx* ctx) {
  if (!ctx) return;
  for (Dev* d : ctx->devs) {
    (void)hipSetDevice(d->id);
    if (d->st) (void)hipStreamSynchronize(d->st);
    if (d->scratch) (void)hipFree(d->scratch);
    if (d->gtab) (void)hipFree(d->gtab);
    if (d->d_blob) (void)hipFree(d->d_blob);
    if (d->d_off) (void)hipFree(d->d_off);
    if (d->d_len) (void)hipFree(d->d_len);
    if (d->h_bits) (void)hipHostFree(d->h_bits);
    if (d->kqt) (void)hipFree(d->kqt);
    if (d->kzq) (void)hipFree(d->kzq);
    if (d->kok) (void)hipFree(d->kok);
    for (auto e : d->ev) if (e) (void)hipEventDestroy(e);
    for (auto& rs : d->ring)
      for (auto e : rs) if (e) (void)hipEventDestroy(e);
    if (d->st) (void)hipStreamDestroy(d->st);
    delete d;
  }
  delete ctx;
}

int gv_num_devices(const gv_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int gv_verify_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                   const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                   uint8_t* out_ok) {
  return run_host(ctx, n, pub33, sig64, nullptr, msg_blob, msg_off, msg_len, out_ok, nullptr);
}

int gv_verify_digests(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                      const uint8_t* dig32, uint8_t* out_ok) {
  if (!dig32 && n) return GV_EINVAL;
  return run_host(ctx, n, pub33, sig64, dig32, nullptr, nullptr, nullptr, out_ok, nullptr);
}

int gv_verify_digests_bits(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                           const uint8_t* dig32, uint64_t* out_bits) {
  if (!dig32 && n) return GV_EINVAL;
  return run_host(ctx, n, pub33, sig64, dig32, nullptr, nullptr, nullptr, nullptr, out_bits);
}

int gv_verify_msgs_bits(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64,
                        const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                        uint64_t* out_bits) {
  return run_host(ctx, n, pub33, sig64, nullptr, msg_blob, msg_off, msg_len, nullptr, out_bits);
}

static int dev_common(gv_ctx* ctx, int slot, size_t n, const void* pub, const void* sig, void* bits,
                      Dev** dout) {
  if (!ctx) return GV_EINVAL;
  if (ctx->fault_inject) return GV_EFAULT;
  if (slot < 0 || slot >= (int)ctx->devs.size()) return GV_ENODEV;
  if (n == 0) return GV_OK;
  if (!pub || !sig || !bits) return GV_EINVAL;
  if (((uintptr_t)pub & 3) || ((uintptr_t)sig & 3)) return GV_EINVAL;
  if (n > 0xFFFFFF00ull) return GV_EINVAL;
  *dout = ctx->devs[slot];
  return GV_OK;
}

int gv_dev_verify_digests(gv_ctx* ctx, int dev_slot, size_t n, const void* d_pub33,
                          const void* d_sig64, const void* d_dig32, void* d_bits, void* stream) {
  Dev* d = nullptr;
  int rc = dev_common(ctx, dev_slot, n, d_pub33, d_sig64, d_bits, &d);
  if (rc || n == 0) return rc;
  if (!d_dig32 || ((uintptr_t)d_dig32 & 3)) return GV_EINVAL;
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  hipStream_t st = stream ? (hipStream_t)stream : d->st;
  return launch(ctx, d, n, (const uint8_t*)d_pub33, (const uint8_t*)d_sig64, (const uint8_t*)d_dig32,
                nullptr, nullptr, nullptr, (uint64_t*)d_bits, st);
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
  hipStream_t st = stream ? (hipStream_t)stream : d->st;
  return launch(ctx, d, n, (const uint8_t*)d_pub33, (const uint8_t*)d_sig64, nullptr,
                (const uint8_t*)d_msg_blob, (const uint64_t*)d_msg_off, (const uint32_t*)d_msg_len,
                (uint64_t*)d_bits, st);
}

// ---- key arena
int gv_keys_load(gv_ctx* ctx, size_t n, const uint8_t* pub33, uint32_t* slot_out) {
  if (!ctx) return GV_EINVAL;
  if (n == 0) return GV_OK;
  if (!pub33 || !slot_out) return GV_EINVAL;
  std::lock_guard<std::mutex> kl(ctx->keys_mu);
  const size_t base = ctx->keys;
  if (base + n > 0xFFFFFF00ull) return GV_EINVAL;
  for (Dev* d : ctx->devs) {                    // every device holds every key
    std::lock_guard<std::mutex> lk(d->mu);
    CK(hipSetDevice(d->id));
    int rc = ensure_keys(d, base + n, base, d->st);
    if (rc) return rc;
    for (size_t c0 = 0; c0 < n; c0 += ctx->max_batch) {
      const size_t cn = std::min(ctx->max_batch, n - c0);
      const size_t C = round_up(cn, 256);
      rc = ensure_cap(d, C);
      if (rc) return rc;
      CK(hipMemcpyAsync(d->d_pub, pub33 + c0 * 33, cn * 33, hipMemcpyHostToDevice, d->st));
      CK(gvk_keys_build(d->d_pub, (uint32_t)cn, (uint32_t)C, d->in_x, d->in_pfx, d->in_r, d->in_s, d->in_e,
                        d->qtab + C * GV_QTAB_N * GV_QENT_WORDS, (uint32_t)(base + c0), d->kqt, d->kzq,
                        (uint32_t)d->kcap, d->kok, d->st));
    }
    CK(hipStreamSynchronize(d->st));
  }
  ctx->keys = base + n;
  for (size_t i = 0; i < n; ++i) slot_out[i] = (uint32_t)(base + i);
  return GV_OK;
}

int gv_keys_reset(gv_ctx* ctx) {
  if (!ctx) return GV_EINVAL;
  std::lock_guard<std::mutex> kl(ctx->keys_mu);
  ctx->keys = 0;
  return GV_OK;
}

size_t gv_keys_count(const gv_ctx* ctx) { return ctx ? ctx->keys : 0; }

int gv_verify_digests_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                            const uint8_t* dig32, uint8_t* out_ok) {
  if (n && (!slot || !dig32)) return GV_EINVAL;
  return run_host(ctx, n, nullptr, sig64, dig32, nullptr, nullptr, nullptr, out_ok, nullptr, slot);
}

int gv_verify_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                         const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                         uint8_t* out_ok) {
  if (n && !slot) return GV_EINVAL;
  return run_host(ctx, n, nullptr, sig64, nullptr, msg_blob, msg_off, msg_len, out_ok, nullptr, slot);
}

int gv_dev_verify_digests_keyed(gv_ctx* ctx, int dev_slot, size_t n, const void* d_slot, const void* d_sig64,
                                const void* d_dig32, void* d_bits, void* stream) {
  Dev* d = nullptr;
  int rc = dev_common(ctx, dev_slot, n, d_slot, d_sig64, d_bits, &d);
  if (rc || n == 0) return rc;
  if (!d_dig32 || ((uintptr_t)d_dig32 & 3)) return GV_EINVAL;
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  hipStream_t st = stream ? (hipStream_t)stream : d->st;
  return launch(ctx, d, n, nullptr, (const uint8_t*)d_sig64, (const uint8_t*)d_dig32, nullptr, nullptr, nullptr,
                (uint64_t*)d_bits, st, (const uint32_t*)d_slot);
}

int gv_set_option(gv_ctx* ctx, const char* key, long long val) {
  if (!ctx || !key) return GV_EINVAL;
  if (!strcmp(key, "lat_max")) {
    if (val < 0) return GV_EINVAL;
    ctx->lat_max = (size_t)val;
  } else if (!strcmp(key, "max_batch")) {
    if (val < 256) return GV_EINVAL;
    ctx->max_batch = round_up((size_t)val, 256);
  } else if (!strcmp(key, "time_kernels")) {
    ctx->time_kernels = val != 0;
  } else if (!strcmp(key, "fault_inject")) {
    ctx->fault_inject = val != 0;
  } else {
    return GV_EINVAL;
  }
  return GV_OK;
}

int gv_last_stage_ms(gv_ctx* ctx, int dev_slot, float* unpack_ms, float* prep_ms, float* ecmult_ms) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  if (!ctx->time_kernels) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  if (d->last < 0) return GV_EINVAL;
  CK(hipSetDevice(d->id));
  hipEvent_t* e = d->ring[d->last];
  CK(hipEventSynchronize(e[2]));
  float a = 0, b = 0, c = 0;
  CK(hipEventElapsedTime(&a, e[3], e[0]));
  CK(hipEventElapsedTime(&b, e[0], e[1]));
  CK(hipEventElapsedTime(&c, e[1], e[2]));
  if (unpack_ms) *unpack_ms = a;
  if (prep_ms) *prep_ms = b;
  if (ecmult_ms) *ecmult_ms = c;
  return GV_OK;
}

int gv_stage_stats(gv_ctx* ctx, int dev_slot, int* count, double* unpack_ms, double* prep_ms,
                   double* ecmult_ms) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  double sa = 0, sb = 0, sc = 0;
  const int cnt = d->ring_count;
  for (int k = 0; k < cnt; ++k) {
    hipEvent_t* e = d->ring[(d->ring_next - 1 - k + Dev::kRing) % Dev::kRing];
    CK(hipEventSynchronize(e[2]));
    float a = 0, b = 0, c = 0;
    CK(hipEventElapsedTime(&a, e[3], e[0]));
    CK(hipEventElapsedTime(&b, e[0], e[1]));
    CK(hipEventElapsedTime(&c, e[1], e[2]));
    sa += a; sb += b; sc += c;
  }
  d->ring_count = 0;
  if (count) *count = cnt;
  if (unpack_ms) *unpack_ms = cnt ? sa / cnt : 0.0;
  if (prep_ms) *prep_ms = cnt ? sb / cnt : 0.0;
  if (ecmult_ms) *ecmult_ms = cnt ? sc / cnt : 0.0;
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
  CK(hipMemcpyAsync(dst, src, bytes, k, d->st));
  CK(hipStreamSynchronize(d->st));
  return GV_OK;
}

int gv_dev_sync(gv_ctx* ctx, int dev_slot) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size()) return GV_EINVAL;
  Dev* d = ctx->devs[dev_slot];
  CK(hipSetDevice(d->id));
  CK(hipStreamSynchronize(d->st));
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

int gv_debug_op(gv_ctx* ctx, int dev_slot, int op, size_t n, const uint32_t* in, uint32_t* out) {
  if (!ctx || dev_slot < 0 || dev_slot >= (int)ctx->devs.size() || !in || !out) return GV_EINVAL;
  if (n == 0) return GV_OK;
  Dev* d = ctx->devs[dev_slot];
  std::lock_guard<std::mutex> lk(d->mu);
  CK(hipSetDevice(d->id));
  const size_t npad = round_up(n, 256);
  uint32_t *din = nullptr, *dout = nullptr;
  CK(hipMalloc(&din, npad * 64));
  if (hipMalloc(&dout, npad * 64) != hipSuccess) { (void)hipFree(din); return GV_ENOMEM; }
  int rc = GV_OK;
  if (hipMemsetAsync(din, 0, npad * 64, d->st) != hipSuccess ||
      hipMemcpyAsync(din, in, n * 64, hipMemcpyHostToDevice, d->st) != hipSuccess ||
      gvk_debug(op, (uint32_t)n, din, dout, d->st) != hipSuccess ||
      hipMemcpyAsync(out, dout, n * 64, hipMemcpyDeviceToHost, d->st) != hipSuccess ||
      hipStreamSynchronize(d->st) != hipSuccess)
    rc = GV_EHIP;
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}

}  // extern "C"
