// fake_gpuverify.cpp -- test infrastructure for the sanitizer builds of the
// host mirror (tests/test_sanitizers.py): the subset of include/gpuverify.h
// that host/gvhost.cpp calls, answered on the CPU.  secp256k1 verdicts come
// from the oracle (oracle/secp256k1_oracle.c, compiled into the harness);
// ed25519 from OpenSSL.  Keys "loaded" into the arenas are kept as bytes.
// This is NOT the product library (which has no CPU path and fails with
// GV_ENODEV without a GPU); it lets ASan / UBSan / TSan watch the host
// mirror's own threads -- the DeliverTx pool, the replay helper thread, the
// CheckTx window -- and the pinned-buffer / key-slot bookkeeping they share.
#include <openssl/evp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <future>
#include <map>
#include <mutex>
#include <vector>

#include "gpuverify.h"

extern "C" int oracle_verify_digest(const uint8_t pub[33], const uint8_t sig[64], const uint8_t digest[32]);

struct gv_ctx {
  bool trust = getenv("GVFAKE_TRUST") != nullptr;   // host-front timing builds: every verdict true, no math
  std::mutex mu;
  std::vector<uint8_t> keys;      // 33 B per slot
  std::vector<uint8_t> ed_keys;   // 32 B per slot
  std::atomic<uint64_t> gen{0}, ed_gen{0};
  std::atomic<uint64_t> calls{0};
  std::mutex qmu;                 // the asynchronous entry points: ticket -> the batch's result
  std::map<uint64_t, std::future<int>> queued;
  uint64_t next_ticket = 1;
};

// gv_keys_load / gv_keys_reset wait for every queued batch first (the
// library's contract: a queued keyed batch never sees a slot move)
static void quiesce(gv_ctx* ctx) {
  std::lock_guard<std::mutex> g(ctx->qmu);
  for (auto& q : ctx->queued) q.second.wait();
}

extern "C" {

gv_ctx* gvfake_open(void) { return new gv_ctx(); }
void gvfake_close(gv_ctx* c) { delete c; }
uint64_t gvfake_calls(gv_ctx* c) { return c->calls.load(); }

int gv_verify_digests(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32,
                      uint8_t* out_ok) {
  if (!ctx || (n && (!pub33 || !sig64 || !dig32 || !out_ok))) return GV_EINVAL;
  ctx->calls++;
  if (ctx->trust) { memset(out_ok, 1, n); return GV_OK; }
  for (size_t i = 0; i < n; ++i) out_ok[i] = (uint8_t)oracle_verify_digest(pub33 + 33 * i, sig64 + 64 * i, dig32 + 32 * i);
  return GV_OK;
}

int gv_keys_load(gv_ctx* ctx, size_t n, const uint8_t* pub33, uint32_t* slot_out) {
  if (!ctx || (n && (!pub33 || !slot_out))) return GV_EINVAL;
  quiesce(ctx);
  std::lock_guard<std::mutex> g(ctx->mu);
  const size_t base = ctx->keys.size() / 33;
  ctx->keys.insert(ctx->keys.end(), pub33, pub33 + 33 * n);
  for (size_t i = 0; i < n; ++i) slot_out[i] = (uint32_t)(base + i);
  return GV_OK;
}
int gv_keys_reset(gv_ctx* ctx) {
  quiesce(ctx);
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->keys.clear();
  ctx->gen++;
  return GV_OK;
}
size_t gv_keys_count(const gv_ctx* ctx) {
  std::lock_guard<std::mutex> g(const_cast<gv_ctx*>(ctx)->mu);
  return ctx->keys.size() / 33;
}
uint64_t gv_keys_generation(const gv_ctx* ctx) { return ctx->gen.load(); }

int gv_verify_digests_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64, const uint8_t* dig32,
                            uint8_t* out_ok) {
  if (!ctx || (n && (!slot || !sig64 || !dig32 || !out_ok))) return GV_EINVAL;
  ctx->calls++;
  if (ctx->trust) { memset(out_ok, 1, n); return GV_OK; }
  std::lock_guard<std::mutex> g(ctx->mu);
  const size_t cnt = ctx->keys.size() / 33;
  for (size_t i = 0; i < n; ++i)
    out_ok[i] = slot[i] < cnt ? (uint8_t)oracle_verify_digest(&ctx->keys[33 * (size_t)slot[i]], sig64 + 64 * i,
                                                              dig32 + 32 * i)
                              : 0;
  return GV_OK;
}

// the message entry points: SHA-256 of each message here, then the digest path
static std::vector<uint8_t> hash_msgs(size_t n, const uint8_t* blob, const uint64_t* off, const uint32_t* len) {
  std::vector<uint8_t> d(32 * n);
  for (size_t i = 0; i < n; ++i) {
    unsigned int dl = 32;
    EVP_Digest(len[i] ? blob + off[i] : (const uint8_t*)"", len[i], &d[32 * i], &dl, EVP_sha256(), nullptr);
  }
  return d;
}
int gv_verify_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* msg_blob,
                   const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* out_ok) {
  if (!ctx || (n && (!msg_off || !msg_len))) return GV_EINVAL;
  const std::vector<uint8_t> d = hash_msgs(n, msg_blob, msg_off, msg_len);
  return gv_verify_digests(ctx, n, pub33, sig64, d.data(), out_ok);
}
int gv_verify_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64, const uint8_t* msg_blob,
                         const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* out_ok) {
  if (!ctx || (n && (!msg_off || !msg_len))) return GV_EINVAL;
  const std::vector<uint8_t> d = hash_msgs(n, msg_blob, msg_off, msg_len);
  return gv_verify_digests_keyed(ctx, n, slot, sig64, d.data(), out_ok);
}

}  // extern "C"
// asynchronous batches: each runs on a thread of its own, gv_wait joins it
template <class F>
static int submit(gv_ctx* ctx, uint64_t* ticket, F f) {
  if (!ctx || !ticket) return GV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->qmu);
  *ticket = ctx->next_ticket++;
  ctx->queued.emplace(*ticket, std::async(std::launch::async, f));
  return GV_OK;
}
extern "C" {
int gv_submit_digests(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32,
                      uint8_t* out_ok, uint64_t* ticket) {
  return submit(ctx, ticket, [=] { return gv_verify_digests(ctx, n, pub33, sig64, dig32, out_ok); });
}
int gv_submit_digests_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64, const uint8_t* dig32,
                            uint8_t* out_ok, uint64_t* ticket) {
  return submit(ctx, ticket, [=] { return gv_verify_digests_keyed(ctx, n, slot, sig64, dig32, out_ok); });
}
int gv_submit_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* msg_blob,
                   const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* out_ok, uint64_t* ticket) {
  return submit(ctx, ticket, [=] { return gv_verify_msgs(ctx, n, pub33, sig64, msg_blob, msg_off, msg_len, out_ok); });
}
int gv_submit_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64, const uint8_t* msg_blob,
                         const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* out_ok, uint64_t* ticket) {
  return submit(ctx, ticket,
                [=] { return gv_verify_msgs_keyed(ctx, n, slot, sig64, msg_blob, msg_off, msg_len, out_ok); });
}
int gv_wait(gv_ctx* ctx, uint64_t ticket) {
  if (!ctx) return GV_EINVAL;
  std::future<int> f;
  {
    std::lock_guard<std::mutex> g(ctx->qmu);
    auto it = ctx->queued.find(ticket);
    if (it == ctx->queued.end()) return GV_EINVAL;
    f = std::move(it->second);
    ctx->queued.erase(it);
  }
  return f.get();
}

static uint8_t ed_verify(const uint8_t* pub32, const uint8_t* sig64, const uint8_t* msg, size_t len) {
  EVP_PKEY* k = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, nullptr, pub32, 32);
  if (!k) return 0;
  EVP_MD_CTX* m = EVP_MD_CTX_new();
  uint8_t ok = 0;
  if (m && EVP_DigestVerifyInit(m, nullptr, nullptr, nullptr, k) == 1)
    ok = EVP_DigestVerify(m, sig64, 64, msg ? msg : (const uint8_t*)"", len) == 1;
  EVP_MD_CTX_free(m);
  EVP_PKEY_free(k);
  return ok;
}

int gv_verify_ed25519_msgs(gv_ctx* ctx, size_t n, const uint8_t* pub32, const uint8_t* sig64,
                           const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                           uint8_t* out_ok) {
  if (!ctx || (n && (!pub32 || !sig64 || !msg_off || !msg_len || !out_ok))) return GV_EINVAL;
  ctx->calls++;
  if (ctx->trust) { memset(out_ok, 1, n); return GV_OK; }
  for (size_t i = 0; i < n; ++i)
    out_ok[i] = ed_verify(pub32 + 32 * i, sig64 + 64 * i, msg_len[i] ? msg_blob + msg_off[i] : nullptr, msg_len[i]);
  return GV_OK;
}

int gv_ed_keys_load(gv_ctx* ctx, size_t n, const uint8_t* pub32, uint32_t* slot_out) {
  if (!ctx || (n && (!pub32 || !slot_out))) return GV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  const size_t base = ctx->ed_keys.size() / 32;
  ctx->ed_keys.insert(ctx->ed_keys.end(), pub32, pub32 + 32 * n);
  for (size_t i = 0; i < n; ++i) slot_out[i] = (uint32_t)(base + i);
  return GV_OK;
}
int gv_ed_keys_reset(gv_ctx* ctx) {
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->ed_keys.clear();
  ctx->ed_gen++;
  return GV_OK;
}
size_t gv_ed_keys_count(const gv_ctx* ctx) {
  std::lock_guard<std::mutex> g(const_cast<gv_ctx*>(ctx)->mu);
  return ctx->ed_keys.size() / 32;
}
uint64_t gv_ed_keys_generation(const gv_ctx* ctx) { return ctx->ed_gen.load(); }

int gv_verify_ed25519_msgs_keyed(gv_ctx* ctx, size_t n, const uint32_t* slot, const uint8_t* sig64,
                                 const uint8_t* msg_blob, const uint64_t* msg_off, const uint32_t* msg_len,
                                 uint8_t* out_ok) {
  if (!ctx || (n && (!slot || !sig64 || !msg_off || !msg_len || !out_ok))) return GV_EINVAL;
  ctx->calls++;
  if (ctx->trust) { memset(out_ok, 1, n); return GV_OK; }
  std::vector<uint8_t> keys;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    keys = ctx->ed_keys;
  }
  const size_t cnt = keys.size() / 32;
  for (size_t i = 0; i < n; ++i)
    out_ok[i] = slot[i] < cnt ? ed_verify(&keys[32 * (size_t)slot[i]], sig64 + 64 * i,
                                          msg_len[i] ? msg_blob + msg_off[i] : nullptr, msg_len[i])
                              : 0;
  return GV_OK;
}

int gv_host_alloc(gv_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out) return GV_EINVAL;
  *out = malloc(bytes ? bytes : 1);
  return *out ? GV_OK : GV_ENOMEM;
}
int gv_host_free(gv_ctx* ctx, void* p) {
  (void)ctx;
  free(p);
  return GV_OK;
}

}  // extern "C"
