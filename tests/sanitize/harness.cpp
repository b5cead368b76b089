// harness.cpp -- drives the host mirror (host/gvhost.cpp) from several
// threads under ASan + UBSan or TSan (tests/test_sanitizers.py; reference
// test-race target: Makefile:123-124).  Verdicts from the CPU fake
// (fake_gpuverify.cpp over the oracle).  Reads a fixture (written by the
// test with txkit): accounts, blocks, CheckTx txs grouped per thread.
//   1. gvh_deliver_blocks (pipelined: block b+1's pre-verification and its
//      batch on the helper thread while block b's DeliverTx loop runs on the
//      8-thread pool; gpu_hash on: message batches) == gvh_deliver_block_codes
//      block by block (host digests) == gvh_ante
//      tx by tx: same codes, same final accounts;
//   2. gvh_checktx from 8 threads at once (the accumulation window, shared
//      batches; each thread signs for its own accounts) == gvh_ante in the
//      same per-thread order.
// Prints {"blocks": [...], "check": [...]} (codes) and exits 0, or exits 1
// with the first difference; a sanitizer report aborts with its own code.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <thread>
#include <vector>

#include "gvhost.h"

extern "C" gv_ctx* gvfake_open(void);
extern "C" void gvfake_close(gv_ctx*);
extern "C" uint64_t gvfake_calls(gv_ctx*);

struct Reader {
  std::vector<uint8_t> b;
  size_t o = 0;
  uint32_t u32() { uint32_t v; memcpy(&v, &b.at(o), 4); o += 4; return v; }
  uint64_t u64() { uint64_t v; memcpy(&v, &b.at(o), 8); o += 8; return v; }
  std::vector<uint8_t> bytes() {
    const uint32_t n = u32();
    std::vector<uint8_t> v(b.begin() + o, b.begin() + o + n);
    o += n;
    return v;
  }
};

struct Acc { uint8_t addr[20]; uint64_t number, seq; std::vector<uint8_t> pub; };

static std::string chain;
static int64_t height;
static std::vector<Acc> accs;

static gvh_app* fresh(gv_ctx* ctx) {
  gvh_app* app = gvh_app_new(ctx);
  gvh_set_context(app, chain.c_str(), height, 0, 0);
  gvh_set_threads(app, 8);
  for (const Acc& a : accs)
    gvh_set_account(app, a.addr, a.number, a.seq, a.pub.empty() ? nullptr : a.pub.data(), a.pub.size());
  return app;
}

static std::vector<std::vector<uint8_t>> state(gvh_app* app) {
  std::vector<std::vector<uint8_t>> out;
  for (const Acc& a : accs) {
    uint64_t num = 0, seq = 0;
    size_t pl = 0;
    std::vector<uint8_t> pub(512);
    gvh_get_account(app, a.addr, &num, &seq, pub.data(), &pl);
    pub.resize(pl);
    pub.insert(pub.end(), (uint8_t*)&num, (uint8_t*)&num + 8);
    pub.insert(pub.end(), (uint8_t*)&seq, (uint8_t*)&seq + 8);
    out.push_back(pub);
  }
  return out;
}

static int fail(const char* what) {
  fprintf(stderr, "harness: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  if (argc != 2) return fail("usage: harness fixture.bin");
  Reader r;
  {
    FILE* f = fopen(argv[1], "rb");
    if (!f) return fail("cannot open fixture");
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) r.b.insert(r.b.end(), buf, buf + k);
    fclose(f);
  }
  if (r.b.size() < 6 || memcmp(r.b.data(), "GVSAN1", 6)) return fail("bad magic");
  r.o = 6;
  {
    auto c = r.bytes();
    chain.assign(c.begin(), c.end());
  }
  height = (int64_t)r.u64();
  for (uint32_t n = r.u32(); n; --n) {
    Acc a;
    memcpy(a.addr, &r.b.at(r.o), 20);
    r.o += 20;
    a.number = r.u64();
    a.seq = r.u64();
    a.pub = r.bytes();
    accs.push_back(a);
  }
  std::vector<std::vector<std::vector<uint8_t>>> blocks(r.u32());
  for (auto& bl : blocks)
    for (uint32_t n = r.u32(); n; --n) bl.push_back(r.bytes());
  std::vector<std::vector<std::vector<uint8_t>>> check(r.u32());   // per thread
  for (auto& th : check)
    for (uint32_t n = r.u32(); n; --n) th.push_back(r.bytes());

  gv_ctx* ctx = gvfake_open();
  // 1a. pipelined replay
  std::vector<const uint8_t*> ptr;
  std::vector<size_t> len, ntx;
  for (auto& bl : blocks) {
    ntx.push_back(bl.size());
    for (auto& t : bl) { ptr.push_back(t.data()); len.push_back(t.size()); }
  }
  std::vector<uint32_t> piped(ptr.size());
  gvh_app* a1 = fresh(ctx);
  gvh_set_gpu_hash(a1, 1);
  if (gvh_deliver_blocks(a1, blocks.size(), ntx.data(), ptr.data(), len.data(), piped.data()) != GVH_OK)
    return fail("gvh_deliver_blocks");
  // 1b. block by block
  gvh_app* a2 = fresh(ctx);
  std::vector<uint32_t> one;
  size_t o = 0;
  for (auto& bl : blocks) {
    std::vector<uint32_t> c(bl.size());
    if (gvh_deliver_block_codes(a2, bl.size(), ptr.data() + o, len.data() + o, c.data()) != GVH_OK)
      return fail("gvh_deliver_block_codes");
    one.insert(one.end(), c.begin(), c.end());
    o += bl.size();
  }
  // 1c. tx by tx, no pre-verification
  gvh_app* a3 = fresh(ctx);
  std::vector<uint32_t> serial;
  for (size_t i = 0; i < ptr.size(); ++i) {
    gvh_result res;
    if (gvh_ante(a3, ptr[i], len[i], 0, &res) != GVH_OK) return fail("gvh_ante");
    serial.push_back(res.code);
  }
  if (piped != one) return fail("deliver_blocks codes != block by block");
  if (one != serial) return fail("block codes != serial ante");
  if (state(a1) != state(a2) || state(a2) != state(a3)) return fail("final accounts differ");

  // 2. concurrent CheckTx through the window vs serial ante
  gvh_app* a4 = fresh(ctx);
  gvh_set_window(a4, 64, 200);
  std::vector<std::vector<uint32_t>> got(check.size());
  std::vector<std::thread> th;
  std::vector<int> rcs(check.size(), GVH_OK);
  for (size_t t = 0; t < check.size(); ++t)
    th.emplace_back([&, t]() {
      for (auto& tx : check[t]) {
        gvh_result res;
        const int rc = gvh_checktx(a4, tx.data(), tx.size(), &res);
        if (rc != GVH_OK) rcs[t] = rc;
        got[t].push_back(res.code);
      }
    });
  for (auto& x : th) x.join();
  for (int rc : rcs)
    if (rc != GVH_OK) return fail("gvh_checktx");
  gvh_app* a5 = fresh(ctx);
  std::vector<uint32_t> cflat, sflat;
  for (size_t t = 0; t < check.size(); ++t)
    for (size_t i = 0; i < check[t].size(); ++i) {
      gvh_result res;
      if (gvh_ante(a5, check[t][i].data(), check[t][i].size(), 0, &res) != GVH_OK) return fail("gvh_ante (check)");
      sflat.push_back(res.code);
      cflat.push_back(got[t][i]);
    }
  if (cflat != sflat) return fail("concurrent CheckTx codes != serial ante");
  if (state(a4) != state(a5)) return fail("CheckTx final accounts differ");
  gvh_stats st;
  gvh_get_stats(a4, &st);
  // freed together at the end: an app allocated where a freed one lived would
  // reuse its std::mutex words, which TSan (no constructor call to see)
  // reports as a lock of a destroyed mutex
  for (gvh_app* a : {a1, a2, a3, a4, a5}) gvh_app_free(a);
  printf("{\"blocks\": [");
  for (size_t i = 0; i < serial.size(); ++i) printf("%s%u", i ? ", " : "", serial[i]);
  printf("], \"check\": [");
  for (size_t i = 0; i < cflat.size(); ++i) printf("%s%u", i ? ", " : "", cflat[i]);
  printf("], \"windows\": %llu, \"verifier_calls\": %llu}\n", (unsigned long long)st.windows,
         (unsigned long long)gvfake_calls(ctx));
  gvfake_close(ctx);
  return 0;
}
