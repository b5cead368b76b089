// front_bench.cpp -- the host mirror's block-path front on the CPU, one
// thread by default, no GPU (a deterministic per-tx cost of
// decode / sequence prediction / plans / pack / DeliverTx loop, accepted
// against a committed figure rather than the shared GPU boxes' +-40 % host
// noise).  host/gvhost.cpp over the CPU fake verifier
// (tests/sanitize/fake_gpuverify.cpp) with GVFAKE_TRUST=1: every verdict true,
// no verification math, so what is timed is PreVerifyTxs' host stages
// (x/auth/types/stdtx.go:248-259 sign bytes, :321-338 amino decode) and the
// DeliverTx ante loop (baseapp/abci.go:203-221).  GVH_PROFILE laps go to
// stderr; tools/front_cost.py writes the fixture and takes the medians.
//
// Fixture "GVFRT1": chain (u32 len + bytes), height (u64), accounts (u32 n;
// addr[20], number u64, sequence u64, pub (u32 len + bytes)), blocks (u32 n;
// each u32 ntx, each tx u32 len + bytes).
// usage: front_bench FIXTURE [threads] [reps]  ->  one JSON line on stdout
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "gvhost.h"

extern "C" gv_ctx* gvfake_open(void);

namespace {
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
struct Acc {
  uint8_t addr[20];
  uint64_t number, seq;
  std::vector<uint8_t> pub;
};
}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: front_bench FIXTURE [threads] [reps]\n"); return 2; }
  const int threads = argc > 2 ? atoi(argv[2]) : 1;
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  Reader r;
  {
    FILE* f = fopen(argv[1], "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", argv[1]); return 2; }
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) r.b.insert(r.b.end(), buf, buf + k);
    fclose(f);
  }
  if (r.b.size() < 6 || memcmp(r.b.data(), "GVFRT1", 6)) { fprintf(stderr, "bad magic\n"); return 2; }
  r.o = 6;
  const std::vector<uint8_t> cb = r.bytes();
  const std::string chain(cb.begin(), cb.end());
  const int64_t height = (int64_t)r.u64();
  std::vector<Acc> accs(r.u32());
  for (Acc& a : accs) {
    memcpy(a.addr, &r.b.at(r.o), 20);
    r.o += 20;
    a.number = r.u64();
    a.seq = r.u64();
    a.pub = r.bytes();
  }
  std::vector<std::vector<std::vector<uint8_t>>> blocks(r.u32());
  for (auto& bl : blocks)
    for (uint32_t n = r.u32(); n; --n) bl.push_back(r.bytes());

  gv_ctx* ctx = gvfake_open();
  size_t bad = 0;
  printf("{\"threads\": %d, \"block_ms\": [", threads);
  for (int rep = 0; rep < reps; ++rep) {
    gvh_app* app = gvh_app_new(ctx);
    gvh_set_context(app, chain.c_str(), height, 0, 0);
    gvh_set_threads(app, threads);
    for (const Acc& a : accs)
      gvh_set_account(app, a.addr, a.number, a.seq, a.pub.empty() ? nullptr : a.pub.data(), a.pub.size());
    printf("%s[", rep ? ", " : "");
    for (size_t b = 0; b < blocks.size(); ++b) {
      std::vector<const uint8_t*> ptr;
      std::vector<size_t> len;
      for (auto& t : blocks[b]) { ptr.push_back(t.data()); len.push_back(t.size()); }
      std::vector<uint32_t> codes(ptr.size());
      fprintf(stderr, "block %zu\n", b);
      const auto t0 = std::chrono::steady_clock::now();
      if (gvh_deliver_block_codes(app, ptr.size(), ptr.data(), len.data(), codes.data()) != GVH_OK) {
        fprintf(stderr, "gvh_deliver_block_codes failed\n");
        return 1;
      }
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      for (uint32_t c : codes) bad += c != 0;
      printf("%s%.3f", b ? ", " : "", ms);
    }
    printf("]");
    gvh_app_free(app);
  }
  printf("], \"ntx\": [");
  for (size_t b = 0; b < blocks.size(); ++b) printf("%s%zu", b ? ", " : "", blocks[b].size());
  printf("], \"nonzero_codes\": %zu}\n", bad);
  return bad ? 1 : 0;
}
