// CPU harness for the runtime's host staging (csrc/gv_stage.h) with fake
// devices: a host batch is split by run_sliced over nd devices, each slice
// stages its chunks (pageable source -> per-device "pinned" buffer) through
// its device's own Pool with par_copy_segs and then "computes" (a sleep
// standing in for H2D + kernels).  Prints one JSON line: per device the
// staging intervals and the threads that ran its pool parts, the whole
// call's wall time and whether every staged byte matches the source.
//
// usage: stage_harness ND ITEMS CHUNK THREADS_PER_DEV COMPUTE_US_PER_CHUNK
//        stage_harness --threads CPUS ND   (gvstage::stage_pool_threads)
#include <chrono>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../cosmos-sdk-rootchain_amd/csrc/gv_stage.h"

using namespace gvstage;
using clk = std::chrono::steady_clock;

struct FakeDev {
  Pool* pool = nullptr;
  Worker* worker = nullptr;
  std::vector<uint8_t> pinned;                 // the staging buffer of one chunk (sig | dig | keys)
  std::vector<std::pair<double, double>> stage;  // [start, end) ms of each chunk's staging
  std::set<std::thread::id> threads;           // threads that ran this device's pool parts
  std::mutex m;
  bool ok = true;
  double enter = 0;                            // ms at which the slice started
};

int main(int argc, char** argv) {
  if (argc == 4 && !strcmp(argv[1], "--threads")) {     // the per-device staging budget
    printf("%d\n", stage_pool_threads(atoi(argv[2]), atoi(argv[3])));
    return 0;
  }
  if (argc < 6) return 2;
  const int nd = atoi(argv[1]);
  const size_t n = strtoull(argv[2], nullptr, 10), chunk = strtoull(argv[3], nullptr, 10);
  const int tpd = atoi(argv[4]);
  const int compute_us = atoi(argv[5]);
  // a C2-shaped pageable batch: 33-byte keys, 64-byte signatures, 32-byte digests
  std::vector<uint8_t> pub(n * 33), sig(n * 64), dig(n * 32);
  for (size_t i = 0; i < pub.size(); ++i) pub[i] = (uint8_t)(i * 131 + 7);
  for (size_t i = 0; i < sig.size(); ++i) sig[i] = (uint8_t)(i * 17 + 3);
  for (size_t i = 0; i < dig.size(); ++i) dig[i] = (uint8_t)(i * 29 + 11);
  std::vector<FakeDev> devs(nd);
  std::vector<Worker*> ws(nd, nullptr);
  for (int k = 0; k < nd; ++k) {
    devs[k].pool = new Pool(tpd - 1);
    if (k > 0) devs[k].worker = ws[k] = new Worker();
    devs[k].pinned.resize(chunk * (33 + 64 + 32));
  }
  // every slice waits here until all nd are in flight (5 s at most): run_sliced
  // must run them at once, or the barrier times out and "concurrent" is false
  std::atomic<int> arrived{0};
  std::atomic<bool> concurrent{true};
  const auto t0 = clk::now();
  auto ms = [&](clk::time_point t) { return std::chrono::duration<double, std::milli>(t - t0).count(); };
  const int rc = run_sliced(ws, n, 256, [&](size_t k, size_t lo, size_t hi) {
    FakeDev& d = devs[k];
    d.enter = ms(clk::now());
    arrived.fetch_add(1);
    for (const auto until = clk::now() + std::chrono::seconds(5); arrived.load() < nd;) {
      if (clk::now() > until) {
        concurrent = false;
        break;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    for (size_t c0 = lo; c0 < hi; c0 += chunk) {
      const size_t cn = std::min(chunk, hi - c0);
      uint8_t* h = d.pinned.data();
      const CopySeg segs[3] = {CopySeg{h, sig.data() + c0 * 64, cn * 64},
                               CopySeg{h + cn * 64, dig.data() + c0 * 32, cn * 32},
                               CopySeg{h + cn * 96, pub.data() + c0 * 33, cn * 33}};
      const auto a = clk::now();
      par_copy_segs(d.pool, segs, 3);
      const auto b = clk::now();
      d.stage.emplace_back(ms(a), ms(b));
      d.ok = d.ok && !memcmp(h, sig.data() + c0 * 64, cn * 64) && !memcmp(h + cn * 64, dig.data() + c0 * 32, cn * 32) &&
             !memcmp(h + cn * 96, pub.data() + c0 * 33, cn * 33);
      // which threads this device's pool puts on a job (the same Pool::run the copies use)
      d.pool->run(d.pool->size(), [&](int) {
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        std::lock_guard<std::mutex> lk(d.m);
        d.threads.insert(std::this_thread::get_id());
      });
      std::this_thread::sleep_for(std::chrono::microseconds(compute_us));   // H2D + kernels stand-in
    }
    return 0;
  });
  const double wall = ms(clk::now());
  // thread ids -> small integers, shared across devices so overlaps show
  std::map<std::thread::id, int> tid;
  for (auto& d : devs)
    for (auto t : d.threads) tid.emplace(t, (int)tid.size());
  printf("{\"concurrent\": %s, \"rc\": %d, \"nd\": %d, \"items\": %zu, \"chunk\": %zu, \"threads_per_dev\": %d, \"wall_ms\": %.3f, \"devs\": [",
         concurrent.load() ? "true" : "false", rc, nd, n, chunk, tpd, wall);
  for (int k = 0; k < nd; ++k) {
    FakeDev& d = devs[k];
    printf("%s{\"ok\": %s, \"enter\": %.3f, \"stage\": [", k ? ", " : "", d.ok ? "true" : "false", d.enter);
    for (size_t i = 0; i < d.stage.size(); ++i) printf("%s[%.3f, %.3f]", i ? ", " : "", d.stage[i].first, d.stage[i].second);
    printf("], \"threads\": [");
    int j = 0;
    for (auto t : d.threads) printf("%s%d", j++ ? ", " : "", tid[t]);
    printf("]}");
  }
  printf("]}\n");
  for (auto& d : devs) {
    delete d.worker;
    delete d.pool;
  }
  return rc;
}
