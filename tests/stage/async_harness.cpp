// CPU harness of the asynchronous host-batch queue (csrc/gv_async.h: the
// queue, tickets and quiesce behind gv_submit_* / gv_wait) with fake devices
// (the node submits through this path; on hardware it only ever
// ran on one GPU).  Each fake device's lane stages its slice's input through
// its own gvstage::Pool (par_copy_segs, as the runtime's staging does),
// "computes" (a sleep standing in for H2D + kernels) and writes one verdict
// byte per item, f(item's input bytes), into the caller's output.
//
//   1. every device's slice of the first batch must be in flight at once (a
//      barrier across the lanes, 5 s at most);
//   2. several submitter threads queue batches of ragged sizes (0, under one
//      256-item slice, past every device) and wait their tickets out of order;
//      every verdict byte must be f(input), every ticket waited once (a second
//      wait and a never-issued ticket answer "unknown");
//   3. a key-load thread holds Quiesce repeatedly while they submit: inside
//      it no batch is pending and no lane runs a slice;
//   4. a device that fails (fail_queued, as a failed hipSetDevice) fails its
//      batches' tickets and only theirs.
// Prints one JSON line; exit 0 when every check held.  Built plain and with
// ThreadSanitizer (tests/test_stage_devices.py).
//
// usage: async_harness ND SUBMITTERS BATCHES_PER_SUBMITTER COMPUTE_US
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../cosmos-sdk-rootchain_amd/csrc/gv_async.h"

using namespace gvstage;
using clk = std::chrono::steady_clock;

namespace {
constexpr int kUnknown = -1, kDevErr = -3;

struct Batch {                                   // a host batch: n items of 97 bytes (sig64 | dig32 | 1)
  const uint8_t* in = nullptr;
  uint8_t* out = nullptr;
  uint32_t tag = 0;                              // which submitter / batch (fail checks)
};
uint8_t verdict(const uint8_t* item) {           // the fake "verification"
  uint32_t h = 2166136261u;
  for (int i = 0; i < 97; ++i) h = (h ^ item[i]) * 16777619u;
  return (uint8_t)(h & 1u);
}

struct FakeDev {
  Pool* pool = nullptr;
  std::vector<uint8_t> pinned;
};
}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  const int nd = atoi(argv[1]), nsub = atoi(argv[2]), per_sub = atoi(argv[3]), compute_us = atoi(argv[4]);
  std::vector<FakeDev> devs(nd);
  for (FakeDev& d : devs) d.pool = new Pool(1);

  std::atomic<int> first_arrived{0}, active{0}, quiesce_violations{0}, bad_bytes{0};
  std::atomic<bool> concurrent{true};
  std::atomic<int> fail_dev{-1};                  // device whose lane fails its queue (check 4)
  gvasync::Lanes<Batch>* lanes = nullptr;
  lanes = new gvasync::Lanes<Batch>((size_t)nd, [&](size_t k) {
    FakeDev& d = devs[k];
    if (fail_dev.load() == (int)k) {              // a failed hipSetDevice: the whole queue fails
      lanes->fail_queued(k, kDevErr);
      return;
    }
    gvasync::Slice<Batch> sl;
    while (lanes->pop(k, sl)) {
      active.fetch_add(1);
      if (sl.job->hb.tag == 0xFFFFFFFFu) {        // check 1: the first batch's slices meet here
        first_arrived.fetch_add(1);
        for (const auto until = clk::now() + std::chrono::seconds(5); first_arrived.load() < nd;) {
          if (clk::now() > until) {
            concurrent = false;
            break;
          }
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
      }
      const Batch& b = sl.job->hb;
      const size_t chunk = 4096;
      for (size_t c0 = sl.lo; c0 < sl.hi; c0 += chunk) {
        const size_t cn = std::min(chunk, sl.hi - c0);
        d.pinned.resize(cn * 97);
        const CopySeg seg{d.pinned.data(), b.in + c0 * 97, cn * 97};
        par_copy_segs(d.pool, &seg, 1);
        std::this_thread::sleep_for(std::chrono::microseconds(compute_us));
        for (size_t i = 0; i < cn; ++i) b.out[c0 + i] = verdict(d.pinned.data() + i * 97);
      }
      active.fetch_sub(1);
      lanes->finish(sl, 0);
    }
  });

  // 1. the first batch: one slice per device, all in flight at once
  const size_t n0 = (size_t)nd * 256 * 3;
  std::vector<uint8_t> in0(n0 * 97), out0(n0, 0xEE);
  for (size_t i = 0; i < in0.size(); ++i) in0[i] = (uint8_t)(i * 131 + 7);
  const uint64_t t0 = lanes->submit(Batch{in0.data(), out0.data(), 0xFFFFFFFFu}, n0);
  int rc0 = lanes->wait(t0, kUnknown);
  for (size_t i = 0; i < n0; ++i) bad_bytes += out0[i] != verdict(&in0[i * 97]);
  const int rewait = lanes->wait(t0, kUnknown), never = lanes->wait(987654321ull, kUnknown);

  // 2 + 3. submitters with ragged batches, waits out of order; a quiescing key loader
  std::atomic<bool> stop_loader{false};
  std::atomic<int> quiesces{0}, waited{0}, wrong_rc{0};
  std::thread loader([&] {
    while (!stop_loader.load()) {
      {
        typename gvasync::Lanes<Batch>::Quiesce q(lanes);
        if (lanes->pending() != 0 || active.load() != 0) quiesce_violations++;
        std::this_thread::sleep_for(std::chrono::microseconds(300));
        if (lanes->pending() != 0 || active.load() != 0) quiesce_violations++;
      }
      quiesces++;
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
  });
  std::vector<std::thread> subs;
  for (int s = 0; s < nsub; ++s)
    subs.emplace_back([&, s] {
      std::mt19937_64 rng(0x5EED + s);
      const size_t sizes[] = {0, 1, 255, 256, 257, 1000, (size_t)nd * 256, (size_t)nd * 256 + 1, 20000, 70001};
      std::vector<std::vector<uint8_t>> ins(per_sub), outs(per_sub);
      std::vector<uint64_t> tick(per_sub);
      for (int j = 0; j < per_sub; ++j) {
        const size_t n = sizes[rng() % (sizeof sizes / sizeof sizes[0])];
        ins[j].resize(n * 97 + 1);
        for (auto& v : ins[j]) v = (uint8_t)rng();
        outs[j].assign(n, 0xEE);
        tick[j] = lanes->submit(Batch{ins[j].data(), outs[j].data(), (uint32_t)(s * 1000 + j)}, n);
      }
      std::vector<int> order(per_sub);
      for (int j = 0; j < per_sub; ++j) order[j] = j;
      std::shuffle(order.begin(), order.end(), rng);
      for (int j : order) {
        if (lanes->wait(tick[j], kUnknown) != 0) wrong_rc++;
        waited++;
        for (size_t i = 0; i < outs[j].size(); ++i) bad_bytes += outs[j][i] != verdict(&ins[j][i * 97]);
      }
    });
  for (auto& t : subs) t.join();
  stop_loader = true;
  loader.join();

  // 4. a failing device: the batch spanning it fails, a batch on the others alone does not
  fail_dev = nd - 1;
  const size_t n4 = (size_t)nd * 256 * 2;
  std::vector<uint8_t> in4(n4 * 97, 1), out4(n4);
  const int rc_span = lanes->wait(lanes->submit(Batch{in4.data(), out4.data(), 7}, n4), kUnknown);
  const int rc_small = lanes->wait(lanes->submit(Batch{in4.data(), out4.data(), 8}, 100), kUnknown);   // device 0 only
  fail_dev = -1;
  const size_t held = lanes->tickets_held();
  lanes->close();
  delete lanes;
  for (FakeDev& d : devs) delete d.pool;

  const bool ok = rc0 == 0 && rewait == kUnknown && never == kUnknown && concurrent.load() && bad_bytes.load() == 0 &&
                  wrong_rc.load() == 0 && quiesce_violations.load() == 0 && waited.load() == nsub * per_sub &&
                  rc_span == kDevErr && rc_small == 0 && held == 0;
  printf("{\"ok\": %s, \"concurrent\": %s, \"first_rc\": %d, \"rewait\": %d, \"never\": %d, \"bad_bytes\": %d, "
         "\"waited\": %d, \"wrong_rc\": %d, \"quiesces\": %d, \"quiesce_violations\": %d, \"failed_device_rc\": %d, "
         "\"other_devices_rc\": %d, \"tickets_left\": %zu}\n",
         ok ? "true" : "false", concurrent.load() ? "true" : "false", rc0, rewait, never, bad_bytes.load(),
         waited.load(), wrong_rc.load(), quiesces.load(), quiesce_violations.load(), rc_span, rc_small, held);
  return ok ? 0 : 1;
}
