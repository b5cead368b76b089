// gv_stage.h -- host-side staging helpers of the runtime (gv_runtime.cpp):
// the per-device staging thread pool, the parallel memcpy of pageable caller
// buffers into pinned staging, the per-device worker thread and the split of
// a host batch into one contiguous slice per device.  No HIP in here, so the
// CPU test harness (tests/stage/stage_harness.cpp) drives the same code with
// fake devices.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <sched.h>
#include <thread>
#include <vector>

namespace gvstage {

inline size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

// Runs fn(part) for part in [0, parts) on the caller plus the pool's
// persistent threads.  One pool PER DEVICE (stage_pool_threads: the staging
// budget split over the devices), so the slices of a host batch stage
// concurrently instead of queueing their copies behind each other's in one
// FIFO.  run() may still be called from several threads at once (concurrent
// callers of one context): each call is a job whose parts any idle thread of
// the pool, or its own caller, claims.
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size() + 1; }
  void run(int parts, const std::function<void(int)>& fn) {
    parts = std::max(1, std::min(parts, size()));
    if (parts == 1) { fn(0); return; }
    auto job = std::make_shared<Job>();
    job->fn = &fn;
    job->parts = parts;
    {
      std::lock_guard<std::mutex> lk(m_);
      jobs_.push_back(job);
    }
    cv_.notify_all();
    for (int p; (p = job->next.fetch_add(1)) < parts;) {   // the caller works too
      fn(p);
      finish(*job);
    }
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [&] { return job->done == parts; });
    drop(job.get());
  }

 private:
  struct Job {
    const std::function<void(int)>* fn = nullptr;
    int parts = 0;
    std::atomic<int> next{0};
    int done = 0;                                  // guarded by m_
  };
  void finish(Job& j) {
    std::lock_guard<std::mutex> lk(m_);
    if (++j.done == j.parts) done_cv_.notify_all();
  }
  void drop(Job* j) {                              // m_ held
    for (size_t i = 0; i < jobs_.size(); ++i)
      if (jobs_[i].get() == j) { jobs_.erase(jobs_.begin() + i); return; }
  }
  void loop() {
    for (;;) {
      std::shared_ptr<Job> job;
      int p = 0;
      {
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
          if (quit_) return;
          while (!jobs_.empty()) {                 // a job with parts left to claim
            p = jobs_.front()->next.fetch_add(1);
            if (p < jobs_.front()->parts) { job = jobs_.front(); break; }
            jobs_.erase(jobs_.begin());            // fully claimed: its caller finishes it
          }
          if (job) break;
          cv_.wait(lk);
        }
      }
      (*job->fn)(p);
      finish(*job);
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::shared_ptr<Job>> jobs_;
  bool quit_ = false;
};

// CPUs this process may run on: the affinity mask, capped by the cgroup v2
// CPU quota when one is set (a GPU box shows 256 CPUs under a 16-CPU quota).
inline int host_cpus() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {0};
    long long period = 0;
    if (fscanf(f, "%31s %lld", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
      const long long q = atoll(quota);
      if (q > 0) n = std::min<long long>(n, std::max<long long>(1, (q + period - 1) / period));
    }
    fclose(f);
  }
  return std::max(1, n);
}

// memcpy split over the pool (large copies only: one core streams ~10 GB/s)
inline void par_copy(Pool* pool, void* dst, const void* src, size_t bytes) {
  constexpr size_t kMin = size_t(1) << 20;
  if (!pool || bytes < kMin) { if (bytes) memcpy(dst, src, bytes); return; }
  const int parts = (int)std::min<size_t>(pool->size(), bytes / (kMin / 2));
  const size_t per = round_up((bytes + parts - 1) / parts, 4096);
  pool->run(parts, [&](int p) {
    const size_t lo = std::min(bytes, p * per), hi = std::min(bytes, lo + per);
    if (hi > lo) memcpy((uint8_t*)dst + lo, (const uint8_t*)src + lo, hi - lo);
  });
}

// Several copies as one pool pass: the total is cut into equal byte ranges,
// one per thread, each range spanning whichever segments it covers.
struct CopySeg {
  uint8_t* dst;
  const uint8_t* src;
  size_t bytes;
};
inline void par_copy_segs(Pool* pool, const CopySeg* seg, int ns) {
  constexpr size_t kMin = size_t(1) << 20;
  size_t total = 0;
  for (int i = 0; i < ns; ++i) total += seg[i].bytes;
  auto copy_range = [&](size_t lo, size_t hi) {       // [lo, hi) of the concatenation
    size_t base = 0;
    for (int i = 0; i < ns && lo < hi; base += seg[i].bytes, ++i) {
      const size_t a = std::max(lo, base), b = std::min(hi, base + seg[i].bytes);
      if (a < b) memcpy(seg[i].dst + (a - base), seg[i].src + (a - base), b - a);
    }
  };
  if (!pool || total < kMin) { copy_range(0, total); return; }
  const int parts = (int)std::min<size_t>(pool->size(), total / (kMin / 2));
  const size_t per = round_up((total + parts - 1) / parts, 4096);
  pool->run(parts, [&](int p) { copy_range(std::min(total, p * per), std::min(total, (p + 1) * per)); });
}

// One persistent thread per extra device: runs the device's slices of host
// batches, in the order they were posted.  Every post gets its own future, so
// concurrent callers of one context (gv_ctx is thread-safe) each wait for
// THEIR slice, never for another caller's.
class Worker {
 public:
  Worker() : th_([this] { loop(); }) {}
  ~Worker() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  std::future<int> post(std::function<int()> job) {
    auto task = std::make_shared<std::packaged_task<int()>>(std::move(job));
    std::future<int> f = task->get_future();
    {
      std::lock_guard<std::mutex> lk(m_);
      q_.push_back([task] { (*task)(); });
    }
    cv_.notify_all();
    return f;
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [this] { return quit_ || !q_.empty(); });
        if (q_.empty()) return;                  // quit with nothing left
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool quit_ = false;
  std::thread th_;
};


// Staging threads per device (the caller included): half the CPUs this
// process may use -- the callers, HIP's own threads and the node keep the
// rest -- split over the devices, at most 8 each and at least 1 (the slice's
// own thread).  One GPU: min(8, cpus / 2); eight GPUs on a 16-CPU quota: 1.
inline int stage_pool_threads(int cpus, int n_dev) {
  return std::max(1, std::min(8, cpus / 2 / std::max(1, n_dev)));
}

// Items [0, n) in one contiguous slice per device, multiples of `align`:
// device 0's on the calling thread, device k's on workers[k] (workers[0]
// unused), all at once.  Returns the first non-zero slice result.
template <class F>
int run_sliced(const std::vector<Worker*>& workers, size_t n, size_t align, F&& slice) {
  const size_t nd = workers.size();
  const size_t per = round_up((n + nd - 1) / nd, align);
  std::vector<int> rcs(nd, 0);
  std::vector<std::future<int>> futs(nd);
  for (size_t k = 1; k < nd; ++k) {
    const size_t lo = std::min(n, k * per), hi = std::min(n, (k + 1) * per);
    if (lo >= hi) continue;
    futs[k] = workers[k]->post([&slice, k, lo, hi]() { return slice(k, lo, hi); });
  }
  rcs[0] = slice(size_t(0), size_t(0), std::min(n, per));
  for (size_t k = 1; k < nd; ++k)
    if (futs[k].valid()) rcs[k] = futs[k].get();
  for (int rc : rcs)
    if (rc) return rc;
  return 0;
}

}  // namespace gvstage
