// gv_async.h -- the queue behind gv_submit_* / gv_wait (gv_runtime.cpp):
// tickets, one slice queue and one lane thread per device, a batch's
// completion over its device slices, and the quiesce a key load holds.  No
// HIP in here: the device part of a lane (staging, key grouping, the chunks
// on the device) is a callback, so the CPU harness
// (tests/stage/async_harness.cpp) drives this same queue with fake
// devices, under ThreadSanitizer too.
#pragma once
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "gv_stage.h"

namespace gvasync {

// One submitted batch: the caller's arguments and its device slices' state.
template <class Batch>
struct Job {
  Batch hb;
  int left = 0;                                   // device slices not finished (Lanes::m_)
  int rc = 0;                                     // the first slice error
  bool done = false;
};
// Items [lo, hi) of a job, for one device.
template <class Batch>
struct Slice {
  std::shared_ptr<Job<Batch>> job;
  size_t lo = 0, hi = 0;
};

template <class Batch>
class Lanes {
 public:
  using SliceT = Slice<Batch>;
  // run(k): device k's lane body, called by device k's lane thread whenever
  // its queue holds a slice.  It takes slices with pop(k, ..) -- until that
  // returns false, or fewer if it chooses (it is called again while the
  // queue holds slices) -- and reports each one with finish(); it returns
  // once every slice it popped is finished.
  Lanes(size_t ndev, std::function<void(size_t)> run) : q_(ndev), run_(std::move(run)) {
    for (size_t k = 0; k < ndev; ++k) lanes_.emplace_back([this, k] { lane(k); });
  }
  ~Lanes() { close(); }
  Lanes(const Lanes&) = delete;
  Lanes& operator=(const Lanes&) = delete;

  // The lanes finish every queued slice, then quit (gv_close).  Jobs never
  // waited for are freed with the object.
  void close() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : lanes_)
      if (t.joinable()) t.join();
  }

  // Queue a batch of n items: contiguous 256-aligned slices, one per device
  // (as the synchronous path splits).  Waits while a Quiesce is held.
  // Returns the ticket.
  uint64_t submit(const Batch& hb, size_t n) {
    auto job = std::make_shared<Job<Batch>>();
    job->hb = hb;
    const size_t nd = q_.size();
    const size_t per = gvstage::round_up((n + nd - 1) / (nd ? nd : 1), 256);
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return quiescing_ == 0; });   // a key load / reset in progress
    for (size_t k = 0; k < nd; ++k) {
      const size_t lo = std::min(n, k * per), hi = std::min(n, (k + 1) * per);
      if (lo >= hi) continue;
      q_[k].push_back(SliceT{job, lo, hi});
      ++job->left;
    }
    if (job->left == 0) job->done = true;
    else ++pending_;
    const uint64_t t = next_ticket_++;
    jobs_.emplace(t, job);
    cv_.notify_all();
    return t;
  }

  // Blocks until the ticket's batch is done and returns its result (0 or the
  // first slice error); `unknown` for a ticket never issued or already
  // waited for.  Waiting is also a ticket's release.
  int wait(uint64_t ticket, int unknown) {
    std::unique_lock<std::mutex> lk(m_);
    auto it = jobs_.find(ticket);
    if (it == jobs_.end()) return unknown;
    std::shared_ptr<Job<Batch>> j = it->second;
    jobs_.erase(it);                               // a second wait on it is `unknown`
    cv_.wait(lk, [&] { return j->done; });
    return j->rc;
  }

  // Lane side: the next slice of device k, or false when its queue is empty.
  bool pop(size_t k, SliceT& out) {
    std::lock_guard<std::mutex> lk(m_);
    if (q_[k].empty()) return false;
    out = q_[k].front();
    q_[k].pop_front();
    return true;
  }
  // Lane side: a popped slice is finished (rc: its error, 0 if none).
  void finish(const SliceT& sl, int rc) {
    std::lock_guard<std::mutex> lk(m_);
    end_slice(sl, rc);
    cv_.notify_all();
  }
  // Lane side: every slice still queued for device k fails with rc.
  void fail_queued(size_t k, int rc) {
    std::lock_guard<std::mutex> lk(m_);
    for (SliceT& sl : q_[k]) end_slice(sl, rc);
    q_[k].clear();
    cv_.notify_all();
  }

  // Held by gv_keys_load / gv_keys_reset: the constructor waits until no
  // submitted batch is pending (a keyed batch must never read a slot that
  // moves), and submissions wait until the destructor -- a caller that keeps
  // queueing batches can neither starve the load nor slip one in under it.
  class Quiesce {
   public:
    explicit Quiesce(Lanes* l) : l_(l) {
      if (!l_) return;
      std::unique_lock<std::mutex> lk(l_->m_);
      ++l_->quiescing_;
      l_->cv_.wait(lk, [&] { return l_->pending_ == 0; });
    }
    ~Quiesce() {
      if (!l_) return;
      std::lock_guard<std::mutex> lk(l_->m_);
      --l_->quiescing_;
      l_->cv_.notify_all();
    }
    Quiesce(const Quiesce&) = delete;
    Quiesce& operator=(const Quiesce&) = delete;

   private:
    Lanes* l_;
  };

  size_t pending() {
    std::lock_guard<std::mutex> lk(m_);
    return pending_;
  }
  size_t tickets_held() {
    std::lock_guard<std::mutex> lk(m_);
    return jobs_.size();
  }

 private:
  void end_slice(const SliceT& sl, int rc) {      // m_ held
    if (rc && !sl.job->rc) sl.job->rc = rc;
    if (--sl.job->left == 0) {
      sl.job->done = true;
      --pending_;
    }
  }
  void lane(size_t k) {
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return quit_ || !q_[k].empty(); });
        if (q_[k].empty()) return;                // quit, nothing left
      }
      run_(k);
    }
  }

  std::mutex m_;
  std::condition_variable cv_;                    // lanes: work or quit; waiters: a job done; submitters: quiesce over
  std::vector<std::deque<SliceT>> q_;             // per device
  std::function<void(size_t)> run_;
  std::vector<std::thread> lanes_;
  std::unordered_map<uint64_t, std::shared_ptr<Job<Batch>>> jobs_;
  uint64_t next_ticket_ = 1;
  size_t pending_ = 0;                            // jobs submitted, not done
  int quiescing_ = 0;
  bool quit_ = false;
};

}  // namespace gvasync
