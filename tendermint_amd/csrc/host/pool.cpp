// Worker pool behind tmh::pool_for (pool.h).
#include "pool.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

namespace tmh {

namespace {

thread_local bool t_in_pool = false;  // a pool worker, or a caller running a pool job

class WorkerPool {
 public:
  explicit WorkerPool(size_t workers) {
    for (size_t w = 0; w < workers; w++) std::thread([this, w] { loop(w); }).detach();
    nworkers_ = workers;
  }

  size_t workers() const { return nworkers_; }

  // false: busy (the caller runs the loop itself)
  bool run(size_t n, size_t helpers, void (*fn)(void *, size_t), void *ctx) {
    std::unique_lock<std::mutex> job_lock(job_mu_, std::try_to_lock);
    if (!job_lock.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = fn;
      ctx_ = ctx;
      n_ = n;
      next_.store(0, std::memory_order_relaxed);
      want_ = helpers;
      pending_ = helpers;
      gen_++;
    }
    cv_.notify_all();
    t_in_pool = true;
    drain();
    t_in_pool = false;
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    return true;
  }

 private:
  void drain() {
    for (size_t i; (i = next_.fetch_add(1, std::memory_order_relaxed)) < n_;) fn_(ctx_, i);
  }

  void loop(size_t w) {
    t_in_pool = true;
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (w >= want_) continue;  // not needed for this job
      }
      drain();
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }

  std::mutex job_mu_;  // one job at a time
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  void (*fn_)(void *, size_t) = nullptr;
  void *ctx_ = nullptr;
  size_t n_ = 0, want_ = 0, pending_ = 0, nworkers_ = 0;
  std::atomic<size_t> next_{0};
  uint64_t gen_ = 0;
};

WorkerPool &pool() {
  static WorkerPool *p = new WorkerPool(pool_threads() - 1);  // never destroyed: workers outlive exit
  return *p;
}

}  // namespace

size_t pool_threads() {
  static const size_t hw = [] {
    const char *e = std::getenv("TMV_HOST_THREADS");
    const long v = e ? std::atol(e) : 0;
    return v > 0 ? (size_t)v : (size_t)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  }();
  return hw;
}

void pool_for(size_t n, size_t max_threads, void (*fn)(void *, size_t), void *ctx) {
  const size_t nt = std::min({max_threads, n, pool_threads()});
  if (nt <= 1 || t_in_pool || !pool().run(n, std::min(nt - 1, pool().workers()), fn, ctx)) {
    for (size_t i = 0; i < n; i++) fn(ctx, i);
  }
}

}  // namespace tmh
