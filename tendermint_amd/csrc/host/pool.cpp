// Worker pool behind tmh::pool_for (pool.h).
#include "pool.h"
#include "../knobs.h"

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

// Jobs run side by side: every caller drains its own job and idle workers
// join whichever posted job still has indices left (up to its helper
// count), so two host-layer calls on different threads -- one planning a
// window while the other waits on the GPU -- both get workers.
class WorkerPool {
 public:
  explicit WorkerPool(size_t workers) {
    for (size_t w = 0; w < workers; w++) std::thread([this] { loop(); }).detach();
    nworkers_ = workers;
  }

  size_t workers() const { return nworkers_; }

  void run(size_t n, size_t helpers, void (*fn)(void *, size_t), void *ctx) {
    Job job;
    job.fn = fn;
    job.ctx = ctx;
    job.n = n;
    job.want = helpers;
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.push_back(&job);
    }
    cv_.notify_all();
    t_in_pool = true;
    drain(job);
    t_in_pool = false;
    std::unique_lock<std::mutex> lk(mu_);
    // no helper can join once the job is off the list; wait for those in it
    jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &job));
    done_cv_.wait(lk, [&] { return job.helpers == 0; });
  }

 private:
  struct Job {
    void (*fn)(void *, size_t) = nullptr;
    void *ctx = nullptr;
    size_t n = 0, want = 0, helpers = 0;  // helpers: workers inside drain (under mu_)
    std::atomic<size_t> next{0};
  };

  static void drain(Job &j) {
    for (size_t i; (i = j.next.fetch_add(1, std::memory_order_relaxed)) < j.n;) j.fn(j.ctx, i);
  }

  Job *pick() {  // under mu_
    for (Job *j : jobs_)
      if (j->helpers < j->want && j->next.load(std::memory_order_relaxed) < j->n) return j;
    return nullptr;
  }

  void loop() {
    t_in_pool = true;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      Job *j;
      cv_.wait(lk, [&] { return (j = pick()) != nullptr; });
      j->helpers++;
      lk.unlock();
      drain(*j);
      lk.lock();
      if (--j->helpers == 0) done_cv_.notify_all();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<Job *> jobs_;
  size_t nworkers_ = 0;
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
  if (nt <= 1 || t_in_pool) {
    for (size_t i = 0; i < n; i++) fn(ctx, i);
    return;
  }
  pool().run(n, std::min(nt - 1, pool().workers()), fn, ctx);
}


namespace {
constexpr size_t kReapBacklog = 3;

class Reaper {
 public:
  Reaper() { std::thread([this] { loop(); }).detach(); }
  bool post(std::unique_ptr<Garbage> &g) {
    std::lock_guard<std::mutex> lk(mu_);
    if (q_.size() >= kReapBacklog) return false;
    q_.push_back(std::move(g));
    cv_.notify_one();
    return true;
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return !q_.empty(); });
      std::unique_ptr<Garbage> g = std::move(q_.front());
      q_.erase(q_.begin());
      lk.unlock();
      g.reset();
      lk.lock();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::unique_ptr<Garbage>> q_;
};
}  // namespace

bool host_timing() {
  static const bool on = std::getenv("TMV_HOST_TIMING") != nullptr;
  return on;
}

bool reap(std::unique_ptr<Garbage> &g) {
  static const bool on = [] {  // A/B (knobs.h): TMV_DEFERRED_RELEASE=0 frees inline
    const char *e = tmv::ab_knob("TMV_DEFERRED_RELEASE");
    return !(e && e[0] == '0');
  }();
  if (!on) return false;
  // never destroyed: its detached thread waits on the condition variable
  static Reaper *r = new Reaper;
  return r->post(g);
}

}  // namespace tmh
