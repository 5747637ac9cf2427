// A process-wide pool of host worker threads for the engine's parallel
// loops (packing, planning, key lookups, staging copies).  Spawning and
// joining 15 threads costs ~0.2-0.5 ms, several times per commit window;
// the pool's workers sleep on a condition variable between jobs instead.
// Jobs of different caller threads run side by side (idle workers join any
// job with work left); a loop nested in a pool job runs on its thread.
#pragma once
#include <cstddef>
#include <memory>
#include <tuple>
#include <type_traits>
#include <utility>

namespace tmh {

// Calls fn(ctx, i) for every i in [0, n) on up to max_threads threads
// (the caller included).  Returns when all calls have finished.
void pool_for(size_t n, size_t max_threads, void (*fn)(void *, size_t), void *ctx);

// Threads the pool may use: min(16, hardware threads), or TMV_HOST_THREADS.
size_t pool_threads();
// TMV_HOST_TIMING set: the engine and the host layer print phase timings to
// stderr (profiling aid; read once).
bool host_timing();

// Deferred release: a call's converted objects (validator sets, commits,
// plans: ~10^4 small heap objects per commit window, 0.3-1.2 ms to free) are
// handed to one background thread instead of being freed before the call
// returns.  At most kReapBacklog bundles wait; past that the caller frees its
// own, so memory stays bounded when calls outpace the reaper.
// TMV_DEFERRED_RELEASE=0 frees on the caller (A/B).
struct Garbage {
  virtual ~Garbage() = default;
};
template <class... T>
struct GarbageOf final : Garbage {
  std::tuple<T...> items;
  explicit GarbageOf(T &&...t) : items(std::move(t)...) {}
};
// Takes ownership; returns false (and frees nothing) when the caller must
// free the bundle itself (reaper off or backlogged).
bool reap(std::unique_ptr<Garbage> &g);
template <class... T>
void release_later(T &&...t) {
  std::unique_ptr<Garbage> g(new GarbageOf<std::remove_reference_t<T>...>(std::move(t)...));
  reap(g);  // if it declined, g (the bundle) is destroyed here, on the caller
}

template <class F>
void parallel_for_n(size_t n, size_t max_threads, F &&fn) {
  using Fn = std::remove_reference_t<F>;
  pool_for(n, max_threads, [](void *c, size_t i) { (*static_cast<Fn *>(c))(i); }, const_cast<void *>(static_cast<const void *>(&fn)));
}

}  // namespace tmh
