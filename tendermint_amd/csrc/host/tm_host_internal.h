// Helpers shared by the host layer's C-ABI translation units
// (tm_host_abi.cpp: batch verifier and commit checks; tm_light_abi.cpp:
// light-client verification).  Not part of the public C-ABI.
#pragma once
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <unordered_map>

#include "../../../include/tmhost.h"
#include "pool.h"
#include "tm_types.h"

// Sets the calling thread's tmv_last_error() text (defined by the runtime,
// and by the CPU test double); the host layer moves a worker thread's error
// to the caller's thread with it.
extern "C" void tmv_internal_set_error(const char *msg);

namespace tmh_internal {

// Phase timing of a host-layer call, printed to stderr when the environment
// variable TMV_HOST_TIMING is set (profiling aid).
struct PhaseTimer {
  const char *tag;
  bool on = tmh::host_timing();
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit PhaseTimer(const char *tag_) : tag(tag_) {}
  void mark(const char *what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[%s] %-8s %9.3f ms\n", tag, what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};
// Marks `what` when it goes out of scope: declared right after the timer,
// before a call's containers, it times their destruction.
struct PhaseEnd {
  PhaseTimer &tm;
  const char *what;
  ~PhaseEnd() { tm.mark(what); }
};

void put_err(char *err, size_t cap, const std::string &s);
tmh::KeyType to_kind(uint8_t k);
tmh::Bytes bytes_of(const uint8_t *p, size_t n);
tmh::BlockID block_id_of(const tmv_block_id &b);
std::unique_ptr<tmh::ValidatorSet> vals_of(const tmv_validator *vals, uint32_t n_vals, int32_t proposer_index);
std::unique_ptr<tmh::Commit> commit_of(const tmv_commit *commit);

// Validator sets and commits a caller has already converted (the light
// layer), looked up by the C struct they came from, so verify_commits does
// not convert them again.
struct Converted {
  std::unordered_map<const void *, const tmh::ValidatorSet *> vals;  // key: tmv_commit_job::vals
  std::unordered_map<const void *, const tmh::Commit *> commits;     // key: tmv_commit_job::commit
};

// tmv_verify_commits, plus not_enough[j] = 1 when job j's error is
// types.ErrNotEnoughVotingPowerSigned (may be NULL).
int verify_commits(tmv_ctx *ctx, const tmv_commit_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                   size_t err_stride, uint8_t *not_enough, const Converted *conv = nullptr);

// Run fn(i) for i in [0, n) on the host worker pool (serial when small).
template <class F>
void parallel_for(size_t n, size_t min_per_thread, F fn) {
  tmh::parallel_for_n(n, n / std::max<size_t>(1, min_per_thread), fn);
}

// Jobs per slice of a large tmv_verify_commits / tmv_light_verify_many call
// (TMV_HOST_SLICE; 0 = no slicing).
uint32_t host_slice_jobs();

// Pipelined host layer: jobs [0, n_jobs) cut into slices that two threads
// (the caller and a persistent partner thread) take in turn, each running
// run_slice(lo, hi) -- a whole host-layer pass over those jobs.  The engine
// serialises calls per device, so while one slice's engine call holds the
// GPU the other slice's host phases (convert, hash packing, plan, dedup,
// sign-bytes templates, packing) run: window k + 1 is prepared while window
// k verifies.  Every job's result is its own (sharing only saves work), so
// slicing changes no result.  Returns the sum of the slices' returns, or the
// first negative one.
// Returns the first infrastructure error (< 0) of any slice, else the sum of
// the slices' results.  On an error its slice's message (tmv_last_error on
// the thread that ran it) becomes the caller thread's last error, and
// *fail_lo (if given) is that slice's first job, read after every slice
// has finished.
int run_sliced(uint32_t n_jobs, int (*run_slice)(void *, uint32_t, uint32_t), void *ctx,
               uint32_t *fail_lo = nullptr);

}  // namespace tmh_internal
