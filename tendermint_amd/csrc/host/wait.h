// Bounded waits for device work (SURVEY §5 failure handling): a hung or
// faulted kernel must not block a caller forever.  The runtime polls
// hipStreamQuery / hipEventQuery through poll_until against a deadline
// (TMV_DEVICE_TIMEOUT_MS, default 60 s, 0 = unbounded) and reports
// TMV_ERR_TIMEOUT; the caller (the Go shim) then re-verifies
// on the CPU.  Header-only and device-free so the CPU suite tests it.
#pragma once
#include <chrono>
#include <cstdint>
#include <thread>

namespace tmh {

enum class Poll { kReady = 0, kError = 1, kTimeout = 2 };

// query() returns 0 when done, 1 while pending, anything else on error.
// Spins (yielding) for the first 5 ms so short and medium launches keep
// their latency -- a sleep rounds up to the timer slack (~50 us), which a
// 200 us spin phase put on every ~0.2 ms VerifyCommit (C1 p50 0.24 ->
// 0.30 ms) -- then sleeps 20 us between polls.
template <class Q>
Poll poll_until(Q query, int64_t timeout_ms) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (;;) {
    const int q = query();
    if (q == 0) return Poll::kReady;
    if (q != 1) return Poll::kError;
    const auto el = clk::now() - t0;
    if (timeout_ms > 0 && el > std::chrono::milliseconds(timeout_ms)) return Poll::kTimeout;
    if (el < std::chrono::milliseconds(5)) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

}  // namespace tmh
