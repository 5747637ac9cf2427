// Part boundaries and caller-page locking of a streamed host-buffer chunk
// (tmverify_runtime.cpp, stage_and_launch / batch_check /
// mixed_check_streamed).  Pure host arithmetic, unit-tested on the CPU
// (tests/test_stream_plan.py through tests/native/commit_check.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace tmh {

// Part boundaries of a streamed batch-equation launch of n entries in groups
// of m: whole groups, the first part `first` entries, then parts doubling
// up to `part` (ramp; without it every later part is `part`), each rounded
// up to a group edge; the last part ends at n.
inline std::vector<uint32_t> stream_part_bounds(uint32_t n, uint32_t m, uint32_t first, uint32_t part, bool ramp) {
  std::vector<uint32_t> b{0};
  uint32_t want = std::max<uint32_t>(1, first);
  part = std::max<uint32_t>(1, part);
  while (b.back() < n) {
    const uint64_t e1 = std::min<uint64_t>(n, ((uint64_t)b.back() + want + m - 1) / m * m);
    b.push_back((uint32_t)e1);
    want = ramp ? (uint32_t)std::min<uint64_t>(part, 2ull * want) : part;
  }
  return b;
}

// The same schedule for a streamed mixed chunk (its parts are split by kind
// on the device, so they need not end on group edges), with at most
// max_parts parts: the later parts grow until they fit.
inline std::vector<uint32_t> mixed_part_bounds(uint32_t n, uint32_t first, uint32_t part, bool ramp,
                                               uint32_t max_parts) {
  first = std::max<uint32_t>(1, first);
  uint64_t part_len = std::max<uint32_t>(1, part);
  const uint32_t slack = ramp ? 32 : 0;  // the ramp's extra parts: < 32 doublings
  while ((n - std::min(n, first) + part_len - 1) / part_len + 1 + slack > max_parts) part_len *= 2;
  std::vector<uint32_t> b{0};
  for (uint64_t want = first; b.back() < n; want = ramp ? std::min<uint64_t>(part_len, 2 * want) : part_len)
    b.push_back((uint32_t)std::min<uint64_t>(n, b.back() + want));
  return b;
}

// Caller pages locked for direct DMA, per span (pk, sig, msg, kind) of a
// chunk: the whole pages inside the first part that has some, then, at the
// next part, every whole page of the rest of the span in one range -- two
// ranges per span, each wholly inside the caller's bytes (a neighbouring
// buffer's registration never collides).  Bytes outside the locked pages go
// through the staging; a span whose range cannot be locked is staged for the
// rest of the chunk (`failed`).
struct SpanPins {
  uintptr_t lo = 0, mid = 0, hi = 0;  // locked [lo, mid) and [mid, hi) (mid == hi: one range)
  bool failed = false;
};

// The range to lock for the part [s0, s1) of a span ending at span_end
// (page: the page size), if any: true and [*r0, *r1) when one is due.
inline bool next_pin_range(const SpanPins &r, uintptr_t s0, uintptr_t s1, uintptr_t span_end, uintptr_t page,
                           uintptr_t *r0, uintptr_t *r1) {
  if (r.failed || s1 <= r.hi) return false;
  if (r.hi && r.hi >= (span_end & ~(page - 1))) return false;  // the rest is locked already
  const uintptr_t a = r.hi ? r.hi : (s0 + page - 1) & ~(page - 1);
  const uintptr_t z = (r.hi ? span_end : s1) & ~(page - 1);
  if (z < a + page) return false;
  *r0 = a;
  *r1 = z;
  return true;
}

// Record a locked range (after next_pin_range and a successful lock).
inline void commit_pin_range(SpanPins &r, uintptr_t r0, uintptr_t r1) {
  if (!r.hi) r.lo = r0;
  r.mid = r.hi ? r.hi : r1;
  r.hi = r1;
}

// The part's bytes [s0, s1) DMA'd from locked pages: offsets [*d0, *d1)
// (d0 == d1: none, all staged), one DMA per locked range -- split at *cut
// (*cut == *d1: no split); the bytes before d0 and from d1 are staged.
inline void direct_piece(const SpanPins &r, uintptr_t s0, uintptr_t s1, size_t *d0, size_t *d1, size_t *cut) {
  *d0 = *d1 = *cut = 0;
  if (!r.hi) return;
  const uintptr_t c0 = std::max(s0, r.lo), c1 = std::min(s1, r.hi);
  if (c1 <= c0) return;
  *d0 = c0 - s0;
  *d1 = c1 - s0;
  *cut = r.mid > c0 && r.mid < c1 ? r.mid - s0 : *d1;
}

}  // namespace tmh
