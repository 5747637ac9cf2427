// Shard and chunk plan of a host-buffer batch (tmverify_runtime.cpp,
// run_batch): the batch is cut into one contiguous shard per device (tiny
// batches stay on one device), each shard into chunks that rotate over the
// device's host lanes, so a chunk's staging and copy overlap the previous
// chunk's kernels.  Pure host arithmetic, unit-tested on the CPU
// (tests/test_shard_plan.py through tests/native/commit_check.cpp).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace tmh {

struct ShardPlan {
  uint32_t shards = 0;
  std::vector<uint32_t> bounds;   // shard s covers [bounds[s], bounds[s + 1])
  std::vector<uint32_t> nchunks;  // chunks of shard s
  uint32_t max_chunks = 0;

  // chunk k of shard s covers [chunk_lo(s, k), chunk_lo(s, k + 1))
  uint32_t chunk_lo(uint32_t s, uint32_t k) const {
    const uint32_t len = bounds[s + 1] - bounds[s];
    return bounds[s] + (uint32_t)((uint64_t)len * k / nchunks[s]);
  }
};

// n entries over ndev devices, chunks of host_chunk entries (at least 2048):
// shards = min(ndev, n / 1024) (at least 1), equal contiguous ranges; a
// shard of len entries gets min(len / (chunk / 2), max(4, len / chunk))
// chunks (at least 1): at least chunk / 2 entries each, 4 once there is
// room, then chunk each -- fewer, larger chunks keep the key-merged form's
// per-chunk sort and launch chain cheap.
inline ShardPlan plan_shards(uint32_t n, uint32_t ndev, uint32_t host_chunk) {
  ShardPlan p;
  p.shards = std::max<uint32_t>(1, std::min<uint32_t>(ndev, n / 1024));
  p.bounds.resize(p.shards + 1);
  for (uint32_t s = 0; s <= p.shards; s++) p.bounds[s] = (uint32_t)((uint64_t)n * s / p.shards);
  const uint32_t chunk = std::max<uint32_t>(2048, host_chunk);
  p.nchunks.resize(p.shards);
  for (uint32_t s = 0; s < p.shards; s++) {
    const uint32_t len = p.bounds[s + 1] - p.bounds[s];
    p.nchunks[s] = std::max<uint32_t>(1, std::min<uint32_t>(len / (chunk / 2), std::max<uint32_t>(4, len / chunk)));
    p.max_chunks = std::max(p.max_chunks, p.nchunks[s]);
  }
  return p;
}

}  // namespace tmh
