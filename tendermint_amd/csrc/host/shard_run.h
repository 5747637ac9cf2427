// The order in which a host-buffer batch's chunks are staged, launched and
// harvested over the devices of a context (tmverify_runtime.cpp run_batch):
// chunk k of every shard, then chunk k + 1, so the devices work side by side;
// a chunk goes to lane k % lanes of its device, whose previous chunk is
// harvested first (its staging is reused); at the end every lane of every
// device is drained.  Written once for the runtime and for the CPU test
// double (tests/native/commit_check.cpp), which runs it over simulated
// devices so a multi-device context's placement is tested without GPUs.
#pragma once
#include <stdint.h>

#include "shard_plan.h"

namespace tmh {

// harvest(shard, lane, ok) waits for the lane's chunk in flight (if any) and,
// when ok, takes its results; it returns 0 or an error code.
// launch(shard, lane, lo, hi) stages entries [lo, hi) and starts them; 0 or
// an error.  Returns the first error; after one, the remaining lanes are
// still drained (harvest with ok = false) and nothing more is launched.
template <class Harvest, class Launch>
int run_shard_plan(const ShardPlan &plan, uint32_t lanes, Harvest harvest, Launch launch) {
  int rc = 0;
  for (uint32_t k = 0; k < plan.max_chunks && rc == 0; k++) {
    for (uint32_t s = 0; s < plan.shards && rc == 0; s++) {
      if (k >= plan.nchunks[s]) continue;
      const uint32_t lane = k % lanes;
      rc = harvest(s, lane, true);  // the lane's previous chunk
      if (rc != 0) break;
      rc = launch(s, lane, plan.chunk_lo(s, k), plan.chunk_lo(s, k + 1));
    }
  }
  for (uint32_t s = 0; s < plan.shards; s++)
    for (uint32_t lane = 0; lane < lanes; lane++) {
      const int r = harvest(s, lane, rc == 0);
      if (rc == 0) rc = r;
    }
  return rc;
}

}  // namespace tmh
