// Small device helpers shared by the verification and batch-check kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmv {

__device__ __forceinline__ void load_words_unaligned(uint32_t w[8], const uint8_t *p) {
#pragma unroll
  for (int i = 0; i < 8; i++)
    w[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
           ((uint32_t)p[4 * i + 3] << 24);
}

__device__ __forceinline__ void load_words_aligned(uint32_t w[8], const uint8_t *p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  const uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// Entry count of a launch: on the device for partitioned (mixed) batches.
__device__ __forceinline__ uint32_t entry_count(const uint32_t *count_ptr, uint32_t n) {
  return count_ptr ? *count_ptr : n;
}

}  // namespace tmv
