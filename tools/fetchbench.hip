// FETCH_SIZE calibration on gfx950 (MI355X_MICROARCH.md: "other access widths
// are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Three kernels read a known number of bytes once each, far
// past the 256 MiB Infinity Cache:
//   k_stream     16 B per lane, fully coalesced (the guide's calibrated case)
//   k_runs160    k_msm_wpart's pattern: one lane per run of 32 consecutive
//                160-byte extended points (ge_p3, 4-byte aligned), read from
//                the top down, neighbouring lanes 32 x 160 B apart
//   k_gather160  one 160-byte point per lane at a scattered index (chunk
//                partials joined by bucket_value)
// Run under rocprofv3 --pmc FETCH_SIZE (tools/profile_r03.sh); each kernel
// prints its byte count, so FETCH_SIZE / bytes is the correction per pattern.
//   hipcc -O3 --offload-arch=gfx950 -I tendermint_amd/csrc tools/fetchbench.hip -o tools/fetchbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "curve25519.h"

using namespace tmv;

struct pt160 { fe X, Y, Z, T; };  // ge_p3's layout: 160 B, 4-byte aligned

__global__ void __launch_bounds__(256) k_stream(const uint4 *in, uint32_t n16, uint32_t *sink) {
  uint32_t acc = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads
}

__global__ void __launch_bounds__(256) k_runs160(const pt160 *in, uint32_t lanes, uint32_t *sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= lanes) return;
  uint32_t acc = 0;
  const pt160 *run = in + 32ull * t;
  for (int i = 31; i >= 0; i--) {
    const pt160 p = run[i];
#pragma unroll
    for (int k = 0; k < 10; k++) acc ^= (uint32_t)(p.X.v[k] ^ p.Y.v[k] ^ p.Z.v[k] ^ p.T.v[k]);
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_gather160(const pt160 *in, const uint32_t *idx, uint32_t lanes,
                                                   uint32_t *sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= lanes) return;
  const pt160 p = in[idx[t]];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) acc ^= (uint32_t)(p.X.v[k] ^ p.Y.v[k] ^ p.Z.v[k] ^ p.T.v[k]);
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const size_t bytes = 2ull << 30;  // 2 GiB: 8x the Infinity Cache
  uint8_t *buf;
  uint32_t *sink, *idx;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(buf, 1, bytes));
  const uint32_t n_pts = (uint32_t)(bytes / sizeof(pt160));
  const uint32_t run_lanes = n_pts / 32;
  const uint32_t g_lanes = n_pts / 4;  // a quarter of the points, scattered
  std::vector<uint32_t> h_idx(g_lanes);
  uint64_t s = 88172645463325252ull;
  for (uint32_t i = 0; i < g_lanes; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h_idx[i] = (uint32_t)(s % n_pts);
  }
  CK(hipMalloc(&idx, 4ull * g_lanes));
  CK(hipMemcpy(idx, h_idx.data(), 4ull * g_lanes, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  const uint32_t n16 = (uint32_t)(bytes / 16);
  hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const uint4 *>(buf), n16, sink);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_runs160, dim3((run_lanes + 255) / 256), dim3(256), 0, 0, reinterpret_cast<const pt160 *>(buf),
                     run_lanes, sink);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_gather160, dim3((g_lanes + 255) / 256), dim3(256), 0, 0, reinterpret_cast<const pt160 *>(buf),
                     idx, g_lanes, sink);
  CK(hipDeviceSynchronize());
  printf("{\"k_stream_bytes\": %zu, \"k_runs160_bytes\": %zu, \"k_gather160_bytes\": %zu, "
         "\"k_gather160_idx_bytes\": %zu}\n",
         (size_t)n16 * 16, (size_t)run_lanes * 32 * sizeof(pt160), (size_t)g_lanes * sizeof(pt160),
         (size_t)g_lanes * 4);
  return 0;
}
