// Microbenchmark: the cost of the half-size scalar reduction (halfscalar.h,
// Lehmer steps on 50-bit leading digits in doubles) per entry, against a
// field multiply, in throughput (many waves per SIMD).  Decides whether a
// per-entry lattice basis (both batch weights ~192 bits) can pay for itself.
//
//   hipcc -O3 --offload-arch=gfx950 -I tendermint_amd/csrc tools/reduce_bench.hip -o tools/reduce_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "halfscalar.h"

using namespace tmv;

__global__ void __launch_bounds__(256) k_reduce(const uint32_t *ks, uint32_t *out, int reps) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = ks[8ull * t + i];
  uint32_t acc = 0;
  for (int r = 0; r < reps; r++) {
    uint32_t u[4], v[4];
    bool neg;
    const bool ok = half::reduce(u, neg, v, k);
    acc ^= u[0] ^ v[1] ^ (ok ? 1u : 0u) ^ (neg ? 2u : 0u);
    k[0] ^= acc & 1u;  // a dependency between repetitions (k stays < l: bit 0 only)
  }
  out[t] = acc;
}

__global__ void __launch_bounds__(256) k_mul(const uint32_t *ks, uint32_t *out, int reps) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe f, g;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f.v[i] = (int32_t)(ks[8ull * t + (i & 7)] & 0x1ffffff) - (1 << 24);
    g.v[i] = (int32_t)(ks[8ull * t + ((i + 3) & 7)] & 0x1ffffff) - (1 << 24);
  }
  for (int r = 0; r < reps; r++) fe_mul(f, f, g);
  uint32_t w[8];
  fe_to_words(w, f);
  out[t] = w[0] ^ w[7];
}

int main() {
  const int blocks = 4096, threads = blocks * 256;
  std::vector<uint32_t> hk(8ull * threads);
  uint64_t x = 0x1234567887654321ull;
  for (size_t i = 0; i < hk.size(); i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    hk[i] = (uint32_t)x;
    if (i % 8 == 7) hk[i] &= 0x0fffffffu;  // k < 2^252 < l
  }
  uint32_t *dk, *dout;
  hipMalloc(&dk, hk.size() * 4);
  hipMalloc(&dout, threads * 4);
  hipMemcpy(dk, hk.data(), hk.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float t_red = 0, t_mul = 0;
  const int reps_red = 8, reps_mul = 64;
  for (int rep = 0; rep < 4; rep++) {
    float t;
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_reduce, dim3(blocks), dim3(256), 0, 0, dk, dout, reps_red);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&t, e0, e1);
    if (rep) t_red += t / 3;
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(256), 0, 0, dk, dout, reps_mul);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&t, e0, e1);
    if (rep) t_mul += t / 3;
  }
  const double per_red = t_red * 1e6 / ((double)threads * reps_red);  // ns per reduction, chip-wide throughput
  const double per_mul = t_mul * 1e6 / ((double)threads * reps_mul);
  printf("{\"reduce_ns_chip\": %.5f, \"fe_mul_ns_chip\": %.5f, \"reduce_in_fe_muls\": %.1f, \"threads\": %d}\n", per_red,
         per_mul, per_red / per_mul, threads);
  return 0;
}
