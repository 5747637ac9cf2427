// Microbenchmark: peak integer-multiply throughput on MI355X (gfx950).
// Measures P_mul: 32x32->64 multiply-add products per second
// chip-wide for v_mad_u64_u32 / v_mad_i64_i32, plus the 24-bit and 32-bit
// low/high forms and v_fma_f64 for comparison.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define ITERS 4096

__global__ void k_mad_u64(uint64_t *out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
  uint64_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc[c] = c + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = (uint64_t)(a + c) * b + acc[c];
    a += (uint32_t)acc[0];
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_i64(int64_t *out, int32_t seed) {
  int32_t a = seed ^ threadIdx.x, b = seed * 7 + blockIdx.x;
  int64_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc[c] = c + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = (int64_t)(a + c) * b + acc[c];
    a += (int32_t)acc[0];
  }
  int64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_lo32(uint32_t *out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x;
  uint32_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc[c] = c + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = acc[c] * (a + c) + c;
    a ^= acc[1];
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_u24(uint32_t *out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x;
  uint32_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc[c] = c + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = __umul24(acc[c], a + c) + c;
    a ^= acc[1];
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma_f64(double *out, double seed) {
  double a = seed + threadIdx.x;
  double acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc[c] = c + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = fma(acc[c], 0.999999, a);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  const int threads = 256, blocks = cus * 8;  // 8 waves/SIMD worth
  void *buf;
  hipMalloc(&buf, (size_t)blocks * threads * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const double ops = (double)blocks * threads * ITERS * CHAINS;
  float ms;
  double r[5];
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0); hipLaunchKernelGGL(k_mad_u64, dim3(blocks), dim3(threads), 0, 0, (uint64_t *)buf, 12345u + rep);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); r[0] = ops / (ms * 1e-3);
    hipEventRecord(e0); hipLaunchKernelGGL(k_mad_i64, dim3(blocks), dim3(threads), 0, 0, (int64_t *)buf, 12345 + rep);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); r[1] = ops / (ms * 1e-3);
    hipEventRecord(e0); hipLaunchKernelGGL(k_mul_lo32, dim3(blocks), dim3(threads), 0, 0, (uint32_t *)buf, 12345u + rep);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); r[2] = ops / (ms * 1e-3);
    hipEventRecord(e0); hipLaunchKernelGGL(k_mul_u24, dim3(blocks), dim3(threads), 0, 0, (uint32_t *)buf, 12345u + rep);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); r[3] = ops / (ms * 1e-3);
    hipEventRecord(e0); hipLaunchKernelGGL(k_fma_f64, dim3(blocks), dim3(threads), 0, 0, (double *)buf, 1.0 + rep);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); r[4] = ops / (ms * 1e-3);
  }
  printf("{\"cus\": %d, \"clock_khz\": %d, \"mad_u64_u32_per_s\": %.4e, \"mad_i64_i32_per_s\": %.4e, "
         "\"mul_lo_u32_per_s\": %.4e, \"mul_u24_per_s\": %.4e, \"fma_f64_per_s\": %.4e}\n",
         cus, clk, r[0], r[1], r[2], r[3], r[4]);
  return 0;
}
