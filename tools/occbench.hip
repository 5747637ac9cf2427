// Throughput vs. number of resident waves (64-thread blocks) for the two
// candidate multiply instructions of the field arithmetic: v_mad_i64_i32 and
// v_fma_f64.  Answers: how much of a SIMD's multiply rate does ONE wave get
// (the 10k-signature batch runs about one wave per SIMD)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 16
#define ITERS 2048

__global__ void __launch_bounds__(64) k_mad(int64_t *out, int32_t seed) {
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

__global__ void __launch_bounds__(64) k_fma(double *out, double seed) {
  double a = seed + threadIdx.x;
  double acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc[c] = c + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc[c] = fma(acc[c], 0.999999, a + c);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  void *buf;
  hipMalloc(&buf, (size_t)65536 * 64 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int waves[] = {256, 512, 768, 1024, 1536, 2048, 4096, 8192, 16384};
  printf("{\"rows\": [");
  for (int wi = 0; wi < 9; wi++) {
    const int w = waves[wi];
    const double ops = (double)w * 64 * ITERS * CHAINS;
    float ms_m = 0, ms_f = 0, t;
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0); hipLaunchKernelGGL(k_mad, dim3(w), dim3(64), 0, 0, (int64_t *)buf, 123 + rep);
      hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&t, e0, e1); if (rep) ms_m += t / 2;
      hipEventRecord(e0); hipLaunchKernelGGL(k_fma, dim3(w), dim3(64), 0, 0, (double *)buf, 1.0 + rep);
      hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&t, e0, e1); if (rep) ms_f += t / 2;
    }
    printf("%s{\"waves\": %d, \"mad_ms\": %.4f, \"mad_per_s\": %.4e, \"fma_ms\": %.4f, \"fma_per_s\": %.4e}",
           wi ? ", " : "", w, ms_m, ops / (ms_m * 1e-3), ms_f, ops / (ms_f * 1e-3));
  }
  printf("]}\n");
  return 0;
}
