// Field-arithmetic A/B: the radix-2^25.5 integer field (curve25519.h,
// v_mad_i64_i32) against the radix-2^21.25 FP64 field (fe64.h, v_fma_f64)
// on the decompression square-root chain z^((p-5)/8) and on plain
// squaring / multiply chains.  Checks that both produce the same canonical
// words for every input, then prints one JSON line of rates.
//   hipcc -O3 --offload-arch=gfx950 -I tendermint_amd/csrc -I tools tools/fieldbench.hip -o /tmp/fieldbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "curve25519.h"
#include "fe64.h"

using namespace tmv;

#define SQ_ITERS 256

__global__ void __launch_bounds__(256) k_pow_int(const uint32_t *in, uint32_t *out, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  fe z, h;
  fe_from_words(z, in + 8 * t);
  fe_pow22523(h, z);
  fe_to_words(out + 8 * t, h);
}

__global__ void __launch_bounds__(256) k_pow_fd(const uint32_t *in, uint32_t *out, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  fe z, h;
  fe_from_words(z, in + 8 * t);
  fe_pow22523_fd(h, z);
  fe_to_words(out + 8 * t, h);
}

// two independent chains of x <- x^2 * y per thread (one sq + one mul)
__global__ void __launch_bounds__(256) k_chain_int(const uint32_t *in, uint32_t *out, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  fe a, b, y;
  fe_from_words(a, in + 8 * t);
  fe_from_words(b, in + 8 * ((t + 1) % n));
  fe_from_words(y, in + 8 * ((t + 2) % n));
  for (int i = 0; i < SQ_ITERS; i++) {
    fe_sq(a, a); fe_mul(a, a, y);
    fe_sq(b, b); fe_mul(b, b, y);
  }
  fe_add(a, a, b);
  fe_to_words(out + 8 * t, a);
}

__global__ void __launch_bounds__(256) k_chain_fd(const uint32_t *in, uint32_t *out, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  fe a0, b0, y0;
  fe_from_words(a0, in + 8 * t);
  fe_from_words(b0, in + 8 * ((t + 1) % n));
  fe_from_words(y0, in + 8 * ((t + 2) % n));
  fd a, b, y;
  fd_from_fe(a, a0); fd_from_fe(b, b0); fd_from_fe(y, y0);
  for (int i = 0; i < SQ_ITERS; i++) {
    fd_sq(a, a); fd_mul(a, a, y);
    fd_sq(b, b); fd_mul(b, b, y);
  }
  fd_add(a, a, b);
  fe r;
  fe_from_fd(r, a);
  fe_to_words(out + 8 * t, r);
}

static float time_kernel(void (*k)(const uint32_t *, uint32_t *, int), const uint32_t *in, uint32_t *out, int n) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, in, out, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return best;
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : (1 << 20);
  std::mt19937_64 rng(7);
  std::vector<uint32_t> h_in(8ull * n);
  for (auto &w : h_in) w = (uint32_t)rng();
  for (int i = 0; i < n; i++) h_in[8ull * i + 7] &= 0x7fffffffu;
  // edge inputs: 0, 1, p - 1, p, 2^255 - 1 (lax values >= p)
  const uint32_t P[8] = {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                         0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
  for (int k = 0; k < 5 && k < n; k++) {
    for (int w = 0; w < 8; w++) {
      uint32_t v = 0;
      if (k == 1) v = w == 0;
      if (k == 2) v = w == 0 ? P[0] - 1 : P[w];
      if (k == 3) v = P[w];
      if (k == 4) v = w == 7 ? 0x7fffffffu : 0xffffffffu;
      h_in[8 * k + w] = v;
    }
  }
  uint32_t *d_in, *d_a, *d_b;
  hipMalloc(&d_in, 32ull * n);
  hipMalloc(&d_a, 32ull * n);
  hipMalloc(&d_b, 32ull * n);
  hipMemcpy(d_in, h_in.data(), 32ull * n, hipMemcpyHostToDevice);
  std::vector<uint32_t> ra(8ull * n), rb(8ull * n);

  const float pow_int = time_kernel(k_pow_int, d_in, d_a, n);
  const float pow_fd = time_kernel(k_pow_fd, d_in, d_b, n);
  hipMemcpy(ra.data(), d_a, 32ull * n, hipMemcpyDeviceToHost);
  hipMemcpy(rb.data(), d_b, 32ull * n, hipMemcpyDeviceToHost);
  long pow_mismatch = 0;
  for (size_t i = 0; i < ra.size(); i++) pow_mismatch += ra[i] != rb[i];
  // host check of a few entries against the host build of the int chain
  long host_mismatch = 0;
  for (int t = 0; t < n && t < 64; t++) {
    fe z, h;
    fe_from_words(z, &h_in[8 * t]);
    fe_pow22523(h, z);
    uint32_t w[8];
    fe_to_words(w, h);
    host_mismatch += memcmp(w, &ra[8 * t], 32) != 0;
    fd a, b;
    fd_from_fe(a, z);
    fd_pow22523(b, a);
    fe_from_fd(h, b);
    fe_to_words(w, h);
    host_mismatch += memcmp(w, &rb[8 * t], 32) != 0;
  }

  const float ch_int = time_kernel(k_chain_int, d_in, d_a, n);
  const float ch_fd = time_kernel(k_chain_fd, d_in, d_b, n);
  hipMemcpy(ra.data(), d_a, 32ull * n, hipMemcpyDeviceToHost);
  hipMemcpy(rb.data(), d_b, 32ull * n, hipMemcpyDeviceToHost);
  long chain_mismatch = 0;
  for (size_t i = 0; i < ra.size(); i++) chain_mismatch += ra[i] != rb[i];

  const double pow_ops = 265.0 * n;  // 254 sq + 11 mul per exponentiation
  const double ch_ops = 4.0 * SQ_ITERS * n;
  printf("{\"n\": %d, \"pow_int_ms\": %.4f, \"pow_fd_ms\": %.4f, \"pow_speedup\": %.3f, "
         "\"pow_int_fieldops_per_s\": %.4e, \"pow_fd_fieldops_per_s\": %.4e, \"pow_mismatch_words\": %ld, "
         "\"host_mismatch\": %ld, \"chain_int_ms\": %.4f, \"chain_fd_ms\": %.4f, \"chain_speedup\": %.3f, "
         "\"chain_int_fieldops_per_s\": %.4e, \"chain_fd_fieldops_per_s\": %.4e, \"chain_mismatch_words\": %ld}\n",
         n, pow_int, pow_fd, pow_int / pow_fd, pow_ops / (pow_int * 1e-3), pow_ops / (pow_fd * 1e-3), pow_mismatch,
         host_mismatch, ch_int, ch_fd, ch_int / ch_fd, ch_ops / (ch_int * 1e-3), ch_ops / (ch_fd * 1e-3),
         chain_mismatch);
  return (pow_mismatch || chain_mismatch || host_mismatch) ? 1 : 0;
}
