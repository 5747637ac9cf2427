// Host-to-device copy rates on one GPU (development tool): pinned or
// registered host memory, 1 / 2 / 4 copy streams (SDMA), and a copy kernel
// that reads the mapped host pages itself (uint4 loads from many waves).
//   hipcc --offload-arch=gfx950 -O2 tools/h2dbench.hip -o tools/h2dbench && ./tools/h2dbench [MiB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void __launch_bounds__(256) k_pull(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

static double copy_streams(void *d, const void *h, size_t bytes, int ns, std::vector<hipStream_t> &st, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  double best = 1e30;
  for (int r = 0; r < reps; r++) {
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    const size_t per = (bytes / ns + 4095) & ~(size_t)4095;
    for (int s = 0; s < ns; s++) {
      const size_t lo = per * s;
      if (lo >= bytes) break;
      const size_t len = std::min(per, bytes - lo);
      CK(hipMemcpyAsync((char *)d + lo, (const char *)h + lo, len, hipMemcpyHostToDevice, st[s]));
    }
    CK(hipDeviceSynchronize());
    best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  return bytes / best / 1e9;
}

static double pull(void *d, const void *hdev, size_t bytes, int blocks, int reps) {
  double best = 1e30;
  for (int r = 0; r < reps; r++) {
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_pull, dim3(blocks), dim3(256), 0, 0, (const uint4 *)hdev, (uint4 *)d, bytes / 16);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  return bytes / best / 1e9;
}

int main(int argc, char **argv) {
  const size_t mib = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 128;
  const size_t bytes = mib << 20;
  void *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  std::memset(h, 1, bytes);
  CK(hipMalloc(&d, bytes));
  std::vector<hipStream_t> st(8);
  for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::printf("{\"bytes\": %zu", bytes);
  for (int ns : {1, 2, 4, 8}) std::printf(", \"pinned_streams%d_GBps\": %.2f", ns, copy_streams(d, h, bytes, ns, st, 5));
  void *hdev = nullptr;
  CK(hipHostGetDevicePointer(&hdev, h, 0));
  for (int blocks : {256, 1024, 4096})
    std::printf(", \"pull_kernel_%d_GBps\": %.2f", blocks, pull(d, hdev, bytes, blocks, 5));
  // registered (malloc'd) memory
  void *m = std::aligned_alloc(4096, bytes);
  std::memset(m, 2, bytes);
  const auto t0 = std::chrono::steady_clock::now();
  CK(hipHostRegister(m, bytes, hipHostRegisterMapped));
  const double reg_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::printf(", \"register_ms\": %.3f", reg_ms);
  for (int ns : {1, 2, 4}) std::printf(", \"registered_streams%d_GBps\": %.2f", ns, copy_streams(d, m, bytes, ns, st, 5));
  void *mdev = nullptr;
  CK(hipHostGetDevicePointer(&mdev, m, 0));
  for (int blocks : {1024, 4096})
    std::printf(", \"registered_pull_%d_GBps\": %.2f", blocks, pull(d, mdev, bytes, blocks, 5));
  CK(hipHostUnregister(m));
  std::printf("}\n");
  return 0;
}
