// MI355X (gfx950) verification kernels.
//
// k_ed25519_verify: one lane per signature, full ZIP-215 verification
// (SHA-512 challenge, scalar reduction, lax decompression of A and R,
// [S]B by a 32x8 base-point comb in global memory, [k]A by signed radix-16
// windows, cofactored identity test).  All integer VALU work — the
// 32x32->64 multiply-adds of the radix-2^25.5 field dominate (see DESIGN.md
// for the roofline), so there is no MFMA or LDS tiling here.
#include <hip/hip_runtime.h>
#include "ed25519_core.h"
#include "verify_kernels.h"

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

__global__ void __launch_bounds__(kVerifyBlock)
k_ed25519_verify(const uint8_t *__restrict__ pk, const uint8_t *__restrict__ sig,
                 const uint8_t *__restrict__ msg, const uint32_t *__restrict__ msg_off, uint32_t n,
                 const ge_precomp *__restrict__ btable, uint8_t *__restrict__ valid, int aligned) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t a_w[8], r_w[8], s_w[8];
  if (aligned) {
    load_words_aligned(a_w, pk + 32ull * i);
    load_words_aligned(r_w, sig + 64ull * i);
    load_words_aligned(s_w, sig + 64ull * i + 32);
  } else {
    load_words_unaligned(a_w, pk + 32ull * i);
    load_words_unaligned(r_w, sig + 64ull * i);
    load_words_unaligned(s_w, sig + 64ull * i + 32);
  }
  const uint32_t o0 = msg_off[i], o1 = msg_off[i + 1];
  const bool ok = ed25519_verify_core(a_w, r_w, s_w, msg + o0, o1 - o0, btable);
  valid[i] = ok ? 1 : 0;
}

hipError_t launch_ed25519_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                 const uint32_t *msg_off, uint32_t n, const ge_precomp *btable,
                                 uint8_t *valid, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  const uint32_t blocks = (n + kVerifyBlock - 1) / kVerifyBlock;
  hipLaunchKernelGGL(k_ed25519_verify, dim3(blocks), dim3(kVerifyBlock), 0, stream, pk, sig, msg, msg_off, n,
                     btable, valid, aligned);
  return hipGetLastError();
}

}  // namespace tmv
