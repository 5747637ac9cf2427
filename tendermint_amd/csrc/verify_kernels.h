// Launch wrappers for the verification kernels (verify_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "curve25519.h"

namespace tmv {

constexpr int kVerifyBlock = 256;
constexpr int kQuadBlock = 64;    // one wave = 16 signatures per block

// Per-signature workspace of the latency path (device memory).
struct Ed25519Work {
  fe *negA;        // n x 4 fe, P3Q layout of -A
  fe *Rc;          // n x 4 fe, CachedQ layout of R
  uint32_t *k;     // n x 8 words, k mod l
  uint8_t *flags;  // 2n bytes: decode ok for A (2i) and R (2i+1)
  static size_t bytes(uint32_t n) { return (size_t)n * (160 + 160 + 32 + 2) + 64; }
};

hipError_t launch_ed25519_verify_quad(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                      const uint32_t *msg_off, uint32_t n, const fe *btab_q, Ed25519Work w,
                                      uint8_t *valid, hipStream_t stream);

hipError_t launch_ed25519_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                 const uint32_t *msg_off, uint32_t n, const ge_precomp *btable,
                                 uint8_t *valid, hipStream_t stream);

}  // namespace tmv
