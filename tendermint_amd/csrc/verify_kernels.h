// Launch wrappers for the verification kernels (verify_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "curve25519.h"

namespace tmv {

constexpr int kVerifyBlock = 256;

struct ge_precomp;

hipError_t launch_ed25519_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                 const uint32_t *msg_off, uint32_t n, const ge_precomp *btable,
                                 uint8_t *valid, hipStream_t stream);

}  // namespace tmv
