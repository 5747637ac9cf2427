// Device-side vote sign-bytes (tmv_verify_votes): each lane writes one
// vote's canonical message (votes.h) into the batch's message buffer, where
// the verification kernels read it as if the host had sent it.  The host
// sends 16 bytes per vote plus one template per commit instead of ~120 bytes
// of encoded message; the kernel is pure byte movement (HBM/L2-bound, a few
// microseconds per 100k votes next to ~1 ms of verification).
#include <hip/hip_runtime.h>
#include "verify_kernels.h"
#include "votes.h"

namespace tmv {

__device__ __forceinline__ uint8_t *put_uvarint(uint8_t *p, uint64_t x) {
  while (x >= 0x80) { *p++ = (uint8_t)(x | 0x80); x >>= 7; }
  *p++ = (uint8_t)x;
  return p;
}

__device__ __forceinline__ uint8_t *put_bytes(uint8_t *p, const uint8_t *src, uint32_t n) {
  for (uint32_t k = 0; k < n; k++) p[k] = src[k];
  return p + n;
}

__global__ void __launch_bounds__(256)
k_vote_signbytes(const tmv_vote *__restrict__ votes, const VoteTab *__restrict__ tab,
                 const uint8_t *__restrict__ blob, const uint32_t *__restrict__ off, uint32_t n,
                 uint8_t *__restrict__ msg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const tmv_vote v = votes[i];
  const VoteTab t = tab[v.tmpl & ~TMV_VOTE_WITH_BLOCK];
  uint8_t *p = msg + off[i];
  p = put_uvarint(p, vote_body_len(t, v));
  p = put_bytes(p, blob + t.head_at, t.head_len);
  if (v.tmpl & TMV_VOTE_WITH_BLOCK) p = put_bytes(p, blob + t.block_at, t.block_len);
  *p++ = 0x2a;
  p = put_uvarint(p, vote_ts_inner(v.ts_seconds, v.ts_nanos));
  if (v.ts_seconds != 0) { *p++ = 0x08; p = put_uvarint(p, (uint64_t)v.ts_seconds); }
  if (v.ts_nanos != 0) { *p++ = 0x10; p = put_uvarint(p, (uint64_t)(int64_t)v.ts_nanos); }
  put_bytes(p, blob + t.chain_at, t.chain_len);
}

// Template indices are checked on the host (tmv_verify_votes) before launch.
hipError_t launch_vote_signbytes(const tmv_vote *votes, const VoteTab *tab, const uint8_t *blob,
                                 const uint32_t *off, uint32_t n, uint8_t *msg, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_vote_signbytes, dim3((n + 255) / 256), dim3(256), 0, stream, votes, tab, blob, off, n, msg);
  return hipGetLastError();
}

}  // namespace tmv
