// Multi-batch launches (tmv_verify_batches_device): K independent device
// batches are gathered into one contiguous batch, verified by one pipeline,
// and each batch's statuses are scattered back to its own output.  Entries
// never mix verdicts across batches (the per-entry vector is exact); batching
// only widens the launches, the way a node draining a queue of commits or
// blocks would.  Pure data movement (HBM-bound).
#include <hip/hip_runtime.h>
#include "verify_kernels.h"

namespace tmv {

// Batches [0, nb) of one BatchRefs cover gathered entries [start[0],
// start[nb]) and message bytes [msg_base[0], msg_base[nb]) (a launch of more
// than kMaxBatches batches passes several BatchRefs).
__device__ __forceinline__ uint32_t batch_of(const BatchRefs &r, uint32_t e) {
  uint32_t b = 0;
  for (uint32_t k = 1; k < r.nb; k++) b = (e >= r.start[k]) ? k : b;
  return b;
}

// Batch holding gathered message byte x (msg_base is ascending).
__device__ __forceinline__ uint32_t batch_of_byte(const BatchRefs &r, uint32_t x) {
  uint32_t b = 0;
  for (uint32_t k = 1; k < r.nb; k++) b = (x >= r.msg_base[k]) ? k : b;
  return b;
}

// Lane t: entry t's key and signature (16-byte vector copies when the source
// is aligned) and rebased message offset, and gathered message bytes
// [16 t, 16 t + 16).  A batch's messages are one contiguous run in its
// source and in the gathered buffer, so consecutive lanes copy consecutive
// bytes (coalesced) instead of each lane walking its own message.
__global__ void __launch_bounds__(256)
k_gather(BatchRefs r, uint8_t *__restrict__ pk, uint8_t *__restrict__ sig, uint32_t *__restrict__ off,
         uint8_t *__restrict__ msg) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t N = r.start[r.nb], M = r.msg_base[r.nb];
  if (r.start[0] + t < N) {
    const uint32_t e = r.start[0] + t;
    const uint32_t b = batch_of(r, e), i = e - r.start[b];
    const uint8_t *spk = r.pk[b] + 32ull * i, *ssig = r.sig[b] + 64ull * i;
    if (((((uintptr_t)spk) | ((uintptr_t)ssig)) & 15) == 0) {
      const uint4 *a = reinterpret_cast<const uint4 *>(spk);
      const uint4 *s = reinterpret_cast<const uint4 *>(ssig);
      uint4 *da = reinterpret_cast<uint4 *>(pk + 32ull * e);
      uint4 *ds = reinterpret_cast<uint4 *>(sig + 64ull * e);
      da[0] = a[0]; da[1] = a[1];
      ds[0] = s[0]; ds[1] = s[1]; ds[2] = s[2]; ds[3] = s[3];
    } else {
      for (int q = 0; q < 32; q++) pk[32ull * e + q] = spk[q];
      for (int q = 0; q < 64; q++) sig[64ull * e + q] = ssig[q];
    }
    const uint32_t *so = r.off[b];
    off[e] = r.msg_base[b] + (so[i] - so[0]);
    if (e + 1 == N) off[N] = r.msg_base[b] + (so[i + 1] - so[0]);
  }
  const uint32_t x0 = r.msg_base[0] + 16 * t;
  if (x0 >= M) return;
  uint32_t b = batch_of_byte(r, x0);
  const uint32_t x1 = min(M, x0 + 16);
  for (uint32_t x = x0; x < x1; x++) {
    while (b + 1 < r.nb && x >= r.msg_base[b + 1]) b++;  // a 16-byte span may cross into the next batch
    msg[x] = r.msg[b][r.off[b][0] + (x - r.msg_base[b])];
  }
}

__global__ void __launch_bounds__(256)
k_scatter(BatchRefs r, const int8_t *__restrict__ status) {
  const uint32_t e = r.start[0] + blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= r.start[r.nb]) return;
  const uint32_t b = batch_of(r, e);
  r.out[b][e - r.start[b]] = status[e];
}

hipError_t launch_gather(const BatchRefs &r, uint8_t *pk, uint8_t *sig, uint32_t *off, uint8_t *msg,
                         hipStream_t stream) {
  const uint32_t N = r.start[r.nb] - r.start[0];
  if (N == 0) return hipSuccess;
  const uint32_t lanes = max(N, (r.msg_base[r.nb] - r.msg_base[0] + 15) / 16);
  hipLaunchKernelGGL(k_gather, dim3((lanes + 255) / 256), dim3(256), 0, stream, r, pk, sig, off, msg);
  return hipGetLastError();
}

hipError_t launch_scatter(const BatchRefs &r, const int8_t *status, hipStream_t stream) {
  const uint32_t N = r.start[r.nb] - r.start[0];
  if (N == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter, dim3((N + 255) / 256), dim3(256), 0, stream, r, status);
  return hipGetLastError();
}

}  // namespace tmv
