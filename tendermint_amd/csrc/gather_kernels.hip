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

// 16 bytes from any byte address: aligned dword loads (each holds at least
// one wanted byte, so none reaches past the source's last page) shifted
// together.
__device__ __forceinline__ uint4 load16_any(const uint8_t *src) {
  const uintptr_t a = (uintptr_t)src;
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t *p = reinterpret_cast<const uint32_t *>(a - sh);
  const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3];
  if (sh == 0) return make_uint4(w0, w1, w2, w3);
  const uint32_t w4 = p[4];
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                    __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}

// Lane t: entry t's key and signature (16-byte vector copies when the source
// is aligned) and rebased message offset, and the t-th 16-byte-aligned span
// of the gathered message bytes.  A batch's messages are one contiguous run
// in its source and in the gathered buffer, so a span inside one batch is one
// 16-byte store; spans at the run's ends or across a batch boundary go byte
// by byte.
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
  // spans start where msg + x is 16-byte aligned
  const int64_t mis = (int64_t)((uintptr_t)msg & 15);
  const int64_t x0 = ((((int64_t)r.msg_base[0] + mis) & ~(int64_t)15) - mis) + 16 * (int64_t)t;
  if (x0 >= (int64_t)M) return;
  const uint32_t lo = (uint32_t)max(x0, (int64_t)r.msg_base[0]);
  const uint32_t hi = (uint32_t)min((int64_t)M, x0 + 16);
  uint32_t b = batch_of_byte(r, lo);
  if ((int64_t)lo == x0 && hi == lo + 16 && (b + 1 == r.nb || hi <= r.msg_base[b + 1])) {
    const uint8_t *src = r.msg[b] + r.off[b][0] + (lo - r.msg_base[b]);
    *reinterpret_cast<uint4 *>(msg + lo) = load16_any(src);
    return;
  }
  for (uint32_t x = lo; x < hi; x++) {
    while (b + 1 < r.nb && x >= r.msg_base[b + 1]) b++;  // a span may cross into the next batch
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
  // one more span than the bytes need: spans are aligned to msg's address
  const uint32_t lanes = max(N, (r.msg_base[r.nb] - r.msg_base[0]) / 16 + 2);
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
