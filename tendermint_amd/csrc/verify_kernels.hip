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
#include "quad.h"
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

// ---------------------------------------------------------------------------
// Latency path: prep kernel (one lane per point) + quad kernel (4 lanes per
// signature).
//
// k_ed25519_prep stores -A in P3Q layout, R in CachedQ layout and k; decode
// failures are recorded in flags (2 bytes per signature).

// Task-uniform waves: lanes [0, n) decode A_i, [n, 2n) decode R_i and
// [2n, 3n) hash k_i = SHA-512(R||A||M) mod l, so no wave mixes the
// decompression and SHA-512 code paths and the three run side by side.
__global__ void __launch_bounds__(kVerifyBlock)
k_ed25519_prep(const uint8_t *__restrict__ pk, const uint8_t *__restrict__ sig, const uint8_t *__restrict__ msg,
               const uint32_t *__restrict__ msg_off, uint32_t n, Ed25519Work w, int aligned) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 3 * n) return;
  const uint32_t task = j / n;
  const uint32_t i = j - task * n;
  uint32_t a_w[8], r_w[8];
  if (task != 1) {
    if (aligned) load_words_aligned(a_w, pk + 32ull * i);
    else load_words_unaligned(a_w, pk + 32ull * i);
  }
  if (task != 0) {
    if (aligned) load_words_aligned(r_w, sig + 64ull * i);
    else load_words_unaligned(r_w, sig + 64ull * i);
  }
  if (task == 2) {
    uint32_t h[16], k[8];
    const uint32_t o0 = msg_off[i], o1 = msg_off[i + 1];
    sha512_pq_msg(h, r_w, a_w, msg + o0, o1 - o0);
    sc_reduce512(k, h);
    uint4 *kd = reinterpret_cast<uint4 *>(w.k + 8ull * i);
    kd[0] = make_uint4(k[0], k[1], k[2], k[3]);
    kd[1] = make_uint4(k[4], k[5], k[6], k[7]);
    return;
  }
  const bool isA = task == 0;
  ge_p3 P;
  const bool ok = ge_decode_zip215(P, isA ? a_w : r_w);
  if (!ok) ge_p3_identity(P);  // keep limbs bounded; the flag rejects the entry
  w.flags[2 * i + (isA ? 0 : 1)] = ok ? 1 : 0;
  fe *dst = (isA ? w.negA : w.Rc) + 4ull * i;
  if (isA) {
    fe t;
    fe_neg(t, P.X); dst[0] = t;
    dst[1] = P.Y;
    fe_one(t); dst[2] = t;
    fe_neg(t, P.T); dst[3] = t;
  } else {
    ge_cached c;
    ge_p3_to_cached(c, P);
    fe t;
    fe_carry(t, c.YmX); dst[0] = t;
    fe_carry(t, c.YpX); dst[1] = t;
    dst[2] = c.T2d;
    dst[3] = c.Z;
  }
}

// Signed radix-16 recoding written straight to LDS (lanes with c >= 2 skip).
__device__ __forceinline__ void recode16_store(int8_t *dst, const uint32_t s[8], bool store) {
  int carry = 0;
#pragma unroll
  for (int i = 0; i < 64; i++) {
    int e = (int)((s[i >> 3] >> (4 * (i & 7))) & 15) + carry;
    if (i < 63) {
      carry = (e + 8) >> 4;
      e -= carry * 16;
    }
    if (store) dst[i] = (int8_t)e;
  }
}

constexpr int kQuadSigs = kQuadBlock / 4;

// k_ed25519_verify_quad: acc = sum over 64 signed radix-16 windows of
// 16*acc + e_i(k)(-A) + e_i(S)B (Straus, shared doublings), then
// [8](acc - R) == O.  Each signature occupies one quad.
__global__ void __launch_bounds__(kQuadBlock)
k_ed25519_verify_quad(const uint8_t *__restrict__ sig, Ed25519Work w, const fe *__restrict__ btab_q, uint32_t n,
                      uint8_t *__restrict__ valid, int aligned) {
  __shared__ fe tabA[kQuadSigs * 8 * 4];
  __shared__ fe tabB[8 * 4];
  __shared__ int8_t dig[kQuadSigs][2][64];
  const int c = threadIdx.x & 3;
  const int q = threadIdx.x >> 2;
  const uint32_t raw = blockIdx.x * kQuadSigs + q;
  const bool live = raw < n;
  const uint32_t i = live ? raw : n - 1;
  for (int t = threadIdx.x; t < 32; t += kQuadBlock) tabB[t] = btab_q[t];

  uint32_t s_w[8];
  if (aligned) load_words_aligned(s_w, sig + 64ull * i + 32);
  else load_words_unaligned(s_w, sig + 64ull * i + 32);
  const bool s_ok = sc_is_canonical(s_w);
  {
    uint32_t k_w[8];
    const uint4 *kp = reinterpret_cast<const uint4 *>(w.k + 8ull * i);
    const uint4 k0 = kp[0], k1 = kp[1];
    k_w[0] = k0.x; k_w[1] = k0.y; k_w[2] = k0.z; k_w[3] = k0.w;
    k_w[4] = k1.x; k_w[5] = k1.y; k_w[6] = k1.z; k_w[7] = k1.w;
    uint32_t sc[8];
#pragma unroll
    for (int t = 0; t < 8; t++) sc[t] = (c & 1) ? s_w[t] : k_w[t];
    recode16_store(&dig[q][c & 1][0], sc, c < 2);
  }
  const bool dec_ok = w.flags[2 * i] && w.flags[2 * i + 1];

  // table of (m+1)(-A), m < 8, in CachedQ layout
  fe P = w.negA[4ull * i + c];
  fe r, Pm, Q, Q0;
  quad::to_cached(Q0, P);
  tabA[(q * 8 + 0) * 4 + c] = Q0;
  quad::dbl(r, P);
  quad::p1p1_to_p3(Pm, r);
  quad::to_cached(Q, Pm);
  tabA[(q * 8 + 1) * 4 + c] = Q;
  for (int m = 2; m < 8; m++) {
    quad::add(r, Pm, Q0);
    quad::p1p1_to_p3(Pm, r);
    quad::to_cached(Q, Pm);
    tabA[(q * 8 + m) * 4 + c] = Q;
  }
  __syncthreads();

  fe acc;
  quad::p3_identity(acc);
  for (int wdx = 63; wdx >= 0; wdx--) {
    if (wdx != 63) {
#pragma unroll
      for (int d = 0; d < 4; d++) {
        quad::dbl(r, acc);
        quad::p1p1_to_p3(acc, r);
      }
    }
    const int da = dig[q][0][wdx];
    const int db = dig[q][1][wdx];
    fe e, idq;
    quad::cached_identity(idq);
    const int aa = da < 0 ? -da : da;
    e = tabA[(q * 8 + (aa ? aa - 1 : 0)) * 4 + c];
    fe_cmov(e, idq, aa == 0);
    quad::cached_cneg(e, da < 0);
    quad::add(r, acc, e);
    quad::p1p1_to_p3(acc, r);
    const int ab = db < 0 ? -db : db;
    e = tabB[(ab ? ab - 1 : 0) * 4 + c];
    fe_cmov(e, idq, ab == 0);
    quad::cached_cneg(e, db < 0);
    quad::add(r, acc, e);
    quad::p1p1_to_p3(acc, r);
  }
  fe Rq = w.Rc[4ull * i + c];
  quad::cached_cneg(Rq, true);
  quad::add(r, acc, Rq);
  quad::p1p1_to_p3(acc, r);
  const bool ok = quad::is_identity_times8(acc) && s_ok && dec_ok;
  if (live && c == 0) valid[i] = ok ? 1 : 0;
}

hipError_t launch_ed25519_verify_quad(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                      const uint32_t *msg_off, uint32_t n, const fe *btab_q, Ed25519Work w,
                                      uint8_t *valid, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  const uint32_t pblocks = (3 * n + kVerifyBlock - 1) / kVerifyBlock;
  hipLaunchKernelGGL(k_ed25519_prep, dim3(pblocks), dim3(kVerifyBlock), 0, stream, pk, sig, msg, msg_off, n, w,
                     aligned);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t qblocks = (n + kQuadSigs - 1) / kQuadSigs;
  hipLaunchKernelGGL(k_ed25519_verify_quad, dim3(qblocks), dim3(kQuadBlock), 0, stream, sig, w, btab_q, n, valid,
                     aligned);
  return hipGetLastError();
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
