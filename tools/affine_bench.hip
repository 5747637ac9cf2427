// Microbenchmark: batch-affine bucket additions against
// the accumulation's mixed addition.  k_msm_accum adds each bucket entry with
// ge_madd (extended + affine Niels point: 7 field multiplications, ~1,400
// VALU instructions).  The CPU literature's alternative is the affine
// addition on a Montgomery / short-Weierstrass model -- lambda = dv / du,
// u3 = lambda^2 - A - u1 - u2, v3 = lambda (u1 - u3) - v1: 2M + 1S + one
// inversion -- with the inversions of many independent additions shared by
// Montgomery's trick (3M per element + one inversion per batch).  On a GPU
// the batch must be independent bucket chains held by the lanes of a wave:
// each lane keeps K affine accumulators, the K denominators' product is
// formed in the lane, the lanes' products are scanned across the wave
// (inclusive prefix and suffix, 6 shuffle levels each), every lane computes
// the one inversion of the wave's product (SIMT: the chain costs every lane
// its full instruction stream), then each lane walks its K elements back.
// The exceptional denominators (u1 == u2: a doubling, P + (-P), a
// small-order point) are detected and replaced by 1 so the product stays
// invertible (a real kernel would then redo those entries on a slow path;
// the check is counted, the slow path is not).
//
// Both kernels run chip-wide (4096 x 256 threads) on random field elements
// from a 4,096-entry table in L2, as the accumulation gathers its points;
// the birational map of every input point to the Montgomery model (one more
// batched inversion per point) is NOT charged to the affine side.  Prints
// one JSON line: ns per addition chip-wide for ge_madd and for batch-affine
// with K = 4 / 8 / 16 accumulators per lane, the ratios, and the registers /
// scratch of each kernel come from `-Rpass-analysis=kernel-resource-usage`.
// The host check compares one wave's affine round against a host
// restatement (the same fe functions compiled for the host).
//
//   hipcc -O3 --offload-arch=gfx950 -I tendermint_amd/csrc tools/affine_bench.hip -o tools/affine_bench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#include "curve25519.h"

using namespace tmv;

namespace {

constexpr int kTable = 4096;
constexpr int32_t kMontA = 486662;

__host__ __device__ inline uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// ---------------------------------------------------------------- ge_madd
__global__ void __launch_bounds__(256) k_madd(const ge_precomp *__restrict__ tab, ge_p3 *out, int rounds) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  ge_p3 acc;
  const ge_precomp &q0 = tab[mix(t) & (kTable - 1)];
  fe_sub(acc.X, q0.ypx, q0.ymx);
  fe_add(acc.Y, q0.ypx, q0.ymx);
  fe_one(acc.Z);
  fe_mul(acc.T, acc.X, acc.Y);
#pragma unroll 1
  for (int r = 0; r < rounds; r++) {
    const ge_precomp q = tab[mix(t * 977u + (uint32_t)r) & (kTable - 1)];
    ge_p1p1 p;
    ge_madd(p, acc, q);
    ge_p1p1_to_p3(acc, p);
  }
  out[t] = acc;
}

// ---------------------------------------------------------- batch affine
__device__ inline void fe_shfl_up(fe &h, const fe &f, int d) {
#pragma unroll
  for (int k = 0; k < 10; k++) h.v[k] = __shfl_up(f.v[k], d, 64);
}
__device__ inline void fe_shfl_down(fe &h, const fe &f, int d) {
#pragma unroll
  for (int k = 0; k < 10; k++) h.v[k] = __shfl_down(f.v[k], d, 64);
}
__device__ inline void fe_shfl(fe &h, const fe &f, int lane) {
#pragma unroll
  for (int k = 0; k < 10; k++) h.v[k] = __shfl(f.v[k], lane, 64);
}

// lam = dv / du for one element given its inverse; accumulator <- acc + P
__host__ __device__ inline void affine_finish(fe &u, fe &v, const fe &pu, const fe &pv, const fe &inv) {
  fe dv, lam, l2, t, u3, v3;
  fe_sub(dv, pv, v);
  fe_carry(dv, dv);
  fe_mul(lam, dv, inv);
  fe_sq(l2, lam);
  fe_add(t, u, pu);        // u1 + u2 (level 2)
  t.v[0] += kMontA;        // + A
  fe_sub(u3, l2, t);
  fe_carry(u3, u3);
  fe_sub(t, u, u3);
  fe_carry(t, t);
  fe_mul(v3, lam, t);
  fe_sub(v3, v3, v);
  fe_carry(v3, v3);
  u = u3;
  v = v3;
}

// register budget up to 2 waves per SIMD (256 VGPRs): the K accumulators and
// prefix products stay in registers (the default budget spilled them)
template <int K>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) k_affine(const fe *__restrict__ tab, fe *out, int rounds, uint32_t *exc) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  fe u[K], v[K], c[K];
#pragma unroll
  for (int j = 0; j < K; j++) {
    const uint32_t i = mix(t * 31u + (uint32_t)j + 0x9e3779b9u) & (kTable - 1);
    u[j] = tab[2 * i];
    v[j] = tab[2 * i + 1];
  }
  uint32_t nexc = 0;
#pragma unroll 1
  for (int r = 0; r < rounds; r++) {
    // denominators du_j = pu_j - u_j, their prefix products in the lane
#pragma unroll
    for (int j = 0; j < K; j++) {
      const uint32_t i = mix(t * 977u + (uint32_t)(r * K + j)) & (kTable - 1);
      fe du;
      fe_sub(du, tab[2 * i], u[j]);
      fe_carry(du, du);
      const bool z = fe_is_zero(du);  // exceptional: doubling / P + (-P) / small order
      nexc += z;
      fe one;
      fe_one(one);
      fe_cmov(du, one, z);
      if (j == 0) c[0] = du;
      else fe_mul(c[j], c[j - 1], du);
    }
    // the lanes' products: inclusive prefix and suffix scans over the wave
    fe pre = c[K - 1], suf = c[K - 1], o;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      fe_shfl_up(o, pre, d);
      if (lane >= d) fe_mul(pre, pre, o);
      fe_shfl_down(o, suf, d);
      if (lane + d < 64) fe_mul(suf, suf, o);
    }
    fe total, inv;
    fe_shfl(total, pre, 63);
    fe_invert(inv, total);  // every lane: one inversion per wave and round
    // the inverse of this lane's product: inv * (prefix before it) * (suffix after it)
    fe before, after, one;
    fe_one(one);
    fe_shfl_up(before, pre, 1);
    fe_shfl_down(after, suf, 1);
    if (lane == 0) before = one;
    if (lane == 63) after = one;
    fe_mul(inv, inv, before);
    fe_mul(inv, inv, after);
    // back through the lane's elements: 1 / du_j = inv * c_(j-1), inv *= du_j
#pragma unroll
    for (int j = K - 1; j >= 0; j--) {
      const uint32_t i = mix(t * 977u + (uint32_t)(r * K + j)) & (kTable - 1);
      const fe pu = tab[2 * i], pv = tab[2 * i + 1];
      fe inv_j;
      if (j > 0) {
        fe_mul(inv_j, inv, c[j - 1]);
        fe du;
        fe_sub(du, pu, u[j]);
        fe_carry(du, du);
        fe_cmov(du, one, fe_is_zero(du));
        fe_mul(inv, inv, du);
      } else {
        inv_j = inv;
      }
      affine_finish(u[j], v[j], pu, pv, inv_j);
    }
  }
  fe acc = u[0];
#pragma unroll
  for (int j = 1; j < K; j++) fe_add(acc, acc, u[j]);
  out[t] = acc;
  if (nexc) atomicAdd(exc, nexc);
}

// host restatement of one lane's first round for K = 4 (lane products scanned
// in order): the affine sums of (u_j, v_j) + (pu_j, pv_j) with direct inversions
int host_check(const std::vector<fe> &tab, const std::vector<fe> &dev_u0) {
  (void)dev_u0;
  int bad = 0;
  for (uint32_t t = 0; t < 64; t++) {
    for (int j = 0; j < 4; j++) {
      const uint32_t i0 = mix(t * 31u + (uint32_t)j + 0x9e3779b9u) & (kTable - 1), i1 = mix(t * 977u + (uint32_t)j) & (kTable - 1);
      fe u = tab[2 * i0], v = tab[2 * i0 + 1], du, inv;
      fe_sub(du, tab[2 * i1], u);
      fe_carry(du, du);
      fe_invert(inv, du);
      fe u_ref = u, v_ref = v;
      affine_finish(u_ref, v_ref, tab[2 * i1], tab[2 * i1 + 1], inv);
      // lambda (u2 - u1) == v2 - v1 after the step (the defining relation)
      fe dv, lam, chk;
      fe_sub(dv, tab[2 * i1 + 1], v);
      fe_carry(dv, dv);
      fe_mul(lam, dv, inv);
      fe_mul(chk, lam, du);
      bad += !fe_eq(chk, dv);
    }
  }
  return bad;
}

}  // namespace

// device check: one wave, one round of k_affine<4> against the host's direct inversions
__global__ void k_affine_check(const fe *__restrict__ tab, fe *out_u, fe *out_v) {
  const int lane = threadIdx.x;
  constexpr int K = 4;
  fe u[K], v[K], c[K], one;
  fe_one(one);
  for (int j = 0; j < K; j++) {
    const uint32_t i = mix((uint32_t)lane * 31u + (uint32_t)j + 0x9e3779b9u) & (kTable - 1);
    u[j] = tab[2 * i];
    v[j] = tab[2 * i + 1];
  }
  for (int j = 0; j < K; j++) {
    const uint32_t i = mix((uint32_t)lane * 977u + (uint32_t)j) & (kTable - 1);
    fe du;
    fe_sub(du, tab[2 * i], u[j]);
    fe_carry(du, du);
    if (j == 0) c[0] = du;
    else fe_mul(c[j], c[j - 1], du);
  }
  fe pre = c[K - 1], suf = c[K - 1], o;
  for (int d = 1; d < 64; d <<= 1) {
    fe_shfl_up(o, pre, d);
    if (lane >= d) fe_mul(pre, pre, o);
    fe_shfl_down(o, suf, d);
    if (lane + d < 64) fe_mul(suf, suf, o);
  }
  fe total, inv, before, after;
  fe_shfl(total, pre, 63);
  fe_invert(inv, total);
  fe_shfl_up(before, pre, 1);
  fe_shfl_down(after, suf, 1);
  if (lane == 0) before = one;
  if (lane == 63) after = one;
  fe_mul(inv, inv, before);
  fe_mul(inv, inv, after);
  for (int j = K - 1; j >= 0; j--) {
    const uint32_t i = mix((uint32_t)lane * 977u + (uint32_t)j) & (kTable - 1);
    fe inv_j;
    if (j > 0) {
      fe_mul(inv_j, inv, c[j - 1]);
      fe du;
      fe_sub(du, tab[2 * i], u[j]);
      fe_carry(du, du);
      fe_mul(inv, inv, du);
    } else {
      inv_j = inv;
    }
    affine_finish(u[j], v[j], tab[2 * i], tab[2 * i + 1], inv_j);
    out_u[lane * K + j] = u[j];
    out_v[lane * K + j] = v[j];
  }
}

int main() {
  // random field elements (reduced), as (u, v) pairs and as Niels triples
  std::vector<fe> tab(2 * kTable);
  std::vector<ge_precomp> ntab(kTable);
  uint64_t x = 0x243f6a8885a308d3ull;
  auto rnd = [&]() {
    uint32_t w[8];
    for (int k = 0; k < 8; k++) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      w[k] = (uint32_t)x;
    }
    w[7] &= 0x7fffffffu;
    fe f;
    fe_from_words(f, w);
    return f;
  };
  for (int i = 0; i < 2 * kTable; i++) tab[i] = rnd();
  for (int i = 0; i < kTable; i++) ntab[i] = ge_precomp{rnd(), rnd(), rnd()};
  fe *dtab;
  ge_precomp *dntab;
  hipMalloc(&dtab, tab.size() * sizeof(fe));
  hipMalloc(&dntab, ntab.size() * sizeof(ge_precomp));
  hipMemcpy(dtab, tab.data(), tab.size() * sizeof(fe), hipMemcpyHostToDevice);
  hipMemcpy(dntab, ntab.data(), ntab.size() * sizeof(ge_precomp), hipMemcpyHostToDevice);

  // correctness: one wave's round against direct inversions on the host
  fe *du_, *dv_;
  hipMalloc(&du_, 256 * sizeof(fe));
  hipMalloc(&dv_, 256 * sizeof(fe));
  hipLaunchKernelGGL(k_affine_check, dim3(1), dim3(64), 0, 0, dtab, du_, dv_);
  std::vector<fe> gu(256), gv(256);
  hipMemcpy(gu.data(), du_, 256 * sizeof(fe), hipMemcpyDeviceToHost);
  hipMemcpy(gv.data(), dv_, 256 * sizeof(fe), hipMemcpyDeviceToHost);
  int mism = 0;
  for (uint32_t lane = 0; lane < 64; lane++)
    for (int j = 0; j < 4; j++) {
      const uint32_t i0 = mix(lane * 31u + (uint32_t)j + 0x9e3779b9u) & (kTable - 1), i1 = mix(lane * 977u + (uint32_t)j) & (kTable - 1);
      fe u = tab[2 * i0], v = tab[2 * i0 + 1], du, inv;
      fe_sub(du, tab[2 * i1], u);
      fe_carry(du, du);
      fe_invert(inv, du);
      affine_finish(u, v, tab[2 * i1], tab[2 * i1 + 1], inv);
      mism += !fe_eq(u, gu[lane * 4 + j]) || !fe_eq(v, gv[lane * 4 + j]);
    }
  const int host_bad = host_check(tab, gu);

  const int blocks = 4096, threads = blocks * 256;
  ge_p3 *o1;
  fe *o2;
  uint32_t *exc;
  hipMalloc(&o1, (size_t)threads * sizeof(ge_p3));
  hipMalloc(&o2, (size_t)threads * sizeof(fe));
  hipMalloc(&exc, 4);
  hipMemset(exc, 0, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int madd_rounds = 64;
  const int aff_adds = 64;  // additions per lane for every K
  double ns[4] = {0, 0, 0, 0};
  for (int rep = 0; rep < 4; rep++) {
    for (int v = 0; v < 4; v++) {
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL(k_madd, dim3(blocks), dim3(256), 0, 0, dntab, o1, madd_rounds);
      if (v == 1) hipLaunchKernelGGL(k_affine<4>, dim3(blocks), dim3(256), 0, 0, dtab, o2, aff_adds / 4, exc);
      if (v == 2) hipLaunchKernelGGL(k_affine<8>, dim3(blocks), dim3(256), 0, 0, dtab, o2, aff_adds / 8, exc);
      if (v == 3) hipLaunchKernelGGL(k_affine<16>, dim3(blocks), dim3(256), 0, 0, dtab, o2, aff_adds / 16, exc);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      const double adds = (double)threads * (v == 0 ? madd_rounds : aff_adds);
      if (rep) ns[v] += t * 1e6 / adds / 3;
    }
  }
  uint32_t nexc = 0;
  hipMemcpy(&nexc, exc, 4, hipMemcpyDeviceToHost);
  const hipError_t err = hipGetLastError();
  printf("{\"ns_per_add_chipwide\": {\"ge_madd\": %.5f, \"affine_k4\": %.5f, \"affine_k8\": %.5f, "
         "\"affine_k16\": %.5f}, \"ratio_vs_madd\": {\"k4\": %.3f, \"k8\": %.3f, \"k16\": %.3f}, "
         "\"device_round_vs_host_mismatches\": %d, \"host_relation_failures\": %d, \"exceptional_denominators\": %u, "
         "\"hip_error\": \"%s\"}\n",
         ns[0], ns[1], ns[2], ns[3], ns[1] / ns[0], ns[2] / ns[0], ns[3] / ns[0], mism, host_bad, nexc,
         hipGetErrorString(err));
  return 0;
}
