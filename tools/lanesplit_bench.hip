// Microbenchmark: does a field multiply split over a
// lane pair shorten the one-wave chains (k_msm_horner, the per-entry check)?
//
// The quad formulas (quad.h) give each lane one squaring + one multiply per
// doubling.  Eight lanes per point would give each coordinate a lane pair.
// Squarings cannot be split without losing their symmetry (55 products), so a
// pair squares redundantly (both lanes hold the whole coordinate), and only
// the multiply is split: lane L of the pair computes the columns of parity L
// (5 columns x 10 products) from lane-dependent operand tables --
//   F_L[i] = f_i << (L == 0 && i odd)     (the radix-2^25.5 factor 2)
//   G_L[m] = g_(m+L), or 19 g_(m+L+10) where m + L < 0 (the wrap)
// so both lanes run one instruction stream; the two-round carry hands each
// column's quotient to the partner lane by DPP, and the limbs are broadcast
// back so both lanes hold the product.
//
// Two dependent chains, K iterations of (h = f^2; f = h g):
//   one:  one lane per chain (fe_sq + fe_mul, the quad formulas' per-lane work)
//   pair: a lane pair per chain (fe_sq on both lanes + the split multiply)
// at 1 wave per SIMD (the per-entry fallback of a 125k launch) and at 1/8
// (Horner).  Prints one JSON line: ns per iteration of each, their ratio, and
// whether the two chains end on the same field element for every chain.
//
//   hipcc -O3 --offload-arch=gfx950 -I tendermint_amd/csrc tools/lanesplit_bench.hip -o lanesplit_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "curve25519.h"

using namespace tmv;

namespace {

template <int CTRL>
__device__ __forceinline__ int32_t dpp32(int32_t x) { return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true); }
__device__ __forceinline__ int64_t dpp64(int64_t x) {
  const int32_t lo = dpp32<0xB1>((int32_t)(uint32_t)x), hi = dpp32<0xB1>((int32_t)(x >> 32));  // quad_perm [1,0,3,2]
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// h = f g on a lane pair; f, g whole on both lanes, h whole on both lanes.
__device__ __forceinline__ void mul_pair(fe &h, const fe &f, const fe &g) {
  const int L = (int)(threadIdx.x & 1);
  int32_t F[10], g19[10], G0[19], G[18];
#pragma unroll
  for (int i = 0; i < 10; i++) F[i] = (i & 1) ? (f.v[i] << (1 - L)) : f.v[i];
#pragma unroll
  for (int j = 1; j < 10; j++) g19[j] = mul19(g.v[j]);
#pragma unroll
  for (int m = -9; m <= 9; m++) G0[m + 9] = m >= 0 ? g.v[m] : g19[m + 10];
#pragma unroll
  for (int m = -9; m <= 8; m++) G[m + 9] = L ? G0[m + 10] : G0[m + 9];
  int64_t bias = L ? ((int64_t)1 << 24) : ((int64_t)1 << 25);
  asm("" : "+v"(bias));
  const int sh = L ? 25 : 26;
  int64_t c[5];
#pragma unroll
  for (int s = 0; s < 5; s++) {
    c[s] = mad_acc(F[0], G[2 * s + 9], bias);
#pragma unroll
    for (int i = 1; i < 10; i++) c[s] = mad_acc(F[i], G[2 * s - i + 9], c[s]);
  }
  // round 1: quotients to the next column (lane 0's column 2s takes lane 1's
  // 2s - 1, or 19 x column 9's; lane 1's 2s + 1 takes lane 0's 2s)
  int64_t k[5], snd[5];
#pragma unroll
  for (int s = 0; s < 5; s++) {
    k[s] = c[s] >> sh;
    c[s] -= k[s] * ((int64_t)1 << sh);
  }
  const int64_t k19 = k[4] * 19;
#pragma unroll
  for (int s = 0; s < 5; s++) snd[s] = L ? (s ? k[s - 1] : k19) : k[s];
#pragma unroll
  for (int s = 0; s < 5; s++) c[s] += dpp64(snd[s]);
  // round 2: the small quotients, the same hand-off on 32-bit values
  int32_t q[5], snd2[5], own[5];
#pragma unroll
  for (int s = 0; s < 5; s++) {
    q[s] = (int32_t)(c[s] >> sh);
    c[s] -= (int64_t)q[s] * ((int64_t)1 << sh);
  }
  const int32_t q19 = mul19(q[4]);
#pragma unroll
  for (int s = 0; s < 5; s++) snd2[s] = L ? (s ? q[s - 1] : q19) : q[s];
#pragma unroll
  for (int s = 0; s < 5; s++) own[s] = (int32_t)(c[s] - bias) + dpp32<0xB1>(snd2[s]);
  // both lanes take the whole product: even limbs from lane 0, odd from lane 1
#pragma unroll
  for (int s = 0; s < 5; s++) {
    h.v[2 * s] = dpp32<0xA0>(own[s]);      // quad_perm [0,0,2,2]
    h.v[2 * s + 1] = dpp32<0xF5>(own[s]);  // quad_perm [1,1,3,3]
  }
}

__device__ __forceinline__ void load_fe(fe &f, const int32_t *p) {
#pragma unroll
  for (int i = 0; i < 10; i++) f.v[i] = p[i];
}

template <bool PAIR>
__global__ void __launch_bounds__(64) k_chain(const int32_t *in_f, const int32_t *in_g, uint32_t *out, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t chain = PAIR ? t >> 1 : t;  // the pair kernel: one chain per lane pair
  fe f, g, h;
  load_fe(f, in_f + 10 * chain);
  load_fe(g, in_g + 10 * chain);
  for (int it = 0; it < iters; it++) {
    fe_sq(h, f);
    if (PAIR) mul_pair(f, h, g);
    else fe_mul(f, h, g);
  }
  uint32_t w[8];
  fe_to_words(w, f);
#pragma unroll
  for (int i = 0; i < 8; i++) out[8ull * t + i] = w[i];
}

}  // namespace

int main() {
  const int iters = 2000;
  const int sizes[2] = {1024, 128};  // blocks of one wave: 1 per SIMD, 1 per 8 SIMDs
  const int maxb = 1024, lanes = maxb * 64;
  std::vector<int32_t> hf(10ull * lanes), hg(10ull * lanes);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  for (size_t i = 0; i < hf.size(); i++) {
    const int bits = (i % 10) & 1 ? 24 : 25;  // level-1 limbs
    hf[i] = (int32_t)(rnd() % (2ull << bits)) - (1 << bits);
    hg[i] = (int32_t)(rnd() % (2ull << bits)) - (1 << bits);
  }
  int32_t *df, *dg;
  uint32_t *o1, *o2;
  hipMalloc(&df, hf.size() * 4);
  hipMalloc(&dg, hg.size() * 4);
  hipMalloc(&o1, 8ull * lanes * 4);
  hipMalloc(&o2, 8ull * lanes * 4);
  hipMemcpy(df, hf.data(), hf.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dg, hg.data(), hg.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("{");
  for (int si = 0; si < 2; si++) {
    const int blocks = sizes[si];
    float ms[2] = {0, 0};
    for (int rep = 0; rep < 4; rep++) {
      for (int v = 0; v < 2; v++) {
        hipEventRecord(e0, 0);
        if (v == 0) hipLaunchKernelGGL(k_chain<false>, dim3(blocks), dim3(64), 0, 0, df, dg, o1, iters);
        else hipLaunchKernelGGL(k_chain<true>, dim3(blocks), dim3(64), 0, 0, df, dg, o2, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float t;
        hipEventElapsedTime(&t, e0, e1);
        if (rep > 0) ms[v] += t / 3;
      }
    }
    // chain p of the pair kernel (lanes 2p, 2p+1) against chain p of the one-lane kernel (lane p)
    std::vector<uint32_t> r1(8ull * blocks * 64), r2(8ull * blocks * 64);
    hipMemcpy(r1.data(), o1, r1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r2.data(), o2, r2.size() * 4, hipMemcpyDeviceToHost);
    bool same = true;
    for (int t = 0; t < blocks * 64; t++)
      for (int i = 0; i < 8; i++) same = same && r2[8ull * t + i] == r1[8ull * (t >> 1) + i];
    printf("%s\"waves_%d\": {\"one_lane_ns_per_iter\": %.2f, \"lane_pair_ns_per_iter\": %.2f, \"ratio\": %.3f, "
           "\"same_result\": %s}",
           si ? ", " : "", blocks, ms[0] * 1e6 / iters, ms[1] * 1e6 / iters, ms[1] / ms[0], same ? "true" : "false");
  }
  printf(", \"iters\": %d, \"note\": \"per iteration: one squaring + one multiply (a quad doubling's per-lane work); "
         "lane_pair: the multiply split over two lanes\"}\n", iters);
  return 0;
}
