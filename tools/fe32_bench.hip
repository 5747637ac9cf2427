// Microbenchmark: field multiply in eight 32-bit words (radix 2^32, value <
// 2^256, 64 v_mad_u64_u32 column products with the carry out of bit 64
// counted, 8 more for the 2^256 == 38 fold) against the radix-2^25.5 fe_mul
// (100 v_mad_i64_i32), in throughput (many waves per SIMD).  The throughput
// kernels are bound by the multiply-adds (k_msm_accum issues them at ~0.9 of
// the measured peak with ~0.8 other VALU instructions per multiply-add
// alongside); this asks whether 28% fewer multiply-adds pay for ~2x the
// other instructions.  Prints one JSON line: ns per multiply chip-wide for
// each, their ratio, and whether both chains end on the same field element.
//
//   hipcc -O3 --offload-arch=gfx950 -I tendermint_amd/csrc tools/fe32_bench.hip -o tools/fe32_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "curve25519.h"

using namespace tmv;

namespace {

struct fe32 {
  uint32_t w[8];
};

// acc = a b + acc; the carry out of bit 64 is added to ovf
#ifndef FE32_ASM
#define FE32_ASM 1
#endif
#if !FE32_ASM || !defined(__HIP_DEVICE_COMPILE__)
__host__ __device__ __forceinline__ void mad_ovf(uint64_t &acc, uint32_t &ovf, uint32_t a, uint32_t b) {
  const uint64_t r = acc + (uint64_t)a * b;
  ovf += r < acc;
  acc = r;
}
__host__ __device__ __forceinline__ void mad_ovf0(uint64_t &acc, uint32_t &ovf, uint32_t a, uint32_t b) {
  const uint64_t r = acc + (uint64_t)a * b;
  ovf = r < acc;
  acc = r;
}
#else
__device__ __forceinline__ void mad_ovf(uint64_t &acc, uint32_t &ovf, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32_e64 %1, %2, %1, 0, %2"
      : "+v"(acc), "+v"(ovf), "=&s"(cc)
      : "v"(a), "v"(b));
}
// the same for a column's second product: ovf starts at the carry
__device__ __forceinline__ void mad_ovf0(uint64_t &acc, uint32_t &ovf, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32_e64 %1, %2, 0, 0, %2"
      : "+v"(acc), "=v"(ovf), "=&s"(cc)
      : "v"(a), "v"(b));
}
#endif

// h = f g mod 2^255 - 19, any inputs < 2^256, result < 2^256
__host__ __device__ __forceinline__ void fe32_mul(fe32 &h, const fe32 &f, const fe32 &g) {
  uint64_t acc[15];
  uint32_t ovf[15];
#pragma unroll
  for (int k = 0; k < 15; k++) {
    const int i0 = k < 8 ? 0 : k - 7;
    acc[k] = (uint64_t)f.w[i0] * g.w[k - i0];
    ovf[k] = 0;  // (columns 0 and 14: one product)
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int k = i + j, i0 = k < 8 ? 0 : k - 7;
      if (i == i0 + 1) mad_ovf0(acc[k], ovf[k], f.w[i], g.w[j]);
      else if (i > i0 + 1) mad_ovf(acc[k], ovf[k], f.w[i], g.w[j]);
    }
  }
  uint32_t r[16];
  r[0] = (uint32_t)acc[0];
  uint32_t clo = (uint32_t)(acc[0] >> 32), chi = 0;  // carry into column k: chi:clo
#pragma unroll
  for (int k = 1; k < 15; k++) {
    unsigned c;
    r[k] = __builtin_addc((uint32_t)acc[k], clo, 0u, &c);
    clo = __builtin_addc((uint32_t)(acc[k] >> 32), chi, c, &c);
    chi = ovf[k] + c;
  }
  r[15] = clo;
  // fold: r_lo + 38 r_hi
  uint64_t cc = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t s = (uint64_t)r[8 + j] * 38u + r[j] + cc;
    h.w[j] = (uint32_t)s;
    cc = s >> 32;
  }
  unsigned c1;
  h.w[0] = __builtin_addc(h.w[0], (uint32_t)cc * 38u, 0u, &c1);
#pragma unroll
  for (int j = 1; j < 8; j++) h.w[j] = __builtin_addc(h.w[j], 0u, c1, &c1);
  h.w[0] += 38u * c1;  // wrapped: h < 2^12 now, no further carry
}

__host__ __device__ __forceinline__ void fe32_to_words(uint32_t out[8], const fe32 &h) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = h.w[i];
  const uint32_t top = w[7] >> 31;
  w[7] &= 0x7fffffffu;
  fe f;
  fe_from_words(f, w);
  f.v[0] += 19 * (int32_t)top;
  fe_to_words(out, f);
}

__host__ __device__ __forceinline__ void fe32_add(fe32 &h, const fe32 &f, const fe32 &g) {
  unsigned c;
  h.w[0] = __builtin_addc(f.w[0], g.w[0], 0u, &c);
#pragma unroll
  for (int j = 1; j < 8; j++) h.w[j] = __builtin_addc(f.w[j], g.w[j], c, &c);
  h.w[0] = __builtin_addc(h.w[0], 38u * c, 0u, &c);  // 2^256 == 38
#pragma unroll
  for (int j = 1; j < 8; j++) h.w[j] = __builtin_addc(h.w[j], 0u, c, &c);
  h.w[0] += 38u * c;
}

__host__ __device__ __forceinline__ void fe32_sub(fe32 &h, const fe32 &f, const fe32 &g) {
  unsigned b;
  h.w[0] = __builtin_subc(f.w[0], g.w[0], 0u, &b);
#pragma unroll
  for (int j = 1; j < 8; j++) h.w[j] = __builtin_subc(f.w[j], g.w[j], b, &b);
  h.w[0] = __builtin_subc(h.w[0], 38u * b, 0u, &b);  // wrapped by 2^256 == 38
#pragma unroll
  for (int j = 1; j < 8; j++) h.w[j] = __builtin_subc(h.w[j], 0u, b, &b);
  h.w[0] -= 38u * b;
}

struct p3_32 {
  fe32 X, Y, Z, T;
};
struct niels32 {
  fe32 ypx, ymx, xy2d;
};

// p += q (q affine Niels), the accumulation step of k_msm_accum
__host__ __device__ __forceinline__ void madd32(p3_32 &p, const niels32 &q) {
  fe32 a, b, c, dd, t, E, F, G, H;
  fe32_sub(t, p.Y, p.X);
  fe32_mul(a, t, q.ymx);
  fe32_add(t, p.Y, p.X);
  fe32_mul(b, t, q.ypx);
  fe32_mul(c, p.T, q.xy2d);
  fe32_add(dd, p.Z, p.Z);
  fe32_sub(E, b, a);
  fe32_add(H, b, a);
  fe32_add(G, dd, c);
  fe32_sub(F, dd, c);
  fe32_mul(p.X, E, F);
  fe32_mul(p.Y, H, G);
  fe32_mul(p.Z, G, F);
  fe32_mul(p.T, E, H);
}

__host__ __device__ __forceinline__ void load32(fe32 &f, const uint32_t *p) {
#pragma unroll
  for (int i = 0; i < 8; i++) f.w[i] = p[i];
}

// 16 Niels points per lane (7 x 8 words: ypx, ymx, xy2d; the words of
// arbitrary field elements: the formulas are identities mod p either way)
__global__ void __launch_bounds__(256) k_madd(const uint32_t *in, const fe *tab, uint32_t *out, int reps) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  ge_p3 p;
  fe_from_words(p.X, in + 32ull * t);
  fe_from_words(p.Y, in + 32ull * t + 8);
  fe_from_words(p.Z, in + 32ull * t + 16);
  fe_from_words(p.T, in + 32ull * t + 24);
  fe_carry(p.X, p.X); fe_carry(p.Y, p.Y); fe_carry(p.Z, p.Z); fe_carry(p.T, p.T);
  for (int r = 0; r < reps; r++) {
    const fe *q = tab + 3ull * ((t + r) & 4095);  // level 1, as k_msm_accum's points
    ge_precomp np;
    np.ypx = q[0];
    np.ymx = q[1];
    np.xy2d = q[2];
    ge_p1p1 s;
    ge_madd(s, p, np);
    ge_p1p1_to_p3(p, s);
  }
  fe_to_words(out + 32ull * t, p.X);
  fe_to_words(out + 32ull * t + 8, p.Y);
  fe_to_words(out + 32ull * t + 16, p.Z);
  fe_to_words(out + 32ull * t + 24, p.T);
}

__global__ void __launch_bounds__(256) k_madd32(const uint32_t *in, const uint32_t *tab, uint32_t *out, int reps) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  p3_32 p;
  load32(p.X, in + 32ull * t);
  load32(p.Y, in + 32ull * t + 8);
  load32(p.Z, in + 32ull * t + 16);
  load32(p.T, in + 32ull * t + 24);
  for (int r = 0; r < reps; r++) {
    const uint32_t *q = tab + 24ull * ((t + r) & 4095);
    niels32 np;
    load32(np.ypx, q);
    load32(np.ymx, q + 8);
    load32(np.xy2d, q + 16);
    madd32(p, np);
  }
  fe32_to_words(out + 32ull * t, p.X);
  fe32_to_words(out + 32ull * t + 8, p.Y);
  fe32_to_words(out + 32ull * t + 16, p.Z);
  fe32_to_words(out + 32ull * t + 24, p.T);
}

__global__ void __launch_bounds__(256) k_mul(const uint32_t *in, uint32_t *out, int reps) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe f, g;
  fe_from_words(f, in + 16ull * t);
  fe_from_words(g, in + 16ull * t + 8);
  for (int r = 0; r < reps; r++) fe_mul(f, f, g);
  fe_to_words(out + 8ull * t, f);
}

__global__ void __launch_bounds__(256) k_mul32(const uint32_t *in, uint32_t *out, int reps) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe32 f, g;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    f.w[i] = in[16ull * t + i];
    g.w[i] = in[16ull * t + 8 + i];
  }
  for (int r = 0; r < reps; r++) fe32_mul(f, f, g);
  fe32_to_words(out + 8ull * t, f);
}

}  // namespace

// host check of the word-radix formulas against ge_madd (both compiled for the host)
static size_t host_check() {
  uint64_t x = 0x0123456789abcdefull;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint32_t)x; };
  size_t bad = 0;
  {  // the primitives alone
    size_t bm = 0, ba = 0, bs = 0;
    for (int it = 0; it < 2000; it++) {
      uint32_t u[8], v[8], a[8], b[8];
      for (int i = 0; i < 8; i++) { u[i] = rnd() & (i == 7 ? 0x7fffffffu : ~0u); v[i] = rnd() & (i == 7 ? 0x7fffffffu : ~0u); }
      fe f, g, h;
      fe_from_words(f, u); fe_from_words(g, v);
      fe32 F, G, H;
      load32(F, u); load32(G, v);
      fe_mul(h, f, g); fe32_mul(H, F, G); fe_to_words(a, h); fe32_to_words(b, H);
      for (int i = 0; i < 8; i++) bm += a[i] != b[i];
      fe_add(h, f, g); fe32_add(H, F, G); fe_to_words(a, h); fe32_to_words(b, H);
      for (int i = 0; i < 8; i++) ba += a[i] != b[i];
      fe_sub(h, f, g); fe32_sub(H, F, G); fe_to_words(a, h); fe32_to_words(b, H);
      for (int i = 0; i < 8; i++) bs += a[i] != b[i];
    }
    printf("{\"mul\": %zu, \"add\": %zu, \"sub\": %zu}\n", bm, ba, bs);
  }
  for (int it = 0; it < 2000; it++) {
    uint32_t w[7][8];
    for (int a = 0; a < 7; a++)
      for (int i = 0; i < 8; i++) w[a][i] = rnd() & (i == 7 ? 0x7fffffffu : 0xffffffffu);
    ge_p3 p;
    ge_precomp q;
    fe_from_words(p.X, w[0]); fe_from_words(p.Y, w[1]); fe_from_words(p.Z, w[2]); fe_from_words(p.T, w[3]);
    fe_from_words(q.ypx, w[4]); fe_from_words(q.ymx, w[5]); fe_from_words(q.xy2d, w[6]);
    fe *all[7] = {&p.X, &p.Y, &p.Z, &p.T, &q.ypx, &q.ymx, &q.xy2d};
    for (fe *e : all) fe_carry(*e, *e);  // exact limbs are level 2: bring to 1 (ge_decode_zip215 does)
    p3_32 p2;
    niels32 q2;
    load32(p2.X, w[0]); load32(p2.Y, w[1]); load32(p2.Z, w[2]); load32(p2.T, w[3]);
    load32(q2.ypx, w[4]); load32(q2.ymx, w[5]); load32(q2.xy2d, w[6]);
    for (int r = 0; r < 3; r++) {
      ge_p1p1 s1;
      ge_madd(s1, p, q);
      ge_p1p1_to_p3(p, s1);
      madd32(p2, q2);
    }
    uint32_t a[8], b[8];
    const fe *fs[4] = {&p.X, &p.Y, &p.Z, &p.T};
    const fe32 *gs[4] = {&p2.X, &p2.Y, &p2.Z, &p2.T};
    for (int c = 0; c < 4; c++) {
      fe_to_words(a, *fs[c]);
      fe32_to_words(b, *gs[c]);
      for (int i = 0; i < 8; i++) bad += a[i] != b[i];
    }
  }
  return bad;
}

int main(int argc, char **argv) {
  if (argc > 1) {
    printf("{\"host_madd_words_differing\": %zu}\n", host_check());
    return 0;
  }
  const int blocks = 4096, threads = blocks * 256;
  std::vector<uint32_t> hin(16ull * threads);
  uint64_t x = 0x243f6a8885a308d3ull;
  for (size_t i = 0; i < hin.size(); i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    hin[i] = (uint32_t)x;
    if (i % 8 == 7) hin[i] &= 0x7fffffffu;  // < 2^255 (fe_from_words drops bit 255)
  }
  uint32_t *din, *o1, *o2;
  hipMalloc(&din, hin.size() * 4);
  hipMalloc(&o1, 8ull * threads * 4);
  hipMalloc(&o2, 8ull * threads * 4);
  hipMemcpy(din, hin.data(), hin.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 64;
  float ms[2] = {0, 0};
  for (int rep = 0; rep < 4; rep++) {
    for (int v = 0; v < 2; v++) {
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(256), 0, 0, din, o1, reps);
      else hipLaunchKernelGGL(k_mul32, dim3(blocks), dim3(256), 0, 0, din, o2, reps);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      if (rep) ms[v] += t / 3;
    }
  }
  // the same chains on one wave per SIMD (1024 one-wave blocks): latency-bound, as the
  // per-entry check and the Horner chain run
  const int lreps = 512;
  float lm[2] = {0, 0};
  for (int rep = 0; rep < 4; rep++) {
    for (int v = 0; v < 2; v++) {
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL(k_mul, dim3(1024), dim3(64), 0, 0, din, o1, lreps);
      else hipLaunchKernelGGL(k_mul32, dim3(1024), dim3(64), 0, 0, din, o2, lreps);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      if (rep) lm[v] += t / 3;
    }
  }
  hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(256), 0, 0, din, o1, reps);
  hipLaunchKernelGGL(k_mul32, dim3(blocks), dim3(256), 0, 0, din, o2, reps);
  std::vector<uint32_t> r1(8ull * threads), r2(8ull * threads);
  hipMemcpy(r1.data(), o1, r1.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(r2.data(), o2, r2.size() * 4, hipMemcpyDeviceToHost);
  size_t diff = 0;
  for (size_t i = 0; i < r1.size(); i++) diff += r1[i] != r2[i];
  const double n = (double)threads * reps;
  // the mixed addition: 32 words of point per lane, a 4096-entry Niels table
  std::vector<uint32_t> hp(32ull * threads), ht(24ull * 4096);
  for (size_t i = 0; i < hp.size(); i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    hp[i] = (uint32_t)x & (i % 8 == 7 ? 0x7fffffffu : 0xffffffffu);
  }
  for (size_t i = 0; i < ht.size(); i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    ht[i] = (uint32_t)x & (i % 8 == 7 ? 0x7fffffffu : 0xffffffffu);
  }
  std::vector<fe> hf(3ull * 4096);
  for (size_t i = 0; i < hf.size(); i++) {
    fe_from_words(hf[i], &ht[8 * i]);
    fe_carry(hf[i], hf[i]);
  }
  uint32_t *dp, *dt, *q1, *q2;
  fe *dtf;
  hipMalloc(&dp, hp.size() * 4);
  hipMalloc(&dt, ht.size() * 4);
  hipMalloc(&dtf, hf.size() * sizeof(fe));
  hipMemcpy(dtf, hf.data(), hf.size() * sizeof(fe), hipMemcpyHostToDevice);
  hipMalloc(&q1, hp.size() * 4);
  hipMalloc(&q2, hp.size() * 4);
  hipMemcpy(dp, hp.data(), hp.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dt, ht.data(), ht.size() * 4, hipMemcpyHostToDevice);
  const int areps = 32;
  float am[2] = {0, 0};
  for (int rep = 0; rep < 4; rep++) {
    for (int v = 0; v < 2; v++) {
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL(k_madd, dim3(blocks), dim3(256), 0, 0, dp, dtf, q1, areps);
      else hipLaunchKernelGGL(k_madd32, dim3(blocks), dim3(256), 0, 0, dp, dt, q2, areps);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      if (rep) am[v] += t / 3;
    }
  }
  std::vector<uint32_t> a1(hp.size()), a2(hp.size());
  hipMemcpy(a1.data(), q1, a1.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(a2.data(), q2, a2.size() * 4, hipMemcpyDeviceToHost);
  size_t adiff = 0;
  for (size_t i = 0; i < a1.size(); i++) adiff += a1[i] != a2[i];
  const double an = (double)threads * areps;
  printf("{\"fe_mul_ns_chip\": %.5f, \"fe32_mul_ns_chip\": %.5f, \"mul_ratio\": %.3f, \"mul_words_differing\": %zu, "
         "\"madd_ns_chip\": %.5f, \"madd32_ns_chip\": %.5f, \"madd_ratio\": %.3f, \"madd_words_differing\": %zu, "
         "\"lone_wave_fe_mul_ns\": %.2f, \"lone_wave_fe32_mul_ns\": %.2f, \"lone_wave_ratio\": %.3f, "
         "\"threads\": %d, \"reps\": %d, \"madd_reps\": %d}\n",
         ms[0] * 1e6 / n, ms[1] * 1e6 / n, ms[1] / ms[0], diff, am[0] * 1e6 / an, am[1] * 1e6 / an, am[1] / am[0],
         adiff, lm[0] * 1e6 / lreps, lm[1] * 1e6 / lreps, lm[1] / lm[0], threads, reps, areps);
  return 0;
}
