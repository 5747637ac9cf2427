// Comb helpers shared by the key-cached kernels (verify_kernels.hip) and the
// key-merged batch equation (msm_kernels.hip): scalar recodings written to
// LDS and the prefetching table-addition loop.
#pragma once
#include "quad.h"

namespace tmv {

// Signed radix-16 recoding written straight to LDS (lanes with store = false skip).
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

// Signed radix-16 recoding into ND digits, the top one absorbing the carry
// (a value below 2^(4 ND - 1) gives a top digit <= 8)
template <int ND>
__device__ __forceinline__ void recode16_n(int8_t *dst, const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int i = 0; i < ND; i++) {
    int e = (int)((s[i >> 3] >> (4 * (i & 7))) & 15) + carry;
    if (i < ND - 1) {
      carry = (e + 8) >> 4;
      e -= carry * 16;
    }
    dst[i] = (int8_t)e;
  }
}

// Signed radix-256 recoding (32 digits in [-128, 127], top digit absorbs the
// carry) for the fixed base B, written to LDS.
__device__ __forceinline__ void recode256_store(int8_t *dst, const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    int e = (int)((s[i >> 2] >> (8 * (i & 3))) & 255) + carry;
    if (i < 31) {
      carry = (e + 128) >> 8;
      e -= carry * 256;
    }
    dst[i] = (int8_t)e;
  }
}

// N table additions (quad-lane, CachedQ entries) with kCombAhead entries in
// flight: the tables live in HBM / the Infinity Cache (a key is 80 KB), so
// one entry of prefetch left the loop waiting on memory latency.
// entry_at(t, digit) returns this lane's coordinate of entry t and its digit.
constexpr int kCombAhead = 8;

template <int N, class EntryAt>
__device__ __forceinline__ void comb_accumulate(fe &acc, const fe &idq, EntryAt entry_at) {
  static_assert(N % kCombAhead == 0, "comb length must be a multiple of the prefetch depth");
  // named registers, not an array, so the ring stays out of scratch
  fe b0, b1, b2, b3, b4, b5, b6, b7;
  int d0, d1, d2, d3, d4, d5, d6, d7;
  b0 = *entry_at(0, d0); b1 = *entry_at(1, d1); b2 = *entry_at(2, d2); b3 = *entry_at(3, d3);
  b4 = *entry_at(4, d4); b5 = *entry_at(5, d5); b6 = *entry_at(6, d6); b7 = *entry_at(7, d7);
  fe r;
  auto step = [&](fe &b, int &d, int next) {
    fe ent = b;
    const int dd = d;
    if (next < N) b = *entry_at(next, d);
    fe_cmov(ent, idq, dd == 0);
    quad::cached_cneg(ent, dd < 0);
    quad::add(r, acc, ent);
    quad::p1p1_to_p3(acc, r);
  };
  for (int t0 = 0; t0 < N; t0 += kCombAhead) {
    step(b0, d0, t0 + 8); step(b1, d1, t0 + 9); step(b2, d2, t0 + 10); step(b3, d3, t0 + 11);
    step(b4, d4, t0 + 12); step(b5, d5, t0 + 13); step(b6, d6, t0 + 14); step(b7, d7, t0 + 15);
  }
}

}  // namespace tmv
