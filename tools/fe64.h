// GF(2^255-19) on the FP64 VALU: twelve double limbs in radix 2^21.25.
//
// CDNA4 issues v_fma_f64 at the full VALU rate and v_mad_i64_i32 at half
// (profiles/occbench_r01.json: 3.65e13 vs 1.97e13 lane-ops/s).  This
// experiment asks whether the long squaring chains -- the square root
// inside point decompression, ~250 squarings per point -- run faster on the
// FP64 pipe.  Measured (tools/fieldbench.hip, profiles/r02/fieldbench*.json):
// no.  Both forms are issue-bound, and the FP64 carries (4 adds per limb)
// and prescales cost what the full-rate FMAs save.  Not used by the product.
//
// Representation: limb j is an integer multiple of 2^P_j held exactly in a
// double, P = ceil(21.25 j) = {0, 22, 43, 64, 85, 107, 128, 149, 170, 192,
// 213, 234} (widths 22/21/21/21 repeating, P_12 = 255).  A product of limbs
// i and j is a multiple of 2^(P_i + P_j) >= 2^P_(i+j), so it lands in column
// i + j with no shifting; columns >= 12 wrap with the factor 19 * 2^-255
// (2^255 == 19), folded into a prescaled copy of one operand.  Every column
// sum is an integer multiple of its column's 2^P_c below 2^(53 + P_c), so
// every FMA is exact (round-to-nearest never engages).
//
// Level discipline as in curve25519.h: a carried element ("level 1") has
// |limb_j| <= 2^(w_j - 1) * 2^P_j; sums add levels; multiply inputs must be
// level <= 3 (column bound 2^52.13 * 2^P_c for level 3 x 3, computed in
// tests/test_fe64.py).  Carries round to nearest with the 1.5 * 2^(52 + P)
// constant: t = x + C rounds x to a multiple of 2^P (|x| < 2^(51 + P)), and
// hi = t - C, lo = x - hi are exact.
#pragma once
#include "curve25519.h"

namespace tmv {

struct fd { double v[12]; };

namespace fd_detail {
constexpr int kPos[13] = {0, 22, 43, 64, 85, 107, 128, 149, 170, 192, 213, 234, 255};

constexpr double p2(int e) {
  double r = 1.0;
  if (e >= 0) {
    for (int i = 0; i < e; i++) r *= 2.0;
  } else {
    for (int i = 0; i < -e; i++) r *= 0.5;
  }
  return r;
}
constexpr double kRound(int j) { return 1.5 * p2(52 + kPos[j]); }  // rounds to multiples of 2^P_j
constexpr double kWrap = 19.0 * p2(-255);
}  // namespace fd_detail

// Move column j's multiple of 2^P_(j+1) into column j + 1 (j = 11 wraps into
// column 0 times 19 * 2^-255).
template <int J>
TMV_HD void fd_carry_step(double *c) {
  using namespace fd_detail;
  constexpr double C = kRound(J + 1);
  const double hi = (c[J] + C) - C;
  c[J] -= hi;
  if (J == 11) c[0] = __builtin_fma(hi, kWrap, c[0]);
  else c[(J + 1) % 12] += hi;
}

// Two interleaved chains, 0 -> 6 and 5 -> 11 -> 0 -> 1 (like fe_carry_wide):
// the second chain takes column 5's raw sum first, so the first chain's last
// step (5 -> 6) and the final 0 -> 1 only add a few bits to limbs already
// carried.
TMV_HD void fd_carry(fd &h, double *c) {
  fd_carry_step<0>(c);  fd_carry_step<5>(c);
  fd_carry_step<1>(c);  fd_carry_step<6>(c);
  fd_carry_step<2>(c);  fd_carry_step<7>(c);
  fd_carry_step<3>(c);  fd_carry_step<8>(c);
  fd_carry_step<4>(c);  fd_carry_step<9>(c);
  fd_carry_step<5>(c);  fd_carry_step<10>(c);
  fd_carry_step<11>(c);
  fd_carry_step<0>(c);
#pragma unroll
  for (int i = 0; i < 12; i++) h.v[i] = c[i];
}

TMV_HD void fd_add(fd &h, const fd &f, const fd &g) {
#pragma unroll
  for (int i = 0; i < 12; i++) h.v[i] = f.v[i] + g.v[i];
}
TMV_HD void fd_sub(fd &h, const fd &f, const fd &g) {
#pragma unroll
  for (int i = 0; i < 12; i++) h.v[i] = f.v[i] - g.v[i];
}

// h = f * g: 144 FMAs + 11 prescales + the carry.
TMV_HD void fd_mul(fd &h, const fd &f, const fd &g) {
  using namespace fd_detail;
  double g19[12], c[12];
#pragma unroll
  for (int j = 1; j < 12; j++) g19[j] = g.v[j] * kWrap;
#pragma unroll
  for (int k = 0; k < 12; k++) c[k] = 0.0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int j = 0; j < 12; j++) {
      if (i + j < 12) c[i + j] = __builtin_fma(f.v[i], g.v[j], c[i + j]);
      else            c[i + j - 12] = __builtin_fma(f.v[i], g19[j], c[i + j - 12]);
    }
  }
  fd_carry(h, c);
}

// h = f^2: 78 FMAs (cross terms on 2 f_i, wrapped terms on 19 * 2^-255 f_j,
// j >= 6) + 17 prescales + the carry.
TMV_HD void fd_sq(fd &h, const fd &f) {
  using namespace fd_detail;
  double f2[11], f19[12], c[12];
#pragma unroll
  for (int i = 0; i < 11; i++) f2[i] = f.v[i] + f.v[i];
#pragma unroll
  for (int j = 6; j < 12; j++) f19[j] = f.v[j] * kWrap;
#pragma unroll
  for (int k = 0; k < 12; k++) c[k] = 0.0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int j = i; j < 12; j++) {
      const int k = i + j;
      if (i == j) {
        if (k < 12) c[k] = __builtin_fma(f.v[i], f.v[i], c[k]);
        else        c[k - 12] = __builtin_fma(f.v[i], f19[i], c[k - 12]);
      } else {
        if (k < 12) c[k] = __builtin_fma(f2[i], f.v[j], c[k]);
        else        c[k - 12] = __builtin_fma(f2[i], f19[j], c[k - 12]);
      }
    }
  }
  fd_carry(h, c);
}

TMV_HD void fd_sqn(fd &h, const fd &f, int n) {
  fd_sq(h, f);
  for (int i = 1; i < n; i++) fd_sq(h, h);
}

// radix 2^25.5 int limbs -> radix 2^21.25 doubles.  Int limb i (bit p_i)
// lands in the column with the largest P_j <= p_i, then one carry pass.
TMV_HD void fd_from_fe(fd &h, const fe &f) {
  using namespace fd_detail;
  constexpr int pi[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  constexpr int col[10] = {0, 1, 2, 3, 4, 6, 7, 8, 9, 10};
  double c[12];
#pragma unroll
  for (int k = 0; k < 12; k++) c[k] = 0.0;
#pragma unroll
  for (int i = 0; i < 10; i++) c[col[i]] = (double)f.v[i] * p2(pi[i]);
  fd_carry(h, c);
}

// radix 2^21.25 doubles (level <= 3) -> radix 2^25.5 int limbs, level 1.
TMV_HD void fe_from_fd(fe &h, const fd &f) {
  using namespace fd_detail;
  constexpr int pi[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  int64_t c[10];
#pragma unroll
  for (int i = 0; i < 10; i++) c[i] = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) {
    int i = 0;
#pragma unroll
    for (int t = 0; t < 10; t++) if (pi[t] <= kPos[j]) i = t;
    const int64_t k = (int64_t)(f.v[j] * p2(-kPos[j]));  // exact integer, |k| < 2^24
    c[i] += k * ((int64_t)1 << (kPos[j] - pi[i]));
  }
  fe_carry_wide(h, c);
}

// h = z^((p-5)/8) = z^(2^252 - 3) on the FP64 pipe (same chain as fe_pow22523).
TMV_HD void fd_pow22523(fd &h, const fd &z) {
  fd t0, t1, t2;
  fd_sq(t0, z);            // 2
  fd_sqn(t1, t0, 2);       // 8
  fd_mul(t1, z, t1);       // 9
  fd_mul(t0, t0, t1);      // 11
  fd_sq(t0, t0);           // 22
  fd_mul(t0, t1, t0);      // 2^5 - 1
  fd_sqn(t1, t0, 5);
  fd_mul(t0, t1, t0);      // 2^10 - 1
  fd_sqn(t1, t0, 10);
  fd_mul(t1, t1, t0);      // 2^20 - 1
  fd_sqn(t2, t1, 20);
  fd_mul(t1, t2, t1);      // 2^40 - 1
  fd_sqn(t1, t1, 10);
  fd_mul(t0, t1, t0);      // 2^50 - 1
  fd_sqn(t1, t0, 50);
  fd_mul(t1, t1, t0);      // 2^100 - 1
  fd_sqn(t2, t1, 100);
  fd_mul(t1, t2, t1);      // 2^200 - 1
  fd_sqn(t1, t1, 50);
  fd_mul(t0, t1, t0);      // 2^250 - 1
  fd_sqn(t0, t0, 2);       // 2^252 - 4
  fd_mul(h, t0, z);        // 2^252 - 3
}

// fe_pow22523 with the chain on the FP64 pipe.
TMV_HD void fe_pow22523_fd(fe &h, const fe &z) {
  fd a, b;
  fd_from_fe(a, z);
  fd_pow22523(b, a);
  fe_from_fd(h, b);
}

}  // namespace tmv
