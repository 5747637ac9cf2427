// Half-size scalars for single-signature verification (lattice reduction in
// dimension 2; T. Pornin, "Optimized Lattice Basis Reduction in Dimension 2,
// and Fast Schnorr and EdDSA Signature Verification", eprint 2020/454).
//
// A signature is checked as  [8]([s]B - R - [k]A) == O  (ZIP-215, cofactored;
// crypto/ed25519/ed25519.go:27-31 -> curve25519-voi) or, for sr25519,
// [s]B - [k]A == R modulo the 4-torsion (Ristretto equality).  [k]A costs a
// 252-doubling chain.  For small integers (u, v) with v == u k (mod l),
// |u|, v < 2^127,
//     [u]([s]B - R - [k]A) == [u s mod l]B - [u]R - [v]A   (mod E[8])
// because [u k]A and [v]A differ by a multiple of [l]A, which is 8-torsion
// (4-torsion for Ristretto points, which lie in 2E).  Both sides of the test
// live in the prime-order part after [8] (Ristretto: modulo E[4]), where [u]
// with u != 0 mod l is a bijection, so
//     [8]([s]B - R - [k]A) == O  <=>  [8]([b]B + [u](-R) + [v](-A)) == O,
//     b = u s mod l,
// and the same with "is in E[4]" for sr25519.  The right-hand side needs
// ~124 doublings (127-bit u, v) plus two fixed-base tables for b (B and
// [2^128]B): the verification chain drops from 252 to 124 doublings at the
// price of an R table and this reduction.  The validity bit is identical for
// every input (an exact equivalence, not a probabilistic one).
//
// (u, v) is the first remainder below 2^126 of the extended Euclidean
// algorithm on (l, k): r_i == t_i k (mod l), |t_i| r_{i-1} <= l, so at the
// first r_i < 2^126 (r_{i-1} >= 2^126) |t_i| < 2^126.6.  The quotients come
// from Lehmer's algorithm (Knuth TAOCP 4.5.2, Algorithm L) on 50-bit leading
// digits held in doubles, with Lehmer's test making every emulated quotient
// the true one; the 2x2 cofactor matrix (entries < 2^31) is then applied to
// the exact 256-bit remainders and the cofactor magnitudes (which only add:
// Euclid's t_i alternate in sign).  A first step Lehmer cannot decide (equal
// leading digits, or a quotient too large for them) subtracts a certain
// lower bound of the quotient exactly.  Quotients >= 2^31 (probability
// ~2^-24 per signature for a hash-derived k) and any result out of bounds
// return ok = false: the caller then verifies with the full 253-bit k
// (u = 1, v = k, b = s) -- slower, same result.
#pragma once
#include <stdint.h>
#include "curve25519.h"
#include "msm.h"

#if !defined(__HIPCC__)
#include <cmath>
#endif

namespace tmv {
namespace half {

constexpr int kLeadBits = 50;   // leading digits: sums with the cofactors stay < 2^53 (exact in doubles)
constexpr int kMaxOuter = 24;   // Lehmer rounds (random k: 6 on average, 7 at most in 2^17 samples)
constexpr double kMaxCof = 2147483648.0;  // 2^31: cofactor matrix entries fit int32

// word i of an 8-word number, 0 past the top, for a run-time i (unrolled select)
TMV_HD uint32_t pick(const uint32_t r[8], int i) {
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) x = (i == j) ? r[j] : x;
  return x;
}

TMV_HD int bitlen8(const uint32_t r[8]) {
  int bl = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int c = r[j] ? 32 * j + 32 - __builtin_clz(r[j]) : 0;
    bl = r[j] ? c : bl;
  }
  return bl;
}

// floor(r / 2^e) for e >= 0, truncated to its low 64 bits (callers choose e
// so that it is < 2^kLeadBits)
TMV_HD uint64_t shr64(const uint32_t r[8], int e) {
  const int wi = e >> 5, sh = e & 31;
  const uint64_t w0 = pick(r, wi), w1 = pick(r, wi + 1), w2 = pick(r, wi + 2);
  const uint64_t lo = w0 | (w1 << 32);
  return sh ? (lo >> sh) | (w2 << (64 - sh)) : lo;
}

// floor(n / d) for integers 0 <= n < 2^53, 0 < d < 2^53 held in doubles
TMV_HD double floor_div(double n, double d) {
  double q = floor(n / d);
  const double rem = fma(-q, d, n);  // exact: an integer of magnitude < 2^53
  q = rem < 0 ? q - 1 : (rem >= d ? q + 1 : q);
  return q;
}

// floor(n / d) for integers 0 <= n < 2^53, 0 < d < 2^53 held in doubles,
// from a reciprocal (v_rcp_f64 on the device, no IEEE division sequence) and
// a remainder correction; *ok = false when the result is not certified
// exactly (the caller then ends its Lehmer round early -- always safe).
// The division sequence was most of reduce()'s cost: 70.7 field multiplies
// of chip time per reduction (tools/reduce_bench.hip), nearly all of it in
// the two IEEE divisions of every Lehmer step.
TMV_HD double floor_div_rcp(double n, double d, bool &ok) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double r = __builtin_amdgcn_rcp(d);
#else
  const double r = 1.0 / d;
#endif
  double q = floor(n * r);
  double rem = fma(-q, d, n);
  q = rem < 0 ? q - 1 : (rem >= d ? q + 1 : q);
  rem = fma(-q, d, n);
  ok = rem >= 0 && rem < d;
  return q;
}

// x = a * y (a < 2^32): 9 words
TMV_HD void mul_1(uint32_t x[9], uint32_t a, const uint32_t y[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t t = (uint64_t)a * y[i] + c;
    x[i] = (uint32_t)t;
    c = t >> 32;
  }
  x[8] = (uint32_t)c;
}

// r = x - y (9 words, x >= y), low 8 words kept (the result fits)
TMV_HD void sub_9(uint32_t r[8], const uint32_t x[9], const uint32_t y[9]) {
  int64_t b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int64_t d = (int64_t)x[i] - y[i] + b;
    r[i] = (uint32_t)d;
    b = d >> 32;
  }
}

// T = a * x + b * y over 5-word magnitudes (the cofactors stay < 2^131)
TMV_HD void lin_5(uint32_t T[5], uint32_t a, const uint32_t x[5], uint32_t b, const uint32_t y[5]) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t p = (uint64_t)a * x[i] + c;        // < 2^64
    const uint64_t q = (uint64_t)b * y[i] + (uint32_t)p;
    T[i] = (uint32_t)q;
    c = (p >> 32) + (q >> 32);
  }
}

// 9-word compare x < y
TMV_HD bool lt9(const uint32_t x[9], const uint32_t y[9]) {
  int r = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) r = x[i] > y[i] ? 1 : (x[i] < y[i] ? -1 : r);
  return r < 0;
}

// 8-word compare x >= y
TMV_HD bool geq8(const uint32_t x[8], const uint32_t y[8]) {
  int r = 0;  // 1: x > y, -1: x < y, decided by the highest differing word
#pragma unroll
  for (int i = 0; i < 8; i++) r = x[i] > y[i] ? 1 : (x[i] < y[i] ? -1 : r);
  return r >= 0;
}

// Outputs: u (magnitude, 4 words), u_neg, v (4 words), with v == u k (mod l)
// for the signed u; returns false (slow path) when the reduction cannot finish
// within its bounds.  k < l.
TMV_HD bool reduce(uint32_t u_out[4], bool &u_neg, uint32_t v_out[4], const uint32_t k[8]) {
  uint32_t r0[8], r1[8], T0[5] = {0, 0, 0, 0, 0}, T1[5] = {1, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 8; i++) { r0[i] = scl::l(i); r1[i] = k[i]; }
  int par = 0;  // sign of t1 = (-1)^par (Euclid's cofactors alternate)
  bool ok = true;
  for (int outer = 0; outer < kMaxOuter; outer++) {
    // loop while r1 >= 2^126: words 4..7 nonzero or bit 30 of word 3 set
    const bool big = (r1[4] | r1[5] | r1[6] | r1[7]) != 0 || (r1[3] >> 30) != 0;
    if (!big) break;
    const int e = bitlen8(r0) - kLeadBits;  // r0 > r1 >= 2^126, so e > 0
    double uh = (double)shr64(r0, e), vh = (double)shr64(r1, e);
    const double thr = ldexp(1.0, 126 - e);  // 2^126 / 2^e
    double A = 1, B = 0, C = 0, D = 1;
    int steps = 0;
    for (int it = 0; it < 64; it++) {  // ~12 steps per round; bounded
      const double dc = vh + C, dd = vh + D;
      if (!(dc > 0 && dd > 0)) break;
      bool exact;
      const double q = floor_div_rcp(uh + A, dc, exact);
      // Lehmer's test: the quotient must also be floor((uh + B) / dd), i.e.
      // 0 <= (uh + B) - q dd < dd (one multiply-add, not a second division)
      const double rem2 = fma(-q, dd, uh + B);
      if (!exact || rem2 < 0 || rem2 >= dd) break;  // not certain
      const double nC = fma(-q, C, A), nD = fma(-q, D, B);
      if (fabs(nC) >= kMaxCof || fabs(nD) >= kMaxCof) break;
      A = C; B = D; C = nC; D = nD;
      const double nv = fma(-q, vh, uh);
      uh = vh; vh = nv;
      steps++;
      // stop right after the step that may take r1 below 2^126 (the
      // emulated remainder is within |C| + |D| of the true one / 2^e)
      if (vh < thr + fabs(C) + fabs(D) + 2) break;
    }
    if (steps == 0) {
      // Lehmer's test could not certify even the first quotient (equal
      // leading digits, or a quotient large against vh's precision).  Take
      // q1 = max(1, floor(uh / (vh + 1))) <= floor(r0 / r1) and subtract
      // q1 r1 from r0 exactly: a whole Euclid step when the result is below
      // r1 (then swap), else a partial one (the next round finishes it with
      // the smaller r0's sharper digits).  t0 - q1 t1 keeps t0's sign
      // (Euclid's cofactors alternate), so its magnitude is T0 + q1 T1.
      double q1 = floor_div(uh, vh + 1);
      q1 = q1 < 1 ? 1 : q1;
      if (q1 >= kMaxCof) { ok = false; break; }  // quotient >= 2^31: slow path
      const uint32_t qq = (uint32_t)q1;
      uint32_t x[9], y[9], rem[8], nT0[5];
#pragma unroll
      for (int i = 0; i < 8; i++) x[i] = r0[i];
      x[8] = 0;
      mul_1(y, qq, r1);
      sub_9(rem, x, y);  // >= 0: q1 <= the true quotient
      lin_5(nT0, 1u, T0, qq, T1);
      if (geq8(rem, r1)) {  // partial step: r0 shrinks, roles stay
#pragma unroll
        for (int i = 0; i < 8; i++) r0[i] = rem[i];
#pragma unroll
        for (int i = 0; i < 5; i++) T0[i] = nT0[i];
      } else {  // whole step
#pragma unroll
        for (int i = 0; i < 8; i++) { r0[i] = r1[i]; r1[i] = rem[i]; }
#pragma unroll
        for (int i = 0; i < 5; i++) { T0[i] = T1[i]; T1[i] = nT0[i]; }
        par ^= 1;
      }
      continue;
    }
    // apply the cofactor matrix: signs alternate with the step parity
    // (even: A, D >= 0 >= B, C; odd: the reverse), so every new remainder is
    // a difference of two nonnegative products and every cofactor a sum
    const uint32_t a = (uint32_t)fabs(A), b = (uint32_t)fabs(B), c = (uint32_t)fabs(C), d = (uint32_t)fabs(D);
    uint32_t pa[9], pb[9], pc[9], pd[9];
    mul_1(pa, a, r0);
    mul_1(pb, b, r1);
    mul_1(pc, c, r0);
    mul_1(pd, d, r1);
    const bool odd = steps & 1;
    uint32_t n0[8], n1[8];
    if (odd) { sub_9(n0, pb, pa); sub_9(n1, pc, pd); }
    else { sub_9(n0, pa, pb); sub_9(n1, pd, pc); }
    uint32_t nT0[5], nT1[5];
    lin_5(nT0, a, T0, b, T1);
    lin_5(nT1, c, T0, d, T1);
#pragma unroll
    for (int i = 0; i < 8; i++) { r0[i] = n0[i]; r1[i] = n1[i]; }
#pragma unroll
    for (int i = 0; i < 5; i++) { T0[i] = nT0[i]; T1[i] = nT1[i]; }
    par ^= steps & 1;
  }
  // done iff r1 < 2^126; bounds: v = r1 < 2^127, |u| = T1 < 2^127
  const bool r1_small = (r1[4] | r1[5] | r1[6] | r1[7]) == 0 && (r1[3] >> 30) == 0;
  const bool u_small = T1[4] == 0 && (T1[3] >> 31) == 0;
  ok = ok && r1_small && u_small;
#pragma unroll
  for (int i = 0; i < 4; i++) { u_out[i] = T1[i]; v_out[i] = r1[i]; }
  u_neg = par != 0;
  return ok;
}


// Scalars of the short check: fast (reduce() succeeded): |u|, v < 2^127 and
// b = |u| s mod l, the B and R terms negated when u < 0; slow: u = 1, v = k,
// b = s (the plain 253-bit check).
struct Scalars {
  uint32_t u[8], v[8], b[8];
  bool u_neg, fast;
};
// The same from a reduction done elsewhere (u4, u_neg, v4, fast: reduce()'s outputs).
TMV_HD void scalars_from(Scalars &o, const uint32_t u4[4], bool neg, const uint32_t v4[4], bool fast,
                         const uint32_t k[8], const uint32_t s[8]) {
  o.fast = fast;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    o.u[i] = o.fast ? (i < 4 ? u4[i] : 0u) : (i == 0 ? 1u : 0u);
    o.v[i] = o.fast ? (i < 4 ? v4[i] : 0u) : k[i];
  }
  o.u_neg = o.fast && neg;
  if (o.fast) sc_mul_mod(o.b, o.u, 4, s);
  else {
#pragma unroll
    for (int i = 0; i < 8; i++) o.b[i] = s[i];
  }
}

TMV_HD void scalars(Scalars &o, const uint32_t k[8], const uint32_t s[8]) {
  uint32_t u4[4], v4[4];
  bool neg = false;
  o.fast = reduce(u4, neg, v4, k);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    o.u[i] = o.fast ? (i < 4 ? u4[i] : 0u) : (i == 0 ? 1u : 0u);
    o.v[i] = o.fast ? (i < 4 ? v4[i] : 0u) : k[i];
  }
  o.u_neg = o.fast && neg;
  if (o.fast) sc_mul_mod(o.b, o.u, 4, s);
  else {
#pragma unroll
    for (int i = 0; i < 8; i++) o.b[i] = s[i];
  }
}

}  // namespace half
}  // namespace tmv
