// GF(2^255-19) field, edwards25519 group and scalar-mod-l arithmetic for the
// MI355X verification kernels.  Compiled for gfx950 (device) and, unchanged,
// for the host (the runtime precomputes the base-point table with it and the
// CPU test tests/native/test_arith.cpp runs it with limb-bound assertions).
//
// Replaces the field/point/scalar internals of the absent third-party module
// curve25519-voi (go.mod:22) that sit behind crypto/ed25519/ed25519.go:173-233
// and crypto/sr25519/{pubkey.go:49-62,batch.go:23-47}.
//
// Representation: radix 2^25.5 — ten signed 32-bit limbs alternating 26/25
// bits.  One field multiply = 100 32x32->64 multiply-adds (v_mad_i64_i32 on
// CDNA4's VALU; this is integer work, MFMA does not apply).
//
// Limb-magnitude discipline ("level"): every mul/sq output is carried
// (|limb| <= 2^25 on 26-bit positions, 2^24 on 25-bit positions, level 1).
// Sums/differences add levels.  Multiply inputs must be level <= 3 so that
// 19*g fits int32 and the 64-bit column sums cannot overflow.  Each formula
// below is annotated with the level of its intermediates; TMV_BOUNDS_CHECK
// (host only) asserts it.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TMV_HD __host__ __device__ __forceinline__
#define TMV_DEV __device__ __forceinline__
#else
#define TMV_HD inline
#define TMV_DEV inline
#endif

#ifdef TMV_BOUNDS_CHECK
#include <cassert>
#include <cstdlib>
#define TMV_ASSERT_LEVEL(f, lvl)                                               \
  do {                                                                         \
    for (int _i = 0; _i < 10; _i++) {                                          \
      int64_t _b = (int64_t)(lvl) << ((_i & 1) ? 24 : 25);                     \
      int64_t _x = (f).v[_i];                                                  \
      if (_x > _b + ((int64_t)1 << 20) || _x < -_b - ((int64_t)1 << 20)) {     \
        assert(!"field limb exceeds level bound");                             \
      }                                                                        \
    }                                                                          \
  } while (0)
#else
#define TMV_ASSERT_LEVEL(f, lvl) do { } while (0)
#endif

namespace tmv {

struct fe { int32_t v[10]; };

TMV_HD void fe_zero(fe &h) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = 0;
}
TMV_HD void fe_one(fe &h) { fe_zero(h); h.v[0] = 1; }

TMV_HD void fe_add(fe &h, const fe &f, const fe &g) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
}
TMV_HD void fe_sub(fe &h, const fe &f, const fe &g) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = f.v[i] - g.v[i];
}
TMV_HD void fe_neg(fe &h, const fe &f) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = -f.v[i];
}
// branch-free conditional move: h = b ? g : h
TMV_HD void fe_cmov(fe &h, const fe &g, bool b) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = b ? g.v[i] : h.v[i];
}

// Rounding bias of column i: it is carried with a shift of 26 (even i) or
// 25 (odd i) bits, rounded to nearest: k = (c + 2^(shift-1)) >> shift.
TMV_HD int64_t carry_bias(int i) { return (int64_t)1 << ((i & 1) ? 24 : 25); }
// Column accumulation c + a * b as one v_mad_i64_i32, written out on the
// device: left to itself the compiler splits each column into partial sums
// joined by extra 64-bit adds and moves a constant addend (the carry bias
// below) to a separate add at the end -- 10 + 10 extra adds per multiply.
// Ten independent columns give the scheduler enough parallelism.
TMV_HD int64_t mad_acc(int32_t a, int32_t b, int64_t c) {
  int64_t r = c + (int64_t)a * b;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(r));  // no instruction: keeps the column one chain
#endif
  return r;
}
// carry_bias(i) + a * b (the column's first product; the bias from an SGPR pair)
TMV_HD int64_t mad_bias(int32_t a, int32_t b, int i) {
  int64_t bias = carry_bias(i);
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+s"(bias));  // an opaque addend, so the multiply-add takes it
#endif
  return mad_acc(a, b, bias);
}

// Carry a column-sum vector back to level 1.  Two interleaved chains
// (0->1->2->3->4 and 4->5->...->9->0->1) for ILP.  The columns arrive
// already holding their rounding bias (c[i] = carry_bias(i) + sum: the
// multiplies start each column's accumulation at its bias instead of 0), so
// a step is k = c >> shift (no rounding add), the remainder keeps the bias
// through later carries into it, and each limb drops it once at the end --
// the same limbs as rounding every step, 12 fewer 64-bit adds per multiply.
TMV_HD void fe_carry_biased(fe &h, int64_t c[10]) {
  int64_t k;
  k = c[0] >> 26; c[1] += k; c[0] -= k * ((int64_t)1 << 26);
  k = c[4] >> 26; c[5] += k; c[4] -= k * ((int64_t)1 << 26);
  k = c[1] >> 25; c[2] += k; c[1] -= k * ((int64_t)1 << 25);
  k = c[5] >> 25; c[6] += k; c[5] -= k * ((int64_t)1 << 25);
  k = c[2] >> 26; c[3] += k; c[2] -= k * ((int64_t)1 << 26);
  k = c[6] >> 26; c[7] += k; c[6] -= k * ((int64_t)1 << 26);
  k = c[3] >> 25; c[4] += k; c[3] -= k * ((int64_t)1 << 25);
  k = c[7] >> 25; c[8] += k; c[7] -= k * ((int64_t)1 << 25);
  k = c[4] >> 26; c[5] += k; c[4] -= k * ((int64_t)1 << 26);
  k = c[8] >> 26; c[9] += k; c[8] -= k * ((int64_t)1 << 26);
  k = c[9] >> 25; c[0] += k * 19; c[9] -= k * ((int64_t)1 << 25);
  k = c[0] >> 26; c[1] += k; c[0] -= k * ((int64_t)1 << 26);
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = (int32_t)(c[i] - carry_bias(i));
}

// The same carry in two parallel rounds (latency form): every column's
// quotient at once, added to the next column; then once more for the small
// second-round quotients.  Two dependent steps instead of the twelve-step
// chain, ~20 more instructions; the limbs are level 1 plus at most 19 * 2^12
// (a different representation of the same element: results encode the same).
// Used by the quad formulas (one wave's dependent chain: Horner, the
// per-entry checks), not by the throughput kernels (TMV_QUAD_PCARRY).
TMV_HD void fe_carry_biased_par(fe &h, int64_t c[10]) {
  int64_t k[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int sh = (i & 1) ? 25 : 26;
    k[i] = c[i] >> sh;
    c[i] -= k[i] * ((int64_t)1 << sh);  // [0, 2^sh): the bias is still in it
  }
#pragma unroll
  for (int i = 9; i >= 1; i--) c[i] += k[i - 1];
  c[0] += k[9] * 19;
  int32_t k2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int sh = (i & 1) ? 25 : 26;
    k2[i] = (int32_t)(c[i] >> sh);
    c[i] -= (int64_t)k2[i] * ((int64_t)1 << sh);
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t in = i ? k2[i - 1] : k2[9] * 19;
    h.v[i] = (int32_t)(c[i] - carry_bias(i)) + in;
  }
}

// The same for columns without the bias.
TMV_HD void fe_carry_wide(fe &h, int64_t c[10]) {
#pragma unroll
  for (int i = 0; i < 10; i++) c[i] += carry_bias(i);
  fe_carry_biased(h, c);
}

// Re-carry any level <= 3 value to level 1.
TMV_HD void fe_carry(fe &h, const fe &f) {
  int64_t c[10];
#pragma unroll
  for (int i = 0; i < 10; i++) c[i] = (int64_t)f.v[i] + carry_bias(i);
  fe_carry_biased(h, c);
}

// 19 x as two full-rate shift-adds (v_mul_lo_u32 is quarter rate on CDNA4)
// (the compiler folds plain shift-adds back into v_mul_lo_u32, hence asm)
TMV_HD int32_t mul19(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  int32_t t, r;
  asm("v_lshl_add_u32 %0, %1, 1, %1" : "=v"(t) : "v"(x));
  asm("v_lshl_add_u32 %0, %1, 4, %2" : "=v"(r) : "v"(x), "v"(t));
  return r;
#else
  return (int32_t)((uint32_t)x * 19u);
#endif
}

// h = f * g.  Column k collects f_i g_j with i+j == k, plus 19 f_i g_j for
// i+j == k+10 (2^255 == 19).  Odd*odd limb products carry an extra factor 2
// (25.5-bit radix).
TMV_HD void fe_mul(fe &h, const fe &f, const fe &g) {
  TMV_ASSERT_LEVEL(f, 3);
  TMV_ASSERT_LEVEL(g, 3);
  int32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = mul19(g.v[i]);
    f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
  }
  int64_t c[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const int32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      if (i == 0) c[j] = mad_bias(a, g.v[j], j);  // column j starts at its bias
      else if (i + j < 10) c[i + j] = mad_acc(a, g.v[j], c[i + j]);
      else                 c[i + j - 10] = mad_acc(a, g19[j], c[i + j - 10]);
    }
  }
  fe_carry_biased(h, c);
}

// fe_mul with the two-round carry (quad formulas, latency-bound chains)
TMV_HD void fe_mul_par(fe &h, const fe &f, const fe &g) {
  TMV_ASSERT_LEVEL(f, 3);
  TMV_ASSERT_LEVEL(g, 3);
  int32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = mul19(g.v[i]);
    f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
  }
  int64_t c[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const int32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      if (i == 0) c[j] = mad_bias(a, g.v[j], j);
      else if (i + j < 10) c[i + j] = mad_acc(a, g.v[j], c[i + j]);
      else                 c[i + j - 10] = mad_acc(a, g19[j], c[i + j - 10]);
    }
  }
  fe_carry_biased_par(h, c);
}

// h = f^2 (55 products via symmetry)
TMV_HD void fe_sq(fe &h, const fe &f) {
  TMV_ASSERT_LEVEL(f, 3);
  int32_t f2[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { f2[i] = 2 * f.v[i]; f19[i] = mul19(f.v[i]); }
  // column k starts at its bias with its first product: (0, k) for k <= 9,
  // then (k - 9, 9) for the wrapped columns 0..8 (i + j = k + 10)
  int64_t c[10];
  bool started[10] = {false, false, false, false, false, false, false, false, false, false};
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      // f_i f_j appears twice for i != j; odd*odd carries another factor 2
      const int oddodd = (i & 1) && (j & 1);
      int32_t a = (i == j) ? f.v[i] : f2[i];
      if (oddodd) a = 2 * a;
      const int k = i + j < 10 ? i + j : i + j - 10;
      const int32_t b = i + j < 10 ? f.v[j] : f19[j];
      if (!started[k]) { c[k] = mad_bias(a, b, k); started[k] = true; }
      else c[k] = mad_acc(a, b, c[k]);
    }
  }
  fe_carry_biased(h, c);
}

// h = 2 f^2
TMV_HD void fe_sq2(fe &h, const fe &f) {
  fe t;
  fe_sq(t, f);
  fe_add(t, t, t);  // level 2
  fe_carry(h, t);   // callers treat the result as level 1
}

// h = f^2 with floor carries: limbs in [0, 2^26) / [0, 2^25) (limb 1 up to
// 2^25 + 2^13), not centred.  Such limbs are below the level-3 bound
// (3 * 2^25), so they may be squared again, but not added to anything: only
// the inner squarings of fe_sqn produce them.  Saves the ten bias
// subtractions of the centred carry (the columns start at 0).
TMV_HD void fe_sq_floor(fe &h, const fe &f) {
  TMV_ASSERT_LEVEL(f, 3);
  int32_t f2[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { f2[i] = 2 * f.v[i]; f19[i] = mul19(f.v[i]); }
  int64_t zero = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+s"(zero));  // an opaque zero addend: each column one v_mad_i64_i32 chain
#endif
  int64_t c[10];
  bool started[10] = {false, false, false, false, false, false, false, false, false, false};
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      const int oddodd = (i & 1) && (j & 1);
      int32_t a = (i == j) ? f.v[i] : f2[i];
      if (oddodd) a = 2 * a;
      const int k = i + j < 10 ? i + j : i + j - 10;
      const int32_t b = i + j < 10 ? f.v[j] : f19[j];
      c[k] = mad_acc(a, b, started[k] ? c[k] : zero);
      started[k] = true;
    }
  }
  int64_t k;
  k = c[0] >> 26; c[1] += k; c[0] -= k * ((int64_t)1 << 26);
  k = c[4] >> 26; c[5] += k; c[4] -= k * ((int64_t)1 << 26);
  k = c[1] >> 25; c[2] += k; c[1] -= k * ((int64_t)1 << 25);
  k = c[5] >> 25; c[6] += k; c[5] -= k * ((int64_t)1 << 25);
  k = c[2] >> 26; c[3] += k; c[2] -= k * ((int64_t)1 << 26);
  k = c[6] >> 26; c[7] += k; c[6] -= k * ((int64_t)1 << 26);
  k = c[3] >> 25; c[4] += k; c[3] -= k * ((int64_t)1 << 25);
  k = c[7] >> 25; c[8] += k; c[7] -= k * ((int64_t)1 << 25);
  k = c[4] >> 26; c[5] += k; c[4] -= k * ((int64_t)1 << 26);
  k = c[8] >> 26; c[9] += k; c[8] -= k * ((int64_t)1 << 26);
  k = c[9] >> 25; c[0] += k * 19; c[9] -= k * ((int64_t)1 << 25);
  k = c[0] >> 26; c[1] += k; c[0] -= k * ((int64_t)1 << 26);
#pragma unroll
  for (int i = 0; i < 10; i++) {
    int32_t v = (int32_t)c[i];
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(v));  // hide the limbs' sign: knowing them >= 0 the compiler
                        // turns the next squaring's products into unsigned
                        // mads with extra moves (151 vs 122 instructions)
#endif
    h.v[i] = v;
  }
}

// h = f^(2^n): the inner squarings with floor carries, the last centred
// (level 1).  TMV_SQN_FLOOR=0: every squaring centred.
#ifndef TMV_SQN_FLOOR
#define TMV_SQN_FLOOR 1
#endif
TMV_HD void fe_sqn(fe &h, const fe &f, int n) {
#if TMV_SQN_FLOOR
  if (n == 1) {
    fe_sq(h, f);
    return;
  }
  fe_sq_floor(h, f);
  for (int i = 2; i < n; i++) fe_sq_floor(h, h);
  fe_sq(h, h);
#else
  fe_sq(h, f);
  for (int i = 1; i < n; i++) fe_sq(h, h);
#endif
}

// Bit positions of the ten limbs.
#define TMV_LIMB_POS {0, 26, 51, 77, 102, 128, 153, 179, 204, 230}

// Load 255 bits (bit 255 ignored) from eight little-endian 32-bit words.
// The value may be >= p (lax decoding accepts it); limbs are exact, level 1.
TMV_HD void fe_from_words(fe &h, const uint32_t w[8]) {
  const int pos[10] = TMV_LIMB_POS;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int p = pos[i], width = (i & 1) ? 25 : 26;
    const int wi = p >> 5, sh = p & 31;
    uint64_t x = w[wi];
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << 32;
    uint32_t limb = (uint32_t)(x >> sh) & ((1u << width) - 1);
    h.v[i] = (int32_t)limb;
  }
  // limb 9 covers bits 230..254; bit 255 was masked by width (25 bits)
}

TMV_HD void fe_from_bytes(fe &h, const uint8_t s[32]) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++)
    w[i] = (uint32_t)s[4 * i] | ((uint32_t)s[4 * i + 1] << 8) |
           ((uint32_t)s[4 * i + 2] << 16) | ((uint32_t)s[4 * i + 3] << 24);
  fe_from_words(h, w);
}

// Canonical (fully reduced) little-endian words.  Input level <= 3.
TMV_HD void fe_to_words(uint32_t w[8], const fe &f) {
  int64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = f.v[i];
  // bring to level 1 first (handles level-3 inputs)
  {
    fe t;
    fe_carry_wide(t, h);
#pragma unroll
    for (int i = 0; i < 10; i++) h[i] = t.v[i];
  }
  // q = floor((h + 19) / 2^255) in {0, 1} (h in (-2^255, 2^256) after carry)
  int64_t q = (19 * h[9] + ((int64_t)1 << 24)) >> 25;
#pragma unroll
  for (int i = 0; i < 10; i++) q = (h[i] + q) >> ((i & 1) ? 25 : 26);
  h[0] += 19 * q;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int sh = (i & 1) ? 25 : 26;
    int64_t k = h[i] >> sh;
    h[i + 1] += k;
    h[i] -= k * ((int64_t)1 << sh);
  }
  h[9] -= (h[9] >> 25) * ((int64_t)1 << 25);
  // pack: limbs are now in [0, 2^width)
  const int pos[10] = TMV_LIMB_POS;
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint64_t limb = (uint64_t)h[i];
    const int wi = pos[i] >> 5, sh = pos[i] & 31;
    w[wi] |= (uint32_t)(limb << sh);
    if (wi + 1 < 8 && sh) w[wi + 1] |= (uint32_t)(limb >> (32 - sh));
  }
}

TMV_HD bool fe_is_zero(const fe &f) {
  uint32_t w[8];
  fe_to_words(w, f);
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r |= w[i];
  return r == 0;
}
TMV_HD bool fe_is_negative(const fe &f) {
  uint32_t w[8];
  fe_to_words(w, f);
  return w[0] & 1;
}
TMV_HD bool fe_eq(const fe &a, const fe &b) {
  fe d;
  fe_sub(d, a, b);
  return fe_is_zero(d);
}

// h = z^((p-5)/8) = z^(2^252 - 3)
TMV_HD void fe_pow22523(fe &h, const fe &z) {
  fe t0, t1, t2;
  fe_sq(t0, z);            // 2
  fe_sqn(t1, t0, 2);       // 8
  fe_mul(t1, z, t1);       // 9
  fe_mul(t0, t0, t1);      // 11
  fe_sq(t0, t0);           // 22
  fe_mul(t0, t1, t0);      // 2^5 - 1
  fe_sqn(t1, t0, 5);
  fe_mul(t0, t1, t0);      // 2^10 - 1
  fe_sqn(t1, t0, 10);
  fe_mul(t1, t1, t0);      // 2^20 - 1
  fe_sqn(t2, t1, 20);
  fe_mul(t1, t2, t1);      // 2^40 - 1
  fe_sqn(t1, t1, 10);
  fe_mul(t0, t1, t0);      // 2^50 - 1
  fe_sqn(t1, t0, 50);
  fe_mul(t1, t1, t0);      // 2^100 - 1
  fe_sqn(t2, t1, 100);
  fe_mul(t1, t2, t1);      // 2^200 - 1
  fe_sqn(t1, t1, 50);
  fe_mul(t0, t1, t0);      // 2^250 - 1
  fe_sqn(t0, t0, 2);       // 2^252 - 4
  fe_mul(h, t0, z);        // 2^252 - 3
}

// h = z^(p-2) = z^-1
TMV_HD void fe_invert(fe &h, const fe &z) {
  fe t0, t1, t2, t3;
  fe_sq(t0, z);            // 2
  fe_sqn(t1, t0, 2);       // 8
  fe_mul(t1, z, t1);       // 9
  fe_mul(t0, t0, t1);      // 11
  fe_sq(t2, t0);           // 22
  fe_mul(t1, t1, t2);      // 2^5 - 1
  fe_sqn(t2, t1, 5);
  fe_mul(t1, t2, t1);      // 2^10 - 1
  fe_sqn(t2, t1, 10);
  fe_mul(t2, t2, t1);      // 2^20 - 1
  fe_sqn(t3, t2, 20);
  fe_mul(t2, t3, t2);      // 2^40 - 1
  fe_sqn(t2, t2, 10);
  fe_mul(t1, t2, t1);      // 2^50 - 1
  fe_sqn(t2, t1, 50);
  fe_mul(t2, t2, t1);      // 2^100 - 1
  fe_sqn(t3, t2, 100);
  fe_mul(t2, t3, t2);      // 2^200 - 1
  fe_sqn(t2, t2, 50);
  fe_mul(t1, t2, t1);      // 2^250 - 1
  fe_sqn(t1, t1, 5);       // 2^255 - 32
  fe_mul(h, t1, t0);       // 2^255 - 21
}

// ---------------------------------------------------------------- constants
// Limb images (level 1) of the curve constants; derived in
// tests/test_arith_constants.py from the integers they encode.
struct consts {
  static TMV_HD fe d()      { return fe{{-10913610, 13857413, -15372611, 6949391, 114729, -8787816, -6275908, -3247719, -18696448, -12055116}}; }
  static TMV_HD fe d2()     { return fe{{-21827239, -5839606, -30745221, 13898782, 229458, 15978800, -12551817, -6495438, 29715968, 9444199}}; }
  static TMV_HD fe sqrtm1() { return fe{{-32595792, -7943725, 9377950, 3500415, 12389472, -272473, -25146209, -2005654, 326686, 11406482}}; }
  static TMV_HD fe invsqrt_a_minus_d() { return fe{{6111485, 4156064, -27798727, 12243468, -25904040, 120897, 20826367, -7060776, 6093568, -1986012}}; }
};

// ---------------------------------------------------------------- points
// Extended twisted Edwards (a = -1): x = X/Z, y = Y/Z, xy = T/Z.
struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };            // completed: x = X/Z, y = Y/T
struct ge_cached { fe YpX, YmX, Z, T2d; };
struct ge_precomp { fe ypx, ymx, xy2d; };      // affine Niels form, Z = 1

TMV_HD void ge_p3_identity(ge_p3 &h) { fe_zero(h.X); fe_one(h.Y); fe_one(h.Z); fe_zero(h.T); }
TMV_HD void ge_precomp_identity(ge_precomp &h) { fe_one(h.ypx); fe_one(h.ymx); fe_zero(h.xy2d); }

TMV_HD void ge_p1p1_to_p2(ge_p2 &r, const ge_p1p1 &p) {  // (Z Y: Z's x2 form shared with Z T)
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
}
// (X T, Z Y, Z T, X Y: the right operands -- T, Y -- and the left ones -- X,
// Z -- each serve two products, so their x19 and odd-limb x2 forms are built
// once per conversion: 25 fewer VALU instructions than (X T, Y Z, Z T, X Y),
// the same limbs -- a product's columns do not depend on operand order)
TMV_HD void ge_p1p1_to_p3(ge_p3 &r, const ge_p1p1 &p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}
TMV_HD void ge_p3_to_p2(ge_p2 &r, const ge_p3 &p) { r.X = p.X; r.Y = p.Y; r.Z = p.Z; }
// completed -> cached without the extended form in between (five
// multiplications, as p1p1_to_p3 + p3_to_cached, when T itself is not needed)
TMV_HD void ge_p1p1_to_cached(ge_cached &r, const ge_p1p1 &p) {
  fe x, y, t;
  fe_mul(x, p.X, p.T);
  fe_mul(y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(t, p.X, p.Y);
  fe_mul(r.T2d, t, consts::d2());
  fe_add(r.YpX, y, x);                // level 2
  fe_sub(r.YmX, y, x);                // level 2
}

TMV_HD void ge_p3_to_cached(ge_cached &r, const ge_p3 &p) {
  fe_add(r.YpX, p.Y, p.X);            // level 2
  fe_sub(r.YmX, p.Y, p.X);            // level 2
  r.Z = p.Z;
  fe_mul(r.T2d, p.T, consts::d2());
}

// dbl-2008-hwcd, a = -1; output is the negation of (E, H, G, F) on every
// coordinate, which is the same projective point.
TMV_HD void ge_p2_dbl(ge_p1p1 &r, const ge_p2 &p) {
  fe XX, YY, ZZ2, S, AA;
  fe_sq(XX, p.X);
  fe_sq(YY, p.Y);
  fe_sq2(ZZ2, p.Z);
  fe_add(S, p.X, p.Y);                 // level <= 2
  fe_sq(AA, S);
  fe_add(r.Y, YY, XX);                 // 2
  fe_sub(r.Z, YY, XX);                 // 2
  fe_sub(r.X, AA, r.Y);                // 3
  fe_sub(r.T, ZZ2, r.Z);               // 3
}
TMV_HD void ge_p3_dbl(ge_p1p1 &r, const ge_p3 &p) {
  ge_p2 q;
  ge_p3_to_p2(q, p);
  ge_p2_dbl(r, q);
}

// add-2008-hwcd-3 (k = 2d): p + q
TMV_HD void ge_add(ge_p1p1 &r, const ge_p3 &p, const ge_cached &q) {
  fe a, b, c, dd, t;
  fe_sub(t, p.Y, p.X); fe_mul(a, t, q.YmX);
  fe_add(t, p.Y, p.X); fe_mul(b, t, q.YpX);
  fe_mul(c, p.T, q.T2d);
  fe_mul(dd, p.Z, q.Z);
  fe_add(dd, dd, dd);                  // 2
  fe_sub(r.X, b, a);                   // 2  E
  fe_add(r.Y, b, a);                   // 2  H
  fe_add(r.Z, dd, c);                  // 3  G
  fe_sub(r.T, dd, c);                  // 3  F
}
// p - q
TMV_HD void ge_sub(ge_p1p1 &r, const ge_p3 &p, const ge_cached &q) {
  fe a, b, c, dd, t;
  fe_sub(t, p.Y, p.X); fe_mul(a, t, q.YpX);
  fe_add(t, p.Y, p.X); fe_mul(b, t, q.YmX);
  fe_mul(c, p.T, q.T2d);
  fe_mul(dd, p.Z, q.Z);
  fe_add(dd, dd, dd);
  fe_sub(r.X, b, a);
  fe_add(r.Y, b, a);
  fe_sub(r.Z, dd, c);
  fe_add(r.T, dd, c);
}
// mixed add with an affine Niels point (Z = 1)
TMV_HD void ge_madd(ge_p1p1 &r, const ge_p3 &p, const ge_precomp &q) {
  fe a, b, c, dd, t;
  fe_sub(t, p.Y, p.X); fe_mul(a, t, q.ymx);
  fe_add(t, p.Y, p.X); fe_mul(b, t, q.ypx);
  fe_mul(c, p.T, q.xy2d);
  fe_add(dd, p.Z, p.Z);                // 2
  fe_sub(r.X, b, a);
  fe_add(r.Y, b, a);
  fe_add(r.Z, dd, c);
  fe_sub(r.T, dd, c);
}

TMV_HD void ge_p3_neg(ge_p3 &r, const ge_p3 &p) {
  fe_neg(r.X, p.X); r.Y = p.Y; r.Z = p.Z; fe_neg(r.T, p.T);
}

// Every verdict below also requires Z != 0: the complete formulas never give a
// point Z == 0, so only a result never computed (e.g. an unwritten, zeroed
// workspace slot, (0 : 0 : 0 : 0)) has it -- and it would otherwise pass
// X == 0, Y == Z.  A missing write then fails a check instead of passing it.
TMV_HD bool ge_p3_is_identity(const ge_p3 &p) {
  return fe_is_zero(p.X) && fe_eq(p.Y, p.Z) && !fe_is_zero(p.Z);
}

// Cofactored identity test: [8]p == O.
TMV_HD bool ge_p3_is_small_order_or_identity_times8(const ge_p3 &p) {
  ge_p1p1 t;
  ge_p2 q;
  ge_p3_dbl(t, p);
  ge_p1p1_to_p2(q, t);
  ge_p2_dbl(t, q);
  ge_p1p1_to_p2(q, t);
  ge_p2_dbl(t, q);
  ge_p1p1_to_p2(q, t);
  return fe_is_zero(q.X) && fe_eq(q.Y, q.Z) && !fe_is_zero(q.Z);
}

// ZIP-215 lax decoding of an edwards25519 point (crypto/ed25519/ed25519.go:27-29
// options): y is taken mod p (y >= p accepted), x recovered from
// x^2 = (y^2-1)/(d y^2+1); non-square -> reject; x == 0 with sign bit 1 is
// accepted ("negative zero").
TMV_HD bool ge_decode_zip215(ge_p3 &h, const uint32_t w[8]) {
  fe u, v, v3, vxx, chk, x, one;
  fe_from_words(h.Y, w);
  fe_carry(h.Y, h.Y);                  // exact limbs are level 2; bring to 1
  fe_one(h.Z);
  fe_one(one);
  fe_sq(u, h.Y);
  fe_mul(v, u, consts::d());
  fe_sub(u, u, one);                   // u = y^2 - 1      (2)
  fe_add(v, v, one);                   // v = d y^2 + 1    (2)
  fe_sq(v3, v);
  fe_mul(v3, v3, v);                   // v^3
  fe_sq(x, v3);
  fe_mul(x, x, v);                     // v^7
  fe_mul(x, x, u);                     // u v^7
  fe_pow22523(x, x);
  fe_mul(x, x, v3);
  fe_mul(x, x, u);                     // x = u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, x);
  fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u);                 // 3
  if (!fe_is_zero(chk)) {
    fe_add(chk, vxx, u);
    if (!fe_is_zero(chk)) return false;
    fe_mul(x, x, consts::sqrtm1());
  }
  const bool sign = (w[7] >> 31) & 1;
  if (fe_is_negative(x) != sign) fe_neg(x, x);
  h.X = x;
  fe_mul(h.T, h.X, h.Y);
  return true;
}

// ---------------------------------------------------------------- ristretto255
// (crypto/sr25519 -> curve25519-voi primitives/sr25519, go.mod:22)

// (was_square, r): r = sqrt(u/v) or sqrt(i u/v), r non-negative.
TMV_HD bool fe_sqrt_ratio_i(fe &r, const fe &u, const fe &v) {
  fe v3, v7, t, check, nu, nui, rp;
  fe_sq(v3, v);
  fe_mul(v3, v3, v);
  fe_sq(v7, v3);
  fe_mul(v7, v7, v);
  fe_mul(t, u, v7);
  fe_pow22523(t, t);
  fe_mul(t, t, v3);
  fe_mul(r, t, u);
  fe_sq(check, r);
  fe_mul(check, check, v);
  fe_neg(nu, u);
  fe_mul(nui, nu, consts::sqrtm1());
  const bool correct = fe_eq(check, u);
  const bool flipped = fe_eq(check, nu);
  const bool flipped_i = fe_eq(check, nui);
  fe_mul(rp, r, consts::sqrtm1());
  if (flipped || flipped_i) r = rp;
  if (fe_is_negative(r)) fe_neg(r, r);
  return correct || flipped;
}

// Canonical Ristretto255 decoding (non-canonical or negative s, non-square,
// negative t or y == 0 reject).
TMV_HD bool ristretto_decode(ge_p3 &h, const uint32_t w[8]) {
  fe s, ss, u1, u2, u2sq, v, t, I, Dx, Dy, x, y, one;
  fe_from_words(s, w);
  uint32_t chk[8];
  fe_to_words(chk, s);
  bool canon = true;
  for (int i = 0; i < 8; i++) canon = canon && (chk[i] == w[i]);
  if (!canon || (chk[0] & 1)) return false;  // >= p, bit 255 set, or negative
  fe_carry(s, s);
  fe_one(one);
  fe_sq(ss, s);
  fe_sub(u1, one, ss);                 // 2
  fe_add(u2, one, ss);                 // 2
  fe_sq(u2sq, u2);
  fe_sq(t, u1);
  fe_mul(t, t, consts::d());
  fe_neg(t, t);
  fe_sub(v, t, u2sq);                  // -(d u1^2) - u2^2   (2)
  fe_mul(t, v, u2sq);
  const bool ok = fe_sqrt_ratio_i(I, one, t);
  fe_mul(Dx, I, u2);
  fe_mul(Dy, I, Dx);
  fe_mul(Dy, Dy, v);
  fe_add(x, s, s);
  fe_mul(x, x, Dx);
  if (fe_is_negative(x)) fe_neg(x, x);
  fe_mul(y, u1, Dy);
  fe_mul(t, x, y);
  if (!ok || fe_is_negative(t) || fe_is_zero(y)) return false;
  h.X = x; h.Y = y; fe_one(h.Z); h.T = t;
  return true;
}

// Ristretto255 encoding (used by the host-side test factory to make keys and
// signatures; verification never encodes).
TMV_HD void ristretto_encode(uint32_t out[8], const ge_p3 &p) {
  fe u1, u2, t, invsqrt, den1, den2, zinv, ix, iy, ench, X, Y, den_inv, one, s;
  fe_add(t, p.Z, p.Y);
  fe_sub(u1, p.Z, p.Y);
  fe_mul(u1, t, u1);                   // (Z+Y)(Z-Y)
  fe_mul(u2, p.X, p.Y);
  fe_sq(t, u2);
  fe_mul(t, t, u1);
  fe_one(one);
  (void)fe_sqrt_ratio_i(invsqrt, one, t);
  fe_mul(den1, invsqrt, u1);
  fe_mul(den2, invsqrt, u2);
  fe_mul(zinv, den1, den2);
  fe_mul(zinv, zinv, p.T);
  fe_mul(ix, p.X, consts::sqrtm1());
  fe_mul(iy, p.Y, consts::sqrtm1());
  fe_mul(ench, den1, consts::invsqrt_a_minus_d());
  fe_mul(t, p.T, zinv);
  const bool rotate = fe_is_negative(t);
  if (rotate) { X = iy; Y = ix; den_inv = ench; }
  else { X = p.X; Y = p.Y; den_inv = den2; }
  fe_mul(t, X, zinv);
  if (fe_is_negative(t)) fe_neg(Y, Y);
  fe_sub(t, p.Z, Y);
  fe_mul(s, den_inv, t);
  if (fe_is_negative(s)) fe_neg(s, s);
  fe_to_words(out, s);
}

// Ristretto equality: X1 Y2 == Y1 X2 or Y1 Y2 == X1 X2 (and Z1, Z2 != 0).
TMV_HD bool ristretto_equal(const ge_p3 &a, const ge_p3 &b) {
  if (fe_is_zero(a.Z) || fe_is_zero(b.Z)) return false;
  fe l, r;
  fe_mul(l, a.X, b.Y);
  fe_mul(r, a.Y, b.X);
  if (fe_eq(l, r)) return true;
  fe_mul(l, a.Y, b.Y);
  fe_mul(r, a.X, b.X);
  return fe_eq(l, r);
}

// ---------------------------------------------------------------- scalars
// l = 2^252 + 27742317777372353535851937790883648493, little-endian words.
struct scl {
  static TMV_HD uint32_t l(int i) {
    const uint32_t L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u};
    return L[i];
  }
  static TMV_HD uint32_t mu(int i) {  // floor(2^512 / l), 9 words
    const uint32_t M[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                           0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
    return M[i];
  }
};

// s < l ?  (strict canonical scalar, ZIP-215 rule for S)
TMV_HD bool sc_is_canonical(const uint32_t s[8]) {
  for (int i = 7; i >= 0; i--) {
    if (s[i] < scl::l(i)) return true;
    if (s[i] > scl::l(i)) return false;
  }
  return false;
}

// r = x mod l for a 512-bit x (16 little-endian words); Barrett (HAC 14.42)
// with b = 2^32, k = 8.
TMV_HD void sc_reduce512(uint32_t r[8], const uint32_t x[16]) {
  // q2 = floor(x / b^7) * mu ; only words 9..17 (q3) are needed, but the
  // full product keeps the carries exact.
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; i++) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
    const uint64_t a = x[7 + i];
#pragma unroll
    for (int j = 0; j < 9; j++) {
      uint64_t t = a * scl::mu(j) + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  // r2 = (q3 * l) mod b^9
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint64_t carry = 0;
    const uint64_t a = q2[9 + i];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (i + j >= 9) break;
      uint64_t t = a * scl::l(j) + r2[i + j] + carry;
      r2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    if (i == 0) r2[8] = (uint32_t)carry;  // rows i >= 1 carry past word 8
  }
  // t = (x mod b^9) - r2 mod b^9
  uint32_t t[9];
  int64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    int64_t d = (int64_t)x[i] - r2[i] + borrow;
    t[i] = (uint32_t)d;
    borrow = d >> 32;  // 0 or -1
  }
  // at most two subtractions of l
  for (int it = 0; it < 2; it++) {
    bool ge = t[8] != 0;
    if (!ge) {
      ge = true;
      for (int i = 7; i >= 0; i--) {
        if (t[i] > scl::l(i)) { ge = true; break; }
        if (t[i] < scl::l(i)) { ge = false; break; }
      }
    }
    if (ge) {
      int64_t b = 0;
#pragma unroll
      for (int i = 0; i < 9; i++) {
        int64_t d = (int64_t)t[i] - (i < 8 ? scl::l(i) : 0u) + b;
        t[i] = (uint32_t)d;
        b = d >> 32;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = t[i];
}

// Signed radix-16 recoding: 64 digits in [-8, 8], sum e_i 16^i = s.
// Requires s < 2^255 (true for s < l and any reduced scalar).
TMV_HD void sc_signed_radix16(int8_t e[64], const uint32_t s[8]) {
#pragma unroll
  for (int i = 0; i < 64; i++) e[i] = (int8_t)((s[i >> 3] >> (4 * (i & 7))) & 15);
  int carry = 0;
#pragma unroll
  for (int i = 0; i < 63; i++) {
    e[i] = (int8_t)(e[i] + carry);
    carry = (e[i] + 8) >> 4;
    e[i] = (int8_t)(e[i] - carry * 16);
  }
  e[63] = (int8_t)(e[63] + carry);
}

}  // namespace tmv
