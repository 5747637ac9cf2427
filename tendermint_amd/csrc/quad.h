// Quad-lane edwards25519 arithmetic: one point spread over the 4 lanes of a
// DPP quad (lane c holds coordinate c), so a point doubling costs each lane
// one squaring + one multiply and an addition two multiplies — 4-way
// parallel twisted-Edwards formulas (add-2008-hwcd-3 / dbl-2008-hwcd, a=-1)
// with the linear glue done by quad_perm DPP moves (free cross-lane reads
// inside a quad, no LDS).  Used by the latency kernel k_ed25519_verify_quad.
//
// Lane layouts (c = lane & 3):
//   P3Q      (X, Y, Z, T)                 extended point
//   P1P1R    (E, G, F, H)                 completed point (x = E/G, y = H/F);
//            the older glue (TMV_QUAD_GLUE=0) uses P1P1Q (E, H, G, F)
//   CachedQ  (Y-X, Y+X, 2dT, Z)           addend; B-table entries have Z = 1
// Every branch below is quad-uniform or lane-select only: DPP requires all
// four lanes of a quad to be active.
#pragma once
#include "curve25519.h"

namespace tmv {
namespace quad {

constexpr int qp(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }

template <int CTRL>
TMV_DEV void fe_dpp(fe &h, const fe &f) {
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = __builtin_amdgcn_mov_dpp(f.v[i], CTRL, 0xF, 0xF, true);
}

// h = s * f for a per-lane s in {-1, 0, +1}
TMV_DEV void fe_signed(fe &h, const fe &f, int s) {
  const int32_t m = s < 0 ? -1 : 0;
  const int32_t keep = s != 0 ? -1 : 0;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = ((f.v[i] ^ m) - m) & keep;
}

// Carry of the quad formulas' products: the two-round parallel form
// (TMV_QUAD_PCARRY=1) or the twelve-step chain (0).
#ifndef TMV_QUAD_PCARRY
#define TMV_QUAD_PCARRY 0
#endif
TMV_DEV void qcarry(fe &h, int64_t c[10]) {
#if TMV_QUAD_PCARRY
  fe_carry_biased_par(h, c);
#else
  fe_carry_biased(h, c);
#endif
}
TMV_DEV void qmul(fe &h, const fe &f, const fe &g) {
#if TMV_QUAD_PCARRY
  fe_mul_par(h, f, g);
#else
  fe_mul(h, f, g);
#endif
}

// h = f^2 << sh (sh in {0, 1}, per lane), carried to level 1
#ifndef TMV_SQ_BIAS
#define TMV_SQ_BIAS 1
#endif
TMV_DEV void fe_sq_shift(fe &h, const fe &f, int sh) {
#if TMV_SQ_BIAS
  // 2^sh f^2 with the left operands taken from f << sh, each column started
  // at its carry bias by its first product (mad_bias, as fe_sq): no 64-bit
  // shift of the columns and no bias adds before the carry
  int32_t g[10], g2[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g[i] = (int32_t)((uint32_t)f.v[i] << sh);
    g2[i] = 2 * g[i];
    f19[i] = mul19(f.v[i]);
  }
  int64_t c[10];
  bool started[10] = {false, false, false, false, false, false, false, false, false, false};
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      const int oddodd = (i & 1) && (j & 1);
      int32_t a = (i == j) ? g[i] : g2[i];
      if (oddodd) a = 2 * a;
      const int k = i + j < 10 ? i + j : i + j - 10;
      const int32_t b = i + j < 10 ? f.v[j] : f19[j];
      if (!started[k]) { c[k] = mad_bias(a, b, k); started[k] = true; }
      else c[k] = mad_acc(a, b, c[k]);
    }
  }
  qcarry(h, c);
#else
  int32_t f2[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; i++) { f2[i] = 2 * f.v[i]; f19[i] = mul19(f.v[i]); }
  int64_t c[10];
#pragma unroll
  for (int k = 0; k < 10; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
#pragma unroll
    for (int j = i; j < 10; j++) {
      const int oddodd = (i & 1) && (j & 1);
      int32_t a = (i == j) ? f.v[i] : f2[i];
      if (oddodd) a = 2 * a;
      if (i + j < 10) c[i + j] += (int64_t)a * f.v[j];
      else            c[i + j - 10] += (int64_t)a * f19[j];
    }
  }
#pragma unroll
  for (int k = 0; k < 10; k++) c[k] = c[k] << sh;
  fe_carry_wide(h, c);
#endif
}

TMV_DEV int lane4() { return (int)(threadIdx.x & 3); }

TMV_DEV void p3_identity(fe &p) {
  const int c = lane4();
  fe_zero(p);
  p.v[0] = (c == 1 || c == 2) ? 1 : 0;
}
TMV_DEV void cached_identity(fe &q) {
  const int c = lane4();
  fe_zero(q);
  q.v[0] = (c == 2) ? 0 : 1;
}

// Linear glue with fused DPP operands (TMV_QUAD_GLUE, default): every
// cross-lane read feeds a VOP2 op directly (v_and / v_xor / v_add _dpp), and a
// per-lane sign is an XOR with -1 completed by one +1 per negated term in the
// limb's final add, so a limb of the doubling's glue is 7 instructions and of
// the addition's 8 (the selects / negations of the older form below took
// about 20 and 14; the values are identical).
#ifndef TMV_QUAD_GLUE
#define TMV_QUAD_GLUE 1
#endif
template <int CTRL>
TMV_DEV int32_t dpp(int32_t x) { return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true); }
// A lane mask (0 / -1) the compiler cannot see through: an AND with a mask it
// knows came from a compare becomes a v_cndmask (VOP3, no DPP operand), so
// the DPP read would stay a separate v_mov_b32_dpp
TMV_DEV int32_t lane_mask(bool b) {
  int32_t m = b ? -1 : 0;
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(m));
#endif
  return m;
}

#if TMV_QUAD_GLUE
// Completed points in the rotated layout P1P1R (E, G, F, H): each lane owns
// one factor of its P3Q product (X = E F, Y = G H, Z = F G, T = H E -- the
// products walk the cycle E-F-G-H), so p1p1_to_p3 reads one operand across
// lanes instead of two (10 DPP moves per conversion instead of 20; the
// multiply-add takes no DPP operand).

// P1P1R -> P3Q: lane c multiplies its own value by lane (2, 3, 1, 0)[c]'s
TMV_DEV void p1p1_to_p3(fe &p, const fe &r) {
  fe o2;
  fe_dpp<qp(2, 3, 1, 0)>(o2, r);
  qmul(p, r, o2);
}

// P3Q -> P1P1R doubling: squares of (X, Y, Z, X+Y) with 2Z^2 on lane 2, then
// E = S3 - S1 - S0, G = S1 - S0, F = S2 - S1 + S0, H = S1 + S0 (all negated
// relative to dbl-2008-hwcd, same projective point).
TMV_DEV void dbl(fe &r, const fe &p) {
  const int c = lane4();
  const int32_t k3 = lane_mask(c == 3);
  fe s;
#pragma unroll
  for (int i = 0; i < 10; i++)  // X, Y, Z, X + Y (level 2)
    s.v[i] = dpp<qp(0, 1, 2, 0)>(p.v[i]) + (dpp<qp(1, 1, 1, 1)>(p.v[i]) & k3);
  fe S;
  fe_sq_shift(S, s, c == 2 ? 1 : 0);
  // lane: 0: S3 - S1 - S0, 1: S1 - S0, 2: S2 - S1 + S0, 3: S1 + S0
  const int32_t kb = lane_mask(c == 0 || c == 2);  // base S3 (lane 0) / S2 (lane 2)
  const int32_t m1 = (c == 0 || c == 2) ? -1 : 0;  // -S1
  const int32_t m0 = (c == 0 || c == 1) ? -1 : 0;  // -S0
  const int32_t corr = -(m1 + m0);
#pragma unroll
  for (int i = 0; i < 10; i++)
    r.v[i] = (dpp<qp(3, 3, 2, 2)>(S.v[i]) & kb) + (dpp<qp(1, 1, 1, 1)>(S.v[i]) ^ m1) +
             (dpp<qp(0, 0, 0, 0)>(S.v[i]) ^ m0) + corr;  // level 3
}

// (Y-X, Y+X, T, Z) of a P3Q point (level 2): the first half of add / to_cached
TMV_DEV void ymx_ypx(fe &t, const fe &p) {
  const int c = lane4();
  const int32_t k = lane_mask(c <= 1), m = c == 0 ? -1 : 0, corr = c == 0 ? 1 : 0;
#pragma unroll
  for (int i = 0; i < 10; i++) t.v[i] = dpp<qp(1, 1, 3, 2)>(p.v[i]) + (((dpp<qp(0, 0, 0, 0)>(p.v[i]) & k) ^ m) + corr);
}

// P3Q + CachedQ -> P1P1R
TMV_DEV void add(fe &r, const fe &p, const fe &q) {
  const int c = lane4();
  fe op1, M;
  ymx_ypx(op1, p);                          // Y-X, Y+X, T, Z
  qmul(M, op1, q);                        // A, B, C, D
  const int32_t k2 = lane_mask(c == 1 || c == 2);  // 2D on lanes 1, 2
  const int32_t mv = (c == 0 || c == 2) ? -1 : 0, corr = -mv;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const int32_t u = dpp<qp(1, 3, 3, 1)>(M.v[i]) + (dpp<qp(1, 3, 3, 1)>(M.v[i]) & k2);  // B, 2D, 2D, B
    r.v[i] = u + (dpp<qp(0, 2, 2, 0)>(M.v[i]) ^ mv) + corr;  // B-A, 2D+C, 2D-C, B+A (level 3)
  }
}

// q -> -q in CachedQ when neg (quad-uniform flag): swap lanes 0/1, negate lane 2
TMV_DEV void cached_cneg(fe &q, bool neg) {
  const int c = lane4();
  const int32_t m = c == 2 ? -1 : 0, corr = -m;
  fe t;
#pragma unroll
  for (int i = 0; i < 10; i++) t.v[i] = (dpp<qp(1, 0, 2, 3)>(q.v[i]) ^ m) + corr;
  fe_cmov(q, t, neg);
}

// P3Q -> CachedQ: (Y-X, Y+X, 2dT, Z)
TMV_DEV void to_cached(fe &q, const fe &p) {
  const int c = lane4();
  fe t, k;
  ymx_ypx(t, p);
  if (c == 2) {
    k = consts::d2();
  } else {
    fe_one(k);
  }
  qmul(q, t, k);                          // lane 2 scales by 2d; others re-carry
}
#else
// (older glue, P1P1Q layout (E, H, G, F))
// P1P1Q -> P3Q: (E F, H G, G F, E H)
TMV_DEV void p1p1_to_p3(fe &p, const fe &r) {
  fe o1, o2;
  fe_dpp<qp(0, 1, 2, 0)>(o1, r);
  fe_dpp<qp(3, 2, 3, 1)>(o2, r);
  qmul(p, o1, o2);
}

// P3Q -> P1P1Q doubling: squares of (X, Y, Z, X+Y) with 2Z^2 on lane 2, then
// E = S3 - S1 - S0, H = S1 + S0, G = S1 - S0, F = S2 - S1 + S0 (all negated
// relative to dbl-2008-hwcd, same projective point).
TMV_DEV void dbl(fe &r, const fe &p) {
  const int c = lane4();
  fe a, b, s;
  fe_dpp<qp(0, 1, 2, 0)>(a, p);
  fe_dpp<qp(1, 1, 1, 1)>(b, p);
  fe_signed(b, b, c == 3 ? 1 : 0);
  fe_add(s, a, b);                          // lane 3: X + Y (level 2)
  fe S;
  fe_sq_shift(S, s, c == 2 ? 1 : 0);
  fe base, s1, s0;
  fe_dpp<qp(3, 3, 2, 2)>(base, S);
  fe_signed(base, base, (c == 0 || c == 3) ? 1 : 0);
  fe_dpp<qp(1, 1, 1, 1)>(s1, S);
  fe_signed(s1, s1, (c == 0 || c == 3) ? -1 : 1);
  fe_dpp<qp(0, 0, 0, 0)>(s0, S);
  fe_signed(s0, s0, (c == 0 || c == 2) ? -1 : 1);
  fe_add(r, base, s1);
  fe_add(r, r, s0);                         // level 3
}

// P3Q + CachedQ -> P1P1Q
TMV_DEV void add(fe &r, const fe &p, const fe &q) {
  const int c = lane4();
  fe a, b, op1, M;
  fe_dpp<qp(1, 1, 3, 2)>(a, p);             // Y, Y, T, Z
  fe_dpp<qp(0, 0, 0, 0)>(b, p);             // X
  fe_signed(b, b, c == 0 ? -1 : (c == 1 ? 1 : 0));
  fe_add(op1, a, b);                        // Y-X, Y+X, T, Z (level 2)
  qmul(M, op1, q);                        // A, B, C, D
  fe u, v;
  fe_dpp<qp(1, 1, 3, 3)>(u, M);             // B, B, D, D
  fe_dpp<qp(0, 0, 2, 2)>(v, M);             // A, A, C, C
  if (c >= 2) fe_add(u, u, u);              // 2D (lane select, no DPP inside)
  fe_signed(v, v, (c == 0 || c == 3) ? -1 : 1);
  fe_add(r, u, v);                          // B-A, B+A, 2D+C, 2D-C (level 3)
}

// q -> -q in CachedQ when neg (quad-uniform flag): swap lanes 0/1, negate lane 2
TMV_DEV void cached_cneg(fe &q, bool neg) {
  const int c = lane4();
  fe t;
  fe_dpp<qp(1, 0, 2, 3)>(t, q);
  fe_signed(t, t, c == 2 ? -1 : 1);
  fe_cmov(q, t, neg);
}

// P3Q -> CachedQ: (Y-X, Y+X, 2dT, Z)
TMV_DEV void to_cached(fe &q, const fe &p) {
  const int c = lane4();
  fe a, b, t, k;
  fe_dpp<qp(1, 1, 3, 2)>(a, p);
  fe_dpp<qp(0, 0, 0, 0)>(b, p);
  fe_signed(b, b, c == 0 ? -1 : (c == 1 ? 1 : 0));
  fe_add(t, a, b);
  if (c == 2) {
    k = consts::d2();
  } else {
    fe_one(k);
  }
  qmul(q, t, k);                          // lane 2 scales by 2d; others re-carry
}

#endif

// [8]P == O on a P3Q point: X == 0 and Y == Z.  Returns the quad verdict on
// every lane of the quad.
TMV_DEV bool is_identity_times8(const fe &p) {
  const int c = lane4();
  fe q = p, r;
  for (int i = 0; i < 3; i++) {
    dbl(r, q);
    p1p1_to_p3(q, r);
  }
  fe z;
  fe_dpp<qp(2, 2, 2, 2)>(z, q);
  fe_signed(z, z, c == 1 ? 1 : 0);
  fe d;
  fe_sub(d, q, z);                          // lane 0: X, lane 1: Y - Z, lane 2: Z
  const int zero = fe_is_zero(d) ? 1 : 0;
  const int z0 = __builtin_amdgcn_mov_dpp(zero, qp(0, 0, 0, 0), 0xF, 0xF, false);
  const int z1 = __builtin_amdgcn_mov_dpp(zero, qp(1, 1, 1, 1), 0xF, 0xF, false);
  const int z2 = __builtin_amdgcn_mov_dpp(zero, qp(2, 2, 2, 2), 0xF, 0xF, false);
  return (z0 & z1 & (z2 ^ 1)) != 0;         // Z == 0 only for a never-computed point (ge_p3_is_identity)
}

// Ristretto identity of a P3Q point (equal to O modulo the 4-torsion: X == 0
// or Y == 0).  Quad verdict on every lane.
TMV_DEV bool is_ristretto_identity(const fe &p) {
  const int zero = fe_is_zero(p) ? 1 : 0;  // lane 0: X, lane 1: Y, lane 2: Z
  const int z0 = __builtin_amdgcn_mov_dpp(zero, qp(0, 0, 0, 0), 0xF, 0xF, false);
  const int z1 = __builtin_amdgcn_mov_dpp(zero, qp(1, 1, 1, 1), 0xF, 0xF, false);
  const int z2 = __builtin_amdgcn_mov_dpp(zero, qp(2, 2, 2, 2), 0xF, 0xF, false);
  return ((z0 | z1) & (z2 ^ 1)) != 0;
}

// Z1 != 0 and Z2 != 0 (lane 2 of each P3Q point): the equalities below hold
// for a never-computed (0 : 0 : 0 : 0) point against anything.  Quad verdict.
TMV_DEV bool both_z_nonzero(const fe &a, const fe &b) {
  const int nz = (fe_is_zero(a) || fe_is_zero(b)) ? 0 : 1;  // lane 2: Z1, Z2
  return __builtin_amdgcn_mov_dpp(nz, qp(2, 2, 2, 2), 0xF, 0xF, false) != 0;
}

// Equality of two P3Q points: X1 Z2 == X2 Z1 and Y1 Z2 == Y2 Z1.  Quad
// verdict on every lane.
TMV_DEV bool p3_equal(const fe &a, const fe &b) {
  const int c = lane4();
  fe ta, tb, za, zb, o1, o2, p, d;
  fe_dpp<qp(0, 1, 0, 1)>(ta, a);            // X1, Y1, X1, Y1
  fe_dpp<qp(0, 1, 0, 1)>(tb, b);            // X2, Y2, X2, Y2
  fe_dpp<qp(2, 2, 2, 2)>(za, a);            // Z1
  fe_dpp<qp(2, 2, 2, 2)>(zb, b);            // Z2
  o1 = ta;
  fe_cmov(o1, tb, c >= 2);                  // X1, Y1, X2, Y2
  o2 = zb;
  fe_cmov(o2, za, c >= 2);                  // Z2, Z2, Z1, Z1
  qmul(p, o1, o2);
  fe_dpp<qp(2, 3, 0, 1)>(d, p);
  fe_sub(d, p, d);                          // lane 0: X1 Z2 - X2 Z1, lane 1: Y1 Z2 - Y2 Z1
  const int zero = fe_is_zero(d) ? 1 : 0;
  const int z0 = __builtin_amdgcn_mov_dpp(zero, qp(0, 0, 0, 0), 0xF, 0xF, false);
  const int z1 = __builtin_amdgcn_mov_dpp(zero, qp(1, 1, 1, 1), 0xF, 0xF, false);
  return (z0 & z1) != 0 && both_z_nonzero(a, b);
}

// Ristretto equality of two P3Q points a (acc) and b (R):
// X1 Y2 == Y1 X2 or Y1 Y2 == X1 X2.  Quad verdict on every lane.
TMV_DEV bool ristretto_equal(const fe &a, const fe &b) {
  fe o1, o2, p, d;
  fe_dpp<qp(0, 1, 1, 0)>(o1, a);            // X1, Y1, Y1, X1
  fe_dpp<qp(1, 0, 1, 0)>(o2, b);            // Y2, X2, Y2, X2
  qmul(p, o1, o2);
  fe_dpp<qp(1, 1, 3, 3)>(d, p);
  fe_sub(d, p, d);                          // lane 0: X1Y2 - Y1X2, lane 2: Y1Y2 - X1X2
  const int zero = fe_is_zero(d) ? 1 : 0;
  const int z0 = __builtin_amdgcn_mov_dpp(zero, qp(0, 0, 0, 0), 0xF, 0xF, false);
  const int z2 = __builtin_amdgcn_mov_dpp(zero, qp(2, 2, 2, 2), 0xF, 0xF, false);
  return (z0 | z2) != 0 && both_z_nonzero(a, b);
}

}  // namespace quad
}  // namespace tmv
