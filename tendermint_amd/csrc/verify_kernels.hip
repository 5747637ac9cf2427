// MI355X (gfx950) verification kernels.
//
// k_ed25519_verify: one lane per signature, full ZIP-215 verification
// (SHA-512 challenge, scalar reduction, lax decompression of A and R,
// [S]B by a 32x8 base-point comb in global memory, [k]A by signed radix-16
// windows, cofactored identity test).  All integer VALU work — the
// 32x32->64 multiply-adds of the radix-2^25.5 field dominate (see DESIGN.md
// for the roofline), so there is no MFMA or LDS tiling here.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include "ed25519_core.h"
#include "quad.h"
#include "sr25519_core.h"
#include "verify_kernels.h"
#include "kernel_util.h"
#include "comb.h"
#include "halfscalar.h"
#include "ktimer.h"

namespace tmv {

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
// Latency path: prep kernel (one lane per point / hash) + quad kernel (4
// lanes per signature), templated on the scheme (SR = false: ed25519 ZIP-215,
// SR = true: sr25519).  Entries may be addressed through an index list
// (mixed batches): entry e of this launch is original signature idx[e], and
// the entry count may live in device memory (count_ptr) so the partition
// kernel never has to round-trip to the host.
//
// k_prep stores -A in P3Q layout, R (ed25519: CachedQ; sr25519: P3Q) and k;
// decode failures go to flags (4 bytes per entry: A ok, R ok, s ok, -).

// Decode blocks (lanes [0, m) decode A, [m, 2m) decode R) and hash blocks
// (one lane per entry: SHA-512 + Barrett, or the merlin transcript).
template <bool SR>
__device__ __forceinline__ void prep_decode_block(uint32_t bx, const uint8_t *__restrict__ pk,
                                                  const uint8_t *__restrict__ sig, const uint32_t *__restrict__ idx,
                                                  const uint32_t *count_ptr, uint32_t n, Ed25519Work w, int aligned) {
  const uint32_t m = entry_count(count_ptr, n);
  const uint32_t j = bx * blockDim.x + threadIdx.x;
  if (j >= 2 * m) return;
  const bool isA = j < m;
  const uint32_t e = isA ? j : j - m;
  const uint32_t i = idx ? idx[e] : e;
  uint32_t p_w[8];
  const uint8_t *src = isA ? pk + 32ull * i : sig + 64ull * i;
  if (aligned) load_words_aligned(p_w, src);
  else load_words_unaligned(p_w, src);
  ge_p3 P;
  bool ok;
  if (SR) ok = ristretto_decode(P, p_w);
  else ok = ge_decode_zip215(P, p_w);
  if (!ok) ge_p3_identity(P);  // keep limbs bounded; the flag rejects the entry
  w.flags[4 * e + (isA ? 0 : 1)] = ok ? 1 : 0;
  if (w.niels) {  // -P in affine Niels form for the batch equation (Z = 1)
    niels_pt np;
    fe t;
    fe_sub(t, P.Y, P.X); fe_carry(np.ypx, t);
    fe_add(t, P.Y, P.X); fe_carry(np.ymx, t);
    fe_mul(t, P.T, consts::d2()); fe_neg(np.xy2d, t);
    np.pad[0] = np.pad[1] = 0;
    niels_store(w.niels, 2ull * e + (isA ? 1 : 0), np);
  }
  fe *dst = (isA ? w.negA : w.Rc) + 4ull * e;
  if (isA || SR) {
    fe t;
    if (isA) fe_neg(t, P.X); else t = P.X;
    dst[0] = t;
    dst[1] = P.Y;
    fe_one(t); dst[2] = t;
    if (isA) fe_neg(t, P.T); else t = P.T;
    dst[3] = t;
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

template <bool SR>
__device__ __forceinline__ void prep_hash_block(uint32_t bx, const uint8_t *__restrict__ pk,
                                                const uint8_t *__restrict__ sig, const uint8_t *__restrict__ msg,
                                                const uint32_t *__restrict__ msg_off, const uint32_t *__restrict__ idx,
                                                const uint32_t *count_ptr, uint32_t n, Ed25519Work w,
                                                const strobe_t *__restrict__ prefix, int aligned) {
  const uint32_t m = entry_count(count_ptr, n);
  const uint32_t e = bx * blockDim.x + threadIdx.x;
  if (e >= m) return;
  const uint32_t i = idx ? idx[e] : e;
  uint32_t a_w[8], r_w[8];
  if (aligned) {
    load_words_aligned(a_w, pk + 32ull * i);
    load_words_aligned(r_w, sig + 64ull * i);
  } else {
    load_words_unaligned(a_w, pk + 32ull * i);
    load_words_unaligned(r_w, sig + 64ull * i);
  }
  uint32_t k[8];
  const uint32_t o0 = msg_off[i], o1 = msg_off[i + 1];
  if constexpr (SR) {
    __shared__ uint64_t strobe_lanes[25][kVerifyBlock];
    sr25519_challenge_lds<kVerifyBlock>(k, *prefix, &strobe_lanes[0][threadIdx.x], a_w, r_w, msg + o0, o1 - o0);
  } else {
    uint32_t h[16];
    sha512_pq_msg(h, r_w, a_w, msg + o0, o1 - o0);
    sc_reduce512(k, h);
  }
  uint4 *kd = reinterpret_cast<uint4 *>(w.k + 8ull * e);
  kd[0] = make_uint4(k[0], k[1], k[2], k[3]);
  kd[1] = make_uint4(k[4], k[5], k[6], k[7]);
  if (w.hs) {  // per-entry pipeline: the half-size scalars, once per entry
    uint32_t u[4], v[4];
    bool neg = false;
    const bool fast = half::reduce(u, neg, v, k);
    uint4 *hd = reinterpret_cast<uint4 *>(w.hs + 12ull * e);
    hd[0] = make_uint4(u[0], u[1], u[2], u[3]);
    hd[1] = make_uint4(v[0], v[1], v[2], v[3]);
    hd[2] = make_uint4((fast ? 1u : 0u) | (neg ? 2u : 0u), 0u, 0u, 0u);
  }
}

// Both halves of the prep in one launch: blocks [0, dblocks) decode, the
// rest hash, so the hash does not wait behind the decode's sqrt chains
// (round 2, against two kernels: one 10k batch 1.047 -> 0.987 ms through the
// batch equation, 0.546 -> 0.491 ms per entry).
template <bool SR>
__global__ void __launch_bounds__(kVerifyBlock)
k_prep_fused(const uint8_t *__restrict__ pk, const uint8_t *__restrict__ sig, const uint8_t *__restrict__ msg,
             const uint32_t *__restrict__ msg_off, const uint32_t *__restrict__ idx, const uint32_t *count_ptr,
             uint32_t n, Ed25519Work w, const strobe_t *__restrict__ prefix, int aligned, uint32_t dblocks) {
  if (blockIdx.x < dblocks) prep_decode_block<SR>(blockIdx.x, pk, sig, idx, count_ptr, n, w, aligned);
  else prep_hash_block<SR>(blockIdx.x - dblocks, pk, sig, msg, msg_off, idx, count_ptr, n, w, prefix, aligned);
}

constexpr int kQuadSigs = kQuadBlock / 4;

// Digits of one quad's scalars in LDS: v (the -A scalar, radix 16: 32
// digits, 64 on the slow path), b (the B scalar, radix 256: 32 digits), u
// (the -R scalar, radix 16: 32 digits).
constexpr int kDigV = 0, kDigB = 64, kDigU = 96, kDigBytes = 128;

// (m+1) P, m < 8, in CachedQ layout, for a P3Q point P (one doubling, six
// additions; tab[4 m + c] is lane c's coordinate)
TMV_DEV void quad_multiples(fe *tab, const fe &P) {
  const int c = threadIdx.x & 3;
  fe r, Pm, Q, Q0;
  quad::to_cached(Q0, P);
  tab[0 * 4 + c] = Q0;
  quad::dbl(r, P);
  quad::p1p1_to_p3(Pm, r);
  quad::to_cached(Q, Pm);
  tab[1 * 4 + c] = Q;
  for (int t = 2; t < 8; t++) {
    quad::add(r, Pm, Q0);
    quad::p1p1_to_p3(Pm, r);
    quad::to_cached(Q, Pm);
    tab[t * 4 + c] = Q;
  }
}

// -R in P3Q layout from the prep's R: sr25519 keeps R itself in P3Q (negate
// X and T); ed25519 keeps its CachedQ (Y-X, Y+X, 2dT, Z), from which
// (-2X, 2Y, 2Z, -2T) -- the same projective point -- is one multiply per
// lane: lanes 0 / 1 re-carry (Y-X) -+ (Y+X), lane 2 doubles Z, lane 3
// scales 2dT by -1/d.
template <bool SR>
TMV_DEV void neg_r_p3(fe &P, const fe &Rc) {
  const int c = threadIdx.x & 3;
  if (SR) {
    if (c == 0 || c == 3) fe_neg(P, Rc);
    else P = Rc;
    return;
  }
  fe o, t, K;
  quad::fe_dpp<quad::qp(1, 0, 3, 2)>(o, Rc);  // lane 0 <- Y+X, 1 <- Y-X, 2 <- Z, 3 <- 2dT
  if (c == 0) fe_sub(t, Rc, o);
  else if (c == 1) fe_add(t, Rc, o);
  else t = o;
  if (c == 3) {
    const uint32_t w[8] = {0x323607aau, 0xda1f0d89u, 0xbd86abd1u, 0xf4a22967u,
                           0x32463099u, 0xd4e9deebu, 0xeb2a31bcu, 0x3f6f812du};  // -1/d mod p
    fe_from_words(K, w);
  } else {
    fe_zero(K);
    K.v[0] = c == 2 ? 2 : 1;
  }
  quad::qmul(P, t, K);
}

// k_verify_quad: one signature per quad, with half-size scalars
// (halfscalar.h): every lane reduces k to (u, v), v == u k (mod l), |u|, v <
// 2^127, and b = |u| s mod l, then the quad evaluates
//   acc = sum over 32 signed radix-16 windows of 16 acc + v_i(-A) + u_i(-R)
//         [+ b_j B + b_(j+16) [2^128]B on even windows, radix-256 digits of b
//          against the 128-entry tables of B and [2^128]B multiples]
// (Straus, 124 shared doublings; the B and R terms negated when u < 0) and
//   ed25519: [8] acc == O       (ZIP-215 cofactored)
//   sr25519: acc in E[4]        (Ristretto identity)
// -- the same validity as [8]([s]B - R - [k]A) == O / Ristretto equality for
// every input (halfscalar.h).  An entry whose reduction does not finish
// (quotient >= 2^31, ~2^-24 of hash-derived k) or every entry when half_on
// == 0 takes the full scalars (u = 1, v = k, b = s: 64 windows, 252
// doublings -- the check of rounds 1-4).  Writes out[i] (ed25519 1/0;
// sr25519 1/0/-1/-2 as int8).
// GT: the 8-entry tables of -A and -R live in a global scratch (w.tabA,
// L2-resident while the wave runs) instead of LDS (40 KB per wave), so LDS
// does not cap residency; each window's entries are loaded before its four
// doublings, like the B entries.
// One 16-entry block (blk) of k_verify_quad; every return before the
// __syncthreads is block-uniform except the passing-group branch, which
// k_verify_quad_list never takes.
template <bool SR, bool GT>
__device__ __forceinline__ void quad_block(uint32_t blk, fe *tab_lds, int8_t (*dig)[kDigBytes],
                                           const uint8_t *__restrict__ sig, const uint32_t *__restrict__ idx,
                                           const uint32_t *count_ptr, uint32_t n, const Ed25519Work &w,
                                           const fe *__restrict__ btab_q, uint8_t *__restrict__ out, int aligned,
                                           const uint8_t *__restrict__ group_ok, uint32_t group_log2,
                                           const uint8_t *__restrict__ sub_ok,
                                           const uint32_t *__restrict__ fail_list,
                                           const uint32_t *__restrict__ fail_count,
                                           const uint32_t *__restrict__ fb_list, uint32_t nl, int half_on) {
  const uint32_t m = entry_count(count_ptr, n);
  const int c = threadIdx.x & 3;
  const int q = threadIdx.x >> 2;
  // Entry list (fb_list, the located fallback): quad q of block b verifies
  // entry fb_list[16 b + q].  Compacted fallback (fail_list): block b covers
  // the b-th 16-entry block of the failing groups k_msm_horner listed.  In
  // both, every other entry already holds its pre-check status (written by
  // k_msm_sort).  Otherwise block b covers entries [16 b, 16 b + 16).
  uint32_t b0 = 0, e;
  bool live;
  if (fb_list) {
    if (blk * kQuadSigs >= nl) return;  // block-uniform
    const uint32_t t = blk * kQuadSigs + q;
    live = t < nl;
    e = fb_list[live ? t : nl - 1];
  } else {
    if (fail_list) {
      const uint32_t per_log2 = group_log2 - 4;  // 16-entry blocks per group
      if (blk >= (*fail_count << per_log2)) return;  // block-uniform
      b0 = (fail_list[blk >> per_log2] << group_log2) + ((blk & ((1u << per_log2) - 1)) << 4);
    } else {
      b0 = blk * kQuadSigs;
    }
    if (b0 >= m) return;  // block-uniform
    const uint32_t raw = b0 + q;
    live = raw < m;
    e = live ? raw : m - 1;
  }
  const uint32_t i = idx ? idx[e] : e;
  // Batch equation held for this block's group (groups are >= 32 entries, so
  // the test is block-uniform): every entry that passed decoding and the S
  // check is valid; the rest keep their pre-check status.
  // With the sub-group verdicts (k_msm_subcheck) a block of a failing group
  // passes when every sub-group it covers passed.
  bool pass = false;
  if (group_ok && !fb_list) {
    pass = !fail_list && group_ok[b0 >> group_log2];
    if (!pass && sub_ok) {
      pass = true;
      for (uint32_t s = b0 >> kSubGroupLog2; s <= (b0 + kQuadSigs - 1) >> kSubGroupLog2; s++) pass = pass && sub_ok[s];
    }
  }
  if (pass) {
    if (!live || c != 0) return;
    uint32_t s_raw[8], s_w[8];
    if (aligned) load_words_aligned(s_raw, sig + 64ull * i + 32);
    else load_words_unaligned(s_raw, sig + 64ull * i + 32);
    bool s_ok;
    if (SR) {
      s_ok = sr25519_decode_s(s_w, s_raw);
    } else {
      s_ok = sc_is_canonical(s_raw);
    }
    const bool a_ok = w.flags[4 * e] != 0;
    const bool r_ok = w.flags[4 * e + 1] != 0;
    const int status = SR ? (!a_ok ? -1 : (!s_ok ? -2 : (r_ok ? 1 : 0))) : ((a_ok && r_ok && s_ok) ? 1 : 0);
    out[i] = (uint8_t)(int8_t)status;
    return;
  }

  uint32_t s_raw[8], s_w[8];
  if (aligned) load_words_aligned(s_raw, sig + 64ull * i + 32);
  else load_words_unaligned(s_raw, sig + 64ull * i + 32);
  bool s_ok;
  if (SR) {
    s_ok = sr25519_decode_s(s_w, s_raw);
  } else {
#pragma unroll
    for (int t = 0; t < 8; t++) s_w[t] = s_raw[t];
    s_ok = sc_is_canonical(s_w);
  }
  if (!s_ok) s_w[7] &= 0x0fffffffu;  // keep the recoding in range; entry is rejected anyway
  bool fast, neg_u;
  {
    uint32_t k_w[8];
    const uint4 *kp = reinterpret_cast<const uint4 *>(w.k + 8ull * e);
    const uint4 k0 = kp[0], k1 = kp[1];
    k_w[0] = k0.x; k_w[1] = k0.y; k_w[2] = k0.z; k_w[3] = k0.w;
    k_w[4] = k1.x; k_w[5] = k1.y; k_w[6] = k1.z; k_w[7] = k1.w;
    // every lane of the quad reduces the same k (no exchange needed); lane 0
    // recodes v, lane 1 b, lane 2 u
    half::Scalars sc;
    if (half_on == 1 && w.hs) {  // reduced once by the prep's hash lane
      const uint4 *hp = reinterpret_cast<const uint4 *>(w.hs + 12ull * e);
      const uint4 hu = hp[0], hv = hp[1], hf = hp[2];
      const uint32_t u4[4] = {hu.x, hu.y, hu.z, hu.w}, v4[4] = {hv.x, hv.y, hv.z, hv.w};
      half::scalars_from(sc, u4, (hf.x & 2u) != 0, v4, (hf.x & 1u) != 0, k_w, s_w);
    } else if (half_on == 1 || (half_on == 2 && e % 3 != 0)) {  // 2 (tests): every third entry on the full-k path
      half::scalars(sc, k_w, s_w);
    } else {
#pragma unroll
      for (int t = 0; t < 8; t++) { sc.u[t] = t == 0; sc.v[t] = k_w[t]; sc.b[t] = s_w[t]; }
      sc.fast = false;
      sc.u_neg = false;
    }
    fast = sc.fast;
    neg_u = sc.u_neg;
    if (c == 0) {
      if (fast) recode16_n<32>(&dig[q][kDigV], sc.v);
      else recode16_n<64>(&dig[q][kDigV], sc.v);
    } else if (c == 1) {
      recode256_store(&dig[q][kDigB], sc.b);
    } else if (c == 2) {
      recode16_n<32>(&dig[q][kDigU], sc.u);
    }
  }
  const bool a_ok = w.flags[4 * e] != 0;
  const bool r_ok = w.flags[4 * e + 1] != 0;

  // tables of (m+1)(-A) and (m+1)(-R), m < 8, in CachedQ layout
  fe *tabA = GT ? w.tabA + 64ull * e : tab_lds + q * 64;
  fe *tabR = tabA + 32;
  quad_multiples(tabA, w.negA[4ull * e + c]);
  {
    fe nR;
    neg_r_p3<SR>(nR, w.Rc[4ull * e + c]);
    quad_multiples(tabR, nR);
  }
  __syncthreads();  // digits (and the LDS tables) written by other lanes

  fe acc, r;
  quad::p3_identity(acc);
  fe idq;
  quad::cached_identity(idq);
  // windows: 32 (fast) or 64 (full k); the wave runs to its longest quad
  const int nw = fast ? 32 : 64;
  const int nw_wave = __ballot(!fast) ? 64 : 32;
  const fe *btab_hi = btab_q + 4 * kBaseQuadEntries;  // (m+1) [2^128]B
  // The 40 KB of B tables are read through L1 (not staged in LDS, which
  // would cap the kernel near one wave per SIMD); each window's entries are
  // loaded before its four doublings so the latency is hidden.
  for (int wdx = nw_wave - 1; wdx >= 0; wdx--) {
    if (wdx >= nw) continue;  // quad-uniform: only the full-k quads run windows 32..63
    const bool even = (wdx & 1) == 0;
    const int da = dig[q][kDigV + wdx];
    const int du = wdx < 32 ? dig[q][kDigU + wdx] : 0;
    const int db = even ? dig[q][kDigB + (wdx >> 1)] : 0;
    const int dh = (even && fast) ? dig[q][kDigB + 16 + (wdx >> 1)] : 0;
    const int aa = da < 0 ? -da : da, au = du < 0 ? -du : du, ab = db < 0 ? -db : db, ah = dh < 0 ? -dh : dh;
    fe aent = tabA[(aa ? aa - 1 : 0) * 4 + c];
    fe rent = tabR[(au ? au - 1 : 0) * 4 + c];
    fe bent, hent;
    if (even) {
      bent = btab_q[(ab ? ab - 1 : 0) * 4 + c];
      if (fast) hent = btab_hi[(ah ? ah - 1 : 0) * 4 + c];
    }
    if (wdx != nw - 1) {
#pragma unroll
      for (int d = 0; d < 4; d++) {
        quad::dbl(r, acc);
        quad::p1p1_to_p3(acc, r);
      }
    }
    fe_cmov(aent, idq, aa == 0);
    quad::cached_cneg(aent, da < 0);
    quad::add(r, acc, aent);
    quad::p1p1_to_p3(acc, r);
    if (wdx < 32) {  // u's digits (the slow path: u = 1, only window 0)
      fe_cmov(rent, idq, au == 0);
      quad::cached_cneg(rent, (du < 0) != neg_u);
      quad::add(r, acc, rent);
      quad::p1p1_to_p3(acc, r);
    }
    if (even) {  // b digit j weighs 256^j = 16^(2j); the top 16 digits on [2^128]B
      fe_cmov(bent, idq, ab == 0);
      quad::cached_cneg(bent, (db < 0) != neg_u);
      quad::add(r, acc, bent);
      quad::p1p1_to_p3(acc, r);
      if (fast) {
        fe_cmov(hent, idq, ah == 0);
        quad::cached_cneg(hent, (dh < 0) != neg_u);
        quad::add(r, acc, hent);
        quad::p1p1_to_p3(acc, r);
      }
    }
  }
  int status;
  if (SR) {
    const bool eq = quad::is_ristretto_identity(acc);
    status = !a_ok ? -1 : (!s_ok ? -2 : (!r_ok ? 0 : (eq ? 1 : 0)));
  } else {
    const bool ok = quad::is_identity_times8(acc) && s_ok && a_ok && r_ok;
    status = ok ? 1 : 0;
  }
  if (live && c == 0) out[i] = (uint8_t)(int8_t)status;
}


template <bool SR, bool GT>
__global__ void __launch_bounds__(kQuadBlock)
k_verify_quad(const uint8_t *__restrict__ sig, const uint32_t *__restrict__ idx, const uint32_t *count_ptr,
              uint32_t n, Ed25519Work w, const fe *__restrict__ btab_q, uint8_t *__restrict__ out, int aligned,
              const uint8_t *__restrict__ group_ok, uint32_t group_log2, const uint8_t *__restrict__ sub_ok,
              const uint32_t *__restrict__ fail_list, const uint32_t *__restrict__ fail_count,
              const uint32_t *__restrict__ fb_list, const uint32_t *__restrict__ fb_count, int half_on) {
  __shared__ fe tab_lds[GT ? 4 : kQuadSigs * 16 * 4];
  __shared__ int8_t dig[kQuadSigs][kDigBytes];
  quad_block<SR, GT>(blockIdx.x, tab_lds, dig, sig, idx, count_ptr, n, w, btab_q, out, aligned, group_ok,
                     group_log2, sub_ok, fail_list, fail_count, fb_list, fb_list ? *fb_count : 0u, half_on);
}

// The located fallback's entry list (k_loc_search) is usually a few entries
// but may hold every entry, so a grid sized for the worst case is mostly
// blocks that exit at once, and dispatching them is what the launch costs.
// Here a bounded grid strides over the list's 16-entry blocks instead.
template <bool SR>
__global__ void __launch_bounds__(kQuadBlock)
k_verify_quad_list(const uint8_t *__restrict__ sig, const uint32_t *__restrict__ idx, const uint32_t *count_ptr,
                   uint32_t n, Ed25519Work w, const fe *__restrict__ btab_q, uint8_t *__restrict__ out,
                   int aligned, const uint32_t *__restrict__ fb_list, const uint32_t *__restrict__ fb_count,
                   int half_on) {
  __shared__ fe tab_lds[4];
  __shared__ int8_t dig[kQuadSigs][kDigBytes];
  const uint32_t nl = *fb_count;
  for (uint32_t blk = blockIdx.x; blk * kQuadSigs < nl; blk += gridDim.x) {
    quad_block<SR, true>(blk, tab_lds, dig, sig, idx, count_ptr, n, w, btab_q, out, aligned, nullptr, 0u, nullptr,
                         nullptr, nullptr, fb_list, nl, half_on);
    __syncthreads();  // dig is rewritten by the next block
  }
}

// Mixed batches: split indices by key kind (TMV_KIND_ED25519 = 0,
// TMV_KIND_SR25519 = 1).  Order inside a list is irrelevant: results are
// scattered back by original index.  Unknown kinds get status 0.
// Ranks inside the workgroup come from wave ballots and the per-wave counts,
// so a workgroup of 256 entries makes one atomic per kind (not one per
// entry: 0.36 ms per 1M entries with per-entry atomics, profiles/r03/
// c5_trace); entries keep their order inside a workgroup.
__global__ void __launch_bounds__(256)
k_partition(const uint8_t *__restrict__ kind, uint32_t n, uint32_t *counts, uint32_t *idx_ed,
            uint32_t *idx_sr, uint8_t *__restrict__ out) {
  __shared__ uint32_t wcnt[2][4];
  __shared__ uint32_t base[2];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool in = i < n;
  const uint8_t k = in ? kind[i] : 255;
  if (in && k > 1) out[i] = 0;  // unknown key kind: not verified
  const uint64_t b0 = __ballot(k == 0), b1 = __ballot(k == 1);
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  if (lane == 0) {
    wcnt[0][wave] = (uint32_t)__popcll(b0);
    wcnt[1][wave] = (uint32_t)__popcll(b1);
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const uint32_t t = threadIdx.x;
    base[t] = atomicAdd(&counts[t], wcnt[t][0] + wcnt[t][1] + wcnt[t][2] + wcnt[t][3]);
  }
  __syncthreads();
  if (k > 1) return;
  uint32_t at = base[k] + (uint32_t)__popcll((k == 0 ? b0 : b1) & below);
  for (uint32_t w = 0; w < wave; w++) at += wcnt[k][w];
  (k == 0 ? idx_ed : idx_sr)[at] = i;
}

// The same split for the entries [lo, hi) of a streamed mixed launch: a
// part's entries of kind k go to idx_k[base_k + j], j < the part's count of
// that kind (the host counts each part's kinds, so base_k is known before the
// part lands); cursor (2 words, zeroed) numbers them, counts[k] accumulates
// the launch's totals (tmv_metrics / tmv_batch_stats).
__global__ void __launch_bounds__(256)
k_partition_range(const uint8_t *__restrict__ kind, uint32_t lo, uint32_t hi, uint32_t base_ed, uint32_t base_sr,
                  uint32_t *cursor, uint32_t *counts, uint32_t *idx_ed, uint32_t *idx_sr, uint8_t *out) {
  __shared__ uint32_t wcnt[2][4];
  __shared__ uint32_t base[2];
  const uint32_t i = lo + blockIdx.x * 256 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool in = i < hi;
  const uint8_t k = in ? kind[i] : 255;
  if (in && k > 1) out[i] = 0;  // unknown key kind: not verified
  const uint64_t b0 = __ballot(k == 0), b1 = __ballot(k == 1);
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  if (lane == 0) {
    wcnt[0][wave] = (uint32_t)__popcll(b0);
    wcnt[1][wave] = (uint32_t)__popcll(b1);
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const uint32_t t = threadIdx.x;
    const uint32_t tot = wcnt[t][0] + wcnt[t][1] + wcnt[t][2] + wcnt[t][3];
    base[t] = (t ? base_sr : base_ed) + atomicAdd(&cursor[t], tot);
    atomicAdd(&counts[t], tot);
  }
  __syncthreads();
  if (k > 1) return;
  uint32_t at = base[k] + (uint32_t)__popcll((k == 0 ? b0 : b1) & below);
  for (uint32_t w = 0; w < wave; w++) at += wcnt[k][w];
  (k == 0 ? idx_ed : idx_sr)[at] = i;
}

// ---------------------------------------------------------------------------
// Key-cached path (validator keys repeat across commits: the device-resident
// analogue of the reference's LRU caching verifier,
// crypto/ed25519/ed25519.go:31,56).  A cached key is stored as a 64-row comb
// of -A: row i holds (m+1) 16^i (-A), m < 8, in CachedQ layout (80 KB/key),
// so [k](-A) needs 64 table additions and no doublings.

// Key tables are built in two launches, so a batch of new keys (a light
// client's window brings one per height) is not one long chain per key:
//   k_key_bases  one quad per key: decode (every lane redundantly), then the
//                64 row bases 16^i (-A) -- the 252-doubling chain, each base
//                to a P3Q scratch and its 1x entry to the table;
//   k_key_rows   one quad per (key, row): multiples 2..8 of the row base
//                (one doubling, six additions).
// One quad per key doing both took a ~700-operation chain (64 rows x (1
// doubling + 6 additions + 4 doublings)).
template <bool SR>
__global__ void __launch_bounds__(kQuadBlock)
k_key_bases(const uint8_t *__restrict__ keys, const uint32_t *__restrict__ slots, uint32_t m, KeyTable kt,
            fe *__restrict__ bases) {
  const int c = threadIdx.x & 3;
  const uint32_t raw = blockIdx.x * kQuadSigs + (threadIdx.x >> 2);
  const bool live = raw < m;
  const uint32_t e = live ? raw : m - 1;
  uint32_t a_w[8];
  load_words_unaligned(a_w, keys + 32ull * e);
  ge_p3 A;
  bool ok = SR ? ristretto_decode(A, a_w) : ge_decode_zip215(A, a_w);
  if (!ok) ge_p3_identity(A);
  // -A in P3Q layout on this lane
  fe P;
  if (c == 0) fe_neg(P, A.X);
  else if (c == 1) P = A.Y;
  else if (c == 2) fe_one(P);
  else fe_neg(P, A.T);
  const uint32_t slot = slots[e];
  fe *row = kt.tab + (size_t)slot * kKeyRowsEntries * 4;
  fe *base = bases + (size_t)e * 64 * 4;
  fe r, Q0;
  for (int i = 0; i < 64; i++) {
    quad::to_cached(Q0, P);
    if (live) {
      base[i * 4 + c] = P;
      row[(i * 8 + 0) * 4 + c] = Q0;
    }
    if (i < 63) {
#pragma unroll
      for (int d = 0; d < 4; d++) {
        quad::dbl(r, P);
        quad::p1p1_to_p3(P, r);
      }
    }
  }
  if (live && c == 0) kt.ok[slot] = ok ? 1 : 0;
}

__global__ void __launch_bounds__(kQuadBlock)
k_key_rows(const uint32_t *__restrict__ slots, uint32_t m, KeyTable kt, const fe *__restrict__ bases) {
  const int c = threadIdx.x & 3;
  const uint32_t raw = blockIdx.x * kQuadSigs + (threadIdx.x >> 2);  // (key, row)
  const bool live = raw < 64 * m;
  const uint32_t q = live ? raw : 64 * m - 1;
  const uint32_t e = q >> 6, i = q & 63;
  const fe P = bases[((size_t)e * 64 + i) * 4 + c];
  fe *row = kt.tab + (size_t)slots[e] * kKeyRowsEntries * 4 + (size_t)i * 8 * 4;
  fe r, Pm, Q, Q0;
  quad::to_cached(Q0, P);
  quad::dbl(r, P);
  quad::p1p1_to_p3(Pm, r);
  quad::to_cached(Q, Pm);
  if (live) row[1 * 4 + c] = Q;
  for (int t = 2; t < 8; t++) {
    quad::add(r, Pm, Q0);
    quad::p1p1_to_p3(Pm, r);
    quad::to_cached(Q, Pm);
    if (live) row[t * 4 + c] = Q;
  }
}

// Lanes [0, m) decode R, [m, 2m) compute the challenge (SHA-512 or merlin).
template <bool SR>
__global__ void __launch_bounds__(kVerifyBlock)
k_prep_cached(const uint8_t *__restrict__ pk, const uint8_t *__restrict__ sig, const uint8_t *__restrict__ msg,
              const uint32_t *__restrict__ msg_off, const uint32_t *__restrict__ idx, uint32_t n, Ed25519Work w,
              const strobe_t *__restrict__ prefix, int aligned) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const uint32_t task = j / n;
  const uint32_t e = j - task * n;  // work slot; the entry read is idx[e] (key order) or e
  const uint32_t i = idx ? idx[e] : e;
  uint32_t a_w[8], r_w[8];
  if (aligned) load_words_aligned(r_w, sig + 64ull * i);
  else load_words_unaligned(r_w, sig + 64ull * i);
  if (task == 1) {
    if (aligned) load_words_aligned(a_w, pk + 32ull * i);
    else load_words_unaligned(a_w, pk + 32ull * i);
    uint32_t k[8];
    const uint32_t o0 = msg_off[i], o1 = msg_off[i + 1];
    if constexpr (SR) {
      __shared__ uint64_t strobe_lanes[25][kVerifyBlock];
      sr25519_challenge_lds<kVerifyBlock>(k, *prefix, &strobe_lanes[0][threadIdx.x], a_w, r_w, msg + o0, o1 - o0);
    } else {
      uint32_t h[16];
      sha512_pq_msg(h, r_w, a_w, msg + o0, o1 - o0);
      sc_reduce512(k, h);
    }
    uint4 *kd = reinterpret_cast<uint4 *>(w.k + 8ull * e);
    kd[0] = make_uint4(k[0], k[1], k[2], k[3]);
    kd[1] = make_uint4(k[4], k[5], k[6], k[7]);
    return;
  }
  ge_p3 P;
  bool ok = SR ? ristretto_decode(P, r_w) : ge_decode_zip215(P, r_w);
  if (!ok) ge_p3_identity(P);
  w.flags[4 * e + 1] = ok ? 1 : 0;
  if (w.niels) {  // -R in affine Niels form for the key-merged batch equation (point index e)
    niels_pt np;
    fe t;
    fe_sub(t, P.Y, P.X); fe_carry(np.ypx, t);
    fe_add(t, P.Y, P.X); fe_carry(np.ymx, t);
    fe_mul(t, P.T, consts::d2()); fe_neg(np.xy2d, t);
    np.pad[0] = np.pad[1] = 0;
    niels_store(w.niels, e, np);
  }
  fe *dst = w.Rc + 4ull * e;
  if (SR) {
    dst[0] = P.X; dst[1] = P.Y;
    fe t; fe_one(t); dst[2] = t;
    dst[3] = P.T;
  } else {
    ge_cached cc;
    ge_p3_to_cached(cc, P);
    fe t;
    fe_carry(t, cc.YmX); dst[0] = t;
    fe_carry(t, cc.YpX); dst[1] = t;
    dst[2] = cc.T2d;
    dst[3] = cc.Z;
  }
}

// acc = sum_i e_i(k) 16^i(-A) [key comb] + sum_j d_j(s) 256^j B [base comb];
// no doublings.  Table entries are prefetched kCombAhead additions ahead.
template <bool SR>
__global__ void __launch_bounds__(kQuadBlock)
k_verify_comb(const uint8_t *__restrict__ sig, const uint32_t *__restrict__ key_slot, const uint32_t *__restrict__ idx,
              uint32_t n, Ed25519Work w, KeyTable kt, const fe *__restrict__ bcomb, uint8_t *__restrict__ out,
              int aligned, const uint8_t *__restrict__ group_ok, uint32_t group_log2) {
  __shared__ int8_t dig[kQuadSigs][2][64];
  if (blockIdx.x * kQuadSigs >= n) return;
  const int c = threadIdx.x & 3;
  const int q = threadIdx.x >> 2;
  const uint32_t raw = blockIdx.x * kQuadSigs + q;
  const bool live = raw < n;
  const uint32_t e = live ? raw : n - 1;  // work slot (key order with idx)
  const uint32_t i = idx ? idx[e] : e;    // entry: input rows, key slot, status
  uint32_t s_raw[8], s_w[8];
  if (aligned) load_words_aligned(s_raw, sig + 64ull * i + 32);
  else load_words_unaligned(s_raw, sig + 64ull * i + 32);
  bool s_ok;
  if (SR) {
    s_ok = sr25519_decode_s(s_w, s_raw);
  } else {
#pragma unroll
    for (int t = 0; t < 8; t++) s_w[t] = s_raw[t];
    s_ok = sc_is_canonical(s_w);
  }
  // key-merged batch equation held for this block's group (groups are >= 32
  // entries: block-uniform): the pre-checks decide every entry
  if (group_ok && group_ok[(blockIdx.x * kQuadSigs) >> group_log2]) {
    if (!live || c != 0) return;
    const bool a_ok = kt.ok[key_slot[i]] != 0;
    const bool r_ok = w.flags[4 * e + 1] != 0;
    const int status = SR ? (!a_ok ? -1 : (!s_ok ? -2 : (r_ok ? 1 : 0))) : ((a_ok && r_ok && s_ok) ? 1 : 0);
    out[i] = (uint8_t)(int8_t)status;
    return;
  }
  if (!s_ok) s_w[7] &= 0x0fffffffu;
  {
    uint32_t k_w[8];
    const uint4 *kp = reinterpret_cast<const uint4 *>(w.k + 8ull * e);
    const uint4 k0 = kp[0], k1 = kp[1];
    k_w[0] = k0.x; k_w[1] = k0.y; k_w[2] = k0.z; k_w[3] = k0.w;
    k_w[4] = k1.x; k_w[5] = k1.y; k_w[6] = k1.z; k_w[7] = k1.w;
    if (c == 1) recode256_store(&dig[q][1][0], s_w);
    else recode16_store(&dig[q][0][0], k_w, c == 0);
  }
  __syncthreads();
  const uint32_t slot = key_slot[i];
  const bool a_ok = kt.ok[slot] != 0;
  const bool r_ok = w.flags[4 * e + 1] != 0;
  const fe *krow = kt.tab + (size_t)slot * kKeyRowsEntries * 4;
  fe acc, r, idq;
  quad::p3_identity(acc);
  quad::cached_identity(idq);
  // 64 key-comb additions then 32 base-comb additions, one entry prefetched
  auto entry_at = [&](int t, int &dsg) -> const fe * {
    if (t < 64) {
      dsg = dig[q][0][t];
      const int a = dsg < 0 ? -dsg : dsg;
      return krow + ((t * 8) + (a ? a - 1 : 0)) * 4 + c;
    }
    dsg = dig[q][1][t - 64];
    const int a = dsg < 0 ? -dsg : dsg;
    return bcomb + (((t - 64) * kBaseQuadEntries) + (a ? a - 1 : 0)) * 4 + c;
  };
  comb_accumulate<96>(acc, idq, entry_at);
  int status;
  if (SR) {
    const fe Rq = w.Rc[4ull * e + c];
    const bool eq = quad::ristretto_equal(acc, Rq);
    status = !a_ok ? -1 : (!s_ok ? -2 : (!r_ok ? 0 : (eq ? 1 : 0)));
  } else {
    fe Rq = w.Rc[4ull * e + c];
    quad::cached_cneg(Rq, true);
    quad::add(r, acc, Rq);
    quad::p1p1_to_p3(acc, r);
    status = (quad::is_identity_times8(acc) && s_ok && a_ok && r_ok) ? 1 : 0;
  }
  if (live && c == 0) out[i] = (uint8_t)(int8_t)status;
}

// Latency form of the key-cached path (small batches: VerifyCommit).  The
// comb sum needs k but not R, so the work of 16 signatures is spread over a
// workgroup of four waves (round 3's two-wave form ran the 96 comb additions
// as one quad chain after the hash, ~40% longer than the R decode): wave 1
// decodes the R's; wave 2 runs the 32 base-comb
// additions (s is known at once); waves 0 and 3 each hash (the same SHA-512 /
// transcript, computed twice so neither waits for the other) and run half of
// the 64 key-comb additions; wave 0 then adds the other partial sums (LDS)
// and makes the final check.  Critical path: max(R decode, hash + 32
// additions) + 2 additions + the check.  One __syncthreads per wave.
template <bool SR>
__global__ void __launch_bounds__(4 * kQuadBlock)
k_verify_cached_fused4(const uint8_t *__restrict__ pk, const uint8_t *__restrict__ sig,
                       const uint8_t *__restrict__ msg, const uint32_t *__restrict__ msg_off,
                       const uint32_t *__restrict__ key_slot, uint32_t n, KeyTable kt, const fe *__restrict__ bcomb,
                       const strobe_t *__restrict__ prefix, uint8_t *__restrict__ out, int aligned) {
  __shared__ int8_t dig_k[2][kQuadSigs][64];  // waves 0 / 3: their own recoding of k
  __shared__ int8_t dig_s[kQuadSigs][32];     // wave 2: s in radix 256
  __shared__ fe part[2][kQuadSigs][4];        // P3Q partial sums of waves 2 and 3
  __shared__ fe Rs[kQuadSigs][4];
  __shared__ uint8_t rok[kQuadSigs];
  const uint32_t base = blockIdx.x * kQuadSigs;
  if (base >= n) return;  // block-uniform
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  if (wave == 1) {
    if (lane < kQuadSigs) {
      const uint32_t i = min(base + lane, n - 1);
      uint32_t r_w[8];
      if (aligned) load_words_aligned(r_w, sig + 64ull * i);
      else load_words_unaligned(r_w, sig + 64ull * i);
      ge_p3 P;
      const bool ok = SR ? ristretto_decode(P, r_w) : ge_decode_zip215(P, r_w);
      if (!ok) ge_p3_identity(P);
      rok[lane] = ok ? 1 : 0;
      if (SR) {
        Rs[lane][0] = P.X; Rs[lane][1] = P.Y;
        fe t; fe_one(t); Rs[lane][2] = t;
        Rs[lane][3] = P.T;
      } else {  // CachedQ of R, negated by the final check
        ge_cached cc;
        ge_p3_to_cached(cc, P);
        fe t;
        fe_carry(t, cc.YmX); Rs[lane][0] = t;
        fe_carry(t, cc.YpX); Rs[lane][1] = t;
        Rs[lane][2] = cc.T2d;
        Rs[lane][3] = cc.Z;
      }
    }
    __syncthreads();
    return;
  }
  const int c = lane & 3;
  const int q = lane >> 2;
  const uint32_t raw = base + q;
  const bool live = raw < n;
  const uint32_t i = live ? raw : n - 1;
  fe acc, r, idq;
  quad::p3_identity(acc);
  quad::cached_identity(idq);
  if (wave == 2) {  // base comb: Σ d_t(s) (256^t B), 32 additions
    uint32_t s_raw[8], s_w[8];
    if (aligned) load_words_aligned(s_raw, sig + 64ull * i + 32);
    else load_words_unaligned(s_raw, sig + 64ull * i + 32);
    bool s_ok;
    if (SR) {
      s_ok = sr25519_decode_s(s_w, s_raw);
    } else {
#pragma unroll
      for (int t = 0; t < 8; t++) s_w[t] = s_raw[t];
      s_ok = sc_is_canonical(s_w);
    }
    if (!s_ok) s_w[7] &= 0x0fffffffu;  // keep the recoding in range; the entry is rejected anyway
    if (c == 1) recode256_store(&dig_s[q][0], s_w);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    auto entry_at = [&](int t, int &dsg) -> const fe * {
      dsg = dig_s[q][t];
      const int a = dsg < 0 ? -dsg : dsg;
      return bcomb + ((t * kBaseQuadEntries) + (a ? a - 1 : 0)) * 4 + c;
    };
    comb_accumulate<32>(acc, idq, entry_at);
    part[0][q][c] = acc;
    __syncthreads();
    return;
  }
  // waves 0 and 3: the challenge k, then key-comb rows [32 h, 32 h + 32)
  const int h = wave == 3 ? 1 : 0;
  if (c == 0) {
    uint32_t k_w[8];
    uint32_t a_w[8], r_w[8];
    if (aligned) {
      load_words_aligned(a_w, pk + 32ull * i);
      load_words_aligned(r_w, sig + 64ull * i);
    } else {
      load_words_unaligned(a_w, pk + 32ull * i);
      load_words_unaligned(r_w, sig + 64ull * i);
    }
    const uint32_t o0 = msg_off[i], o1 = msg_off[i + 1];
    if constexpr (SR) {  // transcript state in LDS, one slot per quad and wave
      __shared__ uint64_t strobe_lanes[2][25][kQuadSigs];
      sr25519_challenge_lds<kQuadSigs>(k_w, *prefix, &strobe_lanes[h][0][q], a_w, r_w, msg + o0, o1 - o0);
    } else {
      uint32_t hh[16];
      sha512_pq_msg(hh, r_w, a_w, msg + o0, o1 - o0);
      sc_reduce512(k_w, hh);
    }
    recode16_store(&dig_k[h][q][0], k_w, true);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const uint32_t slot = key_slot[i];
  const fe *krow = kt.tab + (size_t)slot * kKeyRowsEntries * 4;
  auto entry_at = [&](int t, int &dsg) -> const fe * {
    const int tt = t + 32 * h;
    dsg = dig_k[h][q][tt];
    const int a = dsg < 0 ? -dsg : dsg;
    return krow + ((tt * 8) + (a ? a - 1 : 0)) * 4 + c;
  };
  comb_accumulate<32>(acc, idq, entry_at);
  if (wave == 3) {
    part[1][q][c] = acc;
    __syncthreads();
    return;
  }
  // wave 0: the S check, the other partial sums, the final check
  uint32_t s_raw[8], s_w[8];
  if (aligned) load_words_aligned(s_raw, sig + 64ull * i + 32);
  else load_words_unaligned(s_raw, sig + 64ull * i + 32);
  bool s_ok;
  if (SR) {
    s_ok = sr25519_decode_s(s_w, s_raw);
  } else {
#pragma unroll
    for (int t = 0; t < 8; t++) s_w[t] = s_raw[t];
    s_ok = sc_is_canonical(s_w);
  }
  const bool a_ok = kt.ok[slot] != 0;
  __syncthreads();  // partial sums and R's written
#pragma unroll
  for (int pi = 0; pi < 2; pi++) {
    fe pc;
    quad::to_cached(pc, part[pi][q][c]);
    quad::add(r, acc, pc);
    quad::p1p1_to_p3(acc, r);
  }
  const bool r_ok = rok[q] != 0;
  int status;
  if (SR) {
    const fe Rq = Rs[q][c];
    const bool eq = quad::ristretto_equal(acc, Rq);
    status = !a_ok ? -1 : (!s_ok ? -2 : (!r_ok ? 0 : (eq ? 1 : 0)));
  } else {
    fe Rq = Rs[q][c];
    quad::cached_cneg(Rq, true);
    quad::add(r, acc, Rq);
    quad::p1p1_to_p3(acc, r);
    status = (quad::is_identity_times8(acc) && s_ok && a_ok && r_ok) ? 1 : 0;
  }
  if (live && c == 0) out[i] = (uint8_t)(int8_t)status;
}

hipError_t launch_key_build(bool sr, const uint8_t *keys, const uint32_t *slots, uint32_t m, KeyTable kt,
                            fe *bases, hipStream_t stream) {
  if (m == 0) return hipSuccess;
  const uint32_t blocks = (m + kQuadSigs - 1) / kQuadSigs;
  if (sr) hipLaunchKernelGGL(k_key_bases<true>, dim3(blocks), dim3(kQuadBlock), 0, stream, keys, slots, m, kt, bases);
  else hipLaunchKernelGGL(k_key_bases<false>, dim3(blocks), dim3(kQuadBlock), 0, stream, keys, slots, m, kt, bases);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t rblocks = (uint32_t)((64ull * m + kQuadSigs - 1) / kQuadSigs);
  hipLaunchKernelGGL(k_key_rows, dim3(rblocks), dim3(kQuadBlock), 0, stream, slots, m, kt, (const fe *)bases);
  return hipGetLastError();
}

hipError_t launch_verify_cached(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                const uint32_t *msg_off, const uint32_t *key_slot, uint32_t n, KeyTable kt,
                                const fe *bcomb, const strobe_t *prefix, Ed25519Work w, uint8_t *out,
                                uint32_t fused_max, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  if (n <= fused_max) {  // latency-bound: one fused kernel
    const uint32_t blocks = (n + kQuadSigs - 1) / kQuadSigs;
    if (sr) hipLaunchKernelGGL(k_verify_cached_fused4<true>, dim3(blocks), dim3(4 * kQuadBlock), 0, stream, pk, sig,
                               msg, msg_off, key_slot, n, kt, bcomb, prefix, out, aligned);
    else hipLaunchKernelGGL(k_verify_cached_fused4<false>, dim3(blocks), dim3(4 * kQuadBlock), 0, stream, pk, sig,
                            msg, msg_off, key_slot, n, kt, bcomb, prefix, out, aligned);
    return hipGetLastError();
  }
  w.niels = nullptr;
  const uint32_t pblocks = (uint32_t)((2ull * n + kVerifyBlock - 1) / kVerifyBlock);
  if (sr) hipLaunchKernelGGL(k_prep_cached<true>, dim3(pblocks), dim3(kVerifyBlock), 0, stream, pk, sig, msg, msg_off, nullptr, n, w, prefix, aligned);
  else hipLaunchKernelGGL(k_prep_cached<false>, dim3(pblocks), dim3(kVerifyBlock), 0, stream, pk, sig, msg, msg_off, nullptr, n, w, prefix, aligned);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t qblocks = (n + kQuadSigs - 1) / kQuadSigs;
  if (sr) hipLaunchKernelGGL(k_verify_comb<true>, dim3(qblocks), dim3(kQuadBlock), 0, stream, sig, key_slot, nullptr, n, w, kt, bcomb, out,
                             aligned, nullptr, 0u);
  else hipLaunchKernelGGL(k_verify_comb<false>, dim3(qblocks), dim3(kQuadBlock), 0, stream, sig, key_slot, nullptr, n, w, kt, bcomb, out,
                          aligned, nullptr, 0u);
  return hipGetLastError();
}

template <bool SR>
hipError_t launch_prep_cached(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off,
                              const uint32_t *idx, uint32_t n, const strobe_t *prefix, Ed25519Work w, int aligned,
                              hipStream_t stream) {
  const uint32_t pblocks = (uint32_t)((2ull * n + kVerifyBlock - 1) / kVerifyBlock);
  hipLaunchKernelGGL(k_prep_cached<SR>, dim3(pblocks), dim3(kVerifyBlock), 0, stream, pk, sig, msg, msg_off, idx, n, w,
                     prefix, aligned);
  return hipGetLastError();
}
template hipError_t launch_prep_cached<false>(const uint8_t *, const uint8_t *, const uint8_t *, const uint32_t *,
                                              const uint32_t *, uint32_t, const strobe_t *, Ed25519Work, int,
                                              hipStream_t);
template hipError_t launch_prep_cached<true>(const uint8_t *, const uint8_t *, const uint8_t *, const uint32_t *,
                                             const uint32_t *, uint32_t, const strobe_t *, Ed25519Work, int,
                                             hipStream_t);

template <bool SR>
hipError_t launch_comb_fallback(const uint8_t *sig, const uint32_t *key_slot, const uint32_t *idx, uint32_t n,
                                Ed25519Work w, KeyTable kt, const fe *bcomb, uint8_t *out, int aligned,
                                const uint8_t *group_ok, uint32_t group_log2, hipStream_t stream) {
  const uint32_t qblocks = (n + kQuadSigs - 1) / kQuadSigs;
  hipLaunchKernelGGL(k_verify_comb<SR>, dim3(qblocks), dim3(kQuadBlock), 0, stream, sig, key_slot, idx, n, w, kt, bcomb,
                     out, aligned, group_ok, group_log2);
  return hipGetLastError();
}
template hipError_t launch_comb_fallback<false>(const uint8_t *, const uint32_t *, const uint32_t *, uint32_t,
                                                Ed25519Work, KeyTable, const fe *, uint8_t *, int, const uint8_t *,
                                                uint32_t, hipStream_t);
template hipError_t launch_comb_fallback<true>(const uint8_t *, const uint32_t *, const uint32_t *, uint32_t,
                                               Ed25519Work, KeyTable, const fe *, uint8_t *, int, const uint8_t *,
                                               uint32_t, hipStream_t);

// k_verify_quad's -A tables: LDS or global scratch.  Measured on the C2 bench
// in one GPU call (profiles/r01_msm/ab_quad_table.log, when the quad kernel
// still ran every entry): LDS 72.8 / 73.5 M/s, global 70.8 / 71.2 M/s (5
// instead of 2 waves per SIMD, but every window's entry then comes from L2);
// per entry 45.6-45.7 M/s either way.  As the batch-equation fallback almost
// every block exits at once, and the 22.5 KB of LDS a block holds only caps
// how fast the grid drains: global there (C2 bench, profiles/r02_close/
// ab_quad_fallback.txt: 101.5 / 101.8 -> 102.8 / 102.5 M/s), LDS for the
// per-entry pipeline while its grid fits that residency.
//
// Half-size scalars in the per-entry checks (halfscalar.h): mode 1 (the
// product).  Test aid (tmv_internal_option "half_scalars", never set by a
// deployment): 0 verifies every entry with the full k, 2 puts every third
// entry on the full-k path beside half-size quads of the same wave -- the
// path an entry whose reduction does not finish (~2^-24 of hash outputs)
// takes, which random tests would otherwise never reach.
static std::atomic<int> g_half_mode{1};
void set_half_scalar_mode(int mode) { g_half_mode = mode == 0 || mode == 2 ? mode : 1; }
static int half_scalars_on() { return g_half_mode.load(std::memory_order_relaxed); }

template <bool SR>
static void launch_quad(uint32_t qblocks, hipStream_t stream, const uint8_t *sig, const uint32_t *idx,
                        const uint32_t *count_ptr, uint32_t n, Ed25519Work w, const fe *btab_q, uint8_t *out,
                        int aligned, const uint8_t *group_ok, uint32_t group_log2,
                        const uint8_t *sub_ok = nullptr, const uint32_t *fail_list = nullptr,
                        const uint32_t *fail_count = nullptr, const uint32_t *fb_list = nullptr,
                        const uint32_t *fb_count = nullptr, bool fallback = false) {
  const int half = half_scalars_on();
  // LDS tables hold 40 KB per wave (3 waves per CU): only while the grid fits
  // that residency, else global
  const bool global = fallback || qblocks > 3u * 256u;
  if (global)
    hipLaunchKernelGGL((k_verify_quad<SR, true>), dim3(qblocks), dim3(kQuadBlock), 0, stream, sig, idx, count_ptr, n,
                       w, btab_q, out, aligned, group_ok, group_log2, sub_ok, fail_list, fail_count, fb_list,
                       fb_count, half);
  else
    hipLaunchKernelGGL((k_verify_quad<SR, false>), dim3(qblocks), dim3(kQuadBlock), 0, stream, sig, idx, count_ptr, n,
                       w, btab_q, out, aligned, group_ok, group_log2, sub_ok, fail_list, fail_count, fb_list,
                       fb_count, half);
}

static int is_aligned(const void *a, const void *b) {
  return ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0;
}

template <bool SR>
static hipError_t launch_pipeline(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                  const uint32_t *msg_off, const uint32_t *idx, const uint32_t *count_ptr,
                                  uint32_t n, const fe *btab_q, const strobe_t *prefix, Ed25519Work w,
                                  uint8_t *out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int aligned = is_aligned(pk, sig);
  w.hs = w.hs_buf;  // the prep's hash lane reduces k once per entry (10k launch 0.331 -> 0.299 ms, round 5)
  hipError_t e = launch_prep<SR>(pk, sig, msg, msg_off, idx, count_ptr, n, prefix, w, aligned, stream);
  if (e != hipSuccess) return e;
  const uint32_t qblocks = (n + kQuadSigs - 1) / kQuadSigs;
  launch_quad<SR>(qblocks, stream, sig, idx, count_ptr, n, w, btab_q, out, aligned, nullptr, 0u);
  return hipGetLastError();
}

// Row H: after the batch equation, re-verify only the entries of failed
// groups (blocks of passing groups exit after writing the pre-check status).
template <bool SR>
hipError_t launch_quad_fallback(const uint8_t *sig, const uint32_t *idx, const uint32_t *count_ptr, uint32_t n,
                                const fe *btab_q, Ed25519Work w, const uint8_t *group_ok, uint32_t group_log2,
                                uint8_t *out, int aligned, hipStream_t stream, const uint8_t *sub_ok,
                                const uint32_t *fail_list, const uint32_t *fail_count, const uint32_t *fb_list,
                                const uint32_t *fb_count) {
  // compacted / entry list: a grid for every group failing (blocks past the
  // failing count exit at once)
  const uint32_t qblocks = fb_list ? (n + kQuadSigs - 1) / kQuadSigs
                           : fail_list ? ((((n + (1u << group_log2) - 1) >> group_log2)) << (group_log2 - 4))
                                       : (n + kQuadSigs - 1) / kQuadSigs;
  if (fb_list) {
    // at most 16 waves per CU (the kernel fits 5 per SIMD); blocks stride over the list
    const uint32_t grid = qblocks < 256u * 16u ? qblocks : 256u * 16u;
    hipLaunchKernelGGL(k_verify_quad_list<SR>, dim3(grid), dim3(kQuadBlock), 0, stream, sig, idx, count_ptr, n, w,
                       btab_q, out, aligned, fb_list, fb_count, half_scalars_on());
    return hipGetLastError();
  }
  launch_quad<SR>(qblocks, stream, sig, idx, count_ptr, n, w, btab_q, out, aligned, group_ok, group_log2, sub_ok,
                  fail_list, fail_count, fb_list, fb_count, true);
  return hipGetLastError();
}
template hipError_t launch_quad_fallback<false>(const uint8_t *, const uint32_t *, const uint32_t *, uint32_t,
                                                const fe *, Ed25519Work, const uint8_t *, uint32_t, uint8_t *, int,
                                                hipStream_t, const uint8_t *, const uint32_t *, const uint32_t *,
                                                const uint32_t *, const uint32_t *);
template hipError_t launch_quad_fallback<true>(const uint8_t *, const uint32_t *, const uint32_t *, uint32_t,
                                               const fe *, Ed25519Work, const uint8_t *, uint32_t, uint8_t *, int,
                                               hipStream_t, const uint8_t *, const uint32_t *, const uint32_t *,
                                               const uint32_t *, const uint32_t *);

template <bool SR>
hipError_t launch_prep(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off,
                       const uint32_t *idx, const uint32_t *count_ptr, uint32_t n, const strobe_t *prefix,
                       Ed25519Work w, int aligned, hipStream_t stream) {
  const uint32_t dblocks = (uint32_t)((2ull * n + kVerifyBlock - 1) / kVerifyBlock);
  const uint32_t hblocks = (n + kVerifyBlock - 1) / kVerifyBlock;
  void *tk = ktimer::begin(ktimer::kPrep, stream);
  hipLaunchKernelGGL(k_prep_fused<SR>, dim3(dblocks + hblocks), dim3(kVerifyBlock), 0, stream, pk, sig, msg, msg_off,
                     idx, count_ptr, n, w, prefix, aligned, dblocks);
  const hipError_t e = hipGetLastError();
  ktimer::end(tk, stream);
  return e;
}
template hipError_t launch_prep<false>(const uint8_t *, const uint8_t *, const uint8_t *, const uint32_t *,
                                       const uint32_t *, const uint32_t *, uint32_t, const strobe_t *, Ed25519Work,
                                       int, hipStream_t);
template hipError_t launch_prep<true>(const uint8_t *, const uint8_t *, const uint8_t *, const uint32_t *,
                                      const uint32_t *, const uint32_t *, uint32_t, const strobe_t *, Ed25519Work,
                                      int, hipStream_t);

hipError_t launch_ed25519_verify_quad(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                      const uint32_t *msg_off, uint32_t n, const fe *btab_q, Ed25519Work w,
                                      uint8_t *valid, hipStream_t stream) {
  return launch_pipeline<false>(pk, sig, msg, msg_off, nullptr, nullptr, n, btab_q, nullptr, w, valid, stream);
}

hipError_t launch_sr25519_verify_quad(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                      const uint32_t *msg_off, uint32_t n, const fe *btab_q, const strobe_t *prefix,
                                      Ed25519Work w, int8_t *status, hipStream_t stream) {
  return launch_pipeline<true>(pk, sig, msg, msg_off, nullptr, nullptr, n, btab_q, prefix, w,
                               reinterpret_cast<uint8_t *>(status), stream);
}

hipError_t launch_mixed_verify(const uint8_t *kind, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                               const uint32_t *msg_off, uint32_t n, const fe *btab_q, const strobe_t *prefix,
                               Ed25519Work w_ed, Ed25519Work w_sr, uint32_t *counts, uint32_t *idx_ed,
                               uint32_t *idx_sr, int8_t *status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(counts, 0, 2 * sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  uint8_t *out = reinterpret_cast<uint8_t *>(status);
  hipLaunchKernelGGL(k_partition, dim3((n + 255) / 256), dim3(256), 0, stream, kind, n, counts, idx_ed, idx_sr, out);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  e = launch_pipeline<false>(pk, sig, msg, msg_off, idx_ed, counts, n, btab_q, prefix, w_ed, out, stream);
  if (e != hipSuccess) return e;
  return launch_pipeline<true>(pk, sig, msg, msg_off, idx_sr, counts + 1, n, btab_q, prefix, w_sr, out, stream);
}

hipError_t launch_partition_range(const uint8_t *kind, uint32_t lo, uint32_t hi, uint32_t base_ed, uint32_t base_sr,
                                  uint32_t *cursor, uint32_t *counts, uint32_t *idx_ed, uint32_t *idx_sr, uint8_t *out,
                                  hipStream_t stream) {
  if (hi <= lo) return hipSuccess;
  hipLaunchKernelGGL(k_partition_range, dim3((hi - lo + 255) / 256), dim3(256), 0, stream, kind, lo, hi, base_ed,
                     base_sr, cursor, counts, idx_ed, idx_sr, out);
  return hipGetLastError();
}

hipError_t launch_partition(const uint8_t *kind, uint32_t n, uint32_t *counts, uint32_t *idx_ed, uint32_t *idx_sr,
                            uint8_t *out, hipStream_t stream) {
  hipError_t e = hipMemsetAsync(counts, 0, 2 * sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_partition, dim3((n + 255) / 256), dim3(256), 0, stream, kind, n, counts, idx_ed, idx_sr, out);
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
