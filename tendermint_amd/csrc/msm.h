// Random-linear-combination batch check: the
// device analogue of curve25519-voi's BatchVerifier.Verify behind
// crypto/ed25519/ed25519.go:231-233 and crypto/sr25519/batch.go:44-47.
//
// For a group g of entries (m consecutive signatures of one key kind) with
// random 128-bit z_i (device ChaCha20, key drawn from getrandom per call):
//   T_g = [sum z_i s_i mod l] B + sum [z_i] (-R_i) + sum [z_i k_i mod l] (-A_i)
// ed25519 (ZIP-215, cofactored): group passes iff [8] T_g == O
// sr25519 (Ristretto):           group passes iff T_g is the Ristretto identity
// Entries that failed decoding / the S check are left out of the sums (their
// status is already known).  A passing group makes every remaining entry
// valid (false accept probability <= 2^-128 per group, as voi's); a failing
// group's entries are verified one by one (row H: k_verify_quad with the
// group verdicts), so the validity vector is exact.
//
// Pippenger over the 2m+1 points of a group with signed c-bit digits:
//   k_msm_sort   one workgroup per group: scalars, digits, LDS counting sort
//                of (window, |digit|) bucket entries into the group's region
//   k_msm_accum  one lane per L consecutive sorted entries: runs of one
//                bucket are summed (mixed additions, Niels points); runs that
//                cross a chunk edge leave partial sums
//   k_msm_wpart  one lane per (group, window, part): running sums over the
//                part's H/P buckets (bucket values merge chunk partials)
//   k_msm_wsum   one lane per (group, window): joins the P parts into the
//                window sum S_w = sum_j (j+1) bucket_j (P > 1 only: with one
//                lane per window its T is S_w)
//   k_msm_horner one quad per group: T_g = sum_w 2^(c w) S_w (Horner, quad-lane
//                arithmetic) and the group verdict
//
// Key-merged form (batches whose keys sit in the
// device key cache, e.g. commits of one validator set): entries are ordered
// by key, so a group holds few distinct keys, and the A terms collapse to
// one scalar per (group, key):  sum_i [z_i k_i](-A_i) = sum_key [W_key](-A_key)
// with W_key = sum z_i k_i mod l.  The MSM then covers only the m R points
// (ceil(129/c) windows of the 128-bit z_i: Horner needs ~129 doublings, not
// ~253), and each key term and the B term are comb sums over the cached
// tables (64 and 32 additions, no doublings):
//   k_msm_sort<KM>  z_i digits only; w_i = z_i k_i and the B scalar to HBM
//   k_msm_items     one quad per run of one key inside a group (W_key, key
//                   comb) and per group (B scalar, base comb)
//   k_msm_horner<KM> Horner over the R windows + the group's item points
// The per-entry fallback of failing groups is the key-cached comb kernel.
#pragma once
#include <stdint.h>
#include "curve25519.h"

namespace tmv {

constexpr uint32_t kMsmWideRows = 65536;     // (group, window) rows from which k_msm_wpart runs one lane per window
constexpr int kMsmChunkMax = 32;             // sorted entries per accumulation lane: 16 or 32
constexpr uint32_t kMsmEmpty = 0xffffffffu;  // padding entry / no bucket
constexpr int kMsmSortBlock = 256;
// Buckets cut by chunk edges are joined by k_msm_accum (neighbouring lanes of
// a wave) and k_msm_join_list (the rest, from a packed list) before the
// running sums, which then read whole buckets only.
constexpr uint32_t kSubGroupLog2 = 3;        // k_msm_subcheck: 8 entries per sub-group
constexpr uint32_t kSubGroup = 1u << kSubGroupLog2;

// Affine Niels point padded to one 128-byte line.
struct alignas(16) niels_pt {
  fe ypx, ymx, xy2d;
  int32_t pad[2];
};

// Points of the batch equation are stored as (+P, -P) pairs (pts[2 i] and
// pts[2 i + 1] for point i), so a sorted entry's (index << 1 | negate) word
// is its slot and the bucket sums load the signed point as it is -- no
// per-entry swap and negation.  -DTMV_NIELS_PAIR=0: one slot per point.
#ifndef TMV_NIELS_PAIR
#define TMV_NIELS_PAIR 0
#endif
constexpr uint32_t kNielsPer = TMV_NIELS_PAIR ? 2 : 1;

// -P of a Niels point: (y - x, y + x, -2dxy)
TMV_HD niels_pt niels_negate(const niels_pt &p) {
  niels_pt r;
  r.ypx = p.ymx;
  r.ymx = p.ypx;
  fe_neg(r.xy2d, p.xy2d);
  r.pad[0] = r.pad[1] = 0;
  return r;
}

// Store point i's Niels form (and, paired, its negation).
TMV_HD void niels_store(niels_pt *pts, uint64_t i, const niels_pt &p) {
  if (kNielsPer == 2) {
    pts[2 * i] = p;
    pts[2 * i + 1] = niels_negate(p);
  } else {
    pts[i] = p;
  }
}

struct MsmParams {
  uint32_t m_log2;   // group size = 1 << m_log2 (>= 5, so a 16-signature quad block never spans groups)
  uint32_t c;        // window bits
  uint32_t W;        // windows for a scalar < 2^253: ceil(254 / c)
  uint32_t WR;       // windows for z < 2^128: ceil(129 / c)
  uint32_t H;        // buckets per window = 2^(c-1)
  uint32_t cap;      // sorted-entry slots per group (multiple of kMsmChunkMax)
  uint32_t groups;   // groups allocated = ceil(n / m)
  uint32_t P;        // lanes per window in k_msm_wpart (power of two <= H)
  uint32_t L;        // sorted entries per k_msm_accum lane (16 or 32)
  uint32_t merged;   // key-merged form: R points only, W = WR
  uint32_t sub;      // 1: sub-group bisection (k_msm_subcheck) of failing groups; set by the runtime

  TMV_HD uint32_t m() const { return 1u << m_log2; }
  // windows of the located pass's R weights z (j + 1) < 2^(128 + m_log2)
  // (signed digits need one bit more, as WR for z < 2^128)
  TMV_HD uint32_t WL() const { return (129 + m_log2 + c - 1) / c; }
  TMV_HD uint32_t buckets_per_group() const { return W * H; }
  // Bucket of (window w, |digit| - 1 = i) inside its group: window-major.
  // (|digit|-major, so that k_msm_wpart's lanes -- one per window -- read
  // adjacent buckets, measured slower: k_msm_sort's histogram and scatter
  // lose more than the running sums gain, 122.0-122.8 vs 122.8-123.6 M/s,
  // profiles/r03/ab_join_compact.txt.)
  TMV_HD uint32_t bucket(uint32_t w, uint32_t i) const { return w * H + i; }
  TMV_HD uint32_t chunks_per_group() const { return cap / L; }
  // window-part slots the workspace holds per (group, window).  The located
  // fallback's second MSM runs its running sums with the launch's own P
  // (one lane per window at the located sizes): round 5's 4 lanes per window
  // shortened the chain but cost 2.75x the additions plus the k_msm_wsum
  // join, and a 2.56M launch's 3,744 failing groups are throughput work --
  // C2 bench +1.3% (4 of 4 same-box pairs), 2.56M alone 19.53 / 19.74 ->
  // 19.27 / 19.30 ms, 500k and 1M equal or better
  // (profiles/r06/ab_loc_parts_bench.txt)
  TMV_HD uint32_t wpart_slots() const { return P; }

  static MsmParams make(uint32_t n, uint32_t m_log2, uint32_t c, bool merged = false) {
    MsmParams p;
    p.m_log2 = m_log2;
    p.c = c;
    p.merged = merged ? 1 : 0;
    p.sub = 0;
    p.WR = (129 + c - 1) / c;
    p.W = merged ? p.WR : (254 + c - 1) / c;
    p.H = 1u << (c - 1);
    const uint32_t m = 1u << m_log2;
    // entries per group <= nonzero digits: R weights z < 2^128 (WR windows;
    // the located pass's z (j + 1) < 2^(128 + m_log2), WL windows), A
    // weights and the B scalar < l (W windows)
    const uint32_t rw = p.WR > p.WL() ? p.WR : p.WL();
    const uint32_t slots = merged ? m * p.WR : m * rw + (m + 1) * p.W;
    p.cap = (slots + kMsmChunkMax - 1) / kMsmChunkMax * kMsmChunkMax;
    // chunk length at least the mean bucket size of the low windows (2m / H
    // entries) so buckets rarely span chunks (few partials to merge);
    // measured: 16 beats 8 at m = 64 (C2) and 32 at m = 1024 (1M honest)
    const uint32_t mean = (merged ? m : 2 * m) / p.H;
    p.L = mean <= 16 ? 16 : 32;
    p.groups = (n + m - 1) >> m_log2;
    // P minimises the latency chain: 2 H/P running-sum additions per part,
    // then 3 P additions + log2(H/P) doublings to join the parts
    uint32_t best = ~0u;
    for (uint32_t P = 1; P <= p.H; P *= 2) {
      uint32_t lg = 0;
      while ((p.H / P) >> (lg + 1)) lg++;
      const uint32_t chain = 2 * (p.H / P) + 3 * P + lg;
      if (chain < best) { best = chain; p.P = P; }
    }
    // a launch with this many (group, window) rows is throughput-bound: one
    // lane per window does the fewest additions (2 H, no joins; the parts
    // cost 2 H + ~3 P + log2(H / P) per window) and the window sums are the
    // lanes' T, so k_msm_wsum is skipped.  C2 bench: 82.9 / 84.1 (P = 4) ->
    // 85.0 / 86.2 M/s (P = 1), profiles/r03/ab_parts.txt
    if ((uint64_t)p.groups * p.W >= kMsmWideRows) p.P = 1;
    return p;
  }
};

// Device workspace of the batch check (all per launch stream).
struct MsmWork {
  niels_pt *pts;       // points 2n+1: [2e] = -R_e, [2e+1] = -A_e, [2n] = B; kNielsPer slots each
  uint32_t *ent_pt;    // groups x cap: point index << 1 | negate
  uint32_t *ent_bk;    // groups x cap: global bucket id, kMsmEmpty for padding
  uint32_t *bk_start;  // groups x W x H: first sorted slot of the bucket
  uint32_t *bk_cnt;    // groups x W x H
  ge_p3 *bk_sum;       // groups x W x H: sums of buckets that fit in one chunk
  ge_p3 *part_first;   // chunks: run that began in an earlier chunk and ends here
  ge_p3 *part_last;    // chunks: run that continues into the next chunk
  uint32_t *join_b;    // chunks: the buckets k_msm_join_list joins from their chunk partials, packed at the front,
                       // *join_count of them
  uint32_t *join_count;  // groups: [g0] counts the list of the view starting at group g0 (parts of a
                         // launch may run at once); reset by every k_msm_sort, appended by k_msm_accum
  ge_p3 *wpart;        // groups x W x P x 2: (T, U) of each window part
  ge_p3 *wsum;         // groups x W: window sums
  uint8_t *group_ok;   // groups
  // 1 when a group's bucket entries would not fit its cap slots (cannot
  // happen: MsmParams::make bounds the digits; k_msm_sort then leaves the
  // group empty and the flag fails it).  [g]: group g (k_msm_horner),
  // [groups + f]: the located pass's slot f (k_loc_search)
  uint8_t *sort_ovf;   // 2 x groups
  uint32_t n_pts;      // index of B (= 2n)
  // sub-group bisection of failing groups (k_msm_subcheck; null in the
  // key-merged form, whose fallback is the key-cached comb)
  uint32_t *fail_count;  // failing groups (reset by k_msm_sort, counted by k_msm_horner)
  uint32_t *fail_list;   // groups: ids of the failing groups
  uint8_t *sub_ok;       // groups x m / kSubGroup: verdict of each sub-group of a failing group
  fe *tabR;              // n x 8 x 4 fe: k_msm_subcheck's tables of -R (its -A tables use Ed25519Work::tabA)
  // located fallback (msm_kernels.hip, k_loc_*): failing group f's sums T
  // and T' = sum (j+1) z_j Delta_j, the entries left to verify one by one
  fe *fail_T;            // groups x 8 fe: [8f .. 8f+3] T (P3Q lanes), [8f+4 .. 8f+7] T'
  uint32_t *loc_count;   // failing groups x m: entry count of the locate MSM (device)
  uint32_t *fb_count;    // entries in fb_list
  uint32_t *loc_found;   // failing groups whose one bad entry the search named (tmv_metrics)
  uint32_t *fb_list;     // n: work indices verified one by one
  // key-merged form only (null otherwise)
  uint32_t *wscal;     // n x 8 words: z_e k_e mod l (0 for entries left out)
  uint32_t *bscal;     // groups x 8 words: B scalar of the group
  fe *item_pt;         // (runs + groups) x 4 fe, P3Q: key-run and B-term points

  // item capacity of the key-merged form: runs (<= n + groups) + groups
  static size_t max_items(uint32_t n, const MsmParams &p) { return (size_t)n + 2ull * p.groups; }

  static size_t bytes(uint32_t n, const MsmParams &p) {
    const size_t G = p.groups, bk = (size_t)G * p.buckets_per_group(), ent = (size_t)G * p.cap;
    const size_t chunks = ent / p.L;
    size_t b = (2ull * n + 1) * kNielsPer * sizeof(niels_pt) + 8 * ent + 8 * bk + bk * sizeof(ge_p3) +
               2 * chunks * sizeof(ge_p3) + 4 * chunks + G * p.W * (2ull * p.wpart_slots() + 1) * sizeof(ge_p3) + G + 2 * G +
               18 * 16 + 4 * G;
    if (p.merged) b += 32ull * n + 32 * G + max_items(n, p) * 4 * sizeof(fe);
    else b += 16 + 4 * G + (G << p.m_log2) / kSubGroup + 16 + (size_t)n * 32 * sizeof(fe) + 3 * 16 +
              G * 8 * sizeof(fe) + 16 + 4ull * n + 2 * 16 + 4 * G + 2 * 16 + G * 4 * sizeof(fe) + 16;
    return b;
  }
  static MsmWork carve(void *base, uint32_t n, const MsmParams &p) {
    auto up = [](size_t x) { return (x + 15) & ~size_t(15); };
    uint8_t *b = static_cast<uint8_t *>(base);
    const size_t G = p.groups, bk = (size_t)G * p.buckets_per_group(), ent = (size_t)G * p.cap;
    const size_t chunks = ent / p.L;
    MsmWork w;
    size_t o = 0;
    w.pts = reinterpret_cast<niels_pt *>(b + o); o = up(o + (2ull * n + 1) * kNielsPer * sizeof(niels_pt));
    w.ent_pt = reinterpret_cast<uint32_t *>(b + o); o = up(o + 4 * ent);
    w.ent_bk = reinterpret_cast<uint32_t *>(b + o); o = up(o + 4 * ent);
    w.bk_start = reinterpret_cast<uint32_t *>(b + o); o = up(o + 4 * bk);
    w.bk_cnt = reinterpret_cast<uint32_t *>(b + o); o = up(o + 4 * bk);
    w.bk_sum = reinterpret_cast<ge_p3 *>(b + o); o = up(o + bk * sizeof(ge_p3));
    w.part_first = reinterpret_cast<ge_p3 *>(b + o); o = up(o + chunks * sizeof(ge_p3));
    w.part_last = reinterpret_cast<ge_p3 *>(b + o); o = up(o + chunks * sizeof(ge_p3));
    w.join_b = reinterpret_cast<uint32_t *>(b + o); o = up(o + 4 * chunks);
    w.join_count = reinterpret_cast<uint32_t *>(b + o); o = up(o + 4 * G);
    w.wpart = reinterpret_cast<ge_p3 *>(b + o); o = up(o + G * p.W * 2ull * p.wpart_slots() * sizeof(ge_p3));
    w.wsum = reinterpret_cast<ge_p3 *>(b + o); o = up(o + G * p.W * sizeof(ge_p3));
    w.group_ok = b + o; o = up(o + G);
    w.sort_ovf = b + o; o = up(o + 2 * G);
    w.n_pts = 2 * n;
    w.wscal = w.bscal = nullptr;
    w.item_pt = nullptr;
    w.fail_count = w.fail_list = nullptr;
    w.sub_ok = nullptr;
    w.tabR = nullptr;
    w.fail_T = nullptr;
    w.loc_count = w.fb_count = w.fb_list = w.loc_found = nullptr;
    if (!p.merged) {
      w.fail_count = reinterpret_cast<uint32_t *>(b + o); o = up(o + 16);
      w.fail_list = reinterpret_cast<uint32_t *>(b + o); o = up(o + 4 * G);
      w.sub_ok = b + o; o = up(o + (G << p.m_log2) / kSubGroup);
      w.tabR = reinterpret_cast<fe *>(b + o); o = up(o + (size_t)n * 32 * sizeof(fe));
      w.fail_T = reinterpret_cast<fe *>(b + o); o = up(o + G * 8 * sizeof(fe));
      w.loc_count = reinterpret_cast<uint32_t *>(b + o);
      w.fb_count = w.loc_count + 1;
      w.loc_found = w.loc_count + 2;
      o = up(o + 16);
      w.fb_list = reinterpret_cast<uint32_t *>(b + o); o = up(o + 4ull * n);
    }
    if (p.merged) {
      w.wscal = reinterpret_cast<uint32_t *>(b + o); o = up(o + 32ull * n);
      w.bscal = reinterpret_cast<uint32_t *>(b + o); o = up(o + 32 * G);
      w.item_pt = reinterpret_cast<fe *>(b + o);
    }
    return w;
  }
};

// Per-call randomness: ChaCha20 key (from getrandom, or a caller seed in
// tests) and a nonce that separates the launches of one call.
struct MsmSeed {
  uint32_t key[8];
  uint32_t nonce[3];
};

// ---------------------------------------------------------------- ChaCha20
// RFC 8439 block function; z_e = first 16 bytes of block (key, counter = e,
// nonce).  Row I: the reference draws z from rand.Reader
// (crypto/ed25519/ed25519.go:232).
TMV_HD uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

#define TMV_QR(a, b, c, d)              \
  a += b; d ^= a; d = rotl32(d, 16);    \
  c += d; b ^= c; b = rotl32(b, 12);    \
  a += b; d ^= a; d = rotl32(d, 8);     \
  c += d; b ^= c; b = rotl32(b, 7);

TMV_HD void chacha20_block(uint32_t out[16], const uint32_t key[8], uint32_t counter, const uint32_t nonce[3]) {
  uint32_t x[16];
  x[0] = 0x61707865u; x[1] = 0x3320646eu; x[2] = 0x79622d32u; x[3] = 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; i++) x[4 + i] = key[i];
  x[12] = counter;
  x[13] = nonce[0]; x[14] = nonce[1]; x[15] = nonce[2];
  uint32_t s[16];
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = x[i];
#pragma unroll 1
  for (int r = 0; r < 10; r++) {
    TMV_QR(s[0], s[4], s[8], s[12]);
    TMV_QR(s[1], s[5], s[9], s[13]);
    TMV_QR(s[2], s[6], s[10], s[14]);
    TMV_QR(s[3], s[7], s[11], s[15]);
    TMV_QR(s[0], s[5], s[10], s[15]);
    TMV_QR(s[1], s[6], s[11], s[12]);
    TMV_QR(s[2], s[7], s[8], s[13]);
    TMV_QR(s[3], s[4], s[9], s[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = s[i] + x[i];
}
#undef TMV_QR

// The affine Niels point (y+x, y-x) as an extended point.  (E, H, G, F) =
// (ypx - ymx, ypx + ymx, 2, 2) is the completed form of O + q, so
// X = E F = 2E, Y = H G = 2H, Z = G F = 4, T = E H: one multiply instead of
// the seven of a mixed addition onto the identity.
TMV_HD void niels_to_p3(ge_p3 &r, const fe &ypx, const fe &ymx) {
  fe e, h;
  fe_sub(e, ypx, ymx);  // level 2
  fe_add(h, ypx, ymx);  // level 2
  fe_mul(r.T, e, h);
  fe_add(e, e, e);      // level 4: carried below
  fe_add(h, h, h);
  fe_carry(r.X, e);
  fe_carry(r.Y, h);
  fe_zero(r.Z);
  r.Z.v[0] = 4;
}

// ---------------------------------------------------------------- scalars
// r = (a * b) mod l, a: na words (na <= 8), b: 8 words.
TMV_HD void sc_mul_mod(uint32_t r[8], const uint32_t *a, int na, const uint32_t b[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = 0;
  // unrolled (na is a constant at every call site): with a rolled loop x[i + j]
  // was a run-time register index (s_set_gpr_idx) and x[] partly in scratch
#pragma unroll
  for (int i = 0; i < na; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  sc_reduce512(r, x);
}

// Signed digit of window w (c bits) of a scalar of nw words, given the carry
// of window w-1; top window keeps a digit in [0, 2^(c-1)] (no carry out).
TMV_HD int sc_window_digit(const uint32_t *s, int nw, uint32_t w, uint32_t c, bool top, int &carry) {
  const uint32_t bit = w * c;
  const uint32_t wi = bit >> 5, sh = bit & 31;
  uint64_t x = wi < (uint32_t)nw ? s[wi] : 0;
  if (wi + 1 < (uint32_t)nw) x |= (uint64_t)s[wi + 1] << 32;
  int d = (int)((x >> sh) & ((1u << c) - 1)) + carry;
  if (!top && d >= (1 << (c - 1))) {
    d -= 1 << c;
    carry = 1;
  } else {
    carry = 0;
  }
  return d;
}

}  // namespace tmv
