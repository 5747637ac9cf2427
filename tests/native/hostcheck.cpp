// Host build of the exact device arithmetic (tendermint_amd/csrc/*.h) with
// limb-bound assertions (TMV_BOUNDS_CHECK).  Loaded by tests/test_arith_host.py
// and compared with the CPU oracle; no GPU needed.
#include <cstdint>
#include <cstring>
#include <vector>
#include "../../tendermint_amd/csrc/ed25519_core.h"
#include "../../tendermint_amd/csrc/sr25519_core.h"
#include "../../tendermint_amd/csrc/halfscalar.h"

using namespace tmv;

static std::vector<ge_precomp> g_table;

static void load_words(uint32_t w[8], const uint8_t *b) {
  for (int i = 0; i < 8; i++)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
}

extern "C" int hostcheck_ed25519_verify_batch(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                              const uint32_t *off, uint32_t n, uint8_t *out) {
  if (g_table.empty()) {
    g_table.resize(kBaseTableRows * kBaseTableCols);
    build_base_table(g_table.data());
  }
  int all = n > 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t a[8], r[8], s[8];
    load_words(a, pk + 32 * i);
    load_words(r, sig + 64 * i);
    load_words(s, sig + 64 * i + 32);
    out[i] = ed25519_verify_core(a, r, s, msg + off[i], off[i + 1] - off[i], g_table.data());
    all &= out[i];
  }
  return all;
}

extern "C" void hostcheck_sc_reduce512(const uint8_t in[64], uint8_t out[32]) {
  uint32_t x[16], r[8];
  for (int i = 0; i < 16; i++)
    x[i] = (uint32_t)in[4 * i] | ((uint32_t)in[4 * i + 1] << 8) | ((uint32_t)in[4 * i + 2] << 16) |
           ((uint32_t)in[4 * i + 3] << 24);
  sc_reduce512(r, x);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(r[i] >> (8 * j));
}

// fe_mul_par (two-round carry, the quad formulas' TMV_QUAD_PCARRY form)
// against fe_mul on limbs given directly (level <= 3 extremes included):
// `rounds` chained products of each; returns 1 when every pair encodes the
// same element (the limb bounds are asserted under TMV_BOUNDS_CHECK).
extern "C" int hostcheck_fe_mul_par(const int32_t fl[10], const int32_t gl[10], int rounds) {
  fe x, y, a, b;
  for (int i = 0; i < 10; i++) { x.v[i] = fl[i]; y.v[i] = gl[i]; }
  fe_mul(a, x, y);
  fe_mul_par(b, x, y);
  for (int r = 0; r <= rounds; r++) {
    uint32_t wa[8], wb[8];
    fe_to_words(wa, a);
    fe_to_words(wb, b);
    for (int i = 0; i < 8; i++)
      if (wa[i] != wb[i]) return 0;
    fe t;
    fe_add(t, b, b);  // level 2 (from the slightly wider par output)
    fe_add(t, t, b);  // ~level 3
    fe sa;
    fe_add(sa, a, a);
    fe_add(sa, sa, a);
    fe_mul(a, sa, a);
    fe_mul_par(b, t, b);
  }
  return 1;
}

// fe_pow22523 (the square-root exponent (p - 5) / 8; fe_sqn's floor-carry
// squarings inside) and fe_invert of a 32-byte input.
extern "C" void hostcheck_fe_pow(const uint8_t a[32], uint8_t pow_out[32], uint8_t inv_out[32]) {
  uint32_t w[8];
  memcpy(w, a, 32);
  fe x, y;
  fe_from_words(x, w);
  fe_pow22523(y, x);
  fe_to_words(w, y);
  memcpy(pow_out, w, 32);
  fe_from_words(x, reinterpret_cast<const uint32_t *>(a));
  fe_invert(y, x);
  fe_to_words(w, y);
  memcpy(inv_out, w, 32);
}

extern "C" void hostcheck_fe_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  fe x, y, z;
  fe_from_bytes(x, a);
  fe_from_bytes(y, b);
  fe_carry(x, x);
  fe_carry(y, y);
  fe_mul(z, x, y);
  uint32_t w[8];
  fe_to_words(w, z);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

extern "C" void hostcheck_sha512_pq_msg(const uint8_t *p, const uint8_t *q, const uint8_t *m, uint32_t mlen,
                                        uint8_t out[64]) {
  uint32_t P[8], Q[8], h[16];
  load_words(P, p);
  load_words(Q, q);
  sha512_pq_msg(h, P, Q, m, mlen);
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
}

extern "C" void hostcheck_sr25519_status_batch(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                               const uint32_t *off, uint32_t n, int8_t *out) {
  if (g_table.empty()) {
    g_table.resize(kBaseTableRows * kBaseTableCols);
    build_base_table(g_table.data());
  }
  strobe_t prefix;
  sr25519_context_prefix(prefix);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t a[8], r[8], s[8];
    load_words(a, pk + 32 * i);
    load_words(r, sig + 64 * i);
    load_words(s, sig + 64 * i + 32);
    out[i] = (int8_t)sr25519_verify_core(a, r, s, msg + off[i], off[i + 1] - off[i], prefix, g_table.data());
  }
}

extern "C" void hostcheck_merlin_test(uint8_t out[32]) {
  // merlin "test protocol" vector through the same STROBE code
  strobe_t s;
  strobe_init(s);
  strobe_begin_op(s, 16 | 2);
  strobe_absorb(s, reinterpret_cast<const uint8_t *>("Merlin v1.0"), 11);
  merlin_append(s, "dom-sep", 7, reinterpret_cast<const uint8_t *>("test protocol"), 13);
  merlin_append(s, "some label", 10, reinterpret_cast<const uint8_t *>("some data"), 9);
  strobe_begin_op(s, 16 | 2);
  strobe_absorb(s, reinterpret_cast<const uint8_t *>("challenge"), 9);
  const uint8_t len[4] = {32, 0, 0, 0};
  strobe_absorb(s, len, 4);
  strobe_begin_op(s, 1 | 2 | 4);
  strobe_prf(s, out, 32);
}

// Device ChaCha20 block function (msm.h, row I: the batch weights z_i) on the
// host: key and nonce as RFC 8439 bytes (little-endian words), one block.
#include "../../tendermint_amd/csrc/msm.h"
extern "C" void hostcheck_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                                         uint8_t out[64]) {
  uint32_t k[8], n[3], o[16];
  load_words(k, key);
  for (int i = 0; i < 3; i++)
    n[i] = (uint32_t)nonce[4 * i] | ((uint32_t)nonce[4 * i + 1] << 8) | ((uint32_t)nonce[4 * i + 2] << 16) |
           ((uint32_t)nonce[4 * i + 3] << 24);
  chacha20_block(o, k, counter, n);
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(o[i] >> (8 * j));
}

// sr25519 challenge k for (pk, R, M) through the generic STROBE path (fast =
// 0) or the register-state transcript for vote-sized messages (fast = 1;
// returns 0 when the message length is outside its range).
extern "C" int hostcheck_sr25519_challenge(const uint8_t pk[32], const uint8_t r[32], const uint8_t *m, uint32_t mlen,
                                           int fast, uint8_t out[32]) {
  strobe_t prefix;
  sr25519_context_prefix(prefix);
  uint32_t a[8], rw[8], k[8];
  load_words(a, pk);
  load_words(rw, r);
  if (fast) {
    if (!sr25519_fast_eligible(prefix, mlen)) return 0;
    uint64_t slot[25];
    for (int i = 0; i < 25; i++) slot[i] = 0x0123456789abcdefULL * (i + 1);  // stale LDS contents
    sr25519_challenge_fast<1>(k, prefix, slot, a, rw, m, mlen);
  } else {
    sr25519_challenge(k, prefix, a, rw, m, mlen);
  }
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(k[i] >> (8 * j));
  return 1;
}

// ge_p1p1_to_cached (the running sums' U) against p1p1_to_p3 + p3_to_cached
// on points decoded from the given encodings, each added to the next: returns
// the number of (point, coordinate) pairs that differ (0 expected).
extern "C" int hostcheck_p1p1_to_cached(const uint8_t *enc, uint32_t n) {
  int bad = 0, pairs = 0;  // -1 when fewer than 50 pairs decoded (nothing checked)
  for (uint32_t i = 0; i + 1 < n; i++) {
    uint32_t w0[8], w1[8];
    load_words(w0, enc + 32 * i);
    load_words(w1, enc + 32 * (i + 1));
    ge_p3 a, b;
    if (!ge_decode_zip215(a, w0) || !ge_decode_zip215(b, w1)) continue;
    pairs++;
    ge_cached bc, direct, via;
    ge_p3_to_cached(bc, b);
    ge_p1p1 r;
    ge_add(r, a, bc);
    ge_p1p1_to_cached(direct, r);
    ge_p3 p;
    ge_p1p1_to_p3(p, r);
    ge_p3_to_cached(via, p);
    const fe *x[4] = {&direct.YpX, &direct.YmX, &direct.Z, &direct.T2d};
    const fe *y[4] = {&via.YpX, &via.YmX, &via.Z, &via.T2d};
    for (int c = 0; c < 4; c++) {
      uint32_t u[8], v[8];
      fe t;
      fe_carry(t, *x[c]);
      fe_to_words(u, t);
      fe_carry(t, *y[c]);
      fe_to_words(v, t);
      if (std::memcmp(u, v, sizeof u)) bad++;
    }
  }
  return pairs < 50 ? -1 : bad;
}

// ---------------------------------------------------------------------------
// Half-size scalars (halfscalar.h): the lattice reduction and the short
// verification equation, on the host with single-lane point arithmetic.

// k (32 bytes LE, k < l) -> u (16 bytes, magnitude), v (16 bytes), *u_neg;
// returns 1 when the reduction finished (fast path), 0 for the slow path.
extern "C" int hostcheck_half_reduce(const uint8_t k32[32], uint8_t u16[16], uint8_t v16[16], int *u_neg) {
  uint32_t k[8], u[4], v[4];
  load_words(k, k32);
  bool neg = false;
  const bool ok = half::reduce(u, neg, v, k);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      u16[4 * i + j] = (uint8_t)(u[i] >> (8 * j));
      v16[4 * i + j] = (uint8_t)(v[i] >> (8 * j));
    }
  *u_neg = neg ? 1 : 0;
  return ok ? 1 : 0;
}

// acc = sigma ([b]B + [|u|](-R)) + [v](-A) with single-lane arithmetic
static void half_acc(ge_p3 &acc, const half::Scalars &sc, const ge_p3 &A, const ge_p3 &R) {
  ge_p3 nA, nR, bB, uR, vA;
  ge_p3_neg(nA, A);
  ge_p3_neg(nR, R);
  ge_scalarmult_base(bB, sc.b, g_table.data());
  ge_scalarmult_var(uR, sc.u, nR);
  ge_scalarmult_var(vA, sc.v, nA);
  ge_cached c;
  ge_p1p1 t;
  ge_p3 x;
  ge_p3_to_cached(c, uR);
  ge_add(t, bB, c);
  ge_p1p1_to_p3(x, t);
  if (sc.u_neg) ge_p3_neg(x, x);
  ge_p3_to_cached(c, vA);
  ge_add(t, x, c);
  ge_p1p1_to_p3(acc, t);
}

// ed25519 (sr = 0: 1 / 0) or sr25519 (sr = 1: 1 / 0 / -1 / -2) verification
// through the half-size scalars; *n_slow counts entries on the slow path.
extern "C" void hostcheck_verify_half(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *off,
                                      uint32_t n, int sr, int8_t *out, int *n_slow) {
  if (g_table.empty()) {
    g_table.resize(kBaseTableRows * kBaseTableCols);
    build_base_table(g_table.data());
  }
  strobe_t prefix;
  sr25519_context_prefix(prefix);
  int slow = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t a[8], r[8], s[8], k[8];
    load_words(a, pk + 32 * i);
    load_words(r, sig + 64 * i);
    load_words(s, sig + 64 * i + 32);
    ge_p3 A, R, acc;
    const uint8_t *m = msg + off[i];
    const uint32_t mlen = off[i + 1] - off[i];
    if (sr) {
      uint32_t sd[8];
      if (!ristretto_decode(A, a)) { out[i] = -1; continue; }
      if (!sr25519_decode_s(sd, s)) { out[i] = -2; continue; }
      if (!ristretto_decode(R, r)) { out[i] = 0; continue; }
      sr25519_challenge(k, prefix, a, r, m, mlen);
      half::Scalars sc;
      half::scalars(sc, k, sd);
      slow += sc.fast ? 0 : 1;
      half_acc(acc, sc, A, R);
      out[i] = (fe_is_zero(acc.X) || fe_is_zero(acc.Y)) ? 1 : 0;  // Ristretto identity
    } else {
      if (!sc_is_canonical(s) || !ge_decode_zip215(A, a) || !ge_decode_zip215(R, r)) { out[i] = 0; continue; }
      uint32_t h[16];
      sha512_pq_msg(h, r, a, m, mlen);
      sc_reduce512(k, h);
      half::Scalars sc;
      half::scalars(sc, k, s);
      slow += sc.fast ? 0 : 1;
      half_acc(acc, sc, A, R);
      out[i] = ge_p3_is_small_order_or_identity_times8(acc) ? 1 : 0;
    }
  }
  *n_slow = slow;
}

// Verdicts on a never-computed point (0 : 0 : 0 : 0) -- e.g. an unwritten,
// zeroed workspace slot -- and on the identity: returns 1 when every
// identity / equality check rejects the former and accepts the latter.
extern "C" int hostcheck_degenerate_verdicts() {
  ge_p3 z, id;
  fe_zero(z.X); fe_zero(z.Y); fe_zero(z.Z); fe_zero(z.T);
  ge_p3_identity(id);
  const bool rej = !ge_p3_is_identity(z) && !ge_p3_is_small_order_or_identity_times8(z) &&
                   !ristretto_equal(z, id) && !ristretto_equal(id, z) && !ristretto_equal(z, z);
  const bool acc = ge_p3_is_identity(id) && ge_p3_is_small_order_or_identity_times8(id) && ristretto_equal(id, id);
  return rej && acc ? 1 : 0;
}
