// Host-side sr25519 key/signature factory for synthetic workloads (the
// analogue of the reference's test factories; input generation only, never
// verification).  Built with g++ from the same arithmetic headers the GPU
// kernels use.  Signing follows schnorrkel (crypto/sr25519/privkey.go:45-65):
// the reference draws the witness from crypto/rand; here it is
// r = SHA-512("witness" || nonce || nonce_seed || M) mod l so fixtures are
// reproducible (verification does not depend on how r was chosen).
#include <openssl/evp.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>
#include "../../csrc/ed25519_core.h"
#include "../../csrc/merlin_dev.h"

using namespace tmv;

namespace {

struct Sha512 {
  uint64_t h[8];
  uint8_t buf[128];
  size_t blen = 0;
  uint64_t total = 0;
  Sha512() { sha512_init(h); }
  void block(const uint8_t *p) {
    uint64_t w[16];
    for (int i = 0; i < 16; i++) {
      uint64_t v = 0;
      for (int j = 0; j < 8; j++) v = (v << 8) | p[8 * i + j];
      w[i] = v;
    }
    sha512_compress(h, w);
  }
  void update(const uint8_t *m, size_t n) {
    total += n;
    while (n) {
      size_t take = std::min<size_t>(128 - blen, n);
      memcpy(buf + blen, m, take);
      blen += take; m += take; n -= take;
      if (blen == 128) { block(buf); blen = 0; }
    }
  }
  void final(uint8_t out[64]) {
    uint64_t bits = total * 8;
    uint8_t pad = 0x80, z = 0;
    update(&pad, 1);
    while (blen != 112) update(&z, 1);
    uint8_t len[16] = {0};
    for (int i = 0; i < 8; i++) len[15 - i] = (uint8_t)(bits >> (8 * i));
    update(len, 16);
    for (int i = 0; i < 8; i++)
      for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(h[i] >> (56 - 8 * j));
  }
};

std::vector<ge_precomp> &table() {
  static std::vector<ge_precomp> t;
  if (t.empty()) {
    t.resize(kBaseTableRows * kBaseTableCols);
    build_base_table(t.data());
  }
  return t;
}

void words(uint32_t w[8], const uint8_t *b) {
  for (int i = 0; i < 8; i++)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
}
void bytes(uint8_t *b, const uint32_t w[8]) {
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 4; j++) b[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

// MiniSecretKey.ExpandEd25519: key = clamp(h[0:32]) / 8, nonce = h[32:64]
void expand(const uint8_t mini[32], uint32_t key[8], uint8_t nonce[32]) {
  Sha512 s;
  s.update(mini, 32);
  uint8_t h[64];
  s.final(h);
  uint8_t k[32];
  memcpy(k, h, 32);
  k[0] &= 248;
  k[31] &= 63;
  k[31] |= 64;
  uint8_t carry = 0;  // divide by 8 (little-endian right shift by 3)
  for (int i = 31; i >= 0; i--) {
    uint8_t v = k[i];
    k[i] = (uint8_t)((v >> 3) | (carry << 5));
    carry = v & 7;
  }
  words(key, k);
  memcpy(nonce, h + 32, 32);
}

// r = a*b + c mod l
void sc_muladd(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t x[16] = {0};
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
    for (int j = 0; j < 8; j++) {
      uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  uint64_t carry = 0;
  for (int i = 0; i < 16; i++) {
    uint64_t t = (uint64_t)x[i] + (i < 8 ? c[i] : 0) + carry;
    x[i] = (uint32_t)t;
    carry = t >> 32;
  }
  sc_reduce512(r, x);
}

size_t put_uvarint(uint8_t *p, uint64_t u) {
  size_t n = 0;
  while (u >= 0x80) {
    p[n++] = (uint8_t)(u | 0x80);
    u >>= 7;
  }
  p[n++] = (uint8_t)u;
  return n;
}

// One commit vote's sign-bytes from its fixed parts (types/vote.go:149-157,
// SURVEY Appendix B): uvarint(L) || head || 2a len {08 secs, 10 nanos} ||
// 32 len chain.  head = the CanonicalVote fields before the timestamp (type,
// height, round, block ID).  Returns the length.
size_t vote_message(uint8_t *out, const uint8_t *head, uint32_t head_len, const uint8_t *chain, uint32_t chain_len,
                    int64_t secs, int32_t nanos) {
  uint8_t ts[24];
  size_t tl = 0;
  if (secs) { ts[tl++] = 0x08; tl += put_uvarint(ts + tl, (uint64_t)secs); }
  if (nanos) { ts[tl++] = 0x10; tl += put_uvarint(ts + tl, (uint64_t)(int64_t)nanos); }
  uint8_t tsl[10], chl[10];
  const size_t tsl_n = put_uvarint(tsl, tl), chl_n = chain_len ? put_uvarint(chl, chain_len) : 0;
  const size_t body = head_len + 1 + tsl_n + tl + (chain_len ? 1 + chl_n + chain_len : 0);
  uint8_t *p = out;
  p += put_uvarint(p, body);
  memcpy(p, head, head_len); p += head_len;
  *p++ = 0x2a; memcpy(p, tsl, tsl_n); p += tsl_n; memcpy(p, ts, tl); p += tl;
  if (chain_len) { *p++ = 0x32; memcpy(p, chl, chl_n); p += chl_n; memcpy(p, chain, chain_len); p += chain_len; }
  return (size_t)(p - out);
}

template <typename F>
void parallel_for(uint32_t n, int threads, F f) {
  if (threads < 1) threads = 1;
  if ((uint32_t)threads > n) threads = n ? (int)n : 1;
  std::vector<std::thread> ts;
  for (int t = 1; t < threads; t++)
    ts.emplace_back([=, &f] { f((uint32_t)((uint64_t)n * t / threads), (uint32_t)((uint64_t)n * (t + 1) / threads)); });
  f(0, (uint32_t)((uint64_t)n / threads));
  for (auto &t : ts) t.join();
}

// Ed25519 point encoding (RFC 8032 §5.1.2): y with the sign of x on bit 255.
void ed25519_encode(uint8_t out[32], const ge_p3 &p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  uint32_t w[8];
  fe_to_words(w, y);
  bytes(out, w);
  if (fe_is_negative(x)) out[31] |= 0x80;
}

void sc_from_hash(uint32_t r[8], const uint8_t h[64]) {
  uint32_t hw[16];
  for (int i = 0; i < 16; i++)
    hw[i] = (uint32_t)h[4 * i] | ((uint32_t)h[4 * i + 1] << 8) | ((uint32_t)h[4 * i + 2] << 16) |
            ((uint32_t)h[4 * i + 3] << 24);
  sc_reduce512(r, hw);
}

// RFC 8032 §5.1.5 key expansion: a = clamp(SHA-512(seed)[0:32]) (kept mod
// l: [a]B is the same point), prefix = SHA-512(seed)[32:64], A = [a]B.
struct Ed25519Key {
  uint32_t a[8];
  uint8_t prefix[32], A[32];
};

Ed25519Key ed25519_expand(const uint8_t seed[32]) {
  Ed25519Key k;
  Sha512 s;
  s.update(seed, 32);
  uint8_t h[64];
  s.final(h);
  h[0] &= 248;
  h[31] &= 63;
  h[31] |= 64;
  uint8_t wide[64] = {0};
  memcpy(wide, h, 32);
  sc_from_hash(k.a, wide);
  memcpy(k.prefix, h + 32, 32);
  ge_p3 A;
  ge_scalarmult_base(A, k.a, table().data());
  ed25519_encode(k.A, A);
  return k;
}

// RFC 8032 §5.1.6: r = SHA-512(prefix || M) mod l, R = [r]B,
// k = SHA-512(R || A || M) mod l, S = r + k a mod l.
void ed25519_sign(uint8_t sig[64], const Ed25519Key &key, const uint8_t *m, size_t mlen) {
  uint8_t h[64];
  Sha512 s1;
  s1.update(key.prefix, 32);
  s1.update(m, mlen);
  s1.final(h);
  uint32_t r[8];
  sc_from_hash(r, h);
  ge_p3 R;
  ge_scalarmult_base(R, r, table().data());
  ed25519_encode(sig, R);
  Sha512 s2;
  s2.update(sig, 32);
  s2.update(key.A, 32);
  s2.update(m, mlen);
  s2.final(h);
  uint32_t k[8], S[8];
  sc_from_hash(k, h);
  sc_muladd(S, k, key.a, r);
  bytes(sig + 32, S);
}

}  // namespace

extern "C" {

// Messages of n commit votes that share every field but the timestamp
// (types/block.go:853-854).  Writes them back to back into out (capacity
// n * (head_len + chain_len + 48) is always enough) and the n + 1 offsets.
// Returns the total length.
size_t tmf_vote_messages(const uint8_t *head, uint32_t head_len, const uint8_t *chain, uint32_t chain_len,
                         const int64_t *secs, const int32_t *nanos, uint32_t n, uint8_t *out, uint32_t *off) {
  size_t o = 0;
  off[0] = 0;
  for (uint32_t i = 0; i < n; i++) {
    o += vote_message(out + o, head, head_len, chain, chain_len, secs[i], nanos[i]);
    off[i + 1] = (uint32_t)o;
  }
  return o;
}

// RFC 8032 Ed25519 signatures of n messages by OpenSSL 3 (byte-identical to
// curve25519-voi ed25519.Sign, crypto/ed25519/ed25519.go:88-91): message i
// (msg[off[i] .. off[i+1])) is signed by key key_idx[i] of the n_keys 32-byte
// seeds.  pk_out (n_keys x 32, may be NULL) receives the public keys.  Input
// generation only.  Returns 0, or -1 if OpenSSL failed.
int tmf_ed25519_sign_many(const uint8_t *seeds, uint32_t n_keys, const uint32_t *key_idx, const uint8_t *msg,
                          const uint32_t *off, uint32_t n, uint8_t *sig_out, uint8_t *pk_out, int threads) {
  std::vector<EVP_PKEY *> keys(n_keys, nullptr);
  bool ok = true;
  for (uint32_t k = 0; k < n_keys && ok; k++) {
    keys[k] = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, seeds + 32ull * k, 32);
    ok = keys[k] != nullptr;
    size_t len = 32;
    if (ok && pk_out) ok = EVP_PKEY_get_raw_public_key(keys[k], pk_out + 32ull * k, &len) == 1 && len == 32;
  }
  std::atomic<bool> good{ok};
  if (ok)
    parallel_for(n, threads, [&](uint32_t lo, uint32_t hi) {
      EVP_MD_CTX *ctx = EVP_MD_CTX_new();
      for (uint32_t i = lo; i < hi && ctx; i++) {
        size_t sl = 64;
        EVP_MD_CTX_reset(ctx);  // a one-shot Ed25519 context signs once
        if (key_idx[i] >= n_keys || EVP_DigestSignInit(ctx, nullptr, nullptr, nullptr, keys[key_idx[i]]) != 1 ||
            EVP_DigestSign(ctx, sig_out + 64ull * i, &sl, msg + off[i], off[i + 1] - off[i]) != 1 || sl != 64) {
          good = false;
          break;
        }
      }
      if (!ctx) good = false;
      EVP_MD_CTX_free(ctx);
    });
  for (EVP_PKEY *k : keys) EVP_PKEY_free(k);
  return good ? 0 : -1;
}

// The same signatures (RFC 8032, deterministic) from this file's own
// arithmetic instead of OpenSSL: ~10x faster per thread and free of
// OpenSSL 3's provider-lock contention, for chain-sized fixtures.
// tests/test_factory.py pins it byte for byte to tmf_ed25519_sign_many.
int tmf_ed25519_sign_fast(const uint8_t *seeds, uint32_t n_keys, const uint32_t *key_idx, const uint8_t *msg,
                          const uint32_t *off, uint32_t n, uint8_t *sig_out, int threads) {
  for (uint32_t i = 0; i < n; i++)
    if (key_idx[i] >= n_keys) return -1;
  (void)table();  // built once, before the threads read it
  std::vector<Ed25519Key> keys(n_keys);
  parallel_for(n_keys, threads, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t k = lo; k < hi; k++) keys[k] = ed25519_expand(seeds + 32ull * k);
  });
  parallel_for(n, threads, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; i++)
      ed25519_sign(sig_out + 64ull * i, keys[key_idx[i]], msg + off[i], off[i + 1] - off[i]);
  });
  return 0;
}

void tmf_sr25519_public_key(const uint8_t mini[32], uint8_t pk[32]) {
  uint32_t key[8];
  uint8_t nonce[32];
  expand(mini, key, nonce);
  ge_p3 A;
  ge_scalarmult_base(A, key, table().data());
  uint32_t w[8];
  ristretto_encode(w, A);
  bytes(pk, w);
}

void tmf_sr25519_sign(const uint8_t mini[32], const uint8_t *msg, size_t mlen, const uint8_t *nonce_seed,
                      size_t seed_len, uint8_t sig[64]) {
  uint32_t key[8];
  uint8_t nonce[32];
  expand(mini, key, nonce);
  ge_p3 A;
  ge_scalarmult_base(A, key, table().data());
  uint32_t pk_w[8];
  ristretto_encode(pk_w, A);
  // witness
  Sha512 s;
  s.update(reinterpret_cast<const uint8_t *>("witness"), 7);
  s.update(nonce, 32);
  s.update(nonce_seed, seed_len);
  s.update(msg, mlen);
  uint8_t h[64];
  s.final(h);
  uint32_t hw[16], r[8];
  for (int i = 0; i < 16; i++)
    hw[i] = (uint32_t)h[4 * i] | ((uint32_t)h[4 * i + 1] << 8) | ((uint32_t)h[4 * i + 2] << 16) |
            ((uint32_t)h[4 * i + 3] << 24);
  sc_reduce512(r, hw);
  ge_p3 R;
  ge_scalarmult_base(R, r, table().data());
  uint32_t r_w[8];
  ristretto_encode(r_w, R);
  strobe_t prefix;
  sr25519_context_prefix(prefix);
  uint32_t k[8];
  sr25519_challenge(k, prefix, pk_w, r_w, msg, (uint32_t)mlen);
  uint32_t sc[8];
  sc_muladd(sc, k, key, r);
  bytes(sig, r_w);
  bytes(sig + 32, sc);
  sig[63] |= 0x80;
}

}  // extern "C"
