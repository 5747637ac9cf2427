// Host-side sr25519 key/signature factory for synthetic workloads (the
// analogue of the reference's test factories; input generation only, never
// verification).  Built with g++ from the same arithmetic headers the GPU
// kernels use.  Signing follows schnorrkel (crypto/sr25519/privkey.go:45-65):
// the reference draws the witness from crypto/rand; here it is
// r = SHA-512("witness" || nonce || nonce_seed || M) mod l so fixtures are
// reproducible (verification does not depend on how r was chosen).
#include <cstdint>
#include <cstring>
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

}  // namespace

extern "C" {

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
