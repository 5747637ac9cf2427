// One-signature sr25519 (Schnorrkel) verification, host+device, matching
// crypto/sr25519/pubkey.go:49-62 and the Add-time checks of
// crypto/sr25519/batch.go:30-37.  Status: 1 valid, 0 invalid,
// -1 public key does not decode (Add error), -2 signature encoding rejected
// (marker bit / non-canonical s: Add error).
#pragma once
#include "ed25519_core.h"
#include "merlin_dev.h"

namespace tmv {

TMV_HD int sr25519_verify_core(const uint32_t pk_w[8], const uint32_t r_w[8], const uint32_t s_w[8],
                               const uint8_t *msg, uint32_t mlen, const strobe_t &prefix,
                               const ge_precomp *btable) {
  ge_p3 A, R;
  if (!ristretto_decode(A, pk_w)) return -1;
  uint32_t s[8];
  if (!sr25519_decode_s(s, s_w)) return -2;
  if (!ristretto_decode(R, r_w)) return 0;
  uint32_t k[8];
  sr25519_challenge(k, prefix, pk_w, r_w, msg, mlen);
  ge_p3 sB, kA, Rp;
  ge_scalarmult_base(sB, s, btable);
  ge_scalarmult_var(kA, k, A);
  ge_cached c;
  ge_p1p1 t;
  ge_p3_to_cached(c, kA);
  ge_sub(t, sB, c);
  ge_p1p1_to_p3(Rp, t);
  return ristretto_equal(Rp, R) ? 1 : 0;
}

}  // namespace tmv
