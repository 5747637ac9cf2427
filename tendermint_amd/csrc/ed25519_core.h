// One-signature ZIP-215 ed25519 verification, written once for the device
// kernels and the host-side arithmetic test.
//
// Contract (crypto/ed25519/ed25519.go:27-29,173-180; curve25519-voi
// VerifyOptionsZIP_215, go.mod:22):
//   S < l (strict)             -> else reject
//   A, R decode (lax, ZIP-215) -> else reject
//   k = SHA-512(R || A || M) mod l, on the original 32-byte encodings
//   accept iff [8]([S]B - R - [k]A) == O
#pragma once
#include "curve25519.h"
#include "sha512_dev.h"

namespace tmv {

// Base-point comb table: entry (j, m) = (m+1) * 256^j * B, j < 32, m < 8,
// affine Niels form.  30,720 bytes; built once per device by the runtime.
constexpr int kBaseTableRows = 32;
constexpr int kBaseTableCols = 8;

TMV_HD void ge_precomp_select(ge_precomp &t, const ge_precomp *row, int e) {
  const int neg = e < 0;
  const int a = neg ? -e : e;
  if (a == 0) {
    ge_precomp_identity(t);
  } else {
    t = row[a - 1];
  }
  if (neg) {
    fe tmp = t.ypx;
    t.ypx = t.ymx;
    t.ymx = tmp;
    fe_neg(t.xy2d, t.xy2d);
  }
}

TMV_HD void ge_cached_identity(ge_cached &c) {
  fe_one(c.YpX); fe_one(c.YmX); fe_one(c.Z); fe_zero(c.T2d);
}

// h = [s]B with s < 2^255, via the 32x8 comb: sum odd digits, x16, sum even.
TMV_HD void ge_scalarmult_base(ge_p3 &h, const uint32_t s[8], const ge_precomp *table) {
  int8_t e[64];
  sc_signed_radix16(e, s);
  ge_p1p1 r;
  ge_p2 s2;
  ge_precomp t;
  ge_p3_identity(h);
  for (int i = 1; i < 64; i += 2) {
    ge_precomp_select(t, table + (i / 2) * kBaseTableCols, e[i]);
    ge_madd(r, h, t);
    ge_p1p1_to_p3(h, r);
  }
  ge_p3_dbl(r, h);  ge_p1p1_to_p2(s2, r);
  ge_p2_dbl(r, s2); ge_p1p1_to_p2(s2, r);
  ge_p2_dbl(r, s2); ge_p1p1_to_p2(s2, r);
  ge_p2_dbl(r, s2); ge_p1p1_to_p3(h, r);
  for (int i = 0; i < 64; i += 2) {
    ge_precomp_select(t, table + (i / 2) * kBaseTableCols, e[i]);
    ge_madd(r, h, t);
    ge_p1p1_to_p3(h, r);
  }
}

// h = [s]P with s < 2^255, signed radix-16 fixed windows (63 x (4 dbl + 1 add)).
TMV_HD void ge_scalarmult_var(ge_p3 &h, const uint32_t s[8], const ge_p3 &P) {
  int8_t e[64];
  sc_signed_radix16(e, s);
  ge_cached tab[8];
  ge_p1p1 r;
  ge_p2 q;
  ge_p3 t;
  // tab[m] = (m+1) P
  ge_p3_to_cached(tab[0], P);
  ge_p3_dbl(r, P);
  ge_p1p1_to_p3(t, r);
  ge_p3_to_cached(tab[1], t);
  for (int m = 2; m < 8; m++) {
    ge_add(r, P, tab[m - 1]);   // (m+1)P = P + mP
    ge_p1p1_to_p3(t, r);
    ge_p3_to_cached(tab[m], t);
  }
  ge_p3_identity(h);
  for (int i = 63; i >= 0; i--) {
    if (i != 63) {
      ge_p3_dbl(r, h);  ge_p1p1_to_p2(q, r);
      ge_p2_dbl(r, q);  ge_p1p1_to_p2(q, r);
      ge_p2_dbl(r, q);  ge_p1p1_to_p2(q, r);
      ge_p2_dbl(r, q);  ge_p1p1_to_p3(h, r);
    }
    const int ei = e[i];
    const int a = ei < 0 ? -ei : ei;
    ge_cached c;
    if (a == 0) {
      ge_cached_identity(c);
    } else {
      c = tab[a - 1];
    }
    if (ei < 0) {
      ge_sub(r, h, c);
    } else {
      ge_add(r, h, c);
    }
    ge_p1p1_to_p3(h, r);
  }
}

// Full single verification.  pk_w, r_w, s_w: 8 little-endian words each.
TMV_HD bool ed25519_verify_core(const uint32_t pk_w[8], const uint32_t r_w[8], const uint32_t s_w[8],
                                const uint8_t *msg, uint32_t mlen, const ge_precomp *btable) {
  if (!sc_is_canonical(s_w)) return false;
  ge_p3 A, R;
  if (!ge_decode_zip215(A, pk_w)) return false;
  if (!ge_decode_zip215(R, r_w)) return false;
  uint32_t h[16], k[8];
  sha512_pq_msg(h, r_w, pk_w, msg, mlen);
  sc_reduce512(k, h);
  // Q = [S]B - [k]A - R
  ge_p3 sB, kA, Q;
  ge_scalarmult_base(sB, s_w, btable);
  ge_scalarmult_var(kA, k, A);
  ge_cached c;
  ge_p1p1 r;
  ge_p3_to_cached(c, kA);
  ge_sub(r, sB, c);
  ge_p1p1_to_p3(Q, r);
  ge_p3_to_cached(c, R);
  ge_sub(r, Q, c);
  ge_p1p1_to_p3(Q, r);
  return ge_p3_is_small_order_or_identity_times8(Q);
}

// Base-point table construction (host or device).
TMV_HD void ge_p3_to_precomp(ge_precomp &o, const ge_p3 &p) {
  fe zi, x, y, t;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_add(t, y, x); fe_carry(o.ypx, t);
  fe_sub(t, y, x); fe_carry(o.ymx, t);
  fe_mul(t, x, y);
  fe_mul(o.xy2d, t, consts::d2());
}

TMV_HD void ed25519_base_point(ge_p3 &B) {
  // y = 4/5, x even: encoding 0x58 0x66 ... 0x66
  uint32_t w[8];
  w[0] = 0x66666658u;
  for (int i = 1; i < 8; i++) w[i] = 0x66666666u;
  ge_decode_zip215(B, w);
}

inline void build_base_table(ge_precomp *table) {
  ge_p3 B, P, Q;
  ed25519_base_point(B);
  P = B;
  for (int j = 0; j < kBaseTableRows; j++) {
    ge_cached pc;
    ge_p3_to_cached(pc, P);
    Q = P;
    for (int m = 0; m < kBaseTableCols; m++) {
      ge_p3_to_precomp(table[j * kBaseTableCols + m], Q);
      ge_p1p1 r;
      ge_add(r, Q, pc);
      ge_p1p1_to_p3(Q, r);
    }
    // P *= 256
    for (int d = 0; d < 8; d++) {
      ge_p1p1 r;
      ge_p3_dbl(r, P);
      ge_p1p1_to_p3(P, r);
    }
  }
}

}  // namespace tmv
