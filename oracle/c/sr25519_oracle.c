/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle for sr25519 (Schnorrkel / Ristretto255
 * / merlin), restating the published algorithm behind
 *   crypto/sr25519/pubkey.go:49-62   PubKey.VerifySignature
 *   crypto/sr25519/batch.go:23-47    BatchVerifier.Add / Verify
 *   crypto/sr25519/privkey.go:18     empty signing context
 * implemented upstream in curve25519-voi primitives/sr25519 (go.mod:22,
 * absent).  Pinned against oracle/sr25519_ref.py by tests/test_oracle.py.
 */
#include <stdint.h>
#include <string.h>
#include <pthread.h>

#include "sha512.h"
#include "keccak.h"
#include "oracle_common.h"

/* (was_square, r): r = sqrt(u/v) or sqrt(i u / v), non-negative */
static int fe_sqrt_ratio_i(fe *r, const fe *u, const fe *v) {
    fe v3, v7, t, check, nu, nui, rp;
    fe_sq(&v3, v); fe_mul(&v3, &v3, v);
    fe_sq(&v7, &v3); fe_mul(&v7, &v7, v);
    fe_mul(&t, u, &v7);
    fe_pow22523(&t, &t);
    fe_mul(&t, &t, &v3); fe_mul(r, &t, u);
    fe_sq(&check, r); fe_mul(&check, &check, v);
    fe_neg(&nu, u);
    fe_mul(&nui, &nu, &FE_SQRTM1);
    int correct = fe_eq(&check, u);
    int flipped = fe_eq(&check, &nu);
    int flipped_i = fe_eq(&check, &nui);
    fe_mul(&rp, r, &FE_SQRTM1);
    if (flipped || flipped_i) *r = rp;
    if (fe_isneg(r)) fe_neg(r, r);
    return correct || flipped;
}

static int ristretto_decode(ge *p, const uint8_t b[32]) {
    fe s, ss, u1, u2, u2sq, v, t, I, Dx, Dy, x, y, one;
    uint8_t chk[32];
    fe_frombytes(&s, b);
    fe_tobytes(chk, &s);
    if (memcmp(chk, b, 32) != 0) return 0; /* non-canonical (>= p or bit 255) */
    if (fe_isneg(&s)) return 0;
    fe_1(&one);
    fe_sq(&ss, &s);
    fe_sub(&u1, &one, &ss);
    fe_add(&u2, &one, &ss);
    fe_sq(&u2sq, &u2);
    fe_sq(&t, &u1); fe_mul(&t, &t, &FE_D); fe_neg(&t, &t);
    fe_sub(&v, &t, &u2sq);
    fe_mul(&t, &v, &u2sq);
    int ok = fe_sqrt_ratio_i(&I, &one, &t);
    fe_mul(&Dx, &I, &u2);
    fe_mul(&Dy, &I, &Dx); fe_mul(&Dy, &Dy, &v);
    fe_add(&x, &s, &s); fe_mul(&x, &x, &Dx);
    if (fe_isneg(&x)) fe_neg(&x, &x);
    fe_mul(&y, &u1, &Dy);
    fe_mul(&t, &x, &y);
    if (!ok || fe_isneg(&t) || fe_iszero(&y)) return 0;
    p->X = x; p->Y = y; fe_1(&p->Z); p->T = t;
    return 1;
}

static int ristretto_eq(const ge *a, const ge *b) {
    fe l, r;
    fe_mul(&l, &a->X, &b->Y); fe_mul(&r, &a->Y, &b->X);
    if (fe_eq(&l, &r)) return 1;
    fe_mul(&l, &a->Y, &b->Y); fe_mul(&r, &a->X, &b->X);
    return fe_eq(&l, &r);
}

/* status codes shared with the product C-ABI (include/tmverify.h) */
#define SR_OK 1
#define SR_INVALID 0
#define SR_ADDERR_PUBKEY (-1)
#define SR_ADDERR_SIG (-2)

/* Add-time checks: returns 0 if Add would succeed, else SR_ADDERR_* */
int oracle_sr25519_add_check(const uint8_t *pk, const uint8_t *sig) {
    init_consts();
    ge A;
    if (!ristretto_decode(&A, pk)) return SR_ADDERR_PUBKEY;
    if (!(sig[63] & 128)) return SR_ADDERR_SIG;
    uint8_t s[32];
    memcpy(s, sig + 32, 32);
    s[31] &= 127;
    if (!sc_is_canonical(s)) return SR_ADDERR_SIG;
    return 0;
}

int oracle_sr25519_verify(const uint8_t *pk, const uint8_t *msg, size_t mlen, const uint8_t *sig) {
    init_consts();
    if (oracle_sr25519_add_check(pk, sig) != 0) return 0;
    ge A, R;
    ristretto_decode(&A, pk);
    if (!ristretto_decode(&R, sig)) return 0;
    uint8_t s[32];
    memcpy(s, sig + 32, 32);
    s[31] &= 127;
    merlin_t t;
    merlin_init(&t, "SigningContext");
    merlin_append(&t, "", (const uint8_t *)"", 0);
    merlin_append(&t, "sign-bytes", msg, mlen);
    merlin_append(&t, "proto-name", (const uint8_t *)"Schnorr-sig", 11);
    merlin_append(&t, "sign:pk", pk, 32);
    merlin_append(&t, "sign:R", sig, 32);
    uint8_t wide[64], k[32];
    merlin_challenge(&t, "sign:c", wide, 64);
    sc_reduce64(k, wide);
    ge nA, Rp;
    ge_neg(&nA, &A);
    ge_double_scalarmult(&Rp, s, &GE_B, k, &nA);
    return ristretto_eq(&Rp, &R);
}

typedef struct {
    const uint8_t *pk, *sig, *msg; const uint32_t *off; int8_t *out; size_t lo, hi;
} srjob_t;

static void *sr_worker(void *arg) {
    srjob_t *j = (srjob_t *)arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        int a = oracle_sr25519_add_check(j->pk + 32 * i, j->sig + 64 * i);
        j->out[i] = a ? (int8_t)a
                      : (int8_t)oracle_sr25519_verify(j->pk + 32 * i, j->msg + j->off[i],
                                                      j->off[i + 1] - j->off[i], j->sig + 64 * i);
    }
    return NULL;
}

/* per-entry status: 1 valid, 0 invalid, <0 Add error */
void oracle_sr25519_status_batch(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                 const uint32_t *msg_off, size_t n, int8_t *out, int threads) {
    init_consts();
    if (n == 0) return;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if ((size_t)threads > n) threads = (int)n;
    pthread_t th[256];
    srjob_t jobs[256];
    size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t lo = t * per, hi = (t + 1) * per < n ? (t + 1) * per : n;
        if (lo > hi) lo = hi;
        jobs[t] = (srjob_t){pk, sig, msg, msg_off, out, lo, hi};
        if (threads == 1) sr_worker(&jobs[t]); else pthread_create(&th[t], NULL, sr_worker, &jobs[t]);
    }
    if (threads > 1) for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

void oracle_merlin_test(uint8_t out[32]) {
    merlin_t t;
    merlin_init(&t, "test protocol");
    merlin_append(&t, "some label", (const uint8_t *)"some data", 9);
    merlin_challenge(&t, "challenge", out, 32);
}

int oracle_ristretto_decode(const uint8_t b[32], uint8_t x_out[32], uint8_t y_out[32]) {
    init_consts();
    ge p;
    if (!ristretto_decode(&p, b)) return 0;
    fe_tobytes(x_out, &p.X); fe_tobytes(y_out, &p.Y);
    return 1;
}
