/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load this library; the product path never
 * does.
 *
 * Plain-C restatement of the ed25519 ZIP-215 verification Tendermint runs
 * behind crypto.BatchVerifier:
 *   crypto/ed25519/ed25519.go:27-29    verify options = ZIP-215
 *   crypto/ed25519/ed25519.go:173-180  PubKey.VerifySignature
 *   crypto/ed25519/ed25519.go:209-233  BatchVerifier.Add / Verify
 * The arithmetic follows the published algorithm of the (absent) third-party
 * module github.com/oasisprotocol/curve25519-voi
 * v0.0.0-20210609091139-0a56a4bca00b (go.mod:22): lax point decoding,
 * strict S < l, k = SHA-512(R||A||M) mod l, cofactored [8]([S]B-R-[k]A) == O.
 * Batch semantics: empty -> (0, no vector); vector == per-entry verify.
 *
 * Pinned against oracle/ed25519_ref.py (itself pinned to OpenSSL and
 * RFC 8032) by tests/test_oracle.py.
 *
 * Field arithmetic (radix 2^51) lives in oracle_common.h.
 */
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#include "sha512.h"

#include "oracle_common.h"

int oracle_ed25519_verify(const uint8_t *pk, const uint8_t *msg, size_t mlen, const uint8_t *sig) {
    init_consts();
    if (!sc_is_canonical(sig + 32)) return 0;
    ge A, R;
    if (!ge_decode_lax(&A, pk)) return 0;
    if (!ge_decode_lax(&R, sig)) return 0;
    uint8_t h[64], k[32];
    sha512_ctx c;
    sha512_init(&c);
    sha512_update(&c, sig, 32);
    sha512_update(&c, pk, 32);
    sha512_update(&c, msg, mlen);
    sha512_final(&c, h);
    sc_reduce64(k, h);
    /* Q = [S]B + [k](-A) - R */
    ge nA, Q, nR;
    ge_neg(&nA, &A);
    ge_double_scalarmult(&Q, sig + 32, &GE_B, k, &nA);
    ge_neg(&nR, &R);
    ge_add(&Q, &Q, &nR);
    ge_dbl(&Q, &Q); ge_dbl(&Q, &Q); ge_dbl(&Q, &Q);
    return ge_is_ident(&Q);
}

/* ---- batch API over the same packed layout the product C-ABI uses ----
 * pk: n*32, sig: n*64, msg: concatenated, msg_off: n+1 offsets.
 * Returns 1 if all valid, 0 otherwise (and 0 for n == 0, voi semantics). */
typedef struct {
    const uint8_t *pk, *sig, *msg; const uint32_t *off; uint8_t *out;
    size_t lo, hi;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (size_t i = j->lo; i < j->hi; i++)
        j->out[i] = (uint8_t)oracle_ed25519_verify(j->pk + 32 * i, j->msg + j->off[i],
                                                  j->off[i + 1] - j->off[i], j->sig + 64 * i);
    return NULL;
}

int oracle_ed25519_verify_batch(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                const uint32_t *msg_off, size_t n, uint8_t *valid_out, int threads) {
    init_consts();
    if (n == 0) return 0;
    if (threads < 1) threads = 1;
    if ((size_t)threads > n) threads = (int)n;
    pthread_t th[256];
    job_t jobs[256];
    if (threads > 256) threads = 256;
    size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){pk, sig, msg, msg_off, valid_out, t * per, (t + 1) * per < n ? (t + 1) * per : n};
        if (jobs[t].lo >= jobs[t].hi) { jobs[t].lo = jobs[t].hi = 0; }
        if (threads == 1) worker(&jobs[t]); else pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    if (threads > 1) for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    int ok = 1;
    for (size_t i = 0; i < n; i++) ok &= valid_out[i];
    return ok;
}

/* exposed helpers for tests */
void oracle_sha512(const uint8_t *m, size_t n, uint8_t out[64]) {
    sha512_ctx c; sha512_init(&c); sha512_update(&c, m, n); sha512_final(&c, out);
}
void oracle_sc_reduce64(uint8_t out[32], const uint8_t in[64]) { sc_reduce64(out, in); }
int oracle_ge_decode_lax(const uint8_t s[32], uint8_t x_out[32], uint8_t y_out[32]) {
    init_consts();
    ge p; if (!ge_decode_lax(&p, s)) return 0;
    fe_tobytes(x_out, &p.X); fe_tobytes(y_out, &p.Y); return 1;
}
