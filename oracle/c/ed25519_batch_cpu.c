/*
 * TEST INFRASTRUCTURE ONLY — CPU baseline.  Only bench.py's cpu_baseline leg
 * (and tests/test_oracle.py, which checks it against the per-entry oracle)
 * load this; the product path never does.
 *
 * A plain-C restatement of the batch verification the reference runs on the
 * CPU: curve25519-voi's ed25519 BatchVerifier.Verify behind
 * crypto/ed25519/ed25519.go:231-233 (module
 * github.com/oasisprotocol/curve25519-voi v0.0.0-20210609091139-0a56a4bca00b,
 * go.mod:22, absent here).  Its published algorithm: every Add'ed entry is
 * decoded and hashed; one random linear combination
 *   [8]( sum z_i R_i + sum (z_i k_i) A_i - (sum z_i s_i) B ) == O
 * with 128-bit random z_i is checked by one multi-scalar multiplication
 * (Pippenger buckets); if it fails (or an entry does not decode / has a
 * non-canonical S) every entry is verified on its own, so the validity
 * vector equals per-entry verification.  The arithmetic reuses
 * oracle_common.h (radix 2^51, unified extended additions); z_i come from a
 * per-thread splitmix64 stream seeded from the caller's seed (this is a
 * timing baseline and a checker, not a production verifier).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "sha512.h"

#include "oracle_common.h"

int oracle_ed25519_verify(const uint8_t *pk, const uint8_t *msg, size_t mlen, const uint8_t *sig);

static uint64_t splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void load_words(uint64_t w[4], const uint8_t b[32]) {
    for (int i = 0; i < 4; i++) { w[i] = 0; for (int j = 0; j < 8; j++) w[i] |= (uint64_t)b[8 * i + j] << (8 * j); }
}

/* out = z * k mod l (z: 2 words, k: 4 words) */
static void sc_mul_zk(uint8_t out[32], const uint64_t z[2], const uint64_t k[4]) {
    uint64_t p[8] = {0};
    for (int i = 0; i < 2; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)z[i] * k[j] + p[i + j];
            p[i + j] = (uint64_t)c;
            c >>= 64;
        }
        p[i + 4] = (uint64_t)c;
    }
    uint8_t b[64];
    for (int i = 0; i < 64; i++) b[i] = (uint8_t)(p[i / 8] >> (8 * (i % 8)));
    sc_reduce64(out, b);
}

/* acc (8 words) += z * s */
static void sc_acc_zs(uint64_t acc[8], const uint64_t z[2], const uint64_t s[4]) {
    uint64_t p[6] = {0};
    for (int i = 0; i < 2; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)z[i] * s[j] + p[i + j];
            p[i + j] = (uint64_t)c;
            c >>= 64;
        }
        p[i + 4] = (uint64_t)c;
    }
    u128 c = 0;
    for (int i = 0; i < 8; i++) {
        c += (u128)acc[i] + (i < 6 ? p[i] : 0);
        acc[i] = (uint64_t)c;
        c >>= 64;
    }
}

/* bits [bit, bit + c) of a little-endian scalar of nbytes bytes */
static int digit_at(const uint8_t *s, int nbytes, int bit, int c) {
    uint64_t x = 0;
    const int b0 = bit >> 3;
    for (int i = 0; i < 8 && b0 + i < nbytes; i++) x |= (uint64_t)s[b0 + i] << (8 * i);
    return (int)((x >> (bit & 7)) & ((1u << c) - 1));
}

typedef struct {
    ge *pts;        /* 2m + 1 points: R_i, A_i, ..., B */
    uint8_t *sc;    /* 32 bytes per point */
    uint8_t *nb;    /* scalar bytes per point (16 for z_i, 32 otherwise) */
    ge *bucket;
} scratch_t;

/* one random linear combination over entries [lo, hi); 1 iff it holds and
 * every entry decodes with a canonical S */
static int batch_equation(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *off,
                          size_t lo, size_t hi, uint64_t *rng, scratch_t *sc) {
    const size_t m = hi - lo;
    uint64_t acc[8] = {0};
    for (size_t e = 0; e < m; e++) {
        const size_t i = lo + e;
        const uint8_t *A = pk + 32 * i, *R = sig + 64 * i, *S = sig + 64 * i + 32;
        if (!sc_is_canonical(S)) return 0;
        if (!ge_decode_lax(&sc->pts[2 * e], R)) return 0;
        if (!ge_decode_lax(&sc->pts[2 * e + 1], A)) return 0;
        uint8_t h[64], k[32];
        sha512_ctx c;
        sha512_init(&c);
        sha512_update(&c, R, 32);
        sha512_update(&c, A, 32);
        sha512_update(&c, msg + off[i], off[i + 1] - off[i]);
        sha512_final(&c, h);
        sc_reduce64(k, h);
        uint64_t z[2] = {splitmix64(rng), splitmix64(rng)}, kw[4], sw[4];
        load_words(kw, k);
        load_words(sw, S);
        uint8_t *zr = sc->sc + 32 * (2 * e);
        memset(zr, 0, 32);
        for (int b = 0; b < 16; b++) zr[b] = (uint8_t)(z[b / 8] >> (8 * (b % 8)));
        sc->nb[2 * e] = 16;
        sc_mul_zk(sc->sc + 32 * (2 * e + 1), z, kw);   /* A_i: z_i k_i */
        sc->nb[2 * e + 1] = 32;
        sc_acc_zs(acc, z, sw);
    }
    /* R and A terms enter negated: [8](sum z s B - sum z R - sum z k A) == O */
    for (size_t p = 0; p < 2 * m; p++) ge_neg(&sc->pts[p], &sc->pts[p]);
    uint8_t wide[64], bs[32];
    for (int i = 0; i < 64; i++) wide[i] = (uint8_t)(acc[i / 8] >> (8 * (i % 8)));
    sc_reduce64(bs, wide);
    sc->pts[2 * m] = GE_B;
    memcpy(sc->sc + 32 * (2 * m), bs, 32);
    sc->nb[2 * m] = 32;
    const size_t np = 2 * m + 1;
    /* Pippenger, unsigned c-bit windows */
    const int c = np >= 512 ? 8 : np >= 128 ? 6 : 4;
    const int nbk = (1 << c) - 1, W = (253 + c - 1) / c;
    ge total;
    ge_ident(&total);
    for (int w = W - 1; w >= 0; w--) {
        for (int d = 0; d < c; d++) ge_dbl(&total, &total);
        for (int b = 0; b < nbk; b++) ge_ident(&sc->bucket[b]);
        for (size_t p = 0; p < np; p++) {
            if (w * c >= 8 * sc->nb[p]) continue;
            const int d = digit_at(sc->sc + 32 * p, sc->nb[p], w * c, c);
            if (d) ge_add(&sc->bucket[d - 1], &sc->bucket[d - 1], &sc->pts[p]);
        }
        ge run, sum;
        ge_ident(&run);
        ge_ident(&sum);
        for (int b = nbk - 1; b >= 0; b--) {
            ge_add(&run, &run, &sc->bucket[b]);
            ge_add(&sum, &sum, &run);
        }
        ge_add(&total, &total, &sum);
    }
    ge_dbl(&total, &total);
    ge_dbl(&total, &total);
    ge_dbl(&total, &total);
    return ge_is_ident(&total);
}

typedef struct {
    const uint8_t *pk, *sig, *msg;
    const uint32_t *off;
    uint8_t *out;
    size_t n, batch, first, step;  /* batches first, first + step, ... */
    uint64_t seed;
    size_t batches_failed;
} bjob_t;

static void *bworker(void *arg) {
    bjob_t *j = (bjob_t *)arg;
    scratch_t sc;
    sc.pts = (ge *)malloc(sizeof(ge) * (2 * j->batch + 1));
    sc.sc = (uint8_t *)malloc(32 * (2 * j->batch + 1));
    sc.nb = (uint8_t *)malloc(2 * j->batch + 1);
    sc.bucket = (ge *)malloc(sizeof(ge) * 255);
    uint64_t rng = j->seed;
    const size_t nb = (j->n + j->batch - 1) / j->batch;
    for (size_t b = j->first; b < nb; b += j->step) {
        const size_t lo = b * j->batch, hi = lo + j->batch < j->n ? lo + j->batch : j->n;
        if (batch_equation(j->pk, j->sig, j->msg, j->off, lo, hi, &rng, &sc)) {
            memset(j->out + lo, 1, hi - lo);
        } else {  /* voi: a failing batch is verified entry by entry */
            j->batches_failed++;
            for (size_t i = lo; i < hi; i++)
                j->out[i] = (uint8_t)oracle_ed25519_verify(j->pk + 32 * i, j->msg + j->off[i],
                                                          j->off[i + 1] - j->off[i], j->sig + 64 * i);
        }
    }
    free(sc.pts);
    free(sc.sc);
    free(sc.nb);
    free(sc.bucket);
    return NULL;
}

/* voi-style batch verification of n packed entries in batches of `batch`
 * entries (one BatchVerifier per batch), batches spread over `threads`
 * threads.  Returns 1 iff every entry is valid; out gets the exact vector;
 * *failed_out (optional) the number of batches whose equation failed. */
int oracle_ed25519_batch_verify_voi(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                    const uint32_t *msg_off, size_t n, uint8_t *out, int threads, size_t batch,
                                    uint64_t seed, size_t *failed_out) {
    init_consts();
    if (n == 0) return 0;
    if (batch < 1) batch = 1;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    bjob_t jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (bjob_t){pk, sig, msg, msg_off, out, n, batch, (size_t)t, (size_t)threads,
                           seed ^ (0xA5A5A5A5ULL * (uint64_t)(t + 1)), 0};
        if (threads == 1) bworker(&jobs[t]);
        else pthread_create(&th[t], NULL, bworker, &jobs[t]);
    }
    if (threads > 1) for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    size_t failed = 0;
    for (int t = 0; t < threads; t++) failed += jobs[t].batches_failed;
    if (failed_out) *failed_out = failed;
    int ok = 1;
    for (size_t i = 0; i < n; i++) ok &= out[i];
    return ok;
}

static size_t put_uvarint(uint8_t *p, uint64_t u) {
    size_t n = 0;
    while (u >= 0x80) { p[n++] = (uint8_t)(u | 0x80); u >>= 7; }
    p[n++] = (uint8_t)u;
    return n;
}

/* One commit vote's sign-bytes (types/vote.go:149-157 VoteSignBytes =
 * MarshalDelimited(CanonicalVote)): uvarint(L) || head ||
 * 2a len {08 secs, 10 nanos} || 32 len chain_id, head = the fields before the
 * timestamp (type, height, round, block ID). */
static size_t vote_sign_bytes(uint8_t *out, const uint8_t *head, uint32_t head_len, const uint8_t *chain,
                              uint32_t chain_len, int64_t secs, int32_t nanos) {
    uint8_t ts[24], tsl[10], chl[10];
    size_t tl = 0;
    if (secs) { ts[tl++] = 0x08; tl += put_uvarint(ts + tl, (uint64_t)secs); }
    if (nanos) { ts[tl++] = 0x10; tl += put_uvarint(ts + tl, (uint64_t)(int64_t)nanos); }
    const size_t tsl_n = put_uvarint(tsl, tl), chl_n = chain_len ? put_uvarint(chl, chain_len) : 0;
    const size_t body = head_len + 1 + tsl_n + tl + (chain_len ? 1 + chl_n + chain_len : 0);
    uint8_t *p = out;
    p += put_uvarint(p, body);
    memcpy(p, head, head_len); p += head_len;
    *p++ = 0x2a; memcpy(p, tsl, tsl_n); p += tsl_n; memcpy(p, ts, tl); p += tl;
    if (chain_len) { *p++ = 0x32; memcpy(p, chl, chl_n); p += chl_n; memcpy(p, chain, chain_len); p += chain_len; }
    return (size_t)(p - out);
}

/* bench.py's C1 CPU baseline: the signature work of types.VerifyCommit on one
 * commit of n votes (types/validation.go:154-258 verifyCommitBatch), on the
 * calling thread -- every vote's sign-bytes (Commit.VoteSignBytes,
 * types/block.go:836-862), then one voi-style batch of the n entries
 * (BatchVerifier.Verify, crypto/ed25519/ed25519.go:231-233: one random linear
 * combination, entry by entry if it fails).  A is decoded per entry (voi's
 * expanded-key cache is not restated).  Returns 1 iff every entry is valid;
 * out gets the vector. */
int oracle_verify_commit_cpu(const uint8_t *head, uint32_t head_len, const uint8_t *chain, uint32_t chain_len,
                             const int64_t *secs, const int32_t *nanos, const uint8_t *pk, const uint8_t *sig,
                             uint32_t n, uint8_t *out, uint64_t seed) {
    init_consts();
    if (n == 0) return 0;
    const size_t cap = (size_t)n * (head_len + chain_len + 48);
    uint8_t *msg = (uint8_t *)malloc(cap);
    uint32_t *off = (uint32_t *)malloc(4 * ((size_t)n + 1));
    size_t o = 0;
    off[0] = 0;
    for (uint32_t i = 0; i < n; i++) {
        o += vote_sign_bytes(msg + o, head, head_len, chain, chain_len, secs[i], nanos[i]);
        off[i + 1] = (uint32_t)o;
    }
    size_t failed = 0;
    const int ok = oracle_ed25519_batch_verify_voi(pk, sig, msg, off, n, out, 1, n, seed, &failed);
    free(msg);
    free(off);
    return ok;
}
