/* TEST INFRASTRUCTURE ONLY — Keccak-f[1600], STROBE-128 (merlin subset) and
 * merlin transcripts for the sr25519 CPU oracle.  Restates the published
 * merlin/STROBE algorithms used by curve25519-voi primitives/merlin
 * (go.mod:22; absent here).  Pinned against oracle/sr25519_ref.py, which is
 * pinned to hashlib.sha3_256 and the published merlin test vector. */
#ifndef ORACLE_KECCAK_H
#define ORACLE_KECCAK_H
#include <stdint.h>
#include <string.h>

static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KECCAK_ROTC[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14,
                                    27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
static const int KECCAK_PILN[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4,
                                    15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};

static void keccak_f1600(uint8_t st8[200]) {
    uint64_t s[25], bc[5], t;
    for (int i = 0; i < 25; i++) {
        uint64_t v = 0;
        for (int j = 7; j >= 0; j--) v = (v << 8) | st8[8 * i + j];
        s[i] = v;
    }
    for (int r = 0; r < 24; r++) {
        for (int i = 0; i < 5; i++) bc[i] = s[i] ^ s[i + 5] ^ s[i + 10] ^ s[i + 15] ^ s[i + 20];
        for (int i = 0; i < 5; i++) {
            t = bc[(i + 4) % 5] ^ ((bc[(i + 1) % 5] << 1) | (bc[(i + 1) % 5] >> 63));
            for (int j = 0; j < 25; j += 5) s[j + i] ^= t;
        }
        t = s[1];
        for (int i = 0; i < 24; i++) {
            int j = KECCAK_PILN[i];
            bc[0] = s[j];
            s[j] = (t << KECCAK_ROTC[i]) | (t >> (64 - KECCAK_ROTC[i]));
            t = bc[0];
        }
        for (int j = 0; j < 25; j += 5) {
            for (int i = 0; i < 5; i++) bc[i] = s[j + i];
            for (int i = 0; i < 5; i++) s[j + i] ^= (~bc[(i + 1) % 5]) & bc[(i + 2) % 5];
        }
        s[0] ^= KECCAK_RC[r];
    }
    for (int i = 0; i < 25; i++)
        for (int j = 0; j < 8; j++) st8[8 * i + j] = (uint8_t)(s[i] >> (8 * j));
}

#define STROBE_R 166
enum { FLAG_I = 1, FLAG_A = 2, FLAG_C = 4, FLAG_T = 8, FLAG_M = 16, FLAG_K = 32 };

typedef struct { uint8_t st[200]; uint8_t pos, pos_begin, cur_flags; } strobe128;

static void strobe_run_f(strobe128 *s) {
    s->st[s->pos] ^= s->pos_begin;
    s->st[s->pos + 1] ^= 0x04;
    s->st[STROBE_R + 1] ^= 0x80;
    keccak_f1600(s->st);
    s->pos = 0;
    s->pos_begin = 0;
}

static void strobe_absorb(strobe128 *s, const uint8_t *d, size_t n) {
    for (size_t i = 0; i < n; i++) {
        s->st[s->pos++] ^= d[i];
        if (s->pos == STROBE_R) strobe_run_f(s);
    }
}

static void strobe_squeeze(strobe128 *s, uint8_t *out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        out[i] = s->st[s->pos];
        s->st[s->pos++] = 0;
        if (s->pos == STROBE_R) strobe_run_f(s);
    }
}

static void strobe_begin_op(strobe128 *s, uint8_t flags, int more) {
    if (more) return; /* caller guarantees cur_flags == flags */
    uint8_t hdr[2] = {s->pos_begin, flags};
    s->pos_begin = (uint8_t)(s->pos + 1);
    s->cur_flags = flags;
    strobe_absorb(s, hdr, 2);
    if ((flags & (FLAG_C | FLAG_K)) && s->pos != 0) strobe_run_f(s);
}

static void strobe_meta_ad(strobe128 *s, const uint8_t *d, size_t n, int more) {
    strobe_begin_op(s, FLAG_M | FLAG_A, more);
    strobe_absorb(s, d, n);
}
static void strobe_ad(strobe128 *s, const uint8_t *d, size_t n, int more) {
    strobe_begin_op(s, FLAG_A, more);
    strobe_absorb(s, d, n);
}
static void strobe_prf(strobe128 *s, uint8_t *out, size_t n) {
    strobe_begin_op(s, FLAG_I | FLAG_A | FLAG_C, 0);
    strobe_squeeze(s, out, n);
}

static void strobe_init(strobe128 *s, const uint8_t *label, size_t n) {
    memset(s, 0, sizeof *s);
    const uint8_t hdr[6] = {1, STROBE_R + 2, 1, 0, 1, 96};
    memcpy(s->st, hdr, 6);
    memcpy(s->st + 6, "STROBEv1.0.2", 12);
    keccak_f1600(s->st);
    strobe_meta_ad(s, label, n, 0);
}

typedef struct { strobe128 s; } merlin_t;

static void merlin_append(merlin_t *t, const char *label, const uint8_t *m, size_t n) {
    uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
    strobe_meta_ad(&t->s, (const uint8_t *)label, strlen(label), 0);
    strobe_meta_ad(&t->s, len, 4, 1);
    strobe_ad(&t->s, m, n, 0);
}

static void merlin_init(merlin_t *t, const char *label) {
    strobe_init(&t->s, (const uint8_t *)"Merlin v1.0", 11);
    merlin_append(t, "dom-sep", (const uint8_t *)label, strlen(label));
}

static void merlin_challenge(merlin_t *t, const char *label, uint8_t *out, size_t n) {
    uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
    strobe_meta_ad(&t->s, (const uint8_t *)label, strlen(label), 0);
    strobe_meta_ad(&t->s, len, 4, 1);
    strobe_prf(&t->s, out, n);
}
#endif
