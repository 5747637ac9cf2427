/* TEST INFRASTRUCTURE ONLY — shared GF(2^255-19), Edwards-point and
 * scalar-mod-l arithmetic for the CPU oracle (ed25519_oracle.c,
 * sr25519_oracle.c).  Restates the published curve25519 algorithms behind
 * curve25519-voi (go.mod:22); see ed25519_oracle.c for the contract. */
#ifndef ORACLE_COMMON_H
#define ORACLE_COMMON_H
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[5]; } fe;

static const uint64_t M51 = (1ULL << 51) - 1;

static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
static void fe_copy(fe *h, const fe *f) { *h = *f; }

static void fe_carry(fe *h) {
    uint64_t c;
    for (int i = 0; i < 4; i++) { c = h->v[i] >> 51; h->v[i] &= M51; h->v[i + 1] += c; }
    c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
    c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
}

static void fe_add(fe *h, const fe *f, const fe *g) {
    for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + g->v[i];
    fe_carry(h);
}

/* h = f - g, computed as f + 4p - g so limbs stay non-negative */
static void fe_sub(fe *h, const fe *f, const fe *g) {
    static const uint64_t fourp[5] = {
        0x1FFFFFFFFFFFB4ULL, 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL,
        0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL};
    for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + fourp[i] - g->v[i];
    fe_carry(h);
}

static void fe_neg(fe *h, const fe *f) { fe z; fe_0(&z); fe_sub(h, &z, f); }

static void fe_mul(fe *h, const fe *f, const fe *g) {
    const uint64_t *a = f->v, *b = g->v;
    uint64_t b19[5];
    for (int i = 0; i < 5; i++) b19[i] = b[i] * 19;
    u128 t0 = (u128)a[0]*b[0] + (u128)a[1]*b19[4] + (u128)a[2]*b19[3] + (u128)a[3]*b19[2] + (u128)a[4]*b19[1];
    u128 t1 = (u128)a[0]*b[1] + (u128)a[1]*b[0] + (u128)a[2]*b19[4] + (u128)a[3]*b19[3] + (u128)a[4]*b19[2];
    u128 t2 = (u128)a[0]*b[2] + (u128)a[1]*b[1] + (u128)a[2]*b[0] + (u128)a[3]*b19[4] + (u128)a[4]*b19[3];
    u128 t3 = (u128)a[0]*b[3] + (u128)a[1]*b[2] + (u128)a[2]*b[1] + (u128)a[3]*b[0] + (u128)a[4]*b19[4];
    u128 t4 = (u128)a[0]*b[4] + (u128)a[1]*b[3] + (u128)a[2]*b[2] + (u128)a[3]*b[1] + (u128)a[4]*b[0];
    uint64_t c;
    t1 += (uint64_t)(t0 >> 51); uint64_t r0 = (uint64_t)t0 & M51;
    t2 += (uint64_t)(t1 >> 51); uint64_t r1 = (uint64_t)t1 & M51;
    t3 += (uint64_t)(t2 >> 51); uint64_t r2 = (uint64_t)t2 & M51;
    t4 += (uint64_t)(t3 >> 51); uint64_t r3 = (uint64_t)t3 & M51;
    c = (uint64_t)(t4 >> 51); uint64_t r4 = (uint64_t)t4 & M51;
    r0 += c * 19; c = r0 >> 51; r0 &= M51; r1 += c;
    h->v[0] = r0; h->v[1] = r1; h->v[2] = r2; h->v[3] = r3; h->v[4] = r4;
}

static void fe_sq(fe *h, const fe *f) { fe_mul(h, f, f); }

static void fe_frombytes(fe *h, const uint8_t s[32]) {
    uint64_t w[4];
    for (int i = 0; i < 4; i++) {
        w[i] = 0;
        for (int j = 7; j >= 0; j--) w[i] = (w[i] << 8) | s[8 * i + j];
    }
    w[3] &= 0x7FFFFFFFFFFFFFFFULL; /* drop the sign bit; y >= p is reduced lazily (lax) */
    h->v[0] = w[0] & M51;
    h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
    h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
    h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
    h->v[4] = (w[3] >> 12) & M51;
}

/* fully reduced little-endian encoding */
static void fe_tobytes(uint8_t s[32], const fe *f) {
    fe t = *f;
    fe_carry(&t);
    /* now t < 2^255 + small; subtract p if t >= p */
    uint64_t q = (t.v[0] + 19) >> 51;
    q = (t.v[1] + q) >> 51;
    q = (t.v[2] + q) >> 51;
    q = (t.v[3] + q) >> 51;
    q = (t.v[4] + q) >> 51;
    t.v[0] += 19 * q;
    uint64_t c;
    c = t.v[0] >> 51; t.v[0] &= M51; t.v[1] += c;
    c = t.v[1] >> 51; t.v[1] &= M51; t.v[2] += c;
    c = t.v[2] >> 51; t.v[2] &= M51; t.v[3] += c;
    c = t.v[3] >> 51; t.v[3] &= M51; t.v[4] += c;
    t.v[4] &= M51;
    uint64_t w[4];
    w[0] = t.v[0] | (t.v[1] << 51);
    w[1] = (t.v[1] >> 13) | (t.v[2] << 38);
    w[2] = (t.v[2] >> 26) | (t.v[3] << 25);
    w[3] = (t.v[3] >> 39) | (t.v[4] << 12);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static int fe_iszero(const fe *f) {
    uint8_t s[32]; fe_tobytes(s, f);
    uint8_t r = 0; for (int i = 0; i < 32; i++) r |= s[i];
    return r == 0;
}
static int fe_isneg(const fe *f) { uint8_t s[32]; fe_tobytes(s, f); return s[0] & 1; }
static int fe_eq(const fe *a, const fe *b) { fe d; fe_sub(&d, a, b); return fe_iszero(&d); }

static void fe_pow2k(fe *h, const fe *f, int k) { fe_sq(h, f); for (int i = 1; i < k; i++) fe_sq(h, h); }

/* h = f^((p-5)/8) = f^(2^252 - 3) */
static void fe_pow22523(fe *h, const fe *z) {
    fe t0, t1, t2;
    fe_sq(&t0, z);             /* 2 */
    fe_pow2k(&t1, &t0, 2);     /* 8 */
    fe_mul(&t1, z, &t1);       /* 9 */
    fe_mul(&t0, &t0, &t1);     /* 11 */
    fe_sq(&t0, &t0);           /* 22 */
    fe_mul(&t0, &t1, &t0);     /* 2^5-1 */
    fe_pow2k(&t1, &t0, 5);
    fe_mul(&t0, &t1, &t0);     /* 2^10-1 */
    fe_pow2k(&t1, &t0, 10);
    fe_mul(&t1, &t1, &t0);     /* 2^20-1 */
    fe_pow2k(&t2, &t1, 20);
    fe_mul(&t1, &t2, &t1);     /* 2^40-1 */
    fe_pow2k(&t1, &t1, 10);
    fe_mul(&t0, &t1, &t0);     /* 2^50-1 */
    fe_pow2k(&t1, &t0, 50);
    fe_mul(&t1, &t1, &t0);     /* 2^100-1 */
    fe_pow2k(&t2, &t1, 100);
    fe_mul(&t1, &t2, &t1);     /* 2^200-1 */
    fe_pow2k(&t1, &t1, 50);
    fe_mul(&t0, &t1, &t0);     /* 2^250-1 */
    fe_pow2k(&t0, &t0, 2);     /* 2^252-4 */
    fe_mul(h, &t0, z);         /* 2^252-3 */
}

/* constants */
static fe FE_D, FE_D2, FE_SQRTM1;
static int consts_ready = 0;

static void fe_from_u64le(fe *h, const char *hex) {
    uint8_t b[32];
    for (int i = 0; i < 32; i++) {
        int hi = hex[2 * i], lo = hex[2 * i + 1];
        hi = hi <= '9' ? hi - '0' : hi - 'a' + 10;
        lo = lo <= '9' ? lo - '0' : lo - 'a' + 10;
        b[i] = (uint8_t)(hi * 16 + lo);
    }
    fe_frombytes(h, b);
}

typedef struct { fe X, Y, Z, T; } ge;
static ge GE_B;

static void init_consts(void) {
    if (consts_ready) return;
    /* little-endian encodings */
    fe_from_u64le(&FE_D, "a3785913ca4deb75abd841414d0a700098e879777940c78c73fe6f2bee6c0352");
    fe_add(&FE_D2, &FE_D, &FE_D);
    fe_from_u64le(&FE_SQRTM1, "b0a00e4a271beec478e42fad0618432fa7d7fb3d99004d2b0bdfc14f8024832b");
    fe_from_u64le(&GE_B.X, "1ad5258f602d56c9b2a7259560c72c695cdcd6fd31e2a4c0fe536ecdd3366921");
    fe_from_u64le(&GE_B.Y, "5866666666666666666666666666666666666666666666666666666666666666");
    fe_1(&GE_B.Z);
    fe_mul(&GE_B.T, &GE_B.X, &GE_B.Y);
    consts_ready = 1;
}

static void ge_ident(ge *p) { fe_0(&p->X); fe_1(&p->Y); fe_1(&p->Z); fe_0(&p->T); }

/* unified addition, extended coordinates (a = -1) */
static void ge_add(ge *r, const ge *p, const ge *q) {
    fe A, B, C, Dd, E, F, G, H, t;
    fe_sub(&A, &p->Y, &p->X); fe_sub(&t, &q->Y, &q->X); fe_mul(&A, &A, &t);
    fe_add(&B, &p->Y, &p->X); fe_add(&t, &q->Y, &q->X); fe_mul(&B, &B, &t);
    fe_mul(&C, &p->T, &q->T); fe_mul(&C, &C, &FE_D2);
    fe_mul(&Dd, &p->Z, &q->Z); fe_add(&Dd, &Dd, &Dd);
    fe_sub(&E, &B, &A); fe_sub(&F, &Dd, &C); fe_add(&G, &Dd, &C); fe_add(&H, &B, &A);
    fe_mul(&r->X, &E, &F); fe_mul(&r->Y, &G, &H); fe_mul(&r->Z, &F, &G); fe_mul(&r->T, &E, &H);
}

static void ge_dbl(ge *r, const ge *p) {
    fe A, B, C, E, F, G, H, t;
    fe_sq(&A, &p->X); fe_sq(&B, &p->Y); fe_sq(&C, &p->Z); fe_add(&C, &C, &C);
    fe_add(&t, &p->X, &p->Y); fe_sq(&t, &t);
    fe_add(&H, &A, &B);          /* H = A + B */
    fe_sub(&E, &H, &t);          /* E = A + B - (X+Y)^2 = -2XY */
    fe_sub(&G, &A, &B);          /* G = A - B  (a = -1: -A + B negated) */
    fe_add(&F, &C, &G);          /* F = C + G */
    /* with a=-1: X3 = E*F, Y3 = G*H, Z3 = F*G, T3 = E*H (signs consistent) */
    fe_mul(&r->X, &E, &F); fe_mul(&r->Y, &G, &H); fe_mul(&r->Z, &F, &G); fe_mul(&r->T, &E, &H);
}

static void ge_neg(ge *r, const ge *p) { fe_neg(&r->X, &p->X); r->Y = p->Y; r->Z = p->Z; fe_neg(&r->T, &p->T); }

static int ge_is_ident(const ge *p) { return fe_iszero(&p->X) && fe_eq(&p->Y, &p->Z); }

/* ZIP-215 lax decode; returns 1 on success */
static int ge_decode_lax(ge *p, const uint8_t s[32]) {
    fe u, v, v3, vxx, chk, x, y;
    int sign = s[31] >> 7;
    fe_frombytes(&y, s);
    fe one; fe_1(&one);
    fe_sq(&u, &y);
    fe_mul(&v, &u, &FE_D);
    fe_sub(&u, &u, &one);        /* u = y^2 - 1 */
    fe_add(&v, &v, &one);        /* v = d y^2 + 1 */
    fe_sq(&v3, &v); fe_mul(&v3, &v3, &v);       /* v^3 */
    fe_sq(&x, &v3); fe_mul(&x, &x, &v); fe_mul(&x, &x, &u); /* u v^7 */
    fe_pow22523(&x, &x);
    fe_mul(&x, &x, &v3); fe_mul(&x, &x, &u);    /* x = u v^3 (u v^7)^((p-5)/8) */
    fe_sq(&vxx, &x); fe_mul(&vxx, &vxx, &v);
    fe_sub(&chk, &vxx, &u);
    if (!fe_iszero(&chk)) {
        fe_add(&chk, &vxx, &u);
        if (!fe_iszero(&chk)) return 0;
        fe_mul(&x, &x, &FE_SQRTM1);
    }
    if (fe_isneg(&x) != sign) fe_neg(&x, &x);
    p->X = x; p->Y = y; fe_1(&p->Z); fe_mul(&p->T, &x, &y);
    return 1;
}

/* l = 2^252 + 27742317777372353535851937790883648493, little-endian */
static const uint8_t L_BYTES[32] = {
    0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7, 0xa2, 0xde, 0xf9, 0xde, 0x14,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x10};

static int sc_is_canonical(const uint8_t s[32]) {
    for (int i = 31; i >= 0; i--) {
        if (s[i] < L_BYTES[i]) return 1;
        if (s[i] > L_BYTES[i]) return 0;
    }
    return 0; /* equal to l */
}

/* reduce a 64-byte little-endian integer mod l: Barrett reduction (HAC
 * 14.42) in base 2^64, k = 4 words, mu = floor(2^512 / l) (5 words) */
static void sc_reduce64(uint8_t out[32], const uint8_t in[64]) {
    static const uint64_t MU[5] = {0xed9ce5a30a2c131bULL, 0x2106215d086329a7ULL, 0xffffffffffffffebULL,
                                   0xffffffffffffffffULL, 0x000000000000000fULL};
    static const uint64_t LW[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0x0000000000000000ULL,
                                   0x1000000000000000ULL};
    uint64_t x[8] = {0};
    for (int i = 0; i < 64; i++) x[i / 8] |= (uint64_t)in[i] << (8 * (i % 8));
    /* q1 = x >> 192 (5 words); q2 = q1 * mu (10 words); q3 = q2 >> 320 */
    uint64_t q2[10] = {0};
    for (int i = 0; i < 5; i++) {
        u128 c = 0;
        for (int j = 0; j < 5; j++) {
            c += (u128)x[3 + i] * MU[j] + q2[i + j];
            q2[i + j] = (uint64_t)c;
            c >>= 64;
        }
        q2[i + 5] = (uint64_t)c;
    }
    const uint64_t *q3 = q2 + 5;
    /* r2 = (q3 * l) mod 2^320 */
    uint64_t r2[5] = {0};
    for (int i = 0; i < 5; i++) {
        u128 c = 0;
        for (int j = 0; j < 4 && i + j < 5; j++) {
            c += (u128)q3[i] * LW[j] + r2[i + j];
            r2[i + j] = (uint64_t)c;
            c >>= 64;
        }
        if (i == 0) r2[4] = (uint64_t)c;  /* row 0's carry; later rows' carries fall past 2^320 */
    }
    /* r = (x mod 2^320) - r2 (mod 2^320), then subtract l while r >= l */
    uint64_t r[5];
    u128 br = 0;
    for (int i = 0; i < 5; i++) {
        u128 d = (u128)x[i] - r2[i] - br;
        r[i] = (uint64_t)d;
        br = (d >> 64) ? 1 : 0;
    }
    for (int it = 0; it < 3; it++) {
        int ge_ = r[4] != 0;
        if (!ge_) {
            ge_ = 1;
            for (int i = 3; i >= 0; i--) {
                if (r[i] > LW[i]) { ge_ = 1; break; }
                if (r[i] < LW[i]) { ge_ = 0; break; }
            }
        }
        if (!ge_) break;
        br = 0;
        for (int i = 0; i < 5; i++) {
            u128 d = (u128)r[i] - (i < 4 ? LW[i] : 0) - br;
            r[i] = (uint64_t)d;
            br = (d >> 64) ? 1 : 0;
        }
    }
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(r[i / 8] >> (8 * (i % 8)));
}

/* r = [a]P + [b]Q, 4-bit fixed windows (Straus), variable time */
static void ge_double_scalarmult(ge *r, const uint8_t a[32], const ge *P, const uint8_t b[32], const ge *Q) {
    ge tp[16], tq[16];
    ge_ident(&tp[0]); ge_ident(&tq[0]);
    tp[1] = *P; tq[1] = *Q;
    for (int i = 2; i < 16; i++) { ge_add(&tp[i], &tp[i - 1], P); ge_add(&tq[i], &tq[i - 1], Q); }
    ge acc; ge_ident(&acc);
    for (int i = 63; i >= 0; i--) {
        for (int j = 0; j < 4; j++) ge_dbl(&acc, &acc);
        int da = (a[i / 2] >> (4 * (i & 1))) & 15;
        int db = (b[i / 2] >> (4 * (i & 1))) & 15;
        if (da) ge_add(&acc, &acc, &tp[da]);
        if (db) ge_add(&acc, &acc, &tq[db]);
    }
    *r = acc;
}


#endif
