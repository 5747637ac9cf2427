// Keccak-f[1600], STROBE-128 (the subset merlin uses) and the schnorrkel
// signing transcript, for the sr25519 challenge
//   k = merlin("SigningContext"; "" -> ctx ""; "sign-bytes" -> M;
//              "proto-name" -> "Schnorr-sig"; "sign:pk" -> A; "sign:R" -> R;
//              challenge "sign:c", 64 bytes) mod l
// (crypto/sr25519/{privkey.go:18,batch.go:39}; curve25519-voi
// primitives/merlin + primitives/sr25519, go.mod:22).  Host+device: the
// constant prefix (through the empty context) is absorbed once on the host
// and handed to the kernels as a 203-byte state.
#pragma once
#include "curve25519.h"

namespace tmv {

// 64-bit rotate left: on the device two v_alignbit_b32 for a compile-time n
// (the shift pair the compiler emits otherwise costs three or four)
TMV_HD uint64_t rotl64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (n == 0) return x;
  const int r = 64 - n;  // rotate right by r
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t a = r < 32 ? hi : lo, b = r < 32 ? lo : hi;
  const int k = r & 31;
  if (k == 0) return ((uint64_t)a << 32) | b;
  return ((uint64_t)__builtin_amdgcn_alignbit(b, a, k) << 32) | __builtin_amdgcn_alignbit(a, b, k);
#else
  return n ? ((x << n) | (x >> (64 - n))) : x;
#endif
}

// Round constants in device constant memory (scalar loads by the
// wave-uniform round index), as kSha512K.
#if defined(__HIP_DEVICE_COMPILE__)
__constant__
#endif
static const uint64_t kKeccakRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

// One Keccak-f[1600] round on 25 lanes (lane x + 5y): theta, rho + pi, chi
// unrolled (every lane index a compile-time register), iota by the caller.
TMV_HD void keccak_round(uint64_t a[25]) {
  const int rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  uint64_t c[5], b[25];
#pragma unroll
  for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
  for (int x = 0; x < 5; x++) {
    const uint64_t d = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
#pragma unroll
    for (int y = 0; y < 25; y += 5) a[y + x] ^= d;
  }
#pragma unroll
  for (int x = 0; x < 5; x++)
#pragma unroll
    for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(a[x + 5 * y], rho[x + 5 * y]);
#pragma unroll
  for (int y = 0; y < 25; y += 5)
#pragma unroll
    for (int x = 0; x < 5; x++) a[y + x] = b[y + x] ^ (~b[y + (x + 1) % 5] & b[y + (x + 2) % 5]);
}

// Keccak-f[1600] with the round loop rolled on the device: one ~270-
// instruction round body per permutation site instead of 24 (an unrolled
// permutation is ~6,500 instructions, and the transcript inlines several).
TMV_HD void keccak_f1600_lanes(uint64_t a[25]) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
  for (int round = 0; round < 24; round++) {
    keccak_round(a);
    a[0] ^= kKeccakRC[round];
  }
}

constexpr int kStrobeR = 166;

// STROBE-128 state held as the 25 Keccak lanes (state byte p is byte p & 7 of
// lane p >> 3, little-endian, as Keccak defines it) + the position registers.
// Absorb/squeeze touch one lane per <= 8 bytes and F runs on the lanes in
// place: no byte-array pack/unpack around the permutation.
struct strobe_t {
  uint64_t a[25];
  uint32_t pos, pos_begin, cur_flags;
  TMV_HD uint64_t &lane(uint32_t i) { return a[i]; }
};

// The same state with its lanes in LDS, lane-interleaved (lane i of thread t
// at base[i * STRIDE + t]: conflict-free, and the dynamically indexed state
// stays out of scratch).  The kernels' transcript workspace.
template <int STRIDE>
struct strobe_lds_t {
  uint64_t *base;
  uint32_t pos, pos_begin, cur_flags;
  TMV_HD uint64_t &lane(uint32_t i) { return base[i * STRIDE]; }
};

template <class S>
TMV_HD void strobe_xor_byte(S &s, uint32_t p, uint8_t b) { s.lane(p >> 3) ^= (uint64_t)b << (8 * (p & 7)); }

template <class S>
TMV_HD void strobe_run_f(S &s) {
  strobe_xor_byte(s, s.pos, (uint8_t)s.pos_begin);
  strobe_xor_byte(s, s.pos + 1, 0x04);
  strobe_xor_byte(s, kStrobeR + 1, 0x80);
  uint64_t a[25];  // F on registers
  for (int i = 0; i < 25; i++) a[i] = s.lane(i);
  keccak_f1600_lanes(a);
  for (int i = 0; i < 25; i++) s.lane(i) = a[i];
  s.pos = 0;
  s.pos_begin = 0;
}

// Fresh STROBE-128 instance before any operation: header, version string, F.
TMV_HD void strobe_init(strobe_t &s) {
  for (int i = 0; i < 25; i++) s.a[i] = 0;
  const uint8_t hdr[6] = {1, kStrobeR + 2, 1, 0, 1, 96};
  for (int i = 0; i < 6; i++) strobe_xor_byte(s, i, hdr[i]);
  const char *v = "STROBEv1.0.2";
  for (int i = 0; i < 12; i++) strobe_xor_byte(s, 6 + i, (uint8_t)v[i]);
  keccak_f1600_lanes(s.a);
  s.pos = 0; s.pos_begin = 0; s.cur_flags = 0;
}

// XOR d[0..n) into the rate, a lane-sized chunk at a time.
template <class S>
TMV_HD void strobe_absorb(S &s, const uint8_t *d, uint32_t n) {
  uint32_t i = 0;
  while (i < n) {
    const uint32_t sh = s.pos & 7;
    uint32_t c = 8 - sh;
    if (c > kStrobeR - s.pos) c = kStrobeR - s.pos;
    if (c > n - i) c = n - i;
    uint64_t v = 0;
    for (uint32_t j = 0; j < c; j++) v |= (uint64_t)d[i + j] << (8 * j);
    s.lane(s.pos >> 3) ^= v << (8 * sh);
    s.pos += c;
    i += c;
    if (s.pos == kStrobeR) strobe_run_f(s);
  }
}
template <class S>
TMV_HD void strobe_absorb_byte(S &s, uint8_t b) {
  strobe_xor_byte(s, s.pos++, b);
  if (s.pos == kStrobeR) strobe_run_f(s);
}

// PRF squeeze after begin_op(I|A|C): out = state bytes, which are then zeroed.
template <class S>
TMV_HD void strobe_prf(S &s, uint8_t *out, uint32_t n) {
  uint32_t i = 0;
  while (i < n) {
    const uint32_t sh = s.pos & 7;
    uint32_t c = 8 - sh;
    if (c > kStrobeR - s.pos) c = kStrobeR - s.pos;
    if (c > n - i) c = n - i;
    const uint64_t lane = s.lane(s.pos >> 3);
    for (uint32_t j = 0; j < c; j++) out[i + j] = (uint8_t)(lane >> (8 * (sh + j)));
    const uint64_t mask = (c == 8) ? ~0ULL : (((1ULL << (8 * c)) - 1) << (8 * sh));
    s.lane(s.pos >> 3) = lane & ~mask;
    s.pos += c;
    i += c;
    if (s.pos == kStrobeR) strobe_run_f(s);
  }
}

// begin_op for a fresh (more == false) operation
template <class S>
TMV_HD void strobe_begin_op(S &s, uint8_t flags) {
  const uint8_t old_begin = (uint8_t)s.pos_begin;
  s.pos_begin = s.pos + 1;
  s.cur_flags = flags;
  strobe_absorb_byte(s, old_begin);
  strobe_absorb_byte(s, flags);
  if ((flags & (4 | 32)) && s.pos != 0) strobe_run_f(s);  // C or K forces F
}

// merlin append_message(label, message): meta_ad(label); meta_ad(le32(len), more); ad(message)
template <class S>
TMV_HD void merlin_append(S &s, const char *label, uint32_t llen, const uint8_t *m, uint32_t n) {
  strobe_begin_op(s, 16 | 2);  // M | A
  strobe_absorb(s, reinterpret_cast<const uint8_t *>(label), llen);
  const uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
  strobe_absorb(s, len, 4);    // meta_ad(..., more = true): no begin_op
  strobe_begin_op(s, 2);       // A
  strobe_absorb(s, m, n);
}

// merlin append with the message given as 8 little-endian words (32 bytes)
template <class S>
TMV_HD void merlin_append_words(S &s, const char *label, uint32_t llen, const uint32_t w[8]) {
  uint8_t b[32];
  for (int i = 0; i < 32; i++) b[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  merlin_append(s, label, llen, b, 32);
}

// challenge_bytes(label, 64) -> out (64 bytes as 16 LE words)
template <class S>
TMV_HD void merlin_challenge64(S &s, const char *label, uint32_t llen, uint32_t out[16]) {
  strobe_begin_op(s, 16 | 2);
  strobe_absorb(s, reinterpret_cast<const uint8_t *>(label), llen);
  const uint8_t len[4] = {64, 0, 0, 0};
  strobe_absorb(s, len, 4);
  strobe_begin_op(s, 1 | 2 | 4);  // I | A | C  (prf)
  uint8_t b[64];
  strobe_prf(s, b, 64);
  for (int i = 0; i < 16; i++)
    out[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
             ((uint32_t)b[4 * i + 3] << 24);
}

// Transcript state after merlin("SigningContext") + append("", ctx = "")
// (crypto/sr25519/privkey.go:18): computed once on the host.
inline void sr25519_context_prefix(strobe_t &s) {
  strobe_init(s);
  // Strobe128::new("Merlin v1.0"): meta_ad(label, false)
  strobe_begin_op(s, 16 | 2);
  strobe_absorb(s, reinterpret_cast<const uint8_t *>("Merlin v1.0"), 11);
  // Transcript::new("SigningContext"): append_message("dom-sep", label)
  merlin_append(s, "dom-sep", 7, reinterpret_cast<const uint8_t *>("SigningContext"), 14);
  // SigningContext::new(ctx = ""): append_message("", "")
  merlin_append(s, "", 0, reinterpret_cast<const uint8_t *>(""), 0);
}

// k = challenge mod l for (pk, R, M), s holding the context prefix on entry.
template <class S>
TMV_HD void sr25519_challenge_from(uint32_t k[8], S &s, const uint32_t pk_w[8], const uint32_t r_w[8],
                                   const uint8_t *m, uint32_t mlen) {
  merlin_append(s, "sign-bytes", 10, m, mlen);
  merlin_append(s, "proto-name", 10, reinterpret_cast<const uint8_t *>("Schnorr-sig"), 11);
  merlin_append_words(s, "sign:pk", 7, pk_w);
  merlin_append_words(s, "sign:R", 6, r_w);
  uint32_t wide[16];
  merlin_challenge64(s, "sign:c", 6, wide);
  sc_reduce512(k, wide);
}

TMV_HD void sr25519_challenge(uint32_t k[8], const strobe_t &prefix, const uint32_t pk_w[8],
                              const uint32_t r_w[8], const uint8_t *m, uint32_t mlen) {
  strobe_t s = prefix;
  sr25519_challenge_from(k, s, pk_w, r_w, m, mlen);
}

// ---- the transcript for vote-sized messages, state in registers ----
// After the context prefix (pos 50) a message of 98..127 bytes (vote
// sign-bytes are 109-125) puts every absorbed byte at a fixed place in
// exactly two Keccak blocks:
//   block 1: [50] prefix pos_begin, [51] M|A, [52,62) "sign-bytes",
//            [62,66) le32(mlen), [66] 51, [67] A, [68,166) message [0,98),
//            F padding [166] 67 (pos_begin), [167] 0x04 ^ 0x80;
//   block 2: [0,q) message [98,mlen), q = mlen - 98, then the framing of
//            proto-name / sign:pk / sign:R / sign:c (kSrSuffix: constant
//            bytes, pos_begin bytes that are q + a constant, pk at +44, R at
//            +90), the forced F of begin_op(I|A|C) at q + 136 with padding
//            [q+136] q+135, [q+137] 0x04, [167] 0x80;
// then the 64 challenge bytes are lanes 0..7.  These are the positions
// strobe_begin_op / strobe_absorb / strobe_run_f above produce, step by step
// (checked against them for every length and message alignment by
// tests/test_arith_host.py::test_sr25519_transcript_fast_path).  Block 1 is
// XORed into the register state lane by lane; block 2, which starts q bytes
// into the block, is assembled in the caller's LDS slot as dwords (the shift
// by q becomes an address) and read back as lanes.  The generic path's
// byte-wise absorb with the state in LDS made the sr25519 hash 3.1x the
// ed25519 SHA-512 (k_prep_hash 511 vs 164 us per 500k).
constexpr uint32_t kSrFastPrefixPos = 50, kSrFastMinLen = 98, kSrFastMaxLen = 127;
constexpr int kSrSuffixWords = 35;  // 138 bytes
struct SrSuffix {
  uint32_t t[kSrSuffixWords];   // little-endian dwords of the framing at q = 0
  uint32_t qm[kSrSuffixWords];  // 1 in each byte that holds q + a constant
  int o;
  constexpr SrSuffix() : t(), qm(), o(0) {}
  constexpr void put(uint32_t v, bool qdep = false) {
    t[o >> 2] |= (v & 0xffu) << (8 * (o & 3));
    if (qdep) qm[o >> 2] |= 1u << (8 * (o & 3));
    o++;
  }
  constexpr void str(const char *c) {
    while (*c) put((uint8_t)*c++);
  }
  constexpr void le32(uint32_t v) {
    for (int i = 0; i < 4; i++) put(v >> (8 * i));
  }
  constexpr void skip(int n) { o += n; }
};
constexpr SrSuffix make_sr_suffix() {
  SrSuffix x;
  x.put(0); x.put(16 | 2); x.str("proto-name"); x.le32(11); x.put(1, true); x.put(2); x.str("Schnorr-sig");
  x.put(17, true); x.put(16 | 2); x.str("sign:pk"); x.le32(32); x.put(30, true); x.put(2); x.skip(32);
  x.put(43, true); x.put(16 | 2); x.str("sign:R"); x.le32(32); x.put(77, true); x.put(2); x.skip(32);
  x.put(89, true); x.put(16 | 2); x.str("sign:c"); x.le32(64); x.put(123, true); x.put(1 | 2 | 4);
  x.put(135, true); x.put(0x04);
  return x;
}
constexpr SrSuffix kSrSuffix = make_sr_suffix();
static_assert(kSrSuffix.o == 138, "sr25519 transcript framing length");

TMV_HD bool sr25519_fast_eligible(const strobe_t &prefix, uint32_t mlen) {
  return prefix.pos == kSrFastPrefixPos && mlen >= kSrFastMinLen && mlen <= kSrFastMaxLen;
}

// Message bytes [off, off + 4) as a little-endian dword.  Device: aligned
// dword loads clamped to the one holding the last message byte, funnel-
// shifted (bytes past the message are garbage; callers mask them).
struct MsgWords {
  const uint8_t *m;
  uint32_t mlen;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t *mw;
  uint32_t sh, last;
  TMV_HD MsgWords(const uint8_t *m_, uint32_t n) : m(m_), mlen(n) {
    sh = (uint32_t)((uintptr_t)m & 3);
    mw = reinterpret_cast<const uint32_t *>((uintptr_t)m - sh);
    last = (sh + n - 1) >> 2;
  }
  TMV_HD uint32_t at(uint32_t off) const {
    const uint32_t a = sh + off, i = a >> 2;
    const uint32_t d0 = mw[i < last ? i : last], d1 = mw[i + 1 < last ? i + 1 : last];
    return __builtin_amdgcn_alignbit(d1, d0, 8 * (a & 3));
  }
#else
  TMV_HD MsgWords(const uint8_t *m_, uint32_t n) : m(m_), mlen(n) {}
  TMV_HD uint32_t at(uint32_t off) const {
    uint32_t v = 0;
    for (uint32_t j = 0; j < 4; j++)
      if (off + j < mlen) v |= (uint32_t)m[off + j] << (8 * j);
    return v;
  }
#endif
};

// k for sr25519_fast_eligible transcripts; base = the caller's LDS slot
// (&lds[0][t] of a uint64_t [25][STRIDE] array), used for block 2.
template <int STRIDE>
TMV_HD void sr25519_challenge_fast(uint32_t k[8], const strobe_t &prefix, uint64_t *base, const uint32_t pk_w[8],
                                   const uint32_t r_w[8], const uint8_t *m, uint32_t mlen) {
  const MsgWords msg(m, mlen);
  uint64_t a[25];
#pragma unroll
  for (int i = 0; i < 25; i++) a[i] = prefix.a[i];
  auto lane = [](uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; };
  constexpr uint32_t kSign = 's' | ('i' << 8) | ('g' << 16) | ('n' << 24);
  constexpr uint32_t kByte = '-' | ('b' << 8) | ('y' << 16) | ('t' << 24);
  a[6] ^= lane(((prefix.pos_begin & 0xffu) << 16) | ((16u | 2u) << 24), kSign);
  a[7] ^= lane(kByte, 'e' | ('s' << 8) | (mlen << 16));
  a[8] ^= lane((51u << 16) | (2u << 24), msg.at(0));
#pragma unroll
  for (int j = 0; j < 11; j++) a[9 + j] ^= lane(msg.at(4 + 8 * j), msg.at(8 + 8 * j));
  a[20] ^= lane(msg.at(92), (msg.at(96) & 0xffffu) | (67u << 16) | (0x84u << 24));
  keccak_f1600_lanes(a);

  // block 2 in LDS: dword j of this lane's slot
  auto dw = [base](uint32_t j) -> uint32_t & {
    return reinterpret_cast<uint32_t *>(base + (size_t)(j >> 1) * STRIDE)[j & 1];
  };
  const uint32_t q = mlen - kSrFastMinLen, r = q & 3, qb = q >> 2;
  uint32_t tq = 0;
#pragma unroll
  for (uint32_t j = 0; j < 8; j++) {  // message tail [98, mlen)
    uint32_t v = msg.at(kSrFastMinLen + 4 * j);
    const int32_t rem = (int32_t)q - (int32_t)(4 * j);
    v = rem >= 4 ? v : (rem <= 0 ? 0u : v & ((1u << (8 * rem)) - 1));
    dw(j) = v;
    tq = qb == j ? v : tq;
  }
  uint32_t sfx[kSrSuffixWords];
#pragma unroll
  for (int j = 0; j < kSrSuffixWords; j++) sfx[j] = kSrSuffix.t[j] + q * kSrSuffix.qm[j];
#pragma unroll
  for (int j = 0; j < 8; j++) sfx[11 + j] = pk_w[j];  // pk at +44
  sfx[22] |= r_w[0] << 16;                             // R at +90
#pragma unroll
  for (int j = 0; j < 7; j++) sfx[23 + j] = (r_w[j] >> 16) | (r_w[j + 1] << 16);
  sfx[30] |= r_w[7] >> 16;
  const uint32_t rs = 32 - 8 * r;  // the framing moved up by r bytes within dwords, qb dwords by address
#pragma unroll
  for (int j = 0; j <= kSrSuffixWords; j++) {
    const uint32_t lo = j ? sfx[j - 1] : 0u, hi = j < kSrSuffixWords ? sfx[j] : 0u;
    const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> rs);
    dw(qb + j) = j ? v : (v | tq);
  }
#pragma unroll
  for (int j = kSrSuffixWords + 1; j < kSrSuffixWords + 7; j++) dw(qb + j) = 0;  // through dword 41
#pragma unroll
  for (int i = 0; i < 21; i++) a[i] ^= lane(dw(2 * i), dw(2 * i + 1));  // as written: uint32_t accesses
  a[20] ^= 0x80ull << 56;
  keccak_f1600_lanes(a);
  uint32_t wide[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    wide[2 * i] = (uint32_t)a[i];
    wide[2 * i + 1] = (uint32_t)(a[i] >> 32);
  }
  sc_reduce512(k, wide);
}

// Same, with the transcript state in the caller's LDS slot (base = &lds[0][t]
// of a uint64_t [25][STRIDE] array); vote-sized messages take the fast path.
template <int STRIDE>
TMV_HD void sr25519_challenge_lds(uint32_t k[8], const strobe_t &prefix, uint64_t *base, const uint32_t pk_w[8],
                                      const uint32_t r_w[8], const uint8_t *m, uint32_t mlen) {
#ifndef TMV_SR_FAST_TRANSCRIPT
#define TMV_SR_FAST_TRANSCRIPT 1
#endif
  if (TMV_SR_FAST_TRANSCRIPT && sr25519_fast_eligible(prefix, mlen)) {
    sr25519_challenge_fast<STRIDE>(k, prefix, base, pk_w, r_w, m, mlen);
    return;
  }
  strobe_lds_t<STRIDE> s;
  s.base = base;
  for (int i = 0; i < 25; i++) s.lane(i) = prefix.a[i];
  s.pos = prefix.pos; s.pos_begin = prefix.pos_begin; s.cur_flags = prefix.cur_flags;
  sr25519_challenge_from(k, s, pk_w, r_w, m, mlen);
}

// Signature.UnmarshalBinary checks: schnorrkel marker bit, canonical s.
// s_out = s with the marker cleared.  Returns false on an Add-time error.
TMV_HD bool sr25519_decode_s(uint32_t s_out[8], const uint32_t s_w[8]) {
  for (int i = 0; i < 8; i++) s_out[i] = s_w[i];
  if (!(s_w[7] & 0x80000000u)) return false;
  s_out[7] &= 0x7fffffffu;
  return sc_is_canonical(s_out);
}

}  // namespace tmv
