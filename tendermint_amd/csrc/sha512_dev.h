// SHA-512 (FIPS 180-4) for the verification kernels: the challenge hash
// k = SHA-512(R || A || M) of crypto/ed25519 (Go crypto/sha512 in the
// reference).  64-bit words are emulated on 32-bit VALU by the compiler
// (rotates lower to v_alignbit pairs).  Host+device so the CPU tests run it.
#pragma once
#include "curve25519.h"

namespace tmv {

// Round constants: device constant memory, read with scalar loads (the
// round index is wave-uniform).  A function-local table indexed by the round
// counter was materialised in VGPRs and read through s_set_gpr_idx (~30
// moves per round).
#if defined(__HIP_DEVICE_COMPILE__)
__constant__
#endif
static const uint64_t kSha512K[80] = {
        0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
        0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
        0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
        0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
        0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
        0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
        0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
        0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
        0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
        0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
        0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
        0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
        0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
        0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
        0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
        0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
        0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
        0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
        0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
        0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

// 64-bit rotate: two v_alignbit_b32 on the device (the shift pair the
// compiler emits otherwise costs three instructions)
TMV_HD uint64_t rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t a = n < 32 ? hi : lo, b = n < 32 ? lo : hi;  // n is a compile-time constant
  const int k = n & 31;
  if (k == 0) return ((uint64_t)a << 32) | b;
  return ((uint64_t)__builtin_amdgcn_alignbit(b, a, k) << 32) | __builtin_amdgcn_alignbit(a, b, k);
#else
  return (x >> n) | (x << (64 - n));
#endif
}

// One compression of a 16-word (big-endian-decoded) block into h[8]: 16
// rounds on the block's words, then four passes of 16 with the message
// schedule, each unrolled, so every schedule index is a compile-time
// register (t & 15 == i), no branch sits inside a pass (a per-round
// "first pass?" test made the register allocator copy w[] at every round),
// and only the round constant is read by pass index.
TMV_HD void sha512_compress(uint64_t h[8], uint64_t w[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  auto round = [&](uint64_t wt, uint64_t kt) {
    const uint64_t S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
    const uint64_t ch = (e & f) ^ (~e & g);
    const uint64_t t1 = hh + S1 + ch + kt + wt;
    const uint64_t S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
    const uint64_t x = a ^ b;
    const uint64_t mj = (x & c) | (~x & a);  // majority: c where a != b, else a (one bit-field insert)
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  };
#pragma unroll
  for (int i = 0; i < 16; i++) round(w[i], kSha512K[i]);
  for (int r = 1; r < 5; r++) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint64_t s0 = rotr64(w15, 1) ^ rotr64(w15, 8) ^ (w15 >> 7);
      const uint64_t s1 = rotr64(w2, 19) ^ rotr64(w2, 61) ^ (w2 >> 6);
      w[i] += s0 + w[(i + 9) & 15] + s1;
      round(w[i], kSha512K[16 * r + i]);
    }
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

TMV_HD void sha512_init(uint64_t h[8]) {
  h[0] = 0x6a09e667f3bcc908ULL; h[1] = 0xbb67ae8584caa73bULL;
  h[2] = 0x3c6ef372fe94f82bULL; h[3] = 0xa54ff53a5f1d36f1ULL;
  h[4] = 0x510e527fade682d1ULL; h[5] = 0x9b05688c2b3e6c1fULL;
  h[6] = 0x1f83d9abfb41bd6bULL; h[7] = 0x5be0cd19137e2179ULL;
}

TMV_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// SHA-512 of P || Q || M where P and Q are 32-byte values given as
// little-endian u32 words (R and A of a signature) and M is mlen bytes at m.
// Output: the 64-byte digest as 16 little-endian u32 words (so the
// digest-as-integer for sc_reduce512 is direct).
TMV_HD void sha512_pq_msg(uint32_t out[16], const uint32_t P[8], const uint32_t Q[8],
                          const uint8_t *m, uint32_t mlen) {
  uint64_t h[8];
  sha512_init(h);
  const uint64_t total = 64ull + mlen;
  const uint32_t nblocks = (uint32_t)((total + 17 + 127) / 128);
#if defined(__HIP_DEVICE_COMPILE__)
  // message bytes from aligned dword loads: dword indices clamped to the one
  // holding the last message byte (so every load stays inside that byte's
  // page, and none is made for an empty message), funnel-shifted by the
  // message's misalignment, bytes past the end masked off -- no branch per
  // word on the lane's message length
  const uint32_t sh = (uint32_t)((uintptr_t)m & 3);
  const uint32_t *mw = reinterpret_cast<const uint32_t *>((uintptr_t)m - sh);
  const uint32_t last = mlen ? (sh + mlen - 1) >> 2 : 0;
#endif
  for (uint32_t blk = 0; blk < nblocks; blk++) {
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
      const uint64_t base = (uint64_t)blk * 128 + 8 * t;
      uint64_t word;
      if (blk == 0 && t < 8) {
        // bytes of P||Q: word t covers u32 words 2t, 2t+1 (little-endian bytes)
        const uint32_t lo = t < 4 ? P[2 * t] : Q[2 * t - 8];
        const uint32_t hi = t < 4 ? P[2 * t + 1] : Q[2 * t + 1 - 8];
        word = ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
      } else {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t off = (uint32_t)(base - 64);  // message offset of the word's first byte
        const uint32_t d0i = (sh + off) >> 2;
        uint32_t d0 = 0, d1 = 0, d2 = 0;
        if (mlen) {
          d0 = mw[d0i < last ? d0i : last];
          d1 = mw[d0i + 1 < last ? d0i + 1 : last];
          d2 = mw[d0i + 2 < last ? d0i + 2 : last];
        }
        const uint32_t b_lo = __builtin_amdgcn_alignbit(d1, d0, 8 * sh);  // bytes off .. off+3
        const uint32_t b_hi = __builtin_amdgcn_alignbit(d2, d1, 8 * sh);  // bytes off+4 .. off+7
        uint64_t x = ((uint64_t)b_hi << 32) | b_lo;
        const int32_t rem = (int32_t)mlen - (int32_t)off;  // message bytes from off on
        if (rem < 8) {
          const uint32_t v = rem > 0 ? (uint32_t)rem : 0u;
          x &= ((uint64_t)1 << (8 * v)) - 1;
          if (rem >= 0) x |= (uint64_t)0x80 << (8 * v);  // pad byte right after the message
        }
        word = ((uint64_t)__builtin_bswap32((uint32_t)x) << 32) | __builtin_bswap32((uint32_t)(x >> 32));
#else
        word = 0;
        for (int b = 0; b < 8; b++) {
          const uint64_t q = base + b;
          uint32_t byte;
          if (q < 64) {
            const uint32_t wv = q < 32 ? P[q >> 2] : Q[(q - 32) >> 2];
            byte = (wv >> (8 * (q & 3))) & 0xff;
          } else if (q < total) {
            byte = m[q - 64];
          } else if (q == total) {
            byte = 0x80;
          } else {
            byte = 0;
          }
          word = (word << 8) | byte;
        }
#endif
        if (blk == nblocks - 1 && t == 15) word = total * 8;  // length (< 2^64 bits)
      }
      w[t] = word;
    }
    sha512_compress(h, w);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    // digest bytes are big-endian per word; re-express as LE u32 words
    out[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

}  // namespace tmv
