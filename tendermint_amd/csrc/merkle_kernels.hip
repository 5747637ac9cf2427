// ValidatorSet.Hash on the device: the light client
// checks every new header's ValidatorsHash against the supplied set
// (light/verifier.go:266), i.e. ValidatorSet.Hash (types/validator_set.go:
// 344-350) = merkle.HashFromByteSlices over Validator.Bytes()
// (types/validator.go:154-170: SimpleValidator{pub_key, voting_power}
// protobuf), RFC 6962 leaves SHA-256(0x00 || bytes) and inner nodes
// SHA-256(0x01 || left || right) (crypto/merkle/hash.go, tree.go:11-27).
//
// Many sets per launch (a light client's or blocksync's window of headers):
//   k_valset_leaves  one lane per validator: encode SimpleValidator into a
//                    single SHA-256 block (<= 48 bytes with the prefix) and
//                    hash it
//   k_merkle_leaves  one lane per leaf of arbitrary length (tmv_merkle_roots:
//                    the 14 proto-encoded fields of Header.Hash,
//                    types/block.go:447-478, or any HashFromByteSlices input):
//                    SHA-256(0x00 || leaf) over as many blocks as it needs
//   k_merkle_tree    one workgroup per set: the levels of the tree, pairing
//                    (0,1), (2,3), ... and promoting an odd last node --
//                    the same tree as the reference's split at the largest
//                    power of two below n (tree.go:68-99, its iterative form,
//                    equal by TestHashAlternatives) -- ping-ponging between
//                    two scratch arrays, one barrier per level.
// Node hashes stay as 8 SHA-256 state words; only the roots are serialised.
#include <hip/hip_runtime.h>
#include "sha256_dev.h"
#include "valset.h"

namespace tmv {


__global__ void __launch_bounds__(256)
k_valset_leaves(const uint8_t *__restrict__ pk, const uint8_t *__restrict__ kind, const int64_t *__restrict__ power,
                uint32_t n_vals, uint32_t *__restrict__ node) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_vals) return;
  // varint of the power (proto int64: two's complement, 10 bytes if negative);
  // proto3 omits a zero power
  const int64_t p = power[v];
  uint64_t u = (uint64_t)p;
  uint32_t vb[10];
  int vlen = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const bool more = (u >> 7) != 0;
    vb[i] = (uint32_t)(u & 0x7f) | (more ? 0x80u : 0u);
    if (vlen == i && (u != 0 || i == 0)) vlen = i + 1;
    u >>= 7;
  }
  const int tail = p != 0 ? 1 + vlen : 0;  // 0x10 tag + varint
  const int len = 37 + tail;               // 0x00 prefix + 36 bytes of pub_key field + tail
  const uint8_t *k = pk + 32ull * v;
  const uint32_t tag = kind[v] == kValsetSr25519 ? 0x1au : 0x0au;  // PublicKey oneof: ed25519 = 1, sr25519 = 3
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int pos = 4 * i + j;
      uint32_t b;
      if (pos == 0) b = 0x00;        // leaf prefix
      else if (pos == 1) b = 0x0a;   // SimpleValidator.pub_key, length-delimited
      else if (pos == 2) b = 0x22;   // 34 bytes
      else if (pos == 3) b = tag;
      else if (pos == 4) b = 0x20;   // 32-byte key
      else if (pos < 37) b = k[pos - 5];
      else if (pos < 56) {  // tail, then the 0x80 pad byte at len (<= 48), zeros
        const int t = pos - 37;
        b = t == 0 ? 0x10u : (t <= 10 ? vb[t >= 1 && t <= 10 ? t - 1 : 0] : 0u);
        if (pos == len) b = 0x80;
        else if (pos > len) b = 0;
      } else if (pos == 62) {
        b = (uint32_t)(len * 8) >> 8;
      } else if (pos == 63) {
        b = (uint32_t)(len * 8) & 0xff;
      } else {
        b = 0;
      }
      word = (word << 8) | b;
    }
    w[i] = word;
  }
  uint32_t st[8];
  sha256_init(st);
  sha256_compress(st, w);
  uint4 *o = reinterpret_cast<uint4 *>(node + 8ull * v);
  o[0] = make_uint4(st[0], st[1], st[2], st[3]);
  o[1] = make_uint4(st[4], st[5], st[6], st[7]);
}

__device__ __forceinline__ void load_node(uint32_t h[8], const uint32_t *p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  const uint4 a = q[0], b = q[1];
  h[0] = a.x; h[1] = a.y; h[2] = a.z; h[3] = a.w;
  h[4] = b.x; h[5] = b.y; h[6] = b.z; h[7] = b.w;
}

__device__ __forceinline__ void store_node(uint32_t *p, const uint32_t h[8]) {
  uint4 *q = reinterpret_cast<uint4 *>(p);
  q[0] = make_uint4(h[0], h[1], h[2], h[3]);
  q[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

// RFC 6962 leaf of an arbitrary byte string, one lane per leaf: the padded
// message 0x00 || leaf || 0x80 || 0* || bitlen(64) is assembled a block at a
// time from global memory (leaves are short: header fields, <= 2 blocks).
__global__ void __launch_bounds__(256)
k_merkle_leaves(const uint8_t *__restrict__ data, const uint32_t *__restrict__ leaf_off, uint32_t n_leaves,
                uint32_t *__restrict__ node) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_leaves) return;
  const uint32_t base = leaf_off[i];
  const uint32_t total = leaf_off[i + 1] - base + 1;  // with the 0x00 prefix
  const uint32_t nblk = (total + 72) / 64;            // room for 0x80 and the 8-byte length
  const uint32_t end = 64 * nblk;
  const uint64_t bits = (uint64_t)total * 8;
  uint32_t st[8];
  sha256_init(st);
  for (uint32_t k = 0; k < nblk; k++) {
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t pos = 64 * k + 4 * q + j;
        uint32_t byte = 0;
        if (pos == 0) byte = 0x00;
        else if (pos < total) byte = data[base + pos - 1];
        else if (pos == total) byte = 0x80;
        else if (pos >= end - 8) byte = (uint32_t)(bits >> (8 * (end - 1 - pos))) & 0xffu;
        word = (word << 8) | byte;
      }
      w[q] = word;
    }
    sha256_compress(st, w);
  }
  uint4 *o = reinterpret_cast<uint4 *>(node + 8ull * i);
  o[0] = make_uint4(st[0], st[1], st[2], st[3]);
  o[1] = make_uint4(st[4], st[5], st[6], st[7]);
}

template <int kTreeBlock>
__global__ void __launch_bounds__(kTreeBlock)
k_merkle_tree(const uint32_t *__restrict__ set_off, uint32_t n_sets, uint32_t *node_a, uint32_t *node_b,
              uint8_t *__restrict__ out) {
  const uint32_t s = blockIdx.x;
  if (s >= n_sets) return;
  const uint32_t base = set_off[s], n = set_off[s + 1] - base;
  uint32_t root[8];
  if (n == 0) {  // emptyHash(): SHA-256 of the empty string
    if (threadIdx.x != 0) return;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = 0;
    w[0] = 0x80000000u;
    sha256_init(root);
    sha256_compress(root, w);
  } else {
    uint32_t *cur = node_a + 8ull * base, *nxt = node_b + 8ull * base;
    uint32_t size = n;
    while (size > 1) {  // block-uniform
      const uint32_t half = size >> 1;
      for (uint32_t i = threadIdx.x; i < half; i += kTreeBlock) {
        uint32_t l[8], r[8], h[8];
        load_node(l, cur + 16ull * i);
        load_node(r, cur + 16ull * i + 8);
        sha256_inner(h, l, r);
        store_node(nxt + 8ull * i, h);
      }
      if ((size & 1) && threadIdx.x == 0) {
        uint32_t h[8];
        load_node(h, cur + 8ull * (size - 1));
        store_node(nxt + 8ull * half, h);
      }
      __syncthreads();  // this level's nodes written (workgroup-scope fence)
      uint32_t *t = cur; cur = nxt; nxt = t;
      size = half + (size & 1);
    }
    if (threadIdx.x != 0) return;
    load_node(root, cur);
  }
  uint8_t *o = out + 32ull * s;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    o[4 * i] = (uint8_t)(root[i] >> 24);
    o[4 * i + 1] = (uint8_t)(root[i] >> 16);
    o[4 * i + 2] = (uint8_t)(root[i] >> 8);
    o[4 * i + 3] = (uint8_t)root[i];
  }
}

hipError_t launch_valset_hashes(const uint8_t *pk, const uint8_t *kind, const int64_t *power, uint32_t n_vals,
                                const uint32_t *set_off, uint32_t n_sets, uint32_t *node_a, uint32_t *node_b,
                                uint8_t *out, hipStream_t stream) {
  if (n_vals) {
    hipLaunchKernelGGL(k_valset_leaves, dim3((n_vals + 255) / 256), dim3(256), 0, stream, pk, kind, power, n_vals,
                       node_a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (n_sets) hipLaunchKernelGGL(k_merkle_tree<256>, dim3(n_sets), dim3(256), 0, stream, set_off, n_sets, node_a,
                                 node_b, out);
  return hipGetLastError();
}

hipError_t launch_merkle_roots(const uint8_t *data, const uint32_t *leaf_off, uint32_t n_leaves,
                               const uint32_t *tree_off, uint32_t n_trees, uint32_t max_leaves, uint32_t *node_a,
                               uint32_t *node_b, uint8_t *out, hipStream_t stream) {
  if (n_leaves) {
    hipLaunchKernelGGL(k_merkle_leaves, dim3((n_leaves + 255) / 256), dim3(256), 0, stream, data, leaf_off, n_leaves,
                       node_a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (!n_trees) return hipGetLastError();
  // small trees (Header.Hash: 14 leaves) take one wave per tree
  if (max_leaves <= 128)
    hipLaunchKernelGGL(k_merkle_tree<64>, dim3(n_trees), dim3(64), 0, stream, tree_off, n_trees, node_a, node_b, out);
  else
    hipLaunchKernelGGL(k_merkle_tree<256>, dim3(n_trees), dim3(256), 0, stream, tree_off, n_trees, node_a, node_b,
                       out);
  return hipGetLastError();
}

}  // namespace tmv
