// Device ValidatorSet.Hash (merkle_kernels.hip): launch wrapper shared with
// the runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmv {

constexpr uint8_t kValsetEd25519 = 0;  // TMV_KIND_ED25519: PublicKey oneof field 1
constexpr uint8_t kValsetSr25519 = 1;  // TMV_KIND_SR25519: PublicKey oneof field 3

// node_a / node_b: n_vals x 8 words each (leaf hashes, then the levels).
// set_off: n_sets + 1 offsets into the validator arrays; out: n_sets x 32 B.
hipError_t launch_valset_hashes(const uint8_t *pk, const uint8_t *kind, const int64_t *power, uint32_t n_vals,
                                const uint32_t *set_off, uint32_t n_sets, uint32_t *node_a, uint32_t *node_b,
                                uint8_t *out, hipStream_t stream);

// merkle.HashFromByteSlices of n_trees trees (tmv_merkle_roots): leaf i is
// data[leaf_off[i], leaf_off[i+1]); tree t holds leaves [tree_off[t],
// tree_off[t+1]) and has at most max_leaves of them.  node_a / node_b:
// n_leaves x 8 words each; out: n_trees x 32 B.
hipError_t launch_merkle_roots(const uint8_t *data, const uint32_t *leaf_off, uint32_t n_leaves,
                               const uint32_t *tree_off, uint32_t n_trees, uint32_t max_leaves, uint32_t *node_a,
                               uint32_t *node_b, uint8_t *out, hipStream_t stream);

}  // namespace tmv
