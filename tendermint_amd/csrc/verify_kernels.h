// Launch wrappers for the verification kernels (verify_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "curve25519.h"
#include "merlin_dev.h"
#include "msm.h"
#include "../../include/tmverify.h"

namespace tmv {

constexpr int kVerifyBlock = 256;
constexpr int kQuadBlock = 64;    // one wave = 16 signatures per block
constexpr int kBaseQuadEntries = 128;  // (m+1)B, m < 128, CachedQ layout (20 KB), then (m+1)[2^128]B

// Per-signature workspace of the latency path (device memory).
struct Ed25519Work {
  fe *negA;        // n x 4 fe, P3Q layout of -A
  fe *Rc;          // n x 4 fe, CachedQ layout of R
  uint32_t *k;     // n x 8 words, k mod l
  uint8_t *flags;  // 4n bytes: decode ok for A (4e), R (4e+1)
  niels_pt *niels; // batch check only (else null): [2e] = -R_e, [2e+1] = -A_e
  fe *tabA;        // n x 16 x 4 fe: k_verify_quad's tables of -A (8 x 4 fe) and -R (8 x 4 fe) when kept in global memory
  // per-entry pipeline only (launch_pipeline sets hs = hs_buf; null
  // elsewhere): the prep's hash lane reduces k to the half-size scalars once
  // per entry -- n x 12 words: |u| (4), v (4), fast | u_neg << 1, 3 spare --
  // instead of every lane of the entry's quad repeating the reduction
  uint32_t *hs;
  uint32_t *hs_buf;
  static size_t bytes(uint32_t n) { return (size_t)n * (160 + 160 + 32 + 4 + 2560 + 48) + 256; }
  // carve a workspace for n entries out of base (16-byte aligned pieces)
  static Ed25519Work carve(void *base, uint32_t n) {
    uint8_t *b = static_cast<uint8_t *>(base);
    Ed25519Work w;
    w.negA = reinterpret_cast<fe *>(b);
    w.Rc = reinterpret_cast<fe *>(b + 160ull * n);
    w.k = reinterpret_cast<uint32_t *>(b + 320ull * n);
    w.flags = b + 352ull * n;
    w.tabA = reinterpret_cast<fe *>(b + ((356ull * n + 15) & ~15ull));
    w.hs_buf = reinterpret_cast<uint32_t *>(b + ((356ull * n + 15) & ~15ull) + 2560ull * n);
    w.hs = nullptr;
    w.niels = nullptr;
    return w;
  }
};

hipError_t launch_ed25519_verify_quad(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                      const uint32_t *msg_off, uint32_t n, const fe *btab_q, Ed25519Work w,
                                      uint8_t *valid, hipStream_t stream);

// Device-resident expanded-key table (key-cached path).
constexpr int kKeyRowsEntries = 64 * 8;  // rows x multiples per key
struct KeyTable {
  fe *tab;       // capacity x 64 x 8 x 4 fe  (81,920 B per key)
  uint8_t *ok;   // capacity bytes: key decoded
  static size_t bytes_per_key() { return (size_t)kKeyRowsEntries * 4 * sizeof(fe); }
};

// bases: scratch of key_build_scratch(m) bytes (the row bases, P3Q)
hipError_t launch_key_build(bool sr, const uint8_t *keys, const uint32_t *slots, uint32_t m, KeyTable kt,
                            fe *bases, hipStream_t stream);
inline size_t key_build_scratch(uint32_t m) { return (size_t)m * 64 * 4 * sizeof(fe); }
// fused_max: batches up to this size use the one-kernel latency form
// (k_verify_cached_fused), larger ones k_prep_cached + k_verify_comb.
hipError_t launch_verify_cached(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                const uint32_t *msg_off, const uint32_t *key_slot, uint32_t n, KeyTable kt,
                                const fe *bcomb, const strobe_t *prefix, Ed25519Work w, uint8_t *out,
                                uint32_t fused_max, hipStream_t stream);

hipError_t launch_sr25519_verify_quad(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                      const uint32_t *msg_off, uint32_t n, const fe *btab_q, const strobe_t *prefix,
                                      Ed25519Work w, int8_t *status, hipStream_t stream);

hipError_t launch_mixed_verify(const uint8_t *kind, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                               const uint32_t *msg_off, uint32_t n, const fe *btab_q, const strobe_t *prefix,
                               Ed25519Work w_ed, Ed25519Work w_sr, uint32_t *counts, uint32_t *idx_ed,
                               uint32_t *idx_sr, int8_t *status, hipStream_t stream);

// Batch-equation pipeline (msm.h): k_prep -> k_msm_sort -> k_msm_accum ->
// k_msm_wpart -> k_msm_wsum -> k_msm_horner -> k_verify_quad over the failed
// groups only.  Single key kind (sr = false: ed25519, true: sr25519);
// idx/count_ptr as for the mixed path.
hipError_t launch_batch_check(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                              const uint32_t *msg_off, const uint32_t *idx, const uint32_t *count_ptr, uint32_t n,
                              const fe *btab_q, const strobe_t *prefix, Ed25519Work w, MsmWork mw,
                              const MsmParams &p, const MsmSeed &seed, uint8_t *out, hipStream_t stream);
// The same launch in pieces, for inputs that arrive in parts (the streamed
// host path): the throughput stages (prep, sort, bucket and window sums) of
// entries [e0, e1) of a contiguous n-entry launch -- e0 a multiple of the
// group size, e1 too unless e1 = n -- once those entries are in device
// memory, then, after every part, the latency stages of the whole launch
// (Horner, located / per-entry fallback).  Parts may be enqueued on the
// stream one by one, each behind its own copy.
hipError_t launch_batch_check_part(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                   const uint32_t *msg_off, uint32_t n, uint32_t e0, uint32_t e1, const fe *btab_q,
                                   const strobe_t *prefix, Ed25519Work w, MsmWork mw, const MsmParams &p,
                                   const MsmSeed &seed, uint8_t *out, hipStream_t stream);
hipError_t launch_batch_check_tail(bool sr, const uint8_t *pk, const uint8_t *sig, uint32_t n, const fe *btab_q,
                                   Ed25519Work w, MsmWork mw, const MsmParams &p, const MsmSeed &seed,
                                   uint8_t *out, hipStream_t stream);
// Mixed batch through the batch equation: partition, then one pipeline per
// kind (p: the ed25519 half's parameters, p_sr: the sr25519 half's); with
// ks, the sr25519 pipeline runs on ks->helper (forked after the
// partition, joined back into `stream` at the end).
struct KindStreams {
  hipStream_t helper;
  hipEvent_t fork, join;
};
hipError_t launch_mixed_batch_check(const uint8_t *kind, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                    const uint32_t *msg_off, uint32_t n, const fe *btab_q, const strobe_t *prefix,
                                    Ed25519Work w_ed, Ed25519Work w_sr, MsmWork m_ed, MsmWork m_sr,
                                    const MsmParams &p, const MsmParams &p_sr, const MsmSeed &seed_ed,
                                    const MsmSeed &seed_sr, uint32_t *counts, uint32_t *idx_ed, uint32_t *idx_sr,
                                    int8_t *status, hipStream_t stream, const KindStreams *ks = nullptr);

// Pieces of the pipelines, shared with msm_kernels.hip.
template <bool SR>
hipError_t launch_prep(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off,
                       const uint32_t *idx, const uint32_t *count_ptr, uint32_t n, const strobe_t *prefix,
                       Ed25519Work w, int aligned, hipStream_t stream);
template <bool SR>
hipError_t launch_quad_fallback(const uint8_t *sig, const uint32_t *idx, const uint32_t *count_ptr, uint32_t n,
                                const fe *btab_q, Ed25519Work w, const uint8_t *group_ok, uint32_t group_log2,
                                uint8_t *out, int aligned, hipStream_t stream, const uint8_t *sub_ok = nullptr,
                                const uint32_t *fail_list = nullptr, const uint32_t *fail_count = nullptr,
                                const uint32_t *fb_list = nullptr, const uint32_t *fb_count = nullptr);
// Default for MsmParams::sub: k_msm_subcheck runs before the per-entry
// fallback for groups of 2^m_log2 (m >= 256; tmv_set_batch_options can
// override it per context).
bool subcheck_enabled(uint32_t m_log2);
// Test build (-DTMV_CHECKS) counters since the last reset: joins named by
// k_msm_accum, joins done by k_msm_join_list, buckets with entries left
// unwritten.  false in a product build.
bool read_checks(uint32_t out[3], bool reset);
// Test aid (tmv_internal_option "half_scalars"): 1 = the product's half-size
// scalars, 0 = every entry on the full-k chain, 2 = every third entry.
void set_half_scalar_mode(int mode);
// Launches of at least this many entries use the located fallback
// (TMV_LOCATE_MIN, 0 = never).
uint32_t locate_min_entries();
// Whether a batch-equation launch of n entries with these parameters runs
// the located fallback (tmv_metrics reads its counters).
bool locate_enabled(uint32_t n, const MsmParams &p);
hipError_t launch_partition(const uint8_t *kind, uint32_t n, uint32_t *counts, uint32_t *idx_ed, uint32_t *idx_sr,
                            uint8_t *out, hipStream_t stream);
// Streamed mixed launches: the entries [lo, hi) of a part go to
// idx_ed[base_ed ..] / idx_sr[base_sr ..] (bases from the host's count of the
// earlier parts' kinds; cursor: 2 zeroed words per part).
hipError_t launch_partition_range(const uint8_t *kind, uint32_t lo, uint32_t hi, uint32_t base_ed, uint32_t base_sr,
                                  uint32_t *cursor, uint32_t *counts, uint32_t *idx_ed, uint32_t *idx_sr, uint8_t *out,
                                  hipStream_t stream);
// One kind's pipeline of a streamed mixed launch, over work slots whose
// entries are idx[e] (global indices into pk / sig / msg_off / out): the
// throughput stages of slots [e0, e1) (e0 on a group edge, e1 too unless it
// is the kind's last slot), then, after every part, the tail over n slots.
// nb (>= n) is the slot bound the workspaces were carved for.
hipError_t launch_batch_check_part_idx(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                       const uint32_t *msg_off, const uint32_t *idx, uint32_t nb, uint32_t e0,
                                       uint32_t e1, const fe *btab_q, const strobe_t *prefix, Ed25519Work w, MsmWork mw,
                                       const MsmParams &p, const MsmSeed &seed, uint8_t *out, hipStream_t stream);
hipError_t launch_batch_check_tail_idx(bool sr, const uint8_t *pk, const uint8_t *sig, const uint32_t *idx, uint32_t n,
                                       const fe *btab_q, Ed25519Work w, MsmWork mw, const MsmParams &p,
                                       const MsmSeed &seed, uint8_t *out, hipStream_t stream);

// Multi-batch launches (gather_kernels.hip): up to kMaxBatches device
// batches, passed by value as kernel arguments.
constexpr uint32_t kMaxBatches = 64;  // BatchRefs stays under the 4 KB kernel-argument limit
struct BatchRefs {
  const uint8_t *pk[kMaxBatches];
  const uint8_t *sig[kMaxBatches];
  const uint8_t *msg[kMaxBatches];
  const uint32_t *off[kMaxBatches];
  int8_t *out[kMaxBatches];
  uint32_t start[kMaxBatches + 1];     // first gathered entry of each batch
  uint32_t msg_base[kMaxBatches + 1];  // first gathered message byte of each batch
  uint32_t nb;
};
hipError_t launch_gather(const BatchRefs &r, uint8_t *pk, uint8_t *sig, uint32_t *off, uint8_t *msg,
                         hipStream_t stream);
hipError_t launch_scatter(const BatchRefs &r, const int8_t *status, hipStream_t stream);

// Key-merged batch equation (msm.h): R decode + challenge with Niels(-R) in
// w.niels, and the key-cached comb verification of the entries of failing
// groups (passing groups' entries take their pre-check status).
// With idx, work slot e reads entry idx[e] (the key order) and writes the
// status of idx[e]; per-entry work arrays are indexed by e.
template <bool SR>
hipError_t launch_prep_cached(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off,
                              const uint32_t *idx, uint32_t n, const strobe_t *prefix, Ed25519Work w, int aligned,
                              hipStream_t stream);
template <bool SR>
hipError_t launch_comb_fallback(const uint8_t *sig, const uint32_t *key_slot, const uint32_t *idx, uint32_t n,
                                Ed25519Work w, KeyTable kt, const fe *bcomb, uint8_t *out, int aligned,
                                const uint8_t *group_ok, uint32_t group_log2, hipStream_t stream);
// Runs of one key inside a group, in key order: run r covers work slots
// [lo[r], lo[r + 1]) of key slot slot[r]; group g's runs are
// [group_run0[g], group_run0[g + 1]).  order[e] is the entry at work slot e.
struct KeyRuns {
  const uint32_t *lo;
  const uint32_t *slot;
  const uint32_t *group_run0;
  const uint32_t *order;
  uint32_t n_runs;
};
hipError_t launch_key_merged_check(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                   const uint32_t *msg_off, const uint32_t *key_slot, KeyRuns runs, uint32_t n,
                                   KeyTable kt, const fe *bcomb, const strobe_t *prefix, Ed25519Work w, MsmWork mw,
                                   const MsmParams &p, const MsmSeed &seed, uint8_t *out, hipStream_t stream);

// Vote sign-bytes from templates (signbytes_kernels.hip, votes.h).
struct VoteTab;
hipError_t launch_vote_signbytes(const tmv_vote *votes, const VoteTab *tab, const uint8_t *blob,
                                 const uint32_t *off, uint32_t n, uint8_t *msg, hipStream_t stream);

hipError_t launch_ed25519_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                 const uint32_t *msg_off, uint32_t n, const ge_precomp *btable,
                                 uint8_t *valid, hipStream_t stream);

}  // namespace tmv
