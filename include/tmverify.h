/*
 * tmverify.h — C-ABI of the MI355X signature-verification engine
 * (libtmgpu.so).  Plain pointers and sizes only; no torch or HIP types.
 *
 * This is the L0 replacement behind Tendermint's crypto.BatchVerifier
 * (crypto/crypto.go:66-76).  Each entry point names the reference interface
 * it replaces; INTEGRATION.md shows the cgo binding a maintainer adds to
 * crypto/ed25519, crypto/sr25519 and crypto/batch.
 *
 * Packed batch layout (shared by every batch entry point):
 *   pk      n x 32 bytes, entry i at pk + 32*i
 *   sig     n x 64 bytes, entry i at sig + 64*i  (R || S)
 *   msg     concatenated messages
 *   msg_off n+1 offsets into msg; message i = msg[msg_off[i] .. msg_off[i+1])
 *
 * Return codes of the batch entry points:
 *   TMV_ALL_VALID (1)   n > 0 and every entry verified
 *   TMV_NOT_ALL   (0)   some entry failed, or n == 0 (voi: an empty batch
 *                       verifies false)
 *   < 0                 infrastructure error (no device, allocation, launch,
 *                       TMV_ERR_TIMEOUT);
 *                       the validity vector is then unspecified and the
 *                       caller must not treat any entry as verified.
 */
#ifndef TMVERIFY_H
#define TMVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMV_ALL_VALID 1
#define TMV_NOT_ALL 0
#define TMV_ERR_ARG (-1)
#define TMV_ERR_NO_DEVICE (-2)
#define TMV_ERR_NOMEM (-3)
#define TMV_ERR_LAUNCH (-4)
/* A device wait exceeded $TMV_DEVICE_TIMEOUT_MS (default 60000; 0 = wait
 * forever).  The context's device work is then in an unknown state: the
 * context refuses further work (every call returns TMV_ERR_TIMEOUT); the
 * caller verifies on the CPU and may tmv_close / tmv_open a new context.
 * Pages of the caller's buffers (inputs and status array) that a streamed
 * call had registered for direct DMA stay page-locked after a failed call: the
 * device may still read them, so they are never unregistered under it (and
 * the library keeps no record that could unregister them once reused). */
#define TMV_ERR_TIMEOUT (-5)
/* The OS random source (getrandom) failed while drawing a batch equation's
 * weights (the reference's rand.Reader error, crypto/ed25519/ed25519.go:232);
 * nothing was launched.  tmv_last_error() names the errno. */
#define TMV_ERR_RANDOM (-6)

/* Per-entry sr25519 status (tmv_sr25519_verify_batch, tmv_verify_mixed_batch):
 *   1 valid, 0 invalid, TMV_SR_ADDERR_* = BatchVerifier.Add would have
 *   returned an error (crypto/sr25519/batch.go:30-37). */
#define TMV_SR_ADDERR_PUBKEY (-1)
#define TMV_SR_ADDERR_SIG (-2)

/* Key kinds for tmv_verify_mixed_batch (crypto/batch/batch.go:11-21). */
#define TMV_KIND_ED25519 0
#define TMV_KIND_SR25519 1

typedef struct tmv_ctx tmv_ctx;

/* Open a context on the GPUs selected by device_mask (bit i = HIP device i;
 * 0 = all visible devices).  Builds the per-device base-point tables.
 * Returns NULL on failure (tmv_last_error() says why). */
tmv_ctx *tmv_open(uint32_t device_mask);
/* TEST AID, not for deployments: as tmv_open, but each selected GPU joins the
 * context as `logical` devices (1..8: own streams, lanes, workspaces, key
 * cache), so the multi-device shard / harvest path runs on a one-GPU box.
 * tmv_num_devices then counts logical devices, while the device-pointer entry
 * points still name a GPU by its HIP id (its first logical device).
 * Announces itself on stderr when logical > 1. */
tmv_ctx *tmv_open_logical(uint32_t device_mask, int logical);
void tmv_close(tmv_ctx *ctx);
int tmv_num_devices(const tmv_ctx *ctx);
const char *tmv_last_error(void);
/* "tmverify-mi355x <ver> (gfx950) src=<digest> git=<head>": the source digest
   (tendermint_amd/csrc/src_digest.py over the sources this library is built
   from) and the git HEAD compiled in by the Makefile. */
const char *tmv_version(void);

/* ed25519 batch verification with ZIP-215 semantics.
 * Replaces: crypto/ed25519/ed25519.go:231-233 BatchVerifier.Verify (after the
 * Adds of :209-229 have been collected into the packed arrays; the Go-side
 * Add keeps its type/length checks and error strings).
 * Multi-device contexts shard the batch by contiguous index ranges.
 * valid_out[i] = 1/0 in Add order. */
int tmv_ed25519_verify_batch(tmv_ctx *ctx, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                             const uint32_t *msg_off, uint32_t n, uint8_t *valid_out);

/* Single ed25519 verification.
 * Replaces: crypto/ed25519/ed25519.go:173-180 PubKey.VerifySignature
 * (returns 0 when sig_len != 64, as the reference does).  Returns 1/0 or <0. */
int tmv_ed25519_verify(tmv_ctx *ctx, const uint8_t *pk, const uint8_t *msg, size_t msg_len,
                       const uint8_t *sig, size_t sig_len);

/* sr25519 batch verification (Schnorrkel, empty signing context).
 * Replaces: crypto/sr25519/batch.go:23-47 Add + Verify.  status_out[i] is
 * 1 / 0 / TMV_SR_ADDERR_*; the return value is TMV_ALL_VALID only if every
 * status is 1. */
int tmv_sr25519_verify_batch(tmv_ctx *ctx, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                             const uint32_t *msg_off, uint32_t n, int8_t *status_out);

/* Mixed ed25519 + sr25519 batch in one launch; kind[i] = TMV_KIND_*.
 * status_out as for sr25519 (ed25519 entries are 1/0). */
int tmv_verify_mixed_batch(tmv_ctx *ctx, const uint8_t *kind, const uint8_t *pk, const uint8_t *sig,
                           const uint8_t *msg, const uint32_t *msg_off, uint32_t n, int8_t *status_out);

/* Batch verification with options.  flags:
 *   TMV_FLAG_KEY_CACHE  keep expanded public keys on the device (LRU of
 *   TMV_KEY_CACHE_CAPACITY keys per device, default 4,096 = voi's cache size,
 *   crypto/ed25519/ed25519.go:31,56).  A cached key is a 64-row comb of -A
 *   (80 KB), so [k]A needs no doublings; the first batch that sees a key
 *   pays its table build.  Batches with more distinct keys than the cache
 *   holds take the uncached path transparently.  Results are identical
 *   either way.
 * Replaces the caching verifier behind crypto/ed25519/ed25519.go:173-233
 * (ed25519) and crypto/sr25519/batch.go:23-47 (sr25519).  status_out as for
 * tmv_sr25519_verify_batch (ed25519 entries are 1/0). */
#define TMV_FLAG_KEY_CACHE 1u
int tmv_verify_batch_ex(tmv_ctx *ctx, uint8_t key_kind, uint32_t flags, const uint8_t *pk, const uint8_t *sig,
                        const uint8_t *msg, const uint32_t *msg_off, uint32_t n, int8_t *status_out);
/* Batch equation (random linear combination), the
 * check voi's BatchVerifier.Verify runs (crypto/ed25519/ed25519.go:231-233,
 * crypto/sr25519/batch.go:44-47): entries are split into groups of
 * 2^group_log2 consecutive signatures of one kind; each group is checked with
 * one multi-scalar multiplication under fresh 128-bit random weights
 * (ed25519: cofactored [8](...) == O, ZIP-215; sr25519: Ristretto identity)
 * and the entries of a failing group are verified one by one, so the
 * validity vector is the same as per-entry verification (false accept
 * probability <= 2^-128 per group, as the reference's).
 *   TMV_FLAG_BATCH_EQUATION  use it for this call
 *   TMV_FLAG_PER_ENTRY       never use it for this call
 * Neither flag: batch equation when n >= $TMV_MSM_MIN (default 32768, key-
 * cached batches 16384; the variable sets both, 0 = never): smaller batches
 * are latency-bound and verify faster per entry.
 * TMV_FLAG_BATCH_EQUATION overrides TMV_FLAG_KEY_CACHE. */
#define TMV_FLAG_BATCH_EQUATION 2u
#define TMV_FLAG_PER_ENTRY 4u
/* group_log2: 0 = default (6) or 5..10; window_bits: 0 = chosen from the group
 * size, or 4..9; seed32: NULL = a fresh getrandom() key per call (production),
 * else a fixed ChaCha20 key (tests: reproducible weights).
 * opt_flags: TMV_BATCHOPT_STATS = count group verdicts (host-buffer calls;
 * costs one small device read per call); TMV_BATCHOPT_SUBCHECK_ON / _OFF =
 * re-check failing groups by sub-groups of 8 before the per-entry fallback
 * (default: for groups of >= 256 entries); with it off,
 * launches of >= $TMV_LOCATE_MIN (400000) entries locate a failing group's
 * one bad entry by a second, index-weighted equation. */
#define TMV_BATCHOPT_STATS 1u
#define TMV_BATCHOPT_SUBCHECK_ON 2u
#define TMV_BATCHOPT_SUBCHECK_OFF 4u
int tmv_set_batch_options(tmv_ctx *ctx, uint32_t group_log2, uint32_t window_bits, const uint8_t *seed32,
                          uint32_t opt_flags);
/* Groups checked / failed since the context was opened (TMV_BATCHOPT_STATS). */
int tmv_batch_stats(tmv_ctx *ctx, uint64_t *groups, uint64_t *groups_failed);
/* ValidatorSet.Hash of n_sets validator sets in one launch (SURVEY §8(f)
 * rank 4): replaces types/validator_set.go:344-350 (merkle.HashFromByteSlices,
 * crypto/merkle/tree.go:11-27, over Validator.Bytes(), types/validator.go:
 * 154-170), as the light client checks it per header (light/verifier.go:266).
 * Set s holds validators [set_off[s], set_off[s+1]) in set order; validator
 * i: pk + 32*i, key_kind[i] (TMV_KIND_ED25519 / TMV_KIND_SR25519; secp256k1
 * keys are not supported), power[i].  hash_out: n_sets x 32 bytes (an empty
 * set hashes to SHA-256(""), as the reference).  set_off[0] must be 0.
 * Synchronous; 0 or < 0 on error. */
int tmv_validator_set_hashes(tmv_ctx *ctx, const uint8_t *pk, const uint8_t *key_kind, const int64_t *power,
                             const uint32_t *set_off, uint32_t n_sets, uint8_t *hash_out);
/* merkle.HashFromByteSlices of n_trees trees in one launch (crypto/merkle/
 * tree.go:11-27: RFC 6962 leaves SHA-256(0x00 || leaf), inner nodes
 * SHA-256(0x01 || l || r), split at the largest power of two below n).  The
 * host layer uses it for Header.Hash (types/block.go:447-478: 14 proto-encoded
 * fields per header) across a light client's window of headers.
 * Leaf i = data[leaf_off[i], leaf_off[i+1]) (n_leaves + 1 offsets,
 * leaf_off[0] = 0); tree t = leaves [tree_off[t], tree_off[t+1]) (n_trees + 1
 * offsets, tree_off[0] = 0, tree_off[n_trees] = n_leaves; an empty tree
 * hashes to SHA-256("")).  hash_out: n_trees x 32 bytes.  Synchronous; 0 or
 * < 0 on error. */
int tmv_merkle_roots(tmv_ctx *ctx, const uint8_t *data, const uint32_t *leaf_off, uint32_t n_leaves,
                     const uint32_t *tree_off, uint32_t n_trees, uint8_t *hash_out);
/* Sub-groups of failing groups checked / failed (k_msm_subcheck: a failing
 * group's sub-groups of 8 entries are re-checked with the same equation
 * before entry-by-entry verification; TMV_BATCHOPT_STATS; 0 with
 * the sub-group check off).  No reference counterpart (voi verifies a failing batch
 * entry by entry, crypto/ed25519/ed25519.go:231-233). */
int tmv_subgroup_stats(tmv_ctx *ctx, uint64_t *subgroups, uint64_t *subgroups_failed);
/* Mixed batch with flags (see tmv_verify_mixed_batch). */
int tmv_verify_mixed_batch_ex(tmv_ctx *ctx, uint32_t flags, const uint8_t *kind, const uint8_t *pk,
                              const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off, uint32_t n,
                              int8_t *status_out);

/* Live kernel timing (profiling aid; bench.py's roofline object).  enable != 0:
 * every later launch of the timed kernels -- "k_msm_accum" (batch-equation
 * bucket sums), "k_msm_wpart" (window running sums), "k_prep_fused" (decode +
 * challenge) -- is bracketed by HIP timing events on the stream it runs on
 * (process-wide, two event records per launch); 0 turns it off.
 * tmv_kernel_timing_read waits for the recorded launches of `kernel`, returns
 * their summed duration and count, and forgets them.  No reference
 * counterpart (Go's benchmarks time whole calls). */
int tmv_kernel_timing(tmv_ctx *ctx, int enable);
int tmv_kernel_timing_read(tmv_ctx *ctx, const char *kernel, double *total_ms, uint64_t *launches);

/* Cumulative key-cache counters over the context's devices. */
int tmv_key_cache_stats(tmv_ctx *ctx, uint64_t *hits, uint64_t *misses, uint32_t *used, uint32_t *capacity);

/* Library metrics (verifies/s, batch size, fallback count, H2D
 * bytes -- the reference exports its own per package through Prometheus,
 * e.g. internal/consensus/metrics.gen.go; a Go shim would publish these).
 * Cumulative since tmv_open or the last tmv_metrics_reset.  The group fields
 * count host-buffer calls made with TMV_BATCHOPT_STATS
 * (tmv_set_batch_options); the rest are always kept. */
typedef struct tmv_metrics {
  uint64_t calls;               /* verification calls (host-buffer and device-resident entry points) */
  uint64_t signatures;          /* entries submitted to them */
  uint64_t max_batch;           /* largest call, in entries */
  uint64_t batch_eq_signatures; /* entries verified through the batch equation */
  uint64_t host_signatures;     /* entries of host-buffer calls */
  double host_seconds;          /* busy wall time of host-buffer calls: the union of their intervals, so calls
                                   in flight together count once (end-to-end rate = host_signatures / it);
                                   a call still in flight is not yet counted */
  uint64_t h2d_bytes;           /* host-to-device bytes of host-buffer calls (zero-copy reads not counted) */
  uint64_t d2h_bytes;           /* device-to-host bytes of host-buffer calls */
  uint64_t groups;              /* batch-equation groups checked (TMV_BATCHOPT_STATS) */
  uint64_t groups_failed;       /* of which failed */
  uint64_t located_groups;      /* failing groups whose one bad entry the located pass named */
  uint64_t fallback_signatures; /* entries verified one by one after failing groups */
  uint64_t key_cache_hits;      /* expanded-key cache (TMV_FLAG_KEY_CACHE) */
  uint64_t key_cache_misses;
} tmv_metrics;
int tmv_metrics_read(tmv_ctx *ctx, tmv_metrics *out);
int tmv_metrics_reset(tmv_ctx *ctx);

/* Device-resident variants: every pointer is device memory on HIP device
 * `device` (inputs already in HBM), `stream` is a hipStream_t (NULL = the
 * context's own stream for that device).  Asynchronous: the call enqueues the
 * kernel and returns TMV_NOT_ALL immediately (the verdict is in d_valid once
 * the stream is synchronised), or <0 on a launch error.  Used by the
 * multi-GPU sharded path (one process per GPU) and by bench.py. */
int tmv_ed25519_verify_batch_device(tmv_ctx *ctx, int device, const uint8_t *d_pk, const uint8_t *d_sig,
                                    const uint8_t *d_msg, const uint32_t *d_msg_off, uint32_t n,
                                    uint8_t *d_valid, void *stream);
int tmv_verify_mixed_batch_device(tmv_ctx *ctx, int device, const uint8_t *d_kind, const uint8_t *d_pk,
                                  const uint8_t *d_sig, const uint8_t *d_msg, const uint32_t *d_msg_off,
                                  uint32_t n, int8_t *d_status, void *stream);
/* Device-resident batch with flags; key_kind TMV_KIND_ED25519, TMV_KIND_SR25519
 * or TMV_KIND_MIXED (then d_kind gives each entry's kind).  d_status as for
 * tmv_sr25519_verify_batch (ed25519 entries 1/0). */
#define TMV_KIND_MIXED 2
int tmv_verify_batch_device_ex(tmv_ctx *ctx, int device, uint8_t key_kind, uint32_t flags, const uint8_t *d_kind,
                               const uint8_t *d_pk, const uint8_t *d_sig, const uint8_t *d_msg,
                               const uint32_t *d_msg_off, uint32_t n, int8_t *d_status, void *stream);

/* Several independent device-resident batches in one pipeline: the batches
 * are gathered into one contiguous batch on the device, verified together
 * (per-entry or batch equation, per flags) and each batch's statuses are
 * written to its own d_status (as tmv_verify_batch_device_ex).  Verdicts are
 * per entry, so this equals n_batches separate calls; it only widens the
 * launches (a node draining a queue of batches, blocksync look-ahead).
 * msg_bytes = msg_off[n] - msg_off[0].  Up to TMV_MAX_BATCHES batches (and
 * 2^26 entries in all); key_kind TMV_KIND_ED25519 or TMV_KIND_SR25519.
 * Asynchronous like the other device-resident entry points. */
#define TMV_MAX_BATCHES 256
typedef struct tmv_batch_ref {
  const uint8_t *pk;
  const uint8_t *sig;
  const uint8_t *msg;
  const uint32_t *msg_off;
  uint32_t n;
  uint32_t msg_bytes;
  int8_t *status;
} tmv_batch_ref;
int tmv_verify_batches_device(tmv_ctx *ctx, int device, uint8_t key_kind, uint32_t flags,
                              const tmv_batch_ref *batches, uint32_t n_batches, void *stream);

/* ---- Device-side vote sign-bytes ----
 * The canonical votes of one commit differ only in the timestamp and in
 * whether field 4 (the BlockID) is present: Commit.VoteSignBytes,
 * types/block.go:836-862, over CanonicalizeVote, types/canonical.go:52-63.
 * The caller encodes the shared fields once per (commit, chain_id) -- a
 * template, see tmv_vote_template_encode in tmhost.h -- and sends 16 bytes
 * per vote instead of the ~120-byte message; the device writes
 *   uvarint(len(body)) || head || [block] || 0x2a uvarint(len(ts)) ts || chain
 * into HBM, where ts = [0x08 uvarint(seconds)] [0x10 uvarint(nanos)] (proto3:
 * zero fields omitted), byte-identical to types.VoteSignBytes. */
typedef struct tmv_vote_template {
  const uint8_t *head;  /* fields 1-3 (type, height, round) */
  uint32_t head_len;
  const uint8_t *block; /* field 4, the commit's BlockID (empty when nil) */
  uint32_t block_len;
  const uint8_t *chain; /* field 6, chain_id (empty when "") */
  uint32_t chain_len;
} tmv_vote_template;

#define TMV_VOTE_WITH_BLOCK 0x80000000u /* tmpl bit: BlockIDFlagCommit, field 4 included */

typedef struct tmv_vote {
  int64_t ts_seconds;
  int32_t ts_nanos;
  uint32_t tmpl; /* template index | TMV_VOTE_WITH_BLOCK */
} tmv_vote;

/* tmv_verify_batch_ex over device-built sign-bytes: entry i signs the
 * message of votes[i].  Same flags, statuses and return values as
 * tmv_verify_batch_ex (TMV_ERR_ARG for a template index >= n_tmpl). */
int tmv_verify_votes(tmv_ctx *ctx, uint8_t key_kind, uint32_t flags, const tmv_vote_template *tmpl,
                     uint32_t n_tmpl, const tmv_vote *votes, const uint8_t *pk, const uint8_t *sig, uint32_t n,
                     int8_t *status_out);

/* The messages the device builds for tmv_verify_votes, copied back (tests,
 * tools).  msg_off_out gets n + 1 offsets; msg_out (capacity msg_cap) the
 * concatenated messages, or is skipped when NULL.  Returns the total length,
 * or < 0 (TMV_ERR_ARG if msg_cap is too small). */
int64_t tmv_vote_sign_bytes_device(tmv_ctx *ctx, const tmv_vote_template *tmpl, uint32_t n_tmpl,
                                   const tmv_vote *votes, uint32_t n, uint8_t *msg_out, size_t msg_cap,
                                   uint32_t *msg_off_out);

#ifdef __cplusplus
}
#endif
#endif /* TMVERIFY_H */
