/*
 * tmhost.h — C-ABI of the host layer above the verification engine
 * (libtmgpu.so): the crypto.BatchVerifier object, canonical vote sign-bytes
 * and the commit verifiers, implemented in C++ (tendermint_amd/csrc/host/)
 * over include/tmverify.h.  Plain pointers and sizes only.
 *
 * These are the entry points a Go cgo shim binds:
 *   tmv_batch_*        crypto.BatchVerifier (crypto/crypto.go:66-76) created
 *                      by batch.CreateBatchVerifier (crypto/batch/batch.go:11-21)
 *   tmv_vote_sign_bytes types.VoteSignBytes (types/vote.go:149-157)
 *   tmv_verify_commit  types.VerifyCommit / VerifyCommitLight /
 *                      VerifyCommitLightTrusting (types/validation.go:27,61,96)
 *   tmv_light_verify   light.Verify / VerifyAdjacent / VerifyNonAdjacent
 *                      (light/verifier.go:33-177)
 *   tmv_header_hashes  types.Header.Hash (types/block.go:447-478)
 */
#ifndef TMHOST_H
#define TMHOST_H

#include <stddef.h>
#include <stdint.h>

#include "tmverify.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Key kinds: TMV_KIND_ED25519, TMV_KIND_SR25519; anything else is a key type
 * without batch support (e.g. secp256k1, crypto/batch/batch.go:13-20). */
#define TMV_KIND_OTHER 255

/* ---- crypto.BatchVerifier ---- */
typedef struct tmv_batch tmv_batch;

/* batch.CreateBatchVerifier: NULL when key_kind has no batch verifier. */
tmv_batch *tmv_batch_new(tmv_ctx *ctx, uint8_t key_kind);
/* Add: returns 0, or 1 with the reference's error text in err (type and
 * length checks: crypto/ed25519/ed25519.go:209-224,
 * crypto/sr25519/batch.go:23-28).  Curve-decoding failures of sr25519 keys
 * and signatures are reported by tmv_batch_verify (deferred Add error). */
int tmv_batch_add(tmv_batch *b, uint8_t key_kind, const uint8_t *pk, size_t pk_len, const uint8_t *msg,
                  size_t msg_len, const uint8_t *sig, size_t sig_len, char *err, size_t err_cap);
size_t tmv_batch_len(const tmv_batch *b);
/* Verify: 1 all valid, 0 not (or empty), 2 a deferred Add error (index in
 * *add_err_index, text in err), < 0 infrastructure error.  valid_out gets
 * one byte per entry in Add order. */
int tmv_batch_verify(tmv_batch *b, uint8_t *valid_out, int64_t *add_err_index, char *err, size_t err_cap);
void tmv_batch_free(tmv_batch *b);

/* ---- commit data ---- */
typedef struct {
  const uint8_t *hash;
  uint32_t hash_len;
  uint32_t psh_total;
  const uint8_t *psh_hash;
  uint32_t psh_hash_len;
} tmv_block_id;

typedef struct {
  const uint8_t *address;
  uint32_t address_len;
  const uint8_t *pub_key;
  uint32_t pub_key_len;
  uint8_t key_kind;
  int64_t voting_power;
  int64_t proposer_priority;
} tmv_validator;

typedef struct {
  uint8_t block_id_flag; /* 1 absent, 2 commit, 3 nil */
  const uint8_t *validator_address;
  uint32_t validator_address_len;
  int64_t ts_seconds;
  int32_t ts_nanos;
  const uint8_t *signature;
  uint32_t signature_len;
} tmv_commit_sig;

typedef struct {
  int64_t height;
  int32_t round;
  tmv_block_id block_id;
  const tmv_commit_sig *sigs;
  uint32_t n_sigs;
} tmv_commit;

/* types.VoteSignBytes for (chain_id, type, height, round, block_id or NULL
 * for nil, timestamp).  Returns the length; writes min(len, cap) bytes. */
size_t tmv_vote_sign_bytes(const char *chain_id, int32_t vote_type, int64_t height, int32_t round,
                           const tmv_block_id *block_id, int64_t ts_seconds, int32_t ts_nanos, uint8_t *out,
                           size_t cap);

/* The vote template of tmv_verify_votes (tmverify.h) for (chain_id, type,
 * height, round, block_id or NULL for nil): the three segments are written
 * back to back into out (head, then block, then chain) and their lengths
 * into lens[3].  Returns the total length; writes min(total, cap) bytes. */
size_t tmv_vote_template_encode(const char *chain_id, int32_t vote_type, int64_t height, int32_t round,
                                const tmv_block_id *block_id, uint8_t *out, size_t cap, uint32_t lens[3]);

#define TMV_COMMIT_FULL 0           /* types.VerifyCommit */
#define TMV_COMMIT_LIGHT 1          /* types.VerifyCommitLight */
#define TMV_COMMIT_LIGHT_TRUSTING 2 /* types.VerifyCommitLightTrusting */

/* Verify a commit against a validator set.  vals == NULL means a nil
 * validator set, commit == NULL a nil commit.  proposer_index < 0 derives
 * the proposer from priorities.  block_id / height are ignored for
 * LIGHT_TRUSTING; trust_num / trust_den only apply to it.
 * Returns 0 (ok), 1 (verification error; text in err, byte-identical to the
 * reference's error), < 0 infrastructure error. */
int tmv_verify_commit(tmv_ctx *ctx, int mode, const char *chain_id, const tmv_validator *vals, uint32_t n_vals,
                      int32_t proposer_index, const tmv_block_id *block_id, int64_t height, const tmv_commit *commit,
                      int64_t trust_num, int64_t trust_den, char *err, size_t err_cap);

/* Many commit checks in one device batch (cross-commit batching: blocksync
 * look-ahead, light-client sequential headers).  Each job is
 * one tmv_verify_commit call; results[j] = 0 ok / 1 error (text at
 * errs + j*err_stride), identical to calling tmv_verify_commit per job.
 * Jobs that pass the same tmv_commit pointer share signature entries (a
 * commit that blocksync checks light and then full is verified once).
 * Returns the number of failed jobs, or < 0 on an infrastructure error. */
typedef struct {
  int mode;
  const char *chain_id;
  const tmv_validator *vals;
  uint32_t n_vals;
  int32_t proposer_index;
  const tmv_block_id *block_id;
  int64_t height;
  const tmv_commit *commit;
  int64_t trust_num;
  int64_t trust_den;
} tmv_commit_job;

int tmv_verify_commits(tmv_ctx *ctx, const tmv_commit_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                       size_t err_stride);

/* ---- consensus votes (ADR-064 batched vote verification) ---- */
/* The parts of a types.Vote (types/vote.go:50-62) Vote.Verify reads, with
 * the signing validator's public key (val.PubKey, looked up by the caller
 * from ValidatorIndex as VoteSet.addVote does, types/vote_set.go:183-199). */
typedef struct {
  int32_t type; /* SignedMsgType: 1 prevote, 2 precommit */
  int64_t height;
  int32_t round;
  const tmv_block_id *block_id; /* NULL (or a nil BlockID) = vote for nil */
  int64_t ts_seconds;
  int32_t ts_nanos;
  const uint8_t *validator_address;
  uint32_t validator_address_len;
  const uint8_t *signature;
  uint32_t signature_len;
  uint8_t key_kind; /* TMV_KIND_ED25519 / TMV_KIND_SR25519 */
  const uint8_t *pub_key;
  uint32_t pub_key_len;
} tmv_vote_in;

#define TMV_VOTE_OK 0
#define TMV_VOTE_ERR_INVALID_ADDRESS 1   /* types.ErrVoteInvalidValidatorAddress */
#define TMV_VOTE_ERR_INVALID_SIGNATURE 2 /* types.ErrVoteInvalidSignature */

/* Vote.Verify(chainID, pubKey) (types/vote.go:226-243: address check, then
 * PubKey.VerifySignature over VoteSignBytes) of n votes in ONE signature
 * batch: the batched vote verification ADR-064 describes for consensus
 * (docs/architecture/adr-064-batch-verification.md:58-64: once 2/3+ of the
 * votes have arrived they are verified together).  results[i] = TMV_VOTE_*,
 * identical to verifying vote i alone.  Returns the number of failed votes,
 * or < 0 on an infrastructure error. */
int tmv_verify_vote_batch(tmv_ctx *ctx, const char *chain_id, const tmv_vote_in *votes, uint32_t n,
                          int32_t *results);

/* ---- light client (light/verifier.go) ---- */
typedef struct {
  const uint8_t *p;
  uint32_t len;
} tmv_bytes;

/* types.Header (types/block.go:338-366); chain_id NUL-terminated. */
typedef struct {
  uint64_t version_block, version_app;
  const char *chain_id;
  int64_t height;
  int64_t time_seconds;
  int32_t time_nanos;
  tmv_block_id last_block_id;
  tmv_bytes last_commit_hash, data_hash, validators_hash, next_validators_hash, consensus_hash, app_hash,
      last_results_hash, evidence_hash, proposer_address;
} tmv_header;

/* types.SignedHeader (types/light.go:131-136); NULL members = nil. */
typedef struct {
  const tmv_header *header;
  const tmv_commit *commit;
} tmv_signed_header;

/* types.ValidatorSet (proposer_index < 0: derived from the priorities). */
typedef struct {
  const tmv_validator *vals;
  uint32_t n_vals;
  int32_t proposer_index;
} tmv_validator_set;

/* Header.Hash (types/block.go:447-478) of n headers; has_hash[i] = 0 when the
 * reference returns nil (empty ValidatorsHash), else hash_out + 32*i holds it.
 * Many headers go to the device in one tmv_merkle_roots launch.  0 or < 0. */
int tmv_header_hashes(tmv_ctx *ctx, const tmv_header *headers, uint32_t n, uint8_t *hash_out, uint8_t *has_hash);

#define TMV_LIGHT_VERIFY 0       /* light.Verify (light/verifier.go:158-177) */
#define TMV_LIGHT_ADJACENT 1     /* light.VerifyAdjacent (light/verifier.go:106-155) */
#define TMV_LIGHT_NON_ADJACENT 2 /* light.VerifyNonAdjacent (light/verifier.go:33-91) */

/* Result classes (light/errors.go:15-40): the reference's error types. */
#define TMV_LIGHT_OK 0
#define TMV_LIGHT_ERR_INVALID_HEADER 1     /* light.ErrInvalidHeader */
#define TMV_LIGHT_ERR_OLD_HEADER_EXPIRED 2 /* light.ErrOldHeaderExpired */
#define TMV_LIGHT_ERR_CANT_TRUST 3         /* light.ErrNewValSetCantBeTrusted */
#define TMV_LIGHT_ERR_OTHER 4              /* a plain error (errors.New / fmt.Errorf) */

/* One light-client verification: the arguments of light.Verify /
 * VerifyAdjacent / VerifyNonAdjacent.  trusted_vals = the trusted header's
 * next validators (unused by VerifyAdjacent); times are UTC; trust level
 * = trust_num / trust_den (tmmath.Fraction). */
typedef struct {
  int mode; /* TMV_LIGHT_VERIFY / _ADJACENT / _NON_ADJACENT */
  const tmv_signed_header *trusted;
  const tmv_validator_set *trusted_vals;
  const tmv_signed_header *untrusted;
  const tmv_validator_set *untrusted_vals;
  int64_t trusting_period_ns;
  int64_t now_seconds;
  int32_t now_nanos;
  int64_t max_clock_drift_ns;
  uint64_t trust_num, trust_den;
} tmv_light_job;

/* Many light verifications in one pass: header and validator-set hashes of
 * all jobs in one device launch each, every commit check of all jobs in one
 * signature batch (tmv_verify_commits).  results[j] = TMV_LIGHT_* class,
 * error text at errs + j*err_stride, each identical to a tmv_light_verify
 * of job j alone.  Returns the number of failed jobs or < 0 (infrastructure). */
int tmv_light_verify_many(tmv_ctx *ctx, const tmv_light_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                          size_t err_stride);
/* One job: returns its TMV_LIGHT_* class (text in err) or < 0. */
int tmv_light_verify(tmv_ctx *ctx, const tmv_light_job *job, char *err, size_t err_cap);

#ifdef __cplusplus
}
#endif
#endif /* TMHOST_H */
