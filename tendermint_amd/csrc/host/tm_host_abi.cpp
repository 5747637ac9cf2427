// C-ABI of the host layer (include/tmhost.h): crypto.BatchVerifier objects
// backed by the GPU entry points of include/tmverify.h, canonical vote
// sign-bytes, and the commit verifiers of tm_types.h instantiated with them.
// Only the public tmv_* C-ABI is used to reach the device (layering).
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/tmhost.h"
#include "../../../include/tmverify.h"
#include "tm_types.h"

namespace {

void put_err(char *err, size_t cap, const std::string &s) {
  if (!err || cap == 0) return;
  const size_t n = std::min(cap - 1, s.size());
  std::memcpy(err, s.data(), n);
  err[n] = 0;
}

const uint8_t kL[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                        0xa2, 0xde, 0xf9, 0xde, 0x14, 0,    0,    0,    0,    0,    0,
                        0,    0,    0,    0,    0,    0,    0,    0,    0,    0x10};

bool scalar_canonical(const uint8_t s[32]) {
  for (int i = 31; i >= 0; i--) {
    if (s[i] < kL[i]) return true;
    if (s[i] > kL[i]) return false;
  }
  return false;
}

// Packed entries + GPU verify.
class GpuBatch : public tmh::BatchVerifier {
 public:
  GpuBatch(tmv_ctx *ctx, tmh::KeyType kind) : ctx_(ctx), kind_(kind) { off_.push_back(0); }

  tmh::Error Add(const tmh::PubKey &key, const tmh::Bytes &msg, const tmh::Bytes &sig) override {
    if (kind_ == tmh::KeyType::Ed25519) {
      // crypto/ed25519/ed25519.go:209-224
      if (key.type != tmh::KeyType::Ed25519) return std::string("pubkey is not Ed25519");
      if (key.bytes.size() != 32)
        return "pubkey size is incorrect; expected: 32, got " + std::to_string(key.bytes.size());
      if (sig.size() != 64) return std::string("invalid signature");
      push(key.bytes.data(), msg, sig.data(), "");
      return std::nullopt;
    }
    // crypto/sr25519/batch.go:23-28: type check is synchronous ...
    if (key.type != tmh::KeyType::Sr25519) return std::string("sr25519: pubkey is not sr25519");
    // ... decoding failures are resolved on the device (status -1 / -2 with
    // the public key taking precedence, like the reference's Add order).
    if (key.bytes.size() != 32) {
      return "sr25519: invalid public key: sr25519: bad PublicKey size: " + std::to_string(key.bytes.size());
    }
    std::string sig_err;
    uint8_t s64[64] = {0};
    if (sig.size() != 64) {
      sig_err = "sr25519: unable to decode signature: sr25519: bad Signature size: " + std::to_string(sig.size());
    } else {
      std::memcpy(s64, sig.data(), 64);
      uint8_t s[32];
      std::memcpy(s, s64 + 32, 32);
      if (!(s[31] & 0x80)) {
        sig_err = "sr25519: unable to decode signature: sr25519: signature is not marked as a schnorrkel signature";
      } else {
        s[31] &= 0x7f;
        if (!scalar_canonical(s)) sig_err = "sr25519: unable to decode signature: sr25519: non-canonical scalar";
      }
    }
    push(key.bytes.data(), msg, s64, sig_err);
    return std::nullopt;
  }

  std::pair<bool, std::vector<bool>> Verify() override {
    const uint32_t n = (uint32_t)sig_err_.size();
    std::vector<bool> valid(n, false);
    deferred_.reset();
    if (n == 0) return {false, valid};
    std::vector<uint8_t> out(n);
    int rc;
    // Validator keys repeat across commits: use the device key cache (the
    // reference's LRU caching verifier, crypto/ed25519/ed25519.go:31).
    static const uint8_t z = 0;
    rc = tmv_verify_batch_ex(ctx_, kind_ == tmh::KeyType::Ed25519 ? TMV_KIND_ED25519 : TMV_KIND_SR25519,
                             TMV_FLAG_KEY_CACHE, pk_.data(), sig_.data(), msg_.empty() ? &z : msg_.data(),
                             off_.data(), n, reinterpret_cast<int8_t *>(out.data()));
    if (rc < 0) {
      infra_error_ = rc;
      return {false, valid};
    }
    bool all = true;
    for (uint32_t i = 0; i < n; i++) {
      const int8_t st = (int8_t)out[i];
      valid[i] = st == 1;
      all = all && valid[i];
      if (!deferred_ && st < 0) {
        if (st == TMV_SR_ADDERR_PUBKEY)
          deferred_ = std::make_pair((size_t)i, std::string("sr25519: invalid public key: sr25519: failed to "
                                                            "decompress public key"));
        else
          deferred_ = std::make_pair((size_t)i, sig_err_[i].empty()
                                                    ? std::string("sr25519: unable to decode signature")
                                                    : sig_err_[i]);
      }
    }
    return {all, valid};
  }

  std::optional<std::pair<size_t, std::string>> DeferredAddError() const override { return deferred_; }
  bool MayDeferAddErrors() const override { return kind_ == tmh::KeyType::Sr25519; }

  size_t size() const { return sig_err_.size(); }
  int infra_error() const { return infra_error_; }

 private:
  void push(const uint8_t *pk, const tmh::Bytes &msg, const uint8_t *sig, const std::string &sig_err) {
    pk_.insert(pk_.end(), pk, pk + 32);
    sig_.insert(sig_.end(), sig, sig + 64);
    msg_.insert(msg_.end(), msg.begin(), msg.end());
    off_.push_back((uint32_t)msg_.size());
    sig_err_.push_back(sig_err);
  }

  tmv_ctx *ctx_;
  tmh::KeyType kind_;
  std::vector<uint8_t> pk_, sig_, msg_;
  std::vector<uint32_t> off_;
  std::vector<std::string> sig_err_;
  std::optional<std::pair<size_t, std::string>> deferred_;
  int infra_error_ = 0;
};

tmh::KeyType to_kind(uint8_t k) {
  return k == TMV_KIND_ED25519 ? tmh::KeyType::Ed25519 : k == TMV_KIND_SR25519 ? tmh::KeyType::Sr25519
                                                                             : tmh::KeyType::Other;
}

tmh::Bytes bytes_of(const uint8_t *p, size_t n) { return p && n ? tmh::Bytes(p, p + n) : tmh::Bytes(); }

tmh::BlockID block_id_of(const tmv_block_id &b) {
  tmh::BlockID r;
  r.hash = bytes_of(b.hash, b.hash_len);
  r.part_set_header.total = b.psh_total;
  r.part_set_header.hash = bytes_of(b.psh_hash, b.psh_hash_len);
  return r;
}

}  // namespace

struct tmv_batch {
  std::unique_ptr<GpuBatch> impl;
};

extern "C" {

tmv_batch *tmv_batch_new(tmv_ctx *ctx, uint8_t key_kind) {
  if (!ctx) return nullptr;
  const tmh::KeyType k = to_kind(key_kind);
  if (k == tmh::KeyType::Other) return nullptr;  // crypto/batch/batch.go:21
  auto b = new tmv_batch;
  b->impl = std::make_unique<GpuBatch>(ctx, k);
  return b;
}

int tmv_batch_add(tmv_batch *b, uint8_t key_kind, const uint8_t *pk, size_t pk_len, const uint8_t *msg,
                  size_t msg_len, const uint8_t *sig, size_t sig_len, char *err, size_t err_cap) {
  if (!b) return TMV_ERR_ARG;
  tmh::PubKey key{to_kind(key_kind), bytes_of(pk, pk_len)};
  tmh::Error e = b->impl->Add(key, bytes_of(msg, msg_len), bytes_of(sig, sig_len));
  if (e) {
    put_err(err, err_cap, *e);
    return 1;
  }
  return 0;
}

size_t tmv_batch_len(const tmv_batch *b) { return b ? b->impl->size() : 0; }

int tmv_batch_verify(tmv_batch *b, uint8_t *valid_out, int64_t *add_err_index, char *err, size_t err_cap) {
  if (!b) return TMV_ERR_ARG;
  auto [ok, valid] = b->impl->Verify();
  if (b->impl->infra_error() < 0) {
    put_err(err, err_cap, tmv_last_error());
    return b->impl->infra_error();
  }
  for (size_t i = 0; i < valid.size(); i++)
    if (valid_out) valid_out[i] = valid[i] ? 1 : 0;
  if (auto d = b->impl->DeferredAddError()) {
    if (add_err_index) *add_err_index = (int64_t)d->first;
    put_err(err, err_cap, d->second);
    return 2;
  }
  return ok ? 1 : 0;
}

void tmv_batch_free(tmv_batch *b) { delete b; }

size_t tmv_vote_sign_bytes(const char *chain_id, int32_t vote_type, int64_t height, int32_t round,
                           const tmv_block_id *block_id, int64_t ts_seconds, int32_t ts_nanos, uint8_t *out,
                           size_t cap) {
  tmh::BlockID bid;
  if (block_id) bid = block_id_of(*block_id);
  tmh::Timestamp ts{ts_seconds, ts_nanos};
  tmh::Bytes sb = tmh::VoteSignBytes(chain_id ? chain_id : "", vote_type, height, round, block_id ? &bid : nullptr, ts);
  if (out) std::memcpy(out, sb.data(), std::min(cap, sb.size()));
  return sb.size();
}

int tmv_verify_commit(tmv_ctx *ctx, int mode, const char *chain_id, const tmv_validator *vals, uint32_t n_vals,
                      int32_t proposer_index, const tmv_block_id *block_id, int64_t height, const tmv_commit *commit,
                      int64_t trust_num, int64_t trust_den, char *err, size_t err_cap) {
  if (!ctx) {
    put_err(err, err_cap, "null context");
    return TMV_ERR_ARG;
  }
  std::unique_ptr<tmh::ValidatorSet> vs;
  if (vals) {
    vs = std::make_unique<tmh::ValidatorSet>();
    vs->validators.resize(n_vals);
    for (uint32_t i = 0; i < n_vals; i++) {
      tmh::Validator &v = vs->validators[i];
      v.address = bytes_of(vals[i].address, vals[i].address_len);
      v.pub_key = tmh::PubKey{to_kind(vals[i].key_kind), bytes_of(vals[i].pub_key, vals[i].pub_key_len)};
      v.voting_power = vals[i].voting_power;
      v.proposer_priority = vals[i].proposer_priority;
    }
    vs->proposer = proposer_index;
  }
  std::unique_ptr<tmh::Commit> cm;
  if (commit) {
    cm = std::make_unique<tmh::Commit>();
    cm->height = commit->height;
    cm->round = commit->round;
    cm->block_id = block_id_of(commit->block_id);
    cm->signatures.resize(commit->n_sigs);
    for (uint32_t i = 0; i < commit->n_sigs; i++) {
      const tmv_commit_sig &s = commit->sigs[i];
      tmh::CommitSig &c = cm->signatures[i];
      c.block_id_flag = (tmh::BlockIDFlag)s.block_id_flag;
      c.validator_address = bytes_of(s.validator_address, s.validator_address_len);
      c.timestamp = tmh::Timestamp{s.ts_seconds, s.ts_nanos};
      c.signature = bytes_of(s.signature, s.signature_len);
    }
  }
  int infra = 0;
  tmh::CommitVerifier cv;
  std::vector<GpuBatch *> made;
  cv.make_batch = [&](tmh::KeyType k) -> std::unique_ptr<tmh::BatchVerifier> {
    auto b = std::make_unique<GpuBatch>(ctx, k);
    made.push_back(b.get());
    return b;
  };
  cv.verify_single = [&](const tmh::PubKey &pk, const tmh::Bytes &msg, const tmh::Bytes &sig) -> bool {
    // PubKey.VerifySignature (crypto/ed25519/ed25519.go:173-180; crypto/sr25519/pubkey.go:49-62)
    if (pk.type == tmh::KeyType::Ed25519) {
      if (pk.bytes.size() != 32) return false;
      int r = tmv_ed25519_verify(ctx, pk.bytes.data(), msg.data(), msg.size(), sig.data(), sig.size());
      if (r < 0) { infra = r; return false; }
      return r == 1;
    }
    if (pk.type == tmh::KeyType::Sr25519) {
      if (pk.bytes.size() != 32 || sig.size() != 64) return false;
      uint32_t off[2] = {0, (uint32_t)msg.size()};
      int8_t st = 0;
      static const uint8_t z = 0;
      int r = tmv_sr25519_verify_batch(ctx, pk.bytes.data(), sig.data(), msg.empty() ? &z : msg.data(), off, 1, &st);
      if (r < 0) { infra = r; return false; }
      return st == 1;
    }
    return false;  // key types without a GPU verifier are out of scope
  };
  tmh::BlockID bid = block_id ? block_id_of(*block_id) : tmh::BlockID{};
  const std::string cid = chain_id ? chain_id : "";
  tmh::Error e;
  switch (mode) {
    case TMV_COMMIT_FULL: e = cv.VerifyCommit(cid, vs.get(), bid, height, cm.get()); break;
    case TMV_COMMIT_LIGHT: e = cv.VerifyCommitLight(cid, vs.get(), bid, height, cm.get()); break;
    case TMV_COMMIT_LIGHT_TRUSTING: e = cv.VerifyCommitLightTrusting(cid, vs.get(), cm.get(), trust_num, trust_den); break;
    default: put_err(err, err_cap, "unknown mode"); return TMV_ERR_ARG;
  }
  for (GpuBatch *b : made)
    if (b->infra_error() < 0) infra = b->infra_error();
  if (infra < 0) {
    put_err(err, err_cap, tmv_last_error());
    return infra;
  }
  if (e) {
    put_err(err, err_cap, *e);
    return 1;
  }
  put_err(err, err_cap, "");
  return 0;
}

}  // extern "C"
