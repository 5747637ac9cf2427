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

// Packed entries + GPU verify.
class GpuBatch : public tmh::BatchVerifier {
 public:
  GpuBatch(tmv_ctx *ctx, tmh::KeyType kind) : ctx_(ctx), kind_(kind) { off_.push_back(0); }

  tmh::Error Add(const tmh::PubKey &key, const tmh::Bytes &msg, const tmh::Bytes &sig) override {
    tmh::AddCheck ac = tmh::CheckAdd(kind_, key, sig);
    if (ac.sync) return ac.sync;
    push(key.bytes.data(), msg, ac.sig64.data(), ac.deferred_sig);
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
          deferred_ = std::make_pair((size_t)i, tmh::DeferredPubKeyError());
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

}  // extern "C"

namespace {

// Signature backend over the device: entries split by key kind, each kind one
// tmv_verify_batch_ex call with the key cache (validator keys repeat);
// identical (commit, index, key) entries — blocksync verifies each commit
// twice, light then full — are verified once.
struct GpuBackend {
  tmv_ctx *ctx;
  int infra = 0;
  std::vector<int8_t> operator()(const std::vector<tmh::SigEntry> &es) {
    std::vector<int8_t> st(es.size(), 0);
    for (int kind = 0; kind < 2; kind++) {
      const tmh::KeyType kt = kind == 0 ? tmh::KeyType::Ed25519 : tmh::KeyType::Sr25519;
      std::vector<uint32_t> idx;
      std::vector<uint8_t> pk, sig, msg;
      std::vector<uint32_t> off{0};
      for (size_t i = 0; i < es.size(); i++) {
        const tmh::SigEntry &e = es[i];
        if (e.kind != kt) continue;
        if (e.pk->size() != 32 || e.sig.size() != 64) continue;  // VerifySignature: false
        idx.push_back((uint32_t)i);
        pk.insert(pk.end(), e.pk->begin(), e.pk->end());
        sig.insert(sig.end(), e.sig.begin(), e.sig.end());
        msg.insert(msg.end(), e.msg.begin(), e.msg.end());
        off.push_back((uint32_t)msg.size());
      }
      if (idx.empty()) continue;
      std::vector<int8_t> out(idx.size());
      static const uint8_t z = 0;
      const int rc = tmv_verify_batch_ex(ctx, kind == 0 ? TMV_KIND_ED25519 : TMV_KIND_SR25519, TMV_FLAG_KEY_CACHE,
                                         pk.data(), sig.data(), msg.empty() ? &z : msg.data(), off.data(),
                                         (uint32_t)idx.size(), out.data());
      if (rc < 0) { infra = rc; continue; }
      for (size_t t = 0; t < idx.size(); t++) st[idx[t]] = out[t];
    }
    return st;
  }
};

struct OwnedCommitArgs {
  std::unique_ptr<tmh::ValidatorSet> vals;
  tmh::Commit *commit = nullptr;
  tmh::BlockID block_id;
};

std::unique_ptr<tmh::ValidatorSet> vals_of(const tmv_validator *vals, uint32_t n_vals, int32_t proposer_index) {
  if (!vals) return nullptr;
  auto vs = std::make_unique<tmh::ValidatorSet>();
  vs->validators.resize(n_vals);
  for (uint32_t i = 0; i < n_vals; i++) {
    tmh::Validator &v = vs->validators[i];
    v.address = bytes_of(vals[i].address, vals[i].address_len);
    v.pub_key = tmh::PubKey{to_kind(vals[i].key_kind), bytes_of(vals[i].pub_key, vals[i].pub_key_len)};
    v.voting_power = vals[i].voting_power;
    v.proposer_priority = vals[i].proposer_priority;
  }
  vs->proposer = proposer_index;
  return vs;
}

std::unique_ptr<tmh::Commit> commit_of(const tmv_commit *commit) {
  if (!commit) return nullptr;
  auto cm = std::make_unique<tmh::Commit>();
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
  return cm;
}

}  // namespace

extern "C" {

int tmv_verify_commits(tmv_ctx *ctx, const tmv_commit_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                       size_t err_stride) {
  if (!ctx || (!jobs && n_jobs)) return TMV_ERR_ARG;
  // Convert once per distinct validator set / commit pointer (a commit
  // checked twice, as blocksync does, shares its entries).
  std::unordered_map<const void *, std::unique_ptr<tmh::ValidatorSet>> vmap;
  std::unordered_map<const void *, std::unique_ptr<tmh::Commit>> cmap;
  std::vector<tmh::CommitPlan> plans(n_jobs);
  for (uint32_t j = 0; j < n_jobs; j++) {
    const tmv_commit_job &jb = jobs[j];
    tmh::ValidatorSet *vs = nullptr;
    if (jb.vals) {
      auto &slot = vmap[jb.vals];
      if (!slot) slot = vals_of(jb.vals, jb.n_vals, jb.proposer_index);
      vs = slot.get();
    }
    tmh::Commit *cm = nullptr;
    if (jb.commit) {
      auto &slot = cmap[jb.commit];
      if (!slot) slot = commit_of(jb.commit);
      cm = slot.get();
    }
    const tmh::BlockID bid = jb.block_id ? block_id_of(*jb.block_id) : tmh::BlockID{};
    if (jb.mode < 0 || jb.mode > 2) return TMV_ERR_ARG;
    plans[j] = tmh::CommitVerifier::Plan((tmh::CommitVerifier::Mode)jb.mode, jb.chain_id ? jb.chain_id : "", vs, bid,
                                         jb.height, cm, jb.trust_num, jb.trust_den);
  }
  // dedupe identical entries across plans (same commit object, index, key)
  std::vector<tmh::SigEntry> uniq;
  std::vector<std::vector<uint32_t>> where(n_jobs);
  std::unordered_map<std::string, uint32_t> seen;
  for (uint32_t j = 0; j < n_jobs; j++) {
    const tmh::CommitPlan &pl = plans[j];
    if (pl.early) continue;
    where[j].resize(pl.entries.size());
    for (size_t e = 0; e < pl.entries.size(); e++) {
      std::string key(reinterpret_cast<const char *>(&pl.commit), sizeof(void *));
      const int si = pl.sig_idx[e];
      const void *pkp = pl.entries[e].pk;
      key.append(reinterpret_cast<const char *>(&si), sizeof si);
      key.append(reinterpret_cast<const char *>(&pkp), sizeof pkp);
      key.push_back(pl.batch ? 'b' : 's');
      auto it = seen.find(key);
      if (it != seen.end() && uniq[it->second].msg == pl.entries[e].msg) {
        where[j][e] = it->second;
      } else {
        where[j][e] = (uint32_t)uniq.size();
        seen[key] = (uint32_t)uniq.size();
        uniq.push_back(pl.entries[e]);
      }
    }
  }
  GpuBackend be{ctx};
  std::vector<int8_t> st = uniq.empty() ? std::vector<int8_t>() : be(uniq);
  if (be.infra < 0) {
    if (errs && err_stride) put_err(errs, err_stride, tmv_last_error());
    return be.infra;
  }
  int bad = 0;
  std::vector<int8_t> buf;
  for (uint32_t j = 0; j < n_jobs; j++) {
    buf.resize(where[j].size());
    for (size_t e = 0; e < where[j].size(); e++) buf[e] = st[where[j][e]];
    tmh::Error e = tmh::CommitVerifier::Finish(plans[j], buf.data());
    if (results) results[j] = e ? 1 : 0;
    if (errs && err_stride) put_err(errs + (size_t)j * err_stride, err_stride, e ? *e : std::string());
    bad += e ? 1 : 0;
  }
  return bad;
}

int tmv_verify_commit(tmv_ctx *ctx, int mode, const char *chain_id, const tmv_validator *vals, uint32_t n_vals,
                      int32_t proposer_index, const tmv_block_id *block_id, int64_t height, const tmv_commit *commit,
                      int64_t trust_num, int64_t trust_den, char *err, size_t err_cap) {
  if (!ctx) {
    put_err(err, err_cap, "null context");
    return TMV_ERR_ARG;
  }
  tmv_commit_job jb{mode, chain_id, vals, n_vals, proposer_index, block_id, height, commit, trust_num, trust_den};
  int32_t res = 0;
  const int rc = tmv_verify_commits(ctx, &jb, 1, &res, err, err_cap);
  if (rc < 0) return rc;
  return res;
}

}  // extern "C"
