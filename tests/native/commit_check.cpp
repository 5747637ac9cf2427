// CPU test harness for the commit-verification control flow
// (tendermint_amd/csrc/host/tm_types.h) with a test-double signature scheme,
// like the reference's mocks: "signature" = SHA-512(pk || 0^32 || msg).
// sr25519 test keys starting with 0xFF fail to decode (deferred Add error),
// sr25519 signatures without the schnorrkel marker bit are rejected at Add.
// Exposes the same entry point shape as tmv_verify_commit minus the context.
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tmhost.h"
#include "../../tendermint_amd/csrc/host/tm_types.h"
#include "../../tendermint_amd/csrc/sha512_dev.h"

namespace {

using namespace tmh;

Bytes fake_sig(const Bytes &pk, const Bytes &msg) {
  uint32_t P[8] = {0}, Q[8] = {0}, h[16];
  for (size_t i = 0; i < 32 && i < pk.size(); i++) P[i / 4] |= (uint32_t)pk[i] << (8 * (i % 4));
  tmv::sha512_pq_msg(h, P, Q, msg.data(), (uint32_t)msg.size());
  Bytes s(64);
  for (int i = 0; i < 64; i++) s[i] = (uint8_t)(h[i / 4] >> (8 * (i % 4)));
  return s;
}

bool fake_valid(const PubKey &pk, const Bytes &msg, const Bytes &sig) {
  if (sig.size() != 64) return false;
  Bytes want = fake_sig(pk.bytes, msg);
  if (pk.type == KeyType::Sr25519) {
    if (!(sig[63] & 0x80)) return false;
    want[63] |= 0x80;
  }
  return want == sig;
}

class FakeBatch : public BatchVerifier {
 public:
  explicit FakeBatch(KeyType k) : kind_(k) {}
  Error Add(const PubKey &key, const Bytes &msg, const Bytes &sig) override {
    if (kind_ == KeyType::Ed25519) {
      if (key.type != KeyType::Ed25519) return std::string("pubkey is not Ed25519");
      if (key.bytes.size() != 32) return "pubkey size is incorrect; expected: 32, got " + std::to_string(key.bytes.size());
      if (sig.size() != 64) return std::string("invalid signature");
    } else {
      if (key.type != KeyType::Sr25519) return std::string("sr25519: pubkey is not sr25519");
    }
    e_.push_back({key, msg, sig});
    return std::nullopt;
  }
  std::pair<bool, std::vector<bool>> Verify() override {
    std::vector<bool> v(e_.size());
    bool all = !e_.empty();
    deferred_.reset();
    for (size_t i = 0; i < e_.size(); i++) {
      const auto &x = e_[i];
      if (kind_ == KeyType::Sr25519 && !deferred_) {
        if (!x.key.bytes.empty() && x.key.bytes[0] == 0xFF)
          deferred_ = std::make_pair(i, std::string("sr25519: invalid public key: test"));
        else if (x.sig.size() != 64 || !(x.sig[63] & 0x80))
          deferred_ = std::make_pair(i, std::string("sr25519: unable to decode signature: test"));
      }
      v[i] = fake_valid(x.key, x.msg, x.sig);
      all = all && v[i];
    }
    return {all, v};
  }
  std::optional<std::pair<size_t, std::string>> DeferredAddError() const override { return deferred_; }
  bool MayDeferAddErrors() const override { return kind_ == KeyType::Sr25519; }

 private:
  struct E { PubKey key; Bytes msg, sig; };
  KeyType kind_;
  std::vector<E> e_;
  std::optional<std::pair<size_t, std::string>> deferred_;
};

Bytes b(const uint8_t *p, size_t n) { return p && n ? Bytes(p, p + n) : Bytes(); }

KeyType kind(uint8_t k) { return k == 0 ? KeyType::Ed25519 : k == 1 ? KeyType::Sr25519 : KeyType::Other; }

}  // namespace

extern "C" {
int commitcheck_batches_made = 0;
int commitcheck_singles_made = 0;
}

extern "C" int commitcheck_verify_commit(int mode, const char *chain_id, const tmv_validator *vals, uint32_t n_vals,
                                         int32_t proposer_index, const tmv_block_id *block_id, int64_t height,
                                         const tmv_commit *commit, int64_t trust_num, int64_t trust_den, char *err,
                                         size_t err_cap) {
  std::unique_ptr<ValidatorSet> vs;
  if (vals) {
    vs = std::make_unique<ValidatorSet>();
    for (uint32_t i = 0; i < n_vals; i++)
      vs->validators.push_back(Validator{b(vals[i].address, vals[i].address_len),
                                         PubKey{kind(vals[i].key_kind), b(vals[i].pub_key, vals[i].pub_key_len)},
                                         vals[i].voting_power, vals[i].proposer_priority});
    vs->proposer = proposer_index;
  }
  auto bid_of = [](const tmv_block_id &x) {
    BlockID r;
    r.hash = b(x.hash, x.hash_len);
    r.part_set_header.total = x.psh_total;
    r.part_set_header.hash = b(x.psh_hash, x.psh_hash_len);
    return r;
  };
  std::unique_ptr<Commit> cm;
  if (commit) {
    cm = std::make_unique<Commit>();
    cm->height = commit->height;
    cm->round = commit->round;
    cm->block_id = bid_of(commit->block_id);
    for (uint32_t i = 0; i < commit->n_sigs; i++) {
      const tmv_commit_sig &s = commit->sigs[i];
      cm->signatures.push_back(CommitSig{(BlockIDFlag)s.block_id_flag, b(s.validator_address, s.validator_address_len),
                                         Timestamp{s.ts_seconds, s.ts_nanos}, b(s.signature, s.signature_len)});
    }
  }
  CommitVerifier cv;
  cv.make_batch = [](KeyType k) -> std::unique_ptr<BatchVerifier> {
    commitcheck_batches_made++;
    return std::make_unique<FakeBatch>(k);
  };
  cv.verify_single = [](const PubKey &pk, const Bytes &msg, const Bytes &sig) {
    commitcheck_singles_made++;
    return fake_valid(pk, msg, sig);
  };
  BlockID bid = block_id ? bid_of(*block_id) : BlockID{};
  Error e;
  if (mode == 0) e = cv.VerifyCommit(chain_id, vs.get(), bid, height, cm.get());
  else if (mode == 1) e = cv.VerifyCommitLight(chain_id, vs.get(), bid, height, cm.get());
  else e = cv.VerifyCommitLightTrusting(chain_id, vs.get(), cm.get(), trust_num, trust_den);
  const std::string s = e ? *e : std::string();
  std::strncpy(err, s.c_str(), err_cap - 1);
  err[err_cap - 1] = 0;
  return e ? 1 : 0;
}

extern "C" size_t commitcheck_canonical_time(int64_t secs, int32_t nanos, char *out, size_t cap) {
  std::string s = CanonicalTime(Timestamp{secs, nanos});
  std::strncpy(out, s.c_str(), cap - 1);
  out[cap - 1] = 0;
  return s.size();
}
