// CPU test harness for the commit-verification control flow
// (tendermint_amd/csrc/host/tm_types.h) with a test-double signature scheme,
// like the reference's mocks: "signature" = SHA-512(pk || 0^32 || msg).
// sr25519 test keys starting with 0xFF fail to decode (status -1) and
// sr25519 signatures without the schnorrkel marker are rejected (-2).
#include <cstring>
#include <memory>
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

int8_t fake_status(const SigEntry &e) {
  if (e.kind == KeyType::Sr25519) {
    if (!e.pk->empty() && (*e.pk)[0] == 0xFF) return -1;
    if (e.sig.size() != 64 || !(e.sig[63] & 0x80)) return -2;
    Bytes want = fake_sig(*e.pk, e.msg);
    want[63] |= 0x80;
    return want == e.sig ? 1 : 0;
  }
  if (e.sig.size() != 64) return 0;
  return fake_sig(*e.pk, e.msg) == e.sig ? 1 : 0;
}

Bytes b(const uint8_t *p, size_t n) { return p && n ? Bytes(p, p + n) : Bytes(); }
KeyType kind(uint8_t k) { return k == 0 ? KeyType::Ed25519 : k == 1 ? KeyType::Sr25519 : KeyType::Other; }

std::unique_ptr<ValidatorSet> vals_of(const tmv_validator *vals, uint32_t n, int32_t prop) {
  if (!vals) return nullptr;
  auto vs = std::make_unique<ValidatorSet>();
  for (uint32_t i = 0; i < n; i++)
    vs->validators.push_back(Validator{b(vals[i].address, vals[i].address_len),
                                       PubKey{kind(vals[i].key_kind), b(vals[i].pub_key, vals[i].pub_key_len)},
                                       vals[i].voting_power, vals[i].proposer_priority});
  vs->proposer = prop;
  return vs;
}

BlockID bid_of(const tmv_block_id &x) {
  BlockID r;
  r.hash = b(x.hash, x.hash_len);
  r.part_set_header.total = x.psh_total;
  r.part_set_header.hash = b(x.psh_hash, x.psh_hash_len);
  return r;
}

std::unique_ptr<Commit> commit_of(const tmv_commit *commit) {
  if (!commit) return nullptr;
  auto cm = std::make_unique<Commit>();
  cm->height = commit->height;
  cm->round = commit->round;
  cm->block_id = bid_of(commit->block_id);
  for (uint32_t i = 0; i < commit->n_sigs; i++) {
    const tmv_commit_sig &s = commit->sigs[i];
    cm->signatures.push_back(CommitSig{(BlockIDFlag)s.block_id_flag, b(s.validator_address, s.validator_address_len),
                                       Timestamp{s.ts_seconds, s.ts_nanos}, b(s.signature, s.signature_len)});
  }
  return cm;
}

}  // namespace

extern "C" {
int commitcheck_backend_calls = 0;
int commitcheck_entries_verified = 0;

// Same contract as tmv_verify_commits (include/tmhost.h), fake signatures.
int commitcheck_verify_commits(const tmv_commit_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                               size_t err_stride) {
  std::vector<std::unique_ptr<ValidatorSet>> vs;
  std::vector<std::unique_ptr<Commit>> cs;
  std::vector<CommitPlan> plans;
  for (uint32_t j = 0; j < n_jobs; j++) {
    const tmv_commit_job &jb = jobs[j];
    vs.push_back(vals_of(jb.vals, jb.n_vals, jb.proposer_index));
    cs.push_back(commit_of(jb.commit));
    const BlockID bid = jb.block_id ? bid_of(*jb.block_id) : BlockID{};
    plans.push_back(CommitVerifier::Plan((CommitVerifier::Mode)jb.mode, jb.chain_id ? jb.chain_id : "", vs.back().get(),
                                         bid, jb.height, cs.back().get(), jb.trust_num, jb.trust_den));
  }
  CommitVerifier cv;
  cv.backend = [](const std::vector<SigEntry> &es) {
    commitcheck_backend_calls++;
    commitcheck_entries_verified += (int)es.size();
    std::vector<int8_t> st(es.size());
    for (size_t i = 0; i < es.size(); i++) st[i] = fake_status(es[i]);
    return st;
  };
  std::vector<Error> out = cv.VerifyMany(plans);
  int bad = 0;
  for (uint32_t j = 0; j < n_jobs; j++) {
    if (results) results[j] = out[j] ? 1 : 0;
    const std::string s = out[j] ? *out[j] : std::string();
    char *dst = errs + (size_t)j * err_stride;
    std::strncpy(dst, s.c_str(), err_stride - 1);
    dst[err_stride - 1] = 0;
    bad += out[j] ? 1 : 0;
  }
  return bad;
}

int commitcheck_verify_commit(int mode, const char *chain_id, const tmv_validator *vals, uint32_t n_vals,
                              int32_t proposer_index, const tmv_block_id *block_id, int64_t height,
                              const tmv_commit *commit, int64_t trust_num, int64_t trust_den, char *err,
                              size_t err_cap) {
  tmv_commit_job jb{mode, chain_id, vals, n_vals, proposer_index, block_id, height, commit, trust_num, trust_den};
  int32_t r = 0;
  commitcheck_verify_commits(&jb, 1, &r, err, err_cap);
  return r;
}

size_t commitcheck_canonical_time(int64_t secs, int32_t nanos, char *out, size_t cap) {
  std::string s = CanonicalTime(Timestamp{secs, nanos});
  std::strncpy(out, s.c_str(), cap - 1);
  out[cap - 1] = 0;
  return s.size();
}
}
