// C-ABI of the host layer (include/tmhost.h): crypto.BatchVerifier objects
// backed by the GPU entry points of include/tmverify.h, canonical vote
// sign-bytes, and the commit verifiers of tm_types.h instantiated with them.
// Only the public tmv_* C-ABI is used to reach the device (layering).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <string>
#include <vector>

#include "../../../include/tmhost.h"
#include "../../../include/tmverify.h"
#include "pool.h"
#include "tm_host_internal.h"
#include "tm_light.h"
#include "tm_types.h"

namespace tmh_internal {

// Default 600 jobs: a call of >= 1,200 jobs (a C4 window: 600 blocks, a
// light and a full check each) runs as two slices on two threads, one
// slice's host phases beside the other's engine call.  Round 4, one box:
// C4 one window at a time 122-126k -> 130-139k blocks/s; three slices (500)
// 88-100k (35k-signature key-merged launches are latency-bound).  Round 3
// measured slicing slower, before calls on one device could overlap (lane
// claims) and before the deferred release.  Read on every call (tests
// change it).
uint32_t host_slice_jobs() {
  const char *e = std::getenv("TMV_HOST_SLICE");
  return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 600u;
}

namespace {
// The partner thread of run_sliced: runs one posted task at a time.
class Partner {
 public:
  Partner() { std::thread([this] { loop(); }).detach(); }
  void post(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu_);
    task_ = std::move(f);
    busy_ = true;
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return !busy_; });
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return (bool)task_; });
      std::function<void()> f = std::move(task_);
      task_ = nullptr;
      lk.unlock();
      f();
      lk.lock();
      busy_ = false;
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::function<void()> task_;
  bool busy_ = false;
};
}  // namespace

int run_sliced(uint32_t n_jobs, int (*run_slice)(void *, uint32_t, uint32_t), void *ctx, uint32_t *fail_lo) {
  const uint32_t target = host_slice_jobs();
  if (fail_lo) *fail_lo = 0;
  if (!target || n_jobs < 2 * target) return run_slice(ctx, 0, n_jobs);
  // one partner per process: concurrent sliced calls queue for it (the
  // second caller runs its slices alone)
  // never destroyed: the detached thread waits on its condition variable
  // until exit (destroying it under a waiter blocks at exit)
  static Partner *partner = new Partner;
  static std::mutex *partner_mu = new std::mutex;
  std::unique_lock<std::mutex> own(*partner_mu, std::try_to_lock);
  const uint32_t ns = (n_jobs + target - 1) / target, per = (n_jobs + ns - 1) / ns;
  std::atomic<uint32_t> next{0};
  std::atomic<int> bad{0}, err{0};
  // the first failing slice's message and first job (its thread's last
  // error is thread-local: the caller reads its own after the join)
  std::mutex emu;
  std::string emsg;
  uint32_t elo = 0;
  auto work = [&] {
    for (uint32_t k; (k = next.fetch_add(1)) < ns;) {
      const uint32_t lo = k * per, hi = std::min(n_jobs, lo + per);
      if (lo >= hi) continue;
      const int r = run_slice(ctx, lo, hi);
      if (r < 0) {
        int z = 0;
        if (err.compare_exchange_strong(z, r)) {
          std::lock_guard<std::mutex> lk(emu);
          emsg = tmv_last_error();
          elo = lo;
        }
      } else {
        bad.fetch_add(r);
      }
    }
  };
  if (own.owns_lock()) partner->post(work);
  work();
  if (own.owns_lock()) partner->wait();
  if (err.load()) {
    std::lock_guard<std::mutex> lk(emu);
    tmv_internal_set_error(emsg.c_str());
    if (fail_lo) *fail_lo = elo;
    return err.load();
  }
  return bad.load();
}

void put_err(char *err, size_t cap, const std::string &s) {
  if (!err || cap == 0) return;
  const size_t n = std::min(cap - 1, s.size());
  std::memcpy(err, s.data(), n);
  err[n] = 0;
}

}  // namespace tmh_internal

using namespace tmh_internal;

namespace {

// Packed entries + GPU verify.
class GpuBatch : public tmh::BatchVerifier {
 public:
  GpuBatch(tmv_ctx *ctx, tmh::KeyType kind) : ctx_(ctx), kind_(kind) { off_.push_back(0); }

  tmh::Error Add(const tmh::PubKey &key, const tmh::Bytes &msg, const tmh::Bytes &sig) override {
    tmh::AddCheck ac = tmh::CheckAdd(kind_, key, sig);
    if (ac.sync) return ac.sync;
    push(key.bytes.data(), msg, ac.sig64, ac.deferred_sig);
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

}  // namespace

namespace tmh_internal {

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

}  // namespace tmh_internal

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
  tmh::PubKey key{to_kind(key_kind), tmh::ByteView(pk, pk_len)};
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

size_t tmv_vote_template_encode(const char *chain_id, int32_t vote_type, int64_t height, int32_t round,
                                const tmv_block_id *block_id, uint8_t *out, size_t cap, uint32_t lens[3]) {
  tmh::BlockID bid;
  if (block_id) bid = block_id_of(*block_id);
  const tmh::VoteTemplate t =
      tmh::EncodeVoteTemplate(chain_id ? chain_id : "", vote_type, height, round, block_id ? &bid : nullptr);
  if (lens) {
    lens[0] = t.head_len;
    lens[1] = t.block_len;
    lens[2] = t.chain_len;
  }
  if (out) std::memcpy(out, t.bytes.data(), std::min(cap, t.bytes.size()));
  return t.bytes.size();
}

}  // extern "C"

namespace {

// Signature backend over the device: entries split by key kind, each kind one
// tmv_verify_votes call with the key cache (validator keys repeat).  The
// sign-bytes are built on the device from one template per (commit,
// chain_id) plus 16 bytes per vote; public keys and signatures are packed in
// parallel.
// Packing buffers reused across calls on a thread: fresh multi-megabyte
// vectors would be new mappings, page-faulted in on every call.
struct PackBuffers {
  std::vector<uint8_t> cls;
  std::vector<uint32_t> idx, off;
  std::vector<uint8_t> pk, sig, msg;
  std::vector<tmv_vote> votes;
  std::vector<int8_t> out;
};

// Entry e of plan pl.
struct VoteRef {
  const tmh::CommitPlan *pl;
  uint32_t e;
  const tmh::SigEntry &entry() const { return pl->entries[e]; }
};

// Batches below this size send host-encoded messages (one launch less on
// the latency path, e.g. a single VerifyCommit); larger ones build the
// sign-bytes on the device.  TMV_DEVICE_SIGNBYTES_MIN overrides.
static uint32_t device_signbytes_min() {
  static const uint32_t v = [] {
    const char *e = std::getenv("TMV_DEVICE_SIGNBYTES_MIN");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 4096u;
  }();
  return v;
}

struct GpuBackend {
  tmv_ctx *ctx;
  int infra = 0;
  void operator()(const std::vector<VoteRef> &es, std::vector<int8_t> &st) {
    static thread_local PackBuffers tls;
    PackBuffers &pb = tls;  // the workers below must use this thread's buffers, not their own
    PhaseTimer tm("tmv_verify_commits");
    st.assign(es.size(), 0);
    // one template per (commit object, chain_id): entries come plan by plan,
    // so the plans' runs are found first, each run's template is looked up
    // once (serially: ~10^3 runs), and the entries are filled in parallel
    std::vector<tmh::VoteTemplate> tmpls;
    std::unordered_map<const tmh::CommitPlan *, uint32_t> plan_tmpl;
    std::unordered_map<const tmh::Commit *, std::vector<std::pair<const std::string *, uint32_t>>> by_commit;
    std::vector<uint32_t> ent_tmpl(es.size());
    std::vector<std::pair<size_t, uint32_t>> runs;  // (first entry, template) of each run of one plan
    std::vector<const tmh::CommitPlan *> tmpl_src;  // a plan of each template's (commit, chain_id)
    for (size_t i = 0; i < es.size(); i++) {
      const tmh::CommitPlan *pl = es[i].pl;
      if (i && pl == es[i - 1].pl) continue;
      auto [it, fresh] = plan_tmpl.emplace(pl, 0);
      if (fresh) {
        auto &chains = by_commit[pl->commit];
        uint32_t t = UINT32_MAX;
        for (auto &c : chains)
          if (*c.first == pl->chain_id) t = c.second;
        if (t == UINT32_MAX) {  // encoded below, in parallel
          t = (uint32_t)tmpl_src.size();
          tmpl_src.push_back(pl);
          chains.emplace_back(&pl->chain_id, t);
        }
        it->second = t;
      }
      runs.emplace_back(i, it->second);
    }
    runs.emplace_back(es.size(), 0u);
    tmpls.resize(tmpl_src.size());
    parallel_for(tmpl_src.size(), 16, [&](size_t t) {
      const tmh::CommitPlan *pl = tmpl_src[t];
      const tmh::Commit &cm = *pl->commit;
      tmpls[t] = tmh::EncodeVoteTemplate(pl->chain_id, tmh::kPrecommitType, cm.height, cm.round, &cm.block_id);
    });
    parallel_for(runs.size() - 1, 32, [&](size_t r) {
      std::fill(ent_tmpl.begin() + runs[r].first, ent_tmpl.begin() + runs[r + 1].first, runs[r].second);
    });
    tm.mark("b:tmpl");
    std::vector<tmv_vote_template> tv(tmpls.size());
    for (size_t t = 0; t < tmpls.size(); t++) {
      const tmh::VoteTemplate &vt = tmpls[t];
      const uint8_t *b = vt.bytes.data();
      tv[t] = tmv_vote_template{b, vt.head_len, b + vt.head_len, vt.block_len, b + vt.head_len + vt.block_len,
                                vt.chain_len};
    }
    // verifier kind of every entry (2: not verified -- VerifySignature is
    // false for a wrong key or signature size), classified in parallel
    // chunks, then each kind's index list is filled chunk by chunk
    constexpr size_t kChunk = 4096;
    const size_t nch = (es.size() + kChunk - 1) / kChunk;
    pb.cls.resize(es.size());
    std::vector<uint32_t> ccount(2 * nch + 2, 0);
    parallel_for(nch, 1, [&](size_t c) {
      uint32_t k0 = 0, k1 = 0;
      for (size_t i = c * kChunk; i < std::min(es.size(), c * kChunk + kChunk); i++) {
        const tmh::SigEntry &e = es[i].entry();
        uint8_t k = e.kind == tmh::KeyType::Ed25519 ? 0 : (e.kind == tmh::KeyType::Sr25519 ? 1 : 2);
        if (e.pk.size() != 32 || e.sig_len != 64) k = 2;
        pb.cls[i] = k;
        k0 += k == 0;
        k1 += k == 1;
      }
      ccount[2 * c] = k0;
      ccount[2 * c + 1] = k1;
    });
    uint32_t kind_n[2] = {0, 0};
    for (size_t c = 0; c < nch; c++)
      for (int k = 0; k < 2; k++) {
        const uint32_t v = ccount[2 * c + k];
        ccount[2 * c + k] = kind_n[k];
        kind_n[k] += v;
      }
    pb.idx.resize((size_t)kind_n[0] + kind_n[1]);
    parallel_for(nch, 1, [&](size_t c) {
      uint32_t at[2] = {ccount[2 * c], kind_n[0] + ccount[2 * c + 1]};
      for (size_t i = c * kChunk; i < std::min(es.size(), c * kChunk + kChunk); i++) {
        const uint8_t k = pb.cls[i];
        if (k < 2) pb.idx[at[k]++] = (uint32_t)i;
      }
    });
    tm.mark("b:cls");
    for (int kind = 0; kind < 2; kind++) {
      const uint32_t *kidx = pb.idx.data() + (kind == 0 ? 0 : kind_n[0]);
      const size_t m = kind_n[kind];
      if (m == 0) continue;
      pb.pk.resize(32 * m);
      pb.sig.resize(64 * m);
      pb.votes.resize(m);
      pb.out.resize(m);
      parallel_for((m + 1023) / 1024, 1, [&](size_t c) {
        for (size_t t = c * 1024; t < std::min(m, c * 1024 + 1024); t++) {
          const VoteRef &r = es[kidx[t]];
          const tmh::SigEntry &e = r.entry();
          const tmh::CommitSig &cs = r.pl->commit->signatures[(size_t)r.pl->sig_idx[r.e]];
          std::memcpy(&pb.pk[32 * t], e.pk.data(), 32);
          std::memcpy(&pb.sig[64 * t], e.sig, 64);
          pb.votes[t] = tmv_vote{cs.timestamp.seconds, cs.timestamp.nanos,
                                 ent_tmpl[kidx[t]] |
                                     (cs.block_id_flag == tmh::BlockIDFlagCommit ? TMV_VOTE_WITH_BLOCK : 0u)};
        }
      });
      tm.mark("b:pack");
      int rc;
      if (m >= device_signbytes_min()) {
        rc = tmv_verify_votes(ctx, kind == 0 ? TMV_KIND_ED25519 : TMV_KIND_SR25519, TMV_FLAG_KEY_CACHE, tv.data(),
                              (uint32_t)tv.size(), pb.votes.data(), pb.pk.data(), pb.sig.data(), (uint32_t)m,
                              pb.out.data());
      } else {  // host-encoded messages, same templates
        pb.off.assign(1, 0);
        pb.msg.clear();
        for (size_t t = 0; t < m; t++) {
          const tmv_vote &v = pb.votes[t];
          const tmh::VoteTemplate &vt = tmpls[v.tmpl & ~TMV_VOTE_WITH_BLOCK];
          tmh::AppendVoteFromTemplate(pb.msg, vt, (v.tmpl & TMV_VOTE_WITH_BLOCK) != 0,
                                      tmh::Timestamp{v.ts_seconds, v.ts_nanos});
          pb.off.push_back((uint32_t)pb.msg.size());
        }
        if (pb.msg.empty()) pb.msg.push_back(0);
        rc = tmv_verify_batch_ex(ctx, kind == 0 ? TMV_KIND_ED25519 : TMV_KIND_SR25519, TMV_FLAG_KEY_CACHE,
                                 pb.pk.data(), pb.sig.data(), pb.msg.data(), pb.off.data(), (uint32_t)m,
                                 pb.out.data());
      }
      tm.mark("b:engine");
      if (rc < 0) { infra = rc; continue; }
      parallel_for((m + kChunk - 1) / kChunk, 4, [&](size_t c) {
        for (size_t t = c * kChunk; t < std::min(m, c * kChunk + kChunk); t++) st[kidx[t]] = pb.out[t];
      });
      tm.mark("b:scatter");
    }
  }
};

}  // namespace

namespace tmh_internal {

std::unique_ptr<tmh::ValidatorSet> vals_of(const tmv_validator *vals, uint32_t n_vals, int32_t proposer_index) {
  if (!vals) return nullptr;
  auto vs = std::make_unique<tmh::ValidatorSet>();
  vs->validators.resize(n_vals);
  for (uint32_t i = 0; i < n_vals; i++) {
    tmh::Validator &v = vs->validators[i];
    v.address = tmh::ByteView(vals[i].address, vals[i].address_len);
    v.pub_key = tmh::PubKey{to_kind(vals[i].key_kind), tmh::ByteView(vals[i].pub_key, vals[i].pub_key_len)};
    v.voting_power = vals[i].voting_power;
    v.proposer_priority = vals[i].proposer_priority;
  }
  vs->proposer = proposer_index;
  vs->UpdateTotalVotingPower();
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
    c.validator_address = tmh::ByteView(s.validator_address, s.validator_address_len);
    c.timestamp = tmh::Timestamp{s.ts_seconds, s.ts_nanos};
    c.signature = tmh::ByteView(s.signature, s.signature_len);
  }
  return cm;
}

int verify_commits(tmv_ctx *ctx, const tmv_commit_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                   size_t err_stride, uint8_t *not_enough, const Converted *conv) {
  if (!ctx || (!jobs && n_jobs)) return TMV_ERR_ARG;
  for (uint32_t j = 0; j < n_jobs; j++)
    if (jobs[j].mode < 0 || jobs[j].mode > 2) return TMV_ERR_ARG;
  PhaseTimer tm("tmv_verify_commits");
  const PhaseEnd tm_end{tm, "release"};
  // Convert once per distinct validator set / commit pointer (a commit
  // checked twice, as blocksync does, shares its entries), in parallel.
  std::unordered_map<const void *, size_t> vidx, cidx;
  std::vector<const tmv_commit_job *> vsrc, csrc;
  std::vector<size_t> jv(n_jobs, SIZE_MAX), jc(n_jobs, SIZE_MAX);
  for (uint32_t j = 0; j < n_jobs; j++) {
    if (jobs[j].vals) {
      auto [it, fresh] = vidx.emplace(jobs[j].vals, vsrc.size());
      if (fresh) vsrc.push_back(&jobs[j]);
      jv[j] = it->second;
    }
    if (jobs[j].commit) {
      auto [it, fresh] = cidx.emplace(jobs[j].commit, csrc.size());
      if (fresh) csrc.push_back(&jobs[j]);
      jc[j] = it->second;
    }
  }
  // owned conversions (own_*) and the objects the checks read (vsets /
  // commits: the owned ones or the caller's already converted ones)
  std::vector<std::unique_ptr<tmh::ValidatorSet>> own_v(vsrc.size());
  std::vector<std::unique_ptr<tmh::Commit>> own_c(csrc.size());
  std::vector<const tmh::ValidatorSet *> vsets(vsrc.size(), nullptr);
  std::vector<const tmh::Commit *> commits(csrc.size(), nullptr);
  parallel_for(vsrc.size() + csrc.size(), 4, [&](size_t i) {
    if (i < vsrc.size()) {
      if (conv) {
        auto it = conv->vals.find(vsrc[i]->vals);
        if (it != conv->vals.end() && it->second->Size() == vsrc[i]->n_vals &&
            it->second->proposer == vsrc[i]->proposer_index) {
          vsets[i] = it->second;
          return;
        }
      }
      own_v[i] = vals_of(vsrc[i]->vals, vsrc[i]->n_vals, vsrc[i]->proposer_index);
      vsets[i] = own_v[i].get();
    } else {
      const size_t c = i - vsrc.size();
      if (conv) {
        auto it = conv->commits.find(csrc[c]->commit);
        if (it != conv->commits.end()) { commits[c] = it->second; return; }
      }
      own_c[c] = commit_of(csrc[c]->commit);
      commits[c] = own_c[c].get();
    }
  });
  tm.mark("convert");
  std::vector<tmh::CommitPlan> plans(n_jobs);
  parallel_for(n_jobs, 4, [&](size_t j) {
    const tmv_commit_job &jb = jobs[j];
    const tmh::BlockID bid = jb.block_id ? block_id_of(*jb.block_id) : tmh::BlockID{};
    plans[j] = tmh::CommitVerifier::Plan((tmh::CommitVerifier::Mode)jb.mode, jb.chain_id ? jb.chain_id : "",
                                         jv[j] == SIZE_MAX ? nullptr : vsets[jv[j]], bid, jb.height,
                                         jc[j] == SIZE_MAX ? nullptr : commits[jc[j]], jb.trust_num,
                                         jb.trust_den);
  });
  tm.mark("plan");
  // dedupe identical entries across plans: same commit object and signature
  // index, same public key object, same verifier kind and the same chain_id
  // (hence the same message).  Only jobs over one commit object can share
  // entries, so commits are deduplicated independently, in parallel, into
  // flat arrays: pass 1 gives each entry a commit-local unique index (bit 31
  // marks its first occurrence), pass 2 places the unique entries commit by
  // commit and rebases the indices.
  std::vector<size_t> joff(n_jobs + 1, 0);
  for (uint32_t j = 0; j < n_jobs; j++)
    joff[j + 1] = joff[j] + (plans[j].early ? 0 : plans[j].entries.size());
  std::vector<uint32_t> where(joff[n_jobs]);
  std::vector<std::vector<uint32_t>> by_commit(commits.size());
  std::vector<uint32_t> solo;  // jobs with entries but no commit index (none today; kept general)
  for (uint32_t j = 0; j < n_jobs; j++) {
    if (plans[j].early || plans[j].entries.empty()) continue;
    if (jc[j] != SIZE_MAX) by_commit[jc[j]].push_back(j);
    else solo.push_back(j);
  }
  constexpr uint32_t kFirst = 0x80000000u;
  std::vector<uint32_t> n_new(commits.size() + 1, 0);
  parallel_for(commits.size(), 8, [&](size_t c) {
    const auto &js = by_commit[c];
    if (js.empty()) return;
    static thread_local std::vector<uint32_t> slot[2];  // commit-local index per signature, per kind
    static thread_local std::vector<std::pair<uint32_t, uint32_t>> first;  // (job, entry) of each local index
    uint32_t cnt = 0;
    if (js.size() == 1) {  // nothing to share
      const uint32_t j = js[0];
      for (size_t e = 0; e < plans[j].entries.size(); e++) where[joff[j] + e] = kFirst | cnt++;
      n_new[c] = cnt;
      return;
    }
    bool used[2] = {false, false};
    first.clear();
    for (uint32_t j : js) {
      const tmh::CommitPlan &pl = plans[j];
      const int kind = pl.batch ? 1 : 0;
      std::vector<uint32_t> &sl = slot[kind];
      if (!used[kind]) { sl.assign(pl.commit->signatures.size(), UINT32_MAX); used[kind] = true; }
      for (size_t e = 0; e < pl.entries.size(); e++) {
        const tmh::SigEntry &en = pl.entries[e];
        uint32_t &u = sl[(size_t)pl.sig_idx[e]];
        if (u != UINT32_MAX) {
          const tmh::CommitPlan &fpl = plans[first[u].first];  // first occurrence of u
          if (fpl.entries[first[u].second].pk.data() == en.pk.data() && (&fpl == &pl || fpl.chain_id == pl.chain_id)) {
            where[joff[j] + e] = u;
            continue;
          }
        }
        u = cnt++;
        first.emplace_back(j, (uint32_t)e);
        where[joff[j] + e] = kFirst | u;
      }
    }
    n_new[c] = cnt;
  });
  std::vector<uint32_t> cbase(commits.size() + 1, 0);
  for (size_t c = 0; c < commits.size(); c++) cbase[c + 1] = cbase[c] + n_new[c];
  size_t total = cbase[commits.size()];
  for (uint32_t j : solo) total += plans[j].entries.size();
  std::vector<VoteRef> uniq(total);
  parallel_for(commits.size(), 64, [&](size_t c) {
    for (uint32_t j : by_commit[c])
      for (size_t e = 0; e < plans[j].entries.size(); e++) {
        uint32_t &w = where[joff[j] + e];
        if (w & kFirst) {
          w = cbase[c] + (w & ~kFirst);
          uniq[w] = VoteRef{&plans[j], (uint32_t)e};
        } else {
          w += cbase[c];
        }
      }
  });
  {
    uint32_t u = cbase[commits.size()];
    for (uint32_t j : solo)
      for (size_t e = 0; e < plans[j].entries.size(); e++) {
        where[joff[j] + e] = u;
        uniq[u++] = VoteRef{&plans[j], (uint32_t)e};
      }
  }
  tm.mark("dedup");
  GpuBackend be{ctx};
  std::vector<int8_t> st;
  if (!uniq.empty()) be(uniq, st);
  tm.mark("verify");
  if (be.infra < 0) {
    if (errs && err_stride) put_err(errs, err_stride, tmv_last_error());
    return be.infra;
  }
  std::atomic<int> bad{0};
  parallel_for(n_jobs, 64, [&](size_t j) {
    static thread_local std::vector<int8_t> buf;
    buf.resize(joff[j + 1] - joff[j]);
    for (size_t e = 0; e < buf.size(); e++) buf[e] = st[where[joff[j] + e]];
    bool ne = false;
    tmh::Error e = tmh::CommitVerifier::Finish(plans[j], buf.data(), &ne);
    if (results) results[j] = e ? 1 : 0;
    if (not_enough) not_enough[j] = ne ? 1 : 0;
    if (errs && err_stride) put_err(errs + j * err_stride, err_stride, e ? *e : std::string());
    if (e) bad.fetch_add(1, std::memory_order_relaxed);
  });
  tm.mark("finish");
  // the converted sets, commits and plans are ~10^4 small heap objects per
  // window: handed to the reaper thread (pool.h), or freed here in parallel
  // when it is backlogged (freed on one thread they took ~7 ms of a C3 window)
  {
    std::unique_ptr<tmh::Garbage> g(new tmh::GarbageOf<decltype(own_v), decltype(own_c), decltype(plans)>(
        std::move(own_v), std::move(own_c), std::move(plans)));
    if (!tmh::reap(g)) {
      auto &[gv, gc, gp] = static_cast<tmh::GarbageOf<decltype(own_v), decltype(own_c), decltype(plans)> &>(*g).items;
      parallel_for(std::max(gv.size(), std::max(gc.size(), gp.size())), 16, [&](size_t i) {
        if (i < gv.size()) gv[i].reset();
        if (i < gc.size()) gc[i].reset();
        if (i < gp.size()) gp[i] = tmh::CommitPlan();
      });
    }
  }
  return bad.load();
}

}  // namespace tmh_internal

extern "C" {

int tmv_verify_commits(tmv_ctx *ctx, const tmv_commit_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                       size_t err_stride) {
  if (!ctx || (!jobs && n_jobs)) return TMV_ERR_ARG;
  struct Call {
    tmv_ctx *ctx;
    const tmv_commit_job *jobs;
    int32_t *results;
    char *errs;
    size_t stride;
  } c{ctx, jobs, results, errs, err_stride};
  uint32_t fail_lo = 0;
  const int rc = run_sliced(n_jobs, [](void *p, uint32_t lo, uint32_t hi) {
    const Call &c = *static_cast<const Call *>(p);
    return verify_commits(c.ctx, c.jobs + lo, hi - lo, c.results ? c.results + lo : nullptr,
                          c.errs && c.stride ? c.errs + (size_t)lo * c.stride : nullptr, c.stride, nullptr);
  }, &c, &fail_lo);
  // an infrastructure error's text goes to errs[0] (after every slice ended)
  if (rc < 0 && fail_lo && errs && err_stride) std::memcpy(errs, errs + (size_t)fail_lo * err_stride, err_stride);
  return rc;
}

int tmv_verify_vote_batch(tmv_ctx *ctx, const char *chain_id, const tmv_vote_in *votes, uint32_t n,
                          int32_t *results) {
  if (!ctx || (n && (!votes || !results))) return TMV_ERR_ARG;
  const std::string chain = chain_id ? chain_id : "";
  // address check (pubKey.Address() == vote.ValidatorAddress, crypto.AddressHash
  // = SHA-256(pub key)[:20]), then one batch per key kind over the votes'
  // canonical sign-bytes; VerifySignature semantics: a wrong signature length
  // or an undecodable sr25519 key / signature is an invalid signature.
  std::vector<uint8_t> kind(n, 2);
  parallel_for(n, 256, [&](size_t i) {
    const tmv_vote_in &v = votes[i];
    uint32_t st[8];
    static const uint8_t none = 0;
    tmh::Sha256Bytes(st, nullptr, 0, v.pub_key ? v.pub_key : &none, v.pub_key_len);
    uint8_t addr[20];
    for (int k = 0; k < 20; k++) addr[k] = (uint8_t)(st[k / 4] >> (24 - 8 * (k % 4)));
    const bool addr_ok = v.validator_address_len == 20 && v.validator_address &&
                         std::memcmp(addr, v.validator_address, 20) == 0;
    if (!addr_ok) { results[i] = TMV_VOTE_ERR_INVALID_ADDRESS; return; }
    results[i] = TMV_VOTE_ERR_INVALID_SIGNATURE;
    if (v.pub_key_len != 32 || v.signature_len != 64 || !v.signature) return;
    if (v.key_kind == TMV_KIND_ED25519 || v.key_kind == TMV_KIND_SR25519) kind[i] = v.key_kind;
  });
  for (uint8_t k = 0; k < 2; k++) {
    std::vector<uint32_t> idx;
    for (uint32_t i = 0; i < n; i++)
      if (kind[i] == k) idx.push_back(i);
    if (idx.empty()) continue;
    const size_t m = idx.size();
    std::vector<uint8_t> pk(32 * m), sig(64 * m), msg;
    std::vector<uint32_t> off(m + 1, 0);
    std::vector<tmh::BlockID> bids(m);
    for (size_t t = 0; t < m; t++) {
      const tmv_vote_in &v = votes[idx[t]];
      std::memcpy(&pk[32 * t], v.pub_key, 32);
      std::memcpy(&sig[64 * t], v.signature, 64);
      if (v.block_id) bids[t] = block_id_of(*v.block_id);
      tmh::AppendVoteSignBytes(msg, chain, v.type, v.height, v.round, v.block_id ? &bids[t] : nullptr,
                               tmh::Timestamp{v.ts_seconds, v.ts_nanos});
      off[t + 1] = (uint32_t)msg.size();
    }
    std::vector<int8_t> st(m);
    const int rc = tmv_verify_batch_ex(ctx, k, TMV_FLAG_KEY_CACHE, pk.data(), sig.data(), msg.data(), off.data(),
                                       (uint32_t)m, st.data());
    if (rc < 0) return rc;
    for (size_t t = 0; t < m; t++)
      if (st[t] == 1) results[idx[t]] = TMV_VOTE_OK;
  }
  int bad = 0;
  for (uint32_t i = 0; i < n; i++) bad += results[i] != TMV_VOTE_OK;
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
