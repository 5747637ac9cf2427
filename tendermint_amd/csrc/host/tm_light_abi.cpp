// C-ABI of the light-client verification (include/tmhost.h: tmv_light_verify,
// tmv_light_verify_many, tmv_header_hashes) over tm_light.h.  A window of
// light-client checks (a sequential or skipping light client's prefetched
// headers) is verified in one pass: the header hashes of all jobs in one
// tmv_merkle_roots launch, the supplied validator sets' hashes in one
// tmv_validator_set_hashes launch, and every commit check of every job in one
// signature batch (tmv_verify_commits).  Each job's result equals its own
// light.Verify / VerifyAdjacent / VerifyNonAdjacent (light/verifier.go:33-177).
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <system_error>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../../include/tmhost.h"
#include "../../../include/tmverify.h"
#include "tm_host_internal.h"
#include "tm_light.h"

using namespace tmh_internal;

namespace {

tmh::ByteView bytes_of(const tmv_bytes &b) { return tmh::ByteView(b.p, b.len); }

std::unique_ptr<tmh::Header> header_of(const tmv_header &h) {
  auto o = std::make_unique<tmh::Header>();
  o->version_block = h.version_block;
  o->version_app = h.version_app;
  o->chain_id = h.chain_id ? h.chain_id : "";
  o->height = h.height;
  o->time = tmh::Timestamp{h.time_seconds, h.time_nanos};
  o->last_block_id = block_id_of(h.last_block_id);
  o->last_commit_hash = bytes_of(h.last_commit_hash);
  o->data_hash = bytes_of(h.data_hash);
  o->validators_hash = bytes_of(h.validators_hash);
  o->next_validators_hash = bytes_of(h.next_validators_hash);
  o->consensus_hash = bytes_of(h.consensus_hash);
  o->app_hash = bytes_of(h.app_hash);
  o->last_results_hash = bytes_of(h.last_results_hash);
  o->evidence_hash = bytes_of(h.evidence_hash);
  o->proposer_address = bytes_of(h.proposer_address);
  return o;
}

// Below this many hashes per call the host computes them (no launch on the
// latency path, e.g. one light.Verify); TMV_DEVICE_HASH_MIN overrides.
uint32_t device_hash_min() {
  static const uint32_t v = [] {
    const char *e = std::getenv("TMV_DEVICE_HASH_MIN");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 32u;
  }();
  return v;
}

// Header.Hash of each header (empty = nil).  Device: one tmv_merkle_roots
// launch over the 14 leaves of every header that has a ValidatorsHash.
int header_hashes(tmv_ctx *ctx, const std::vector<const tmh::Header *> &hs, std::vector<tmh::Bytes> &out) {
  out.assign(hs.size(), tmh::Bytes());
  std::vector<uint32_t> live;
  for (uint32_t i = 0; i < hs.size(); i++)
    if (hs[i] && !hs[i]->validators_hash.empty()) live.push_back(i);
  if (live.size() < device_hash_min()) {
    parallel_for(live.size(), 16, [&](size_t k) { out[live[k]] = tmh::HeaderHashHost(*hs[live[k]]); });
    return 0;
  }
  tmh::Bytes blob;
  std::vector<uint32_t> leaf_off{0}, tree_off{0};
  blob.reserve(live.size() * 400);
  leaf_off.reserve(live.size() * tmh::kHeaderLeaves + 1);
  for (uint32_t i : live) {
    tmh::AppendHeaderLeaves(*hs[i], blob, leaf_off);
    tree_off.push_back((uint32_t)(leaf_off.size() - 1));
  }
  std::vector<uint8_t> roots(32 * live.size());
  const int rc = tmv_merkle_roots(ctx, blob.empty() ? nullptr : blob.data(), leaf_off.data(),
                                  (uint32_t)(leaf_off.size() - 1), tree_off.data(), (uint32_t)live.size(),
                                  roots.data());
  if (rc < 0) return rc;
  for (size_t k = 0; k < live.size(); k++) out[live[k]].assign(roots.begin() + 32 * k, roots.begin() + 32 * k + 32);
  return 0;
}

// ValidatorSet.Hash of each set.  Device: one tmv_validator_set_hashes launch
// over the sets whose keys are all ed25519 / sr25519; the rest on the host.
int valset_hashes(tmv_ctx *ctx, const std::vector<const tmh::ValidatorSet *> &vs,
                  const std::vector<const tmv_validator_set *> &src, std::vector<tmh::Bytes> &out) {
  out.assign(vs.size(), tmh::Bytes());
  std::vector<uint32_t> dev, host;
  for (uint32_t i = 0; i < vs.size(); i++) {
    if (!vs[i]) continue;
    bool ok = true;
    for (const tmh::Validator &v : vs[i]->validators)
      ok = ok && v.pub_key.type != tmh::KeyType::Other && v.pub_key.bytes.size() == 32;
    (ok ? dev : host).push_back(i);
  }
  if (dev.size() < device_hash_min()) {
    host.insert(host.end(), dev.begin(), dev.end());
    dev.clear();
  }
  parallel_for(host.size(), 4, [&](size_t k) { out[host[k]] = tmh::ValidatorSetHashHost(*vs[host[k]]); });
  if (dev.empty()) return 0;
  // pack the sets' keys, kinds and powers (offsets first, then the sets in
  // parallel: a light window holds ~10^5 validators)
  std::vector<uint32_t> off(dev.size() + 1, 0);
  for (size_t k = 0; k < dev.size(); k++) off[k + 1] = off[k] + src[dev[k]]->n_vals;
  const size_t total = off.back();
  std::vector<uint8_t> pk(32 * total), kind(total);
  std::vector<int64_t> power(total);
  parallel_for(dev.size(), 16, [&](size_t k) {
    const tmv_validator_set &s = *src[dev[k]];
    for (uint32_t v = 0; v < s.n_vals; v++) {
      std::memcpy(pk.data() + 32ull * (off[k] + v), s.vals[v].pub_key, 32);
      kind[off[k] + v] = s.vals[v].key_kind;
      power[off[k] + v] = s.vals[v].voting_power;
    }
  });
  std::vector<uint8_t> roots(32 * dev.size());
  const int rc = tmv_validator_set_hashes(ctx, pk.empty() ? nullptr : pk.data(), kind.empty() ? nullptr : kind.data(),
                                          power.empty() ? nullptr : power.data(), off.data(), (uint32_t)dev.size(),
                                          roots.data());
  if (rc < 0) return rc;
  for (size_t k = 0; k < dev.size(); k++) out[dev[k]].assign(roots.begin() + 32 * k, roots.begin() + 32 * k + 32);
  return 0;
}

template <class T>
struct Interner {  // distinct C pointers -> dense indices
  std::unordered_map<const T *, uint32_t> idx;
  std::vector<const T *> src;
  uint32_t operator()(const T *p) {
    if (!p) return UINT32_MAX;
    auto [it, fresh] = idx.emplace(p, (uint32_t)src.size());
    if (fresh) src.push_back(p);
    return it->second;
  }
};

int light_verify_slice(tmv_ctx *ctx, const tmv_light_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                       size_t err_stride);

}  // namespace

extern "C" {

int tmv_header_hashes(tmv_ctx *ctx, const tmv_header *headers, uint32_t n, uint8_t *hash_out, uint8_t *has_hash) {
  if (!ctx || (n && (!headers || !hash_out))) return TMV_ERR_ARG;
  std::vector<std::unique_ptr<tmh::Header>> hs(n);
  parallel_for(n, 64, [&](size_t i) { hs[i] = header_of(headers[i]); });
  std::vector<const tmh::Header *> ptrs(n);
  for (uint32_t i = 0; i < n; i++) ptrs[i] = hs[i].get();
  std::vector<tmh::Bytes> out;
  const int rc = header_hashes(ctx, ptrs, out);
  if (rc < 0) return rc;
  for (uint32_t i = 0; i < n; i++) {
    if (has_hash) has_hash[i] = out[i].empty() ? 0 : 1;
    if (out[i].empty()) std::memset(hash_out + 32 * i, 0, 32);
    else std::memcpy(hash_out + 32 * i, out[i].data(), 32);
  }
  return 0;
}

int tmv_light_verify_many(tmv_ctx *ctx, const tmv_light_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                          size_t err_stride) {
  if (!ctx || (!jobs && n_jobs)) return TMV_ERR_ARG;
  for (uint32_t j = 0; j < n_jobs; j++)
    if (jobs[j].mode < TMV_LIGHT_VERIFY || jobs[j].mode > TMV_LIGHT_NON_ADJACENT) return TMV_ERR_ARG;
  struct Call {
    tmv_ctx *ctx;
    const tmv_light_job *jobs;
    int32_t *results;
    char *errs;
    size_t stride;
  } c{ctx, jobs, results, errs, err_stride};
  uint32_t fail_lo = 0;
  const int rc = run_sliced(n_jobs, [](void *p, uint32_t lo, uint32_t hi) {
    const Call &c = *static_cast<const Call *>(p);
    return light_verify_slice(c.ctx, c.jobs + lo, hi - lo, c.results ? c.results + lo : nullptr,
                              c.errs && c.stride ? c.errs + (size_t)lo * c.stride : nullptr, c.stride);
  }, &c, &fail_lo);
  // an infrastructure error's text goes to errs[0] (after every slice ended)
  if (rc < 0 && fail_lo && errs && err_stride) std::memcpy(errs, errs + (size_t)fail_lo * err_stride, err_stride);
  return rc;
}

}  // extern "C"

namespace {

// One pass of the light checks over jobs (tmv_light_verify_many's slices).
int light_verify_slice(tmv_ctx *ctx, const tmv_light_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                       size_t err_stride) {
  PhaseTimer tm("tmv_light_verify_many");
  const PhaseEnd tm_end{tm, "release"};
  // distinct headers, commits and validator sets, converted once
  Interner<tmv_header> H;
  Interner<tmv_commit> C;
  Interner<tmv_validator_set> V;
  struct Ref {
    uint32_t th, tc, uh, uc, tv, uv;
  };
  std::vector<Ref> refs(n_jobs);
  for (uint32_t j = 0; j < n_jobs; j++) {
    const tmv_light_job &jb = jobs[j];
    Ref &r = refs[j];
    r.th = jb.trusted ? H(jb.trusted->header) : UINT32_MAX;
    r.tc = jb.trusted ? C(jb.trusted->commit) : UINT32_MAX;
    r.uh = jb.untrusted ? H(jb.untrusted->header) : UINT32_MAX;
    r.uc = jb.untrusted ? C(jb.untrusted->commit) : UINT32_MAX;
    r.tv = V(jb.trusted_vals);
    r.uv = V(jb.untrusted_vals);
  }
  std::vector<std::unique_ptr<tmh::Header>> headers(H.src.size());
  std::vector<std::unique_ptr<tmh::Commit>> commits(C.src.size());
  std::vector<std::unique_ptr<tmh::ValidatorSet>> vsets(V.src.size());
  const size_t nh = headers.size(), nc = commits.size();
  parallel_for(nh + nc + vsets.size(), 16, [&](size_t i) {
    if (i < nh) headers[i] = header_of(*H.src[i]);
    else if (i < nh + nc) commits[i - nh] = commit_of(C.src[i - nh]);
    else vsets[i - nh - nc] = vals_of(V.src[i - nh - nc]->vals, V.src[i - nh - nc]->n_vals,
                                      V.src[i - nh - nc]->proposer_index);
  });
  tm.mark("convert");
  // hashes the checks may need: Header.Hash of untrusted headers,
  // ValidatorSet.Hash of untrusted validator sets
  std::vector<uint8_t> need_h(nh, 0), need_v(vsets.size(), 0);
  for (const Ref &r : refs) {
    if (r.uh != UINT32_MAX) need_h[r.uh] = 1;
    if (r.uv != UINT32_MAX) need_v[r.uv] = 1;
  }
  std::vector<const tmh::Header *> hq(nh, nullptr);
  for (size_t i = 0; i < nh; i++)
    if (need_h[i]) hq[i] = headers[i].get();
  std::vector<const tmh::ValidatorSet *> vq(vsets.size(), nullptr);
  for (size_t i = 0; i < vsets.size(); i++)
    if (need_v[i]) vq[i] = vsets[i].get();
  // The hashes run beside the signature checks: Header.Hash and
  // ValidatorSet.Hash only decide two comparisons in PlanLight (the commit's
  // BlockID hash, the header's ValidatorsHash), so every job is first planned
  // as if both matched -- the hashes the header claims -- and its commit
  // checks are verified while a helper thread hashes; a job whose real hashes
  // differ ends in PlanLight's early error (ahead of any commit check in the
  // reference's order) and its speculative commit results are dropped.  A job
  // whose hashes match has exactly the speculative plan.
  std::vector<tmh::Bytes> hh, vh;
  int hrc = 0;
  std::string hash_error;
  auto hash_job = [&] {
    hrc = header_hashes(ctx, hq, hh);
    if (hrc >= 0) hrc = valset_hashes(ctx, vq, V.src, vh);
    if (hrc < 0) hash_error = tmv_last_error();
  };
  std::thread hasher;
  try {
    hasher = std::thread(hash_job);
  } catch (const std::system_error &) {
    hash_job();  // no thread to be had: hash first, inline (the results are the same)
  }
  struct Join {
    std::thread &t;
    ~Join() { if (t.joinable()) t.join(); }
  } join_hasher{hasher};
  static const tmh::Bytes kNone;
  auto light_job = [&](uint32_t j) {
    const tmv_light_job &jb = jobs[j];
    const Ref &r = refs[j];
    tmh::LightJob lj;
    lj.mode = (tmh::LightMode)jb.mode;
    lj.trusted = tmh::SignedHeader{r.th == UINT32_MAX ? nullptr : headers[r.th].get(),
                                   r.tc == UINT32_MAX ? nullptr : commits[r.tc].get()};
    lj.untrusted = tmh::SignedHeader{r.uh == UINT32_MAX ? nullptr : headers[r.uh].get(),
                                     r.uc == UINT32_MAX ? nullptr : commits[r.uc].get()};
    lj.trusted_vals = r.tv == UINT32_MAX ? nullptr : vsets[r.tv].get();
    lj.untrusted_vals = r.uv == UINT32_MAX ? nullptr : vsets[r.uv].get();
    lj.trusting_period_ns = jb.trusting_period_ns;
    lj.now = tmh::Timestamp{jb.now_seconds, jb.now_nanos};
    lj.max_clock_drift_ns = jb.max_clock_drift_ns;
    lj.trust_num = jb.trust_num;
    lj.trust_den = jb.trust_den;
    return lj;
  };
  // speculative plans: the hashes the untrusted header and commit claim
  std::vector<tmh::LightPlan> plans(n_jobs);
  parallel_for(n_jobs, 16, [&](size_t j) {
    const tmh::LightJob lj = light_job((uint32_t)j);
    tmh::Bytes claim_h, claim_v;
    if (lj.untrusted.commit) claim_h.assign(lj.untrusted.commit->block_id.hash.begin(),
                                            lj.untrusted.commit->block_id.hash.end());
    if (lj.untrusted.header) claim_v.assign(lj.untrusted.header->validators_hash.begin(),
                                            lj.untrusted.header->validators_hash.end());
    plans[j] = tmh::PlanLight(lj, claim_h, claim_v);
  });
  tm.mark("plan");
  // the commit checks of every job, one signature batch
  std::vector<tmv_commit_job> cj;
  std::vector<uint32_t> cfirst(n_jobs + 1, 0);
  for (uint32_t j = 0; j < n_jobs; j++) {
    const tmv_light_job &jb = jobs[j];
    for (const tmh::LightCommitCheck &ck : plans[j].checks) {
      const tmv_validator_set *vs = ck.mode == tmh::CommitVerifier::kLightTrusting ? jb.trusted_vals : jb.untrusted_vals;
      const tmv_commit *commit = jb.untrusted->commit;
      cj.push_back(tmv_commit_job{(int)ck.mode, jb.trusted->header->chain_id ? jb.trusted->header->chain_id : "",
                                  vs ? vs->vals : nullptr, vs ? vs->n_vals : 0, vs ? vs->proposer_index : -1,
                                  &commit->block_id, ck.height, commit, ck.trust_num, ck.trust_den});
      if (!vs) cj.back().vals = nullptr;
    }
    cfirst[j + 1] = (uint32_t)cj.size();
  }
  constexpr size_t kStride = 1024;
  std::vector<int32_t> cres(cj.size());
  std::vector<uint8_t> cne(cj.size());
  std::vector<char> cerr(cj.size() * kStride);
  if (!cj.empty()) {
    // the sets and commits converted above are the ones the checks read
    Converted conv;
    conv.vals.reserve(vsets.size());
    for (size_t i = 0; i < vsets.size(); i++)
      if (vsets[i]) conv.vals.emplace(V.src[i]->vals, vsets[i].get());
    conv.commits.reserve(commits.size());
    for (size_t i = 0; i < commits.size(); i++)
      if (commits[i]) conv.commits.emplace(C.src[i], commits[i].get());
    const int rc = verify_commits(ctx, cj.data(), (uint32_t)cj.size(), cres.data(), cerr.data(), kStride, cne.data(),
                                  &conv);
    if (rc < 0) {
      if (errs && err_stride) put_err(errs, err_stride, std::string(cerr.data()));
      return rc;
    }
  }
  tm.mark("commits");
  hasher.join();
  tm.mark("hashes joined");
  if (hrc < 0) {
    tmv_internal_set_error(hash_error.c_str());
    if (errs && err_stride) put_err(errs, err_stride, hash_error);
    return hrc;
  }
  // the real plans; a job whose hashes differ from the claimed ones now
  // carries its early error (and none of the speculative checks)
  parallel_for(n_jobs, 16, [&](size_t j) {
    const Ref &r = refs[j];
    const tmh::LightPlan real = tmh::PlanLight(light_job((uint32_t)j), r.uh == UINT32_MAX ? kNone : hh[r.uh],
                                               r.uv == UINT32_MAX ? kNone : vh[r.uv]);
    if (real.early) plans[j].early = real.early;
  });
  int bad = 0;
  for (uint32_t j = 0; j < n_jobs; j++) {
    const size_t k = plans[j].checks.size();
    std::vector<tmh::Error> e(k);
    std::unique_ptr<bool[]> ne(new bool[k + 1]);
    for (size_t i = 0; i < k; i++) {
      const uint32_t c = cfirst[j] + (uint32_t)i;
      if (cres[c]) e[i] = std::string(&cerr[c * kStride]);
      ne[i] = cne[c] != 0;
    }
    const tmh::LightResult lr = tmh::FinishLight(plans[j], e.data(), ne.get());
    if (results) results[j] = lr.kind;
    if (errs && err_stride) put_err(errs + (size_t)j * err_stride, err_stride, lr.text);
    bad += lr.kind != tmh::kLightOk;
  }
  tm.mark("finish");
  // many small heap objects (validators, signatures, plans): to the reaper
  // thread (pool.h), or freed here in parallel when it is backlogged
  using Bundle = tmh::GarbageOf<decltype(headers), decltype(commits), decltype(vsets), decltype(plans)>;
  std::unique_ptr<tmh::Garbage> g(new Bundle(std::move(headers), std::move(commits), std::move(vsets),
                                             std::move(plans)));
  if (!tmh::reap(g)) {
    auto &[gh, gc, gv, gp] = static_cast<Bundle &>(*g).items;
    const size_t nrel = std::max({gh.size(), gc.size(), gv.size(), gp.size()});
    parallel_for(nrel, 16, [&](size_t i) {
      if (i < gh.size()) gh[i].reset();
      if (i < gc.size()) gc[i].reset();
      if (i < gv.size()) gv[i].reset();
      if (i < gp.size()) gp[i] = tmh::LightPlan();
    });
  }
  return bad;
}

}  // namespace

extern "C" {

int tmv_light_verify(tmv_ctx *ctx, const tmv_light_job *job, char *err, size_t err_cap) {
  if (!job) return TMV_ERR_ARG;
  int32_t res = 0;
  const int rc = tmv_light_verify_many(ctx, job, 1, &res, err, err_cap);
  return rc < 0 ? rc : res;
}

}  // extern "C"
