// CPU test harness for the commit-verification and light-client control flow
// (tendermint_amd/csrc/host/tm_types.h, tm_light.h) with a test-double
// signature scheme, like the reference's mocks: "signature" =
// SHA-512(pk || 0^32 || msg).  sr25519 test keys starting with 0xFF fail to
// decode (status -1) and sr25519 signatures without the schnorrkel marker are
// rejected (-2).  commitcheck_set_real_signatures(1) switches the double to
// the C oracle (oracle/c, linked as liboracle.so: test infrastructure) so the
// reference's own signed fixtures (light/mbt) run through the product's host
// code on the CPU.
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <atomic>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tmhost.h"
#include "../../include/tmverify.h"
#include "../../tendermint_amd/csrc/host/tm_light.h"
#include "../../tendermint_amd/csrc/host/shard_plan.h"
#include "../../tendermint_amd/csrc/host/stream_plan.h"
#include "../../tendermint_amd/csrc/host/shard_run.h"
#include "../../tendermint_amd/csrc/host/wait.h"
#include "../../tendermint_amd/csrc/host/tm_types.h"
#include "../../tendermint_amd/csrc/sha512_dev.h"

extern "C" {
int oracle_ed25519_verify(const uint8_t *pk, const uint8_t *msg, size_t mlen, const uint8_t *sig);
int oracle_sr25519_add_check(const uint8_t *pk, const uint8_t *sig);
int oracle_sr25519_verify(const uint8_t *pk, const uint8_t *msg, size_t mlen, const uint8_t *sig);
}

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

int g_real = 0;  // commitcheck_set_real_signatures

int8_t fake_status(KeyType kind, const Bytes &pk, const Bytes &msg, const Bytes &sig) {
  if (g_real) {
    if (kind == KeyType::Sr25519) {
      const int a = oracle_sr25519_add_check(pk.data(), sig.data());  // 0 ok, -1 key, -2 signature
      if (a < 0) return (int8_t)a;
      return (int8_t)oracle_sr25519_verify(pk.data(), msg.data(), msg.size(), sig.data());
    }
    return (int8_t)oracle_ed25519_verify(pk.data(), msg.data(), msg.size(), sig.data());
  }
  if (kind == KeyType::Sr25519) {
    if (!pk.empty() && pk[0] == 0xFF) return -1;
    if (sig.size() != 64 || !(sig[63] & 0x80)) return -2;
    Bytes want = fake_sig(pk, msg);
    want[63] |= 0x80;
    return want == sig ? 1 : 0;
  }
  if (sig.size() != 64) return 0;
  return fake_sig(pk, msg) == sig ? 1 : 0;
}

}  // namespace

// The host layer under test is the product's own tm_host_abi.cpp, linked
// into this library; only the device entry points it calls
// (include/tmverify.h) are replaced by the test double below.
struct tmv_ctx {
  int unused;
};

extern "C" {
std::atomic<int> commitcheck_backend_calls{0};  // read as a plain int through ctypes (same layout)
std::atomic<int> commitcheck_entries_verified{0};
int g_skip_hash = 0;  // timing of the host layer alone (tools only)
// the next device call returns this infrastructure error (e.g.
// TMV_ERR_TIMEOUT), on whichever thread makes it, and leaves a message
// naming that thread as its last error
std::atomic<int> g_fail_next{0};

void commitcheck_fail_next(int rc) { g_fail_next.store(rc); }

// tmh::poll_until (host/wait.h, the runtime's bounded device waits) against a
// query that completes after `ready_after` polls (< 0: never) or fails.
int commitcheck_poll(int ready_after, int fail, int64_t timeout_ms, double *elapsed_ms) {
  int polls = 0;
  const auto t0 = std::chrono::steady_clock::now();
  const tmh::Poll r = tmh::poll_until([&] {
    polls++;
    if (fail) return 2;
    return ready_after >= 0 && polls > ready_after ? 0 : 1;
  }, timeout_ms);
  *elapsed_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return (int)r;
}

static thread_local std::string g_fake_error;
const char *tmv_last_error(void) { return g_fake_error.empty() ? "fake device error" : g_fake_error.c_str(); }
void tmv_internal_set_error(const char *msg) { g_fake_error = msg ? msg : ""; }
static int take_failure() {
  const int rc = g_fail_next.exchange(0);
  if (rc) {
    char buf[96];
    snprintf(buf, sizeof(buf), "fake infrastructure error on thread %zx",
             std::hash<std::thread::id>()(std::this_thread::get_id()));
    g_fake_error = buf;
  }
  return rc;
}

// Simulated devices: a context of g_devices devices runs every batch through
// the runtime's shard plan and launch / harvest order (host/shard_plan.h,
// host/shard_run.h) -- a launch computes its chunk into the lane's buffer
// (device memory), a harvest copies it to the caller's vector (the D2H) --
// and logs each step, so a multi-device context's placement is checked on
// the CPU.
static uint32_t g_devices = 1, g_chunk = 262144, g_lanes = 2;
static std::vector<uint32_t> g_steps;  // (kind 0 launch / 1 harvest, device, lane, lo, hi) per step
// sliced host-layer calls (TMV_HOST_SLICE) reach the double from two threads
// at once: the step log is appended under this lock (it was not, and the
// concurrent appends corrupted the heap under CPU load)
static std::mutex g_steps_mu;

void commitcheck_set_devices(uint32_t devices, uint32_t host_chunk, uint32_t lanes) {
  g_devices = devices ? devices : 1;
  g_chunk = host_chunk;
  g_lanes = lanes ? lanes : 1;
  std::lock_guard<std::mutex> lk(g_steps_mu);
  g_steps.clear();
}

// Copies up to cap steps (5 words each) and clears the log; returns the count.
uint32_t commitcheck_steps(uint32_t *out, uint32_t cap) {
  std::lock_guard<std::mutex> lk(g_steps_mu);
  const uint32_t n = (uint32_t)(g_steps.size() / 5);
  for (uint32_t i = 0; i < std::min(n, cap) * 5; i++) out[i] = g_steps[i];
  g_steps.clear();
  return n;
}
}

template <class F>
static void run_devices(uint32_t n, int8_t *status_out, F status_of) {
  const tmh::ShardPlan plan = tmh::plan_shards(n, g_devices, g_chunk);
  struct Lane {
    uint32_t lo = 0, n = 0;
    std::vector<int8_t> buf;
  };
  std::vector<std::vector<Lane>> lanes(plan.shards, std::vector<Lane>(g_lanes));
  tmh::run_shard_plan(
      plan, g_lanes,
      [&](uint32_t s, uint32_t l, bool ok) -> int {
        Lane &ln = lanes[s][l];
        if (!ln.n) return 0;
        if (ok) std::memcpy(status_out + ln.lo, ln.buf.data(), ln.n);
        {
          std::lock_guard<std::mutex> lk(g_steps_mu);
          g_steps.insert(g_steps.end(), {1u, s, l, ln.lo, ln.lo + ln.n});
        }
        ln.n = 0;
        return 0;
      },
      [&](uint32_t s, uint32_t l, uint32_t lo, uint32_t hi) -> int {
        Lane &ln = lanes[s][l];
        ln.buf.resize(hi - lo);
        for (uint32_t i = lo; i < hi; i++) ln.buf[i - lo] = status_of(i);
        ln.lo = lo;
        ln.n = hi - lo;
        {
          std::lock_guard<std::mutex> lk(g_steps_mu);
          g_steps.insert(g_steps.end(), {0u, s, l, lo, hi});
        }
        return 0;
      });
}

extern "C" {

int tmv_verify_batch_ex(tmv_ctx *, uint8_t key_kind, uint32_t, const uint8_t *pk, const uint8_t *sig,
                        const uint8_t *msg, const uint32_t *msg_off, uint32_t n, int8_t *status_out) {
  if (const int rc = take_failure()) return rc;
  commitcheck_backend_calls++;
  commitcheck_entries_verified += (int)n;
  run_devices(n, status_out, [&](uint32_t i) -> int8_t {
    const Bytes key(pk + 32 * i, pk + 32 * i + 32);
    return g_skip_hash ? 1
                       : fake_status(key_kind == TMV_KIND_SR25519 ? KeyType::Sr25519 : KeyType::Ed25519, key,
                                     Bytes(msg + msg_off[i], msg + msg_off[i + 1]), Bytes(sig + 64 * i, sig + 64 * i + 64));
  });
  bool all = n > 0;
  for (uint32_t i = 0; i < n; i++) all = all && status_out[i] == 1;
  return all ? TMV_ALL_VALID : TMV_NOT_ALL;
}

// The message the device builds for a vote (include/tmverify.h,
// tmv_verify_votes), assembled here independently of the product's encoder
// so that the CPU suite checks the template split against the reference's
// sign-bytes (tests compare with oracle-encoded messages).
static void put_uvarint(Bytes &out, uint64_t x) {
  while (x >= 0x80) { out.push_back((uint8_t)(x | 0x80)); x >>= 7; }
  out.push_back((uint8_t)x);
}
static Bytes vote_message(const tmv_vote_template &t, const tmv_vote &v) {
  Bytes ts;
  if (v.ts_seconds != 0) { ts.push_back(0x08); put_uvarint(ts, (uint64_t)v.ts_seconds); }
  if (v.ts_nanos != 0) { ts.push_back(0x10); put_uvarint(ts, (uint64_t)(int64_t)v.ts_nanos); }
  Bytes body(t.head, t.head + t.head_len);
  if (v.tmpl & TMV_VOTE_WITH_BLOCK) body.insert(body.end(), t.block, t.block + t.block_len);
  body.push_back(0x2a);
  put_uvarint(body, ts.size());
  body.insert(body.end(), ts.begin(), ts.end());
  body.insert(body.end(), t.chain, t.chain + t.chain_len);
  Bytes msg;
  put_uvarint(msg, body.size());
  msg.insert(msg.end(), body.begin(), body.end());
  return msg;
}

int tmv_verify_votes(tmv_ctx *, uint8_t key_kind, uint32_t, const tmv_vote_template *tmpl, uint32_t n_tmpl,
                     const tmv_vote *votes, const uint8_t *pk, const uint8_t *sig, uint32_t n, int8_t *status_out) {
  if (const int rc = take_failure()) return rc;
  commitcheck_backend_calls++;
  commitcheck_entries_verified += (int)n;
  for (uint32_t i = 0; i < n; i++)
    if ((votes[i].tmpl & ~TMV_VOTE_WITH_BLOCK) >= n_tmpl) return TMV_ERR_ARG;
  run_devices(n, status_out, [&](uint32_t i) -> int8_t {
    const uint32_t t = votes[i].tmpl & ~TMV_VOTE_WITH_BLOCK;
    const Bytes key(pk + 32 * i, pk + 32 * i + 32);
    return g_skip_hash ? 1
                       : fake_status(key_kind == TMV_KIND_SR25519 ? KeyType::Sr25519 : KeyType::Ed25519, key,
                                     vote_message(tmpl[t], votes[i]), Bytes(sig + 64 * i, sig + 64 * i + 64));
  });
  bool all = n > 0;
  for (uint32_t i = 0; i < n; i++) all = all && status_out[i] == 1;
  return all ? TMV_ALL_VALID : TMV_NOT_ALL;
}

// Device hashing entry points (include/tmverify.h) on the host: the light
// layer sends large windows to them.
int tmv_merkle_roots(tmv_ctx *, const uint8_t *data, const uint32_t *leaf_off, uint32_t n_leaves,
                     const uint32_t *tree_off, uint32_t n_trees, uint8_t *hash_out) {
  commitcheck_backend_calls++;
  if (tree_off[n_trees] != n_leaves) return TMV_ERR_ARG;
  for (uint32_t t = 0; t < n_trees; t++)
    MerkleRootHost(data, leaf_off + tree_off[t], tree_off[t + 1] - tree_off[t], hash_out + 32 * t);
  return 0;
}

int tmv_validator_set_hashes(tmv_ctx *, const uint8_t *pk, const uint8_t *key_kind, const int64_t *power,
                             const uint32_t *set_off, uint32_t n_sets, uint8_t *hash_out) {
  commitcheck_backend_calls++;
  for (uint32_t s = 0; s < n_sets; s++) {
    ValidatorSet vs;
    for (uint32_t i = set_off[s]; i < set_off[s + 1]; i++) {
      Validator v;
      v.pub_key = PubKey{key_kind[i] == TMV_KIND_SR25519 ? KeyType::Sr25519 : KeyType::Ed25519,
                         ByteView(pk + 32 * i, 32)};
      v.voting_power = power[i];
      vs.validators.push_back(v);
    }
    const Bytes h = ValidatorSetHashHost(vs);
    std::memcpy(hash_out + 32 * s, h.data(), 32);
  }
  return 0;
}

static tmv_ctx g_ctx;

void commitcheck_set_real_signatures(int on) { g_real = on; }

tmv_ctx *commitcheck_ctx(void) { return &g_ctx; }

int commitcheck_verify_vote_batch(tmv_ctx *, const char *chain_id, const tmv_vote_in *votes, uint32_t n,
                                  int32_t *results) {
  return tmv_verify_vote_batch(&g_ctx, chain_id, votes, n, results);
}

int commitcheck_light_verify_many(const tmv_light_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                                  size_t err_stride) {
  return tmv_light_verify_many(&g_ctx, jobs, n_jobs, results, errs, err_stride);
}

int commitcheck_header_hashes(const tmv_header *headers, uint32_t n, uint8_t *hash_out, uint8_t *has_hash) {
  return tmv_header_hashes(&g_ctx, headers, n, hash_out, has_hash);
}

size_t commitcheck_go_format(int what, int64_t a, int32_t b, char *out, size_t cap) {
  std::string s = what == 0 ? GoTime(Timestamp{a, b}) : what == 1 ? GoDuration(a) : GoQuote(std::string(out));
  std::strncpy(out, s.c_str(), cap - 1);
  out[cap - 1] = 0;
  return s.size();
}

// Same contract as tmv_verify_commits (include/tmhost.h), fake signatures.
int commitcheck_verify_commits(const tmv_commit_job *jobs, uint32_t n_jobs, int32_t *results, char *errs,
                               size_t err_stride) {
  return tmv_verify_commits(&g_ctx, jobs, n_jobs, results, errs, err_stride);
}

int commitcheck_verify_commit(int mode, const char *chain_id, const tmv_validator *vals, uint32_t n_vals,
                              int32_t proposer_index, const tmv_block_id *block_id, int64_t height,
                              const tmv_commit *commit, int64_t trust_num, int64_t trust_den, char *err,
                              size_t err_cap) {
  return tmv_verify_commit(&g_ctx, mode, chain_id, vals, n_vals, proposer_index, block_id, height, commit, trust_num,
                           trust_den, err, err_cap);
}

size_t commitcheck_canonical_time(int64_t secs, int32_t nanos, char *out, size_t cap) {
  std::string s = CanonicalTime(Timestamp{secs, nanos});
  std::strncpy(out, s.c_str(), cap - 1);
  out[cap - 1] = 0;
  return s.size();
}
}

// The runtime's shard / chunk plan of a host-buffer batch (host/shard_plan.h,
// used by run_batch), in launch order: (device, lo, hi, chunk k) per chunk.
// Returns the number of chunks written (or needed, if cap is short).
extern "C" uint32_t commitcheck_shard_plan(uint32_t n, uint32_t ndev, uint32_t host_chunk, uint32_t *out,
                                           uint32_t cap) {
  const tmh::ShardPlan p = tmh::plan_shards(n, ndev, host_chunk);
  uint32_t w = 0;
  for (uint32_t k = 0; k < p.max_chunks; k++)
    for (uint32_t s = 0; s < p.shards; s++) {
      if (k >= p.nchunks[s]) continue;
      if (w < cap) {
        out[4 * w] = s;
        out[4 * w + 1] = p.chunk_lo(s, k);
        out[4 * w + 2] = p.chunk_lo(s, k + 1);
        out[4 * w + 3] = k;
      }
      w++;
    }
  return w;
}

// The runtime's streamed part schedules (host/stream_plan.h): boundaries of
// a one-kind launch (group-aligned) or of a mixed chunk (kind = 1).
// Returns the number of boundaries written (or needed, if cap is short).
extern "C" uint32_t commitcheck_stream_parts(uint32_t n, uint32_t m, uint32_t first, uint32_t part, int ramp, int mixed,
                                             uint32_t max_parts, uint32_t *out, uint32_t cap) {
  const std::vector<uint32_t> b = mixed ? tmh::mixed_part_bounds(n, first, part, ramp != 0, max_parts)
                                        : tmh::stream_part_bounds(n, m, first, part, ramp != 0);
  for (size_t i = 0; i < b.size() && i < cap; i++) out[i] = b[i];
  return (uint32_t)b.size();
}

// The runtime's caller-page locking over one span split into parts
// (host/stream_plan.h, stage_and_launch's feed): span [base, base + len) in
// parts of the given lengths, page size `page`, the lock attempt number
// `fail_at` (0-based, < 0: none) failing.  Per part: [d0, d1, cut]; then the
// locked ranges [r0, r1) in order.  Returns the number of locked ranges
// (out: 3 x parts words, then 2 x ranges words, at most 8 ranges).
extern "C" uint32_t commitcheck_pin_walk(uint64_t base, const uint64_t *part_len, uint32_t parts, uint64_t page,
                                         int fail_at, uint64_t min_len, uint64_t *out) {
  tmh::SpanPins r;
  uint64_t end = base;
  for (uint32_t i = 0; i < parts; i++) end += part_len[i];
  uint64_t s0 = base;
  uint32_t ranges = 0;
  int attempts = 0;
  for (uint32_t i = 0; i < parts; i++) {
    const uint64_t s1 = s0 + part_len[i];
    size_t d0 = 0, d1 = 0, cut = 0;
    if (!r.failed && part_len[i] >= min_len) {
      uintptr_t r0, r1;
      bool ok = true;
      if (tmh::next_pin_range(r, s0, s1, end, page, &r0, &r1)) {
        if (attempts++ == fail_at) {
          r.failed = true;
          ok = false;
        } else {
          tmh::commit_pin_range(r, r0, r1);
          out[3ull * parts + 2 * ranges] = r0;
          out[3ull * parts + 2 * ranges + 1] = r1;
          ranges++;
        }
      }
      if (ok) tmh::direct_piece(r, s0, s1, &d0, &d1, &cut);
    }
    out[3 * i] = d0;
    out[3 * i + 1] = d1;
    out[3 * i + 2] = cut;
    s0 = s1;
  }
  return ranges;
}
