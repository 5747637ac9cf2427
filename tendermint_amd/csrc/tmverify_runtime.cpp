// Host runtime behind include/tmverify.h: device discovery, per-device
// base-point tables, pinned staging, streams and the shard-by-index
// multi-GPU split.  Compiled by hipcc into libtmgpu.so.
//
// There is deliberately no CPU fallback in this library: if the device path
// fails the call returns < 0 and the caller decides (the Go shim
// re-verifies on CPU).  Product code never links the test oracle.
#include <hip/hip_runtime.h>
#include <sys/random.h>

#include <cerrno>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <list>
#include <unordered_map>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tmverify.h"
#include "ed25519_core.h"
#include "merlin_dev.h"
#include "host/pool.h"
#include "host/shard_plan.h"
#include "host/stream_plan.h"
#include "host/shard_run.h"
#include "host/wait.h"
#include "knobs.h"
#include "ktimer.h"
#include "verify_kernels.h"
#include "votes.h"
#include "valset.h"

namespace {

thread_local std::string g_last_error;

void set_error(const char *where, hipError_t e) {
  g_last_error = std::string(where) + ": " + hipGetErrorString(e);
}
void set_error(const std::string &s) { g_last_error = s; }

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// Large staging copies into pinned memory use several host threads (one
// thread moves ~10 GB/s; a 1M-signature batch is ~220 MB).
void par_memcpy(void *dst, const void *src, size_t n) {
  const size_t kChunk = size_t(2) << 20;
  if (n < 2 * kChunk) { std::memcpy(dst, src, n); return; }
  const size_t chunks = (n + kChunk - 1) / kChunk;
  tmh::parallel_for_n(chunks, 8, [&](size_t c) {
    const size_t lo = c * kChunk, len = std::min(n, lo + kChunk) - lo;
    std::memcpy(static_cast<char *>(dst) + lo, static_cast<const char *>(src) + lo, len);
  });
}

// Several staging copies at once, cut into pieces spread over the host pool.
struct CopySpan {
  void *dst;
  const void *src;
  size_t n;
};
void par_memcpy_spans(const CopySpan *sp, size_t count) {
  const size_t kPiece = size_t(512) << 10;
  std::vector<std::pair<size_t, size_t>> pieces;  // (span, offset)
  for (size_t i = 0; i < count; i++)
    for (size_t o = 0; o < sp[i].n; o += kPiece) pieces.emplace_back(i, o);
  if (pieces.size() < 4) {
    for (size_t i = 0; i < count; i++) std::memcpy(sp[i].dst, sp[i].src, sp[i].n);
    return;
  }
  tmh::parallel_for_n(pieces.size(), 16, [&](size_t k) {
    const CopySpan &c = sp[pieces[k].first];
    const size_t o = pieces[k].second, len = std::min(c.n, o + kPiece) - o;
    std::memcpy(static_cast<char *>(c.dst) + o, static_cast<const char *>(c.src) + o, len);
  });
}

struct DeviceBuf {
  void *ptr = nullptr;
  size_t cap = 0;
  bool pinned = false;
  void *dev = nullptr;  // pinned buffers: the device's address of the same memory
  hipError_t ensure(size_t bytes, bool host_pinned) {
    if (bytes <= cap) return hipSuccess;
    release();
    size_t want = std::max<size_t>(bytes, 1 << 20);
    want = want + want / 4;
    hipError_t e = host_pinned ? hipHostMalloc(&ptr, want, hipHostMallocDefault) : hipMalloc(&ptr, want);
    if (e != hipSuccess) { ptr = nullptr; cap = 0; return e; }
    cap = want;
    pinned = host_pinned;
    dev = nullptr;
    if (pinned && hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess) dev = nullptr;
    return hipSuccess;
  }
  void release() {
    if (!ptr) return;
    if (pinned) (void)hipHostFree(ptr); else (void)hipFree(ptr);
    ptr = nullptr;
    dev = nullptr;
    cap = 0;
  }
};

// Open-addressing (linear probing, tombstones) index of cached keys.  Keys
// are public keys, i.e. uniformly random bytes, so 8 of them are the hash.
struct KeyIndex {
  struct Ent { std::array<uint8_t, 33> key; uint32_t slot; uint8_t state; };  // 0 empty, 1 full, 2 deleted
  std::vector<Ent> t;
  size_t live = 0, used = 0;
  static uint64_t hash(const uint8_t *k33) {
    uint64_t h;
    std::memcpy(&h, k33 + 1, 8);
    return (h ^ (h >> 29) ^ ((uint64_t)k33[0] << 63)) * 0x9E3779B97F4A7C15ull;
  }
  void init(size_t cap) {
    size_t sz = 16;
    while (sz < 4 * cap) sz <<= 1;
    t.assign(sz, Ent{{}, 0, 0});
    live = used = 0;
  }
  // returns slot or UINT32_MAX
  uint32_t find(const uint8_t *k33) const {
    const size_t mask = t.size() - 1;
    for (size_t i = hash(k33) & mask;; i = (i + 1) & mask) {
      const Ent &e = t[i];
      if (e.state == 0) return UINT32_MAX;
      if (e.state == 1 && std::memcmp(e.key.data(), k33, 33) == 0) return e.slot;
    }
  }
  void insert(const uint8_t *k33, uint32_t slot) {
    if (2 * (used + 1) > t.size()) rehash();
    const size_t mask = t.size() - 1;
    size_t i = hash(k33) & mask;
    while (t[i].state == 1) i = (i + 1) & mask;
    if (t[i].state == 0) used++;
    std::memcpy(t[i].key.data(), k33, 33);
    t[i].slot = slot;
    t[i].state = 1;
    live++;
  }
  void erase(const uint8_t *k33) {
    const size_t mask = t.size() - 1;
    for (size_t i = hash(k33) & mask;; i = (i + 1) & mask) {
      Ent &e = t[i];
      if (e.state == 0) return;
      if (e.state == 1 && std::memcmp(e.key.data(), k33, 33) == 0) { e.state = 2; live--; return; }
    }
  }
  void rehash() {  // drops tombstones; doubles the table when over a quarter full
    std::vector<Ent> old;
    old.swap(t);
    t.assign(4 * live >= old.size() ? 2 * old.size() : old.size(), Ent{{}, 0, 0});
    live = used = 0;
    for (const Ent &e : old)
      if (e.state == 1) insert(e.key.data(), e.slot);
  }
  size_t size() const { return live; }
};

// Scratch of one launch stream: prep outputs (Ed25519Work), mixed-batch
// partition, and the event that orders reuse of these buffers.
struct Workspace {
  DeviceBuf work, work2, idx, msm, msm2, gather;
  hipEvent_t done = nullptr;
  // mixed batch-equation launches: the sr25519 pipeline's stream and its
  // fork / join events (created on first use)
  tmv::KindStreams kinds{nullptr, nullptr, nullptr};
  // last batch-equation launch on this stream (for tmv_batch_stats)
  const uint8_t *group_ok[2] = {nullptr, nullptr};
  const uint8_t *sub_ok[2] = {nullptr, nullptr};  // sub-group verdicts (k_msm_subcheck), if it ran
  uint32_t groups = 0, m_log2 = 0, n = 0;
  uint32_t m_log2_sr = 0;  // mixed: the sr25519 half's group size (m_log2 is the ed25519 half's)
  const uint32_t *counts = nullptr;  // mixed launches: per-kind entry counts on the device
  const uint32_t *loc[2] = {nullptr, nullptr};  // located pass ran: its (slots, fb_count, found) words
};

// One lane of the host-buffer pipeline: a stream with its own pinned and
// device staging.  Large host batches are cut into chunks that alternate
// between two lanes, so chunk k+1's staging and H2D copy overlap chunk k's
// kernels (the reference's "double-buffered hipMemcpyAsync on side streams").
struct HostLane {
  hipStream_t stream = nullptr;
  DeviceBuf h_in, d_in, h_out, d_out;
  uint32_t lo = 0, n = 0;  // chunk in flight (n == 0: idle)
  // streamed batch-equation chunks: the parts' H2D copies run on `copy`,
  // each followed by an event the kernels of its part wait for (created on
  // first use)
  hipStream_t copy = nullptr;
  std::vector<hipEvent_t> part_ready;
  // odd parts run their kernels on `helper`, so two parts' kernels overlap;
  // `join` orders the launch's tail after them
  hipStream_t helper = nullptr;
  hipEvent_t join = nullptr;
  // streamed mixed chunks: one event per part after its kind partition
  std::vector<hipEvent_t> part_split;
  // caller pages pinned for the chunk in flight (streamed path, direct DMA);
  // unregistered when the chunk is harvested
  std::vector<void *> pinned;
  void unpin() {
    for (void *p : pinned) (void)hipHostUnregister(p);
    pinned.clear();
  }
};
constexpr int kLanes = 4;  // streams per device; TMV_HOST_LANES of them carry chunks

struct Device {
  int id = -1;
  // device-pointer entry points called with stream = NULL run here; the host
  // lanes have streams of their own, so such a call never shares a lane's
  // stream (or its workspace) with a host-buffer call in flight
  hipStream_t stream = nullptr;  // created on first use (context_stream)
  std::once_flag stream_once;
  HostLane lane[kLanes];
  tmv::ge_precomp *d_btable = nullptr;   // 32x8 comb (single-lane kernel)
  tmv::fe *d_btab_q = nullptr;           // 8 x CachedQ multiples of B (quad kernel)
  tmv::strobe_t *d_prefix = nullptr;     // sr25519 transcript prefix (empty context)
  // one workspace per launch stream, so device-resident batches issued on
  // different caller streams run concurrently (the context's own stream is
  // one of them)
  std::unordered_map<hipStream_t, std::unique_ptr<Workspace>> ws;
  hipEvent_t work_done = nullptr;        // after the latest key-table build (cumulative: each build waits on the last)
  hipEvent_t kbuild_copied = nullptr;    // the latest build's keys left the pinned staging
  tmv::fe *d_bcomb = nullptr;            // 32 x 128 CachedQ: (m+1) 256^j B (key-cached path)
  // expanded-key cache (device table + host LRU index)
  tmv::KeyTable kt{nullptr, nullptr};
  uint32_t kcap = 0;
  KeyIndex kindex;                                  // (kind, key bytes) -> slot
  std::list<uint32_t> klru;                         // front = most recently used
  std::vector<std::list<uint32_t>::iterator> kpos;
  std::vector<std::array<uint8_t, 33>> kslot_key;
  std::vector<uint64_t> kslot_epoch;
  std::vector<uint8_t> kseen;  // resolve_keys: slots found, per lookup part
  uint64_t kepoch = 0, khits = 0, kmisses = 0;
  DeviceBuf d_kbuild, h_kbuild;
  DeviceBuf d_valset, h_valset;  // tmv_validator_set_hashes staging
  // host-buffer launches: key slots of the shard and the per-chunk key
  // histograms of the key-merged form's counting sort
  std::vector<uint32_t> slots, key_count;
  std::mutex mu;
  // lanes claimed by host-buffer calls (run_batch).  A call holds `mu` while
  // it stages and launches a chunk, not while it waits for the device, so
  // calls on different lanes (a caller's windows in flight) overlap; a chunk
  // in flight is `lane[l].n != 0`, which resolve_keys waits for before a
  // new key may evict a slot
  bool lane_busy[kLanes] = {};
  std::condition_variable lane_cv;
  // a device wait timed out: its work is in an unknown state, so every later
  // call on this device returns TMV_ERR_TIMEOUT (include/tmverify.h)
  std::atomic<bool> faulted{false};
};

// Caller pages that stayed registered after a failed or skipped wait (the
// chunk's DMA may still be in flight, so they were not unregistered; see the
// harvest in run_batch).  A stale registration would let a later copy through
// those virtual addresses -- after the caller freed and the allocator reused
// them -- hit the old pinned pages, so each range is unregistered as soon as
// the streams that could still read it report idle: checked (never waited
// for) at every tmv_open, tmv_close and host-buffer call.
struct LeakedPin {
  int dev;
  hipStream_t copy, stream;
  void *p;
};
std::mutex g_leak_mu;
std::vector<LeakedPin> g_leaked;

void leak_pins(int dev, HostLane &ln) {
  std::lock_guard<std::mutex> lk(g_leak_mu);
  for (void *p : ln.pinned) g_leaked.push_back({dev, ln.copy, ln.stream, p});
  ln.pinned.clear();
}

// Unregister every leaked range whose streams have drained (a range whose
// device never drains stays registered, with that device's leaked buffers).
void release_leaked_pins() {
  std::lock_guard<std::mutex> lk(g_leak_mu);
  if (g_leaked.empty()) return;
  // the caller's current device is restored on return (this runs inside
  // tmv_open / tmv_close / host-buffer calls, on the caller's thread)
  int cur = -1;
  const bool have_cur = hipGetDevice(&cur) == hipSuccess;
  struct Restore {
    bool on;
    int dev;
    ~Restore() { if (on) (void)hipSetDevice(dev); }
  } restore{have_cur, cur};
  std::vector<LeakedPin> keep;
  for (const LeakedPin &x : g_leaked) {
    (void)hipSetDevice(x.dev);
    const bool idle = (!x.copy || hipStreamQuery(x.copy) == hipSuccess) &&
                      (!x.stream || hipStreamQuery(x.stream) == hipSuccess);
    (void)hipGetLastError();
    if (idle) (void)hipHostUnregister(x.p);
    else keep.push_back(x);
  }
  g_leaked.swap(keep);
}

size_t leaked_pin_count() {
  std::lock_guard<std::mutex> lk(g_leak_mu);
  return g_leaked.size();
}

// Kernel choice: the quad (4 lanes / signature) path wins while the batch is
// too small to fill the chip one lane per signature; the single-lane kernel
// has less glue per signature and wins on large batches.
constexpr uint32_t kQuadMax = 49152;
int g_kernel_override = -1;  // A/B (TMV_KERNEL=quad|single): -1 auto, 0 single, 1 quad
// Batch equation (msm.h) by default from this many entries up (TMV_MSM_MIN,
// 0 = never): below it a batch is latency-bound and the per-entry pipeline
// beats the batch check's longer chain; above it the batch check does 2-3x
// less work.  Set from launches alone at the end of round 4
// (profiles/r04/crossover.txt): per entry 0.43 / 0.66 / 0.96 / 1.26 ms at
// 16k / 24k / 32k / 48k C2 entries, the batch equation 0.87 / 0.90 / 0.96 /
// 1.10 ms -- equal at 32k (was 16384).  Key-cached batches (the key-merged
// form against the comb kernel) keep 16384 (g_km_min); TMV_MSM_MIN sets
// both.  Flags override per call.
uint32_t g_msm_min = 32768;
uint32_t g_km_min = 16384;
uint32_t g_msm_chunk = 0;  // A/B (TMV_MSM_CHUNK): 16 or 32 overrides the chunk length
uint32_t g_msm_parts = 0;  // A/B (TMV_MSM_PARTS): running-sum lanes per window (power of two <= H)
// Key-cached batches up to this size run as one fused latency kernel
// (TMV_CACHED_FUSED_MAX; commit-sized calls such as VerifyCommit).
uint32_t g_cached_fused_max = 4096;
// Fused-path batches read their inputs and write their statuses in pinned
// host memory instead of copying (A/B: TMV_ZERO_COPY=0 turns it off).
int g_zero_copy = 1;
// Host-buffer batches of at least this many entries per device are
// pipelined in chunks (of half to one of these) over two lanes
// (TMV_HOST_CHUNK).
uint32_t g_host_chunk = 262144;
// Mixed ed25519 + sr25519 host batches on the batch equation are streamed
// (mixed_check_streamed, round 5: C5 1M end to end 16.0 -> 11.0-11.3 ms);
// A/B (TMV_MIXED_STREAM=0): unstreamed, in chunks of g_mixed_chunk, the
// second's copy beside the first's kernels.
int g_mixed_stream = 1;
uint32_t g_mixed_chunk = 786432;
// Lanes the chunks rotate over (A/B: TMV_HOST_LANES, 1..kLanes).
uint32_t g_host_lanes = 2;
// Bound on every wait for device work (TMV_DEVICE_TIMEOUT_MS, 0 = none).
int64_t g_timeout_ms = 60000;
// Streamed host batches (uncached batch equation): a chunk's inputs are
// staged and copied in parts -- the first of g_stream_first entries, then
// g_stream_part each (rounded to whole groups) -- and each part's throughput
// kernels start as soon as its copy lands, so one pipeline covers the chunk
// (one latency tail) while the rest is still being staged
// (TMV_STREAM_FIRST, TMV_STREAM_PART).  Such batches are cut into chunks of
// up to g_stream_chunk entries per device (TMV_STREAM_CHUNK).  A/B:
// TMV_STREAM=0 (no streaming), TMV_STREAM_TWO=0 (every part on the lane's
// stream), TMV_SR_GROUP_LOG2 (group size of uncached sr25519 launches).
int g_stream = 1;
int g_stream_two = 1;
uint32_t g_sr_group_log2 = 0;
// Round 2, 320k C2 entries end to end (parts on two streams): 5.7 ms with
// parts of 32k / 64k, 5.85-6.0 with 32k / 128k; one stream 6.05-6.3;
// unstreamed (two lanes of 80k chunks) 6.9 ms.  Round 3 (faster kernels,
// the caller's pages DMA'd directly), the bench's 640k entries: parts of
// 128k 82.7-83.8 M/s, 64k 77.3-79.1, 256k 78.9-79.8; a first part of 16k
// or 64k changes nothing (profiles/r03/e2e_parts.txt).  2.56 M entries per
// call: chunks of up to 4 M (one pipeline) 106 M/s, 2 M (two pipelines of
// 1.28 M on two lanes) 98 M/s, 1 M 87 M/s (profiles/r03/e2e_chunk.txt)
uint32_t g_stream_first = 32768, g_stream_part = 131072, g_stream_chunk = 1u << 22;
// Part sizes double from g_stream_first up to g_stream_part (32k, 64k,
// 128k, ...), so the second part lands while the first one's kernels run
// instead of the device idling for a whole 128k part's copy (round 6, same
// box, A/B TMV_STREAM_RAMP=0: 2.56M C2 call 22.29 / 22.12 -> 21.83 / 21.65
// ms, C5 1M mixed 11.48 -> 11.19 ms; profiles/r06/ab_e2e_ramp.txt)
int g_stream_ramp = 1;
constexpr uint32_t kMaxStreamParts = 512;  // bound on a streamed mixed chunk's parts (4 M / 128k + 1 = 33 by default)
// Streamed parts DMA straight from the caller's buffers: each part pins the
// whole pages of its pk / sig / msg spans (hipHostRegister, disjoint page
// ranges part to part) while earlier parts run, and only the bytes outside
// them (< 4 KiB per span and part) go through the lane's pinned staging
// (A/B: TMV_REGISTER=0 stages everything).  A span whose pages cannot be
// pinned (already pinned, read-only mapping, ...) is staged.
int g_register = 1;

void read_env() {
  static std::once_flag once;
  std::call_once(once, [] {
    // production knobs
    const char *mm = getenv("TMV_MSM_MIN");
    if (mm) g_msm_min = g_km_min = (uint32_t)strtoul(mm, nullptr, 10);
    const char *cf = getenv("TMV_CACHED_FUSED_MAX");
    if (cf) g_cached_fused_max = (uint32_t)strtoul(cf, nullptr, 10);
    const char *hc = getenv("TMV_HOST_CHUNK");
    if (hc) g_host_chunk = std::max<uint32_t>(1, (uint32_t)strtoul(hc, nullptr, 10));
    const char *to = getenv("TMV_DEVICE_TIMEOUT_MS");
    if (to) g_timeout_ms = strtoll(to, nullptr, 10);
    const char *sf = getenv("TMV_STREAM_FIRST");
    if (sf) g_stream_first = std::max<uint32_t>(1, (uint32_t)strtoul(sf, nullptr, 10));
    const char *sp = getenv("TMV_STREAM_PART");
    if (sp) g_stream_part = std::max<uint32_t>(1, (uint32_t)strtoul(sp, nullptr, 10));
    const char *sc = getenv("TMV_STREAM_CHUNK");
    if (sc) g_stream_chunk = std::max<uint32_t>(2048, (uint32_t)strtoul(sc, nullptr, 10));
    // A/B switches: read only by a -DTMV_AB build (knobs.h)
    const char *k = tmv::ab_knob("TMV_KERNEL");
    if (k && !strcmp(k, "quad")) g_kernel_override = 1;
    if (k && !strcmp(k, "single")) g_kernel_override = 0;
    const char *zc = tmv::ab_knob("TMV_ZERO_COPY");
    if (zc) g_zero_copy = atoi(zc);
    const char *ms = tmv::ab_knob("TMV_MIXED_STREAM");
    if (ms) g_mixed_stream = atoi(ms);
    const char *mxc = tmv::ab_knob("TMV_MIXED_CHUNK");
    if (mxc) g_mixed_chunk = std::max<uint32_t>(1, (uint32_t)strtoul(mxc, nullptr, 10));
    const char *hl = tmv::ab_knob("TMV_HOST_LANES");
    if (hl) g_host_lanes = std::min<uint32_t>(kLanes, std::max<uint32_t>(1, (uint32_t)strtoul(hl, nullptr, 10)));
    const char *mp = tmv::ab_knob("TMV_MSM_PARTS");
    if (mp) g_msm_parts = (uint32_t)strtoul(mp, nullptr, 10);
    const char *mc = tmv::ab_knob("TMV_MSM_CHUNK");
    if (mc) g_msm_chunk = (uint32_t)strtoul(mc, nullptr, 10);
    const char *st = tmv::ab_knob("TMV_STREAM");
    if (st) g_stream = atoi(st);
    const char *sg = tmv::ab_knob("TMV_SR_GROUP_LOG2");
    if (sg) g_sr_group_log2 = (uint32_t)strtoul(sg, nullptr, 10);
    const char *s2 = tmv::ab_knob("TMV_STREAM_TWO");
    if (s2) g_stream_two = atoi(s2);
    const char *rp = tmv::ab_knob("TMV_STREAM_RAMP");
    if (rp) g_stream_ramp = atoi(rp);
    const char *rg = tmv::ab_knob("TMV_REGISTER");
    if (rg) g_register = atoi(rg);
  });
}

// The context's own stream (device-pointer calls with stream = NULL, the
// hashing entry points), created on first use; NULL if creation failed.
hipStream_t context_stream(Device &d) {
  std::call_once(d.stream_once, [&] {
    (void)hipSetDevice(d.id);
    if (hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess) d.stream = nullptr;
  });
  return d.stream;
}

// Bounded waits (host/wait.h).  hipErrorNotReady = timed out (the device is
// then marked faulted); any other error is the device's.
hipError_t wait_stream(Device &d, hipStream_t s) {
  read_env();
  hipError_t err = hipSuccess;
  const tmh::Poll r = tmh::poll_until([&] {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return 0;
    if (e == hipErrorNotReady) return 1;
    err = e;
    return 2;
  }, g_timeout_ms);
  if (r == tmh::Poll::kTimeout) {
    d.faulted = true;
    set_error("device wait exceeded TMV_DEVICE_TIMEOUT_MS (" + std::to_string(g_timeout_ms) + " ms)");
    return hipErrorNotReady;
  }
  return err;
}
hipError_t wait_event(Device &d, hipEvent_t ev) {
  read_env();
  hipError_t err = hipSuccess;
  const tmh::Poll r = tmh::poll_until([&] {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return 0;
    if (e == hipErrorNotReady) return 1;
    err = e;
    return 2;
  }, g_timeout_ms);
  if (r == tmh::Poll::kTimeout) {
    d.faulted = true;
    set_error("device wait exceeded TMV_DEVICE_TIMEOUT_MS (" + std::to_string(g_timeout_ms) + " ms)");
    return hipErrorNotReady;
  }
  return err;
}
int wait_rc(hipError_t e) { return e == hipErrorNotReady ? TMV_ERR_TIMEOUT : TMV_ERR_LAUNCH; }
int faulted_rc(Device &d) {
  set_error("device timed out earlier (TMV_ERR_TIMEOUT); open a new context");
  return TMV_ERR_TIMEOUT;
}

// Batch-equation parameters for n entries.  Group size: the caller's, else
// 64 (a group of m fails with probability ~ m x the rate of entries that are
// invalid yet decode; 64 keeps the per-entry fallback near 10% of a batch
// with 0.2% such entries, as in BASELINE configs[1]).  Window: minimises
// bucket additions + per-window running sums for that m (c in [4, 9]).
// The key-merged form (merged = true; keyed batches are commit traffic,
// nearly always valid) defaults to groups of 256: its MSM has only the R
// points and its fallback is the cheaper key-cached comb.
// Cost of a bucket's running sum relative to a bucket entry's addition in the
// window choice below.  2.2 from the kernels' per-item times picked c = 6 for
// groups of 128; c = 5 measured faster (2.56M launch alone 20.95 -> 19.94 ms,
// profiles/r05/ab_window.txt): fuller buckets (16 entries, one chunk) split
// and join less, and the 2H-addition running-sum chain halves.  3.0 keeps
// c = 5 for groups of 64 and 128.
constexpr double kRunningSumWeight = 3.0;
static double running_sum_weight() {  // A/B of the weight (TMV_RS_WEIGHT, read per launch)
  const char *e = tmv::ab_knob("TMV_RS_WEIGHT");
  return e ? atof(e) : kRunningSumWeight;
}
tmv::MsmParams msm_params(uint32_t n, uint32_t m_log2, uint32_t c, bool merged = false, bool ed_only = false,
                          int sub = -1) {
  // uncached ed25519 launches large enough for the located fallback
  // (tmv::locate_min_entries): groups of 128 (c = 6 by the cost model) --
  // a failing group costs one located entry, not 128 verifications; C2
  // bench 98.1-98.3 -> 100.7-100.8 M/s, groups of 256: 91.7-92.0
  // (profiles/r02_close/ab_group.txt).  sr25519 / mixed batches keep 64
  // (the factory's sr25519 corruption rate puts two bad entries in too many
  // groups of 128).
  const uint32_t lmin = tmv::locate_min_entries();
  if (m_log2 == 0) m_log2 = merged ? 8 : (ed_only && lmin && n >= lmin ? 7 : 6);
  m_log2 = std::max<uint32_t>(5, std::min<uint32_t>(10, m_log2));
  if (c == 0) {
    const double m = double(1u << m_log2), rsw = running_sum_weight();
    double best = 1e30;
    for (uint32_t cc = 4; cc <= 9; cc++) {
      const double W = (254 + cc - 1) / cc, WR = (129 + cc - 1) / cc, H = double(1u << (cc - 1));
      const double cost = merged ? m * WR + 2.2 * WR * H : m * (W + WR) + rsw * W * H;
      if (cost < best) { best = cost; c = cc; }
    }
  }
  c = std::max<uint32_t>(4, std::min<uint32_t>(9, c));
  tmv::MsmParams p = tmv::MsmParams::make(n, m_log2, c, merged);
  if (g_msm_chunk == 16 || g_msm_chunk == 32) p.L = g_msm_chunk;
  if (g_msm_parts && g_msm_parts <= p.H && !(g_msm_parts & (g_msm_parts - 1))) p.P = g_msm_parts;
  // sub-group bisection: the context's choice, else the default policy
  // (the key-merged form's fallback is the key-cached comb: never)
  p.sub = merged ? 0 : (sub < 0 ? (tmv::subcheck_enabled(m_log2) ? 1 : 0) : (uint32_t)sub);
  return p;
}

// Phase timing of the host-buffer path, printed to stderr when
// TMV_HOST_TIMING is set (profiling aid; the host layer prints its own).
struct EngineTimer {
  bool on = tmh::host_timing();
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char *what, uint32_t n) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[tmv_engine] %-8s %9.3f ms (n=%u)\n", what,
            std::chrono::duration<double, std::milli>(now - t).count(), n);
    t = now;
  }
};

// Packed staging layout for one shard: pk | sig | off | msg (16-B aligned).
struct Layout {
  size_t pk, sig, off, msg, total;
  Layout(uint32_t n, size_t msg_bytes) {
    pk = 0;
    sig = align16(pk + 32ull * n);
    off = align16(sig + 64ull * n);
    msg = align16(off + 4ull * (n + 1));
    total = align16(msg + std::max<size_t>(msg_bytes, 1));
  }
};

// How one launch verifies: per entry, or through the batch equation with
// these parameters and this randomness.
struct LaunchOpts {
  bool batch_eq = false;
  tmv::MsmParams p{};      // single-kind launches; the sr25519 half of a mixed one
  tmv::MsmParams p_ed{};   // the ed25519 half of a mixed launch
  tmv::MsmParams p_ed_streamed{};  // ... of a streamed one (mixed_check_streamed)
  tmv::MsmSeed seed[2]{};  // [kind]
  int err = 0;             // < 0: no launch (the weights' key could not be drawn)
};

// Test aid (tmv_internal_random_fault): the next `count` getrandom calls
// fail with errno `err` (count < 0: every call).
std::atomic<int> g_rand_fault_err{0}, g_rand_fault_count{0};

// The key of a launch's ChaCha20 weights from the OS (the reference draws z
// from rand.Reader, crypto/ed25519/ed25519.go:232, and a Reader error
// reaches its caller).  Short reads and EINTR are retried; any other failure
// (ENOSYS, a seccomp EPERM, ...) returns TMV_ERR_RANDOM instead of spinning.
int draw_weight_key(uint8_t key[32]) {
  size_t got = 0;
  while (got < 32) {
    ssize_t r;
    int fc = g_rand_fault_count.load();
    if (fc != 0) {
      if (fc > 0) g_rand_fault_count.fetch_sub(1);
      errno = g_rand_fault_err.load();
      r = -1;
    } else {
      r = getrandom(key + got, 32 - got, 0);
    }
    if (r > 0) {
      got += (size_t)r;
    } else if (r < 0 && errno == EINTR) {
      continue;
    } else {
      set_error(std::string("getrandom: ") + (r < 0 ? strerror(errno) : "no bytes"));
      return TMV_ERR_RANDOM;
    }
  }
  return 0;
}

}  // namespace

struct tmv_ctx {
  std::vector<std::unique_ptr<Device>> devs;
  // batch-equation options (tmv_set_batch_options)
  uint32_t msm_m_log2 = 0, msm_c = 0;
  int msm_sub = -1;  // TMV_BATCHOPT_SUBCHECK_ON / _OFF, -1 = default
  bool fixed_seed = false, stats = false;
  uint8_t seed[32] = {0};
  std::atomic<uint64_t> launches{0};
  std::atomic<uint64_t> groups{0}, groups_failed{0}, subgroups{0}, subgroups_failed{0};
  // tmv_metrics
  std::atomic<uint64_t> m_calls{0}, m_sigs{0}, m_max{0}, m_beq{0}, m_host_sigs{0}, m_host_ns{0}, m_h2d{0}, m_d2h{0},
      m_located{0}, m_fallback{0};
  uint64_t khits_base = 0, kmiss_base = 0;
  std::mutex opt_mu;
  // m_host_ns is busy wall time: the union of the host-buffer calls'
  // intervals (calls overlap -- lane claims, windows in flight -- so summing
  // each call's duration would count shared time more than once)
  std::mutex host_mu;
  uint32_t host_inflight = 0;
  std::chrono::steady_clock::time_point host_t0;

  void host_enter() {
    std::lock_guard<std::mutex> lk(host_mu);
    if (host_inflight++ == 0) host_t0 = std::chrono::steady_clock::now();
  }
  void host_leave(uint64_t n) {
    std::lock_guard<std::mutex> lk(host_mu);
    m_host_sigs += n;
    if (--host_inflight == 0)
      m_host_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                       std::chrono::steady_clock::now() - host_t0).count();
  }

  void count_call(uint64_t n) {
    m_calls++;
    m_sigs += n;
    uint64_t cur = m_max.load();
    while (n > cur && !m_max.compare_exchange_weak(cur, n)) {
    }
  }
};

// Options of one launch of n entries: per-entry or batch equation (flags,
// else TMV_MSM_MIN), parameters and fresh randomness.
static LaunchOpts make_opts(tmv_ctx *ctx, uint32_t flags, uint32_t n, bool merged = false, bool ed_only = false) {
  read_env();
  LaunchOpts o;
  if (flags & TMV_FLAG_PER_ENTRY) o.batch_eq = false;
  else if (flags & TMV_FLAG_BATCH_EQUATION) o.batch_eq = true;
  else {
    const uint32_t thr = merged ? g_km_min : g_msm_min;
    o.batch_eq = thr > 0 && n >= thr;
  }
  if (!o.batch_eq) return o;
  ctx->m_beq += n;
  uint8_t key[32];
  bool fixed;
  {
    std::lock_guard<std::mutex> lk(ctx->opt_mu);  // tmv_set_batch_options writes these
    o.p = msm_params(n, ctx->msm_m_log2 ? ctx->msm_m_log2 : (!merged && !ed_only ? g_sr_group_log2 : 0), ctx->msm_c,
                     merged, ed_only, ctx->msm_sub);
    // mixed launches: each kind's half its own group size -- ed25519 takes
    // the located-fallback groups of 128 at the size ed25519-only launches
    // do, sr25519 keeps 64 (msm_params); both stay the caller's when set
    o.p_ed = merged || ed_only ? o.p : msm_params(n, ctx->msm_m_log2, ctx->msm_c, false, true, ctx->msm_sub);
    // streamed, the ed25519 half keeps groups of 64 too: a part's window
    // parts are latency-bound (~1k groups per part and kind), and c = 6's
    // 2H = 64-addition running sums (groups of 128) cost more than the
    // located fallback saves -- C5 1M mixed end to end 11.6 -> 11.2 ms
    // (profiles/r05/mixed_stream/)
    o.p_ed_streamed = merged || ed_only ? o.p
                                        : msm_params(n, ctx->msm_m_log2 ? ctx->msm_m_log2 : 6, ctx->msm_c, false, true,
                                                     ctx->msm_sub);
    fixed = ctx->fixed_seed;
    if (fixed) std::memcpy(key, ctx->seed, 32);
  }
  if (!fixed && (o.err = draw_weight_key(key)) != 0) return o;
  const uint64_t ctr = ctx->launches.fetch_add(1);
  for (int k = 0; k < 2; k++) {
    std::memcpy(o.seed[k].key, key, 32);
    o.seed[k].nonce[0] = (uint32_t)ctr;
    o.seed[k].nonce[1] = (uint32_t)(ctr >> 32);
    o.seed[k].nonce[2] = (uint32_t)k;
  }
  return o;
}

// Group verdicts of the last batch-equation launch on stream s (synchronised
// by the caller) into the context's counters.
static void collect_stats(tmv_ctx *ctx, Device &d, hipStream_t s) {
  auto it = d.ws.find(s);
  if (it == d.ws.end() || !it->second->group_ok[0]) return;
  Workspace &w = *it->second;
  uint32_t live[2] = {0, 0}, live_n[2] = {0, 0};
  if (w.counts) {
    uint32_t c[2];
    if (hipMemcpy(c, w.counts, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return;
    for (int k = 0; k < 2; k++) {
      const uint32_t ml = k ? w.m_log2_sr : w.m_log2;
      live[k] = (c[k] + (1u << ml) - 1) >> ml;
      live_n[k] = c[k];
    }
  } else {
    live[0] = w.groups;
  }
  for (int k = 0; k < 2; k++) {
    if (!w.group_ok[k] || !live[k]) continue;
    const uint32_t mlog = k ? w.m_log2_sr : w.m_log2;
    std::vector<uint8_t> ok(live[k]);
    if (hipMemcpy(ok.data(), w.group_ok[k], live[k], hipMemcpyDeviceToHost) != hipSuccess) return;
    uint64_t failed = 0;
    for (uint8_t v : ok) failed += v ? 0 : 1;
    ctx->groups += live[k];
    ctx->groups_failed += failed;
    if (failed && w.loc[k]) {  // located pass: its search counted the entries it left to verify
      uint32_t lc[4];
      if (hipMemcpy(lc, w.loc[k], sizeof(lc), hipMemcpyDeviceToHost) != hipSuccess) return;
      ctx->m_fallback += lc[1];
      ctx->m_located += lc[2];
    } else if (failed && !w.sub_ok[k]) {  // every entry of a failing group
      const uint32_t m = 1u << mlog, nk = w.counts ? live_n[k] : w.n;
      for (uint32_t g = 0; g < live[k]; g++)
        if (!ok[g]) ctx->m_fallback += std::min<uint32_t>(m, nk - g * m);
    }
    if (!w.sub_ok[k] || !failed) continue;
    // sub-groups of the failing groups (the only ones k_msm_subcheck writes)
    const uint32_t per = 1u << (mlog - tmv::kSubGroupLog2);
    std::vector<uint8_t> sub((size_t)live[k] * per);
    if (hipMemcpy(sub.data(), w.sub_ok[k], sub.size(), hipMemcpyDeviceToHost) != hipSuccess) return;
    uint64_t sfail = 0;
    for (uint32_t g = 0; g < live[k]; g++)
      if (!ok[g])
        for (uint32_t j = 0; j < per; j++) sfail += sub[(size_t)g * per + j] ? 0 : 1;
    ctx->subgroups += failed * per;
    ctx->subgroups_failed += sfail;
    // per-entry fallback by 16-entry blocks holding a failing sub-group
    for (uint32_t g = 0; g < live[k]; g++)
      if (!ok[g])
        for (uint32_t j = 0; j + 1 < per + 1; j += 2) {
          const bool bad = !sub[(size_t)g * per + j] || (j + 1 < per && !sub[(size_t)g * per + j + 1]);
          if (bad) ctx->m_fallback += 2 * tmv::kSubGroup;
        }
  }
  w.group_ok[0] = w.group_ok[1] = nullptr;
  w.sub_ok[0] = w.sub_ok[1] = nullptr;
  w.loc[0] = w.loc[1] = nullptr;
}

static int init_device(Device &d) {
  hipError_t e = hipSetDevice(d.id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  // The lanes' streams are created first and the context's own stream only
  // when a call first needs it (context_stream): HIP spreads streams over
  // its hardware queues (GPU_MAX_HW_QUEUES = 4) in creation order, and with
  // the context stream created ahead of the lanes a streamed host call's
  // copy stream shared a queue with its lane's kernels -- end to end 105 ->
  // 82 M/s on 2.56 M-entry calls (profiles/r04/e2e_lane0.txt).
  for (int l = 0; l < kLanes; l++) {
    e = hipStreamCreateWithFlags(&d.lane[l].stream, hipStreamNonBlocking);
    if (e != hipSuccess) { set_error("hipStreamCreate", e); return TMV_ERR_NO_DEVICE; }
  }
  std::vector<tmv::ge_precomp> table(tmv::kBaseTableRows * tmv::kBaseTableCols);
  tmv::build_base_table(table.data());
  const size_t bytes = table.size() * sizeof(tmv::ge_precomp);
  e = hipMalloc(&d.d_btable, bytes);
  if (e != hipSuccess) { set_error("hipMalloc(btable)", e); return TMV_ERR_NOMEM; }
  e = hipMemcpy(d.d_btable, table.data(), bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) { set_error("hipMemcpy(btable)", e); return TMV_ERR_NO_DEVICE; }
  // quad B tables: entry m = (m+1)B, then entry kBaseQuadEntries + m =
  // (m+1)[2^128]B (the half-size scalars' top digits), m < kBaseQuadEntries,
  // as (ymx, ypx, xy2d, 1)
  std::vector<tmv::fe> bq(2 * 4 * tmv::kBaseQuadEntries);
  {
    tmv::ge_p3 B;
    tmv::ed25519_base_point(B);
    for (int h = 0; h < 2; h++) {
      if (h == 1)
        for (int d = 0; d < 128; d++) {  // B <- [2^128]B
          tmv::ge_p1p1 t;
          tmv::ge_p3_dbl(t, B);
          tmv::ge_p1p1_to_p3(B, t);
        }
      tmv::ge_cached bc;
      tmv::ge_p3_to_cached(bc, B);
      tmv::ge_p3 P = B;
      for (int m = 0; m < tmv::kBaseQuadEntries; m++) {
        tmv::ge_precomp pc;
        tmv::ge_p3_to_precomp(pc, P);
        tmv::fe *o = &bq[4 * (h * tmv::kBaseQuadEntries + m)];
        o[0] = pc.ymx;
        o[1] = pc.ypx;
        o[2] = pc.xy2d;
        tmv::fe_one(o[3]);
        tmv::ge_p1p1 t;
        tmv::ge_add(t, P, bc);
        tmv::ge_p1p1_to_p3(P, t);
      }
    }
  }
  e = hipMalloc(&d.d_btab_q, bq.size() * sizeof(tmv::fe));
  if (e != hipSuccess) { set_error("hipMalloc(btab_q)", e); return TMV_ERR_NOMEM; }
  e = hipMemcpy(d.d_btab_q, bq.data(), bq.size() * sizeof(tmv::fe), hipMemcpyHostToDevice);
  if (e != hipSuccess) { set_error("hipMemcpy(btab_q)", e); return TMV_ERR_NO_DEVICE; }
  tmv::strobe_t prefix;
  tmv::sr25519_context_prefix(prefix);
  e = hipMalloc(&d.d_prefix, sizeof(prefix));
  if (e != hipSuccess) { set_error("hipMalloc(prefix)", e); return TMV_ERR_NOMEM; }
  e = hipMemcpy(d.d_prefix, &prefix, sizeof(prefix), hipMemcpyHostToDevice);
  if (e != hipSuccess) { set_error("hipMemcpy(prefix)", e); return TMV_ERR_NO_DEVICE; }
  e = hipEventCreateWithFlags(&d.work_done, hipEventDisableTiming);
  if (e != hipSuccess) { set_error("hipEventCreate", e); return TMV_ERR_NO_DEVICE; }
  // base comb for the key-cached path: row j, entry m = (m+1) 256^j B (CachedQ, Z kept)
  {
    std::vector<tmv::fe> bc((size_t)32 * tmv::kBaseQuadEntries * 4);
    tmv::ge_p3 row, P;
    tmv::ed25519_base_point(row);
    for (int j = 0; j < 32; j++) {
      tmv::ge_cached rc;
      tmv::ge_p3_to_cached(rc, row);
      P = row;
      for (int m = 0; m < tmv::kBaseQuadEntries; m++) {
        tmv::ge_cached c;
        tmv::ge_p3_to_cached(c, P);
        tmv::fe *o = &bc[((size_t)j * tmv::kBaseQuadEntries + m) * 4];
        tmv::fe_carry(o[0], c.YmX);
        tmv::fe_carry(o[1], c.YpX);
        o[2] = c.T2d;
        o[3] = c.Z;
        tmv::ge_p1p1 t;
        tmv::ge_add(t, P, rc);
        tmv::ge_p1p1_to_p3(P, t);
      }
      for (int d = 0; d < 8; d++) {  // row *= 256
        tmv::ge_p1p1 t;
        tmv::ge_p3_dbl(t, row);
        tmv::ge_p1p1_to_p3(row, t);
      }
    }
    e = hipMalloc(&d.d_bcomb, bc.size() * sizeof(tmv::fe));
    if (e != hipSuccess) { set_error("hipMalloc(bcomb)", e); return TMV_ERR_NOMEM; }
    e = hipMemcpy(d.d_bcomb, bc.data(), bc.size() * sizeof(tmv::fe), hipMemcpyHostToDevice);
    if (e != hipSuccess) { set_error("hipMemcpy(bcomb)", e); return TMV_ERR_NO_DEVICE; }
  }
  const char *kc = getenv("TMV_KEY_CACHE_CAPACITY");
  d.kcap = kc ? (uint32_t)strtoul(kc, nullptr, 10) : 4096u;  // voi's LRU size (crypto/ed25519/ed25519.go:56)
  return 0;
}

// Resolve the key slot of every entry, building the comb tables of missing
// keys on the device.  Returns 1 if the batch has more distinct keys than the
// cache holds (caller uses the uncached path), 0 on success, < 0 on error.
// Caller holds d.mu.  slots_out: n entries (host memory).
static int resolve_keys(Device &d, bool sr, const uint8_t *pk, uint32_t n, uint32_t *slots_out, hipStream_t s) {
  if (d.kcap == 0) return 1;
  hipError_t e;
  if (!d.kt.tab) {
    if ((e = hipMalloc(&d.kt.tab, (size_t)d.kcap * tmv::KeyTable::bytes_per_key())) != hipSuccess) {
      set_error("hipMalloc(key table)", e);
      d.kt.tab = nullptr;
      return 1;  // no room: fall back to the uncached path
    }
    if ((e = hipMalloc(&d.kt.ok, d.kcap)) != hipSuccess) { set_error("hipMalloc(key ok)", e); return TMV_ERR_NOMEM; }
    d.kpos.resize(d.kcap);
    d.kslot_key.resize(d.kcap);
    d.kslot_epoch.assign(d.kcap, 0);
  }
  if (d.kindex.t.empty()) d.kindex.init(d.kcap);
  const uint64_t epoch = ++d.kepoch;
  std::vector<uint32_t> miss_idx;
  std::vector<uint32_t> miss_slot;
  // 1) read-only lookups, in parallel for large batches (runs of one key
  //    reuse the previous answer); each part marks the slots it found and
  //    counts its misses
  constexpr uint32_t kParts = 16;
  const uint32_t parts = n >= 16384 ? kParts : 1;
  d.kseen.assign((size_t)parts * d.kcap, 0);
  uint32_t misses[kParts] = {0};
  // missing entries by (entry part p, key part q): list p * parts + q, in
  // entry order; q = a key's hash bits, so every distinct key lives in one q
  std::vector<std::vector<uint32_t>> mb((size_t)parts * parts);
  auto key_part = [&](const uint8_t *k33) -> uint32_t {
    return parts == 1 ? 0u : (uint32_t)(KeyIndex::hash(k33) >> 58) & (kParts - 1);
  };
  auto lookup = [&](uint32_t part) {
    const uint32_t lo = (uint32_t)((uint64_t)n * part / parts), hi = (uint32_t)((uint64_t)n * (part + 1) / parts);
    uint8_t *seen = d.kseen.data() + (size_t)part * d.kcap;
    uint8_t key[33];
    key[0] = sr ? 1 : 0;
    const uint8_t *last_pk = nullptr;
    uint32_t last_slot = UINT32_MAX, miss = 0, last_q = 0;
    for (uint32_t i = lo; i < hi; i++) {
      const uint8_t *p = pk + 32ull * i;
      if (last_pk && std::memcmp(p, last_pk, 32) == 0) {
        slots_out[i] = last_slot;
        if (last_slot == UINT32_MAX) {
          miss++;
          mb[(size_t)part * parts + last_q].push_back(i);
        }
        continue;
      }
      std::memcpy(key + 1, p, 32);
      last_slot = slots_out[i] = d.kindex.find(key);
      last_pk = p;
      if (last_slot == UINT32_MAX) {
        miss++;
        last_q = key_part(key);
        mb[(size_t)part * parts + last_q].push_back(i);
      } else {
        seen[last_slot] = 1;
      }
    }
    misses[part] = miss;
  };
  if (parts > 1) tmh::parallel_for_n(parts, kParts, lookup);
  else lookup(0);
  uint32_t n_miss = 0;
  for (uint32_t t = 0; t < parts; t++) n_miss += misses[t];
  // 2) pin every key found to this batch (epoch) before any miss may evict
  uint32_t distinct = 0;
  for (uint32_t slot = 0; slot < d.kcap; slot++) {
    bool hit = false;
    for (uint32_t t = 0; t < parts && !hit; t++) hit = d.kseen[(size_t)t * d.kcap + slot] != 0;
    if (!hit) continue;
    d.kslot_epoch[slot] = epoch;
    distinct++;
    d.klru.splice(d.klru.begin(), d.klru, d.kpos[slot]);
    d.khits++;
  }
  // tables built by earlier batches (possibly on other streams, not waited
  // for on the host) are complete before this batch's kernels read them
  (void)hipStreamWaitEvent(s, d.work_done, 0);
  if (n_miss == 0) return 0;
  // new keys may evict slots: let chunks still in flight on other lanes finish
  for (HostLane &l : d.lane)
    if (l.n && l.stream != s) {
      const hipError_t we = wait_stream(d, l.stream);
      if (we != hipSuccess) return wait_rc(we);
    }
  // 3) misses.  Distinct missing keys per key part q, in parallel (each
  //    part reads its lists in entry order, so the result is deterministic);
  //    then decide, before touching the index, whether the batch fits:
  //    bailing out after inserting keys whose tables were never built would
  //    leave stale entries behind.  (Serially over every missing entry this
  //    cost ~1.5 ms per C3 window, where ~60k of 67k entries name one of the
  //    window's 1,000 new keys.)
  struct MissPart {
    KeyIndex ix;                  // distinct new key -> ordinal in first / slot
    std::vector<uint32_t> first;  // entry of its first occurrence
    std::vector<uint32_t> slot;   // its cache slot
  };
  std::vector<MissPart> mp(parts);
  std::vector<uint32_t> ord(n);  // missing entry -> its key's ordinal in its part
  auto dedupe = [&](uint32_t q) {
    MissPart &m = mp[q];
    m.ix.init(16);
    uint8_t k[33];
    k[0] = sr ? 1 : 0;
    for (uint32_t p = 0; p < parts; p++)
      for (uint32_t i : mb[(size_t)p * parts + q]) {
        if (i > 0 && slots_out[i - 1] == UINT32_MAX && std::memcmp(pk + 32ull * i, pk + 32ull * (i - 1), 32) == 0) {
          ord[i] = ord[i - 1];  // a run of one key (same list: same key part, entry order)
          continue;
        }
        std::memcpy(k + 1, pk + 32ull * i, 32);
        uint32_t o = m.ix.find(k);
        if (o == UINT32_MAX) {
          o = (uint32_t)m.first.size();
          m.ix.insert(k, o);
          m.first.push_back(i);
        }
        ord[i] = o;
      }
  };
  if (parts > 1) tmh::parallel_for_n(parts, kParts, dedupe);
  else dedupe(0);
  for (uint32_t q = 0; q < parts; q++) distinct += (uint32_t)mp[q].first.size();
  if (distinct > d.kcap) return 1;
  uint8_t key[33];
  key[0] = sr ? 1 : 0;
  //    then give each new key a slot (LRU victims are never keys of this
  //    batch: every key found above is pinned to this epoch)
  for (uint32_t q = 0; q < parts; q++) {
    MissPart &m = mp[q];
    m.slot.resize(m.first.size());
    for (size_t t = 0; t < m.first.size(); t++) {
      const uint32_t i = m.first[t];
      std::memcpy(key + 1, pk + 32ull * i, 32);
      uint32_t slot;
      if (d.kindex.size() < d.kcap && d.klru.size() < d.kcap) {
        slot = (uint32_t)d.klru.size();
        d.klru.push_front(slot);
      } else {
        slot = d.klru.back();  // least recently used; never one pinned by this batch
        d.kindex.erase(d.kslot_key[slot].data());
        d.klru.splice(d.klru.begin(), d.klru, d.kpos[slot]);
      }
      d.kpos[slot] = d.klru.begin();
      std::memcpy(d.kslot_key[slot].data(), key, 33);
      d.kslot_epoch[slot] = epoch;
      d.kindex.insert(key, slot);
      m.slot[t] = slot;
      miss_idx.push_back(i);
      miss_slot.push_back(slot);
      d.kmisses++;
    }
  }
  //    and every missing entry its key's slot
  for (uint32_t q = 0; q < parts; q++) {
    const MissPart &m = mp[q];
    for (uint32_t p = 0; p < parts; p++)
      for (uint32_t i : mb[(size_t)p * parts + q]) slots_out[i] = m.slot[ord[i]];
  }
  const uint32_t m = (uint32_t)miss_idx.size();
  if (m) {
    // keys, slots, then the row-base scratch of the two-launch build
    const size_t soff = (32ull * m + 15) & ~size_t(15), boff = (soff + 4ull * m + 15) & ~size_t(15);
    const size_t bytes = boff + tmv::key_build_scratch(m);
    const size_t hbytes = soff + 4ull * m;
    // the previous build's copy must have left the staging before it is
    // rewritten (or regrown); its kernel need not have finished
    if (d.kbuild_copied && (e = wait_event(d, d.kbuild_copied)) != hipSuccess) return wait_rc(e);
    if ((e = d.h_kbuild.ensure(hbytes, true)) != hipSuccess) { set_error("hipHostMalloc", e); return TMV_ERR_NOMEM; }
    if (bytes > d.d_kbuild.cap) {
      if ((e = wait_event(d, d.work_done)) != hipSuccess) return wait_rc(e);
      if ((e = d.d_kbuild.ensure(bytes, false)) != hipSuccess) { set_error("hipMalloc", e); return TMV_ERR_NOMEM; }
    }
    (void)hipStreamWaitEvent(s, d.work_done, 0);
    uint8_t *h = static_cast<uint8_t *>(d.h_kbuild.ptr);
    for (uint32_t t = 0; t < m; t++) std::memcpy(h + 32ull * t, pk + 32ull * miss_idx[t], 32);
    std::memcpy(h + soff, miss_slot.data(), 4ull * m);
    if ((e = hipMemcpyAsync(d.d_kbuild.ptr, h, soff + 4ull * m, hipMemcpyHostToDevice, s)) != hipSuccess) {
      set_error("hipMemcpyAsync(keys)", e);
      return TMV_ERR_LAUNCH;
    }
    if (!d.kbuild_copied && (e = hipEventCreateWithFlags(&d.kbuild_copied, hipEventDisableTiming)) != hipSuccess) {
      d.kbuild_copied = nullptr;
      set_error("hipEventCreate", e);
      return TMV_ERR_NO_DEVICE;
    }
    (void)hipEventRecord(d.kbuild_copied, s);
    uint8_t *dk = static_cast<uint8_t *>(d.d_kbuild.ptr);
    if ((e = tmv::launch_key_build(sr, dk, reinterpret_cast<uint32_t *>(dk + soff), m, d.kt,
                                   reinterpret_cast<tmv::fe *>(dk + boff), s)) != hipSuccess) {
      set_error("key-table build launch", e);
      return TMV_ERR_LAUNCH;
    }
    // no host wait: this stream's kernels follow the build in order, later
    // batches on other streams wait on work_done (above), the next build
    // waits for kbuild_copied before reusing the staging
    (void)hipEventRecord(d.work_done, s);
  }
  return 0;
}

// The workspace of stream s, big enough for n entries, with this launch
// ordered after the previous user of that workspace.  Caller holds d.mu.
static Workspace *reserve_work(Device &d, uint32_t n, bool mixed, hipStream_t s, int *rc,
                               const tmv::MsmParams *mp = nullptr, const tmv::MsmParams *mp2 = nullptr) {
  auto &slot = d.ws[s];
  if (!slot) {
    slot = std::make_unique<Workspace>();
    hipError_t e = hipEventCreateWithFlags(&slot->done, hipEventDisableTiming);
    if (e != hipSuccess) { set_error("hipEventCreate", e); *rc = TMV_ERR_NO_DEVICE; d.ws.erase(s); return nullptr; }
  }
  Workspace &w = *slot;
  const size_t need = tmv::Ed25519Work::bytes(n);
  const size_t idx_need = 2ull * 4 * n + 64 + 4ull * 2 * kMaxStreamParts;  // + streamed mixed parts' cursors
  const size_t msm_need = mp ? tmv::MsmWork::bytes(n, *mp) : 0;
  const size_t msm2_need = mp ? tmv::MsmWork::bytes(n, mp2 ? *mp2 : *mp) : 0;
  if (need > w.work.cap || (mixed && (need > w.work2.cap || idx_need > w.idx.cap)) || msm_need > w.msm.cap ||
      (mixed && msm2_need > w.msm2.cap)) {
    hipError_t e = wait_event(d, w.done);  // old buffers may still be in use
    if (e != hipSuccess) { *rc = wait_rc(e); return nullptr; }
    if ((e = w.work.ensure(need, false)) != hipSuccess) { set_error("hipMalloc(work)", e); *rc = TMV_ERR_NOMEM; return nullptr; }
    if (mixed) {
      if ((e = w.work2.ensure(need, false)) != hipSuccess) { set_error("hipMalloc(work2)", e); *rc = TMV_ERR_NOMEM; return nullptr; }
      if ((e = w.idx.ensure(idx_need, false)) != hipSuccess) { set_error("hipMalloc(idx)", e); *rc = TMV_ERR_NOMEM; return nullptr; }
    }
    if (msm_need) {
      if ((e = w.msm.ensure(msm_need, false)) != hipSuccess) { set_error("hipMalloc(msm)", e); *rc = TMV_ERR_NOMEM; return nullptr; }
      if (mixed && (e = w.msm2.ensure(msm2_need, false)) != hipSuccess) {
        set_error("hipMalloc(msm2)", e);
        *rc = TMV_ERR_NOMEM;
        return nullptr;
      }
    }
  }
  *rc = 0;
  return &w;
}

// Stages the inputs of entries [e0, e1) of a streamed launch and enqueues
// their copy; *ready = an event recorded after it (stage_and_launch); 0 or < 0.
using PartFeeder = std::function<int(uint32_t e0, uint32_t e1, hipEvent_t *ready)>;

// Part boundaries of a streamed launch of n entries: whole groups, the first
// part g_stream_first entries, then g_stream_part each.
static std::vector<uint32_t> stream_parts(uint32_t n, uint32_t m) {
  return tmh::stream_part_bounds(n, m, g_stream_first, g_stream_part, g_stream_ramp != 0);
}

// feed: streamed launch, parts alternating between s and s2 (if given,
// joined back into s by `join` before the tail).
static int batch_check(Device &d, const LaunchOpts &o, bool sr, const uint8_t *pk, const uint8_t *sig,
                       const uint8_t *msg, const uint32_t *off, uint32_t n, uint8_t *out, hipStream_t s,
                       const PartFeeder *feed = nullptr, hipStream_t s2 = nullptr, hipEvent_t join = nullptr) {
  int rc;
  Workspace *ws = reserve_work(d, n, false, s, &rc, &o.p);
  if (!ws) return rc;
  tmv::Ed25519Work w = tmv::Ed25519Work::carve(ws->work.ptr, n);
  tmv::MsmWork mw = tmv::MsmWork::carve(ws->msm.ptr, n, o.p);
  hipError_t e;
  if (feed) {  // parts as their inputs land, then one tail
    const std::vector<uint32_t> b = stream_parts(n, o.p.m());
    const bool two = s2 && join && b.size() > 2;
    for (size_t j = 0; j + 1 < b.size(); j++) {
      hipEvent_t ready = nullptr;
      if ((rc = (*feed)(b[j], b[j + 1], &ready)) != 0) return rc;
      const hipStream_t t = two && (j & 1) ? s2 : s;
      if ((e = hipStreamWaitEvent(t, ready, 0)) != hipSuccess) { set_error("part wait", e); return TMV_ERR_LAUNCH; }
      e = tmv::launch_batch_check_part(sr, pk, sig, msg, off, n, b[j], b[j + 1], d.d_btab_q, d.d_prefix, w, mw, o.p,
                                       o.seed[sr ? 1 : 0], out, t);
      if (e != hipSuccess) { set_error("batch check part launch", e); return TMV_ERR_LAUNCH; }
    }
    if (two && ((e = hipEventRecord(join, s2)) != hipSuccess || (e = hipStreamWaitEvent(s, join, 0)) != hipSuccess)) {
      set_error("part join", e);
      return TMV_ERR_LAUNCH;
    }
    e = tmv::launch_batch_check_tail(sr, pk, sig, n, d.d_btab_q, w, mw, o.p, o.seed[sr ? 1 : 0], out, s);
  } else {
    e = tmv::launch_batch_check(sr, pk, sig, msg, off, nullptr, nullptr, n, d.d_btab_q, d.d_prefix, w, mw, o.p,
                                o.seed[sr ? 1 : 0], out, s);
  }
  if (e != hipSuccess) { set_error("batch check launch", e); return TMV_ERR_LAUNCH; }
  ws->group_ok[0] = mw.group_ok;
  ws->group_ok[1] = nullptr;
  ws->sub_ok[0] = o.p.sub ? mw.sub_ok : nullptr;
  ws->sub_ok[1] = nullptr;
  ws->groups = (n + o.p.m() - 1) >> o.p.m_log2;
  ws->m_log2 = ws->m_log2_sr = o.p.m_log2;
  ws->n = n;
  ws->counts = nullptr;
  ws->loc[0] = tmv::locate_enabled(n, o.p) ? mw.loc_count : nullptr;
  ws->loc[1] = nullptr;
  (void)hipEventRecord(ws->done, s);
  return 0;
}

// Streamed mixed ed25519 + sr25519 chunk (SURVEY 8(a) rows 7 / G-I with
// crypto/batch/batch.go:11-21's mixed batches): the inputs land part by part
// (feed), each part is split by key kind on the device into the two kinds'
// work-slot lists at bases the host knows (it counts each part's kinds from
// the caller's kind array), and each kind's pipeline runs the throughput
// stages of the groups the parts so far complete -- the ed25519 pipeline on
// s, the sr25519 one on s2 -- then one tail per kind (Horner, fallback).  The
// same kernels and the same validity vector as the unstreamed mixed launch;
// only the part schedule differs.
static int mixed_check_streamed(Device &d, const LaunchOpts &o_in, const uint8_t *kind_h, const uint8_t *kind_d,
                                const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *off,
                                uint32_t n, uint8_t *out, hipStream_t s, hipStream_t s2, hipEvent_t join,
                                std::vector<hipEvent_t> &split_ev, const PartFeeder &feed) {
  LaunchOpts o = o_in;
  o.p_ed = o_in.p_ed_streamed;
  int rc;
  Workspace *ws = reserve_work(d, n, true, s, &rc, &o.p_ed, &o.p);
  if (!ws) return rc;
  if (!s2 || !join) s2 = s;  // no helper stream, or no event to join it back: one stream (as batch_check)
  tmv::Ed25519Work w_ed = tmv::Ed25519Work::carve(ws->work.ptr, n);
  tmv::Ed25519Work w_sr = tmv::Ed25519Work::carve(ws->work2.ptr, n);
  // workspaces carved for n slots per kind (the kinds' counts are known only
  // part by part); the pipelines' B point sits at slot 2n of each
  tmv::MsmWork m_ed = tmv::MsmWork::carve(ws->msm.ptr, n, o.p_ed);
  tmv::MsmWork m_sr = tmv::MsmWork::carve(ws->msm2.ptr, n, o.p);
  uint32_t *ib = static_cast<uint32_t *>(ws->idx.ptr);
  uint32_t *counts = ib, *idx_ed = ib + 16, *idx_sr = ib + 16 + n, *cursor = ib + 16 + 2ull * n;
  // parts: the one-kind schedule (a short first part), at most kMaxStreamParts
  const std::vector<uint32_t> b =
      tmh::mixed_part_bounds(n, g_stream_first, g_stream_part, g_stream_ramp != 0, kMaxStreamParts);
  const size_t parts = b.size() - 1;
  hipError_t e;
  if ((e = hipMemsetAsync(ib, 0, 64, s)) != hipSuccess ||
      (e = hipMemsetAsync(cursor, 0, 8ull * parts, s)) != hipSuccess) {
    set_error("hipMemsetAsync", e);
    return TMV_ERR_LAUNCH;
  }
  while (split_ev.size() < parts) {
    hipEvent_t ev;
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) {
      set_error("hipEventCreate", e);
      return TMV_ERR_NO_DEVICE;
    }
    split_ev.push_back(ev);
  }
  const uint32_t g_ed = o.p_ed.m(), g_sr = o.p.m();  // group sizes
  uint32_t base_ed = 0, base_sr = 0, done_ed = 0, done_sr = 0;  // slots assigned / slots launched
  for (size_t j = 0; j < parts; j++) {
    const uint32_t a = b[j], z = b[j + 1];
    hipEvent_t ready = nullptr;
    if ((rc = feed(a, z, &ready)) != 0) return rc;
    uint32_t c_ed = 0, c_sr = 0;
    for (uint32_t i = a; i < z; i++) {
      c_ed += kind_h[i] == TMV_KIND_ED25519;
      c_sr += kind_h[i] == TMV_KIND_SR25519;
    }
    if ((e = hipStreamWaitEvent(s, ready, 0)) != hipSuccess) { set_error("part wait", e); return TMV_ERR_LAUNCH; }
    if ((e = tmv::launch_partition_range(kind_d, a, z, base_ed, base_sr, cursor + 2 * j, counts, idx_ed, idx_sr, out,
                                         s)) != hipSuccess ||
        (e = hipEventRecord(split_ev[j], s)) != hipSuccess) {
      set_error("part partition", e);
      return TMV_ERR_LAUNCH;
    }
    base_ed += c_ed;
    base_sr += c_sr;
    const bool last = j + 1 == parts;
    // slots of whole groups now assigned (the last part: every slot)
    const uint32_t hi_ed = last ? base_ed : base_ed / g_ed * g_ed, hi_sr = last ? base_sr : base_sr / g_sr * g_sr;
    if (hi_ed > done_ed) {
      e = tmv::launch_batch_check_part_idx(false, pk, sig, msg, off, idx_ed, n, done_ed, hi_ed, d.d_btab_q, d.d_prefix,
                                           w_ed, m_ed, o.p_ed, o.seed[0], out, s);
      if (e != hipSuccess) { set_error("mixed part launch", e); return TMV_ERR_LAUNCH; }
      done_ed = hi_ed;
    }
    if (hi_sr > done_sr) {
      if ((e = hipStreamWaitEvent(s2, split_ev[j], 0)) != hipSuccess) { set_error("part wait", e); return TMV_ERR_LAUNCH; }
      e = tmv::launch_batch_check_part_idx(true, pk, sig, msg, off, idx_sr, n, done_sr, hi_sr, d.d_btab_q, d.d_prefix,
                                           w_sr, m_sr, o.p, o.seed[1], out, s2);
      if (e != hipSuccess) { set_error("mixed part launch", e); return TMV_ERR_LAUNCH; }
      done_sr = hi_sr;
    }
  }
  // the tails: ed25519 on s, sr25519 on s2 (after its last partition), joined into s
  if ((e = hipStreamWaitEvent(s2, split_ev[parts - 1], 0)) != hipSuccess) { set_error("part wait", e); return TMV_ERR_LAUNCH; }
  if ((e = tmv::launch_batch_check_tail_idx(true, pk, sig, idx_sr, base_sr, d.d_btab_q, w_sr, m_sr, o.p, o.seed[1], out,
                                            s2)) != hipSuccess ||
      (e = tmv::launch_batch_check_tail_idx(false, pk, sig, idx_ed, base_ed, d.d_btab_q, w_ed, m_ed, o.p_ed, o.seed[0],
                                            out, s)) != hipSuccess) {
    set_error("mixed tail launch", e);
    return TMV_ERR_LAUNCH;
  }
  if (s2 != s && ((e = hipEventRecord(join, s2)) != hipSuccess || (e = hipStreamWaitEvent(s, join, 0)) != hipSuccess)) {
    set_error("part join", e);
    return TMV_ERR_LAUNCH;
  }
  ws->group_ok[0] = m_ed.group_ok;
  ws->group_ok[1] = m_sr.group_ok;
  ws->sub_ok[0] = o.p_ed.sub ? m_ed.sub_ok : nullptr;
  ws->sub_ok[1] = o.p.sub ? m_sr.sub_ok : nullptr;
  ws->groups = (base_ed + g_ed - 1) / g_ed;
  ws->m_log2 = o.p_ed.m_log2;
  ws->m_log2_sr = o.p.m_log2;
  ws->n = n;
  ws->counts = counts;
  ws->loc[0] = tmv::locate_enabled(base_ed, o.p_ed) ? m_ed.loc_count : nullptr;
  ws->loc[1] = tmv::locate_enabled(base_sr, o.p) ? m_sr.loc_count : nullptr;
  (void)hipEventRecord(ws->done, s);
  return 0;
}

static int launch_sr25519(Device &d, const LaunchOpts &o, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                          const uint32_t *off, uint32_t n, int8_t *status, hipStream_t s) {
  if (o.batch_eq) return batch_check(d, o, true, pk, sig, msg, off, n, reinterpret_cast<uint8_t *>(status), s);
  int rc;
  Workspace *ws = reserve_work(d, n, false, s, &rc);
  if (!ws) return rc;
  tmv::Ed25519Work w = tmv::Ed25519Work::carve(ws->work.ptr, n);
  hipError_t e = tmv::launch_sr25519_verify_quad(pk, sig, msg, off, n, d.d_btab_q, d.d_prefix, w, status, s);
  if (e != hipSuccess) { set_error("sr25519 launch", e); return TMV_ERR_LAUNCH; }
  (void)hipEventRecord(ws->done, s);
  return 0;
}

static int launch_mixed(Device &d, const LaunchOpts &o, const uint8_t *kind, const uint8_t *pk, const uint8_t *sig,
                        const uint8_t *msg, const uint32_t *off, uint32_t n, int8_t *status, hipStream_t s) {
  int rc;
  Workspace *ws = reserve_work(d, n, true, s, &rc, o.batch_eq ? &o.p_ed : nullptr, o.batch_eq ? &o.p : nullptr);
  if (!ws) return rc;
  tmv::Ed25519Work w1 = tmv::Ed25519Work::carve(ws->work.ptr, n);
  tmv::Ed25519Work w2 = tmv::Ed25519Work::carve(ws->work2.ptr, n);
  uint32_t *ib = static_cast<uint32_t *>(ws->idx.ptr);
  uint32_t *counts = ib, *idx_ed = ib + 16, *idx_sr = ib + 16 + n;
  hipError_t e;
  if (o.batch_eq) {
    tmv::MsmWork m1 = tmv::MsmWork::carve(ws->msm.ptr, n, o.p_ed);
    tmv::MsmWork m2 = tmv::MsmWork::carve(ws->msm2.ptr, n, o.p);
    read_env();
    tmv::KindStreams &ks = ws->kinds;
    if (!ks.helper) {
      if (hipStreamCreateWithFlags(&ks.helper, hipStreamNonBlocking) != hipSuccess) ks.helper = nullptr;
      if (hipEventCreateWithFlags(&ks.fork, hipEventDisableTiming) != hipSuccess) ks.fork = nullptr;
      if (hipEventCreateWithFlags(&ks.join, hipEventDisableTiming) != hipSuccess) ks.join = nullptr;
    }
    e = tmv::launch_mixed_batch_check(kind, pk, sig, msg, off, n, d.d_btab_q, d.d_prefix, w1, w2, m1, m2, o.p_ed,
                                      o.p, o.seed[0], o.seed[1], counts, idx_ed, idx_sr, status, s,
                                      &ks);
    ws->group_ok[0] = m1.group_ok;
    ws->group_ok[1] = m2.group_ok;
    ws->sub_ok[0] = o.p_ed.sub ? m1.sub_ok : nullptr;
    ws->sub_ok[1] = o.p.sub ? m2.sub_ok : nullptr;
    ws->groups = o.p_ed.groups;
    ws->m_log2 = o.p_ed.m_log2;
    ws->m_log2_sr = o.p.m_log2;
    ws->n = n;
    ws->counts = counts;
    ws->loc[0] = tmv::locate_enabled(n, o.p_ed) ? m1.loc_count : nullptr;
    ws->loc[1] = tmv::locate_enabled(n, o.p) ? m2.loc_count : nullptr;
  } else {
    e = tmv::launch_mixed_verify(kind, pk, sig, msg, off, n, d.d_btab_q, d.d_prefix, w1, w2, counts, idx_ed, idx_sr,
                                 status, s);
  }
  if (e != hipSuccess) { set_error("mixed launch", e); return TMV_ERR_LAUNCH; }
  (void)hipEventRecord(ws->done, s);
  return 0;
}

static int launch_cached(Device &d, bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                         const uint32_t *off, const uint32_t *slots, uint32_t n, uint8_t *out, hipStream_t s) {
  int rc;
  Workspace *ws = reserve_work(d, n, false, s, &rc);
  if (!ws) return rc;
  tmv::Ed25519Work w = tmv::Ed25519Work::carve(ws->work.ptr, n);
  read_env();
  hipError_t e = tmv::launch_verify_cached(sr, pk, sig, msg, off, slots, n, d.kt, d.d_bcomb, d.d_prefix, w, out,
                                           g_cached_fused_max, s);
  if (e != hipSuccess) { set_error("cached verify launch", e); return TMV_ERR_LAUNCH; }
  (void)hipEventRecord(ws->done, s);
  return 0;
}

// Key-merged batch equation over a key-ordered batch (msm.h).
static int launch_key_merged(Device &d, const LaunchOpts &o, bool sr, const uint8_t *pk, const uint8_t *sig,
                             const uint8_t *msg, const uint32_t *off, const uint32_t *slots, tmv::KeyRuns runs,
                             uint32_t n, uint8_t *out, hipStream_t s) {
  int rc;
  Workspace *ws = reserve_work(d, n, false, s, &rc, &o.p);
  if (!ws) return rc;
  tmv::Ed25519Work w = tmv::Ed25519Work::carve(ws->work.ptr, n);
  tmv::MsmWork mw = tmv::MsmWork::carve(ws->msm.ptr, n, o.p);
  hipError_t e = tmv::launch_key_merged_check(sr, pk, sig, msg, off, slots, runs, n, d.kt, d.d_bcomb, d.d_prefix, w,
                                              mw, o.p, o.seed[sr ? 1 : 0], out, s);
  if (e != hipSuccess) { set_error("key-merged check launch", e); return TMV_ERR_LAUNCH; }
  ws->group_ok[0] = mw.group_ok;
  ws->group_ok[1] = nullptr;
  ws->sub_ok[0] = ws->sub_ok[1] = nullptr;
  ws->groups = o.p.groups;
  ws->m_log2 = ws->m_log2_sr = o.p.m_log2;
  ws->n = n;
  ws->counts = nullptr;
  ws->loc[0] = ws->loc[1] = nullptr;  // the key-cached comb fallback checks every entry of a failing group
  (void)hipEventRecord(ws->done, s);
  return 0;
}

// Enqueue ed25519 verification of n device-resident entries on stream s.
// Caller holds d.mu.  Chooses the quad or single-lane kernel.
static int launch_ed25519(Device &d, const LaunchOpts &o, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                          const uint32_t *off, uint32_t n, uint8_t *valid, hipStream_t s) {
  if (o.batch_eq) return batch_check(d, o, false, pk, sig, msg, off, n, valid, s);
  read_env();
  const bool quad = g_kernel_override == 1 || (g_kernel_override == -1 && n <= kQuadMax);
  hipError_t e;
  if (!quad) {
    e = tmv::launch_ed25519_verify(pk, sig, msg, off, n, d.d_btable, valid, s);
    if (e != hipSuccess) { set_error("k_ed25519_verify launch", e); return TMV_ERR_LAUNCH; }
    return 0;
  }
  int rc;
  Workspace *ws = reserve_work(d, n, false, s, &rc);
  if (!ws) return rc;
  tmv::Ed25519Work w = tmv::Ed25519Work::carve(ws->work.ptr, n);
  e = tmv::launch_ed25519_verify_quad(pk, sig, msg, off, n, d.d_btab_q, w, valid, s);
  if (e != hipSuccess) { set_error("k_ed25519_verify_quad launch", e); return TMV_ERR_LAUNCH; }
  (void)hipEventRecord(ws->done, s);
  return 0;
}

static uint32_t mixed_stream_chunk(size_t free_bytes);

extern "C" {

int tmv_kernel_timing(tmv_ctx *ctx, int enable) {
  if (!ctx) { set_error("null context"); return TMV_ERR_ARG; }
  tmv::ktimer::set(enable != 0);
  return 0;
}

int tmv_kernel_timing_read(tmv_ctx *ctx, const char *kernel, double *total_ms, uint64_t *launches) {
  if (!ctx || !kernel || !total_ms || !launches) { set_error("null argument"); return TMV_ERR_ARG; }
  tmv::ktimer::Kernel k;
  if (!strcmp(kernel, "k_msm_accum")) k = tmv::ktimer::kAccum;
  else if (!strcmp(kernel, "k_msm_wpart")) k = tmv::ktimer::kWpart;
  else if (!strcmp(kernel, "k_prep_fused")) k = tmv::ktimer::kPrep;
  else { set_error("unknown timed kernel"); return TMV_ERR_ARG; }
  *total_ms = 0;
  *launches = 0;
  const int e = tmv::ktimer::read(k, total_ms, launches);
  if (e) { set_error("hipEventElapsedTime", (hipError_t)e); return TMV_ERR_LAUNCH; }
  return 0;
}

const char *tmv_last_error(void) { return g_last_error.c_str(); }
void tmv_internal_set_error(const char *msg) { g_last_error = msg ? msg : ""; }

// Test aids (tests/test_failure_handling.py): inject getrandom failures and
// draw one weights key the way every batch-equation launch does.
void tmv_internal_random_fault(int err, int count) {
  g_rand_fault_err = err;
  g_rand_fault_count = count;
}
// Test aid: switches the engine's tests set on paths that random inputs
// almost never reach.  "half_scalars" = 1 (the product), 0 (every entry's
// per-entry check on the full-k chain) or 2 (every third entry).  Returns 0,
// or TMV_ERR_ARG for an unknown name.  Never called by the Go shim.
int tmv_internal_option(const char *name, int64_t value) {
  if (name && !strcmp(name, "half_scalars")) {
    tmv::set_half_scalar_mode((int)value);
    return 0;
  }
  set_error("unknown internal option");
  return TMV_ERR_ARG;
}
// Test build counters (-DTMV_CHECKS, tools/build_checks.sh): out[0] joins
// k_msm_accum named, out[1] joins k_msm_join_list did, out[2] buckets with
// entries whose sum was never written; reset != 0 zeroes them.  Returns 0,
// or TMV_ERR_ARG in a product build (no counters compiled in).
int tmv_internal_checks(uint32_t *out3, int reset) {
  if (!out3) { set_error("null argument"); return TMV_ERR_ARG; }
  if (!tmv::read_checks(out3, reset != 0)) {
    set_error("not a TMV_CHECKS build, or the device read failed");
    return TMV_ERR_ARG;
  }
  return 0;
}
int64_t tmv_internal_mixed_stream_chunk(uint64_t free_bytes) {
  read_env();
  return mixed_stream_chunk((size_t)free_bytes);
}
int tmv_internal_draw_key(uint8_t *out32) {
  if (!out32) { set_error("null argument"); return TMV_ERR_ARG; }
  return draw_weight_key(out32);
}

tmv_ctx *tmv_open(uint32_t device_mask) { return tmv_open_logical(device_mask, 1); }

tmv_ctx *tmv_open_logical(uint32_t device_mask, int logical) {
  release_leaked_pins();
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    set_error(e != hipSuccess ? std::string("hipGetDeviceCount: ") + hipGetErrorString(e)
                              : std::string("no HIP device visible"));
    return nullptr;
  }
  // logical > 1 (test aid, tmv_open_logical only): each selected GPU joins the
  // context as that many devices -- own streams, lanes, workspaces and key
  // cache -- so the multi-device shard / launch / harvest path of run_batch
  // runs on real streams on a one-GPU box.  Device-pointer entry points name
  // a GPU by its HIP id and reach its first logical device.
  logical = std::max(1, std::min(8, logical));
  if (logical > 1)
    fprintf(stderr, "tmverify: TEST AID tmv_open_logical: every GPU opened as %d logical devices\n", logical);
  auto ctx = std::make_unique<tmv_ctx>();
  for (int i = 0; i < count && i < 32; i++) {
    if (device_mask != 0 && !(device_mask & (1u << i))) continue;
    for (int k = 0; k < logical; k++) {
      auto d = std::make_unique<Device>();
      d->id = i;
      if (init_device(*d) != 0) {
        tmv_close(ctx.release());
        return nullptr;
      }
      ctx->devs.push_back(std::move(d));
    }
  }
  if (ctx->devs.empty()) {
    set_error("device_mask selects no visible device");
    return nullptr;
  }
  return ctx.release();
}

void tmv_close(tmv_ctx *ctx) {
  if (!ctx) return;
  for (auto &d : ctx->devs) {  // drain the healthy devices first, so their leaked ranges are released
    if (d->faulted) continue;
    (void)hipSetDevice(d->id);
    for (HostLane &l : d->lane) {
      if (l.stream) (void)hipStreamSynchronize(l.stream);
      if (l.copy) (void)hipStreamSynchronize(l.copy);
    }
  }
  release_leaked_pins();
  for (auto &d : ctx->devs) {
    (void)hipSetDevice(d->id);
    if (d->faulted) continue;  // work still running on its buffers: leak them rather than free them under it
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    for (HostLane &l : d->lane) {
      if (l.stream) (void)hipStreamSynchronize(l.stream);
      if (l.copy) (void)hipStreamSynchronize(l.copy);
      for (hipEvent_t ev : l.part_ready) (void)hipEventDestroy(ev);
      l.part_ready.clear();
      for (hipEvent_t ev : l.part_split) (void)hipEventDestroy(ev);
      l.part_split.clear();
      if (l.copy) (void)hipStreamDestroy(l.copy);
      l.copy = nullptr;
      if (l.helper) (void)hipStreamSynchronize(l.helper);
      if (l.helper) (void)hipStreamDestroy(l.helper);
      if (l.join) (void)hipEventDestroy(l.join);
      l.helper = nullptr;
      l.join = nullptr;
      l.d_in.release();
      l.d_out.release();
      l.h_in.release();
      l.h_out.release();
    }
    for (auto &kv : d->ws) {
      if (kv.second->done) (void)hipEventSynchronize(kv.second->done);
      kv.second->work.release();
      kv.second->work2.release();
      kv.second->idx.release();
      kv.second->msm.release();
      kv.second->msm2.release();
      kv.second->gather.release();
      if (kv.second->done) (void)hipEventDestroy(kv.second->done);
      tmv::KindStreams &ks = kv.second->kinds;
      if (ks.helper) (void)hipStreamSynchronize(ks.helper);
      if (ks.fork) (void)hipEventDestroy(ks.fork);
      if (ks.join) (void)hipEventDestroy(ks.join);
      if (ks.helper) (void)hipStreamDestroy(ks.helper);
    }
    d->ws.clear();
    if (d->work_done) (void)hipEventSynchronize(d->work_done);  // the last key build (not waited for on the host)
    d->d_kbuild.release();
    d->h_kbuild.release();
    if (d->kt.tab) (void)hipFree(d->kt.tab);
    if (d->kt.ok) (void)hipFree(d->kt.ok);
    if (d->d_bcomb) (void)hipFree(d->d_bcomb);
    if (d->d_prefix) (void)hipFree(d->d_prefix);
    if (d->d_btab_q) (void)hipFree(d->d_btab_q);
    if (d->work_done) (void)hipEventDestroy(d->work_done);
    if (d->kbuild_copied) (void)hipEventDestroy(d->kbuild_copied);
    if (d->d_btable) (void)hipFree(d->d_btable);
    for (int l = 0; l < kLanes; l++)
      if (d->lane[l].stream) (void)hipStreamDestroy(d->lane[l].stream);
    if (d->stream) (void)hipStreamDestroy(d->stream);
  }
  delete ctx;
}

int tmv_num_devices(const tmv_ctx *ctx) { return ctx ? (int)ctx->devs.size() : 0; }

}  // extern "C"

enum class Scheme { Ed25519, Sr25519, Mixed, Ed25519Cached, Sr25519Cached };

// Messages built on the device from vote templates (tmv_verify_votes):
// the host sends the votes and the template table + blob; msg_off still
// holds the host-computed offsets of the messages the device will write.
struct VoteSrc {
  const tmv_vote *votes;
  const uint8_t *tab;  // n_tmpl VoteTab, then the template bytes
  size_t tab_bytes, blob_at;
};

// Stage one contiguous shard [lo, hi) to device d and launch; does not sync.
// Layout: pk | sig | off | msg | kind or key slots | votes | templates | key
// runs | key order (16-B aligned pieces).  Key-cached batches resolve their
// slots first; the key-merged batch equation gets the key order of the
// entries (a counting sort by slot) and the runs of one key inside a group,
// and its kernels read the entries through that order.
static int stage_and_launch(tmv_ctx *ctx, uint32_t flags, Device &d, HostLane &ln, Scheme sch, const uint8_t *kind,
                            const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off,
                            uint32_t lo, uint32_t hi, const VoteSrc *vs) {
  const uint32_t n = hi - lo;
  const size_t mbytes = (size_t)msg_off[hi] - msg_off[lo];
  Layout L(n, mbytes);
  bool cached = sch == Scheme::Ed25519Cached || sch == Scheme::Sr25519Cached;
  const bool sr = sch == Scheme::Sr25519Cached || sch == Scheme::Sr25519;
  hipError_t e = hipSetDevice(d.id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  EngineTimer tm;
  if (cached) {
    d.slots.resize(n);
    const int kr = resolve_keys(d, sr, pk + 32ull * lo, n, d.slots.data(), ln.stream);
    if (kr < 0) return kr;
    if (kr == 1) {  // more distinct keys than the cache holds: uncached path
      sch = sr ? Scheme::Sr25519 : Scheme::Ed25519;
      cached = false;
    }
  }
  tm.mark("keys", n);
  LaunchOpts o = make_opts(ctx, flags, n, cached, sch == Scheme::Ed25519 || sch == Scheme::Ed25519Cached);
  if (o.err) return o.err;
  // key-merged form: worth it while a group holds few keys (runs <= n / 2)
  bool merged = cached && o.batch_eq;
  uint32_t distinct = 0;
  const uint32_t kc = d.kcap;
  constexpr uint32_t kSortChunks = 16;
  if (merged) {  // per-chunk key histograms (parallel), for a stable counting sort
    d.key_count.assign((size_t)kSortChunks * kc, 0);
    const uint32_t *sl = d.slots.data();
    uint32_t *hist = d.key_count.data();
    tmh::parallel_for_n(kSortChunks, kSortChunks, [&](size_t c) {
      const uint32_t j0 = (uint32_t)((uint64_t)n * c / kSortChunks), j1 = (uint32_t)((uint64_t)n * (c + 1) / kSortChunks);
      uint32_t *hc = hist + c * kc;
      for (uint32_t j = j0; j < j1; j++) hc[sl[j]]++;
    });
    for (uint32_t k = 0; k < kc; k++) {
      uint32_t t = 0;
      for (uint32_t c = 0; c < kSortChunks; c++) t += hist[(size_t)c * kc + k];
      distinct += t != 0;
    }
    if ((uint64_t)distinct + o.p.groups > n / 2) merged = false;
  }
  if (cached && !merged) o.batch_eq = false;  // key-cached per-entry path
  read_env();
  const bool mixed_stream = sch == Scheme::Mixed && g_mixed_stream;
  if (g_stream && !cached && !vs && (sch == Scheme::Ed25519 || sch == Scheme::Sr25519 || mixed_stream) &&
      o.batch_eq && n > g_stream_first) {
    // streamed: stage and copy part by part, each part's kernels behind its
    // copy (mixed chunks: the kind bytes too, after the other inputs)
    const size_t kind_at = L.total, in_total = L.total + (mixed_stream ? align16(n) : 0);
    if ((e = ln.h_in.ensure(in_total, true)) != hipSuccess) { set_error("hipHostMalloc", e); return TMV_ERR_NOMEM; }
    if ((e = ln.d_in.ensure(in_total, false)) != hipSuccess) { set_error("hipMalloc", e); return TMV_ERR_NOMEM; }
    if ((e = ln.h_out.ensure(n, true)) != hipSuccess) { set_error("hipHostMalloc", e); return TMV_ERR_NOMEM; }
    if ((e = ln.d_out.ensure(n, false)) != hipSuccess) { set_error("hipMalloc", e); return TMV_ERR_NOMEM; }
    if (!ln.copy && (e = hipStreamCreateWithFlags(&ln.copy, hipStreamNonBlocking)) != hipSuccess) {
      ln.copy = nullptr;
      set_error("hipStreamCreate", e);
      return TMV_ERR_NO_DEVICE;
    }
    uint8_t *h = static_cast<uint8_t *>(ln.h_in.ptr), *dd = static_cast<uint8_t *>(ln.d_in.ptr);
    uint32_t *off = reinterpret_cast<uint32_t *>(h + L.off);
    const uint32_t base = msg_off[lo];
    size_t part = 0;
    if ((g_stream_two || mixed_stream) && !ln.helper) {
      if (hipStreamCreateWithFlags(&ln.helper, hipStreamNonBlocking) != hipSuccess) ln.helper = nullptr;
      else if (hipEventCreateWithFlags(&ln.join, hipEventDisableTiming) != hipSuccess) ln.join = nullptr;
    }
    bool pin_ok = g_register != 0;
    double pin_ms = 0;
    ln.unpin();
    // Caller pages pinned for direct DMA, per span (pk, sig, msg, kind): the
    // whole pages inside part 0's bytes, then at part 1 every whole page
    // inside the rest of the chunk's span, in one range (registering costs
    // ~2 us a range and unregistering ~4.5 us: a 2.56M call used to unpin 63
    // per-part ranges in 0.28 ms, and stage a sub-page tail per part and
    // span).  Only pages wholly inside the caller's span are registered, so
    // a neighbouring buffer's registration never collides; the bytes outside
    // the registered pages (part 0's head and tail, the chunk's last tail)
    // go through the lane's pinned staging, and so does a span whose range
    // cannot be registered (read-only, already registered), for the rest of
    // the chunk.
    constexpr uintptr_t kPage = 4096;
    tmh::SpanPins reg[4];  // host/stream_plan.h
    const uintptr_t span_end[4] = {(uintptr_t)(pk + 32ull * (lo + n)), (uintptr_t)(sig + 64ull * (lo + n)),
                                   mbytes ? (uintptr_t)(msg + msg_off[lo + n]) : 0,
                                   mixed_stream ? (uintptr_t)(kind + lo + n) : 0};
    const PartFeeder feed = [&](uint32_t a, uint32_t b, hipEvent_t *ready) -> int {
      for (uint32_t i = a; i <= b; i++) off[i] = msg_off[lo + i] - base;
      const size_t m0 = off[a], m1 = off[b];
      // per span: [dst offset, caller bytes, length]; [d0, d1) of it is
      // DMA'd from registered pages, the rest staged
      struct Span {
        size_t at;
        const uint8_t *src;
        size_t len;
        size_t d0, d1, cut;
      } sp[4] = {{L.pk + 32ull * a, pk + 32ull * (lo + a), 32ull * (b - a), 0, 0, 0},
                 {L.sig + 64ull * a, sig + 64ull * (lo + a), 64ull * (b - a), 0, 0, 0},
                 {L.msg + m0, msg + base + m0, m1 - m0, 0, 0, 0},
                 {kind_at + a, mixed_stream ? kind + lo + a : nullptr, mixed_stream ? (size_t)(b - a) : 0, 0, 0, 0}};
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < 4; k++) {
        Span &x = sp[k];
        tmh::SpanPins &r = reg[k];
        if (!pin_ok || r.failed || x.len < 4 * kPage) continue;
        const uintptr_t s0 = (uintptr_t)x.src, s1 = s0 + x.len;
        uintptr_t r0, r1;
        if (tmh::next_pin_range(r, s0, s1, span_end[k], kPage, &r0, &r1)) {
          if (hipHostRegister(reinterpret_cast<void *>(r0), r1 - r0, hipHostRegisterDefault) != hipSuccess) {
            (void)hipGetLastError();
            r.failed = true;  // stage this span for the rest of the chunk
            continue;
          }
          ln.pinned.push_back(reinterpret_cast<void *>(r0));
          tmh::commit_pin_range(r, r0, r1);
        }
        tmh::direct_piece(r, s0, s1, &x.d0, &x.d1, &x.cut);
      }
      pin_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      CopySpan cs[8];
      size_t ncs = 0;
      for (const Span &x : sp) {
        if (!x.len) continue;
        if (x.d1 == 0) {
          cs[ncs++] = {h + x.at, x.src, x.len};
          continue;
        }
        if (x.d0) cs[ncs++] = {h + x.at, x.src, x.d0};
        if (x.d1 < x.len) cs[ncs++] = {h + x.at + x.d1, x.src + x.d1, x.len - x.d1};
      }
      par_memcpy_spans(cs, ncs);
      if (part >= ln.part_ready.size()) {
        hipEvent_t ev;
        hipError_t ce = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (ce != hipSuccess) { set_error("hipEventCreate", ce); return TMV_ERR_NO_DEVICE; }
        ln.part_ready.push_back(ev);
      }
      hipEvent_t ev = ln.part_ready[part++];
      hipError_t ce;
      auto h2d = [&](size_t at, const void *src, size_t len) -> bool {
        if (!len) return true;
        if ((ce = hipMemcpyAsync(dd + at, src, len, hipMemcpyHostToDevice, ln.copy)) != hipSuccess) {
          set_error("hipMemcpyAsync(H2D)", ce);
          return false;
        }
        ctx->m_h2d += len;
        return true;
      };
      if (!h2d(L.off + 4ull * a, h + L.off + 4ull * a, 4ull * (b - a + 1))) return TMV_ERR_LAUNCH;
      for (int k = 0; k < 4; k++) {
        const Span &x = sp[k];
        bool ok;
        if (x.d1 == 0) {
          ok = h2d(x.at, h + x.at, x.len);
        } else {  // staged head, the locked middle (one DMA per locked range), staged tail
          const size_t cut = x.cut;
          ok = h2d(x.at, h + x.at, x.d0) && h2d(x.at + x.d0, x.src + x.d0, cut - x.d0) &&
               h2d(x.at + cut, x.src + cut, x.d1 - cut) && h2d(x.at + x.d1, h + x.at + x.d1, x.len - x.d1);
        }
        if (!ok) return TMV_ERR_LAUNCH;
      }
      if ((ce = hipEventRecord(ev, ln.copy)) != hipSuccess) {
        set_error("part event", ce);
        return TMV_ERR_LAUNCH;
      }
      *ready = ev;
      return 0;
    };
    tm.mark("stage", n);
    const int rc =
        mixed_stream
            ? mixed_check_streamed(d, o, kind + lo, dd + kind_at, dd + L.pk, dd + L.sig, dd + L.msg,
                                   reinterpret_cast<const uint32_t *>(dd + L.off), n,
                                   static_cast<uint8_t *>(ln.d_out.ptr), ln.stream, ln.helper,
                                   ln.join, ln.part_split, feed)
            : batch_check(d, o, sr, dd + L.pk, dd + L.sig, dd + L.msg, reinterpret_cast<const uint32_t *>(dd + L.off), n,
                          static_cast<uint8_t *>(ln.d_out.ptr), ln.stream, &feed, g_stream_two ? ln.helper : nullptr,
                          g_stream_two ? ln.join : nullptr);
    // an error after parts were enqueued: they still use the lane's buffers
    // and the caller's registered pages, so drain before returning
    auto drain = [&](int r) {
      const bool drained = wait_stream(d, ln.copy) == hipSuccess;
      if (ln.helper) (void)wait_stream(d, ln.helper);
      if (wait_stream(d, ln.stream) == hipSuccess && drained) ln.unpin();
      else ln.pinned.clear();  // copies may be in flight: leave the pages registered (see run_batch)
      return r;
    };
    if (rc != 0) return drain(rc);
    if (tm.on) fprintf(stderr, "[tmv_engine] pinning %9.3f ms (%zu ranges)\n", pin_ms, ln.pinned.size());
    tm.mark("parts staged + launched", n);
    // statuses through the lane's staging (a late DMA after a device
    // timeout must not land in caller memory the call no longer owns)
    if ((e = hipMemcpyAsync(ln.h_out.ptr, ln.d_out.ptr, n, hipMemcpyDeviceToHost, ln.stream)) != hipSuccess) {
      set_error("hipMemcpyAsync(D2H)", e);
      return drain(TMV_ERR_LAUNCH);
    }
    ctx->m_d2h += n;
    return 0;
  }
  const uint32_t G = merged ? o.p.groups : 0;
  const size_t kind_at = L.total;
  const size_t votes_at = L.total + (sch == Scheme::Mixed ? align16(n) : 0) + (cached ? align16(4ull * n) : 0);
  const size_t tab_at = votes_at + (vs ? align16(sizeof(tmv_vote) * n) : 0);
  const size_t runs_at = tab_at + (vs ? align16(vs->tab_bytes) : 0);
  const size_t run_cap = (size_t)distinct + G;  // key segments cut at group edges
  const size_t order_at = runs_at + align16(4ull * (2 * run_cap + 1 + G + 1));
  const size_t total = merged ? order_at + align16(4ull * n) : runs_at;
  if ((e = ln.h_in.ensure(total, true)) != hipSuccess) { set_error("hipHostMalloc", e); return TMV_ERR_NOMEM; }
  if ((e = ln.d_in.ensure(total, false)) != hipSuccess) { set_error("hipMalloc", e); return TMV_ERR_NOMEM; }
  if ((e = ln.h_out.ensure(n, true)) != hipSuccess) { set_error("hipHostMalloc", e); return TMV_ERR_NOMEM; }
  if ((e = ln.d_out.ensure(n, false)) != hipSuccess) { set_error("hipMalloc", e); return TMV_ERR_NOMEM; }
  uint8_t *h = static_cast<uint8_t *>(ln.h_in.ptr);
  uint32_t *off = reinterpret_cast<uint32_t *>(h + L.off);
  const uint32_t base = msg_off[lo];
  par_memcpy(h + L.pk, pk + 32ull * lo, 32ull * n);
  par_memcpy(h + L.sig, sig + 64ull * lo, 64ull * n);
  for (uint32_t i = 0; i <= n; i++) off[i] = msg_off[lo + i] - base;
  if (vs) {
    par_memcpy(h + votes_at, vs->votes + lo, sizeof(tmv_vote) * n);
    std::memcpy(h + tab_at, vs->tab, vs->tab_bytes);
  } else if (mbytes) {
    par_memcpy(h + L.msg, msg + base, mbytes);
  }
  if (sch == Scheme::Mixed) std::memcpy(h + kind_at, kind + lo, n);
  if (cached) std::memcpy(h + kind_at, d.slots.data(), 4ull * n);
  uint32_t n_runs = 0;
  if (merged) {
    // key order of the work slots: stable counting sort, chunks scattered in parallel
    uint32_t *hist = d.key_count.data();
    std::vector<uint32_t> key_start(kc + 1);
    uint32_t run = 0;
    for (uint32_t k = 0; k < kc; k++) {
      key_start[k] = run;
      for (uint32_t c = 0; c < kSortChunks; c++) {
        const uint32_t v = hist[(size_t)c * kc + k];
        hist[(size_t)c * kc + k] = run;
        run += v;
      }
    }
    key_start[kc] = run;
    uint32_t *order = reinterpret_cast<uint32_t *>(h + order_at);
    const uint32_t *sl = d.slots.data();
    tmh::parallel_for_n(kSortChunks, kSortChunks, [&](size_t c) {
      const uint32_t j0 = (uint32_t)((uint64_t)n * c / kSortChunks), j1 = (uint32_t)((uint64_t)n * (c + 1) / kSortChunks);
      uint32_t *cur = hist + c * kc;
      for (uint32_t j = j0; j < j1; j++) order[cur[sl[j]]++] = j;
    });
    // runs: key segments [key_start[k], key_start[k+1]) cut at group edges
    uint32_t *rlo = reinterpret_cast<uint32_t *>(h + runs_at);
    uint32_t *rslot = rlo + run_cap + 1;
    uint32_t *rg0 = rslot + run_cap;
    const uint32_t m = o.p.m();
    uint32_t g = 0;
    for (uint32_t k = 0; k < kc; k++) {
      uint32_t a0 = key_start[k];
      const uint32_t a1 = key_start[k + 1];
      while (a0 < a1) {
        while (g < G && (g << o.p.m_log2) <= a0) rg0[g++] = n_runs;
        rlo[n_runs] = a0;
        rslot[n_runs] = k;
        n_runs++;
        a0 = std::min(a1, (a0 / m + 1) * m);
      }
    }
    while (g < G) rg0[g++] = n_runs;
    rlo[n_runs] = n;
    rg0[G] = n_runs;
  }
  tm.mark("stage", n);
  // Small key-cached batches (the VerifyCommit latency path) skip both
  // copies: the fused kernel reads the pinned staging and writes the
  // statuses to pinned memory over PCIe (coherent host memory).
  const bool zero_copy = g_zero_copy && cached && !merged && !vs && n <= g_cached_fused_max && ln.h_in.dev &&
                         ln.h_out.dev;
  uint8_t *dd = static_cast<uint8_t *>(zero_copy ? ln.h_in.dev : ln.d_in.ptr);
  const uint32_t *doff = reinterpret_cast<uint32_t *>(dd + L.off);
  if (zero_copy) {
    // inputs are read in place
  } else if (vs) {  // everything but the message region, which the device writes
    if ((e = hipMemcpyAsync(dd, h, L.msg, hipMemcpyHostToDevice, ln.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(dd + L.total, h + L.total, total - L.total, hipMemcpyHostToDevice, ln.stream)) !=
            hipSuccess) {
      set_error("hipMemcpyAsync(H2D)", e);
      return TMV_ERR_LAUNCH;
    }
    ctx->m_h2d += L.msg + (total - L.total);
    const tmv::VoteTab *tab = reinterpret_cast<const tmv::VoteTab *>(dd + tab_at);
    if ((e = tmv::launch_vote_signbytes(reinterpret_cast<const tmv_vote *>(dd + votes_at), tab,
                                        dd + tab_at + vs->blob_at, doff, n, dd + L.msg, ln.stream)) != hipSuccess) {
      set_error("k_vote_signbytes", e);
      return TMV_ERR_LAUNCH;
    }
  } else if ((e = hipMemcpyAsync(ln.d_in.ptr, h, total, hipMemcpyHostToDevice, ln.stream)) != hipSuccess) {
    set_error("hipMemcpyAsync(H2D)", e);
    return TMV_ERR_LAUNCH;
  } else {
    ctx->m_h2d += total;
  }
  uint8_t *out = static_cast<uint8_t *>(zero_copy ? ln.h_out.dev : ln.d_out.ptr);
  const uint32_t *dslots = reinterpret_cast<const uint32_t *>(dd + kind_at);
  int rc;
  switch (sch) {
    case Scheme::Ed25519:
      rc = launch_ed25519(d, o, dd + L.pk, dd + L.sig, dd + L.msg, doff, n, out, ln.stream);
      break;
    case Scheme::Sr25519:
      rc = launch_sr25519(d, o, dd + L.pk, dd + L.sig, dd + L.msg, doff, n, reinterpret_cast<int8_t *>(out), ln.stream);
      break;
    case Scheme::Ed25519Cached:
    case Scheme::Sr25519Cached:
      if (merged) {
        const uint32_t *rlo = reinterpret_cast<const uint32_t *>(dd + runs_at);
        const tmv::KeyRuns runs{rlo, rlo + run_cap + 1, rlo + 2 * run_cap + 1,
                                reinterpret_cast<const uint32_t *>(dd + order_at), n_runs};
        rc = launch_key_merged(d, o, sr, dd + L.pk, dd + L.sig, dd + L.msg, doff, dslots, runs, n, out, ln.stream);
      } else {
        rc = launch_cached(d, sr, dd + L.pk, dd + L.sig, dd + L.msg, doff, dslots, n, out, ln.stream);
      }
      break;
    default:
      rc = launch_mixed(d, o, dd + kind_at, dd + L.pk, dd + L.sig, dd + L.msg, doff, n, reinterpret_cast<int8_t *>(out),
                        ln.stream);
  }
  if (rc != 0) return rc;
  if (zero_copy) return 0;
  if ((e = hipMemcpyAsync(ln.h_out.ptr, ln.d_out.ptr, n, hipMemcpyDeviceToHost, ln.stream)) != hipSuccess) {
    set_error("hipMemcpyAsync(D2H)", e);
    return TMV_ERR_LAUNCH;
  }
  ctx->m_d2h += n;
  return 0;
}

// Entries per streamed mixed chunk.  mixed_check_streamed carves both
// kinds' per-entry scratch and MSM workspaces for the whole chunk (the kinds'
// counts are known only part by part), ~20 KB per entry, and a lane's
// workspace only grows: the chunk is capped so that the host lanes' workspaces
// together take at most half of the device memory free at the call (3.7M
// entries on an idle MI355X; a smaller device gets smaller chunks instead of
// TMV_ERR_NOMEM).
static uint32_t mixed_stream_chunk(size_t free_bytes) {
  constexpr uint32_t kN = 1u << 20;
  const tmv::MsmParams p = tmv::MsmParams::make(kN, 6, 5);
  const double per_entry = (2.0 * tmv::Ed25519Work::bytes(kN) + 2.0 * tmv::MsmWork::bytes(kN, p)) / kN;
  const double fit = (double)free_bytes / 2.0 / (std::max<uint32_t>(1, g_host_lanes) * per_entry);
  const uint32_t c = (uint32_t)std::min<double>(g_stream_chunk, fit) & ~65535u;
  return std::max<uint32_t>(c, 65536u);
}

// Host-buffer batch: shard by contiguous index ranges over the context's
// devices, stage, launch, gather.  out gets 1 byte per entry.
static int run_batch(tmv_ctx *ctx, Scheme sch, const uint8_t *kind, const uint8_t *pk, const uint8_t *sig,
                     const uint8_t *msg, const uint32_t *msg_off, uint32_t n, uint8_t *out, uint32_t flags = 0,
                     const VoteSrc *vs = nullptr) {
  if (!ctx) { set_error("null context"); return TMV_ERR_ARG; }
  if (n == 0) return TMV_NOT_ALL;
  if (!pk || !sig || !msg_off || !out || (sch == Scheme::Mixed && !kind) ||
      (!msg && !vs && msg_off[n] != msg_off[0])) {
    set_error("null argument");
    return TMV_ERR_ARG;
  }
  read_env();
  if (leaked_pin_count()) release_leaked_pins();
  ctx->count_call(n);
  ctx->host_enter();
  struct HostTime {  // busy wall time of host-buffer calls into tmv_metrics, on every return
    tmv_ctx *c;
    uint32_t n;
    ~HostTime() { c->host_leave(n); }
  } host_time{ctx, n};
  // streamed batch-equation chunks are large (one pipeline, one tail each);
  // other paths alternate smaller chunks over the lanes
  const uint32_t per_dev = n / (uint32_t)ctx->devs.size();
  const bool streamable = g_stream && !vs && (sch == Scheme::Ed25519 || sch == Scheme::Sr25519) &&
                          !(flags & TMV_FLAG_PER_ENTRY) &&
                          ((flags & TMV_FLAG_BATCH_EQUATION) || (g_msm_min > 0 && per_dev >= g_msm_min));
  const bool mixed_batch_eq = sch == Scheme::Mixed && !vs && !(flags & TMV_FLAG_PER_ENTRY) &&
                              ((flags & TMV_FLAG_BATCH_EQUATION) || (g_msm_min > 0 && per_dev >= g_msm_min));
  const bool mixed_streamed = mixed_batch_eq && g_stream && g_mixed_stream;
  uint32_t chunk = streamable ? g_stream_chunk : (mixed_batch_eq ? g_mixed_chunk : g_host_chunk);
  if (mixed_streamed) {
    size_t free_b = 0, total_b = 0;
    if (hipSetDevice(ctx->devs[0]->id) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
      (void)hipGetLastError();
      free_b = 0;
    }
    chunk = free_b ? mixed_stream_chunk(free_b) : g_mixed_chunk;
  }
  const tmh::ShardPlan plan = tmh::plan_shards(n, (uint32_t)ctx->devs.size(), chunk);
  const uint32_t shards = plan.shards;
  // claim g_host_lanes lanes per device (devices in order, so concurrent
  // calls cannot deadlock); released on every return
  struct Claims {
    tmv_ctx *ctx;
    uint32_t nl, claimed = 0;
    std::vector<std::array<uint32_t, kLanes>> lane;
    ~Claims() {
      for (uint32_t s = 0; s < claimed; s++) {
        Device &d = *ctx->devs[s];
        {
          std::lock_guard<std::mutex> lk(d.mu);
          for (uint32_t j = 0; j < nl; j++) d.lane_busy[lane[s][j]] = false;
        }
        d.lane_cv.notify_all();
      }
    }
  } claims{ctx, std::min<uint32_t>(g_host_lanes, kLanes), 0, std::vector<std::array<uint32_t, kLanes>>(shards)};
  for (uint32_t s = 0; s < shards; s++) {
    Device &d = *ctx->devs[s];
    std::unique_lock<std::mutex> lk(d.mu);
    d.lane_cv.wait(lk, [&] {
      uint32_t free = 0;
      for (uint32_t l = 0; l < kLanes; l++) free += !d.lane_busy[l];
      return free >= claims.nl || d.faulted;
    });
    if (d.faulted) return faulted_rc(d);
    for (uint32_t l = 0, j = 0; l < kLanes && j < claims.nl; l++)
      if (!d.lane_busy[l]) {
        d.lane_busy[l] = true;
        claims.lane[s][j++] = l;
      }
    claims.claimed = s + 1;
  }
  EngineTimer tm;
  // chunk k of every shard, then chunk k + 1: the devices work side by side
  // (host/shard_run.h; the CPU test double runs the same order)
  int rc = tmh::run_shard_plan(
      plan, g_host_lanes,
      [&](uint32_t s, uint32_t lane, bool ok) -> int {
        Device &d = *ctx->devs[s];
        HostLane &ln = d.lane[claims.lane[s][lane]];
        if (ln.n == 0) return 0;  // this call is the lane's only writer
        (void)hipSetDevice(d.id);
        int r = 0;
        if (ok || !d.faulted) {  // the wait runs without the device lock
          const hipError_t e = wait_stream(d, ln.stream);
          if (e != hipSuccess) {
            if (e != hipErrorNotReady) set_error("hipStreamSynchronize", e);
            r = wait_rc(e);
          }
        }
        tm.mark("waited", ln.n);
        if (ok && r == 0) std::memcpy(out + ln.lo, ln.h_out.ptr, ln.n);
        tm.mark("copied out", ln.n);
        // the chunk's copies are done (its stream waited on every part's copy);
        // if they may not be (a failed or skipped wait), the caller's pages
        // stay registered and only the records are dropped: unregistering
        // under a DMA in flight, or later, after the caller freed the
        // memory, would be worse (include/tmverify.h, TMV_ERR_TIMEOUT)
        if (r == 0 && (ok || !d.faulted)) ln.unpin();
        else leak_pins(d.id, ln);  // released once its streams drain (release_leaked_pins)
        tm.mark("unpinned", ln.n);
        std::lock_guard<std::mutex> lk(d.mu);
        if (ok && r == 0 && ctx->stats) collect_stats(ctx, d, ln.stream);
        ln.n = 0;
        return r;
      },
      [&](uint32_t s, uint32_t lane, uint32_t c0, uint32_t c1) -> int {
        Device &d = *ctx->devs[s];
        HostLane &ln = d.lane[claims.lane[s][lane]];
        (void)hipSetDevice(d.id);
        std::lock_guard<std::mutex> lk(d.mu);  // key cache, device scratch, workspaces
        if (d.faulted) return faulted_rc(d);
        const int r = stage_and_launch(ctx, flags, d, ln, sch, kind, pk, sig, msg, msg_off, c0, c1, vs);
        if (r == 0) {
          ln.lo = c0;
          ln.n = c1 - c0;
        }
        return r;
      });
  tm.mark("synced", n);
  if (rc != 0) return rc;
  for (uint32_t i = 0; i < n; i++)
    if (out[i] != 1) return TMV_NOT_ALL;
  return TMV_ALL_VALID;
}

// Template table + blob for k_vote_signbytes, and the offsets of every
// vote's message (host-side sizing with the device's own length functions).
static int prepare_votes(const tmv_vote_template *tmpl, uint32_t n_tmpl, const tmv_vote *votes, uint32_t n,
                         std::vector<uint8_t> &tab, size_t &blob_at, std::vector<uint32_t> &off) {
  if ((!tmpl && n_tmpl) || (!votes && n)) { set_error("null argument"); return TMV_ERR_ARG; }
  std::vector<tmv::VoteTab> vt(n_tmpl);
  uint64_t blob = 0;
  for (uint32_t t = 0; t < n_tmpl; t++) {
    const tmv_vote_template &T = tmpl[t];
    if ((T.head_len && !T.head) || (T.block_len && !T.block) || (T.chain_len && !T.chain)) {
      set_error("null template segment");
      return TMV_ERR_ARG;
    }
    vt[t] = tmv::VoteTab{(uint32_t)blob, T.head_len, (uint32_t)(blob + T.head_len), T.block_len,
                         (uint32_t)(blob + T.head_len + T.block_len), T.chain_len};
    blob += (uint64_t)T.head_len + T.block_len + T.chain_len;
    if (blob > (1u << 30)) { set_error("vote templates too large"); return TMV_ERR_ARG; }
  }
  blob_at = align16(sizeof(tmv::VoteTab) * n_tmpl);
  tab.resize(blob_at + blob);
  if (n_tmpl) std::memcpy(tab.data(), vt.data(), sizeof(tmv::VoteTab) * n_tmpl);
  for (uint32_t t = 0; t < n_tmpl; t++) {
    uint8_t *b = tab.data() + blob_at + vt[t].head_at;
    if (tmpl[t].head_len) std::memcpy(b, tmpl[t].head, tmpl[t].head_len);
    if (tmpl[t].block_len) std::memcpy(b + tmpl[t].head_len, tmpl[t].block, tmpl[t].block_len);
    if (tmpl[t].chain_len) std::memcpy(b + tmpl[t].head_len + tmpl[t].block_len, tmpl[t].chain, tmpl[t].chain_len);
  }
  off.resize((size_t)n + 1);
  off[0] = 0;
  uint64_t acc = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t t = votes[i].tmpl & ~TMV_VOTE_WITH_BLOCK;
    if (t >= n_tmpl) { set_error("vote template index out of range"); return TMV_ERR_ARG; }
    acc += tmv::vote_msg_len(vt[t], votes[i]);
    if (acc > UINT32_MAX) { set_error("vote messages exceed 4 GiB"); return TMV_ERR_ARG; }
    off[i + 1] = (uint32_t)acc;
  }
  return 0;
}

static Device *find_device(tmv_ctx *ctx, int device) {
  if (!ctx) return nullptr;
  for (auto &d : ctx->devs)
    if (d->id == device) return d.get();
  return nullptr;
}

extern "C" {

int tmv_ed25519_verify_batch(tmv_ctx *ctx, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                             const uint32_t *msg_off, uint32_t n, uint8_t *valid_out) {
  return run_batch(ctx, Scheme::Ed25519, nullptr, pk, sig, msg, msg_off, n, valid_out);
}

int tmv_sr25519_verify_batch(tmv_ctx *ctx, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                             const uint32_t *msg_off, uint32_t n, int8_t *status_out) {
  return run_batch(ctx, Scheme::Sr25519, nullptr, pk, sig, msg, msg_off, n, reinterpret_cast<uint8_t *>(status_out));
}

int tmv_verify_mixed_batch(tmv_ctx *ctx, const uint8_t *kind, const uint8_t *pk, const uint8_t *sig,
                           const uint8_t *msg, const uint32_t *msg_off, uint32_t n, int8_t *status_out) {
  return run_batch(ctx, Scheme::Mixed, kind, pk, sig, msg, msg_off, n, reinterpret_cast<uint8_t *>(status_out));
}

int tmv_verify_batch_ex(tmv_ctx *ctx, uint8_t key_kind, uint32_t flags, const uint8_t *pk, const uint8_t *sig,
                        const uint8_t *msg, const uint32_t *msg_off, uint32_t n, int8_t *status_out) {
  const bool cache = (flags & TMV_FLAG_KEY_CACHE) != 0;
  Scheme sch;
  if (key_kind == TMV_KIND_ED25519) sch = cache ? Scheme::Ed25519Cached : Scheme::Ed25519;
  else if (key_kind == TMV_KIND_SR25519) sch = cache ? Scheme::Sr25519Cached : Scheme::Sr25519;
  else { set_error("unsupported key kind"); return TMV_ERR_ARG; }
  return run_batch(ctx, sch, nullptr, pk, sig, msg, msg_off, n, reinterpret_cast<uint8_t *>(status_out), flags);
}

int tmv_verify_mixed_batch_ex(tmv_ctx *ctx, uint32_t flags, const uint8_t *kind, const uint8_t *pk,
                              const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off, uint32_t n,
                              int8_t *status_out) {
  return run_batch(ctx, Scheme::Mixed, kind, pk, sig, msg, msg_off, n, reinterpret_cast<uint8_t *>(status_out),
                   flags);
}

int tmv_verify_votes(tmv_ctx *ctx, uint8_t key_kind, uint32_t flags, const tmv_vote_template *tmpl,
                     uint32_t n_tmpl, const tmv_vote *votes, const uint8_t *pk, const uint8_t *sig, uint32_t n,
                     int8_t *status_out) {
  if (!ctx) { set_error("null context"); return TMV_ERR_ARG; }
  const bool cache = (flags & TMV_FLAG_KEY_CACHE) != 0;
  Scheme sch;
  if (key_kind == TMV_KIND_ED25519) sch = cache ? Scheme::Ed25519Cached : Scheme::Ed25519;
  else if (key_kind == TMV_KIND_SR25519) sch = cache ? Scheme::Sr25519Cached : Scheme::Sr25519;
  else { set_error("unsupported key kind"); return TMV_ERR_ARG; }
  static thread_local std::vector<uint8_t> tab;
  static thread_local std::vector<uint32_t> off;
  size_t blob_at = 0;
  EngineTimer tm;
  const int pr = prepare_votes(tmpl, n_tmpl, votes, n, tab, blob_at, off);
  if (pr < 0) return pr;
  tm.mark("votes", n);
  const VoteSrc vs{votes, tab.data(), tab.size(), blob_at};
  return run_batch(ctx, sch, nullptr, pk, sig, nullptr, off.data(), n, reinterpret_cast<uint8_t *>(status_out),
                   flags, &vs);
}

int64_t tmv_vote_sign_bytes_device(tmv_ctx *ctx, const tmv_vote_template *tmpl, uint32_t n_tmpl,
                                   const tmv_vote *votes, uint32_t n, uint8_t *msg_out, size_t msg_cap,
                                   uint32_t *msg_off_out) {
  if (!ctx || !msg_off_out) { set_error("null argument"); return TMV_ERR_ARG; }
  std::vector<uint8_t> tab;
  std::vector<uint32_t> off;
  size_t blob_at = 0;
  const int pr = prepare_votes(tmpl, n_tmpl, votes, n, tab, blob_at, off);
  if (pr < 0) return pr;
  std::memcpy(msg_off_out, off.data(), sizeof(uint32_t) * ((size_t)n + 1));
  const size_t total = off[n];
  if (!msg_out || n == 0) return (int64_t)total;
  if (msg_cap < total) { set_error("msg_cap too small"); return TMV_ERR_ARG; }
  Device &d = *ctx->devs[0];
  std::lock_guard<std::mutex> lk(d.mu);
  if (d.faulted) return faulted_rc(d);
  hipError_t e = hipSetDevice(d.id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  const size_t v_at = 0, t_at = align16(sizeof(tmv_vote) * n), o_at = t_at + align16(tab.size()),
               m_at = o_at + align16(4ull * (n + 1)), bytes = m_at + std::max<size_t>(total, 1);
  hipStream_t s = context_stream(d);
  if (!s) { set_error("hipStreamCreate failed"); return TMV_ERR_NO_DEVICE; }
  uint8_t *dev = nullptr;
  if ((e = hipMalloc(&dev, bytes)) != hipSuccess) { set_error("hipMalloc", e); return TMV_ERR_NOMEM; }
  int rc = 0;
  if ((e = hipMemcpyAsync(dev + v_at, votes, sizeof(tmv_vote) * n, hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = hipMemcpyAsync(dev + t_at, tab.data(), tab.size(), hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = hipMemcpyAsync(dev + o_at, off.data(), 4ull * (n + 1), hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = tmv::launch_vote_signbytes(reinterpret_cast<const tmv_vote *>(dev + v_at),
                                      reinterpret_cast<const tmv::VoteTab *>(dev + t_at), dev + t_at + blob_at,
                                      reinterpret_cast<const uint32_t *>(dev + o_at), n, dev + m_at, s)) !=
          hipSuccess ||
      (e = hipMemcpyAsync(msg_out, dev + m_at, total, hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = wait_stream(d, s)) != hipSuccess) {
    if (e != hipErrorNotReady) set_error("tmv_vote_sign_bytes_device", e);
    rc = wait_rc(e);
  }
  if (!d.faulted) (void)hipFree(dev);
  return rc < 0 ? rc : (int64_t)total;
}

int tmv_set_batch_options(tmv_ctx *ctx, uint32_t group_log2, uint32_t window_bits, const uint8_t *seed32,
                          uint32_t opt_flags) {
  if (!ctx) { set_error("null context"); return TMV_ERR_ARG; }
  if ((group_log2 && (group_log2 < 5 || group_log2 > 10)) || (window_bits && (window_bits < 4 || window_bits > 9))) {
    set_error("group_log2 must be 0 or 5..10, window_bits 0 or 4..9");
    return TMV_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(ctx->opt_mu);
  ctx->msm_m_log2 = group_log2;
  ctx->msm_c = window_bits;
  ctx->fixed_seed = seed32 != nullptr;
  if (seed32) std::memcpy(ctx->seed, seed32, 32);
  ctx->stats = (opt_flags & TMV_BATCHOPT_STATS) != 0;
  ctx->msm_sub = (opt_flags & TMV_BATCHOPT_SUBCHECK_ON) ? 1 : (opt_flags & TMV_BATCHOPT_SUBCHECK_OFF) ? 0 : -1;
  return 0;
}

int tmv_batch_stats(tmv_ctx *ctx, uint64_t *groups, uint64_t *groups_failed) {
  if (!ctx) return TMV_ERR_ARG;
  if (groups) *groups = ctx->groups.load();
  if (groups_failed) *groups_failed = ctx->groups_failed.load();
  return 0;
}

int tmv_subgroup_stats(tmv_ctx *ctx, uint64_t *subgroups, uint64_t *subgroups_failed) {
  if (!ctx) return TMV_ERR_ARG;
  if (subgroups) *subgroups = ctx->subgroups.load();
  if (subgroups_failed) *subgroups_failed = ctx->subgroups_failed.load();
  return 0;
}

int tmv_key_cache_stats(tmv_ctx *ctx, uint64_t *hits, uint64_t *misses, uint32_t *used, uint32_t *capacity) {
  if (!ctx) return TMV_ERR_ARG;
  uint64_t h = 0, m = 0;
  uint32_t u = 0, c = 0;
  for (auto &d : ctx->devs) {
    std::lock_guard<std::mutex> lk(d->mu);
    h += d->khits; m += d->kmisses; u += (uint32_t)d->kindex.size(); c += d->kcap;
  }
  if (hits) *hits = h;
  if (misses) *misses = m;
  if (used) *used = u;
  if (capacity) *capacity = c;
  return 0;
}

int tmv_metrics_read(tmv_ctx *ctx, tmv_metrics *out) {
  if (!ctx || !out) { set_error("null argument"); return TMV_ERR_ARG; }
  std::memset(out, 0, sizeof(*out));
  out->calls = ctx->m_calls;
  out->signatures = ctx->m_sigs;
  out->max_batch = ctx->m_max;
  out->batch_eq_signatures = ctx->m_beq;
  out->host_signatures = ctx->m_host_sigs;
  out->host_seconds = (double)ctx->m_host_ns.load() * 1e-9;
  out->h2d_bytes = ctx->m_h2d;
  out->d2h_bytes = ctx->m_d2h;
  out->groups = ctx->groups;
  out->groups_failed = ctx->groups_failed;
  out->located_groups = ctx->m_located;
  out->fallback_signatures = ctx->m_fallback;
  uint64_t h = 0, m = 0;
  for (auto &d : ctx->devs) {
    std::lock_guard<std::mutex> lk(d->mu);
    h += d->khits;
    m += d->kmisses;
  }
  out->key_cache_hits = h - ctx->khits_base;
  out->key_cache_misses = m - ctx->kmiss_base;
  return 0;
}

int tmv_metrics_reset(tmv_ctx *ctx) {
  if (!ctx) { set_error("null context"); return TMV_ERR_ARG; }
  for (auto *a : {&ctx->m_calls, &ctx->m_sigs, &ctx->m_max, &ctx->m_beq, &ctx->m_host_sigs, &ctx->m_host_ns,
                  &ctx->m_h2d, &ctx->m_d2h, &ctx->m_located, &ctx->m_fallback, &ctx->groups, &ctx->groups_failed,
                  &ctx->subgroups, &ctx->subgroups_failed})
    a->store(0);
  uint64_t h = 0, m = 0;
  for (auto &d : ctx->devs) {
    std::lock_guard<std::mutex> lk(d->mu);
    h += d->khits;
    m += d->kmisses;
  }
  ctx->khits_base = h;
  ctx->kmiss_base = m;
  return 0;
}

int tmv_verify_mixed_batch_device(tmv_ctx *ctx, int device, const uint8_t *d_kind, const uint8_t *d_pk,
                                  const uint8_t *d_sig, const uint8_t *d_msg, const uint32_t *d_msg_off, uint32_t n,
                                  int8_t *d_status, void *stream) {
  Device *dev = find_device(ctx, device);
  if (!dev) { set_error("device not in context"); return TMV_ERR_ARG; }
  if (dev->faulted) return faulted_rc(*dev);
  if (n == 0) return TMV_NOT_ALL;
  hipError_t e = hipSetDevice(dev->id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : context_stream(*dev);
  if (!s) { set_error("hipStreamCreate failed"); return TMV_ERR_NO_DEVICE; }
  const LaunchOpts o = make_opts(ctx, 0, n);
  if (o.err) return o.err;
  ctx->count_call(n);
  std::lock_guard<std::mutex> lk(dev->mu);
  int rc = launch_mixed(*dev, o, d_kind, d_pk, d_sig, d_msg, d_msg_off, n, d_status, s);
  return rc != 0 ? rc : TMV_NOT_ALL;
}

int tmv_verify_batch_device_ex(tmv_ctx *ctx, int device, uint8_t key_kind, uint32_t flags, const uint8_t *d_kind,
                               const uint8_t *d_pk, const uint8_t *d_sig, const uint8_t *d_msg,
                               const uint32_t *d_msg_off, uint32_t n, int8_t *d_status, void *stream) {
  Device *dev = find_device(ctx, device);
  if (!dev) { set_error("device not in context"); return TMV_ERR_ARG; }
  if (dev->faulted) return faulted_rc(*dev);
  if (n == 0) return TMV_NOT_ALL;
  if (key_kind == TMV_KIND_MIXED && !d_kind) { set_error("mixed batch without kinds"); return TMV_ERR_ARG; }
  if (key_kind > TMV_KIND_MIXED) { set_error("unsupported key kind"); return TMV_ERR_ARG; }
  hipError_t e = hipSetDevice(dev->id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : context_stream(*dev);
  if (!s) { set_error("hipStreamCreate failed"); return TMV_ERR_NO_DEVICE; }
  const LaunchOpts o = make_opts(ctx, flags, n, false, key_kind == TMV_KIND_ED25519);
  if (o.err) return o.err;
  ctx->count_call(n);
  std::lock_guard<std::mutex> lk(dev->mu);
  uint8_t *out = reinterpret_cast<uint8_t *>(d_status);
  int rc;
  if (key_kind == TMV_KIND_ED25519) rc = launch_ed25519(*dev, o, d_pk, d_sig, d_msg, d_msg_off, n, out, s);
  else if (key_kind == TMV_KIND_SR25519) rc = launch_sr25519(*dev, o, d_pk, d_sig, d_msg, d_msg_off, n, d_status, s);
  else rc = launch_mixed(*dev, o, d_kind, d_pk, d_sig, d_msg, d_msg_off, n, d_status, s);
  return rc != 0 ? rc : TMV_NOT_ALL;
}

int tmv_verify_batches_device(tmv_ctx *ctx, int device, uint8_t key_kind, uint32_t flags,
                              const tmv_batch_ref *batches, uint32_t n_batches, void *stream) {
  Device *dev = find_device(ctx, device);
  if (!dev) { set_error("device not in context"); return TMV_ERR_ARG; }
  if (dev->faulted) return faulted_rc(*dev);
  if (key_kind != TMV_KIND_ED25519 && key_kind != TMV_KIND_SR25519) {
    set_error("tmv_verify_batches_device: key_kind must be ed25519 or sr25519");
    return TMV_ERR_ARG;
  }
  if (n_batches == 0 || n_batches > TMV_MAX_BATCHES || !batches) {
    set_error("tmv_verify_batches_device: 1..256 batches");
    return TMV_ERR_ARG;
  }
  // one BatchRefs (kernel argument) per kMaxBatches batches; entry and
  // message offsets are global over the launch
  const uint32_t n_refs = (n_batches + tmv::kMaxBatches - 1) / tmv::kMaxBatches;
  std::vector<tmv::BatchRefs> refs(n_refs);
  uint64_t N = 0, M = 0;
  for (uint32_t b = 0; b < n_batches; b++) {
    const tmv_batch_ref &x = batches[b];
    if (x.n && (!x.pk || !x.sig || !x.msg_off || !x.status || (!x.msg && x.msg_bytes))) {
      set_error("tmv_verify_batches_device: null pointer in a non-empty batch");
      return TMV_ERR_ARG;
    }
    if (!x.n && x.msg_bytes) {
      set_error("tmv_verify_batches_device: message bytes in an empty batch");
      return TMV_ERR_ARG;
    }
    tmv::BatchRefs &r = refs[b / tmv::kMaxBatches];
    const uint32_t k = b % tmv::kMaxBatches;
    r.pk[k] = x.pk; r.sig[k] = x.sig; r.msg[k] = x.msg; r.off[k] = x.msg_off; r.out[k] = x.status;
    r.start[k] = (uint32_t)N;
    r.msg_base[k] = (uint32_t)M;
    r.nb = k + 1;
    N += x.n;
    M += x.msg_bytes;
    if (N > 0xffffffffull / 64 || M > 0xffffffffull) { set_error("tmv_verify_batches_device: too large"); return TMV_ERR_ARG; }
    r.start[k + 1] = (uint32_t)N;
    r.msg_base[k + 1] = (uint32_t)M;
  }
  if (N == 0) return TMV_NOT_ALL;
  hipError_t e = hipSetDevice(dev->id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : context_stream(*dev);
  if (!s) { set_error("hipStreamCreate failed"); return TMV_ERR_NO_DEVICE; }
  const uint32_t n = (uint32_t)N;
  const LaunchOpts o = make_opts(ctx, flags, n, false, key_kind == TMV_KIND_ED25519);
  if (o.err) return o.err;
  ctx->count_call(n);
  std::lock_guard<std::mutex> lk(dev->mu);
  int rc;
  Workspace *ws = reserve_work(*dev, n, false, s, &rc, o.batch_eq ? &o.p : nullptr);
  if (!ws) return rc;
  Layout L(n, (size_t)M);
  const size_t need = L.total + align16(n);
  if (need > ws->gather.cap) {
    if ((e = wait_event(*dev, ws->done)) != hipSuccess) return wait_rc(e);
    if ((e = ws->gather.ensure(need, false)) != hipSuccess) { set_error("hipMalloc(gather)", e); return TMV_ERR_NOMEM; }
  }
  uint8_t *g = static_cast<uint8_t *>(ws->gather.ptr);
  uint32_t *goff = reinterpret_cast<uint32_t *>(g + L.off);
  int8_t *gst = reinterpret_cast<int8_t *>(g + L.total);
  for (const tmv::BatchRefs &r : refs)
    if ((e = tmv::launch_gather(r, g + L.pk, g + L.sig, goff, g + L.msg, s)) != hipSuccess) {
      set_error("gather launch", e);
      return TMV_ERR_LAUNCH;
    }
  if (key_kind == TMV_KIND_ED25519)
    rc = launch_ed25519(*dev, o, g + L.pk, g + L.sig, g + L.msg, goff, n, reinterpret_cast<uint8_t *>(gst), s);
  else
    rc = launch_sr25519(*dev, o, g + L.pk, g + L.sig, g + L.msg, goff, n, gst, s);
  if (rc != 0) return rc;
  for (const tmv::BatchRefs &r : refs)
    if ((e = tmv::launch_scatter(r, gst, s)) != hipSuccess) { set_error("scatter launch", e); return TMV_ERR_LAUNCH; }
  (void)hipEventRecord(ws->done, s);
  return TMV_NOT_ALL;
}

// ValidatorSet.Hash of many sets in one launch (SURVEY §8(f) rank 4;
// types/validator_set.go:344-350).  Synchronous, host buffers.
int tmv_validator_set_hashes(tmv_ctx *ctx, const uint8_t *pk, const uint8_t *key_kind, const int64_t *power,
                             const uint32_t *set_off, uint32_t n_sets, uint8_t *hash_out) {
  if (!ctx || ctx->devs.empty()) { set_error("null context"); return TMV_ERR_ARG; }
  if (n_sets == 0) return 0;
  if (!set_off || !hash_out) { set_error("tmv_validator_set_hashes: null pointer"); return TMV_ERR_ARG; }
  if (set_off[0] != 0) { set_error("tmv_validator_set_hashes: set_off[0] must be 0"); return TMV_ERR_ARG; }
  for (uint32_t s = 0; s < n_sets; s++)
    if (set_off[s + 1] < set_off[s]) { set_error("tmv_validator_set_hashes: set_off decreasing"); return TMV_ERR_ARG; }
  const uint32_t n = set_off[n_sets];
  if (n && (!pk || !key_kind || !power)) { set_error("tmv_validator_set_hashes: null pointer"); return TMV_ERR_ARG; }
  if (n > (1u << 26)) { set_error("tmv_validator_set_hashes: too many validators"); return TMV_ERR_ARG; }
  for (uint32_t i = 0; i < n; i++)
    if (key_kind[i] != TMV_KIND_ED25519 && key_kind[i] != TMV_KIND_SR25519) {
      set_error("tmv_validator_set_hashes: key kind must be ed25519 or sr25519");
      return TMV_ERR_ARG;
    }
  Device &d = *ctx->devs[0];
  std::lock_guard<std::mutex> lk(d.mu);
  if (d.faulted) return faulted_rc(d);
  hipError_t e = hipSetDevice(d.id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  // staging: power | set_off | pk | kind, then (device only) two node arrays and the roots
  const size_t o_off = align16(8ull * n), o_pk = o_off + align16(4ull * (n_sets + 1));
  const size_t o_kind = o_pk + align16(32ull * n), in_bytes = o_kind + align16(n);
  const size_t o_na = in_bytes, o_nb = o_na + 32ull * n, o_out = o_nb + 32ull * n;
  const size_t dev_bytes = o_out + 32ull * n_sets;
  hipStream_t s = context_stream(d);
  if (!s) { set_error("hipStreamCreate failed"); return TMV_ERR_NO_DEVICE; }
  if ((e = wait_stream(d, s)) != hipSuccess) return wait_rc(e);  // staging may still feed an earlier call
  if ((e = d.h_valset.ensure(in_bytes, true)) != hipSuccess) { set_error("hipHostMalloc", e); return TMV_ERR_NOMEM; }
  if ((e = d.d_valset.ensure(dev_bytes, false)) != hipSuccess) { set_error("hipMalloc", e); return TMV_ERR_NOMEM; }
  uint8_t *h = static_cast<uint8_t *>(d.h_valset.ptr);
  if (n) {
    std::memcpy(h, power, 8ull * n);
    std::memcpy(h + o_pk, pk, 32ull * n);
    std::memcpy(h + o_kind, key_kind, n);
  }
  std::memcpy(h + o_off, set_off, 4ull * (n_sets + 1));
  uint8_t *g = static_cast<uint8_t *>(d.d_valset.ptr);
  if ((e = hipMemcpyAsync(g, h, in_bytes, hipMemcpyHostToDevice, s)) != hipSuccess) {
    set_error("hipMemcpyAsync(valset)", e);
    return TMV_ERR_LAUNCH;
  }
  e = tmv::launch_valset_hashes(g + o_pk, g + o_kind, reinterpret_cast<const int64_t *>(g), n,
                                reinterpret_cast<const uint32_t *>(g + o_off), n_sets,
                                reinterpret_cast<uint32_t *>(g + o_na), reinterpret_cast<uint32_t *>(g + o_nb),
                                g + o_out, s);
  if (e != hipSuccess) { set_error("valset hash launch", e); return TMV_ERR_LAUNCH; }
  if ((e = hipMemcpyAsync(hash_out, g + o_out, 32ull * n_sets, hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = wait_stream(d, s)) != hipSuccess) {
    if (e != hipErrorNotReady) set_error("valset hash readback", e);
    return wait_rc(e);
  }
  return 0;
}

int tmv_merkle_roots(tmv_ctx *ctx, const uint8_t *data, const uint32_t *leaf_off, uint32_t n_leaves,
                     const uint32_t *tree_off, uint32_t n_trees, uint8_t *hash_out) {
  if (!ctx || ctx->devs.empty()) { set_error("null context"); return TMV_ERR_ARG; }
  if (n_trees == 0) return 0;
  if (!leaf_off || !tree_off || !hash_out) { set_error("tmv_merkle_roots: null pointer"); return TMV_ERR_ARG; }
  if (leaf_off[0] != 0 || tree_off[0] != 0 || tree_off[n_trees] != n_leaves) {
    set_error("tmv_merkle_roots: offsets must start at 0 and tree_off must end at n_leaves");
    return TMV_ERR_ARG;
  }
  uint32_t max_leaves = 0;
  for (uint32_t t = 0; t < n_trees; t++) {
    if (tree_off[t + 1] < tree_off[t]) { set_error("tmv_merkle_roots: tree_off decreasing"); return TMV_ERR_ARG; }
    max_leaves = std::max(max_leaves, tree_off[t + 1] - tree_off[t]);
  }
  for (uint32_t i = 0; i < n_leaves; i++)
    if (leaf_off[i + 1] < leaf_off[i]) { set_error("tmv_merkle_roots: leaf_off decreasing"); return TMV_ERR_ARG; }
  const uint32_t bytes = leaf_off[n_leaves];
  if (bytes && !data) { set_error("tmv_merkle_roots: null data"); return TMV_ERR_ARG; }
  if (n_leaves > (1u << 26) || bytes > (1u << 30)) { set_error("tmv_merkle_roots: input too large"); return TMV_ERR_ARG; }
  Device &d = *ctx->devs[0];
  std::lock_guard<std::mutex> lk(d.mu);
  if (d.faulted) return faulted_rc(d);
  hipError_t e = hipSetDevice(d.id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  // staging: leaf_off | tree_off | data, then (device only) two node arrays and the roots
  const size_t o_tree = align16(4ull * (n_leaves + 1)), o_data = o_tree + align16(4ull * (n_trees + 1));
  const size_t in_bytes = o_data + align16(bytes);
  const size_t o_na = in_bytes, o_nb = o_na + 32ull * n_leaves, o_out = o_nb + 32ull * n_leaves;
  const size_t dev_bytes = o_out + 32ull * n_trees;
  hipStream_t s = context_stream(d);
  if (!s) { set_error("hipStreamCreate failed"); return TMV_ERR_NO_DEVICE; }
  if ((e = wait_stream(d, s)) != hipSuccess) return wait_rc(e);  // staging shared with tmv_validator_set_hashes
  if ((e = d.h_valset.ensure(in_bytes, true)) != hipSuccess) { set_error("hipHostMalloc", e); return TMV_ERR_NOMEM; }
  if ((e = d.d_valset.ensure(dev_bytes, false)) != hipSuccess) { set_error("hipMalloc", e); return TMV_ERR_NOMEM; }
  uint8_t *h = static_cast<uint8_t *>(d.h_valset.ptr);
  std::memcpy(h, leaf_off, 4ull * (n_leaves + 1));
  std::memcpy(h + o_tree, tree_off, 4ull * (n_trees + 1));
  if (bytes) std::memcpy(h + o_data, data, bytes);
  uint8_t *g = static_cast<uint8_t *>(d.d_valset.ptr);
  if ((e = hipMemcpyAsync(g, h, in_bytes, hipMemcpyHostToDevice, s)) != hipSuccess) {
    set_error("hipMemcpyAsync(merkle)", e);
    return TMV_ERR_LAUNCH;
  }
  e = tmv::launch_merkle_roots(g + o_data, reinterpret_cast<const uint32_t *>(g), n_leaves,
                               reinterpret_cast<const uint32_t *>(g + o_tree), n_trees, max_leaves,
                               reinterpret_cast<uint32_t *>(g + o_na), reinterpret_cast<uint32_t *>(g + o_nb),
                               g + o_out, s);
  if (e != hipSuccess) { set_error("merkle launch", e); return TMV_ERR_LAUNCH; }
  if ((e = hipMemcpyAsync(hash_out, g + o_out, 32ull * n_trees, hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = wait_stream(d, s)) != hipSuccess) {
    if (e != hipErrorNotReady) set_error("merkle readback", e);
    return wait_rc(e);
  }
  return 0;
}

}  // extern "C"

extern "C" {

int tmv_ed25519_verify(tmv_ctx *ctx, const uint8_t *pk, const uint8_t *msg, size_t msg_len, const uint8_t *sig,
                       size_t sig_len) {
  if (sig_len != 64) return 0;  // crypto/ed25519/ed25519.go:175-177
  if (msg_len > 0xffffffffu) { set_error("message too long"); return TMV_ERR_ARG; }
  uint32_t off[2] = {0, (uint32_t)msg_len};
  uint8_t v = 0;
  static const uint8_t empty = 0;
  int rc = tmv_ed25519_verify_batch(ctx, pk, sig, msg ? msg : &empty, off, 1, &v);
  return rc < 0 ? rc : (int)v;
}

int tmv_ed25519_verify_batch_device(tmv_ctx *ctx, int device, const uint8_t *d_pk, const uint8_t *d_sig,
                                    const uint8_t *d_msg, const uint32_t *d_msg_off, uint32_t n, uint8_t *d_valid,
                                    void *stream) {
  Device *dev = find_device(ctx, device);
  if (!dev) { set_error("device not in context"); return TMV_ERR_ARG; }
  if (dev->faulted) return faulted_rc(*dev);
  if (n == 0) return TMV_NOT_ALL;
  hipError_t e = hipSetDevice(dev->id);
  if (e != hipSuccess) { set_error("hipSetDevice", e); return TMV_ERR_NO_DEVICE; }
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : context_stream(*dev);
  if (!s) { set_error("hipStreamCreate failed"); return TMV_ERR_NO_DEVICE; }
  const LaunchOpts o = make_opts(ctx, 0, n, false, true);
  if (o.err) return o.err;
  ctx->count_call(n);
  std::lock_guard<std::mutex> lk(dev->mu);
  int rc = launch_ed25519(*dev, o, d_pk, d_sig, d_msg, d_msg_off, n, d_valid, s);
  return rc != 0 ? rc : TMV_NOT_ALL;
}

}  // extern "C"

