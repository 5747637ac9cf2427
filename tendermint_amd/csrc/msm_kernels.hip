// Batch-equation kernels (msm.h): the random-linear-combination check that
// curve25519-voi's BatchVerifier.Verify performs behind
// crypto/ed25519/ed25519.go:231-233 and crypto/sr25519/batch.go:44-47, laid
// out for CDNA4: groups of m signatures, Pippenger buckets found by an LDS
// counting sort, bucket sums by independent lanes over fixed-size chunks of
// the sorted entries (no atomics on points), and a per-group Horner
// combination in quad-lane arithmetic (quad.h).  All integer VALU work.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>
#include "ed25519_core.h"
#include "kernel_util.h"
#include "comb.h"
#include "quad.h"
#include "ktimer.h"
#include "verify_kernels.h"
#include "halfscalar.h"

#include <atomic>
#include <mutex>
#include <vector>

namespace tmv {

namespace ktimer {
namespace {
struct Pair {
  int k;
  hipEvent_t a, b;
};
std::atomic<bool> g_on{false};
std::mutex g_mu;
std::vector<Pair *> g_done[kCount];  // recorded pairs per kernel
std::vector<hipEvent_t> g_free;      // recycled timing events
hipEvent_t take_event() {
  hipEvent_t e = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_free.empty()) { e = g_free.back(); g_free.pop_back(); }
  }
  if (!e && hipEventCreate(&e) != hipSuccess) e = nullptr;
  return e;
}
}  // namespace

void set(bool on) { g_on.store(on); }
bool on() { return g_on.load(std::memory_order_relaxed); }

void *begin(Kernel k, hipStream_t s) {
  if (!on()) return nullptr;
  Pair *p = new Pair{k, take_event(), take_event()};
  if (!p->a || !p->b || hipEventRecord(p->a, s) != hipSuccess) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (p->a) g_free.push_back(p->a);
    if (p->b) g_free.push_back(p->b);
    delete p;
    return nullptr;
  }
  return p;
}

void end(void *token, hipStream_t s) {
  if (!token) return;
  Pair *p = static_cast<Pair *>(token);
  (void)hipEventRecord(p->b, s);
  std::lock_guard<std::mutex> lk(g_mu);
  g_done[p->k].push_back(p);
}

int read(Kernel k, double *ms, uint64_t *launches) {
  std::vector<Pair *> v;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    v.swap(g_done[k]);
  }
  int rc = 0;
  for (Pair *p : v) {
    float t = 0.f;
    hipError_t e = hipEventSynchronize(p->b);
    if (e == hipSuccess) e = hipEventElapsedTime(&t, p->a, p->b);
    if (e == hipSuccess) {
      *ms += t;
      *launches += 1;
    } else if (!rc) {
      rc = (int)e;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    g_free.push_back(p->a);
    g_free.push_back(p->b);
    delete p;
  }
  return rc;
}

}  // namespace ktimer

namespace {

template <int V>
struct StaticIndex {
  static constexpr int value = V;
};

// Signed c-bit digits of a scalar read window after window: a 64-bit buffer
// of the next bits, refilled from the scalar's next word once every ~32 / c
// windows.  The reader owns a copy of the words and shifts them down by one
// at each refill, so every register index is a compile-time constant (no
// select chain, no scratch, no s_set_gpr_idx); the top window keeps
// [0, 2^(c-1)] (callers size the window count so it fits).  Round 4 measured
// a reader that refilled through a run-time word index: no faster, the
// scalars in scratch (profiles/r04/ab_sort_reader.txt).
template <int NW>
struct DigitReader {
  uint32_t wd[NW];  // the words not yet in buf, lowest first
  uint64_t buf;     // bits [pos, pos + avail) of the scalar, zeros above
  uint32_t avail;
  int carry;
  __device__ __forceinline__ void init(const uint32_t *s) {
#pragma unroll
    for (int k = 0; k < NW; k++) wd[k] = s[k];
    buf = 0;
    avail = 0;
    carry = 0;
  }
  __device__ __forceinline__ int next(uint32_t c, bool top) {
    if (avail < c) {  // avail + 32 <= 40: fits
      buf |= (uint64_t)wd[0] << avail;
#pragma unroll
      for (int k = 0; k + 1 < NW; k++) wd[k] = wd[k + 1];
      wd[NW - 1] = 0;
      avail += 32;
    }
    int d = (int)(buf & ((1u << c) - 1)) + carry;
    buf >>= c;
    avail -= c;
    if (!top && d >= (1 << (c - 1))) {
      d -= 1 << c;
      carry = 1;
    } else {
      carry = 0;
    }
    return d;
  }
};

// For every nonzero digit of a scalar: f(bucket within group, negative).
template <int NW, typename F>
__device__ __forceinline__ void for_each_digit(const uint32_t *s, uint32_t windows, const MsmParams &p, F f) {
  DigitReader<NW> rd;
  rd.init(s);
  for (uint32_t w = 0; w < windows; w++) {
    const int d = rd.next(p.c, w + 1 == windows);
    if (d != 0) f(p.bucket(w, (uint32_t)((d < 0 ? -d : d) - 1)), d < 0);
  }
}

__device__ __forceinline__ void p3_add(ge_p3 &a, const ge_p3 &b) {
  ge_cached c;
  ge_p3_to_cached(c, b);
  ge_p1p1 r;
  ge_add(r, a, c);
  ge_p1p1_to_p3(a, r);
}

__device__ __forceinline__ void p3_dbl(ge_p3 &a) {
  ge_p1p1 r;
  ge_p3_dbl(r, a);
  ge_p1p1_to_p3(a, r);
}

}  // namespace

// One workgroup per group of m entries}  // namespace

// One workgroup per group of m entries: z_e, z_e k_e mod l, sum z_e s_e mod l
// (the B scalar), then a counting sort of the (window, |digit|) bucket entries
// of the 2m+1 points into the group's slots of ent_pt/ent_bk.  KM (key-merged
// form): only the m R points are sorted; z_e k_e and the B scalar go to
// mw.wscal / mw.bscal for k_msm_items, and the key's decode status comes from
// the key cache.  LOC (located fallback): block f sorts the f-th FAILING
// group into slot f with every weight multiplied by (j + 1), j the entry's
// index in its group, so the same bucket stages compute
// T'_f = sum (j+1) z_j Delta_j (z_j (j+1) < 2^(128 + m_log2): p.WL() R
// windows).
template <bool SR, bool KM, int BS = kMsmSortBlock, bool LOC = false>
__global__ void __launch_bounds__(BS)
k_msm_sort(const uint8_t *__restrict__ sig, const uint32_t *__restrict__ idx, const uint32_t *count_ptr, uint32_t n,
           Ed25519Work w, MsmWork mw, MsmParams p, MsmSeed seed, const fe *__restrict__ btab_q, int aligned,
           const uint32_t *__restrict__ key_slot, const uint8_t *__restrict__ key_ok, uint8_t *__restrict__ out,
           uint32_t e_base) {
  extern __shared__ uint32_t smem[];
  const uint32_t cnt = entry_count(count_ptr, n);
  const uint32_t tid = threadIdx.x;
  uint32_t g = blockIdx.x;  // LOC: the slot; the group is fail_list[slot]
  if (g == 0 && tid == 0) *mw.join_count = 0;  // the next k_msm_accum appends its joins
  if (LOC) {
    const uint32_t nf = *mw.fail_count;
    if (g == 0 && tid == 0) {
      *mw.loc_count = nf << p.m_log2;  // the bucket stages' entry count: nf slots
      *mw.fb_count = 0;                // k_loc_search appends the entries left to verify
      *mw.loc_found = 0;
    }
    if (g >= nf) return;  // block-uniform
  }
  const uint32_t slot = g;
  if (LOC) g = mw.fail_list[slot];
  const uint32_t e0 = g << p.m_log2;
  if (!KM && !LOC && g == 0 && tid == 0) {  // B as a Niels point (btab_q entry 0 = (ymx, ypx, xy2d, 1) of 1*B)
    niels_pt bp;
    bp.ymx = btab_q[0];
    bp.ypx = btab_q[1];
    bp.xy2d = btab_q[2];
    bp.pad[0] = bp.pad[1] = 0;
    niels_store(mw.pts, mw.n_pts, bp);
    if (mw.fail_count) *mw.fail_count = 0;  // k_msm_horner appends the failing groups
  }
  if (e0 >= cnt) return;  // block-uniform
  const uint32_t mlive = min(p.m(), cnt - e0);
  const uint32_t WH = p.W * p.H;
  uint32_t *hist = smem;                       // WH counters, then cursors
  uint32_t *red = smem + WH;                   // BS x 9 words
  uint32_t *scan = red + BS * 9;    // BS + 1

  constexpr int R = 4;  // entries per thread: m <= 4 * BS
  constexpr int ZW = LOC ? 5 : 4;  // words of the R weight (LOC: z (j + 1) < 2^(128 + m_log2), m_log2 <= 31)
  const uint32_t WRz = LOC ? p.WL() : p.WR;
  uint32_t z[R][ZW], wv[R][8];
  bool live[R];
  uint32_t acc[9];
#pragma unroll
  for (int t = 0; t < 9; t++) acc[t] = 0;
  // one copy of the weight computation per entry slot r (a compile-time
  // index): as a loop the body is too large for the unroller, and z[r] /
  // wv[r] / live[r] became run-time register indices (s_set_gpr_idx) and
  // scratch
  auto weigh = [&](auto rc) {
    constexpr int r = decltype(rc)::value;
    live[r] = false;
#pragma unroll
    for (int t = 0; t < ZW; t++) z[r][t] = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) wv[r][t] = 0;
    const uint32_t j = tid + r * BS;
    if (j >= mlive) return;
    const uint32_t e = e0 + j;
    const uint32_t i = idx ? idx[e] : e;
    uint32_t s_raw[8], s[8];
    if (aligned) load_words_aligned(s_raw, sig + 64ull * i + 32);
    else load_words_unaligned(s_raw, sig + 64ull * i + 32);
    bool s_ok;
    if (SR) {
      s_ok = sr25519_decode_s(s, s_raw);
    } else {
#pragma unroll
      for (int t = 0; t < 8; t++) s[t] = s_raw[t];
      s_ok = sc_is_canonical(s);
    }
    const bool a_ok = KM ? key_ok[key_slot[i]] != 0 : w.flags[4 * e] != 0;
    if (!KM && !LOC && out) {  // pre-check status; the compacted fallback rewrites failing groups' entries
      const bool r_ok = w.flags[4 * e + 1] != 0;
      const int st = SR ? (!a_ok ? -1 : (!s_ok ? -2 : (r_ok ? 1 : 0))) : ((a_ok && r_ok && s_ok) ? 1 : 0);
      out[i] = (uint8_t)(int8_t)st;
    }
    if (!(s_ok && a_ok && w.flags[4 * e + 1])) {  // left out of the sums
      if (KM) {
        uint4 *wd = reinterpret_cast<uint4 *>(mw.wscal + 8ull * e);
        wd[0] = wd[1] = make_uint4(0, 0, 0, 0);
      }
      return;
    }
    live[r] = true;
    uint32_t blk[16];
    chacha20_block(blk, seed.key, e_base + e, seed.nonce);  // counter = the entry's index in the whole launch
#pragma unroll
    for (int t = 0; t < 4; t++) z[r][t] = blk[t];
    uint32_t k[8];
    const uint4 *kp = reinterpret_cast<const uint4 *>(w.k + 8ull * e);
    const uint4 k0 = kp[0], k1 = kp[1];
    k[0] = k0.x; k[1] = k0.y; k[2] = k0.z; k[3] = k0.w;
    k[4] = k1.x; k[5] = k1.y; k[6] = k1.z; k[7] = k1.w;
    sc_mul_mod(wv[r], z[r], 4, k);
    if constexpr (LOC) {  // weights times (j + 1): z (j + 1) exactly, z k (j + 1) mod l
      const uint32_t jj = j + 1;
      uint64_t cy = 0;
#pragma unroll
      for (int t = 0; t < 4; t++) {
        cy += (uint64_t)z[r][t] * jj;
        z[r][t] = (uint32_t)cy;
        cy >>= 32;
      }
      z[r][4] = (uint32_t)cy;
      uint32_t t8[8];
#pragma unroll
      for (int t = 0; t < 8; t++) t8[t] = wv[r][t];
      sc_mul_mod(wv[r], &jj, 1, t8);
    }
    if (KM) {
      uint4 *wd = reinterpret_cast<uint4 *>(mw.wscal + 8ull * e);
      wd[0] = make_uint4(wv[r][0], wv[r][1], wv[r][2], wv[r][3]);
      wd[1] = make_uint4(wv[r][4], wv[r][5], wv[r][6], wv[r][7]);
    }
    uint32_t u[8];
    sc_mul_mod(u, z[r], ZW, s);  // LOC: (z (j + 1)) s mod l
    uint64_t c = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
      c += (uint64_t)acc[t] + u[t];
      acc[t] = (uint32_t)c;
      c >>= 32;
    }
    acc[8] += (uint32_t)c;
  };
  weigh(StaticIndex<0>{});
  weigh(StaticIndex<1>{});
  weigh(StaticIndex<2>{});
  weigh(StaticIndex<3>{});
  static_assert(R == 4, "one weigh() call per entry slot");
  // B scalar = (sum of z_e s_e) mod l: block tree sum (< m l < 2^264), then Barrett
#pragma unroll
  for (int t = 0; t < 9; t++) red[tid * 9 + t] = acc[t];
  __syncthreads();
  for (uint32_t stride = BS / 2; stride > 0; stride >>= 1) {
    if (tid < stride) {
      uint64_t c = 0;
      for (int t = 0; t < 9; t++) {
        c += (uint64_t)red[tid * 9 + t] + red[(tid + stride) * 9 + t];
        red[tid * 9 + t] = (uint32_t)c;
        c >>= 32;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    uint32_t x[16], b[8];
    for (int t = 0; t < 16; t++) x[t] = t < 9 ? red[t] : 0;
    sc_reduce512(b, x);
    for (int t = 0; t < 8; t++) red[t] = b[t];
    if (KM)
      for (int t = 0; t < 8; t++) mw.bscal[8ull * g + t] = b[t];
  }
  for (uint32_t t = tid; t < WH; t += BS) hist[t] = 0;
  __syncthreads();
  uint32_t bsc[8];
#pragma unroll
  for (int t = 0; t < 8; t++) bsc[t] = red[t];

  // pass 1: bucket sizes
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (!live[r]) continue;
    for_each_digit<ZW>(z[r], WRz, p, [&](uint32_t bk, bool) { atomicAdd(&hist[bk], 1u); });
    if (!KM) for_each_digit<8>(wv[r], p.W, p, [&](uint32_t bk, bool) { atomicAdd(&hist[bk], 1u); });
  }
  if (!KM && tid == 0) for_each_digit<8>(bsc, p.W, p, [&](uint32_t bk, bool) { atomicAdd(&hist[bk], 1u); });
  __syncthreads();

  // exclusive scan: contiguous segments per thread, thread 0 scans the totals
  const uint32_t seg = (WH + BS - 1) / BS;
  const uint32_t lo = min(WH, tid * seg), hi = min(WH, lo + seg);
  uint32_t local = 0;
  for (uint32_t t = lo; t < hi; t++) local += hist[t];
  scan[tid] = local;
  __syncthreads();
  if (tid == 0) {
    uint32_t run = 0;
    for (int t = 0; t < BS; t++) {
      const uint32_t v = scan[t];
      scan[t] = run;
      run += v;
    }
    scan[BS] = run;
  }
  __syncthreads();
  const uint32_t gbase = slot * p.cap;
  const uint32_t bbase = slot * WH;
  // more entries than slots cannot happen (MsmParams::make sizes cap by the
  // digits that can occur); if it did, leave the group empty and flag it so
  // k_msm_horner / k_loc_search fail it -- never a wrong sum
  const bool ovf = scan[BS] > p.cap;  // block-uniform
  if (tid == 0) mw.sort_ovf[(LOC ? p.groups : 0) + slot] = ovf ? 1 : 0;
  if (ovf) {
    for (uint32_t t = tid; t < WH; t += BS) {
      mw.bk_start[bbase + t] = gbase;
      mw.bk_cnt[bbase + t] = 0;
    }
    for (uint32_t t = tid; t < p.cap; t += BS) mw.ent_bk[gbase + t] = kMsmEmpty;
    return;
  }
  {
    uint32_t off = scan[tid];
    for (uint32_t t = lo; t < hi; t++) {
      const uint32_t c = hist[t];
      mw.bk_start[bbase + t] = gbase + off;
      mw.bk_cnt[bbase + t] = c;
      hist[t] = off;  // cursor
      off += c;
    }
  }
  __syncthreads();

  // pass 2: scatter (point index << 1 | negate); stored points are -R, -A, +B.
  // Window by window: a window's H buckets are one contiguous slot range, so
  // its entries are placed in LDS first and then stored in order -- coalesced
  // lines, where scattering each entry straight to memory left partly
  // written lines behind (3.4x the sorted bytes in WRITE_SIZE).
  uint32_t *ent_pt = mw.ent_pt + gbase;
  uint32_t *ent_bk = mw.ent_bk + gbase;
  const uint32_t wcap = 2 * p.m() + 1;  // entries one window can hold: m R + m A digits + B
  uint32_t *st_pt = scan + BS + 1, *st_bk = st_pt + wcap;
  DigitReader<ZW> rz[R];
  DigitReader<8> rw[R], rb;
#pragma unroll
  for (int r = 0; r < R; r++) {
    rz[r].init(z[r]);
    rw[r].init(wv[r]);
  }
  rb.init(bsc);
  const uint32_t total = scan[BS];
  for (uint32_t w = 0; w < p.W; w++) {
    const uint32_t wbeg = hist[p.bucket(w, 0)];
    const uint32_t wend = w + 1 < p.W ? hist[p.bucket(w + 1, 0)] : total;
    __syncthreads();  // bounds read (and the previous window stored) before the cursors move
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (!live[r]) continue;
      const uint32_t e = e0 + tid + r * BS;
      if (w < WRz) {
        const int d = rz[r].next(p.c, w + 1 == WRz);
        if (d != 0) {
          const uint32_t bk = p.bucket(w, (uint32_t)((d < 0 ? -d : d) - 1));
          const uint32_t pos = atomicAdd(&hist[bk], 1u) - wbeg;  // < cap: checked above
          st_pt[pos] = ((KM ? e : 2 * e) << 1) | (d < 0 ? 1u : 0u);
          st_bk[pos] = bbase + bk;
        }
      }
      if (!KM) {
        const int d = rw[r].next(p.c, w + 1 == p.W);
        if (d != 0) {
          const uint32_t bk = p.bucket(w, (uint32_t)((d < 0 ? -d : d) - 1));
          const uint32_t pos = atomicAdd(&hist[bk], 1u) - wbeg;
          st_pt[pos] = ((2 * e + 1) << 1) | (d < 0 ? 1u : 0u);
          st_bk[pos] = bbase + bk;
        }
      }
    }
    if (!KM && tid == 0) {
      const int d = rb.next(p.c, w + 1 == p.W);
      if (d != 0) {
        const uint32_t bk = p.bucket(w, (uint32_t)((d < 0 ? -d : d) - 1));
        const uint32_t pos = atomicAdd(&hist[bk], 1u) - wbeg;
        st_pt[pos] = (mw.n_pts << 1) | (d < 0 ? 1u : 0u);
        st_bk[pos] = bbase + bk;
      }
    }
    __syncthreads();
    for (uint32_t i = tid; i < wend - wbeg; i += BS) {
      ent_pt[wbeg + i] = st_pt[i];
      ent_bk[wbeg + i] = st_bk[i];
    }
  }
  for (uint32_t t = total + tid; t < p.cap; t += BS) ent_bk[t] = kMsmEmpty;
}

#ifdef TMV_CHECKS
// Test build (-DTMV_CHECKS, tools/build_checks.sh; tests/test_gpu_checks.py
// reads these through tmv_internal_checks): joins named by k_msm_accum, joins
// k_msm_join_list found in its list, and buckets with entries whose sum was
// never written (k_check_buckets).  Round 5's lost-join race -- a part's sort
// resetting the list counter under another part's appends -- makes the
// first two differ and the third non-zero, where the product fails the
// groups closed (Z != 0 verdicts) and pays a fallback.
__device__ uint32_t g_joins_named, g_joins_done, g_buckets_unwritten;
#endif

// One lane per chunk of L sorted entries: sums each run of equal
// bucket ids with mixed additions.  A run that is the whole bucket goes to
// bk_sum.  A bucket cut by chunk edges: the lane whose run opens it holds
// the open run at its chunk's end, the lane whose chunk it ends in holds
// its first run.  When those are neighbouring lanes of one wave (a bucket
// over two chunks -- nearly every cut bucket: chunks hold 16 entries, the
// mean bucket 4-8), the second lane leaves its run in LDS and the first
// adds it after the loop and stores the whole bucket: no partials leave the
// wave.  The rest (a wave's edge, buckets over three or more chunks) keep
// their runs in part_last / part_first and name the bucket in join_b at the
// chunk of its last run, for k_msm_join_list.
// Register budget: the compiler's choice (145 VGPRs, 3 waves per SIMD); 4
// waves (128 VGPRs, 26 spilled) measured slower (profiles/r03/
// ab_register_budget.txt).  The chunk's bucket / point words are loaded as
// uint4 into register arrays that the rolled loop indexes by its wave-uniform
// counter (v_movrels): faster than reading them entry by entry, or than also
// prefetching the next Niels point (profiles/r04/ab_accum_r04m.txt) -- the
// gathers' latency, not the selects, is what the loop waits on.
template <int L>
__global__ void __launch_bounds__(256)
k_msm_accum(const uint32_t *count_ptr, uint32_t n, MsmWork mw, MsmParams p) {
  __shared__ ge_p3 first_run[256];  // a lane's first run, joined by its wave neighbour (40 KB)
  // blocks b and b + 8 share an XCD (round-robin dispatch): give each XCD a
  // contiguous range of the LIVE chunks so a group's points stay in one L2
  // (mixed batches size the grid for n but use only their kind's groups)
  const uint32_t cpg = p.chunks_per_group();
  const uint32_t live_groups = (entry_count(count_ptr, n) + p.m() - 1) >> p.m_log2;
  const uint32_t live_blocks = (live_groups * cpg + blockDim.x - 1) / blockDim.x;
  const uint32_t per_xcd = (live_blocks + 7) / 8;
  if ((blockIdx.x >> 3) >= per_xcd) return;
  const uint32_t lb = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const uint32_t t = lb * blockDim.x + threadIdx.x;
  const uint32_t g = t / cpg;
  if (g >= live_groups) return;
  const uint32_t base = t * L;
  const uint32_t lane = threadIdx.x & 63;
  // the chunk's words in registers: the loop below is not unrolled (L copies
  // of a 1,400-instruction body), so bk[q] / pt[q] are read with v_movrels
  // under s_set_gpr_idx (q is wave-uniform)
  uint32_t bk[L], pt[L];
  {
    const uint4 *b4 = reinterpret_cast<const uint4 *>(mw.ent_bk + base);
    const uint4 *p4 = reinterpret_cast<const uint4 *>(mw.ent_pt + base);
#pragma unroll
    for (int q = 0; q < L / 4; q++) {
      const uint4 x = b4[q], y = p4[q];
      bk[4 * q] = x.x; bk[4 * q + 1] = x.y; bk[4 * q + 2] = x.z; bk[4 * q + 3] = x.w;
      pt[4 * q] = y.x; pt[4 * q + 1] = y.y; pt[4 * q + 2] = y.z; pt[4 * q + 3] = y.w;
    }
  }
  if (bk[0] == kMsmEmpty) return;  // padding: nothing to sum or join
  uint32_t join = kMsmEmpty;  // this chunk's join_b
  auto flush = [&](uint32_t b, uint32_t rs, uint32_t re, const ge_p3 &acc) {
    const uint32_t bs = mw.bk_start[b], be = bs + mw.bk_cnt[b];
    if (rs == bs && re == be) {
      mw.bk_sum[b] = acc;
    } else if (re == base + L && re < be) {
      mw.part_last[t] = acc;  // (the open run at the chunk's end: see below)
    } else if (lane != 0 && bs >= base - L) {  // ends here, opened by the previous lane
      first_run[threadIdx.x] = acc;
    } else {
      mw.part_first[t] = acc;
      join = b;
    }
  };
  // every lane's first run starts at entry 0: take that point as the
  // accumulator (one multiply) instead of adding it to the identity (seven)
  ge_p3 acc;
  const uint32_t pt0 = pt[0];
  if (kNielsPer == 2) {  // the signed point's own slot
    const niels_pt P = mw.pts[pt0];
    niels_to_p3(acc, P.ypx, P.ymx);
  } else {
    const niels_pt P = mw.pts[pt0 >> 1];
    const bool neg = pt0 & 1;
    niels_to_p3(acc, neg ? P.ymx : P.ypx, neg ? P.ypx : P.ymx);
  }
  uint32_t cur = bk[0], rs = base;
  uint32_t j = 1;
  bool more = true;
  uint32_t bn = bk[1], pn = pt[1];  // loaded one entry ahead
#pragma unroll
  for (int q = 1; q < L; q++) {
    const uint32_t bq = bn, pq = pn;
    if (q + 1 < L) {
      bn = bk[q + 1];
      pn = pt[q + 1];
    }
    more = more && bq != kMsmEmpty;  // padding only follows the last bucket
    if (!more) continue;
    if (bq != cur) {
      flush(cur, rs, base + q, acc);
      ge_p3_identity(acc);
      cur = bq;
      rs = base + q;
    }
    ge_precomp np;
    const niels_pt P = mw.pts[kNielsPer == 2 ? pq : pq >> 1];
    if (kNielsPer == 2) {
      np.ypx = P.ypx;
      np.ymx = P.ymx;
      np.xy2d = P.xy2d;
    } else {
      const bool neg = pq & 1;
      np.ypx = neg ? P.ymx : P.ypx;
      np.ymx = neg ? P.ypx : P.ymx;
      fe_neg(np.xy2d, P.xy2d);
      fe_cmov(np.xy2d, P.xy2d, !neg);
    }
    ge_p1p1 r;
    ge_madd(r, acc, np);
    ge_p1p1_to_p3(acc, r);
    j = q + 1;
  }
  // the last run: whole, ending in this chunk, or open at the chunk's end
  const uint32_t bs = mw.bk_start[cur], be = bs + mw.bk_cnt[cur];
  const uint32_t re = base + j;
  const bool open = re == base + L && re < be;
  const bool join_next = open && bs >= base && lane != 63 && be <= base + 2 * L;
  if (!open) flush(cur, rs, re, acc);
  else if (!join_next) mw.part_last[t] = acc;
  // the first runs are in LDS: wave-local exchange, no workgroup barrier
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (join_next) {
    p3_add(acc, first_run[threadIdx.x + 1]);
    mw.bk_sum[cur] = acc;
  }
  // append this wave's joins to the launch's list: one atomic per wave, by
  // its lowest joining lane
  const uint64_t jm = __ballot(join != kMsmEmpty);
  if (jm) {  // wave-uniform
    const int leader = __ffsll((unsigned long long)jm) - 1;
    uint32_t jb = 0;
    if ((int)lane == leader) jb = atomicAdd(mw.join_count, (uint32_t)__popcll(jm));
    jb = __shfl(jb, leader);
    if (join != kMsmEmpty) mw.join_b[jb + __popcll(jm & ((1ull << lane) - 1))] = join;
#ifdef TMV_CHECKS
    if ((int)lane == leader) atomicAdd(&g_joins_named, (uint32_t)__popcll(jm));
#endif
  }
}

// The buckets k_msm_accum could not join inside a wave (~7% of the chunks at
// the bench's shape): k_msm_accum appended them to a packed list (one atomic
// per wave), and this kernel strides over it with every lane busy.  (Rounds
// 2-5 scanned one join word per chunk instead: 2.56M join 577 -> 381 us per
// launch with the list, profiles/r05/ab_join_list.txt.)
__global__ void __launch_bounds__(256)
k_msm_join_list(MsmWork mw, MsmParams p) {
  const uint32_t cnt = *mw.join_count;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
    // a listed bucket spans two or more chunks: the run that left its first
    // chunk, the middle chunks, the run that ended in its last (bucket_value,
    // written out so the partials stay in registers, not scratch)
    const uint32_t b = mw.join_b[i];
    const uint32_t bs = mw.bk_start[b], t0 = bs / p.L, t1 = (bs + mw.bk_cnt[b] - 1) / p.L;
    ge_p3 acc = mw.part_last[t0];
    for (uint32_t t = t0 + 1; t < t1; t++) {
      const ge_p3 q = mw.part_last[t];
      p3_add(acc, q);
    }
    const ge_p3 q = mw.part_first[t1];
    p3_add(acc, q);
    mw.bk_sum[b] = acc;
#ifdef TMV_CHECKS
    atomicAdd(&g_joins_done, 1u);
#endif
  }
}

// Running sums: register budget the compiler's choice (178 VGPRs, 2 waves;
// 3 waves measured the same, profiles/r03/ab_register_budget.txt); loading
// the next bucket's sum one step ahead measured no faster (the kernel waits
// on its addition chains, profiles/r04/ab_wpart_prefetch.txt).

// A window sum as k_msm_horner reads it: the top window (Horner's start) as a
// P3Q point (X, Y, Z, T), every other window already in CachedQ order
// (Y-X, Y+X, 2dT, Z, carried), so Horner's chain adds it without a
// to_cached multiply of its own (one field multiplication per window here,
// on the running-sum lane, instead of one per window on Horner's chain).
__device__ __forceinline__ void store_window_sum(ge_p3 *dst, const ge_p3 &S, bool top) {
  if (top) {
    *dst = S;
    return;
  }
  ge_p3 q;
  fe t;
  fe_sub(t, S.Y, S.X);
  fe_carry(q.X, t);
  fe_add(t, S.Y, S.X);
  fe_carry(q.Y, t);
  fe_mul(q.Z, S.T, consts::d2());
  q.T = S.Z;
  *dst = q;
}

// Window parts: lane (g, w, q) sums buckets [q s, (q+1) s) of window w with
// the running-sum trick: T = sum_i (i+1) B_{qs+i}, U = sum_i B_{qs+i}.
// Buckets are whole (joined by k_msm_accum or k_msm_join_list).  One lane per
// window (P = 1) keeps U in cached form only: U += B adds the P3 bucket sum
// to the cached U and converts the result straight back, T += U takes that
// cached U -- 17 multiplications a bucket instead of 18.
__global__ void __launch_bounds__(256)
k_msm_wpart(const uint32_t *count_ptr, uint32_t n, MsmWork mw, MsmParams p) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t per_group = p.W * p.P;
  const uint32_t g = t / per_group;
  if (g >= p.groups || (g << p.m_log2) >= entry_count(count_ptr, n)) return;
  const uint32_t r = t - g * per_group, wdx = r / p.P, part = r % p.P;
  const uint32_t s = p.H / p.P;
  ge_p3 U, T;
  bool u_set = false, t_set = false;
  const uint32_t gb = g * p.W * p.H, i0 = part * s;
  if (p.P == 1) {  // U only as the cached addend; T starts as the first B
    ge_cached Uc;
    uint32_t cnt = mw.bk_cnt[gb + p.bucket(wdx, s - 1)];
    for (int i = (int)s - 1; i >= 0; i--) {
      const uint32_t c_i = cnt;
      if (i > 0) cnt = mw.bk_cnt[gb + p.bucket(wdx, (uint32_t)i - 1)];
      ge_p1p1 rr;
      bool first = false;
      if (c_i) {
        const ge_p3 B = mw.bk_sum[gb + p.bucket(wdx, (uint32_t)i)];
        if (u_set) {
          ge_add(rr, B, Uc);
          ge_p1p1_to_cached(Uc, rr);
        } else {
          ge_p3_to_cached(Uc, B);
          T = B;
          u_set = t_set = first = true;
        }
      }
      if (u_set && !first) {
        ge_add(rr, T, Uc);
        ge_p1p1_to_p3(T, rr);
      }
    }
  } else {
    // the next bucket's count is loaded one iteration ahead, so only its
    // point load is exposed
    uint32_t cnt = mw.bk_cnt[gb + p.bucket(wdx, i0 + s - 1)];
    for (int i = (int)s - 1; i >= 0; i--) {
      const uint32_t c_i = cnt;
      if (i > 0) cnt = mw.bk_cnt[gb + p.bucket(wdx, i0 + (uint32_t)i - 1)];
      if (c_i) {
        const ge_p3 B = mw.bk_sum[gb + p.bucket(wdx, i0 + (uint32_t)i)];
        if (u_set) p3_add(U, B);
        else { U = B; u_set = true; }
      }
      if (u_set) {
        if (t_set) p3_add(T, U);
        else { T = U; t_set = true; }
      }
    }
  }
  if (!u_set) ge_p3_identity(U);
  if (!t_set) ge_p3_identity(T);
  if (p.P > 1) {
    mw.wpart[2ull * t] = T;
    mw.wpart[2ull * t + 1] = U;
  } else {  // T is the window sum: k_msm_horner reads it
    store_window_sum(&mw.wpart[2ull * t], T, wdx == p.W - 1);
  }
}

// Window sums: S_w = sum_q T_q + s * sum_q q U_q (s = H / P).
__global__ void __launch_bounds__(256)
k_msm_wsum(const uint32_t *count_ptr, uint32_t n, MsmWork mw, MsmParams p) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = t / p.W;
  if (g >= p.groups || (g << p.m_log2) >= entry_count(count_ptr, n)) return;
  const ge_p3 *wp = mw.wpart + 2ull * t * p.P;
  ge_p3 acc;
  if (p.P > 1) {
    ge_p3 r = wp[2 * (p.P - 1) + 1];
    acc = r;
    for (uint32_t q = p.P - 2; q >= 1; q--) {
      p3_add(r, wp[2 * q + 1]);
      p3_add(acc, r);
    }
    for (uint32_t d = p.H / p.P; d > 1; d >>= 1) p3_dbl(acc);
    for (uint32_t q = 0; q < p.P; q++) p3_add(acc, wp[2 * q]);
  } else {
    acc = wp[0];
  }
  store_window_sum(&mw.wsum[t], acc, t - g * p.W == p.W - 1);
}

// Group verdicts: one quad per group (lane c holds coordinate c), 16 groups
// per wave; T_g = sum_w 2^(c w) S_w by Horner, then
//   ed25519: [8] T_g == O;  sr25519: T_g is the Ristretto identity.
// A failing group's T_g goes to mw.fail_T at its place in the failing list.
// LOC: the same Horner over the locate MSM's slots (count_ptr = loc_count),
// T'_f to mw.fail_T, no verdict.
template <bool SR, bool KM, bool LOC>
__device__ __forceinline__ void horner_block(uint32_t bx, const uint32_t *count_ptr, uint32_t n, MsmWork mw,
                                             const MsmParams &p, const uint32_t *__restrict__ group_run0,
                                             uint32_t n_runs) {
  const uint32_t live_groups = (entry_count(count_ptr, n) + p.m() - 1) >> p.m_log2;
  if (bx * 16 >= live_groups) return;  // block-uniform
  const uint32_t raw = bx * 16 + (threadIdx.x >> 2);
  const bool live = raw < live_groups;
  const uint32_t g = live ? raw : live_groups - 1;  // whole quads stay active for DPP
  const int c = (int)(threadIdx.x & 3);
  // one running-sum lane per window (P = 1): its T is the window sum, read
  // in place (k_msm_wsum does not run)
  const uint32_t st = p.P == 1 ? 2 : 1;
  const ge_p3 *S = p.P == 1 ? mw.wpart + 2ull * g * p.W : mw.wsum + (size_t)g * p.W;
  fe acc = reinterpret_cast<const fe *>(&S[st * (p.W - 1)])[c];
  fe r, q, qc;
  for (int wI = (int)p.W - 2; wI >= 0; wI--) {
    qc = reinterpret_cast<const fe *>(&S[st * wI])[c];  // CachedQ (store_window_sum), loaded ahead
    for (uint32_t d = 0; d < p.c; d++) {
      quad::dbl(r, acc);
      quad::p1p1_to_p3(acc, r);
    }
    quad::add(r, acc, qc);
    quad::p1p1_to_p3(acc, r);
  }
  if (KM) {  // + the group's key-run points and its B-term point (k_msm_items)
    const uint32_t r0 = group_run0[g], r1 = group_run0[g + 1];
    for (uint32_t it = r0; it <= r1; it++) {
      q = mw.item_pt[4ull * (it < r1 ? it : n_runs + g) + c];
      quad::to_cached(qc, q);
      quad::add(r, acc, qc);
      quad::p1p1_to_p3(acc, r);
    }
  }
  if (LOC) {
    if (live) mw.fail_T[8ull * g + 4 + c] = acc;
    return;
  }
  bool ok;
  if (SR) {
    fe id;
    quad::p3_identity(id);
    ok = quad::ristretto_equal(acc, id);
  } else {
    ok = quad::is_identity_times8(acc);
  }
  ok = ok && !mw.sort_ovf[g];
  int f = -1;
  if (live && c == 0) {
    mw.group_ok[g] = ok ? 1 : 0;
    if (!ok && mw.fail_list) {
      f = (int)atomicAdd(mw.fail_count, 1u);
      mw.fail_list[f] = g;
    }
  }
  f = __builtin_amdgcn_mov_dpp(f, quad::qp(0, 0, 0, 0), 0xF, 0xF, false);  // the quad's lane 0
  if (f >= 0 && mw.fail_T) mw.fail_T[8ull * f + c] = acc;
}

template <bool SR, bool KM, bool LOC = false>
__global__ void __launch_bounds__(64)
k_msm_horner(const uint32_t *count_ptr, uint32_t n, MsmWork mw, MsmParams p, const uint32_t *__restrict__ group_run0,
             uint32_t n_runs) {
  horner_block<SR, KM, LOC>(blockIdx.x, count_ptr, n, mw, p, group_run0, n_runs);
}

// Horner with helpers (launches below the located fallback's size): blocks
// [0, hblocks) are k_msm_horner's, raised to s_setprio 3, and the rest reduce
// every entry's k to its half-size scalars (halfscalar.h) into w.hs_buf, so
// the per-entry fallback of the failing groups skips its reduction.  The
// Horner chain occupies about one SIMD in eight; the reductions run on the
// idle ones while it does (a 125k launch: ~33 us of chip time inside a
// ~225 us chain), not after it.
template <bool SR>
__global__ void __launch_bounds__(64)
k_msm_horner_helped(const uint32_t *count_ptr, uint32_t n, MsmWork mw, MsmParams p, Ed25519Work w,
                    uint32_t hblocks) {
  if (blockIdx.x < hblocks) {  // block-uniform
    __builtin_amdgcn_s_setprio(3);
    horner_block<SR, false, false>(blockIdx.x, count_ptr, n, mw, p, nullptr, 0u);
    return;
  }
  const uint32_t e = (blockIdx.x - hblocks) * 64 + threadIdx.x;
  if (e >= entry_count(count_ptr, n)) return;
  const uint4 *kp = reinterpret_cast<const uint4 *>(w.k + 8ull * e);
  const uint4 k0 = kp[0], k1 = kp[1];
  const uint32_t k[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
  uint32_t u[4], v[4];
  bool neg = false;
  const bool fast = half::reduce(u, neg, v, k);
  uint4 *hd = reinterpret_cast<uint4 *>(w.hs_buf + 12ull * e);
  hd[0] = make_uint4(u[0], u[1], u[2], u[3]);
  hd[1] = make_uint4(v[0], v[1], v[2], v[3]);
  hd[2] = make_uint4((fast ? 1u : 0u) | (neg ? 2u : 0u), 0u, 0u, 0u);
}

// Located fallback, search stage: one wave per failing group (slot f).  With
// M = [8] T_f and M' = [8] T'_f (sr25519: T and T' themselves, compared as
// Ristretto points), the group holds exactly one entry j whose term is not
// torsion iff M' = [j + 1] M: M has prime order l and (j + 1) < l, so j is
// unique; with two or more such entries a match needs the random weights to
// satisfy a fixed linear relation (probability ~2^-128 per candidate).
// Quad q tries j = q, q + 16, ...: [q + 1] M, then + [16] M each step.  One
// match: only entry j is verified one by one (every other entry keeps its
// pre-check status); otherwise every entry of the group is.
template <bool SR>
__global__ void __launch_bounds__(64)
k_loc_search(const uint32_t *count_ptr, uint32_t n, MsmWork mw, MsmParams p) {
  __shared__ int s_cnt, s_j;
  __shared__ uint32_t s_base;
  const uint32_t f = blockIdx.x;
  if (f >= *mw.fail_count) return;  // block-uniform
  const int c = (int)(threadIdx.x & 3), q = (int)(threadIdx.x >> 2);
  if (threadIdx.x == 0) {
    s_cnt = 0;
    s_j = -1;
  }
  fe M = mw.fail_T[8ull * f + c], Mp = mw.fail_T[8ull * f + 4 + c], r;
  if (!SR) {
    for (int i = 0; i < 3; i++) {
      quad::dbl(r, M);
      quad::p1p1_to_p3(M, r);
      quad::dbl(r, Mp);
      quad::p1p1_to_p3(Mp, r);
    }
  }
  fe Mc, Dc, P = M, D = M;
  quad::to_cached(Mc, M);
  const int k = q + 1;  // <= 16; quad-uniform
  for (int b = 30 - __builtin_clz((unsigned)k); b >= 0; b--) {
    quad::dbl(r, P);
    quad::p1p1_to_p3(P, r);
    if ((k >> b) & 1) {
      quad::add(r, P, Mc);
      quad::p1p1_to_p3(P, r);
    }
  }
  for (int i = 0; i < 4; i++) {
    quad::dbl(r, D);
    quad::p1p1_to_p3(D, r);
  }
  quad::to_cached(Dc, D);
  __syncthreads();  // s_cnt / s_j initialised
  const uint32_t m = p.m();
  for (uint32_t j = (uint32_t)q; j < m; j += 16) {
    const bool eq = SR ? quad::ristretto_equal(P, Mp) : quad::p3_equal(P, Mp);
    if (eq && c == 0) {
      atomicAdd(&s_cnt, 1);
      s_j = (int)j;
    }
    quad::add(r, P, Dc);
    quad::p1p1_to_p3(P, r);
  }
  __syncthreads();
  const uint32_t e0 = mw.fail_list[f] << p.m_log2;
  const uint32_t mlive = min(m, entry_count(count_ptr, n) - e0);
  const bool ovf = mw.sort_ovf[p.groups + f];
  if (s_cnt == 1 && (uint32_t)s_j < mlive && !ovf) {  // block-uniform
    if (threadIdx.x == 0) {
      mw.fb_list[atomicAdd(mw.fb_count, 1u)] = e0 + (uint32_t)s_j;
      atomicAdd(mw.loc_found, 1u);
    }
    return;
  }
  if (threadIdx.x == 0) s_base = atomicAdd(mw.fb_count, mlive);
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < mlive; t += 64) mw.fb_list[s_base + t] = e0 + t;
}

// Sub-group bisection (row H, before the per-entry fallback): a failing group
// usually holds one bad signature, so instead of verifying all m entries one
// by one, each sub-group of kSubGroup = 8 entries of a failing group is
// checked with the same equation and the same z_i,
//   T = [sum z_i s_i]B + sum [z_i](-R_i) + sum [z_i k_i](-A_i),
// by Straus with shared doublings (64 signed radix-16 windows; the 128-bit
// z_i need only the low 33; B digits radix 256 on even windows): 252
// doublings + ~810 additions for 8 entries, against 8 x (252 + 96) per
// entry.  Only the 16-entry fallback blocks holding a failing sub-group then
// verify entry by entry.  One quad per sub-group (lane c holds coordinate c);
// the failing groups come from k_msm_horner's list, so quads are dense.
// A passing sub-group carries the same <= 2^-128 false-accept bound as a
// group (z_i independent of the inputs).  Tables of (j+1)(-A), (j+1)(-R),
// j < 8, go to global scratch (w.tabA / mw.tabR, written and read by the
// same lane).
template <bool SR>
__global__ void __launch_bounds__(64)
k_msm_subcheck(const uint8_t *__restrict__ sig, const uint32_t *__restrict__ idx, const uint32_t *count_ptr,
               uint32_t n, Ed25519Work w, MsmWork mw, MsmParams p, MsmSeed seed, const fe *__restrict__ btab_q,
               int aligned, const uint32_t *__restrict__ list, const uint32_t *list_count) {
  constexpr int kQ = 16;                           // quads (sub-groups) per wave
  __shared__ int8_t dig[kQ][kSubGroup][2][64];     // [0]: z k mod l, [1]: z (33 digits used)
  __shared__ int8_t bdig[kQ][32];
  const uint32_t subs = *list_count << (p.m_log2 - kSubGroupLog2);
  if (blockIdx.x * kQ >= subs) return;  // block-uniform
  const int c = (int)(threadIdx.x & 3);
  const int q = (int)(threadIdx.x >> 2);
  const uint32_t raw = blockIdx.x * kQ + q;
  const bool live = raw < subs;
  const uint32_t t = live ? raw : subs - 1;  // whole quads stay active for DPP
  const uint32_t sh = p.m_log2 - kSubGroupLog2;
  const uint32_t g = list[t >> sh];
  const uint32_t e0 = (g << p.m_log2) + ((t & ((1u << sh) - 1)) << kSubGroupLog2);
  const uint32_t cnt = entry_count(count_ptr, n);

  // scalars: lane c takes entries c and c + 4 (as k_msm_sort forms them)
  uint32_t bacc[9];
#pragma unroll
  for (int u = 0; u < 9; u++) bacc[u] = 0;
  uint8_t in_sum = 0;  // bit jj: entry jj is part of the sums (all lanes learn it below)
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int jj = c + 4 * h;
    const uint32_t e = e0 + jj;
    uint32_t z[8], wv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) z[u] = wv[u] = 0;
    if (e < cnt) {
      const uint32_t i = idx ? idx[e] : e;
      uint32_t s_raw[8], s[8];
      if (aligned) load_words_aligned(s_raw, sig + 64ull * i + 32);
      else load_words_unaligned(s_raw, sig + 64ull * i + 32);
      bool s_ok;
      if (SR) {
        s_ok = sr25519_decode_s(s, s_raw);
      } else {
#pragma unroll
        for (int u = 0; u < 8; u++) s[u] = s_raw[u];
        s_ok = sc_is_canonical(s);
      }
      if (s_ok && w.flags[4 * e] && w.flags[4 * e + 1]) {
        in_sum |= (uint8_t)(1u << jj);
        uint32_t blk[16];
        chacha20_block(blk, seed.key, e, seed.nonce);
#pragma unroll
        for (int u = 0; u < 4; u++) z[u] = blk[u];
        uint32_t k[8];
        const uint4 *kp = reinterpret_cast<const uint4 *>(w.k + 8ull * e);
        const uint4 k0 = kp[0], k1 = kp[1];
        k[0] = k0.x; k[1] = k0.y; k[2] = k0.z; k[3] = k0.w;
        k[4] = k1.x; k[5] = k1.y; k[6] = k1.z; k[7] = k1.w;
        sc_mul_mod(wv, z, 4, k);
        uint32_t zs[8];
        sc_mul_mod(zs, z, 4, s);
        uint64_t cy = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
          cy += (uint64_t)bacc[u] + zs[u];
          bacc[u] = (uint32_t)cy;
          cy >>= 32;
        }
        bacc[8] += (uint32_t)cy;
      }
    }
    recode16_store(&dig[q][jj][0][0], wv, true);
    recode16_store(&dig[q][jj][1][0], z, true);
  }
  // B scalar: sum over the quad (each lane < 2 l, the total < 2^256), mod l
#pragma unroll
  for (int x = 1; x <= 2; x <<= 1) {
    uint32_t o[9];
#pragma unroll
    for (int u = 0; u < 9; u++) o[u] = (uint32_t)__shfl_xor((int)bacc[u], x, 4);
    uint64_t cy = 0;
#pragma unroll
    for (int u = 0; u < 9; u++) {
      cy += (uint64_t)bacc[u] + o[u];
      bacc[u] = (uint32_t)cy;
      cy >>= 32;
    }
  }
  in_sum |= (uint8_t)__shfl_xor((int)in_sum, 1, 4);
  in_sum |= (uint8_t)__shfl_xor((int)in_sum, 2, 4);
  if (c == 0) {
    uint32_t x[16], b[8];
#pragma unroll
    for (int u = 0; u < 16; u++) x[u] = u < 9 ? bacc[u] : 0;
    sc_reduce512(b, x);
    recode256_store(&bdig[q][0], b);
  }

  // tables of (j+1)(-R_e), (j+1)(-A_e) from the affine Niels points
  // (y+x, y-x, 2dxy): P3 = (2E, 2H, 4, E H) with E = ypx - ymx, H = ypx + ymx
#pragma unroll 1
  for (int jj = 0; jj < (int)kSubGroup; jj++) {
    if (!((in_sum >> jj) & 1)) continue;  // quad-uniform
    const uint32_t e = e0 + jj;
#pragma unroll 1
    for (int ra = 0; ra < 2; ra++) {
      const niels_pt &np = mw.pts[(2ull * e + ra) * kNielsPer];
      fe E, H, P;
      fe_sub(E, np.ypx, np.ymx);
      fe_add(H, np.ypx, np.ymx);
      fe_mul(P, E, H);  // T (every lane: quad-uniform work)
      if (c == 0) { fe_add(E, E, E); fe_carry(P, E); }
      else if (c == 1) { fe_add(H, H, H); fe_carry(P, H); }
      else if (c == 2) { fe_zero(P); P.v[0] = 4; }
      fe *tab = (ra ? w.tabA : mw.tabR) + 32ull * e;
      fe r, Pm, Q, Q0;
      quad::to_cached(Q0, P);
      tab[c] = Q0;
      quad::dbl(r, P);
      quad::p1p1_to_p3(Pm, r);
      quad::to_cached(Q, Pm);
      tab[4 + c] = Q;
      for (int m = 2; m < 8; m++) {
        quad::add(r, Pm, Q0);
        quad::p1p1_to_p3(Pm, r);
        quad::to_cached(Q, Pm);
        tab[m * 4 + c] = Q;
      }
    }
  }
  __syncthreads();  // digits written by other lanes (one wave per block)

  // Straus: 64 windows; per window 8 A additions, 8 R additions (windows <=
  // 32), one B addition (even windows), each addend loaded one addition
  // ahead (the window's first one before its doublings).  Entries left out
  // (or past the batch end, whose table slots may lie past the scratch) read
  // a B-table entry and add the identity.
  const fe *tA = w.tabA + 32ull * e0 + c;
  const fe *tR = mw.tabR + 32ull * e0 + c;
  auto adds_in = [](int wdx) { return 8 + (wdx <= 32 ? 8 : 0) + ((wdx & 1) ? 0 : 1); };
  auto fetch = [&](int wdx, int k, int &d) -> fe {
    if (k < 16) {
      const int jj = k & 7;
      const bool in = (in_sum >> jj) & 1;
      d = in ? dig[q][jj][k >> 3][wdx] : 0;
      const int a = d < 0 ? -d : d;
      return in ? (k < 8 ? tA : tR)[32 * jj + (a ? a - 1 : 0) * 4] : btab_q[c];
    }
    d = bdig[q][wdx >> 1];
    const int a = d < 0 ? -d : d;
    return btab_q[(a ? a - 1 : 0) * 4 + c];
  };
  fe idq, acc, r, nxt;
  int dn;
  quad::cached_identity(idq);
  quad::p3_identity(acc);
  nxt = fetch(63, 0, dn);
#pragma unroll 1
  for (int wdx = 63; wdx >= 0; wdx--) {
    if (wdx != 63) {
#pragma unroll
      for (int u = 0; u < 4; u++) {
        quad::dbl(r, acc);
        quad::p1p1_to_p3(acc, r);
      }
    }
    const int na = adds_in(wdx);
#pragma unroll 1
    for (int k = 0; k < na; k++) {
      fe ent = nxt;
      const int d = dn;
      if (k + 1 < na) {
        const int kn = (k + 1 >= 8 && wdx > 32) ? 16 : k + 1;  // a window > 32 has no R additions
        nxt = fetch(wdx, kn, dn);
      } else if (wdx > 0) {
        nxt = fetch(wdx - 1, 0, dn);
      }
      fe_cmov(ent, idq, d == 0);
      quad::cached_cneg(ent, d < 0);
      quad::add(r, acc, ent);
      quad::p1p1_to_p3(acc, r);
    }
  }
  bool ok;
  if (SR) {
    fe id;
    quad::p3_identity(id);
    ok = quad::ristretto_equal(acc, id);
  } else {
    ok = quad::is_identity_times8(acc);
  }
  if (live && c == 0) mw.sub_ok[e0 >> kSubGroupLog2] = ok ? 1 : 0;
}

// Dynamic LDS of k_msm_sort: the bucket counters / cursors, the scalar
// reduction, the scan, and one window's staged entries (point, bucket).
static size_t sort_smem(const MsmParams &p, uint32_t bs) {
  return ((size_t)p.W * p.H + bs * 9 + bs + 1 + 2 * (2 * p.m() + 1)) * sizeof(uint32_t);
}

#ifdef TMV_CHECKS
// Test build: every bucket with entries must have a sum written by this
// launch.  The bucket sums are zeroed before the accumulation runs, so a
// bucket whose join was lost keeps Z == 0 and is counted here.
__global__ void __launch_bounds__(256)
k_check_buckets(const uint32_t *count_ptr, uint32_t n, MsmWork mw, MsmParams p) {
  const uint32_t live_groups = (entry_count(count_ptr, n) + p.m() - 1) >> p.m_log2;
  const uint64_t nb = (uint64_t)live_groups * p.W * p.H;
  for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * blockDim.x) {
    if (!mw.bk_cnt[b]) continue;
    const fe &z = mw.bk_sum[b].Z;
    bool zero = true;
#pragma unroll
    for (int k = 0; k < 10; k++) zero = zero && z.v[k] == 0;
    if (zero) atomicAdd(&g_buckets_unwritten, 1u);
  }
}
#endif

// Bucket sums, window parts and window sums (shared by both forms).
// timed: bracket the first two kernels with the live kernel timer (the
// located fallback's second pass over the failing groups is not timed).
static hipError_t launch_buckets(const uint32_t *count_ptr, uint32_t n, MsmWork mw, const MsmParams &p,
                                 hipStream_t stream, bool timed = true) {
  const uint64_t chunks = (uint64_t)p.groups * p.chunks_per_group();
  const uint32_t ablocks = (uint32_t)((chunks + 255) / 256), per_xcd = (ablocks + 7) / 8;
  hipError_t e;
#ifdef TMV_CHECKS
  if ((e = hipMemsetAsync(mw.bk_sum, 0, (size_t)p.groups * p.W * p.H * sizeof(ge_p3), stream)) != hipSuccess) return e;
#endif
  void *tk = timed ? ktimer::begin(ktimer::kAccum, stream) : nullptr;
  if (p.L == 16)
    hipLaunchKernelGGL(k_msm_accum<16>, dim3(8 * per_xcd), dim3(256), 0, stream, count_ptr, n, mw, p);
  else
    hipLaunchKernelGGL(k_msm_accum<32>, dim3(8 * per_xcd), dim3(256), 0, stream, count_ptr, n, mw, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  ktimer::end(tk, stream);
  // lanes for ~3% of the chunks (C2 names ~2.5%); more joins stride
  const uint32_t jblocks = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((chunks / 32 + 255) / 256, 1), 8192);
  hipLaunchKernelGGL(k_msm_join_list, dim3(jblocks), dim3(256), 0, stream, mw, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
#ifdef TMV_CHECKS
  hipLaunchKernelGGL(k_check_buckets, dim3(1024), dim3(256), 0, stream, count_ptr, n, mw, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
#endif
  const uint64_t parts = (uint64_t)p.groups * p.W * p.P;
  tk = timed ? ktimer::begin(ktimer::kWpart, stream) : nullptr;
  hipLaunchKernelGGL(k_msm_wpart, dim3((uint32_t)((parts + 255) / 256)), dim3(256), 0, stream, count_ptr, n, mw, p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  ktimer::end(tk, stream);
  if (p.P == 1) return hipSuccess;  // the parts are the window sums
  const uint64_t rows = (uint64_t)p.groups * p.W;
  hipLaunchKernelGGL(k_msm_wsum, dim3((uint32_t)((rows + 255) / 256)), dim3(256), 0, stream, count_ptr, n, mw, p);
  return hipGetLastError();
}

// Sub-group bisection is worth its latency only for large groups: measured
// on C5 (1M mixed, ~1% invalid, one launch): m = 64 16.2 ms without, 16.9 ms
// with; m = 256 20.2 ms without, 19.4 ms with; the C2 bench (m = 64, 4
// launches in flight) 76.3 vs 69.7 M/s -- the check is a ~1.1k-addition
// chain per quad that lengthens every launch's critical path by ~1.4 ms.
// Default: groups of >= 256 entries (tmv_set_batch_options can force it on
// or off per context).
bool subcheck_enabled(uint32_t m_log2) { return m_log2 >= 8; }

// Test build counters (TMV_CHECKS), summed over every launch since the last
// reset; false in a product build.
bool read_checks(uint32_t out[3], bool reset) {
#ifdef TMV_CHECKS
  uint32_t v[3] = {0, 0, 0};
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(&v[0], HIP_SYMBOL(g_joins_named), 4) != hipSuccess ||
      hipMemcpyFromSymbol(&v[1], HIP_SYMBOL(g_joins_done), 4) != hipSuccess ||
      hipMemcpyFromSymbol(&v[2], HIP_SYMBOL(g_buckets_unwritten), 4) != hipSuccess)
    return false;
  for (int k = 0; k < 3; k++) out[k] = v[k];
  if (reset) {
    const uint32_t z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_joins_named), &z, 4);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_joins_done), &z, 4);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_buckets_unwritten), &z, 4);
  }
  return true;
#else
  (void)out;
  (void)reset;
  return false;
#endif
}

// Located fallback (k_msm_sort<LOC> .. k_loc_search): for launches of at
// least this many entries (TMV_LOCATE_MIN, 0 = never) a failing group gets a
// second, index-weighted MSM that names its one bad entry, so one entry is
// verified instead of the whole group; two bad entries in a group still
// fall back to all of them.  Less work (the second MSM costs about one
// group's share of the pipeline, the per-entry fallback ~64 verifications),
// a longer chain (a second Horner), so it pays where throughput, not the
// launch's latency, sets the rate.  C2 launches alone (profiles/r05/
// ab_locate_min.txt), located vs not: 250k 2.99 vs 2.65-2.70 ms, 500k 4.80 vs
// 4.73-4.81, 1M 8.67-8.92 vs 9.40.  Round 5 measured and removed two
// refinements for the groups the search cannot name (two or more bad
// entries): sub-group checks (profiles/r03/ab_loc_subcheck.txt) and a
// bisection MSM (profiles/r05/ab_loc_bisect.txt) -- both fewer one-by-one
// entries, both slower launches.  (Read at every launch: tests cover the
// located path below the default.)
static uint32_t locate_min() {
  const char *e = getenv("TMV_LOCATE_MIN");
  return e ? (uint32_t)strtoul(e, nullptr, 10) : 400000u;
}

uint32_t locate_min_entries() { return locate_min(); }

bool locate_enabled(uint32_t n, const MsmParams &p) {
  const uint32_t lmin = locate_min();
  return lmin && n >= lmin && !p.sub && p.WL() <= p.W;
}

// Views of a launch's work arrays for the entries of groups [g0, ...): the
// throughput stages of one part of a launch run on these exactly as on
// a whole batch (indices inside a view are relative), and the whole-launch
// stages (Horner, fallback) read the same arrays through the full structs.
static Ed25519Work work_view(Ed25519Work w, uint64_t e0) {
  w.negA += 4 * e0;
  w.Rc += 4 * e0;
  w.k += 8 * e0;
  w.flags += 4 * e0;
  w.tabA += 64 * e0;  // k_verify_quad's stride (k_msm_subcheck, tail only, uses 32 of it)
  w.hs_buf += 12 * e0;  // (w.hs stays null: the batch paths reduce in their fallback)
  return w;
}
static MsmWork msm_view(MsmWork mw, const MsmParams &p, uint32_t n, uint64_t g0) {
  const uint64_t e0 = g0 << p.m_log2, wh = (uint64_t)p.W * p.H;
  mw.pts += 2 * e0 * kNielsPer;
  mw.n_pts = (uint32_t)(2ull * n - 2 * e0);  // B keeps the launch's slot 2n
  mw.ent_pt += g0 * p.cap;
  mw.ent_bk += g0 * p.cap;
  mw.bk_start += g0 * wh;
  mw.bk_cnt += g0 * wh;
  mw.bk_sum += g0 * wh;
  mw.part_first += g0 * p.chunks_per_group();
  mw.part_last += g0 * p.chunks_per_group();
  mw.join_b += g0 * p.chunks_per_group();
  mw.join_count += g0;  // the view's own counter: parts may run at once
  mw.wpart += g0 * p.W * 2ull * p.P;
  mw.wsum += g0 * p.W;
  mw.group_ok += g0;
  mw.sort_ovf += g0;  // [g] of the part's groups (the located half is the tail's, full structs)
  if (mw.sub_ok) mw.sub_ok += (g0 << p.m_log2) / kSubGroup;
  if (mw.tabR) mw.tabR += 32 * e0;
  return mw;
}

// k_msm_sort over every group (LOC: every failing group's slot).  Groups of
// <= 256 entries take 64-thread workgroups (4 entries per thread at most):
// a 64-entry group in a 256-thread workgroup left 3 of 4 waves idle but
// resident through the sort's LDS phases (C2 bench, round 1: 80.4 / 80.7 ->
// 84.8 / 84.7 M/s).
template <bool SR, bool LOC>
static hipError_t launch_sort(const uint8_t *sig, const uint32_t *idx, const uint32_t *count_ptr, uint32_t n,
                              uint32_t e_base, const fe *btab_q, Ed25519Work w, MsmWork mw, const MsmParams &p,
                              const MsmSeed &seed, uint8_t *out, int aligned, hipStream_t stream) {
  if (p.m_log2 <= 8)
    hipLaunchKernelGGL((k_msm_sort<SR, false, 64, LOC>), dim3(p.groups), dim3(64), sort_smem(p, 64), stream, sig, idx,
                       count_ptr, n, w, mw, p, seed, btab_q, aligned, nullptr, nullptr, out, e_base);
  else
    hipLaunchKernelGGL((k_msm_sort<SR, false, kMsmSortBlock, LOC>), dim3(p.groups), dim3(kMsmSortBlock),
                       sort_smem(p, kMsmSortBlock), stream, sig, idx, count_ptr, n, w, mw, p, seed, btab_q, aligned,
                       nullptr, nullptr, out, e_base);
  return hipGetLastError();
}

// Throughput stages (prep, sort, bucket sums, window sums) of entries
// [e_base, e_base + n) of a launch; w / mw / out / pk / sig / msg_off are
// already offset to the part.
template <bool SR>
static hipError_t launch_part(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off,
                              const uint32_t *idx, const uint32_t *count_ptr, uint32_t n, uint32_t e_base,
                              const fe *btab_q, const strobe_t *prefix, Ed25519Work w, MsmWork mw,
                              const MsmParams &p, const MsmSeed &seed, uint8_t *out, int aligned,
                              hipStream_t stream) {
  w.niels = mw.pts;
  hipError_t e = launch_prep<SR>(pk, sig, msg, msg_off, idx, count_ptr, n, prefix, w, aligned, stream);
  if (e != hipSuccess) return e;
  if ((e = launch_sort<SR, false>(sig, idx, count_ptr, n, e_base, btab_q, w, mw, p, seed, out, aligned, stream)) !=
      hipSuccess)
    return e;
  return launch_buckets(count_ptr, n, mw, p, stream);
}

// Latency stages of a whole launch: Horner over every group, then the
// located fallback (large launches) or the per-entry fallback of the failing
// groups.  Below the located size Horner runs beside helper workgroups that
// reduce every entry's k for the fallback (k_msm_horner_helped; 125k
// fallback 273 -> 238 us, profiles/r05/ab_horner_help.txt).
template <bool SR>
static hipError_t launch_tail(const uint8_t *sig, const uint32_t *idx, const uint32_t *count_ptr, uint32_t n,
                              const fe *btab_q, Ed25519Work w, MsmWork mw, const MsmParams &p, const MsmSeed &seed,
                              uint8_t *out, int aligned, hipStream_t stream) {
  hipError_t e;
  const bool located = locate_enabled(n, p);
  const bool helped = !located && w.hs_buf;
  const uint32_t hblocks = (p.groups + 15) / 16;
  if (helped) {
    hipLaunchKernelGGL(k_msm_horner_helped<SR>, dim3(hblocks + (n + 63) / 64), dim3(64), 0, stream, count_ptr, n, mw,
                       p, w, hblocks);
    w.hs = w.hs_buf;  // the fallback below takes the reductions
  } else {
    hipLaunchKernelGGL((k_msm_horner<SR, false>), dim3(hblocks), dim3(64), 0, stream, count_ptr, n, mw, p, nullptr,
                       0u);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (located) {
    // second MSM over the failing groups (slot f = f-th failing group), then
    // the search, then one-by-one verification of the listed entries only
    if ((e = launch_sort<SR, true>(sig, idx, count_ptr, n, 0u, btab_q, w, mw, p, seed, nullptr, aligned, stream)) !=
        hipSuccess)
      return e;
    const uint32_t n_slots = p.groups << p.m_log2;
    if ((e = launch_buckets(mw.loc_count, n_slots, mw, p, stream, false)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_msm_horner<SR, false, true>), dim3((p.groups + 15) / 16), dim3(64), 0, stream,
                       mw.loc_count, n_slots, mw, p, nullptr, 0u);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_loc_search<SR>, dim3(p.groups), dim3(64), 0, stream, count_ptr, n, mw, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return launch_quad_fallback<SR>(sig, idx, count_ptr, n, btab_q, w, mw.group_ok, p.m_log2, out, aligned, stream,
                                    nullptr, nullptr, nullptr, mw.fb_list, mw.fb_count);
  }
  const uint8_t *sub_ok = nullptr;
  if (p.sub) {
    // grid for every group failing; blocks past the failing count exit at once
    const uint64_t subs = (uint64_t)p.groups << (p.m_log2 - kSubGroupLog2);
    hipLaunchKernelGGL(k_msm_subcheck<SR>, dim3((uint32_t)((subs + 15) / 16)), dim3(64), 0, stream, sig, idx,
                       count_ptr, n, w, mw, p, seed, btab_q, aligned, (const uint32_t *)mw.fail_list,
                       (const uint32_t *)mw.fail_count);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    sub_ok = mw.sub_ok;
  }
  // the failing groups' entries only (k_msm_horner's list; every entry's
  // pre-check status was written by k_msm_sort)
  return launch_quad_fallback<SR>(sig, idx, count_ptr, n, btab_q, w, mw.group_ok, p.m_log2, out, aligned, stream,
                                  sub_ok, mw.fail_list, mw.fail_count);
}

template <bool SR>
static hipError_t launch_check(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off,
                               const uint32_t *idx, const uint32_t *count_ptr, uint32_t n, const fe *btab_q,
                               const strobe_t *prefix, Ed25519Work w, MsmWork mw, const MsmParams &p,
                               const MsmSeed &seed, uint8_t *out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  w.niels = mw.pts;
  hipError_t e = launch_part<SR>(pk, sig, msg, msg_off, idx, count_ptr, n, 0u, btab_q, prefix, w, mw, p, seed, out,
                                 aligned, stream);
  if (e != hipSuccess) return e;
  return launch_tail<SR>(sig, idx, count_ptr, n, btab_q, w, mw, p, seed, out, aligned, stream);
}

hipError_t launch_batch_check_part(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                   const uint32_t *msg_off, uint32_t n, uint32_t e0, uint32_t e1, const fe *btab_q,
                                   const strobe_t *prefix, Ed25519Work w, MsmWork mw, const MsmParams &p,
                                   const MsmSeed &seed, uint8_t *out, hipStream_t stream) {
  // a part is whole groups: it starts on a group edge and ends on one or at n
  if (e0 >= e1 || e1 > n || (e0 & (p.m() - 1)) || (e1 != n && (e1 & (p.m() - 1)))) return hipErrorInvalidValue;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  const uint32_t g0 = e0 >> p.m_log2;
  MsmParams pp = p;
  pp.groups = ((e1 - e0) + p.m() - 1) >> p.m_log2;
  w.niels = mw.pts;
  const uint64_t E = e0;
  if (sr)
    return launch_part<true>(pk + 32 * E, sig + 64 * E, msg, msg_off + E, nullptr, nullptr, e1 - e0, e0, btab_q,
                             prefix, work_view(w, E), msm_view(mw, p, n, g0), pp, seed, out ? out + E : nullptr,
                             aligned, stream);
  return launch_part<false>(pk + 32 * E, sig + 64 * E, msg, msg_off + E, nullptr, nullptr, e1 - e0, e0, btab_q,
                            prefix, work_view(w, E), msm_view(mw, p, n, g0), pp, seed, out ? out + E : nullptr,
                            aligned, stream);
}

hipError_t launch_batch_check_tail(bool sr, const uint8_t *pk, const uint8_t *sig, uint32_t n, const fe *btab_q,
                                   Ed25519Work w, MsmWork mw, const MsmParams &p, const MsmSeed &seed,
                                   uint8_t *out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  w.niels = mw.pts;
  if (sr) return launch_tail<true>(sig, nullptr, nullptr, n, btab_q, w, mw, p, seed, out, aligned, stream);
  return launch_tail<false>(sig, nullptr, nullptr, n, btab_q, w, mw, p, seed, out, aligned, stream);
}

hipError_t launch_batch_check_part_idx(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                       const uint32_t *msg_off, const uint32_t *idx, uint32_t nb, uint32_t e0,
                                       uint32_t e1, const fe *btab_q, const strobe_t *prefix, Ed25519Work w, MsmWork mw,
                                       const MsmParams &p, const MsmSeed &seed, uint8_t *out, hipStream_t stream) {
  if (e0 >= e1 || e1 > nb || (e0 & (p.m() - 1))) return hipErrorInvalidValue;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  const uint32_t g0 = e0 >> p.m_log2;
  MsmParams pp = p;
  pp.groups = ((e1 - e0) + p.m() - 1) >> p.m_log2;
  w.niels = mw.pts;
  // the entries stay where they are (idx holds their global indices, out is
  // indexed by them); the work arrays are views at slot e0
  if (sr)
    return launch_part<true>(pk, sig, msg, msg_off, idx + e0, nullptr, e1 - e0, e0, btab_q, prefix, work_view(w, e0),
                             msm_view(mw, p, nb, g0), pp, seed, out, aligned, stream);
  return launch_part<false>(pk, sig, msg, msg_off, idx + e0, nullptr, e1 - e0, e0, btab_q, prefix, work_view(w, e0),
                            msm_view(mw, p, nb, g0), pp, seed, out, aligned, stream);
}

hipError_t launch_batch_check_tail_idx(bool sr, const uint8_t *pk, const uint8_t *sig, const uint32_t *idx, uint32_t n,
                                       const fe *btab_q, Ed25519Work w, MsmWork mw, const MsmParams &p,
                                       const MsmSeed &seed, uint8_t *out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  w.niels = mw.pts;
  if (sr) return launch_tail<true>(sig, idx, nullptr, n, btab_q, w, mw, p, seed, out, aligned, stream);
  return launch_tail<false>(sig, idx, nullptr, n, btab_q, w, mw, p, seed, out, aligned, stream);
}

// Key-merged form: one quad per item.  Items [0, n_runs) are runs of one key
// inside a group: W = sum of z_e k_e over the run (mod l), then [W](-A) from
// the key's comb (64 additions).  Item n_runs + g is group g's B term:
// [sum z_e s_e]B from the base comb (32 additions).  Lane 0 of the quad
// forms the scalar and its digits; all four lanes add (quad arithmetic).
__global__ void __launch_bounds__(kQuadBlock)
k_msm_items(KeyRuns runs, uint32_t n_items, MsmWork mw, KeyTable kt, const fe *__restrict__ bcomb) {
  constexpr int kItems = kQuadBlock / 4;
  __shared__ int8_t dig[kItems][64];
  if (blockIdx.x * kItems >= n_items) return;  // block-uniform
  const int c = threadIdx.x & 3;
  const int q = threadIdx.x >> 2;
  const uint32_t raw = blockIdx.x * kItems + q;
  const bool live = raw < n_items;
  const uint32_t it = live ? raw : n_items - 1;
  const bool key = it < runs.n_runs;  // quad-uniform; runs precede B terms
  if (c == 0) {
    uint32_t sc[8];
    if (key) {
      uint32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t e = runs.lo[it]; e < runs.lo[it + 1]; e++) {
        const uint4 *wp = reinterpret_cast<const uint4 *>(mw.wscal + 8ull * e);
        const uint4 a = wp[0], b = wp[1];
        const uint32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint64_t cy = 0;
#pragma unroll
        for (int t = 0; t < 8; t++) {
          cy += (uint64_t)acc[t] + v[t];
          acc[t] = (uint32_t)cy;
          cy >>= 32;
        }
        acc[8] += (uint32_t)cy;
      }
      uint32_t x[16];
#pragma unroll
      for (int t = 0; t < 16; t++) x[t] = t < 9 ? acc[t] : 0;
      sc_reduce512(sc, x);
      recode16_store(&dig[q][0], sc, true);
    } else {
      const uint32_t *bs = mw.bscal + 8ull * (it - runs.n_runs);
#pragma unroll
      for (int t = 0; t < 8; t++) sc[t] = bs[t];
      recode256_store(&dig[q][0], sc);
    }
  }
  __syncthreads();  // one wave per block
  fe acc, idq;
  quad::p3_identity(acc);
  quad::cached_identity(idq);
  if (key) {
    const fe *krow = kt.tab + (size_t)runs.slot[it] * kKeyRowsEntries * 4;
    comb_accumulate<64>(acc, idq, [&](int t, int &dsg) -> const fe * {
      dsg = dig[q][t];
      const int a = dsg < 0 ? -dsg : dsg;
      return krow + ((t * 8) + (a ? a - 1 : 0)) * 4 + c;
    });
  } else {
    comb_accumulate<32>(acc, idq, [&](int t, int &dsg) -> const fe * {
      dsg = dig[q][t];
      const int a = dsg < 0 ? -dsg : dsg;
      return bcomb + ((t * kBaseQuadEntries) + (a ? a - 1 : 0)) * 4 + c;
    });
  }
  if (live) mw.item_pt[4ull * it + c] = acc;
}

template <bool SR>
static hipError_t launch_km(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, const uint32_t *msg_off,
                            const uint32_t *key_slot, KeyRuns runs, uint32_t n, KeyTable kt, const fe *bcomb,
                            const strobe_t *prefix, Ed25519Work w, MsmWork mw, const MsmParams &p,
                            const MsmSeed &seed, uint8_t *out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int aligned = ((((uintptr_t)pk) | ((uintptr_t)sig)) & 15) == 0;
  w.niels = mw.pts;
  hipError_t e = launch_prep_cached<SR>(pk, sig, msg, msg_off, runs.order, n, prefix, w, aligned, stream);
  if (e != hipSuccess) return e;
  const size_t smem = sort_smem(p, kMsmSortBlock);
  hipLaunchKernelGGL((k_msm_sort<SR, true>), dim3(p.groups), dim3(kMsmSortBlock), smem, stream, sig, runs.order, nullptr,
                     n, w, mw, p, seed, nullptr, aligned, key_slot, kt.ok, nullptr, 0u);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = launch_buckets(nullptr, n, mw, p, stream)) != hipSuccess) return e;
  const uint32_t n_items = runs.n_runs + p.groups;
  hipLaunchKernelGGL(k_msm_items, dim3((n_items + 15) / 16), dim3(kQuadBlock), 0, stream, runs, n_items, mw, kt, bcomb);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((k_msm_horner<SR, true>), dim3((p.groups + 15) / 16), dim3(64), 0, stream, nullptr, n, mw, p,
                     runs.group_run0, runs.n_runs);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return launch_comb_fallback<SR>(sig, key_slot, runs.order, n, w, kt, bcomb, out, aligned, mw.group_ok, p.m_log2,
                                  stream);
}

hipError_t launch_key_merged_check(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                   const uint32_t *msg_off, const uint32_t *key_slot, KeyRuns runs, uint32_t n,
                                   KeyTable kt, const fe *bcomb, const strobe_t *prefix, Ed25519Work w, MsmWork mw,
                                   const MsmParams &p, const MsmSeed &seed, uint8_t *out, hipStream_t stream) {
  if (sr) return launch_km<true>(pk, sig, msg, msg_off, key_slot, runs, n, kt, bcomb, prefix, w, mw, p, seed, out, stream);
  return launch_km<false>(pk, sig, msg, msg_off, key_slot, runs, n, kt, bcomb, prefix, w, mw, p, seed, out, stream);
}

hipError_t launch_batch_check(bool sr, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                              const uint32_t *msg_off, const uint32_t *idx, const uint32_t *count_ptr, uint32_t n,
                              const fe *btab_q, const strobe_t *prefix, Ed25519Work w, MsmWork mw,
                              const MsmParams &p, const MsmSeed &seed, uint8_t *out, hipStream_t stream) {
  if (sr) return launch_check<true>(pk, sig, msg, msg_off, idx, count_ptr, n, btab_q, prefix, w, mw, p, seed, out, stream);
  return launch_check<false>(pk, sig, msg, msg_off, idx, count_ptr, n, btab_q, prefix, w, mw, p, seed, out, stream);
}

hipError_t launch_mixed_batch_check(const uint8_t *kind, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg,
                                    const uint32_t *msg_off, uint32_t n, const fe *btab_q, const strobe_t *prefix,
                                    Ed25519Work w_ed, Ed25519Work w_sr, MsmWork m_ed, MsmWork m_sr,
                                    const MsmParams &p, const MsmParams &p_sr, const MsmSeed &seed_ed,
                                    const MsmSeed &seed_sr,
                                    uint32_t *counts, uint32_t *idx_ed, uint32_t *idx_sr, int8_t *status,
                                    hipStream_t stream, const KindStreams *ks) {
  if (n == 0) return hipSuccess;
  uint8_t *out = reinterpret_cast<uint8_t *>(status);
  hipError_t e = launch_partition(kind, n, counts, idx_ed, idx_sr, out, stream);
  if (e != hipSuccess) return e;
  // the sr25519 pipeline on the helper stream, forked after the partition
  // and joined at the end: the two kinds' pipelines (own work arrays, own
  // entries of `out`) overlap, so one kind's latency tail runs beside the
  // other's throughput stages
  hipStream_t s_sr = stream;
  if (ks && ks->helper && ks->fork && ks->join) {
    if ((e = hipEventRecord(ks->fork, stream)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(ks->helper, ks->fork, 0)) != hipSuccess) return e;
    s_sr = ks->helper;
  }
  e = launch_check<true>(pk, sig, msg, msg_off, idx_sr, counts + 1, n, btab_q, prefix, w_sr, m_sr, p_sr, seed_sr,
                         out, s_sr);
  if (e != hipSuccess) return e;
  e = launch_check<false>(pk, sig, msg, msg_off, idx_ed, counts, n, btab_q, prefix, w_ed, m_ed, p, seed_ed, out,
                          stream);
  if (e != hipSuccess) return e;
  if (s_sr != stream) {
    if ((e = hipEventRecord(ks->join, s_sr)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(stream, ks->join, 0)) != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace tmv
