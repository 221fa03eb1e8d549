// Fused device ops of the routed serving step (see router.h).
#include "router.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <string>

#include "hbm_cache.h"
#include "step_comm.h"
#include "trace.h"

#define RT_OK(expr)                                                                     \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw Error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + #expr); \
  } while (0)

namespace shellac {

namespace {

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
constexpr int kB = 256;
constexpr int64_t kGroupRows = 2048;  // rows per workgroup in the counting sort
constexpr int kMaxBuckets = 4097;

int group_grid(int64_t n, int64_t rows_per_group = kGroupRows) {
  int64_t g = (n + rows_per_group - 1) / rows_per_group;
  return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 1024);
}

int grid1(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>((n + kB - 1) / kB, 1), 8192); }

__device__ __forceinline__ int ring_owner_of(const Digest& k, const uint32_t* __restrict__ pts,
                                             const int32_t* __restrict__ own, int npts) {
  const uint32_t p = ring_position(k);
  int lo = 0, hi = npts;  // first point >= p (wrapping)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (pts[mid] < p) lo = mid + 1; else hi = mid;
  }
  return own[lo == npts ? 0 : lo];
}

// The ring (points + owners) staged in LDS for a kernel's binary searches: a search over
// global memory is ~11 dependent L2 round trips per key (k_route_hist took 27 us for 1M
// keys, most of it waiting). Rings of up to kRingLds points (25 shards x 160) fit;
// bigger ones are searched in place. Every thread of the workgroup must call it.
constexpr int kRingLds = 4096;
struct RingView {
  const uint32_t* pts;
  const int32_t* own;
};
__device__ __forceinline__ RingView stage_ring(const uint32_t* __restrict__ pts,
                                               const int32_t* __restrict__ own, int npts,
                                               uint32_t* s_pts, int32_t* s_own) {
  if (npts > kRingLds) return RingView{pts, own};
  for (int k = threadIdx.x; k < npts; k += blockDim.x) {
    s_pts[k] = pts[k];
    s_own[k] = own[k];
  }
  __syncthreads();
  return RingView{s_pts, s_own};
}

// The hot set as an open-addressing hash set (linear probing, load <= 1/2, an all-zero
// slot is empty): one or two bucket loads per key instead of the directory + binary
// search over the sorted set it replaced (5-6 dependent loads: ~100 us for a 64K-row SET
// batch beside the coalescing probe at 8 ranks).
__device__ __forceinline__ uint64_t hot_slot(const Digest& k, uint64_t mask) {
  return (k.lo ^ (k.hi * 0x9E3779B97F4A7C15ull)) & mask;
}
__device__ __forceinline__ bool hot_hash_has(const Digest& k, const Digest* __restrict__ tab,
                                             uint64_t mask) {
  for (uint64_t i = hot_slot(k, mask);; i = (i + 1) & mask) {
    const Digest e = tab[i];
    if (e.lo == k.lo && e.hi == k.hi) return true;
    if (e.lo == 0 && e.hi == 0) return false;
  }
}
__global__ __launch_bounds__(256) void k_hot_hash_build(const Digest* __restrict__ hot, int64_t n,
                                                        Digest* __restrict__ tab, uint64_t mask) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)gridDim.x * 256) {
    const Digest k = hot[j];
    if (k.lo == 0 && k.hi == 0) continue;  // the empty marker (never a real digest in practice)
    // claim a slot by its 128 bits: CAS on lo, then hi (a slot whose lo we won but whose
    // hi another builder set cannot happen: lo is claimed from 0 exactly once)
    for (uint64_t i = hot_slot(k, mask);; i = (i + 1) & mask) {
      unsigned long long* lo = reinterpret_cast<unsigned long long*>(&tab[i].lo);
      const unsigned long long old = atomicCAS(lo, 0ull, (unsigned long long)k.lo);
      if (old == 0ull) {
        tab[i].hi = k.hi;
        break;
      }
      if (old == k.lo) {
        // same low word: the slot is this digest only if hi matches (set by its claimer
        // before this kernel ends; duplicates in `hot` cannot occur, it is a set)
        break;
      }
    }
  }
}

__device__ __forceinline__ uint64_t align16(uint64_t v) { return (v + 15) & ~15ull; }

// --- counting sort -----------------------------------------------------------------
// table[d * G + b] = rows of workgroup b's contiguous range with dest d.
__global__ __launch_bounds__(kB) void k_gr_hist(const int32_t* __restrict__ dest, int64_t n,
                                                int32_t nb, int64_t plen,
                                                uint64_t* __restrict__ table) {
  extern __shared__ uint32_t s_c[];
  for (int d = threadIdx.x; d < nb; d += kB) s_c[d] = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * plen, i1 = min(n, i0 + plen);
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kB) atomicAdd(&s_c[dest[i]], 1u);
  __syncthreads();
  for (int d = threadIdx.x; d < nb; d += kB) table[(int64_t)d * gridDim.x + blockIdx.x] = s_c[d];
}

// One workgroup: exclusive scan of table[0..T) in place; counts[d] = bucket totals.
// Optionally (xtable != nullptr, routed GET plan) also writes the GET column of the
// exchange row, xtable[d * xstride] = counts[d] for d < nb - 1, and
// extras = {counts[nb - 1] (local replica hits), *rl_off_n (their response bytes)}.
__global__ __launch_bounds__(1024) void k_gr_scan(uint64_t* __restrict__ table, int64_t T,
                                                  int32_t nb, int32_t G,
                                                  int64_t* __restrict__ counts,
                                                  int64_t* __restrict__ xtable = nullptr,
                                                  const uint64_t* __restrict__ rl_off_n = nullptr,
                                                  int64_t* __restrict__ extras = nullptr,
                                                  int xstride = 3) {
  __shared__ unsigned long long s_w[16];
  __shared__ unsigned long long s_total;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t per = (T + 1023) / 1024;
  const int64_t a = min(T, per * t), b = min(T, a + per);
  unsigned long long mine = 0;
  for (int64_t i = a; i < b; ++i) mine += table[i];
  unsigned long long inc = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  if (t == 0) {
    unsigned long long run = 0;
    for (int k = 0; k < 16; ++k) {
      const unsigned long long v = s_w[k];
      s_w[k] = run;
      run += v;
    }
    s_total = run;
  }
  __syncthreads();
  unsigned long long run = s_w[w] + inc - mine;
  for (int64_t i = a; i < b; ++i) {
    const unsigned long long v = table[i];
    table[i] = run;
    run += v;
  }
  __syncthreads();
  for (int d = t; d < nb; d += 1024) {
    const uint64_t s0 = table[(int64_t)d * G];
    const uint64_t s1 = d + 1 < nb ? table[(int64_t)(d + 1) * G] : s_total;
    counts[d] = (int64_t)(s1 - s0);
    if (xtable) {
      if (d < nb - 1) xtable[(int64_t)d * xstride] = (int64_t)(s1 - s0);
      else {
        extras[0] = (int64_t)(s1 - s0);
        extras[1] = rl_off_n ? (int64_t)*rl_off_n : 0;
      }
    }
  }
}

__global__ __launch_bounds__(kB) void k_gr_scatter(const int32_t* __restrict__ dest, int64_t n,
                                                   int32_t nb, int64_t plen,
                                                   const uint64_t* __restrict__ table,
                                                   const uint32_t* __restrict__ rows,
                                                   int32_t row_words, uint32_t* __restrict__ out,
                                                   int64_t* __restrict__ perm) {
  extern __shared__ uint32_t s_cur[];
  for (int d = threadIdx.x; d < nb; d += kB) s_cur[d] = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * plen, i1 = min(n, i0 + plen);
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kB) {
    const int d = dest[i];
    const int64_t pos =
        (int64_t)table[(int64_t)d * gridDim.x + blockIdx.x] + atomicAdd(&s_cur[d], 1u);
    if (perm) perm[i] = pos;
    if (rows)
      for (int k = 0; k < row_words; ++k) out[pos * row_words + k] = rows[i * row_words + k];
  }
}

void hist_and_scan(const int32_t* dest, int64_t n, int32_t nb, uint64_t* ws, int64_t* counts,
                   int* G_out, int64_t* plen_out, hipStream_t s) {
  SH_CHECK(nb >= 1 && nb <= kMaxBuckets, "too many buckets");
  const int G = group_grid(n);
  const int64_t plen = (n + G - 1) / G;
  hipLaunchKernelGGL(k_gr_hist, dim3(G), dim3(kB), nb * sizeof(uint32_t), s, dest, n, nb, plen, ws);
  hipLaunchKernelGGL(k_gr_scan, dim3(1), dim3(1024), 0, s, ws, (int64_t)nb * G, nb, G, counts);
  RT_OK(hipGetLastError());
  *G_out = G;
  *plen_out = plen;
}

// --- GET / SET planning ------------------------------------------------------------
__global__ __launch_bounds__(kB) void k_route_gets(const Digest* __restrict__ keys, int64_t n,
                                                   const uint64_t* __restrict__ rsize,
                                                   const uint32_t* __restrict__ pts,
                                                   const int32_t* __restrict__ own, int npts,
                                                   int32_t w, int32_t* __restrict__ dest) {
  for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB)
    dest[i] = (rsize && rsize[i] > 0) ? w : ring_owner_of(keys[i], pts, own, npts);
}

// Routed GET plan, fused: dest of every key of this workgroup's contiguous range
// (owner, or `w` for a local replica hit) + its LDS histogram into table[d * G + b]
// (the k_gr_hist layout, so k_gr_scan / k_gr_scatter follow unchanged).
// With GET coalescing (`first`), a duplicate row (first[i] != i) stays local too: it
// is answered from its claiming row after the step (expand_coalesced), so it is never
// sent; `ndup` counts them (one atomic per workgroup).
__global__ __launch_bounds__(kB) void k_route_hist(const Digest* __restrict__ keys, int64_t n,
                                                   const uint64_t* __restrict__ rsize,
                                                   const uint32_t* __restrict__ pts,
                                                   const int32_t* __restrict__ own, int npts,
                                                   int32_t w, int64_t plen,
                                                   int32_t* __restrict__ dest,
                                                   uint64_t* __restrict__ table,
                                                   const uint32_t* __restrict__ first,
                                                   unsigned long long* __restrict__ ndup) {
  extern __shared__ uint32_t s_c[];
  __shared__ unsigned int s_dup;
  __shared__ uint32_t s_pts[kRingLds];
  __shared__ int32_t s_own[kRingLds];
  const int nb = w + 1;
  for (int d = threadIdx.x; d < nb; d += kB) s_c[d] = 0;
  if (threadIdx.x == 0) s_dup = 0;
  const RingView rv = stage_ring(pts, own, npts, s_pts, s_own);  // (barrier inside)
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * plen, i1 = min(n, i0 + plen);
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kB) {
    const bool dup = first && first[i] != (uint32_t)i;
    const int d = (dup || (rsize && rsize[i] > 0)) ? w : ring_owner_of(keys[i], rv.pts, rv.own, npts);
    dest[i] = d;
    atomicAdd(&s_c[d], 1u);
    if (dup) atomicAdd(&s_dup, 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < nb; d += kB) table[(int64_t)d * gridDim.x + blockIdx.x] = s_c[d];
  if (threadIdx.x == 0 && ndup && s_dup) atomicAdd(ndup, (unsigned long long)s_dup);
}

// The SET planner's input rows: workgroups [0, Gc) take the rows the previous step carried
// over (count on the device, clamped to the carry capacity, split evenly over the Gc
// workgroups), workgroups [Gc, Gc + Gs) the batch, plen rows each, so a carried row always
// sorts before the batch's rows of its destination (the batch's newer SETs win the
// owner's dedupe). A carried row keeps its destination and tier (cdest = rank | tier << 29):
// it is not routed again. Per-row outputs (owner, vpad): carried row j at j, batch row j at
// ccap + j.
struct SetRows {
  const Digest* keys;
  const uint32_t* vlen;
  const uint32_t* flags;
  const uint32_t* expire;
  const uint64_t* val_off;
  uint64_t values_base;
  int64_t n;
  const Digest* pkeys;  // owner copies' digests (simulated world), else null
  const Digest* ckeys;
  const uint32_t* cvlen;
  const uint32_t* cflags;
  const uint32_t* cexpire;
  const uint64_t* cval;  // absolute value addresses
  const int32_t* cdest;
  const unsigned long long* cn;
  int64_t ccap;
  int32_t Gc;
};
constexpr int kTierBit = 29;  // forced destination's tier (carried rows)
constexpr int kFanBit = 30;   // fan out to every rank (hot key)

__device__ __forceinline__ void set_range(const SetRows& r, int64_t plen, bool* carry,
                                          int64_t* i0, int64_t* i1, int64_t* v0) {
  const int b = blockIdx.x;
  *carry = b < r.Gc;
  if (*carry) {
    const int64_t nc = min((int64_t)*r.cn, r.ccap);
    const int64_t pc = (nc + r.Gc - 1) / r.Gc;
    *i0 = min(nc, (int64_t)b * pc);
    *i1 = min(nc, *i0 + pc);
    *v0 = 0;
  } else {
    *i0 = (int64_t)(b - r.Gc) * plen;
    *i1 = min(r.n, *i0 + plen);
    *v0 = r.ccap;
  }
}

// SET planning, fused: input row j goes to its owner and (fan-out) to every rank when
// its key is hot (tier 0 = owner copy, tier 1 = replica copy). Each workgroup handles
// a contiguous range: owner / padded length per row, and the rows AND value bytes per
// destination in one packed 64-bit LDS counter (rows | bytes << 32) so k_ps_scatter
// can hand out row slots and byte ranges in the same order.
__global__ __launch_bounds__(kB) void k_ps_dest_hist(
    SetRows sr, const uint32_t* __restrict__ pts, const int32_t* __restrict__ own, int npts,
    const Digest* __restrict__ hot_tab, uint64_t hot_mask,
    int32_t nb, int64_t plen, int32_t w, int32_t* __restrict__ owner,
    uint32_t* __restrict__ vpad, uint64_t* __restrict__ tcnt, uint64_t* __restrict__ tbytes) {
  extern __shared__ unsigned long long s_cb[];
  __shared__ uint32_t s_pts[kRingLds];
  __shared__ int32_t s_own[kRingLds];
  for (int d = threadIdx.x; d < nb; d += kB) s_cb[d] = 0;
  const RingView rv = stage_ring(pts, own, npts, s_pts, s_own);
  __syncthreads();
  bool carry;
  int64_t i0, i1, v0;
  set_range(sr, plen, &carry, &i0, &i1, &v0);
  for (int64_t j = i0 + threadIdx.x; j < i1; j += kB) {
    int ow;
    uint32_t vl;
    bool h = false;
    if (carry) {
      ow = sr.cdest[j];
      vl = sr.cvlen[j];
    } else {
      const Digest k = sr.keys[j];
      const int o = ring_owner_of(k, rv.pts, rv.own, npts);
      h = hot_tab != nullptr && hot_hash_has(k, hot_tab, hot_mask);
      ow = h ? (o | (1 << kFanBit)) : o;
      vl = sr.vlen[j];
    }
    owner[v0 + j] = ow;
    const uint32_t vp = vl == kSkipVlen ? 0u : (uint32_t)align16(vl);
    vpad[v0 + j] = vp;
    const unsigned long long inc = 1ull | ((unsigned long long)vp << 32);
    if (h) {
      for (int r = 0; r < w; ++r) atomicAdd(&s_cb[r], inc);
    } else {
      atomicAdd(&s_cb[ow & ((1 << kTierBit) - 1)], inc);
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < nb; d += kB) {
    const uint64_t c = s_cb[d];
    tcnt[(int64_t)d * gridDim.x + blockIdx.x] = c & 0xFFFFFFFFull;
    tbytes[(int64_t)d * gridDim.x + blockIdx.x] = c >> 32;
  }
}

// One workgroup: block-wide exclusive scan of t[0..T) in place, returns the total.
__device__ unsigned long long block_scan_inplace(uint64_t* __restrict__ t, int64_t T,
                                                 unsigned long long* s_w) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t per = (T + 1023) / 1024;
  const int64_t a = min(T, per * tid), b = min(T, a + per);
  unsigned long long mine = 0;
  for (int64_t i = a; i < b; ++i) mine += t[i];
  unsigned long long inc = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  __syncthreads();
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  if (tid == 0) {
    unsigned long long run = 0;
    for (int k = 0; k < 16; ++k) {
      const unsigned long long v = s_w[k];
      s_w[k] = run;
      run += v;
    }
    s_w[16] = run;
  }
  __syncthreads();
  unsigned long long run = s_w[wv] + inc - mine;
  for (int64_t i = a; i < b; ++i) {
    const unsigned long long v = t[i];
    t[i] = run;
    run += v;
  }
  const unsigned long long total = s_w[16];
  __syncthreads();
  return total;
}

// Scans both SET tables, then writes the SET blocks of this rank's exchange row:
// rows_col[p] = SET rows to peer p, bytes_col[p] = their value bytes (k_gr_scan writes
// the GET block on the other stream).
__global__ __launch_bounds__(1024) void k_ps_scan(uint64_t* __restrict__ tcnt,
                                                  uint64_t* __restrict__ tbytes, int32_t nb,
                                                  int32_t G, int64_t* __restrict__ cnt_s,
                                                  int64_t* __restrict__ rows_col,
                                                  int64_t* __restrict__ bytes_col) {
  __shared__ unsigned long long s_w[17];
  const int64_t T = (int64_t)nb * G;
  const unsigned long long tc = block_scan_inplace(tcnt, T, s_w);
  const unsigned long long tb = block_scan_inplace(tbytes, T, s_w);
  __syncthreads();
  const int w = nb - 1;
  for (int d = threadIdx.x; d < nb; d += 1024) {
    const uint64_t c1 = d + 1 < nb ? tcnt[(int64_t)(d + 1) * G] : tc;
    const uint64_t b1 = d + 1 < nb ? tbytes[(int64_t)(d + 1) * G] : tb;
    const int64_t c = (int64_t)(c1 - tcnt[(int64_t)d * G]);
    cnt_s[d] = c;
    if (d < w) {
      rows_col[d] = c;
      bytes_col[d] = (int64_t)(b1 - tbytes[(int64_t)d * G]);
    }
  }
}

// rec = {lo, hi, vlen | flags << 32, expire | (voff | tier << 31) << 32} where voff is
// the value's offset inside the destination peer's value block.
__global__ __launch_bounds__(kB) void k_ps_scatter(
    SetRows sr, int32_t nb, int64_t plen, const uint64_t* __restrict__ tcnt,
    const uint64_t* __restrict__ tbytes, const int32_t* __restrict__ owner,
    const uint32_t* __restrict__ vpad, int32_t w, int64_t* __restrict__ srec,
    uint64_t* __restrict__ sval, uint64_t* __restrict__ svoff) {
  extern __shared__ unsigned long long s_cb[];
  for (int d = threadIdx.x; d < nb; d += kB) s_cb[d] = 0;
  __syncthreads();
  const int G = gridDim.x;
  bool carry;
  int64_t i0, i1, v0;
  set_range(sr, plen, &carry, &i0, &i1, &v0);
  for (int64_t j = i0 + threadIdx.x; j < i1; j += kB) {
    const int ow = owner[v0 + j];
    const bool fan = (ow >> kFanBit) & 1;
    const int o = ow & ((1 << kTierBit) - 1);
    const uint64_t pad = vpad[v0 + j];
    Digest k;
    uint64_t r2, ex, src;
    if (carry) {
      k = sr.ckeys[j];
      r2 = (uint64_t)sr.cvlen[j] | ((uint64_t)sr.cflags[j] << 32);
      ex = sr.cexpire[j];
      src = sr.cval[j];
    } else {
      k = sr.keys[j];
      r2 = (uint64_t)sr.vlen[j] | ((uint64_t)(sr.flags ? sr.flags[j] : 0u) << 32);
      ex = sr.expire ? sr.expire[j] : 0u;
      src = sr.values_base + sr.val_off[j];
    }
    const int r0 = fan ? 0 : o, r1 = fan ? w : o + 1;
    for (int d = r0; d < r1; ++d) {
      const unsigned long long old = atomicAdd(&s_cb[d], 1ull | (pad << 32));
      const int64_t pos = (int64_t)tcnt[(int64_t)d * G + blockIdx.x] + (int64_t)(old & 0xFFFFFFFFull);
      const uint64_t vglob = tbytes[(int64_t)d * G + blockIdx.x] + (old >> 32);
      const uint64_t voff = vglob - tbytes[(int64_t)d * G];  // within the peer's value block
      const uint64_t tier = fan ? (d != o ? 1ull : 0ull) : (uint64_t)((ow >> kTierBit) & 1);
      int64_t* rec = srec + pos * 4;
      const Digest kk = (!carry && tier == 0 && sr.pkeys) ? sr.pkeys[j] : k;
      rec[0] = (int64_t)kk.lo;
      rec[1] = (int64_t)kk.hi;
      rec[2] = (int64_t)r2;
      rec[3] = (int64_t)(ex | ((voff | (tier << 31)) << 32));
      sval[pos] = src;
      svoff[pos] = vglob;
    }
  }
}

// Two-launch exclusive scan of n values (out[n] = total) that needs no sentinel:
// per-workgroup sums over contiguous ranges, then each workgroup adds the sums before it.
constexpr int kScanItems = 4096;
__global__ __launch_bounds__(kB) void k_scan_parts(const uint64_t* __restrict__ in, int64_t n,
                                                   uint64_t* __restrict__ parts) {
  __shared__ unsigned long long s_w[kB / 64];
  const int64_t i0 = (int64_t)blockIdx.x * kScanItems, i1 = min(n, i0 + kScanItems);
  unsigned long long v = 0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kB) v += in[i];
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int k = 0; k < kB / 64; ++k) t += s_w[k];
    parts[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kB) void k_scan_apply(const uint64_t* __restrict__ in, int64_t n,
                                                   const uint64_t* __restrict__ parts,
                                                   uint64_t* __restrict__ out) {
  __shared__ unsigned long long s_w[kB / 64];
  __shared__ unsigned long long s_base;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long pre = 0;
  for (int k = threadIdx.x; k < (int)blockIdx.x; k += kB) pre += parts[k];
  for (int d = 32; d > 0; d >>= 1) pre += __shfl_xor(pre, d);
  if (lane == 0) s_w[wv] = pre;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int k = 0; k < kB / 64; ++k) t += s_w[k];
    s_base = t;
  }
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * kScanItems, i1 = min(n, i0 + kScanItems);
  constexpr int per = kScanItems / kB;
  const int64_t a = min(i1, i0 + (int64_t)per * threadIdx.x), b = min(i1, a + per);
  unsigned long long mine = 0;
  for (int64_t i = a; i < b; ++i) mine += in[i];
  unsigned long long inc = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  __syncthreads();
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  unsigned long long run = s_base + inc - mine;
  for (int k = 0; k < wv; ++k) run += s_w[k];
  for (int64_t i = a; i < b; ++i) {
    out[i] = run;
    run += in[i];
  }
  if (b == n && a < b) out[n] = run;
  if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
}

}  // namespace

int64_t group_ws_words(int64_t n, int32_t nb) { return (int64_t)nb * group_grid(n) + 8; }

void group_rows(const int32_t* dest, int64_t n, int32_t nb, const void* rows, int32_t row_bytes,
                void* out_rows, int64_t* perm, int64_t* counts, uint64_t* ws, hipStream_t s) {
  SH_CHECK(row_bytes % 4 == 0, "row bytes must be a multiple of 4");
  if (n <= 0) {
    RT_OK(hipMemsetAsync(counts, 0, nb * sizeof(int64_t), s));
    return;
  }
  int G;
  int64_t plen;
  hist_and_scan(dest, n, nb, ws, counts, &G, &plen, s);
  hipLaunchKernelGGL(k_gr_scatter, dim3(G), dim3(kB), nb * sizeof(uint32_t), s, dest, n, nb, plen,
                     ws, (const uint32_t*)rows, row_bytes / 4, (uint32_t*)out_rows, perm);
  RT_OK(hipGetLastError());
}

void route_gets(const Digest* keys, int64_t n, const uint64_t* replica_size,
                const uint32_t* ring_pts, const int32_t* ring_owner, int32_t npts, int32_t w,
                int32_t* dest, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_route_gets, dim3(grid1(n)), dim3(kB), 0, s, keys, n, replica_size, ring_pts,
                     ring_owner, npts, w, dest);
  RT_OK(hipGetLastError());
}

// Exclusive scan with out[n] = total; parts needs ceil(n / kScanItems) words.
void scan_u64(const uint64_t* in, int64_t n, uint64_t* parts, uint64_t* out, hipStream_t s) {
  const int g = (int)std::max<int64_t>(1, (n + kScanItems - 1) / kScanItems);
  hipLaunchKernelGGL(k_scan_parts, dim3(g), dim3(kB), 0, s, in, n, parts);
  hipLaunchKernelGGL(k_scan_apply, dim3(g), dim3(kB), 0, s, in, n, parts, out);
  RT_OK(hipGetLastError());
}

int64_t scan_parts_words(int64_t n) { return (n + kScanItems - 1) / kScanItems + 1; }

}  // namespace shellac


// =====================================================================================
// RoutedStep: the device-driven routed step (see router.h for the layouts)
// =====================================================================================
namespace shellac {

namespace {

enum Slot {
  kRlLoc, kRlSize0, kRlSize1, kRlOff0, kRlOff1, kDestG, kRoute0, kRoute1, kCntG, kWsG,
  kCoTab, kFirst0, kFirst1, kOwnerS, kVpad, kTcnt, kTbytes, kSrec, kSval, kSvoff, kCntS,
  kOwnCnt, kLkLoc, kLkSize, kLkOff, kDstA, kDstB, kSrcA, kSrcB, kHdr, kUsed, kRb, kTab,
  kSegOff, kSegSrc, kTcnt1, kTbytes1, kCntS1, kSegOffF, kSegSrcF,
  kRkeys, kV0, kV1, kFl, kEx, kRoff, kReserve, kSrec1, kSval1, kSvoff1,
  // RoutedStep::step's own exchange buffers (the multi-call path gets them from Python)
  kRowB, kMatB, kGB, kR0, kR1, kS0, kS1, kRs0, kRs1, kNumSlots
};

// Slot of G a requester writes peer p's rows into: self = W-1, others W + o(p).
__device__ __forceinline__ int64_t g_slot(int p, int me, int W) {
  return p == me ? (int64_t)(W - 1) : (int64_t)W + (p < me ? p : p - 1);
}

// Counting-sort scatter of the GET rows into the request slots of G: peer p's rows go to
// its slot at their rank j within p's bucket (j >= capG: overflow, not written).
// route[i] = p << 32 | j for a row sent to p, -1 for a row answered locally (replica
// hit or coalesced duplicate).
__global__ __launch_bounds__(kB) void k_gr_scatter_slots(
    const int32_t* __restrict__ dest, int64_t n, int32_t nb, int64_t plen,
    const uint64_t* __restrict__ table, const Digest* __restrict__ keys, int64_t capG,
    int32_t me, uint8_t* __restrict__ G, int64_t* __restrict__ route) {
  // (keys: what the owner probes — the request digests, or their probe digests in a
  // simulated world, RoutedStep::set_probe_keys)
  extern __shared__ uint32_t s_cur[];
  const int W = nb - 1;
  for (int d = threadIdx.x; d < nb; d += kB) s_cur[d] = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * plen, i1 = min(n, i0 + plen);
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kB) {
    const int d = dest[i];
    const int64_t pos =
        (int64_t)table[(int64_t)d * gridDim.x + blockIdx.x] + atomicAdd(&s_cur[d], 1u);
    if (d == W) {
      route[i] = -1;
      continue;
    }
    const int64_t j = pos - (int64_t)table[(int64_t)d * gridDim.x];
    route[i] = ((int64_t)d << 32) | j;
    if (j < capG)
      reinterpret_cast<Digest*>(G)[g_slot(d, me, W) * capG + j] = keys[i];
  }
}

// Log bytes this step's received SETs may append to the main shard (records, padded
// values, the CLOCK hand's reinsertion budget): the owner probe treats what they will
// overwrite as evicted, so the SET chain can run beside the reply gather.
// One launch with k_derive's work: the rows each owner slot holds (own_cnt).
__global__ void k_owner_prep(const int64_t* __restrict__ mat, int64_t K, int32_t W, int32_t me,
                             int64_t capG, uint64_t rmax, uint64_t ahead,
                             int64_t* __restrict__ own_cnt, uint64_t* __restrict__ out) {
  for (int s = threadIdx.x; s < W; s += blockDim.x) {
    const int q = s == W - 1 ? me : (s < me ? s : s + 1);
    own_cnt[s] = min(mat[(int64_t)q * K + me], capG);
  }
  if (threadIdx.x != 0) return;
  uint64_t rows = 0, bytes = 0;
  for (int q = 0; q < W; ++q) {
    rows += (uint64_t)mat[(int64_t)q * K + W + me];
    bytes += (uint64_t)mat[(int64_t)q * K + 2 * W + me];
  }
  // `ahead`: the next step's SET bytes too (look-ahead, RoutedStep::step): its append may
  // then run before the next probe, beside this step's owner phase
  *out = 48 * rows + bytes + rmax + ahead;
}

// Reply bytes the owner probe found per requester (before any drop): out[q].
__global__ void k_demand(const uint64_t* __restrict__ lk_off, int32_t W, int32_t me, int64_t capG,
                         int64_t* __restrict__ out) {
  for (int s = threadIdx.x; s < W; s += blockDim.x) {
    const int q = s == W - 1 ? me : (s < me ? s : s + 1);
    out[q] = (int64_t)(lk_off[(int64_t)(s + 1) * capG] - lk_off[(int64_t)s * capG]);
  }
}

// Owner, reply slots as segments of one plain gather per destination buffer (others: R,
// self: data's self slot). Slot s = [header (capG x u64) | records | slack], as segments
// [header | one per row | slack] (capG + 2 per slot): the header segment copies the
// headers k_reply_prep wrote into `hdr`, the slack segment is a kSegSkip gap (the slot's
// unused tail: neither read nor written), so the segments tile the buffer.
// used[s] = the bytes of slot s's longest row prefix that fits capD (rows past it are
// dropped: header 0, no bytes).
// Also k_demand's work (rb[q] = reply bytes for requester q) and rb[W] = 0 (the dropped
// rows counter k_reply_prep adds to): one launch instead of three.
__global__ void k_reply_used(const uint64_t* __restrict__ lk_off, int32_t W, int32_t me,
                             int64_t capG, int64_t capD, int64_t slotR,
                             const uint64_t* __restrict__ hdr, uint64_t* __restrict__ used,
                             uint64_t* __restrict__ offA, uint64_t* __restrict__ srcA,
                             uint64_t* __restrict__ offB, uint64_t* __restrict__ srcB,
                             int64_t* __restrict__ rb) {
  const int64_t per = capG + 2;
  if (threadIdx.x == 0) rb[W] = 0;
  for (int s = threadIdx.x; s < W; s += blockDim.x) {
    const uint64_t base = lk_off[s * capG];
    const int q = s == W - 1 ? me : (s < me ? s : s + 1);
    rb[q] = (int64_t)(lk_off[(int64_t)(s + 1) * capG] - base);
    int64_t lo = 0, hi = capG;  // the largest j with lk_off[s capG + j] - base <= capD
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (lk_off[s * capG + mid] - base <= (uint64_t)capD) lo = mid; else hi = mid - 1;
    }
    const uint64_t u = lk_off[s * capG + lo] - base;
    used[s] = u;
    const bool self = s == W - 1;
    uint64_t* off = self ? offB : offA + s * per;
    uint64_t* src = self ? srcB : srcA + s * per;
    const uint64_t sb = self ? 0 : (uint64_t)s * (uint64_t)slotR;
    off[0] = sb;
    src[0] = (uint64_t)(uintptr_t)(hdr + s * capG);
    const uint64_t gap = (uint64_t)capG * 8 + u;
    off[capG + 1] = sb + gap;
    src[capG + 1] = kSegSkip;  // the slot's unused tail: a gap (was copied onto itself)
  }
  if (threadIdx.x == 0) {
    offA[(int64_t)(W - 1) * per] = (uint64_t)(W - 1) * (uint64_t)slotR;
    offB[per] = (uint64_t)slotR;
  }
}

__global__ __launch_bounds__(kB) void k_reply_prep(
    const uint64_t* __restrict__ lk_loc, const uint64_t* __restrict__ lk_size,
    const uint64_t* __restrict__ lk_off, const int64_t* __restrict__ own_cnt,
    const uint64_t* __restrict__ used, int32_t W, int64_t capG, int64_t slotR,
    const uint8_t* __restrict__ log, uint64_t* __restrict__ hdr, uint64_t* __restrict__ offA,
    uint64_t* __restrict__ srcA, uint64_t* __restrict__ offB, uint64_t* __restrict__ srcB,
    unsigned long long* __restrict__ dropped) {
  const int64_t rows = (int64_t)W * capG, per = capG + 2;
  for (int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * kB) {
    const int64_t s = r / capG, j = r - s * capG;
    const uint64_t sz = lk_size[r];
    const uint64_t off_in = lk_off[r] - lk_off[s * capG];
    const bool keep = sz > 0 && off_in + sz <= used[s];
    const bool self = s == W - 1;
    const uint64_t sb = self ? 0 : (uint64_t)s * (uint64_t)slotR;
    uint64_t* off = self ? offB : offA + s * per;
    uint64_t* src = self ? srcB : srcA + s * per;
    // zero-length rows (misses, padding, dropped) sit where the next kept row starts
    off[1 + j] = sb + (uint64_t)capG * 8 + min(off_in, used[s]);
    src[1 + j] = keep ? (uint64_t)(uintptr_t)(log + lk_loc[r]) : 0ull;
    hdr[r] = keep ? (sz << 32 | off_in) : 0ull;
    if (j < own_cnt[s] && sz > 0 && !keep) atomicAdd(dropped, 1ull);
  }
}

// Requester: (size, off) of every request row in `data` (0, 0 = miss; duplicates are
// filled in from their claimer by expand_coalesced afterwards).
// A coalesced duplicate (first[i] != i) takes its claiming row's record: each row
// evaluates its claimer directly, so no second expansion pass is needed. The local
// region holds the replica hits only if their total fit capL (one plain gather).
__global__ __launch_bounds__(kB) void k_assemble_slots(
    const int64_t* __restrict__ route, const uint32_t* __restrict__ first, int64_t n,
    int32_t W, int32_t me, int64_t capG, int64_t capL, int64_t slotR,
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ rl_size,
    const uint64_t* __restrict__ rl_off, uint64_t* __restrict__ out_size,
    uint64_t* __restrict__ out_off) {
  const bool local_ok = rl_size && rl_off[n] <= (uint64_t)capL;
  for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
    const int64_t c = first ? (int64_t)first[i] : i;
    const int64_t r = route[c];
    uint64_t sz = 0, off = 0;
    if (r < 0) {
      if (local_ok && rl_size[c] > 0) {
        sz = rl_size[c];
        off = rl_off[c];
      }
    } else {
      const int p = (int)(r >> 32);
      const int64_t j = r & 0xFFFFFFFFll;
      if (j < capG) {
        const int rs = p == me ? W - 1 : (p < me ? p : p - 1);
        const uint64_t base = (uint64_t)capL + (uint64_t)rs * (uint64_t)slotR;
        const uint64_t h = reinterpret_cast<const uint64_t*>(data + base)[j];
        sz = h >> 32;
        if (sz) off = base + (uint64_t)capG * 8 + (h & 0xFFFFFFFFull);
      }
    }
    out_size[i] = sz;
    out_off[i] = off;
  }
}

// SET send buffer segments: per destination d (send order: others by rank, self last)
// one segment of its records and one per value row. tab (rank order, per d):
// [Sstart (W+1) | Bstart (W) | Psend (W) | segbase (W)].
__global__ __launch_bounds__(kB) void k_set_segs(const uint64_t* __restrict__ tab, int32_t W,
                                                 int64_t rows, const uint64_t* __restrict__ sval,
                                                 const uint64_t* __restrict__ svoff,
                                                 uint64_t srec_base, uint64_t total,
                                                 uint64_t* __restrict__ seg_off,
                                                 uint64_t* __restrict__ seg_src) {
  const uint64_t* Sst = tab;
  const uint64_t* Bst = tab + W + 1;
  const uint64_t* Ps = Bst + W;
  const uint64_t* sb = Ps + W;
  for (int64_t t = (int64_t)blockIdx.x * kB + threadIdx.x; t <= rows + W;
       t += (int64_t)gridDim.x * kB) {
    if (t == rows + W) {
      seg_off[rows + W] = total;
    } else if (t >= rows) {  // destination d's record block
      const int d = (int)(t - rows);
      seg_off[sb[d]] = Ps[d];
      seg_src[sb[d]] = srec_base + 32 * Sst[d];
    } else {  // value row t (grouped by destination in rank order)
      int lo = 0, hi = W;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (Sst[mid] <= (uint64_t)t) lo = mid; else hi = mid;
      }
      const uint64_t nrec = Sst[lo + 1] - Sst[lo];
      const int64_t k = (int64_t)sb[lo] + 1 + (t - (int64_t)Sst[lo]);
      seg_off[k] = Ps[lo] + 32 * nrec + (svoff[t] - Bst[lo]);
      seg_src[k] = sval[t];
    }
  }
}

// Received SET rows (sources: others by rank, self last) -> store arguments. tab per
// source k: [first row (W+1) | record block address (W) | value block address (W)].
// The self block (k = W - 1) is not packed: its records are the planner's own (srec) and
// its values stay where the caller's batch holds them (self_sval: absolute addresses).
__global__ __launch_bounds__(kB) void k_rs_fill_slots(
    const uint64_t* __restrict__ tab, int32_t W, int64_t ms, Digest* __restrict__ keys,
    uint32_t* __restrict__ vlen0, uint32_t* __restrict__ vlen1, uint32_t* __restrict__ flags,
    uint32_t* __restrict__ expire, uint64_t* __restrict__ roff,
    const uint64_t* __restrict__ self_sval) {
  const uint64_t* first = tab;
  const uint64_t* rec = tab + W + 1;
  const uint64_t* val = rec + W;
  for (int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x; r < ms; r += (int64_t)gridDim.x * kB) {
    int lo = 0, hi = W;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (first[mid] <= (uint64_t)r) lo = mid; else hi = mid;
    }
    const int64_t* rr = reinterpret_cast<const int64_t*>(rec[lo] + 32 * (r - (int64_t)first[lo]));
    keys[r] = Digest{(uint64_t)rr[0], (uint64_t)rr[1]};
    const uint32_t vl = (uint32_t)rr[2];
    const uint64_t hi32 = (uint64_t)rr[3] >> 32;
    const uint32_t tier = (uint32_t)(hi32 >> 31);
    vlen0[r] = tier == 0 ? vl : kSkipVlen;
    vlen1[r] = tier == 1 ? vl : kSkipVlen;
    flags[r] = (uint32_t)((uint64_t)rr[2] >> 32);
    expire[r] = (uint32_t)rr[3];
    // absolute: the store's values base is 0
    roff[r] = lo == W - 1 ? self_sval[r - (int64_t)first[lo]] : val[lo] + (hi32 & 0x7FFFFFFFull);
  }
}

int64_t align_up64(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// ---- fixed-slot SET exchange (RoutedStep::step) -----------------------------------------
// set_meta_ words (W ranks): [slot headers {rows, bytes} x W (16-B aligned) | fit (W) |
// fit bytes (W) | segment base (W) | nseg, self block start, routed rows, 0...].
struct SetMeta {
  int W;
  __device__ __forceinline__ uint64_t* hdr(uint64_t* m) const { return m; }
  __device__ __forceinline__ uint64_t* fit(uint64_t* m) const { return m + 2 * W; }
  __device__ __forceinline__ uint64_t* fitb(uint64_t* m) const { return m + 3 * W; }
  __device__ __forceinline__ uint64_t* segbase(uint64_t* m) const { return m + 4 * W; }
  __device__ __forceinline__ uint64_t* tail(uint64_t* m) const { return m + 5 * W; }
};
int64_t set_meta_words(int W) { return 5 * (int64_t)W + 8; }

__device__ __forceinline__ uint32_t rec_vpad(const int64_t* rec) {
  const uint32_t vl = (uint32_t)rec[2];
  return vl == kSkipVlen ? 0u : (uint32_t)align16(vl);
}

// One workgroup. Per destination d (rank order): the rows that fit its slot (a prefix of
// its block: row j fits while j < capR and its value ends within capB; value offsets grow
// with j), their bytes, the slot header {rows, bytes} (others), and the segment bases of
// the send buffer's segment list (per other rank: header, records, gap, one per row, tail).
__global__ __launch_bounds__(256) void k_set_fit(const uint64_t* __restrict__ tcnt,
                                                 const uint64_t* __restrict__ tbytes, int64_t G,
                                                 const int64_t* __restrict__ cnt_s,
                                                 const int64_t* __restrict__ srec,
                                                 const uint64_t* __restrict__ svoff, int32_t W,
                                                 int32_t me, int64_t capS, int64_t capSB,
                                                 int64_t capSelf, int64_t capSelfB,
                                                 uint64_t* __restrict__ meta) {
  const SetMeta sm{W};
  for (int d = threadIdx.x; d < W; d += blockDim.x) {
    const uint64_t sst = tcnt[(int64_t)d * G], bst = tbytes[(int64_t)d * G];
    const int64_t cnt = cnt_s[d];
    const int64_t capR = d == me ? capSelf : capS;
    const uint64_t capB = (uint64_t)(d == me ? capSelfB : capSB);
    auto end_of = [&](int64_t j) {
      return svoff[sst + j] - bst + rec_vpad(srec + 4 * (sst + j));
    };
    int64_t lo = 0, hi = min(cnt, capR);  // largest f in [lo, hi] whose row f-1 fits
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (end_of(mid - 1) <= capB) lo = mid; else hi = mid - 1;
    }
    const uint64_t fb = lo ? end_of(lo - 1) : 0;
    sm.fit(meta)[d] = (uint64_t)lo;
    sm.fitb(meta)[d] = fb;
    if (d != me) {
      const int k = d < me ? d : d - 1;
      sm.hdr(meta)[2 * k] = (uint64_t)lo;
      sm.hdr(meta)[2 * k + 1] = fb;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t sb = 0, rows = 0;
    for (int d = 0; d < W; ++d) {
      rows += (uint64_t)cnt_s[d];
      if (d == me) continue;
      sm.segbase(meta)[d] = sb;
      sb += 4 + (uint64_t)cnt_s[d];
    }
    sm.tail(meta)[0] = sb;                           // segments of the send buffer
    sm.tail(meta)[1] = tcnt[(int64_t)me * G];        // first row of the self block
    sm.tail(meta)[2] = rows;                         // routed rows (all destinations)
  }
}

// The carry of one row that did not fit (its block's slot, or the self capacity): key,
// metadata, destination + tier and a copy of its value bytes (the caller's batch may be
// gone next step) into the carry buffers of this step's parity. ctr = {rows, bytes} of
// this parity; tot = {rows, bytes, lost} since construction.
struct CarryOut {
  Digest* keys;
  uint32_t* vlen;
  uint32_t* flags;
  uint32_t* expire;
  uint64_t* val;
  int32_t* dest;
  uint8_t* bytes;
  int64_t cap;
  uint64_t bcap;
  unsigned long long* ctr;
  unsigned long long* tot;
};
__device__ void carry_row(const CarryOut& co, const int64_t* __restrict__ rec, uint64_t src,
                          int d, int me) {
  const uint32_t vl = (uint32_t)rec[2];
  const uint64_t r3 = (uint64_t)rec[3];
  const uint32_t vp = rec_vpad(rec);
  const unsigned long long slot = atomicAdd(co.ctr, 1ull);
  if (slot >= (unsigned long long)co.cap) {
    atomicAdd(co.tot + 2, 1ull);
    return;
  }
  const unsigned long long at = vp ? atomicAdd(co.ctr + 1, (unsigned long long)vp) : 0ull;
  co.keys[slot] = Digest{(uint64_t)rec[0], (uint64_t)rec[1]};
  co.flags[slot] = (uint32_t)((uint64_t)rec[2] >> 32);
  co.expire[slot] = (uint32_t)r3;
  if (at + vp > co.bcap) {  // no room for the value: a skip row (counted as lost)
    co.vlen[slot] = kSkipVlen;
    co.dest[slot] = me;
    co.val[slot] = 0;
    atomicAdd(co.tot + 2, 1ull);
    return;
  }
  co.vlen[slot] = vl;
  co.dest[slot] = d | (int)((r3 >> 63) << kTierBit);
  co.val[slot] = (uint64_t)(uintptr_t)(co.bytes + at);
  const u32x4v* s4 = reinterpret_cast<const u32x4v*>((uintptr_t)src);
  u32x4v* d4 = reinterpret_cast<u32x4v*>(co.bytes + at);
  for (uint32_t c = 0; c < vp / 16; ++c) d4[c] = s4[c];
  atomicAdd(co.tot, 1ull);
  atomicAdd(co.tot + 1, (unsigned long long)vp);
}

// The send buffer's segment list (slots in o-order = rank order without this rank; slot =
// [header 16 B | capS records | capSB value bytes]), and the carry of every routed row that
// does not fit. Threads: one per routed row, then one per destination (its fixed
// segments), then one for the end offset.
constexpr int kSegLds = 1024;
__global__ __launch_bounds__(kB) void k_set_pack_segs(
    const uint64_t* __restrict__ meta_c, const uint64_t* __restrict__ tcnt,
    const uint64_t* __restrict__ tbytes, int64_t G, const int64_t* __restrict__ cnt_s,
    const int64_t* __restrict__ srec, const uint64_t* __restrict__ sval,
    const uint64_t* __restrict__ svoff, int32_t W, int32_t me, int64_t capS, int64_t slotS,
    int64_t tmax, uint64_t* __restrict__ seg_off, uint64_t* __restrict__ seg_src,
    CarryOut co) {
  __shared__ uint64_t s_sst[kSegLds + 1];
  uint64_t* meta = const_cast<uint64_t*>(meta_c);
  const SetMeta sm{W};
  const bool lds = W <= kSegLds;
  if (lds) {
    for (int d = threadIdx.x; d < W; d += kB) s_sst[d] = tcnt[(int64_t)d * G];
    if (threadIdx.x == 0) s_sst[W] = sm.tail(meta)[2];
    __syncthreads();
  }
  const int64_t total = (int64_t)sm.tail(meta)[2];
  const uint64_t val0 = 16 + 32 * (uint64_t)capS;
  for (int64_t t = (int64_t)blockIdx.x * kB + threadIdx.x; t < tmax; t += (int64_t)gridDim.x * kB) {
    if (t < total) {
      int lo = 0, hi = W;  // the block holding row t: last d with sst[d] <= t
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        const uint64_t v = lds ? s_sst[mid] : tcnt[(int64_t)mid * G];
        if (v <= (uint64_t)t) lo = mid; else hi = mid;
      }
      const int d = lo;
      const uint64_t sst = lds ? s_sst[d] : tcnt[(int64_t)d * G];
      const int64_t j = t - (int64_t)sst;
      const bool keep = (uint64_t)j < sm.fit(meta)[d];
      if (d != me) {
        const int k = d < me ? d : d - 1;
        const uint64_t vo = svoff[t] - tbytes[(int64_t)d * G];
        const int64_t q = (int64_t)sm.segbase(meta)[d] + 3 + j;
        seg_off[q] = (uint64_t)k * slotS + val0 + min(vo, sm.fitb(meta)[d]);
        seg_src[q] = keep ? sval[t] : 0ull;
      }
      if (!keep) carry_row(co, srec + 4 * t, sval[t], d, me);
    } else if (t < total + W) {
      const int d = (int)(t - total);
      if (d == me) continue;
      const int k = d < me ? d : d - 1;
      const uint64_t base = (uint64_t)k * slotS, f = sm.fit(meta)[d];
      const int64_t q = (int64_t)sm.segbase(meta)[d];
      seg_off[q] = base;
      seg_src[q] = (uint64_t)(uintptr_t)(sm.hdr(meta) + 2 * k);
      seg_off[q + 1] = base + 16;
      seg_src[q + 1] = (uint64_t)(uintptr_t)(srec + 4 * (int64_t)tcnt[(int64_t)d * G]);
      seg_off[q + 2] = base + 16 + 32 * f;
      seg_src[q + 2] = kSegSkip;
      seg_off[q + 3 + cnt_s[d]] = base + val0 + sm.fitb(meta)[d];
      seg_src[q + 3 + cnt_s[d]] = kSegSkip;
    } else if (t == total + W) {
      seg_off[sm.tail(meta)[0]] = (uint64_t)(W - 1) * slotS;
    }
  }
}

// Received SET rows in fixed positions: [source slots (o-order) x capS | capSelf own rows].
// Row j of slot k is a SET when j < the slot header's row count; an own row when it is
// within the self block's fit. Every other row is a skip row (kSkipVlen in both tiers).
__global__ __launch_bounds__(kB) void k_rs_fill_fixed(
    const uint8_t* __restrict__ Rs, int64_t slotS, int64_t capS, int32_t W,
    const uint64_t* __restrict__ meta_c, int32_t me, const int64_t* __restrict__ srec,
    const uint64_t* __restrict__ sval, int64_t nrows, Digest* __restrict__ keys,
    uint32_t* __restrict__ vlen0, uint32_t* __restrict__ vlen1, uint32_t* __restrict__ flags,
    uint32_t* __restrict__ expire, uint64_t* __restrict__ roff) {
  uint64_t* meta = const_cast<uint64_t*>(meta_c);
  const SetMeta sm{W};
  const int64_t others = (int64_t)(W - 1) * capS;
  for (int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * kB) {
    const int64_t* rr = nullptr;
    uint64_t vbase = 0, vabs = 0;
    if (r < others) {
      const int64_t k = r / capS, j = r - k * capS;
      const uint8_t* slot = Rs + k * slotS;
      if ((uint64_t)j < reinterpret_cast<const uint64_t*>(slot)[0]) {
        rr = reinterpret_cast<const int64_t*>(slot + 16 + 32 * j);
        vbase = (uint64_t)(uintptr_t)(slot + 16 + 32 * capS);
      }
    } else {
      const int64_t j = r - others;
      if ((uint64_t)j < sm.fit(meta)[me]) {
        const int64_t t = (int64_t)sm.tail(meta)[1] + j;
        rr = srec + 4 * t;
        vabs = sval[t];
      }
    }
    if (!rr) {
      keys[r] = Digest{0, 0};
      vlen0[r] = vlen1[r] = kSkipVlen;
      flags[r] = expire[r] = 0;
      roff[r] = 0;
      continue;
    }
    keys[r] = Digest{(uint64_t)rr[0], (uint64_t)rr[1]};
    const uint32_t vl = (uint32_t)rr[2];
    const uint64_t hi32 = (uint64_t)rr[3] >> 32;
    const uint32_t tier = (uint32_t)(hi32 >> 31);
    vlen0[r] = tier == 0 ? vl : kSkipVlen;
    vlen1[r] = tier == 1 ? vl : kSkipVlen;
    flags[r] = (uint32_t)((uint64_t)rr[2] >> 32);
    expire[r] = (uint32_t)rr[3];
    roff[r] = rr == nullptr ? 0 : (vabs ? vabs : vbase + (hi32 & 0x7FFFFFFFull));
  }
}

}  // namespace

const StepStreams& step_streams(int device) {
  static std::mutex mu;
  static std::vector<StepStreams> pool(64);
  SH_CHECK(device >= 0 && device < 64, "bad device");
  std::lock_guard<std::mutex> lk(mu);
  StepStreams& p = pool[device];
  if (!p.plan) {
    RT_OK(hipSetDevice(device));
    // Which streams share a hardware queue (4 per process, handed out round robin as
    // streams are first used) decides whether the plan runs beside the reply gather. Make
    // sure the null stream (torch's default) holds its queue, then take the other three
    // for the step: call this before anything else creates streams (bench.py does, via
    // ops.cache.reserve_step_streams) and the step's four streams never share.
    void* scratch = nullptr;
    RT_OK(hipMalloc(&scratch, 64));
    RT_OK(hipMemsetAsync(scratch, 0, 64, nullptr));
    RT_OK(hipStreamSynchronize(nullptr));
    RT_OK(hipFree(scratch));
    // SHELLAC_STREAM_PRIO="plan,set,asm" (A/B): per-stream priorities, clamped to the
    // device's range (on this image least 1, greatest -1); default: all normal
    int prio[3] = {0, 0, 0};
    if (const char* e = getenv("SHELLAC_STREAM_PRIO")) {
      int lo = 0, hi = 0;
      RT_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      (void)sscanf(e, "%d,%d,%d", &prio[0], &prio[1], &prio[2]);
      for (int& x : prio) x = std::max(hi, std::min(lo, x));
      fprintf(stderr, "[shellac] step stream priorities plan %d set %d asm %d (least %d greatest %d)\n",
              prio[0], prio[1], prio[2], lo, hi);
    }
    RT_OK(hipStreamCreateWithPriority(&p.plan, hipStreamNonBlocking, prio[0]));
    RT_OK(hipStreamCreateWithPriority(&p.set, hipStreamNonBlocking, prio[1]));
    RT_OK(hipStreamCreateWithPriority(&p.asm_, hipStreamNonBlocking, prio[2]));
    // measured: with the plan stream sharing the assembly's queue the simulated 8-rank step
    // took 0.93 ms (the plan waited behind the mirrored reply copy), sharing the main
    // stream's 0.50 ms at one rank (behind the reply gather)
  }
  return p;
}

RoutedStep::RoutedStep(int world, int rank, int device)
    : w_(world), rank_(rank), device_(device), bufs_(kNumSlots) {
  SH_CHECK(world >= 1 && world < kMaxBuckets, "bad world size");
  RT_OK(hipSetDevice(device_));
  (void)step_streams(device_);  // the process's first streams take the hardware queues
  const size_t K = (size_t)row_words();
  RT_OK(hipHostMalloc(&host_mat_, K * (size_t)world * sizeof(int64_t), hipHostMallocDefault));
  RT_OK(hipHostMalloc(&host_ring_, kPend * K * (size_t)world * sizeof(int64_t),
                      hipHostMallocDefault));
  RT_OK(hipHostMalloc(&host_dmat_, (size_t)world * (size_t)world * sizeof(int64_t),
                      hipHostMallocDefault));
  // two parities: a step's H2D copies of its tables may still be queued on the SET
  // stream when the next step's host code fills the other half
  RT_OK(hipHostMalloc(&host_tab_, 2 * (8 * (size_t)world + 8) * sizeof(uint64_t),
                      hipHostMallocDefault));
  for (hipEvent_t* e : {&ev_fork_, &ev_pjoin_, &ev_pub_, &ev_sfork_, &ev_join_, &ev_asm_[0],
                        &ev_asm_[1], &ev_probe_, &ev_local_, &ev_rfork_, &ev_reply_[0],
                        &ev_reply_[1], &ev_pfork_, &ev_plan_, &ev_rep_, &ev_start_,
                        &ev_gdone_[0], &ev_gdone_[1], &ev_carry_[0], &ev_carry_[1], &ev_c1_,
                        &ev_c2_, &ev_pack_, &ev_hot_, &ev_sdone_[0], &ev_sdone_[1]})
    RT_OK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  for (hipEvent_t& e : ev_ring_) RT_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // carry counters ([parity][rows, bytes], totals [rows, bytes, lost]) and the SET slot
  // metadata: zeroed once here (construction, not the serving path)
  RT_OK(hipMalloc(&cctr_, 8 * sizeof(unsigned long long)));
  RT_OK(hipMemset(cctr_, 0, 8 * sizeof(unsigned long long)));
  for (uint64_t*& m : set_meta_) {
    RT_OK(hipMalloc(&m, set_meta_words(world) * sizeof(uint64_t)));
    RT_OK(hipMemset(m, 0, set_meta_words(world) * sizeof(uint64_t)));
  }
  RT_OK(hipDeviceSynchronize());
}

RoutedStep::~RoutedStep() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  reap(true);
  for (auto& b : bufs_) (void)hipFree(b.p);
  if (hot_tab_) (void)hipFree(hot_tab_);
  for (int p = 0; p < 2; ++p)
    for (void* q : {(void*)ck_[p], (void*)cvl_[p], (void*)cfl_[p], (void*)cex_[p],
                    (void*)cval_[p], (void*)cdst_[p], (void*)cbytes_[p]})
      if (q) (void)hipFree(q);
  (void)hipFree(cctr_);
  for (uint64_t* m : set_meta_) (void)hipFree(m);
  (void)hipHostFree(host_mat_);
  (void)hipHostFree(host_ring_);
  (void)hipHostFree(host_dmat_);
  (void)hipHostFree(host_tab_);
  for (hipEvent_t e : {ev_fork_, ev_pjoin_, ev_pub_, ev_sfork_, ev_join_, ev_asm_[0], ev_asm_[1],
                       ev_probe_, ev_local_, ev_rfork_, ev_reply_[0], ev_reply_[1], ev_pfork_,
                       ev_plan_, ev_rep_, ev_start_, ev_gdone_[0], ev_gdone_[1], ev_carry_[0],
                       ev_carry_[1], ev_c1_, ev_c2_, ev_pack_, ev_hot_, ev_sdone_[0], ev_sdone_[1]})
    (void)hipEventDestroy(e);
  for (hipEvent_t e : ev_ring_) (void)hipEventDestroy(e);
}

void RoutedStep::set_ring(const uint32_t* pts, const int32_t* owner, int32_t npts) {
  pts_ = pts;
  own_ = owner;
  npts_ = npts;
}

// ---- deferred frees -------------------------------------------------------------------
void RoutedStep::note_stream(hipStream_t s) {
  if (std::find(seen_streams_.begin(), seen_streams_.end(), s) == seen_streams_.end())
    seen_streams_.push_back(s);
}

void RoutedStep::retire(void* p) {
  if (!p) return;
  const StepStreams& ss = step_streams(device_);
  Dead d{p, {}};
  std::vector<hipStream_t> all = seen_streams_;
  for (hipStream_t x : {ss.plan, ss.set, ss.asm_})
    if (std::find(all.begin(), all.end(), x) == all.end()) all.push_back(x);
  for (hipStream_t x : all) {
    hipEvent_t e;
    RT_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    RT_OK(hipEventRecord(e, x));
    d.ev.push_back(e);
  }
  dead_.push_back(std::move(d));
}

void RoutedStep::reap(bool all) {
  for (size_t i = 0; i < dead_.size();) {
    bool done = true;
    for (hipEvent_t e : dead_[i].ev)
      if (all) (void)hipEventSynchronize(e);
      else if (hipEventQuery(e) != hipSuccess) done = false;
    if (!done) {
      ++i;
      continue;
    }
    for (hipEvent_t e : dead_[i].ev) (void)hipEventDestroy(e);
    (void)hipFree(dead_[i].p);
    dead_.erase(dead_.begin() + (long)i);
  }
}

void RoutedStep::set_hot(const Digest* hot, int64_t nhot, const int64_t* dir, bool changed) {
  hot_ = hot;
  nhot_ = hot ? nhot : 0;
  hot_dir_ = hot ? dir : nullptr;
  if (!hot || nhot <= 0) return;
  // called every step: build once per hot set (`changed`: new contents, maybe at the
  // same address)
  if (!changed && hot == hot_built_ && nhot == nhot_built_) return;
  // a new hot set (replica refresh): a new hash set, built on the plan stream (the next
  // plan waits for it); the old one is freed once the steps queued before have passed
  // (no device synchronisation: in-flight collectives on other ranks are never waited for)
  RT_OK(hipSetDevice(device_));
  uint64_t slots = 1024;
  while (slots < 2 * (uint64_t)nhot) slots *= 2;
  retire(hot_tab_);
  RT_OK(hipMalloc(&hot_tab_, slots * sizeof(Digest)));
  hipStream_t bs = step_streams(device_).plan;
  RT_OK(hipMemsetAsync(hot_tab_, 0, slots * sizeof(Digest), bs));
  hot_mask_ = slots - 1;
  const int g = (int)std::min<int64_t>((nhot + 255) / 256, 4096);
  hipLaunchKernelGGL(k_hot_hash_build, dim3(g), dim3(256), 0, bs, hot, nhot, hot_tab_, hot_mask_);
  RT_OK(hipGetLastError());
  RT_OK(hipEventRecord(ev_hot_, bs));
  hot_pending_ = true;
  hot_built_ = hot;
  nhot_built_ = nhot;
}

template <typename T>
T* RoutedStep::buf(int slot, size_t count) {
  Buf& b = bufs_[slot];
  const size_t need = std::max<size_t>(count, 1) * sizeof(T);
  if (b.cap < need) {
    // grow-only; the old block may still be read by queued work: freed once it has passed
    retire(b.p);
    const size_t cap = (need + need / 4 + 255) & ~(size_t)255;
    RT_OK(hipMalloc(&b.p, cap));
    b.cap = cap;
  }
  return static_cast<T*>(b.p);
}

// ---- capacities ---------------------------------------------------------------------
// Slack over the largest demand of the last kHist steps: 10 % (+256 rows) for the GET
// slots, 5 % (+256 KiB) for the reply data — per-peer demand of a step varies by ~1 %
// (Zipf batches of 1M rows), so an overflow needs a shift in the workload, which the
// next steps absorb; the local region is per rank and costs no link bytes (10 % + 1 MiB).
// The SET slots take the same slack (rows, value bytes); a SET that does not fit is
// carried into the next step, never lost.
namespace {
constexpr size_t kHist = 16;
void push_hist(std::vector<int64_t>* h, int64_t v) {
  h->push_back(v);
  if (h->size() > kHist) h->erase(h->begin());
}
int64_t hist_max(const std::vector<int64_t>& h) {
  int64_t m = 0;
  for (int64_t v : h) m = std::max(m, v);
  return m;
}
}  // namespace

std::vector<int64_t> RoutedStep::caps(int64_t n) const {
  // the local region is this rank's own: sized per GET row from its history (no
  // agreement needed), calibrated by a host read when there is none yet
  const bool cal_l = hist_lr_.empty() && n > 0;
  double lr = 0;
  for (double v : hist_lr_) lr = std::max(lr, v);
  const int64_t l = cal_l ? capL_ : align_up64((int64_t)(lr * 1.15 * (double)n) + (1 << 20), 4096);
  if (ovr_[0] > 0 && !calibrating_)
    return {align_up64(ovr_[0], 2), align_up64(ovr_[1], 16), align_up64(ovr_[2], 16), 0, 0};
  if (calibrating_) return {std::max<int64_t>(align_up64(n, 64), 64), capD_, l, 1, cal_l};
  const int64_t g = align_up64(hist_max(hist_g_) * 11 / 10 + 256, 64);
  const int64_t d = align_up64(hist_max(hist_d_) * 21 / 20 + (256 << 10), 4096);
  return {g, d, l, 0, cal_l};
}

std::vector<int64_t> RoutedStep::set_caps() const {
  if (ovr_s_[0] > 0)
    return {align_up64(ovr_s_[0], 2), align_up64(ovr_s_[1], 16), align_up64(ovr_s_[2], 2),
            align_up64(ovr_s_[3], 16)};
  return {align_up64(hist_max(hist_s_) * 11 / 10 + 256, 64),
          align_up64(hist_max(hist_sb_) * 21 / 20 + (256 << 10), 4096),
          align_up64(hist_max(hist_self_) * 11 / 10 + 256, 64),
          align_up64(hist_max(hist_selfb_) * 21 / 20 + (256 << 10), 4096)};
}

void RoutedStep::reset_caps() {
  // pending matrices still count in the statistics, not in the new history
  for (Pend& p : pend_) {
    RT_OK(hipEventSynchronize(ev_ring_[p.slot]));
    if (!p.stats_done)
      add_stats(note_matrix(host_ring_ + (size_t)p.slot * row_words() * w_, p.n, p.capG, false));
  }
  pend_.clear();
  for (auto* h : {&hist_g_, &hist_d_, &hist_s_, &hist_sb_, &hist_self_, &hist_selfb_}) h->clear();
  hist_lr_.clear();
  calibrating_ = true;
  capD_ = capL_ = 0;
}

// History (hist) and this rank's statistics of one all-gathered matrix:
// [n_local, n_dup, GET rows sent off-rank, rows over capG, reply rows dropped].
std::vector<int64_t> RoutedStep::note_matrix(const int64_t* m, int64_t n, int64_t capG, bool hist) {
  const int W = w_, me = rank_;
  const int64_t K = row_words();
  if (hist) {
    int64_t mg = 0, md = 0, ms = 0, mb = 0, mself = 0, mselfb = 0;
    for (int r = 0; r < W; ++r)
      for (int p = 0; p < W; ++p) {
        mg = std::max(mg, m[r * K + p]);
        md = std::max(md, m[r * K + 3 * W + p]);
        if (p == r) {
          mself = std::max(mself, m[r * K + W + p]);
          mselfb = std::max(mselfb, m[r * K + 2 * W + p]);
        } else {
          ms = std::max(ms, m[r * K + W + p]);
          mb = std::max(mb, m[r * K + 2 * W + p]);
        }
      }
    push_hist(&hist_g_, mg);
    // the reply column is the previous step's demand (none before the first step)
    if (!calibrating_) push_hist(&hist_d_, md);
    push_hist(&hist_s_, ms);
    push_hist(&hist_sb_, mb);
    push_hist(&hist_self_, mself);
    push_hist(&hist_selfb_, mselfb);
    if (n > 0) {
      hist_lr_.push_back((double)m[me * K + 4 * W + 1] / (double)n);
      if (hist_lr_.size() > kHist) hist_lr_.erase(hist_lr_.begin());
    }
    calibrating_ = false;
  }
  int64_t over = 0, off_rank = 0;
  for (int p = 0; p < W; ++p) {
    over += std::max<int64_t>(0, m[me * K + p] - capG);
    if (p != me) off_rank += m[me * K + p];
  }
  return {m[me * K + 4 * W], m[me * K + 4 * W + 2], off_rank, over, m[me * K + 4 * W + 3]};
}

void RoutedStep::add_stats(const std::vector<int64_t>& st) {
  for (size_t i = 0; i < stat_acc_.size() && i < st.size(); ++i) stat_acc_[i] += st[i];
}

// Matrices published by step(), oldest first: statistics once, history (hist) for the
// steps up to `upto`, in step order; an entry leaves once its history is in. The host
// waits for a matrix only when its step is that old (two steps: long complete).
void RoutedStep::harvest(int64_t upto, bool hist) {
  for (Pend& p : pend_) {
    if (p.step > upto) break;
    if (p.stats_done && (!hist || p.hist_done)) continue;
    RT_OK(hipEventSynchronize(ev_ring_[p.slot]));
    const int64_t* m = host_ring_ + (size_t)p.slot * row_words() * w_;
    const std::vector<int64_t> st = note_matrix(m, p.n, p.capG, hist && !p.hist_done);
    if (!p.stats_done) add_stats(st);
    p.stats_done = true;
    if (hist) p.hist_done = true;
  }
  while (!pend_.empty() && pend_.front().hist_done) pend_.pop_front();
}

void RoutedStep::harvest_all() { harvest(INT64_MAX, false); }

std::vector<int64_t> RoutedStep::take_stats() {
  std::vector<int64_t> out = stat_acc_;
  std::fill(stat_acc_.begin(), stat_acc_.end(), 0);
  return out;
}

std::vector<int64_t> RoutedStep::carry_stats() {
  unsigned long long h[3] = {0, 0, 0};
  RT_OK(hipSetDevice(device_));
  RT_OK(hipDeviceSynchronize());
  RT_OK(hipMemcpy(h, cctr_ + 4, sizeof(h), hipMemcpyDeviceToHost));
  return {(int64_t)h[0], (int64_t)h[1], (int64_t)h[2]};
}

void RoutedStep::ensure_carry(int64_t rows, uint64_t bytes) {
  // parity P only (this step's pack writes it); the other parity holds what the previous
  // step carried and this step's plan reads it
  const int P = par_;
  rows = std::max<int64_t>(rows, 1024);
  bytes = std::max<uint64_t>(align_up64((int64_t)bytes, 16), 1 << 20);
  if (ck_[P] && ccap_p_[P] >= rows && cbcap_p_[P] >= bytes) return;
  for (void* q : {(void*)ck_[P], (void*)cvl_[P], (void*)cfl_[P], (void*)cex_[P], (void*)cval_[P],
                  (void*)cdst_[P], (void*)cbytes_[P]})
    retire(q);
  const int64_t r = rows + rows / 4;
  const uint64_t b = (bytes + bytes / 4 + 255) & ~(uint64_t)255;
  RT_OK(hipMalloc(&ck_[P], r * sizeof(Digest)));
  RT_OK(hipMalloc(&cvl_[P], r * sizeof(uint32_t)));
  RT_OK(hipMalloc(&cfl_[P], r * sizeof(uint32_t)));
  RT_OK(hipMalloc(&cex_[P], r * sizeof(uint32_t)));
  RT_OK(hipMalloc(&cval_[P], r * sizeof(uint64_t)));
  RT_OK(hipMalloc(&cdst_[P], r * sizeof(int32_t)));
  RT_OK(hipMalloc(&cbytes_[P], b));
  ccap_p_[P] = r;
  cbcap_p_[P] = b;
}

// ---- plan ---------------------------------------------------------------------------
void RoutedStep::plan(const Digest* keys, int64_t n, HbmCache* replica, uint32_t now,
                      const Digest* skeys, const uint32_t* svlen, const uint32_t* sflags,
                      const uint32_t* sexpire, const uint64_t* sval_off, const uint8_t* svalues,
                      int64_t ns, bool fanout, uint8_t* G, int64_t* row, hipStream_t s,
                      bool coalesce) {
  SH_CHECK(pts_ && own_ && npts_ > 0, "RoutedStep: ring not set");
  SH_CHECK(n < (1ll << 31), "RoutedStep: GET batch too large");
  if (!in_step_) {  // a multi-call step: the next step() plans on `s`, no look-ahead
    pfork_valid_ = false;
    gdone_valid_[0] = gdone_valid_[1] = false;
  }
  const int W = w_;
  const int nb = W + 1;
  const std::vector<int64_t> c = caps(n);
  capG_ = c[0];
  if (!calibrating_) capD_ = c[1];
  if (!c[4]) capL_ = c[2];
  par_ ^= 1;
  const int P = par_;
  n_ = n;
  ns_ = ns;
  values_ = svalues;
  have_replica_ = replica != nullptr;
  replica_ = replica;
  published_ = false;
  // the deferred assemble of the step two back reads this parity's buffers
  if (asm_pending_[P]) {
    RT_OK(hipStreamWaitEvent(s, ev_asm_[P], 0));
    asm_pending_[P] = false;
  }
  // every buffer first
  first_ = nullptr;
  uint32_t* co_tab = nullptr;
  int64_t co_slots = 0;
  if (coalesce && n > 0) {
    co_slots = coalesce_table_slots(n);
    co_tab = buf<uint32_t>(kCoTab, co_slots);
    first_ = buf<uint32_t>(P ? kFirst1 : kFirst0, n);
  }
  rl_size_ = rl_off_ = nullptr;
  if (replica) {
    rl_loc_ = buf<uint64_t>(kRlLoc, n);
    rl_size_ = buf<uint64_t>(P ? kRlSize1 : kRlSize0, n + 1);
    rl_off_ = buf<uint64_t>(P ? kRlOff1 : kRlOff0, n + 1);
  }
  int32_t* dest_g = buf<int32_t>(kDestG, n);
  route_ = buf<int64_t>(P ? kRoute1 : kRoute0, n);
  int64_t* cnt_g = buf<int64_t>(kCntG, nb);
  const int64_t ng = std::max<int64_t>(n, 1);
  const int Gg = group_grid(ng);
  const int64_t plen_g = (ng + Gg - 1) / Gg;
  uint64_t* ws_g = buf<uint64_t>(kWsG, group_ws_words(ng, nb));
  // the SET rows the previous step carried over (step() writes them; none otherwise):
  // Gc workgroups of them ahead of the batch's Gs
  const int Pc = P ^ 1;
  const bool have_carry = carry_written_[Pc] && ck_[Pc] != nullptr;
  const int64_t ccap = have_carry ? ccap_p_[Pc] : 0;
  const int64_t nsx = std::max<int64_t>(ns, 1);
  const int Gs = group_grid(nsx, 256);
  const int64_t plen_s = (nsx + Gs - 1) / Gs;
  // (a carry is rare and small: a few workgroups share it, whatever its capacity)
  const int Gc = have_carry ? 16 : 0;
  const int Gt = Gs + Gc;
  // upper bound of routed SET rows (a carried row goes to its one destination)
  const int64_t mcap = (fanout ? ns * W : ns) + ccap;
  gt_ = Gt;
  nrouted_max_ = mcap;
  int32_t* owner_s = buf<int32_t>(kOwnerS, (size_t)(ccap + ns));
  uint32_t* vpad = buf<uint32_t>(kVpad, (size_t)(ccap + ns));
  // by parity: the previous step's fixed-slot pack (SET stream) may still read them
  uint64_t* tcnt = buf<uint64_t>(P ? kTcnt1 : kTcnt, (size_t)nb * Gt);
  uint64_t* tbytes = buf<uint64_t>(P ? kTbytes1 : kTbytes, (size_t)nb * Gt);
  // by parity: the previous step's SET packing (on the SET stream) may still read them
  srec_ = buf<int64_t>(P ? kSrec1 : kSrec, 4 * (size_t)mcap);
  sval_ = buf<uint64_t>(P ? kSval1 : kSval, mcap);
  svoff_ = buf<uint64_t>(P ? kSvoff1 : kSvoff, mcap);
  cnt_s_ = buf<int64_t>(P ? kCntS1 : kCntS, nb);
  rb_ = buf<int64_t>(kRb, W + 1);
  if (hist_g_.empty() && calibrating_) RT_OK(hipMemsetAsync(rb_, 0, (W + 1) * sizeof(int64_t), s));

  // the previous step's reply demand and dropped rows ride in this row
  RT_OK(hipMemsetAsync(row + 4 * W, 0, kExtras * sizeof(int64_t), s));
  RT_OK(hipMemcpyAsync(row + 3 * W, rb_, W * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  RT_OK(hipMemcpyAsync(row + 4 * W + 3, rb_ + W, sizeof(int64_t), hipMemcpyDeviceToDevice, s));

  // SET planning on the side stream (owner + hot fan-out, counting sort with value-byte
  // ranges), concurrently with the replica probe and GET sort on `s`
  // (inside step() the planner already runs beside the previous step's reply gather, and
  // a fourth concurrent stream would share a hardware queue with another: 4 per process)
  if (!in_step_ && !side_) {
    const StepStreams& ps = step_streams(device_);
    side_ = ps.set;  // the multi-call path's SET planning (the SET side is idle then)
  }
  hipStream_t ss = in_step_ ? s : side_;
  if (ss != s) {
    RT_OK(hipEventRecord(ev_fork_, s));
    RT_OK(hipStreamWaitEvent(ss, ev_fork_, 0));
  }
  if (hot_pending_) {  // a new hot hash set is being built on the plan stream
    RT_OK(hipStreamWaitEvent(ss, ev_hot_, 0));
    hot_pending_ = false;
  }
  // this step's carry counters (its pack adds to them); the step two back's plan has read them
  RT_OK(hipMemsetAsync(cctr_ + 2 * P, 0, 2 * sizeof(unsigned long long), ss));
  const SetRows sr{skeys, svlen, sflags, sexpire, sval_off, (uint64_t)(uintptr_t)svalues, ns,
                   spkeys_, ck_[Pc], cvl_[Pc], cfl_[Pc], cex_[Pc], cval_[Pc], cdst_[Pc], cctr_ + 2 * Pc,
                   ccap, Gc};
  hipLaunchKernelGGL(k_ps_dest_hist, dim3(Gt), dim3(kB), nb * sizeof(unsigned long long), ss, sr,
                     pts_, own_, npts_, fanout && nhot_ > 0 ? hot_tab_ : nullptr, hot_mask_, nb,
                     plen_s, W, owner_s, vpad, tcnt, tbytes);
  hipLaunchKernelGGL(k_ps_scan, dim3(1), dim3(1024), 0, ss, tcnt, tbytes, nb, Gt, cnt_s_,
                     row + W, row + 2 * W);
  if (ns > 0 || Gc > 0)
    hipLaunchKernelGGL(k_ps_scatter, dim3(Gt), dim3(kB), nb * sizeof(unsigned long long), ss, sr,
                       nb, plen_s, tcnt, tbytes, owner_s, vpad, W, srec_, sval_, svoff_);
  RT_OK(hipGetLastError());
  carry_written_[Pc] = false;  // consumed (its value bytes stay put until this step's SETs)
  if (ss != s) RT_OK(hipEventRecord(ev_pjoin_, ss));

  // GET rows: coalesce duplicates (answered from their claimer), replica probe, owner
  // (or bucket W = answered here), counting sort straight into the request slots
  if (first_ && replica)
    replica->lookup_coalesced(keys, n, co_tab, co_slots, first_, rl_loc_, rl_size_, rl_off_, now,
                              s);
  else if (first_)
    coalesce_keys(keys, n, co_tab, co_slots, first_, s);
  else if (replica)
    replica->lookup(keys, n, rl_loc_, rl_size_, rl_off_, now, s);
  int64_t* extras = row + 4 * W;
  hipLaunchKernelGGL(k_route_hist, dim3(Gg), dim3(kB), nb * sizeof(uint32_t), s, keys, n, rl_size_,
                     pts_, own_, npts_, W, plen_g, dest_g, ws_g, first_,
                     reinterpret_cast<unsigned long long*>(extras + 2));
  hipLaunchKernelGGL(k_gr_scan, dim3(1), dim3(1024), 0, s, ws_g, (int64_t)nb * Gg, nb, Gg, cnt_g,
                     row, replica ? rl_off_ + n : nullptr, extras, 1);
  if (n > 0)
    hipLaunchKernelGGL(k_gr_scatter_slots, dim3(Gg), dim3(kB), nb * sizeof(uint32_t), s, dest_g, n,
                       nb, plen_g, ws_g, pkeys_ ? pkeys_ : keys, capG_, rank_, G, route_);
  RT_OK(hipGetLastError());
  if (ss != s) RT_OK(hipStreamWaitEvent(s, ev_pjoin_, 0));  // join: the row is complete
}

void RoutedStep::publish(const int64_t* mat, hipStream_t s) {
  const int W = w_;
  const int64_t K = row_words();
  mat_dev_ = mat;  // owner_probe derives the owner slot counts from it
  RT_OK(hipMemcpyAsync(host_mat_, mat, (size_t)W * K * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  RT_OK(hipEventRecord(ev_pub_, s));
  published_ = true;
}

void RoutedStep::calibrate_local() {
  SH_CHECK(published_, "RoutedStep: publish before calibrate_local");
  RT_OK(hipEventSynchronize(ev_pub_));
  const int64_t lb = host_mat_[rank_ * row_words() + 4 * w_ + 1];
  capL_ = align_up64(lb * 23 / 20 + (1 << 20), 4096);
}

// ---- owner --------------------------------------------------------------------------
void RoutedStep::owner_probe(const uint8_t* G, HbmCache* shard, uint32_t now, hipStream_t s) {
  const int W = w_;
  // the last step's SET chain writes the main shard: the probe comes after it
  join_sets(s);
  const int64_t rows = (int64_t)W * capG_;
  lk_loc_ = buf<uint64_t>(kLkLoc, rows);
  lk_size_ = buf<uint64_t>(kLkSize, rows + 1);
  lk_off_ = buf<uint64_t>(kLkOff, rows + 1);
  // this step's SETs are appended beside the reply gather (store_sets): reserve their
  // bytes, computed on the device from the all-gathered matrix (no host read)
  uint64_t* reserve = buf<uint64_t>(kReserve, 1);
  own_cnt_ = buf<int64_t>(kOwnCnt, W);
  // look-ahead (native step only): 5/4 of the largest recent SET payload plus the CLOCK
  // reinsertion budget, the most the next step's main-shard SET chain can append
  // (only while the log is far from wrapping: a SET that runs early never runs the CLOCK
  // hand, so no reinsertion budget needs reserving; near the wrap every SET waits for its
  // own probe and no look-ahead is reserved, which would cost hit ratio)
  const uint64_t rmax = (uint64_t)shard->reinsert_max();
  ahead_prev_ = ahead_;
  const uint64_t est = pay_hist_.empty() ? 0 : (uint64_t)hist_max(pay_hist_) * 5 / 4;
  ahead_ = in_step_ && est && !shard->would_reclaim(est) ? est : 0;
  hipLaunchKernelGGL(k_owner_prep, dim3(1), dim3(64), 0, s, mat_dev_, row_words(), W, rank_, capG_,
                     rmax, ahead_, own_cnt_, reserve);
  RT_OK(hipGetLastError());
  shard->lookup_slots(reinterpret_cast<const Digest*>(G), W, capG_, own_cnt_, lk_loc_, lk_size_,
                      lk_off_, now, s, reserve);
}

void RoutedStep::owner_demand(int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_demand, dim3(1), dim3(64), 0, s, lk_off_, w_, rank_, capG_, out);
  RT_OK(hipGetLastError());
}

void RoutedStep::calibrate_reply(const int64_t* dmat) {
  const int W = w_;
  RT_OK(hipMemcpy(host_dmat_, dmat, (size_t)W * W * sizeof(int64_t), hipMemcpyDeviceToHost));
  int64_t m = 0;
  for (int i = 0; i < W * W; ++i) m = std::max(m, host_dmat_[i]);
  push_hist(&hist_d_, m);
  capD_ = align_up64(m * 21 / 20 + (256 << 10), 4096);
}

void RoutedStep::owner_reply(HbmCache* shard, uint8_t* R, uint8_t* data, hipStream_t s) {
  const int W = w_;
  const int64_t rows = (int64_t)W * capG_;
  const int64_t slotR = capG_ * 8 + capD_;
  const int64_t per = capG_ + 2;
  SH_CHECK(capD_ > 0 && capD_ % 16 == 0, "RoutedStep: reply capacity not set");
  uint64_t* hdr = buf<uint64_t>(kHdr, rows);
  uint64_t* used = buf<uint64_t>(kUsed, W);
  uint64_t* offA = buf<uint64_t>(kDstA, (size_t)(W - 1) * per + 1);
  uint64_t* srcA = buf<uint64_t>(kSrcA, (size_t)(W - 1) * per + 1);
  uint64_t* offB = buf<uint64_t>(kDstB, per + 1);
  uint64_t* srcB = buf<uint64_t>(kSrcB, per);
  uint8_t* self_slot = data + capL_ + (int64_t)(W - 1) * slotR;
  hipLaunchKernelGGL(k_reply_used, dim3(1), dim3(64), 0, s, lk_off_, W, rank_, capG_, capD_, slotR,
                     hdr, used, offA, srcA, offB, srcB, rb_);
  hipLaunchKernelGGL(k_reply_prep, dim3(grid1(rows)), dim3(kB), 0, s, lk_loc_, lk_size_, lk_off_,
                     own_cnt_, used, W, capG_, slotR, shard->log_ptr(), hdr, offA, srcA, offB,
                     srcB, reinterpret_cast<unsigned long long*>(rb_ + W));
  RT_OK(hipGetLastError());
  // from here on nothing on `s` touches what the next step's plan writes (it may run
  // beside the reply gather: RoutedStep::step with an inputs-ready event)
  RT_OK(hipEventRecord(ev_pfork_, s));
  if (W > 1) segcopy(nullptr, srcA, offA, (int64_t)(W - 1) * per, R, s);
  segcopy(nullptr, srcB, offB, per, self_slot, s);
}

void RoutedStep::gather_local(uint8_t* data, hipStream_t s) {
  // all-or-nothing: nothing lands when the total outgrew capL (assemble then answers the
  // replica hits as misses; the next steps' capL grows from the observed bytes)
  if (!have_replica_ || !replica_ || n_ <= 0) return;
  replica_->gather(rl_loc_, rl_off_, n_, data, s, (uint64_t)capL_);
}

// ---- SETs ---------------------------------------------------------------------------
std::vector<int64_t> RoutedStep::set_splits() {
  SH_CHECK(published_, "RoutedStep: publish before set_splits");
  const int W = w_, me = rank_;
  const int64_t K = row_words();
  // the matrices of earlier native steps first (history in step order)
  harvest(INT64_MAX, true);
  RT_OK(hipEventSynchronize(ev_pub_));
  mat_.assign(host_mat_, host_mat_ + (size_t)W * K);
  // overflow: GET rows this rank could not send (its slots were full)
  const std::vector<int64_t> st = note_matrix(mat_.data(), n_, capG_, true);
  const int64_t off_rank = st[2], over = st[3];
  sset_.assign(W, 0);
  rset_.assign(W, 0);
  ns_rows_ = ms_ = 0;
  for (int p = 0; p < W; ++p) {
    sset_[p] = 32 * mat_[me * K + W + p] + mat_[me * K + 2 * W + p];
    rset_[p] = 32 * mat_[p * K + W + me] + mat_[p * K + 2 * W + me];
    ns_rows_ += mat_[me * K + W + p];
    ms_ += mat_[p * K + W + me];
    // value offsets travel as 31-bit fields in the SET records
    SH_CHECK(mat_[me * K + 2 * W + p] < (1ll << 31) && mat_[p * K + 2 * W + me] < (1ll << 31),
             "SET values for one peer exceed 2 GiB per step; split the batch");
  }
  std::vector<int64_t> out(2 * W + 5);
  for (int p = 0; p < W; ++p) {
    out[p] = sset_[p];
    out[W + p] = rset_[p];
  }
  out[2 * W] = mat_[me * K + 4 * W];      // n_local (replica hits + duplicates)
  out[2 * W + 1] = mat_[me * K + 4 * W + 2];  // duplicates
  out[2 * W + 2] = off_rank;
  out[2 * W + 3] = over;
  out[2 * W + 4] = mat_[me * K + 4 * W + 3];  // reply rows this shard dropped (last step)
  return out;
}

void RoutedStep::pack_sets(uint8_t* S, hipStream_t s) {
  const int W = w_, me = rank_;
  const int64_t K = row_words();
  // tab: [Sstart (W+1) | Bstart (W) | Psend (W) | segbase (W)] in rank order; send order
  // is the other ranks by rank, then self
  uint64_t* t = host_tab_ + (size_t)par_ * (8 * (size_t)W + 8);
  uint64_t* Sst = t;
  uint64_t* Bst = t + W + 1;
  uint64_t* Ps = Bst + W;
  uint64_t* sb = Ps + W;
  Sst[0] = 0;
  uint64_t b = 0;
  for (int p = 0; p < W; ++p) {
    Sst[p + 1] = Sst[p] + (uint64_t)mat_[me * K + W + p];
    Bst[p] = b;
    b += (uint64_t)mat_[me * K + 2 * W + p];
  }
  uint64_t pos = 0, seg = 0;
  for (int k = 0; k < W; ++k) {
    const int d = k == W - 1 ? me : (k < me ? k : k + 1);
    Ps[d] = pos;
    sb[d] = seg;
    pos += (uint64_t)sset_[d];
    seg += 1 + (uint64_t)mat_[me * K + W + d];
  }
  self_row0_ = (int64_t)Sst[me];
  // the self block (last in send order) is not copied: store_sets reads its records and
  // values where the planner left them, so S holds the other ranks' blocks only
  const int64_t nseg_out = (int64_t)sb[me];
  if (nseg_out == 0) return;
  const size_t words = 5 * (size_t)W + 1;
  uint64_t* dtab = buf<uint64_t>(kTab, 8 * (size_t)W + 8);
  const int64_t nseg = W + ns_rows_;
  uint64_t* seg_off = buf<uint64_t>(kSegOff, nseg + 1);
  uint64_t* seg_src = buf<uint64_t>(kSegSrc, nseg);
  RT_OK(hipMemcpyAsync(dtab, t, words * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_set_segs, dim3(grid1(ns_rows_ + W + 1)), dim3(kB), 0, s, dtab, W, ns_rows_,
                     sval_, svoff_, (uint64_t)(uintptr_t)srec_, pos, seg_off, seg_src);
  RT_OK(hipGetLastError());
  // seg_off[sb[me]] = Ps[me]: the end of the other ranks' blocks
  segcopy(nullptr, seg_src, seg_off, nseg_out, S, s);
}

void RoutedStep::store_sets(const uint8_t* Rs, HbmCache* shard, HbmCache* replica, uint32_t now,
                            hipStream_t s, hipStream_t sset, bool replica_on_sset,
                            hipEvent_t index_after, bool allow_reclaim) {
  const int W = w_, me = rank_;
  const int64_t K = row_words();
  const int64_t ms = ms_;
  if (ms <= 0) return;
  // per source k (others by rank, self last): first row, record block, value block
  uint64_t* t = host_tab_ + (size_t)par_ * (8 * (size_t)W + 8) + 5 * (size_t)W + 1;
  uint64_t* first = t;
  uint64_t* rec = t + W + 1;
  uint64_t* val = rec + W;
  uint64_t row0 = 0, rpos = 0, recv_bytes = 0;
  for (int k = 0; k < W; ++k) {
    const int q = k == W - 1 ? me : (k < me ? k : k + 1);
    const uint64_t rows = (uint64_t)mat_[q * K + W + me];
    first[k] = row0;
    // self: the planner's records (values by absolute address, self_sval below)
    const uint64_t base =
        q == me ? (uint64_t)(uintptr_t)(srec_ + 4 * self_row0_) : (uint64_t)(uintptr_t)Rs + rpos;
    rec[k] = base;
    val[k] = base + 32 * rows;
    row0 += rows;
    recv_bytes += (uint64_t)mat_[q * K + 2 * W + me];
    if (q != me) rpos += (uint64_t)rset_[q];
  }
  first[W] = row0;
  uint64_t* dtab = buf<uint64_t>(kTab, 8 * (size_t)W + 8) + 5 * (size_t)W + 1;
  Digest* rkeys = buf<Digest>(kRkeys, ms);
  uint32_t* v0 = buf<uint32_t>(kV0, ms);
  uint32_t* v1 = buf<uint32_t>(kV1, ms);
  uint32_t* fl = buf<uint32_t>(kFl, ms);
  uint32_t* ex = buf<uint32_t>(kEx, ms);
  uint64_t* roff = buf<uint64_t>(kRoff, ms);
  RT_OK(hipMemcpyAsync(dtab, t, (3 * (size_t)W + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                       sset));
  hipLaunchKernelGGL(k_rs_fill_slots, dim3(grid1(ms)), dim3(kB), 0, sset, dtab, W, ms, rkeys, v0,
                     v1, fl, ex, roff, sval_ + self_row0_);
  RT_OK(hipGetLastError());
  RT_OK(hipEventRecord(ev_sfork_, sset));  // the store arguments are ready
  const uint64_t bound = 48 * (uint64_t)ms + recv_bytes;
  if (replica && replica_on_sset) {
    // native step: the local gather already ran on this stream (it reads the replica log
    // these rows may overwrite); the next step's plan (replica probe) waits for ev_rep_
    replica->store(rkeys, nullptr, roff, v1, fl, ex, ms, bound, now, sset);
    RT_OK(hipEventRecord(ev_rep_, sset));
    rep_pending_ = true;
  }
  // Main shard (tier 0) on the SET stream, after this step's owner probe (or, early
  // under a look-ahead reserve, after the previous step's reply gather with
  // `index_after` = this probe): the probes reserved these bytes (k_owner_prep), so the
  // append never touches a record a reply gather reads. The next owner_probe joins it.
  shard->store(rkeys, nullptr, roff, v0, fl, ex, ms, bound, now, sset, index_after,
               allow_reclaim);
  RT_OK(hipEventRecord(ev_join_, sset));
  sets_pending_ = true;
  // replica (tier 1) on `s`, after this step's local gather (same stream) and the fill
  if (replica && !replica_on_sset) {
    RT_OK(hipStreamWaitEvent(s, ev_sfork_, 0));
    replica->store(rkeys, nullptr, roff, v1, fl, ex, ms, bound, now, s);
  }
}

// ---- assemble -------------------------------------------------------------------------
void RoutedStep::assemble(const uint8_t* data, uint64_t* out_size, uint64_t* out_off,
                          hipStream_t s) {
  const int P = par_;
  if (n_ > 0) {
    const int64_t slotR = capG_ * 8 + capD_;
    hipLaunchKernelGGL(k_assemble_slots, dim3(grid1(n_)), dim3(kB), 0, s, route_, first_, n_, w_,
                       rank_, capG_, capL_, slotR, data, have_replica_ ? rl_size_ : nullptr,
                       have_replica_ ? rl_off_ : nullptr, out_size, out_off);
    RT_OK(hipGetLastError());
  }
  RT_OK(hipEventRecord(ev_asm_[P], s));
  asm_pending_[P] = true;
}

// ---- fixed-slot SETs (step()) -------------------------------------------------------------
// Send buffer S = [W-1 slots, o-order], slot = [16-B header {rows, bytes} | capS records |
// capSB value bytes]: k_set_fit finds each destination's fitting prefix, k_set_pack_segs
// writes the segment list (and carries every row past the prefix), segcopy_dev moves the
// bytes; all on the SET stream, sized from the device (no host read).
void RoutedStep::pack_fixed(uint8_t* S, int64_t slotS, const std::vector<int64_t>& sc,
                            hipStream_t ps) {
  const int W = w_, me = rank_, P = par_;
  const uint64_t* tcnt = buf<uint64_t>(P ? kTcnt1 : kTcnt, 1);
  const uint64_t* tbytes = buf<uint64_t>(P ? kTbytes1 : kTbytes, 1);
  const int64_t nseg_max = 4 * (int64_t)W + nrouted_max_;
  uint64_t* seg_off = buf<uint64_t>(kSegOffF, nseg_max + 1);
  uint64_t* seg_src = buf<uint64_t>(kSegSrcF, nseg_max + 1);
  uint64_t* meta = set_meta_[P];
  hipLaunchKernelGGL(k_set_fit, dim3(1), dim3(256), 0, ps, tcnt, tbytes, gt_, cnt_s_, srec_,
                     svoff_, W, me, sc[0], sc[1], sc[2], sc[3], meta);
  const CarryOut co{ck_[P],  cvl_[P],     cfl_[P],      cex_[P],      cval_[P],    cdst_[P],
                    cbytes_[P], ccap_p_[P], cbcap_p_[P], cctr_ + 2 * P, cctr_ + 4};
  const int64_t tmax = nrouted_max_ + W + 1;
  hipLaunchKernelGGL(k_set_pack_segs, dim3(grid1(tmax)), dim3(kB), 0, ps, meta, tcnt, tbytes,
                     gt_, cnt_s_, srec_, sval_, svoff_, W, me, sc[0], slotS, tmax, seg_off,
                     seg_src, co);
  RT_OK(hipGetLastError());
  if (W > 1) segcopy_dev(seg_src, seg_off, reinterpret_cast<const int64_t*>(meta + 5 * W), S, ps);
  RT_OK(hipEventRecord(ev_pack_, ps));  // the SET exchange sends S
  carry_written_[P] = true;  // the next plan (same stream) reads the carry
}

// Received SETs in fixed rows [others' slots x capS | capSelf own rows] -> the replica
// (tier 1) and the main shard (tier 0), both on the SET stream.
void RoutedStep::store_fixed(const uint8_t* Rs, int64_t slotS, const std::vector<int64_t>& sc,
                             HbmCache* shard, HbmCache* replica, uint32_t now, hipStream_t sset,
                             hipEvent_t index_after, bool allow_reclaim) {
  const int W = w_;
  const int64_t nrows = (int64_t)(W - 1) * sc[0] + sc[2];
  if (nrows <= 0) return;
  Digest* rkeys = buf<Digest>(kRkeys, nrows);
  uint32_t* v0 = buf<uint32_t>(kV0, nrows);
  uint32_t* v1 = buf<uint32_t>(kV1, nrows);
  uint32_t* fl = buf<uint32_t>(kFl, nrows);
  uint32_t* ex = buf<uint32_t>(kEx, nrows);
  uint64_t* roff = buf<uint64_t>(kRoff, nrows);
  hipLaunchKernelGGL(k_rs_fill_fixed, dim3(grid1(nrows)), dim3(kB), 0, sset, Rs, slotS, sc[0], W,
                     set_meta_[par_], rank_, srec_, sval_, nrows, rkeys, v0, v1, fl, ex, roff);
  RT_OK(hipGetLastError());
  RT_OK(hipEventRecord(ev_sfork_, sset));
  const uint64_t bound = 48 * (uint64_t)nrows + (uint64_t)(W - 1) * sc[1] + (uint64_t)sc[3];
  if (replica) {
    // the local gather already ran on this stream (it reads the replica log these rows
    // may overwrite); the next step's plan (replica probe) waits for ev_rep_
    replica->store(rkeys, nullptr, roff, v1, fl, ex, nrows, bound, now, sset);
    RT_OK(hipEventRecord(ev_rep_, sset));
    rep_pending_ = true;
  }
  shard->store(rkeys, nullptr, roff, v0, fl, ex, nrows, bound, now, sset, index_after,
               allow_reclaim);
  RT_OK(hipEventRecord(ev_join_, sset));
  sets_pending_ = true;
}

// ---- the whole step, natively ----------------------------------------------------------
void RoutedStep::set_comm(std::shared_ptr<StepComm> c) {
  SH_CHECK(!c || (c->world() == w_ && c->rank() == rank_), "RoutedStep: comm of another job");
  comm_ = std::move(c);
}

template <typename F>
void RoutedStep::collective(hipStream_t home, hipStream_t comm_stream, int ch, F issue) {
  if (!single_) {
    issue(home, ch);
    return;
  }
  // single: every collective on the comm stream and the control communicator, in issue
  // order; events carry the data dependencies in and out
  if (home != comm_stream) {
    RT_OK(hipEventRecord(ev_c1_, home));
    RT_OK(hipStreamWaitEvent(comm_stream, ev_c1_, 0));
  }
  issue(comm_stream, (int)StepComm::kCtrl);
  if (home != comm_stream) {
    RT_OK(hipEventRecord(ev_c2_, comm_stream));
    RT_OK(hipStreamWaitEvent(home, ev_c2_, 0));
  }
}

std::vector<int64_t> RoutedStep::prepare(int64_t n) {
  harvest(step_id_ - 2, true);
  return caps(n);
}

std::vector<int64_t> RoutedStep::step(const Digest* keys, int64_t n, HbmCache* replica,
                                      uint32_t now, const Digest* skeys, const uint32_t* svlen,
                                      const uint32_t* sflags, const uint32_t* sexpire,
                                      const uint64_t* sval_off, const uint8_t* svalues, int64_t ns,
                                      bool fanout, bool coalesce, HbmCache* shard, uint8_t* data,
                                      uint64_t* out_size, uint64_t* out_off, hipStream_t s,
                                      hipStream_t sset, hipStream_t sasm,
                                      hipEvent_t inputs_ready, int64_t svalues_bytes) {
  SH_CHECK(comm_, "RoutedStep::step: no communicator (set_comm)");
  const int W = w_, me = rank_;
  // the reply transfer and the assembly share one stream: the caller's `sasm` (torch owns
  // it, so tensors recorded on it never outlive it), else the executor's own; in single
  // mode it carries every collective of the step
  hipStream_t cs = sasm;
  // The step's streams come from a per-device pool created once per process and never
  // destroyed (like torch's stream pool): tensors the caller recorded on them can never
  // outlive them, and the first streams of a process get the hardware queues to
  // themselves (4 per process, taken round robin). A CU-masked queue of their own each
  // measured 2-3x slower (0.95 vs 0.47 ms one rank, 2.4 vs 0.83 ms simulated 8 ranks).
  if (!plan_stream_) {
    const StepStreams& ss = step_streams(device_);
    plan_stream_ = ss.plan;
    set_stream_ = ss.set;
    asm_stream_ = ss.asm_;
  }
  if (!sasm) cs = asm_stream_;
  if (!sset) sset = set_stream_;
  note_stream(s);
  note_stream(cs);
  note_stream(sset);
  reap(false);
  // capacities of this step: the matrices of the steps up to two back (every rank the same)
  harvest(step_id_ - 2, true);
  const int64_t K = row_words();
  {
    const std::vector<int64_t> c = caps(n);
    // (a rank without a local-region history yet, c[4], still steps natively so that every
    // rank takes the same path: its replica hits that outgrow the old capL are misses)
    SH_CHECK(!c[3], "RoutedStep::step: a calibrating step takes the multi-call path");
  }
  const std::vector<int64_t> sc = set_caps();
  sv_bytes_ = svalues_bytes;
  // o(p): the position of peer p among the other ranks
  auto o = [me](int p) { return p < me ? p : p - 1; };
  int64_t* row = buf<int64_t>(kRowB, K);
  int64_t* mat = buf<int64_t>(kMatB, (size_t)K * W);
  int64_t slotS = 0;
  uint8_t* Sbuf = nullptr;
  if (!row_init_) {
    RT_OK(hipMemsetAsync(row, 0, K * sizeof(int64_t), s));
    row_init_ = true;
  }
  {
    const int64_t gslot = 16 * caps(n)[0];
    uint8_t* G = buf<uint8_t>(kGB, (size_t)(2 * W - 1) * gslot);
    {
      TraceRange t("serve.plan");
      // With an inputs-ready event the plan runs on its own stream, beside the previous
      // step's reply gather: it waits for the inputs, for the previous step's owner side
      // to be done with what the plan rewrites (ev_pfork_) and for the previous replica
      // store (its probe must see those SETs). Without one, everything queued on `s`
      // before this call is the plan's input (the caller may have produced the keys).
      hipStream_t ps = s;
      if (inputs_ready) {
        ps = plan_stream_;
        RT_OK(hipStreamWaitEvent(ps, inputs_ready, 0));
        if (pfork_valid_) {
          RT_OK(hipStreamWaitEvent(ps, ev_pfork_, 0));
          if (rep_pending_) RT_OK(hipStreamWaitEvent(ps, ev_rep_, 0));
        } else {
          RT_OK(hipEventRecord(ev_start_, s));
          RT_OK(hipStreamWaitEvent(ps, ev_start_, 0));
        }
      }
      in_step_ = true;
      plan(keys, n, replica, now, skeys, svlen, sflags, sexpire, sval_off, svalues, ns, fanout, G,
           row, ps, coalesce);
      in_step_ = false;
      RT_OK(hipEventRecord(ev_plan_, ps));  // the SET stream starts from the plan's output
      if (ps != s) RT_OK(hipStreamWaitEvent(s, ev_plan_, 0));
      // The SET send buffer, packed right behind the plan on its stream (beside this step's
      // GET exchange), once the SET side of the step two back (same parity: its send
      // buffer, slot metadata and carry bytes) is done. This step's carry holds twice
      // the batch's routed rows and a bounded copy of the values (a row finding no room is
      // counted as lost).
      const int P = par_;
      if (sdone_valid_[P]) RT_OK(hipStreamWaitEvent(ps, ev_sdone_[P], 0));
      ensure_carry(2 * (fanout ? ns * W : ns),
                   std::max<uint64_t>(2 * (uint64_t)std::max<int64_t>(svalues_bytes, 0), 64ull << 20));
      slotS = 16 + 32 * sc[0] + sc[1];
      Sbuf = buf<uint8_t>(P ? kS1 : kS0, (size_t)std::max<int64_t>((W - 1) * slotS, 16));
      pack_fixed(Sbuf, slotS, sc, ps);
    }
    {
      TraceRange t("serve.row_allgather");
      // the all-gather, the matrix into the pinned ring (read two steps later) and the
      // request exchange, one collective hop in single mode
      const int slot = ring_next_;
      for (const Pend& q : pend_) SH_CHECK(q.slot != slot, "RoutedStep: matrix ring overrun");
      ring_next_ = (ring_next_ + 1) % kPend;
      collective(s, cs, StepComm::kCtrl, [&](hipStream_t st, int ch) {
        comm_->all_gather(mat, row, K, 4, st, ch);
        RT_OK(hipMemcpyAsync(host_ring_ + (size_t)slot * K * W, mat, (size_t)W * K * sizeof(int64_t),
                             hipMemcpyDeviceToHost, st));
        RT_OK(hipEventRecord(ev_ring_[slot], st));
        if (W > 1) {
          // G = [recv: W-1 slots | self | send: W-1 slots], others in o-order on both sides
          std::vector<int64_t> off_r(W, 0), off_s(W, 0), sz(W, gslot);
          for (int p = 0; p < W; ++p)
            if (p != me) {
              off_r[p] = o(p) * gslot;
              off_s[p] = (int64_t)W * gslot + o(p) * gslot;
            }
          sz[me] = 0;
          comm_->all_to_all(G, off_r, sz, G, off_s, sz, st, ch);
        }
      });
      pend_.push_back(Pend{step_id_, n, capG_, slot, false, false});
      mat_dev_ = mat;  // owner_probe derives the owner slot counts from it
      published_ = false;
    }
    TraceRange t("serve.owner");
    in_step_ = true;  // owner_probe reserves the look-ahead
    owner_probe(G, shard, now, s);
    in_step_ = false;
  }
  const int P = par_;
  // The SET stream starts once the plan is done (the local gather reads its replica
  // locations; packing its SET rows); its main-shard append waits below for what the
  // reserves require, its index insert for this probe
  RT_OK(hipEventRecord(ev_probe_, s));
  RT_OK(hipStreamWaitEvent(sset, ev_plan_, 0));
  // the local (replica) gather on the SET stream, beside the reply gather: the replica
  // store follows it there, so the next step's replica probe need not wait for the reply
  gather_local(data, sset);
  RT_OK(hipEventRecord(ev_local_, sset));
  const int64_t slotR = capG_ * 8 + capD_;
  uint8_t* R = buf<uint8_t>(P ? kR1 : kR0, (size_t)std::max<int64_t>((W - 1) * slotR, 16));
  // the reply transfer of two steps back read this parity's R
  if (reply_pending_[P]) {
    RT_OK(hipStreamWaitEvent(s, ev_reply_[P], 0));
    reply_pending_[P] = false;
  }
  {
    TraceRange t("serve.reply");
    owner_reply(shard, R, data, s);
    // the reply slots (others' in R, the own one in `data`) are written
    RT_OK(hipEventRecord(ev_rfork_, s));
    RT_OK(hipEventRecord(ev_gdone_[P], s));  // this step's log reads are done
    gdone_valid_[P] = true;
    RT_OK(hipStreamWaitEvent(cs, ev_rfork_, 0));
    if (W > 1) {
      // the reply transfer on the comm stream: the SET exchange and the next step's
      // planning run beside it
      collective(cs, cs, StepComm::kData, [&](hipStream_t st, int ch) {
        std::vector<int64_t> off_r(W, 0), off_s(W, 0), sz(W, slotR);
        for (int p = 0; p < W; ++p)
          if (p != me) {
            off_s[p] = o(p) * slotR;
            off_r[p] = capL_ + o(p) * slotR;
          }
        sz[me] = 0;
        comm_->all_to_all(data, off_r, sz, R, off_s, sz, st, ch);
      });
      RT_OK(hipEventRecord(ev_reply_[P], cs));
      reply_pending_[P] = true;
    }
    pfork_valid_ = true;
  }
  {
    TraceRange t("serve.assemble");
    // behind this step's reply transfer on the same stream (and the local gather)
    RT_OK(hipStreamWaitEvent(cs, ev_local_, 0));
    assemble(data, out_size, out_off, cs);
  }
  {
    TraceRange t("serve.set_exchange");
    uint8_t* Rs = buf<uint8_t>(P ? kRs1 : kRs0, (size_t)std::max<int64_t>((W - 1) * slotS, 16));
    // Where the main-shard append may start. This step's probe reserved its bytes (the
    // reply gather never reads them); if the previous probe reserved them too
    // (look-ahead: this step's bytes within its margin), the append needs only the
    // previous step's reply gather done and runs beside this owner phase, with the index
    // insert alone waiting for the probe. Otherwise everything waits for the probe. The
    // payload bound comes from the slot capacities (no host read of the matrix).
    const int64_t nrows = (int64_t)(W - 1) * sc[0] + sc[2];
    const int64_t pay = 48 * nrows + (int64_t)(W - 1) * sc[1] + sc[3];
    const bool early = gdone_valid_[P ^ 1] && ahead_prev_ >= (uint64_t)pay &&
                       !shard->would_reclaim((uint64_t)pay);
    early_sets_ += early ? 1 : 0;
    push_hist(&pay_hist_, pay);
    RT_OK(hipStreamWaitEvent(sset, ev_pack_, 0));
    if (W > 1) {
      // every rank sends every other rank one full slot (fixed size: no split sizes)
      collective(sset, cs, StepComm::kSet, [&](hipStream_t st, int ch) {
        std::vector<int64_t> off_s(W, 0), off_r(W, 0), sz(W, slotS);
        for (int p = 0; p < W; ++p)
          if (p != me) off_s[p] = off_r[p] = o(p) * slotS;
        sz[me] = 0;
        comm_->all_to_all(Rs, off_r, sz, Sbuf, off_s, sz, st, ch);
      });
    }
    // the transfer needs only the packed slots; the stores wait for what the reserves need
    RT_OK(hipStreamWaitEvent(sset, early ? ev_gdone_[P ^ 1] : ev_probe_, 0));
    store_fixed(Rs, slotS, sc, shard, replica, now, sset, early ? ev_probe_ : nullptr,
                /*allow_reclaim=*/!early);
    RT_OK(hipEventRecord(ev_sdone_[P], sset));  // the SET side of this parity is done
    sdone_valid_[P] = true;
  }
  ++step_id_;
  return take_stats();
}

void RoutedStep::join_sets(hipStream_t s) {
  if (!sets_pending_) return;
  RT_OK(hipStreamWaitEvent(s, ev_join_, 0));
  sets_pending_ = false;
}

}  // namespace shellac
