// Fused device ops of the routed serving step (see router.h).
#include "router.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "hbm_cache.h"

#define RT_OK(expr)                                                                     \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw Error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + #expr); \
  } while (0)

namespace shellac {

namespace {

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

// Membership in the hot set, sorted by the signed low word (torch's sort of column 0).
// `dir` (optional, 65537 entries) narrows the search to the keys sharing the top 16
// bits of the order-preserving unsigned image of lo, ~nhot/65536 of them.
__device__ __forceinline__ bool is_hot(const Digest& k, const Digest* __restrict__ hot,
                                       int64_t nhot, const int64_t* __restrict__ dir) {
  const int64_t x = (int64_t)k.lo;
  int64_t lo = 0, hi = nhot;
  if (dir) {
    const uint32_t b = (uint32_t)((k.lo ^ (1ull << 63)) >> 48);
    lo = dir[b];
    hi = dir[b + 1];
  }
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)hot[mid].lo < x) lo = mid + 1; else hi = mid;
  }
  for (int64_t i = lo; i < nhot && (int64_t)hot[i].lo == x; ++i)
    if (hot[i].hi == k.hi) return true;
  return false;
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
// exchange table, xtable[d * 3] = counts[d] for d < nb - 1, and
// extras = {counts[nb - 1] (local replica hits), *rl_off_n (their response bytes)}.
__global__ __launch_bounds__(1024) void k_gr_scan(uint64_t* __restrict__ table, int64_t T,
                                                  int32_t nb, int32_t G,
                                                  int64_t* __restrict__ counts,
                                                  int64_t* __restrict__ xtable = nullptr,
                                                  const uint64_t* __restrict__ rl_off_n = nullptr,
                                                  int64_t* __restrict__ extras = nullptr) {
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
      if (d < nb - 1) xtable[(int64_t)d * 3] = (int64_t)(s1 - s0);
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
  const int nb = w + 1;
  for (int d = threadIdx.x; d < nb; d += kB) s_c[d] = 0;
  if (threadIdx.x == 0) s_dup = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * plen, i1 = min(n, i0 + plen);
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kB) {
    const bool dup = first && first[i] != (uint32_t)i;
    const int d = (dup || (rsize && rsize[i] > 0)) ? w : ring_owner_of(keys[i], pts, own, npts);
    dest[i] = d;
    atomicAdd(&s_c[d], 1u);
    if (dup) atomicAdd(&s_dup, 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < nb; d += kB) table[(int64_t)d * gridDim.x + blockIdx.x] = s_c[d];
  if (threadIdx.x == 0 && ndup && s_dup) atomicAdd(ndup, (unsigned long long)s_dup);
}

// SET planning, fused: input row j goes to its owner and (fan-out) to every rank when
// its key is hot (tier 0 = owner copy, tier 1 = replica copy). Each workgroup handles
// a contiguous range: owner / padded length per row, and the rows AND value bytes per
// destination in one packed 64-bit LDS counter (rows | bytes << 32) so k_ps_scatter
// can hand out row slots and byte ranges in the same order.
__global__ __launch_bounds__(kB) void k_ps_dest_hist(
    const Digest* __restrict__ keys, const uint32_t* __restrict__ vlen, int64_t ns,
    const uint32_t* __restrict__ pts, const int32_t* __restrict__ own, int npts,
    const Digest* __restrict__ hot, int64_t nhot, const int64_t* __restrict__ hot_dir,
    int32_t nb, int64_t plen, int32_t w, int32_t* __restrict__ owner,
    uint32_t* __restrict__ vpad, uint64_t* __restrict__ tcnt, uint64_t* __restrict__ tbytes) {
  extern __shared__ unsigned long long s_cb[];
  for (int d = threadIdx.x; d < nb; d += kB) s_cb[d] = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * plen, i1 = min(ns, i0 + plen);
  for (int64_t j = i0 + threadIdx.x; j < i1; j += kB) {
    const Digest k = keys[j];
    const int o = ring_owner_of(k, pts, own, npts);
    const bool h = nhot > 0 && is_hot(k, hot, nhot, hot_dir);
    owner[j] = h ? (o | (1 << 30)) : o;  // bit 30: fan out to every rank
    const uint32_t vl = vlen[j];
    const uint32_t vp = vl == kSkipVlen ? 0u : (uint32_t)align16(vl);
    vpad[j] = vp;
    const unsigned long long inc = 1ull | ((unsigned long long)vp << 32);
    if (h) {
      for (int r = 0; r < w; ++r) atomicAdd(&s_cb[r], inc);
    } else {
      atomicAdd(&s_cb[o], inc);
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

// Scans both SET tables, then writes the SET columns of the per-peer exchange table:
// table[p * 3 + 1] = SET rows, table[p * 3 + 2] = SET value bytes (k_gr_scan writes
// column 0 on the other stream).
__global__ __launch_bounds__(1024) void k_ps_scan(uint64_t* __restrict__ tcnt,
                                                  uint64_t* __restrict__ tbytes, int32_t nb,
                                                  int32_t G, int64_t* __restrict__ cnt_s,
                                                  int64_t* __restrict__ table) {
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
      table[d * 3 + 1] = c;
      table[d * 3 + 2] = (int64_t)(b1 - tbytes[(int64_t)d * G]);
    }
  }
}

// rec = {lo, hi, vlen | flags << 32, expire | (voff | tier << 31) << 32} where voff is
// the value's offset inside the destination peer's value block.
__global__ __launch_bounds__(kB) void k_ps_scatter(
    int64_t ns, int32_t nb, int64_t plen, const uint64_t* __restrict__ tcnt,
    const uint64_t* __restrict__ tbytes, const Digest* __restrict__ keys,
    const uint32_t* __restrict__ vlen, const uint32_t* __restrict__ flags,
    const uint32_t* __restrict__ expire, const uint64_t* __restrict__ val_off,
    uint64_t values_base, const int32_t* __restrict__ owner, const uint32_t* __restrict__ vpad,
    int32_t w, int64_t* __restrict__ srec, uint64_t* __restrict__ sval,
    uint64_t* __restrict__ svoff) {
  extern __shared__ unsigned long long s_cb[];
  for (int d = threadIdx.x; d < nb; d += kB) s_cb[d] = 0;
  __syncthreads();
  const int G = gridDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * plen, i1 = min(ns, i0 + plen);
  for (int64_t j = i0 + threadIdx.x; j < i1; j += kB) {
    const int ow = owner[j];
    const bool fan = (ow >> 30) != 0;
    const int o = ow & ((1 << 30) - 1);
    const uint64_t pad = vpad[j];
    const Digest k = keys[j];
    const uint64_t r2 = (uint64_t)vlen[j] | ((uint64_t)(flags ? flags[j] : 0u) << 32);
    const uint64_t ex = expire ? expire[j] : 0u;
    const uint64_t src = values_base + val_off[j];
    const int r0 = fan ? 0 : o, r1 = fan ? w : o + 1;
    for (int d = r0; d < r1; ++d) {
      const unsigned long long old = atomicAdd(&s_cb[d], 1ull | (pad << 32));
      const int64_t pos = (int64_t)tcnt[(int64_t)d * G + blockIdx.x] + (int64_t)(old & 0xFFFFFFFFull);
      const uint64_t vglob = tbytes[(int64_t)d * G + blockIdx.x] + (old >> 32);
      const uint64_t voff = vglob - tbytes[(int64_t)d * G];  // within the peer's value block
      const uint64_t tier = d != o ? 1ull : 0ull;
      int64_t* rec = srec + pos * 4;
      rec[0] = (int64_t)k.lo;
      rec[1] = (int64_t)k.hi;
      rec[2] = (int64_t)r2;
      rec[3] = (int64_t)(ex | ((voff | (tier << 31)) << 32));
      sval[pos] = src;
      svoff[pos] = vglob;
    }
  }
}

// Request buffer: a request region [G_0 | R_0 | G_1 | R_1 | ...] (digests and SET
// records, exchanged synchronously) followed by a value region [V_0 | V_1 | ...] (SET
// payloads, exchanged asynchronously so they stay off the critical path to the owner
// lookup). Destination offsets follow from the exchange table, so no scan:
// segments G_p = 2p, R_p = 2p + 1, value row i = 2w + i; seg_off[2w + ns] = total bytes.
__global__ __launch_bounds__(kB) void k_send_segs(const int64_t* __restrict__ table,
                                                  const uint64_t* __restrict__ svoff,
                                                  const uint64_t* __restrict__ sval,
                                                  uint64_t gk_base, uint64_t srec_base, int32_t w,
                                                  int64_t ns, uint64_t* __restrict__ seg_off,
                                                  uint64_t* __restrict__ seg_src) {
  extern __shared__ int64_t s_pre[];  // S[w+1] SET rows, Gp[w+1] GET rows, P[w+1] request starts
  int64_t* S = s_pre;
  int64_t* Gp = S + (w + 1);
  int64_t* P = Gp + (w + 1);
  __shared__ int64_t s_vtot;
  if (threadIdx.x == 0) {
    S[0] = Gp[0] = P[0] = 0;
    int64_t vt = 0;
    for (int p = 0; p < w; ++p) {
      const int64_t g = table[p * 3], sr = table[p * 3 + 1];
      S[p + 1] = S[p] + sr;
      Gp[p + 1] = Gp[p] + g;
      P[p + 1] = P[p] + 16 * g + 32 * sr;
      vt += table[p * 3 + 2];
    }
    s_vtot = vt;
  }
  __syncthreads();
  const uint64_t req = (uint64_t)P[w];
  const int64_t total = ns + w;
  for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i <= total;
       i += (int64_t)gridDim.x * kB) {
    if (i == total) {
      seg_off[2 * w + ns] = req + (uint64_t)s_vtot;
    } else if (i < ns) {
      seg_off[2 * w + i] = req + svoff[i];  // svoff: global byte offset in peer order
      seg_src[2 * w + i] = sval[i];
    } else {
      const int p = (int)(i - ns);
      const int64_t g = Gp[p + 1] - Gp[p];
      seg_off[2 * p] = (uint64_t)P[p];
      seg_src[2 * p] = gk_base + 16 * (uint64_t)Gp[p];
      seg_off[2 * p + 1] = (uint64_t)(P[p] + 16 * g);
      seg_src[2 * p + 1] = srec_base + 32 * (uint64_t)S[p];
    }
  }
}

// De-interleave the received request region into [all G | all R]: 2w segments + end.
__global__ void k_recv_segs(const int64_t* __restrict__ rtable, uint64_t recv_base, int32_t w,
                            uint64_t* __restrict__ seg_off, uint64_t* __restrict__ seg_src) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t q0 = 0, g0 = 0, r0 = 0, gtot = 0;
  for (int q = 0; q < w; ++q) gtot += 16 * (uint64_t)rtable[q * 3];
  for (int q = 0; q < w; ++q) {
    const uint64_t a = (uint64_t)rtable[q * 3], b = (uint64_t)rtable[q * 3 + 1];
    seg_off[q] = g0;
    seg_src[q] = recv_base + q0;
    seg_off[w + q] = gtot + r0;
    seg_src[w + q] = recv_base + q0 + 16 * a;
    g0 += 16 * a;
    r0 += 32 * b;
    q0 += 16 * a + 32 * b;  // the value region follows all request chunks
  }
  seg_off[2 * w] = gtot + r0;
}

__global__ __launch_bounds__(kB) void k_rs_fill(
    const int64_t* __restrict__ rrec, int64_t ms, const int64_t* __restrict__ rtable, int32_t w,
    Digest* __restrict__ keys, uint32_t* __restrict__ vlen0, uint32_t* __restrict__ vlen1,
    uint32_t* __restrict__ flags, uint32_t* __restrict__ expire, uint64_t* __restrict__ roff) {
  extern __shared__ int64_t s_q[];  // first[w+1], vstart[w]
  int64_t* first = s_q;
  int64_t* vstart = s_q + (w + 1);
  if (threadIdx.x == 0) {
    int64_t v0 = 0;  // value region starts after every source's request chunk
    for (int q = 0; q < w; ++q) v0 += 16 * rtable[q * 3] + 32 * rtable[q * 3 + 1];
    first[0] = 0;
    for (int q = 0; q < w; ++q) {
      vstart[q] = v0;
      first[q + 1] = first[q] + rtable[q * 3 + 1];
      v0 += rtable[q * 3 + 2];
    }
  }
  __syncthreads();
  for (int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x; r < ms; r += (int64_t)gridDim.x * kB) {
    int lo = 0, hi = w;  // source q with first[q] <= r < first[q+1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (first[mid] <= r) lo = mid; else hi = mid;
    }
    const int64_t* rec = rrec + r * 4;
    keys[r] = Digest{(uint64_t)rec[0], (uint64_t)rec[1]};
    const uint32_t vl = (uint32_t)rec[2];
    const uint64_t hi32 = (uint64_t)rec[3] >> 32;
    const uint32_t tier = (uint32_t)(hi32 >> 31);
    vlen0[r] = tier == 0 ? vl : kSkipVlen;
    vlen1[r] = tier == 1 ? vl : kSkipVlen;
    flags[r] = (uint32_t)((uint64_t)rec[2] >> 32);
    expire[r] = (uint32_t)rec[3];
    roff[r] = (uint64_t)vstart[lo] + (hi32 & 0x7FFFFFFFull);
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

__global__ void k_reply_bytes(const uint64_t* __restrict__ lk_off,
                              const int64_t* __restrict__ rtable,
                              const uint64_t* __restrict__ gscan,
                              const int64_t* __restrict__ table, int32_t w,
                              int64_t* __restrict__ bytes) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t R = 0, G = 0;
  for (int q = 0; q < w; ++q) {
    const int64_t a = rtable[q * 3], g = table[q * 3];
    bytes[q] = (int64_t)(lk_off[R + a] - lk_off[R]);
    bytes[w + q] = (int64_t)(gscan[G + g] - gscan[G]);
    R += a;
    G += g;
  }
}

__global__ __launch_bounds__(kB) void k_assemble(const int64_t* __restrict__ perm, int64_t n,
                                                 int64_t n_remote,
                                                 const uint64_t* __restrict__ sizes_back,
                                                 const uint64_t* __restrict__ gscan,
                                                 const uint64_t* __restrict__ rl_size,
                                                 const uint64_t* __restrict__ rl_off,
                                                 uint64_t local_bytes, uint64_t* __restrict__ size,
                                                 uint64_t* __restrict__ off) {
  for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
    if (rl_size && rl_size[i] > 0) {
      size[i] = rl_size[i];
      off[i] = rl_off[i];
      continue;
    }
    const int64_t p = perm[i];
    if (p < n_remote) {
      size[i] = sizes_back[p];
      off[i] = gscan[p] + local_bytes;
    } else {
      size[i] = 0;
      off[i] = local_bytes;
    }
  }
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
// RoutedStep
// =====================================================================================
namespace shellac {

namespace {
enum Slot {
  kRlLoc, kRlSize, kRlOff, kDestG, kGk, kPermG, kCntG, kWsG, kOwnerS, kVpad, kTcnt,
  kTbytes, kSrec, kSval, kSvoff, kCntS, kSegOff, kSegSrc, kBody, kRSegOff, kRSegSrc,
  kLkLoc, kLkOff, kGscan, kParts, kNbytes, kRkeys, kV0, kV1, kFl, kEx, kRoff, kCoTab, kFirst,
  kNumSlots
};
}  // namespace

RoutedStep::RoutedStep(int world, int rank, int device)
    : w_(world), rank_(rank), device_(device), bufs_(kNumSlots) {
  SH_CHECK(world >= 1 && world < kMaxBuckets, "bad world size");
  RT_OK(hipSetDevice(device_));
  RT_OK(hipHostMalloc(&host_, (8 * (size_t)world + 8) * sizeof(int64_t), hipHostMallocDefault));
  RT_OK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  RT_OK(hipStreamCreateWithFlags(&store_side_, hipStreamNonBlocking));
  RT_OK(hipEventCreateWithFlags(&ev_sfork_, hipEventDisableTiming));
  RT_OK(hipStreamCreateWithFlags(&local_side_, hipStreamNonBlocking));
  RT_OK(hipEventCreateWithFlags(&ev_lfork_, hipEventDisableTiming));
  RT_OK(hipEventCreateWithFlags(&ev_ljoin_, hipEventDisableTiming));
  RT_OK(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
  RT_OK(hipEventCreateWithFlags(&ev_fill_, hipEventDisableTiming));
  RT_OK(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
  RT_OK(hipEventCreateWithFlags(&ev_pjoin_, hipEventDisableTiming));
}

RoutedStep::~RoutedStep() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (auto& b : bufs_) (void)hipFree(b.p);
  (void)hipHostFree(host_);
  (void)hipEventDestroy(ev_fork_);
  (void)hipEventDestroy(ev_fill_);
  (void)hipEventDestroy(ev_join_);
  (void)hipEventDestroy(ev_pjoin_);
  (void)hipEventDestroy(ev_sfork_);
  (void)hipEventDestroy(ev_lfork_);
  (void)hipEventDestroy(ev_ljoin_);
  (void)hipStreamDestroy(side_);
  (void)hipStreamDestroy(store_side_);
  (void)hipStreamDestroy(local_side_);
}

void RoutedStep::set_ring(const uint32_t* pts, const int32_t* owner, int32_t npts) {
  pts_ = pts;
  own_ = owner;
  npts_ = npts;
}

void RoutedStep::set_hot(const Digest* hot, int64_t nhot, const int64_t* dir) {
  hot_ = hot;
  nhot_ = hot ? nhot : 0;
  hot_dir_ = hot ? dir : nullptr;
}

template <typename T>
T* RoutedStep::buf(int slot, size_t count) {
  Buf& b = bufs_[slot];
  const size_t need = std::max<size_t>(count, 1) * sizeof(T);
  if (b.cap < need) {
    // grow-only; the old block may still be read by queued work on this device
    if (b.p) {
      RT_OK(hipDeviceSynchronize());
      RT_OK(hipFree(b.p));
    }
    const size_t cap = (need + need / 4 + 255) & ~(size_t)255;
    RT_OK(hipMalloc(&b.p, cap));
    b.cap = cap;
  }
  return static_cast<T*>(b.p);
}

void RoutedStep::plan(const Digest* keys, int64_t n, HbmCache* replica, uint32_t now,
                      const Digest* skeys, const uint32_t* svlen, const uint32_t* sflags,
                      const uint32_t* sexpire, const uint64_t* sval_off, const uint8_t* svalues,
                      int64_t ns, bool fanout, int64_t* table, hipStream_t s, bool coalesce) {
  SH_CHECK(pts_ && own_ && npts_ > 0, "RoutedStep: ring not set");
  const int W = w_;
  const int nb = W + 1;
  n_ = n;
  values_ = svalues;
  have_replica_ = replica != nullptr;
  replica_ = replica;
  local_done_ = false;
  table_ = table;
  int64_t* extras = table + 6 * W;  // [table | rtable | extras]: one D2H in read_counts
  first_ = nullptr;
  uint32_t* co_tab = nullptr;
  int64_t co_slots = 0;
  if (coalesce && n > 0) {
    co_slots = coalesce_table_slots(n);
    co_tab = buf<uint32_t>(kCoTab, co_slots);
    first_ = buf<uint32_t>(kFirst, n);
  }
  // every buffer first (buf() may reallocate, which synchronises the device)
  uint64_t* rl_size = nullptr;
  if (replica) {
    rl_loc_ = buf<uint64_t>(kRlLoc, n);
    rl_size = rl_size_ = buf<uint64_t>(kRlSize, n + 1);
    rl_off_ = buf<uint64_t>(kRlOff, n + 1);
  }
  int32_t* dest_g = buf<int32_t>(kDestG, n);
  gk_ = buf<Digest>(kGk, n);
  perm_g_ = buf<int64_t>(kPermG, n);
  cnt_g_ = buf<int64_t>(kCntG, nb);
  const int64_t ng = std::max<int64_t>(n, 1);
  const int Gg = group_grid(ng);
  const int64_t plen_g = (ng + Gg - 1) / Gg;
  uint64_t* ws_g = buf<uint64_t>(kWsG, group_ws_words(ng, nb));
  // SET rows fan out up to W ways: smaller ranges per workgroup than the GET sort
  const int64_t nsx = std::max<int64_t>(ns, 1);
  const int Gs = group_grid(nsx, 256);
  const int64_t plen_s = (nsx + Gs - 1) / Gs;
  const int64_t mcap = fanout ? ns * W : ns;  // upper bound of routed SET rows
  int32_t* owner_s = buf<int32_t>(kOwnerS, ns);
  uint32_t* vpad = buf<uint32_t>(kVpad, ns);
  uint64_t* tcnt = buf<uint64_t>(kTcnt, (size_t)nb * Gs);
  uint64_t* tbytes = buf<uint64_t>(kTbytes, (size_t)nb * Gs);
  srec_ = buf<int64_t>(kSrec, 4 * (size_t)mcap);
  sval_ = buf<uint64_t>(kSval, mcap);
  svoff_ = buf<uint64_t>(kSvoff, mcap);
  cnt_s_ = buf<int64_t>(kCntS, nb);

  // SET planning on the side stream (owner + hot fan-out, counting sort with value-byte
  // ranges), concurrently with the replica probe and GET sort on `s`
  RT_OK(hipEventRecord(ev_fork_, s));
  RT_OK(hipStreamWaitEvent(side_, ev_fork_, 0));
  hipLaunchKernelGGL(k_ps_dest_hist, dim3(Gs), dim3(kB), nb * sizeof(unsigned long long), side_,
                     skeys, svlen, ns, pts_, own_, npts_, fanout ? hot_ : nullptr,
                     fanout ? nhot_ : 0, fanout ? hot_dir_ : nullptr, nb, plen_s, W, owner_s,
                     vpad, tcnt, tbytes);
  hipLaunchKernelGGL(k_ps_scan, dim3(1), dim3(1024), 0, side_, tcnt, tbytes, nb, Gs, cnt_s_,
                     table);
  if (ns > 0)
    hipLaunchKernelGGL(k_ps_scatter, dim3(Gs), dim3(kB), nb * sizeof(unsigned long long), side_,
                       ns, nb, plen_s, tcnt, tbytes, skeys, svlen, sflags, sexpire, sval_off,
                       (uint64_t)(uintptr_t)svalues, owner_s, vpad, W, srec_, sval_, svoff_);
  RT_OK(hipGetLastError());
  RT_OK(hipEventRecord(ev_pjoin_, side_));

  // GET rows: coalesce duplicates (they stay local and are filled in by finish), owner
  // (or bucket W = local replica hit / duplicate), counting sort by owner
  RT_OK(hipMemsetAsync(extras + 2, 0, sizeof(int64_t), s));
  if (first_ && replica)  // one pass: each digest's claiming row probes the replica
    replica->lookup_coalesced(keys, n, co_tab, co_slots, first_, rl_loc_, rl_size_, rl_off_, now,
                              s);
  else if (first_)
    coalesce_keys(keys, n, co_tab, co_slots, first_, s);
  else if (replica)
    replica->lookup(keys, n, rl_loc_, rl_size_, rl_off_, now, s);
  hipLaunchKernelGGL(k_route_hist, dim3(Gg), dim3(kB), nb * sizeof(uint32_t), s, keys, n, rl_size,
                     pts_, own_, npts_, W, plen_g, dest_g, ws_g, first_,
                     reinterpret_cast<unsigned long long*>(extras + 2));
  hipLaunchKernelGGL(k_gr_scan, dim3(1), dim3(1024), 0, s, ws_g, (int64_t)nb * Gg, nb, Gg, cnt_g_,
                     table, replica ? rl_off_ + n : nullptr, extras);
  if (n > 0)
    hipLaunchKernelGGL(k_gr_scatter, dim3(Gg), dim3(kB), nb * sizeof(uint32_t), s, dest_g, n, nb,
                       plen_g, ws_g, (const uint32_t*)keys, 4, (uint32_t*)gk_, perm_g_);
  RT_OK(hipGetLastError());
  RT_OK(hipStreamWaitEvent(s, ev_pjoin_, 0));  // join: the table is complete
}

std::vector<int64_t> RoutedStep::read_counts(const int64_t* rtable, hipStream_t s) {
  const int W = w_;
  rtable_ = rtable;
  SH_CHECK(rtable == table_ + 3 * W, "RoutedStep: rtable must follow table (one D2H)");
  RT_OK(hipMemcpyAsync(host_, table_, (6 * W + 3) * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  RT_OK(hipStreamSynchronize(s));
  std::vector<int64_t> out(host_, host_ + 6 * W + 3);
  n_local_ = out[6 * W];
  local_bytes_ = (uint64_t)out[6 * W + 1];
  n_remote_ = n_ - n_local_;
  ns_ = mg_ = ms_ = 0;
  for (int p = 0; p < W; ++p) {
    ns_ += out[3 * p + 1];
    mg_ += out[3 * W + 3 * p];
    ms_ += out[3 * W + 3 * p + 1];
    // value offsets travel as 31-bit fields in the SET records
    SH_CHECK(out[3 * p + 2] < (1ll << 31) && out[3 * W + 3 * p + 2] < (1ll << 31),
             "SET values for one peer exceed 2 GiB per step; split the batch");
  }
  return out;
}

void RoutedStep::pack(uint8_t* send, hipStream_t s) {
  const int W = w_;
  const int64_t nseg = 2 * (int64_t)W + ns_;
  uint64_t* seg_off = buf<uint64_t>(kSegOff, nseg + 1);
  uint64_t* seg_src = buf<uint64_t>(kSegSrc, nseg);
  hipLaunchKernelGGL(k_send_segs, dim3(grid1(ns_ + W + 1)), dim3(kB), 3 * (W + 1) * sizeof(int64_t),
                     s, table_, svoff_, sval_, (uint64_t)(uintptr_t)gk_,
                     (uint64_t)(uintptr_t)srec_, W, ns_, seg_off, seg_src);
  RT_OK(hipGetLastError());
  segcopy(nullptr, seg_src, seg_off, nseg, send, s);
}

void RoutedStep::owner(const uint8_t* recv, HbmCache* shard, uint32_t now, uint64_t* sizes_out,
                       hipStream_t s) {
  const int W = w_;
  // the last step's SET chain reads the body arena (rrec_) and writes the main shard:
  // both are about to be reused
  join_sets(s);
  uint8_t* body = buf<uint8_t>(kBody, 16 * mg_ + 32 * ms_ + 16);
  uint64_t* roff = buf<uint64_t>(kRSegOff, 2 * W + 1);
  uint64_t* rsrc = buf<uint64_t>(kRSegSrc, 2 * W);
  hipLaunchKernelGGL(k_recv_segs, dim3(1), dim3(64), 0, s, rtable_, (uint64_t)(uintptr_t)recv, W,
                     roff, rsrc);
  RT_OK(hipGetLastError());
  segcopy(nullptr, rsrc, roff, 2 * W, body, s);
  rrec_ = reinterpret_cast<const int64_t*>(body + 16 * mg_);
  lk_loc_ = buf<uint64_t>(kLkLoc, mg_);
  lk_off_ = buf<uint64_t>(kLkOff, mg_ + 1);
  shard->lookup(reinterpret_cast<const Digest*>(body), mg_, lk_loc_, sizes_out, lk_off_, now, s);
}

std::vector<int64_t> RoutedStep::reply_sizes(const uint64_t* sizes_in, hipStream_t s) {
  const int W = w_;
  sizes_in_ = sizes_in;
  gscan_ = buf<uint64_t>(kGscan, n_remote_ + 1);
  scan_u64(sizes_in, n_remote_, buf<uint64_t>(kParts, scan_parts_words(n_remote_)), gscan_, s);
  int64_t* nb = buf<int64_t>(kNbytes, 2 * W);
  hipLaunchKernelGGL(k_reply_bytes, dim3(1), dim3(64), 0, s, lk_off_, rtable_, gscan_, table_, W,
                     nb);
  RT_OK(hipGetLastError());
  RT_OK(hipMemcpyAsync(host_ + 6 * W + 2, nb, 2 * W * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  RT_OK(hipStreamSynchronize(s));
  return std::vector<int64_t>(host_ + 6 * W + 2, host_ + 8 * W + 2);
}

void RoutedStep::gather_replies(HbmCache* shard, uint8_t* reply, hipStream_t s) {
  if (mg_ > 0) shard->gather(lk_loc_, lk_off_, mg_, reply, s);
}

// Received-SET unpacking and the main-shard SET chain on the side stream, after the work
// queued on `s` so far (the reply gather). Queuing it before host sync 2 instead (with the
// owner lookup reserving its log bytes), to fill the GPU's idle time there, was measured
// slower: simulated 8 ranks 0.83 / 0.82 vs 0.83 / 0.79 ms per step, 2 ranks 0.80 / 0.84 vs
// 0.77 / 0.79 — the SET chain then competes with the owner probe and reply gather.
void RoutedStep::fork_store(const uint8_t* recv, int64_t recv_bytes, HbmCache* shard,
                            uint32_t now, hipStream_t s) {
  const int64_t ms = ms_;
  const uint64_t bound = 48 * (uint64_t)ms + (uint64_t)recv_bytes;
  Digest* rkeys = buf<Digest>(kRkeys, ms);
  uint32_t* v0 = buf<uint32_t>(kV0, ms);
  uint32_t* v1 = buf<uint32_t>(kV1, ms);
  uint32_t* fl = buf<uint32_t>(kFl, ms);
  uint32_t* ex = buf<uint32_t>(kEx, ms);
  uint64_t* roff = buf<uint64_t>(kRoff, ms);
  RT_OK(hipEventRecord(ev_sfork_, s));
  RT_OK(hipStreamWaitEvent(store_side_, ev_sfork_, 0));
  hipLaunchKernelGGL(k_rs_fill, dim3(grid1(ms)), dim3(kB), (2 * w_ + 1) * sizeof(int64_t),
                     store_side_, rrec_, ms, rtable_, w_, rkeys, v0, v1, fl, ex, roff);
  RT_OK(hipGetLastError());
  RT_OK(hipEventRecord(ev_fill_, store_side_));
  shard->store(rkeys, recv, roff, v0, fl, ex, ms, bound, now, store_side_);
  RT_OK(hipEventRecord(ev_join_, store_side_));
  sets_pending_ = true;
}

void RoutedStep::gather_local(uint8_t* data, hipStream_t s) {
  if (!(have_replica_ && replica_ && n_local_ > 0 && local_bytes_ > 0)) return;
  RT_OK(hipEventRecord(ev_lfork_, s));
  RT_OK(hipStreamWaitEvent(local_side_, ev_lfork_, 0));
  replica_->gather(rl_loc_, rl_off_, n_, data, local_side_);
  RT_OK(hipEventRecord(ev_ljoin_, local_side_));
  local_pending_ = true;
  local_done_ = true;
}

void RoutedStep::join_local(hipStream_t s) {
  if (!local_pending_) return;
  RT_OK(hipStreamWaitEvent(s, ev_ljoin_, 0));
  local_pending_ = false;
}

void RoutedStep::join_sets(hipStream_t s) {
  if (!sets_pending_) return;
  RT_OK(hipStreamWaitEvent(s, ev_join_, 0));
  sets_pending_ = false;
}

void RoutedStep::finish(uint8_t* data, const uint8_t* recv, int64_t recv_bytes, HbmCache* shard,
                        HbmCache* replica, uint32_t now, uint64_t* out_size, uint64_t* out_off,
                        hipStream_t s) {
  const int64_t ms = ms_;
  uint32_t *v1 = nullptr, *fl = nullptr, *ex = nullptr;
  Digest* rkeys = nullptr;
  uint64_t* roff = nullptr;
  const uint64_t bound = 48 * (uint64_t)ms + (uint64_t)recv_bytes;
  if (ms > 0) {
    // fork: received-SET unpacking and the main-shard SET chain (latency-bound small
    // grids) go to the side stream, concurrently with the bandwidth-bound replica
    // gather below. They touch different shards; everything the caller queued before
    // (reply gather from the main shard, the wait for the SET payloads) comes first.
    fork_store(recv, recv_bytes, shard, now, s);
    rkeys = buf<Digest>(kRkeys, ms);  // filled by k_rs_fill on the side stream (ev_fill_)
    v1 = buf<uint32_t>(kV1, ms);
    fl = buf<uint32_t>(kFl, ms);
    ex = buf<uint32_t>(kEx, ms);
    roff = buf<uint64_t>(kRoff, ms);
  }
  if (local_done_) join_local(s);  // gathered early (gather_local) on the local stream
  else if (have_replica_ && replica && n_local_ > 0) replica->gather(rl_loc_, rl_off_, n_, data, s);
  // k_rs_fill reads rtable_, which the next step's count exchange overwrites: later work
  // on `s` (and the collectives ordered after it) waits for the fill
  if (ms > 0) RT_OK(hipStreamWaitEvent(s, ev_fill_, 0));
  if (ms > 0 && replica) {
    // the replica's own SET rows (tier 1) go after its gather: they may overwrite
    // log bytes the gather reads (the fill they read was waited for above)
    replica->store(rkeys, recv, roff, v1, fl, ex, ms, bound, now, s);
  }
  if (n_ > 0)
    hipLaunchKernelGGL(k_assemble, dim3(grid1(n_)), dim3(kB), 0, s, perm_g_, n_, n_remote_,
                       sizes_in_, gscan_, have_replica_ ? rl_size_ : nullptr,
                       have_replica_ ? rl_off_ : nullptr, local_bytes_, out_size, out_off);
  RT_OK(hipGetLastError());
  if (first_) expand_coalesced(first_, n_, out_size, out_off, s);  // duplicates: claimer's record
  // join: later work sees the SETs. Deferred (default), the next step's plan (replica
  // probe, routing: no main-shard access) runs concurrently with the SET chain and its
  // owner() joins
  if (!defer_join_) join_sets(s);
}

}  // namespace shellac
