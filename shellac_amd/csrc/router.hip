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

int group_grid(int64_t n) {
  int64_t g = (n + kGroupRows - 1) / kGroupRows;
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
__device__ __forceinline__ bool is_hot(const Digest& k, const Digest* __restrict__ hot,
                                       int64_t nhot) {
  const int64_t x = (int64_t)k.lo;
  int64_t lo = 0, hi = nhot;
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
__global__ __launch_bounds__(1024) void k_gr_scan(uint64_t* __restrict__ table, int64_t T,
                                                  int32_t nb, int32_t G,
                                                  int64_t* __restrict__ counts) {
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

__global__ __launch_bounds__(kB) void k_ps_dest(const Digest* __restrict__ keys, int64_t ns,
                                                const uint32_t* __restrict__ pts,
                                                const int32_t* __restrict__ own, int npts,
                                                const Digest* __restrict__ hot, int64_t nhot,
                                                int32_t w, bool fanout,
                                                int32_t* __restrict__ dest,
                                                int32_t* __restrict__ owner) {
  for (int64_t j = (int64_t)blockIdx.x * kB + threadIdx.x; j < ns; j += (int64_t)gridDim.x * kB) {
    const Digest k = keys[j];
    const int o = ring_owner_of(k, pts, own, npts);
    owner[j] = o;
    if (!fanout) {
      dest[j] = o;
      continue;
    }
    const bool h = nhot > 0 && is_hot(k, hot, nhot);
    for (int r = 0; r < w; ++r) dest[j * w + r] = (r == o || h) ? r : w;
  }
}

__global__ __launch_bounds__(kB) void k_ps_scatter(
    const int32_t* __restrict__ dest, int64_t m, int32_t nb, int64_t plen,
    const uint64_t* __restrict__ table, const Digest* __restrict__ keys,
    const uint32_t* __restrict__ vlen, const uint32_t* __restrict__ flags,
    const uint32_t* __restrict__ expire, const uint64_t* __restrict__ val_off,
    uint64_t values_base, const int32_t* __restrict__ owner, int32_t w, bool fanout,
    int64_t* __restrict__ srec, uint64_t* __restrict__ sval, uint64_t* __restrict__ spad) {
  extern __shared__ uint32_t s_cur[];
  for (int d = threadIdx.x; d < nb; d += kB) s_cur[d] = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * plen, i1 = min(m, i0 + plen);
  for (int64_t v = i0 + threadIdx.x; v < i1; v += kB) {
    const int d = dest[v];
    const int64_t pos =
        (int64_t)table[(int64_t)d * gridDim.x + blockIdx.x] + atomicAdd(&s_cur[d], 1u);
    const int64_t j = fanout ? v / w : v;
    const int r = fanout ? (int)(v - j * w) : owner[j];
    const uint32_t tier = (fanout && r != owner[j]) ? 1u : 0u;
    const Digest k = keys[j];
    const uint32_t vl = vlen[j];
    int64_t* rec = srec + pos * 4;
    rec[0] = (int64_t)k.lo;
    rec[1] = (int64_t)k.hi;
    rec[2] = (int64_t)((uint64_t)vl | ((uint64_t)(flags ? flags[j] : 0u) << 32));
    rec[3] = (int64_t)((uint64_t)(expire ? expire[j] : 0u) | ((uint64_t)tier << 32));
    sval[pos] = values_base + val_off[j];
    spad[pos] = (d < w && vl != kSkipVlen) ? align16(vl) : 0;
  }
}

__global__ void k_plan_table(const int64_t* __restrict__ cnt_g, const int64_t* __restrict__ cnt_s,
                             const uint64_t* __restrict__ vscan, int32_t w,
                             int64_t* __restrict__ table) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t S = 0;
  for (int p = 0; p < w; ++p) {
    table[p * 3 + 0] = cnt_g[p];
    table[p * 3 + 1] = cnt_s[p];
    table[p * 3 + 2] = (int64_t)(vscan[S + cnt_s[p]] - vscan[S]);
    S += cnt_s[p];
  }
}

// Per-peer prefix sums staged in LDS by every workgroup (w is small).
__global__ __launch_bounds__(kB) void k_send_segs(const int64_t* __restrict__ cnt_g,
                                                  const int64_t* __restrict__ cnt_s,
                                                  const uint64_t* __restrict__ spad,
                                                  const uint64_t* __restrict__ sval,
                                                  uint64_t gk_base, uint64_t srec_base, int32_t w,
                                                  int64_t ns, uint64_t* __restrict__ seg_len,
                                                  uint64_t* __restrict__ seg_src) {
  extern __shared__ int64_t s_pre[];  // S[w+1], Gp[w+1]
  int64_t* S = s_pre;
  int64_t* Gp = s_pre + (w + 1);
  if (threadIdx.x == 0) {
    S[0] = Gp[0] = 0;
    for (int p = 0; p < w; ++p) {
      S[p + 1] = S[p] + cnt_s[p];
      Gp[p + 1] = Gp[p] + cnt_g[p];
    }
  }
  __syncthreads();
  const int64_t total = ns + w;
  for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kB) {
    if (i < ns) {
      int lo = 0, hi = w;  // last p with S[p] <= i
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (S[mid] <= i) lo = mid; else hi = mid;
      }
      const int64_t seg = i + 2 * lo + 2;
      seg_len[seg] = spad[i];
      seg_src[seg] = sval[i];
    } else {
      const int p = (int)(i - ns);
      const int64_t g = 2 * p + S[p];
      seg_len[g] = 16 * (uint64_t)cnt_g[p];
      seg_src[g] = gk_base + 16 * (uint64_t)Gp[p];
      seg_len[g + 1] = 32 * (uint64_t)cnt_s[p];
      seg_src[g + 1] = srec_base + 32 * (uint64_t)S[p];
    }
  }
}

__global__ void k_recv_segs(const int64_t* __restrict__ rtable, uint64_t recv_base, int32_t w,
                            uint64_t* __restrict__ seg_len, uint64_t* __restrict__ seg_src) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t q0 = 0;
  for (int q = 0; q < w; ++q) {
    const uint64_t a = (uint64_t)rtable[q * 3], b = (uint64_t)rtable[q * 3 + 1],
                   c = (uint64_t)rtable[q * 3 + 2];
    seg_len[q] = 16 * a;
    seg_src[q] = recv_base + q0;
    seg_len[w + q] = 32 * b;
    seg_src[w + q] = recv_base + q0 + 16 * a;
    q0 += 16 * a + 32 * b + c;
  }
}

__global__ __launch_bounds__(kB) void k_rs_pad(const int64_t* __restrict__ rrec, int64_t ms,
                                               uint64_t* __restrict__ rpad) {
  for (int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x; r <= ms; r += (int64_t)gridDim.x * kB) {
    if (r == ms) {
      rpad[ms] = 0;
      continue;
    }
    const uint32_t vl = (uint32_t)rrec[r * 4 + 2];
    rpad[r] = vl == kSkipVlen ? 0 : align16(vl);
  }
}

__global__ __launch_bounds__(kB) void k_rs_fill(
    const int64_t* __restrict__ rrec, int64_t ms, const int64_t* __restrict__ rtable, int32_t w,
    const uint64_t* __restrict__ rscan, Digest* __restrict__ keys, uint32_t* __restrict__ vlen0,
    uint32_t* __restrict__ vlen1, uint32_t* __restrict__ flags, uint32_t* __restrict__ expire,
    uint64_t* __restrict__ roff) {
  extern __shared__ int64_t s_q[];  // first[w+1], vstart[w]
  int64_t* first = s_q;
  int64_t* vstart = s_q + (w + 1);
  if (threadIdx.x == 0) {
    int64_t q0 = 0;
    first[0] = 0;
    for (int q = 0; q < w; ++q) {
      const int64_t a = rtable[q * 3], b = rtable[q * 3 + 1], c = rtable[q * 3 + 2];
      vstart[q] = q0 + 16 * a + 32 * b;
      first[q + 1] = first[q] + b;
      q0 += 16 * a + 32 * b + c;
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
    const uint32_t tier = (uint32_t)((uint64_t)rec[3] >> 32);
    vlen0[r] = tier == 0 ? vl : kSkipVlen;
    vlen1[r] = tier == 1 ? vl : kSkipVlen;
    flags[r] = (uint32_t)((uint64_t)rec[2] >> 32);
    expire[r] = (uint32_t)rec[3];
    roff[r] = (uint64_t)vstart[lo] + (rscan[r] - rscan[first[lo]]);
  }
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

void plan_sets(const Digest* keys, const uint32_t* vlen, const uint32_t* flags,
               const uint32_t* expire, const uint64_t* val_off, int64_t ns, uint64_t values_base,
               const uint32_t* ring_pts, const int32_t* ring_owner, int32_t npts,
               const Digest* hot, int64_t nhot, int32_t w, bool fanout, int32_t* dest_ws,
               int32_t* owner_ws, uint64_t* ws, int64_t* srec, uint64_t* sval, uint64_t* spad,
               int64_t* counts, hipStream_t s) {
  const int64_t m = fanout ? ns * w : ns;
  if (m <= 0) {
    RT_OK(hipMemsetAsync(counts, 0, (w + 1) * sizeof(int64_t), s));
    return;
  }
  hipLaunchKernelGGL(k_ps_dest, dim3(grid1(ns)), dim3(kB), 0, s, keys, ns, ring_pts, ring_owner,
                     npts, hot, nhot, w, fanout, dest_ws, owner_ws);
  int G;
  int64_t plen;
  hist_and_scan(dest_ws, m, w + 1, ws, counts, &G, &plen, s);
  hipLaunchKernelGGL(k_ps_scatter, dim3(G), dim3(kB), (w + 1) * sizeof(uint32_t), s, dest_ws, m,
                     w + 1, plen, ws, keys, vlen, flags, expire, val_off, values_base, owner_ws, w,
                     fanout, srec, sval, spad);
  RT_OK(hipGetLastError());
}

void plan_table(const int64_t* cnt_g, const int64_t* cnt_s, const uint64_t* vscan, int32_t w,
                int64_t* table, hipStream_t s) {
  hipLaunchKernelGGL(k_plan_table, dim3(1), dim3(64), 0, s, cnt_g, cnt_s, vscan, w, table);
  RT_OK(hipGetLastError());
}

void send_segments(const int64_t* cnt_g, const int64_t* cnt_s, const uint64_t* spad,
                   const uint64_t* sval, uint64_t gk_base, uint64_t srec_base, int32_t w,
                   int64_t ns, uint64_t* seg_len, uint64_t* seg_src, hipStream_t s) {
  hipLaunchKernelGGL(k_send_segs, dim3(grid1(ns + w)), dim3(kB), 2 * (w + 1) * sizeof(int64_t), s,
                     cnt_g, cnt_s, spad, sval, gk_base, srec_base, w, ns, seg_len, seg_src);
  RT_OK(hipGetLastError());
}

void recv_segments(const int64_t* rtable, uint64_t recv_base, int32_t w, uint64_t* seg_len,
                   uint64_t* seg_src, hipStream_t s) {
  hipLaunchKernelGGL(k_recv_segs, dim3(1), dim3(64), 0, s, rtable, recv_base, w, seg_len, seg_src);
  RT_OK(hipGetLastError());
}

void recv_sets(const int64_t* rrec, int64_t ms, const int64_t* rtable, int32_t w,
               uint64_t* rpad_ws, uint64_t* rscan_ws, void* scan_tmp, size_t scan_tmp_bytes,
               Digest* keys, uint32_t* vlen0, uint32_t* vlen1, uint32_t* flags, uint32_t* expire,
               uint64_t* roff, hipStream_t s) {
  if (ms <= 0) return;
  hipLaunchKernelGGL(k_rs_pad, dim3(grid1(ms + 1)), dim3(kB), 0, s, rrec, ms, rpad_ws);
  device_exclusive_scan(rpad_ws, rscan_ws, ms, scan_tmp, scan_tmp_bytes, s);
  hipLaunchKernelGGL(k_rs_fill, dim3(grid1(ms)), dim3(kB), (2 * w + 1) * sizeof(int64_t), s, rrec,
                     ms, rtable, w, rscan_ws, keys, vlen0, vlen1, flags, expire, roff);
  RT_OK(hipGetLastError());
}

void reply_bytes(const uint64_t* lk_off, const int64_t* rtable, const uint64_t* gscan,
                 const int64_t* table, int32_t w, int64_t* bytes, hipStream_t s) {
  hipLaunchKernelGGL(k_reply_bytes, dim3(1), dim3(64), 0, s, lk_off, rtable, gscan, table, w,
                     bytes);
  RT_OK(hipGetLastError());
}

void assemble_response(const int64_t* perm_g, int64_t n, int64_t n_remote,
                       const uint64_t* sizes_back, const uint64_t* gscan,
                       const uint64_t* rl_size, const uint64_t* rl_off, uint64_t local_bytes,
                       uint64_t* size, uint64_t* off, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_assemble, dim3(grid1(n)), dim3(kB), 0, s, perm_g, n, n_remote, sizes_back,
                     gscan, rl_size, rl_off, local_bytes, size, off);
  RT_OK(hipGetLastError());
}

}  // namespace shellac

// =====================================================================================
// RoutedStep
// =====================================================================================
namespace shellac {

namespace {
enum Slot {
  kRlLoc, kRlSize, kRlOff, kDestG, kGk, kPermG, kCntG, kWsG, kDestS, kOwnerS, kSrec, kSval,
  kSpad, kCntS, kWsS, kVscan, kExtras, kSegLen, kSegSrc, kSegOff, kBody, kRSegLen, kRSegSrc,
  kRSegOff, kLkLoc, kLkOff, kGin, kGscan, kNbytes, kRpad, kRscan, kRkeys, kV0, kV1, kFl, kEx,
  kRoff, kScanTmp, kNumSlots
};
}  // namespace

RoutedStep::RoutedStep(int world, int rank, int device)
    : w_(world), rank_(rank), device_(device), bufs_(kNumSlots) {
  SH_CHECK(world >= 1 && world < kMaxBuckets, "bad world size");
  RT_OK(hipSetDevice(device_));
  RT_OK(hipHostMalloc(&host_, (8 * (size_t)world + 8) * sizeof(int64_t), hipHostMallocDefault));
}

RoutedStep::~RoutedStep() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (auto& b : bufs_) (void)hipFree(b.p);
  (void)hipHostFree(host_);
}

void RoutedStep::set_ring(const uint32_t* pts, const int32_t* owner, int32_t npts) {
  pts_ = pts;
  own_ = owner;
  npts_ = npts;
}

void RoutedStep::set_hot(const Digest* hot, int64_t nhot) {
  hot_ = hot;
  nhot_ = hot ? nhot : 0;
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

uint64_t* RoutedStep::scan(uint64_t* in, uint64_t* out, int64_t n, hipStream_t s) {
  RT_OK(hipMemsetAsync(in + n, 0, sizeof(uint64_t), s));
  const size_t tb = device_scan_tmp_bytes(std::max<int64_t>(n, 1));
  uint8_t* tmp = buf<uint8_t>(kScanTmp, tb);
  device_exclusive_scan(in, out, n, tmp, bufs_[kScanTmp].cap, s);
  return out;
}

void RoutedStep::plan(const Digest* keys, int64_t n, HbmCache* replica, uint32_t now,
                      const Digest* skeys, const uint32_t* svlen, const uint32_t* sflags,
                      const uint32_t* sexpire, const uint64_t* sval_off, const uint8_t* svalues,
                      int64_t ns, bool fanout, int64_t* table, hipStream_t s) {
  SH_CHECK(pts_ && own_ && npts_ > 0, "RoutedStep: ring not set");
  const int W = w_;
  n_ = n;
  values_ = svalues;
  have_replica_ = replica != nullptr;
  table_ = table;
  uint64_t* rl_size = nullptr;
  if (replica) {
    rl_loc_ = buf<uint64_t>(kRlLoc, n);
    rl_size = rl_size_ = buf<uint64_t>(kRlSize, n + 1);
    rl_off_ = buf<uint64_t>(kRlOff, n + 1);
    replica->lookup(keys, n, rl_loc_, rl_size_, rl_off_, now, s);
  }
  int32_t* dest_g = buf<int32_t>(kDestG, n);
  route_gets(keys, n, rl_size, pts_, own_, npts_, W, dest_g, s);
  gk_ = buf<Digest>(kGk, n);
  perm_g_ = buf<int64_t>(kPermG, n);
  cnt_g_ = buf<int64_t>(kCntG, W + 1);
  group_rows(dest_g, n, W + 1, keys, 16, gk_, perm_g_, cnt_g_,
             buf<uint64_t>(kWsG, group_ws_words(std::max<int64_t>(n, 1), W + 1)), s);
  m_ = fanout ? ns * W : ns;
  srec_ = buf<int64_t>(kSrec, 4 * (size_t)m_);
  sval_ = buf<uint64_t>(kSval, m_);
  spad_ = buf<uint64_t>(kSpad, m_ + 1);
  cnt_s_ = buf<int64_t>(kCntS, W + 1);
  plan_sets(skeys, svlen, sflags, sexpire, sval_off, ns, (uint64_t)(uintptr_t)svalues, pts_, own_,
            npts_, fanout ? hot_ : nullptr, fanout ? nhot_ : 0, W, fanout,
            buf<int32_t>(kDestS, m_), buf<int32_t>(kOwnerS, ns),
            buf<uint64_t>(kWsS, group_ws_words(std::max<int64_t>(m_, 1), W + 1)), srec_, sval_,
            spad_, cnt_s_, s);
  uint64_t* vscan = scan(spad_, buf<uint64_t>(kVscan, m_ + 1), m_, s);
  plan_table(cnt_g_, cnt_s_, vscan, W, table, s);
  int64_t* extras = buf<int64_t>(kExtras, 2);
  RT_OK(hipMemcpyAsync(extras, cnt_g_ + W, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  if (replica)
    RT_OK(hipMemcpyAsync(extras + 1, rl_off_ + n, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  else
    RT_OK(hipMemsetAsync(extras + 1, 0, sizeof(int64_t), s));
}

std::vector<int64_t> RoutedStep::read_counts(const int64_t* rtable, hipStream_t s) {
  const int W = w_;
  rtable_ = rtable;
  RT_OK(hipMemcpyAsync(host_, table_, 3 * W * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  RT_OK(hipMemcpyAsync(host_ + 3 * W, rtable, 3 * W * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  RT_OK(hipMemcpyAsync(host_ + 6 * W, bufs_[kExtras].p, 2 * sizeof(int64_t),
                       hipMemcpyDeviceToHost, s));
  RT_OK(hipStreamSynchronize(s));
  std::vector<int64_t> out(host_, host_ + 6 * W + 2);
  n_local_ = out[6 * W];
  local_bytes_ = (uint64_t)out[6 * W + 1];
  n_remote_ = n_ - n_local_;
  ns_ = mg_ = ms_ = 0;
  for (int p = 0; p < W; ++p) {
    ns_ += out[3 * p + 1];
    mg_ += out[3 * W + 3 * p];
    ms_ += out[3 * W + 3 * p + 1];
  }
  return out;
}

void RoutedStep::pack(uint8_t* send, hipStream_t s) {
  const int64_t nseg = 2 * (int64_t)w_ + ns_;
  uint64_t* seg_len = buf<uint64_t>(kSegLen, nseg + 1);
  uint64_t* seg_src = buf<uint64_t>(kSegSrc, nseg);
  send_segments(cnt_g_, cnt_s_, spad_, sval_, (uint64_t)(uintptr_t)gk_,
                (uint64_t)(uintptr_t)srec_, w_, ns_, seg_len, seg_src, s);
  uint64_t* seg_off = scan(seg_len, buf<uint64_t>(kSegOff, nseg + 1), nseg, s);
  segcopy(nullptr, seg_src, seg_off, nseg, send, s);
}

void RoutedStep::owner(const uint8_t* recv, HbmCache* shard, uint32_t now, uint64_t* sizes_out,
                       hipStream_t s) {
  const int64_t W2 = 2 * (int64_t)w_;
  uint8_t* body = buf<uint8_t>(kBody, 16 * mg_ + 32 * ms_ + 16);
  uint64_t* rlen = buf<uint64_t>(kRSegLen, W2 + 1);
  uint64_t* rsrc = buf<uint64_t>(kRSegSrc, W2);
  recv_segments(rtable_, (uint64_t)(uintptr_t)recv, w_, rlen, rsrc, s);
  uint64_t* roff = scan(rlen, buf<uint64_t>(kRSegOff, W2 + 1), W2, s);
  segcopy(nullptr, rsrc, roff, W2, body, s);
  rrec_ = reinterpret_cast<const int64_t*>(body + 16 * mg_);
  lk_loc_ = buf<uint64_t>(kLkLoc, mg_);
  lk_off_ = buf<uint64_t>(kLkOff, mg_ + 1);
  shard->lookup(reinterpret_cast<const Digest*>(body), mg_, lk_loc_, sizes_out, lk_off_, now, s);
}

std::vector<int64_t> RoutedStep::reply_sizes(const uint64_t* sizes_in, hipStream_t s) {
  const int W = w_;
  sizes_in_ = sizes_in;
  uint64_t* gin = buf<uint64_t>(kGin, n_remote_ + 1);
  if (n_remote_ > 0)
    RT_OK(hipMemcpyAsync(gin, sizes_in, n_remote_ * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
  gscan_ = scan(gin, buf<uint64_t>(kGscan, n_remote_ + 1), n_remote_, s);
  int64_t* nb = buf<int64_t>(kNbytes, 2 * W);
  reply_bytes(lk_off_, rtable_, gscan_, table_, W, nb, s);
  RT_OK(hipMemcpyAsync(host_ + 6 * W + 2, nb, 2 * W * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  RT_OK(hipStreamSynchronize(s));
  return std::vector<int64_t>(host_ + 6 * W + 2, host_ + 8 * W + 2);
}

void RoutedStep::gather_replies(HbmCache* shard, uint8_t* reply, hipStream_t s) {
  if (mg_ > 0) shard->gather(lk_loc_, lk_off_, mg_, reply, s);
}

void RoutedStep::finish(uint8_t* data, const uint8_t* recv, int64_t recv_bytes, HbmCache* shard,
                        HbmCache* replica, uint32_t now, uint64_t* out_size, uint64_t* out_off,
                        hipStream_t s) {
  if (have_replica_ && replica && n_local_ > 0) replica->gather(rl_loc_, rl_off_, n_, data, s);
  if (ms_ > 0) {
    const int64_t ms = ms_;
    uint64_t* rpad = buf<uint64_t>(kRpad, ms + 1);
    uint64_t* rscan = buf<uint64_t>(kRscan, ms + 1);
    Digest* rkeys = buf<Digest>(kRkeys, ms);
    uint32_t* v0 = buf<uint32_t>(kV0, ms);
    uint32_t* v1 = buf<uint32_t>(kV1, ms);
    uint32_t* fl = buf<uint32_t>(kFl, ms);
    uint32_t* ex = buf<uint32_t>(kEx, ms);
    uint64_t* roff = buf<uint64_t>(kRoff, ms);
    uint8_t* tmp = buf<uint8_t>(kScanTmp, device_scan_tmp_bytes(ms));
    recv_sets(rrec_, ms, rtable_, w_, rpad, rscan, tmp, bufs_[kScanTmp].cap, rkeys, v0, v1, fl, ex,
              roff, s);
    const uint64_t bound = 48 * (uint64_t)ms + (uint64_t)recv_bytes;
    shard->store(rkeys, recv, roff, v0, fl, ex, ms, bound, now, s);
    if (replica) replica->store(rkeys, recv, roff, v1, fl, ex, ms, bound, now, s);
  }
  assemble_response(perm_g_, n_, n_remote_, sizes_in_, gscan_, have_replica_ ? rl_size_ : nullptr,
                    have_replica_ ? rl_off_ : nullptr, local_bytes_, out_size, out_off, s);
}

}  // namespace shellac
