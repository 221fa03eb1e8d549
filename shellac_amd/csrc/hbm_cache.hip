// HIP/CDNA4 kernels and host driver for the HBM cache shard (see hbm_cache.h).
//
// Kernel map (all wave64, 256-thread workgroups):
//   k_coalesce     GET request collapsing: each workgroup collapses a 1024-key chunk
//                  in an LDS table, its local claimers claim a global open-addressing
//                  table (a plain load, then one CAS where the slot is still free),
//                  and (PROBE) the global claimers are probed by 8-lane groups.
//   k_probe        8 lanes per key, digests staged in LDS, 3 keys in flight per
//                  group: the group reads the first bucket (one 128-B line) and only
//                  on a miss the second; pair-lane shuffles join the {digest} and
//                  {loc,vlen,expire} halves of each entry, max-reduce picks the
//                  newest live match. No dependent read of the value log.
//   k_segcopy      load-balanced byte mover: each workgroup owns a 64 KiB tile
//                  of the *output*, finds the segments covering it (block-wide
//                  128-ary search, then per-lane binary search of offsets staged
//                  in LDS) and every lane moves 16 x 16 B, so item-size skew
//                  never idles lanes. Used for GET gathers, SET log writes and
//                  packing SET payloads for the all-to-all.
//   k_set_dedupe   batch-local open-addressing table: the last SET of a key in a
//                  batch wins (request order = memcached/HTTP pipelining order).
//   k_set_copy     load-balanced writer of [ItemHeader|value] into the log at
//                  head + exclusive-scan(item sizes): batch allocation is a scan.
//   k_set_index    4 lanes per key: two-choice insert with a 64-bit CAS on the
//                  entry's loc word; replaces the key's own entry, else a dead
//                  slot in the emptier bucket, else evicts the oldest item;
//                  workgroup 0 publishes the new log head into the other of two
//                  ping-pong head slots, and every item resets its dedupe slot.
//   k_set_fixup    rewrites the digest words of entries a later insert of the same
//                  batch re-claimed (the CAS arbitrates loc only).
//   All per-op counters are block-reduced and added to one of 64 counter
//   shards (one atomic per block per field; same-address fan-in measured at
//   ~12 ns/atomic would otherwise serialise a 64K-wave probe into milliseconds).
//   k_expand(_out), k_small_get, k_delete, k_sweep, k_export, k_digest, k_route*,
//   k_permute, k_mfma_hello.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "hbm_cache.h"
#include "trace.h"

namespace shellac {

#define HIP_OK(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      throw Error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + #expr + \
                  " [" + __FILE__ + ":" + std::to_string(__LINE__) + "]");             \
  } while (0)

namespace {

constexpr int kBlock = 256;
constexpr int kTileSegCap = 1024;          // segments staged in LDS per tile
constexpr int kMaxGrid = 2048;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Tuned constants (round-2 sweeps, profiles/archive/r1_probe_grid_sweep.log,
// r1_segcopy_store_ab.log, r1_overlap_sweep.log; the A/B knobs are gone):
//  * k_probe / k_coalesce grids cap at kMaxGrid workgroups (halving the grid nearly
//    doubled a 1M-key probe: it is bound by random lines in flight);
//  * segcopy: 4 x 16-B loads in flight per lane, 8 waves/SIMD, nontemporal stores
//    (-3.5 % gather time against plain stores), a 16 KiB minimum tile, and 48/64 of the
//    co-resident slots so a concurrent SET chain gets CUs (a gather at 3/4 of the slots is
//    as fast as at all of them: memory-bound).
constexpr int kSegMinTile = 1024;  // 16-B chunks
constexpr int kSegOcc64 = 48;

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

inline int grid_for(int64_t work_items, int per_block, int cap = 8192) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
  for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s);
  return v;
}

constexpr int kCtrShards = 64;  // counters spread over 64 cache lines (no same-address fan-in)

// Block-wide sum of up to 3 per-thread counters, then ONE atomic per field per
// block into this block's counter shard. Every thread of the block must call it.
__device__ __forceinline__ void block_count(CacheCounters* shards, unsigned long long a,
                                            unsigned long long CacheCounters::*fa,
                                            unsigned long long b = 0,
                                            unsigned long long CacheCounters::*fb = nullptr,
                                            unsigned long long c = 0,
                                            unsigned long long CacheCounters::*fc = nullptr) {
  __shared__ unsigned long long s_red[3][kBlock / 64];
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_red[0][w] = a;
    s_red[1][w] = b;
    s_red[2][w] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t0 = 0, t1 = 0, t2 = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
      t0 += s_red[0][k];
      t1 += s_red[1][k];
      t2 += s_red[2][k];
    }
    CacheCounters* c_ = shards + (blockIdx.x & (kCtrShards - 1));
    if (t0) atomicAdd(&(c_->*fa), t0);
    if (fb && t1) atomicAdd(&(c_->*fb), t1);
    if (fc && t2) atomicAdd(&(c_->*fc), t2);
  }
  __syncthreads();  // s_red may be reused by a following call
}

// Block-wide sum of v written to part[blockIdx.x] (every thread must call it).
__device__ __forceinline__ void block_partial(unsigned long long v, uint64_t* __restrict__ part) {
  __shared__ unsigned long long s_p[kBlock / 64];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_p[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) t += s_p[k];
    part[blockIdx.x] = t;
  }
  __syncthreads();  // s_p may be reused by a following call
}

// ---- decoupled look-back (single-pass scans across workgroups) -------------------------
// Workgroups are dispatched in blockIdx order, so when workgroup b waits for b-1's word,
// b-1 is resident or done: the chain always completes. The state words are reset by the
// launch's last workgroup (self-cleaning, no memset between launches).
constexpr unsigned long long kLbAgg = 1ull << 62;    // look-back state: aggregate ready
constexpr unsigned long long kLbIncl = 2ull << 62;   // inclusive prefix ready
constexpr unsigned long long kLbVal = (1ull << 62) - 1;
constexpr uint32_t kLbSpinLimit = 1u << 22;          // a predecessor that never publishes

// Wave 0 (all 64 lanes): publish this workgroup's aggregate, return the sum of every
// earlier workgroup's (exclusive prefix). The wave reads 64 predecessors' words per step
// (lane l -> workgroup b-1-l) and stops at the nearest inclusive prefix: a walk over
// thousands of aggregate-only predecessors is then a few dependent loads, not one per
// predecessor (one lane at a time made a 1024-group coalescing probe 2x slower).
// *fail on a predecessor that never published.
__device__ __forceinline__ unsigned long long lookback_exclusive(unsigned long long* state,
                                                                unsigned long long agg,
                                                                int* fail) {
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0) {
    if (lane == 0)
      __hip_atomic_store(state, kLbIncl | agg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0)
    __hip_atomic_store(state + blockIdx.x, kLbAgg | agg, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long base = 0;
  int64_t end = (int64_t)blockIdx.x;  // window: workgroups [end-64, end)
  uint32_t spins = 0;
  for (;;) {
    const int64_t p = end - 1 - lane;
    const unsigned long long st =
        p >= 0 ? __hip_atomic_load(state + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
               : kLbIncl;  // before workgroup 0: an inclusive zero
    const unsigned long long incl = __ballot((st & kLbIncl) != 0);
    const int stop = incl ? __ffsll((long long)incl) - 1 : 63;  // last lane that counts
    const unsigned long long notready = __ballot(st == 0);
    const unsigned long long need = stop == 63 ? ~0ull : ((2ull << stop) - 1ull);
    if (notready & need) {
      if (++spins > kLbSpinLimit) {
        if (lane == 0) *fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    unsigned long long v = lane <= stop ? (st & kLbVal) : 0ull;
    base += wave_sum(v);
    if (incl) break;
    end -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(state + blockIdx.x, kLbIncl | (base + agg), __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_AGENT);
  return base;
}

// Every thread: the launch's last workgroup to get here clears the look-back words.
__device__ __forceinline__ void lookback_done(unsigned long long* state, unsigned int* done) {
  __shared__ int s_last_lb;
  __syncthreads();
  if (threadIdx.x == 0) s_last_lb = atomicAdd(done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (s_last_lb) {
    for (unsigned k = threadIdx.x; k < gridDim.x; k += kBlock) state[k] = 0ull;
    if (threadIdx.x == 0) atomicExch(done, 0u);
  }
}

// Items per workgroup when n items are split into contiguous ranges over `grid` groups.
__host__ __device__ __forceinline__ int64_t part_len(int64_t n, int grid) {
  return (n + grid - 1) / grid;
}

// Second half of a two-kernel exclusive scan whose first half is fused into the
// producer (k_probe / k_set_size write one partial sum per workgroup over contiguous
// ranges of `plen` items). Workgroup b covers producer groups [b*q, (b+1)*q): it sums
// the partials before its range, then each wave scans a contiguous quarter of the range,
// 64 items per step.
// off[n] = total. Replaces hipcub's init + scan pair (one launch, no lookback state).
// `part_cnt` / `cnt` (optional): the same scan over (size[i] != 0), i.e. each item's
// ordinal among the non-empty ones (the CLOCK ring's entry per stored SET row).
__global__ __launch_bounds__(kBlock) void k_offsets(const uint64_t* __restrict__ size, int64_t n,
                                                    const uint64_t* __restrict__ part, int nparts,
                                                    int64_t plen, int q,
                                                    uint64_t* __restrict__ off,
                                                    uint64_t* __restrict__ host_total,
                                                    const uint64_t* __restrict__ part_cnt,
                                                    uint64_t* __restrict__ cnt,
                                                    const uint64_t* __restrict__ claim_head,
                                                    unsigned long long* __restrict__ claim) {
  __shared__ unsigned long long s_w[2][kBlock / 64];
  __shared__ unsigned long long s_base[2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int p0 = blockIdx.x * q;
  unsigned long long pre = 0, prec = 0;
  for (int k = threadIdx.x; k < p0 && k < nparts; k += kBlock) {
    pre += part[k];
    if (cnt) prec += part_cnt[k];
  }
  pre = wave_sum(pre);
  prec = wave_sum(prec);
  if (lane == 0) {
    s_w[0][w] = pre;
    s_w[1][w] = prec;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    unsigned long long t = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) t += s_w[threadIdx.x][k];
    s_base[threadIdx.x] = t;
  }
  __syncthreads();
  const int64_t i0 = (int64_t)p0 * plen;
  const int64_t i1 = min(n, (int64_t)(p0 + q) * plen);
  // Wave w scans the contiguous sub-range [a, b) of the workgroup's range, 64 items per
  // step with coalesced loads and stores (one lane per item, a shuffle scan per step).
  // Pass 1 sums each wave's sub-range so every wave knows its base; pass 2 re-reads it
  // (from cache) and scans. (Lane-contiguous runs of `per` items made every load and
  // store instruction touch 64 different lines: 27 us per 1M items beside the SET append,
  // now 20 us. The step did not move, 0.319-0.321 vs 0.320-0.323 ms over three rounds
  // (profiles/archive/r2_offsets_ab.log): the gather then starts earlier into the SET append.)
  // Up to kOffRegs x 64 items per wave (the lookup's 1M rows: 512) are loaded once, all
  // in flight together, and scanned from registers: the two dependent passes of 64 items
  // per step were latency-bound, 20-28 us per 1M rows between the lookup and the gather.
  const int64_t len = i1 > i0 ? i1 - i0 : 0;
  const int64_t per = ((len + kBlock / 64 - 1) / (kBlock / 64) + 63) / 64 * 64;
  const int64_t a = min(i1, i0 + per * w), b = min(i1, a + per);
  constexpr int kOffRegs = 8;
  const bool in_regs = per <= 64 * kOffRegs;  // uniform across the launch
  uint64_t rv[kOffRegs];
  unsigned long long ws = 0, wc = 0;
  if (in_regs) {
#pragma unroll
    for (int u = 0; u < kOffRegs; ++u) {
      const int64_t i = a + u * 64 + lane;
      rv[u] = i < b ? size[i] : 0;
      ws += rv[u];
      wc += rv[u] ? 1 : 0;
    }
  } else {
    for (int64_t i = a + lane; i < b; i += 64) {
      const uint64_t v = size[i];
      ws += v;
      wc += v ? 1 : 0;
    }
  }
  ws = wave_sum(ws);
  wc = wave_sum(wc);
  __syncthreads();  // s_w is reused
  if (lane == 0) {
    s_w[0][w] = ws;
    s_w[1][w] = wc;
  }
  __syncthreads();
  unsigned long long run = s_base[0], runc = s_base[1];
  for (int k = 0; k < w; ++k) {
    run += s_w[0][k];
    runc += s_w[1][k];
  }
  if (in_regs) {
#pragma unroll
    for (int u = 0; u < kOffRegs; ++u) {
      const int64_t i = a + u * 64 + lane;
      const uint64_t v = rv[u];
      const unsigned long long c = v ? 1 : 0;
      unsigned long long inc = v, incc = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long o = __shfl_up(inc, d);
        const unsigned long long oc = __shfl_up(incc, d);
        if (lane >= d) {
          inc += o;
          incc += oc;
        }
      }
      if (i < b) {
        off[i] = run + inc - v;
        if (cnt) cnt[i] = runc + incc - c;
      }
      run += __shfl(inc, 63);
      runc += __shfl(incc, 63);
    }
  }
  for (int64_t t = a; !in_regs && t < b; t += 64) {
    const int64_t i = t + lane;
    const uint64_t v = i < b ? size[i] : 0;
    const unsigned long long c = v ? 1 : 0;
    unsigned long long inc = v, incc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long o = __shfl_up(inc, d);
      const unsigned long long oc = __shfl_up(incc, d);
      if (lane >= d) {
        inc += o;
        incc += oc;
      }
    }
    if (i < b) {
      off[i] = run + inc - v;
      if (cnt) cnt[i] = runc + incc - c;
    }
    run += __shfl(inc, 63);
    runc += __shfl(incc, 63);
  }
  if (i1 == n && threadIdx.x == 0) {  // every workgroup whose range ends at n: the total
    unsigned long long tot = s_base[0], totc = s_base[1];
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
      tot += s_w[0][k];
      totc += s_w[1][k];
    }
    off[n] = tot;
    if (cnt) cnt[n] = totc;
    if (host_total)
      __hip_atomic_store(host_total, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // a SET batch's sizes: claim the log bytes its append will write before the append
    // kernel starts (the edge server re-checks its copies against this word)
    if (claim) atomicMax(claim, (unsigned long long)(*claim_head + tot));
  }
}

__device__ __forceinline__ uint64_t pack2(uint32_t lo, uint32_t hi) {
  return ((uint64_t)hi << 32) | lo;
}

constexpr int kCoProbe = 3;   // keys an 8-lane group of k_probe probes concurrently (loads in flight)
constexpr int kProbeTile = 512;  // digests k_probe stages in LDS at a time

// One 8-lane group's match of digest `d` against the bucket quarter-entry `v` its lane
// l8 loaded: pair-lane shuffles join entry halves, max-reduce keeps the newest live
// match. hl = stored loc (0: none), hv = its raw vlen word (kRefBit included), he = its
// entry within the bucket; uniform in the group.
__device__ __forceinline__ void group_match(const uint4 v, const Digest& d, int l8,
                                            uint64_t head, uint64_t cap, uint32_t now,
                                            uint64_t* hl_out, uint32_t* hv_out,
                                            int* he_out = nullptr) {
  const uint64_t a = pack2(v.x, v.y);   // even lane: d0   | odd lane: loc
  const uint64_t c = pack2(v.z, v.w);   // even lane: d1   | odd lane: vlen | expire<<32
  const uint64_t pa = __shfl_xor(a, 1);
  const uint64_t pc = __shfl_xor(c, 1);
  const bool hit = (l8 & 1) == 0 && a == d.lo && c == d.hi &&
                   entry_live(pa, (uint32_t)(pc >> 32), head, cap, now);
  uint64_t hl = hit ? pa : 0;
  uint32_t hv = hit ? (uint32_t)pc : 0;
  int he = l8 >> 1;
#pragma unroll
  for (int sh = 2; sh < 8; sh <<= 1) {
    const uint64_t ol = __shfl_xor(hl, sh);
    const uint32_t ov = __shfl_xor(hv, sh);
    const int oe = __shfl_xor(he, sh);
    if (ol > hl) { hl = ol; hv = ov; he = oe; }
  }
  *hl_out = hl;
  *hv_out = hv;
  if (he_out) *he_out = he;
}

// CLOCK reference: a hit on an entry whose bit is clear sets it (one atomic the first
// time an object is read per hand lap; hot objects already carry the bit, so a Zipf
// probe stream almost never writes).
__device__ __forceinline__ void mark_ref(Entry* index, uint64_t bucket, int e, uint32_t hv) {
  if (!(hv & kRefBit)) atomicOr(&index[bucket * kEntriesPerBucket + e].vlen, kRefBit);
}

// ---------------------------------------------------------------------------------
// GET: probe
// ---------------------------------------------------------------------------------
// One 8-lane group per key: the group reads the key's first bucket (128 B, 16 B per
// lane; even lanes hold digests, odd lanes loc/vlen/expire) and only on a miss its
// second bucket. SETs fill the first bucket first, so a hit usually costs one line.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_probe(const Digest* __restrict__ keys, int64_t n,
                                                  Entry* __restrict__ index, uint64_t mask,
                                                  const uint64_t* __restrict__ head_ptr,
                                                  uint64_t reserve, uint64_t cap, uint32_t now,
                                                  uint64_t* __restrict__ out_loc,
                                                  uint64_t* __restrict__ out_size,
                                                  CacheCounters* __restrict__ ctr,
                                                  uint64_t* __restrict__ part,
                                                  const uint32_t* __restrict__ first,
                                                  int64_t slot_rows,
                                                  const int64_t* __restrict__ slot_cnt,
                                                  const uint64_t* __restrict__ reserve_dev) {
  const int l8 = threadIdx.x & 7;
  // `reserve` (+ *reserve_dev, a device-computed bound): bytes about to be appended
  // before this lookup's gather runs; objects that those appends will overwrite are
  // already treated as evicted
  const uint64_t head = *head_ptr + reserve + (reserve_dev ? *reserve_dev : 0ull);
  unsigned long long hits = 0, bytes = 0, ops = 0, psum = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) out_size[n] = 0;
  // contiguous key range per workgroup (k_offsets scans it from the partial sums)
  const int64_t plen = part_len(n, gridDim.x);
  const int64_t i1 = min(n, (int64_t)(blockIdx.x + 1) * plen);
  // The range is probed in tiles staged through LDS: one coalesced pass loads the
  // tile's digests (and coalescing flags), so the only dependent global access per key
  // is its bucket line. Each 8-lane group keeps kCoProbe bucket loads in flight (a probe
  // is latency-bound: measured 65 us per 1M keys whether 1M or 300K of them probed,
  // when every key also waited for its own digest load).
  __shared__ Digest s_k[kProbeTile];
  __shared__ uint8_t s_go[kProbeTile];
  constexpr int kG = kBlock / 8;
  for (int64_t t0 = (int64_t)blockIdx.x * plen; t0 < i1; t0 += kProbeTile) {
    const int cnt = (int)min((int64_t)kProbeTile, i1 - t0);
    for (int k = threadIdx.x; k < cnt; k += kBlock) {
      s_k[k] = keys[t0 + k];
      const int64_t i = t0 + k;
      // duplicates skip; in a slotted batch (slot_cnt) rows past their slot's count are
      // padding and skip too (answered as misses, not counted)
      s_go[k] = (!first || first[i] == (uint32_t)i) &&
                (!slot_cnt || i % slot_rows < slot_cnt[i / slot_rows]);
    }
    __syncthreads();
    for (int q0 = threadIdx.x >> 3; q0 < cnt; q0 += kG * kCoProbe) {
      uint4 vb[kCoProbe];
#pragma unroll
      for (int p = 0; p < kCoProbe; ++p) {
        const int q = q0 + p * kG;  // uniform in the 8-lane group
        if (q < cnt && s_go[q])
          vb[p] = reinterpret_cast<const uint4*>(index + bucket1(s_k[q], mask) * kEntriesPerBucket)[l8];
      }
#pragma unroll
      for (int p = 0; p < kCoProbe; ++p) {
        const int q = q0 + p * kG;
        if (q >= cnt) continue;
        const int64_t i = t0 + q;
        if (!s_go[q]) {  // coalesced duplicate: served from its first row
          if (l8 == 0) {
            out_loc[i] = kMissLoc;
            out_size[i] = 0;
          }
          continue;
        }
        const Digest d = s_k[q];
        uint64_t hl;
        uint32_t hv;
        int he;
        uint64_t hb = bucket1(d, mask);
        group_match(vb[p], d, l8, head, cap, now, &hl, &hv, &he);
        if (hl == 0) {  // second bucket only on a miss in the first (uniform in the group)
          hb = bucket2(d, mask);
          const uint4 v2 = reinterpret_cast<const uint4*>(index + hb * kEntriesPerBucket)[l8];
          group_match(v2, d, l8, head, cap, now, &hl, &hv, &he);
        }
        if (l8 == 0) {
          ++ops;
          if (hl) {
            mark_ref(index, hb, he, hv);
            hv = entry_vlen(hv);
            out_loc[i] = (hl - 1) % cap;
            out_size[i] = item_bytes(hv);
            ++hits;
            bytes += hv;
            psum += item_bytes(hv);
          } else {
            out_loc[i] = kMissLoc;
            out_size[i] = 0;
          }
        }
      }
    }
    __syncthreads();  // the tile's LDS is reused
  }
  block_count(ctr, ops, &CacheCounters::get_ops, hits, &CacheCounters::get_hits, bytes,
              &CacheCounters::get_bytes);
  block_partial(psum, part);
}

// ---------------------------------------------------------------------------------
// GET coalescing (request collapsing inside a batch)
// ---------------------------------------------------------------------------------
// A Zipf request batch repeats its hot keys many times (1M Zipf(0.99) requests over 4M
// objects hold ~1/3 distinct keys). first[i] = the row that serves row i: one row per
// distinct digest claims a slot of an open-addressing table (u32 row+1, linear probing,
// <= 50 % load) with one CAS; every other row of that digest finds the claim and points
// at it. The probe and the gather then touch only claiming rows, and k_expand gives
// each duplicate its claimer's (off, size) afterwards: duplicates share one record in
// the response buffer, as a proxy hands one cached object to many clients.
// Contention: a hot key repeats ~60K times in a 1M batch, and a same-address atomic
// costs ~12 ns serialised, so one global CAS per request spent ~0.3 ms on the hottest
// key alone (measured: 330 us per 1M-key batch). Each workgroup therefore first
// collapses its own chunk of 1024 keys in an LDS table, and only its local claimers go
// to the global table: a key's global atomics are bounded by the number of chunks.
// Every local claimer reads the global slot before it CASes: the ~780K claims of a 1M
// Zipf batch are bound by the memory-side atomics' throughput, and a slot another chunk
// already took costs a load instead of an atomic (round 5 read first only for keys repeated
// in the chunk; reading first for all took the lookup from 101.7 to 97.1 us).
// PROBE: the global claimer of a digest also probes the shard's index for it (one lane
// reads the 128-B bucket), so coalescing and lookup are one pass over the batch, and
// the workgroup's contiguous row range yields the partial sums k_offsets scans.
constexpr int kCoPer = 4;                   // keys per thread per chunk
constexpr int kCoKeys = kBlock * kCoPer;    // keys per chunk
constexpr int kCoSlots = 2 * kCoKeys;       // LDS table slots (<= 50 % load)

// 4 waves per SIMD (<= 128 VGPRs): the 1024-key chunks of a 1M batch (1024 workgroups)
// are all resident at once (4 per CU, 33 KB LDS each) — at 130 VGPRs (3 waves) a
// quarter of them ran as a second round (151 vs 95 us)
template <bool PROBE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_coalesce(
    const Digest* __restrict__ keys, int64_t n, int64_t plen, uint32_t* __restrict__ tab,
    uint32_t tmask, uint32_t* __restrict__ first, uint32_t* __restrict__ cslot,
    Entry* __restrict__ index, uint64_t mask, const uint64_t* __restrict__ head_ptr,
    uint64_t reserve, uint64_t cap, uint32_t now, uint64_t* __restrict__ out_loc,
    uint64_t* __restrict__ out_size, CacheCounters* __restrict__ ctr,
    uint64_t* __restrict__ part, int local_only, uint64_t* __restrict__ woff) {
  __shared__ Digest s_k[kCoKeys];       // the chunk's digests (LDS compares, probe input)
  // woff (PROBE, optional): each row's exclusive offset within this workgroup's rows (the
  // gather adds the prefix of the workgroup totals, k_block_prefix): the chunk's sizes are
  // kept in s_tab (free after the local claims) and scanned at the end of the chunk
  __shared__ unsigned long long s_wt[kBlock / 64], s_run;
  if (threadIdx.x == 0) s_run = 0;
  __shared__ uint32_t s_tab[kCoSlots];  // local row + 1
  __shared__ uint32_t s_rep[kCoKeys];   // global claimer of each local claimer
  __shared__ uint32_t s_dup[kCoKeys];   // local duplicates of each local claimer
  __shared__ uint32_t s_q[PROBE ? kCoKeys : 1];   // rows this chunk probes
  __shared__ int s_qn;
  const uint64_t head = PROBE ? *head_ptr + reserve : 0;
  const int l8 = threadIdx.x & 7;
  unsigned long long ops = 0, hits = 0, bytes = 0, psum = 0, dups = 0;
  const int64_t r0 = (int64_t)blockIdx.x * plen, r1 = min(n, r0 + plen);
  for (int64_t base = r0; base < r1; base += kCoKeys) {
    const int cnt = (int)min((int64_t)kCoKeys, r1 - base);
    for (int k = threadIdx.x; k < kCoSlots; k += kBlock) s_tab[k] = 0;
    for (int k = threadIdx.x; k < kCoKeys; k += kBlock) s_dup[k] = 0;
    if (threadIdx.x == 0) s_qn = 0;
    Digest dk[kCoPer];
    uint32_t lrep[kCoPer];
    // 0. stage the chunk (rows strided by kBlock: coalesced 16-B loads)
#pragma unroll
    for (int u = 0; u < kCoPer; ++u) {
      const int j = u * kBlock + threadIdx.x;
      lrep[u] = (uint32_t)j;
      if (j < cnt) {
        dk[u] = keys[base + j];
        s_k[j] = dk[u];
      }
    }
    __syncthreads();
    // 1. local claims in LDS
#pragma unroll
    for (int u = 0; u < kCoPer; ++u) {
      const int j = u * kBlock + threadIdx.x;
      if (j >= cnt) continue;
      const Digest d = dk[u];
      uint32_t h = (uint32_t)d.lo & (kCoSlots - 1);
      for (int step = 0; step < kCoSlots; ++step) {
        const uint32_t v = atomicCAS(&s_tab[h], 0u, (uint32_t)j + 1u);
        if (v == 0) break;
        const Digest o = s_k[v - 1];
        if (o.lo == d.lo && o.hi == d.hi) {
          lrep[u] = v - 1;
          atomicAdd(&s_dup[v - 1], 1u);
          break;
        }
        h = (h + 1) & (kCoSlots - 1);
      }
    }
    __syncthreads();
    // 2. local claimers claim globally; global claimers queue for the probe. The first
    //    attempt of all kCoPer rows is issued back to back (independent loads / CASes in
    //    flight together), then each row resolves; a probed chain (slot held by another
    //    digest) continues one row at a time. local_only: chunk-local collapsing only
    //    (no global atomics; a digest repeated across chunks is probed and copied once
    //    per chunk — still exact results).
    {
      bool act[kCoPer];
      uint32_t hh[kCoPer], vv[kCoPer];
#pragma unroll
      for (int u = 0; u < kCoPer; ++u) {
        const int j = u * kBlock + threadIdx.x;
        act[u] = !local_only && j < cnt && lrep[u] == (uint32_t)j;
        hh[u] = (uint32_t)(dk[u].hi ^ (dk[u].hi >> 29)) & tmask;
        // read before the CAS: a slot another chunk's claimer already holds needs no atomic
        // (the global claims are bound by the memory-side atomics' throughput: ~52 of the
        // lookup's ~100 us; reading first took the lookup from 101.7 to 97.1 us,
        // profiles/archive/r6_fused_gather_rejected/README.md)
        vv[u] = act[u] ? __hip_atomic_load(tab + hh[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0u;
      }
#pragma unroll
      for (int u = 0; u < kCoPer; ++u)
        if (act[u] && vv[u] == 0)
          vv[u] = atomicCAS(tab + hh[u], 0u, (uint32_t)(base + u * kBlock + threadIdx.x) + 1u);
      Digest oo[kCoPer];
#pragma unroll
      for (int u = 0; u < kCoPer; ++u)
        if (act[u] && vv[u] != 0) oo[u] = keys[vv[u] - 1];
#pragma unroll
      for (int u = 0; u < kCoPer; ++u) {
        const int j = u * kBlock + threadIdx.x;
        if (j >= cnt || lrep[u] != (uint32_t)j) continue;
        const Digest d = dk[u];
        const uint32_t i = (uint32_t)(base + j);
        uint32_t rep = i, h = hh[u];
        if (act[u] && vv[u] != 0) {
          if (oo[u].lo == d.lo && oo[u].hi == d.hi) {
            rep = vv[u] - 1;
          } else {  // collision with another digest: linear probing, one row at a time
            for (uint32_t step = 0; step < tmask; ++step) {
              h = (h + 1) & tmask;
              uint32_t v = __hip_atomic_load(tab + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (v == 0) {
                v = atomicCAS(tab + h, 0u, i + 1u);
                if (v == 0) break;  // claimed
              }
              const Digest o = keys[v - 1];
              if (o.lo == d.lo && o.hi == d.hi) {
                rep = v - 1;
                break;
              }
            }
          }
        }
        s_rep[j] = rep;
        if (rep == i) {
          if (cslot) cslot[i] = local_only ? 0u : h;  // k_expand_out clears it
          if (PROBE) s_q[atomicAdd(&s_qn, 1)] = (uint32_t)j;
        }
      }
    }
    __syncthreads();
    if (PROBE) {
      // 2b. probe the queued digests, one 8-lane group per digest (each lane one 16-B
      //     quarter-entry of the 128-B bucket, as k_probe), kCoProbe digests per group
      //     in flight; results go straight to out_loc / out_size
      const int qn = s_qn;
      constexpr int kG = kBlock / 8;
      for (int q0 = threadIdx.x >> 3; q0 < qn; q0 += kG * kCoProbe) {
        uint4 vb[kCoProbe];
#pragma unroll
        for (int p = 0; p < kCoProbe; ++p) {
          const int q = q0 + p * kG;  // uniform in the 8-lane group
          if (q < qn)
            vb[p] = reinterpret_cast<const uint4*>(
                index + bucket1(s_k[s_q[q]], mask) * kEntriesPerBucket)[l8];
        }
#pragma unroll
        for (int p = 0; p < kCoProbe; ++p) {
          const int q = q0 + p * kG;
          if (q >= qn) continue;
          const int j = (int)s_q[q];
          const Digest d = s_k[j];
          uint64_t hl;
          uint32_t hv;
          int he;
          uint64_t hb = bucket1(d, mask);
          group_match(vb[p], d, l8, head, cap, now, &hl, &hv, &he);
          if (hl == 0) {  // second bucket only on a miss in the first (uniform in the group)
            hb = bucket2(d, mask);
            const uint4 v2 = reinterpret_cast<const uint4*>(index + hb * kEntriesPerBucket)[l8];
            group_match(v2, d, l8, head, cap, now, &hl, &hv, &he);
          }
          if (l8 == 0) {
            if (hl) mark_ref(index, hb, he, hv);
            hv = entry_vlen(hv);
            ++ops;
            out_loc[base + j] = hl ? (hl - 1) % cap : kMissLoc;
            out_size[base + j] = hl ? item_bytes(hv) : 0;
            if (woff) s_tab[j] = hl ? (uint32_t)item_bytes(hv) : 0u;
            if (hl) {
              ++hits;
              bytes += hv;
              psum += item_bytes(hv);
            }
          }
        }
      }
    }
    // 3. every row takes its local claimer's global claimer; non-claimers are empty
#pragma unroll
    for (int u = 0; u < kCoPer; ++u) {
      const int j = u * kBlock + threadIdx.x;
      if (j >= cnt) continue;
      const uint32_t f = s_rep[lrep[u]];
      first[base + j] = f;
      if (PROBE && f != (uint32_t)(base + j)) {
        out_loc[base + j] = kMissLoc;
        out_size[base + j] = 0;
        if (woff) s_tab[j] = 0u;
        ++dups;
      }
    }
    __syncthreads();  // LDS is reused by the next chunk
    if (PROBE && woff) {
      // the chunk's exclusive offsets from its sizes (kCoPer consecutive rows per thread)
      const int t4 = threadIdx.x * kCoPer;
      uint32_t v[kCoPer];
      unsigned long long ts = 0;
#pragma unroll
      for (int u = 0; u < kCoPer; ++u) {
        v[u] = t4 + u < cnt ? s_tab[t4 + u] : 0u;
        ts += v[u];
      }
      const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
      unsigned long long inc = ts;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long o = __shfl_up(inc, d);
        if (lane >= d) inc += o;
      }
      if (lane == 63) s_wt[wv] = inc;
      __syncthreads();
      unsigned long long ex = s_run + inc - ts, tot = 0;
#pragma unroll
      for (int k = 0; k < kBlock / 64; ++k) {
        if (k < wv) ex += s_wt[k];
        tot += s_wt[k];
      }
#pragma unroll
      for (int u = 0; u < kCoPer; ++u) {
        if (t4 + u < cnt) woff[base + t4 + u] = ex;
        ex += v[u];
      }
      __syncthreads();  // s_run and s_wt read by every thread
      if (threadIdx.x == 0) s_run += tot;
      // (the next chunk's first barrier orders s_run's update before its scan)
    }
  }
  if (PROBE) {
    if (blockIdx.x == 0 && threadIdx.x == 0) out_size[n] = 0;
    block_count(ctr, ops, &CacheCounters::get_ops, hits, &CacheCounters::get_hits, bytes,
                &CacheCounters::get_bytes);
    block_count(ctr, dups, &CacheCounters::get_coalesced);
    block_partial(psum, part);  // k_offsets scans the partials
  }
}

// The exclusive prefix of the coalescing lookup's per-workgroup totals (at most kMaxGrid):
// prefix[b] = bytes of workgroups < b, prefix[nparts] = the total, also published to the
// pinned host slot (the unsynced gather's size check). One workgroup; with the lookup's
// block-local offsets it replaces the 1M-row offsets scan (BlockedOff).
static_assert(HbmCache::kLookupPrefixWords == kMaxGrid + 1, "prefix words: kMaxGrid + 1");
__global__ __launch_bounds__(kBlock) void k_block_prefix(const uint64_t* __restrict__ part,
                                                         int nparts,
                                                         uint64_t* __restrict__ prefix,
                                                         uint64_t* __restrict__ host_total) {
  constexpr int kPer = kMaxGrid / kBlock;
  __shared__ unsigned long long s_w[kBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t v[kPer];
  unsigned long long ts = 0;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = threadIdx.x * kPer + u;
    v[u] = i < nparts ? part[i] : 0;
    ts += v[u];
  }
  unsigned long long inc = ts;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  unsigned long long ex = inc - ts;
  for (int k = 0; k < w; ++k) ex += s_w[k];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = threadIdx.x * kPer + u;
    if (i < nparts) prefix[i] = ex;
    ex += v[u];
  }
  if (threadIdx.x == kBlock - 1) {
    prefix[nparts] = ex;
    if (host_total)
      __hip_atomic_store(host_total, (uint64_t)ex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// In place: every duplicate row takes its claiming row's (size, off). Only claiming rows
// are read and only duplicate rows are written, so rows never race. Runs after the
// gather (which needs the scan in `off` intact).
__global__ __launch_bounds__(kBlock) void k_expand(const uint32_t* __restrict__ first, int64_t n,
                                                   uint64_t* __restrict__ size,
                                                   uint64_t* __restrict__ off) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const uint32_t f = first[i];
    if (f != (uint32_t)i) {
      size[i] = size[f];
      off[i] = off[f];
    }
  }
}

// Out of place (may run concurrently with the gather, which reads size/off): every row
// takes its claimer's (size, off) into out_size/out_off, and every claimer clears its
// slot of the coalescing table, so the next batch needs no table memset.
__global__ __launch_bounds__(kBlock) void k_expand_out(const uint32_t* __restrict__ first,
                                                       int64_t n,
                                                       const uint64_t* __restrict__ size,
                                                       const uint64_t* __restrict__ off,
                                                       uint64_t* __restrict__ out_size,
                                                       uint64_t* __restrict__ out_off,
                                                       uint32_t* __restrict__ tab,
                                                       const uint32_t* __restrict__ cslot) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const uint32_t f = first[i];
    out_size[i] = size[f];
    out_off[i] = off[f];
    if (f == (uint32_t)i && tab) tab[cslot[i]] = 0u;
  }
}

// ---------------------------------------------------------------------------------
// Load-balanced segmented copy
// ---------------------------------------------------------------------------------
// Last index j in [lo, hi) with off[j] <= x (off non-decreasing).
template <typename T>
__device__ __forceinline__ int64_t seg_search(const T* off, int64_t lo, int64_t hi, uint64_t x) {
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if ((uint64_t)off[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t seg_search_global(const uint64_t* off, int64_t n, uint64_t x) {
  // last j in [0, n) with off[j] <= x
  int64_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (off[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

// Segment offsets of a byte mover: a plain array, or (Blocked) the coalescing lookup's
// block-local offsets plus the exclusive prefix of its per-workgroup totals — off(j) =
// prefix[j >> shift] + local[j] for j < n, the total for j >= n (no 1M-row scan between
// the lookup and the gather: k_block_prefix scans only the workgroup totals).
struct PlainOff {
  const uint64_t* __restrict__ p;
  __device__ __forceinline__ uint64_t operator[](int64_t j) const { return p[j]; }
};
struct BlockedOff {
  const uint64_t* __restrict__ local;
  const uint64_t* __restrict__ prefix;
  int64_t n;
  int shift;
  __device__ __forceinline__ uint64_t operator[](int64_t j) const {
    return j < n ? prefix[j >> shift] + local[j] : prefix[((n - 1) >> shift) + 1];
  }
};

// Cooperative search: each half of the block (128 lanes) finds, for its own x,
// the last j in [0, n1) with off[j] <= x by 128-ary narrowing (one load per lane
// per round, ~3 rounds for 10^6 segments) instead of one lane's ~20 dependent
// loads. Every thread of the block must call it; results land in s_res[0..1].
template <typename Off>
__device__ __forceinline__ void block_find2(const Off off, int64_t n1,
                                            uint64_t x0, uint64_t x1, int64_t* s_lo,
                                            int64_t* s_hi, int* s_cnt) {
  const int h = threadIdx.x >> 7, t = threadIdx.x & 127, w = threadIdx.x >> 6;
  const uint64_t x = h ? x1 : x0;
  if (threadIdx.x < 2) {
    s_lo[threadIdx.x] = 0;
    s_hi[threadIdx.x] = n1;
  }
  __syncthreads();
  for (int round = 0; round < 16; ++round) {
    const int64_t lo = s_lo[h], hi = s_hi[h];
    const bool done = (s_hi[0] - s_lo[0] <= 1) && (s_hi[1] - s_lo[1] <= 1);
    if (done) break;  // uniform: every thread read the same LDS words
    const int64_t len = hi - lo;
    // probe p_t = lo + ceil(len*(t+1)/128) for t < 127 (p_t in (lo, hi))
    bool ok = false;
    if (len > 1 && t < 127) {
      const int64_t p = lo + (len * (t + 1) + 127) / 128;
      ok = p < hi && off[p] <= x;
    }
    const unsigned long long b = __ballot(ok);
    __syncthreads();  // all lanes have read s_lo/s_hi of this round
    if ((threadIdx.x & 63) == 0) s_cnt[w] = __popcll(b);
    __syncthreads();
    if (t == 0 && len > 1) {
      const int k = s_cnt[2 * h] + s_cnt[2 * h + 1];  // probes 0..k-1 passed (monotone)
      const int64_t nlo = k > 0 ? lo + (len * k + 127) / 128 : lo;
      const int64_t nhi = k < 127 ? lo + (len * (k + 1) + 127) / 128 : hi;
      s_lo[h] = nlo;
      s_hi[h] = nhi < hi ? nhi : hi;
    }
    __syncthreads();
  }
}

// A value every lane holds equally, moved to scalar registers.
__device__ __forceinline__ int64_t uniform64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Last j in [lo, hi) with off[j] <= x, given off[lo] <= x (off non-decreasing), by the
// whole block in 256-ary narrowing rounds (one load per thread per round). Every thread of
// the block must call it; s_b (2 words) and s_cnt (kBlock / 64) are scratch in LDS.
template <typename Off>
__device__ __forceinline__ int64_t block_last_le(const Off off, int64_t lo,
                                                 int64_t hi, uint64_t x, int64_t* s_b,
                                                 int* s_cnt) {
  __syncthreads();  // s_b free
  if (threadIdx.x == 0) {
    s_b[0] = lo;
    s_b[1] = hi;
  }
  __syncthreads();
  for (;;) {
    const int64_t l = s_b[0], h = s_b[1];
    if (h - l <= 1) break;  // uniform: every thread read the same LDS words
    const int64_t len = h - l;
    bool ok = false;
    if (threadIdx.x < kBlock - 1) {
      const int64_t q = l + (len * (threadIdx.x + 1) + kBlock - 1) / kBlock;
      ok = q < h && off[q] <= x;
    }
    const unsigned long long b = __ballot(ok);
    __syncthreads();  // every thread has read s_b
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = __popcll(b);
    __syncthreads();
    if (threadIdx.x == 0) {
      int k = 0;
#pragma unroll
      for (int w = 0; w < kBlock / 64; ++w) k += s_cnt[w];  // probes 0..k-1 passed (monotone)
      const int64_t nlo = k > 0 ? l + (len * k + kBlock - 1) / kBlock : l;
      const int64_t nhi = k < kBlock - 1 ? l + (len * (k + 1) + kBlock - 1) / kBlock : h;
      s_b[0] = nlo;
      s_b[1] = nhi < h ? nhi : h;
    }
    __syncthreads();
  }
  return s_b[0];
}

// A coalesced GET's per-request answers, done by the gather's workgroups after their
// copies (a grid-stride tail, n = 0: none): row i takes its claimer's (size, off), and
// every claimer clears its slot of the coalescing table (k_expand_out's work, without a
// launch or a stream of its own).
struct ExpandTail {
  const uint32_t* first = nullptr;
  int64_t n = 0;
  const uint64_t* size = nullptr;
  const uint64_t* off = nullptr;
  uint64_t* out_size = nullptr;
  uint64_t* out_off = nullptr;
  uint32_t* tab = nullptr;
  const uint32_t* cslot = nullptr;
  const uint64_t* prefix = nullptr;  // non-null: `off` holds block-local offsets (BlockedOff)
  int shift = 0;
};
__device__ __forceinline__ void expand_tail(const ExpandTail& ex) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < ex.n;
       i += (int64_t)gridDim.x * kBlock) {
    const uint32_t f = ex.first[i];
    ex.out_size[i] = ex.size[f];
    ex.out_off[i] = ex.prefix ? ex.prefix[f >> ex.shift] + ex.off[f] : ex.off[f];
    if (f == (uint32_t)i && ex.tab) ex.tab[ex.cslot[i]] = 0u;
  }
}

// Mode 0 (gather/pack): chunk at byte x of segment j comes from src + src_off[j] + w;
// a segment whose src_off is kSegSkip is a gap (its bytes are left as they are).
// Mode 2 (sized gather): as mode 0, but segment j holds only seg_len[j] bytes (passed in
// the `head_ptr` slot) and is copied only when it ends within `cap`; the bytes between a
// segment's end and the next segment's start are left untouched (gaps, headers written
// by someone else), and segments past `cap` are dropped instead of the whole copy.
// Mode 4: mode 0 with BlockedOff segment offsets (`dst_off` block-local, ex.prefix/shift).
// Mode 3: mode 0 with the segment count read from the device word `head_ptr` points at
// (a plan whose segment list the GPU built: no host read of its length).
// Mode 1 (SET log write): w < 32 synthesises the ItemHeader, else value bytes from
// src + src_off[j] + (w - 32); destination = log + (base + dst_off[j]) % cap + w, where
// the batch is at most cap/2 so the modulo is one compare against the wrap point.
// The grid is exactly the number of co-resident workgroups; workgroup b owns the
// contiguous destination range [b*span, (b+1)*span), so every workgroup moves the same
// bytes in one pass (no tail round). One cooperative search finds the segments holding
// the range's first and last byte; their offsets are then staged in LDS kTileSegCap at
// a time, and every lane walks its chunks (256 x 16 B apart) with a galloping search
// over the staged offsets, issuing U independent 16-B loads before their stores.
// GLDS: the source loads land in LDS by LDS-DMA (`global_load_lds_dwordx4`, no VGPR
// destination; a per-wave staging area of U KiB, lane-linear), then each lane reads back
// its own 16 B for the store; the segment tables then stage 512 segments per pass so a
// workgroup's LDS stays at ~24 KB (benchmarks/native/gather_glds_micro.hip: the gather's
// pattern alone, 304 MiB: 133.5 us by LDS-DMA vs 151.6-157.6 us through VGPRs, but no gain
// once 16 KB more LDS per workgroup lowers the co-resident count).
template <int MODE, int U, int WAVES, bool NTSTORE = false, bool GLDS = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) void k_segcopy(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const uint64_t* __restrict__ dst_off, int64_t n, uint8_t* __restrict__ dst,
    // MODE 1 extras
    const Digest* __restrict__ keys, const uint32_t* __restrict__ vlen,
    const uint32_t* __restrict__ flags, const uint32_t* __restrict__ expire,
    const uint64_t* __restrict__ head_ptr, uint64_t cap, int min_tile, ExpandTail ex) {
  // the copy (a uniform early exit per workgroup skips to the expand tail)
  do {
  // mode 2 stages a length per segment too: fewer segments per pass keep 8 waves/SIMD
  constexpr int TSC = MODE == 2 ? 768 : GLDS ? 512 : kTileSegCap;
  __shared__ uint64_t s_off[TSC + 1];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[GLDS ? kBlock / 64 : 1][GLDS ? U : 1]
                                                         [GLDS ? 1024 : 16];
  __shared__ uint64_t s_src[TSC];
  __shared__ int64_t s_lo[2], s_hi[2];
  __shared__ int s_cnt[kBlock / 64];
  if (MODE == 3) n = *reinterpret_cast<const int64_t*>(head_ptr);  // count on the device
  using Off = typename std::conditional<MODE == 4, BlockedOff, PlainOff>::type;
  Off doff;
  if constexpr (MODE == 4)
    doff = BlockedOff{dst_off, ex.prefix, n, ex.shift};
  else
    doff = PlainOff{dst_off};
  const uint64_t total = doff[n];
  if ((MODE == 0 || MODE == 3 || MODE == 4) && total > cap) break;  // destination capacity
  const uint64_t* __restrict__ seg_len = MODE == 2 ? head_ptr : nullptr;
  __shared__ uint32_t s_len[MODE == 2 ? TSC : 1];  // records < 4 GiB
  const int64_t nchunks = (int64_t)(total >> 4);
  const uint64_t base = MODE == 1 ? *head_ptr % cap : 0;
  (void)s_len;
  int64_t span = (nchunks + gridDim.x - 1) / gridDim.x;
  span = (span + kBlock - 1) & ~(int64_t)(kBlock - 1);
  if (span < min_tile) span = min_tile;
  const int64_t r0 = (int64_t)blockIdx.x * span;
  const int64_t r1 = min(r0 + span, nchunks);
  if (r0 >= r1) break;
  block_find2(doff, n + 1, (uint64_t)r0 << 4, ((uint64_t)r1 << 4) - 1, s_lo, s_hi, s_cnt);
  // (the pass bounds are uniform: scalar registers, and scalar loads below)
  const int64_t ja = uniform64(s_lo[0]), jb = uniform64(s_lo[1]);
  for (int64_t j0 = ja; j0 <= jb; j0 += TSC) {
    if (j0 > ja && j0 < jb) {
      // A later pass that starts in a run of empty segments (equal offsets) skips to the
      // run's last member, which starts the next segment holding bytes, by one block
      // search: the combined CLOCK batch has runs of 10^4-10^5 empty rows (window entries
      // not re-appended), and staging them 1024 at a time made the workgroup whose range
      // spans such a run the append's straggler (250 us instead of 45 for a 105 MiB
      // append, alone).
      const uint64_t o0 = doff[j0];
      if (doff[j0 + 1] == o0) j0 = uniform64(block_last_le(doff, j0, jb + 1, o0, s_lo, s_cnt));
    }
    const int cnt = (int)min((int64_t)TSC, jb - j0 + 1);
    __syncthreads();  // previous pass done with s_off / s_src (and s_lo read above)
    for (int k = threadIdx.x; k <= cnt; k += kBlock) s_off[k] = doff[j0 + k];
    for (int k = threadIdx.x; k < cnt; k += kBlock) s_src[k] = src_off[j0 + k];
    if (MODE == 2)
      for (int k = threadIdx.x; k < cnt; k += kBlock) {
        const uint64_t st = dst_off[j0 + k], ln = seg_len[j0 + k];
        s_len[k] = st + ln <= cap ? (uint32_t)ln : 0u;  // past the capacity: dropped
      }
    __syncthreads();
    const int64_t c0 = max(r0, (int64_t)(s_off[0] >> 4));
    const int64_t c1 = min(r1, (int64_t)(s_off[cnt] >> 4));
    int jl = 0;
    const int64_t nu = (c1 - c0 + kBlock - 1) / kBlock;  // chunks per lane in this pass
#pragma unroll 1
    for (int64_t u0 = 0; u0 < nu; u0 += U) {
      const u32x4* sp[U];
      u32x4 v[U];
      uint64_t dofs[MODE == 1 ? U : 1];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t c = c0 + (u0 + u) * kBlock + threadIdx.x;
        sp[u] = nullptr;
        if (c >= c1) continue;
        const uint64_t x = (uint64_t)c << 4;
        // galloping search: last k >= jl with s_off[k] <= x (s_off[jl] <= x holds)
        int step = 1, hi;
        while (jl + step < cnt && s_off[jl + step] <= x) {
          jl += step;
          step <<= 1;
        }
        hi = min(jl + step, cnt);
        while (hi - jl > 1) {
          const int mid = (jl + hi) >> 1;
          if (s_off[mid] <= x) jl = mid; else hi = mid;
        }
        const uint64_t seg_start = s_off[jl];
        const uint64_t seg_src = s_src[jl];
        const uint64_t w = x - seg_start;
        if (MODE == 2) {
          if (x < seg_start || w >= s_len[jl]) continue;  // gap / dropped: untouched
          sp[u] = reinterpret_cast<const u32x4*>((uintptr_t)src + seg_src + w);
        } else if (MODE == 0 || MODE == 3 || MODE == 4) {
          // a kSegSkip source leaves the segment's bytes untouched (no load, no store)
          if (seg_src == kSegSkip) continue;
          // integer address math: src may be null with absolute addresses in src_off
          sp[u] = reinterpret_cast<const u32x4*>((uintptr_t)src + seg_src + w);
        } else {
          const int64_t j = j0 + jl;
          const uint64_t p = base + seg_start;
          dofs[u] = (p >= cap ? p - cap : p) + w;
          if (w == 0) {
            const Digest d = keys[j];
            v[u] = u32x4{(uint32_t)d.lo, (uint32_t)(d.lo >> 32), (uint32_t)d.hi,
                         (uint32_t)(d.hi >> 32)};
          } else if (w == 16) {
            v[u] = u32x4{vlen[j], flags ? flags[j] : 0u, expire ? expire[j] : 0u, kItemMagic};
          } else {
            sp[u] = reinterpret_cast<const u32x4*>((uintptr_t)src + seg_src +
                                                   (w - kItemHeaderBytes));
          }
        }
      }
      if constexpr (GLDS) {
        const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (sp[u])
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void*)sp[u],
                (__attribute__((address_space(3))) void*)&s_stage[wv][u][0], 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMAs have landed in LDS
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (sp[u]) v[u] = *reinterpret_cast<const u32x4*>(&s_stage[wv][u][lane * 16]);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (sp[u]) v[u] = __builtin_nontemporal_load(sp[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t c = c0 + (u0 + u) * kBlock + threadIdx.x;
        if (c >= c1 || (MODE != 1 && !sp[u])) continue;
        const uint64_t d = MODE == 1 ? dofs[MODE == 1 ? u : 0] : (uint64_t)c << 4;
        if (NTSTORE)
          __builtin_nontemporal_store(v[u], reinterpret_cast<u32x4*>(dst + d));
        else
          *reinterpret_cast<u32x4*>(dst + d) = v[u];
      }
    }
  }
  } while (false);
  if (ex.n) expand_tail(ex);
}

// Co-resident workgroups of a kernel on the current device (occupancy x CUs), cached.
template <typename K>
int resident_grid(K kernel, int* cache) {
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] == 0) {
    int per_cu = 0, cus = 0;
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0));
    HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    cache[dev] = per_cu > 0 && cus > 0 ? per_cu * cus : kMaxGrid;
  }
  return cache[dev];
}

// The byte mover's launch: 4 loads in flight per lane, 8 waves/SIMD, nontemporal stores,
// kSegOcc64/64 of the co-resident slots (see the tuned constants above).
// (SHELLAC_SEGOCC_<MODE> = slots / 64 overrides kSegOcc64 for one mode: A/B experiments)
inline int seg_occ64(int mode) {
  static int occ[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
  if (occ[mode] < 0) {
    const std::string v = "SHELLAC_SEGOCC_" + std::to_string(mode);
    const char* e = getenv(v.c_str());
    const int x = e ? atoi(e) : 0;
    occ[mode] = x >= 1 && x <= 64 ? x : kSegOcc64;
  }
  return occ[mode];
}

// SHELLAC_GLDS=1 (A/B): the gather (modes 0 / 4) stages its loads by LDS-DMA, with the
// workgroup count of the register version (its co-resident count x the mode's slot share)
inline bool seg_glds() {
  static const int on = [] {
    const char* e = getenv("SHELLAC_GLDS");
    return e && atoi(e) != 0 ? 1 : 0;
  }();
  return on != 0;
}

template <int MODE, typename... Args>
void launch_segcopy_ex(hipStream_t s, const ExpandTail& ex, Args... args) {
  static int grid[64];
  const auto kern = k_segcopy<MODE, 4, 8, true>;
  const int g = std::max(1, resident_grid(kern, grid) * seg_occ64(MODE) / 64);
  if constexpr (MODE == 0 || MODE == 4) {
    if (seg_glds()) {
      static int ggrid[64];
      const auto gk = k_segcopy<MODE, 4, 8, true, true>;
      hipLaunchKernelGGL(gk, dim3(std::min(g, resident_grid(gk, ggrid))), dim3(kBlock), 0, s,
                         args..., kSegMinTile, ex);
      return;
    }
  }
  hipLaunchKernelGGL(kern, dim3(g), dim3(kBlock), 0, s, args..., kSegMinTile, ex);
}
template <int MODE, typename... Args>
void launch_segcopy(hipStream_t s, Args... args) {
  launch_segcopy_ex<MODE>(s, ExpandTail{}, args...);
}

// A launch that also completes `*stop` (when set; the event is then taken): the event rides
// on the kernel's own completion signal (hipExtLaunchKernel's stop event) instead of a
// marker packet queued behind it. A marker costs the next kernel of its queue ~2.7 us, and a
// stream waiting on a recorded event starts ~2.4 us later than on a stop event
// (profiles/r6_hop).
template <typename K, typename... A>
void launch_stop(hipEvent_t* stop, K kern, dim3 g, dim3 b, hipStream_t s, A... args) {
  hipEvent_t e = stop ? *stop : nullptr;
  if (e) {
    *stop = nullptr;
    hipExtLaunchKernelGGL(kern, g, b, 0, s, nullptr, e, 0, args...);
  } else {
    hipLaunchKernelGGL(kern, g, b, 0, s, args...);
  }
}

// ---------------------------------------------------------------------------------
// Edge GET (the HTTP proxy's micro-batches): probe + scan + gather in ONE launch, each
// key probed once. Workgroup b owns keys [32b, 32b+32) (one 8-lane group per key): it
// probes them, scans their sizes in LDS, learns the byte offset of its range by a
// decoupled look-back over its predecessors' published aggregates (workgroups are
// dispatched in order, so every predecessor is resident or done), then copies its own
// records. keys / off_out / out may be mapped host memory, so a batch needs no copies:
// the response lands in pinned host memory ready for writev.
// ---------------------------------------------------------------------------------
constexpr int kEdgeKeys = kBlock / 8;   // keys per workgroup

__global__ __launch_bounds__(kBlock) void k_edge_get(
    const Digest* __restrict__ keys, int64_t n, Entry* __restrict__ index, uint64_t mask,
    const uint64_t* __restrict__ head_ptr, uint64_t cap, uint32_t now,
    const uint8_t* __restrict__ log, uint8_t* __restrict__ out, uint64_t out_cap,
    uint64_t* __restrict__ off_out, CacheCounters* __restrict__ ctr,
    unsigned long long* __restrict__ state, unsigned int* __restrict__ done_ctr,
    uint64_t* __restrict__ done_slot) {
  __shared__ uint64_t s_off[kEdgeKeys + 1];
  __shared__ uint64_t s_loc[kEdgeKeys];
  __shared__ unsigned long long s_base;
  __shared__ int s_fail;
  const int g = threadIdx.x >> 3, l8 = threadIdx.x & 7, lane = threadIdx.x & 63;
  const int64_t i0 = (int64_t)blockIdx.x * kEdgeKeys;
  const int cnt = (int)min((int64_t)kEdgeKeys, n - i0);
  const uint64_t head = *head_ptr;
  uint64_t hl = 0;
  uint32_t hv = 0;
  if (g < cnt) {
    const Digest d = keys[i0 + g];
    int he = 0;
    uint64_t hb = bucket1(d, mask);
    group_match(reinterpret_cast<const uint4*>(index + hb * kEntriesPerBucket)[l8], d, l8, head,
                cap, now, &hl, &hv, &he);
    if (hl == 0) {
      hb = bucket2(d, mask);
      group_match(reinterpret_cast<const uint4*>(index + hb * kEntriesPerBucket)[l8], d, l8,
                  head, cap, now, &hl, &hv, &he);
    }
    if (hl && l8 == 0) mark_ref(index, hb, he, hv);
    hv = entry_vlen(hv);
  }
  if (l8 == 0) {
    s_loc[g] = hl ? (hl - 1) % cap : 0;
    s_off[g] = hl ? item_bytes(hv) : 0;
  }
  if (threadIdx.x == 0) s_fail = 0;
  __syncthreads();
  // wave 0: exclusive scan of the 32 sizes, publish the aggregate, look back
  if (threadIdx.x < 64) {
    const uint64_t v = lane < kEdgeKeys ? s_off[lane] : 0;
    uint64_t inc = v;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
      const uint64_t o = __shfl_up(inc, dd);
      if (lane >= dd) inc += o;
    }
    const uint64_t agg = __shfl(inc, 63);
    // never hangs: a predecessor that never publishes marks the batch failed
    const unsigned long long base = lookback_exclusive(state, agg, &s_fail);
    if (lane == 0) s_base = base;
    if (lane <= kEdgeKeys) s_off[lane] = inc - v;  // exclusive; s_off[32] = agg
  }
  __syncthreads();
  const uint64_t base = s_base;
  const uint64_t agg = s_off[kEdgeKeys];
  const bool fail = s_fail != 0;
  for (int k = threadIdx.x; k < cnt; k += kBlock) off_out[i0 + k] = base + s_off[k];
  const bool last_wg = i0 + kEdgeKeys >= n;
  if (last_wg && threadIdx.x == 0) off_out[n] = base + agg;
  block_count(ctr, (unsigned long long)(threadIdx.x == 0 ? cnt : 0), &CacheCounters::get_ops,
              (unsigned long long)(l8 == 0 && hl ? 1 : 0), &CacheCounters::get_hits,
              (unsigned long long)(l8 == 0 && hl ? hv : 0), &CacheCounters::get_bytes);
  // copy this workgroup's records (skipped if the batch outgrew the buffer: the caller
  // sees off_out[n] > out_cap and repeats the batch into a bigger one)
  if (!fail && base + agg <= out_cap) {
    const int64_t nchunks = (int64_t)(agg >> 4);
    int jl = 0;
    for (int64_t c = threadIdx.x; c < nchunks; c += kBlock) {
      const uint64_t x = (uint64_t)c << 4;
      while (jl + 1 < cnt && s_off[jl + 1] <= x) ++jl;  // monotone per lane
      const u32x4 v = __builtin_nontemporal_load(
          reinterpret_cast<const u32x4*>(log + s_loc[jl] + (x - s_off[jl])));
      *reinterpret_cast<u32x4*>(out + base + x) = v;
    }
  }
  // Completion signal without a stream sync: every wave drains its own stores (vmcnt)
  // around a system-scope release fence (ROCm 7.2 can drop the fence's own wait), the
  // workgroup counts itself done, and the last one resets the counter and the look-back
  // state for the next launch, then publishes the total (or kSlotFailed) into the pinned
  // host slot the batcher thread polls.
  if (done_slot) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    if (fail) atomicOr(done_ctr + 1, 1u);
    s_last = atomicAdd(done_ctr, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last) {
    __shared__ unsigned long long s_total;
    if (threadIdx.x == 0)  // the last range's inclusive prefix = the batch total
      s_total = __hip_atomic_load(state + gridDim.x - 1, __ATOMIC_ACQUIRE,
                                  __HIP_MEMORY_SCOPE_AGENT) & kLbVal;
    __syncthreads();
    for (unsigned k = threadIdx.x; k < gridDim.x; k += kBlock) state[k] = 0ull;
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned int failed = atomicExch(done_ctr + 1, 0u);
      atomicExch(done_ctr, 0u);
      __threadfence_system();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (done_slot) {
        const uint64_t total = failed ? HbmCache::kSlotFailed : (uint64_t)s_total;
        __hip_atomic_store(done_slot, total, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// Persistent edge-GET server (HbmCache::serve_get). One 512-thread workgroup stays
// resident and polls a ring of jobs in pinned, coherent host memory, so a micro-batch
// costs no kernel launch (profiles/archive/r2_edge_get_latency.log: a launch + completion round
// trip is 14-19 us of the proxy's 25-33 us batch).
// Transport: a job is 64 granules of 16 B, each {payload word, tag = ticket + 1}: five
// header granules (arena, capacity, offsets array, n | now, host slot) and two per key.
// Wave 0 polls the whole job with one 16-B load per lane — one PCIe round trip — and
// takes it when every granule it covers carries the ticket's tag (the host writes each
// granule with one 16-B store, so a granule is never torn): no separate read of the job
// after its sequence word.
// Coherence: other CUs' SET kernels write the index and the log and release them (kernel
// end, or k_set_small's agent release before its index insert); the server reads both
// with nontemporal loads, which bypass the CU's L1 (L2-served), so no acquire fence per
// job. A SET chain still running may overwrite a record while it is being copied: every
// SET batch first raises the claim word (the furthest log byte its append writes;
// k_offsets / k_set_small, before the append), the probe treats anything the claim
// reaches as evicted, and after every copy load of a round has returned the claim is read
// again: a record it now reaches is stored with a zeroed magic word (a miss at the
// batcher's header check) — a seqlock. An index entry a concurrent insert has
// half-written can pair a digest with another key's record: the header check rejects it.
// Exit: when the host sets the stop word, after `idle` ticks without a job, or after
// `life` ticks of running (so a device-wide synchronisation elsewhere never waits on it
// for long); it records the tickets it consumed and its epoch, and serve_kick relaunches
// it when jobs are outstanding. Per job, lane 0 records five wall-clock stamps (poll
// issue, job seen, probed, copied, publish) for serve_trace().
// ---------------------------------------------------------------------------------
constexpr int kSrvBlock = 512;
constexpr int kSrvPollWave = kSrvBlock / 64 - 1;  // the last wave polls; the others work
constexpr int kSrvWorkers = kSrvPollWave * 64;
constexpr int kSrvGroups = kSrvWorkers / 8;
static_assert(HbmCache::kServeKeys <= kSrvGroups, "one probe pass per job");
constexpr int kSrvUnroll = 16;  // 16-B chunks in flight per lane: 128 KiB per round
constexpr int kSrvGranules = 64;
constexpr int kSrvHdr = 5;
static_assert(kSrvHdr + 2 * HbmCache::kServeKeys <= kSrvGranules, "a job is one wave's load");

struct SrvGranule {
  uint64_t v, tag;
};
struct SrvJob {  // one ring slot (1 KiB), host-written
  SrvGranule g[kSrvGranules];
};
// control words, each on its own line: the exited epoch, the stop word, then each server
// block's consumed count (block b at kCtlConsumed + 8 b)
constexpr int kCtlExited = 8, kCtlStop = 16, kCtlConsumed = HbmCache::kSrvCtlConsumed;
constexpr int kCtlWords = kCtlConsumed + 8 * HbmCache::kServeBlocksMax;
// The server exits after this long without a job (the next job relaunches it) and after
// this long in all (a device-wide synchronisation elsewhere waits at most that long).
constexpr uint64_t kSrvIdleUs = 1000, kSrvLifeUs = 10000;
constexpr int kSrvTrace = 64;  // jobs whose phase stamps are kept (ring)

// Lane `lane`'s 16-B granule of ring slot `t`: a system-coherent load (sc0 sc1: past every
// GPU cache) of host memory the host rewrites — a plain or nontemporal load of it can be
// served stale from a cache, and a poll that misses a job then waits for the server's
// idle exit (measured: ~0.5 ms a job). Waits for its own return. (A buffer-load builtin
// with the same cache policy measured 2.5 us per round trip against 1.4 for this.)
__device__ __forceinline__ u32x4 poll_slot(const SrvJob* ring, uint64_t t, int lane) {
  const void* p = &ring[t % HbmCache::kServeRing].g[lane];
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(v)
               : "v"(p)
               : "memory");
  return v;
}
__device__ __forceinline__ uint64_t sys_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t agent_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane l8's 16-B quarter of a bucket, read past the CU's L1 (nontemporal: L2-served)
__device__ __forceinline__ uint4 nt_bucket_quarter(const Entry* index, uint64_t b, int l8) {
  const u32x4 v = __builtin_nontemporal_load(
      reinterpret_cast<const u32x4*>(index + b * kEntriesPerBucket) + l8);
  return uint4{v.x, v.y, v.z, v.w};
}
// newest log head any kernel has published or claimed (head slots 0/1, claim word 4)
__device__ __forceinline__ uint64_t newest_head(const uint64_t* heads) {
  return max(max(agent_load(heads), agent_load(heads + 1)), agent_load(heads + 4));
}

// Several server blocks (HbmCache::serve_blocks): block b serves the tickets T with
// T % nblk == b from a ring of its own, so jobs of different submitters (the batcher,
// each reactor) are served side by side. The blocks leave together: a block stranded
// alone would keep the others' jobs waiting for the relaunch until it idles. `sync`
// (device memory, zeroed at launch): [0] the last job's publish tick of any block (idle
// means all idle), [1] blocks that have exited (the last one out writes the exited
// epoch), [2] set by the first block that decides to leave (lifetime, idle, stop): every
// block checks it before each poll.
__global__ __launch_bounds__(kSrvBlock) void k_edge_server(
    const SrvJob* __restrict__ ring, uint64_t* __restrict__ ctl, uint64_t* __restrict__ slots,
    Entry* __restrict__ index, uint64_t mask, const uint64_t* __restrict__ heads, uint64_t cap,
    const uint8_t* __restrict__ log, CacheCounters* __restrict__ ctr,
    uint64_t* __restrict__ trace, uint64_t epoch, uint64_t idle_ticks, uint64_t life_ticks,
    uint64_t* __restrict__ sync, int nblk) {
  constexpr int K = HbmCache::kServeKeys;
  const int blk = blockIdx.x;
  ring += (size_t)blk * HbmCache::kServeRing;
  uint64_t* const consumed = ctl + kCtlConsumed + 8 * blk;
  __shared__ Digest s_key[K];
  __shared__ uint64_t s_loc[K];      // physical record offset
  __shared__ uint64_t s_lg[K];       // logical record start + 1 (0: miss)
  __shared__ uint64_t s_off[K + 1];
  __shared__ uint64_t s_job[kSrvHdr];  // out, out_cap, off, n | now << 32, slot
  __shared__ uint64_t s_head;
  __shared__ uint64_t s_t[3];          // poll issued, job seen (poller); last publish (tid 0)
  __shared__ int s_cmd;
  __shared__ unsigned long long s_cnt[3][kSrvBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = tid >> 3, l8 = tid & 7;
  const bool worker = w != kSrvPollWave;
  uint64_t ticket = sys_load(consumed);  // this block's tickets: T = ticket * nblk + blk
  const uint64_t t_start = (uint64_t)wall_clock64();
  if (tid == 0) s_t[2] = t_start;
  u32x4 pre = u32x4{0u, 0u, 0u, 0u};
  bool have_pre = false;
  __syncthreads();
  for (;;) {
    // ---- wait for the next job. The poller wave reads all of it per poll (one 16-B
    //      granule a lane); while the workers probe a job it reads the next slot ahead:
    //      when the host has queued that job meanwhile (back-to-back batches) it is there
    //      when this one is done, and the round trip hid under the probe.
    if (!worker) {
      const uint64_t want = ticket + 1;
      int cmd = 1;
      uint64_t t_poll = 0;
      for (;;) {
        // another block is leaving: leave too (its jobs and ours wait for the relaunch, so
        // every block goes at once, at most one job apart)
        if (nblk > 1 && __shfl((int)(lane == 0 && agent_load(sync + 2) != 0), 0)) break;
        u32x4 gv;
        t_poll = (uint64_t)wall_clock64();
        if (have_pre) {
          gv = pre;
          have_pre = false;
        } else {
          gv = poll_slot(ring, ticket, lane);
        }
        const uint64_t v = pack2(gv.x, gv.y), tag = pack2(gv.z, gv.w);
        const uint64_t nn = __shfl(v, 3) & 0xffffffffu;     // n, from granule 3
        const bool hdr_ok = __shfl((int)(tag == want), 3) != 0;
        const bool mine = lane < kSrvHdr + 2 * (int)(hdr_ok ? min(nn, (uint64_t)K) : 0);
        if (hdr_ok && __ballot(mine && tag != want) == 0ull) {
          if (lane < kSrvHdr) s_job[lane] = v;
          const int kk = (lane - kSrvHdr) >> 1;
          if (lane >= kSrvHdr && mine) {
            if (((lane - kSrvHdr) & 1) == 0) s_key[kk].lo = v;
            else s_key[kk].hi = v;
          }
          cmd = 0;
          break;
        }
        const uint64_t t = (uint64_t)wall_clock64();
        // (another block's publish may be newer than t: compare, do not subtract)
        const bool quit =
            lane == 0 && (sys_load(ctl + kCtlStop) ||
                          t > max(s_t[2], agent_load(sync)) + idle_ticks || t - t_start > life_ticks);
        if (__shfl((int)quit, 0)) {
          if (lane == 0 && nblk > 1)
            __hip_atomic_store(sync + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (lane == 0) {
        s_cmd = cmd;
        s_t[0] = t_poll;
        s_t[1] = (uint64_t)wall_clock64();
      }
    }
    __syncthreads();
    if (s_cmd) break;
    const int n = (int)(s_job[3] & 0xffffffffu);
    const uint32_t now = (uint32_t)(s_job[3] >> 32);
    uint8_t* const out = reinterpret_cast<uint8_t*>(s_job[0]);
    const uint64_t out_cap = s_job[1];
    uint64_t* const off_out = reinterpret_cast<uint64_t*>(s_job[2]);
    // ---- probe: one 8-lane group of the workers per key, nontemporal (L2-served) bucket
    //      reads, issued together with the (L2-hot) head words the liveness test needs
    unsigned long long ops = 0, hits = 0, bytes = 0;
    if (!worker) {  // read ahead (consumed when this job is done)
      pre = poll_slot(ring, ticket + 1, lane);
      have_pre = true;
    }
    for (int k = g; worker && k - g < n; k += kSrvGroups) {
      uint64_t hl = 0;
      uint32_t hv = 0;
      if (k < n) {
        const Digest d = s_key[k];
        int he = 0;
        uint64_t hb = bucket1(d, mask);
        const uint4 q1 = nt_bucket_quarter(index, hb, l8);
        // each lane judges its own entry: lanes may see different (all valid) heads
        const uint64_t head = newest_head(heads);
        group_match(q1, d, l8, head, cap, now, &hl, &hv, &he);
        if (hl == 0) {
          hb = bucket2(d, mask);
          group_match(nt_bucket_quarter(index, hb, l8), d, l8, head, cap, now, &hl, &hv, &he);
        }
        if (hl && l8 == 0) mark_ref(index, hb, he, hv);
        hv = entry_vlen(hv);
        if (l8 == 0) {
          s_lg[k] = hl;
          s_loc[k] = hl ? (hl - 1) % cap : 0;
          s_off[k] = hl ? item_bytes(hv) : 0;
          ++ops;
          hits += hl ? 1 : 0;
          bytes += hl ? hv : 0;
        }
      }
    }
    __syncthreads();
    // ---- exclusive scan of the sizes (wave 0, two keys per lane: K <= 128)
    if (w == 0) {
      const uint64_t a = lane < n ? s_off[lane] : 0;
      const uint64_t b = lane + 64 < n ? s_off[lane + 64] : 0;
      uint64_t ia = a, ib = b;
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const uint64_t oa = __shfl_up(ia, dd), ob = __shfl_up(ib, dd);
        if (lane >= dd) {
          ia += oa;
          ib += ob;
        }
      }
      const uint64_t ta = __shfl(ia, 63), tb = __shfl(ib, 63);
      if (lane < n) s_off[lane] = ia - a;
      if (lane + 64 < n) s_off[lane + 64] = ta + ib - b;
      if (lane == 0) s_off[n] = ta + tb;
    }
    __syncthreads();
    const uint64_t t_probed = (uint64_t)wall_clock64();
    const uint64_t total = s_off[n];
    if (worker)
      for (int k = tid; k <= n; k += kSrvWorkers) off_out[k] = s_off[k];
    // ---- stream the records in rounds of kSrvUnroll chunks per worker lane: loads, then
    //      (all loads of the round returned) the claim check, then the stores. Nothing
    //      when the records outgrow the arena (the caller regathers).
    const int64_t nch = total <= out_cap ? (int64_t)(total >> 4) : 0;
    for (int64_t c0 = 0; c0 < nch; c0 += (int64_t)kSrvWorkers * kSrvUnroll) {
      u32x4 v[kSrvUnroll];
      int rec[kSrvUnroll];
#pragma unroll
      for (int u = 0; u < kSrvUnroll; ++u) {
        const int64_t c = c0 + (int64_t)u * kSrvWorkers + tid;
        rec[u] = -1;
        if (worker && c < nch) {
          const uint64_t x = (uint64_t)c << 4;
          int lo = 0, hi = n - 1;  // the record holding byte x: last k with s_off[k] <= x
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_off[mid] <= x) lo = mid;
            else hi = mid - 1;
          }
          v[u] = __builtin_nontemporal_load(
              reinterpret_cast<const u32x4*>(log + s_loc[lo] + (x - s_off[lo])));
          rec[u] = lo;
        }
      }
      if (worker) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) s_head = newest_head(heads);
      __syncthreads();
      const uint64_t c2 = s_head;
#pragma unroll
      for (int u = 0; u < kSrvUnroll; ++u) {
        if (rec[u] < 0) continue;
        const uint64_t x = (uint64_t)(c0 + (int64_t)u * kSrvWorkers + tid) << 4;
        // a record the claim now reaches may be torn: zero its magic word (miss)
        if (x - s_off[rec[u]] == 16 && !(c2 <= (s_lg[rec[u]] - 1) + cap))
          v[u] = u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(out + x) = v[u];
      }
    }
    // ---- completion: every worker wave drains its stores, then one system-scope publish
    //      (the poller's outstanding read-ahead is not waited for)
    if (worker) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // A job of several rounds: a record's chunks after its header round were loaded after
    // the only check that covered its magic word. Every load has returned now: read the
    // claim once more and turn every record it reaches into a miss (magic word zeroed)
    // before the publish. (One round: the round's own check covered every chunk.)
    if (nch > (int64_t)kSrvWorkers * kSrvUnroll) {
      if (tid == 0) s_head = newest_head(heads);
      __syncthreads();
      const uint64_t c3 = s_head;
      for (int k = tid; worker && k < n; k += kSrvWorkers)
        if (s_lg[k] && !(c3 <= (s_lg[k] - 1) + cap))
          *reinterpret_cast<uint32_t*>(out + s_off[k] + 28) = 0u;
      if (worker) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const uint64_t t_copied = (uint64_t)wall_clock64();
    const uint64_t gticket = ticket * (uint64_t)nblk + (uint64_t)blk;
    if (tid == 0) {
      // the job's phase stamps first, so they are in place when the host sees the slot
      uint64_t* tr = trace + (gticket % kSrvTrace) * 8;
      tr[0] = gticket;
      tr[1] = s_t[0];
      tr[2] = s_t[1];
      tr[3] = t_probed;
      tr[4] = t_copied;
      tr[5] = (uint64_t)wall_clock64();
      tr[6] = (uint64_t)n;
      tr[7] = total;
      __threadfence_system();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(slots + s_job[4], total, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(consumed, ticket + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      s_t[2] = (uint64_t)wall_clock64();
      if (nblk > 1)
        __hip_atomic_fetch_max(sync, s_t[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- counters (off the latency path)
    ops = wave_sum(ops);
    hits = wave_sum(hits);
    bytes = wave_sum(bytes);
    if (lane == 0) {
      s_cnt[0][w] = ops;
      s_cnt[1][w] = hits;
      s_cnt[2][w] = bytes;
    }
    __syncthreads();
    if (tid == 0) {
      unsigned long long t0 = 0, t1 = 0, t2 = 0;
#pragma unroll
      for (int k = 0; k < kSrvBlock / 64; ++k) {
        t0 += s_cnt[0][k];
        t1 += s_cnt[1][k];
        t2 += s_cnt[2][k];
      }
      CacheCounters* c_ = ctr + (gticket & (kCtrShards - 1));
      if (t0) atomicAdd(&c_->get_ops, t0);
      if (t1) atomicAdd(&c_->get_hits, t1);
      if (t2) atomicAdd(&c_->get_bytes, t2);
    }
    ++ticket;
    __syncthreads();  // LDS is reused by the next job
  }
  if (tid == 0) {
    __hip_atomic_store(consumed, ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t out = __hip_atomic_fetch_add(sync + 1, 1ull, __ATOMIC_ACQ_REL,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (out + 1 == (uint64_t)nblk)  // the last block out: every ticket it could take is done
      __hip_atomic_store(ctl + kCtlExited, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------------------------
// SET
// ---------------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void k_set_size(const uint32_t* __restrict__ vlen, int64_t n,
                                                     const int* __restrict__ tw,
                                                     const uint32_t* __restrict__ slot_of,
                                                     uint32_t max_item,
                                                     uint64_t* __restrict__ size,
                                                     CacheCounters* __restrict__ ctr,
                                                     uint64_t* __restrict__ part,
                                                     uint64_t* __restrict__ part_cnt) {
  unsigned long long dropped = 0, ops = 0, psum = 0, stored = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) size[n] = 0;
  const int64_t plen = part_len(n, gridDim.x);
  const int64_t i1 = min(n, (int64_t)(blockIdx.x + 1) * plen);
  for (int64_t i = (int64_t)blockIdx.x * plen + threadIdx.x; i < i1; i += kBlock) {
    if (vlen[i] == kSkipVlen) { size[i] = 0; continue; }  // row addressed to another tier
    const bool win = tw[slot_of[i]] == (int)i && vlen[i] <= max_item;
    const uint64_t sz = win ? item_bytes(vlen[i]) : 0;
    size[i] = sz;
    psum += sz;
    ++ops;
    dropped += win ? 0 : 1;
    stored += win ? 1 : 0;
  }
  block_count(ctr, ops, &CacheCounters::set_ops, dropped, &CacheCounters::set_dropped);
  block_partial(psum, part);
  if (part_cnt) block_partial(stored, part_cnt);  // ring ordinals (CLOCK)
}

// SET index insert, 4 lanes per key: lane q reads entry q of both candidate buckets
// (4 x 8-B agent-scope loads each), so a wave keeps 16 keys' bucket reads in flight — the
// insert is latency-bound, and beside the bandwidth-bound gather it only gets the slots
// the gather leaves (a 16-lanes-per-key version took 130-140 us there, this one 39 us).
// Policy: replace the key's own entry, else a dead slot (first bucket while it keeps
// >= 2 free, else the emptier bucket), else move one entry of the pair to its other
// bucket (relocate_one), else evict the oldest; the entry is claimed by a
// CAS on its loc word, the digest / vlen words follow and k_set_fixup repairs entries
// a later insert of the same batch re-claimed. Workgroup 0 publishes the new log head
// into the other ping-pong head slot; every row resets its dedupe-table slot.
// Keep this kernel at <= 64 VGPRs (8 waves/SIMD): beside the gather, which holds 3/4 of
// every SIMD's slots, a 72-VGPR build fits one wave per SIMD instead of two and ran 4x
// slower (126 vs 31 us per 64K-row batch).
// Relocation: when all 8 slots of a new key's bucket pair are live, one of them whose own
// other bucket has a dead slot moves there (one cuckoo step) and the key takes its place;
// only when none can move is the oldest evicted. Without it, inserts racing for a pair's
// last free slots evicted a live key now and then at 30 % slot load (1 key in 40K, in
// about 1 run in 4; a sequential insert of the same keys evicts none).
// Called by the whole 4-lane group, in the all-live case (lane l4 holds entry l4 of each
// bucket in w1 / w2). The lane holding the chosen entry copies it into the dead slot
// (copy_entry: lock the slot's loc, write the words, publish the loc) — so the copy is
// never half-written while live, no two copies interleave their words in one slot, and
// from then on the key has two entries with the same record. Returns, uniform in the group: the entry's index 0-7 (the caller then
// CASes it from the entry's loc to its own) and the copy's slot, or -1 when no entry can
// move, -2 when the copy's CAS lost (re-read and try again). If the caller's
// CAS then fails (the moved key was updated in the meantime, or evicted), it must drop
// the copy (undo_relocation) so no stale duplicate stays behind.
// (Entry words by value: an array argument would put the caller's registers in scratch.)
// claim[i] of a row k_set_index left to k_set_fixup (no index slot id reaches it)
constexpr uint32_t kClaimDeferred = 0xfffffffeu;

struct Reloc {
  uint64_t alt;  // the copy's slot
  int target;    // 0-7, -1 none can move, -2 the copy's CAS lost
};

// Copy an entry {d0, d1, loc, vlen|expire} into the free slot `a` whose loc was `expect`:
// lock the slot first (CAS expect -> kLockedLoc: from then on no other inserter claims,
// matches or copies into it), write the digest and vlen words, then publish the real loc
// behind an agent-scope release. Two inserters that picked the same free slot can no
// longer interleave their digest words: only the one whose lock CAS won writes any.
// Returns whether the copy is in place.
__device__ __forceinline__ bool copy_entry(Entry* __restrict__ a, uint64_t expect, uint64_t d0,
                                           uint64_t d1, uint64_t loc, uint64_t word) {
  if (atomicCAS(reinterpret_cast<unsigned long long*>(&a->loc), (unsigned long long)expect,
                (unsigned long long)kLockedLoc) != expect)
    return false;
  a->d0 = d0;
  a->d1 = d1;
  *reinterpret_cast<uint64_t*>(&a->vlen) = word;
  __hip_atomic_store(&a->loc, loc, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Drop a copy (its loc still `loc`): lock it, clear the digest words, then free it, so
// the moved key's digest never lingers in a free slot beside its live entry and no new
// claimer's words can be overwritten by the clearing.
__device__ __forceinline__ void drop_entry(Entry* __restrict__ a, uint64_t loc) {
  if (atomicCAS(reinterpret_cast<unsigned long long*>(&a->loc), (unsigned long long)loc,
                (unsigned long long)kLockedLoc) != loc)
    return;
  a->d0 = 0;
  a->d1 = 0;
  __hip_atomic_store(&a->loc, (uint64_t)0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Reloc relocate_one(uint64_t p0, uint64_t p1, uint64_t p2, uint64_t p3,
                                         uint64_t r0, uint64_t r1, uint64_t r2, uint64_t r3,
                                         uint64_t b1, uint64_t b2, Entry* __restrict__ index,
                                         uint64_t mask, uint64_t base, uint64_t span,
                                         uint64_t head_new, uint64_t cap, uint32_t now) {
  const int l4 = threadIdx.x & 3;
  const int gbase = threadIdx.x & 60;
  int pick = -1;  // this lane's candidate: 0 (its b1 entry) or 1 (its b2 entry)
  uint64_t a_slot = 0, a_loc = 0;
#pragma unroll 1
  for (int h = 0; h < 2 && pick < 0; ++h) {
    const uint64_t wd0 = h ? r0 : p0, wd1 = h ? r1 : p1, wloc = h ? r2 : p2;
    const uint64_t own = h ? b2 : b1;
    if (wloc - base - 1 < span) continue;  // another row's claim of this batch: not final
    if (wloc == kLockedLoc) continue;      // another inserter's copy in flight
    const Digest de{wd0, wd1};
    const uint64_t x1 = bucket1(de, mask), x2 = bucket2(de, mask);
    const uint64_t ob = x1 == own ? x2 : (x2 == own ? x1 : own);
    if (ob == own) continue;
    const uint64_t* q = reinterpret_cast<const uint64_t*>(index + ob * kEntriesPerBucket);
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {
      const uint64_t l = __hip_atomic_load(q + 4 * k + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t x = __hip_atomic_load(q + 4 * k + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (entry_free(l, (uint32_t)(x >> 32), head_new, cap, now)) {
        pick = h;
        a_slot = ob * kEntriesPerBucket + k;
        a_loc = l;
        break;
      }
    }
  }
  const uint32_t m0 = (uint32_t)((__ballot(pick == 0) >> gbase) & 0xfull);
  const uint32_t m1 = (uint32_t)((__ballot(pick == 1) >> gbase) & 0xfull);
  if (!(m0 | m1)) return Reloc{~0ull, -1};
  const int lane = m0 ? __ffs(m0) - 1 : __ffs(m1) - 1;
  const int target = (m0 ? 0 : 4) + lane;
  int ok = 0;
  if (l4 == lane) ok = copy_entry(index + a_slot, a_loc, m0 ? p0 : r0, m0 ? p1 : r1,
                                  m0 ? p2 : r2, m0 ? p3 : r3);
  ok = __shfl(ok, gbase + lane);
  return Reloc{__shfl(a_slot, gbase + lane), ok ? target : -2};
}

// The caller's CAS of the moved key's old slot failed: drop the copy relocate_one made.
__device__ __forceinline__ void undo_relocation(Entry* __restrict__ index, uint64_t alt,
                                             uint64_t loc) {
  drop_entry(index + alt, loc);
}

// One SET row's index insert by its 4-lane group (uniform arguments across the group;
// `active` false: nothing to insert). Lane 0 writes the claimed entry id to *claim_out
// when the CAS succeeds (the caller pre-sets ~0u); counts evictions / bytes / rows that
// lost their bucket pair past the retry budget. k_set_small's copy of k_set_index's
// loop body (k_set_index keeps its own: sharing this function cost it 12 B/lane of
// scratch at its 64-VGPR budget).
__device__ __forceinline__ void index_insert(
    bool active, const Digest& d, uint64_t myloc, uint32_t myvlen, uint32_t myexp,
    uint32_t* __restrict__ claim_out,
    Entry* __restrict__ index, uint64_t mask, uint64_t base, uint64_t head_new, uint64_t cap,
    uint32_t now, unsigned long long& evicted, unsigned long long& bytes,
    unsigned long long& lost) {
  const int l4 = threadIdx.x & 3;
  const int gbase = threadIdx.x & 60;  // this group's first lane within the wave
  if (!active) return;  // uniform across the 4-lane group
  const uint64_t b1 = bucket1(d, mask), b2 = bucket2(d, mask);
  const uint64_t* q1 = reinterpret_cast<const uint64_t*>(index + b1 * kEntriesPerBucket + l4);
  const uint64_t* q2 = reinterpret_cast<const uint64_t*>(index + b2 * kEntriesPerBucket + l4);
  for (int attempt = 0; attempt < 16; ++attempt) {
    // agent-scope loads: a retry must see other workgroups' CAS results, not stale L1
    uint64_t w1[4], w2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w1[k] = __hip_atomic_load(q1 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      w2[k] = __hip_atomic_load(q2 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // words: d0, d1, loc, vlen | expire << 32. A digest match whose loc belongs to
    // this batch, (base, head_new], is another row's claim whose digest words have not
    // landed yet (dedupe leaves one row per key, so it is never this key's entry):
    // taking it as our own would CAS that row's claim away and lose its SET.
    const uint64_t span = head_new - base;  // locs of this batch: (base, head_new]
    const bool in1 = w1[2] - base - 1 < span || w1[2] == kLockedLoc;
    const bool in2 = w2[2] - base - 1 < span || w2[2] == kLockedLoc;
    const bool m1 = w1[0] == d.lo && w1[1] == d.hi && !in1;
    const bool m2 = w2[0] == d.lo && w2[1] == d.hi && !in2;
    const bool v1 = !entry_free(w1[2], (uint32_t)(w1[3] >> 32), head_new, cap, now);
    const bool v2 = !entry_free(w2[2], (uint32_t)(w2[3] >> 32), head_new, cap, now);
    const uint32_t mmask = (uint32_t)((__ballot(m1) >> gbase) & 0xfull) |
                           ((uint32_t)((__ballot(m2) >> gbase) & 0xfull) << 4);
    const uint32_t lmask = (uint32_t)((__ballot(v1) >> gbase) & 0xfull) |
                           ((uint32_t)((__ballot(v2) >> gbase) & 0xfull) << 4);
    int target;
    bool evict = false;
    uint64_t alt = ~0ull;  // relocation copy (all-live pair), dropped if our CAS fails
    if (mmask) {
      target = __ffs(mmask) - 1;
    } else {
      const uint32_t dead = ~lmask & 0xffu;
      if (dead) {
        const int live1 = __popc(lmask & 0xfu), live2 = __popc(lmask & 0xf0u);
        const uint32_t pref = __popc(dead & 0x0fu) >= 2
                                  ? (dead & 0x0fu)
                                  : (live2 < live1 ? (dead & 0xf0u) : (dead & 0x0fu));
        target = __ffs(pref ? pref : dead) - 1;
      } else {
        const Reloc r = relocate_one(w1[0], w1[1], w1[2], w1[3], w2[0], w2[1], w2[2], w2[3],
                                     b1, b2, index, mask, base, span, head_new, cap, now);
        target = r.target;
        alt = r.alt;
        if (target == -1) {
          uint64_t oldest = ~0ull;
          target = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint64_t le = e < 4 ? __shfl(w1[2], gbase + e) : __shfl(w2[2], gbase + e - 4);
            if (le < oldest) { oldest = le; target = e; }
          }
          evict = true;
        }
      }
    }
    if (target < 0) {  // the relocation's copy lost its slot: re-read
      if (attempt == 15 && l4 == 0) ++lost;
      continue;
    }
    const uint64_t e1 = __shfl(w1[2], gbase + (target & 3));
    const uint64_t e2 = __shfl(w2[2], gbase + (target & 3));
    const uint64_t expected = target < 4 ? e1 : e2;
    Entry* const slot = index + (target < 4 ? b1 : b2) * kEntriesPerBucket + (target & 3);
    int ok = 0;
    if (l4 == 0) {
      const unsigned long long prev = atomicCAS(
          reinterpret_cast<unsigned long long*>(&slot->loc), (unsigned long long)expected,
          (unsigned long long)myloc);
      if (prev == expected) {
        slot->d0 = d.lo;
        slot->d1 = d.hi;
        *reinterpret_cast<uint64_t*>(&slot->vlen) = pack2(myvlen, myexp);
        *claim_out = (uint32_t)(slot - index);
        ok = 1;
        evicted += evict ? 1 : 0;
        bytes += myvlen;
      } else if (alt != ~0ull) {
        undo_relocation(index, alt, expected);
      }
    }
    ok = __shfl(ok, gbase);
    if (ok) break;
    if (attempt == 15 && l4 == 0) ++lost;  // bucket pair contended past the retry budget
  }
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_set_index(
    const Digest* __restrict__ keys, int64_t n, const uint64_t* __restrict__ size,
    const uint64_t* __restrict__ off, const uint32_t* __restrict__ vlen,
    const uint32_t* __restrict__ expire, Entry* __restrict__ index, uint64_t mask,
    const uint64_t* __restrict__ head_ptr, uint64_t* __restrict__ head_next, uint64_t cap,
    uint32_t now, const uint32_t* __restrict__ slot_of, unsigned long long* __restrict__ dd_keys,
    int* __restrict__ dd_win, CacheCounters* __restrict__ ctr, uint32_t* __restrict__ claim,
    const uint64_t* __restrict__ from, int64_t r0, int64_t r1,
    const unsigned long long* __restrict__ r1_dev) {
  // r1_dev: the combined batch's effective hand window (rows past it are skip rows)
  if (r1_dev && (int64_t)*r1_dev < r1) r1 = (int64_t)*r1_dev;
  const int l4 = threadIdx.x & 3;
  const int gbase = threadIdx.x & 60;  // this group's first lane within the wave
  const uint64_t base = *head_ptr;
  const uint64_t head_new = base + off[n];
  const int64_t ngroups = ((int64_t)gridDim.x * kBlock) >> 2;
  unsigned long long evicted = 0, bytes = 0, lost = 0, moved_away = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) *head_next = head_new;
  for (int64_t i = r0 + (((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 2); i < r1; i += ngroups) {
    if (l4 == 0 && vlen[i] != kSkipVlen) {  // leave the dedupe table clean for the next batch
      const uint32_t sl = slot_of[i];
      dd_keys[sl] = 0ull;
      dd_win[sl] = -1;
    }
    if (l4 == 0) claim[i] = ~0u;  // no entry (yet)
    if (size[i] == 0) continue;   // uniform across the 4-lane group
    const Digest d = keys[i];
    const uint64_t myloc = base + off[i] + 1;
    const uint32_t myvlen = vlen[i];
    const uint32_t myexp = expire ? expire[i] : 0u;
    // a CLOCK reinsertion (detached hand): a move of the entry that still points at the
    // item's old location, or nothing (uniform in the group)
    const uint64_t fr = from ? from[i] : 0ull;
    const uint64_t b1 = bucket1(d, mask), b2 = bucket2(d, mask);
    const uint64_t* q1 = reinterpret_cast<const uint64_t*>(index + b1 * kEntriesPerBucket + l4);
    const uint64_t* q2 = reinterpret_cast<const uint64_t*>(index + b2 * kEntriesPerBucket + l4);
    for (int attempt = 0; attempt < 16; ++attempt) {
      // agent-scope loads: a retry must see other workgroups' CAS results, not stale L1
      uint64_t w1[4], w2[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        w1[k] = __hip_atomic_load(q1 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        w2[k] = __hip_atomic_load(q2 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      // words: d0, d1, loc, vlen | expire << 32. A digest match whose loc belongs to
      // this batch, (base, head_new], is another row's claim whose digest words have not
      // landed yet (dedupe leaves one row per key, so it is never this key's entry):
      // taking it as our own would CAS that row's claim away and lose its SET.
      const uint64_t span = head_new - base;  // locs of this batch: (base, head_new]
      const bool in1 = w1[2] - base - 1 < span || w1[2] == kLockedLoc;
      const bool in2 = w2[2] - base - 1 < span || w2[2] == kLockedLoc;
      const bool m1 = w1[0] == d.lo && w1[1] == d.hi && !in1;
      const bool m2 = w2[0] == d.lo && w2[1] == d.hi && !in2;
      const bool v1 = !entry_free(w1[2], (uint32_t)(w1[3] >> 32), head_new, cap, now);
      const bool v2 = !entry_free(w2[2], (uint32_t)(w2[3] >> 32), head_new, cap, now);
      const uint32_t mmask = (uint32_t)((__ballot(m1) >> gbase) & 0xfull) |
                             ((uint32_t)((__ballot(m2) >> gbase) & 0xfull) << 4);
      const uint32_t lmask = (uint32_t)((__ballot(v1) >> gbase) & 0xfull) |
                             ((uint32_t)((__ballot(v2) >> gbase) & 0xfull) << 4);
      int target;
      if (fr) {
        // the move's source entry: the one whose loc is still the old item's (a SET, DELETE
        // or eviction since the hand read the index replaced it: the reinsertion is dropped)
        const uint32_t fmask = (uint32_t)((__ballot(w1[2] == fr) >> gbase) & 0xfull) |
                               ((uint32_t)((__ballot(w2[2] == fr) >> gbase) & 0xfull) << 4);
        if (!fmask) {
          if (l4 == 0) ++moved_away;
          break;
        }
        target = __ffs(fmask) - 1;
      } else if (mmask) {
        target = __ffs(mmask) - 1;
      } else {
        const uint32_t dead = ~lmask & 0xffu;
        if (dead) {
          const int live1 = __popc(lmask & 0xfu), live2 = __popc(lmask & 0xf0u);
          const uint32_t pref = __popc(dead & 0x0fu) >= 2
                                    ? (dead & 0x0fu)
                                    : (live2 < live1 ? (dead & 0xf0u) : (dead & 0x0fu));
          target = __ffs(pref ? pref : dead) - 1;
        } else {
          // all 8 live: k_set_fixup moves one of them or evicts (relocate_one's policy,
          // one lane per row there: here it cost 40 B/lane of scratch at 64 VGPRs)
          if (l4 == 0) claim[i] = kClaimDeferred;
          break;
        }
      }
      const uint64_t e1 = __shfl(w1[2], gbase + (target & 3));
      const uint64_t e2 = __shfl(w2[2], gbase + (target & 3));
      const uint64_t expected = target < 4 ? e1 : e2;
      Entry* const slot = index + (target < 4 ? b1 : b2) * kEntriesPerBucket + (target & 3);
      int ok = 0;
      if (l4 == 0) {
        const unsigned long long prev = atomicCAS(
            reinterpret_cast<unsigned long long*>(&slot->loc), (unsigned long long)expected,
            (unsigned long long)myloc);
        if (prev == expected) {
          slot->d0 = d.lo;
          slot->d1 = d.hi;
          *reinterpret_cast<uint64_t*>(&slot->vlen) = pack2(myvlen, myexp);
          claim[i] = (uint32_t)(slot - index);
          ok = 1;
          bytes += myvlen;
        }
      }
      ok = __shfl(ok, gbase);
      if (ok) break;
      if (fr) {  // the entry moved on between the read and the CAS: drop the reinsertion
        if (l4 == 0) ++moved_away;
        break;
      }
      if (attempt == 15 && l4 == 0) ++lost;  // bucket pair contended past the retry budget
    }
  }
  block_count(ctr, evicted, &CacheCounters::set_evicted, bytes, &CacheCounters::set_bytes, lost,
              &CacheCounters::set_dropped);
  if (from) block_count(ctr, moved_away, &CacheCounters::reinsert_lost);
}

// One row k_set_index deferred (its pair all live), by one thread inside k_set_fixup:
// relocate_one's policy lane-serial — move the first entry (bucket 1, then bucket 2; not
// another claim of this batch) whose other bucket has a dead slot, copying it there
// before its slot is taken, else evict the oldest. Other deferred rows are the only
// concurrent writers that can touch these non-batch entries, hence the CAS retries.
__device__ void deferred_insert(const Digest& d, uint64_t myloc, uint64_t myword,
                                Entry* __restrict__ index, uint64_t mask, uint64_t base,
                                uint64_t span, uint64_t head_new, uint64_t cap, uint32_t now,
                                uint32_t* __restrict__ claim_out, unsigned long long& evicted,
                                unsigned long long& bytes, unsigned long long& lost) {
  const uint64_t bb[2] = {bucket1(d, mask), bucket2(d, mask)};
  for (int attempt = 0; attempt < 16; ++attempt) {
    Entry* target = nullptr;
    Entry* copy = nullptr;
    Entry* victim = nullptr;  // the eviction fallback: the oldest entry not of this batch
    uint64_t expected = 0, oldest = ~0ull;
    bool evict = false;
    for (int e = 0; e < 8 && !target; ++e) {  // a slot that died or freed up meanwhile
      Entry* const x = index + bb[e >> 2] * kEntriesPerBucket + (e & 3);
      const uint64_t l = agent_load(&x->loc);
      const uint64_t w = agent_load(reinterpret_cast<const uint64_t*>(&x->vlen));
      if (l == kLockedLoc) continue;  // another inserter's copy in flight
      if (!entry_live(l, (uint32_t)(w >> 32), head_new, cap, now)) {
        target = x;
        expected = l;
      } else if (l - base - 1 >= span && l < oldest) {
        oldest = l;
        victim = x;
      }
    }
    if (!target) {
      for (int e = 0; e < 8 && !target; ++e) {
        Entry* const x = index + bb[e >> 2] * kEntriesPerBucket + (e & 3);
        const uint64_t l = agent_load(&x->loc);
        if (l - base - 1 < span || l == kLockedLoc) continue;  // a claim of this batch / a copy
        const Digest de{agent_load(&x->d0), agent_load(&x->d1)};
        const uint64_t w = agent_load(reinterpret_cast<const uint64_t*>(&x->vlen));
        // the words belong to loc l only if l is still there (a concurrent insert may have
        // replaced the entry between the loads): re-check after reading them
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (agent_load(&x->loc) != l) continue;
        const uint64_t x1 = bucket1(de, mask), x2 = bucket2(de, mask);
        const uint64_t own = bb[e >> 2];
        const uint64_t ob = x1 == own ? x2 : (x2 == own ? x1 : own);
        if (ob == own) continue;
        for (int k = 0; k < 4; ++k) {
          Entry* const a = index + ob * kEntriesPerBucket + k;
          const uint64_t al = agent_load(&a->loc);
          const uint64_t aw = agent_load(reinterpret_cast<const uint64_t*>(&a->vlen));
          if (!entry_free(al, (uint32_t)(aw >> 32), head_new, cap, now)) continue;
          if (copy_entry(a, al, de.lo, de.hi, l, w)) {
            target = x;
            expected = l;
            copy = a;
          }
          break;  // copied, or lost the slot: take the next candidate
        }
      }
      if (!target && victim) {
        target = victim;
        expected = oldest;
        evict = true;
      }
    }
    if (!target) continue;
    // the row's own entry goes in through the same lock: a concurrent copy can never
    // land its words in the slot between this CAS and the words below
    if (copy_entry(target, expected, d.lo, d.hi, myloc, myword)) {
      *claim_out = (uint32_t)(target - index);
      evicted += evict ? 1 : 0;
      bytes += (uint32_t)myword;
      return;
    }
    if (copy) drop_entry(copy, expected);  // the moved key changed meanwhile: drop the copy
  }
  ++lost;
}

// After k_set_index (kernel boundary: every CAS and word write is visible): each entry
// whose loc is still the one a row of this batch claimed gets that row's digest and
// vlen|expire words again, so no entry pairs one key's digest with another key's loc.
// Rows k_set_index deferred (kClaimDeferred: all 8 slots of the pair live) are inserted
// here first, by deferred_insert.
__global__ __launch_bounds__(kBlock) void k_set_fixup(
    const Digest* __restrict__ keys, int64_t n, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ vlen, const uint32_t* __restrict__ expire,
    const uint64_t* __restrict__ head_ptr, uint32_t* __restrict__ claim,
    Entry* __restrict__ index, const uint64_t* __restrict__ size, uint64_t* __restrict__ ring,
    uint64_t rmask, const uint64_t* __restrict__ ring_tail, uint64_t* __restrict__ ring_tail_next,
    const uint64_t* __restrict__ cnt_off, uint64_t* __restrict__ head_host, uint64_t mask,
    uint64_t cap, uint32_t now, CacheCounters* __restrict__ ctr) {
  const uint64_t base = *head_ptr;
  // item-start ring (CLOCK hand input): every stored row takes the next ring entry in row
  // order = log order (cnt_off: exclusive count of stored rows); the new head goes to the
  // pinned host slot the host's reclaim decision reads
  const uint64_t rtail = ring ? *ring_tail : 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (ring) *ring_tail_next = rtail + cnt_off[n];
    if (head_host)
      __hip_atomic_store(head_host, base + off[n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (ring)
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock)
      if (size[i]) ring[(rtail + cnt_off[i]) & rmask] = base + off[i] + 0;
  unsigned long long evicted = 0, lost = 0, bytes = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    // a row that stored nothing claimed nothing (and past a hand's effective window
    // k_set_index did not reset its claim word)
    if (!size[i]) continue;
    uint32_t c = claim[i];
    if (c == kClaimDeferred) {
      claim[i] = ~0u;
      deferred_insert(keys[i], base + off[i] + 1, pack2(vlen[i], expire ? expire[i] : 0u), index,
                      mask, base, off[n], base + off[n], cap, now, claim + i, evicted, bytes,
                      lost);
      continue;  // its words are final (deferred rows are not re-claimed by the batch)
    }
    if (c == ~0u) continue;
    Entry* const e = index + c;
    if (e->loc != base + off[i] + 1) continue;  // evicted again within the batch
    const Digest d = keys[i];
    e->d0 = d.lo;
    e->d1 = d.hi;
    *reinterpret_cast<uint64_t*>(&e->vlen) = pack2(vlen[i], expire ? expire[i] : 0u);
  }
  block_count(ctr, evicted, &CacheCounters::set_evicted, lost, &CacheCounters::set_dropped, bytes,
              &CacheCounters::set_bytes);
}

// ---------------------------------------------------------------------------------
// Small SET batches (the proxy's fills, memcached sets): the whole chain above in ONE
// workgroup and one launch instead of six — dedupe in an LDS hash table (last writer of
// a digest wins, as k_set_dedupe), sizes and both scans in LDS, the log claim, the append
// (records synthesised like k_segcopy<1>), then, behind an agent-scope release, the
// index insert (index_insert, exactly k_set_index's policy), the fix-up, the CLOCK ring
// entries and the head publication. Rows: kSmallSetRows at most, one per thread.
// ---------------------------------------------------------------------------------
constexpr int kSmallSetRows = kBlock;
constexpr int kSetSmallU = 16;  // 16-B chunks in flight per lane in the append

__global__ __launch_bounds__(kBlock) void k_set_small(
    const Digest* __restrict__ keys, const uint8_t* __restrict__ values,
    const uint64_t* __restrict__ val_off, const uint32_t* __restrict__ vlen,
    const uint32_t* __restrict__ flags, const uint32_t* __restrict__ expire, int n,
    uint32_t max_item, Entry* __restrict__ index, uint64_t mask,
    const uint64_t* __restrict__ head_ptr, uint64_t* __restrict__ head_next,
    unsigned long long* __restrict__ claim_word, uint64_t cap, uint32_t now,
    uint8_t* __restrict__ log, uint64_t* __restrict__ ring, uint64_t rmask,
    const uint64_t* __restrict__ ring_tail, uint64_t* __restrict__ ring_tail_next,
    uint64_t* __restrict__ head_host, CacheCounters* __restrict__ ctr) {
  constexpr int kT = 2 * kSmallSetRows;  // dedupe table slots
  __shared__ unsigned long long s_tk[kT];
  __shared__ int s_tw[kT];
  __shared__ uint64_t s_off[kSmallSetRows + 1];
  __shared__ uint64_t s_src[kSmallSetRows];
  __shared__ uint32_t s_cnt[kSmallSetRows + 1];
  __shared__ uint32_t s_claim[kSmallSetRows];
  __shared__ Digest s_key[kSmallSetRows];
  __shared__ uint32_t s_vl[kSmallSetRows];
  __shared__ uint32_t s_ex[kSmallSetRows];
  __shared__ unsigned long long s_w[2][kBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int k = tid; k < kT; k += kBlock) {
    s_tk[k] = 0ull;
    s_tw[k] = -1;
  }
  __syncthreads();
  // ---- dedupe: last writer of a digest (lo word, as k_set_dedupe) wins
  const bool row = tid < n;
  const uint32_t vl = row ? vlen[tid] : kSkipVlen;
  const bool skip = vl == kSkipVlen;
  Digest d{0, 0};
  int slot = -1;
  s_vl[tid] = vl;
  s_ex[tid] = row && expire ? expire[tid] : 0u;
  if (row && !skip) {
    d = keys[tid];
    s_key[tid] = d;
    const unsigned long long key = d.lo ? d.lo : 1ull;
    uint32_t t = (uint32_t)fmix64(key) & (kT - 1);
    for (int probe = 0; probe < kT; ++probe) {
      const unsigned long long prev = atomicCAS(&s_tk[t], 0ull, key);
      if (prev == 0ull || prev == key) {
        atomicMax(&s_tw[t], tid);
        slot = (int)t;
        break;
      }
      t = (t + 1) & (kT - 1);
    }
  }
  __syncthreads();
  const bool win = slot >= 0 && s_tw[slot] == tid && vl <= max_item;
  const uint64_t sz = win ? item_bytes(vl) : 0;
  // ---- exclusive scans of the sizes and of the stored-row count (CLOCK ring ordinals)
  uint64_t inc = sz;
  uint64_t incc = win ? 1 : 0;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const uint64_t o = __shfl_up(inc, dd), oc = __shfl_up(incc, dd);
    if (lane >= dd) {
      inc += o;
      incc += oc;
    }
  }
  if (lane == 63) {
    s_w[0][w] = inc;
    s_w[1][w] = incc;
  }
  __syncthreads();
  uint64_t pre = 0, prec = 0, tot = 0, totc = 0;
#pragma unroll
  for (int k = 0; k < kBlock / 64; ++k) {
    if (k < w) {
      pre += s_w[0][k];
      prec += s_w[1][k];
    }
    tot += s_w[0][k];
    totc += s_w[1][k];
  }
  const uint64_t my_off = pre + inc - sz;
  s_off[tid] = my_off;
  s_cnt[tid] = (uint32_t)(prec + incc - (win ? 1 : 0));
  s_src[tid] = row && win ? (uint64_t)(uintptr_t)values + val_off[tid] : 0;
  if (tid == 0) {
    s_off[kSmallSetRows] = tot;
    s_cnt[kSmallSetRows] = (uint32_t)totc;
  }
  const uint64_t base = *head_ptr;
  const uint64_t head_new = base + tot;
  // ---- claim the bytes the append writes (the edge server re-checks against it)
  if (tid == 0 && tot) {
    atomicMax(claim_word, (unsigned long long)head_new);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // ---- append: 16-B chunks of the batch's records, header words synthesised. The values
  //      are often in mapped host memory (the proxy's zero-copy staging): kSetSmallU loads
  //      in flight per lane, issued before their stores, so one workgroup is not bound by
  //      one PCIe round trip per chunk.
  const int64_t nch = (int64_t)(tot >> 4);
  const uint64_t pbase = base % cap;
  for (int64_t c0 = 0; c0 < nch; c0 += (int64_t)kBlock * kSetSmallU) {
    u32x4 v[kSetSmallU];
    uint8_t* dst[kSetSmallU];
#pragma unroll
    for (int u = 0; u < kSetSmallU; ++u) {
      const int64_t c = c0 + (int64_t)u * kBlock + tid;
      dst[u] = nullptr;
      if (c >= nch) continue;
      const uint64_t x = (uint64_t)c << 4;
      int lo = 0, hi = n - 1;  // last row with s_off <= x: the record holding byte x
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= x) lo = mid;
        else hi = mid - 1;
      }
      const uint64_t wofs = x - s_off[lo];
      const uint64_t p = pbase + s_off[lo];
      dst[u] = log + (p >= cap ? p - cap : p) + wofs;
      if (wofs == 0) {
        const Digest k = s_key[lo];
        v[u] = u32x4{(uint32_t)k.lo, (uint32_t)(k.lo >> 32), (uint32_t)k.hi,
                     (uint32_t)(k.hi >> 32)};
      } else if (wofs == 16) {
        v[u] = u32x4{s_vl[lo], flags ? flags[lo] : 0u, s_ex[lo], kItemMagic};
      } else {
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
            (uintptr_t)s_src[lo] + (wofs - kItemHeaderBytes)));
      }
    }
#pragma unroll
    for (int u = 0; u < kSetSmallU; ++u)
      if (dst[u]) *reinterpret_cast<u32x4*>(dst[u]) = v[u];
  }
  // ---- release the records before any index entry can point at them
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // ---- index insert, 4 lanes per row
  unsigned long long evicted = 0, bytes = 0, lost = 0;
  for (int i0 = 0; i0 < n; i0 += kBlock / 4) {
    const int i = i0 + (tid >> 2);
    const bool act = i < n && s_off[i + 1] != s_off[i];
    if ((tid & 3) == 0 && i < n) s_claim[i] = ~0u;
    index_insert(act, act ? s_key[i] : Digest{0, 0}, base + s_off[i] + 1, act ? s_vl[i] : 0u,
                 act ? s_ex[i] : 0u, s_claim + (i < n ? i : 0), index, mask, base, head_new,
                 cap, now, evicted, bytes, lost);
  }
  // ---- fix-up (entries a later row of this batch re-claimed), CLOCK ring, head
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (row && win) {
    const uint32_t c = s_claim[tid];
    const uint64_t myloc = base + my_off + 1;
    if (c != ~0u) {
      Entry* const e = index + c;
      if (__hip_atomic_load(&e->loc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == myloc) {
        e->d0 = d.lo;
        e->d1 = d.hi;
        *reinterpret_cast<uint64_t*>(&e->vlen) = pack2(vl, s_ex[tid]);
      }
    }
  }
  const uint64_t rtail = ring ? *ring_tail : 0;
  if (ring && row && win) ring[(rtail + s_cnt[tid]) & rmask] = base + my_off;
  if (tid == 0) {
    *head_next = head_new;
    if (ring) *ring_tail_next = rtail + s_cnt[kSmallSetRows];
    __hip_atomic_store(head_host, head_new, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  block_count(ctr, (unsigned long long)(row && !skip ? 1 : 0), &CacheCounters::set_ops,
              (unsigned long long)(row && !skip && !win ? 1 : 0), &CacheCounters::set_dropped);
  block_count(ctr, evicted, &CacheCounters::set_evicted, bytes, &CacheCounters::set_bytes, lost,
              &CacheCounters::set_dropped);
}

// ---------------------------------------------------------------------------------
// CLOCK eviction: second chances for referenced items before the log overwrites them
// ---------------------------------------------------------------------------------
// The log is a FIFO: a SET batch of B bytes overwrites the oldest B bytes. Before it
// runs, the hand walks the item-start ring (one entry per stored item, in log order)
// from the oldest item: an item whose index entry still points at it, is unexpired and
// was read since the hand last passed it (kRefBit) is re-appended at the head in front
// of the batch (a reinsertion, which also clears the bit); the rest are left to the
// overwrite. The hand stops at the first entry c whose item the overwrite — now
// B + R bytes, R = reinserted bytes of entries [0, c) — does not reach:
//     loc_c >= head - cap + R_c + B        (entries [0, c) consumed)
// R is capped by the reinsertion budget `rmax` (hot items past it just age out).
// Kernels (two launches: the hand is a dependent chain on the SET stream, and a launch
// queued while the GET lookup holds every CU waits for its workgroups to retire):
//   k_rc_scan  per window entry: its loc and hot size (h, 0 when not referenced), a block
//              partial of h, the batch's bytes B; hot entries' rows of the combined batch
//              are written from the header it read (no second header read), the others as
//              skip rows, and the batch's own rows are copied behind the window.
//   k_rc_emit  the exclusive scan of h (block partials of the previous launch + a block
//              scan) gives each entry its reinsertion offset hx and its cut test
//                  meets_j = loc_j + cap >= head + B + min(hx_j, rmax) + lead
//              which is monotone over valid entries (a valid entry's loc grows at least by
//              the hot bytes of the entries before it), so an entry is consumed iff it does
//              not meet the bound: the pick needs no grid-wide cut. The first meeting entry
//              is min-reduced (an atomic, no fence: k_set_dedupe, the next launch on the
//              stream, advances the hand and resets the control words — a last-workgroup
//              hand-off here needs an agent-scope release per workgroup, an L2 write-back
//              beside the gather).
// Lead mode (a log of at least 16 x (batch bound + rmax), HBM serving shards): the hand runs
// lead = rmax + 1.25 B ahead of the overwrite and decides about entries about two batches
// before the log overwrites them. A pick then lies beyond everything the batch can
// overwrite, so the log append copies it straight from its old place — one copy per
// reinserted byte — and, above all, a referenced object has moved before any lookup's
// reserve (the next SET's bytes + rmax, treated as misses) reaches its old copy: without the
// lead every hot object near the tail missed for a step or two per lap (the 5 GiB shard's
// hit ratio 0.963 -> 0.998, profiles/r5x_hand_lead). On a small log (a batch a sizeable
// share of it) deciding two batches early costs hit ratio instead, so there the hand has no
// lead and
//   k_segcopy<2> stages the picked records in scratch (their old bytes lie in the region
//              the batch overwrites, which the previous step's gather may still read).
// The combined batch then runs the ordinary SET chain (dedupe lets the batch's own SETs
// win over a reinsertion of the same key). Host twin: HostCache::reclaim.
constexpr unsigned long long kRcCount = 1ull << 43;  // k_rc_scan / k_rc_emit packed counts
constexpr int kRcScanK = 1;  // window entries per lane of k_rc_scan (SHELLAC_RCSCAN_K)

struct RcArgs {
  const uint64_t* ring;
  uint64_t rmask;
  const uint64_t* ring_tail;  // the last batch whose ring entries are written (see store)
  // [0] hand, [1] batch bytes B, [2] first meeting entry, [3] scanned, [4] entries the last
  // batch consumed (the adaptive window, layout.h hand_window_eff), [5 + parity] the effective
  // window of the batch in hand buffer `parity` (its index pass stops there)
  unsigned long long* ctl;
  int64_t W;      // the window's rows
  int64_t n_new;  // the batch's rows (the window's base 2n + 256; reinsertions <= W - n)
  int parity;     // the hand buffer's: ctl[5 + parity] = this batch's effective window
  const uint64_t* head_ptr;  // the claim word: the head the queued appends will reach
  uint64_t cap;
  uint32_t now;
  uint64_t rmax;
  // 1: the hand runs `lead` = rmax + 1.25 B ahead of the overwrite and its picks are
  // copied straight from the log; 0: no lead, picks staged through scratch (see below)
  uint64_t lead_mode;
};

// The combined SET batch (rows [0, W) reinsertions, [W, W + n) the batch). `from`: a
// picked reinsertion's old entry loc (its index insert is a move from it), 0 otherwise.
struct RcBatch {
  Digest* keys;
  uint64_t* voff;
  uint32_t* vlen;
  uint32_t* flags;
  uint32_t* expire;
  uint64_t* from;
};

// block_partial into part[at] (several 256-entry sub-blocks per workgroup)
__device__ __forceinline__ void block_partial_at(unsigned long long v, uint64_t* __restrict__ part,
                                                 int64_t at) {
  __shared__ unsigned long long s_p[kBlock / 64];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_p[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) t += s_p[k];
    part[at] = t;
  }
  __syncthreads();
}

// K window entries per lane (entries j = (blockIdx.x * K + k) * kBlock + threadIdx.x): the K
// ring -> header -> index chains are issued phase by phase, so each lane keeps K of them in
// flight — the window needs 1/K of the workgroups, which matters beside the gather, which
// holds most of the co-resident slots (the hand scan was latency-bound at 5 %
// of the HBM roofline). Every entry's decision is the single-entry rule's.
template <int K>
__global__ __launch_bounds__(kBlock) void k_rc_scan(RcArgs a, RcBatch cb, const uint8_t* __restrict__ log,
                                                    const Entry* __restrict__ index, uint64_t mask,
                                                    const Digest* __restrict__ keys,
                                                    const uint8_t* __restrict__ values,
                                                    const uint64_t* __restrict__ val_off,
                                                    const uint32_t* __restrict__ vlen_new,
                                                    const uint32_t* __restrict__ flags,
                                                    const uint32_t* __restrict__ expire,
                                                    int64_t n_new, uint32_t max_item,
                                                    uint64_t* __restrict__ rc_loc,
                                                    uint64_t* __restrict__ rc_h,
                                                    uint64_t* __restrict__ part_h) {
  const uint64_t hand = a.ctl[0], rtail = *a.ring_tail, head = *a.head_ptr;
  // the batch's own rows behind the window, and its bytes (upper bound: dedupe losers
  // included)
  unsigned long long best = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n_new;
       i += (int64_t)gridDim.x * kBlock) {
    const uint32_t v = vlen_new[i];
    if (v != kSkipVlen && v <= max_item) best += item_bytes(v);
    const int64_t r = a.W + i;
    cb.keys[r] = keys[i];
    cb.voff[r] = (uint64_t)(uintptr_t)values + val_off[i];
    cb.vlen[r] = v;
    cb.flags[r] = flags ? flags[i] : 0u;
    cb.expire[r] = expire ? expire[i] : 0u;
    cb.from[r] = 0;
  }
  const uint64_t avail = rtail - hand;
  // the entries this hand examines (a detached hand sees the ring tail of the batch before
  // the previous one; rows past the effective window are skip rows): the advance consumes
  // at most these
  const int64_t weff = hand_window_eff(a.n_new, a.ctl[4]);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.ctl[3] = (uint64_t)weff < avail ? (uint64_t)weff : avail;
    a.ctl[5 + a.parity] = (unsigned long long)weff;
  }
  int64_t j[K];
  uint64_t l[K], loc[K], h[K];
  uint4 w0[K], w1[K];
  // 1. the ring entries
#pragma unroll
  for (int k = 0; k < K; ++k) {
    j[k] = ((int64_t)blockIdx.x * K + k) * kBlock + threadIdx.x;
    l[k] = kRingSkip;
    loc[k] = kRingSkip;
    h[k] = 0;
    w0[k] = w1[k] = make_uint4(0, 0, 0, 0);
    if (j[k] < weff && (uint64_t)j[k] < avail) {
      const uint64_t idx = hand + (uint64_t)j[k];
      l[k] = rtail - idx <= a.rmask + 1 ? a.ring[idx & a.rmask] : kRingSkip;
    }
  }
  // 2. the headers of the intact (not overwritten) items
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (l[k] != kRingSkip && head <= l[k] + a.cap) {
      const uint4* hp = reinterpret_cast<const uint4*>(log + l[k] % a.cap);
      w0[k] = hp[0];
      w1[k] = hp[1];
    }
  // 3. the entry pointing at each item: first bucket first, the second only when the first
  // has none (SETs fill the first bucket first, so one 128-B line per window entry usually
  // settles it). A digest match alone does not settle it: a dead entry keeps its digest, so
  // a key can match in one bucket while its live entry is in the other (stopping there
  // dropped live, referenced items: test_serve_steps_return_ground_truth_records). Each
  // entry's {loc, vlen, expire} half is one 16-B load, and a bucket's four are issued
  // together, the K entries' first buckets together (no insert runs beside the hand: the SET
  // chain is on this stream; a concurrent lookup only sets reference bits, read either way)
  uint4 hv[K][kEntriesPerBucket];
  bool found[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    found[k] = false;
    if (l[k] != kRingSkip && w1[k].w == kItemMagic) {
      loc[k] = l[k];
      const Digest d{pack2(w0[k].x, w0[k].y), pack2(w0[k].z, w0[k].w)};
      const uint64_t b = bucket1(d, mask);
#pragma unroll
      for (int e = 0; e < (int)kEntriesPerBucket; ++e)
        hv[k][e] = reinterpret_cast<const uint4*>(index + b * kEntriesPerBucket + e)[1];
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (loc[k] == kRingSkip) continue;
#pragma unroll
    for (int e = 0; e < (int)kEntriesPerBucket; ++e)
      if (pack2(hv[k][e].x, hv[k][e].y) == loc[k] + 1) {
        found[k] = true;
        if ((hv[k][e].z & kRefBit) && (hv[k][e].w == 0 || hv[k][e].w > a.now))
          h[k] = item_bytes(w1[k].x);
      }
    if (!found[k]) {
      const Digest d{pack2(w0[k].x, w0[k].y), pack2(w0[k].z, w0[k].w)};
      const uint64_t b = bucket2(d, mask);
      uint4 h2[kEntriesPerBucket];
#pragma unroll
      for (int e = 0; e < (int)kEntriesPerBucket; ++e)
        h2[e] = reinterpret_cast<const uint4*>(index + b * kEntriesPerBucket + e)[1];
#pragma unroll
      for (int e = 0; e < (int)kEntriesPerBucket; ++e)
        if (pack2(h2[e].x, h2[e].y) == loc[k] + 1) {
          if ((h2[e].z & kRefBit) && (h2[e].w == 0 || h2[e].w > a.now)) h[k] = item_bytes(w1[k].x);
        }
    }
  }
  // 4. the rows
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (j[k] >= weff && j[k] < a.W) {
      // a row past the effective window: a skip row (the SET chain reads nothing else of a
      // row whose vlen says skip; k_rc_emit reads no rc_loc / rc_h past the examined entries)
      cb.vlen[j[k]] = kSkipVlen;
    } else if (j[k] < a.W) {
      rc_loc[j[k]] = loc[k];
      rc_h[j[k]] = h[k];
      // a hot entry's row from the header just read (k_rc_emit fills in its value pointer
      // or turns it into a skip row); every other entry is a skip row already
      cb.keys[j[k]] = h[k] ? Digest{pack2(w0[k].x, w0[k].y), pack2(w0[k].z, w0[k].w)} : Digest{0, 0};
      cb.voff[j[k]] = 0;
      cb.vlen[j[k]] = h[k] ? w1[k].x : kSkipVlen;
      cb.flags[j[k]] = h[k] ? w1[k].y : 0u;
      cb.expire[j[k]] = h[k] ? w1[k].z : 0u;
      cb.from[j[k]] = 0;
    }
    // hot bytes and (bits 43+) hot entries of each 256-entry sub-block, scanned by k_rc_emit
    block_partial_at(h[k] ? h[k] + kRcCount : 0ull, part_h, (int64_t)blockIdx.x * K + k);
  }
  // batch bytes: one atomic per block
  __shared__ unsigned long long s_b[kBlock / 64];
  best = wave_sum(best);
  if ((threadIdx.x & 63) == 0) s_b[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) t += s_b[k];
    if (t) atomicAdd(&a.ctl[1], t);
  }
}

__global__ __launch_bounds__(kBlock) void k_rc_emit(RcArgs a, RcBatch cb,
                                                    const uint8_t* __restrict__ log,
                                                    uint64_t* __restrict__ rc_loc,
                                                    uint64_t* __restrict__ rc_h,
                                                    const uint64_t* __restrict__ part_h,
                                                    uint64_t* __restrict__ rc_hx,
                                                    const uint8_t* __restrict__ scratch,
                                                    CacheCounters* __restrict__ ctr) {
  __shared__ unsigned long long s_w[kBlock / 64];
  __shared__ unsigned long long s_pre;
  // lead mode: a workgroup wholly past the entries the hand examined (k_rc_scan's count)
  // has nothing to pick, cut or plan (its rows are skip rows already)
  if (a.lead_mode && (uint64_t)blockIdx.x * kBlock >= a.ctl[3]) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long pre = 0;
  for (unsigned b = threadIdx.x; b < blockIdx.x; b += kBlock) pre += part_h[b];
  pre = wave_sum(pre);
  if (lane == 0) s_w[w] = pre;
  __syncthreads();
  if (threadIdx.x == 0) s_pre = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool examined = j < a.W && (uint64_t)j < a.ctl[3];
  const uint64_t h = examined ? rc_h[j] : 0;
  const unsigned long long hp = h ? h + kRcCount : 0ull;  // bytes | hot entries << 43
  unsigned long long inc = hp;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  __syncthreads();  // s_w reuse
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  unsigned long long hxp = s_pre + inc - hp;
  for (int k = 0; k < w; ++k) hxp += s_w[k];
  // hot bytes and hot entries before entry j
  const unsigned long long hx = hxp & (kRcCount - 1), hc = hxp / kRcCount;
  bool meets = false;
  unsigned long long nre = 0, bre = 0;
  if (j < a.W) {
    const uint64_t loc = examined ? rc_loc[j] : kRingSkip;
    const uint64_t r = hx < a.rmax ? hx : a.rmax;
    const uint64_t head = *a.head_ptr, bb = a.ctl[1];
    const uint64_t lead = a.lead_mode ? a.rmax + bb + (bb >> 2) : 0;
    meets = loc != kRingSkip && loc + a.cap >= head + bb + r + lead;
    bool pick = false;
    if (h) {
      // lead mode: a pick must lie beyond everything the batch can overwrite (its bytes +
      // the whole budget); an unsafe one (the hand not yet `lead` ahead: the first steps
      // after the log fills, a batch much larger than the last) ages out
      if (!meets && hx + h <= a.rmax && hc < (unsigned long long)(a.W - a.n_new) &&
          (!a.lead_mode || loc + a.cap >= head + bb + a.rmax)) {
        pick = true;
        cb.voff[j] = a.lead_mode ? (uint64_t)(uintptr_t)log + loc % a.cap + kItemHeaderBytes
                                 : (uint64_t)(uintptr_t)scratch + hx + kItemHeaderBytes;
        cb.from[j] = loc + 1;  // indexed as a move from the entry that points here
        ++nre;
        bre += cb.vlen[j];
      } else {
        cb.vlen[j] = kSkipVlen;  // consumed past the budget or unsafe, or not consumed
      }
    }
    if (!a.lead_mode) {
      // the staging copy's plan (k_segcopy<2>, the next launch): entry j's record goes
      // from its log offset to scratch + hx, only when picked (a zero length leaves a gap)
      rc_hx[j] = hx;
      rc_h[j] = pick ? h : 0;
      rc_loc[j] = pick ? loc % a.cap : 0;
      if (j == a.W - 1) rc_hx[a.W] = hx + h;
    }
  }
  // only the first entry meeting the bound matters: one atomic per wave (its lowest lane)
  const unsigned long long mb = __ballot(meets);
  if (mb && lane == __ffsll((long long)mb) - 1) atomicMin(&a.ctl[2], (unsigned long long)j);
  block_count(ctr, nre, &CacheCounters::reinserted, bre, &CacheCounters::reinsert_bytes);
}

// The hand's advance past the consumed entries (k_set_dedupe's block 0, the launch after
// k_rc_emit): consumed = the first entry meeting the bound (none: the whole window).
struct RcAdvance {
  unsigned long long* ctl = nullptr;  // null: this SET batch ran no hand
  const uint64_t* ring_tail = nullptr;
  uint64_t rmask = 0;
  int64_t W = 0;
  const uint64_t* ring = nullptr;
  const uint64_t* head = nullptr;  // the claim word (the head before this batch's append)
  uint64_t cap = 0;
  int catch_up = 1;  // 0: tests only (debug_set_hand), the hand never jumps
};

// A hand behind the overwrite (batches that skipped it while the log filled, e.g. a
// populate that queued dozens of stores before the first completed, or a burst it could not
// keep up with) would spend its windows on items already overwritten while referenced ones
// reach the overwrite unexamined: it jumps to the first entry the overwrite has not reached.
// Ring locations grow along the ring; a skip entry ends the search early (conservative).
// One dependent load when the hand is where it should be; a binary search otherwise.
// HostCache::reclaim_locked does the same.
__device__ __forceinline__ uint64_t hand_catch_up(const uint64_t* ring, uint64_t rmask,
                                                  uint64_t hand, uint64_t rtail, uint64_t head,
                                                  uint64_t cap) {
  auto over = [&](uint64_t idx) {
    const uint64_t l = ring[idx & rmask];
    return l != kRingSkip && head > l + cap;
  };
  if (hand >= rtail || !over(hand)) return hand;
  uint64_t lo = hand + 1, hi = rtail;  // over(lo - 1); the first entry not over in [lo, hi]
  while (lo < hi) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (over(mid)) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void rc_advance(const RcAdvance& r) {
  const uint64_t rtail = *r.ring_tail;
  const uint64_t hand0 = r.ctl[0];
  const uint64_t weff = r.ctl[3];  // the entries the hand examined (k_rc_scan)
  const unsigned long long cut = r.ctl[2];
  const uint64_t consumed = cut != ~0ull && cut < weff ? cut : weff;
  uint64_t hand = hand0 + consumed;
  if (rtail - hand > r.rmask + 1) hand = rtail - (r.rmask + 1);  // ring lapped the hand
  if (r.catch_up) hand = hand_catch_up(r.ring, r.rmask, hand, rtail, *r.head, r.cap);
  r.ctl[0] = hand;
  r.ctl[1] = 0;
  r.ctl[2] = ~0ull;
  r.ctl[3] = 0;
  r.ctl[4] = consumed;  // the next batch's window (hand_window_eff)
}

// SET dedupe (last writer of a digest wins). `adv`: the CLOCK hand step before this batch
// (k_rc_emit) left its cut in the control words; block 0 advances the hand.
__global__ __launch_bounds__(kBlock) void k_set_dedupe(const Digest* __restrict__ keys,
                                                       const uint32_t* __restrict__ vlen, int64_t n,
                                                       unsigned long long* __restrict__ tk,
                                                       int* __restrict__ tw, uint32_t tmask,
                                                       uint32_t* __restrict__ slot_of,
                                                       RcAdvance adv) {
  if (adv.ctl && blockIdx.x == 0 && threadIdx.x == 0) rc_advance(adv);
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    if (vlen[i] == kSkipVlen) { slot_of[i] = 0; continue; }
    const unsigned long long key = keys[i].lo ? keys[i].lo : 1ull;
    uint32_t s = (uint32_t)fmix64(key) & tmask;
    for (uint32_t probe = 0; probe <= tmask; ++probe) {
      const unsigned long long prev = atomicCAS(&tk[s], 0ull, key);
      if (prev == 0ull || prev == key) {
        atomicMax(&tw[s], (int)i);
        slot_of[i] = s;
        break;
      }
      s = (s + 1) & tmask;
    }
  }
}

// ---------------------------------------------------------------------------------
// DELETE / SWEEP
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_delete(const Digest* __restrict__ keys, int64_t n,
                                                   Entry* __restrict__ index, uint64_t mask,
                                                   const uint64_t* __restrict__ head_ptr,
                                                   uint64_t cap, uint32_t now,
                                                   uint8_t* __restrict__ found,
                                                   CacheCounters* __restrict__ ctr) {
  const int l16 = threadIdx.x & 15;
  const uint64_t head = *head_ptr;
  const int64_t ngroups = ((int64_t)gridDim.x * kBlock) >> 4;
  unsigned long long ops = 0, hits = 0;
  for (int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 4; i < n; i += ngroups) {
    const Digest d = keys[i];
    const uint64_t b = (l16 < 8) ? bucket1(d, mask) : bucket2(d, mask);
    Entry* const bucket = index + b * kEntriesPerBucket;
    const uint4 v = reinterpret_cast<const uint4*>(bucket)[l16 & 7];
    const uint64_t a = pack2(v.x, v.y), c = pack2(v.z, v.w);
    const uint64_t pa = __shfl_xor(a, 1), pc = __shfl_xor(c, 1);
    const bool even = (l16 & 1) == 0;
    int was_live = 0;
    if (even && a == d.lo && c == d.hi && pa != 0) {
      Entry* const slot = bucket + ((l16 & 7) >> 1);
      const unsigned long long prev =
          atomicCAS(reinterpret_cast<unsigned long long*>(&slot->loc), (unsigned long long)pa, 0ull);
      if (prev == pa && entry_live(pa, (uint32_t)(pc >> 32), head, cap, now)) was_live = 1;
    }
    const unsigned long long any = __ballot(was_live);
    const int gbase = threadIdx.x & 48;
    const int f = ((any >> gbase) & 0xffffull) != 0;
    if (l16 == 0) {
      ++ops;
      hits += f;
      if (found) found[i] = (uint8_t)f;
    }
  }
  block_count(ctr, ops, &CacheCounters::del_ops, hits, &CacheCounters::del_hits);
}

__global__ __launch_bounds__(kBlock) void k_sweep(Entry* __restrict__ index, uint64_t nslots,
                                                  const uint64_t* __restrict__ head_ptr,
                                                  uint64_t cap, uint32_t now,
                                                  unsigned long long* __restrict__ out,
                                                  CacheCounters* __restrict__ ctr) {
  const uint64_t head = *head_ptr;
  unsigned long long live = 0, bytes = 0, swept = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < nslots;
       k += (uint64_t)gridDim.x * kBlock) {
    Entry* const e = index + k;
    const uint64_t loc = e->loc;
    if (!loc) continue;
    const uint64_t ve = *reinterpret_cast<const uint64_t*>(&e->vlen);
    if (entry_live(loc, (uint32_t)(ve >> 32), head, cap, now)) {
      ++live;
      bytes += item_bytes(entry_vlen((uint32_t)ve));
    } else if (atomicCAS(reinterpret_cast<unsigned long long*>(&e->loc), (unsigned long long)loc,
                         0ull) == loc) {
      ++swept;
    }
  }
  block_count(ctr, swept, &CacheCounters::swept);
  live = wave_sum(live);
  bytes = wave_sum(bytes);
  if ((threadIdx.x & 63) == 0) {
    if (live) atomicAdd(&out[0], live);
    if (bytes) atomicAdd(&out[1], bytes);
  }
}


// Export the digests of all live entries (rebalancing / warm restore). One atomic
// per workgroup per pass reserves the output range; lanes write in block order.
__global__ __launch_bounds__(kBlock) void k_export(const Entry* __restrict__ index, uint64_t nslots,
                                                   const uint64_t* __restrict__ head_ptr,
                                                   uint64_t cap, uint32_t now,
                                                   Digest* __restrict__ out, uint64_t out_cap,
                                                   unsigned long long* __restrict__ counter) {
  __shared__ unsigned int s_wcnt[kBlock / 64];
  __shared__ unsigned long long s_base;
  const uint64_t head = *head_ptr;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t k0 = (uint64_t)blockIdx.x * kBlock; k0 < nslots; k0 += (uint64_t)gridDim.x * kBlock) {
    const uint64_t k = k0 + threadIdx.x;
    bool live = false;
    Digest d{0, 0};
    if (k < nslots) {
      const Entry e = index[k];
      live = entry_live(e.loc, e.expire, head, cap, now);
      d = Digest{e.d0, e.d1};
    }
    const unsigned long long m = __ballot(live);
    if (lane == 0) s_wcnt[w] = (unsigned int)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned int tot = 0;
      for (int i = 0; i < kBlock / 64; ++i) tot += s_wcnt[i];
      s_base = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    unsigned int before = 0;
    for (int i = 0; i < w; ++i) before += s_wcnt[i];
    if (live) {
      const uint64_t pos = s_base + before + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
      if (pos < out_cap) out[pos] = d;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------
// Digest / routing / permutation
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_digest(const uint8_t* __restrict__ bytes,
                                                   const int64_t* __restrict__ offs, int64_t n,
                                                   Digest* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t b = offs[i];
    out[i] = digest_bytes(bytes + b, (uint64_t)(offs[i + 1] - b));
  }
}

__global__ __launch_bounds__(kBlock) void k_route(const Digest* __restrict__ keys, int64_t n,
                                                  const uint32_t* __restrict__ pts,
                                                  const int32_t* __restrict__ owner, int32_t npts,
                                                  int32_t* __restrict__ dest,
                                                  int64_t* __restrict__ counts, int32_t nranks) {
  extern __shared__ unsigned long long s_cnt[];
  for (int r = threadIdx.x; r < nranks; r += kBlock) s_cnt[r] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const uint32_t p = ring_position(keys[i]);
    int lo = 0, hi = npts;  // first point >= p
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (pts[mid] < p) lo = mid + 1; else hi = mid;
    }
    const int r = owner[lo == npts ? 0 : lo];
    dest[i] = r;
    atomicAdd(&s_cnt[r], 1ull);
  }
  __syncthreads();
  for (int r = threadIdx.x; r < nranks; r += kBlock)
    if (s_cnt[r]) atomicAdd(reinterpret_cast<unsigned long long*>(&counts[r]), s_cnt[r]);
}

__global__ __launch_bounds__(kBlock) void k_scatter(const int32_t* __restrict__ dest,
                                                    const int64_t* __restrict__ base, int64_t n,
                                                    int64_t* __restrict__ cursor,
                                                    int64_t* __restrict__ perm) {
  const int lane = threadIdx.x & 63;
  for (int64_t i0 = (int64_t)blockIdx.x * kBlock; i0 < n; i0 += (int64_t)gridDim.x * kBlock) {
    const int64_t i = i0 + threadIdx.x;
    const bool act = i < n;
    const int d = act ? dest[i] : -1;
    // wave-aggregated slot reservation: one atomic per distinct destination per wave
    unsigned long long todo = __ballot(act);
    int64_t pos = 0;
    while (todo) {
      const int leader = __ffsll((long long)todo) - 1;
      const int ld = __shfl(d, leader);
      const unsigned long long same = __ballot(act && d == ld);
      int64_t start = 0;
      if (lane == leader)
        start = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(&cursor[ld]),
                                   (unsigned long long)__popcll(same));
      start = __shfl(start, leader);
      if (d == ld && act) {
        const unsigned long long below = same & ((1ull << lane) - 1ull);
        pos = base[ld] + start + __popcll(below);
      }
      todo &= ~same;
    }
    if (act) perm[i] = pos;
  }
}

__global__ __launch_bounds__(kBlock) void k_permute(const uint32_t* __restrict__ in,
                                                    const int64_t* __restrict__ perm, int64_t n,
                                                    int32_t words, uint32_t* __restrict__ out) {
  const int64_t total = n * words;
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kBlock) {
    const int64_t i = t / words, w = t - i * words;
    out[perm[i] * words + w] = in[t];
  }
}

// Records -> SET rows (see records_to_set in hbm_cache.h).
__global__ __launch_bounds__(kBlock) void k_records_to_set(
    const uint8_t* __restrict__ rec, const uint64_t* __restrict__ off,
    const uint64_t* __restrict__ size, const uint64_t* __restrict__ have, int64_t n,
    Digest* __restrict__ keys, uint64_t* __restrict__ val_off, uint32_t* __restrict__ vlen,
    uint32_t* __restrict__ flags, uint32_t* __restrict__ expire) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const bool skip = size[i] == 0 || (have && have[i] != 0);
    if (skip) {
      keys[i] = Digest{0, 0};
      val_off[i] = 0;
      vlen[i] = kSkipVlen;
      flags[i] = 0;
      expire[i] = 0;
      continue;
    }
    const uint4* hp = reinterpret_cast<const uint4*>(rec + off[i]);
    const uint4 w0 = hp[0], w1 = hp[1];
    keys[i] = Digest{pack2(w0.x, w0.y), pack2(w0.z, w0.w)};
    val_off[i] = off[i] + kItemHeaderBytes;
    vlen[i] = w1.x;
    flags[i] = w1.y;
    expire[i] = w1.z;
  }
}

// ---------------------------------------------------------------------------------
// MFMA hello (platform smoke)
// ---------------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

__global__ __launch_bounds__(64) void k_mfma_hello(const uint16_t* __restrict__ A,
                                                   const uint16_t* __restrict__ B,
                                                   float* __restrict__ C) {
  // tile t: A_t [32 x 16] row-major, B_t [16 x 32] row-major, C_t [32 x 32] row-major
  const int t = blockIdx.x, l = threadIdx.x, r = l & 31, h = l >> 5;
  const uint16_t* a = A + (size_t)t * 32 * 16;
  const uint16_t* b = B + (size_t)t * 16 * 32;
  u16x8_t av, bv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = a[r * 16 + 8 * h + j];      // A[row r][k = 8h + j]
    bv[j] = b[(8 * h + j) * 32 + r];    // B[k = 8h + j][col r]
  }
  f32x16_t acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, av),
                                                __builtin_bit_cast(bf16x8_t, bv), acc, 0, 0, 0);
  float* c = C + (size_t)t * 32 * 32;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    c[row * 32 + r] = acc[i];
  }
}

}  // namespace

// =====================================================================================
// Host side
// =====================================================================================
size_t device_scan_tmp_bytes(int64_t n) {
  size_t bytes = 0;
  HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr,
                                          (uint64_t*)nullptr, (int)(n + 1)));
  return bytes;
}

// k_offsets launch for sizes produced by `grid` workgroups over contiguous ranges.
void launch_offsets(const uint64_t* size, int64_t n, const uint64_t* part, int grid,
                    uint64_t* off, hipStream_t s, uint64_t* host_total = nullptr,
                    int64_t plen_override = 0, const uint64_t* part_cnt = nullptr,
                    uint64_t* cnt = nullptr, const uint64_t* claim_head = nullptr,
                    uint64_t* claim = nullptr) {
  const int64_t plen = plen_override > 0 ? plen_override : part_len(n, grid);
  const int q = (int)std::max<int64_t>(1, 2048 / std::max<int64_t>(plen, 1));
  const int g2 = (grid + q - 1) / q;
  hipLaunchKernelGGL(k_offsets, dim3(g2), dim3(kBlock), 0, s, size, n, part, grid, plen, q, off,
                     host_total, part_cnt, cnt, claim_head,
                     reinterpret_cast<unsigned long long*>(claim));
  HIP_OK(hipGetLastError());
}

void device_exclusive_scan(const uint64_t* in, uint64_t* out, int64_t n, void* tmp,
                           size_t tmp_bytes, hipStream_t s) {
  // in must be readable at [0, n]; the caller guarantees in[n] == 0.
  SH_CHECK(n + 1 < (int64_t)INT32_MAX, "scan too large");
  HIP_OK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, (int)(n + 1), s));
}

void segcopy(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off, int64_t n,
             uint8_t* dst, hipStream_t s, uint64_t dst_cap) {
  if (n <= 0) return;
  launch_segcopy<0>(s, src, src_off, dst_off, n, dst, nullptr, nullptr, nullptr, nullptr, nullptr,
                    dst_cap);
  HIP_OK(hipGetLastError());
}

void segcopy_dev(const uint64_t* src_off, const uint64_t* dst_off, const int64_t* n_dev,
                 uint8_t* dst, hipStream_t s, uint64_t dst_cap) {
  launch_segcopy<3>(s, nullptr, src_off, dst_off, (int64_t)0, dst, nullptr, nullptr, nullptr,
                    nullptr, reinterpret_cast<const uint64_t*>(n_dev), dst_cap);
  HIP_OK(hipGetLastError());
}

void segcopy_sized(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off,
                   const uint64_t* seg_len, int64_t n, uint8_t* dst, hipStream_t s, uint64_t cap) {
  if (n <= 0) return;
  launch_segcopy<2>(s, src, src_off, dst_off, n, dst, nullptr, nullptr, nullptr, nullptr,
                    seg_len, cap);
  HIP_OK(hipGetLastError());
}

int64_t coalesce_table_slots(int64_t n) {
  int64_t t = 1024;
  while (t < 2 * n) t <<= 1;
  return t;
}

void coalesce_keys(const Digest* keys, int64_t n, uint32_t* table, int64_t table_slots,
                   uint32_t* first, hipStream_t s, uint32_t* cslot, bool table_clean) {
  if (n <= 0) return;
  SH_CHECK(n < (1ll << 31), "coalesce: batch too large");
  SH_CHECK(table_slots >= 2 * n && (table_slots & (table_slots - 1)) == 0,
           "coalesce: table needs a power of two >= 2n slots");
  if (!table_clean) HIP_OK(hipMemsetAsync(table, 0, (size_t)table_slots * sizeof(uint32_t), s));
  const int64_t chunks = (n + kCoKeys - 1) / kCoKeys;
  hipLaunchKernelGGL(k_coalesce<false>, dim3((unsigned)chunks), dim3(kBlock), 0, s, keys, n,
                     (int64_t)kCoKeys, table, (uint32_t)(table_slots - 1), first, cslot,
                     nullptr, 0ull, nullptr, 0ull, 0ull, 0u, nullptr, nullptr, nullptr, nullptr,
                     0, nullptr);
  HIP_OK(hipGetLastError());
}

void expand_coalesced(const uint32_t* first, int64_t n, uint64_t* size, uint64_t* off,
                      hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_expand, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, first, n, size,
                     off);
  HIP_OK(hipGetLastError());
}

void expand_coalesced_out(const uint32_t* first, int64_t n, const uint64_t* size,
                          const uint64_t* off, uint64_t* out_size, uint64_t* out_off,
                          uint32_t* table, const uint32_t* cslot, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_expand_out, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, s, first, n,
                     size, off, out_size, out_off, table, cslot);
  HIP_OK(hipGetLastError());
}

void digest_keys(const uint8_t* bytes, const int64_t* offs, int64_t n, Digest* out,
                 hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_digest, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, bytes, offs, n, out);
  HIP_OK(hipGetLastError());
}

void route_keys(const Digest* keys, int64_t n, const uint32_t* ring_pts, const int32_t* ring_owner,
                int32_t npts, int32_t* dest, int64_t* counts, int32_t nranks, hipStream_t s) {
  if (n <= 0) return;
  SH_CHECK(npts > 0 && nranks > 0 && nranks <= 4096, "bad ring");
  hipLaunchKernelGGL(k_route, dim3(grid_for(n, kBlock * 8, 1024)), dim3(kBlock),
                     nranks * sizeof(unsigned long long), s, keys, n, ring_pts, ring_owner, npts,
                     dest, counts, nranks);
  HIP_OK(hipGetLastError());
}

void scatter_by_dest(const int32_t* dest, const int64_t* base, int64_t n, int32_t nranks,
                     int64_t* cursor, int64_t* perm, hipStream_t s) {
  if (n <= 0) return;
  (void)nranks;
  hipLaunchKernelGGL(k_scatter, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, dest, base, n,
                     cursor, perm);
  HIP_OK(hipGetLastError());
}

void permute_records(const void* in, const int64_t* perm, int64_t n, int32_t rec_bytes, void* out,
                     hipStream_t s) {
  if (n <= 0) return;
  SH_CHECK(rec_bytes % 4 == 0, "record size must be a multiple of 4");
  const int32_t words = rec_bytes / 4;
  hipLaunchKernelGGL(k_permute, dim3(grid_for(n * words, kBlock)), dim3(kBlock), 0, s,
                     (const uint32_t*)in, perm, n, words, (uint32_t*)out);
  HIP_OK(hipGetLastError());
}

void records_to_set(const uint8_t* rec, const uint64_t* off, const uint64_t* size,
                    const uint64_t* have_size, int64_t n, Digest* keys, uint64_t* val_off,
                    uint32_t* vlen, uint32_t* flags, uint32_t* expire, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_records_to_set, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, rec, off,
                     size, have_size, n, keys, val_off, vlen, flags, expire);
  HIP_OK(hipGetLastError());
}

void mfma_hello(const uint16_t* a, const uint16_t* b, float* c, int tiles, hipStream_t s) {
  if (tiles <= 0) return;
  hipLaunchKernelGGL(k_mfma_hello, dim3(tiles), dim3(64), 0, s, a, b, c);
  HIP_OK(hipGetLastError());
}

HbmCache::HbmCache(const ShardConfig& cfg) : cfg_(cfg) {
  SH_CHECK(cfg_.nbuckets >= 2 && (cfg_.nbuckets & (cfg_.nbuckets - 1)) == 0,
           "nbuckets must be a power of two >= 2");
  SH_CHECK(cfg_.nbuckets * kEntriesPerBucket < (1ull << 32), "index too large (u32 entry ids)");
  SH_CHECK(cfg_.log_bytes >= 4096 && cfg_.log_bytes % 16 == 0, "log_bytes must be >=4096, %16");
  SH_CHECK(cfg_.max_item > 0 && item_bytes(cfg_.max_item) * 2 <= cfg_.log_bytes,
           "max_item too large for the log");
  DeviceGuard g(cfg_.device);
  const uint64_t slack = item_bytes(cfg_.max_item) + 64;
  HIP_OK(hipMalloc(&log_, cfg_.log_bytes + slack));
  HIP_OK(hipMalloc(&index_, cfg_.nbuckets * kBucketBytes));
  HIP_OK(hipMalloc(&head_, 64));
  HIP_OK(hipMalloc(&ctr_, kCtrShards * sizeof(CacheCounters)));
  HIP_OK(hipMalloc(&scratch_, 64));
  HIP_OK(hipMalloc(&done_ctr_, 64));
  HIP_OK(hipMemset(done_ctr_, 0, 64));
  const size_t lb_words = (size_t)(kSmallGetMax / kEdgeKeys + 1);
  HIP_OK(hipMalloc(&lb_state_, lb_words * sizeof(unsigned long long)));
  HIP_OK(hipMemset(lb_state_, 0, lb_words * sizeof(unsigned long long)));
  HIP_OK(hipMalloc(&part_, 3 * kMaxGrid * sizeof(uint64_t)));
  HIP_OK(hipHostMalloc(&host_buf_, kCtrShards * sizeof(CacheCounters), hipHostMallocDefault));
  HIP_OK(hipHostMalloc(&host_slots_, kHostSlots * sizeof(uint64_t),
                       hipHostMallocMapped | hipHostMallocCoherent));
  memset(host_slots_, 0, kHostSlots * sizeof(uint64_t));
  SH_CHECK(cfg_.serve_blocks >= 1 && cfg_.serve_blocks <= kServeBlocksMax,
           "serve_blocks out of range");
  srv_blocks_ = cfg_.serve_blocks;
  HIP_OK(hipHostMalloc(&srv_ring_, (size_t)kServeRing * srv_blocks_ * sizeof(SrvJob),
                       hipHostMallocMapped | hipHostMallocCoherent));
  memset(srv_ring_, 0, (size_t)kServeRing * srv_blocks_ * sizeof(SrvJob));
  HIP_OK(hipHostMalloc(&srv_ctl_, kCtlWords * sizeof(uint64_t),
                       hipHostMallocMapped | hipHostMallocCoherent));
  memset(srv_ctl_, 0, kCtlWords * sizeof(uint64_t));
  HIP_OK(hipMalloc(&srv_sync_, 64));
  HIP_OK(hipHostMalloc(&srv_trace_, kSrvTrace * 8 * sizeof(uint64_t),
                       hipHostMallocMapped | hipHostMallocCoherent));
  memset(srv_trace_, 0, kSrvTrace * 8 * sizeof(uint64_t));
  {
    int khz = 0;
    HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg_.device));
    if (khz <= 0) khz = 100000;
    srv_khz_ = (uint64_t)khz;
    srv_idle_ticks_ = (uint64_t)khz * kSrvIdleUs / 1000;
    srv_life_ticks_ = (uint64_t)khz * kSrvLifeUs / 1000;
  }
  HIP_OK(hipMemset(index_, 0, cfg_.nbuckets * kBucketBytes));
  HIP_OK(hipMemset(head_, 0, 64));
  HIP_OK(hipMemset(ctr_, 0, kCtrShards * sizeof(CacheCounters)));
  SH_CHECK(cfg_.evict == kEvictFifo || cfg_.evict == kEvictClock, "unknown eviction policy");
  SH_CHECK(cfg_.max_item <= kVlenMask, "max_item must be < 2 GiB (CLOCK bit in vlen)");
  if (cfg_.evict == kEvictClock) {
    rmax_ = reinsert_budget(cfg_.log_bytes, cfg_.reinsert_max);
    ring_cap_ = ring_entries(cfg_.nbuckets);
    HIP_OK(hipMalloc(&ring_, ring_cap_ * sizeof(uint64_t)));
    HIP_OK(hipMalloc(&rc_ctl_, 8 * sizeof(unsigned long long)));
    HIP_OK(hipMemset(rc_ctl_, 0, 8 * sizeof(unsigned long long)));
    HIP_OK(hipMemset(rc_ctl_ + 2, 0xff, sizeof(unsigned long long)));  // no cut yet
    for (HandBuf& b : hb_) HIP_OK(hipMalloc(&b.scratch, rmax_ + 64));
  }
  HIP_OK(hipDeviceSynchronize());
}

HbmCache::~HbmCache() {
  DeviceGuard g(cfg_.device);
  try {
    serve_stop();
  } catch (...) {
  }
  (void)hipDeviceSynchronize();
  if (srv_stream_) (void)hipStreamDestroy(srv_stream_);
  (void)hipHostFree(srv_ring_);
  (void)hipHostFree(srv_ctl_);
  (void)hipHostFree(srv_trace_);
  (void)hipFree(srv_sync_);
  (void)hipFree(log_);
  (void)hipFree(index_);
  (void)hipFree(head_);
  (void)hipFree(ctr_);
  (void)hipFree(scratch_);
  (void)hipFree(done_ctr_);
  (void)hipFree(lb_state_);
  (void)hipFree(part_);
  (void)hipHostFree(host_buf_);
  (void)hipHostFree(host_slots_);
  for (SetWs& w : ws_)
    for (void* p : {(void*)w.dd_keys, (void*)w.dd_win, (void*)w.dd_slot, (void*)w.set_size,
                    (void*)w.set_off, (void*)w.set_claim, (void*)w.set_cnt})
      (void)hipFree(p);
  (void)hipFree(ring_); (void)hipFree(rc_ctl_);
  for (void* p : {(void*)rc_loc_, (void*)rc_h_, (void*)rc_part_, (void*)rc_hx_}) (void)hipFree(p);
  for (HandBuf& b : hb_)
    for (void* p : {(void*)b.keys, (void*)b.voff, (void*)b.from, (void*)b.vlen, (void*)b.flags,
                    (void*)b.expire, (void*)b.scratch})
      (void)hipFree(p);
  reap_retired(true);
  if (ws_ready_) (void)hipEventDestroy(ws_ready_);
  for (const SetStream& x : set_streams_)
    if (x.last) (void)hipEventDestroy(x.last);
}

void HbmCache::retire_group(std::initializer_list<void*> ptrs, uint64_t bytes, hipStream_t s) {
  RetiredGroup g;
  for (void* p : ptrs)
    if (p) g.ptrs.push_back(p);
  if (g.ptrs.empty()) return;
  g.bytes = bytes;
  retired_ever_ += bytes;
  // the growing stream waits for the other SET streams' last stores (their events, not
  // their streams: a stream a caller has destroyed is never touched), then one event
  for (const SetStream& x : set_streams_)
    if (x.s != s && x.last) HIP_OK(hipStreamWaitEvent(s, x.last, 0));
  hipEvent_t e;
  HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipEventRecord(e, s));
  g.ev.push_back(e);
  retired_.push_back(std::move(g));
}

void HbmCache::reap_retired(bool all) {
  for (size_t i = 0; i < retired_.size();) {
    bool done = true;
    for (hipEvent_t e : retired_[i].ev)
      if (all) (void)hipEventSynchronize(e);
      else if (hipEventQuery(e) != hipSuccess) done = false;
    if (!done) {
      ++i;
      continue;
    }
    for (hipEvent_t e : retired_[i].ev) (void)hipEventDestroy(e);
    for (void* p : retired_[i].ptrs) (void)hipFree(p);
    retired_.erase(retired_.begin() + (long)i);
  }
}

uint64_t HbmCache::retired_bytes() {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  reap_retired(false);
  uint64_t b = 0;
  for (const RetiredGroup& r : retired_) b += r.bytes;
  return b;
}

void HbmCache::ws_order(hipStream_t s) {
  if (!ws_ready_ || s == ws_grow_stream_) return;
  if (std::find(ws_ordered_.begin(), ws_ordered_.end(), s) != ws_ordered_.end()) return;
  HIP_OK(hipStreamWaitEvent(s, ws_ready_, 0));  // the grow's table clears land first
  ws_ordered_.push_back(s);
}

void HbmCache::note_stream(hipStream_t s) {
  for (const SetStream& x : set_streams_)
    if (x.s == s) return;
  SetStream x;
  x.s = s;
  // (only orders execution: no system-scope cache flush at every store's end marker)
  HIP_OK(hipEventCreateWithFlags(&x.last, hipEventDisableTiming | hipEventDisableSystemFence));
  set_streams_.push_back(x);
}

void HbmCache::note_store_end(hipStream_t s) {
  for (const SetStream& x : set_streams_)
    if (x.s == s) {
      (void)hipEventRecord(x.last, s);
      return;
    }
}

uint64_t HbmCache::hbm_bytes() const {
  return cfg_.log_bytes + item_bytes(cfg_.max_item) + 64 + cfg_.nbuckets * kBucketBytes +
         ring_cap_ * sizeof(uint64_t) + (hb_[0].scratch ? 2 * (rmax_ + 64) : 0);
}

// Hand-step workspace for windows of w ring entries. Buffers grow without a device
// synchronisation: the old blocks are retired (freed with the cache), since queued work on
// any stream may still read them.
void HbmCache::ensure_rc_ws(int64_t w, hipStream_t s) {
  if (w <= rc_cap_) return;
  int64_t cap = rc_cap_ ? rc_cap_ : 4096;
  while (cap < w) cap *= 2;
  const uint64_t oc = (uint64_t)rc_cap_;
  retire_group({rc_loc_, rc_h_, rc_part_, rc_hx_}, oc * 8 * 2 + (oc / kBlock + 5) * 8 + (oc + 1) * 8,
               s);
  HIP_OK(hipMalloc(&rc_loc_, cap * 8));
  HIP_OK(hipMalloc(&rc_h_, cap * 8));
  HIP_OK(hipMalloc(&rc_part_, (cap / kBlock + 5) * 8));  // + K - 1 sub-blocks of the scan
  HIP_OK(hipMalloc(&rc_hx_, (cap + 1) * 8));
  rc_cap_ = cap;
}

// Hand buffer b for a combined batch of `rows` rows (w reinsertion rows + the batch's own).
void HbmCache::ensure_cb(int b, int64_t rows, hipStream_t s) {
  HandBuf& h = hb_[b];
  if (rows <= h.cap) return;
  int64_t cap = h.cap ? h.cap : 4096;
  while (cap < rows) cap *= 2;
  retire_group({h.keys, h.voff, h.from, h.vlen, h.flags, h.expire}, (uint64_t)h.cap * 44, s);
  HIP_OK(hipMalloc(&h.keys, cap * sizeof(Digest)));
  HIP_OK(hipMalloc(&h.voff, cap * 8));
  HIP_OK(hipMalloc(&h.from, cap * 8));
  HIP_OK(hipMalloc(&h.vlen, cap * 4));
  HIP_OK(hipMalloc(&h.flags, cap * 4));
  HIP_OK(hipMalloc(&h.expire, cap * 4));
  h.cap = cap;
}

bool HbmCache::should_reclaim(uint64_t bytes_bound) const {
  if (cfg_.evict != kEvictClock) return false;
  // head as of the last SET chain that completed (published by k_set_index); up to a
  // few stores may be queued behind it, so reclaim once the log is within 4 batches of
  // wrapping (the hand step decides exactly on the device; skipping is only an
  // optimisation for a log that has not filled yet)
  // (a populate queues dozens of large batches before the first completes, so they can all
  // skip the hand and leave it laps behind the overwrite: rc_advance then jumps it)
  const uint64_t h = __atomic_load_n(host_slots_ + kHeadSlot, __ATOMIC_ACQUIRE);
  return h + 4 * (bytes_bound + rmax_) > cfg_.log_bytes;
}

void HbmCache::reclaim_locked(const Digest* keys, const uint8_t* values, const uint64_t* val_off,
                              const uint32_t* vlen, const uint32_t* flags, const uint32_t* expire,
                              int64_t n, int64_t w, uint64_t rmax, uint32_t now, hipStream_t s,
                              bool detached, bool lead) {
  // The head: the claim word, i.e. the head every queued append will have reached (equal to
  // the head slot once they have run). The ring tail: a detached hand may run before the
  // previous batch's fixup writes its ring entries and tail, so it reads the tail of the
  // batch before that one (the other ping-pong slot), whose entries are written.
  RcArgs a{ring_, ring_cap_ - 1, detached ? next_ring_tail() : cur_ring_tail(), rc_ctl_, w, n,
           hand_b_, claim_ptr(), cfg_.log_bytes, now, rmax, lead ? 1ull : 0ull};
  const int g = (int)((w + kBlock - 1) / kBlock);
  const HandBuf& hb = hb_[hand_b_];
  const RcBatch cb{hb.keys, hb.voff, hb.vlen, hb.flags, hb.expire, hb.from};
  // window entries per lane of the scan (SHELLAC_RCSCAN_K: A/B experiments); its part_h stays
  // one word per 256 entries, rc_part_ is sized for g + K of them
  static const int rk = [] {
    const char* e = getenv("SHELLAC_RCSCAN_K");
    const int v = e ? atoi(e) : kRcScanK;
    return v == 1 || v == 2 || v == 4 ? v : kRcScanK;
  }();
  const int gk = (g + rk - 1) / rk;
  if (rk == 4)
    hipLaunchKernelGGL(k_rc_scan<4>, dim3(gk), dim3(kBlock), 0, s, a, cb, log_, index_,
                       cfg_.nbuckets - 1, keys, values, val_off, vlen, flags, expire, n,
                       cfg_.max_item, rc_loc_, rc_h_, rc_part_);
  else if (rk == 2)
    hipLaunchKernelGGL(k_rc_scan<2>, dim3(gk), dim3(kBlock), 0, s, a, cb, log_, index_,
                       cfg_.nbuckets - 1, keys, values, val_off, vlen, flags, expire, n,
                       cfg_.max_item, rc_loc_, rc_h_, rc_part_);
  else
    hipLaunchKernelGGL(k_rc_scan<1>, dim3(gk), dim3(kBlock), 0, s, a, cb, log_, index_,
                       cfg_.nbuckets - 1, keys, values, val_off, vlen, flags, expire, n,
                       cfg_.max_item, rc_loc_, rc_h_, rc_part_);
  hipLaunchKernelGGL(k_rc_emit, dim3(g), dim3(kBlock), 0, s, a, cb, log_, rc_loc_, rc_h_,
                     rc_part_, rc_hx_, hb.scratch, ctr_);
  if (!lead)
    launch_segcopy<2>(s, log_, rc_loc_, rc_hx_, w, hb.scratch, nullptr, nullptr, nullptr,
                      nullptr, rc_h_, rmax);
  rc_adv_w_ = w;  // the combined batch's dedupe advances the hand
  HIP_OK(hipGetLastError());
}

void HbmCache::ensure_set_ws(int64_t n, hipStream_t s) {
  if (n <= set_cap_) return;
  int64_t cap = set_cap_ ? set_cap_ : 1024;
  while (cap < n) cap *= 2;
  const uint64_t tslots = (uint64_t)cap * 2;
  const uint64_t oc = (uint64_t)set_cap_;
  for (SetWs& w : ws_) {
    // the old workspace may still be read by queued SET chains on other streams: retired
    // until their events say they finished (no device synchronisation on the serving path)
    retire_group({w.dd_keys, w.dd_win, w.dd_slot, w.set_size, w.set_off, w.set_claim, w.set_cnt},
                 2 * oc * 12 + oc * 8 + 3 * (oc + 1) * 8, s);
    HIP_OK(hipMalloc(&w.dd_keys, tslots * sizeof(uint64_t)));
    HIP_OK(hipMalloc(&w.dd_win, tslots * sizeof(int)));
    // the tables are cleared once here, on the stream of the SET that first uses them
    // (ordered before its dedupe; the null stream is not: a non-blocking stream does not
    // wait for it, which once dropped the first batch's rows); k_set_index resets every
    // slot a batch used
    HIP_OK(hipMemsetAsync(w.dd_keys, 0, tslots * sizeof(uint64_t), s));
    HIP_OK(hipMemsetAsync(w.dd_win, 0xff, tslots * sizeof(int), s));
    HIP_OK(hipMalloc(&w.dd_slot, cap * sizeof(uint32_t)));
    HIP_OK(hipMalloc(&w.set_size, (cap + 1) * sizeof(uint64_t)));
    HIP_OK(hipMalloc(&w.set_off, (cap + 1) * sizeof(uint64_t)));
    HIP_OK(hipMalloc(&w.set_claim, cap * sizeof(uint32_t)));
    HIP_OK(hipMalloc(&w.set_cnt, (cap + 1) * sizeof(uint64_t)));
  }
  select_ws(0);
  dd_mask_ = (uint32_t)(tslots - 1);
  set_cap_ = cap;
  ++ws_gen_;
  // a store on another stream waits for these clears (the dedupe tables were
  // read uncleared by a store on a stream the grow was not ordered with)
  if (!ws_ready_) HIP_OK(hipEventCreateWithFlags(&ws_ready_, hipEventDisableTiming));
  HIP_OK(hipEventRecord(ws_ready_, s));
  ws_grow_stream_ = s;
  ws_ordered_.clear();
}

void HbmCache::reserve(int64_t n) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  if (cfg_.evict == kEvictClock && rmax_ && n > 0) {
    // a SET batch of n rows runs as a combined batch of hand_window(n) + n rows once the
    // log wraps: size the hand's workspaces and both hand buffers for it now, so no serving
    // store allocates in steady state
    const int64_t w = hand_window(n);
    ensure_rc_ws(w, nullptr);
    ensure_cb(0, w + n, nullptr);
    ensure_cb(1, w + n, nullptr);
    n = w + n;
  }
  ensure_set_ws(n, nullptr);
  // (a maintenance call, not on the serving path: the null-stream clears land before any
  // stream's next SET, and every grown-out workspace can go)
  HIP_OK(hipDeviceSynchronize());
  reap_retired(true);
}

void HbmCache::lookup(const Digest* keys, int64_t n, uint64_t* loc, uint64_t* size, uint64_t* off,
                      uint32_t now, hipStream_t s, uint64_t reserve, int total_slot,
                      const uint32_t* first) {
  TraceRange tr("hbm.lookup");
  SH_CHECK(total_slot < kHostSlots, "host slot out of range");
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  uint64_t* ht = total_slot >= 0 ? host_slots_ + total_slot : nullptr;
  if (ht) __atomic_store_n(ht, kSlotPending, __ATOMIC_RELEASE);
  if (n <= 0) {
    HIP_OK(hipMemsetAsync(off, 0, sizeof(uint64_t), s));
    if (ht) *ht = 0;
    return;
  }
  const int grid = grid_for(n * 8, kBlock, kMaxGrid);
  hipLaunchKernelGGL(k_probe, dim3(grid), dim3(kBlock), 0, s, keys, n, index_, cfg_.nbuckets - 1,
                     cur_head(), reserve, cfg_.log_bytes, now, loc, size, ctr_, part_, first,
                     (int64_t)1, (const int64_t*)nullptr, (const uint64_t*)nullptr);
  HIP_OK(hipGetLastError());
  launch_offsets(size, n, part_, grid, off, s, ht);
}

void HbmCache::lookup_slots(const Digest* keys, int64_t nslots, int64_t slot_rows,
                            const int64_t* slot_cnt, uint64_t* loc, uint64_t* size, uint64_t* off,
                            uint32_t now, hipStream_t s, const uint64_t* reserve_dev) {
  TraceRange tr("hbm.lookup_slots");
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  const int64_t n = nslots * slot_rows;
  if (n <= 0) {
    HIP_OK(hipMemsetAsync(off, 0, sizeof(uint64_t), s));
    return;
  }
  const int grid = grid_for(n * 8, kBlock, kMaxGrid);
  hipLaunchKernelGGL(k_probe, dim3(grid), dim3(kBlock), 0, s, keys, n, index_, cfg_.nbuckets - 1,
                     cur_head(), (uint64_t)0, cfg_.log_bytes, now, loc, size, ctr_, part_,
                     (const uint32_t*)nullptr, slot_rows, slot_cnt, reserve_dev);
  HIP_OK(hipGetLastError());
  launch_offsets(size, n, part_, grid, off, s, nullptr);
}

int HbmCache::lookup_coalesced(const Digest* keys, int64_t n, uint32_t* table,
                               int64_t table_slots, uint32_t* first, uint64_t* loc,
                               uint64_t* size, uint64_t* off, uint32_t now, hipStream_t s,
                               uint64_t reserve, int total_slot, uint32_t* cslot,
                               bool table_clean, uint64_t* prefix, hipEvent_t index_done) {
  TraceRange tr("hbm.lookup_coalesced");
  SH_CHECK(total_slot < kHostSlots, "host slot out of range");
  SH_CHECK(n < (1ll << 31), "coalesce: batch too large");
  SH_CHECK(table_slots >= 2 * n && (table_slots & (table_slots - 1)) == 0,
           "coalesce: table needs a power of two >= 2n slots");
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  uint64_t* ht = total_slot >= 0 ? host_slots_ + total_slot : nullptr;
  if (ht) __atomic_store_n(ht, kSlotPending, __ATOMIC_RELEASE);
  if (n <= 0) {
    HIP_OK(hipMemsetAsync(off, 0, sizeof(uint64_t), s));
    if (prefix) HIP_OK(hipMemsetAsync(prefix, 0, sizeof(uint64_t), s));
    if (ht) *ht = 0;
    if (index_done) HIP_OK(hipEventRecord(index_done, s));
    return prefix ? 31 : -1;
  }
  if (!table_clean) HIP_OK(hipMemsetAsync(table, 0, (size_t)table_slots * sizeof(uint32_t), s));
  // contiguous whole chunks per workgroup, at most kMaxGrid partial sums
  const int64_t chunks = (n + kCoKeys - 1) / kCoKeys;
  int64_t per = (chunks + kMaxGrid - 1) / kMaxGrid;
  if (prefix)  // a power of two: the gather finds a row's workgroup by a shift
    for (int64_t p2 = 1;; p2 <<= 1)
      if (p2 >= per) {
        per = p2;
        break;
      }
  const int grid = (int)((chunks + per - 1) / per);
  const int64_t plen = per * kCoKeys;
  // (fusing the offsets scan into this kernel — by decoupled look-back, or by one bump
  // allocation per chunk with a compacted hit list — was measured slower: 0.45 and 0.35 vs
  // 0.32 ms per step; see docs/PERF.md)
  launch_stop(&index_done, k_coalesce<true>, dim3(grid), dim3(kBlock), s, keys, n, plen, table,
              (uint32_t)(table_slots - 1), first, cslot, index_, cfg_.nbuckets - 1, cur_head(),
              reserve, cfg_.log_bytes, now, loc, size, ctr_, part_, 0, prefix ? off : nullptr);
  HIP_OK(hipGetLastError());
  if (!prefix) {
    launch_offsets(size, n, part_, grid, off, s, ht, plen);
    return -1;
  }
  hipLaunchKernelGGL(k_block_prefix, dim3(1), dim3(kBlock), 0, s, part_, grid, prefix, ht);
  HIP_OK(hipGetLastError());
  int shift = 0;
  while ((int64_t)1 << shift < plen) ++shift;
  return shift;
}

uint64_t HbmCache::host_slot(int i) const {
  SH_CHECK(i >= 0 && i < kHostSlots, "host slot out of range");
  return __atomic_load_n(host_slots_ + i, __ATOMIC_ACQUIRE);
}

uint64_t HbmCache::wait_host_slot(int i, int64_t timeout_ms) const {
  SH_CHECK(i >= 0 && i < kHostSlots, "host slot out of range");
  const uint64_t* p = host_slots_ + i;
  uint64_t v = __atomic_load_n(p, __ATOMIC_ACQUIRE);
  if (v != kSlotPending) return v;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0;; ++spin) {
    v = __atomic_load_n(p, __ATOMIC_ACQUIRE);
    if (v != kSlotPending) return v;
    if ((spin & 1023) == 1023) {
      const auto el = std::chrono::steady_clock::now() - t0;
      SH_CHECK(std::chrono::duration_cast<std::chrono::milliseconds>(el).count() < timeout_ms,
               "timed out waiting for a lookup total (GPU stalled?)");
    }
    __builtin_ia32_pause();
  }
}

void HbmCache::small_get(const Digest* keys, int64_t n, uint8_t* out, uint64_t out_cap,
                         uint64_t* off, uint32_t now, hipStream_t s, int done_slot) {
  SH_CHECK(n >= 0 && n <= kSmallGetMax, "edge GET batch too large");
  SH_CHECK(done_slot < kHostSlots, "host slot out of range");
  TraceRange tr("hbm.edge_get");
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  uint64_t* ds = done_slot >= 0 ? host_slots_ + done_slot : nullptr;
  if (ds) __atomic_store_n(ds, kSlotPending, __ATOMIC_RELEASE);
  const int grid = (int)std::max<int64_t>(1, (n + kEdgeKeys - 1) / kEdgeKeys);
  hipLaunchKernelGGL(k_edge_get, dim3(grid), dim3(kBlock), 0, s, keys, n, index_,
                     cfg_.nbuckets - 1, cur_head(), cfg_.log_bytes, now, log_, out, out_cap, off,
                     ctr_, lb_state_, done_ctr_, ds);
  HIP_OK(hipGetLastError());
}

void HbmCache::serve_launch_locked() {
  DeviceGuard g(cfg_.device);
  if (!srv_stream_) {
    // A CU mask gives the stream a hardware queue of its own (masked queues are never
    // shared), so no other stream's work waits behind the resident server; the mask
    // itself only keeps the server on the first 64 CUs.
    const uint32_t mask[2] = {0xffffffffu, 0xffffffffu};
    HIP_OK(hipExtStreamCreateWithCUMask(&srv_stream_, 2, mask));
  }
  __atomic_store_n(srv_ctl_ + kCtlStop, 0ull, __ATOMIC_RELEASE);
  ++srv_epoch_;
  SrvJob* ring = nullptr;
  uint64_t *ctl = nullptr, *slots = nullptr, *trace = nullptr;
  HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ring), srv_ring_, 0));
  HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctl), srv_ctl_, 0));
  HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&slots), host_slots_, 0));
  HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&trace), srv_trace_, 0));
  HIP_OK(hipMemsetAsync(srv_sync_, 0, 64, srv_stream_));
  hipLaunchKernelGGL(k_edge_server, dim3(srv_blocks_), dim3(kSrvBlock), 0, srv_stream_, ring, ctl,
                     slots, index_, cfg_.nbuckets - 1, (const uint64_t*)head_, cfg_.log_bytes,
                     log_, ctr_, trace, srv_epoch_, srv_idle_ticks_, srv_life_ticks_, srv_sync_,
                     srv_blocks_);
  HIP_OK(hipGetLastError());
  srv_running_ = true;
  ++srv_launches_;
}

bool HbmCache::serve_get(const Digest* host_keys, int64_t n, uint8_t* out, uint64_t out_cap,
                         uint64_t* off, uint32_t now, int done_slot) {
  if (n < 1 || n > kServeKeys || done_slot < 0 || done_slot >= kHostSlots) return false;
  TraceRange tr("hbm.serve_get");
  std::lock_guard<std::mutex> lk(srv_mu_);
  // ticket T goes to server block T % blocks, as that block's ticket T / blocks
  const uint64_t blk = srv_ticket_ % (uint64_t)srv_blocks_, t = srv_ticket_ / (uint64_t)srv_blocks_;
  const uint64_t consumed = __atomic_load_n(srv_ctl_ + kCtlConsumed + 8 * blk, __ATOMIC_ACQUIRE);
  if (t - consumed >= (uint64_t)kServeRing) return false;  // that block's ring is full
  __atomic_store_n(host_slots_ + done_slot, kSlotPending, __ATOMIC_RELEASE);
  // every 16-B granule is {value, tag}: the value first, then the tag with a release
  // store, so a granule read whole by the device never pairs a new tag with an old value
  SrvGranule* jg = static_cast<SrvJob*>(srv_ring_)[blk * kServeRing + t % kServeRing].g;
  const uint64_t tag = t + 1;
  auto put = [&](int i, uint64_t v) {
    jg[i].v = v;
    __atomic_store_n(&jg[i].tag, tag, __ATOMIC_RELEASE);
  };
  for (int64_t k = 0; k < n; ++k) {
    put(kSrvHdr + 2 * (int)k, host_keys[k].lo);
    put(kSrvHdr + 2 * (int)k + 1, host_keys[k].hi);
  }
  put(0, (uint64_t)(uintptr_t)out);
  put(1, out_cap);
  put(2, (uint64_t)(uintptr_t)off);
  put(4, (uint64_t)done_slot);
  put(3, (uint64_t)(uint32_t)n | ((uint64_t)now << 32));
  __atomic_store_n(&srv_ticket_, srv_ticket_ + 1, __ATOMIC_RELAXED);  // serve_backlog reads it
  if (!srv_running_ ||
      __atomic_load_n(srv_ctl_ + kCtlExited, __ATOMIC_ACQUIRE) == srv_epoch_)
    serve_launch_locked();
  return true;
}

bool HbmCache::serve_get_after(hipStream_t after, const Digest* host_keys, int64_t n,
                               uint8_t* out, uint64_t out_cap, uint64_t* off, uint32_t now,
                               int done_slot) {
  if (n < 1 || n > kServeKeys || done_slot < 0 || done_slot >= kHostSlots) return false;
  {
    // one event per thread and device (the proxy's reactors and test threads submit
    // concurrently); polled, not synchronised (no yield on the submission path)
    DeviceGuard g(cfg_.device);
    thread_local hipEvent_t ev[64] = {};
    SH_CHECK(cfg_.device >= 0 && cfg_.device < 64, "device out of range");
    hipEvent_t& e = ev[cfg_.device];
    if (!e) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_OK(hipEventRecord(e, after));
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      const hipError_t q = hipEventQuery(e);
      if (q == hipSuccess) break;
      SH_CHECK(q == hipErrorNotReady, std::string("event query failed: ") + hipGetErrorString(q));
      if ((spin & 1023) == 1023)
        SH_CHECK(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(30),
                 "timed out waiting for the caller's stream before an edge job");
      __builtin_ia32_pause();
    }
  }
  return serve_get(host_keys, n, out, out_cap, off, now, done_slot);
}

void HbmCache::serve_kick() {
  std::lock_guard<std::mutex> lk(srv_mu_);
  if (srv_running_ && __atomic_load_n(srv_ctl_ + kCtlExited, __ATOMIC_ACQUIRE) != srv_epoch_)
    return;  // running (or launched and about to start)
  srv_running_ = false;
  if (serve_backlog() > 0) serve_launch_locked();
}

std::vector<uint64_t> HbmCache::serve_trace() const {
  std::vector<uint64_t> out(srv_trace_, srv_trace_ + kSrvTrace * 8);
  return out;
}

uint64_t HbmCache::serve_wait(int i, int64_t timeout_ms) {
  SH_CHECK(i >= 0 && i < kHostSlots, "host slot out of range");
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0;; ++spin) {
    const uint64_t v = __atomic_load_n(host_slots_ + i, __ATOMIC_ACQUIRE);
    if (v != kSlotPending) return v;
    if ((spin & 255) == 255) {
      serve_kick();
      const auto el = std::chrono::steady_clock::now() - t0;
      SH_CHECK(std::chrono::duration_cast<std::chrono::milliseconds>(el).count() < timeout_ms,
               "timed out waiting for the edge server");
    }
    __builtin_ia32_pause();
  }
}

void HbmCache::serve_stop() {
  std::lock_guard<std::mutex> lk(srv_mu_);
  if (!srv_running_) return;
  DeviceGuard g(cfg_.device);
  __atomic_store_n(srv_ctl_ + kCtlStop, 1ull, __ATOMIC_RELEASE);
  HIP_OK(hipStreamSynchronize(srv_stream_));
  srv_running_ = false;
}

void HbmCache::gather(const uint64_t* loc, const uint64_t* off, int64_t n, uint8_t* out,
                      hipStream_t s, uint64_t out_cap, const uint32_t* first,
                      const uint64_t* size, uint64_t* out_size, uint64_t* out_off,
                      uint32_t* table, const uint32_t* cslot, const uint64_t* prefix,
                      int shift) {
  TraceRange tr("hbm.gather");
  DeviceGuard g(cfg_.device);
  if (n <= 0) return;
  ExpandTail ex;
  if (first) ex = ExpandTail{first, n, size, off, out_size, out_off, table, cslot};
  ex.prefix = prefix;
  ex.shift = shift;
  if (prefix)  // block-local offsets (lookup_coalesced with a prefix)
    launch_segcopy_ex<4>(s, ex, log_, loc, off, n, out, nullptr, nullptr, nullptr, nullptr,
                         nullptr, out_cap);
  else
    launch_segcopy_ex<0>(s, ex, log_, loc, off, n, out, nullptr, nullptr, nullptr, nullptr,
                         nullptr, out_cap);
  HIP_OK(hipGetLastError());
}

void HbmCache::store(const Digest* keys, const uint8_t* values, const uint64_t* val_off,
                     const uint32_t* vlen, const uint32_t* flags, const uint32_t* expire,
                     int64_t n, uint64_t bytes_bound, uint32_t now, hipStream_t s,
                     hipEvent_t index_after, bool allow_reclaim, hipEvent_t append_after,
                     hipEvent_t append_done, int phase, hipEvent_t plan_done,
                     hipEvent_t done) {
  TraceRange tr("hbm.store");
  if (n <= 0) {
    if (done) HIP_OK(hipEventRecord(done, s));  // nothing queued to carry it
    return;
  }
  SH_CHECK(bytes_bound <= cfg_.log_bytes / 2,
           "SET batch larger than half the log; split the batch");
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  note_stream(s);
  stop_ev_ = done;  // the chain's last kernel (the index fix-up) takes it
  struct EndMark {  // the stream's `last` event, after whatever this call queues
    HbmCache* c;
    hipStream_t s;
    ~EndMark() {
      if (c->stop_ev_) {  // no chain kernel took `done`
        (void)hipEventRecord(c->stop_ev_, s);
        c->stop_ev_ = nullptr;
      }
      c->note_store_end(s);
    }
  } end_mark{this, s};
  if (!retired_.empty()) reap_retired(false);  // grown-out workspaces whose chains finished
  // phase 2: the rest of the chain of the batch a phase-1 call planned
  if (phase == 2) {
    SH_CHECK(pend_.active && pend_.n == n, "store phase 2 without the same batch's phase 1");
    store_tail_locked(now, s, index_after, append_after, append_done);
    return;
  }
  SH_CHECK(!pend_.active, "store: a phase-1 batch is still waiting for its phase 2");
  // the CLOCK hand's reinsertions share the half-log bound with the batch
  const uint64_t rmax = std::min<uint64_t>(rmax_, cfg_.log_bytes / 2 - bytes_bound) / 16 * 16;
  const bool hand = allow_reclaim && rmax && should_reclaim(bytes_bound);
  lead_ = hand_lead(cfg_.log_bytes, bytes_bound, rmax, lead_);  // every batch, as HostCache
  if (!hand && phase == 0 && n <= kSmallSetRows && !index_after && !append_after &&
      !append_done && !plan_done) {
    // one launch for the whole chain (the proxy's small SET batches)
    hipLaunchKernelGGL(k_set_small, dim3(1), dim3(kBlock), 0, s, keys, values, val_off, vlen,
                       flags, expire, (int)n, cfg_.max_item, index_, cfg_.nbuckets - 1,
                       cur_head(), next_head(),
                       reinterpret_cast<unsigned long long*>(claim_ptr()), cfg_.log_bytes, now,
                       log_, ring_, ring_ ? ring_cap_ - 1 : 0ull, cur_ring_tail(),
                       next_ring_tail(), host_slots_ + kHeadSlot, ctr_);
    HIP_OK(hipGetLastError());
    hsel_ ^= 1;
    return;
  }
  // consecutive batches take the two SET workspaces and hand buffers in turn
  Pending p;
  p.active = true;
  p.n = n;
  p.parity = ws_next_;
  ws_next_ ^= 1;
  const bool detached = phase == 1;
  if (hand) {
    const int64_t w = hand_window(n);
    ensure_rc_ws(w, s);
    hand_b_ = p.parity;
    ensure_cb(hand_b_, w + n, s);
    ensure_set_ws(w + n, s);
    reclaim_locked(keys, values, val_off, vlen, flags, expire, n, w, rmax, now, s, detached,
                   lead_);
    // combined batch: reinsertions first (log order), then the batch (its SETs win)
    const HandBuf& hb = hb_[hand_b_];
    p.rows = w + n;
    p.nmove = w;
    p.keys = hb.keys;
    p.values = nullptr;
    p.voff = hb.voff;
    p.vlen = hb.vlen;
    p.flags = hb.flags;
    p.expire = hb.expire;
    p.from = hb.from;
  } else {
    ensure_set_ws(n, s);
    p.rows = n;
    p.keys = keys;
    p.values = values;
    p.voff = val_off;
    p.vlen = vlen;
    p.flags = flags;
    p.expire = expire;
  }
  ws_order(s);
  select_ws(p.parity);
  store_plan_locked(p.keys, p.vlen, p.rows, s, detached);
  if (plan_done) HIP_OK(hipEventRecord(plan_done, s));
  pend_ = p;
  if (detached) return;  // the chain follows in phase 2
  store_tail_locked(now, s, index_after, append_after, append_done);
}

// The planned batch's log append (after `append_after`) and index insert (after
// `index_after`); publishes the new head (the ping-pong slot flips).
void HbmCache::store_tail_locked(uint32_t now, hipStream_t s, hipEvent_t index_after,
                                 hipEvent_t append_after, hipEvent_t append_done) {
  const Pending p = pend_;
  pend_.active = false;
  select_ws(p.parity);
  if (append_after) HIP_OK(hipStreamWaitEvent(s, append_after, 0));
  launch_segcopy<1>(s, p.values, p.voff, set_off_, p.rows, log_, p.keys, p.vlen, p.flags,
                    p.expire, cur_head(), cfg_.log_bytes);
  HIP_OK(hipGetLastError());
  if (append_done) HIP_OK(hipEventRecord(append_done, s));
  store_index_locked(p.keys, p.vlen, p.expire, p.rows, now, s, index_after, p.from, p.nmove,
                     p.nmove ? p.parity : -1);
  hsel_ ^= 1;  // later operations on the stream read the published slot
}

// The SET kernel chain (caller holds mu_, workspace sized): dedupe (last writer wins),
// sizes + fused scan, log append (k_segcopy<1>), two-choice CAS index insert that also
// publishes the new head into the other head slot. The planning kernels (dedupe, sizes,
// scan) touch neither the log, the index nor the head; the log write touches only bytes a
// reserving lookup treats as gone; the index insert (+ fix-up), queued after
// `index_after`, is the only part a concurrent lookup can observe.
void HbmCache::store_locked(const Digest* keys, const uint8_t* values, const uint64_t* val_off,
                            const uint32_t* vlen, const uint32_t* flags, const uint32_t* expire,
                            int64_t n, uint32_t now, hipStream_t s, hipEvent_t index_after,
                            hipEvent_t append_after, hipEvent_t append_done,
                            const uint64_t* from, hipEvent_t plan_done, int64_t nmove) {
  store_plan_locked(keys, vlen, n, s);
  if (plan_done) HIP_OK(hipEventRecord(plan_done, s));
  if (append_after) HIP_OK(hipStreamWaitEvent(s, append_after, 0));
  launch_segcopy<1>(s, values, val_off, set_off_, n, log_, keys, vlen, flags, expire, cur_head(),
                    cfg_.log_bytes);
  HIP_OK(hipGetLastError());
  if (append_done) HIP_OK(hipEventRecord(append_done, s));
  store_index_locked(keys, vlen, expire, n, now, s, index_after, from, nmove);
}

// `detached`: the planning of a phase-1 batch, which may run before the previous batch's
// append and index insert: the ring tail it clamps the hand with is the batch-before's (the
// last one written), and the claim grows from itself (the head every queued append
// reaches) rather than from the head slot the previous index insert has not published yet.
void HbmCache::store_plan_locked(const Digest* keys, const uint32_t* vlen, int64_t n,
                                 hipStream_t s, bool detached) {
  const int grid = grid_for(n, kBlock, kMaxGrid);
  RcAdvance adv;
  if (rc_adv_w_ > 0) {
    adv = RcAdvance{rc_ctl_, detached ? next_ring_tail() : cur_ring_tail(), ring_cap_ - 1,
                    rc_adv_w_, ring_, claim_ptr(), cfg_.log_bytes, catch_up_ ? 1 : 0};
    rc_adv_w_ = 0;
  }
  hipLaunchKernelGGL(k_set_dedupe, dim3(grid), dim3(kBlock), 0, s, keys, vlen, n,
                     (unsigned long long*)dd_keys_, dd_win_, dd_mask_, dd_slot_, adv);
  const int sgrid = grid_for(n, kBlock, kMaxGrid);
  uint64_t* part_cnt = ring_ ? part_ + 2 * kMaxGrid : nullptr;
  hipLaunchKernelGGL(k_set_size, dim3(sgrid), dim3(kBlock), 0, s, vlen, n, dd_win_, dd_slot_,
                     cfg_.max_item, set_size_, ctr_, part_ + kMaxGrid, part_cnt);
  HIP_OK(hipGetLastError());
  launch_offsets(set_size_, n, part_ + kMaxGrid, sgrid, set_off_, s, nullptr, 0, part_cnt,
                 ring_ ? set_cnt_ : nullptr, detached ? claim_ptr() : cur_head(), claim_ptr());
}

void HbmCache::store_index_locked(const Digest* keys, const uint32_t* vlen,
                                  const uint32_t* expire, int64_t n, uint32_t now, hipStream_t s,
                                  hipEvent_t index_after, const uint64_t* from, int64_t nmove,
                                  int win_parity) {
  // the index insert is the only SET kernel a concurrent lookup can observe
  if (index_after) HIP_OK(hipStreamWaitEvent(s, index_after, 0));
  // A combined batch's reinsertions (rows [0, nmove), moves) land in a launch of their own
  // before the batch's rows: a batch row may claim the slot of an item this batch's append
  // overwrites as dead, and must not take a reinserted item's entry from under its move
  // (the host twin runs the rows in this order too).
  if (!from) nmove = 0;
  for (int pass = nmove > 0 ? 0 : 1; pass < 2; ++pass) {
    const int64_t r0 = pass ? nmove : 0, r1 = pass ? n : nmove;
    if (r1 <= r0) continue;
    const int igrid = grid_for((r1 - r0) * 4, kBlock, kMaxGrid);
    hipLaunchKernelGGL(k_set_index, dim3(igrid), dim3(kBlock), 0, s, keys, n, set_size_, set_off_,
                       vlen, expire, index_, cfg_.nbuckets - 1, cur_head(), next_head(),
                       cfg_.log_bytes, now, dd_slot_, (unsigned long long*)dd_keys_, dd_win_,
                       ctr_, set_claim_, pass ? (const uint64_t*)nullptr : from, r0, r1,
                       pass || win_parity < 0 ? nullptr : rc_ctl_ + 5 + win_parity);
  }
  launch_stop(&stop_ev_, k_set_fixup, dim3(grid_for(n, kBlock, kMaxGrid)), dim3(kBlock), s, keys,
              n, set_off_, vlen, expire, cur_head(), set_claim_, index_, set_size_, ring_,
              ring_ ? ring_cap_ - 1 : 0ull, cur_ring_tail(), next_ring_tail(), set_cnt_,
              host_slots_ + kHeadSlot, cfg_.nbuckets - 1, cfg_.log_bytes, now, ctr_);
  HIP_OK(hipGetLastError());
}

void HbmCache::destroy_graph(StoreGraph* g) {
  for (auto& e : g->exec)
    if (e) {
      (void)hipGraphExecDestroy(e);
      e = nullptr;
    }
  g->n = -1;
}

void HbmCache::store_graph(StoreGraph* g, const Digest* keys, const uint8_t* values,
                           const uint64_t* val_off, const uint32_t* vlen, const uint32_t* flags,
                           const uint32_t* expire, int64_t n, uint64_t bytes_bound,
                           uint32_t now, hipStream_t s) {
  TraceRange tr("hbm.store_graph");
  if (n <= 0) return;
  SH_CHECK(s != nullptr, "store_graph needs a created stream (the legacy default stream "
                         "cannot be captured)");
  SH_CHECK(bytes_bound <= cfg_.log_bytes / 2,
           "SET batch larger than half the log; split the batch");
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard dg(cfg_.device);
  ensure_set_ws(n, s);  // before any capture: allocation is not capturable
  ws_order(s);
  select_ws(0);         // (graphs bake the workspace in: always the first)
  const void* ptrs[6] = {keys, values, val_off, vlen, flags, expire};
  bool same = g->n == n && g->bound == bytes_bound && g->now == now && g->ws_gen == ws_gen_ &&
              g->exec[0] && g->exec[1];
  for (int i = 0; same && i < 6; ++i) same = g->ptrs[i] == ptrs[i];
  if (!same) {
    destroy_graph(g);
    const int keep = hsel_;
    for (int p = 0; p < 2; ++p) {
      hsel_ = p;  // the graph for parity p reads head slot p and publishes into 1 - p
      hipGraph_t graph = nullptr;
      HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
      try {
        store_locked(keys, values, val_off, vlen, flags, expire, n, now, s);
      } catch (...) {
        (void)hipStreamEndCapture(s, &graph);
        if (graph) (void)hipGraphDestroy(graph);
        hsel_ = keep;
        throw;
      }
      HIP_OK(hipStreamEndCapture(s, &graph));
      const hipError_t e = hipGraphInstantiate(&g->exec[p], graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      HIP_OK(e);
    }
    hsel_ = keep;
    for (int i = 0; i < 6; ++i) g->ptrs[i] = ptrs[i];
    g->n = n;
    g->bound = bytes_bound;
    g->now = now;
    g->ws_gen = ws_gen_;
    g->captures++;
  }
  HIP_OK(hipGraphLaunch(g->exec[hsel_], s));
  g->launches++;
  hsel_ ^= 1;
}

void HbmCache::remove(const Digest* keys, int64_t n, uint8_t* found, uint32_t now, hipStream_t s) {
  TraceRange tr("hbm.remove");
  if (n <= 0) return;
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  hipLaunchKernelGGL(k_delete, dim3(grid_for(n * 16, kBlock, kMaxGrid)), dim3(kBlock), 0, s, keys, n,
                     index_, cfg_.nbuckets - 1, cur_head(), cfg_.log_bytes, now, found, ctr_);
  HIP_OK(hipGetLastError());
}

void HbmCache::sweep(uint32_t now, hipStream_t s, uint64_t* live_entries, uint64_t* live_bytes) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  unsigned long long* out = scratch_;
  HIP_OK(hipMemsetAsync(out, 0, 2 * sizeof(unsigned long long), s));
  const uint64_t nslots = cfg_.nbuckets * kEntriesPerBucket;
  hipLaunchKernelGGL(k_sweep, dim3(grid_for((int64_t)nslots, kBlock, 4096)), dim3(kBlock), 0, s,
                     index_, nslots, cur_head(), cfg_.log_bytes, now, out, ctr_);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(host_buf_, out, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  reap_retired(false);  // (the idle-time maintenance call: grown-out workspaces that are done)
  if (live_entries) *live_entries = host_buf_[0];
  if (live_bytes) *live_bytes = host_buf_[1];
}

uint64_t HbmCache::export_keys(Digest* out, uint64_t out_cap, uint32_t now, hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  HIP_OK(hipMemsetAsync(scratch_, 0, sizeof(unsigned long long), s));
  const uint64_t nslots = cfg_.nbuckets * kEntriesPerBucket;
  hipLaunchKernelGGL(k_export, dim3(grid_for((int64_t)nslots, kBlock, 4096)), dim3(kBlock), 0, s,
                     index_, nslots, cur_head(), cfg_.log_bytes, now, out, out_cap, scratch_);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(host_buf_, scratch_, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return host_buf_[0];
}

namespace {
struct SnapHeader {
  char magic[8];
  uint64_t version, log_bytes, nbuckets, max_item, head, index_bytes, log_saved, user[4];
};
constexpr char kSnapMagic[8] = {'S', 'H', 'L', 'C', 'S', 'N', 'P', '1'};
}  // namespace

void HbmCache::save(const std::string& path, const uint64_t user[4], hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  HIP_OK(hipStreamSynchronize(s));
  uint64_t head = 0;
  HIP_OK(hipMemcpy(&head, cur_head(), 8, hipMemcpyDeviceToHost));
  const uint64_t slack = item_bytes(cfg_.max_item) + 64;
  SnapHeader h{};
  std::memcpy(h.magic, kSnapMagic, 8);
  h.version = 1;
  h.log_bytes = cfg_.log_bytes;
  h.nbuckets = cfg_.nbuckets;
  h.max_item = cfg_.max_item;
  h.head = head;
  h.index_bytes = cfg_.nbuckets * kBucketBytes;
  h.log_saved = head >= cfg_.log_bytes ? cfg_.log_bytes + slack : std::min(head + slack, cfg_.log_bytes + slack);
  for (int i = 0; i < 4; ++i) h.user[i] = user ? user[i] : 0;
  FILE* f = std::fopen(path.c_str(), "wb");
  SH_CHECK(f, "cannot open snapshot for writing: " + path);
  const size_t chunk = 64u << 20;
  uint8_t* pin = nullptr;
  HIP_OK(hipHostMalloc(&pin, chunk, hipHostMallocDefault));
  bool ok = std::fwrite(&h, sizeof h, 1, f) == 1;
  auto dump = [&](const uint8_t* dev, uint64_t bytes) {
    for (uint64_t o = 0; ok && o < bytes; o += chunk) {
      const size_t n = (size_t)std::min<uint64_t>(chunk, bytes - o);
      HIP_OK(hipMemcpy(pin, dev + o, n, hipMemcpyDeviceToHost));
      ok = std::fwrite(pin, 1, n, f) == n;
    }
  };
  dump(reinterpret_cast<const uint8_t*>(index_), h.index_bytes);
  dump(log_, h.log_saved);
  (void)hipHostFree(pin);
  ok = (std::fclose(f) == 0) && ok;
  SH_CHECK(ok, "snapshot write failed: " + path);
}

void HbmCache::load(const std::string& path, uint64_t user[4], hipStream_t s) {
  serve_stop();  // the snapshot rewrites the index and the log underneath it
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  FILE* f = std::fopen(path.c_str(), "rb");
  SH_CHECK(f, "cannot open snapshot: " + path);
  SnapHeader h{};
  bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, kSnapMagic, 8) == 0;
  if (!ok || h.log_bytes != cfg_.log_bytes || h.nbuckets != cfg_.nbuckets ||
      h.max_item != cfg_.max_item) {
    std::fclose(f);
    throw Error("snapshot " + path + " does not match this shard's geometry");
  }
  HIP_OK(hipStreamSynchronize(s));
  const size_t chunk = 64u << 20;
  uint8_t* pin = nullptr;
  HIP_OK(hipHostMalloc(&pin, chunk, hipHostMallocDefault));
  auto fill = [&](uint8_t* dev, uint64_t bytes) {
    for (uint64_t o = 0; ok && o < bytes; o += chunk) {
      const size_t n = (size_t)std::min<uint64_t>(chunk, bytes - o);
      ok = std::fread(pin, 1, n, f) == n;
      if (ok) HIP_OK(hipMemcpy(dev + o, pin, n, hipMemcpyHostToDevice));
    }
  };
  fill(reinterpret_cast<uint8_t*>(index_), h.index_bytes);
  fill(log_, h.log_saved);
  (void)hipHostFree(pin);
  std::fclose(f);
  SH_CHECK(ok, "snapshot truncated: " + path);
  HIP_OK(hipMemcpy(cur_head(), &h.head, 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(claim_ptr(), &h.head, 8, hipMemcpyHostToDevice));
  // the CLOCK ring is not part of a snapshot: the first lap after a restore is FIFO
  HIP_OK(hipMemset(head_ + 2, 0, 2 * sizeof(uint64_t)));
  if (rc_ctl_) {
    HIP_OK(hipMemset(rc_ctl_, 0, 8 * sizeof(unsigned long long)));
    HIP_OK(hipMemset(rc_ctl_ + 2, 0xff, sizeof(unsigned long long)));
  }
  HIP_OK(hipDeviceSynchronize());  // the null-stream memsets before any other stream's work
  __atomic_store_n(host_slots_ + kHeadSlot, h.head, __ATOMIC_RELEASE);
  if (user)
    for (int i = 0; i < 4; ++i) user[i] = h.user[i];
}

std::vector<uint64_t> HbmCache::debug_bucket(uint64_t b) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  SH_CHECK(b < cfg_.nbuckets, "bucket out of range");
  HIP_OK(hipDeviceSynchronize());
  Entry e[kEntriesPerBucket];
  HIP_OK(hipMemcpy(e, index_ + b * kEntriesPerBucket, sizeof e, hipMemcpyDeviceToHost));
  std::vector<uint64_t> out;
  for (const Entry& x : e)
    for (uint64_t w : {x.d0, x.d1, x.loc, (uint64_t)x.vlen | ((uint64_t)x.expire << 32)})
      out.push_back(w);
  return out;
}

std::vector<uint64_t> HbmCache::debug_hand() {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  HIP_OK(hipDeviceSynchronize());
  uint64_t hand = 0, tail = 0, head = 0, loc = ~0ull;
  if (rc_ctl_) HIP_OK(hipMemcpy(&hand, rc_ctl_, 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&tail, cur_ring_tail(), 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&head, cur_head(), 8, hipMemcpyDeviceToHost));
  if (ring_ && tail > hand && tail - hand <= ring_cap_)
    HIP_OK(hipMemcpy(&loc, ring_ + (hand & (ring_cap_ - 1)), 8, hipMemcpyDeviceToHost));
  unsigned long long ctl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rc_ctl_) HIP_OK(hipMemcpy(ctl, rc_ctl_, sizeof ctl, hipMemcpyDeviceToHost));
  return {hand, tail, head, loc, ctl[4], ctl[5], ctl[6]};
}

void HbmCache::debug_set_hand(uint64_t hand, bool catch_up) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  SH_CHECK(rc_ctl_ != nullptr, "no CLOCK hand (FIFO eviction)");
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(rc_ctl_, &hand, 8, hipMemcpyHostToDevice));
  catch_up_ = catch_up;
}

void HbmCache::debug_set_entry(uint64_t b, int slot, uint64_t d0, uint64_t d1, uint64_t loc,
                               uint32_t vlen, uint32_t expire) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  SH_CHECK(b < cfg_.nbuckets && slot >= 0 && slot < (int)kEntriesPerBucket, "entry out of range");
  HIP_OK(hipDeviceSynchronize());
  const Entry e{d0, d1, loc, vlen, expire};
  HIP_OK(hipMemcpy(index_ + b * kEntriesPerBucket + slot, &e, sizeof e, hipMemcpyHostToDevice));
}

void HbmCache::flush(hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  HIP_OK(hipMemsetAsync(index_, 0, cfg_.nbuckets * kBucketBytes, s));
}

CacheCounters HbmCache::counters(hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  CacheCounters c{};
  HIP_OK(hipMemcpyAsync(host_buf_, ctr_, kCtrShards * sizeof(CacheCounters),
                        hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  const auto* sh = reinterpret_cast<const unsigned long long*>(host_buf_);
  auto* dst = reinterpret_cast<unsigned long long*>(&c);
  constexpr int kWords = sizeof(CacheCounters) / sizeof(unsigned long long);
  for (int k = 0; k < kCtrShards; ++k)
    for (int w = 0; w < kWords; ++w) dst[w] += sh[k * kWords + w];
  return c;
}

uint64_t HbmCache::head(hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  DeviceGuard g(cfg_.device);
  HIP_OK(hipMemcpyAsync(host_buf_, cur_head(), sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return host_buf_[0];
}

}  // namespace shellac
