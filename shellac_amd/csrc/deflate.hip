// Batch gzip on the GPU: one wave per 32 KiB block, greedy LZ77 over an LDS hash table,
// fixed-Huffman DEFLATE codes (RFC 1951 §3.2.6). See deflate.h for the design.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cstring>
#include <stdexcept>

#include "common.h"
#include "deflate.h"
#include "http.h"
#include "huffman.h"

#define GZ_OK(expr)                                                                       \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      throw Error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + #expr);   \
  } while (0)

namespace shellac {
namespace {

constexpr int kHashBits = 12;
constexpr int kHashSize = 1 << kHashBits;
constexpr int kMaxMatch = 258;

__device__ __forceinline__ uint32_t rev(uint32_t code, int len) {
  return __builtin_bitreverse32(code) >> (32 - len);
}

// x^(8n) mod P and (a * b) mod P over GF(2) for the reflected CRC-32 polynomial: the
// register after n more zero bytes is mulx8n(n) * reg, which combines CRCs of slices.
__host__ __device__ inline uint32_t crc_mulmod(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
  }
  return p;
}
__host__ __device__ inline uint32_t crc_x8n(uint64_t n) {
  uint32_t xp = 1u << 31;       // x^0
  uint32_t sq = 1u << 23;       // x^8 (one byte)
  while (n) {
    if (n & 1) xp = crc_mulmod(sq, xp);
    sq = crc_mulmod(sq, sq);
    n >>= 1;
  }
  return xp;
}

__device__ __forceinline__ uint32_t hash4(const uint8_t* s, int p) {
  const uint32_t w = (uint32_t)s[p] | ((uint32_t)s[p + 1] << 8) | ((uint32_t)s[p + 2] << 16) |
                     ((uint32_t)s[p + 3] << 24);
  return (w * 2654435761u) >> (32 - kHashBits);
}

// Symbol of a match length (257..285) / distance (0..29) and its extra bits, by the
// position of the top set bit (RFC 1951 §3.2.5) — no table walk.
__device__ __forceinline__ void len_sym(int len, int* sym, int* nb, uint32_t* val) {
  if (len < 11) {
    *sym = 254 + len; *nb = 0; *val = 0;
  } else if (len == 258) {
    *sym = 285; *nb = 0; *val = 0;
  } else {
    const int L = len - 3;
    const int e = 29 - __clz(L);  // floor(log2 L) - 2
    const int q = (L >> e) & 3;
    *sym = 257 + 4 * e + 4 + q; *nb = e; *val = (uint32_t)(len - 3 - ((4 + q) << e));
  }
}
__device__ __forceinline__ void dist_sym(int dist, int* sym, int* nb, uint32_t* val) {
  const int D = dist - 1;
  if (D < 4) {
    *sym = D; *nb = 0; *val = 0;
  } else {
    const int e = 30 - __clz(D);  // floor(log2 D) - 1
    const int q = (D >> e) & 1;
    *sym = 2 * e + 2 + q; *nb = e; *val = (uint32_t)(D - ((2 + q) << e));
  }
}

// Pass 1: one wave per block; the block, a 4096-entry hash head table and a per-position
// hash chain live in LDS.
//  a. CRC register of the block (lane slices combined by GF(2) multiplies).
//  b. Hash chains, 64 positions per step: every lane hashes its position, finds the lanes
//     of the step with the same hash by 13 ballots (bitwise match), and links to the
//     latest earlier one, or to the head table's entry as of the step; the last lane of
//     each hash then updates the head. prev[p] = the previous position with p's hash.
//  c. Parse, one 1/64 segment of the block per lane: at each position the lane walks up
//     to kChain candidates of the chain, compares 4 bytes at a time (aligned LDS words
//     combined by alignbyte), keeps the longest match, and defers to the next position
//     when that one matches longer (lazy matching, as zlib's levels 4-9). A match never
//     crosses the lane's segment end, so the segments' token lists concatenate.
//  d. The lanes' token lists are compacted into the block's token array (scan of the
//     counts); the literal/length + distance histogram is counted in LDS on the way.
// tab[2b] = src offset, tab[2b+1] = len | final << 32.
constexpr int kChain = 12;        // chain candidates examined per position
constexpr int kNiceLen = 96;      // stop searching at a match this long
constexpr int kLazyLen = 24;      // below this, try the next position (lazy matching)
constexpr int kSegs = 64;         // parse segments per block (one per lane)

__device__ __forceinline__ uint32_t lds_word_at(const uint32_t* w, uint32_t x) {
  // bytes x..x+3 from aligned words (LDS has no unaligned dword reads)
  const uint32_t lo = w[x >> 2], hi = w[(x >> 2) + 1];
  return __builtin_amdgcn_alignbyte(hi, lo, x & 3);
}

// Longest match at p among the chain candidates (length capped at maxl); returns the
// length, *dist the distance.
__device__ __forceinline__ int best_match(const uint8_t* s_in, const uint32_t* s_w,
                                          const uint16_t* s_prev, int p, int maxl, int* dist) {
  int bl = 0, bd = 0;
  int c = s_prev[p];
  for (int depth = 0; c && depth < kChain; ++depth) {
    const int q = c - 1;
    // quick reject: the byte that would extend the best match so far must match
    if (bl < maxl && s_in[q + bl] == s_in[p + bl]) {
      int len = 0;
      while (len < maxl) {
        const uint32_t x = lds_word_at(s_w, (uint32_t)(q + len)) ^ lds_word_at(s_w, (uint32_t)(p + len));
        if (x) {
          len += (int)(__builtin_ctz(x) >> 3);
          break;
        }
        len += 4;
      }
      len = min(len, maxl);
      if (len > bl) {
        bl = len;
        bd = p - q;
        if (bl >= kNiceLen || bl >= maxl) break;
      }
    }
    c = s_prev[q];
  }
  *dist = bd;
  return bl;
}

__global__ __launch_bounds__(64) void k_lz77(const uint8_t* __restrict__ src,
                                             const uint64_t* __restrict__ tab, int64_t nblk,
                                             uint32_t* __restrict__ tok,
                                             uint32_t* __restrict__ stage,
                                             uint32_t* __restrict__ hist,
                                             uint32_t* __restrict__ ntok,
                                             uint32_t* __restrict__ out_crc) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kDeflateBlock + 16];
  __shared__ uint16_t s_prev[kDeflateBlock];
  __shared__ uint16_t s_head[kHashSize];
  __shared__ uint32_t s_hist[kHistSyms];
  const int64_t b = blockIdx.x;
  if (b >= nblk) return;
  const int lane = threadIdx.x;
  const uint64_t off = tab[2 * b];
  const int n = (int)(tab[2 * b + 1] & 0xFFFFFFFFull);
  // blocks start 16-B aligned in the packed input (the host pads every input)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* in4 = reinterpret_cast<const u32x4*>(src + off);
  u32x4* s4 = reinterpret_cast<u32x4*>(s_in);
  const int n16 = (n + 15) / 16;
  for (int i = lane; i < n16; i += 64) s4[i] = in4[i];
  for (int i = n + lane; i < n16 * 16 + 16; i += 64) s_in[i] = 0;  // zero tail (word reads)
  for (int i = lane; i < kHistSyms; i += 64) s_hist[i] = 0;
  // CRC table in the chain array's space (rebuilt below)
  uint32_t* s_crc = reinterpret_cast<uint32_t*>(s_prev);
  for (int i = lane; i < 256; i += 64) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    s_crc[i] = c;
  }
  __syncthreads();
  {
    // CRC register of the block from a zero register (the host folds blocks together)
    const int S = (n + 63) / 64;
    const int a0 = min(n, lane * S), a1 = min(n, a0 + S);
    uint32_t r = 0;
    for (int p = a0; p < a1; ++p) r = s_crc[(r ^ s_in[p]) & 0xFF] ^ (r >> 8);
    r = crc_mulmod(crc_x8n((uint64_t)(n - a1)), r);
    for (int o = 32; o > 0; o >>= 1) r ^= __shfl_xor(r, o);
    if (lane == 0) out_crc[b] = r;
  }
  __syncthreads();
  for (int i = lane; i < kHashSize; i += 64) s_head[i] = 0;
  __syncthreads();
  // b. hash chains
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int p = c0 + lane;
    const bool valid = p + 3 < n;
    const uint32_t h = valid ? hash4(s_in, p) : 0u;
    const uint32_t key = valid ? (h | (1u << kHashBits)) : 0u;  // bit 12: has a hash
    unsigned long long same = ~0ull;
#pragma unroll
    for (int k = 0; k <= kHashBits; ++k) {
      const unsigned long long bal = __ballot((key >> k) & 1u);
      same &= ((key >> k) & 1u) ? bal : ~bal;
    }
    uint32_t cand = valid ? s_head[h] : 0u;
    const unsigned long long earlier = same & below;
    if (earlier) cand = (uint32_t)(c0 + 63 - __clzll((long long)earlier)) + 1;
    if (p < n) s_prev[p] = valid ? (uint16_t)cand : 0;
    const bool last = (same & ~below & ~(1ull << lane)) == 0;
    __builtin_amdgcn_wave_barrier();
    if (valid && last) s_head[h] = (uint16_t)(p + 1);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // c. parse this lane's segment
  const uint32_t* s_w = reinterpret_cast<const uint32_t*>(s_in);
  const int S = (n + kSegs - 1) / kSegs;
  const int a = min(n, lane * S), e = min(n, a + S);
  uint32_t* t = stage + b * (int64_t)kDeflateBlock + (int64_t)lane * S;
  int nt = 0, p = a;
  int nl = -1, nd = 0;  // the next position's search result, when lazy matching made one
  while (p < e) {
    int d = 0;
    int l;
    if (nl >= 0) {
      l = nl;
      d = nd;
    } else {
      l = p + 3 < e ? best_match(s_in, s_w, s_prev, p, min(kMaxMatch, e - p), &d) : 0;
    }
    nl = -1;
    if (l >= 3 && l < kLazyLen && p + 4 < e) {
      int d1 = 0;
      const int l1 = best_match(s_in, s_w, s_prev, p + 1, min(kMaxMatch, e - p - 1), &d1);
      if (l1 > l) {  // a literal now, the longer match next
        nl = l1;
        nd = d1;
        l = 0;
      }
    }
    if (l >= 3) {
      int ls, lb, ds, db;
      uint32_t lv, dv;
      len_sym(l, &ls, &lb, &lv);
      dist_sym(d, &ds, &db, &dv);
      t[nt++] = kTokMatch | ((uint32_t)l << 16) | (uint32_t)(d - 1);
      atomicAdd(&s_hist[ls], 1u);
      atomicAdd(&s_hist[kLitLenSyms + ds], 1u);
      p += l;
    } else {
      const uint32_t lit = s_in[p];
      t[nt++] = lit;
      atomicAdd(&s_hist[lit], 1u);
      p += 1;
    }
  }
  // d. compact the segments' tokens into the block's token array
  uint32_t inc = (uint32_t)nt;
  for (int dd = 1; dd < 64; dd <<= 1) {
    const uint32_t o = __shfl_up(inc, dd);
    if (lane >= dd) inc += o;
  }
  const uint32_t base = inc - (uint32_t)nt;
  uint32_t* dst = tok + b * (int64_t)kDeflateBlock + base;
  for (int k = 0; k < nt; ++k) dst[k] = t[k];
  __syncthreads();
  for (int i = lane; i < kHistSyms; i += 64) hist[b * (int64_t)kHistSyms + i] = s_hist[i];
  if (lane == 63) ntok[b] = inc;
}

// Block planning on the device: one wave per block, its lane 0 runs the shared planner
// (deflate_plan.h) over the block's histogram with the scratch in LDS and writes the plan
// record k_emit encodes with — the batch needs no host round trip between the passes.
__global__ __launch_bounds__(64) void k_plan(const uint64_t* __restrict__ tab, int64_t nblk,
                                             const uint32_t* __restrict__ hist,
                                             uint32_t* __restrict__ plans,
                                             uint32_t* __restrict__ slot) {
  __shared__ PlanScratch s_ws;
  const int64_t b = blockIdx.x;
  if (b >= nblk || threadIdx.x != 0) return;
  const uint64_t meta = tab[2 * b + 1];
  uint32_t* rec = plans + b * (int64_t)kPlanWords;
  plan_block_record(hist + b * (int64_t)kHistSyms, (uint32_t)(meta & 0xFFFFFFFFull),
                    (meta >> 32) != 0, &s_ws, rec);
  // output slot: the planned size, 4-byte aligned, + one word (k_emit stores whole words)
  slot[b] = ((rec[2] + 3) & ~3u) + 4;
}

// Exclusive scan of the blocks' output slots (one workgroup): the compact output layout,
// so the batch's result crosses PCIe at its compressed size, not one stride per block.
__global__ __launch_bounds__(1024) void k_slot_scan(const uint32_t* __restrict__ slot,
                                                    int64_t nblk, uint64_t* __restrict__ off) {
  __shared__ unsigned long long s_w[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t per = (nblk + 1023) / 1024;
  const int64_t a = min(nblk, per * t), e = min(nblk, a + per);
  unsigned long long mine = 0;
  for (int64_t i = a; i < e; ++i) mine += slot[i];
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
    off[nblk] = run;
  }
  __syncthreads();
  unsigned long long run = s_w[w] + inc - mine;
  for (int64_t i = a; i < e; ++i) {
    off[i] = run;
    run += slot[i];
  }
}

// OR `len` (<= 28) bits of v into the LDS bit buffer at bit `pos`.
__device__ __forceinline__ void or_bits(uint32_t* w, uint32_t pos, uint32_t v, int len) {
  if (len == 0) return;
  const uint32_t k = pos >> 5, sh = pos & 31;
  atomicOr(&w[k], v << sh);
  if (sh + len > 32) atomicOr(&w[k + 1], v >> (32 - sh));
}

// Pass 2: one wave per block encodes its tokens with its plan (stored / fixed / dynamic
// codes, k_plan). The codes sit in LDS; each chunk of 64 tokens is placed by
// a wave prefix sum of the tokens' bit lengths and OR-ed into an LDS bit buffer, which is
// then written out whole. A plan record: [mode, header bits, total bytes, codes (316),
// header bytes].
__global__ __launch_bounds__(64) void k_emit(const uint8_t* __restrict__ src,
                                             const uint64_t* __restrict__ tab, int64_t nblk,
                                             const uint32_t* __restrict__ tok,
                                             const uint32_t* __restrict__ ntok,
                                             const uint32_t* __restrict__ plans,
                                             const uint64_t* __restrict__ out_off,
                                             uint8_t* __restrict__ dst,
                                             uint32_t* __restrict__ out_len) {
  __shared__ uint32_t s_code[kHistSyms];
  __shared__ uint32_t s_out[kDeflateStride / 4];
  const int64_t b = blockIdx.x;
  if (b >= nblk) return;
  const int lane = threadIdx.x;
  const uint64_t off = tab[2 * b];
  const int n = (int)(tab[2 * b + 1] & 0xFFFFFFFFull);
  const bool fin = (tab[2 * b + 1] >> 32) != 0;
  const uint32_t* pl = plans + b * (int64_t)kPlanWords;
  const uint32_t mode = pl[0], hbits = pl[1], total = pl[2];
  uint8_t* out = dst + out_off[b];  // 4-byte aligned compact slot
  if (mode == 0) {  // stored: header byte (BFINAL, BTYPE 00, padding), LEN, NLEN, raw bytes
    if (lane == 0) {
      out[0] = fin ? 1 : 0;
      out[1] = (uint8_t)(n & 0xFF);
      out[2] = (uint8_t)(n >> 8);
      out[3] = (uint8_t)(~n & 0xFF);
      out[4] = (uint8_t)((~n >> 8) & 0xFF);
      out_len[b] = (uint32_t)n + 5 | 0x80000000u;  // top bit: stored
    }
    for (int i = lane; i < n; i += 64) out[5 + i] = src[off + i];
    return;
  }
  for (int i = lane; i < kHistSyms; i += 64) s_code[i] = pl[3 + i];
  const int words = (int)((total + 3) / 4) + 1;
  for (int i = lane; i < words; i += 64) s_out[i] = 0;
  __syncthreads();
  const uint8_t* hdr = reinterpret_cast<const uint8_t*>(pl + 3 + kHistSyms);
  uint8_t* s_out8 = reinterpret_cast<uint8_t*>(s_out);
  for (int i = lane; i < (int)((hbits + 7) / 8); i += 64) s_out8[i] = hdr[i];
  __syncthreads();
  uint32_t base = hbits;
  const uint32_t* t = tok + b * (int64_t)kDeflateBlock;
  const int nt = (int)ntok[b];
  for (int c0 = 0; c0 < nt; c0 += 64) {
    const int i = c0 + lane;
    uint32_t av = 0, bv = 0;
    int al = 0, bl = 0;
    if (i < nt) {
      const uint32_t x = t[i];
      if (x & kTokMatch) {
        int ls, lb, ds, db;
        uint32_t lv, dv;
        len_sym((int)((x >> 16) & 0x1FF), &ls, &lb, &lv);
        dist_sym((int)(x & 0xFFFF) + 1, &ds, &db, &dv);
        const uint32_t lc = s_code[ls], dc = s_code[kLitLenSyms + ds];
        al = (int)(lc >> 16) + lb;
        av = (lc & 0xFFFF) | (lv << (lc >> 16));
        bl = (int)(dc >> 16) + db;
        bv = (dc & 0xFFFF) | (dv << (dc >> 16));
      } else {
        const uint32_t lc = s_code[x & 0xFF];
        al = (int)(lc >> 16);
        av = lc & 0xFFFF;
      }
    }
    // inclusive scan of the chunk's bit lengths
    uint32_t inc = (uint32_t)(al + bl);
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= d) inc += o;
    }
    const uint32_t p0 = base + inc - (uint32_t)(al + bl);
    or_bits(s_out, p0, av, al);
    or_bits(s_out, p0 + al, bv, bl);
    base += __shfl(inc, 63);
  }
  __syncthreads();
  if (lane == 0) {
    const uint32_t eob = s_code[256];
    or_bits(s_out, base, eob & 0xFFFF, (int)(eob >> 16));
    base += eob >> 16;
    uint32_t bytes = (base + 7) / 8;
    if (!fin) {  // sync flush: empty stored block (3 zero bits), pad, LEN 0, NLEN 0xFFFF
      bytes = (base + 3 + 7) / 8;
      s_out8[bytes + 2] = 0xFF;
      s_out8[bytes + 3] = 0xFF;
      bytes += 4;
    }
    out_len[b] = bytes;
  }
  __syncthreads();
  uint32_t* o32 = reinterpret_cast<uint32_t*>(out);
  for (int i = lane; i < words; i += 64) o32[i] = s_out[i];
}

// ---------------------------------------------------------------------------------
// Batch inflate (RFC 1951 raw DEFLATE streams, one per gzip member; the host parses the
// gzip framing): one wave per member. Decoding is inherently serial, so the wave runs the
// bit reader and the canonical-Huffman decoder in lockstep (uniform values in every lane)
// while the byte work is spread over the lanes: back-reference copies 64 bytes per step
// (a period-d pattern for d < 64), stored blocks, input refills, output flushes and the
// CRC-32 of the output (lane slices combined by GF(2) multiplies, as the deflate side).
// The 32 KiB window lives in LDS; the output goes to global memory in 1 KiB flushes.
// res[2m] = output bytes | error << 31, res[2m + 1] = CRC-32 of the output.
constexpr int kInfRing = 8192;   // input bytes staged in LDS (two halves)
constexpr int kInfWin = 32768;   // window
constexpr int kInfFlush = 1024;

struct InfHuff {
  uint16_t count[16];
  uint16_t symbol[288];
};

struct InfState {
  const uint8_t* src;
  int64_t in_len;
  int64_t pos;        // next input byte
  int64_t ring_base;  // the ring holds input [ring_base, ring_base + kInfRing)
  uint64_t bitbuf;
  int bitcnt;
};

__device__ void inf_refill_ring(InfState& st, uint8_t* s_ring, int64_t from, int lane) {
  // input [from, from + kInfRing / 2) into its ring half (the wave)
  for (int k = lane; k < kInfRing / 2; k += 64) {
    const int64_t x = from + k;
    s_ring[x & (kInfRing - 1)] = x < st.in_len ? st.src[x] : 0;
  }
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
}

__device__ __forceinline__ uint32_t inf_bits(InfState& st, const uint8_t* s_ring, int n) {
  while (st.bitcnt < n) {
    st.bitbuf |= (uint64_t)s_ring[st.pos & (kInfRing - 1)] << st.bitcnt;
    st.pos++;
    st.bitcnt += 8;
  }
  const uint32_t v = (uint32_t)(st.bitbuf & ((1ull << n) - 1));
  st.bitbuf >>= n;
  st.bitcnt -= n;
  return v;
}

// puff-style canonical decode: one bit at a time against the per-length counts
__device__ __forceinline__ int inf_decode(InfState& st, const uint8_t* s_ring, const InfHuff* h) {
  int code = 0, first = 0, index = 0;
  for (int len = 1; len <= 15; ++len) {
    code |= (int)inf_bits(st, s_ring, 1);
    const int count = h->count[len];
    if (code - count < first) return h->symbol[index + (code - first)];
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

// counts + symbols from code lengths (lane 0 writes); false on an over-subscribed code
__device__ bool inf_construct(InfHuff* h, const uint8_t* len, int n, int lane) {
  bool ok = true;
  if (lane == 0) {
    for (int k = 0; k < 16; ++k) h->count[k] = 0;
    for (int sym = 0; sym < n; ++sym) h->count[len[sym]]++;
    int left = 1;
    for (int k = 1; k < 16; ++k) {
      left <<= 1;
      left -= h->count[k];
      if (left < 0) ok = false;
    }
    uint16_t offs[16];
    offs[1] = 0;
    for (int k = 1; k < 15; ++k) offs[k + 1] = (uint16_t)(offs[k] + h->count[k]);
    for (int sym = 0; sym < n; ++sym)
      if (len[sym]) h->symbol[offs[len[sym]]++] = (uint16_t)sym;
  }
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
  return __shfl(ok ? 1 : 0, 0) != 0;
}

__global__ __launch_bounds__(64) void k_inflate(const uint8_t* __restrict__ in,
                                                const uint64_t* __restrict__ itab,
                                                uint8_t* __restrict__ out,
                                                const uint64_t* __restrict__ otab, int64_t nm,
                                                uint32_t* __restrict__ res) {
  __shared__ uint8_t s_win[kInfWin];
  __shared__ uint8_t s_ring[kInfRing];
  __shared__ uint32_t s_crc[256];
  __shared__ InfHuff s_ll, s_dd;
  __shared__ uint8_t s_len[320];
  const int64_t m = blockIdx.x;
  if (m >= nm) return;
  const int lane = threadIdx.x;
  for (int i = lane; i < 256; i += 64) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    s_crc[i] = c;
  }
  InfState st;
  st.src = in + itab[2 * m];
  st.in_len = (int64_t)itab[2 * m + 1];
  st.pos = 0;
  st.ring_base = 0;
  st.bitbuf = 0;
  st.bitcnt = 0;
  uint8_t* dst = out + otab[2 * m];
  const int64_t cap = (int64_t)otab[2 * m + 1];
  inf_refill_ring(st, s_ring, 0, lane);
  inf_refill_ring(st, s_ring, kInfRing / 2, lane);
  int64_t opos = 0, flushed = 0;
  uint32_t crc = 0xFFFFFFFFu;
  int err = 0;
  // flush s_win[flushed, opos) to the output and fold it into the CRC register
  auto flush = [&]() {
    const int64_t nf = opos - flushed;
    if (nf <= 0) return;
    const int S = (int)((nf + 63) / 64);
    const int64_t a0 = flushed + min((int64_t)lane * S, nf), a1 = min(opos, a0 + S);
    uint32_t r = 0;
    for (int64_t x = a0; x < a1; ++x) {
      const uint8_t byte = s_win[x & (kInfWin - 1)];
      dst[x] = byte;
      r = s_crc[(r ^ byte) & 0xFF] ^ (r >> 8);
    }
    r = crc_mulmod(crc_x8n((uint64_t)(opos - a1)), r);
    for (int o = 32; o > 0; o >>= 1) r ^= __shfl_xor(r, o);
    crc = crc_mulmod(crc_x8n((uint64_t)nf), crc) ^ r;
    flushed = opos;
  };
  auto maybe_refill = [&]() {
    if (st.pos - st.ring_base >= (3 * kInfRing) / 4) {
      inf_refill_ring(st, s_ring, st.ring_base + kInfRing, lane);
      st.ring_base += kInfRing / 2;
    }
  };
  __syncthreads();
  bool last = false;
  while (!last && !err) {
    maybe_refill();
    last = inf_bits(st, s_ring, 1) != 0;
    const uint32_t type = inf_bits(st, s_ring, 2);
    if (type == 0) {  // stored: byte-aligned LEN, NLEN, raw bytes
      st.bitbuf = 0;
      st.bitcnt = 0;  // drop the partial byte (whole bytes were never pre-loaded)
      const uint32_t len = inf_bits(st, s_ring, 16);
      const uint32_t nlen = inf_bits(st, s_ring, 16);
      if ((len ^ 0xFFFFu) != nlen) { err = 1; break; }
      if (opos + len > cap || st.pos + len > st.in_len) { err = 2; break; }
      uint32_t done = 0;
      while (done < len) {
        maybe_refill();
        const uint32_t chunk = min(len - done, (uint32_t)kInfRing / 4);
        if (opos - flushed + chunk > kInfWin - 512) flush();
        for (uint32_t k = lane; k < chunk; k += 64)
          s_win[(opos + k) & (kInfWin - 1)] = s_ring[(st.pos + k) & (kInfRing - 1)];
        __builtin_amdgcn_wave_barrier();
        __syncthreads();
        st.pos += chunk;
        opos += chunk;
        done += chunk;
      }
      continue;
    }
    if (type == 3) { err = 3; break; }
    if (type == 1) {  // fixed codes (RFC 1951 §3.2.6)
      if (lane == 0) {
        for (int sym = 0; sym < 288; ++sym) s_len[sym] = sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : 8;
        for (int sym = 0; sym < 30; ++sym) s_len[288 + sym] = 5;
      }
      __syncthreads();
      inf_construct(&s_ll, s_len, 288, lane);
      inf_construct(&s_dd, s_len + 288, 30, lane);
    } else {  // dynamic codes
      const int nlen = (int)inf_bits(st, s_ring, 5) + 257;
      const int ndist = (int)inf_bits(st, s_ring, 5) + 1;
      const int ncode = (int)inf_bits(st, s_ring, 4) + 4;
      if (nlen > 286 || ndist > 30) { err = 4; break; }
      const int kOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      uint32_t clv[19];
      for (int k = 0; k < 19; ++k) clv[k] = k < ncode ? inf_bits(st, s_ring, 3) : 0;
      if (lane == 0)
        for (int k = 0; k < 19; ++k) s_len[kOrd[k]] = (uint8_t)clv[k];
      __syncthreads();
      if (!inf_construct(&s_ll, s_len, 19, lane)) { err = 5; break; }
      int idx = 0;
      uint8_t prevlen = 0;
      uint8_t lens[316];
      while (idx < nlen + ndist) {
        int sym = inf_decode(st, s_ring, &s_ll);
        if (sym < 0) { err = 6; break; }
        if (sym < 16) {
          lens[idx++] = (uint8_t)sym;
          prevlen = (uint8_t)sym;
        } else {
          int rep;
          uint8_t v = 0;
          if (sym == 16) {
            if (idx == 0) { err = 7; break; }
            v = prevlen;
            rep = 3 + (int)inf_bits(st, s_ring, 2);
          } else if (sym == 17) {
            rep = 3 + (int)inf_bits(st, s_ring, 3);
          } else {
            rep = 11 + (int)inf_bits(st, s_ring, 7);
          }
          if (idx + rep > nlen + ndist) { err = 8; break; }
          while (rep--) lens[idx++] = v;
          if (sym != 16) prevlen = 0;
        }
      }
      if (err) break;
      if (lens[256] == 0) { err = 9; break; }
      if (lane == 0) {
        for (int k = 0; k < 320; ++k) s_len[k] = 0;
        for (int k = 0; k < nlen; ++k) s_len[k] = lens[k];
        for (int k = 0; k < ndist; ++k) s_len[288 + k] = lens[nlen + k];
      }
      __syncthreads();
      inf_construct(&s_ll, s_len, nlen, lane);
      inf_construct(&s_dd, s_len + 288, ndist, lane);
    }
    // the block's symbols
    static constexpr uint16_t kLBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27,
                                            31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
                                            227, 258};
    static constexpr uint8_t kLExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                          2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    static constexpr uint16_t kDBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                            193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
                                            4097, 6145, 8193, 12289, 16385, 24577};
    static constexpr uint8_t kDExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                          6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
    for (;;) {
      maybe_refill();
      if (opos - flushed > kInfWin - 2 * 258 - kInfFlush) flush();
      else if (opos - flushed >= kInfFlush) flush();
      const int sym = inf_decode(st, s_ring, &s_ll);
      if (sym < 0) { err = 10; break; }
      if (sym < 256) {
        if (opos >= cap) { err = 2; break; }
        if (lane == 0) s_win[opos & (kInfWin - 1)] = (uint8_t)sym;
        __builtin_amdgcn_wave_barrier();
        opos++;
        continue;
      }
      if (sym == 256) break;
      const int ls = sym - 257;
      if (ls >= 29) { err = 11; break; }
      const int len = kLBase[ls] + (int)inf_bits(st, s_ring, kLExt[ls]);
      const int ds = inf_decode(st, s_ring, &s_dd);
      if (ds < 0 || ds >= 30) { err = 12; break; }
      const int dist = kDBase[ds] + (int)inf_bits(st, s_ring, kDExt[ds]);
      if (dist > opos) { err = 13; break; }
      if (opos + len > cap) { err = 2; break; }
      __syncthreads();
      for (int k0 = 0; k0 < len; k0 += 64) {
        const int k = k0 + lane;
        uint8_t byte = 0;
        if (k < len) {
          const int64_t srcp = dist < 64 ? opos - dist + (k % dist) : opos - dist + k;
          byte = s_win[srcp & (kInfWin - 1)];
        }
        __syncthreads();
        if (k < len) s_win[(opos + k) & (kInfWin - 1)] = byte;
        __syncthreads();
      }
      opos += len;
    }
  }
  if (!err) flush();
  if (lane == 0) {
    res[2 * m] = (uint32_t)min(opos, (int64_t)0x7FFFFFFF) | (err ? 0x80000000u : 0u);
    res[2 * m + 1] = ~crc;
  }
}

}  // namespace

GpuGzip::GpuGzip(int device) : device_(device) {
  GZ_OK(hipSetDevice(device_));
  GZ_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
}

GpuGzip::~GpuGzip() {
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(stream_);
  for (void* p : {(void*)h_in_, (void*)h_out_, (void*)h_tab_, (void*)h_len_})
    if (p) (void)hipHostFree(p);
  for (void* p : {(void*)d_in_, (void*)d_out_, (void*)d_tab_, (void*)d_len_, (void*)d_res_,
                  (void*)d_plan_, (void*)d_tok_, (void*)d_slot_})
    if (p) (void)hipFree(p);
  (void)hipStreamDestroy(stream_);
}

template <typename T>
T* GpuGzip::grow(T** p, size_t* cap, size_t count, bool host) {
  const size_t need = std::max<size_t>(count, 1) * sizeof(T);
  if (*cap < need) {
    if (*p) {
      if (host) GZ_OK(hipHostFree(*p));
      else GZ_OK(hipFree(*p));
    }
    const size_t c = (need + need / 4 + 4095) & ~(size_t)4095;
    void* q = nullptr;
    if (host) GZ_OK(hipHostMalloc(&q, c, hipHostMallocDefault));
    else GZ_OK(hipMalloc(&q, c));
    *p = static_cast<T*>(q);
    *cap = c;
  }
  return *p;
}

std::vector<std::string> GpuGzip::compress(const std::vector<std::string_view>& in) {
  std::vector<std::string> out;
  run(in, &out, true);
  return out;
}

std::vector<std::string> GpuGzip::deflate(const std::vector<std::string_view>& in) {
  std::vector<std::string> out;
  run(in, &out, false);
  return out;
}

// gzip member -> (raw DEFLATE offset, length, ISIZE, CRC) or false (framing, RFC 1952)
static bool parse_gzip_member(std::string_view z, size_t* off, size_t* len, uint32_t* isize,
                              uint32_t* crc) {
  if (z.size() < 18 || (uint8_t)z[0] != 0x1f || (uint8_t)z[1] != 0x8b || z[2] != 8) return false;
  const uint8_t flg = (uint8_t)z[3];
  size_t p = 10;
  if (flg & 4) {  // FEXTRA
    if (p + 2 > z.size()) return false;
    p += 2 + ((uint8_t)z[p] | ((size_t)(uint8_t)z[p + 1] << 8));
  }
  for (int f : {8, 16}) {  // FNAME, FCOMMENT: zero-terminated
    if (flg & f) {
      while (p < z.size() && z[p]) ++p;
      ++p;
    }
  }
  if (flg & 2) p += 2;  // FHCRC
  if (p + 8 > z.size()) return false;
  auto u32 = [&](size_t q) {
    return (uint32_t)(uint8_t)z[q] | ((uint32_t)(uint8_t)z[q + 1] << 8) |
           ((uint32_t)(uint8_t)z[q + 2] << 16) | ((uint32_t)(uint8_t)z[q + 3] << 24);
  };
  *off = p;
  *len = z.size() - 8 - p;
  *crc = u32(z.size() - 8);
  *isize = u32(z.size() - 4);
  return true;
}

std::vector<std::string> GpuGzip::inflate(const std::vector<std::string_view>& in,
                                          std::vector<uint8_t>* ok, uint64_t max_out) {
  std::lock_guard<std::mutex> lk(mu_);
  GZ_OK(hipSetDevice(device_));
  const size_t nm = in.size();
  std::vector<std::string> out(nm);
  ok->assign(nm, 0);
  if (nm == 0) return out;
  // members whose framing parses and whose ISIZE fits the cap go to the GPU
  std::vector<size_t> doff(nm), dlen(nm), osz(nm);
  std::vector<uint32_t> want_crc(nm);
  size_t packed = 0, obytes = 0;
  for (size_t i = 0; i < nm; ++i) {
    uint32_t isize = 0;
    if (!parse_gzip_member(in[i], &doff[i], &dlen[i], &isize, &want_crc[i]) || isize > max_out) {
      dlen[i] = 0;
      osz[i] = ~(size_t)0;  // not decoded
      continue;
    }
    osz[i] = isize;
    packed += (dlen[i] + 15) & ~(size_t)15;
    obytes += (isize + 15) & ~(size_t)15;
  }
  uint8_t* hin = grow(&h_in_, &h_in_cap_, packed + 16, true);
  uint8_t* din = grow(&d_in_, &d_in_cap_, packed + 16, false);
  uint64_t* htab = grow(&h_tab_, &h_tab_cap_, 4 * nm, true);
  uint64_t* dtab = grow(&d_tab_, &d_tab_cap_, 4 * nm, false);
  uint8_t* dout = grow(&d_out_, &d_out_cap_, obytes + 16, false);
  uint8_t* hout = grow(&h_out_, &h_out_cap_, obytes + 16, true);
  uint32_t* hres = grow(&h_len_, &h_len_cap_, 2 * nm, true);
  uint32_t* dres = grow(&d_len_, &d_len_cap_, 2 * nm, false);
  size_t ip = 0, op = 0;
  for (size_t i = 0; i < nm; ++i) {
    const size_t cap = osz[i] == ~(size_t)0 ? 0 : osz[i];
    if (dlen[i]) std::memcpy(hin + ip, in[i].data() + doff[i], dlen[i]);
    htab[2 * i] = ip;
    htab[2 * i + 1] = dlen[i];
    htab[2 * nm + 2 * i] = op;
    htab[2 * nm + 2 * i + 1] = cap;
    ip += (dlen[i] + 15) & ~(size_t)15;
    op += (cap + 15) & ~(size_t)15;
  }
  GZ_OK(hipMemcpyAsync(din, hin, packed + 16, hipMemcpyHostToDevice, stream_));
  GZ_OK(hipMemcpyAsync(dtab, htab, 4 * nm * sizeof(uint64_t), hipMemcpyHostToDevice, stream_));
  hipLaunchKernelGGL(k_inflate, dim3((unsigned)nm), dim3(64), 0, stream_, din, dtab, dout,
                     dtab + 2 * nm, (int64_t)nm, dres);
  GZ_OK(hipGetLastError());
  GZ_OK(hipMemcpyAsync(hres, dres, 2 * nm * sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  GZ_OK(hipMemcpyAsync(hout, dout, obytes + 16, hipMemcpyDeviceToHost, stream_));
  GZ_OK(hipStreamSynchronize(stream_));
  for (size_t i = 0; i < nm; ++i) {
    if (osz[i] == ~(size_t)0) continue;
    const uint32_t r = hres[2 * i];
    const uint32_t got = r & 0x7FFFFFFFu;
    // a member is good when it decoded without error to exactly ISIZE bytes with its CRC
    if ((r >> 31) || got != osz[i] || hres[2 * i + 1] != want_crc[i]) continue;
    out[i].assign(reinterpret_cast<const char*>(hout + htab[2 * nm + 2 * i]), got);
    (*ok)[i] = 1;
  }
  stats_.inflated += nm;
  return out;
}

void GpuGzip::run(const std::vector<std::string_view>& in, std::vector<std::string>* out,
                  bool gzip) {
  std::lock_guard<std::mutex> lk(mu_);
  GZ_OK(hipSetDevice(device_));
  // block table: every input has at least one block (an empty input: one empty final block)
  // inputs are packed 16-B aligned (the kernel stages blocks with 16-B loads)
  size_t nblk = 0, total = 0, packed = 0;
  for (const auto& s : in) {
    nblk += std::max<size_t>(1, (s.size() + kDeflateBlock - 1) / kDeflateBlock);
    total += s.size();
    packed += (s.size() + 15) & ~(size_t)15;
  }
  out->assign(in.size(), std::string());
  if (in.empty()) return;
  uint8_t* hin = grow(&h_in_, &h_in_cap_, packed + 16, true);
  uint8_t* din = grow(&d_in_, &d_in_cap_, packed + 16, false);
  uint64_t* htab = grow(&h_tab_, &h_tab_cap_, 2 * nblk, true);
  uint64_t* dtab = grow(&d_tab_, &d_tab_cap_, 2 * nblk, false);
  // pass-1 results [histograms (316 per block) | token counts | CRC registers] and pass-2
  // lengths: one D2H each
  const size_t nres = nblk * (size_t)kHistSyms + nblk;
  uint32_t* dres = grow(&d_res_, &d_res_cap_, nres, false);
  // [lengths (nblk) | CRC registers (nblk) | slot offsets (nblk + 1, u64)]: one D2H
  const size_t nlen = 2 * nblk + 2 * (nblk + 1) + 2;
  uint32_t* hlen = grow(&h_len_, &h_len_cap_, nlen, true);
  uint32_t* dlen = grow(&d_len_, &d_len_cap_, nlen, false);
  uint32_t* dslot = grow(&d_slot_, &d_slot_cap_, nblk, false);
  uint64_t* doff = reinterpret_cast<uint64_t*>(dlen + 2 * nblk + ((2 * nblk) & 1));
  const uint64_t* hoff = reinterpret_cast<const uint64_t*>(hlen + 2 * nblk + ((2 * nblk) & 1));
  // tokens: the parse's per-segment lists (stage) compacted into one list per block (tok)
  uint32_t* dtok = grow(&d_tok_, &d_tok_cap_, 2 * nblk * (size_t)kDeflateBlock, false);
  uint32_t* dstage = dtok + nblk * (size_t)kDeflateBlock;
  uint32_t* dplan = grow(&d_plan_, &d_plan_cap_, nblk * (size_t)kPlanWords, false);
  uint32_t* dhist = dres;
  uint32_t* dntok = dres + nblk * (size_t)kHistSyms;
  uint32_t* dcrc = dlen + nblk;
  const uint32_t* hcrc = hlen + nblk;
  const size_t out_bound = packed + 16 * nblk + 64;
  uint8_t* dout = grow(&d_out_, &d_out_cap_, out_bound, false);
  uint8_t* hout = grow(&h_out_, &h_out_cap_, out_bound, true);
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  size_t o = 0, k = 0;
  for (const auto& s : in) {
    if (!s.empty()) std::memcpy(hin + o, s.data(), s.size());
    size_t done = 0;
    do {
      const size_t len = std::min<size_t>(kDeflateBlock, s.size() - done);
      const bool fin = done + len == s.size();
      htab[2 * k] = o + done;
      htab[2 * k + 1] = (uint64_t)len | ((uint64_t)fin << 32);
      ++k;
      done += len;
    } while (done < s.size());
    o += (s.size() + 15) & ~(size_t)15;
  }
  const auto t1 = clk::now();
  GZ_OK(hipMemcpyAsync(din, hin, packed + 16, hipMemcpyHostToDevice, stream_));
  GZ_OK(hipMemcpyAsync(dtab, htab, 2 * nblk * sizeof(uint64_t), hipMemcpyHostToDevice, stream_));
  hipLaunchKernelGGL(k_lz77, dim3((unsigned)nblk), dim3(64), 0, stream_, din, dtab,
                     (int64_t)nblk, dtok, dstage, dhist, dntok, dcrc);
  GZ_OK(hipGetLastError());
  hipLaunchKernelGGL(k_plan, dim3((unsigned)nblk), dim3(64), 0, stream_, dtab, (int64_t)nblk,
                     dhist, dplan, dslot);
  hipLaunchKernelGGL(k_slot_scan, dim3(1), dim3(1024), 0, stream_, dslot, (int64_t)nblk, doff);
  hipLaunchKernelGGL(k_emit, dim3((unsigned)nblk), dim3(64), 0, stream_, din, dtab,
                     (int64_t)nblk, dtok, dntok, dplan, doff, dout, dlen);
  GZ_OK(hipGetLastError());
  // one D2H of [lengths | CRC registers | slot offsets], one of the compact output; its
  // extent is bounded by the stored encoding of every block (the input + 9 B per block)
  GZ_OK(hipMemcpyAsync(hlen, dlen, (2 * nblk + 2 * (nblk + 1)) * sizeof(uint32_t),
                       hipMemcpyDeviceToHost, stream_));
  GZ_OK(hipMemcpyAsync(hout, dout, out_bound, hipMemcpyDeviceToHost, stream_));
  GZ_OK(hipStreamSynchronize(stream_));
  const auto t2 = clk::now();
  // assemble: [gzip header] deflate blocks [CRC-32, ISIZE]
  static const unsigned char kHdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 0xff};
  k = 0;
  for (size_t i = 0; i < in.size(); ++i) {
    const auto& s = in[i];
    const size_t nb = std::max<size_t>(1, (s.size() + kDeflateBlock - 1) / kDeflateBlock);
    size_t bytes = gzip ? 18 : 0;
    for (size_t j = 0; j < nb; ++j) bytes += hlen[k + j] & 0x7FFFFFFFu;
    std::string& r = (*out)[i];
    r.reserve(bytes);
    if (gzip) r.append(reinterpret_cast<const char*>(kHdr), 10);
    // CRC-32 of the input from the blocks' registers: reg <- reg * x^(8 len) + r_block
    uint32_t reg = 0xFFFFFFFFu;
    for (size_t j = 0; j < nb; ++j, ++k) {
      const uint32_t l = hlen[k];
      stats_.stored_blocks += l >> 31;
      r.append(reinterpret_cast<const char*>(hout + hoff[k]), l & 0x7FFFFFFFu);
      const uint64_t blen = std::min<uint64_t>(kDeflateBlock, s.size() - j * kDeflateBlock);
      reg = crc_mulmod(crc_x8n(blen), reg) ^ hcrc[k];
    }
    if (gzip) {
      const uint32_t crc = ~reg;
      const uint32_t isz = (uint32_t)s.size();
      for (int t = 0; t < 4; ++t) r.push_back((char)((crc >> (8 * t)) & 0xFF));
      for (int t = 0; t < 4; ++t) r.push_back((char)((isz >> (8 * t)) & 0xFF));
    }
    stats_.out_bytes += r.size();
  }
  const auto ms = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  stats_.last_pack_ms = ms(t0, t1);
  stats_.last_gpu_ms = ms(t1, t2);
  stats_.last_assemble_ms = ms(t2, clk::now());
  stats_.inputs += in.size();
  stats_.blocks += nblk;
  stats_.in_bytes += total;
}

GzipService::GzipService(int device, int batch_us, size_t max_batch, int workers)
    : batch_us_(batch_us), max_batch_(std::max<size_t>(1, max_batch)) {
  for (int i = 0; i < std::max(1, workers); ++i) gz_.emplace_back(new GpuGzip(device));
  for (auto& g : gz_) {
    GpuGzip* e = g.get();
    th_.emplace_back([this, e] { loop(e); });
  }
}

GzipService::~GzipService() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_)
    if (t.joinable()) t.join();
}

void GzipService::submit(std::string body, Done done) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(Job{std::move(body), std::move(done), false, 0});
  }
  cv_.notify_one();
}

void GzipService::submit_inflate(std::string member, uint64_t max_out, Done done) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(Job{std::move(member), std::move(done), true, max_out});
  }
  cv_.notify_one();
}

// One GpuGzip::inflate call for the batch; members it does not decode (or whose output
// exceeds their own cap) go through zlib here, on the service thread.
void GzipService::run_inflate(GpuGzip* gz, std::vector<Job>& batch) {
  std::vector<std::string_view> v;
  uint64_t cap = 0;
  for (const auto& j : batch) {
    v.emplace_back(j.body);
    cap = std::max(cap, j.max_out);
  }
  std::vector<std::string> out;
  std::vector<uint8_t> okv;
  try {
    out = gz->inflate(v, &okv, cap);
  } catch (const std::exception&) {
    out.assign(batch.size(), std::string());
    okv.assign(batch.size(), 0);
  }
  uint64_t gpu = 0, cpu = 0, bad = 0;
  for (size_t i = 0; i < batch.size(); ++i) {
    if (okv[i] && out[i].size() <= batch[i].max_out) {
      ++gpu;
      batch[i].done(true, std::move(out[i]));
      continue;
    }
    std::string o;
    const bool ok = gzip_decompress(batch[i].body, &o, batch[i].max_out);
    ok ? ++cpu : ++bad;
    batch[i].done(ok, ok ? std::move(o) : std::string());
  }
  std::lock_guard<std::mutex> lk(mu_);
  st_.inflate_batches++;
  st_.inflated_gpu += gpu;
  st_.inflated_cpu += cpu;
  st_.inflate_errors += bad;
}

GzipService::Stats GzipService::totals() {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

void GzipService::stats(StatList* out) {
  const Stats t = totals();
  out->emplace_back("batches", t.batches);
  out->emplace_back("bodies", t.bodies);
  out->emplace_back("in_bytes", t.in_bytes);
  out->emplace_back("out_bytes", t.out_bytes);
  out->emplace_back("errors", t.errors);
  out->emplace_back("inflate_batches", t.inflate_batches);
  out->emplace_back("inflated_gpu", t.inflated_gpu);
  out->emplace_back("inflated_cpu", t.inflated_cpu);
  out->emplace_back("inflate_errors", t.inflate_errors);
}

void GzipService::loop(GpuGzip* gz) {
  std::vector<Job> batch;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty() && stop_) return;
      // collect for up to batch_us after the first submission (or until max_batch)
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(batch_us_);
      cv_.wait_until(lk, until, [&] { return stop_ || q_.size() >= max_batch_; });
      // one kind per batch: the compress or inflate jobs at the front of the queue
      while (!q_.empty() && batch.size() < max_batch_ &&
             (batch.empty() || q_.front().inflate == batch.front().inflate)) {
        batch.push_back(std::move(q_.front()));
        q_.pop_front();
      }
    }
    if (batch.empty()) continue;  // another worker took this window's bodies
    if (batch.front().inflate) {
      run_inflate(gz, batch);
      batch.clear();
      continue;
    }
    std::vector<std::string_view> v;
    v.reserve(batch.size());
    uint64_t inb = 0;
    for (const auto& j : batch) {
      v.emplace_back(j.body);
      inb += j.body.size();
    }
    std::vector<std::string> out;
    bool ok = true;
    try {
      out = gz->compress(v);
    } catch (const std::exception&) {
      ok = false;
    }
    uint64_t outb = 0;
    for (size_t i = 0; i < batch.size(); ++i) {
      if (ok) {
        outb += out[i].size();
        batch[i].done(true, std::move(out[i]));
      } else {
        batch[i].done(false, std::move(batch[i].body));
      }
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      st_.batches++;
      st_.bodies += batch.size();
      st_.in_bytes += inb;
      st_.out_bytes += outb;
      st_.errors += ok ? 0 : 1;
    }
    batch.clear();
  }
}

}  // namespace shellac
