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
// plan record per block: mode, header bits, total bytes, codes, header bytes (<= 640)
constexpr int kPlanWords = 3 + kHistSyms + 160;

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

// Pass 1: one wave per block. The block and a 4096-entry hash head table live in LDS;
// the wave parses greedily (the 64 lanes compare a candidate 64 bytes per ballot and hash
// the positions a match covers in parallel) and writes tokens (huffman.h) plus the
// block's literal/length and distance histogram, and the block's CRC register.
// tab[2b] = src offset, tab[2b+1] = len | final << 32.
__global__ __launch_bounds__(64) void k_lz77(const uint8_t* __restrict__ src,
                                             const uint64_t* __restrict__ tab, int64_t nblk,
                                             uint32_t* __restrict__ tok,
                                             uint32_t* __restrict__ hist,
                                             uint32_t* __restrict__ ntok,
                                             uint32_t* __restrict__ out_crc) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kDeflateBlock + 16];
  __shared__ uint32_t s_head[kHashSize];
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
  for (int i = n + lane; i < n16 * 16 + 16; i += 64) s_in[i] = 0;  // zero tail (hash reads)
  for (int i = lane; i < kHistSyms; i += 64) s_hist[i] = 0;
  // CRC table in the head table's space (it is cleared after the CRC pass)
  for (int i = lane; i < 256; i += 64) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    s_head[i] = c;
  }
  __syncthreads();
  {
    // CRC register of the block from a zero register (the host folds blocks together):
    // lane i takes slice [i*S, min(n, (i+1)*S)), then shifts its register past the
    // bytes after its slice and the wave XORs the registers
    const int S = (n + 63) / 64;
    const int a0 = min(n, lane * S), a1 = min(n, a0 + S);
    uint32_t r = 0;
    for (int p = a0; p < a1; ++p) r = s_head[(r ^ s_in[p]) & 0xFF] ^ (r >> 8);
    r = crc_mulmod(crc_x8n((uint64_t)(n - a1)), r);
    for (int o = 32; o > 0; o >>= 1) r ^= __shfl_xor(r, o);
    if (lane == 0) out_crc[b] = r;
  }
  __syncthreads();
  for (int i = lane; i < kHashSize; i += 64) s_head[i] = 0;
  __syncthreads();

  uint32_t* t = tok + b * (int64_t)kDeflateBlock;
  int nt = 0;
  int pos = 0;
  while (pos < n) {
    int len = 0, dist = 0;
    if (pos + 3 < n) {
      const uint32_t h = hash4(s_in, pos);
      const uint32_t c = s_head[h];
      // one wave per workgroup: its LDS operations complete in issue order, so a wave
      // barrier (no s_barrier, only no code motion across it) orders the read before
      // lane 0 replaces the head
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) s_head[h] = (uint32_t)pos + 1;
      if (c) {
        const int cand = (int)c - 1;
        const int maxl = min(kMaxMatch, n - pos);
        for (int base = 0; base < maxl; base += 64) {
          const int k = base + lane;
          const bool eq = k < maxl && s_in[cand + k] == s_in[pos + k];
          const unsigned long long miss = __ballot(!eq);
          if (miss) {
            len = base + __ffsll((long long)miss) - 1;
            break;
          }
          len = base + 64;
        }
        len = min(len, maxl);
        dist = pos - cand;
      }
    }
    if (len >= 3) {
      if (lane == 0) {
        int ls, lb, ds, db;
        uint32_t lv, dv;
        len_sym(len, &ls, &lb, &lv);
        dist_sym(dist, &ds, &db, &dv);
        t[nt] = kTokMatch | ((uint32_t)len << 16) | (uint32_t)(dist - 1);
        s_hist[ls]++;
        s_hist[kLitLenSyms + ds]++;
      }
      // hash the positions the match covers (latest position wins)
      for (int q = 1 + lane; q < len; q += 64) {
        const int p = pos + q;
        if (p + 3 < n) atomicMax(&s_head[hash4(s_in, p)], (uint32_t)p + 1);
      }
      pos += len;
    } else {
      if (lane == 0) {
        const uint32_t lit = s_in[pos];
        t[nt] = lit;
        s_hist[lit]++;
      }
      pos += 1;
    }
    ++nt;
    __builtin_amdgcn_wave_barrier();  // head-table updates precede the next lookup
  }
  __syncthreads();
  for (int i = lane; i < kHistSyms; i += 64) hist[b * (int64_t)kHistSyms + i] = s_hist[i];
  if (lane == 0) ntok[b] = (uint32_t)nt;
}

// OR `len` (<= 28) bits of v into the LDS bit buffer at bit `pos`.
__device__ __forceinline__ void or_bits(uint32_t* w, uint32_t pos, uint32_t v, int len) {
  if (len == 0) return;
  const uint32_t k = pos >> 5, sh = pos & 31;
  atomicOr(&w[k], v << sh);
  if (sh + len > 32) atomicOr(&w[k + 1], v >> (32 - sh));
}

// Pass 2: one wave per block encodes its tokens with the host's plan (stored / fixed /
// dynamic codes, huffman.cc). The codes sit in LDS; each chunk of 64 tokens is placed by
// a wave prefix sum of the tokens' bit lengths and OR-ed into an LDS bit buffer, which is
// then written out whole. A plan record: [mode, header bits, total bytes, codes (316),
// header bytes].
__global__ __launch_bounds__(64) void k_emit(const uint8_t* __restrict__ src,
                                             const uint64_t* __restrict__ tab, int64_t nblk,
                                             const uint32_t* __restrict__ tok,
                                             const uint32_t* __restrict__ ntok,
                                             const uint32_t* __restrict__ plans,
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
  uint8_t* out = dst + b * (int64_t)kDeflateStride;
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

}  // namespace

GpuGzip::GpuGzip(int device) : device_(device) {
  GZ_OK(hipSetDevice(device_));
  GZ_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
}

GpuGzip::~GpuGzip() {
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(stream_);
  for (void* p : {(void*)h_in_, (void*)h_out_, (void*)h_tab_, (void*)h_len_, (void*)h_res_,
                  (void*)h_plan_})
    if (p) (void)hipHostFree(p);
  for (void* p : {(void*)d_in_, (void*)d_out_, (void*)d_tab_, (void*)d_len_, (void*)d_res_,
                  (void*)d_plan_, (void*)d_tok_})
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
  const size_t nres = nblk * (size_t)kHistSyms + 2 * nblk;
  uint32_t* hres = grow(&h_res_, &h_res_cap_, nres, true);
  uint32_t* dres = grow(&d_res_, &d_res_cap_, nres, false);
  uint32_t* hlen = grow(&h_len_, &h_len_cap_, nblk, true);
  uint32_t* dlen = grow(&d_len_, &d_len_cap_, nblk, false);
  uint32_t* dtok = grow(&d_tok_, &d_tok_cap_, nblk * (size_t)kDeflateBlock, false);
  uint32_t* hplan = grow(&h_plan_, &h_plan_cap_, nblk * (size_t)kPlanWords, true);
  uint32_t* dplan = grow(&d_plan_, &d_plan_cap_, nblk * (size_t)kPlanWords, false);
  uint32_t* dhist = dres;
  uint32_t* dntok = dres + nblk * (size_t)kHistSyms;
  uint32_t* dcrc = dntok + nblk;
  const uint32_t* hhist = hres;
  const uint32_t* hcrc = hres + nblk * (size_t)kHistSyms + nblk;
  uint8_t* dout = grow(&d_out_, &d_out_cap_, nblk * (size_t)kDeflateStride, false);
  uint8_t* hout = grow(&h_out_, &h_out_cap_, nblk * (size_t)kDeflateStride, true);
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
                     (int64_t)nblk, dtok, dhist, dntok, dcrc);
  GZ_OK(hipGetLastError());
  GZ_OK(hipMemcpyAsync(hres, dres, nres * sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  GZ_OK(hipStreamSynchronize(stream_));
  // plan every block (stored / fixed / dynamic codes and header) on a few host threads
  {
    const size_t nth = std::min<size_t>(std::max<size_t>(1, nblk / 64),
                                        std::max(1u, std::min(8u, std::thread::hardware_concurrency() / 2)));
    auto work = [&](size_t lo, size_t hi) {
      BlockPlan bp;
      for (size_t bi = lo; bi < hi; ++bi) {
        const uint64_t meta = htab[2 * bi + 1];
        plan_block(hhist + bi * kHistSyms, (uint32_t)(meta & 0xFFFFFFFFu), (meta >> 32) != 0, &bp);
        uint32_t* rec = hplan + bi * (size_t)kPlanWords;
        rec[0] = (uint32_t)bp.mode;
        rec[1] = bp.header_bits;
        rec[2] = (uint32_t)bp.total_bytes;
        std::memcpy(rec + 3, bp.codes, sizeof(bp.codes));
        SH_CHECK(bp.header.size() <= 4 * (size_t)(kPlanWords - 3 - kHistSyms), "gzip header too long");
        std::memset(rec + 3 + kHistSyms, 0, 4 * (size_t)(kPlanWords - 3 - kHistSyms));
        std::memcpy(rec + 3 + kHistSyms, bp.header.data(), bp.header.size());
      }
    };
    std::vector<std::thread> ths;
    const size_t per = (nblk + nth - 1) / nth;
    for (size_t ti = 1; ti < nth; ++ti)
      ths.emplace_back(work, std::min(nblk, ti * per), std::min(nblk, (ti + 1) * per));
    work(0, std::min(nblk, per));
    for (auto& th : ths) th.join();
  }
  GZ_OK(hipMemcpyAsync(dplan, hplan, nblk * (size_t)kPlanWords * 4, hipMemcpyHostToDevice, stream_));
  hipLaunchKernelGGL(k_emit, dim3((unsigned)nblk), dim3(64), 0, stream_, din, dtab,
                     (int64_t)nblk, dtok, dntok, dplan, dout, dlen);
  GZ_OK(hipGetLastError());
  GZ_OK(hipMemcpyAsync(hlen, dlen, nblk * sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  GZ_OK(hipMemcpyAsync(hout, dout, nblk * (size_t)kDeflateStride, hipMemcpyDeviceToHost, stream_));
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
      r.append(reinterpret_cast<const char*>(hout + k * (size_t)kDeflateStride), l & 0x7FFFFFFFu);
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
    q_.push_back(Job{std::move(body), std::move(done)});
  }
  cv_.notify_one();
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
      const size_t take = std::min(q_.size(), max_batch_);
      for (size_t i = 0; i < take; ++i) {
        batch.push_back(std::move(q_.front()));
        q_.pop_front();
      }
    }
    if (batch.empty()) continue;  // another worker took this window's bodies
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
