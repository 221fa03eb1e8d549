// Batch gzip on the GPU: one wave per 32 KiB block, greedy LZ77 over an LDS hash table,
// fixed-Huffman DEFLATE codes (RFC 1951 §3.2.6). See deflate.h for the design.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>

#include "common.h"
#include "deflate.h"

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

// Wave-uniform LSB-first bit writer into a 4-byte aligned global buffer. Every lane holds
// the same state; lane 0 stores.
struct Bits {
  uint64_t acc = 0;
  int nb = 0;
  uint32_t words = 0;
  uint32_t* out;
  uint32_t cap_words;
  bool over = false;
  __device__ void put(uint32_t v, int n) {  // n <= 32, nb < 32 on entry
    acc |= (uint64_t)v << nb;
    nb += n;
    if (nb >= 32) {
      if (words < cap_words) {
        if (__lane_id() == 0) out[words] = (uint32_t)acc;
      } else {
        over = true;
      }
      ++words;
      acc >>= 32;
      nb -= 32;
    }
  }
};

__device__ __forceinline__ void put_literal(Bits& b, uint32_t lit) {
  if (lit < 144) b.put(rev(0x30 + lit, 8), 8);
  else b.put(rev(0x190 + (lit - 144), 9), 9);
}

// Length (3..258) and distance (1..32768) codes of RFC 1951 §3.2.5 by arithmetic: the
// code tables are "4 codes per extra bit" (lengths) and "2 codes per extra bit"
// (distances) above a few exact codes, so the code index, base and extra-bit count follow
// from the position of the top set bit — no table walk per match.
__device__ __forceinline__ void put_match(Bits& b, int len, int dist) {
  int i, le, lbase;
  if (len < 11) {
    i = len - 3; le = 0; lbase = len;
  } else if (len == 258) {
    i = 28; le = 0; lbase = 258;
  } else {
    const int L = len - 3;
    le = 29 - __clz(L);  // floor(log2 L) - 2
    const int q = (L >> le) & 3;
    i = 4 * le + 4 + q;
    lbase = 3 + ((4 + q) << le);
  }
  const int sym = 257 + i;
  uint32_t code, clen;
  if (sym < 280) {
    code = rev(sym - 256, 7);
    clen = 7;
  } else {
    code = rev(0xC0 + (sym - 280), 8);
    clen = 8;
  }
  b.put(code | ((uint32_t)(len - lbase) << clen), clen + le);
  const int D = dist - 1;
  int j, de, dbase;
  if (D < 4) {
    j = D; de = 0; dbase = dist;
  } else {
    de = 30 - __clz(D);  // floor(log2 D) - 1
    const int q = (D >> de) & 1;
    j = 2 * de + 2 + q;
    dbase = 1 + ((2 + q) << de);
  }
  b.put(rev(j, 5) | ((uint32_t)(dist - dbase) << 5), 5 + de);
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

// One wave per block. tab[b] = src offset | (len | final << 31) << 40 ... kept as two
// words for clarity: tab[2b] = src offset, tab[2b+1] = len | final << 32.
__global__ __launch_bounds__(64) void k_deflate(const uint8_t* __restrict__ src,
                                                const uint64_t* __restrict__ tab, int64_t nblk,
                                                uint8_t* __restrict__ dst,
                                                uint32_t* __restrict__ out_len,
                                                uint32_t* __restrict__ out_crc) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kDeflateBlock + 16];
  __shared__ uint32_t s_head[kHashSize];
  const int64_t b = blockIdx.x;
  if (b >= nblk) return;
  const int lane = threadIdx.x;
  const uint64_t off = tab[2 * b];
  const int n = (int)(tab[2 * b + 1] & 0xFFFFFFFFull);
  const bool fin = (tab[2 * b + 1] >> 32) != 0;
  // blocks start 16-B aligned in the packed input (the host pads every input)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* in4 = reinterpret_cast<const u32x4*>(src + off);
  u32x4* s4 = reinterpret_cast<u32x4*>(s_in);
  const int n16 = (n + 15) / 16;
  for (int i = lane; i < n16; i += 64) s4[i] = in4[i];
  for (int i = n + lane; i < n16 * 16 + 16; i += 64) s_in[i] = 0;  // zero tail (hash reads)
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

  uint8_t* out = dst + b * (int64_t)kDeflateStride;
  Bits bw;
  bw.out = reinterpret_cast<uint32_t*>(out);
  // a compressed block larger than its stored form (5 + n bytes) is abandoned
  bw.cap_words = (uint32_t)((n + 5) / 4);
  bw.put(fin ? 1u : 0u, 1);
  bw.put(1u, 2);  // BTYPE 01: fixed Huffman
  int pos = 0;
  while (pos < n && !bw.over) {
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
      put_match(bw, len, dist);
      // hash the positions the match covers (latest position wins)
      for (int q = 1 + lane; q < len; q += 64) {
        const int p = pos + q;
        if (p + 3 < n) atomicMax(&s_head[hash4(s_in, p)], (uint32_t)p + 1);
      }
      pos += len;
    } else {
      put_literal(bw, s_in[pos]);
      pos += 1;
    }
    __builtin_amdgcn_wave_barrier();  // head-table updates precede the next lookup
  }
  if (!bw.over) {
    bw.put(0u, 7);  // end of block (256)
    if (!fin) bw.put(0u, 3);  // sync flush: empty stored block header (BFINAL 0, BTYPE 00)
    // tail bytes of the bit buffer, then (non-final) LEN = 0, NLEN = 0xFFFF
    const int tail = (bw.nb + 7) / 8;
    const uint32_t total = bw.words * 4 + tail + (fin ? 0 : 4);
    if (total <= (uint32_t)n + 5) {
      if (lane < tail) out[bw.words * 4 + lane] = (uint8_t)(bw.acc >> (8 * lane));
      if (!fin && lane < 4) out[bw.words * 4 + tail + lane] = lane < 2 ? 0x00 : 0xFF;
      if (lane == 0) out_len[b] = total;
      return;
    }
  }
  // stored block: header byte (BFINAL, BTYPE 00, padding), LEN, NLEN, the raw bytes
  if (lane == 0) {
    out[0] = fin ? 1 : 0;
    out[1] = (uint8_t)(n & 0xFF);
    out[2] = (uint8_t)(n >> 8);
    out[3] = (uint8_t)(~n & 0xFF);
    out[4] = (uint8_t)((~n >> 8) & 0xFF);
    out_len[b] = (uint32_t)n + 5 | 0x80000000u;  // top bit: stored
  }
  for (int i = lane; i < n; i += 64) out[5 + i] = s_in[i];
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
  for (void* p : {(void*)d_in_, (void*)d_out_, (void*)d_tab_, (void*)d_len_})
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
  // [compressed length per block | CRC register per block]: one D2H
  uint32_t* hlen = grow(&h_len_, &h_len_cap_, 2 * nblk, true);
  uint32_t* dlen = grow(&d_len_, &d_len_cap_, 2 * nblk, false);
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
  hipLaunchKernelGGL(k_deflate, dim3((unsigned)nblk), dim3(64), 0, stream_, din, dtab,
                     (int64_t)nblk, dout, dlen, dlen + nblk);
  GZ_OK(hipGetLastError());
  GZ_OK(hipMemcpyAsync(hlen, dlen, 2 * nblk * sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
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
      reg = crc_mulmod(crc_x8n(blen), reg) ^ hlen[nblk + k];
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
