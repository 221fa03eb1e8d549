// DEFLATE block planning on the host: stored / fixed / dynamic choice by exact cost,
// length-limited canonical Huffman codes, dynamic header. See huffman.h.
#include "huffman.h"

#include <algorithm>
#include <queue>

namespace shellac {
namespace {

struct Bits {
  std::vector<uint8_t>* out;
  uint64_t nbits = 0;
  void put(uint32_t v, int n) {
    for (int i = 0; i < n; ++i) {
      if ((nbits & 7) == 0) out->push_back(0);
      if ((v >> i) & 1) out->back() |= (uint8_t)(1u << (nbits & 7));
      ++nbits;
    }
  }
};

uint32_t reverse_bits(uint32_t code, int len) {
  uint32_t r = 0;
  for (int i = 0; i < len; ++i) r |= ((code >> i) & 1u) << (len - 1 - i);
  return r;
}

// Canonical codes (RFC 1951 §3.2.2), bit-reversed for LSB-first output.
void canonical(const uint8_t* len, int n, uint32_t* code) {
  int bl_count[16] = {};
  for (int i = 0; i < n; ++i) bl_count[len[i]]++;
  bl_count[0] = 0;
  uint32_t next[16] = {};
  uint32_t c = 0;
  for (int b = 1; b < 16; ++b) {
    c = (c + bl_count[b - 1]) << 1;
    next[b] = c;
  }
  for (int i = 0; i < n; ++i)
    code[i] = len[i] ? reverse_bits(next[len[i]]++, len[i]) : 0;
}

int litlen_extra(int sym) {
  if (sym < 265 || sym == 285) return 0;
  return (sym - 261) / 4;
}
int dist_extra(int j) { return j < 4 ? 0 : (j - 2) / 2; }
int fixed_len(int sym) { return sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : 8; }

}  // namespace

SymExtra len_symbol(int len) {
  if (len < 11) return {257 + len - 3, 0, 0};
  if (len == 258) return {285, 0, 0};
  const int L = len - 3;
  int e = 0;
  while ((L >> (e + 3)) != 0) ++e;  // floor(log2 L) - 2
  const int q = (L >> e) & 3;
  const int base = 3 + ((4 + q) << e);
  return {257 + 4 * e + 4 + q, e, (uint32_t)(len - base)};
}

SymExtra dist_symbol(int dist) {
  const int D = dist - 1;
  if (D < 4) return {D, 0, 0};
  int e = 0;
  while ((D >> (e + 2)) != 0) ++e;  // floor(log2 D) - 1
  const int q = (D >> e) & 1;
  const int base = 1 + ((2 + q) << e);
  return {2 * e + 2 + q, e, (uint32_t)(dist - base)};
}

void huffman_lengths(const uint32_t* freq, int n, int max_len, uint8_t* len) {
  std::fill(len, len + n, 0);
  std::vector<int> used;
  for (int i = 0; i < n; ++i)
    if (freq[i]) used.push_back(i);
  if (used.size() < 2) {  // a one-symbol code is incomplete: give two symbols one bit each
    const int a = used.empty() ? 0 : used[0];
    len[a] = 1;
    len[a == 0 ? 1 : 0] = 1;
    return;
  }
  // Huffman tree: leaves 0..m-1, internal nodes after them
  const int m = (int)used.size();
  std::vector<uint64_t> w(2 * m);
  std::vector<int> parent(2 * m, -1);
  using Item = std::pair<uint64_t, int>;
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
  for (int k = 0; k < m; ++k) {
    w[k] = freq[used[k]];
    pq.push({w[k], k});
  }
  int next = m;
  while (pq.size() > 1) {
    const Item a = pq.top();
    pq.pop();
    const Item b = pq.top();
    pq.pop();
    w[next] = a.first + b.first;
    parent[a.second] = parent[b.second] = next;
    pq.push({w[next], next});
    ++next;
  }
  std::vector<int> depth(next, 0);
  for (int k = next - 2; k >= 0; --k) depth[k] = depth[parent[k]] + 1;
  for (int k = 0; k < m; ++k) len[used[k]] = (uint8_t)std::min(depth[k], max_len);
  // repair to a complete code of lengths <= max_len (Kraft sum == 2^max_len)
  const uint64_t T = 1ull << max_len;
  auto kraft = [&] {
    uint64_t s = 0;
    for (int i : used) s += 1ull << (max_len - len[i]);
    return s;
  };
  uint64_t K = kraft();
  // oversubscribed (from clamping): lengthen the least frequent of the longest codes
  while (K > T) {
    int best = -1;
    for (int i : used)
      if (len[i] < max_len &&
          (best < 0 || len[i] > len[best] || (len[i] == len[best] && freq[i] < freq[best])))
        best = i;
    K -= 1ull << (max_len - len[best] - 1);
    len[best]++;
  }
  // incomplete: shorten the most frequent of the longest codes while it fits
  while (K < T) {
    int best = -1;
    for (int i : used)
      if (len[i] > 1 && K + (1ull << (max_len - len[i])) <= T &&
          (best < 0 || len[i] > len[best] || (len[i] == len[best] && freq[i] > freq[best])))
        best = i;
    if (best < 0) break;  // cannot happen for >= 2 symbols (all terms divide the gap)
    K += 1ull << (max_len - len[best]);
    len[best]--;
  }
}

void plan_block(const uint32_t* hist_in, uint32_t n, bool fin, BlockPlan* out) {
  uint32_t hist[kHistSyms];
  std::copy(hist_in, hist_in + kHistSyms, hist);
  hist[256] += 1;  // end of block
  // bits of the symbols' extra fields (the same under fixed and dynamic codes)
  uint64_t extra = 0;
  for (int s = 257; s < kLitLenSyms; ++s) extra += (uint64_t)hist[s] * litlen_extra(s);
  for (int j = 0; j < kDistSyms; ++j) extra += (uint64_t)hist[kLitLenSyms + j] * dist_extra(j);
  auto bytes_of = [&](uint64_t bits) {  // + sync flush for a non-final block
    if (fin) return (bits + 7) / 8;
    return (bits + 3 + 7) / 8 + 4;
  };
  // fixed
  uint64_t fixed_bits = 3 + extra;
  for (int s = 0; s < kLitLenSyms; ++s) fixed_bits += (uint64_t)hist[s] * fixed_len(s);
  for (int j = 0; j < kDistSyms; ++j) fixed_bits += (uint64_t)hist[kLitLenSyms + j] * 5;
  // dynamic
  uint8_t ll[kLitLenSyms], dl[kDistSyms];
  huffman_lengths(hist, kLitLenSyms, 15, ll);
  huffman_lengths(hist + kLitLenSyms, kDistSyms, 15, dl);
  int hlit = kLitLenSyms, hdist = kDistSyms;
  while (hlit > 257 && ll[hlit - 1] == 0) --hlit;
  while (hdist > 1 && dl[hdist - 1] == 0) --hdist;
  std::vector<uint8_t> seq(ll, ll + hlit);
  seq.insert(seq.end(), dl, dl + hdist);
  struct Rle {
    int sym, nbits;
    uint32_t v;
  };
  std::vector<Rle> rle;
  for (size_t i = 0; i < seq.size();) {
    const uint8_t v = seq[i];
    size_t r = 1;
    while (i + r < seq.size() && seq[i + r] == v) ++r;
    i += r;
    if (v == 0) {
      while (r >= 11) {
        const size_t k = std::min<size_t>(r, 138);
        rle.push_back({18, 7, (uint32_t)(k - 11)});
        r -= k;
      }
      if (r >= 3) {
        rle.push_back({17, 3, (uint32_t)(r - 3)});
        r = 0;
      }
      for (; r; --r) rle.push_back({0, 0, 0});
    } else {
      rle.push_back({v, 0, 0});
      --r;
      while (r >= 3) {
        const size_t k = std::min<size_t>(r, 6);
        rle.push_back({16, 2, (uint32_t)(k - 3)});
        r -= k;
      }
      for (; r; --r) rle.push_back({v, 0, 0});
    }
  }
  uint32_t clf[19] = {};
  for (const Rle& x : rle) clf[x.sym]++;
  uint8_t cll[19];
  huffman_lengths(clf, 19, 7, cll);
  static const int kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  int hclen = 19;
  while (hclen > 4 && cll[kOrder[hclen - 1]] == 0) --hclen;
  uint64_t dyn_bits = 3 + 5 + 5 + 4 + 3ull * hclen + extra;
  for (const Rle& x : rle) dyn_bits += cll[x.sym] + x.nbits;
  for (int s = 0; s < kLitLenSyms; ++s) dyn_bits += (uint64_t)hist[s] * ll[s];
  for (int j = 0; j < kDistSyms; ++j) dyn_bits += (uint64_t)hist[kLitLenSyms + j] * dl[j];

  const uint64_t stored = 5ull + n;
  const uint64_t fb = bytes_of(fixed_bits), db = bytes_of(dyn_bits);
  out->header.clear();
  Bits bw{&out->header};
  if (stored < fb && stored < db) {
    out->mode = 0;
    out->total_bytes = stored;
    out->header_bits = 0;
    return;
  }
  if (fb <= db) {
    out->mode = 1;
    out->total_bytes = fb;
    // the fixed code is defined over 288 literal/length and 32 distance symbols: the
    // canonical assignment must count the unused 286-287 (8-bit) and 30-31 codes too
    uint8_t fl[288], fd[32];
    for (int s = 0; s < 288; ++s) fl[s] = (uint8_t)fixed_len(s);
    std::fill(fd, fd + 32, 5);
    uint32_t c[288];
    canonical(fl, 288, c);
    for (int s = 0; s < kLitLenSyms; ++s) out->codes[s] = c[s] | ((uint32_t)fl[s] << 16);
    canonical(fd, 32, c);
    for (int j = 0; j < kDistSyms; ++j) out->codes[kLitLenSyms + j] = c[j] | (5u << 16);
    bw.put(fin ? 1 : 0, 1);
    bw.put(1, 2);
  } else {
    out->mode = 2;
    out->total_bytes = db;
    uint32_t c[kLitLenSyms];
    canonical(ll, kLitLenSyms, c);
    for (int s = 0; s < kLitLenSyms; ++s) out->codes[s] = c[s] | ((uint32_t)ll[s] << 16);
    canonical(dl, kDistSyms, c);
    for (int j = 0; j < kDistSyms; ++j) out->codes[kLitLenSyms + j] = c[j] | ((uint32_t)dl[j] << 16);
    uint32_t clc[19];
    canonical(cll, 19, clc);
    bw.put(fin ? 1 : 0, 1);
    bw.put(2, 2);
    bw.put((uint32_t)(hlit - 257), 5);
    bw.put((uint32_t)(hdist - 1), 5);
    bw.put((uint32_t)(hclen - 4), 4);
    for (int i = 0; i < hclen; ++i) bw.put(cll[kOrder[i]], 3);
    for (const Rle& x : rle) {
      bw.put(clc[x.sym], cll[x.sym]);
      if (x.nbits) bw.put(x.v, x.nbits);
    }
  }
  out->header_bits = (uint32_t)bw.nbits;
}

std::string deflate_tokens_cpu(const std::vector<uint32_t>& tokens, const std::string& data,
                               bool fin) {
  uint32_t hist[kHistSyms] = {};
  for (uint32_t t : tokens) {
    if (t & kTokMatch) {
      hist[len_symbol((t >> 16) & 0x1FF).sym]++;
      hist[kLitLenSyms + dist_symbol((int)(t & 0xFFFF) + 1).sym]++;
    } else {
      hist[t & 0xFF]++;
    }
  }
  BlockPlan p;
  plan_block(hist, (uint32_t)data.size(), fin, &p);
  std::vector<uint8_t> out;
  if (p.mode == 0) {
    const uint32_t n = (uint32_t)data.size();
    out = {(uint8_t)(fin ? 1 : 0), (uint8_t)(n & 0xFF), (uint8_t)(n >> 8),
           (uint8_t)(~n & 0xFF), (uint8_t)((~n >> 8) & 0xFF)};
    out.insert(out.end(), data.begin(), data.end());
    return std::string(out.begin(), out.end());
  }
  out = p.header;
  Bits bw{&out, p.header_bits};
  auto code = [&](int s) { bw.put(p.codes[s] & 0xFFFF, (int)(p.codes[s] >> 16)); };
  for (uint32_t t : tokens) {
    if (t & kTokMatch) {
      const SymExtra l = len_symbol((t >> 16) & 0x1FF);
      code(l.sym);
      if (l.nbits) bw.put(l.value, l.nbits);
      const SymExtra d = dist_symbol((int)(t & 0xFFFF) + 1);
      code(kLitLenSyms + d.sym);
      if (d.nbits) bw.put(d.value, d.nbits);
    } else {
      code((int)(t & 0xFF));
    }
  }
  code(256);
  if (!fin) {
    bw.put(0, 3);
    while (bw.nbits & 7) bw.put(0, 1);
    out.insert(out.end(), {0x00, 0x00, 0xFF, 0xFF});
  }
  return std::string(out.begin(), out.end());
}

}  // namespace shellac
