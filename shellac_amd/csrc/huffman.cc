// DEFLATE block planning on the host: stored / fixed / dynamic choice by exact cost,
// length-limited canonical Huffman codes, dynamic header. See huffman.h.
#include "huffman.h"

#include <algorithm>

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
  PlanScratch ws;
  plan_huffman_lengths(freq, n, max_len, len, &ws);
}

void plan_block(const uint32_t* hist, uint32_t n, bool fin, BlockPlan* out) {
  PlanScratch ws;
  uint32_t rec[kPlanWords];
  plan_block_record(hist, n, fin, &ws, rec);
  out->mode = (int)rec[0];
  out->header_bits = rec[1];
  out->total_bytes = rec[2];
  for (int i = 0; i < kHistSyms; ++i) out->codes[i] = rec[3 + i];
  const uint8_t* h = reinterpret_cast<const uint8_t*>(rec + 3 + kHistSyms);
  out->header.assign(h, h + (rec[1] + 7) / 8);
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
