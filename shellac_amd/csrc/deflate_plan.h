// DEFLATE block planning (RFC 1951 §3.2.5-3.2.7), one implementation for the GPU and the
// host: from a block's symbol histogram, choose stored / fixed-Huffman / dynamic-Huffman
// by exact bit cost, build length-limited canonical Huffman codes and the dynamic block
// header, and write the plan record k_emit encodes with. The batch gzip (deflate.hip)
// runs it on the device right after its parse (k_plan, one wave per block, so a batch
// needs no host round trip between the passes); huffman.cc runs the same code on the host
// (unit tests, CPU reference encoder), so both make identical choices.
//
// Everything works in caller-provided scratch (LDS on the device, the stack on the host):
// no allocation, no recursion.
#pragma once

#include <cstdint>

#include "common.h"

namespace shellac {

constexpr int kLitLenSyms = 286;  // 0-255 literals, 256 end of block, 257-285 lengths
constexpr int kDistSyms = 30;
constexpr int kHistSyms = kLitLenSyms + kDistSyms;  // histogram layout: [litlen | dist]
constexpr int kPlanHdrWords = 160;                  // dynamic header <= 640 bytes
// plan record per block: [mode, header bits, total bytes, codes (kHistSyms), header]
// codes: bit-reversed code | length << 16
constexpr int kPlanWords = 3 + kHistSyms + kPlanHdrWords;

// Tokens of a parsed block: a literal byte, or a match (len 3..258, dist 1..32768).
constexpr uint32_t kTokMatch = 0x80000000u;

struct PlanScratch {
  uint64_t w[2 * 288];      // Huffman tree node weights
  int16_t parent[2 * 288];
  int16_t depth[2 * 288];
  int16_t heap[288];        // min-heap of node indices by (weight, index)
  int16_t used[288];        // symbols with a non-zero count
  uint32_t hist[kHistSyms];
  uint32_t code[288];
  uint8_t ll[288], dl[32], cll[19], pad_[1];
  uint8_t seq[kHistSyms];   // litlen + dist code lengths, RLE input
  uint16_t rle[kHistSyms];  // RLE of seq: sym | extra value << 5 (extra bits from sym)
};

SH_HD uint32_t plan_reverse_bits(uint32_t code, int len) {
  uint32_t r = 0;
  for (int i = 0; i < len; ++i) r |= ((code >> i) & 1u) << (len - 1 - i);
  return r;
}

// Canonical codes (RFC 1951 §3.2.2), bit-reversed for LSB-first output.
SH_HD void plan_canonical(const uint8_t* len, int n, uint32_t* code) {
  int bl_count[16] = {};
  for (int i = 0; i < n; ++i) bl_count[len[i]]++;
  bl_count[0] = 0;
  uint32_t next[16] = {};
  uint32_t c = 0;
  for (int b = 1; b < 16; ++b) {
    c = (c + (uint32_t)bl_count[b - 1]) << 1;
    next[b] = c;
  }
  for (int i = 0; i < n; ++i) code[i] = len[i] ? plan_reverse_bits(next[len[i]]++, len[i]) : 0;
}

SH_HD int plan_litlen_extra(int sym) { return (sym < 265 || sym == 285) ? 0 : (sym - 261) / 4; }
SH_HD int plan_dist_extra(int j) { return j < 4 ? 0 : (j - 2) / 2; }
SH_HD int plan_fixed_len(int sym) { return sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : 8; }

SH_HD bool plan_heap_less(const PlanScratch* ws, int a, int b) {
  return ws->w[a] < ws->w[b] || (ws->w[a] == ws->w[b] && a < b);
}

SH_HD void plan_heap_push(PlanScratch* ws, int* size, int node) {
  int i = (*size)++;
  while (i > 0) {
    const int p = (i - 1) >> 1;
    if (!plan_heap_less(ws, node, ws->heap[p])) break;
    ws->heap[i] = ws->heap[p];
    i = p;
  }
  ws->heap[i] = (int16_t)node;
}

SH_HD int plan_heap_pop(PlanScratch* ws, int* size) {
  const int top = ws->heap[0];
  const int last = ws->heap[--(*size)];
  int i = 0;
  for (;;) {
    int c = 2 * i + 1;
    if (c >= *size) break;
    if (c + 1 < *size && plan_heap_less(ws, ws->heap[c + 1], ws->heap[c])) ++c;
    if (!plan_heap_less(ws, ws->heap[c], last)) break;
    ws->heap[i] = ws->heap[c];
    i = c;
  }
  if (*size > 0) ws->heap[i] = (int16_t)last;
  return top;
}

// Length-limited Huffman code lengths (a complete code; at least two symbols get codes):
// a Huffman tree, lengths clamped to max_len, then repaired to Kraft sum 2^max_len.
SH_HD void plan_huffman_lengths(const uint32_t* freq, int n, int max_len, uint8_t* len,
                                PlanScratch* ws) {
  int m = 0;
  for (int i = 0; i < n; ++i) {
    len[i] = 0;
    if (freq[i]) ws->used[m++] = (int16_t)i;
  }
  if (m < 2) {  // a one-symbol code is incomplete: give two symbols one bit each
    const int a = m ? ws->used[0] : 0;
    len[a] = 1;
    len[a == 0 ? 1 : 0] = 1;
    return;
  }
  int hs = 0;
  for (int k = 0; k < m; ++k) {
    ws->w[k] = freq[ws->used[k]];
    plan_heap_push(ws, &hs, k);
  }
  int next = m;
  while (hs > 1) {
    const int a = plan_heap_pop(ws, &hs);
    const int b = plan_heap_pop(ws, &hs);
    ws->w[next] = ws->w[a] + ws->w[b];
    ws->parent[a] = ws->parent[b] = (int16_t)next;
    plan_heap_push(ws, &hs, next);
    ++next;
  }
  ws->depth[next - 1] = 0;
  for (int k = next - 2; k >= 0; --k) ws->depth[k] = (int16_t)(ws->depth[ws->parent[k]] + 1);
  for (int k = 0; k < m; ++k) {
    const int d = ws->depth[k];
    len[ws->used[k]] = (uint8_t)(d < max_len ? d : max_len);
  }
  // repair to a complete code of lengths <= max_len (Kraft sum == 2^max_len)
  const uint64_t T = 1ull << max_len;
  uint64_t K = 0;
  for (int k = 0; k < m; ++k) K += 1ull << (max_len - len[ws->used[k]]);
  while (K > T) {  // oversubscribed (clamping): lengthen the least frequent longest code
    int best = -1;
    for (int k = 0; k < m; ++k) {
      const int i = ws->used[k];
      if (len[i] < max_len &&
          (best < 0 || len[i] > len[best] || (len[i] == len[best] && freq[i] < freq[best])))
        best = i;
    }
    K -= 1ull << (max_len - len[best] - 1);
    len[best]++;
  }
  while (K < T) {  // incomplete: shorten the most frequent longest code while it fits
    int best = -1;
    for (int k = 0; k < m; ++k) {
      const int i = ws->used[k];
      if (len[i] > 1 && K + (1ull << (max_len - len[i])) <= T &&
          (best < 0 || len[i] > len[best] || (len[i] == len[best] && freq[i] > freq[best])))
        best = i;
    }
    if (best < 0) break;  // cannot happen for >= 2 symbols (every term divides the gap)
    K += 1ull << (max_len - len[best]);
    len[best]--;
  }
}

// LSB-first bit writer into a zero-initialised byte area.
struct PlanBits {
  uint8_t* out;
  uint32_t cap;
  uint32_t nbits;
  SH_HD void put(uint32_t v, int n) {
    for (int i = 0; i < n; ++i) {
      const uint32_t byte = nbits >> 3;
      if (byte < cap && ((v >> i) & 1u)) out[byte] |= (uint8_t)(1u << (nbits & 7));
      ++nbits;
    }
  }
};

// The plan record of one block from its histogram (hist[256], end of block, is added
// here); n = its input bytes, fin = last block of its member.
SH_HD void plan_block_record(const uint32_t* hist_in, uint32_t n, bool fin, PlanScratch* ws,
                             uint32_t* rec) {
  uint32_t* hist = ws->hist;
  for (int i = 0; i < kHistSyms; ++i) hist[i] = hist_in[i];
  hist[256] += 1;
  uint64_t extra = 0;  // bits of the extra fields (the same under fixed and dynamic codes)
  for (int s = 257; s < kLitLenSyms; ++s) extra += (uint64_t)hist[s] * plan_litlen_extra(s);
  for (int j = 0; j < kDistSyms; ++j) extra += (uint64_t)hist[kLitLenSyms + j] * plan_dist_extra(j);
  uint64_t fixed_bits = 3 + extra;
  for (int s = 0; s < kLitLenSyms; ++s) fixed_bits += (uint64_t)hist[s] * plan_fixed_len(s);
  for (int j = 0; j < kDistSyms; ++j) fixed_bits += (uint64_t)hist[kLitLenSyms + j] * 5;
  uint8_t* ll = ws->ll;
  uint8_t* dl = ws->dl;
  plan_huffman_lengths(hist, kLitLenSyms, 15, ll, ws);
  plan_huffman_lengths(hist + kLitLenSyms, kDistSyms, 15, dl, ws);
  int hlit = kLitLenSyms, hdist = kDistSyms;
  while (hlit > 257 && ll[hlit - 1] == 0) --hlit;
  while (hdist > 1 && dl[hdist - 1] == 0) --hdist;
  int ns = 0;
  for (int i = 0; i < hlit; ++i) ws->seq[ns++] = ll[i];
  for (int i = 0; i < hdist; ++i) ws->seq[ns++] = dl[i];
  // run-length coding of the code lengths (16: repeat previous 3-6, 17: zeros 3-10,
  // 18: zeros 11-138)
  int nr = 0;
  for (int i = 0; i < ns;) {
    const uint8_t v = ws->seq[i];
    int r = 1;
    while (i + r < ns && ws->seq[i + r] == v) ++r;
    i += r;
    if (v == 0) {
      while (r >= 11) {
        const int k = r < 138 ? r : 138;
        ws->rle[nr++] = (uint16_t)(18 | (k - 11) << 5);
        r -= k;
      }
      if (r >= 3) {
        ws->rle[nr++] = (uint16_t)(17 | (r - 3) << 5);
        r = 0;
      }
      for (; r; --r) ws->rle[nr++] = 0;
    } else {
      ws->rle[nr++] = v;
      --r;
      while (r >= 3) {
        const int k = r < 6 ? r : 6;
        ws->rle[nr++] = (uint16_t)(16 | (k - 3) << 5);
        r -= k;
      }
      for (; r; --r) ws->rle[nr++] = v;
    }
  }
  uint32_t clf[19] = {};
  for (int k = 0; k < nr; ++k) clf[ws->rle[k] & 31]++;
  uint8_t* cll = ws->cll;
  plan_huffman_lengths(clf, 19, 7, cll, ws);
  const int kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  const int kRleBits[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
  int hclen = 19;
  while (hclen > 4 && cll[kOrder[hclen - 1]] == 0) --hclen;
  uint64_t dyn_bits = 3 + 5 + 5 + 4 + 3ull * (uint64_t)hclen + extra;
  for (int k = 0; k < nr; ++k) {
    const int s = ws->rle[k] & 31;
    dyn_bits += cll[s] + kRleBits[s];
  }
  for (int s = 0; s < kLitLenSyms; ++s) dyn_bits += (uint64_t)hist[s] * ll[s];
  for (int j = 0; j < kDistSyms; ++j) dyn_bits += (uint64_t)hist[kLitLenSyms + j] * dl[j];
  // + the sync flush (empty stored block) that ends a non-final block
  const uint64_t fb = fin ? (fixed_bits + 7) / 8 : (fixed_bits + 3 + 7) / 8 + 4;
  const uint64_t db = fin ? (dyn_bits + 7) / 8 : (dyn_bits + 3 + 7) / 8 + 4;
  const uint64_t stored = 5ull + n;
  uint8_t* hdr = reinterpret_cast<uint8_t*>(rec + 3 + kHistSyms);
  for (int i = 0; i < kPlanHdrWords; ++i) rec[3 + kHistSyms + i] = 0;
  PlanBits bw{hdr, 4u * kPlanHdrWords, 0};
  uint32_t* codes = rec + 3;
  if (stored < fb && stored < db) {
    rec[0] = 0;
    rec[1] = 0;
    rec[2] = (uint32_t)stored;
    return;
  }
  uint32_t* c = ws->code;
  if (fb <= db) {
    rec[0] = 1;
    rec[2] = (uint32_t)fb;
    // the fixed code is defined over 288 literal/length and 32 distance symbols: the
    // canonical assignment counts the unused 286-287 (8-bit) and 30-31 codes too
    for (int s = 0; s < 288; ++s) ll[s] = (uint8_t)plan_fixed_len(s);
    plan_canonical(ll, 288, c);
    for (int s = 0; s < kLitLenSyms; ++s) codes[s] = c[s] | ((uint32_t)ll[s] << 16);
    for (int j = 0; j < 32; ++j) dl[j] = 5;
    plan_canonical(dl, 32, c);
    for (int j = 0; j < kDistSyms; ++j) codes[kLitLenSyms + j] = c[j] | (5u << 16);
    bw.put(fin ? 1 : 0, 1);
    bw.put(1, 2);
  } else {
    rec[0] = 2;
    rec[2] = (uint32_t)db;
    plan_canonical(ll, kLitLenSyms, c);
    for (int s = 0; s < kLitLenSyms; ++s) codes[s] = c[s] | ((uint32_t)ll[s] << 16);
    plan_canonical(dl, kDistSyms, c);
    for (int j = 0; j < kDistSyms; ++j) codes[kLitLenSyms + j] = c[j] | ((uint32_t)dl[j] << 16);
    plan_canonical(cll, 19, c);
    bw.put(fin ? 1 : 0, 1);
    bw.put(2, 2);
    bw.put((uint32_t)(hlit - 257), 5);
    bw.put((uint32_t)(hdist - 1), 5);
    bw.put((uint32_t)(hclen - 4), 4);
    for (int i = 0; i < hclen; ++i) bw.put(cll[kOrder[i]], 3);
    for (int k = 0; k < nr; ++k) {
      const int s = ws->rle[k] & 31;
      bw.put(c[s], cll[s]);
      if (kRleBits[s]) bw.put((uint32_t)(ws->rle[k] >> 5), kRleBits[s]);
    }
  }
  rec[1] = bw.nbits;
}

}  // namespace shellac
