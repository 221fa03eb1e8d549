// Host API of the DEFLATE block planner (deflate_plan.h, shared with the GPU's k_plan):
// the BlockPlan view of a plan record, Huffman lengths, and a CPU reference encoder of a
// token list for tests.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "deflate_plan.h"

namespace shellac {

inline uint32_t tok_literal(uint32_t b) { return b; }
inline uint32_t tok_match(uint32_t len, uint32_t dist) { return kTokMatch | (len << 16) | (dist - 1); }

// Length / distance symbol of a match and its extra bits (code index arithmetic).
struct SymExtra {
  int sym, nbits;
  uint32_t value;
};
SymExtra len_symbol(int len);    // sym 257..285
SymExtra dist_symbol(int dist);  // sym 0..29

struct BlockPlan {
  int mode = 0;                  // 0 stored, 1 fixed Huffman, 2 dynamic Huffman
  std::vector<uint8_t> header;   // the block's first bits (BFINAL, BTYPE, dynamic tables)
  uint32_t header_bits = 0;
  // per symbol: bit-reversed code | length << 16 (litlen 0..285, then dist 0..29)
  uint32_t codes[kHistSyms] = {};
  uint64_t total_bytes = 0;      // encoded size of the block, sync flush included (non-final)
};

// `hist` counts literal/length symbols (256 = end of block is added here) and distance
// symbols of the block's tokens; `n` is its input size; `fin` marks the last block.
void plan_block(const uint32_t* hist, uint32_t n, bool fin, BlockPlan* out);

// Length-limited Huffman code lengths (complete code; at least two symbols get codes).
void huffman_lengths(const uint32_t* freq, int n, int max_len, uint8_t* len);

// CPU reference: parse-free encoding of a token list with plan_block's codes, for tests.
std::string deflate_tokens_cpu(const std::vector<uint32_t>& tokens, const std::string& data,
                               bool fin);

}  // namespace shellac
