// 128-bit object digest (MurmurHash3_x64_128, seeded) shared by host and device.
//
// The reference keys its memcached objects by the raw request URL string
// (src/python/shellac/server/Server.py:327, :335, :432) and lets libmemcached's
// ketama pick the node. Here every object is keyed by a 128-bit digest of the
// key bytes instead (the Varnish design: objects are looked up by a hash of the
// request, never by the string): the digest is computed once at the edge and
// everything downstream (index probe, shard routing, all-to-all transport,
// log headers) moves fixed 16-byte records instead of variable-length strings.
#pragma once

#include "common.h"

namespace shellac {

constexpr uint64_t kDigestSeed = 0x5348454c4c414321ULL;  // "SHELLAC!"

struct alignas(16) Digest {
  uint64_t lo;
  uint64_t hi;
};

SH_HD uint64_t load_le64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

// MurmurHash3_x64_128 (Austin Appleby, public domain), 64-bit seed variant.
SH_HD Digest digest_bytes(const uint8_t* data, uint64_t len, uint64_t seed = kDigestSeed) {
  const uint64_t c1 = 0x87c37b91114253d5ULL;
  const uint64_t c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = seed, h2 = seed;
  const uint64_t nblocks = len / 16;
  for (uint64_t i = 0; i < nblocks; ++i) {
    uint64_t k1 = load_le64(data + i * 16);
    uint64_t k2 = load_le64(data + i * 16 + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* tail = data + nblocks * 16;
  uint64_t k1 = 0, k2 = 0;
  const uint64_t rem = len & 15;
  for (uint64_t i = rem; i > 8; --i) k2 ^= (uint64_t)tail[i - 1] << (8 * (i - 9));
  if (rem > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
  const uint64_t r1 = rem > 8 ? 8 : rem;
  for (uint64_t i = r1; i > 0; --i) k1 ^= (uint64_t)tail[i - 1] << (8 * (i - 1));
  if (rem > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
  h1 ^= len; h2 ^= len;
  h1 += h2; h2 += h1;
  h1 = fmix64(h1); h2 = fmix64(h2);
  h1 += h2; h2 += h1;
  return Digest{h1, h2};
}

// 32-bit ring position of a digest (consistent-hash ring lookups).
SH_HD uint32_t ring_position(const Digest& d) { return (uint32_t)(d.hi >> 32); }

}  // namespace shellac
