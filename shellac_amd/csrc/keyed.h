// Full-key object identity for the digest-indexed tiers.
//
// The reference keys memcached objects by the full URL (src/python/shellac/server/
// Server.py:327, :335, :432) and memcached compares whole keys. The HBM and DRAM shards
// index by a 128-bit digest (digest.h), so the backends that front them store each value
// as [u16 key length | key bytes | payload] and accept a hit only if the stored key is
// byte-equal to the requested one: two keys whose digests collide (by accident or by a
// crafted URL) read as a miss, never as each other's object.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>

namespace shellac {

constexpr size_t kKeyedPrefix = 2;
constexpr size_t kMaxKeyedKey = 0xffff;

inline size_t keyed_size(size_t klen, size_t plen) { return kKeyedPrefix + klen + plen; }

inline void write_keyed(uint8_t* dst, const std::string& key, const char* payload, size_t plen) {
  const uint16_t kl = (uint16_t)key.size();
  std::memcpy(dst, &kl, kKeyedPrefix);
  std::memcpy(dst + kKeyedPrefix, key.data(), key.size());
  if (plen) std::memcpy(dst + kKeyedPrefix + key.size(), payload, plen);
}

// True if the stored value v[0..n) belongs to `key`; *payload_off = start of the payload.
inline bool keyed_match(const char* v, size_t n, const std::string& key, size_t* payload_off) {
  if (n < kKeyedPrefix) return false;
  uint16_t kl;
  std::memcpy(&kl, v, kKeyedPrefix);
  if (kl != key.size() || n < kKeyedPrefix + kl) return false;
  if (kl && std::memcmp(v + kKeyedPrefix, key.data(), kl) != 0) return false;
  *payload_off = kKeyedPrefix + kl;
  return true;
}

}  // namespace shellac
