// ObjectCache: the host-DRAM cache tier of the proxy (DramBackend, and the L1 in front
// of the HBM shards in TieredBackend).
//
// The reference keeps objects in memcached (src/python/shellac/server/Server.py:81-83,
// get :335, set :432). On the host the hot path is a hit, so objects are immutable
// reference-counted byte strings: a hit hands the reactor a ByteRef to the stored bytes
// (one atomic increment, no copy) and the response goes to writev() from there. Each
// object is one allocation holding [u16 key length | key | payload] (keyed.h): a hit
// requires the full key to match, so a digest collision reads as a miss.
//
// Striped for the reactor threads (a mutex per stripe, digests spread by their high
// bits). Capacity is in bytes; eviction is CLOCK over each stripe's slots (a hit sets
// the reference bit, the hand clears it once before evicting), the host analogue of
// the HBM log's CLOCK reinsertion. TTLs expire lazily on access.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "digest.h"
#include "stream_buf.h"

namespace shellac {

struct ObjectCacheStats {
  uint64_t gets = 0, hits = 0, sets = 0, evictions = 0, expired = 0, key_mismatch = 0;
  uint64_t objects = 0, bytes = 0;
};

class ObjectCache {
 public:
  ObjectCache(uint64_t capacity_bytes, uint32_t max_item, int stripes = 64);
  // Hit: *payload = the object's bytes (shared, no copy), flags and absolute expiry.
  bool get(const std::string& key, const Digest& d, uint32_t now, Bytes* payload,
           uint32_t* flags, uint32_t* expire);
  // Stores a private copy of `payload` (one allocation) keyed by `key`.
  void set(const std::string& key, const Digest& d, const char* payload, size_t n,
           uint32_t flags, uint32_t expire, uint32_t now);
  bool del(const std::string& key, const Digest& d, uint32_t now);
  void clear();
  ObjectCacheStats stats() const;

 private:
  struct Obj {
    Digest d{0, 0};
    std::shared_ptr<const std::string> data;  // [klen | key | payload]; null = free slot
    uint32_t flags = 0, expire = 0;
    uint32_t bytes = 0;
    bool ref = false;
  };
  struct Stripe {
    std::mutex mu;
    std::vector<Obj> slots;
    std::vector<uint32_t> free;     // free slot ids
    std::vector<int32_t> table;     // open addressing: slot id, -1 empty, -2 tombstone
    uint64_t bytes = 0, live = 0, used = 0;  // used = table entries incl. tombstones
    uint32_t hand = 0;
    ObjectCacheStats st;
  };
  Stripe& stripe(const Digest& d) { return *stripes_[(d.hi >> 40) % stripes_.size()]; }
  static int32_t* find(Stripe& s, const Digest& d);
  static void table_insert(Stripe& s, const Digest& d, int32_t slot);
  static void rehash(Stripe& s, size_t cap);
  void erase_slot(Stripe& s, int32_t* pos, std::vector<std::shared_ptr<const std::string>>* dead);
  void evict(Stripe& s, std::vector<std::shared_ptr<const std::string>>* dead);

  uint64_t cap_per_stripe_;
  uint32_t max_item_;
  std::vector<std::unique_ptr<Stripe>> stripes_;
};

}  // namespace shellac
