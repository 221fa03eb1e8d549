// Host-DRAM cache shard with exactly the HBM shard's layout and semantics.
//
// Uses: (a) the cache backend on machines/CI without a GPU, (b) the semantic
// reference the HIP kernels are tested against, (c) the CPU implementation of the
// batch ops when the distributed serving path runs over gloo. Thread-safe (one
// mutex per shard; the proxy stripes keys over several shards for concurrency).
#pragma once

#include <mutex>
#include <string>
#include <vector>

#include "layout.h"

namespace shellac {

class HostCache {
 public:
  // evict: 0 FIFO, 1 CLOCK (as ShardConfig::evict); reinsert_max 0 = auto budget.
  HostCache(uint64_t log_bytes, uint64_t nbuckets, uint32_t max_item, int evict = 1,
            uint64_t reinsert_max = 0);
  ~HostCache();
  HostCache(const HostCache&) = delete;
  HostCache& operator=(const HostCache&) = delete;

  void lookup(const Digest* keys, int64_t n, uint64_t* loc, uint64_t* size, uint64_t* off,
              uint32_t now, uint64_t reserve = 0);
  void gather(const uint64_t* loc, const uint64_t* off, int64_t n, uint8_t* out) const;
  void store(const Digest* keys, const uint8_t* values, const uint64_t* val_off,
             const uint32_t* vlen, const uint32_t* flags, const uint32_t* expire, int64_t n,
             uint32_t now, uint64_t bytes_bound = 0);  // 0: the batch's exact bytes
  void remove(const Digest* keys, int64_t n, uint8_t* found, uint32_t now);
  void sweep(uint32_t now, uint64_t* live_entries, uint64_t* live_bytes);
  void flush();
  // Tests: see HbmCache::debug_bucket / debug_set_entry.
  std::vector<uint64_t> debug_bucket(uint64_t b);
  // {hand (ring index), ring tail, head, the log offset of the hand's item (~0: none)}
  std::vector<uint64_t> debug_hand();
  void debug_set_entry(uint64_t b, int slot, uint64_t d0, uint64_t d1, uint64_t loc,
                       uint32_t vlen, uint32_t expire);
  void debug_set_hand(uint64_t hand, bool catch_up = true);  // HbmCache::debug_set_hand
  uint64_t export_keys(Digest* out, uint64_t out_cap, uint32_t now);
  void save(const std::string& path, const uint64_t user[4]);
  void load(const std::string& path, uint64_t user[4]);
  CacheCounters counters();
  uint64_t head();

  // Single-key conveniences used by the proxy / memcached server. get() copies
  // the value (not the header) into `out` and returns false on miss.
  bool get_one(const Digest& key, std::vector<uint8_t>* out, uint32_t* flags, uint32_t now,
               uint32_t* expire = nullptr);
  bool get_one(const Digest& key, std::string* out, uint32_t* flags, uint32_t now,
               uint32_t* expire = nullptr);
  void set_one(const Digest& key, const uint8_t* value, uint32_t vlen, uint32_t flags,
               uint32_t expire, uint32_t now);

  uint64_t log_bytes() const { return log_bytes_; }
  uint64_t nbuckets() const { return nbuckets_; }
  uint32_t max_item() const { return max_item_; }
  uint64_t reinsert_max() const { return evict_ ? rmax_ : 0; }

 private:
  struct Row {  // one SET row of a (possibly combined) batch
    Digest key;
    const uint8_t* val;
    uint32_t vlen, flags, expire;
    uint64_t from = 0;  // a CLOCK reinsertion: a move of the entry at this loc (see HbmCache)
  };
  bool insert_locked(const Digest& d, uint64_t loc1, uint32_t vlen, uint32_t expire, uint32_t now);
  // mark: a GET (sets the CLOCK reference bit of the entry it finds)
  uint64_t probe_locked(const Digest& d, uint32_t now, uint32_t* vlen, uint64_t reserve = 0,
                        bool mark = false);
  void store_rows_locked(const std::vector<Row>& rows, uint32_t now);
  // CLOCK hand step ahead of a batch of `bytes` log bytes over `n` rows (the device
  // algorithm, sequentially): appends the reinsertion rows to `out`, their records
  // staged in `stage`.
  void reclaim_locked(int64_t n, uint64_t bytes, uint64_t rmax, uint32_t now,
                      std::vector<Row>* out, std::vector<uint8_t>* stage, bool lead_mode);

  uint64_t log_bytes_, nbuckets_, mask_;
  uint32_t max_item_;
  uint8_t* log_ = nullptr;
  size_t log_alloc_ = 0;
  Entry* index_ = nullptr;
  size_t index_alloc_ = 0;
  uint64_t head_ = 0;
  CacheCounters ctr_{};
  mutable std::mutex mu_;
  int evict_ = 1;
  uint64_t rmax_ = 0;
  std::vector<uint64_t> ring_;  // item starts in log order (kRingSkip holes)
  uint64_t ring_tail_ = 0, hand_ = 0;
  uint64_t hand_consumed_ = 0;  // entries the hand consumed last batch (adaptive window)
  bool lead_ = false;  // the hand's mode (layout.h hand_lead, sticky)
  bool catch_up_ = true;  // debug_set_hand
};

// CPU versions of the device batch helpers (same contracts as hbm_cache.h).
void host_exclusive_scan(const uint64_t* in, uint64_t* out, int64_t n);
void host_segcopy(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off, int64_t n,
                  uint8_t* dst);
void host_digest_keys(const uint8_t* bytes, const int64_t* offs, int64_t n, Digest* out);
void host_route_keys(const Digest* keys, int64_t n, const uint32_t* ring_pts,
                     const int32_t* ring_owner, int32_t npts, int32_t* dest, int64_t* counts,
                     int32_t nranks);
void host_scatter_by_dest(const int32_t* dest, const int64_t* base, int64_t n, int32_t nranks,
                          int64_t* cursor, int64_t* perm);
void host_permute_records(const void* in, const int64_t* perm, int64_t n, int32_t rec_bytes,
                          void* out);

}  // namespace shellac
