// Memory layout of one cache shard, shared by the HBM (HIP) and DRAM (host) engines.
//
// A shard is two regions:
//
//   index : nbuckets x 128-byte buckets, 4 x 32-byte Entry each. Every object has
//           two candidate buckets (two-choice hashing), so a probe is exactly two
//           independent cache-line reads and never touches the value log.
//   log   : a circular, append-only byte log of `capacity` bytes (+ one max item
//           of slack so an item that starts near the end never wraps). Items are
//           appended at a monotonically increasing *logical* head; physical offset
//           = logical % capacity. Eviction is FIFO by construction: appending
//           overwrites the oldest bytes. An entry is live iff its item has not
//           been overwritten (head <= loc + capacity) and has not expired.
//
// This replaces the reference's external memcached slab store (Server.py:81-83,
// :335 get, :432 set with time=ttl) with a structure that maps onto HBM: no
// free lists, no per-class slabs, no fragmentation, batch allocation is one
// prefix sum, and lookups are coalesced 128-byte reads.
#pragma once

#include <cstdlib>

#include "digest.h"

namespace shellac {

constexpr uint32_t kEntriesPerBucket = 4;
constexpr uint32_t kBucketBytes = 128;
constexpr uint32_t kItemHeaderBytes = 32;
constexpr uint32_t kItemMagic = 0x5348a11cu;
constexpr uint64_t kMissLoc = ~0ULL;
// vlen sentinel: "this SET row is not for this tier" (skipped, not counted).
constexpr uint32_t kSkipVlen = 0xFFFFFFFFu;

struct alignas(32) Entry {
  uint64_t d0;      // digest.lo
  uint64_t d1;      // digest.hi
  uint64_t loc;     // logical offset of the item header + 1 (0 = empty slot)
  uint32_t vlen;    // value length in bytes | kRefBit (read since the CLOCK hand last passed)
  uint32_t expire;  // absolute expiry (seconds since cache epoch), 0 = never
};
static_assert(sizeof(Entry) == 32, "Entry must be 32 bytes");

// CLOCK reference bit, kept in the top bit of Entry::vlen: set by a GET hit, cleared
// when the eviction hand re-appends the item (a second chance) — see reclaim in
// hbm_cache.h. Values are therefore < 2 GiB (max_item is checked against it).
constexpr uint32_t kRefBit = 0x80000000u;
constexpr uint32_t kVlenMask = 0x7fffffffu;
SH_HD uint32_t entry_vlen(uint32_t v) { return v & kVlenMask; }

// Header written in front of every value in the log; a GET returns header+value.
struct alignas(16) ItemHeader {
  uint64_t d0;
  uint64_t d1;
  uint32_t vlen;
  uint32_t flags;   // opaque client flags (memcached protocol)
  uint32_t expire;
  uint32_t magic;
};
static_assert(sizeof(ItemHeader) == kItemHeaderBytes, "ItemHeader must be 32 bytes");

SH_HD uint64_t item_bytes(uint32_t vlen) { return kItemHeaderBytes + align_up(vlen, 16); }

SH_HD uint64_t bucket1(const Digest& d, uint64_t mask) { return d.lo & mask; }

SH_HD uint64_t bucket2(const Digest& d, uint64_t mask) {
  uint64_t b1 = d.lo & mask;
  uint64_t b2 = fmix64(d.hi ^ rotl64(d.lo, 29)) & mask;
  return b2 == b1 ? (b1 ^ 1) & mask : b2;
}

// An entry's loc while one inserter rewrites its digest / vlen words (a relocation copy
// being written, or one being dropped): neither live (probes and matches skip it) nor free
// (no other inserter may claim it). Only the thread that stored it moves the slot on.
constexpr uint64_t kLockedLoc = ~0ull - 1;

SH_HD bool entry_live(uint64_t loc, uint32_t expire, uint64_t head, uint64_t capacity,
                      uint32_t now) {
  return loc != 0 && loc != kLockedLoc && head <= (loc - 1) + capacity &&
         (expire == 0 || expire > now);
}
// A slot an inserter may claim: neither live nor locked.
SH_HD bool entry_free(uint64_t loc, uint32_t expire, uint64_t head, uint64_t capacity,
                      uint32_t now) {
  return loc != kLockedLoc && !entry_live(loc, expire, head, capacity, now);
}

// CLOCK eviction geometry shared by the HBM and host engines, so both make identical
// decisions: the reinsertion budget per SET batch (`req` bytes, 0 = auto: 1/32 of the
// log clamped to [1 MiB, 1 GiB] and at most 1/4 of it), the hand's window (ring entries
// examined per SET batch of n rows) and the item-start ring size (power of two).
inline uint64_t reinsert_budget(uint64_t log_bytes, uint64_t req) {
  if (req) return req / 16 * 16;
  uint64_t r = log_bytes / 32;
  r = r < (1ull << 20) ? (1ull << 20) : (r > (1ull << 30) ? (1ull << 30) : r);
  return (r < log_bytes / 4 ? r : log_bytes / 4) / 16 * 16;
}
// Window = k * n + 256 entries, k = 2 by default: a batch can reinsert up to about its
// own bytes (write amplification <= 2) before referenced items past the window age out.
// Every window entry costs a scan row and a (skip) row of the combined SET chain, so the
// window is the fixed cost of a SET batch once the log has wrapped: k = 4 made the
// steady-state N=1 step 0.91 ms at a 5 GiB log and 0.41 ms at 16 GiB, k = 2 0.51 / 0.37
// ms with the same hit ratio and reinsertions (profiles/archive/r2_hand_window_ab.log); the
// evict_sim hit ratios are identical for k = 2, 3, 4; k = 1 does not cover the batch's own
// bytes and degrades to FIFO.
// Adaptive window: the hand must pass every item the overwrite reaches, i.e. the items a
// step appended one lap earlier (its SETs + its reinsertions). When a read-heavy step
// reinserts more items than its batch holds, 2n + 256 entries fall behind; behind the
// overwrite the hand can no longer give second chances and every referenced object ages
// out (the host twin: hit ratio 0.43 instead of 0.77 at 2x the log, hot objects lost). So
// the window holds up to kHandWindowMaxK * n + 256 rows, of which the hand examines
//     W_eff = min(W, max(1.5n + 256, 1.25 x (entries it consumed last batch) + 256))
// (a 1.5n base, down from the fixed 2n: the wrapped step -1.5 %, the full cache and the hit
// ratios unchanged, profiles/r5ar_window_base)
// (hand_window_eff; the rest are skip rows without reads), and reinsertions are capped at
// W - n items per batch, so the items a batch appends stay within the window a lap later.
constexpr int64_t kHandWindowK = 3;     // halves: the base window 1.5 n + 256
constexpr int64_t kHandWindowMaxK = 3;
SH_HD int64_t hand_window(int64_t n) {  // the rows of the window (allocation, launch)
  const int64_t w = kHandWindowMaxK * n + 256;
  return w < (1 << 20) ? w : (1 << 20);
}
SH_HD int64_t hand_window_eff(int64_t n, uint64_t consumed_last) {
  const int64_t w = hand_window(n);
  int64_t e = kHandWindowK * n / 2 + 256;
  const uint64_t want = consumed_last + consumed_last / 4 + 256;
  if ((uint64_t)e < want) e = want > (uint64_t)w ? w : (int64_t)want;
  return e < w ? e : w;
}
// Whether the hand runs ahead of the overwrite (lead mode, HbmCache k_rc_emit): on a log of
// at least 16 x (the batch's byte bound + the reinsertion budget). Both engines decide the
// same way from the same bound.
// The decision is sticky (`prev`: the last batch's): a batch bound that straddles the
// threshold flipped the mode from batch to batch, and each switch into lead mode drops the
// referenced items the hand then finds too close to the overwrite to copy (host twin, working
// set 2x the log: hit ratio 0.40 against 0.86). Lead mode is left below 12x.
inline bool hand_lead(uint64_t log_bytes, uint64_t bytes_bound, uint64_t rmax,
                      bool prev = false) {
  return log_bytes >= (prev ? 12 : 16) * (bytes_bound + rmax);
}
inline uint64_t ring_entries(uint64_t nbuckets) {
  uint64_t r = 4096;
  while (r < 2 * nbuckets * kEntriesPerBucket) r <<= 1;
  return r;
}
constexpr uint64_t kRingSkip = ~0ull;  // item-start ring: a SET row that stored nothing

// Counters kept on the device (and mirrored by the host engine). Under GET coalescing
// get_ops / get_hits / get_bytes count distinct keys probed; the duplicate rows a
// batch-mate's record answered are get_coalesced (requests = get_ops + get_coalesced).
struct CacheCounters {
  unsigned long long get_ops;
  unsigned long long get_hits;
  unsigned long long get_bytes;
  unsigned long long set_ops;
  unsigned long long set_bytes;
  unsigned long long set_dropped;   // rejected (too large) or lost a same-batch dedupe
  unsigned long long set_evicted;   // a live entry displaced because both buckets were full
  unsigned long long del_ops;
  unsigned long long del_hits;
  unsigned long long swept;         // dead entries reclaimed by sweep()
  unsigned long long get_coalesced; // duplicate GET rows served by a batch-mate's probe
  unsigned long long reinserted;    // referenced items the CLOCK hand gave a second life
  unsigned long long reinsert_bytes;
  // reinsertions indexed as moves whose entry had moved on (a SET or DELETE of the key
  // landed after the hand read the index): their log bytes are dead on arrival
  unsigned long long reinsert_lost;
  unsigned long long reserved[2];
};
static_assert(sizeof(CacheCounters) == 128, "CacheCounters layout");

}  // namespace shellac
