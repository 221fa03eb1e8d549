// Fused device ops of the routed serving step (models/sharded_cache.py,
// ShardedCache._serve_routed): everything between the collectives runs as a few
// kernels with no host round trips, instead of dozens of small framework ops.
//
// The reference has no equivalent; its "routing" is one ketama pick and one TCP
// round trip per request (src/python/shellac/server/Server.py:335, :432). Here a
// whole batch is routed, grouped by owner, packed, unpacked and reassembled on
// the GPU around four all-to-alls (see the phase list in sharded_cache.py).
//
// Conventions: all pointers are device pointers; int64 counts; `w` = world size;
// bucket `w` collects rows that go nowhere (local replica hits, SET rows of
// ranks that neither own nor replicate the key). Row order inside a bucket is
// unspecified (LDS atomics) but consistent between every output of one call.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <vector>

#include "layout.h"

namespace shellac {

// Words of scratch (uint64) group/plan calls need for n rows into nb buckets.
int64_t group_ws_words(int64_t n, int32_t nb);

// Counting sort of n rows by dest (0..nb-1): counts[nb], perm[i] = grouped position,
// out_rows[perm[i]] = rows[i] (row_bytes multiple of 4; rows may be null).
void group_rows(const int32_t* dest, int64_t n, int32_t nb, const void* rows, int32_t row_bytes,
                void* out_rows, int64_t* perm, int64_t* counts, uint64_t* ws, hipStream_t s);

// GET side: dest = ring owner, or `w` where replica_size[i] > 0 (local replica hit).
void route_gets(const Digest* keys, int64_t n, const uint64_t* replica_size,
                const uint32_t* ring_pts, const int32_t* ring_owner, int32_t npts, int32_t w,
                int32_t* dest, hipStream_t s);

// SET side: route + hot-key fan-out + grouping. With `fanout` every input row j
// becomes w virtual rows (j, r): r receives it if r owns the key (tier 0) or the
// key is in the sorted hot set (tier 1, replica copy). Outputs in grouped order:
// srec[m][4] = {digest lo, hi, vlen | flags << 32, expire | tier << 32},
// sval[m] = values_base + val_off[j] (absolute address), spad[m] = 16-aligned value
// bytes (0 for skip rows and bucket-w rows), counts[w + 1]. m = ns * (fanout ? w : 1).
// Scratch: dest_ws[m] int32, owner_ws[ns] int32, ws = group_ws_words(m, w + 1).
void plan_sets(const Digest* keys, const uint32_t* vlen, const uint32_t* flags,
               const uint32_t* expire, const uint64_t* val_off, int64_t ns, uint64_t values_base,
               const uint32_t* ring_pts, const int32_t* ring_owner, int32_t npts,
               const Digest* hot, int64_t nhot, int32_t w, bool fanout, int32_t* dest_ws,
               int32_t* owner_ws, uint64_t* ws, int64_t* srec, uint64_t* sval, uint64_t* spad,
               int64_t* counts, hipStream_t s);

// table[p] = {GET rows, SET rows, SET value bytes} I send to peer p (int64 [w][3]);
// vscan = exclusive scan of spad (m + 1 entries).
void plan_table(const int64_t* cnt_g, const int64_t* cnt_s, const uint64_t* vscan, int32_t w,
                int64_t* table, hipStream_t s);

// Segment list of the request buffer: per peer p [G_p | R_p | V rows of p], for
// gather_segments. gk / srec are the grouped GET digests and SET records; ns = SET rows
// that leave this rank (host value, sum of cnt_s[0..w)). seg_len / seg_src: 2w + ns.
void send_segments(const int64_t* cnt_g, const int64_t* cnt_s, const uint64_t* spad,
                   const uint64_t* sval, uint64_t gk_base, uint64_t srec_base, int32_t w,
                   int64_t ns, uint64_t* seg_len, uint64_t* seg_src, hipStream_t s);

// Segment list that de-interleaves the received buffer into [all G | all R]
// (2w segments) from the received table rtable[w][3].
void recv_segments(const int64_t* rtable, uint64_t recv_base, int32_t w, uint64_t* seg_len,
                   uint64_t* seg_src, hipStream_t s);

// Received SET rows: keys, per-tier vlen (skip sentinel for the other tier), flags,
// expire and the offset of each value inside the received buffer. rpad_ws / rscan_ws
// are [ms] / [ms + 1] scratch; scan_tmp is device_scan_tmp_bytes(ms) bytes.
void recv_sets(const int64_t* rrec, int64_t ms, const int64_t* rtable, int32_t w,
               uint64_t* rpad_ws, uint64_t* rscan_ws, void* scan_tmp, size_t scan_tmp_bytes,
               Digest* keys, uint32_t* vlen0, uint32_t* vlen1, uint32_t* flags, uint32_t* expire,
               uint64_t* roff, hipStream_t s);

// bytes[0..w) = reply bytes per source q (owner side, from lk_off over rtable GET rows),
// bytes[w..2w) = bytes expected from owner p (requester side, from gscan over table).
void reply_bytes(const uint64_t* lk_off, const int64_t* rtable, const uint64_t* gscan,
                 const int64_t* table, int32_t w, int64_t* bytes, hipStream_t s);

// Response (size, off) in request order: replica hits from (rl_size, rl_off), the rest
// from the grouped remote sizes (sizes_back, gscan) shifted by local_bytes.
void assemble_response(const int64_t* perm_g, int64_t n, int64_t n_remote,
                       const uint64_t* sizes_back, const uint64_t* gscan,
                       const uint64_t* rl_size, const uint64_t* rl_off, uint64_t local_bytes,
                       uint64_t* size, uint64_t* off, hipStream_t s);

class HbmCache;

// The routed serving step of one rank as a native executor: ShardedCache keeps only
// the four collectives (torch.distributed -> RCCL) and hands every buffer in between
// to this object, which keeps its scratch in a grow-only device arena (no allocator
// traffic per step) and reads the two host-visible results (per-peer counts, reply
// byte splits) through pinned memory with one stream sync each.
//
// Call order per step (stream-ordered on `s`):
//   plan -> [a2a table -> rtable] -> read_counts -> pack(send) -> [a2a send -> recv]
//   -> owner(recv, sizes_out) -> [a2a sizes_out -> sizes_in] -> reply_sizes(sizes_in)
//   -> gather_replies(reply) -> [async a2a reply -> data] -> finish(data, ...) -> [wait]
class RoutedStep {
 public:
  RoutedStep(int world, int rank, int device);
  ~RoutedStep();
  RoutedStep(const RoutedStep&) = delete;
  RoutedStep& operator=(const RoutedStep&) = delete;

  void set_ring(const uint32_t* pts, const int32_t* owner, int32_t npts);
  void set_hot(const Digest* hot, int64_t nhot);

  // GET routing (replica probe first when `replica`), SET routing + hot fan-out,
  // per-peer table[w][3] = {GET rows, SET rows, SET value bytes} into `table`.
  void plan(const Digest* keys, int64_t n, HbmCache* replica, uint32_t now,
            const Digest* skeys, const uint32_t* svlen, const uint32_t* sflags,
            const uint32_t* sexpire, const uint64_t* sval_off, const uint8_t* svalues, int64_t ns,
            bool fanout, int64_t* table, hipStream_t s);
  // Host sync 1. Returns [table (3w) | rtable (3w) | n_local | local_bytes].
  std::vector<int64_t> read_counts(const int64_t* rtable, hipStream_t s);
  void pack(uint8_t* send, hipStream_t s);
  // Owner side: de-interleave the received requests, probe `shard`; sizes_out[mg+1].
  void owner(const uint8_t* recv, HbmCache* shard, uint32_t now, uint64_t* sizes_out,
             hipStream_t s);
  // Host sync 2. Returns [reply bytes per source (w) | bytes per owner (w)].
  std::vector<int64_t> reply_sizes(const uint64_t* sizes_in, hipStream_t s);
  void gather_replies(HbmCache* shard, uint8_t* reply, hipStream_t s);
  // Local replica gather into data[0, local_bytes), received SET stores (main shard
  // tier 0, replica tier 1), response (size, off) in request order.
  void finish(uint8_t* data, const uint8_t* recv, int64_t recv_bytes, HbmCache* shard,
              HbmCache* replica, uint32_t now, uint64_t* out_size, uint64_t* out_off,
              hipStream_t s);

  int64_t mg() const { return mg_; }
  int64_t ms() const { return ms_; }
  int64_t n_local() const { return n_local_; }
  int rank() const { return rank_; }

 private:
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
  };
  template <typename T>
  T* buf(int slot, size_t count);
  uint64_t* scan(uint64_t* in, uint64_t* out, int64_t n, hipStream_t s);  // in[n] zeroed here

  int w_, rank_, device_;
  const uint32_t* pts_ = nullptr;
  const int32_t* own_ = nullptr;
  int32_t npts_ = 0;
  const Digest* hot_ = nullptr;
  int64_t nhot_ = 0;
  std::vector<Buf> bufs_;
  int64_t* host_ = nullptr;  // pinned
  // per-step state
  int64_t n_ = 0, m_ = 0, ns_ = 0, mg_ = 0, ms_ = 0, n_local_ = 0, n_remote_ = 0;
  uint64_t local_bytes_ = 0;
  bool have_replica_ = false;
  const uint8_t* values_ = nullptr;
  // device pointers live for one step (arena slots or caller tensors)
  int64_t* table_ = nullptr;
  const int64_t* rtable_ = nullptr;
  uint64_t *rl_loc_ = nullptr, *rl_size_ = nullptr, *rl_off_ = nullptr;
  Digest* gk_ = nullptr;
  int64_t *perm_g_ = nullptr, *cnt_g_ = nullptr, *cnt_s_ = nullptr, *srec_ = nullptr;
  uint64_t *sval_ = nullptr, *spad_ = nullptr;
  const int64_t* rrec_ = nullptr;
  uint64_t *lk_loc_ = nullptr, *lk_off_ = nullptr, *gscan_ = nullptr;
  const uint64_t* sizes_in_ = nullptr;
};

}  // namespace shellac
