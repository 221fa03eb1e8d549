// Fused device ops of the routed serving step (models/sharded_cache.py,
// ShardedCache._serve_routed): everything between the collectives runs as a few
// kernels with no host round trips, instead of dozens of small framework ops.
//
// The reference has no equivalent; its "routing" is one ketama pick and one TCP
// round trip per request (src/python/shellac/server/Server.py:335, :432). Here a
// whole batch is routed, grouped by owner, packed, unpacked and reassembled on
// the GPU around five all-to-alls (see the phase list in sharded_cache.py).
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

// Exclusive scan of n uint64 values into out[0..n] (out[n] = total) in two launches,
// without hipcub's sentinel/temp requirements; parts = scan_parts_words(n) words.
void scan_u64(const uint64_t* in, int64_t n, uint64_t* parts, uint64_t* out, hipStream_t s);
int64_t scan_parts_words(int64_t n);

class HbmCache;

// The routed serving step of one rank as a native executor: ShardedCache keeps only
// the five collectives (torch.distributed -> RCCL) and hands every buffer in between
// to this object, which keeps its scratch in a grow-only device arena (no allocator
// traffic per step) and reads the two host-visible results (per-peer counts, reply
// byte splits) through pinned memory with one stream sync each.
//
// Call order per step (stream-ordered on `s`):
//   plan -> [a2a table -> rtable] -> read_counts -> pack(send)
//   -> [a2a send request region -> recv request region]
//   -> [async a2a send value region -> recv value region]   (SET payloads, off the
//       critical path: only finish() reads them)
//   -> owner(recv, sizes_out) -> [a2a sizes_out -> sizes_in] -> reply_sizes(sizes_in)
//   -> gather_replies(reply) -> [async a2a reply -> data] -> [wait value region]
//   -> finish(data, recv, ...) -> [wait reply a2a before reading data]
// send / recv = [request region: per peer G_p | R_p][value region: per peer V_p].
class RoutedStep {
 public:
  RoutedStep(int world, int rank, int device);
  ~RoutedStep();
  RoutedStep(const RoutedStep&) = delete;
  RoutedStep& operator=(const RoutedStep&) = delete;

  void set_ring(const uint32_t* pts, const int32_t* owner, int32_t npts);
  // Sorted hot set (by signed lo) + optional 65537-entry directory (see is_hot).
  void set_hot(const Digest* hot, int64_t nhot, const int64_t* dir = nullptr);

  // GET routing (replica probe first when `replica`), SET routing + hot fan-out (on a
  // side stream, concurrently), per-peer table[w][3] = {GET rows, SET rows, SET value
  // bytes} into `table`, which must hold 6w + 3 words: [table | rtable | extras].
  // `coalesce`: duplicate GET digests of the batch are not routed; each is answered
  // from the row that claimed its digest (coalesce_keys / expand_coalesced).
  void plan(const Digest* keys, int64_t n, HbmCache* replica, uint32_t now,
            const Digest* skeys, const uint32_t* svlen, const uint32_t* sflags,
            const uint32_t* sexpire, const uint64_t* sval_off, const uint8_t* svalues, int64_t ns,
            bool fanout, int64_t* table, hipStream_t s, bool coalesce = false);
  // Host sync 1 (one D2H; rtable must be table + 3w). Returns
  // [table (3w) | rtable (3w) | n_local | local_bytes | coalesced duplicates] (n_local
  // includes the duplicates).
  std::vector<int64_t> read_counts(const int64_t* rtable, hipStream_t s);
  // send: request region (sum 16 G_p + 32 R_p) then value region (sum V_p).
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
  // `s` waits for the main-shard SET chain of the last finish(). With the deferred join
  // (default) finish() does not wait for it: the chain runs under the next step's plan
  // and the next owner() joins before it touches the main shard, so the caller must
  // keep `recv` alive until then and call join_sets() before any other use of the shard.
  void join_sets(hipStream_t s);
  // Early local gather (after read_counts): the replica hits' records go into
  // data[0, local_bytes) on a third stream while the request exchange, owner lookup and
  // host sync 2 proceed; finish() (or join_local) makes `s` wait for it. `data` must
  // stay allocated until then.
  void gather_local(uint8_t* data, hipStream_t s);
  void join_local(hipStream_t s);
  void set_defer_join(bool on) { defer_join_ = on; }
  bool sets_pending() const { return sets_pending_; }

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
  void fork_store(const uint8_t* recv, int64_t recv_bytes, HbmCache* shard, uint32_t now,
                  hipStream_t s);

  int w_, rank_, device_;
  const uint32_t* pts_ = nullptr;
  const int32_t* own_ = nullptr;
  int32_t npts_ = 0;
  const Digest* hot_ = nullptr;
  int64_t nhot_ = 0;
  const int64_t* hot_dir_ = nullptr;
  std::vector<Buf> bufs_;
  int64_t* host_ = nullptr;  // pinned
  // side stream: the main-shard SET chain runs there while the replica gather runs on
  // the caller's stream (finish); events fork and join the two
  hipStream_t side_ = nullptr;
  hipEvent_t ev_fork_ = nullptr, ev_fill_ = nullptr, ev_join_ = nullptr, ev_pjoin_ = nullptr;
  // store stream: the received-SET chain of the main shard (fork_store). Separate from
  // side_ (the SET planning of plan()), so the next step's planning does not queue
  // behind a deferred SET chain.
  hipStream_t store_side_ = nullptr;
  hipEvent_t ev_sfork_ = nullptr;
  hipStream_t local_side_ = nullptr;  // early replica gather (gather_local)
  hipEvent_t ev_lfork_ = nullptr, ev_ljoin_ = nullptr;
  bool local_pending_ = false, local_done_ = false;
  HbmCache* replica_ = nullptr;
  bool defer_join_ = true, sets_pending_ = false;
  // per-step state
  int64_t n_ = 0, ns_ = 0, mg_ = 0, ms_ = 0, n_local_ = 0, n_remote_ = 0;
  uint64_t local_bytes_ = 0;
  bool have_replica_ = false;
  const uint8_t* values_ = nullptr;
  // device pointers live for one step (arena slots or caller tensors)
  int64_t* table_ = nullptr;
  const int64_t* rtable_ = nullptr;
  uint64_t *rl_loc_ = nullptr, *rl_size_ = nullptr, *rl_off_ = nullptr;
  Digest* gk_ = nullptr;
  int64_t *perm_g_ = nullptr, *cnt_g_ = nullptr, *cnt_s_ = nullptr, *srec_ = nullptr;
  uint64_t *sval_ = nullptr, *svoff_ = nullptr;
  uint32_t* first_ = nullptr;  // coalescing: claiming row of each GET row (null = off)
  const int64_t* rrec_ = nullptr;
  uint64_t *lk_loc_ = nullptr, *lk_off_ = nullptr, *gscan_ = nullptr;
  const uint64_t* sizes_in_ = nullptr;
};

}  // namespace shellac
