// HBM-resident cache shard (one per MI355X GPU) and its batch operations.
//
// Capability parity: this is the "distributed key/value store" side of Shellac,
// which the reference delegates to memcached through pylibmc
// (src/python/shellac/server/Server.py:79-83 client, :335 get, :432 set with
// time=ttl). The README's roadmap item "replacing Memcached with a
// purpose-built cache" (README.md:79) is what this class is.
//
// Every operation is a *batch* of fixed 16-byte digests on a HIP stream; all
// pointer arguments are device pointers unless stated otherwise. No operation
// allocates or synchronises except where documented (lookup_total, sweep,
// counters, reserve), so the batch pipeline can run back-to-back on a stream.
#pragma once

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "layout.h"

namespace shellac {

// Eviction policies of the value log (ShardConfig::evict).
enum : int { kEvictFifo = 0, kEvictClock = 1 };

struct ShardConfig {
  uint64_t log_bytes = 1ull << 30;  // value-log capacity (multiple of 16)
  uint64_t nbuckets = 1ull << 20;   // power of two, 4 entries (128 B) each
  uint32_t max_item = 1u << 20;     // max value bytes (memcached's 1 MB item limit)
  int device = 0;
  // kEvictClock: items read since the hand last passed get re-appended instead of being
  // overwritten (CLOCK / FIFO-reinsertion, memcached-LRU-like hit ratios under
  // capacity pressure). kEvictFifo: plain circular log.
  int evict = kEvictClock;
  uint64_t reinsert_max = 0;  // reinsertion budget per SET batch (bytes); 0 = auto
  int serve_blocks = 8;       // resident edge-server blocks (serve_get jobs side by side)
};

class HbmCache {
 public:
  explicit HbmCache(const ShardConfig& cfg);
  ~HbmCache();
  HbmCache(const HbmCache&) = delete;
  HbmCache& operator=(const HbmCache&) = delete;

  // GET phase 1: probe both candidate buckets of every key. Writes, per key,
  // the physical log offset of the item (kMissLoc on miss) and the bytes the
  // item occupies in a GET response (0 on miss); then an exclusive scan of the
  // sizes into off[0..n] (off[n] = total response bytes).
  // `reserve` > 0 treats objects that the next `reserve` appended bytes will
  // overwrite as misses, so SETs may be queued between this lookup and its gather.
  // `total_slot` >= 0 also writes off[n] straight into host slot `total_slot` (pinned,
  // coherent), readable with host_slot() once the stream has passed the lookup: the
  // response size without a D2H copy.
  // `first` (coalesce_keys output, may be null): rows with first[i] != i are duplicates
  // and are answered as misses without touching the index (expand_coalesced fills them
  // in after the gather).
  void lookup(const Digest* keys, int64_t n, uint64_t* loc, uint64_t* size, uint64_t* off,
              uint32_t now, hipStream_t s, uint64_t reserve = 0, int total_slot = -1,
              const uint32_t* first = nullptr);
  // Coalescing lookup: coalesce_keys and lookup(first=...) in one pass — the row that
  // claims a digest probes the index for it; duplicate rows get size 0 (fill them in
  // with expand_coalesced after the gather). `table`: coalesce_table_slots(n) words.
  // `cslot` (optional, u32 [n]): each claiming row's table slot, for
  // expand_coalesced_out to clear; `table_clean`: the caller guarantees a zeroed table
  // (skips the memset).
  // `prefix` (optional, kMaxGrid + 1 words): block-local offsets — `off` gets each row's
  // offset within its lookup workgroup's rows and `prefix` the exclusive prefix of the
  // workgroup totals (one small scan instead of the n-row one); returns the row shift of a
  // workgroup (its rows are [b << shift, (b + 1) << shift)), for gather(prefix, shift).
  // Without `prefix`: `off` is the exclusive scan of `size`; returns -1.
  // `index_done`: completes with the kernel that reads (and reference-marks) the index, as
  // that kernel's own completion signal (no marker packet between it and the next kernel
  // of `s`): a SET's index insert on another stream may wait for it.
  int lookup_coalesced(const Digest* keys, int64_t n, uint32_t* table, int64_t table_slots,
                       uint32_t* first, uint64_t* loc, uint64_t* size, uint64_t* off,
                       uint32_t now, hipStream_t s, uint64_t reserve = 0, int total_slot = -1,
                       uint32_t* cslot = nullptr, bool table_clean = false,
                       uint64_t* prefix = nullptr, hipEvent_t index_done = nullptr);
  // Slotted lookup (the routed step's owner side): nslots x slot_rows rows, slot k's
  // rows [k * slot_rows, k * slot_rows + slot_cnt[k]) are requests, the rest padding
  // (size 0, not probed, not counted). off = exclusive scan over all rows.
  // `reserve_dev` (optional, device word): a reserve the stream computes before the
  // probe runs (the routed step's received SET bytes), as lookup's `reserve`.
  void lookup_slots(const Digest* keys, int64_t nslots, int64_t slot_rows,
                    const int64_t* slot_cnt, uint64_t* loc, uint64_t* size, uint64_t* off,
                    uint32_t now, hipStream_t s, const uint64_t* reserve_dev = nullptr);
  uint64_t host_slot(int i) const;
  // Spin until the lookup that was given `total_slot` i has written it (no stream or
  // event synchronisation: the kernel's system-scope store is the signal). Throws after
  // timeout_ms. Each lookup that names a slot must be waited for before the slot is reused.
  uint64_t wait_host_slot(int i, int64_t timeout_ms = 10000) const;
  static constexpr int kHostSlots = 64;
  static constexpr int kHeadSlot = kHostSlots - 2;  // the SET chain publishes the head here
  static constexpr uint64_t kSlotPending = ~0ull;
  static constexpr uint64_t kSlotFailed = ~0ull - 1;  // the edge GET could not complete
  // words of a lookup_coalesced `prefix` (the lookup's workgroups, at most 2048, + 1)
  static constexpr int64_t kLookupPrefixWords = 2049;
  // Edge GET (the proxy's micro-batches, n <= kSmallGetMax): probe + scan + gather in
  // one launch, every key probed once (decoupled look-back scan across workgroups).
  // keys / out / off may be mapped host memory (no copies); off[0..n] is always written;
  // off[n] > out_cap means the output is incomplete (nothing is written past out_cap) and
  // the batch must be repeated into a bigger buffer.
  // `done_slot` >= 0: the kernel's last workgroup writes off[n] (or kSlotFailed) into
  // that host slot after every output byte is visible to the host, so
  // wait_host_slot(done_slot) replaces a stream synchronisation. Launches are ordered on
  // their stream (the look-back state is shared), several may be queued at once with
  // distinct slots.
  void small_get(const Digest* keys, int64_t n, uint8_t* out, uint64_t out_cap, uint64_t* off,
                 uint32_t now, hipStream_t s, int done_slot = -1);
  static constexpr int64_t kSmallGetMax = 1 << 17;
  // Persistent edge-GET server: the same contract as small_get for batches of at most
  // kServeKeys rows, answered by one resident workgroup that polls a ring of jobs in
  // pinned host memory — no kernel launch and no stream per batch. The keys are copied
  // into the ring (host pointer); out / off are device views of mapped memory as for
  // small_get, and the total (or kSlotFailed) lands in host slot `done_slot`.
  // Returns false (nothing queued) when the ring is full or n is out of range; the
  // caller then uses small_get. Each call must eventually be followed by serve_kick()
  // calls while its slot is pending (the server exits when idle or at the end of its
  // lifetime, and serve_kick restarts it if jobs are outstanding). Records a SET
  // overwrites while the server copies them come back with a zeroed magic word (the
  // caller treats them as misses). Not ordered against anything on any stream: the
  // caller keeps GETs of keys with SETs / DELETEs in flight on the stream path.
  static constexpr int kServeKeys = 29;   // a job (5 + 2 per key 16-B granules) is one wave's load
  static constexpr int kServeRing = 16;
  bool serve_get(const Digest* host_keys, int64_t n, uint8_t* out, uint64_t out_cap,
                 uint64_t* off, uint32_t now, int done_slot);
  // The same, ordered after the work queued so far on stream `after` only (what the caller
  // queued there to fill `out` / `off`, or SETs it queued on that stream): an event recorded
  // there is host-polled before the job is queued, so the stream-less server never races it.
  // SETs queued on other streams are not covered (ShardedCache queues its SETs on its side
  // and hand streams: call its sync_sets() first).
  bool serve_get_after(hipStream_t after, const Digest* host_keys, int64_t n, uint8_t* out,
                       uint64_t out_cap, uint64_t* off, uint32_t now, int done_slot);
  void serve_kick();
  // server jobs queued or running (the resident workgroup takes them one at a time: a
  // caller with several batches in flight sends the rest down the launched path)
  uint64_t serve_backlog() const {  // any thread (the batcher, reactors submitting directly)
    uint64_t c = 0;
    for (int b = 0; b < srv_blocks_; ++b)
      c += __atomic_load_n(srv_ctl_ + kSrvCtlConsumed + 8 * b, __ATOMIC_ACQUIRE);
    const uint64_t t = __atomic_load_n(&srv_ticket_, __ATOMIC_RELAXED);
    return t > c ? t - c : 0;
  }
  static constexpr int kServeBlocksMax = 8;
  static constexpr int kSrvCtlConsumed = 24;  // control word of block 0's consumed count
  int serve_blocks() const { return srv_blocks_; }
  // wait_host_slot for a serve_get job: spins, relaunching the server when it exited
  uint64_t serve_wait(int done_slot, int64_t timeout_ms = 10000);
  void serve_stop();  // ask the server to exit and wait for it (outstanding jobs stay queued)
  uint64_t serve_launches() const { return srv_launches_; }
  uint64_t serve_jobs() const { return __atomic_load_n(&srv_ticket_, __ATOMIC_RELAXED); }
  // Phase stamps of the last (up to 64) server jobs, wall-clock ticks of the device:
  // rows of {ticket, poll issued, job seen, probed, copied, publish, n, total bytes}; and the
  // tick rate (kHz).
  std::vector<uint64_t> serve_trace() const;
  uint64_t wall_khz() const { return srv_khz_; }
  // GET phase 2: copy each hit's [ItemHeader | value | pad] to out + off[i]. `out` may be
  // pinned host memory (zero-copy); nothing is written when off[n] > out_cap, so the
  // caller can queue the gather before it knows the total and retry if it did not fit.
  // `first` (a coalesced lookup): the gather's workgroups also write every request's
  // (size, off) from its claimer into out_size / out_off and clear the claimers' slots of
  // the coalescing table (expand_coalesced_out's work, no launch of its own).
  void gather(const uint64_t* loc, const uint64_t* off, int64_t n, uint8_t* out, hipStream_t s,
              uint64_t out_cap = ~0ull, const uint32_t* first = nullptr,
              const uint64_t* size = nullptr, uint64_t* out_size = nullptr,
              uint64_t* out_off = nullptr, uint32_t* table = nullptr,
              const uint32_t* cslot = nullptr, const uint64_t* prefix = nullptr,
              int shift = 0);
  // SET a batch. values + val_off[i] holds vlen[i] bytes (val_off 16-byte aligned,
  // the buffer readable 16 bytes past every value). Later duplicates of a key in
  // the same batch win. `bytes_bound` must bound sum(item_bytes(vlen)).
  // `index_after`: the chain up to the log write runs at once, the index insert waits
  // for this event. A lookup enqueued (on another stream) before this store and
  // followed by the event therefore runs concurrently with the SET's dedupe, sizing
  // and log append: it reads the index and the current head slot, which only the index
  // insert changes, and a `reserve` covering this SET keeps its gather off the bytes
  // the append overwrites.
  // `allow_reclaim` false: no CLOCK hand this batch (the append stays within
  // `bytes_bound`; a caller that reserved only that much for it, see would_reclaim).
  // `append_after`: the log append (and what follows) waits for this event; the CLOCK
  // hand, the dedupe and the sizing (reads only) run at once — beside a gather that
  // still reads the region the append will overwrite. `append_done`: recorded right after
  // the log append (a caller can keep its gather from contending with it).
  // `phase` 1 queues only the batch's CLOCK hand, 2 the rest of its chain (0: both).
  // A phase-1 hand is *detached*: it may run as soon as the previous batch's planning is
  // done (`plan_done` of that batch's phase 2), beside that batch's log append and index
  // insert. It reads the head the previous append will reach (the claim word) and the ring
  // tail of the batch before (the last one whose ring entries are written), and its
  // reinsertions are indexed as *moves*: a reinsertion row's insert CASes the entry from
  // the item's old location to the new one, and is dropped when the entry has moved on
  // (a SET or DELETE of the key landed after the hand read the index) — so an early hand
  // can never resurrect a superseded or deleted value. Two hand buffers alternate, so the
  // hand of batch k+1 never writes what batch k's append still reads.
  // `plan_done`: recorded after the batch's planning kernels (dedupe, sizes, offsets).
  // `done`: completes with everything this call queued; carried by the chain's last kernel
  // as its completion signal (profiles/r6_hop: ~2.4 us sooner across queues than a
  // recorded event), or recorded when the call queued no chain.
  void store(const Digest* keys, const uint8_t* values, const uint64_t* val_off,
             const uint32_t* vlen, const uint32_t* flags, const uint32_t* expire, int64_t n,
             uint64_t bytes_bound, uint32_t now, hipStream_t s, hipEvent_t index_after = nullptr,
             bool allow_reclaim = true, hipEvent_t append_after = nullptr,
             hipEvent_t append_done = nullptr, int phase = 0, hipEvent_t plan_done = nullptr,
             hipEvent_t done = nullptr);
  // Whether a SET of `bytes_bound` bytes issued now would run the CLOCK hand (the log is
  // within a few batches of wrapping); the answer can only turn true later.
  bool would_reclaim(uint64_t bytes_bound) const {
    return cfg_.evict == kEvictClock && rmax_ && should_reclaim(bytes_bound);
  }
  // SET through captured hipGraphs, for callers with fixed batch sizes and fixed
  // staging buffers (the proxy's micro-batches, padded to a size class with
  // vlen = kSkipVlen rows). The five SET kernels become one graph launch. A graph bakes
  // in its pointers, `n`, `bytes_bound` and `now` and the head slot it reads, so `g`
  // keeps one executable per head-slot parity and is re-captured whenever any of those
  // (or the SET workspace) changes; `now` changes once a second.
  struct StoreGraph {
    hipGraphExec_t exec[2] = {nullptr, nullptr};
    const void* ptrs[6] = {};
    int64_t n = -1;
    uint64_t bound = 0;
    uint32_t now = 0;
    uint64_t ws_gen = 0;
    uint64_t captures = 0, launches = 0;
  };
  void store_graph(StoreGraph* g, const Digest* keys, const uint8_t* values,
                   const uint64_t* val_off, const uint32_t* vlen, const uint32_t* flags,
                   const uint32_t* expire, int64_t n, uint64_t bytes_bound, uint32_t now,
                   hipStream_t s);
  static void destroy_graph(StoreGraph* g);
  // DELETE a batch; found[i] = 1 if a live entry was removed.
  void remove(const Digest* keys, int64_t n, uint8_t* found, uint32_t now, hipStream_t s);
  // Reclaim index slots whose items expired or were overwritten. Synchronises;
  // returns {live entries, live item bytes}.
  void sweep(uint32_t now, hipStream_t s, uint64_t* live_entries, uint64_t* live_bytes);
  // Digests of every live entry -> out (device, up to out_cap); returns the live
  // count (may exceed out_cap). Synchronises. Used for rebalancing / migration.
  uint64_t export_keys(Digest* out, uint64_t out_cap, uint32_t now, hipStream_t s);
  // Snapshot / warm restore of the whole shard (index + log + head) to a file;
  // `user` carries 4 caller words (e.g. the epoch). load() needs equal geometry.
  void save(const std::string& path, const uint64_t user[4], hipStream_t s);
  void load(const std::string& path, uint64_t user[4], hipStream_t s);
  // Drop everything (memcached FLUSH).
  void flush(hipStream_t s);
  // Tests: read / overwrite one index bucket (4 entries of {d0, d1, loc, vlen | expire
  // << 32}), synchronously. Builds index states no API call produces in a fixed order
  // (e.g. a dead same-digest entry in a key's first bucket beside its live one).
  std::vector<uint64_t> debug_bucket(uint64_t b);
  // {hand (ring index), ring tail, head, the log offset of the hand's item (~0: none), entries
  // the hand consumed last batch, the effective windows of hand buffers 0 and 1}
  std::vector<uint64_t> debug_hand();
  void debug_set_entry(uint64_t b, int slot, uint64_t d0, uint64_t d1, uint64_t loc,
                       uint32_t vlen, uint32_t expire);
  // Tests: move the CLOCK hand to ring index `hand` (e.g. a lap behind the overwrite), and
  // whether the hand may jump to the first entry the overwrite has not reached
  // (hand_catch_up; false isolates it: a hand left behind then spends its windows on
  // overwritten entries).
  void debug_set_hand(uint64_t hand, bool catch_up = true);
  CacheCounters counters(hipStream_t s);
  uint64_t head(hipStream_t s);

  const ShardConfig& config() const { return cfg_; }
  uint8_t* log_ptr() const { return log_; }
  Entry* index_ptr() const { return index_; }
  uint64_t* head_ptr() const { return head_ + hsel_; }
  // Pre-size the SET workspace for batches of n keys, and with CLOCK the hand's workspaces
  // for the combined batch such a SET runs once the log wraps (allocates; synchronises;
  // call outside capture and before serving).
  void reserve(int64_t n);
  // Bytes of grown-out workspaces not freed yet (their chains still running); frees the
  // ones whose chains have finished first.
  uint64_t retired_bytes();
  uint64_t retired_ever() const { return retired_ever_; }  // bytes ever retired (tests)
  uint64_t hbm_bytes() const;
  uint64_t reinsert_max() const { return cfg_.evict == kEvictClock ? rmax_ : 0; }

 private:
  void ensure_set_ws(int64_t n, hipStream_t s);
  void ensure_rc_ws(int64_t w, hipStream_t s);
  void ensure_cb(int b, int64_t rows, hipStream_t s);
  bool should_reclaim(uint64_t bytes_bound) const;
  void reclaim_locked(const Digest* keys, const uint8_t* values, const uint64_t* val_off,
                      const uint32_t* vlen, const uint32_t* flags, const uint32_t* expire,
                      int64_t n, int64_t w, uint64_t rmax, uint32_t now, hipStream_t s,
                      bool detached, bool lead);
  uint64_t* cur_ring_tail() const { return head_ + 2 + hsel_; }
  uint64_t* next_ring_tail() const { return head_ + 2 + (hsel_ ^ 1); }
  // Deferred frees (no device-wide synchronisation on the serving path): a grown buffer's
  // old blocks are retired as a group with one event recorded on the growing call's stream
  // after it has waited for the last store queued on every other stream SET work used
  // (`note_stream`; each store records its stream's `last` event when it returns, so no
  // call ever records on a stream the caller may since have destroyed); reap_retired frees
  // a group once its event has completed (every chain that could read the old blocks has
  // finished) — at the start of every store and in sweep; reserve (which synchronises the
  // device) and the destructor free every group.
  struct RetiredGroup {
    std::vector<void*> ptrs;
    std::vector<hipEvent_t> ev;
    uint64_t bytes = 0;
  };
  void retire_group(std::initializer_list<void*> ptrs, uint64_t bytes, hipStream_t s);
  void reap_retired(bool all);
  void note_stream(hipStream_t s);
  void note_store_end(hipStream_t s);
  std::vector<RetiredGroup> retired_;
  uint64_t retired_ever_ = 0;
  struct SetStream {
    hipStream_t s = nullptr;
    hipEvent_t last = nullptr;  // recorded after the last store queued on s
  };
  std::vector<SetStream> set_streams_;
  // The SET workspace's tables are cleared on the stream of the call that grew them;
  // a store on another stream waits for that (ws_ready_) once (ws_ordered_).
  hipEvent_t ws_ready_ = nullptr;
  hipStream_t ws_grow_stream_ = nullptr;
  std::vector<hipStream_t> ws_ordered_;
  void ws_order(hipStream_t s);
  // CLOCK state
  uint64_t* ring_ = nullptr;           // item-start ring (logical locs, kRingSkip holes)
  uint64_t ring_cap_ = 0;
  unsigned long long* rc_ctl_ = nullptr;  // hand, batch bytes, cut, entries scanned
  bool lead_ = false;  // the hand's mode (layout.h hand_lead, sticky; HostCache keeps the same)
  bool catch_up_ = true;  // debug_set_hand
  uint64_t rmax_ = 0;
  int64_t rc_cap_ = 0;
  uint64_t *rc_loc_ = nullptr, *rc_h_ = nullptr, *rc_part_ = nullptr, *rc_hx_ = nullptr;
  int64_t rc_adv_w_ = 0;
  // store(phase=1) queued a batch's CLOCK hand and planning; store(phase=2) runs the rest
  // of its chain (append, index insert) from this record
  struct Pending {
    bool active = false;
    int64_t n = 0, rows = 0, nmove = 0;  // caller rows; rows of the (combined) batch; moves
    int parity = 0;                       // its SET workspace and hand buffer
    const Digest* keys = nullptr;
    const uint8_t* values = nullptr;
    const uint64_t* voff = nullptr;
    const uint32_t *vlen = nullptr, *flags = nullptr, *expire = nullptr;
    const uint64_t* from = nullptr;
  };
  Pending pend_;
  int hand_b_ = 0;  // the hand buffer reclaim_locked fills
  // The combined SET batch (reinsertion rows, then the batch's own rows) and the staged
  // reinsertion records, two buffers taken in turn (a detached hand fills one while the
  // previous batch's chain still reads the other). `from`: a reinsertion row's old entry
  // loc (a move), 0 for the batch's rows.
  struct HandBuf {
    Digest* keys = nullptr;
    uint64_t* voff = nullptr;
    uint64_t* from = nullptr;
    uint32_t *vlen = nullptr, *flags = nullptr, *expire = nullptr;
    int64_t cap = 0;
    uint8_t* scratch = nullptr;  // staged reinsertions (rmax_ + 64 bytes)
  };
  HandBuf hb_[2];
  // SET workspaces, two taken in turn by consecutive batches (ws_next_): a batch's planning
  // (phase 1) may run while the previous batch's append and index insert still use theirs.
  // The dd_* / set_* members below point at the one in use (select_ws).
  struct SetWs {
    uint64_t* dd_keys = nullptr;
    int* dd_win = nullptr;
    uint32_t* dd_slot = nullptr;
    uint64_t *set_size = nullptr, *set_off = nullptr, *set_cnt = nullptr;
    uint32_t* set_claim = nullptr;
  };
  SetWs ws_[2];
  int ws_next_ = 0;
  void select_ws(int p) {
    const SetWs& w = ws_[p];
    dd_keys_ = w.dd_keys; dd_win_ = w.dd_win; dd_slot_ = w.dd_slot; set_size_ = w.set_size;
    set_off_ = w.set_off; set_cnt_ = w.set_cnt; set_claim_ = w.set_claim;
  }

  ShardConfig cfg_;
  uint8_t* log_ = nullptr;
  Entry* index_ = nullptr;
  uint64_t* head_ = nullptr;         // device: logical write head, 2 ping-pong slots
  int hsel_ = 0;                     // slot holding the current head
  uint64_t* cur_head() const { return head_ + hsel_; }
  // furthest log byte any queued SET append will write (monotone; set before the append)
  uint64_t* claim_ptr() const { return head_ + 4; }
  uint64_t* next_head() const { return head_ + (hsel_ ^ 1); }
  CacheCounters* ctr_ = nullptr;     // device counters (64 shards)
  unsigned long long* scratch_ = nullptr;  // device scratch for reductions
  uint64_t* part_ = nullptr;         // per-workgroup sums: GET sizes, SET sizes, SET counts
  uint64_t* host_buf_ = nullptr;     // pinned scratch for small D2H reads
  uint64_t* host_slots_ = nullptr;   // pinned coherent slots the GPU writes totals into
  // persistent edge-GET server (serve_get): job ring + control words in pinned coherent
  // memory, its own CU-masked stream (a queue of its own: nothing queues behind it)
  void* srv_ring_ = nullptr;
  uint64_t* srv_ctl_ = nullptr;      // [8] exited epoch, [16] stop, [24 + 8 b] block b's consumed
  uint64_t* srv_sync_ = nullptr;     // device: the server blocks' shared idle clock, exit count
  int srv_blocks_ = 1;
  hipStream_t srv_stream_ = nullptr;
  uint64_t srv_ticket_ = 0, srv_epoch_ = 0, srv_launches_ = 0;
  uint64_t srv_idle_ticks_ = 0, srv_life_ticks_ = 0, srv_khz_ = 0;
  uint64_t* srv_trace_ = nullptr;    // pinned: per-job phase stamps (serve_trace)
  bool srv_running_ = false;
  std::mutex srv_mu_;
  void serve_launch_locked();
  unsigned int* done_ctr_ = nullptr; // device: edge-GET workgroups finished + fail flag (self-resetting)
  unsigned long long* lb_state_ = nullptr;  // device: edge-GET look-back words (self-resetting)
  // SET workspace
  int64_t set_cap_ = 0;
  uint64_t* dd_keys_ = nullptr;
  int* dd_win_ = nullptr;
  uint32_t* dd_slot_ = nullptr;
  uint64_t* set_size_ = nullptr;
  uint64_t* set_off_ = nullptr;
  uint32_t* set_claim_ = nullptr;  // entry each SET row claimed (k_set_fixup)
  uint64_t* set_cnt_ = nullptr;    // ring ordinal of each stored SET row (CLOCK)
  uint32_t dd_mask_ = 0;
  uint64_t ws_gen_ = 0;  // bumped when the SET workspace moves (invalidates graphs)
  std::mutex mu_;
  // store(done): the event the call's last kernel carries as its completion signal (taken
  // by that launch; recorded by a marker if the path queued no such kernel)
  hipEvent_t stop_ev_ = nullptr;
  void store_locked(const Digest* keys, const uint8_t* values, const uint64_t* val_off,
                    const uint32_t* vlen, const uint32_t* flags, const uint32_t* expire,
                    int64_t n, uint32_t now, hipStream_t s, hipEvent_t index_after = nullptr,
                    hipEvent_t append_after = nullptr, hipEvent_t append_done = nullptr,
                    const uint64_t* from = nullptr, hipEvent_t plan_done = nullptr,
                    int64_t nmove = 0);
  void store_plan_locked(const Digest* keys, const uint32_t* vlen, int64_t n, hipStream_t s,
                         bool detached = false);
  void store_tail_locked(uint32_t now, hipStream_t s, hipEvent_t index_after,
                         hipEvent_t append_after, hipEvent_t append_done);
  void store_index_locked(const Digest* keys, const uint32_t* vlen, const uint32_t* expire,
                          int64_t n, uint32_t now, hipStream_t s, hipEvent_t index_after,
                          const uint64_t* from = nullptr, int64_t nmove = 0,
                          int win_parity = -1);
};

// ---- Generic device kernels used by the distributed serving path ----------------

// Exclusive scan of in[0..n) into out[0..n] (out[n] = total), u64.
void device_exclusive_scan(const uint64_t* in, uint64_t* out, int64_t n, void* tmp,
                           size_t tmp_bytes, hipStream_t s);
size_t device_scan_tmp_bytes(int64_t n);

// Load-balanced segmented copy: segment i copies (dst_off[i+1]-dst_off[i]) bytes
// from src + src_off[i] to dst + dst_off[i]. All offsets/lengths multiples of 16.
// src_off[i] == kSegSkip: segment i is a gap (nothing read or written).
constexpr uint64_t kSegSkip = ~0ull;
void segcopy(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off, int64_t n,
             uint8_t* dst, hipStream_t s, uint64_t dst_cap = ~0ull);
// Device-count variant (absolute source addresses in src_off): the number of segments is
// *n_dev, read by the kernel, so a segment list the GPU built needs no host read.
void segcopy_dev(const uint64_t* src_off, const uint64_t* dst_off, const int64_t* n_dev,
                 uint8_t* dst, hipStream_t s, uint64_t dst_cap = ~0ull);
// Sized variant: segment i holds seg_len[i] bytes at dst + dst_off[i] (dst_off ascending,
// gaps allowed and left untouched, dst_off[n] = the extent); a segment that does not end
// within `cap` is dropped (the others still land). Offsets / lengths multiples of 16.
void segcopy_sized(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off,
                   const uint64_t* seg_len, int64_t n, uint8_t* dst, hipStream_t s,
                   uint64_t cap = ~0ull);

// GET coalescing: first[i] = the row that serves row i (one row per distinct digest
// serves all its duplicates). `table` is scratch of coalesce_table_slots(n) u32 words.
int64_t coalesce_table_slots(int64_t n);
void coalesce_keys(const Digest* keys, int64_t n, uint32_t* table, int64_t table_slots,
                   uint32_t* first, hipStream_t s, uint32_t* cslot = nullptr,
                   bool table_clean = false);
// After the gather of a coalesced lookup: size[i], off[i] of every duplicate row i :=
// those of first[i] (in place), so each request addresses its claimer's record.
void expand_coalesced(const uint32_t* first, int64_t n, uint64_t* size, uint64_t* off,
                      hipStream_t s);

// Out-of-place variant (may overlap the gather): out_size/out_off[i] := size/off of
// first[i] for every row; claimers clear their table slot (cslot from lookup_coalesced)
// so the table is clean for the next batch.
void expand_coalesced_out(const uint32_t* first, int64_t n, const uint64_t* size,
                          const uint64_t* off, uint64_t* out_size, uint64_t* out_off,
                          uint32_t* table, const uint32_t* cslot, hipStream_t s);

// GET records -> a SET batch (shard migration over xGMI: records gathered on one GPU,
// peer-copied to another, stored there). Row i's record is rec[off[i] .. +size[i]]
// (size 0 = miss); a row whose `have_size[i]` (the destination's own lookup, may be null)
// is non-zero is skipped — insert-if-absent, so a migration never overwrites an object
// the destination has stored since. Outputs: vlen = kSkipVlen for skipped rows.
void records_to_set(const uint8_t* rec, const uint64_t* off, const uint64_t* size,
                    const uint64_t* have_size, int64_t n, Digest* keys, uint64_t* val_off,
                    uint32_t* vlen, uint32_t* flags, uint32_t* expire, hipStream_t s);

// Digest packed key bytes: key i = bytes[offs[i] .. offs[i+1]).
void digest_keys(const uint8_t* bytes, const int64_t* offs, int64_t n, Digest* out,
                 hipStream_t s);

// Consistent-hash routing: dest[i] = owner of the first ring point >= ring_position(keys[i])
// (wrapping), counts[r] += #keys routed to r. `counts` must be zeroed by the caller.
void route_keys(const Digest* keys, int64_t n, const uint32_t* ring_pts, const int32_t* ring_owner,
                int32_t npts, int32_t* dest, int64_t* counts, int32_t nranks, hipStream_t s);

// Stable-within-wave scatter of records by destination: pos = base[dest[i]] + rank,
// perm[i] = pos, out[pos] = in[i] for `rec_bytes`-byte records (16 or 32-multiple of 4).
void scatter_by_dest(const int32_t* dest, const int64_t* base, int64_t n, int32_t nranks,
                     int64_t* cursor, int64_t* perm, hipStream_t s);
void permute_records(const void* in, const int64_t* perm, int64_t n, int32_t rec_bytes, void* out,
                     hipStream_t s);

// MFMA smoke kernel (BASELINE.json platform check): C[32x32] = A[32x16] * B[16x32],
// bf16 inputs, fp32 accumulate, one v_mfma_f32_32x32x16_bf16 per wave.
void mfma_hello(const uint16_t* a, const uint16_t* b, float* c, int tiles, hipStream_t s);

}  // namespace shellac
