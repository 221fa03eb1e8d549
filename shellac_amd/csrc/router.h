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
#include <deque>
#include <memory>
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
class StepComm;

// The native step's streams, one set per device for the whole process (never destroyed).
struct StepStreams {
  hipStream_t plan = nullptr, set = nullptr, asm_ = nullptr;
};
const StepStreams& step_streams(int device);

// The routed serving step of one rank as a native executor, device-driven: no host sync
// between plan and finish. ShardedCache issues the collectives (torch.distributed ->
// RCCL) and hands every buffer in between to this object, which keeps its scratch in a
// grow-only device arena.
//
// Fixed-capacity exchange. The GET requests and the replies travel in per-peer slots of
// a capacity every rank agrees on (capG rows, capD reply bytes), so the all-to-alls need
// no split sizes from the device: counts and per-row (size, offset) ride in-band. The
// capacities come from the demand the ranks observed in earlier steps (one all-gathered
// row per rank per step), the same numbers on every rank, with slack; a row that does
// not fit its slot is answered as a miss (always a valid cache answer) and counted, and
// the next steps' capacities grow. The first step after a reset calibrates the
// capacities with two host reads (the only synchronising step).
// SETs travel the same way in step(): per-peer slots of capS records + capSB value bytes
// with the row / byte count in a 16-B slot header, packed from a segment list the GPU builds
// (k_set_fit, k_set_pack_segs, segcopy_dev). A SET row that does not fit its slot is never
// dropped: it is carried (key, metadata, value bytes) into the next step's plan, ahead of
// that step's own rows, and stored one step later. The host reads nothing in the middle of
// a step: the capacities of step i come from the matrices of steps <= i - 2 (the host waits
// for a matrix two steps old, complete long before), every rank the same.
// (The multi-call path of calibrating steps still exchanges SETs with exact sizes read by
// the host: set_splits / pack_sets / store_sets.)
// Self traffic never enters a collective: a rank probes its own slot in
// place and gathers its own replies straight into the response buffer.
//
// Slot layouts (o(q) = q < rank ? q : q - 1 orders the other ranks):
//   G    = [recv: W-1 slots | self slot | send: W-1 slots], capG x 16-B digests each;
//          the owner probes G[0, W capG) (sources in o-order, self last) in place.
//   R    = [W-1 reply slots] (send), slot o(q) for requester q.
//   data = [local region capL | W-1 reply slots (recv, o-order) | self reply slot]:
//          the response buffer. A reply slot = [capG x u64 (size << 32 | offset)][capD].
//   all-gathered row (K = 4W + 8 int64): [GET rows to p (W) | SET rows to p (W) |
//          SET bytes to p (W) | reply bytes produced for q, previous step (W) |
//          n_local, local_bytes, n_dup, reply rows dropped (previous step), 0 x 4].
// Per step (stream-ordered on `s`):
//   plan(G) -> [all_gather row -> mat] -> publish(mat)
//   -> [a2a G send -> G recv, capG*16 per other rank]
//   -> owner_probe(G) (reserves this step's SET bytes) -> [SET stream forks here]
//   -> (calibration only: owner_demand, all_gather, calibrate_reply)
//   -> owner_reply(R, data) -> [async a2a R -> data, slot bytes per other rank]
//   -> gather_local(data) -> set_splits() (host waits for publish)
//   -> on the SET stream: pack_sets(S) -> [a2a S -> Rs, exact sizes] -> store_sets(Rs),
//      i.e. the main-shard SET chain beside the reply gather
//   -> on a side stream after the reply a2a: assemble(data, out) -> wait() before reading.
//   (step(): the reply transfer and the assembly share the caller's `sasm` stream; the SET
//   exchange uses fixed slots: pack_fixed(S) -> [a2a S -> Rs, slotS per peer] ->
//   store_fixed(Rs), no host read.)
// Communicator modes (step()): `single` (default) issues every collective of a step on ONE
// communicator and ONE stream (the assembly stream) in a fixed order — all-gather, request
// a2a, reply a2a, SET a2a — with events carrying the data dependencies to and from the
// compute streams: every rank sees the same FIFO of collectives, so no two collectives can
// wait on each other. `channels` keeps one communicator per channel on the stream that
// produces its data (the three may run concurrently; see docs/ARCHITECTURE.md).
class RoutedStep {
 public:
  static constexpr int kExtras = 8;
  RoutedStep(int world, int rank, int device);
  ~RoutedStep();
  RoutedStep(const RoutedStep&) = delete;
  RoutedStep& operator=(const RoutedStep&) = delete;

  void set_ring(const uint32_t* pts, const int32_t* owner, int32_t npts);
  // Simulated world (bench.py --simulate-world): the digests the owner probes / stores for
  // the next plan's GET rows and SET rows (routing, replica probes and replica copies keep
  // the request digests). Null: the request digests themselves.
  void set_probe_keys(const Digest* pkeys, const Digest* spkeys) {
    pkeys_ = pkeys;
    spkeys_ = spkeys;
  }
  // Hot set (sorted by signed lo; the directory is kept for the framework-op path). The
  // SET planner probes a hash set built from it on the first call and whenever
  // `changed` (or the pointer / size) says the set is new.
  void set_hot(const Digest* hot, int64_t nhot, const int64_t* dir = nullptr,
               bool changed = false);
  int64_t row_words() const { return 4 * (int64_t)w_ + kExtras; }

  // ---- capacities (identical on every rank: derived from all-gathered rows) ----
  // {capG rows, capD reply bytes, capL local bytes, calibrating, calibrating local} for
  // a GET batch of n rows. While calibrating capG = n (every row fits), capD is set by
  // calibrate_reply during the step; capL (per GET row from this rank's history) by
  // calibrate_local when there is no history yet.
  std::vector<int64_t> caps(int64_t n) const;
  // Before a step: take in the matrices of the steps two back (their history), then caps(n).
  // Call this (not caps) to size a step's buffers: step() does the same harvest first.
  std::vector<int64_t> prepare(int64_t n);
  void reset_caps();  // next step calibrates (new ring, new hot set)
  // Tests: fixed capacities (every rank the same), overriding the policy; 0s clear it.
  void set_cap_override(int64_t capG, int64_t capD, int64_t capL) {
    ovr_ = {capG, capD, capL};
  }
  // SET slot capacities of step(): {capS rows, capSB value bytes per peer slot, capSelf
  // rows, capSelfB bytes stored from this rank's own rows}; from the history like caps().
  std::vector<int64_t> set_caps() const;
  // Tests: fixed SET capacities (every rank the same); 0s clear it.
  void set_set_cap_override(int64_t capS, int64_t capSB, int64_t capSelf, int64_t capSelfB) {
    ovr_s_ = {capS, capSB, capSelf, capSelfB};
  }
  // {SET rows carried into a later step, their bytes, rows lost (carry buffer full)} since
  // construction (host read: waits for the device).
  std::vector<int64_t> carry_stats();
  // Lagged per-step statistics [n_local, n_dup, GET rows sent off-rank, rows over capG,
  // reply rows dropped], summed over the steps harvested since the last call.
  std::vector<int64_t> take_stats();
  // Host: wait for every published step's matrix and add its statistics (not its history:
  // the capacities stay on the two-step lag every rank follows).
  void harvest_all();
  // step(): one communicator and one stream for every collective (default) or one
  // communicator per channel.
  void set_single_comm(bool single) { single_ = single; }
  bool single_comm() const { return single_; }

  // GET routing (coalescing + replica probe first), the digests of peer p's rows written
  // into its slot of G (rows past capG: overflow, answered as misses), SET routing + hot
  // fan-out on a side stream; this rank's all-gather row -> `row`.
  void plan(const Digest* keys, int64_t n, HbmCache* replica, uint32_t now,
            const Digest* skeys, const uint32_t* svlen, const uint32_t* sflags,
            const uint32_t* sexpire, const uint64_t* sval_off, const uint8_t* svalues, int64_t ns,
            bool fanout, uint8_t* G, int64_t* row, hipStream_t s, bool coalesce);
  // After the all-gather: per-source row counts of this rank's owner slots, and the
  // matrix copied to pinned host memory (read by set_splits without stalling the GPU).
  void publish(const int64_t* mat, hipStream_t s);
  // Calibration: wait for the published matrix, fix capL from this step's local bytes.
  void calibrate_local();
  // Owner side: probe the W slots of G in place (padding rows skipped).
  void owner_probe(const uint8_t* G, HbmCache* shard, uint32_t now, hipStream_t s);
  // Reply bytes this shard's probe found per requester -> `out` (W words, device).
  void owner_demand(int64_t* out, hipStream_t s);
  // Calibration: capD from the all-gathered demand (W x W, device; host read).
  void calibrate_reply(const int64_t* dmat);
  // Reply slots: headers (size, offset per row; 0 = miss / dropped) and the records —
  // other requesters' into R, this rank's own straight into data's self slot.
  void owner_reply(HbmCache* shard, uint8_t* R, uint8_t* data, hipStream_t s);
  // The local replica hits' records into data[0, capL).
  void gather_local(uint8_t* data, hipStream_t s);
  // Host: wait for the published matrix; returns [send bytes to p (W) | recv bytes from
  // q (W) | n_local, n_dup, GET rows sent off-rank, rows over capG, reply rows dropped]
  // (self entries included: the SET buffer is [others in rank order | self]).
  std::vector<int64_t> set_splits();
  // SET send buffer: per other rank (rank order) [records 32 B x rows | values]; the
  // self block is never packed. Run on the SET stream (forked from `s` after the probe).
  void pack_sets(uint8_t* S, hipStream_t sset);
  // Received SETs (others from Rs, own straight from the planner's buffers and the
  // caller's batch) into the main shard (tier 0) on the SET stream `sset`, beside the
  // reply gather (the probe reserved their bytes; joined by the next owner_probe), and
  // the replica (tier 1) on `s` after the local gather.
  void store_sets(const uint8_t* Rs, HbmCache* shard, HbmCache* replica, uint32_t now,
                  hipStream_t s, hipStream_t sset, bool replica_on_sset = false,
                  hipEvent_t index_after = nullptr, bool allow_reclaim = true);
  // Per-request (size, off) into `data`, in request order (duplicates: their claimer's
  // record); run on a stream that has waited for the reply all-to-all.
  void assemble(const uint8_t* data, uint64_t* out_size, uint64_t* out_off, hipStream_t s);
  // `s` waits for the main-shard SET chain of the last store_sets.
  void join_sets(hipStream_t s);

  // ---- native step -------------------------------------------------------------------
  // The communicator step() issues its collectives on (RCCL, mirror or callbacks).
  void set_comm(std::shared_ptr<StepComm> c);
  bool has_comm() const { return comm_ != nullptr; }
  // Steps whose main-shard SET append started early under a look-ahead reserve.
  int64_t early_sets() const { return early_sets_; }
  // The whole step in one call, every collective issued from here (no Python between
  // them): plan -> all-gather -> publish -> request a2a -> owner probe -> reply (its
  // transfer on the executor's comm stream) -> local gather -> SET exchange on `sset`
  // -> assemble on `sasm`. Not for a calibrating step (caps(n)[3]: the multi-call path;
  // every rank agrees on it). `data` holds caps(n)[2] + W (8 capG + capD) + 16 bytes; out_size /
  // out_off n words each, valid once `sasm` has passed this step. `sset` / `sasm` 0: the
  // process-wide step streams (step_streams). `inputs_ready`
  // (optional): an event after which the GET keys and the SET batch are complete; then
  // the plan runs on a stream of its own beside the previous step's reply gather instead
  // of after everything queued on `s`. Returns
  // [n_local, n_dup, GET rows sent off-rank, rows over capG, reply rows dropped].
  // `svalues_bytes`: the size of the SET batch's value buffer (sizes the carry buffer).
  // Returns take_stats() (the statistics of earlier steps, two steps behind).
  std::vector<int64_t> step(const Digest* keys, int64_t n, HbmCache* replica, uint32_t now,
                            const Digest* skeys, const uint32_t* svlen, const uint32_t* sflags,
                            const uint32_t* sexpire, const uint64_t* sval_off,
                            const uint8_t* svalues, int64_t ns, bool fanout, bool coalesce,
                            HbmCache* shard, uint8_t* data, uint64_t* out_size,
                            uint64_t* out_off, hipStream_t s, hipStream_t sset,
                            hipStream_t sasm, hipEvent_t inputs_ready = nullptr,
                            int64_t svalues_bytes = 0);
  bool sets_pending() const { return sets_pending_; }
  int rank() const { return rank_; }

 private:
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
  };
  template <typename T>
  T* buf(int slot, size_t count);
  // history (hist = true) and statistics of one all-gathered matrix
  std::vector<int64_t> note_matrix(const int64_t* m, int64_t n, int64_t capG, bool hist);
  void harvest(int64_t upto, bool hist);
  void add_stats(const std::vector<int64_t>& st);
  // fixed-slot SET exchange of step()
  void ensure_carry(int64_t rows, uint64_t bytes);
  void pack_fixed(uint8_t* S, int64_t slotS, const std::vector<int64_t>& sc, hipStream_t ps);
  void store_fixed(const uint8_t* Rs, int64_t slotS, const std::vector<int64_t>& sc,
                   HbmCache* shard, HbmCache* replica, uint32_t now, hipStream_t sset,
                   hipEvent_t index_after, bool allow_reclaim);
  // a collective on `home` (channels) or on the comm stream with event hops (single)
  template <typename F>
  void collective(hipStream_t home, hipStream_t comm_stream, int ch, F issue);
  // deferred frees: a block another step's queued work may still read is freed once events
  // recorded on every stream the executor uses have passed (no device synchronisation)
  void retire(void* p);
  void reap(bool all);
  void note_stream(hipStream_t s);

  int w_, rank_, device_;
  const uint32_t* pts_ = nullptr;
  const int32_t* own_ = nullptr;
  int32_t npts_ = 0;
  const Digest* pkeys_ = nullptr;
  const Digest* spkeys_ = nullptr;
  const Digest* hot_ = nullptr;
  int64_t nhot_ = 0;
  const int64_t* hot_dir_ = nullptr;
  Digest* hot_tab_ = nullptr;  // hash set of the hot digests (built by set_hot)
  uint64_t hot_mask_ = 0;
  const Digest* hot_built_ = nullptr;
  int64_t nhot_built_ = 0;
  std::vector<Buf> bufs_;
  int64_t* host_mat_ = nullptr;   // pinned: the published all-gather matrix
  int64_t* host_dmat_ = nullptr;  // pinned: calibration demand matrix
  uint64_t* host_tab_ = nullptr;  // pinned: per-step SET tables (uploaded)
  hipStream_t side_ = nullptr;  // (streams: the process-wide pool, step_streams)
  hipStream_t plan_stream_ = nullptr;  // step(): the pipelined plan
  hipStream_t set_stream_ = nullptr;   // step() without `sset`: the SET side
  hipStream_t asm_stream_ = nullptr;   // step() without `sasm`: reply transfer + assembly
  hipEvent_t ev_pfork_ = nullptr, ev_plan_ = nullptr, ev_rep_ = nullptr, ev_start_ = nullptr;
  bool pfork_valid_ = false, rep_pending_ = false, in_step_ = false;
  // look-ahead reserve (step()): bytes this / the previous probe reserved for the next
  // step's SETs; recent main-shard SET payload bounds; gather-done events per parity
  uint64_t ahead_ = 0, ahead_prev_ = 0;
  int64_t early_sets_ = 0;
  std::vector<int64_t> pay_hist_;
  hipEvent_t ev_gdone_[2] = {nullptr, nullptr};
  bool gdone_valid_[2] = {false, false};
  std::shared_ptr<StepComm> comm_;
  hipEvent_t ev_probe_ = nullptr, ev_local_ = nullptr, ev_rfork_ = nullptr,
             ev_reply_[2] = {nullptr, nullptr};
  bool reply_pending_[2] = {false, false};
  bool row_init_ = false;
  hipEvent_t ev_fork_ = nullptr, ev_pjoin_ = nullptr, ev_pub_ = nullptr, ev_sfork_ = nullptr,
             ev_join_ = nullptr, ev_asm_[2] = {nullptr, nullptr};
  bool asm_pending_[2] = {false, false};
  bool sets_pending_ = false;
  // capacities and their history (max over the window of the all-gathered demand)
  int64_t capG_ = 0, capD_ = 0, capL_ = 0;
  std::vector<int64_t> ovr_ = {0, 0, 0};
  bool calibrating_ = true;
  std::vector<int64_t> hist_g_, hist_d_;
  std::vector<double> hist_lr_;  // local bytes per GET row
  // per-step state
  int par_ = 0;  // step parity: the buffers the deferred assemble reads
  int64_t n_ = 0, ns_ = 0, ns_rows_ = 0, ms_ = 0;
  bool have_replica_ = false, published_ = false;
  HbmCache* replica_ = nullptr;
  const uint8_t* values_ = nullptr;
  uint64_t *rl_loc_ = nullptr, *rl_size_ = nullptr, *rl_off_ = nullptr;
  uint32_t* first_ = nullptr;
  int64_t* route_ = nullptr;
  int64_t *srec_ = nullptr, *cnt_s_ = nullptr;
  uint64_t *sval_ = nullptr, *svoff_ = nullptr;
  int64_t* own_cnt_ = nullptr;
  const int64_t* mat_dev_ = nullptr;  // the all-gathered matrix (device), from publish
  int64_t self_row0_ = 0;             // first row of the self block in srec_ / sval_
  uint64_t *lk_loc_ = nullptr, *lk_size_ = nullptr, *lk_off_ = nullptr;
  int64_t* rb_ = nullptr;       // reply bytes per requester (W) + dropped rows (1)
  std::vector<int64_t> mat_;    // host copy of this step's matrix (after set_splits)
  // ---- lagged matrices (step()): pinned ring, harvested two steps later ----
  static constexpr int kPend = 4;
  struct Pend {
    int64_t step, n, capG;
    int slot;
    bool hist_done, stats_done;
  };
  std::deque<Pend> pend_;
  int64_t* host_ring_ = nullptr;
  hipEvent_t ev_ring_[kPend] = {};
  int ring_next_ = 0;
  int64_t step_id_ = 0;
  std::vector<int64_t> stat_acc_ = std::vector<int64_t>(5, 0);
  // ---- fixed-slot SETs and the carry (two parities) ----
  std::vector<int64_t> hist_s_, hist_sb_, hist_self_, hist_selfb_;
  std::vector<int64_t> ovr_s_ = {0, 0, 0, 0};
  Digest* ck_[2] = {nullptr, nullptr};
  uint32_t *cvl_[2] = {nullptr, nullptr}, *cfl_[2] = {nullptr, nullptr},
           *cex_[2] = {nullptr, nullptr};
  uint64_t* cval_[2] = {nullptr, nullptr};
  int32_t* cdst_[2] = {nullptr, nullptr};
  uint8_t* cbytes_[2] = {nullptr, nullptr};
  int64_t ccap_p_[2] = {0, 0};     // carry rows per parity
  uint64_t cbcap_p_[2] = {0, 0};   // carry value bytes per parity
  unsigned long long* cctr_ = nullptr;  // [parity][rows, bytes] + totals[rows, bytes, lost]
  bool carry_written_[2] = {false, false};
  hipEvent_t ev_carry_[2] = {nullptr, nullptr};
  int64_t gt_ = 0;       // SET plan workgroups (carry + batch) of this step
  int64_t nrouted_max_ = 0;
  uint64_t* set_meta_[2] = {nullptr, nullptr};  // per parity: headers, fit, segment bases
  hipEvent_t ev_sdone_[2] = {nullptr, nullptr};  // the SET side of a parity is done
  bool sdone_valid_[2] = {false, false};
  int64_t sv_bytes_ = 0;
  bool single_ = true;
  hipEvent_t ev_c1_ = nullptr, ev_c2_ = nullptr, ev_pack_ = nullptr;
  hipEvent_t ev_hot_ = nullptr;
  bool hot_pending_ = false;
  struct Dead {
    void* p;
    std::vector<hipEvent_t> ev;
  };
  std::vector<Dead> dead_;
  std::vector<hipStream_t> seen_streams_;
  std::vector<int64_t> sset_;   // per destination SET bytes (send), rank order
  std::vector<int64_t> rset_;   // per source SET bytes (recv), rank order
};

}  // namespace shellac
