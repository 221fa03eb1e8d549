// Cache backends behind the proxy and the memcached-protocol shard server.
//
// The reference has exactly one: a blocking pylibmc client doing one TCP round
// trip per request inside the reactor (src/python/shellac/server/Server.py:335
// get, :432 set). Here every backend is asynchronous (completions are posted to
// the calling reactor's Executor), so a slow cache never stalls the event loop:
//
//   DramBackend       striped host-DRAM shards (csrc/host_cache.cc), synchronous
//                     fast path, no GPU needed;
//   HbmBackend        one HBM shard per local MI355X (csrc/hbm_cache.hip), fed by a
//                     batcher thread that coalesces the GETs/SETs of all reactors
//                     into one kernel pipeline per GPU per tick;
//   MemcachedBackend  memcached binary protocol over TCP to remote nodes (real
//                     memcached or `shellac-cached`), ketama-routed, pipelined on
//                     persistent connections, with node ejection + retry.
#pragma once

#include <cstdlib>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "digest.h"
#include "host_cache.h"
#include "host_router.h"
#include "ketama.h"
#include "net.h"
#include "object_cache.h"
#include "presence_filter.h"
#include "stream_buf.h"

namespace shellac {

class HbmCache;

class Executor {
 public:
  virtual ~Executor() = default;
  virtual void post(std::function<void()> fn) = 0;  // run fn on the executor's thread
  // Several completions at once (one lock and one wake-up for a whole GPU batch).
  virtual void post_batch(std::vector<std::function<void()>>& fns) {
    for (auto& f : fns) post(std::move(f));
    fns.clear();
  }
};

struct CacheValue {
  Bytes data;
  uint32_t flags = 0;
  int64_t ttl_left = -1;  // seconds of life left: -1 unknown, 0 never expires
};
using GetCallback = std::function<void(bool hit, CacheValue v)>;
using DelCallback = std::function<void(bool found)>;
using StatList = std::vector<std::pair<std::string, uint64_t>>;

// Asynchronous body compressor for the proxy's -z path: `done` runs on the compressor's
// thread (callers post back to their reactor) with ok = false and the original body when
// compression failed. The GPU implementation is GzipService (deflate.h); the proxy
// itself only sees this interface, so it builds without the HIP runtime.
class Compressor {
 public:
  using Done = std::function<void(bool ok, std::string out)>;
  virtual ~Compressor() = default;
  virtual void submit(std::string body, Done done) = 0;
  // gunzip one member off the caller's thread (output capped at max_out bytes); engines
  // without it return false from can_inflate() and the caller decodes inline
  virtual bool can_inflate() const { return false; }
  virtual void submit_inflate(std::string member, uint64_t max_out, Done done) {
    (void)max_out;
    done(false, std::move(member));
  }
  virtual void stats(StatList* out) = 0;
};

class CacheBackend {
 public:
  virtual ~CacheBackend() = default;
  // `done` runs on `ex`'s thread (inline for synchronous backends).
  virtual void get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) = 0;
  virtual void set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
                   uint32_t ttl_s) = 0;
  virtual void del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) = 0;
  virtual void flush() = 0;
  virtual std::string name() const = 0;
  virtual void stats(StatList* out) = 0;
  // Fault injection / drills: take GPU shard `shard` of this tier out of service (or
  // bring it back). Returns false if the tier has no such shard.
  virtual bool inject_shard_down(int shard, bool down) {
    (void)shard;
    (void)down;
    return false;
  }
  // Reactor-direct submission (HbmBackend's edge server): a reactor thread attaches once
  // with itself as `ex`; its GETs may then be held by the tier and sent to the GPU from
  // the reactor's own loop by direct_service(), which also answers finished ones inline —
  // no batcher-thread hop either way. direct_service() returns true while jobs are
  // outstanding (the loop keeps polling instead of blocking); direct_detach() drains them
  // before the thread exits. Wrappers forward; other tiers ignore them.
  virtual void direct_attach(Executor* ex) { (void)ex; }
  virtual bool direct_service() { return false; }
  virtual void direct_detach() {}
  // Hot-object spreading (HbmBackend on several GPUs): re-plan the replicated hot set now;
  // returns the refresh's counts (empty: the tier has none). Wrappers forward.
  virtual StatList hot_refresh() { return {}; }
};

// 32-bit-point ring over digests, identical to shellac_amd.parallel.ring.ShardRing.
class DigestRing {
 public:
  explicit DigestRing(int nshards, int points_per_shard = 160);
  int owner(const Digest& d) const;
  // Owner among the shards whose bit is set in `alive` (ketama ejection: a dead shard's
  // keys move to the next live point); -1 if none is alive.
  int owner(const Digest& d, uint64_t alive) const;
  const std::vector<std::pair<uint32_t, int>>& points() const { return pts_; }

 private:
  std::vector<std::pair<uint32_t, int>> pts_;
};

// Host-DRAM tier: refcounted immutable objects (object_cache.h) — a hit is shared, not
// copied, and the full key is checked; CLOCK eviction by bytes.
class DramBackend : public CacheBackend {
 public:
  DramBackend(uint64_t bytes, uint32_t max_item, int stripes = 64);
  void get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) override;
  void set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
           uint32_t ttl_s) override;
  void del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) override;
  void flush() override;
  std::string name() const override { return "dram"; }
  void stats(StatList* out) override;
  uint32_t now() const;

 private:
  ObjectCache cache_;
  double epoch_;
};

struct HbmBackendConfig {
  std::vector<int> devices{0};
  uint64_t log_bytes_per_gpu = 8ull << 30;
  uint64_t nbuckets_per_gpu = 1ull << 22;
  uint32_t max_item = 1u << 20;
  int batch_us = 0;           // optional linger for batch-mates (0: natural batching)
  int max_batch = 65536;      // requests per batch at most
  int sweep_interval_s = 10;  // idle-time expiry sweep of every shard (0 = off)
  int spin_us = 50;           // a batcher polls its queue this long before blocking
  bool presence_filter = true;  // answer GETs of never-stored digests on the host
  int depth = 3;              // batches in flight per GPU (pinned staging per batch)
  int evict = 1;              // 0 FIFO, 1 CLOCK (ShardConfig::evict)
  int retry_s = 2;            // an ejected GPU shard is retried after this long
  int batch_timeout_ms = 2000;  // a batch unfinished this long ejects its GPU
  bool flush_on_restore = true;  // a shard back from ejection may hold stale objects
  // ...and is then warmed from its peers over xGMI: the objects of its key range that
  // other shards took while it was out are peer-copied back (hipMemcpyPeerAsync)
  bool warm_restore = true;
  // peer copies of the warm restore: "auto" = direct xGMI where hipDeviceCanAccessPeer
  // says so (peer access enabled at start), staged through pinned host memory otherwise;
  // "staged" forces the host path (tests; a node whose xGMI mapping is broken)
  std::string peer_copy = "auto";
  // Pinned response arenas allocated up front per GPU (depth + 2 of this size): pinning
  // host memory mid-run stalled every socket call on the box for up to ~0.5 s
  uint64_t arena_bytes = 16u << 20;
  // GET batches of at most HbmCache::kServeKeys distinct keys go to the GPU's persistent
  // edge server (HbmCache::serve_get: no launch per batch) unless a SET / DELETE of one
  // of their keys is still in flight; off: every batch is a launch on the stream
  bool edge_server = true;
  // server jobs that may be ahead of a batch sent to it: 2 = a batch waits behind at most
  // one job (~4-9 us) rather than take a launch (~15 us) — c=10 284K vs 252K RPS at 1
  // (profiles/archive/r3_http)
  int serve_backlog = 2;
  // resident edge-server blocks per GPU (ShardConfig::serve_blocks): jobs of different
  // submitters are served side by side; serve_backlog counts jobs per block
  int serve_blocks = 8;
  // CPUs the batcher threads run on (thread i on batcher_cpus[i % size]; empty: unpinned)
  std::vector<int> batcher_cpus;
  // Reactor-direct GETs (CacheBackend::direct_attach): an attached reactor writes its own
  // edge-server jobs (at most kServeKeys distinct keys, while fewer than direct_backlog
  // jobs are queued on the server) and polls their completion words in its loop; larger
  // or write-ordered batches still go through the batcher. Needs edge_server.
  bool direct = true;
  int direct_backlog = 4;
  uint64_t direct_arena_bytes = 1u << 20;  // pinned arenas reserved per GPU for them
  int direct_arenas = 32;
  // Hot-object spreading over the shards (more than one device, and
  // flush_on_restore: a restored shard must not keep replicas it missed writes for). The
  // `hot_objects` most requested objects of a sampled GET stream (one GET in `hot_sample`,
  // a power of two) are replicated on every shard: their SETs / DELETEs are written through
  // to every shard, their GETs go to a designated shard chosen to even out the load
  // (objects above `hot_spray_above` of the sampled GETs, default 1/(4N), are sprayed over
  // all shards). A refresh thread re-plans every `hot_refresh_ms` (0: only on request,
  // HbmBackend::hot_refresh) once `hot_min_samples` samples are in, and fetches the
  // records of newly hot objects from their owners over xGMI (at most hot_fill_budget
  // bytes per refresh, hottest first). 0 objects: plain ketama (every key on its owner).
  int hot_objects = 1024;
  int hot_refresh_ms = 1000;
  int hot_sample = 8;
  uint64_t hot_min_samples = 512;
  uint64_t hot_fill_budget = 256ull << 20;
  double hot_spray_above = 0;  // 0: 1 / (4 * shards)
};

// One HBM shard per local MI355X. Each GPU has its own batcher thread: requests are
// routed to their shard's queue by the digest ring, and the batcher keeps up to `depth`
// batches in flight on its stream — GETs as one edge-GET launch that writes hits
// straight into a pinned arena (handed to the reactors as zero-copy ByteRef slices),
// SETs/DELETEs from pinned staging — reaping them in order as their completion slots /
// events fire. A batch that errors or stalls ejects its GPU from the ring (its keys
// fall through to the origin) until retry_s passes and the GPU proves healthy.
class HbmBackend : public CacheBackend {
 public:
  explicit HbmBackend(const HbmBackendConfig& cfg);
  ~HbmBackend() override;
  void get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) override;
  void set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
           uint32_t ttl_s) override;
  void del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) override;
  void flush() override;
  std::string name() const override { return "hbm"; }
  // peer path chosen for src -> dst: 0 same device, 1 direct (peer access), 2 staged
  int peer_path(int src_dev, int dst_dev) const;
  void stats(StatList* out) override;
  bool inject_shard_down(int shard, bool down) override;
  void direct_attach(Executor* ex) override;
  bool direct_service() override;
  void direct_detach() override;

  struct HotFill;
  struct Req {
    int kind;  // 0 get, 1 set, 2 del, 3 barrier, 4 hot-replica fill
    Digest d;
    std::string key;
    Bytes value;
    uint32_t flags = 0, ttl = 0;
    Executor* ex = nullptr;
    GetCallback gcb;
    DelCallback dcb;
    // kinds 3 / 4: runs on the batcher thread once the request's flight has finished on
    // the GPU (ok) or was failed
    std::function<void(bool ok)> ccb;
    std::shared_ptr<HotFill> fill;
  };
  struct Dev;
  struct Direct;
  // One hot-set refresh now (serialised with the refresh thread's); its counts. A no-op
  // with spreading off.
  StatList hot_refresh() override;
  bool hot_spreading() const { return hot_on_; }
  // reactor contexts (host slots kDirectSlot0 + kDirectJobs * context + job)
  static constexpr int kDirectJobs = 2, kDirectSlot0 = 32, kDirectMax = 15;

 private:
  // owner among the shards up in `up` (-1: none)
  int owner_of(const Digest& d, uint64_t up) const;
  // a GET's shard: a hot object's designated / sprayed replica when that shard holds the
  // replicas (spread_mask_) and is up, else the owner
  int route_get(const Digest& d);
  void sample_get(const Digest& d);
  void enqueue_ctl(int dev, std::function<void(bool)> cb);
  void hot_loop();
  StatList hot_refresh_locked();
  void enqueue(int dev, Req r);
  void enqueue_many(int dev, std::vector<Req>& rs);
  uint32_t now() const;
  // SETs / DELETEs accepted and not yet finished on the GPU, counted per digest hash: a
  // reactor-direct GET of such a key goes through the batcher (ordered after them)
  static constexpr size_t kWpend = 1 << 16;
  void write_begin(uint64_t lo) {
    wpend_[lo & (kWpend - 1)].fetch_add(1, std::memory_order_acq_rel);
  }
  void write_end(uint64_t lo) {
    wpend_[lo & (kWpend - 1)].fetch_sub(1, std::memory_order_acq_rel);
  }
  bool writes_pending(uint64_t lo) const {
    return wpend_[lo & (kWpend - 1)].load(std::memory_order_acquire) != 0;
  }
  void direct_submit(Direct& dc, size_t k);
  void direct_reap(Direct& dc, size_t k, int j);

  HbmBackendConfig cfg_;
  DigestRing ring_;
  std::vector<std::unique_ptr<Dev>> devs_;
  std::unique_ptr<std::atomic<uint32_t>[]> wpend_;
  std::mutex direct_mu_;
  std::vector<std::unique_ptr<Direct>> direct_;
  std::vector<uint8_t> peer_ok_;  // [src * n + dst]: peer access enabled (direct xGMI copies)
  std::atomic<uint64_t> up_mask_{0};  // bit i: shard i serves requests
  double epoch_;
  std::atomic<uint64_t> no_shard_misses_{0};
  // ---- hot-object spreading (hot_refresh_locked documents the protocol)
  std::unique_ptr<HostRouter> router_;  // ketama owners + the published hot table
  bool hot_on_ = false;
  // shards holding current replicas of the whole published hot set: a GET may go there
  std::atomic<uint64_t> spread_mask_{0};
  static constexpr int kSampleStripes = 16;
  struct alignas(64) SampleStripe {
    std::mutex mu;
    std::vector<Digest> v;
  };
  std::unique_ptr<SampleStripe[]> samples_;
  std::mutex hot_mu_;  // one refresh at a time; guards the refresh state below
  struct DigestHash {
    size_t operator()(const Digest& d) const { return (size_t)(d.lo ^ (d.hi * 0x9E3779B97F4A7C15ull)); }
  };
  struct DigestEq {
    bool operator()(const Digest& a, const Digest& b) const { return a.lo == b.lo && a.hi == b.hi; }
  };
  std::unordered_map<Digest, uint64_t, DigestHash, DigestEq> hot_counts_;
  std::vector<Digest> hot_set_;     // the published hot set, hottest first
  std::vector<int32_t> hot_rank_;   // its designated ranks (-1: sprayed)
  std::vector<double> hot_weights_;
  std::thread hot_th_;
  std::mutex hot_th_mu_;
  std::condition_variable hot_cv_;
  bool hot_stop_ = false;
  // GETs answered by a non-owner replica, sharded by the routing thread's slot (every
  // reactor counts without sharing a line)
  struct alignas(64) SpreadCtr {
    std::atomic<uint64_t> v{0};
  };
  SpreadCtr hot_spread_gets_[16];
  std::atomic<uint64_t> hot_refreshes_{0}, hot_added_{0}, hot_removed_{0}, hot_filled_{0},
      hot_fill_skipped_{0}, hot_fill_failed_{0}, hot_deferred_{0},
      hot_fill_bytes_{0}, hot_refresh_us_{0}, hot_samples_{0}, hot_objects_{0},
      hot_dropped_replicas_{0};
};

// Two-level cache: a small host-DRAM L1 in front of a big L2 (HBM shards or
// remote nodes). L1 hits cost a hash probe on the reactor thread (~us); L1
// misses go to L2 and promote on hit; writes go to both levels.
class TieredBackend : public CacheBackend {
 public:
  // promote_max: L2 hits larger than this stay in L2 only (served from there every time,
  // zero-copy for the HBM tier) instead of being copied into — and churning — the L1.
  TieredBackend(std::shared_ptr<CacheBackend> l1, std::shared_ptr<CacheBackend> l2,
                uint32_t promote_ttl_s = 60, uint64_t promote_max = 32 << 10);
  void get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) override;
  void set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
           uint32_t ttl_s) override;
  void del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) override;
  void flush() override;
  std::string name() const override { return l1_->name() + "+" + l2_->name(); }
  void stats(StatList* out) override;
  bool inject_shard_down(int shard, bool down) override;
  void direct_attach(Executor* ex) override {
    l1_->direct_attach(ex);
    l2_->direct_attach(ex);
  }
  bool direct_service() override {
    const bool a = l1_->direct_service();
    return l2_->direct_service() || a;
  }
  void direct_detach() override {
    l1_->direct_detach();
    l2_->direct_detach();
  }
  StatList hot_refresh() override { return l2_->hot_refresh(); }

 private:
  std::shared_ptr<CacheBackend> l1_, l2_;
  uint32_t promote_ttl_;
  uint64_t promote_max_;
  std::atomic<uint64_t> promoted_{0}, not_promoted_{0};
  std::atomic<uint64_t> l1_hits_{0}, l2_hits_{0}, misses_{0};
};

// Fault injection: a decorator that makes the wrapped tier misbehave
// on purpose — GETs answered as misses, SETs dropped, answers delayed, or the whole
// tier "down" (every GET misses, every SET is lost) — with probabilities that can be
// changed while the proxy runs. Used by the failure tests and for drills.
struct FaultSpec {
  double get_miss = 0;    // P(GET answered as a miss without asking the tier)
  double set_drop = 0;    // P(SET silently dropped)
  uint32_t delay_us = 0;  // extra latency before every GET/DEL is answered
  bool down = false;      // tier unreachable
  int gpu_down = -1;      // GPU shard K of the tier ejected (HbmBackend ring ejection)
};
FaultSpec parse_fault_spec(const std::string& spec);  // "get_miss=0.1,set_drop=1,delay_us=500,down"

class FaultBackend : public CacheBackend {
 public:
  FaultBackend(std::shared_ptr<CacheBackend> inner, const FaultSpec& spec, uint64_t seed = 1);
  ~FaultBackend() override;
  void get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) override;
  void set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
           uint32_t ttl_s) override;
  void del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) override;
  void flush() override { inner_->flush(); }
  std::string name() const override { return "fault(" + inner_->name() + ")"; }
  void stats(StatList* out) override;
  bool inject_shard_down(int shard, bool down) override;
  void direct_attach(Executor* ex) override { inner_->direct_attach(ex); }
  bool direct_service() override { return inner_->direct_service(); }
  void direct_detach() override { inner_->direct_detach(); }
  StatList hot_refresh() override { return inner_->hot_refresh(); }
  void set_spec(const FaultSpec& spec);
  FaultSpec spec() const;

 private:
  bool roll(double p);
  void later(std::function<void()> fn);  // run after delay_us on the timer thread
  void timer_loop();

  std::shared_ptr<CacheBackend> inner_;
  mutable std::mutex mu_;
  FaultSpec spec_;
  uint64_t rng_;
  std::atomic<uint64_t> injected_miss_{0}, injected_drop_{0}, injected_delay_{0};
  // delay timer
  std::condition_variable cv_;
  std::deque<std::pair<double, std::function<void()>>> timers_;  // FIFO: one fixed delay
  bool stop_ = false;
  std::thread th_;
};

struct MemcachedConfig {
  std::vector<Addr> servers;
  int retry_timeout_s = 2;     // ejected node is retried after this long
  int connect_timeout_ms = 500;
  int op_timeout_ms = 1000;
};

class MemcachedBackend : public CacheBackend {
 public:
  explicit MemcachedBackend(const MemcachedConfig& cfg);
  ~MemcachedBackend() override;
  void get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) override;
  void set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
           uint32_t ttl_s) override;
  void del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) override;
  void flush() override;
  std::string name() const override { return "memcached"; }
  void stats(StatList* out) override;

 private:
  struct Pending {
    uint8_t op;
    Executor* ex;
    GetCallback gcb;
    DelCallback dcb;
    double t0;
  };
  struct Node;
  struct Cmd {
    std::string key;
    uint8_t op;
    Bytes value;
    uint32_t flags, ttl;
    Executor* ex;
    GetCallback gcb;
    DelCallback dcb;
  };
  void loop();
  void submit(Cmd c);
  void node_fail(int idx);
  void drain_commands();
  static std::string wire_key(const std::string& key);

  MemcachedConfig cfg_;
  KetamaRing ring_;
  std::vector<std::unique_ptr<Node>> nodes_;
  int epfd_ = -1, evfd_ = -1;
  std::mutex mu_;
  std::vector<Cmd> inbox_;
  std::atomic<bool> stop_{false};
  std::thread th_;
  std::atomic<uint64_t> gets_{0}, hits_{0}, sets_{0}, errors_{0}, ejections_{0};
};

}  // namespace shellac
