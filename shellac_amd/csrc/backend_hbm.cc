// HbmBackend: the HTTP proxy's (and the memcached node's) cache tier over one HBM shard
// per local MI355X (split from backend.cc so the host-only backends build without ROCm).
//
// Replaces the reference's blocking memcached round trip inside the reactor
// (src/python/shellac/server/Server.py:335 get, :432 set). Per GPU:
//
//   reactors ──get/set/del──▶ queue ──▶ batcher thread ──▶ HIP stream
//                                          │  flight k:   edge GET (keys + offsets in
//                                          │              mapped memory, values into a
//                                          │              pinned arena), SET store,
//                                          │              DELETE, event
//                                          │  up to `depth` flights in flight
//                                          ◀─ reap in order: completion slot / event
//   reactors ◀──post_batch(callbacks)──────┘  hits = ByteRef slices of the arena
//
// A hit never touches a host copy: the GPU writes [ItemHeader | u16 klen | key | payload]
// into pinned memory, the batcher checks the key bytes and hands out a slice of the
// payload that keeps the arena alive until the last client write completes.
#include <pthread.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <unordered_set>

#include "backend.h"
#include "hbm_cache.h"
#include "keyed.h"
#include "trace.h"

namespace shellac {

namespace {
double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

#define HB_OK(expr)                                                                   \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) throw Error(std::string("HIP: ") + hipGetErrorString(_e) + \
                                      " at " #expr);                                  \
  } while (0)

namespace {

// Mapped pinned buffer (host pointer + its device view) that grows on demand.
struct Mapped {
  uint8_t* h = nullptr;
  uint8_t* d = nullptr;
  size_t cap = 0;
  void ensure(size_t bytes) {
    if (bytes <= cap) return;
    size_t c = cap ? cap : 4096;
    while (c < bytes) c *= 2;
    release();
    HB_OK(hipHostMalloc(reinterpret_cast<void**>(&h), c, hipHostMallocMapped));
    HB_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
    cap = c;
  }
  void release() {
    if (h) (void)hipHostFree(h);
    h = d = nullptr;
    cap = 0;
  }
  template <typename T>
  T* host() const { return reinterpret_cast<T*>(h); }
  template <typename T>
  T* dev() const { return reinterpret_cast<T*>(d); }
};

// Device buffer that grows on demand (the hot-set refresh's staging; the caller has set
// the device). Growing frees the old block, so only the refresh thread, which owns these,
// grows them, and never while a fill that reads them is still queued.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  template <typename T>
  T* ensure(size_t bytes) {
    if (bytes > cap) {
      if (p) (void)hipFree(p);
      p = nullptr;
      cap = 0;
      const size_t c = std::max<size_t>({bytes, 4096});
      HB_OK(hipMalloc(&p, c));
      cap = c;
    }
    return static_cast<T*>(p);
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Pinned response arenas. A GET batch gathers into one; its hits are ByteRef slices that
// own a reference, so the arena returns to the pool (not to the allocator) when the last
// response built from it has been written to its client. Pinned allocations and frees
// are slow and hipHostFree waits for the device, so neither happens on a reactor thread:
// give_back() only files the arena; take() (the batcher) picks the smallest one that
// fits and trims the pool beyond kKeepBytes of idle arenas.
class ArenaPool : public std::enable_shared_from_this<ArenaPool> {
 public:
  struct Arena {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t cap = 0;
  };
  static constexpr size_t kKeepBytes = size_t(1) << 30;  // idle arenas kept (per GPU)
  explicit ArenaPool(int device) : device_(device) {}
  ~ArenaPool() {
    for (auto& a : free_) (void)hipHostFree(a.h);
  }
  std::shared_ptr<Arena> take(size_t min_cap) {
    Arena a{};
    std::vector<Arena> trim;
    {
      std::lock_guard<std::mutex> lk(mu_);
      int best = -1;
      for (size_t i = 0; i < free_.size(); ++i)
        if (free_[i].cap >= min_cap && (best < 0 || free_[i].cap < free_[(size_t)best].cap))
          best = (int)i;
      if (best >= 0) {
        a = free_[(size_t)best];
        free_.erase(free_.begin() + best);
        free_bytes_ -= a.cap;
      }
      while (free_bytes_ > kKeepBytes && !free_.empty()) {  // the smallest idle arenas go
        size_t k = 0;
        for (size_t i = 1; i < free_.size(); ++i)
          if (free_[i].cap < free_[k].cap) k = i;
        free_bytes_ -= free_[k].cap;
        trim.push_back(free_[k]);
        free_.erase(free_.begin() + (long)k);
      }
    }
    for (const Arena& t : trim) {
      (void)hipHostFree(t.h);
      allocated_.fetch_sub(t.cap, std::memory_order_relaxed);
      frees_.fetch_add(1, std::memory_order_relaxed);
    }
    if (!a.h) {
      size_t c = 1u << 20;
      while (c < min_cap) c *= 2;
      HB_OK(hipSetDevice(device_));
      const double t0 = wall_s();
      HB_OK(hipHostMalloc(reinterpret_cast<void**>(&a.h), c, hipHostMallocMapped));
      HB_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.d), a.h, 0));
      const uint64_t us = (uint64_t)((wall_s() - t0) * 1e6);
      if (us > alloc_max_us_.load(std::memory_order_relaxed)) alloc_max_us_.store(us);
      a.cap = c;
      allocated_.fetch_add(c, std::memory_order_relaxed);
      allocs_.fetch_add(1, std::memory_order_relaxed);
    }
    auto pool = shared_from_this();
    return std::shared_ptr<Arena>(new Arena(a), [pool](Arena* p) {
      pool->give_back(*p);
      delete p;
    });
  }
  // take() without allocating or trimming (no HIP call: safe on a reactor thread); null
  // when no idle arena fits
  std::shared_ptr<Arena> try_take(size_t min_cap) {
    Arena a{};
    {
      std::lock_guard<std::mutex> lk(mu_);
      int best = -1;
      for (size_t i = 0; i < free_.size(); ++i)
        if (free_[i].cap >= min_cap && (best < 0 || free_[i].cap < free_[(size_t)best].cap))
          best = (int)i;
      if (best < 0) return nullptr;
      a = free_[(size_t)best];
      free_.erase(free_.begin() + best);
      free_bytes_ -= a.cap;
    }
    auto pool = shared_from_this();
    return std::shared_ptr<Arena>(new Arena(a), [pool](Arena* p) {
      pool->give_back(*p);
      delete p;
    });
  }
  // n arenas of cap bytes into the free list (at start-up, before any traffic)
  void reserve(size_t n, size_t cap) {
    std::vector<std::shared_ptr<Arena>> held;
    for (size_t i = 0; i < n; ++i) held.push_back(take(cap));
  }  // returned to the pool here
  uint64_t allocated() const { return allocated_.load(std::memory_order_relaxed); }
  uint64_t allocs() const { return allocs_.load(std::memory_order_relaxed); }
  uint64_t frees() const { return frees_.load(std::memory_order_relaxed); }
  uint64_t alloc_max_us() const { return alloc_max_us_.load(std::memory_order_relaxed); }

 private:
  void give_back(const Arena& a) {  // any thread (often a reactor): no HIP call here
    std::lock_guard<std::mutex> lk(mu_);
    free_.push_back(a);
    free_bytes_ += a.cap;
  }
  int device_;
  std::mutex mu_;
  std::vector<Arena> free_;
  size_t free_bytes_ = 0;
  std::atomic<uint64_t> allocated_{0}, allocs_{0}, frees_{0}, alloc_max_us_{0};
};

}  // namespace

// One batch in flight on a GPU.
struct Flight {
  std::vector<HbmBackend::Req> reqs;
  std::vector<uint32_t> gets, sets, dels;  // request indices by kind
  std::vector<uint32_t> ctls;              // barriers and hot-replica fills
  std::vector<uint32_t> urow;              // GET request -> GPU row (host coalescing)
  size_t rows = 0;                         // distinct GET digests
  Mapped keys, offs, set_keys, set_vals, set_voff, set_meta, del_keys, del_found;
  std::shared_ptr<ArenaPool::Arena> arena;
  std::vector<uint64_t> wkeys;  // SET / DELETE digests (lo words) counted in Dev::pend_w
  bool flush = false;           // a flush runs on the stream right before this flight
  hipEvent_t ev = nullptr;
  int slot = -1;
  bool active = false, got = false;
  bool served = false;  // GETs answered by the persistent edge server (no stream launch)
  uint32_t tnow = 0;
  double t0 = 0;
};

// A hot-replica fill queued on a target shard (HbmBackend::hot_refresh_locked): m records
// gathered on their owners and peer-copied into this shard's staging (krec at koff, digests
// kk), stored by the target's batcher in stream order. Rows whose digest had a SET or DELETE
// queued to this shard since the refresh began (Dev::touched) are dropped at launch: the
// write-through copy is newer than the owner's record read here.
struct HbmBackend::HotFill {
  int64_t m = 0;
  const Digest* kk = nullptr;
  const uint8_t* krec = nullptr;
  const uint64_t* koff = nullptr;
  uint64_t* hsize = nullptr;      // mapped host view of the row sizes (0: no record)
  const uint64_t* dsize = nullptr;  // its device view
  Digest* okeys = nullptr;
  uint64_t* ovoff = nullptr;
  uint32_t* ometa = nullptr;
  uint64_t bound = 0;
  std::vector<uint64_t> lo;  // row digests' low words (the touched check)
  // under the target Dev's mu
  bool cancelled = false, launched = false;
  uint64_t skipped = 0, rows = 0;
};

struct HbmBackend::Dev {
  HbmBackend* be = nullptr;
  int index = 0, device = 0;
  std::unique_ptr<HbmCache> cache;
  hipStream_t stream = nullptr;
  std::shared_ptr<ArenaPool> pool;
  std::vector<std::unique_ptr<Flight>> flights;
  size_t head = 0, inflight = 0;  // oldest flight, flights launched and not yet freed
  // queue (reactor threads -> batcher)
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Req> q;
  std::atomic<size_t> qn{0};
  std::atomic<bool> spinning{false};
  bool stop = false, flush_req = false;
  bool kick = false;  // the shard's state changed (drill set / lifted): wake an idle batcher
  std::atomic<bool> ctl_pending{false};  // flush / filter rebuild requested (no requests needed)
  std::thread th;
  // health
  std::atomic<bool> forced_down{false};
  // back in the ring and still pulling its objects from peers: GETs neither skip on the
  // presence filter nor bypass the batcher (they queue behind the migration)
  std::atomic<bool> restoring{false};
  bool failed = false;
  double retry_at = 0;
  // presence filter (this shard's digests)
  std::shared_ptr<PresenceFilter> filt, filt_next;
  uint64_t filt_bits = 0, filt_rebuild_at = 0;
  bool filt_want_rebuild = false;
  // warm restore over xGMI: a stream for peer work on this GPU and the digest ring on
  // the device (route_keys)
  hipStream_t mstream = nullptr;
  hipStream_t sstream = nullptr;  // stats reads (non-blocking: never waits on other streams)
  uint32_t* d_pts = nullptr;
  int32_t* d_own = nullptr;
  int npts = 0;
  // co-table for host GET coalescing (batcher thread only)
  std::vector<int32_t> co_tab;
  // hot-set refresh: digests (lo) being filled into this shard, and those of them that a
  // SET / DELETE queued here since (both under mu)
  std::unordered_set<uint64_t> filling, touched;
  // refresh staging on this GPU (the refresh thread's): as an owner (snapshot) and as a
  // target (fill)
  DevBuf hs_keys, hs_loc, hs_size, hs_off, hs_rec, hf_keys, hf_rec, hf_off, hf_okeys, hf_voff,
      hf_meta;
  Mapped hf_size;
  std::atomic<uint64_t> eject_gen{0};  // bumped when the shard leaves service
  struct alignas(64) Ctr {
    std::atomic<uint64_t> v{0};
  };
  // GETs routed to this shard (per-shard load), sharded by the routing thread's slot: the
  // reactors never share a counter line
  static constexpr int kCtrShards = 16;
  Ctr routed_gets[kCtrShards];
  uint64_t routed_total() const {
    uint64_t t = 0;
    for (const Ctr& c : routed_gets) t += c.v.load(std::memory_order_relaxed);
    return t;
  }
  // digests (lo word) with a SET / DELETE in a flight not yet reaped, and flushes in
  // flight: a GET of such a key takes the stream path, ordered after them
  std::unordered_map<uint64_t, uint32_t> pend_w;
  std::unordered_set<uint64_t> take_wset;  // take_batch scratch: write digests so far
  uint32_t pend_flush = 0;
  void track_writes(const Flight& f, int dir);
  double avg_row_bytes = 4096;
  // flushes requested and not yet finished on the GPU (any thread reads it: a
  // reactor-direct GET waits for them by going through the batcher)
  std::atomic<uint32_t> flush_pend{0};
  void flush_done() { flush_pend.fetch_sub(1, std::memory_order_acq_rel); }
  // offsets arrays of the reactor-direct jobs on this GPU (mapped; 32 words per job)
  Mapped direct_offs;
  // stats
  std::atomic<uint64_t> batches{0}, batched_reqs{0}, max_batch{0}, batch_ns{0}, coalesced{0},
      filt_skips{0}, filt_rebuilds{0}, sweeps{0}, live_objects{0}, live_bytes{0},
      key_mismatch{0}, failures{0}, ejections{0}, restores{0}, regathers{0}, arena_misses{0},
      dropped{0}, staged_copies{0}, served_batches{0}, ordered_gets{0},
      migrated{0}, migrate_ns{0}, direct_jobs{0}, direct_reqs{0}, direct_fallbacks{0},
      direct_overflows{0}, direct_timeouts{0}, direct_ns{0};

  void loop();
  bool take_batch(std::vector<Req>* out, bool* do_flush, bool* rebuilding);
  void launch(Flight& f);
  bool try_reap(Flight& f, bool block);
  void deliver_gets(Flight& f);
  void deliver_dels(Flight& f);
  void overflow_misses(Flight& f);
  void fail_flight(Flight& f);
  // `unlaunched`: the requests never reached the GPU (their SETs / DELETEs end here)
  void fail_requests(std::vector<Req>& reqs, bool unlaunched);
  void eject(const char* why);
  void maybe_restore();
  uint64_t migrate_from(Dev& src);
  void sweep();
  void finish_filter_rebuild();
  bool up() const { return (be->up_mask_.load(std::memory_order_acquire) >> index) & 1; }
  void set_up(bool on) {
    if (on) be->up_mask_.fetch_or(1ull << index);
    else be->up_mask_.fetch_and(~(1ull << index));
  }
  ~Dev() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& f : flights) {
      for (Mapped* m : {&f->keys, &f->offs, &f->set_keys, &f->set_vals, &f->set_voff,
                        &f->set_meta, &f->del_keys, &f->del_found})
        m->release();
      f->arena.reset();
      if (f->ev) (void)hipEventDestroy(f->ev);
    }
    direct_offs.release();
    for (DevBuf* b : {&hs_keys, &hs_loc, &hs_size, &hs_off, &hs_rec, &hf_keys, &hf_rec, &hf_off,
                      &hf_okeys, &hf_voff, &hf_meta})
      b->release();
    hf_size.release();
    cache.reset();
    if (stream) (void)hipStreamDestroy(stream);
    if (mstream) (void)hipStreamDestroy(mstream);
    if (sstream) (void)hipStreamDestroy(sstream);
    (void)hipFree(d_pts);
    (void)hipFree(d_own);
  }
};

// Host slots the edge GET signals completion through: one per flight.
constexpr int kFlightSlot0 = 8;

// A reactor's direct-submission context (one per attached reactor thread, used only by
// that thread): per GPU, the GETs it accepted this loop iteration and up to kDirectJobs
// edge-server jobs in flight, each answered from its own host slot and pinned arena.
struct HbmBackend::Direct {
  static constexpr int kOffWords = 32;  // >= kServeKeys + 1
  struct Job {
    int slot = -1;
    bool busy = false, answered = false;
    std::vector<Req> reqs;
    std::vector<uint32_t> urow;
    Digest keys[HbmCache::kServeKeys];
    size_t rows = 0;
    uint64_t* offs_h = nullptr;
    uint64_t* offs_d = nullptr;
    std::shared_ptr<ArenaPool::Arena> arena;
    uint32_t tnow = 0;
    double t0 = 0;
  };
  struct PerDev {
    std::vector<Req> pending;
    Job jobs[kDirectJobs];
    double avg_row_bytes = 4096;
  };
  int idx = 0;
  Executor* ex = nullptr;  // the attached reactor (null: context free)
  bool poisoned = false;   // a job never completed: the context is not reused
  std::vector<PerDev> dev;
};

namespace {
// The calling thread's direct context (set by direct_attach on a reactor thread).
struct DirectTls {
  HbmBackend* be = nullptr;
  HbmBackend::Direct* ctx = nullptr;
};
thread_local DirectTls tl_direct;

// Record [ItemHeader | u16 klen | key | payload] at base + o (sz bytes, 0 = miss) checked
// against the request's digest and key; a hit is a ByteRef slice that keeps `owner` alive.
bool read_hit(const uint8_t* base, uint64_t o, uint64_t sz, const Digest& d,
              const std::string& key, uint32_t tnow, const std::shared_ptr<const void>& owner,
              CacheValue* v, bool* mismatch) {
  if (!sz) return false;
  ItemHeader h;
  std::memcpy(&h, base + o, sizeof h);
  if (h.magic != kItemMagic || h.d0 != d.lo || h.d1 != d.hi) return false;
  size_t po = 0;
  const char* val = reinterpret_cast<const char*>(base + o + kItemHeaderBytes);
  if (!keyed_match(val, h.vlen, key, &po)) {
    *mismatch = true;  // digest collision
    return false;
  }
  v->flags = h.flags;
  v->ttl_left = h.expire ? (int64_t)h.expire - (int64_t)tnow : 0;
  v->data = ByteRef(owner, val + po, h.vlen - po);
  return true;
}
}  // namespace


HbmBackend::HbmBackend(const HbmBackendConfig& cfg)
    : cfg_(cfg), ring_((int)cfg.devices.size()), epoch_(wall_s()) {
  SH_CHECK(!cfg_.devices.empty() && cfg_.devices.size() <= 64, "HbmBackend needs 1..64 devices");
  SH_CHECK(cfg_.depth >= 1 && kFlightSlot0 + cfg_.depth <= kDirectSlot0,
           "pipeline depth out of range");
  static_assert(kDirectSlot0 + kDirectJobs * kDirectMax <= HbmCache::kHeadSlot,
                "direct host slots overlap the head slot");
  static_assert(Direct::kOffWords >= HbmCache::kServeKeys + 1, "direct offsets too short");
  SH_CHECK(cfg_.direct_backlog >= 1, "direct_backlog must be >= 1");
  wpend_.reset(new std::atomic<uint32_t>[kWpend]);
  for (size_t i = 0; i < kWpend; ++i) wpend_[i].store(0, std::memory_order_relaxed);
  for (size_t i = 0; i < cfg_.devices.size(); ++i) {
    auto d = std::make_unique<Dev>();
    d->be = this;
    d->index = (int)i;
    d->device = cfg_.devices[i];
    HB_OK(hipSetDevice(d->device));
    ShardConfig sc;
    sc.log_bytes = cfg_.log_bytes_per_gpu / 16 * 16;
    sc.nbuckets = cfg_.nbuckets_per_gpu;
    sc.max_item = cfg_.max_item + (uint32_t)keyed_size(kMaxKeyedKey, 0);
    sc.device = d->device;
    sc.evict = cfg_.evict;
    sc.serve_blocks = cfg_.serve_blocks;
    d->cache = std::make_unique<HbmCache>(sc);
    HB_OK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    HB_OK(hipStreamCreateWithFlags(&d->mstream, hipStreamNonBlocking));
    HB_OK(hipStreamCreateWithFlags(&d->sstream, hipStreamNonBlocking));
    {
      const auto& pts = ring_.points();
      std::vector<uint32_t> hp(pts.size());
      std::vector<int32_t> ho(pts.size());
      for (size_t k = 0; k < pts.size(); ++k) {
        hp[k] = pts[k].first;
        ho[k] = pts[k].second;
      }
      d->npts = (int)pts.size();
      HB_OK(hipMalloc(&d->d_pts, std::max<size_t>(1, hp.size()) * sizeof(uint32_t)));
      HB_OK(hipMalloc(&d->d_own, std::max<size_t>(1, ho.size()) * sizeof(int32_t)));
      HB_OK(hipMemcpy(d->d_pts, hp.data(), hp.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
      HB_OK(hipMemcpy(d->d_own, ho.data(), ho.size() * sizeof(int32_t), hipMemcpyHostToDevice));
      // a pageable-memory hipMemcpy may return before its DMA lands; the batcher's
      // non-blocking streams do not wait for the null stream
      HB_OK(hipDeviceSynchronize());
    }
    d->pool = std::make_shared<ArenaPool>(d->device);
    if (cfg_.arena_bytes) d->pool->reserve((size_t)cfg_.depth + 2, (size_t)cfg_.arena_bytes);
    if (cfg_.direct && cfg_.edge_server) {
      // reactors never allocate pinned memory: their arenas and offsets exist up front
      if (cfg_.direct_arenas > 0 && cfg_.direct_arena_bytes)
        d->pool->reserve((size_t)cfg_.direct_arenas, (size_t)cfg_.direct_arena_bytes);
      d->direct_offs.ensure((size_t)kDirectMax * kDirectJobs * Direct::kOffWords * 8);
    }
    for (int k = 0; k < cfg_.depth; ++k) {
      auto f = std::make_unique<Flight>();
      HB_OK(hipEventCreateWithFlags(&f->ev, hipEventDisableTiming));
      f->slot = kFlightSlot0 + k;
      f->keys.ensure(4096 * sizeof(Digest));
      f->offs.ensure(4097 * 8);
      d->flights.push_back(std::move(f));
    }
    d->cache->reserve(4096);
    if (cfg_.presence_filter) {
      // 16 bits per index slot (capped at 256 MiB): ~2 % false positives when a full
      // index's worth of digests has been added since the last rebuild
      const uint64_t slots = cfg_.nbuckets_per_gpu * kEntriesPerBucket;
      d->filt_bits = std::min<uint64_t>(slots * 16, 1ull << 31);
      d->filt_rebuild_at = slots;
      d->filt = std::make_shared<PresenceFilter>(d->filt_bits);
    }
    up_mask_.fetch_or(1ull << i);
    devs_.push_back(std::move(d));
  }
  if (cfg_.direct && cfg_.edge_server) {
    for (int c = 0; c < kDirectMax; ++c) {
      auto dc = std::make_unique<Direct>();
      dc->idx = c;
      dc->dev.resize(devs_.size());
      for (size_t k = 0; k < devs_.size(); ++k)
        for (int j = 0; j < kDirectJobs; ++j) {
          Direct::Job& jb = dc->dev[k].jobs[j];
          const size_t w = ((size_t)c * kDirectJobs + (size_t)j) * Direct::kOffWords;
          jb.slot = kDirectSlot0 + c * kDirectJobs + j;
          jb.offs_h = devs_[k]->direct_offs.host<uint64_t>() + w;
          jb.offs_d = devs_[k]->direct_offs.dev<uint64_t>() + w;
        }
      direct_.push_back(std::move(dc));
    }
  }
  // Peer access between the shards' GPUs (warm restore copies over xGMI). A pair the
  // runtime cannot map, or every pair under peer_copy = "staged", copies through pinned
  // host memory instead (peer_path / copy_between).
  const size_t nd = devs_.size();
  peer_ok_.assign(nd * nd, 0);
  if (cfg_.peer_copy != "staged") {
    for (size_t i = 0; i < nd; ++i)
      for (size_t j = 0; j < nd; ++j) {
        const int a = devs_[i]->device, b = devs_[j]->device;
        if (a == b) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, b, a) != hipSuccess || !can) continue;
        HB_OK(hipSetDevice(b));  // b (the destination) reads / DMAs from a's memory
        const hipError_t e = hipDeviceEnablePeerAccess(a, 0);
        if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) peer_ok_[i * nd + j] = 1;
        else (void)hipGetLastError();  // clear the sticky error: the pair stays staged
      }
  }
  if (devs_.size() > 1) {
    // DigestRing's points (tests check the owners agree), answered from the span table
    router_ = std::make_unique<HostRouter>((int)devs_.size());
    if (cfg_.hot_objects > 0 && cfg_.flush_on_restore) {
      SH_CHECK(cfg_.hot_sample >= 1 && (cfg_.hot_sample & (cfg_.hot_sample - 1)) == 0,
               "hot_sample must be a power of two");
      hot_on_ = true;
      samples_.reset(new SampleStripe[kSampleStripes]);
      hot_weights_.assign(devs_.size(), 1.0);
      spread_mask_.store(up_mask_.load());
    }
  }
  for (auto& d : devs_) {
    Dev* dp = d.get();
    dp->th = std::thread([dp] { dp->loop(); });
  }
  if (hot_on_ && cfg_.hot_refresh_ms > 0) hot_th_ = std::thread([this] { hot_loop(); });
}

HbmBackend::~HbmBackend() {
  {
    std::lock_guard<std::mutex> lk(hot_th_mu_);
    hot_stop_ = true;
  }
  hot_cv_.notify_all();
  if (hot_th_.joinable()) hot_th_.join();  // first: a refresh waits on the batchers
  for (auto& d : devs_) {
    {
      std::lock_guard<std::mutex> lk(d->mu);
      d->stop = true;
    }
    d->cv.notify_all();
  }
  for (auto& d : devs_)
    if (d->th.joinable()) d->th.join();
}

uint32_t HbmBackend::now() const { return (uint32_t)(wall_s() - epoch_) + 1; }

int HbmBackend::owner_of(const Digest& d, uint64_t up) const {
  if (devs_.size() == 1) return up & 1 ? 0 : -1;
  const uint64_t all = devs_.size() >= 64 ? ~0ull : (1ull << devs_.size()) - 1;
  if ((up & all) == all) return router_->owner(d);  // the span table: one load, two compares
  return ring_.owner(d, up);  // ketama ejection: the next live point
}

namespace {
thread_local uint64_t tl_spray_seq = 0;  // a reactor's stream position (sprayed objects)
thread_local uint32_t tl_sample_ctr = 0;
std::atomic<unsigned> g_sample_slot{0};
thread_local unsigned tl_sample_slot = g_sample_slot.fetch_add(1, std::memory_order_relaxed);
}  // namespace

int HbmBackend::route_get(const Digest& d) {
  const uint64_t up = up_mask_.load(std::memory_order_acquire);
  if (hot_on_) {
    if (((tl_sample_ctr++) & (uint32_t)(cfg_.hot_sample - 1)) == 0) sample_get(d);
    int r = -1;
    {
      const HostRouter::Read rd(*router_);
      const int hr = rd.hot_rank(d);
      if (hr != HostRouter::kNotHot) r = hr >= 0 ? hr : rd.spray(tl_spray_seq++);
    }
    if (r >= 0 && ((up & spread_mask_.load(std::memory_order_acquire)) >> r) & 1) {
      const int o = owner_of(d, up);
      if (r != o) hot_spread_gets_[tl_sample_slot % 16].v.fetch_add(1, std::memory_order_relaxed);
      return r;
    }
  }
  return owner_of(d, up);
}

void HbmBackend::sample_get(const Digest& d) {
  SampleStripe& st = samples_[tl_sample_slot % kSampleStripes];
  std::lock_guard<std::mutex> lk(st.mu);
  if (st.v.size() < (1u << 16)) st.v.push_back(d);  // bounded while no refresh drains it
}

void HbmBackend::enqueue(int k, Req r) {
  Dev& dv = *devs_[k];
  {
    std::lock_guard<std::mutex> lk(dv.mu);
    if (r.kind == 1 && cfg_.presence_filter) {
      dv.filt->add(r.d);
      if (dv.filt_next) dv.filt_next->add(r.d);
    }
    // a write of an object being filled into this shard: the fill must not overwrite it
    if ((r.kind == 1 || r.kind == 2) && !dv.filling.empty() && dv.filling.count(r.d.lo))
      dv.touched.insert(r.d.lo);
    dv.q.push_back(std::move(r));
    dv.qn.store(dv.q.size(), std::memory_order_release);
  }
  if (!dv.spinning.load(std::memory_order_acquire)) dv.cv.notify_one();
}

void HbmBackend::enqueue_many(int k, std::vector<Req>& rs) {
  if (rs.empty()) return;
  Dev& dv = *devs_[k];
  {
    std::lock_guard<std::mutex> lk(dv.mu);
    for (auto& r : rs) dv.q.push_back(std::move(r));  // GETs only: no filter update
    dv.qn.store(dv.q.size(), std::memory_order_release);
  }
  rs.clear();
  if (!dv.spinning.load(std::memory_order_acquire)) dv.cv.notify_one();
}

void HbmBackend::get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) {
  const int k = route_get(d);
  if (k < 0) {  // every shard ejected: the request falls through to the origin
    no_shard_misses_.fetch_add(1, std::memory_order_relaxed);
    done(false, CacheValue{});
    return;
  }
  Dev& dv = *devs_[k];
  if (devs_.size() > 1)
    dv.routed_gets[tl_sample_slot % Dev::kCtrShards].v.fetch_add(1, std::memory_order_relaxed);
  const bool restoring = dv.restoring.load(std::memory_order_acquire);
  if (cfg_.presence_filter && !restoring && !std::atomic_load(&dv.filt)->maybe(d)) {
    dv.filt_skips.fetch_add(1, std::memory_order_relaxed);  // never stored: no GPU batch
    done(false, CacheValue{});
    return;
  }
  Req r;
  r.kind = 0;
  r.d = d;
  r.key = key;
  r.ex = ex;
  r.gcb = std::move(done);
  // Reactor-direct: the calling reactor sends it to the edge server itself at the end of
  // its loop iteration (direct_service), unless a write or flush of this shard it must
  // stay ordered after has not finished on the GPU yet
  Direct* dc = tl_direct.be == this ? tl_direct.ctx : nullptr;
  if (dc && ex == dc->ex && !restoring && dv.flush_pend.load(std::memory_order_acquire) == 0 &&
      !writes_pending(d.lo)) {
    dc->dev[(size_t)k].pending.push_back(std::move(r));
    return;
  }
  enqueue(k, std::move(r));
}

void HbmBackend::set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
                     uint32_t ttl_s) {
  if (!value || value->size() > cfg_.max_item || key.size() > kMaxKeyedKey) return;
  Req r;
  r.kind = 1;
  r.d = d;
  r.key = key;
  r.value = std::move(value);
  r.flags = flags;
  r.ttl = ttl_s;
  if (!hot_on_) {
    const int k = owner_of(d, up_mask_.load(std::memory_order_acquire));
    if (k < 0) return;
    write_begin(d.lo);  // ends when its flight is reaped (or the request is failed)
    enqueue(k, std::move(r));
    return;
  }
  // held until every copy is queued: a refresh's set_hot returns only after this
  const HostRouter::Read rd(*router_);
  const uint64_t up = up_mask_.load(std::memory_order_acquire);
  const int o = owner_of(d, up);
  if (o < 0) return;
  const bool hot = rd.hot_rank(d) != HostRouter::kNotHot;
  write_begin(d.lo);
  if (!hot) {
    enqueue(o, std::move(r));
    return;
  }
  enqueue(o, r);  // write-through: the owner, then every other shard in service
  for (size_t k = 0; k < devs_.size(); ++k) {
    if ((int)k == o || !((up >> k) & 1)) continue;
    write_begin(d.lo);
    enqueue((int)k, r);
  }
}

void HbmBackend::del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) {
  Req r;
  r.kind = 2;
  r.d = d;
  r.key = key;
  r.ex = ex;
  std::unique_ptr<HostRouter::Read> rd;  // write-through: held until every copy is queued
  if (hot_on_) rd = std::make_unique<HostRouter::Read>(*router_);
  const uint64_t up = up_mask_.load(std::memory_order_acquire);
  const int k = owner_of(d, up);
  if (k < 0) {
    if (done) done(false);
    return;
  }
  std::vector<int> to{k};
  if (rd && rd->hot_rank(d) != HostRouter::kNotHot)
    for (size_t j = 0; j < devs_.size(); ++j)
      if ((int)j != k && ((up >> j) & 1)) to.push_back((int)j);
  if (to.size() == 1) {
    r.dcb = std::move(done);
    write_begin(d.lo);
    enqueue(k, std::move(r));
    return;
  }
  // one answer: found anywhere, once every copy is gone
  struct Fan {
    std::atomic<int> left;
    std::atomic<bool> found{false};
    DelCallback cb;
  };
  auto fan = std::make_shared<Fan>();
  fan->left.store((int)to.size());
  fan->cb = std::move(done);
  for (int j : to) {
    Req c = r;
    c.dcb = [fan](bool f) {
      if (f) fan->found.store(true, std::memory_order_relaxed);
      if (fan->left.fetch_sub(1, std::memory_order_acq_rel) == 1 && fan->cb)
        fan->cb(fan->found.load(std::memory_order_relaxed));
    };
    write_begin(d.lo);
    enqueue(j, std::move(c));
  }
}

void HbmBackend::enqueue_ctl(int k, std::function<void(bool)> cb) {
  Req r;
  r.kind = 3;
  r.d = Digest{0, 0};
  r.ccb = std::move(cb);
  enqueue(k, std::move(r));
}

void HbmBackend::flush() {
  for (auto& d : devs_) {
    {
      std::lock_guard<std::mutex> lk(d->mu);
      if (!d->flush_req) d->flush_pend.fetch_add(1, std::memory_order_acq_rel);
      d->flush_req = true;
      d->ctl_pending.store(true, std::memory_order_release);
    }
    d->cv.notify_one();
  }
}

bool HbmBackend::inject_shard_down(int shard, bool down) {
  if (shard < 0 || shard >= (int)devs_.size()) return false;
  Dev& dv = *devs_[shard];
  dv.forced_down.store(down, std::memory_order_release);
  if (down) {
    dv.eject_gen.fetch_add(1, std::memory_order_acq_rel);
    dv.set_up(false);
    spread_mask_.fetch_and(~(1ull << shard), std::memory_order_acq_rel);  // replicas suspect
    dv.ejections++;
  }
  {
    std::lock_guard<std::mutex> lk(dv.mu);
    dv.kick = true;
  }
  dv.cv.notify_one();  // the batcher restores the shard (flushing it) when forced_down clears
  return true;
}

// ---------------------------------------------------------------------------------
// reactor-direct submission: the reactor is its own batcher for
// small GET batches — it writes the edge-server job, polls the job's host slot in its
// loop and answers the requests inline. Replaces the reference's blocking mc.get inside
// the reactor (src/python/shellac/server/Server.py:335) without blocking.
// ---------------------------------------------------------------------------------
void HbmBackend::direct_attach(Executor* ex) {
  if (!ex || direct_.empty() || tl_direct.be == this) return;
  std::lock_guard<std::mutex> lk(direct_mu_);
  for (auto& dc : direct_)
    if (!dc->ex && !dc->poisoned) {
      dc->ex = ex;
      tl_direct = DirectTls{this, dc.get()};
      return;
    }
  // more reactors than contexts: the rest use the batcher
}

void HbmBackend::direct_submit(Direct& dc, size_t k) {
  Dev& dv = *devs_[k];
  Direct::PerDev& pd = dc.dev[k];
  std::vector<Req>& P = pd.pending;
  int free_job = -1;
  for (int j = 0; j < kDirectJobs && free_job < 0; ++j)
    if (!pd.jobs[j].busy) free_job = j;
  // distinct digests (at most kServeKeys: a bigger batch is the batcher's)
  size_t rows = 0;
  Digest keys[HbmCache::kServeKeys];
  std::vector<uint32_t> urow(P.size());
  bool small = true;
  for (size_t i = 0; i < P.size() && small; ++i) {
    size_t u = 0;
    while (u < rows && !(keys[u].lo == P[i].d.lo && keys[u].hi == P[i].d.hi)) ++u;
    if (u == rows) {
      if (rows == (size_t)HbmCache::kServeKeys) {
        small = false;
        break;
      }
      keys[rows++] = P[i].d;
    }
    urow[i] = (uint32_t)u;
  }
  // both jobs busy with a small batch pending: it goes out when one finishes (a few us)
  if (small && free_job < 0) return;
  bool ok = small && dv.up() && dv.flush_pend.load(std::memory_order_acquire) == 0 &&
            dv.cache->serve_backlog() <
                (uint64_t)cfg_.direct_backlog * (uint64_t)dv.cache->serve_blocks();
  Direct::Job* jb = ok ? &pd.jobs[free_job] : nullptr;
  if (ok) {
    jb->arena = dv.pool->try_take((size_t)(pd.avg_row_bytes * 1.5 * (double)rows) + (64u << 10));
    ok = jb->arena != nullptr;
  }
  if (ok) {
    jb->tnow = now();
    std::copy(keys, keys + rows, jb->keys);
    ok = dv.cache->serve_get(jb->keys, (int64_t)rows, jb->arena->d, jb->arena->cap, jb->offs_d,
                             jb->tnow, jb->slot);
    if (!ok) jb->arena.reset();
  }
  if (!ok) {
    dv.direct_fallbacks.fetch_add(P.size(), std::memory_order_relaxed);
    enqueue_many((int)k, P);
    return;
  }
  jb->rows = rows;
  jb->urow.swap(urow);
  jb->reqs.swap(P);
  P.clear();
  jb->busy = true;
  jb->answered = false;
  jb->t0 = wall_s();
  dv.direct_jobs.fetch_add(1, std::memory_order_relaxed);
  dv.direct_reqs.fetch_add(jb->reqs.size(), std::memory_order_relaxed);
  dv.coalesced.fetch_add(jb->reqs.size() - rows, std::memory_order_relaxed);
}

void HbmBackend::direct_reap(Direct& dc, size_t k, int j) {
  Dev& dv = *devs_[k];
  Direct::PerDev& pd = dc.dev[k];
  Direct::Job& jb = pd.jobs[j];
  const uint64_t total = dv.cache->host_slot(jb.slot);
  if (total == HbmCache::kSlotPending) {
    const double el = wall_s() - jb.t0;
    // the server may have exited (idle / lifetime) just before taking the job
    if (el > 20e-6) dv.cache->serve_kick();
    if (!jb.answered && el * 1e3 > cfg_.batch_timeout_ms) {
      // stalled: answer misses now; the job (arena, slot) stays reserved until it ends
      dv.direct_timeouts.fetch_add(1, std::memory_order_relaxed);
      std::vector<Req> rs;
      rs.swap(jb.reqs);
      jb.answered = true;
      for (auto& r : rs)
        if (r.gcb) r.gcb(false, CacheValue{});
    }
    return;
  }
  dv.direct_ns.fetch_add((uint64_t)((wall_s() - jb.t0) * 1e9), std::memory_order_relaxed);
  std::vector<Req> rs;
  rs.swap(jb.reqs);
  std::shared_ptr<ArenaPool::Arena> arena = std::move(jb.arena);
  const bool answered = jb.answered;
  jb.busy = false;
  jb.answered = false;
  if (answered) return;
  if (total == HbmCache::kSlotFailed) {
    for (auto& r : rs) r.gcb(false, CacheValue{});
    return;
  }
  if (jb.rows) pd.avg_row_bytes = 0.9 * pd.avg_row_bytes + 0.1 * ((double)total / (double)jb.rows);
  if (total > arena->cap) {  // the records did not fit (none written): the batcher regathers
    dv.direct_overflows.fetch_add(1, std::memory_order_relaxed);
    enqueue_many((int)k, rs);
    return;
  }
  // answers first, callbacks after: a callback may issue GETs of its own (into pending)
  std::shared_ptr<const void> owner = arena;
  struct Ans {
    bool hit;
    CacheValue v;
  };
  std::vector<Ans> ans(rs.size());
  for (size_t i = 0; i < rs.size(); ++i) {
    const uint32_t u = jb.urow[i];
    const uint64_t o = jb.offs_h[u], sz = jb.offs_h[u + 1] - o;
    bool mismatch = false;
    ans[i].hit = read_hit(arena->h, o, sz, jb.keys[u], rs[i].key, jb.tnow, owner, &ans[i].v,
                          &mismatch);
    if (mismatch) dv.key_mismatch.fetch_add(1, std::memory_order_relaxed);
  }
  for (size_t i = 0; i < rs.size(); ++i) {
    Req& r = rs[i];
    if (r.ex == dc.ex) r.gcb(ans[i].hit, std::move(ans[i].v));
    else if (r.ex) {
      auto cb = std::move(r.gcb);
      r.ex->post([cb = std::move(cb), a = std::move(ans[i])]() mutable { cb(a.hit, std::move(a.v)); });
    } else {
      r.gcb(ans[i].hit, std::move(ans[i].v));
    }
  }
}

bool HbmBackend::direct_service() {
  Direct* dc = tl_direct.be == this ? tl_direct.ctx : nullptr;
  if (!dc) return false;
  bool busy = false;
  for (size_t k = 0; k < devs_.size(); ++k) {
    Direct::PerDev& pd = dc->dev[k];
    for (int j = 0; j < kDirectJobs; ++j)
      if (pd.jobs[j].busy) direct_reap(*dc, k, j);
    if (!pd.pending.empty()) direct_submit(*dc, k);
    for (int j = 0; j < kDirectJobs; ++j) busy |= pd.jobs[j].busy;
    busy |= !pd.pending.empty();
  }
  return busy;
}

void HbmBackend::direct_detach() {
  Direct* dc = tl_direct.be == this ? tl_direct.ctx : nullptr;
  if (!dc) return;
  for (size_t k = 0; k < devs_.size(); ++k) enqueue_many((int)k, dc->dev[k].pending);
  const double until = wall_s() + cfg_.batch_timeout_ms * 1e-3 + 1.0;
  for (;;) {
    bool busy = false;
    for (size_t k = 0; k < devs_.size(); ++k)
      for (int j = 0; j < kDirectJobs; ++j)
        if (dc->dev[k].jobs[j].busy) {
          direct_reap(*dc, k, j);
          busy |= dc->dev[k].jobs[j].busy;
        }
    if (!busy) break;
    if (wall_s() > until) {
      dc->poisoned = true;  // a job never finished: its arena / slot stay reserved
      break;
    }
    __builtin_ia32_pause();
  }
  tl_direct = DirectTls{};
  std::lock_guard<std::mutex> lk(direct_mu_);
  dc->ex = nullptr;
}

// ---------------------------------------------------------------------------------
// batcher
// ---------------------------------------------------------------------------------
bool HbmBackend::Dev::take_batch(std::vector<Req>* out, bool* do_flush, bool* rebuilding) {
  std::unique_lock<std::mutex> lk(mu);
  ctl_pending.store(false, std::memory_order_relaxed);
  if (q.empty() && !flush_req && !filt_want_rebuild) return false;
  const HbmBackendConfig& cfg = be->cfg_;
  if (cfg.batch_us > 0 && (int)q.size() < cfg.max_batch) {
    // optional linger: trade latency for bigger batches
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(cfg.batch_us);
    while (!stop && (int)q.size() < cfg.max_batch &&
           cv.wait_until(lk, deadline) != std::cv_status::timeout) {
    }
  }
  if (filt_want_rebuild) {
    // SETs queued from here on add to filt_next; the ones already queued are in this
    // batch and committed before finish_filter_rebuild() exports the shard's keys
    filt_next = std::make_shared<PresenceFilter>(filt_bits);
    filt_want_rebuild = false;
    *rebuilding = true;
  }
  // A flight runs its GETs before its SETs / DELETEs, so a GET queued behind a write of
  // the same key ends the batch: it goes into the next flight, which is ordered after this
  // one (read-your-writes for a client that re-reads right after a fill; seen as a second
  // origin fetch in test_proxy_reactor_direct_gets when the reactor's GET reached the queue
  // before the batcher took the SET)
  size_t take = std::min(q.size(), (size_t)std::max(cfg.max_batch, 1));
  {
    std::unordered_set<uint64_t>& w = take_wset;
    w.clear();
    for (size_t i = 0; i < take; ++i) {
      const Req& r = q[i];
      if (r.kind == 1 || r.kind == 2) {
        w.insert(r.d.lo);
      } else if (r.kind == 4) {  // a fill ends its flight (it runs after the flight's writes)
        take = i + 1;
        break;
      } else if (r.kind == 0 && !w.empty() && w.count(r.d.lo)) {
        take = i;
        break;
      }
    }
  }
  if (take == q.size()) {
    out->swap(q);
  } else {
    out->assign(std::make_move_iterator(q.begin()), std::make_move_iterator(q.begin() + take));
    q.erase(q.begin(), q.begin() + take);
  }
  qn.store(q.size(), std::memory_order_release);
  *do_flush = flush_req;
  flush_req = false;
  return true;
}

void HbmBackend::Dev::loop() {
  const HbmBackendConfig& cfg = be->cfg_;
  (void)hipSetDevice(device);
  const std::string nm = "shellac-hbm" + std::to_string(device);
  pthread_setname_np(pthread_self(), nm.c_str());
  if (!cfg.batcher_cpus.empty()) {  // a core of its own: it spins on the queue and the GPU
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cfg.batcher_cpus[(size_t)index % cfg.batcher_cpus.size()], &set);
    (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
  }
  std::vector<Req> batch;
  for (;;) {
    bool worked = false;
    // 1. reap the oldest flight (in launch order) once its completion signal fired
    if (inflight) {
      Flight& f = *flights[head];
      bool freed = false;
      try {
        freed = try_reap(f, false);
      } catch (const std::exception& e) {
        std::fprintf(stderr, "[shellac hbm] gpu %d batch failed: %s\n", device, e.what());
        fail_flight(f);
        eject("batch error");
        freed = true;
      }
      if (!freed && f.active && (wall_s() - f.t0) * 1e3 > cfg.batch_timeout_ms) {
        std::fprintf(stderr, "[shellac hbm] gpu %d batch stalled for %d ms\n", device,
                     cfg.batch_timeout_ms);
        fail_flight(f);  // answered as misses; the flight stays busy until the GPU finishes
        eject("stall");
      }
      if (freed) {
        track_writes(f, -1);
        head = (head + 1) % flights.size();
        --inflight;
        worked = true;
      }
    }
    // 2. launch the queued requests as a new flight
    if (inflight < flights.size() &&
        (qn.load(std::memory_order_acquire) || ctl_pending.load(std::memory_order_acquire))) {
      bool do_flush = false, rebuilding = false;
      batch.clear();
      if (take_batch(&batch, &do_flush, &rebuilding)) {
        worked = true;
        if (!up() || failed) {
          fail_requests(batch, true);
          if (do_flush) flush_done();
        } else if (batch.empty()) {
          try {
            // finished before anything else may read the shard: edge-server GETs are not
            // ordered after the stream
            if (do_flush) {
              cache->flush(stream);
              HB_OK(hipStreamSynchronize(stream));
            }
          } catch (const std::exception& e) {
            std::fprintf(stderr, "[shellac hbm] gpu %d flush failed: %s\n", device, e.what());
          }
          if (do_flush) flush_done();
        } else {
          Flight& f = *flights[(head + inflight) % flights.size()];
          f.reqs.swap(batch);
          try {
            if (do_flush) cache->flush(stream);
            f.flush = do_flush;
            launch(f);
            track_writes(f, +1);
            ++inflight;
          } catch (const std::exception& e) {
            std::fprintf(stderr, "[shellac hbm] gpu %d launch failed: %s\n", device, e.what());
            fail_requests(f.reqs, true);
            if (do_flush) flush_done();
            f.flush = false;
            f.reqs.clear();
            f.active = false;
            eject("launch error");
          }
        }
        if (rebuilding) {
          try {
            finish_filter_rebuild();  // export_keys runs after the batch on the stream
          } catch (const std::exception& e) {
            std::fprintf(stderr, "[shellac hbm] presence filter rebuild failed: %s\n", e.what());
            std::lock_guard<std::mutex> lk(mu);
            filt_next.reset();
          }
        } else if (cfg.presence_filter && filt->adds() >= filt_rebuild_at) {
          std::lock_guard<std::mutex> lk(mu);
          filt_want_rebuild = true;
          ctl_pending.store(true, std::memory_order_release);
        }
      }
    }
    if (worked) continue;
    if (inflight) {  // waiting on the GPU: poll (the edge GET signals through host memory)
      if (up()) __builtin_ia32_pause();
      else std::this_thread::sleep_for(std::chrono::microseconds(200));  // ejected, draining
      continue;
    }
    // 3. idle
    if (!up()) maybe_restore();
    if (cfg.spin_us > 0 && qn.load(std::memory_order_acquire) == 0) {
      // poll for up to spin_us before blocking: under steady traffic the next request
      // usually arrives within that window, and catching it saves a futex wake-up
      spinning.store(true, std::memory_order_release);
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(cfg.spin_us);
      while (qn.load(std::memory_order_acquire) == 0 && std::chrono::steady_clock::now() < until)
        __builtin_ia32_pause();
      spinning.store(false, std::memory_order_release);
    }
    std::unique_lock<std::mutex> lk(mu);
    if (stop && q.empty()) return;
    if (!q.empty() || flush_req || filt_want_rebuild || kick) {
      kick = false;
      continue;
    }
    const auto wake = [&] { return stop || !q.empty() || flush_req || filt_want_rebuild || kick; };
    const int wait_s = !up() ? 1 : cfg.sweep_interval_s;
    if (wait_s > 0) {
      if (!cv.wait_for(lk, std::chrono::seconds(wait_s), wake) && up() && cfg.sweep_interval_s > 0) {
        // idle: expire TTL'd objects out of the index now and then
        lk.unlock();
        try {
          sweep();
        } catch (const std::exception& e) {
          std::fprintf(stderr, "[shellac hbm] sweep failed: %s\n", e.what());
        }
      }
    } else {
      cv.wait(lk, wake);
    }
  }
}

void HbmBackend::Dev::launch(Flight& f) {
  TraceRange tr("hbm_backend.launch");
  f.gets.clear();
  f.sets.clear();
  f.dels.clear();
  f.ctls.clear();
  for (uint32_t i = 0; i < f.reqs.size(); ++i) {
    const int kd = f.reqs[i].kind;
    (kd == 0 ? f.gets : kd == 1 ? f.sets : kd == 2 ? f.dels : f.ctls).push_back(i);
  }
  f.tnow = be->now();
  f.t0 = wall_s();
  f.got = f.gets.empty();
  f.active = true;
  f.served = false;
  // ---- GET: coalesce equal digests on the host (a hot object under concurrent clients
  // is one GPU row and one arena record, shared by its requests), then one edge-GET
  // launch: keys and offsets in mapped memory, records straight into a pinned arena
  const size_t n0 = f.gets.size();
  f.rows = 0;
  if (n0) {
    size_t tsz = 16;
    while (tsz < 2 * n0) tsz <<= 1;
    co_tab.assign(tsz, -1);
    f.urow.resize(n0);
    f.keys.ensure(n0 * sizeof(Digest));
    Digest* hk = f.keys.host<Digest>();
    for (size_t j = 0; j < n0; ++j) {
      const Digest& d = f.reqs[f.gets[j]].d;
      for (size_t h = (size_t)(d.hi ^ (d.hi >> 31)) & (tsz - 1);; h = (h + 1) & (tsz - 1)) {
        const int32_t u = co_tab[h];
        if (u < 0) {
          co_tab[h] = (int32_t)f.rows;
          hk[f.rows] = d;
          f.urow[j] = (uint32_t)f.rows++;
          break;
        }
        if (hk[u].lo == d.lo && hk[u].hi == d.hi) {
          f.urow[j] = (uint32_t)u;
          break;
        }
      }
    }
    coalesced += n0 - f.rows;
    f.offs.ensure((f.rows + 1) * 8);
    // arena sized from the running average record size (regathered if it falls short)
    const size_t want = (size_t)(avg_row_bytes * 1.5 * (double)f.rows) + (64u << 10);
    f.arena = pool->take(want);
    // small batches go to the resident edge server unless they must stay ordered after a
    // SET / DELETE / flush still in flight (read-your-writes for memcached clients)
    bool ordered = pend_flush > 0 || f.flush;
    for (size_t u = 0; !ordered && !pend_w.empty() && u < f.rows; ++u)
      ordered = pend_w.count(hk[u].lo) != 0;
    if (ordered) ordered_gets++;
    // ... and only while fewer than serve_backlog jobs are ahead of it: the server takes
    // one job at a time, so under load (several batches in flight) the launched path's
    // many workgroups win (profiles/archive/r3_http: c=1000 with every small batch served 0.95M
    // RPS, launched only 1.13M)
    f.served = be->cfg_.edge_server && !ordered && f.rows <= (size_t)HbmCache::kServeKeys &&
               cache->serve_backlog() <
                   (uint64_t)be->cfg_.serve_backlog * (uint64_t)cache->serve_blocks() &&
               cache->serve_get(hk, (int64_t)f.rows, f.arena->d, f.arena->cap,
                                f.offs.dev<uint64_t>(), f.tnow, f.slot);
    if (f.served) served_batches++;
    else
      cache->small_get(f.keys.dev<Digest>(), (int64_t)f.rows, f.arena->d, f.arena->cap,
                       f.offs.dev<uint64_t>(), f.tnow, stream, f.slot);
  }
  // ---- SET: [klen | key | payload] values packed into mapped staging the SET kernels
  // read directly (no copies), exact log-bytes bound
  const size_t ns = f.sets.size();
  if (ns) {
    f.set_keys.ensure(ns * sizeof(Digest));
    f.set_voff.ensure(ns * 8);
    f.set_meta.ensure(ns * 12);
    size_t bytes = 16;
    for (uint32_t i : f.sets)
      bytes += align_up(keyed_size(f.reqs[i].key.size(), f.reqs[i].value->size()), 16);
    f.set_vals.ensure(bytes);
    Digest* kk = f.set_keys.host<Digest>();
    uint64_t* vo = f.set_voff.host<uint64_t>();
    uint32_t* vl = f.set_meta.host<uint32_t>();
    uint32_t* fl = vl + ns;
    uint32_t* ex = vl + 2 * ns;
    uint64_t off = 0, bound = 0;
    for (size_t j = 0; j < ns; ++j) {
      const Req& r = f.reqs[f.sets[j]];
      const size_t sz = keyed_size(r.key.size(), r.value->size());
      write_keyed(f.set_vals.host<uint8_t>() + off, r.key, r.value->data(), r.value->size());
      kk[j] = r.d;
      vo[j] = off;
      vl[j] = (uint32_t)sz;
      fl[j] = r.flags;
      ex[j] = r.ttl ? f.tnow + r.ttl : 0;
      off += align_up(sz, 16);
      bound += item_bytes((uint32_t)sz);
    }
    cache->store(f.set_keys.dev<Digest>(), f.set_vals.dev<uint8_t>(),
                 f.set_voff.dev<uint64_t>(), f.set_meta.dev<uint32_t>(),
                 f.set_meta.dev<uint32_t>() + ns, f.set_meta.dev<uint32_t>() + 2 * ns,
                 (int64_t)ns, bound, f.tnow, stream);
    for (uint32_t i : f.sets) f.reqs[i].value = Bytes();  // staged: drop the reference
  }
  // ---- DELETE: keys and found flags in mapped memory
  const size_t nd = f.dels.size();
  if (nd) {
    f.del_keys.ensure(nd * sizeof(Digest));
    f.del_found.ensure(nd);
    for (size_t j = 0; j < nd; ++j) f.del_keys.host<Digest>()[j] = f.reqs[f.dels[j]].d;
    cache->remove(f.del_keys.dev<Digest>(), (int64_t)nd, f.del_found.dev<uint8_t>(), f.tnow,
                  stream);
  }
  // ---- hot-replica fills (last in the flight: every write queued before them ran first)
  for (uint32_t i : f.ctls) {
    if (f.reqs[i].kind != 4) continue;
    HotFill& h = *f.reqs[i].fill;
    {
      std::lock_guard<std::mutex> lk(mu);
      if (h.cancelled) continue;  // the refresh gave up on this shard
      h.launched = true;
      for (int64_t j = 0; j < h.m; ++j)
        if (h.hsize[j] && touched.count(h.lo[(size_t)j])) {
          h.hsize[j] = 0;  // a newer write-through copy is (or will be) here
          ++h.skipped;
        } else if (h.hsize[j]) {
          ++h.rows;
        }
    }
    records_to_set(h.krec, h.koff, h.dsize, nullptr, h.m, h.okeys, h.ovoff, h.ometa,
                   h.ometa + h.m, h.ometa + 2 * h.m, stream);
    cache->store(h.okeys, h.krec, h.ovoff, h.ometa, h.ometa + h.m, h.ometa + 2 * h.m, h.m,
                 h.bound, f.tnow, stream);
  }
  HB_OK(hipEventRecord(f.ev, stream));
  batches++;
  batched_reqs += f.reqs.size();
  uint64_t prev = max_batch.load();
  while (f.reqs.size() > prev && !max_batch.compare_exchange_weak(prev, f.reqs.size())) {
  }
}

// Completion of flight f (non-blocking unless `block`): GET results as soon as the edge
// GET's slot fires, DELETE results and the flight's buffers once its event completes.
bool HbmBackend::Dev::try_reap(Flight& f, bool block) {
  if (!f.got && f.active) {
    const uint64_t total = block ? cache->wait_host_slot(f.slot, be->cfg_.batch_timeout_ms)
                                 : cache->host_slot(f.slot);
    if (total == HbmCache::kSlotPending) {
      if (f.served) cache->serve_kick();  // relaunch the server if it exited meanwhile
      return false;
    }
    if (total == HbmCache::kSlotFailed) throw Error("edge GET reported a failed look-back");
    if (f.rows) avg_row_bytes = 0.9 * avg_row_bytes + 0.1 * ((double)total / (double)f.rows);
    if (total > f.arena->cap) {
      // Rare: the records outgrew the arena (the kernel wrote none of them). A second
      // lookup sees exactly the first one's state only when nothing has run since: no
      // SET/DELETE in this flight and no later flight queued on the stream. Otherwise the
      // GETs answer "miss" (always a valid cache answer: the proxy goes to the origin);
      // reading a newer state would reorder them after later SETs.
      if (f.sets.empty() && f.dels.empty() && inflight == 1) {
        regathers++;
        HB_OK(hipEventSynchronize(f.ev));
        f.arena = pool->take(total + (64u << 10));
        cache->small_get(f.keys.dev<Digest>(), (int64_t)f.rows, f.arena->d, f.arena->cap,
                         f.offs.dev<uint64_t>(), f.tnow, stream, f.slot);
        HB_OK(hipEventRecord(f.ev, stream));
        const uint64_t t2 = cache->wait_host_slot(f.slot, be->cfg_.batch_timeout_ms);
        if (t2 == HbmCache::kSlotPending || t2 == HbmCache::kSlotFailed)
          throw Error("edge GET regather failed");
        if (t2 > f.arena->cap) overflow_misses(f);  // cannot happen: state unchanged
        else deliver_gets(f);
      } else {
        overflow_misses(f);
      }
    } else {
      deliver_gets(f);
    }
    f.got = true;
  }
  if (block) {
    HB_OK(hipEventSynchronize(f.ev));
  } else {
    const hipError_t e = hipEventQuery(f.ev);
    if (e == hipErrorNotReady) return false;
    HB_OK(e);
  }
  if (f.active) {
    deliver_dels(f);
    for (uint32_t i : f.ctls)
      if (f.reqs[i].ccb) f.reqs[i].ccb(true);
    batch_ns += (uint64_t)((wall_s() - f.t0) * 1e9);
  }
  f.active = false;
  f.reqs.clear();
  f.arena.reset();  // hits hold their own references
  return true;
}

// dir = +1 when flight f launches, -1 when it is freed: its SET / DELETE digests and
// its flush count as in flight until then.
void HbmBackend::Dev::track_writes(const Flight& f, int dir) {
  Flight& m = const_cast<Flight&>(f);
  if (dir > 0) {
    m.wkeys.clear();
    for (uint32_t i : f.sets) m.wkeys.push_back(f.reqs[i].d.lo);
    for (uint32_t i : f.dels) m.wkeys.push_back(f.reqs[i].d.lo);
    for (uint64_t k : m.wkeys) ++pend_w[k];
    if (f.flush) ++pend_flush;
    return;
  }
  for (uint64_t k : m.wkeys) {
    auto it = pend_w.find(k);
    if (it != pend_w.end() && --it->second == 0) pend_w.erase(it);
    be->write_end(k);
  }
  m.wkeys.clear();
  if (m.flush) {
    if (pend_flush) --pend_flush;
    flush_done();
  }
  m.flush = false;
}

// Group completions per executor: one post_batch (one lock, one wake-up) per reactor.
namespace {
struct PostGroups {
  std::vector<std::pair<Executor*, std::vector<std::function<void()>>>> g;
  std::vector<std::function<void()>>& at(Executor* ex) {
    for (auto& p : g)
      if (p.first == ex) return p.second;
    g.emplace_back(ex, std::vector<std::function<void()>>{});
    return g.back().second;
  }
  void flush() {
    for (auto& p : g) p.first->post_batch(p.second);
    g.clear();
  }
};
}  // namespace

void HbmBackend::Dev::deliver_gets(Flight& f) {
  if (f.gets.empty()) return;
  const uint64_t* off = f.offs.host<uint64_t>();
  const Digest* hk = f.keys.host<Digest>();
  const uint8_t* base = f.arena->h;
  // the arena stays alive while any response built from it does
  std::shared_ptr<const void> owner = f.arena;
  PostGroups pg;
  for (size_t j = 0; j < f.gets.size(); ++j) {
    Req& r = f.reqs[f.gets[j]];
    const uint32_t u = f.urow[j];
    const uint64_t o = off[u], sz = off[u + 1] - o;
    CacheValue v;
    bool mismatch = false;
    const bool hit = read_hit(base, o, sz, hk[u], r.key, f.tnow, owner, &v, &mismatch);
    if (mismatch) key_mismatch.fetch_add(1, std::memory_order_relaxed);
    auto cb = std::move(r.gcb);
    if (r.ex)
      pg.at(r.ex).push_back([cb = std::move(cb), hit, v = std::move(v)]() { cb(hit, v); });
    else
      cb(hit, std::move(v));
  }
  pg.flush();
}

// Every GET of flight f answers "miss" (its records did not fit the arena).
void HbmBackend::Dev::overflow_misses(Flight& f) {
  arena_misses += f.gets.size();
  std::vector<Req> gets;
  for (uint32_t i : f.gets) gets.push_back(std::move(f.reqs[i]));
  fail_requests(gets, false);
}

void HbmBackend::Dev::deliver_dels(Flight& f) {
  if (f.dels.empty()) return;
  PostGroups pg;
  for (size_t j = 0; j < f.dels.size(); ++j) {
    Req& r = f.reqs[f.dels[j]];
    const bool found = f.del_found.host<uint8_t>()[j] != 0;
    auto cb = std::move(r.dcb);
    if (!cb) continue;
    if (r.ex)
      pg.at(r.ex).push_back([cb = std::move(cb), found]() { cb(found); });
    else
      cb(found);
  }
  pg.flush();
}

void HbmBackend::Dev::fail_requests(std::vector<Req>& reqs, bool unlaunched) {
  PostGroups pg;
  for (auto& r : reqs) {
    if (unlaunched && (r.kind == 1 || r.kind == 2)) be->write_end(r.d.lo);
    if (r.kind >= 3) {
      if (r.ccb) r.ccb(false);
      r.ccb = nullptr;
    } else if (r.kind == 0 && r.gcb) {
      auto cb = std::move(r.gcb);
      if (r.ex) pg.at(r.ex).push_back([cb = std::move(cb)]() { cb(false, CacheValue{}); });
      else cb(false, CacheValue{});
    } else if (r.kind == 2 && r.dcb) {
      auto cb = std::move(r.dcb);
      if (r.ex) pg.at(r.ex).push_back([cb = std::move(cb)]() { cb(false); });
      else cb(false);
    } else if (r.kind == 1) {
      dropped++;
    }
  }
  pg.flush();
}

// A failed or stalled flight: its requests are answered (GET miss, DEL not found), the
// flight itself stays reserved until the GPU finishes with its buffers.
void HbmBackend::Dev::fail_flight(Flight& f) {
  failures++;
  if (!f.got) {
    fail_requests(f.reqs, false);
  } else {
    std::vector<Req> rest;
    for (uint32_t i : f.dels) rest.push_back(std::move(f.reqs[i]));
    for (uint32_t i : f.ctls) rest.push_back(std::move(f.reqs[i]));
    fail_requests(rest, false);
  }
  f.got = true;
  f.gets.clear();
  f.dels.clear();
  f.ctls.clear();
  f.active = false;
}

void HbmBackend::Dev::eject(const char* why) {
  if (up()) {
    std::fprintf(stderr, "[shellac hbm] ejecting gpu %d (%s); retry in %d s\n", device, why,
                 be->cfg_.retry_s);
    ejections++;
  }
  failed = true;
  retry_at = wall_s() + be->cfg_.retry_s;
  eject_gen.fetch_add(1, std::memory_order_acq_rel);
  set_up(false);
  be->spread_mask_.fetch_and(~(1ull << index), std::memory_order_acq_rel);
  std::vector<Req> pending;
  {
    std::lock_guard<std::mutex> lk(mu);
    pending.swap(q);
    qn.store(0, std::memory_order_release);
  }
  fail_requests(pending, true);
}

// Bring an ejected shard back: the fault drill was lifted, or retry_s passed and every
// flight has completed (the GPU answers again). Its contents may be stale (SETs routed
// elsewhere while it was out), so it is flushed unless configured otherwise.
void HbmBackend::Dev::maybe_restore() {
  if (forced_down.load(std::memory_order_acquire)) return;
  if (failed && wall_s() < retry_at) return;
  try {
    for (auto& f : flights) HB_OK(hipEventSynchronize(f->ev));
    if (be->cfg_.flush_on_restore) cache->flush(stream);
    HB_OK(hipStreamSynchronize(stream));
  } catch (const std::exception&) {
    retry_at = wall_s() + be->cfg_.retry_s;
    return;
  }
  failed = false;
  for (size_t i = 0; i < inflight; ++i)  // every flight has finished: its writes end
    track_writes(*flights[(head + i) % flights.size()], -1);
  inflight = 0;
  head = 0;
  pend_w.clear();
  pend_flush = 0;
  for (auto& f : flights) {
    f->active = false;
    f->reqs.clear();
    f->arena.reset();
  }
  restores++;
  // Back in the ring first, then warm: objects of this shard's key range that its peers
  // took while it was out are copied back GPU-to-GPU, inserted only where this shard has
  // nothing yet — so a SET that reaches it from now on is never overwritten by an older
  // migrated copy (requests queued meanwhile run after the migration, on this thread).
  restoring.store(true, std::memory_order_release);
  set_up(true);
  uint64_t moved = 0;
  if (be->cfg_.warm_restore && be->cfg_.flush_on_restore) {
    for (auto& other : be->devs_) {
      if (other.get() == this || !other->up()) continue;
      try {
        moved += migrate_from(*other);
      } catch (const std::exception& e) {
        std::fprintf(stderr, "[shellac hbm] warm restore from gpu %d failed: %s\n",
                     other->device, e.what());
      }
    }
  }
  restoring.store(false, std::memory_order_release);
  std::fprintf(stderr, "[shellac hbm] gpu %d back in service (%llu objects warmed from peers)\n",
               device, (unsigned long long)moved);
}

int HbmBackend::peer_path(int src_dev, int dst_dev) const {
  if (cfg_.peer_copy == "staged") return 2;  // forced (tests run it with one GPU)
  if (src_dev == dst_dev) return 0;
  const size_t nd = devs_.size();
  size_t si = nd, di = nd;
  for (size_t i = 0; i < nd; ++i) {
    if (devs_[i]->device == src_dev) si = i;
    if (devs_[i]->device == dst_dev) di = i;
  }
  return si < nd && di < nd && peer_ok_[si * nd + di] ? 1 : 2;
}

namespace {
// src (on src_dev) -> dst (on dst_dev), ordered on `stream` (dst_dev's): a device copy on
// one GPU, a direct peer DMA where peer access is enabled, else staged through pinned
// host memory in 64 MiB pieces (synchronous; the warm restore is off the request path).
void copy_between(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes,
                  hipStream_t stream, int path) {
  if (!bytes) return;
  if (path == 0) {
    HB_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream));
  } else if (path == 1) {
    HB_OK(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, stream));
  } else {
    const size_t piece = std::min<size_t>(bytes, 64u << 20);
    void* h = nullptr;
    HB_OK(hipHostMalloc(&h, piece, hipHostMallocDefault));
    try {
      HB_OK(hipStreamSynchronize(stream));  // earlier work on dst's stream first
      for (size_t o = 0; o < bytes; o += piece) {
        const size_t n = std::min(piece, bytes - o);
        HB_OK(hipSetDevice(src_dev));
        HB_OK(hipMemcpy(h, static_cast<const uint8_t*>(src) + o, n, hipMemcpyDeviceToHost));
        HB_OK(hipSetDevice(dst_dev));
        HB_OK(hipMemcpy(static_cast<uint8_t*>(dst) + o, h, n, hipMemcpyHostToDevice));
      }
    } catch (...) {
      (void)hipHostFree(h);
      throw;
    }
    HB_OK(hipHostFree(h));
  }
}
}  // namespace

// Peer migration src -> this (both GPUs' HbmCache APIs are thread-safe; src's work goes
// on src's migration stream, beside src's own batcher): export src's live digests, route
// them on src's GPU, take the ones this shard owns, look them up and gather their records
// on src, hipMemcpyPeerAsync the records to this GPU, turn them into a SET batch
// (insert-if-absent against this shard's own lookup) and store them; finally delete them
// from src, where nothing routes any more. Chunked so a store stays within half a log.
uint64_t HbmBackend::Dev::migrate_from(Dev& src) {
  TraceRange tr("hbm_backend.migrate");
  const double t0 = wall_s();
  const uint32_t t = be->now();
  const int W = (int)be->devs_.size();
  // ---- on src: live digests and their owners under the full ring
  HB_OK(hipSetDevice(src.device));
  const uint64_t live = src.cache->export_keys(nullptr, 0, t, src.mstream);
  if (!live) {
    HB_OK(hipSetDevice(device));
    return 0;
  }
  Digest* s_keys = nullptr;
  int32_t* s_dest = nullptr;
  int64_t* s_cnt = nullptr;
  HB_OK(hipMalloc(&s_keys, live * sizeof(Digest)));
  HB_OK(hipMalloc(&s_dest, live * sizeof(int32_t)));
  HB_OK(hipMalloc(&s_cnt, W * sizeof(int64_t)));
  std::vector<int32_t> dest;
  std::vector<Digest> keys;
  uint64_t got = 0;
  try {
    got = std::min(live, src.cache->export_keys(s_keys, live, t, src.mstream));
    HB_OK(hipMemsetAsync(s_cnt, 0, W * sizeof(int64_t), src.mstream));
    route_keys(s_keys, (int64_t)got, src.d_pts, src.d_own, src.npts, s_dest, s_cnt, W,
               src.mstream);
    dest.resize(got);
    keys.resize(got);
    HB_OK(hipMemcpyAsync(dest.data(), s_dest, got * sizeof(int32_t), hipMemcpyDeviceToHost,
                         src.mstream));
    HB_OK(hipMemcpyAsync(keys.data(), s_keys, got * sizeof(Digest), hipMemcpyDeviceToHost,
                         src.mstream));
    HB_OK(hipStreamSynchronize(src.mstream));
  } catch (...) {
    (void)hipFree(s_keys); (void)hipFree(s_dest); (void)hipFree(s_cnt);
    throw;
  }
  (void)hipFree(s_dest);
  (void)hipFree(s_cnt);
  std::vector<Digest> mine;
  for (uint64_t i = 0; i < got; ++i)
    if (dest[i] == index) mine.push_back(keys[i]);
  (void)hipFree(s_keys);
  if (be->hot_on_ && !mine.empty()) {
    // hot objects stay where they are: the peers hold write-through replicas (they keep
    // serving the GETs spread to them), and this shard receives the whole hot set from the
    // next refresh's heal fill before it rejoins the spread mask
    const HostRouter::Read rd(*be->router_);
    mine.erase(std::remove_if(mine.begin(), mine.end(),
                              [&](const Digest& d) { return rd.hot_rank(d) != HostRouter::kNotHot; }),
               mine.end());
  }
  if (be->cfg_.presence_filter && !mine.empty()) {  // GETs routed here must not skip them
    std::lock_guard<std::mutex> lk(mu);
    for (const Digest& d : mine) {
      filt->add(d);
      if (filt_next) filt_next->add(d);
    }
  }
  uint64_t moved = 0;
  const uint64_t rec_cap = std::max<uint64_t>(cache->config().log_bytes / 8, 1u << 20);
  const size_t chunk = 65536;
  for (size_t c0 = 0; c0 < mine.size(); c0 += chunk) {
    const int64_t m = (int64_t)std::min(chunk, mine.size() - c0);
    // ---- on src: look the chunk up (misses the tail the next appends will overwrite)
    HB_OK(hipSetDevice(src.device));
    Digest* sk = nullptr;
    uint64_t *sloc = nullptr, *ssize = nullptr, *soff = nullptr;
    uint8_t* srec = nullptr;
    HB_OK(hipMalloc(&sk, m * sizeof(Digest)));
    HB_OK(hipMalloc(&sloc, m * 8));
    HB_OK(hipMalloc(&ssize, (m + 1) * 8));
    HB_OK(hipMalloc(&soff, (m + 1) * 8));
    uint64_t total = 0;
    HB_OK(hipMemcpyAsync(sk, mine.data() + c0, m * sizeof(Digest), hipMemcpyHostToDevice,
                         src.mstream));
    src.cache->lookup(sk, m, sloc, ssize, soff, t, src.mstream, src.cache->config().log_bytes / 8);
    HB_OK(hipMemcpyAsync(&total, soff + m, 8, hipMemcpyDeviceToHost, src.mstream));
    HB_OK(hipStreamSynchronize(src.mstream));
    if (total > rec_cap) total = 0;  // pathological chunk: skip it (objects just miss)
    if (total) {
      HB_OK(hipMalloc(&srec, total + 16));
      src.cache->gather(sloc, soff, m, srec, src.mstream);
      HB_OK(hipStreamSynchronize(src.mstream));
    }
    // ---- to this GPU over xGMI, insert-if-absent, store
    HB_OK(hipSetDevice(device));
    Digest* kk = nullptr;
    uint64_t *koff = nullptr, *ksize = nullptr, *kloc = nullptr, *khave = nullptr,
             *khoff = nullptr, *kvoff = nullptr;
    uint8_t* krec = nullptr;
    uint32_t* kmeta = nullptr;
    Digest* skeys2 = nullptr;
    bool ok = true;
    try {
      if (total) {
        HB_OK(hipMalloc(&kk, m * sizeof(Digest)));
        HB_OK(hipMalloc(&koff, (m + 1) * 8));
        HB_OK(hipMalloc(&ksize, (m + 1) * 8));
        HB_OK(hipMalloc(&kloc, m * 8));
        HB_OK(hipMalloc(&khave, (m + 1) * 8));
        HB_OK(hipMalloc(&khoff, (m + 1) * 8));
        HB_OK(hipMalloc(&kvoff, m * 8));
        HB_OK(hipMalloc(&kmeta, 3 * m * 4));
        HB_OK(hipMalloc(&skeys2, m * sizeof(Digest)));
        HB_OK(hipMalloc(&krec, total + 16));
        const int path = be->peer_path(src.device, device);
        copy_between(krec, device, srec, src.device, total, stream, path);
        copy_between(koff, device, soff, src.device, (m + 1) * 8, stream, path);
        copy_between(ksize, device, ssize, src.device, (m + 1) * 8, stream, path);
        copy_between(kk, device, sk, src.device, m * sizeof(Digest), stream, path);
        if (path == 2) staged_copies++;
        cache->lookup(kk, m, kloc, khave, khoff, t, stream);
        records_to_set(krec, koff, ksize, khave, m, skeys2, kvoff, kmeta, kmeta + m, kmeta + 2 * m,
                       stream);
        cache->store(skeys2, krec, kvoff, kmeta, kmeta + m, kmeta + 2 * m, m, total + 48 * m, t,
                     stream);
        HB_OK(hipStreamSynchronize(stream));
        std::vector<uint64_t> sz(m);
        HB_OK(hipMemcpy(sz.data(), ksize, m * 8, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < m; ++i) moved += sz[i] ? 1 : 0;
      }
    } catch (...) {
      ok = false;
    }
    for (void* p : {(void*)kk, (void*)koff, (void*)ksize, (void*)kloc, (void*)khave,
                    (void*)khoff, (void*)kvoff, (void*)krec, (void*)kmeta, (void*)skeys2})
      (void)hipFree(p);
    // ---- src no longer serves these digests
    HB_OK(hipSetDevice(src.device));
    if (ok && total) {
      src.cache->remove(sk, m, nullptr, t, src.mstream);
      HB_OK(hipStreamSynchronize(src.mstream));
    }
    for (void* p : {(void*)sk, (void*)sloc, (void*)ssize, (void*)soff, (void*)srec})
      (void)hipFree(p);
    HB_OK(hipSetDevice(device));
    if (!ok) throw Error("peer migration chunk failed");
  }
  migrated += moved;
  migrate_ns += (uint64_t)((wall_s() - t0) * 1e9);
  return moved;
}

void HbmBackend::Dev::sweep() {
  TraceRange tr("hbm_backend.sweep");
  uint64_t o = 0, b = 0;
  cache->sweep(be->now(), stream, &o, &b);
  live_objects = o;
  live_bytes = b;
  sweeps++;
}

void HbmBackend::Dev::finish_filter_rebuild() {
  TraceRange tr("hbm_backend.filter_rebuild");
  const uint32_t t = be->now();
  const uint64_t live = cache->export_keys(nullptr, 0, t, stream);
  if (live) {
    // the kernel writes the digests straight into mapped host memory (no device buffer)
    Mapped m;
    m.ensure(live * sizeof(Digest));
    uint64_t got = 0;
    try {
      got = std::min(live, cache->export_keys(m.dev<Digest>(), live, t, stream));
    } catch (...) {
      m.release();
      throw;
    }
    for (uint64_t i = 0; i < got; ++i) filt_next->add(m.host<Digest>()[i]);
    m.release();
  }
  std::lock_guard<std::mutex> lk(mu);
  std::atomic_store(&filt, filt_next);
  filt_next.reset();
  filt_rebuild_at = filt->adds() + be->cfg_.nbuckets_per_gpu * kEntriesPerBucket;
  filt_rebuilds++;
}

// ---------------------------------------------------------------------------------
// hot-object spreading: the reference's ketama client
// sends each key to one node (src/python/shellac/server/Server.py:81-83), so a hot key
// loads one GPU. The hot set follows a sampled GET stream; its objects are replicated on
// every shard in service and their GETs spread by the router's designation / spray.
// ---------------------------------------------------------------------------------
void HbmBackend::hot_loop() {
  pthread_setname_np(pthread_self(), "shellac-hot");
  std::unique_lock<std::mutex> lk(hot_th_mu_);
  while (!hot_stop_) {
    hot_cv_.wait_for(lk, std::chrono::milliseconds(cfg_.hot_refresh_ms), [&] { return hot_stop_; });
    if (hot_stop_) break;
    lk.unlock();
    try {
      hot_refresh();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "[shellac hbm] hot-set refresh failed: %s\n", e.what());
    }
    lk.lock();
  }
}

StatList HbmBackend::hot_refresh() {
  std::lock_guard<std::mutex> lk(hot_mu_);
  return hot_refresh_locked();
}

namespace {
// waits for n completion callbacks (barriers, fills); ok[i] per callback index
struct Waiter {
  std::mutex mu;
  std::condition_variable cv;
  int left = 0;
  std::vector<int> ok;  // 1 ok, 0 failed, -1 pending
  explicit Waiter(int n) : left(n), ok((size_t)n, -1) {}
  std::function<void(bool)> cb(int i) {
    return [this, i](bool good) {
      std::lock_guard<std::mutex> lk(mu);
      ok[(size_t)i] = good ? 1 : 0;
      if (--left == 0) cv.notify_all();
    };
  }
  bool wait(int timeout_ms) {
    std::unique_lock<std::mutex> lk(mu);
    return cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return left == 0; });
  }
  int state(int i) {
    std::lock_guard<std::mutex> lk(mu);
    return ok[(size_t)i];
  }
};
}  // namespace

// One refresh. The order keeps every GET answered by a copy no older than the last SET /
// DELETE that finished before the GET began (HotSpread's refresh_hot, single process):
//  1. plan the new hot set from the sampled counts (plan_hot: top hot_objects, designated
//     greedily from the owners' cold loads, the hottest sprayed);
//  2. every shard in service starts recording writes of the objects about to be filled
//     (Dev::filling / touched);
//  3. router table T1 = the current hot set + the new objects designated to their owners:
//     the new objects' SETs / DELETEs are written through from here on, their GETs still go
//     to their owners. set_hot returns once nothing routes under the old table, so every
//     write routed owner-only has been queued;
//  4. a barrier on each owner: those writes have finished on its GPU;
//  5. the owners look the objects up and gather their records (one snapshot per owner);
//  6. per target shard, the records of the objects it does not own go over xGMI into its
//     staging (copy_between: hipMemcpyPeerAsync, or staged through pinned host memory) and
//     a fill request is queued behind the shard's writes; the batcher drops the rows with
//     a write queued since step 2 (that copy is newer) and stores the rest;
//  7. once every fill has finished, the shards that now hold the whole set join the
//     spread mask, and T2 = the new hot set with its designations is published;
//  8. objects that left the set lose their non-owner replicas (deleted: no SET reaches
//     them any more, and a later promotion must find no stale copy).
// Shards that are down, or eject mid-refresh, drop out of the spread mask (a restored
// shard is flushed and rejoins with a full fill at the next refresh).
StatList HbmBackend::hot_refresh_locked() {
  StatList out;
  if (!hot_on_) return out;
  TraceRange tr("hbm_backend.hot_refresh");
  const double t_start = wall_s();
  const int N = (int)devs_.size();
  // ---- samples -> decayed counts
  uint64_t nsamp = 0;
  for (int i = 0; i < kSampleStripes; ++i) {
    std::vector<Digest> v;
    {
      std::lock_guard<std::mutex> lk(samples_[i].mu);
      v.swap(samples_[i].v);
    }
    nsamp += v.size();
    for (const Digest& d : v) {
      auto it = hot_counts_.find(d);
      if (it != hot_counts_.end()) ++it->second;
      else if (hot_counts_.size() < (1u << 18)) hot_counts_.emplace(d, 1);
    }
  }
  hot_samples_.fetch_add(nsamp, std::memory_order_relaxed);
  uint64_t total = 0;
  for (const auto& kv : hot_counts_) total += kv.second;
  out.emplace_back("samples", total);
  if (total < cfg_.hot_min_samples) {
    out.emplace_back("skipped", 1);
    return out;
  }
  const uint64_t up = up_mask_.load(std::memory_order_acquire);
  std::vector<std::pair<Digest, uint64_t>> counts(hot_counts_.begin(), hot_counts_.end());
  for (auto it = hot_counts_.begin(); it != hot_counts_.end();) {  // halve: recent traffic rules
    it->second >>= 1;
    if (!it->second) it = hot_counts_.erase(it);
    else ++it;
  }
  const double above = cfg_.hot_spray_above > 0 ? cfg_.hot_spray_above : 1.0 / (4.0 * N);
  std::unordered_map<Digest, int32_t, DigestHash, DigestEq> cur;
  for (size_t i = 0; i < hot_set_.size(); ++i) cur.emplace(hot_set_[i], hot_rank_[i]);
  // hysteresis: an object already replicated stays unless a new one is twice as hot (the
  // set's tail would otherwise churn on sampling noise: a fill and a delete per object)
  const std::function<bool(const Digest&)> sticky = [&](const Digest& d) { return cur.count(d) > 0; };
  HotPlan plan = plan_hot(counts, cfg_.hot_objects, N, up,
                          [&](const Digest& d) { return owner_of(d, up); }, above, 2, &sticky,
                          2.0);
  // ---- what changes
  std::unordered_set<Digest, DigestHash, DigestEq> added;
  for (const Digest& d : plan.hot)
    if (!cur.count(d)) added.insert(d);
  const uint64_t mask0 = spread_mask_.load(std::memory_order_acquire) & up;
  const uint64_t heal = up & ~mask0;  // in service, holding no replicas yet (restored, new)
  std::vector<uint64_t> gen0((size_t)N);
  for (int r = 0; r < N; ++r) gen0[(size_t)r] = devs_[(size_t)r]->eject_gen.load();
  // objects to snapshot, hottest first: the new ones, and every planned one for a heal
  std::vector<Digest> fill_objs;
  for (const Digest& d : plan.hot)
    if (heal || added.count(d)) fill_objs.push_back(d);
  // ---- 2. record writes of those objects on every shard in service
  for (int r = 0; r < N; ++r) {
    if (!((up >> r) & 1)) continue;
    Dev& dv = *devs_[(size_t)r];
    std::lock_guard<std::mutex> lk(dv.mu);
    dv.filling.clear();
    dv.touched.clear();
    for (const Digest& d : fill_objs) dv.filling.insert(d.lo);
  }
  auto stop_recording = [&] {
    for (auto& dv : devs_) {
      std::lock_guard<std::mutex> lk(dv->mu);
      dv->filling.clear();
      dv->touched.clear();
    }
  };
  // ---- 3. T1: write-through for the new objects, their GETs at their owners (nothing new:
  // the published table already is T1)
  if (!added.empty()) {
    std::vector<Digest> h(hot_set_);
    std::vector<int32_t> rk(hot_rank_);
    for (const Digest& d : plan.hot)
      if (added.count(d)) {
        h.push_back(d);
        rk.push_back(owner_of(d, up));
      }
    router_->set_hot(h.data(), (int64_t)h.size(), rk.data(), hot_weights_.data());
  }
  const uint32_t t = now();
  const int wait_ms = 2 * cfg_.batch_timeout_ms + 1000;
  // ---- 4. barrier on every owner (source) of an object to fill
  // (an object of the current set owned by a shard being healed is read from a shard that
  // holds its replica: the healed one was flushed, and warm restore leaves hot objects be)
  int replica_src = -1;
  for (int r = 0; r < N && replica_src < 0; ++r)
    if ((mask0 >> r) & 1) replica_src = r;
  std::vector<std::vector<Digest>> by_owner((size_t)N);
  for (const Digest& d : fill_objs) {
    int o = owner_of(d, up);
    if (o >= 0 && ((heal >> o) & 1) && replica_src >= 0 && cur.count(d)) o = replica_src;
    if (o >= 0) by_owner[(size_t)o].push_back(d);
  }
  uint64_t bad = 0;  // shards that failed a barrier or a fill this refresh
  {
    std::vector<int> who;
    for (int o = 0; o < N; ++o)
      if (!by_owner[(size_t)o].empty()) who.push_back(o);
    auto w = std::make_shared<Waiter>((int)who.size());
    for (size_t i = 0; i < who.size(); ++i) {
      auto wp = w;
      auto cb = w->cb((int)i);
      enqueue_ctl(who[i], [wp, cb](bool ok) { cb(ok); });
    }
    w->wait(wait_ms);
    for (size_t i = 0; i < who.size(); ++i)
      if (w->state((int)i) != 1) {
        bad |= 1ull << who[i];
        by_owner[(size_t)who[i]].clear();  // its objects are not filled this time
      }
  }
  // ---- 5. snapshot on each owner
  struct Snap {
    std::vector<Digest> keys;
    std::vector<uint64_t> size, off;
    uint64_t total = 0;
  };
  std::vector<Snap> snap((size_t)N);
  for (int o = 0; o < N; ++o) {
    Snap& sn = snap[(size_t)o];
    sn.keys = by_owner[(size_t)o];
    const int64_t m = (int64_t)sn.keys.size();
    if (!m) continue;
    Dev& od = *devs_[(size_t)o];
    try {
      HB_OK(hipSetDevice(od.device));
      Digest* sk = od.hs_keys.ensure<Digest>((size_t)m * sizeof(Digest));
      uint64_t* sloc = od.hs_loc.ensure<uint64_t>((size_t)m * 8);
      uint64_t* ssz = od.hs_size.ensure<uint64_t>((size_t)(m + 1) * 8);
      uint64_t* soff = od.hs_off.ensure<uint64_t>((size_t)(m + 1) * 8);
      HB_OK(hipMemcpyAsync(sk, sn.keys.data(), (size_t)m * sizeof(Digest), hipMemcpyHostToDevice,
                           od.mstream));
      od.cache->lookup(sk, m, sloc, ssz, soff, t, od.mstream, od.cache->config().log_bytes / 8);
      sn.size.assign((size_t)m + 1, 0);
      sn.off.assign((size_t)m + 1, 0);
      HB_OK(hipMemcpyAsync(sn.size.data(), ssz, (size_t)m * 8, hipMemcpyDeviceToHost, od.mstream));
      HB_OK(hipMemcpyAsync(sn.off.data(), soff, (size_t)(m + 1) * 8, hipMemcpyDeviceToHost,
                           od.mstream));
      HB_OK(hipStreamSynchronize(od.mstream));
      sn.total = sn.off[(size_t)m];
      if (sn.total) {
        uint8_t* srec = od.hs_rec.ensure<uint8_t>(sn.total + 16);
        od.cache->gather(sloc, soff, m, srec, od.mstream);
        HB_OK(hipStreamSynchronize(od.mstream));
      }
    } catch (const std::exception& e) {
      std::fprintf(stderr, "[shellac hbm] hot snapshot on gpu %d failed: %s\n", od.device, e.what());
      bad |= 1ull << o;
      sn = Snap{};
    }
  }
  // ---- budget: new objects hottest first, (targets) x record bytes each
  std::unordered_set<Digest, DigestHash, DigestEq> deferred;
  {
    std::unordered_map<Digest, uint64_t, DigestHash, DigestEq> rec;
    for (int o = 0; o < N; ++o)
      for (size_t i = 0; i < snap[(size_t)o].keys.size(); ++i)
        rec[snap[(size_t)o].keys[i]] = snap[(size_t)o].size[i];
    const uint64_t targets = (uint64_t)std::max(1, __builtin_popcountll(up) - 1);
    uint64_t spent = 0;
    for (const Digest& d : plan.hot) {
      if (!added.count(d)) continue;
      auto it = rec.find(d);
      const uint64_t b = it == rec.end() ? 0 : it->second * targets;
      if (spent + b > cfg_.hot_fill_budget) deferred.insert(d);
      else spent += b;
    }
  }
  // an object is spread after this refresh if it stays (was hot and still is) or was added,
  // snapshot ok (owner did not fail) and within the budget
  std::unordered_set<Digest, DigestHash, DigestEq> filled_ok;
  for (int o = 0; o < N; ++o)
    for (const Digest& d : snap[(size_t)o].keys) filled_ok.insert(d);
  // ---- 6. fills, one per target shard
  std::vector<std::shared_ptr<HotFill>> fills((size_t)N);
  uint64_t fill_bytes = 0;
  std::vector<int> tgt;
  for (int r = 0; r < N; ++r) {
    if (!((up >> r) & 1) || ((bad >> r) & 1)) continue;
    const bool full = (heal >> r) & 1;
    // rows: every snapshot row of the other owners; size 0 where this shard takes no copy
    int64_t m = 0;
    uint64_t bytes = 0;
    for (int o = 0; o < N; ++o)
      if (o != r && snap[(size_t)o].total) {
        m += (int64_t)snap[(size_t)o].keys.size();
        bytes += snap[(size_t)o].total;
      }
    if (!m) continue;
    Dev& td = *devs_[(size_t)r];
    auto h = std::make_shared<HotFill>();
    try {
      HB_OK(hipSetDevice(td.device));
      Digest* kk = td.hf_keys.ensure<Digest>((size_t)m * sizeof(Digest));
      uint8_t* krec = td.hf_rec.ensure<uint8_t>(bytes + 16);
      uint64_t* koff = td.hf_off.ensure<uint64_t>((size_t)(m + 1) * 8);
      h->okeys = td.hf_okeys.ensure<Digest>((size_t)m * sizeof(Digest));
      h->ovoff = td.hf_voff.ensure<uint64_t>((size_t)m * 8);
      h->ometa = td.hf_meta.ensure<uint32_t>((size_t)m * 12);
      td.hf_size.ensure((size_t)(m + 1) * 8);
      std::vector<Digest> keys;
      std::vector<uint64_t> off;
      keys.reserve((size_t)m);
      off.reserve((size_t)m + 1);
      h->hsize = td.hf_size.host<uint64_t>();
      h->dsize = td.hf_size.dev<uint64_t>();
      uint64_t base = 0;
      int64_t row = 0;
      for (int o = 0; o < N; ++o) {
        const Snap& sn = snap[(size_t)o];
        if (o == r || !sn.total) continue;
        Dev& od = *devs_[(size_t)o];
        copy_between(krec + base, td.device, od.hs_rec.p, od.device, sn.total, td.mstream,
                     peer_path(od.device, td.device));
        if (peer_path(od.device, td.device) == 2) td.staged_copies++;
        for (size_t i = 0; i < sn.keys.size(); ++i, ++row) {
          const Digest& d = sn.keys[i];
          keys.push_back(d);
          off.push_back(base + sn.off[i]);
          const bool want = (full || added.count(d)) && !deferred.count(d);
          h->hsize[row] = want ? sn.size[i] : 0;
          h->lo.push_back(d.lo);
          if (want && sn.size[i]) fill_bytes += sn.size[i];
        }
        base += sn.total;
      }
      off.push_back(base);
      HB_OK(hipMemcpyAsync(kk, keys.data(), (size_t)m * sizeof(Digest), hipMemcpyHostToDevice,
                           td.mstream));
      HB_OK(hipMemcpyAsync(koff, off.data(), (size_t)(m + 1) * 8, hipMemcpyHostToDevice,
                           td.mstream));
      HB_OK(hipStreamSynchronize(td.mstream));
      h->m = m;
      h->kk = kk;
      h->krec = krec;
      h->koff = koff;
      h->bound = bytes + 48 * (uint64_t)m;
      if (cfg_.presence_filter) {  // GETs spread here must not skip the replicas
        std::lock_guard<std::mutex> lk(td.mu);
        for (int64_t i = 0; i < m; ++i)
          if (h->hsize[i]) {
            td.filt->add(keys[(size_t)i]);
            if (td.filt_next) td.filt_next->add(keys[(size_t)i]);
          }
      }
    } catch (const std::exception& e) {
      std::fprintf(stderr, "[shellac hbm] hot fill staging on gpu %d failed: %s\n", td.device,
                   e.what());
      bad |= 1ull << r;
      continue;
    }
    fills[(size_t)r] = h;
    tgt.push_back(r);
  }
  {
    auto w = std::make_shared<Waiter>((int)tgt.size());
    for (size_t i = 0; i < tgt.size(); ++i) {
      Req q;
      q.kind = 4;
      q.d = Digest{0, 0};
      q.fill = fills[(size_t)tgt[i]];
      auto wp = w;
      auto cb = w->cb((int)i);
      q.ccb = [wp, cb](bool ok) { cb(ok); };
      enqueue(tgt[i], std::move(q));
    }
    if (!w->wait(wait_ms)) {
      // a shard that never got to its fill: cancel it if not launched (else it completes
      // with its touched check made in time, and only its buffers must outlive it)
      for (size_t i = 0; i < tgt.size(); ++i) {
        if (w->state((int)i) != -1) continue;
        Dev& td = *devs_[(size_t)tgt[i]];
        std::lock_guard<std::mutex> lk(td.mu);
        HotFill& h = *fills[(size_t)tgt[i]];
        if (!h.launched) h.cancelled = true;
        else {  // still running on the GPU: its staging is abandoned (leaked), not reused
          td.hf_keys = DevBuf{}; td.hf_rec = DevBuf{}; td.hf_off = DevBuf{};
          td.hf_okeys = DevBuf{}; td.hf_voff = DevBuf{}; td.hf_meta = DevBuf{};
          td.hf_size = Mapped{};
        }
      }
    }
    uint64_t rows = 0, skipped = 0;
    for (size_t i = 0; i < tgt.size(); ++i) {
      const int r = tgt[i];
      if (w->state((int)i) != 1) {
        bad |= 1ull << r;
        hot_fill_failed_.fetch_add(1, std::memory_order_relaxed);
        continue;
      }
      Dev& td = *devs_[(size_t)r];
      std::lock_guard<std::mutex> lk(td.mu);
      rows += fills[(size_t)r]->rows;
      skipped += fills[(size_t)r]->skipped;
    }
    hot_filled_.fetch_add(rows, std::memory_order_relaxed);
    hot_fill_skipped_.fetch_add(skipped, std::memory_order_relaxed);
    out.emplace_back("filled_rows", rows);
    out.emplace_back("fill_skipped_rows", skipped);
  }
  stop_recording();
  // ---- 7. the spread mask, then T2
  uint64_t mask = (mask0 | heal) & ~bad;
  for (int r = 0; r < N; ++r)
    if (devs_[(size_t)r]->eject_gen.load() != gen0[(size_t)r]) mask &= ~(1ull << r);
  // owners whose barrier or snapshot failed: their new objects are not filled anywhere
  std::vector<Digest> final_hot;
  std::vector<int32_t> final_rank;
  for (size_t i = 0; i < plan.hot.size(); ++i) {
    const Digest& d = plan.hot[i];
    if (added.count(d) && (deferred.count(d) || !filled_ok.count(d))) continue;
    final_hot.push_back(d);
    final_rank.push_back(plan.rank[i]);
  }
  std::vector<double> wts((size_t)N, 0.0);
  double wsum = 0;
  for (int r = 0; r < N; ++r)
    if ((mask >> r) & 1) wsum += (wts[(size_t)r] = plan.weights[(size_t)r]);
  if (wsum <= 0) {  // nowhere to spread: no hot set
    final_hot.clear();
    final_rank.clear();
    wts.assign((size_t)N, 1.0);
  }
  spread_mask_.store(mask, std::memory_order_release);
  for (int r = 0; r < N; ++r)  // an ejection that raced the store above
    if (devs_[(size_t)r]->eject_gen.load() != gen0[(size_t)r] || !devs_[(size_t)r]->up())
      spread_mask_.fetch_and(~(1ull << r), std::memory_order_acq_rel);
  const bool same = added.empty() && final_hot.size() == hot_set_.size() &&
                    final_rank == std::vector<int32_t>(hot_rank_.begin(), hot_rank_.end()) &&
                    wts == hot_weights_ &&
                    std::equal(final_hot.begin(), final_hot.end(), hot_set_.begin(),
                               [](const Digest& x, const Digest& y) { return x.lo == y.lo && x.hi == y.hi; });
  if (!same)  // (an unchanged table is not republished)
    router_->set_hot(final_hot.data(), (int64_t)final_hot.size(), final_rank.data(), wts.data());
  // ---- 8. replicas of objects no longer hot (the old set and this refresh's write-through
  // set minus the new one) go from every shard but their owner
  std::unordered_set<Digest, DigestHash, DigestEq> fin(final_hot.begin(), final_hot.end());
  std::vector<Digest> gone;
  for (const Digest& d : hot_set_)
    if (!fin.count(d)) gone.push_back(d);
  for (const Digest& d : added)
    if (!fin.count(d)) gone.push_back(d);
  const uint64_t up2 = up_mask_.load(std::memory_order_acquire);
  uint64_t dropped = 0;
  for (const Digest& d : gone) {
    const int o = owner_of(d, up2);
    for (int r = 0; r < N; ++r) {
      if (r == o || !((up2 >> r) & 1)) continue;
      Req q;
      q.kind = 2;
      q.d = d;
      write_begin(d.lo);
      enqueue(r, std::move(q));
      ++dropped;
    }
  }
  hot_set_ = std::move(final_hot);
  hot_rank_ = std::move(final_rank);
  hot_weights_ = wts;
  hot_objects_.store(hot_set_.size(), std::memory_order_relaxed);
  uint64_t n_added = 0;
  for (const Digest& d : added) n_added += fin.count(d);
  hot_added_.fetch_add(n_added, std::memory_order_relaxed);
  hot_removed_.fetch_add(gone.size(), std::memory_order_relaxed);
  hot_deferred_.fetch_add(deferred.size(), std::memory_order_relaxed);
  hot_dropped_replicas_.fetch_add(dropped, std::memory_order_relaxed);
  hot_fill_bytes_.fetch_add(fill_bytes, std::memory_order_relaxed);
  hot_refreshes_.fetch_add(1, std::memory_order_relaxed);
  const uint64_t us = (uint64_t)((wall_s() - t_start) * 1e6);
  hot_refresh_us_.store(us, std::memory_order_relaxed);
  out.emplace_back("hot", hot_set_.size());
  out.emplace_back("added", n_added);
  out.emplace_back("removed", gone.size());
  out.emplace_back("deferred", deferred.size());
  out.emplace_back("replicas_dropped", dropped);
  out.emplace_back("fill_bytes", fill_bytes);
  out.emplace_back("spread_mask", spread_mask_.load());
  out.emplace_back("heal_mask", heal);
  out.emplace_back("failed_mask", bad);
  out.emplace_back("hot_share_ppm", (uint64_t)(plan.hot_share * 1e6));
  double pmax = 0, psum = 0;
  int pn = 0;
  for (int r = 0; r < N; ++r)
    if ((up >> r) & 1) {
      pmax = std::max(pmax, plan.planned[(size_t)r]);
      psum += plan.planned[(size_t)r];
      ++pn;
    }
  out.emplace_back("planned_max_over_mean_ppm",
                   psum > 0 ? (uint64_t)(pmax / (psum / pn) * 1e6) : 0);
  out.emplace_back("refresh_us", us);
  return out;
}

void HbmBackend::stats(StatList* out) {
  CacheCounters t{};
  uint64_t hbm = 0;
  auto sum = [&](std::atomic<uint64_t> Dev::*m) {
    uint64_t s = 0;
    for (auto& d : devs_) s += ((*d).*m).load();
    return s;
  };
  for (auto& d : devs_) {
    (void)hipSetDevice(d->device);
    // a stream of its own, non-blocking: the batcher's may be busy, and the legacy null
    // stream would also wait for the resident edge server; counters are advisory
    const CacheCounters c = d->cache->counters(d->sstream);
    t.get_ops += c.get_ops; t.get_hits += c.get_hits; t.set_ops += c.set_ops;
    t.set_bytes += c.set_bytes; t.set_evicted += c.set_evicted; t.del_ops += c.del_ops;
    t.reinserted += c.reinserted; t.reinsert_bytes += c.reinsert_bytes;
    hbm += d->cache->hbm_bytes();
  }
  out->emplace_back("cache_get_ops", t.get_ops);
  out->emplace_back("cache_get_hits", t.get_hits);
  out->emplace_back("cache_set_ops", t.set_ops);
  out->emplace_back("cache_set_bytes", t.set_bytes);
  out->emplace_back("cache_evicted", t.set_evicted);
  out->emplace_back("cache_reinserted", t.reinserted);
  out->emplace_back("cache_reinsert_bytes", t.reinsert_bytes);
  out->emplace_back("hbm_gpus", devs_.size());
  out->emplace_back("hbm_gpus_up", (uint64_t)__builtin_popcountll(up_mask_.load()));
  out->emplace_back("hbm_bytes", hbm);
  out->emplace_back("hbm_pipeline_depth", (uint64_t)cfg_.depth);
  out->emplace_back("hbm_batches", sum(&Dev::batches));
  out->emplace_back("hbm_batched_requests", sum(&Dev::batched_reqs));
  uint64_t mb = 0;
  for (auto& d : devs_) mb = std::max<uint64_t>(mb, d->max_batch.load());
  out->emplace_back("hbm_max_batch", mb);
  out->emplace_back("hbm_batch_ns_total", sum(&Dev::batch_ns));
  out->emplace_back("hbm_sweeps", sum(&Dev::sweeps));
  out->emplace_back("hbm_live_objects", sum(&Dev::live_objects));
  out->emplace_back("hbm_live_bytes", sum(&Dev::live_bytes));
  out->emplace_back("hbm_coalesced_gets", sum(&Dev::coalesced));
  out->emplace_back("hbm_key_mismatch", sum(&Dev::key_mismatch));
  out->emplace_back("hbm_failures", sum(&Dev::failures));
  out->emplace_back("hbm_ejections", sum(&Dev::ejections));
  out->emplace_back("hbm_restores", sum(&Dev::restores));
  out->emplace_back("hbm_regathers", sum(&Dev::regathers));
  out->emplace_back("hbm_arena_misses", sum(&Dev::arena_misses));
  out->emplace_back("hbm_served_batches", sum(&Dev::served_batches));
  out->emplace_back("hbm_ordered_get_batches", sum(&Dev::ordered_gets));
  out->emplace_back("hbm_direct_jobs", sum(&Dev::direct_jobs));
  out->emplace_back("hbm_direct_requests", sum(&Dev::direct_reqs));
  out->emplace_back("hbm_direct_fallback_requests", sum(&Dev::direct_fallbacks));
  out->emplace_back("hbm_direct_overflows", sum(&Dev::direct_overflows));
  out->emplace_back("hbm_direct_timeouts", sum(&Dev::direct_timeouts));
  // submit -> completion seen by the reactor, summed over jobs
  out->emplace_back("hbm_direct_job_ns_total", sum(&Dev::direct_ns));
  uint64_t sl = 0;
  for (auto& d : devs_) sl += d->cache->serve_launches();
  out->emplace_back("hbm_server_launches", sl);
  out->emplace_back("hbm_staged_peer_copies", sum(&Dev::staged_copies));
  uint64_t direct = 0;
  for (uint8_t v : peer_ok_) direct += v;
  out->emplace_back("hbm_peer_pairs_direct", direct);
  out->emplace_back("hbm_migrated", sum(&Dev::migrated));
  out->emplace_back("hbm_migrate_ns", sum(&Dev::migrate_ns));
  out->emplace_back("hbm_dropped_sets", sum(&Dev::dropped));
  out->emplace_back("hbm_no_shard_misses", no_shard_misses_.load());
  // per-shard GET routing (the load hot-object spreading evens out) and the hot set
  for (size_t i = 0; i < devs_.size(); ++i)
    out->emplace_back("hbm_shard_gets_" + std::to_string(i), devs_[i]->routed_total());
  out->emplace_back("hbm_hot_spreading", hot_on_ ? 1 : 0);
  if (hot_on_) {
    out->emplace_back("hbm_hot_objects", hot_objects_.load());
    out->emplace_back("hbm_hot_refreshes", hot_refreshes_.load());
    out->emplace_back("hbm_hot_added", hot_added_.load());
    out->emplace_back("hbm_hot_removed", hot_removed_.load());
    out->emplace_back("hbm_hot_deferred", hot_deferred_.load());
    out->emplace_back("hbm_hot_filled_rows", hot_filled_.load());
    out->emplace_back("hbm_hot_fill_skipped_rows", hot_fill_skipped_.load());
    out->emplace_back("hbm_hot_fill_failures", hot_fill_failed_.load());
    out->emplace_back("hbm_hot_fill_bytes", hot_fill_bytes_.load());
    out->emplace_back("hbm_hot_replicas_dropped", hot_dropped_replicas_.load());
    uint64_t sg = 0;
    for (const SpreadCtr& c : hot_spread_gets_) sg += c.v.load(std::memory_order_relaxed);
    out->emplace_back("hbm_hot_spread_gets", sg);
    out->emplace_back("hbm_hot_samples", hot_samples_.load());
    out->emplace_back("hbm_hot_spread_mask", spread_mask_.load());
    out->emplace_back("hbm_hot_refresh_us_last", hot_refresh_us_.load());
    out->emplace_back("hbm_hot_router_tables", router_->publications());
  }
  uint64_t arena = 0, aallocs = 0, afrees = 0, amax = 0;
  for (auto& d : devs_) {
    amax = std::max<uint64_t>(amax, d->pool->alloc_max_us());
    arena += d->pool->allocated();
    aallocs += d->pool->allocs();
    afrees += d->pool->frees();
  }
  out->emplace_back("hbm_arena_bytes", arena);
  out->emplace_back("hbm_arena_allocs", aallocs);
  out->emplace_back("hbm_arena_frees", afrees);
  out->emplace_back("hbm_arena_alloc_max_us", amax);
  if (cfg_.presence_filter) {
    uint64_t adds = 0;
    for (auto& d : devs_) adds += std::atomic_load(&d->filt)->adds();
    out->emplace_back("hbm_filter_skips", sum(&Dev::filt_skips));
    out->emplace_back("hbm_filter_rebuilds", sum(&Dev::filt_rebuilds));
    out->emplace_back("hbm_filter_adds", adds);
    out->emplace_back("hbm_filter_fill_ppm",
                      (uint64_t)(std::atomic_load(&devs_[0]->filt)->fill() * 1e6));
  }
}

}  // namespace shellac
