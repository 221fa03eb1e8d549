// HbmBackend: the HTTP proxy's batched HIP pipeline over one HBM shard per local GPU
// (split from backend.cc so the host-only backends build without ROCm).
#include <chrono>
#include <cstdio>

#include "backend.h"
#include "hbm_cache.h"
#include "trace.h"

namespace shellac {

namespace {
double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

// =====================================================================================
// HBM
// =====================================================================================
#define HB_OK(expr)                                                                   \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) throw Error(std::string("HIP: ") + hipGetErrorString(_e) + \
                                      " at " #expr);                                  \
  } while (0)

struct HbmBackend::Dev {
  int device = 0;
  std::unique_ptr<HbmCache> cache;
  hipStream_t stream = nullptr;
  size_t n_cap = 0, out_cap = 0, vals_cap = 0;
  Digest *d_keys = nullptr, *h_keys = nullptr;
  Digest* h_keys_dev = nullptr;    // device view of the mapped h_keys
  uint64_t* h_off_dev = nullptr;   // device view of the mapped h_off
  uint64_t *d_loc = nullptr, *d_size = nullptr, *d_off = nullptr, *h_off = nullptr;
  uint8_t* h_out = nullptr;
  uint8_t* h_out_dev = nullptr;  // device view of the pinned h_out (zero-copy gather target)
  uint8_t *d_vals = nullptr, *h_vals = nullptr;
  uint64_t *d_voff = nullptr, *h_voff = nullptr;
  uint32_t *d_meta = nullptr, *h_meta = nullptr;  // [vlen | flags | expire] x n
  uint8_t *d_found = nullptr, *h_found = nullptr;
  // zero-copy SET staging for graph-replayed micro-batches (mapped pinned memory the
  // kernels read directly): keys, value bytes, value offsets, [vlen | flags | expire]
  static constexpr int kSetClasses = 3;
  static constexpr int64_t kSetClass[kSetClasses] = {64, 512, 4096};
  Digest *hs_keys = nullptr, *hs_keys_dev = nullptr;
  uint8_t *hs_vals = nullptr, *hs_vals_dev = nullptr;
  size_t hs_vals_cap = 0;
  uint64_t *hs_voff = nullptr, *hs_voff_dev = nullptr;
  uint32_t *hs_meta = nullptr, *hs_meta_dev = nullptr;
  HbmCache::StoreGraph set_graph[kSetClasses];
  // host-side GET coalescing scratch (batcher thread only)
  std::vector<int32_t> co_tab;
  std::vector<uint32_t> urow;
  std::vector<CacheValue> uval;
  std::vector<uint8_t> uhit;

  void set_device() { HB_OK(hipSetDevice(device)); }

  template <typename T>
  static void map_alloc(T** host, T** dev, size_t bytes) {
    HB_OK(hipHostMalloc(reinterpret_cast<void**>(host), bytes, hipHostMallocMapped));
    HB_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(dev), *host, 0));
  }
  void ensure_set_staging(size_t val_bytes) {
    const int64_t cmax = kSetClass[kSetClasses - 1];
    if (!hs_keys) {
      map_alloc(&hs_keys, &hs_keys_dev, cmax * sizeof(Digest));
      map_alloc(&hs_voff, &hs_voff_dev, cmax * sizeof(uint64_t));
      map_alloc(&hs_meta, &hs_meta_dev, 3 * cmax * sizeof(uint32_t));
      cache->reserve(cmax);
    }
    if (val_bytes > hs_vals_cap) {  // graphs holding the old pointer re-capture
      size_t cap = hs_vals_cap ? hs_vals_cap : (4u << 20);
      while (cap < val_bytes) cap *= 2;
      HB_OK(hipStreamSynchronize(stream));
      (void)hipHostFree(hs_vals);
      map_alloc(&hs_vals, &hs_vals_dev, cap);
      hs_vals_cap = cap;
    }
  }

  void ensure_n(size_t n) {
    if (n <= n_cap) return;
    size_t cap = n_cap ? n_cap : 1024;
    while (cap < n) cap *= 2;
    HB_OK(hipStreamSynchronize(stream));
    (void)hipFree(d_keys); (void)hipHostFree(h_keys); (void)hipFree(d_loc); (void)hipFree(d_size);
    (void)hipFree(d_off); (void)hipHostFree(h_off); (void)hipFree(d_voff); (void)hipHostFree(h_voff);
    (void)hipFree(d_meta); (void)hipHostFree(h_meta); (void)hipFree(d_found); (void)hipHostFree(h_found);
    HB_OK(hipMalloc(&d_keys, cap * sizeof(Digest)));
    HB_OK(hipHostMalloc(&h_keys, cap * sizeof(Digest), hipHostMallocMapped));
    HB_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_keys_dev), h_keys, 0));
    HB_OK(hipMalloc(&d_loc, cap * 8));
    HB_OK(hipMalloc(&d_size, (cap + 1) * 8));
    HB_OK(hipMalloc(&d_off, (cap + 1) * 8));
    HB_OK(hipHostMalloc(&h_off, (cap + 1) * 8, hipHostMallocMapped));
    HB_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_off_dev), h_off, 0));
    HB_OK(hipMalloc(&d_voff, cap * 8));
    HB_OK(hipHostMalloc(&h_voff, cap * 8, hipHostMallocDefault));
    HB_OK(hipMalloc(&d_meta, cap * 12));
    HB_OK(hipHostMalloc(&h_meta, cap * 12, hipHostMallocDefault));
    HB_OK(hipMalloc(&d_found, cap));
    HB_OK(hipHostMalloc(&h_found, cap, hipHostMallocDefault));
    n_cap = cap;
    cache->reserve((int64_t)cap);
  }
  void ensure_out(size_t bytes) {
    if (bytes <= out_cap) return;
    size_t cap = out_cap ? out_cap : (16u << 20);
    while (cap < bytes) cap *= 2;
    HB_OK(hipStreamSynchronize(stream));
    (void)hipHostFree(h_out);
    HB_OK(hipHostMalloc(&h_out, cap, hipHostMallocMapped));
    HB_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_out_dev), h_out, 0));
    out_cap = cap;
  }
  void ensure_vals(size_t bytes) {
    if (bytes <= vals_cap) return;
    size_t cap = vals_cap ? vals_cap : (1u << 20);
    while (cap < bytes) cap *= 2;
    HB_OK(hipStreamSynchronize(stream));
    (void)hipFree(d_vals); (void)hipHostFree(h_vals);
    HB_OK(hipMalloc(&d_vals, cap));
    HB_OK(hipHostMalloc(&h_vals, cap, hipHostMallocDefault));
    vals_cap = cap;
  }
  ~Dev() {
    (void)hipSetDevice(device);
    (void)hipStreamSynchronize(stream);
    cache.reset();
    (void)hipFree(d_keys); (void)hipHostFree(h_keys); (void)hipFree(d_loc); (void)hipFree(d_size);
    (void)hipFree(d_off); (void)hipHostFree(h_off); (void)hipHostFree(h_out);
    (void)hipFree(d_vals); (void)hipHostFree(h_vals); (void)hipFree(d_voff); (void)hipHostFree(h_voff);
    (void)hipFree(d_meta); (void)hipHostFree(h_meta); (void)hipFree(d_found); (void)hipHostFree(h_found);
    for (auto& g : set_graph) HbmCache::destroy_graph(&g);
    (void)hipHostFree(hs_keys); (void)hipHostFree(hs_vals); (void)hipHostFree(hs_voff);
    (void)hipHostFree(hs_meta);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

HbmBackend::HbmBackend(const HbmBackendConfig& cfg)
    : cfg_(cfg), ring_((int)cfg.devices.size()), epoch_(wall_s()) {
  SH_CHECK(!cfg_.devices.empty(), "HbmBackend needs at least one device");
  for (int dev : cfg_.devices) {
    auto d = std::make_unique<Dev>();
    d->device = dev;
    d->set_device();
    ShardConfig sc;
    sc.log_bytes = cfg_.log_bytes_per_gpu / 16 * 16;
    sc.nbuckets = cfg_.nbuckets_per_gpu;
    sc.max_item = cfg_.max_item;
    sc.device = dev;
    d->cache = std::make_unique<HbmCache>(sc);
    HB_OK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    d->ensure_n(4096);
    d->ensure_out(4u << 20);
    d->ensure_vals(4u << 20);
    devs_.push_back(std::move(d));
  }
  if (cfg_.presence_filter) {
    // 16 bits per index slot of every shard (capped at 256 MiB): ~2 % false positives
    // when a full index's worth of digests has been added since the last rebuild
    const uint64_t slots = cfg_.nbuckets_per_gpu * kEntriesPerBucket * devs_.size();
    filt_bits_ = std::min<uint64_t>(slots * 16, 1ull << 31);
    filt_rebuild_at_ = slots;
    filt_ = std::make_shared<PresenceFilter>(filt_bits_);
  }
  th_ = std::thread([this] { loop(); });
}

HbmBackend::~HbmBackend() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

uint32_t HbmBackend::now() const { return (uint32_t)(wall_s() - epoch_) + 1; }

void HbmBackend::get(const std::string&, const Digest& d, Executor* ex, GetCallback done) {
  if (cfg_.presence_filter && !std::atomic_load(&filt_)->maybe(d)) {
    // never stored: a miss without a GPU batch
    filt_skips_.fetch_add(1, std::memory_order_relaxed);
    done(false, CacheValue{});
    return;
  }
  Req r;
  r.kind = 0;
  r.d = d;
  r.ex = ex;
  r.gcb = std::move(done);
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(r));
    qn_.store(q_.size(), std::memory_order_release);
  }
  if (!spinning_.load(std::memory_order_acquire)) cv_.notify_one();
}

void HbmBackend::set(const std::string&, const Digest& d, Bytes value, uint32_t flags,
                     uint32_t ttl_s) {
  if (!value || value->size() > cfg_.max_item) return;
  Req r;
  r.kind = 1;
  r.d = d;
  r.value = std::move(value);
  r.flags = flags;
  r.ttl = ttl_s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (cfg_.presence_filter) {
      filt_->add(d);
      if (filt_next_) filt_next_->add(d);
    }
    q_.push_back(std::move(r));
    qn_.store(q_.size(), std::memory_order_release);
  }
  if (!spinning_.load(std::memory_order_acquire)) cv_.notify_one();
}

void HbmBackend::del(const std::string&, const Digest& d, Executor* ex, DelCallback done) {
  Req r;
  r.kind = 2;
  r.d = d;
  r.ex = ex;
  r.dcb = std::move(done);
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(r));
    qn_.store(q_.size(), std::memory_order_release);
  }
  if (!spinning_.load(std::memory_order_acquire)) cv_.notify_one();
}

void HbmBackend::flush() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    flush_req_ = true;
  }
  cv_.notify_one();
}

void HbmBackend::loop() {
  std::vector<Req> batch;
  for (;;) {
    bool do_flush = false, rebuilding = false;
    // After a batch, poll the queue for up to spin_us before blocking: under steady
    // traffic the next request usually arrives within that window, and catching it here
    // saves the futex wake-up (the producer skips notify while we spin).
    if (cfg_.spin_us > 0 && qn_.load(std::memory_order_acquire) == 0) {
      spinning_.store(true, std::memory_order_release);
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(cfg_.spin_us);
      while (qn_.load(std::memory_order_acquire) == 0 && std::chrono::steady_clock::now() < until)
        __builtin_ia32_pause();
      spinning_.store(false, std::memory_order_release);
    }
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (cfg_.sweep_interval_s > 0) {
        // idle: expire TTL'd objects out of every shard's index now and then (the
        // FIFO log reclaims bytes by itself; expired entries are otherwise only
        // skipped lazily at lookup)
        if (!cv_.wait_for(lk, std::chrono::seconds(cfg_.sweep_interval_s),
                          [&] { return stop_ || !q_.empty() || flush_req_ || filt_want_rebuild_; })) {
          lk.unlock();
          try {
            sweep_all();
          } catch (const std::exception& e) {
            std::fprintf(stderr, "[shellac hbm] sweep failed: %s\n", e.what());
          }
          continue;
        }
      } else {
        cv_.wait(lk, [&] { return stop_ || !q_.empty() || flush_req_ || filt_want_rebuild_; });
      }
      if (stop_ && q_.empty()) return;
      // Natural batching: whatever queued while the previous batch ran goes now. An
      // optional linger (batch_us > 0) trades latency for bigger batches.
      if (cfg_.batch_us > 0) {
        const auto deadline =
            std::chrono::steady_clock::now() + std::chrono::microseconds(cfg_.batch_us);
        while (!stop_ && (int)q_.size() < cfg_.max_batch &&
               cv_.wait_until(lk, deadline) != std::cv_status::timeout) {
        }
      }
      if (filt_want_rebuild_) {
        // SETs queued from here on add to filt_next_; the ones already queued are in
        // `batch` and committed before finish_filter_rebuild() exports the shards' keys
        filt_next_ = std::make_shared<PresenceFilter>(filt_bits_);
        filt_want_rebuild_ = false;
        rebuilding = true;
      }
      batch.swap(q_);
      qn_.store(0, std::memory_order_release);
      do_flush = flush_req_;
      flush_req_ = false;
    }
    const double t0 = wall_s();
    try {
      if (do_flush)
        for (auto& d : devs_) {
          d->set_device();
          d->cache->flush(d->stream);
          HB_OK(hipStreamSynchronize(d->stream));
        }
      if (!batch.empty()) run_batch(batch);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "[shellac hbm] batch failed: %s\n", e.what());
      for (auto& r : batch) {
        if (r.kind == 0 && r.gcb) {
          auto cb = std::move(r.gcb);
          r.ex->post([cb]() { cb(false, CacheValue{}); });
        } else if (r.kind == 2 && r.dcb) {
          auto cb = std::move(r.dcb);
          r.ex->post([cb]() { cb(false); });
        }
      }
    }
    if (rebuilding) {
      try {
        finish_filter_rebuild();
      } catch (const std::exception& e) {
        std::fprintf(stderr, "[shellac hbm] presence filter rebuild failed: %s\n", e.what());
        std::lock_guard<std::mutex> lk(mu_);
        filt_next_.reset();
      }
    } else if (cfg_.presence_filter && filt_->adds() >= filt_rebuild_at_) {
      filt_want_rebuild_ = true;  // read under mu_ by the wait predicate next iteration
    }
    const uint64_t n = batch.size();
    if (n) {
      batches_++;
      batched_reqs_ += n;
      uint64_t prev = max_batch_seen_.load();
      while (n > prev && !max_batch_seen_.compare_exchange_weak(prev, n)) {
      }
      batch_ns_ += (uint64_t)((wall_s() - t0) * 1e9);
    }
    batch.clear();
  }
}

// Host slot the small-GET kernel signals completion through (this backend owns its
// HbmCache instances, so no other user shares the slot).
constexpr int kDoneSlot = HbmCache::kHostSlots - 1;

void HbmBackend::run_batch(std::vector<Req>& batch) {
  TraceRange tr("hbm_backend.batch");
  const size_t nd = devs_.size();
  const uint32_t tnow = now();
  std::vector<std::vector<size_t>> gets(nd), sets(nd), dels(nd);
  for (size_t i = 0; i < batch.size(); ++i) {
    const int o = nd == 1 ? 0 : ring_.owner(batch[i].d);
    (batch[i].kind == 0 ? gets : batch[i].kind == 1 ? sets : dels)[o].push_back(i);
  }
  // ---- GET: H2D keys, probe + scan, gather straight into pinned host memory (skipped
  // by the kernel if the batch does not fit), D2H offsets; one sync per device.
  // Coalesced on the host first: requests for the same digest in one batch (a hot
  // object under concurrent clients) share one GPU row, one copy over PCIe and one
  // CacheValue (the bytes are shared, as the DRAM tier shares them).
  std::vector<size_t> nuniq(nd, 0);
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n0 = gets[k].size();
    if (!n0) continue;
    dv.set_device();
    dv.ensure_n(std::max(n0, std::max(sets[k].size(), dels[k].size())));
    dv.ensure_out(1);
    size_t tsz = 16;
    while (tsz < 2 * n0) tsz <<= 1;
    dv.co_tab.assign(tsz, -1);
    dv.urow.resize(n0);
    size_t n = 0;
    for (size_t j = 0; j < n0; ++j) {
      const Digest& d = batch[gets[k][j]].d;
      for (size_t h = (size_t)(d.hi ^ (d.hi >> 31)) & (tsz - 1);; h = (h + 1) & (tsz - 1)) {
        const int32_t u = dv.co_tab[h];
        if (u < 0) {  // first request for this digest: it gets a GPU row
          dv.co_tab[h] = (int32_t)n;
          dv.h_keys[n] = d;
          dv.urow[j] = (uint32_t)n++;
          break;
        }
        if (dv.h_keys[u].lo == d.lo && dv.h_keys[u].hi == d.hi) {
          dv.urow[j] = (uint32_t)u;
          break;
        }
      }
    }
    nuniq[k] = n;
    coalesced_gets_ += n0 - n;
    if ((int64_t)n <= HbmCache::kSmallGetMax) {
      // one launch, no copies: keys, offsets and values all live in mapped host memory;
      // the kernel's last workgroup signals completion through a pinned host slot
      dv.cache->small_get(dv.h_keys_dev, (int64_t)n, dv.h_out_dev, dv.out_cap, dv.h_off_dev,
                          tnow, dv.stream, kDoneSlot);
      continue;
    }
    HB_OK(hipMemcpyAsync(dv.d_keys, dv.h_keys, n * sizeof(Digest), hipMemcpyHostToDevice, dv.stream));
    dv.cache->lookup(dv.d_keys, (int64_t)n, dv.d_loc, dv.d_size, dv.d_off, tnow, dv.stream);
    dv.cache->gather(dv.d_loc, dv.d_off, (int64_t)n, dv.h_out_dev, dv.stream, dv.out_cap);
    HB_OK(hipMemcpyAsync(dv.h_off, dv.d_off, (n + 1) * 8, hipMemcpyDeviceToHost, dv.stream));
  }
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n = nuniq[k];
    if (!n) continue;
    dv.set_device();
    const bool small = (int64_t)n <= HbmCache::kSmallGetMax;
    if (small)
      dv.cache->wait_host_slot(kDoneSlot, 10000);  // no stream sync on the hit path
    else
      HB_OK(hipStreamSynchronize(dv.stream));
    const uint64_t total = dv.h_off[n];
    if (total > dv.out_cap) {  // rare: grow the zero-copy buffer and gather again
      dv.ensure_out(total);
      if (small)
        dv.cache->small_get(dv.h_keys_dev, (int64_t)n, dv.h_out_dev, dv.out_cap, dv.h_off_dev,
                            tnow, dv.stream);
      else
        dv.cache->gather(dv.d_loc, dv.d_off, (int64_t)n, dv.h_out_dev, dv.stream, dv.out_cap);
      HB_OK(hipStreamSynchronize(dv.stream));
    }
  }
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n = nuniq[k];
    if (!n) continue;
    // one CacheValue per GPU row, shared by that row's requests
    dv.uval.assign(n, CacheValue{});
    dv.uhit.assign(n, 0);
    for (size_t u = 0; u < n; ++u) {
      const uint64_t o = dv.h_off[u], sz = dv.h_off[u + 1] - o;
      if (!sz) continue;
      ItemHeader h;
      std::memcpy(&h, dv.h_out + o, sizeof h);
      if (h.magic == kItemMagic && h.d0 == dv.h_keys[u].lo && h.d1 == dv.h_keys[u].hi) {
        dv.uhit[u] = 1;
        CacheValue& v = dv.uval[u];
        v.flags = h.flags;
        v.ttl_left = h.expire ? (int64_t)h.expire - (int64_t)tnow : 0;
        v.data = std::make_shared<const std::string>(
            reinterpret_cast<const char*>(dv.h_out + o + kItemHeaderBytes), h.vlen);
      }
    }
    for (size_t j = 0; j < gets[k].size(); ++j) {
      Req& r = batch[gets[k][j]];
      const uint32_t u = dv.urow[j];
      const bool hit = dv.uhit[u] != 0;
      CacheValue v = dv.uval[u];
      auto cb = std::move(r.gcb);
      r.ex->post([cb, hit, v]() { cb(hit, v); });
    }
  }
  // ---- SET. Micro-batches: pack into mapped staging padded to a size class (skip
  // rows); the SET kernels read it directly (no copies). SHELLAC_SET_GRAPH=1 replays a
  // captured hipGraph per class instead of launching the chain: measured slower on
  // ROCm 7 (52.8 vs 46.6 us per 64-row batch incl. sync, profiles/r1_small_get_latency.log),
  // so off by default. Larger batches: pinned staging, H2D, store.
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n = sets[k].size();
    if (!n) continue;
    dv.set_device();
    int cls = 0;
    while (cls < Dev::kSetClasses && Dev::kSetClass[cls] < (int64_t)n) ++cls;
    if (cls < Dev::kSetClasses) {
      const int64_t cn = Dev::kSetClass[cls];
      uint64_t bytes = 16;
      for (size_t idx : sets[k]) bytes += align_up(batch[idx].value->size(), 16);
      dv.ensure_set_staging(bytes);
      uint32_t* vl = dv.hs_meta;
      uint32_t* fl = dv.hs_meta + cn;
      uint32_t* ex = dv.hs_meta + 2 * cn;
      uint64_t off = 0;
      for (size_t j = 0; j < n; ++j) {
        const Req& r = batch[sets[k][j]];
        dv.hs_keys[j] = r.d;
        std::memcpy(dv.hs_vals + off, r.value->data(), r.value->size());
        dv.hs_voff[j] = off;
        vl[j] = (uint32_t)r.value->size();
        fl[j] = r.flags;
        ex[j] = r.ttl ? tnow + r.ttl : 0;
        off += align_up(r.value->size(), 16);
      }
      for (int64_t j = (int64_t)n; j < cn; ++j) {  // padding: rows the SET skips
        dv.hs_keys[j] = Digest{0, 0};
        dv.hs_voff[j] = 0;
        vl[j] = kSkipVlen;
        fl[j] = 0;
        ex[j] = 0;
      }
      // the bound only guards against batches over half the log: a class constant
      if (set_graphs_)
        dv.cache->store_graph(&dv.set_graph[cls], dv.hs_keys_dev, dv.hs_vals_dev,
                              dv.hs_voff_dev, dv.hs_meta_dev, dv.hs_meta_dev + cn,
                              dv.hs_meta_dev + 2 * cn, cn, dv.cache->config().log_bytes / 2,
                              tnow, dv.stream);
      else
        dv.cache->store(dv.hs_keys_dev, dv.hs_vals_dev, dv.hs_voff_dev, dv.hs_meta_dev,
                        dv.hs_meta_dev + cn, dv.hs_meta_dev + 2 * cn, cn,
                        dv.cache->config().log_bytes / 2, tnow, dv.stream);
      continue;
    }
    dv.ensure_n(n);
    uint64_t bytes = 16;
    for (size_t idx : sets[k]) bytes += align_up(batch[idx].value->size(), 16);
    dv.ensure_vals(bytes);
    uint64_t off = 0, bound = 0;
    uint32_t* vl = dv.h_meta;
    uint32_t* fl = dv.h_meta + n;
    uint32_t* ex = dv.h_meta + 2 * n;
    for (size_t j = 0; j < n; ++j) {
      const Req& r = batch[sets[k][j]];
      dv.h_keys[j] = r.d;
      std::memcpy(dv.h_vals + off, r.value->data(), r.value->size());
      dv.h_voff[j] = off;
      vl[j] = (uint32_t)r.value->size();
      fl[j] = r.flags;
      ex[j] = r.ttl ? tnow + r.ttl : 0;
      off += align_up(r.value->size(), 16);
      bound += item_bytes(vl[j]);
    }
    HB_OK(hipMemcpyAsync(dv.d_keys, dv.h_keys, n * sizeof(Digest), hipMemcpyHostToDevice, dv.stream));
    HB_OK(hipMemcpyAsync(dv.d_vals, dv.h_vals, off + 16, hipMemcpyHostToDevice, dv.stream));
    HB_OK(hipMemcpyAsync(dv.d_voff, dv.h_voff, n * 8, hipMemcpyHostToDevice, dv.stream));
    HB_OK(hipMemcpyAsync(dv.d_meta, dv.h_meta, n * 12, hipMemcpyHostToDevice, dv.stream));
    dv.cache->store(dv.d_keys, dv.d_vals, dv.d_voff, dv.d_meta, dv.d_meta + n, dv.d_meta + 2 * n,
                    (int64_t)n, bound, tnow, dv.stream);
  }
  // ---- DELETE
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n = dels[k].size();
    if (!n && sets[k].empty()) continue;  // GET-only batch: nothing left on the stream
    dv.set_device();
    if (n) {
      HB_OK(hipStreamSynchronize(dv.stream));  // staging reuse after SET
      dv.ensure_n(n);
      for (size_t j = 0; j < n; ++j) dv.h_keys[j] = batch[dels[k][j]].d;
      HB_OK(hipMemcpyAsync(dv.d_keys, dv.h_keys, n * sizeof(Digest), hipMemcpyHostToDevice, dv.stream));
      dv.cache->remove(dv.d_keys, (int64_t)n, dv.d_found, tnow, dv.stream);
      HB_OK(hipMemcpyAsync(dv.h_found, dv.d_found, n, hipMemcpyDeviceToHost, dv.stream));
    }
    HB_OK(hipStreamSynchronize(dv.stream));
    for (size_t j = 0; j < n; ++j) {
      Req& r = batch[dels[k][j]];
      const bool f = dv.h_found[j] != 0;
      auto cb = std::move(r.dcb);
      if (cb) r.ex->post([cb, f]() { cb(f); });
    }
  }
}

void HbmBackend::sweep_all() {
  TraceRange tr("hbm_backend.sweep");
  const uint32_t t = now();
  uint64_t objs = 0, bytes = 0;
  for (auto& d : devs_) {
    d->set_device();
    uint64_t o = 0, b = 0;
    d->cache->sweep(t, d->stream, &o, &b);
    objs += o;
    bytes += b;
  }
  live_objects_ = objs;
  live_bytes_ = bytes;
  sweeps_++;
}

void HbmBackend::finish_filter_rebuild() {
  TraceRange tr("hbm_backend.filter_rebuild");
  const uint32_t t = now();
  for (auto& d : devs_) {
    d->set_device();
    const uint64_t live = d->cache->export_keys(nullptr, 0, t, d->stream);
    if (!live) continue;
    // the kernel writes the digests straight into mapped host memory (no device buffer)
    Digest *h = nullptr, *hdev = nullptr;
    Dev::map_alloc(&h, &hdev, live * sizeof(Digest));
    uint64_t got = 0;
    try {
      got = std::min(live, d->cache->export_keys(hdev, live, t, d->stream));
    } catch (...) {
      (void)hipHostFree(h);
      throw;
    }
    for (uint64_t i = 0; i < got; ++i) filt_next_->add(h[i]);
    (void)hipHostFree(h);
  }
  std::lock_guard<std::mutex> lk(mu_);
  std::atomic_store(&filt_, filt_next_);
  filt_next_.reset();
  filt_rebuild_at_ = filt_->adds() + cfg_.nbuckets_per_gpu * kEntriesPerBucket * devs_.size();
  filt_rebuilds_++;
}

void HbmBackend::stats(StatList* out) {
  CacheCounters t{};
  uint64_t hbm = 0;
  for (auto& d : devs_) {
    d->set_device();
    const CacheCounters c = d->cache->counters(nullptr);
    t.get_ops += c.get_ops; t.get_hits += c.get_hits; t.set_ops += c.set_ops;
    t.set_bytes += c.set_bytes; t.set_evicted += c.set_evicted; t.del_ops += c.del_ops;
    hbm += d->cache->hbm_bytes();
  }
  out->emplace_back("cache_get_ops", t.get_ops);
  out->emplace_back("cache_get_hits", t.get_hits);
  out->emplace_back("cache_set_ops", t.set_ops);
  out->emplace_back("cache_set_bytes", t.set_bytes);
  out->emplace_back("cache_evicted", t.set_evicted);
  out->emplace_back("hbm_gpus", devs_.size());
  out->emplace_back("hbm_bytes", hbm);
  out->emplace_back("hbm_batches", batches_.load());
  out->emplace_back("hbm_batched_requests", batched_reqs_.load());
  out->emplace_back("hbm_max_batch", max_batch_seen_.load());
  out->emplace_back("hbm_batch_ns_total", batch_ns_.load());
  out->emplace_back("hbm_sweeps", sweeps_.load());
  uint64_t gl = 0, gc = 0;
  for (auto& d : devs_)
    for (auto& g : d->set_graph) {
      gl += g.launches;
      gc += g.captures;
    }
  out->emplace_back("hbm_set_graph_launches", gl);
  out->emplace_back("hbm_set_graph_captures", gc);
  out->emplace_back("hbm_live_objects", live_objects_.load());
  out->emplace_back("hbm_live_bytes", live_bytes_.load());
  out->emplace_back("hbm_coalesced_gets", coalesced_gets_.load());
  if (cfg_.presence_filter) {
    const auto f = std::atomic_load(&filt_);
    out->emplace_back("hbm_filter_skips", filt_skips_.load());
    out->emplace_back("hbm_filter_rebuilds", filt_rebuilds_.load());
    out->emplace_back("hbm_filter_adds", f->adds());
    out->emplace_back("hbm_filter_fill_ppm", (uint64_t)(f->fill() * 1e6));
  }
}

}  // namespace shellac
