// Cache backends: DRAM (striped host shards), HBM (batched HIP pipeline per GPU),
// memcached binary protocol client (ketama, pipelined, ejection + retry).
#include "backend.h"

#include <sys/epoll.h>
#include <sys/eventfd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "hbm_cache.h"
#include "mcproto.h"

namespace shellac {

namespace {
double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

// =====================================================================================
// DigestRing
// =====================================================================================
DigestRing::DigestRing(int nshards, int pps) {
  for (int i = 0; i < nshards; ++i)
    for (int j = 0; j < pps; ++j) {
      const std::string s = "shellac-shard-" + std::to_string(i) + "-" + std::to_string(j);
      const Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(s.data()), s.size());
      pts_.emplace_back((uint32_t)(d.hi >> 32), i);
    }
  std::stable_sort(pts_.begin(), pts_.end(),
                   [](const std::pair<uint32_t, int>& a, const std::pair<uint32_t, int>& b) {
                     return a.first < b.first;
                   });
}

int DigestRing::owner(const Digest& d) const {
  if (pts_.empty()) return 0;
  const uint32_t p = ring_position(d);
  auto it = std::lower_bound(pts_.begin(), pts_.end(), p,
                             [](const std::pair<uint32_t, int>& a, uint32_t v) { return a.first < v; });
  return it == pts_.end() ? pts_.front().second : it->second;
}

// =====================================================================================
// DRAM
// =====================================================================================
DramBackend::DramBackend(uint64_t bytes, uint32_t max_item, int stripes) : epoch_(wall_s()) {
  SH_CHECK(stripes > 0, "stripes");
  const uint64_t per = std::max<uint64_t>(bytes / stripes / 16 * 16, 1ull << 20);
  // ~1 KiB average objects at <= 50% slot load
  uint64_t nb = 2;
  while (nb * 4 * 512 < per) nb *= 2;
  const uint32_t mi = (uint32_t)std::min<uint64_t>(max_item, per / 4);
  for (int i = 0; i < stripes; ++i) shards_.emplace_back(new HostCache(per, nb, mi));
}

uint32_t DramBackend::now() const { return (uint32_t)(wall_s() - epoch_) + 1; }

void DramBackend::get(const std::string&, const Digest& d, Executor*, GetCallback done) {
  std::vector<uint8_t> v;
  uint32_t flags = 0, expire = 0;
  const uint32_t t = now();
  if (shard(d).get_one(d, &v, &flags, t, &expire)) {
    done(true, CacheValue{std::make_shared<const std::string>(v.begin(), v.end()), flags,
                          expire ? (int64_t)expire - t : 0});
  } else {
    done(false, CacheValue{});
  }
}

void DramBackend::set(const std::string&, const Digest& d, Bytes value, uint32_t flags,
                      uint32_t ttl_s) {
  if (!value) return;
  const uint32_t n = now();
  shard(d).set_one(d, reinterpret_cast<const uint8_t*>(value->data()), (uint32_t)value->size(),
                   flags, ttl_s ? n + ttl_s : 0, n);
}

void DramBackend::del(const std::string&, const Digest& d, Executor*, DelCallback done) {
  uint8_t found = 0;
  shard(d).remove(&d, 1, &found, now());
  if (done) done(found != 0);
}

void DramBackend::flush() {
  for (auto& s : shards_) s->flush();
}

void DramBackend::stats(StatList* out) {
  CacheCounters t{};
  for (auto& s : shards_) {
    const CacheCounters c = s->counters();
    t.get_ops += c.get_ops; t.get_hits += c.get_hits; t.set_ops += c.set_ops;
    t.set_bytes += c.set_bytes; t.set_evicted += c.set_evicted; t.del_ops += c.del_ops;
  }
  out->emplace_back("cache_get_ops", t.get_ops);
  out->emplace_back("cache_get_hits", t.get_hits);
  out->emplace_back("cache_set_ops", t.set_ops);
  out->emplace_back("cache_set_bytes", t.set_bytes);
  out->emplace_back("cache_evicted", t.set_evicted);
  out->emplace_back("cache_shards", shards_.size());
}

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
  uint64_t *d_loc = nullptr, *d_size = nullptr, *d_off = nullptr, *h_off = nullptr;
  uint8_t *d_out = nullptr, *h_out = nullptr;
  uint8_t *d_vals = nullptr, *h_vals = nullptr;
  uint64_t *d_voff = nullptr, *h_voff = nullptr;
  uint32_t *d_meta = nullptr, *h_meta = nullptr;  // [vlen | flags | expire] x n
  uint8_t *d_found = nullptr, *h_found = nullptr;

  void set_device() { HB_OK(hipSetDevice(device)); }

  void ensure_n(size_t n) {
    if (n <= n_cap) return;
    size_t cap = n_cap ? n_cap : 1024;
    while (cap < n) cap *= 2;
    HB_OK(hipStreamSynchronize(stream));
    (void)hipFree(d_keys); (void)hipHostFree(h_keys); (void)hipFree(d_loc); (void)hipFree(d_size);
    (void)hipFree(d_off); (void)hipHostFree(h_off); (void)hipFree(d_voff); (void)hipHostFree(h_voff);
    (void)hipFree(d_meta); (void)hipHostFree(h_meta); (void)hipFree(d_found); (void)hipHostFree(h_found);
    HB_OK(hipMalloc(&d_keys, cap * sizeof(Digest)));
    HB_OK(hipHostMalloc(&h_keys, cap * sizeof(Digest), hipHostMallocDefault));
    HB_OK(hipMalloc(&d_loc, cap * 8));
    HB_OK(hipMalloc(&d_size, (cap + 1) * 8));
    HB_OK(hipMalloc(&d_off, (cap + 1) * 8));
    HB_OK(hipHostMalloc(&h_off, (cap + 1) * 8, hipHostMallocDefault));
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
    size_t cap = out_cap ? out_cap : (1u << 20);
    while (cap < bytes) cap *= 2;
    HB_OK(hipStreamSynchronize(stream));
    (void)hipFree(d_out); (void)hipHostFree(h_out);
    HB_OK(hipMalloc(&d_out, cap));
    HB_OK(hipHostMalloc(&h_out, cap, hipHostMallocDefault));
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
    (void)hipFree(d_off); (void)hipHostFree(h_off); (void)hipFree(d_out); (void)hipHostFree(h_out);
    (void)hipFree(d_vals); (void)hipHostFree(h_vals); (void)hipFree(d_voff); (void)hipHostFree(h_voff);
    (void)hipFree(d_meta); (void)hipHostFree(h_meta); (void)hipFree(d_found); (void)hipHostFree(h_found);
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
  Req r;
  r.kind = 0;
  r.d = d;
  r.ex = ex;
  r.gcb = std::move(done);
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(r));
  }
  cv_.notify_one();
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
    q_.push_back(std::move(r));
  }
  cv_.notify_one();
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
  }
  cv_.notify_one();
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
    bool do_flush = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !q_.empty() || flush_req_; });
      if (stop_ && q_.empty()) return;
      // give batch-mates up to batch_us to arrive (a lone request pays at most that)
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(cfg_.batch_us);
      while (!stop_ && (int)q_.size() < cfg_.max_batch &&
             cv_.wait_until(lk, deadline) != std::cv_status::timeout) {
      }
      batch.swap(q_);
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

void HbmBackend::run_batch(std::vector<Req>& batch) {
  const size_t nd = devs_.size();
  const uint32_t tnow = now();
  std::vector<std::vector<size_t>> gets(nd), sets(nd), dels(nd);
  for (size_t i = 0; i < batch.size(); ++i) {
    const int o = nd == 1 ? 0 : ring_.owner(batch[i].d);
    (batch[i].kind == 0 ? gets : batch[i].kind == 1 ? sets : dels)[o].push_back(i);
  }
  // ---- GET phase 1: H2D keys, probe + scan, D2H offsets (all devices in flight)
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n = gets[k].size();
    if (!n) continue;
    dv.set_device();
    dv.ensure_n(std::max(n, std::max(sets[k].size(), dels[k].size())));
    for (size_t j = 0; j < n; ++j) dv.h_keys[j] = batch[gets[k][j]].d;
    HB_OK(hipMemcpyAsync(dv.d_keys, dv.h_keys, n * sizeof(Digest), hipMemcpyHostToDevice, dv.stream));
    dv.cache->lookup(dv.d_keys, (int64_t)n, dv.d_loc, dv.d_size, dv.d_off, tnow, dv.stream);
    HB_OK(hipMemcpyAsync(dv.h_off, dv.d_off, (n + 1) * 8, hipMemcpyDeviceToHost, dv.stream));
  }
  // ---- GET phase 2: gather + D2H values
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n = gets[k].size();
    if (!n) continue;
    dv.set_device();
    HB_OK(hipStreamSynchronize(dv.stream));
    const uint64_t total = dv.h_off[n];
    if (total) {
      dv.ensure_out(total);
      dv.cache->gather(dv.d_loc, dv.d_off, (int64_t)n, dv.d_out, dv.stream);
      HB_OK(hipMemcpyAsync(dv.h_out, dv.d_out, total, hipMemcpyDeviceToHost, dv.stream));
    }
  }
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n = gets[k].size();
    if (!n) continue;
    dv.set_device();
    HB_OK(hipStreamSynchronize(dv.stream));
    for (size_t j = 0; j < n; ++j) {
      Req& r = batch[gets[k][j]];
      const uint64_t o = dv.h_off[j], sz = dv.h_off[j + 1] - o;
      bool hit = false;
      CacheValue v;
      if (sz) {
        ItemHeader h;
        std::memcpy(&h, dv.h_out + o, sizeof h);
        if (h.magic == kItemMagic && h.d0 == r.d.lo && h.d1 == r.d.hi) {
          hit = true;
          v.flags = h.flags;
          v.ttl_left = h.expire ? (int64_t)h.expire - (int64_t)tnow : 0;
          v.data = std::make_shared<const std::string>(
              reinterpret_cast<const char*>(dv.h_out + o + kItemHeaderBytes), h.vlen);
        }
      }
      auto cb = std::move(r.gcb);
      r.ex->post([cb, hit, v]() { cb(hit, v); });
    }
  }
  // ---- SET: pack 16-aligned payloads in pinned staging, H2D, store
  for (size_t k = 0; k < nd; ++k) {
    Dev& dv = *devs_[k];
    const size_t n = sets[k].size();
    if (!n) continue;
    dv.set_device();
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
}

// =====================================================================================
// Tiered (L1 DRAM + L2)
// =====================================================================================
TieredBackend::TieredBackend(std::shared_ptr<CacheBackend> l1, std::shared_ptr<CacheBackend> l2,
                             uint32_t promote_ttl_s)
    : l1_(std::move(l1)), l2_(std::move(l2)), promote_ttl_(promote_ttl_s) {
  SH_CHECK(l1_ && l2_, "tiered backend needs two levels");
}

void TieredBackend::get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) {
  auto l2 = l2_;
  auto l1 = l1_;
  const uint32_t pttl = promote_ttl_;
  l1_->get(key, d, ex, [this, key, d, ex, done, l1, l2, pttl](bool hit, CacheValue v) {
    if (hit) {
      l1_hits_++;
      done(true, std::move(v));
      return;
    }
    l2->get(key, d, ex, [this, key, d, done, l1, pttl](bool hit2, CacheValue v2) {
      if (hit2 && v2.data) {
        l2_hits_++;
        if (v2.ttl_left > 0 || v2.ttl_left == 0 || v2.ttl_left == -1) {
          const uint32_t ttl = v2.ttl_left > 0 ? (uint32_t)v2.ttl_left
                                               : (v2.ttl_left == 0 ? 0u : pttl);
          l1->set(key, d, v2.data, v2.flags, ttl);  // promote
        }
      } else {
        misses_++;
      }
      done(hit2, std::move(v2));
    });
  });
}

void TieredBackend::set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
                        uint32_t ttl_s) {
  l2_->set(key, d, value, flags, ttl_s);
  l1_->set(key, d, std::move(value), flags, ttl_s);
}

void TieredBackend::del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) {
  auto l2 = l2_;
  l1_->del(key, d, ex, [key, d, ex, done, l2](bool f1) {
    l2->del(key, d, ex, [done, f1](bool f2) {
      if (done) done(f1 || f2);
    });
  });
}

void TieredBackend::flush() {
  l1_->flush();
  l2_->flush();
}

void TieredBackend::stats(StatList* out) {
  out->emplace_back("tier_l1_hits", l1_hits_.load());
  out->emplace_back("tier_l2_hits", l2_hits_.load());
  out->emplace_back("tier_misses", misses_.load());
  StatList a, b;
  l1_->stats(&a);
  l2_->stats(&b);
  for (auto& kv : a) out->emplace_back("l1_" + kv.first, kv.second);
  for (auto& kv : b) out->emplace_back("l2_" + kv.first, kv.second);
}

// =====================================================================================
// memcached binary client
// =====================================================================================
struct MemcachedBackend::Node {
  Addr addr;
  int fd = -1;
  bool connected = false;
  double down_until = 0;
  std::string out;
  size_t out_off = 0;
  std::string in;
  uint32_t next_opaque = 1;
  std::deque<std::pair<uint32_t, Pending>> pending;
};

std::string MemcachedBackend::wire_key(const std::string& key) {
  bool ok = key.size() <= 250 && !key.empty();
  for (unsigned char c : key)
    if (c <= 32 || c == 127) { ok = false; break; }
  return ok ? key : "shellac:" + md5_hex(key);
}

MemcachedBackend::MemcachedBackend(const MemcachedConfig& cfg) : cfg_(cfg) {
  SH_CHECK(!cfg_.servers.empty(), "no memcached servers");
  std::vector<KetamaRing::Node> nodes;
  for (const auto& a : cfg_.servers) {
    auto n = std::make_unique<Node>();
    n->addr = a;
    nodes_.push_back(std::move(n));
    nodes.push_back(KetamaRing::Node{a.str(), 1, true});
  }
  ring_ = KetamaRing(nodes);
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = ~0ull;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
  th_ = std::thread([this] { loop(); });
}

MemcachedBackend::~MemcachedBackend() {
  stop_ = true;
  uint64_t one = 1;
  (void)!write(evfd_, &one, 8);
  if (th_.joinable()) th_.join();
  for (auto& n : nodes_)
    if (n->fd >= 0) close(n->fd);
  close(epfd_);
  close(evfd_);
}

void MemcachedBackend::submit(Cmd c) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    inbox_.push_back(std::move(c));
  }
  uint64_t one = 1;
  (void)!write(evfd_, &one, 8);
}

void MemcachedBackend::get(const std::string& key, const Digest&, Executor* ex, GetCallback done) {
  gets_++;
  submit(Cmd{key, mc::GET, nullptr, 0, 0, ex, std::move(done), nullptr});
}

void MemcachedBackend::set(const std::string& key, const Digest&, Bytes value, uint32_t flags,
                           uint32_t ttl_s) {
  sets_++;
  submit(Cmd{key, mc::SET, std::move(value), flags, ttl_s, nullptr, nullptr, nullptr});
}

void MemcachedBackend::del(const std::string& key, const Digest&, Executor* ex, DelCallback done) {
  submit(Cmd{key, mc::DELETE, nullptr, 0, 0, ex, nullptr, std::move(done)});
}

void MemcachedBackend::flush() {
  for (size_t i = 0; i < nodes_.size(); ++i)
    submit(Cmd{std::string("\x01node") + std::to_string(i), mc::FLUSH, nullptr, 0, 0, nullptr,
               nullptr, nullptr});
}

void MemcachedBackend::node_fail(int idx) {
  Node& n = *nodes_[idx];
  if (n.fd >= 0) {
    epoll_ctl(epfd_, EPOLL_CTL_DEL, n.fd, nullptr);
    close(n.fd);
  }
  n.fd = -1;
  n.connected = false;
  n.out.clear();
  n.out_off = 0;
  n.in.clear();
  errors_++;
  ejections_++;
  n.down_until = wall_s() + cfg_.retry_timeout_s;
  ring_.set_alive(idx, false);  // keys remap to the remaining nodes (ketama auto-eject)
  for (auto& p : n.pending) {
    Pending& q = p.second;
    if (q.gcb) {
      auto cb = std::move(q.gcb);
      q.ex->post([cb]() { cb(false, CacheValue{}); });
    } else if (q.dcb) {
      auto cb = std::move(q.dcb);
      q.ex->post([cb]() { cb(false); });
    }
  }
  n.pending.clear();
}

void MemcachedBackend::drain_commands() {
  std::vector<Cmd> cmds;
  {
    std::lock_guard<std::mutex> lk(mu_);
    cmds.swap(inbox_);
  }
  const double t = wall_s();
  for (size_t i = 0; i < nodes_.size(); ++i)  // re-admit ejected nodes after retry timeout
    if (!ring_.node(i).alive && t >= nodes_[i]->down_until) ring_.set_alive(i, true);
  for (auto& c : cmds) {
    int idx;
    if (c.op == mc::FLUSH && !c.key.empty() && c.key[0] == '\x01') {
      idx = std::stoi(c.key.substr(5));
      if (!ring_.node(idx).alive) continue;
    } else {
      idx = ring_.pick(wire_key(c.key));
    }
    if (idx < 0) {  // every node down: fail fast
      if (c.gcb) c.ex->post([cb = std::move(c.gcb)]() { cb(false, CacheValue{}); });
      if (c.dcb) c.ex->post([cb = std::move(c.dcb)]() { cb(false); });
      continue;
    }
    Node& n = *nodes_[idx];
    if (n.fd < 0) {
      n.fd = connect_nonblock(n.addr);
      if (n.fd < 0) {
        node_fail(idx);
        if (c.gcb) c.ex->post([cb = std::move(c.gcb)]() { cb(false, CacheValue{}); });
        if (c.dcb) c.ex->post([cb = std::move(c.dcb)]() { cb(false); });
        continue;
      }
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
      ev.data.u64 = (uint64_t)idx;
      epoll_ctl(epfd_, EPOLL_CTL_ADD, n.fd, &ev);
    }
    const uint32_t op = n.next_opaque++;
    const std::string k = c.op == mc::FLUSH ? std::string() : wire_key(c.key);
    if (c.op == mc::GET) {
      mc::request(n.out, mc::GET, k, "", nullptr, 0, op);
    } else if (c.op == mc::SET) {
      mc::request(n.out, mc::SET, k, mc::set_extras(c.flags, c.ttl), c.value->data(),
                  c.value->size(), op);
    } else if (c.op == mc::DELETE) {
      mc::request(n.out, mc::DELETE, k, "", nullptr, 0, op);
    } else {
      mc::request(n.out, mc::FLUSH, "", "", nullptr, 0, op);
    }
    n.pending.emplace_back(op, Pending{c.op, c.ex, std::move(c.gcb), std::move(c.dcb), t});
  }
  for (size_t i = 0; i < nodes_.size(); ++i) {  // try to write immediately
    Node& n = *nodes_[i];
    if (n.fd < 0 || !n.connected || n.out_off >= n.out.size()) continue;
    const ssize_t w = send(n.fd, n.out.data() + n.out_off, n.out.size() - n.out_off, MSG_NOSIGNAL);
    if (w > 0) n.out_off += (size_t)w;
    if (n.out_off == n.out.size()) { n.out.clear(); n.out_off = 0; }
  }
}

void MemcachedBackend::loop() {
  epoll_event evs[64];
  char buf[65536];
  while (!stop_) {
    const int k = epoll_wait(epfd_, evs, 64, 50);
    for (int e = 0; e < k; ++e) {
      if (evs[e].data.u64 == ~0ull) {
        uint64_t v;
        (void)!read(evfd_, &v, 8);
        continue;
      }
      const int idx = (int)evs[e].data.u64;
      Node& n = *nodes_[idx];
      if (n.fd < 0) continue;
      if (evs[e].events & (EPOLLERR | EPOLLHUP)) { node_fail(idx); continue; }
      if (evs[e].events & EPOLLOUT) {
        if (!n.connected) {
          int err = 0;
          socklen_t el = sizeof err;
          getsockopt(n.fd, SOL_SOCKET, SO_ERROR, &err, &el);
          if (err) { node_fail(idx); continue; }
          n.connected = true;
        }
        while (n.out_off < n.out.size()) {
          const ssize_t w = send(n.fd, n.out.data() + n.out_off, n.out.size() - n.out_off, MSG_NOSIGNAL);
          if (w <= 0) break;
          n.out_off += (size_t)w;
        }
        if (n.out_off >= n.out.size()) { n.out.clear(); n.out_off = 0; }
      }
      if (evs[e].events & (EPOLLIN | EPOLLRDHUP)) {
        bool dead = false;
        for (;;) {
          const ssize_t r = recv(n.fd, buf, sizeof buf, 0);
          if (r > 0) { n.in.append(buf, (size_t)r); continue; }
          if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) dead = true;
          break;
        }
        size_t pos = 0;
        mc::Frame f;
        while (size_t used = mc::next_frame(reinterpret_cast<const uint8_t*>(n.in.data()) + pos,
                                            n.in.size() - pos, &f)) {
          pos += used;
          // responses arrive in request order; skip any stale opaques
          while (!n.pending.empty() && n.pending.front().first != f.h.opaque) {
            Pending& q = n.pending.front().second;
            if (q.gcb) q.ex->post([cb = std::move(q.gcb)]() { cb(false, CacheValue{}); });
            n.pending.pop_front();
          }
          if (n.pending.empty()) continue;
          Pending q = std::move(n.pending.front().second);
          n.pending.pop_front();
          if (q.op == mc::GET && q.gcb) {
            if (f.h.status == mc::OK) {
              hits_++;
              CacheValue v;
              v.flags = f.h.extlen >= 4 ? mc::get32(f.extras) : 0;
              v.data = std::make_shared<const std::string>((const char*)f.value, f.vlen);
              q.ex->post([cb = std::move(q.gcb), v]() { cb(true, v); });
            } else {
              q.ex->post([cb = std::move(q.gcb)]() { cb(false, CacheValue{}); });
            }
          } else if (q.op == mc::DELETE && q.dcb) {
            const bool ok = f.h.status == mc::OK;
            q.ex->post([cb = std::move(q.dcb), ok]() { cb(ok); });
          }
        }
        if (pos) n.in.erase(0, pos);
        if (dead) node_fail(idx);
      }
      if (n.fd >= 0) {
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLRDHUP | (n.out_off < n.out.size() || !n.connected ? EPOLLOUT : 0);
        ev.data.u64 = (uint64_t)idx;
        epoll_ctl(epfd_, EPOLL_CTL_MOD, n.fd, &ev);
      }
    }
    drain_commands();
    // op timeouts: a node that stops answering is ejected
    const double t = wall_s();
    for (size_t i = 0; i < nodes_.size(); ++i) {
      Node& n = *nodes_[i];
      if (n.fd >= 0 && !n.pending.empty() &&
          t - n.pending.front().second.t0 > cfg_.op_timeout_ms / 1000.0)
        node_fail((int)i);
    }
    for (size_t i = 0; i < nodes_.size(); ++i) {
      Node& n = *nodes_[i];
      if (n.fd >= 0 && (n.out_off < n.out.size() || !n.connected)) {
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLRDHUP | EPOLLOUT;
        ev.data.u64 = (uint64_t)i;
        epoll_ctl(epfd_, EPOLL_CTL_MOD, n.fd, &ev);
      }
    }
  }
}

void MemcachedBackend::stats(StatList* out) {
  out->emplace_back("cache_get_ops", gets_.load());
  out->emplace_back("cache_get_hits", hits_.load());
  out->emplace_back("cache_set_ops", sets_.load());
  out->emplace_back("memcached_errors", errors_.load());
  out->emplace_back("memcached_ejections", ejections_.load());
  out->emplace_back("memcached_nodes", nodes_.size());
}

}  // namespace shellac
