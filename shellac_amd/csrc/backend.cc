// Cache backends: DRAM (striped host shards), tiered L1/L2, memcached binary protocol
// client (ketama, pipelined, ejection + retry). The HBM backend (HIP) is in
// backend_hbm.cc so these host-only backends also build without ROCm (sanitizer presets).
#include "backend.h"

#include <sys/epoll.h>
#include <sys/eventfd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "keyed.h"
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

int DigestRing::owner(const Digest& d, uint64_t alive) const {
  if (pts_.empty() || !alive) return -1;
  const uint32_t p = ring_position(d);
  size_t i = std::lower_bound(pts_.begin(), pts_.end(), p,
                              [](const std::pair<uint32_t, int>& a, uint32_t v) {
                                return a.first < v;
                              }) - pts_.begin();
  for (size_t k = 0; k < pts_.size(); ++k) {  // next point of a live shard (wrapping)
    const int o = pts_[(i + k) % pts_.size()].second;
    if ((alive >> o) & 1) return o;
  }
  return -1;
}

// =====================================================================================
// DRAM
// =====================================================================================
DramBackend::DramBackend(uint64_t bytes, uint32_t max_item, int stripes)
    : cache_(bytes, max_item, stripes), epoch_(wall_s()) {}

uint32_t DramBackend::now() const { return (uint32_t)(wall_s() - epoch_) + 1; }

void DramBackend::get(const std::string& key, const Digest& d, Executor*, GetCallback done) {
  const uint32_t t = now();
  CacheValue v;
  uint32_t expire = 0;
  if (cache_.get(key, d, t, &v.data, &v.flags, &expire)) {
    v.ttl_left = expire ? (int64_t)expire - t : 0;
    done(true, std::move(v));
  } else {
    done(false, CacheValue{});
  }
}

void DramBackend::set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
                      uint32_t ttl_s) {
  if (!value) return;
  const uint32_t n = now();
  cache_.set(key, d, value->data(), value->size(), flags, ttl_s ? n + ttl_s : 0, n);
}

void DramBackend::del(const std::string& key, const Digest& d, Executor*, DelCallback done) {
  const bool found = cache_.del(key, d, now());
  if (done) done(found);
}

void DramBackend::flush() { cache_.clear(); }

void DramBackend::stats(StatList* out) {
  const ObjectCacheStats t = cache_.stats();
  out->emplace_back("cache_get_ops", t.gets);
  out->emplace_back("cache_get_hits", t.hits);
  out->emplace_back("cache_set_ops", t.sets);
  out->emplace_back("cache_evicted", t.evictions);
  out->emplace_back("cache_expired", t.expired);
  out->emplace_back("cache_objects", t.objects);
  out->emplace_back("cache_bytes", t.bytes);
  out->emplace_back("cache_key_mismatch", t.key_mismatch);
}

// =====================================================================================
// Tiered (L1 DRAM + L2)
// =====================================================================================
TieredBackend::TieredBackend(std::shared_ptr<CacheBackend> l1, std::shared_ptr<CacheBackend> l2,
                             uint32_t promote_ttl_s, uint64_t promote_max)
    : l1_(std::move(l1)), l2_(std::move(l2)), promote_ttl_(promote_ttl_s),
      promote_max_(promote_max) {
  SH_CHECK(l1_ && l2_, "tiered backend needs two levels");
}

void TieredBackend::get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) {
  // Raw level pointers in the callbacks: the levels live as long as this object, which
  // (like `this` below) must outlive its requests. Copying the shared_ptrs per request
  // made every reactor thread bump the same two reference counts (c=10 hit path:
  // 666K -> see docs/PERF.md).
  CacheBackend* l2 = l2_.get();
  l1_->get(key, d, ex, [this, key, d, ex, l2, done = std::move(done)](bool hit,
                                                                      CacheValue v) mutable {
    if (hit) {
      l1_hits_.fetch_add(1, std::memory_order_relaxed);
      done(true, std::move(v));
      return;
    }
    l2->get(key, d, ex, [this, key, d, done = std::move(done)](bool hit2, CacheValue v2) {
      if (hit2 && v2.data) {
        l2_hits_.fetch_add(1, std::memory_order_relaxed);
        if (v2.data->size() <= promote_max_) {
          // promote with the L2 entry's remaining TTL (0 = no expiry, -1 = unknown)
          const uint32_t ttl = v2.ttl_left > 0 ? (uint32_t)v2.ttl_left
                                               : (v2.ttl_left == 0 ? 0u : promote_ttl_);
          l1_->set(key, d, v2.data, v2.flags, ttl);
          promoted_.fetch_add(1, std::memory_order_relaxed);
        } else {
          not_promoted_.fetch_add(1, std::memory_order_relaxed);
        }
      } else {
        misses_.fetch_add(1, std::memory_order_relaxed);
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
  out->emplace_back("tier_promoted", promoted_.load());
  out->emplace_back("tier_not_promoted_large", not_promoted_.load());
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

// =====================================================================================
// Fault injection
// =====================================================================================
FaultSpec parse_fault_spec(const std::string& spec) {
  FaultSpec f;
  size_t i = 0;
  while (i < spec.size()) {
    size_t j = spec.find(',', i);
    if (j == std::string::npos) j = spec.size();
    const std::string kv = spec.substr(i, j - i);
    i = j + 1;
    if (kv.empty()) continue;
    const size_t eq = kv.find('=');
    const std::string k = kv.substr(0, eq);
    const std::string v = eq == std::string::npos ? "" : kv.substr(eq + 1);
    if (k == "get_miss") f.get_miss = std::stod(v);
    else if (k == "set_drop") f.set_drop = std::stod(v);
    else if (k == "delay_us") f.delay_us = (uint32_t)std::stoul(v);
    else if (k == "down") f.down = v.empty() || v == "1" || v == "true";
    else if (k == "gpu_down") f.gpu_down = std::stoi(v);
    else throw Error("unknown fault '" + k + "' (get_miss, set_drop, delay_us, down, gpu_down)");
  }
  return f;
}

FaultBackend::FaultBackend(std::shared_ptr<CacheBackend> inner, const FaultSpec& spec,
                           uint64_t seed)
    : inner_(std::move(inner)), spec_(FaultSpec{}), rng_(seed * 0x9E3779B97F4A7C15ull + 1) {
  th_ = std::thread([this] { timer_loop(); });
  set_spec(spec);
}

FaultBackend::~FaultBackend() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
}

void FaultBackend::set_spec(const FaultSpec& spec) {
  int old_gpu;
  {
    std::lock_guard<std::mutex> lk(mu_);
    old_gpu = spec_.gpu_down;
    spec_ = spec;
  }
  // gpu_down=K: the GPU tier's shard K is ejected as if it had failed (and restored,
  // flushed, when the drill is lifted)
  if (old_gpu != spec.gpu_down) {
    if (old_gpu >= 0) inner_->inject_shard_down(old_gpu, false);
    if (spec.gpu_down >= 0 && !inner_->inject_shard_down(spec.gpu_down, true))
      throw Error("gpu_down: the cache tier has no GPU shard " + std::to_string(spec.gpu_down));
  }
}

bool FaultBackend::inject_shard_down(int shard, bool down) {
  return inner_->inject_shard_down(shard, down);
}

bool TieredBackend::inject_shard_down(int shard, bool down) {
  return l2_->inject_shard_down(shard, down);
}

FaultSpec FaultBackend::spec() const {
  std::lock_guard<std::mutex> lk(mu_);
  return spec_;
}

bool FaultBackend::roll(double p) {
  if (p <= 0) return false;
  if (p >= 1) return true;
  std::lock_guard<std::mutex> lk(mu_);
  rng_ ^= rng_ << 13;
  rng_ ^= rng_ >> 7;
  rng_ ^= rng_ << 17;
  return (double)(rng_ >> 11) * (1.0 / 9007199254740992.0) < p;
}

void FaultBackend::later(std::function<void()> fn) {
  const FaultSpec f = spec();
  if (!f.delay_us) {
    fn();
    return;
  }
  injected_delay_++;
  {
    std::lock_guard<std::mutex> lk(mu_);
    timers_.emplace_back(wall_s() + f.delay_us * 1e-6, std::move(fn));
  }
  cv_.notify_one();
}

void FaultBackend::timer_loop() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    if (stop_) break;
    if (timers_.empty()) {
      cv_.wait(lk);
      continue;
    }
    const double due = timers_.front().first, t = wall_s();
    if (due > t) {
      // system_clock deadline: libstdc++ maps steady-clock waits to pthread_cond_clockwait,
      // which ThreadSanitizer does not intercept (false reports under the tsan preset)
      cv_.wait_until(lk, std::chrono::system_clock::now() +
                             std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                 std::chrono::duration<double>(due - t)));
      continue;
    }
    auto fn = std::move(timers_.front().second);
    timers_.pop_front();
    lk.unlock();
    fn();
    lk.lock();
  }
  // run what is left so no caller waits forever
  while (!timers_.empty()) {
    auto fn = std::move(timers_.front().second);
    timers_.pop_front();
    lk.unlock();
    fn();
    lk.lock();
  }
}

void FaultBackend::get(const std::string& key, const Digest& d, Executor* ex, GetCallback done) {
  const FaultSpec f = spec();
  if (f.down || roll(f.get_miss)) {
    injected_miss_++;
    if (!f.delay_us) {
      done(false, CacheValue{});
      return;
    }
    later([ex, done] {
      if (ex) ex->post([done] { done(false, CacheValue{}); });
      else done(false, CacheValue{});
    });
    return;
  }
  if (!f.delay_us) {
    inner_->get(key, d, ex, std::move(done));
    return;
  }
  // the delayed lookup runs from the timer thread; a synchronous tier would answer
  // right there, so the answer is always handed back to `ex`
  later([this, key, d, ex, done] {
    inner_->get(key, d, ex, [ex, done](bool hit, CacheValue v) {
      if (ex) ex->post([done, hit, v] { done(hit, v); });
      else done(hit, v);
    });
  });
}

void FaultBackend::set(const std::string& key, const Digest& d, Bytes value, uint32_t flags,
                       uint32_t ttl_s) {
  const FaultSpec f = spec();
  if (f.down || roll(f.set_drop)) {
    injected_drop_++;
    return;
  }
  inner_->set(key, d, std::move(value), flags, ttl_s);
}

void FaultBackend::del(const std::string& key, const Digest& d, Executor* ex, DelCallback done) {
  const FaultSpec f = spec();
  if (f.down) {
    done(false);
    return;
  }
  if (!f.delay_us) {
    inner_->del(key, d, ex, std::move(done));
    return;
  }
  later([this, key, d, ex, done] {
    inner_->del(key, d, ex, [ex, done](bool found) {
      if (ex) ex->post([done, found] { done(found); });
      else done(found);
    });
  });
}

void FaultBackend::stats(StatList* out) {
  inner_->stats(out);
  out->emplace_back("fault_injected_miss", injected_miss_.load());
  out->emplace_back("fault_injected_drop", injected_drop_.load());
  out->emplace_back("fault_injected_delay", injected_delay_.load());
}

}  // namespace shellac
