// Native (host-only) test driver for the sanitizer presets.
//
// The reference is single-threaded and has no sanitizer story; this runtime has
// reactor threads, a memcached IO thread, GPU batcher threads and a fault-delay
// timer thread, so its host code is exercised here under ASan+UBSan and TSan
// (CMakePresets.json: asan, tsan, ubsan). No Python, no GPU: every case drives the
// C++ objects directly.
//
//   cmake --preset tsan && cmake --build --preset tsan && build/tsan/shellac_native_tests
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "backend.h"
#include "digest.h"
#include "host_cache.h"
#include "host_router.h"
#include "http.h"
#include "ketama.h"
#include "loadgen.h"
#include "mcserver.h"
#include "net.h"
#include "proxy.h"
#include "stream_buf.h"

using namespace shellac;

namespace {

int g_fail = 0;
#define CHECK(cond)                                                               \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                                   \
    }                                                                             \
  } while (0)

Digest dg(const std::string& s) { return digest_bytes((const uint8_t*)s.data(), s.size()); }

// ---------------------------------------------------------------------------------
void test_host_cache_oracle() {
  HostCache hc(64 << 20, 1 << 16, 1 << 16);
  std::map<std::string, std::string> oracle;
  std::mt19937_64 rng(1);
  for (int it = 0; it < 20000; ++it) {
    const std::string k = "/k/" + std::to_string(rng() % 3000);
    const int op = (int)(rng() % 10);
    if (op < 5) {
      std::string v(rng() % 700, (char)('a' + rng() % 26));
      hc.set_one(dg(k), (const uint8_t*)v.data(), (uint32_t)v.size(), 7, 0, 1);
      oracle[k] = v;
    } else if (op < 9) {
      std::vector<uint8_t> out;
      uint32_t flags = 0;
      const bool hit = hc.get_one(dg(k), &out, &flags, 1);
      auto it2 = oracle.find(k);
      CHECK(hit == (it2 != oracle.end()));
      if (hit && it2 != oracle.end()) {
        CHECK(std::string(out.begin(), out.end()) == it2->second);
        CHECK(flags == 7);
      }
    } else {
      const Digest d = dg(k);
      uint8_t found = 0;
      hc.remove(&d, 1, &found, 1);
      CHECK((found != 0) == (oracle.erase(k) == 1));
    }
  }
}

// ---------------------------------------------------------------------------------
void test_http_parser_splits_and_garbage() {
  const std::string msgs =
      "GET /a HTTP/1.1\r\nHost: x\r\nAccept-Encoding: gzip\r\n\r\n"
      "POST /p HTTP/1.1\r\nContent-Length: 5\r\n\r\nhello"
      "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n2;x=1\r\nde\r\n0\r\n\r\n";
  std::mt19937 rng(3);
  for (int trial = 0; trial < 300; ++trial) {
    std::vector<std::string> bodies;
    HttpParser p(true);
    size_t i = 0;
    while (i < msgs.size()) {
      const size_t n = std::min(msgs.size() - i, (size_t)(1 + rng() % 17));
      size_t used = 0;
      while (used < n) {
        const size_t u = p.parse(msgs.data() + i + used, n - used);
        CHECK(!p.error());
        used += u;
        if (p.message_complete()) {
          bodies.push_back(p.body());
          p.reset();
        } else if (u == 0) {
          break;
        }
      }
      i += n;
    }
    CHECK(bodies.size() == 3);
    if (bodies.size() == 3) {
      CHECK(bodies[0].empty() && bodies[1] == "hello" && bodies[2] == "abcde");
    }
  }
  // random garbage never crashes and never reads out of bounds
  for (int trial = 0; trial < 2000; ++trial) {
    std::string g(rng() % 300, '\0');
    for (auto& c : g) c = (char)(rng() % 256);
    if (trial % 3 == 0) g = "HTTP/1.1 200 OK\r\nContent-Length: " + g;
    if (trial % 3 == 1) g = "GET / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n" + g;
    HttpParser p(true);
    size_t off = 0;
    while (off < g.size()) {
      const size_t u = p.parse(g.data() + off, g.size() - off);
      if (u == 0 || p.error() || p.message_complete()) break;
      off += u;
    }
    p.finish();
  }
  // gzip roundtrip
  std::string big(100000, 'q');
  std::string z = gzip_compress(big, 6), back;
  CHECK(gzip_decompress(z, &back) && back == big);
}

// ---------------------------------------------------------------------------------
void test_stream_buf() {
  StreamBuf b;
  b.write("hello ");
  b.write_shared(std::make_shared<const std::string>("world"));
  iovec v[4];
  CHECK(b.iov(v, 4) == 2);
  b.ack(3);
  CHECK(b.read() == "lo world");
  b.close();
  CHECK(!b.complete());
  b.ack(8);
  CHECK(b.complete());
}

void test_ketama() {
  KetamaRing r({{"a:11211", 1, true}, {"b:11211", 1, true}, {"c:11211", 2, true}});
  std::vector<int> owner;
  for (int i = 0; i < 1000; ++i) owner.push_back(r.pick("/k" + std::to_string(i)));
  r.set_alive(1, false);
  int moved = 0;
  for (int i = 0; i < 1000; ++i) {
    const int o = r.pick("/k" + std::to_string(i));
    CHECK(o != 1);
    if (owner[i] != 1) moved += o != owner[i];
  }
  CHECK(moved == 0);  // only the ejected node's keys move
}

// The host router's worker pool: threaded routing equals one thread's, call after call
// (the pool is reused), for GETs and SETs, with and without a hot set.
void test_host_router_pool() {
  HostRouter r(8, 64);
  std::vector<Digest> keys(200000);
  uint64_t x = 0x243F6A8885A308D3ull;
  for (auto& d : keys) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    d.lo = x;
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    d.hi = x;
  }
  std::vector<int32_t> rank(4096);
  for (int i = 0; i < 4096; ++i) rank[(size_t)i] = i < 3 ? -1 : i % 8;
  const std::vector<double> w(8, 1.0);
  for (int hot = 0; hot < 2; ++hot) {
    r.set_hot(keys.data(), hot ? 4096 : 0, rank.data(), w.data());
    std::vector<int32_t> d1(keys.size()), dn(keys.size());
    std::vector<int64_t> c1(8, 0), cn(8, 0);
    r.route_gets(keys.data(), (int64_t)keys.size(), 77, d1.data(), c1.data(), 1);
    for (int rep = 0; rep < 3; ++rep) {
      std::fill(cn.begin(), cn.end(), 0);
      r.route_gets(keys.data(), (int64_t)keys.size(), 77, dn.data(), cn.data(), 4);
      CHECK(dn == d1 && cn == c1);
    }
    r.route_sets(keys.data(), (int64_t)keys.size(), d1.data(), c1.data(), 1);
    r.route_sets(keys.data(), (int64_t)keys.size(), dn.data(), cn.data(), 3);
    CHECK(dn == d1);
    int64_t hot_rows = 0;
    for (int32_t v : d1) hot_rows += v < 0;
    CHECK(hot_rows == (hot ? 4096 : 0));
  }
}

// The hot table swapped under routing (the proxy's refresh beside its reactors): readers
// hold Read guards and route small batches while a writer alternates two hot sets. Every
// decision is one of the two tables' (never a torn one), and when set_hot returns no reader
// is still inside a guard on the previous table (the refresh protocol relies on it). Under
// TSAN this is the race check of the lock-free read side.
void test_host_router_hot_swap_concurrent() {
  constexpr int kShards = 8, kReaders = 4;
  HostRouter r(kShards, 64);
  std::vector<Digest> keys(4096);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& d : keys) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    d.lo = x;
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    d.hi = x;
  }
  // table A: keys [0, 1024) on rank i % 8; table B: keys [512, 1512) on rank (i + 3) % 8
  std::vector<int32_t> ra(1024), rb(1000);
  for (int i = 0; i < 1024; ++i) ra[(size_t)i] = i % kShards;
  for (int i = 0; i < 1000; ++i) rb[(size_t)i] = (512 + i + 3) % kShards;
  const std::vector<double> w(kShards, 1.0);
  auto want = [&](int table, int k) {  // the rank table A (0) or B (1) gives key k
    if (table == 0) return k < 1024 ? ra[(size_t)k] : HostRouter::kNotHot;
    return k >= 512 && k < 1512 ? rb[(size_t)(k - 512)] : HostRouter::kNotHot;
  };
  r.set_hot(keys.data(), 1024, ra.data(), w.data());
  std::atomic<bool> stop{false};
  std::atomic<int> bad{0};
  std::atomic<int64_t> held[kReaders];
  std::atomic<uint64_t> decisions{0};
  for (auto& h : held) h.store(-1);
  std::vector<std::thread> th;
  for (int t = 0; t < kReaders; ++t)
    th.emplace_back([&, t] {
      std::vector<int32_t> dest(64);
      std::vector<int64_t> cnt(kShards);
      uint64_t n = 0;
      for (uint32_t it = 0; !stop.load(std::memory_order_acquire); ++it) {
        const int k = (int)((it * 2654435761u + (uint32_t)t * 977u) % 1600u);
        {
          const HostRouter::Read rd(r);
          const int64_t nh = rd.table().nhot;
          held[t].store(nh, std::memory_order_release);
          const int got = rd.hot_rank(keys[(size_t)k]);
          if (!((nh == 1024 && got == want(0, k)) || (nh == 1000 && got == want(1, k))))
            bad.fetch_add(1);
          held[t].store(-1, std::memory_order_release);
        }
        if ((it & 63) == 0) {  // a batch through the routing call (its own guard)
          std::fill(cnt.begin(), cnt.end(), 0);
          r.route_gets(keys.data() + (k & ~63), 64, 0, dest.data(), cnt.data(), 1);
          for (int i = 0; i < 64; ++i) {
            const int kk = (k & ~63) + i;
            const int own = r.owner(keys[(size_t)kk]);
            const int a = want(0, kk) == HostRouter::kNotHot ? own : want(0, kk);
            const int b = want(1, kk) == HostRouter::kNotHot ? own : want(1, kk);
            if (dest[(size_t)i] != a && dest[(size_t)i] != b) bad.fetch_add(1);
          }
        }
        ++n;
      }
      decisions.fetch_add(n);
    });
  for (int rep = 0; rep < 200; ++rep) {
    const bool to_b = rep % 2 == 0;
    const int64_t old = to_b ? 1024 : 1000;
    if (to_b)
      r.set_hot(keys.data() + 512, 1000, rb.data(), w.data());
    else
      r.set_hot(keys.data(), 1024, ra.data(), w.data());
    for (auto& h : held)
      if (h.load(std::memory_order_acquire) == old) bad.fetch_add(1);  // grace period broken
  }
  stop.store(true, std::memory_order_release);
  for (auto& t : th) t.join();
  CHECK(bad.load() == 0);
  CHECK(decisions.load() > 1000);
}

// ---------------------------------------------------------------------------------
// Minimal keep-alive origin: one thread per connection, Content-Length bodies.
class Origin {
 public:
  Origin() {
    fd_ = listen_tcp("127.0.0.1", 0, false, 128);
    fcntl(fd_, F_SETFL, fcntl(fd_, F_GETFL) & ~O_NONBLOCK);  // blocking accept loop
    sockaddr_in a{};
    socklen_t al = sizeof a;
    getsockname(fd_, (sockaddr*)&a, &al);
    port_ = ntohs(a.sin_port);
    th_ = std::thread([this] { accept_loop(); });
  }
  ~Origin() {
    stop_ = true;
    shutdown(fd_, SHUT_RDWR);
    close(fd_);
    th_.join();
    std::lock_guard<std::mutex> lk(mu_);
    for (int c : conns_) shutdown(c, SHUT_RDWR);
    for (auto& t : workers_) t.join();
  }
  uint16_t port() const { return port_; }
  uint64_t hits() const { return hits_; }

 private:
  void accept_loop() {
    for (;;) {
      const int c = accept(fd_, nullptr, nullptr);
      if (c < 0) return;
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) {
        close(c);
        return;
      }
      conns_.push_back(c);
      workers_.emplace_back([this, c] { serve(c); });
    }
  }
  void serve(int c) {
    // accepted sockets are blocking (O_NONBLOCK is not inherited on Linux)
    HttpParser p(true);
    char buf[8192];
    for (;;) {
      const ssize_t r = recv(c, buf, sizeof buf, 0);
      if (r <= 0) break;
      size_t off = 0;
      while (off < (size_t)r) {
        off += p.parse(buf + off, (size_t)r - off);
        if (p.error()) return;
        if (!p.message_complete()) break;
        hits_++;
        std::string body = "<html>" + p.url() + " " + std::string(500 + p.url().size(), 'x') +
                           "</html>";
        std::string resp = "HTTP/1.1 200 OK\r\nContent-Type: text/html\r\nContent-Length: " +
                           std::to_string(body.size()) + "\r\n\r\n" + body;
        size_t w = 0;
        while (w < resp.size()) {
          const ssize_t k = send(c, resp.data() + w, resp.size() - w, MSG_NOSIGNAL);
          if (k <= 0) return;
          w += (size_t)k;
        }
        p.reset();
      }
    }
  }
  int fd_ = -1;
  uint16_t port_ = 0;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> hits_{0};
  std::thread th_;
  std::mutex mu_;
  std::vector<int> conns_;
  std::vector<std::thread> workers_;
};

LoadResult drive(uint16_t port, int paths, int64_t n, int conc, int depth) {
  LoadConfig lc;
  lc.port = port;
  lc.paths.clear();
  for (int i = 0; i < paths; ++i) lc.paths.push_back("/obj/" + std::to_string(i));
  lc.requests = n;
  lc.concurrency = conc;
  lc.depth = depth;
  lc.threads = 2;
  lc.headers = {"Accept-Encoding: gzip"};
  lc.timeout_s = 60;
  return run_load(lc);
}

void test_proxy_threads_dram(const char* fault) {
  Origin o;
  ProxyConfig pc;
  pc.bind = "127.0.0.1";
  pc.port = 0;
  pc.upstreams = resolve_list("127.0.0.1:" + std::to_string(o.port()), 80);
  pc.threads = 4;
  std::shared_ptr<CacheBackend> be = std::make_shared<DramBackend>(64 << 20, 1 << 20, 16);
  if (fault) be = std::make_shared<FaultBackend>(be, parse_fault_spec(fault));
  Proxy px(pc, be);
  px.start();
  const LoadResult r = drive(px.port(), 200, 20000, 32, 4);
  CHECK(r.errors == 0 && r.non2xx == 0);
  CHECK(r.completed == 20000);
  const std::string st = px.stats_json();
  CHECK(st.find("\"errors\":0") != std::string::npos);
  if (!fault) CHECK(o.hits() <= 400);  // collapsed/cached: a handful of fetches per path
  px.stop();
}

void test_proxy_over_memcached_node() {
  // cache node (memcached binary protocol) backed by DRAM, proxy -> tiered(L1, memcached)
  Origin o;
  CacheServerConfig cc;
  cc.bind = "127.0.0.1";
  cc.port = 0;
  cc.threads = 2;
  CacheServer node(cc, std::make_shared<DramBackend>(64 << 20, 1 << 20, 4));
  node.start();
  MemcachedConfig mc;
  mc.servers = resolve_list("127.0.0.1:" + std::to_string(node.port()), 11211);
  auto l2 = std::make_shared<MemcachedBackend>(mc);
  auto tiered = std::make_shared<TieredBackend>(std::make_shared<DramBackend>(1 << 20, 1 << 20, 2),
                                                l2, 60);
  ProxyConfig pc;
  pc.bind = "127.0.0.1";
  pc.port = 0;
  pc.upstreams = resolve_list("127.0.0.1:" + std::to_string(o.port()), 80);
  pc.threads = 3;
  Proxy px(pc, tiered);
  px.start();
  const LoadResult r = drive(px.port(), 3000, 15000, 24, 2);
  CHECK(r.errors == 0 && r.non2xx == 0 && r.completed == 15000);
  CHECK(node.ops() > 0);
  px.stop();
  node.stop();
}

}  // namespace

int main(int argc, char** argv) {
  const std::string only = argc > 1 ? argv[1] : "";
  struct Case {
    const char* name;
    std::function<void()> fn;
  } cases[] = {
      {"host_cache_oracle", test_host_cache_oracle},
      {"http_parser", test_http_parser_splits_and_garbage},
      {"stream_buf", test_stream_buf},
      {"ketama", test_ketama},
      {"host_router_pool", test_host_router_pool},
      {"host_router_hot_swap", test_host_router_hot_swap_concurrent},
      {"proxy_threads_dram", [] { test_proxy_threads_dram(nullptr); }},
      {"proxy_threads_fault", [] { test_proxy_threads_dram("get_miss=0.3,set_drop=0.3,delay_us=200"); }},
      {"proxy_memcached_node", test_proxy_over_memcached_node},
  };
  for (auto& c : cases) {
    if (!only.empty() && only != c.name) continue;
    const int before = g_fail;
    const auto t0 = std::chrono::steady_clock::now();
    try {
      c.fn();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s threw: %s\n", c.name, e.what());
      ++g_fail;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%-24s %s (%.2fs)\n", c.name, g_fail == before ? "ok" : "FAILED", s);
  }
  std::printf("%s\n", g_fail ? "FAILED" : "ALL OK");
  return g_fail ? 1 : 0;
}
