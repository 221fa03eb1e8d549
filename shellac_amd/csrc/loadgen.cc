// Native closed-loop HTTP/1.1 load generator ("ab -k -n N -c C" equivalent).
//
// The reference benchmarks with ApacheBench (benchmarks/run-*.sh:
// `ab -k -n 400 -c 10 -g X.dat -H "Accept-Encoding: gzip"`), which is not
// installed here. This drives C keep-alive connections (optionally pipelined
// `depth` deep) from T epoll threads, issues N requests round-robin over a path
// list, and records per-request latency (send -> last byte) for p50/p99 and an
// ab-style "-g" per-request TSV.
#include "loadgen.h"

#include <sys/epoll.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <deque>
#include <thread>

#include "http.h"

namespace shellac {

namespace {
struct LgConn {
  int fd = -1;
  bool connected = false;
  std::string out;
  size_t out_off = 0;
  std::deque<double> sent;  // send timestamps of in-flight requests
  std::unique_ptr<HttpParser> parser;
  size_t path_idx = 0;
  bool out_armed = true;    // EPOLLOUT in the interest set
};
}  // namespace

LoadResult run_load(const LoadConfig& cfg) {
  SH_CHECK(cfg.concurrency > 0 && cfg.threads > 0 && cfg.requests > 0, "bad load config");
  SH_CHECK(!cfg.paths.empty(), "no paths");
  const Addr addr = resolve(cfg.host + ":" + std::to_string(cfg.port), cfg.port);
  std::atomic<int64_t> issued{0};
  std::vector<std::vector<LoadSample>> per_thread(cfg.threads);
  std::atomic<uint64_t> bytes{0}, errors{0}, non2xx{0}, reconnects{0};
  std::vector<double> connected_at(cfg.threads, 0.0);  // last connection up, per thread
  const double t_start = now_s();

  // serialized requests, one per path (built once)
  std::vector<std::string> reqs;
  for (const auto& path : cfg.paths) {
    std::string r = cfg.method + " " + path + " HTTP/1.1\r\nHost: " + cfg.host + "\r\n";
    if (cfg.keepalive) r += "Connection: keep-alive\r\n";
    for (const auto& h : cfg.headers) r += h + "\r\n";
    r += "\r\n";
    reqs.push_back(std::move(r));
  }
  auto req_bytes = [&](size_t i) -> const std::string& { return reqs[i % reqs.size()]; };

  auto worker = [&](int tid) {
    const int nconn = cfg.concurrency / cfg.threads + (tid < cfg.concurrency % cfg.threads ? 1 : 0);
    const int ep = epoll_create1(EPOLL_CLOEXEC);
    std::vector<LgConn> conns(nconn);
    auto& samples = per_thread[tid];
    samples.reserve((size_t)(cfg.requests / cfg.threads + 16));
    int live = 0;
    auto open_conn = [&](int i) {
      LgConn& c = conns[i];
      c = LgConn();
      c.fd = connect_nonblock(addr);
      if (c.fd < 0) return false;
      c.parser = std::make_unique<HttpParser>(false);
      c.parser->set_eof_body(true);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
      ev.data.u32 = (uint32_t)i;
      epoll_ctl(ep, EPOLL_CTL_ADD, c.fd, &ev);
      ++live;
      return true;
    };
    auto close_conn = [&](int i) {
      LgConn& c = conns[i];
      if (c.fd < 0) return;
      epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
      close(c.fd);
      c.fd = -1;
      --live;
    };
    auto top_up = [&](LgConn& c) {  // keep `depth` requests in flight
      while ((int)c.sent.size() < cfg.depth) {
        // claim request k only while k < requests: a blind fetch_add past the end would
        // inflate `issued`, and a thread whose connection died with requests in flight
        // would then wrongly see nothing left to re-issue (lost requests)
        int64_t k = issued.load();
        do {
          if (k >= cfg.requests) break;
        } while (!issued.compare_exchange_weak(k, k + 1));
        if (k >= cfg.requests) break;
        c.out += req_bytes((size_t)k);
        c.sent.push_back(0);  // timestamp set at send
      }
    };
    // send what is queued right away; returns false on a socket error
    auto flush = [&](LgConn& c) {
      if (!c.connected || c.out_off >= c.out.size()) return true;
      const double t = now_s();
      for (auto& ts : c.sent)
        if (ts == 0) ts = t;
      const ssize_t w = send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (w > 0) c.out_off += (size_t)w;
      if (c.out_off == c.out.size()) {
        c.out.clear();
        c.out_off = 0;
      }
      return w >= 0 || errno == EAGAIN || errno == EWOULDBLOCK;
    };
    // EPOLLOUT only while bytes wait (one epoll_ctl per change, not per event)
    auto rearm = [&](int i) {
      LgConn& c = conns[i];
      if (c.fd < 0) return;
      const bool want = !c.connected || c.out_off < c.out.size();
      if (want == c.out_armed) return;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP | (want ? EPOLLOUT : 0);
      ev.data.u32 = (uint32_t)i;
      epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &ev);
      c.out_armed = want;
    };
    for (int i = 0; i < nconn; ++i) {
      if (open_conn(i)) top_up(conns[i]);
    }
    char buf[1 << 16];
    epoll_event evs[256];
    while (live > 0) {
      const int n = epoll_wait(ep, evs, 256, 1000);
      if (n == 0 && now_s() - t_start > cfg.timeout_s) break;
      for (int e = 0; e < n; ++e) {
        const int i = (int)evs[e].data.u32;
        LgConn& c = conns[i];
        if (c.fd < 0) continue;
        if (evs[e].events & EPOLLOUT) {
          if (!c.connected) {
            int err = 0;
            socklen_t el = sizeof err;
            getsockopt(c.fd, SOL_SOCKET, SO_ERROR, &err, &el);
            if (err) {
              errors += c.sent.size();
              close_conn(i);
              continue;
            }
            c.connected = true;
            connected_at[tid] = std::max(connected_at[tid], now_s() - t_start);
          }
        }
        flush(c);
        if (evs[e].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
          bool dead = false;
          for (;;) {
            const ssize_t r = recv(c.fd, buf, sizeof buf, 0);
            if (r > 0) {
              bytes += (uint64_t)r;
              const char* p = buf;
              size_t left = (size_t)r;
              while (left > 0 && !c.sent.empty()) {
                const size_t used = c.parser->parse(p, left);
                p += used;
                left -= used;
                if (c.parser->error()) { dead = true; break; }
                if (c.parser->message_complete()) {
                  const double t = now_s();
                  const int st = c.parser->status();
                  samples.push_back(LoadSample{c.sent.front() - t_start, t - c.sent.front(), st});
                  if (st < 200 || st >= 300) non2xx++;
                  c.sent.pop_front();
                  const bool ka = c.parser->keep_alive() && cfg.keepalive;
                  c.parser->reset();
                  if (!ka) { dead = true; break; }
                } else if (used == 0) {
                  break;
                }
              }
              if (dead) break;
              if ((size_t)r < sizeof buf) break;
              continue;
            }
            if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) dead = true;
            break;
          }
          if (dead) {
            // server closed with requests in flight: re-issue them on a new connection
            // (a keep-alive server may close at its max-requests limit)
            issued.fetch_sub((int64_t)c.sent.size());
            reconnects++;
            close_conn(i);
            // reconnect if work remains (ab -k semantics when the server closes)
            if (issued.load() < cfg.requests && open_conn(i)) top_up(conns[i]);
            continue;
          }
          top_up(c);
          if (c.sent.empty() && issued.load() >= cfg.requests) {
            close_conn(i);
            continue;
          }
          flush(c);  // the next request leaves in this iteration, not the next one
        }
        rearm(i);
      }
    }
    for (int i = 0; i < nconn; ++i) close_conn(i);
    close(ep);
  };

  std::vector<std::thread> th;
  for (int t = 0; t < cfg.threads; ++t) th.emplace_back(worker, t);
  for (auto& t : th) t.join();
  const double elapsed = now_s() - t_start;

  LoadResult res;
  for (auto& v : per_thread) res.samples.insert(res.samples.end(), v.begin(), v.end());
  std::sort(res.samples.begin(), res.samples.end(),
            [](const LoadSample& a, const LoadSample& b) { return a.start < b.start; });
  res.completed = res.samples.size();
  res.elapsed_s = elapsed;
  res.bytes = bytes;
  res.errors = errors;
  res.non2xx = non2xx;
  res.reconnects = reconnects;
  res.connected_s = *std::max_element(connected_at.begin(), connected_at.end());
  return res;
}

}  // namespace shellac
