// Native closed-loop HTTP/1.1 load generator ("ab -k -n N -c C" equivalent).
//
// The reference benchmarks with ApacheBench (benchmarks/run-*.sh:
// `ab -k -n 400 -c 10 -g X.dat -H "Accept-Encoding: gzip"`), which is not
// installed here. This drives C keep-alive connections (optionally pipelined
// `depth` deep) from T epoll threads, issues N requests round-robin over a path
// list, and records per-request latency (send -> last byte) for p50/p99 and an
// ab-style "-g" per-request TSV.
#include "loadgen.h"

#include <strings.h>
#include <sys/epoll.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <deque>
#include <string_view>
#include <thread>

#include "http.h"

namespace shellac {

namespace {
// Response framing without copying bodies: the head is collected and scanned for the
// status, Content-Length and Connection; the body is skipped by count. A response the
// fast path cannot frame (chunked, or no length) switches the connection to the full
// HttpParser. The load generator then costs a fraction of the proxy it measures.
struct FastFramer {
  std::string head;      // bytes of the current head (until CRLFCRLF)
  uint64_t body_left = 0;
  bool in_body = false;
  int status = 0;
  bool keep_alive = true;

  // Consume from [p, p+n); returns bytes used, sets *done when a response completed,
  // *fallback when the response needs the full parser (nothing consumed then).
  size_t feed(const char* p, size_t n, bool* done, bool* fallback) {
    *done = *fallback = false;
    size_t used = 0;
    if (!in_body) {
      if (head.empty()) {
        // common case: the whole head is in this read; copy only the head, not the body
        const std::string_view v(p, n);
        const size_t e = v.find("\r\n\r\n");
        if (e == std::string_view::npos) {
          head.assign(p, n);
          return n;
        }
        head.assign(p, e + 4);
        used = e + 4;
      } else {
        // append up to the end of the head
        const size_t start = head.size() >= 3 ? head.size() - 3 : 0;
        head.append(p, n);
        const size_t e = head.find("\r\n\r\n", start);
        if (e == std::string::npos) return n;
        used = n - (head.size() - (e + 4));
        head.resize(e + 4);
      }
      if (!parse_head()) {
        *fallback = true;
        return 0;
      }
      in_body = true;
    }
    const size_t take = (size_t)std::min<uint64_t>(body_left, n - used);
    body_left -= take;
    used += take;
    if (body_left == 0) {
      *done = true;
      in_body = false;
      head.clear();
    }
    return used;
  }

  bool parse_head() {
    // "HTTP/1.1 200 ..."
    if (head.size() < 12 || head.compare(0, 5, "HTTP/") != 0) return false;
    status = std::atoi(head.c_str() + 9);
    bool have_len = false;
    keep_alive = head.compare(5, 3, "1.0") != 0;
    size_t pos = head.find("\r\n") + 2;
    while (pos + 2 < head.size()) {
      const size_t eol = head.find("\r\n", pos);
      const size_t colon = head.find(':', pos);
      if (colon != std::string::npos && colon < eol) {
        const size_t nl = colon - pos;
        const char* v = head.c_str() + colon + 1;
        if (nl == 14 && strncasecmp(head.c_str() + pos, "content-length", 14) == 0) {
          body_left = std::strtoull(v, nullptr, 10);
          have_len = true;
        } else if (nl == 17 && strncasecmp(head.c_str() + pos, "transfer-encoding", 17) == 0) {
          return false;  // chunked: the full parser frames it
        } else if (nl == 10 && strncasecmp(head.c_str() + pos, "connection", 10) == 0) {
          const std::string val(v, eol - colon - 1);
          if (strcasestr(val.c_str(), "close")) keep_alive = false;
          else if (strcasestr(val.c_str(), "keep-alive")) keep_alive = true;
        }
      }
      pos = eol + 2;
    }
    if (!have_len) {
      if (status == 204 || status == 304 || status / 100 == 1) body_left = 0;
      else return false;
    }
    return true;
  }
};

struct LgConn {
  int fd = -1;
  bool connected = false;
  std::string out;
  size_t out_off = 0;
  std::deque<std::pair<double, int64_t>> sent;  // in-flight requests: (send time, k)
  std::unique_ptr<HttpParser> parser;  // full parser (fallback framing)
  FastFramer fast;
  bool use_parser = false;
  size_t path_idx = 0;
  bool out_armed = true;    // EPOLLOUT in the interest set
  double t_connect = 0;     // when connect() was called
};
}  // namespace

LoadResult run_load(const LoadConfig& cfg) {
  SH_CHECK(cfg.concurrency > 0 && cfg.threads > 0 && cfg.requests > 0, "bad load config");
  SH_CHECK(!cfg.paths.empty() || cfg.objects > 0, "no paths");
  const Addr addr = resolve(cfg.host + ":" + std::to_string(cfg.port), cfg.port);
  std::atomic<int64_t> issued{0};
  std::vector<std::vector<LoadSample>> per_thread(cfg.threads);
  std::vector<std::vector<double>> conn_lat(cfg.threads), conn_call(cfg.threads);
  std::vector<double> open_loop(cfg.threads, 0.0);
  std::atomic<uint64_t> bytes{0}, errors{0}, non2xx{0}, reconnects{0};
  std::vector<double> connected_at(cfg.threads, 0.0);  // last connection up, per thread

  // serialized requests, one per path (built once)
  std::string tail = " HTTP/1.1\r\nHost: " + cfg.host + "\r\n";
  if (cfg.keepalive) tail += "Connection: keep-alive\r\n";
  for (const auto& h : cfg.headers) tail += h + "\r\n";
  tail += "\r\n";
  std::vector<std::string> reqs;
  for (const auto& path : cfg.paths) reqs.push_back(cfg.method + " " + path + tail);
  // generated paths: Zipf inverse-CDF table over popularity ranks, ranks -> ids by
  // rank * P mod N (P prime and not a divisor of N: a bijection)
  const int64_t nobj = cfg.objects;
  std::vector<double> cdf;
  std::vector<uint32_t> guide;  // guide[b]: first rank whose CDF reaches b / G
  uint64_t mult = 1;
  if (nobj > 0 && cfg.zipf_s > 0) {
    cdf.resize((size_t)nobj);
    double acc = 0;
    for (int64_t r = 0; r < nobj; ++r) {
      acc += std::pow((double)(r + 1), -cfg.zipf_s);
      cdf[(size_t)r] = acc;
    }
    for (auto& v : cdf) v /= acc;
    // guide table: a draw u only searches the ranks of its 1/G bucket (a few adjacent
    // cache lines) instead of ~23 dependent misses through a 64 MB CDF at 8M objects
    const size_t G = 1u << 20;
    guide.resize(G + 1);
    size_t r = 0;
    for (size_t b = 0; b <= G; ++b) {
      const double t = (double)b / (double)G;
      while (r + 1 < cdf.size() && cdf[r] < t) ++r;
      guide[b] = (uint32_t)r;
    }
    mult = 2654435761ull;
    while ((uint64_t)nobj % mult == 0) mult += 2;
  }
  auto gen_req = [&](int64_t k, uint64_t* rng, std::string* out) {
    int64_t id;
    if (cdf.empty()) {
      id = k % nobj;
    } else {
      uint64_t& x = *rng;
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      const double u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
      const size_t b = (size_t)(u * (double)(guide.size() - 1));
      const auto lo = cdf.begin() + guide[b];
      const auto hi = b + 1 < guide.size() ? cdf.begin() + std::min<size_t>(cdf.size(), guide[b + 1] + 1)
                                           : cdf.end();
      const int64_t r = std::lower_bound(lo, hi, u) - cdf.begin();
      id = (int64_t)(((unsigned __int128)std::min<int64_t>(r, nobj - 1) * mult) % (uint64_t)nobj);
    }
    *out += cfg.method;
    *out += ' ';
    *out += cfg.path_prefix;
    *out += std::to_string(id);
    *out += cfg.path_suffix;
    *out += tail;
  };

  reserve_fd_table(cfg.concurrency + 256);
  // the clock starts at the first connection, after the path tables are built (the
  // Zipf CDF of 8M objects alone takes ~0.1 s)
  const double t_start = now_s();
  auto worker = [&](int tid) {
    pin_thread(cfg.cpus, (size_t)tid);
    const int nconn = cfg.concurrency / cfg.threads + (tid < cfg.concurrency % cfg.threads ? 1 : 0);
    uint64_t rng = (cfg.seed + 1) * 0x9E3779B97F4A7C15ull ^ (uint64_t)(tid + 1) * 0xD1B54A32D192ED03ull;
    const int ep = epoll_create1(EPOLL_CLOEXEC);
    std::vector<LgConn> conns(nconn);
    auto& samples = per_thread[tid];
    samples.reserve((size_t)(cfg.requests / cfg.threads + 16));
    int live = 0;
    // requests are claimed from the shared counter 32 at a time (one contended atomic per
    // 32 requests, not per request); a dead connection's in-flight requests go back to
    // this thread's redo list and are re-issued with the same k
    int64_t next_k = 0, end_k = 0;
    std::vector<int64_t> redo;
    uint64_t my_bytes = 0;
    auto claim = [&](int64_t* k) {
      if (!redo.empty()) {
        *k = redo.back();
        redo.pop_back();
        return true;
      }
      if (next_k == end_k) {
        int64_t g = issued.load();
        int64_t take = 0;
        do {
          take = std::min<int64_t>(32, cfg.requests - g);
          if (take <= 0) return false;
        } while (!issued.compare_exchange_weak(g, g + take));
        next_k = g;
        end_k = g + take;
      }
      *k = next_k++;
      return true;
    };
    auto work_left = [&] {
      return !redo.empty() || next_k < end_k || issued.load() < cfg.requests;
    };
    auto open_conn = [&](int i) {
      LgConn& c = conns[i];
      c = LgConn();
      c.t_connect = now_s();
      c.fd = connect_nonblock(addr);
      conn_call[tid].push_back(now_s() - c.t_connect);
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
      // abortive close (RST): a run leaves no TIME_WAIT sockets behind, so the next
      // run's connect() does not crawl through thousands of them for a free port
      const linger lg{1, 0};
      setsockopt(c.fd, SOL_SOCKET, SO_LINGER, &lg, sizeof lg);
      epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
      close(c.fd);
      c.fd = -1;
      --live;
    };
    auto top_up = [&](LgConn& c) {  // keep `depth` requests in flight
      while ((int)c.sent.size() < cfg.depth) {
        int64_t k = 0;
        if (!claim(&k)) break;
        if (nobj > 0) gen_req(k, &rng, &c.out);
        else c.out += reqs[(size_t)k % reqs.size()];
        c.sent.emplace_back(0.0, k);  // timestamp set at send
      }
    };
    // send what is queued right away; returns false on a socket error
    auto flush = [&](LgConn& c) {
      if (!c.connected || c.out_off >= c.out.size()) return true;
      const double t = now_s();
      for (auto& ts : c.sent)
        if (ts.first == 0) ts.first = t;
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
    const double t_open = now_s();
    for (int i = 0; i < nconn; ++i) {
      if (!work_left()) break;  // fewer requests than connections: open only what is used
      if (open_conn(i)) {
        top_up(conns[i]);
        // the other threads claimed the rest: an idle connection would only wait for the
        // server's idle timeout before this thread could finish
        if (conns[i].sent.empty()) close_conn(i);
      }
    }
    open_loop[tid] = now_s() - t_open;
    char buf[1 << 16];
    epoll_event evs[256];
    const double spin_s = cfg.spin_us * 1e-6;
    double last_ev = now_s();
    while (live > 0) {
      const bool spin = spin_s > 0 && now_s() - last_ev < spin_s;
      const int n = epoll_wait(ep, evs, 256, spin ? 0 : 1000);
      if (n > 0 && spin_s > 0) last_ev = now_s();
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
            const double tc = now_s();
            connected_at[tid] = std::max(connected_at[tid], tc - t_start);
            conn_lat[tid].push_back(tc - c.t_connect);
          }
        }
        flush(c);
        if (evs[e].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
          bool dead = false;
          for (;;) {
            const ssize_t r = recv(c.fd, buf, sizeof buf, 0);
            if (r > 0) {
              my_bytes += (uint64_t)r;
              const char* p = buf;
              size_t left = (size_t)r;
              while (left > 0 && !c.sent.empty()) {
                bool complete = false;
                int st = 0;
                bool ka = true;
                size_t used = 0;
                if (!c.use_parser) {
                  bool fallback = false;
                  // the framer keeps the partial head; on fallback replay it to the parser
                  const std::string pending = c.fast.head;
                  used = c.fast.feed(p, left, &complete, &fallback);
                  if (fallback) {
                    c.use_parser = true;
                    const size_t hp = c.parser->parse(pending.data(), pending.size());
                    (void)hp;
                    c.fast = FastFramer();
                    continue;
                  }
                  st = c.fast.status;
                  ka = c.fast.keep_alive;
                } else {
                  used = c.parser->parse(p, left);
                  if (c.parser->error()) { dead = true; break; }
                  complete = c.parser->message_complete();
                  if (complete) {
                    st = c.parser->status();
                    ka = c.parser->keep_alive();
                    c.parser->reset();
                  }
                }
                p += used;
                left -= used;
                if (complete) {
                  const double t = now_s();
                  const double ts = c.sent.front().first;
                  samples.push_back(LoadSample{ts - t_start, t - ts, st});
                  if (st < 200 || st >= 300) non2xx++;
                  c.sent.pop_front();
                  if (!(ka && cfg.keepalive)) { dead = true; break; }
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
            for (const auto& q : c.sent) redo.push_back(q.second);
            reconnects++;
            close_conn(i);
            // reconnect if work remains (ab -k semantics when the server closes)
            if (work_left() && open_conn(i)) top_up(conns[i]);
            continue;
          }
          top_up(c);
          if (c.sent.empty() && !work_left()) {
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
    bytes += my_bytes;
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
  for (auto& v : conn_lat) res.connect_lat.insert(res.connect_lat.end(), v.begin(), v.end());
  for (auto& v : conn_call) res.connect_call.insert(res.connect_call.end(), v.begin(), v.end());
  res.open_loop_s = *std::max_element(open_loop.begin(), open_loop.end());
  return res;
}

}  // namespace shellac
