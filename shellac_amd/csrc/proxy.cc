// Native caching reverse proxy (see proxy.h for the reference map and fixes).
#include "proxy.h"

#include <poll.h>
#include <sys/epoll.h>
#include <pthread.h>
#include <sys/eventfd.h>
#include <sys/timerfd.h>
#include <sys/uio.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <deque>
#include <random>
#include <sstream>
#include <unordered_map>

#include "http.h"

namespace shellac {

namespace {

constexpr uint64_t kListenId = 1, kEventId = 2, kTimerId = 3, kFirstConnId = 16;
constexpr int kHistBuckets = 40;

std::string simple_response(int code, const char* reason, const std::string& server,
                            const std::string& body, const char* ctype = "text/plain",
                            bool close = false) {
  std::string s = "HTTP/1.1 " + std::to_string(code) + " " + reason + "\r\nServer: " + server +
                  "\r\nContent-Type: " + ctype + "\r\nContent-Length: " +
                  std::to_string(body.size()) + "\r\nConnection: " +
                  (close ? "close" : "keep-alive") + "\r\n\r\n";
  return s + body;
}

bool contains_ci(const std::string* h, const char* needle) {
  if (!h) return false;
  return to_lower(*h).find(needle) != std::string::npos;
}

// Cache-Control max-age / s-maxage (seconds), -1 if absent.
long cc_max_age(const std::string* cc) {
  if (!cc) return -1;
  const std::string s = to_lower(*cc);
  long best = -1;
  for (const char* k : {"s-maxage=", "max-age="}) {
    const size_t p = s.find(k);
    if (p != std::string::npos) {
      best = std::strtol(s.c_str() + p + std::strlen(k), nullptr, 10);
      break;
    }
  }
  return best;
}

// ---- content negotiation + Vary (policy "rfc") ----------------------------------------
// The proxy forces `Accept-Encoding: gzip` upstream (Server.py:358), so one URL is cached
// once, usually gzip-coded; a client that did not ask for gzip gets the identity variant
// decoded from it on the way out (deliver()). Responses that Vary on request headers
// other than Accept-Encoding are stored per variant: a marker under the URL key names the
// headers, and the object lives under URL + the request's values of those headers.
const std::string kVaryMarker = "\x01SHELLAC-VARY\n";  // objects always start with "HTTP/"

bool is_vary_marker(std::string_view v) {
  return v.size() >= kVaryMarker.size() && v.compare(0, kVaryMarker.size(), kVaryMarker) == 0;
}

std::vector<std::string> split_names(const std::string& list) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= list.size()) {
    size_t j = list.find(',', i);
    if (j == std::string::npos) j = list.size();
    size_t a = i, b = j;
    while (a < b && (list[a] == ' ' || list[a] == '\t')) ++a;
    while (b > a && (list[b - 1] == ' ' || list[b - 1] == '\t')) --b;
    if (b > a) out.push_back(to_lower(list.substr(a, b - a)));
    i = j + 1;
  }
  return out;
}

// Request headers a response varies on, sorted, without accept-encoding (negotiated by
// the proxy itself); {"*"} = varies on something outside the request (never cached).
std::vector<std::string> vary_names(const HttpParser& r) {
  std::vector<std::string> names;
  for (const auto& h : r.headers()) {
    if (h.first != "vary") continue;
    for (auto& n : split_names(h.second)) {
      if (n == "*") return {"*"};
      if (n != "accept-encoding" && std::find(names.begin(), names.end(), n) == names.end())
        names.push_back(std::move(n));
    }
  }
  std::sort(names.begin(), names.end());
  return names;
}

std::vector<std::string> marker_names(std::string_view v) {
  return split_names(std::string(v.substr(kVaryMarker.size())));
}

// Secondary key of one variant: URL key + the request's values of the varied headers.
// Repeated headers combine in order with "," (RFC 7230 §3.2.2: `X: a` + `X: b` is the
// same field value as `X: a,b`, so they select the same variant), and each combined value
// is length-prefixed, so no value bytes (separators included) can forge another key.
// Names are tokens from the response's Vary header (no separator bytes).
std::string vary_key(const std::string& base, const std::vector<std::string>& names,
                     const std::vector<Header>& req) {
  std::string k = base;
  k += '\x1f';
  std::string v;
  for (const auto& n : names) {
    v.clear();
    bool first = true;
    for (const auto& h : req)
      if (h.first == n) {
        if (!first) v += ',';
        v += h.second;
        first = false;
      }
    k += n;
    k += '=';
    k += std::to_string(v.size());
    k += ':';
    k += v;
  }
  return k;
}

// Does the serialized response's head carry Content-Encoding: gzip?
bool object_is_gzip(std::string_view ov) {
  const size_t eoh = ov.find("\r\n\r\n");
  if (eoh == std::string_view::npos) return false;
  size_t pos = ov.find("\r\n");
  while (pos != std::string_view::npos && pos < eoh) {
    const size_t ls = pos + 2;
    const size_t le = ov.find("\r\n", ls);
    const std::string_view line = ov.substr(ls, le - ls);
    static constexpr std::string_view kCe = "content-encoding:";
    if (line.size() > kCe.size()) {
      bool match = true;
      for (size_t i = 0; i < kCe.size() && match; ++i)
        match = (char)std::tolower((unsigned char)line[i]) == kCe[i];
      if (match) return to_lower(std::string(line.substr(kCe.size()))).find("gzip") != std::string::npos;
    }
    pos = le;
  }
  return false;
}

// Identity variant of a gzip-coded cached response (body inflated, capped at `cap` bytes;
// Content-Encoding dropped, Content-Length recomputed, Vary kept). nullptr on a corrupt
// or oversized body.
Bytes identity_variant(const Bytes& obj, uint64_t cap) {
  HttpParser r(false);
  r.parse(obj->data(), obj->size());
  if (!r.message_complete() && !r.finish()) return nullptr;
  std::string body;
  if (!gzip_decompress(r.body(), &body, cap)) return nullptr;
  r.remove_header("content-encoding");
  r.mutable_body() = std::move(body);
  return std::make_shared<const std::string>(r.serialize());
}

}  // namespace

struct Slot {
  uint64_t seq = 0;
  StreamBuf out;
  bool ready = false;
  bool streaming = false;  // response bytes flow out before the response is complete
  uint64_t stream_up = 0;  // id of the upstream feeding a streamed response
  bool close_after = false;
  std::string fwd;  // serialized request for the miss path (built on the first forward)
  // The parsed request, kept (not serialized) while the cache answers: a hit never pays
  // for re-serializing a request it does not forward. Returned to the reactor's pool.
  std::unique_ptr<HttpParser> req;
  std::string key;
  std::string base_key;  // URL (+Host) key; `key` becomes a variant key after a Vary marker
  Digest d{};
  bool lookup = false, head = false, client_gzip = false;
  bool vary_probe = false;  // `key` is a variant key (second lookup after a marker)
  // request headers, kept for the miss path when a response may Vary (policy rfc)
  std::shared_ptr<const std::vector<Header>> req_headers;
  int attempts = 0;
  double t0 = 0;
};

struct Conn {
  int fd = -1;
  int kind = 0;  // 0 client, 1 upstream
  uint64_t id = 0;
  double ctime = 0, atime = 0;
  bool dead = false;
  bool out_armed = false;
  bool in_paused = false;  // EPOLLIN withheld (backpressure from a slow client)
  virtual ~Conn() = default;
};

struct Upstream;

struct Client : Conn {
  std::unique_ptr<HttpParser> req = std::make_unique<HttpParser>(true);
  std::deque<std::unique_ptr<Slot>> slots;
  uint64_t next_seq = 1;
  Upstream* up = nullptr;
  int nreq = 0;
  bool closing = false;  // stop parsing (bad request / EOF)
  bool eof = false;      // peer finished sending: close after the last response
  bool loopback = false;
};

struct Pend {
  uint64_t client_id, seq;
  std::string key;
  Digest d;
  bool lookup, head, client_gzip;
  std::string base_key;
  std::shared_ptr<const std::vector<Header>> req_headers;
};

struct Upstream : Conn {
  int server = 0;
  bool connected = false;
  StreamBuf out;
  std::unique_ptr<HttpParser> resp;
  std::deque<Pend> pend;
  Client* owner = nullptr;
  double ka_timeout = -1;
  int ka_max = 1 << 30;
  int count = 0;
  bool streaming = false;       // the front response is being streamed through
  bool stream_chunked = false;  // ... re-framed as chunked (unknown length)
};

class Reactor : public Executor {
 public:
  Reactor(Proxy* px, int id, int listen_fd);
  ~Reactor() override;
  void loop();
  void post(std::function<void()> fn) override;
  void post_batch(std::vector<std::function<void()>>& fns) override;
  void wake() {
    uint64_t one = 1;
    (void)!write(evfd_, &one, 8);
  }

  // stats (read by Proxy::stats_json from another thread)
  std::atomic<uint64_t> requests{0}, hits{0}, misses{0}, upstream_reqs{0}, responses{0},
      bytes_out{0}, errors{0}, clients{0}, upstreams{0}, accepts{0}, gc_closed{0},
      cache_sets{0}, bad_requests{0}, upstream_failures{0}, retries{0}, collapsed{0},
      streamed{0}, stream_pauses{0}, gzip_gpu_bodies{0}, gzip_gpu_inflated{0}, identity_decoded{0},
      vary_stored{0},
      vary_hits{0};
  // event-loop health: the longest iteration (events handled between two epoll_waits)
  // and how many took over 10 ms — a reactor that stalls stops accepting connections
  std::atomic<uint64_t> loop_max_us{0}, loop_slow{0}, client_resets{0};
  // longest single step per kind: accept, client event, upstream event, posted
  // completions, timer (gc)
  std::atomic<uint64_t> phase_max_us[5] = {};
  void phase_done(int k, double t0) {
    const uint64_t us = (uint64_t)((now_s() - t0) * 1e6);
    if (us > phase_max_us[k].load(std::memory_order_relaxed)) phase_max_us[k].store(us);
  }
  std::atomic<uint64_t> hist[kHistBuckets] = {};

 private:
  void accept_all();
  void on_client(Client* c, uint32_t ev);
  void on_upstream(Upstream* u, uint32_t ev);
  void on_request(Client* c);
  void on_cache(uint64_t cid, uint64_t seq, bool hit, CacheValue v);
  void forward(Client* c, Slot* s);
  static std::string upstream_request(HttpParser& q);
  std::unique_ptr<HttpParser> take_parser();
  void give_parser(std::unique_ptr<HttpParser> p);
  std::vector<std::unique_ptr<HttpParser>> parser_pool_;
  void on_upstream_response(Upstream* u);
  void finish_response(HttpParser& r, const Pend& p);
  void rewrite_response_headers(HttpParser& r);
  void pause_input(Conn* c, bool paused);
  void rearm(Conn* c);
  bool maybe_stream(Upstream* u);
  void resume_stream(uint64_t up_id);
  void stream_out(Upstream* u, std::string data, bool last);
  Upstream* pick_upstream(Client* c);
  int choose_server();
  void flush_client(Client* c);
  void flush_upstream(Upstream* u);
  void complete_slot(Client* c, Slot* s, Bytes data);
  void deliver(Client* c, Slot* s, Bytes obj);
  void fail_pend(Pend& p, int code, const char* reason);
  void release_waiters(const std::string& key, Bytes obj);
  void close_client(Client* c);
  void close_upstream(Upstream* u);
  void arm(Conn* c, bool out);
  void gc();
  Client* find_client(uint64_t id);
  Slot* find_slot(Client* c, uint64_t seq);
  void drain_posted();
  bool cacheable_response(const HttpParser& r, uint32_t* ttl) const;

  Proxy* px_;
  const ProxyConfig& cfg_;
  int id_;
  int epfd_ = -1, listen_fd_ = -1, evfd_ = -1, timerfd_ = -1;
  uint64_t next_id_ = kFirstConnId;
  std::unordered_map<uint64_t, Conn*> conns_;
  std::vector<Upstream*> pool_;
  std::vector<Conn*> graveyard_;
  std::mutex post_mu_;
  std::vector<std::function<void()>> posted_;
  // the loop is busy-polling (epoll_wait(0), posted work drained every pass): posters
  // skip the eventfd write — a syscall on their side and a read on this one, per
  // completion (the HBM batcher posts one per GPU batch)
  std::atomic<bool> spinning_{false};
  std::mt19937 rng_;
  std::vector<char> buf_;
  // collapsed forwarding: key -> requests waiting on the in-flight miss of the
  // same object (only the first one goes upstream)
  std::unordered_map<std::string, std::vector<std::pair<uint64_t, uint64_t>>> inflight_;
  // servers that answered "Connection: close": never pipeline onto them
  std::vector<char> server_nka_;
};

// =====================================================================================
Reactor::Reactor(Proxy* px, int id, int listen_fd)
    : px_(px), cfg_(px->cfg_), id_(id), listen_fd_(listen_fd), rng_(1234 + id), buf_(1 << 16),
      server_nka_(px->cfg_.upstreams.size(), 0) {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  timerfd_ = timerfd_create(CLOCK_MONOTONIC, TFD_NONBLOCK | TFD_CLOEXEC);
  itimerspec its{};
  its.it_interval.tv_sec = 1;
  its.it_value.tv_sec = 1;
  timerfd_settime(timerfd_, 0, &its, nullptr);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = kListenId;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, listen_fd_, &ev);
  ev.data.u64 = kEventId;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
  ev.data.u64 = kTimerId;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, timerfd_, &ev);
}

Reactor::~Reactor() {
  for (auto& kv : conns_) {
    close(kv.second->fd);
    delete kv.second;
  }
  for (Conn* c : graveyard_) delete c;
  close(listen_fd_);
  close(evfd_);
  close(timerfd_);
  close(epfd_);
}

void Reactor::post(std::function<void()> fn) {
  bool was_empty;
  {
    std::lock_guard<std::mutex> lk(post_mu_);
    was_empty = posted_.empty();
    posted_.push_back(std::move(fn));
  }
  // a non-empty queue already has a wake-up pending; a spinning loop needs none
  if (was_empty && !spinning_.load(std::memory_order_seq_cst)) wake();
}

void Reactor::post_batch(std::vector<std::function<void()>>& fns) {
  if (fns.empty()) return;
  bool was_empty;
  {
    std::lock_guard<std::mutex> lk(post_mu_);
    was_empty = posted_.empty();
    if (was_empty) {
      posted_.swap(fns);
    } else {
      for (auto& f : fns) posted_.push_back(std::move(f));
    }
  }
  fns.clear();
  if (was_empty && !spinning_.load(std::memory_order_seq_cst)) wake();
}

void Reactor::drain_posted() {
  std::vector<std::function<void()>> fns;
  {
    std::lock_guard<std::mutex> lk(post_mu_);
    fns.swap(posted_);
  }
  for (auto& f : fns) f();
}

void Reactor::arm(Conn* c, bool out) {
  if (c->dead || c->out_armed == out) return;
  c->out_armed = out;
  rearm(c);
}

void Reactor::pause_input(Conn* c, bool paused) {
  if (c->dead || c->in_paused == paused) return;
  c->in_paused = paused;
  rearm(c);
}

void Reactor::rearm(Conn* c) {
  epoll_event ev{};
  ev.events = (c->in_paused ? 0u : (uint32_t)(EPOLLIN | EPOLLRDHUP)) |
              (c->out_armed ? (uint32_t)EPOLLOUT : 0u);
  ev.data.u64 = c->id;
  epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev);
}

void Reactor::loop() {
  epoll_event evs[256];
  const double spin_s = cfg_.spin_us * 1e-6;
  double last_work = now_s();
  // the cache tier may take this thread's GETs directly (HbmBackend: the reactor writes
  // the edge-server job and polls its completion below, no batcher thread either way)
  CacheBackend* const be = px_->backend_.get();
  if (be) be->direct_attach(this);
  bool direct_busy = false;
  while (px_->running_) {
    const bool spin = spin_s > 0 && now_s() - last_work < spin_s;
    int timeout_ms = 0;
    if (spin) {
      spinning_.store(true, std::memory_order_seq_cst);
    } else {
      // leaving the spin: a poster that still saw spinning_ did not write the eventfd,
      // so look at the queue after clearing the flag (both seq_cst: one of the two sides
      // sees the other) and block only when it is empty
      spinning_.store(false, std::memory_order_seq_cst);
      std::lock_guard<std::mutex> lk(post_mu_);
      timeout_ms = posted_.empty() && !direct_busy ? 100 : 0;
    }
    const int n = epoll_wait(epfd_, evs, 256, timeout_ms);
    const double t_it = n > 0 ? now_s() : 0;
    if (n > 0 && spin_s > 0) last_work = t_it;
    for (int i = 0; i < n; ++i) {
      const uint64_t id = evs[i].data.u64;
      const double t0 = now_s();
      if (id == kListenId) {
        accept_all();
        phase_done(0, t0);
      } else if (id == kEventId) {
        uint64_t v;
        (void)!read(evfd_, &v, 8);
      } else if (id == kTimerId) {
        uint64_t v;
        (void)!read(timerfd_, &v, 8);
        gc();
        phase_done(4, t0);
      } else {
        auto it = conns_.find(id);
        if (it == conns_.end() || it->second->dead) continue;
        Conn* c = it->second;
        if (c->kind == 0) {
          on_client(static_cast<Client*>(c), evs[i].events);
          phase_done(1, t0);
        } else {
          on_upstream(static_cast<Upstream*>(c), evs[i].events);
          phase_done(2, t0);
        }
      }
    }
    {
      const double t0 = now_s();
      drain_posted();
      // GETs this iteration accepted go to the GPU now; finished ones are answered here
      if (be) {
        direct_busy = be->direct_service();
        if (direct_busy && spin_s > 0) last_work = t0;
      }
      phase_done(3, t0);
    }
    for (Conn* c : graveyard_) delete c;
    graveyard_.clear();
    if (n > 0) {
      const uint64_t us = (uint64_t)((now_s() - t_it) * 1e6);
      if (us > loop_max_us.load(std::memory_order_relaxed)) loop_max_us.store(us);
      if (us > 10000) loop_slow.fetch_add(1, std::memory_order_relaxed);
    }
  }
  if (be) be->direct_detach();  // answers (or hands to the batcher) what it still holds
}

void Reactor::accept_all() {
  for (;;) {
    sockaddr_in sa{};
    socklen_t len = sizeof sa;
    const int fd = accept4(listen_fd_, reinterpret_cast<sockaddr*>(&sa), &len,
                           SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) return;
    set_nodelay(fd);
    auto* c = new Client();
    c->fd = fd;
    c->kind = 0;
    c->id = next_id_++;
    c->ctime = c->atime = now_s();
    c->loopback = (ntohl(sa.sin_addr.s_addr) >> 24) == 127;
    conns_[c->id] = c;
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = c->id;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
    accepts++;
    clients++;
  }
}

Client* Reactor::find_client(uint64_t id) {
  auto it = conns_.find(id);
  if (it == conns_.end() || it->second->dead || it->second->kind != 0) return nullptr;
  return static_cast<Client*>(it->second);
}

Slot* Reactor::find_slot(Client* c, uint64_t seq) {
  for (auto& s : c->slots)
    if (s->seq == seq) return s.get();
  return nullptr;
}

// ---------------------------------------------------------------------------------
// client side
// ---------------------------------------------------------------------------------
void Reactor::on_client(Client* c, uint32_t ev) {
  if (ev & EPOLLOUT) flush_client(c);
  if (c->dead) return;
  if (ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
    for (;;) {
      const ssize_t r = recv(c->fd, buf_.data(), buf_.size(), 0);
      if (r > 0) {
        c->atime = now_s();
        const char* p = buf_.data();
        size_t n = (size_t)r;
        while (n > 0 && !c->dead && !c->closing) {
          const size_t used = c->req->parse(p, n);
          p += used;
          n -= used;
          if (c->req->error()) {
            bad_requests++;
            auto s = std::make_unique<Slot>();
            s->seq = c->next_seq++;
            s->out.write(simple_response(400, "Bad Request", cfg_.server_name, "bad request\n",
                                         "text/plain", true));
            s->out.close();
            s->ready = true;
            s->close_after = true;
            c->slots.push_back(std::move(s));
            c->closing = true;
            break;
          }
          if (c->req->message_complete()) {
            on_request(c);
            if (c->dead) return;
            if (c->req) c->req->reset();
            else c->req = take_parser();  // the request moved into its slot
          } else if (used == 0) {
            break;
          }
        }
        if (c->dead) return;
        if ((size_t)r < buf_.size()) break;
        continue;
      }
      if (r == 0) {  // client EOF: finish every queued response, then close
        c->eof = true;
        c->closing = true;
        if (c->slots.empty()) close_client(c);
        else flush_client(c);
        return;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      // a client that resets its connection has just gone away; not a proxy error
      if (errno == ECONNRESET) client_resets++;
      else errors++;
      close_client(c);
      return;
    }
    flush_client(c);
  }
}

void Reactor::on_request(Client* c) {
  HttpParser& q = *c->req;
  c->nreq++;
  requests++;
  const std::string url = q.url();
  if (cfg_.kill_switch && url == "/kill" && (!cfg_.kill_loopback_only || c->loopback)) {
    // KILL SWITCH (Server.py:329-331: sys.exit(0))
    std::fprintf(stderr, "[shellac] /kill received; shutting down\n");
    px_->stop();
    return;
  }
  auto s = std::make_unique<Slot>();
  Slot* sp = s.get();
  s->seq = c->next_seq++;
  s->t0 = now_s();
  s->close_after = !q.keep_alive() || c->nreq >= cfg_.client_max_reqs;
  if (url == "/_shellac/stats" || url == "/_shellac/metrics") {
    // the same counters as JSON, or in the Prometheus text format for a scraper
    const bool prom = url == "/_shellac/metrics";
    s->out.write(simple_response(200, "OK", cfg_.server_name,
                                 prom ? prometheus_text(px_->stats_json()) : px_->stats_json(),
                                 prom ? "text/plain; version=0.0.4" : "application/json",
                                 s->close_after));
    s->out.close();
    s->ready = true;
    c->slots.push_back(std::move(s));
    flush_client(c);
    return;
  }
  const std::string& method = q.method();
  s->head = method == "HEAD";
  s->client_gzip = contains_ci(q.header("accept-encoding"), "gzip");
  const std::string* host = q.header("host");
  s->key = cfg_.key_host && host ? *host + url : url;  // reference key: URL (Server.py:327)
  s->base_key = s->key;
  s->d = digest_bytes(reinterpret_cast<const uint8_t*>(s->key.data()), s->key.size());
  s->lookup = px_->cfg_.cache_enabled &&
              (cfg_.policy == "reference" || method == "GET") && !q.header("authorization");
  if (s->lookup) s->req = std::move(c->req);  // serialized only if the cache misses
  else s->fwd = upstream_request(q);
  c->slots.push_back(std::move(s));
  if (sp->lookup) {
    const uint64_t cid = c->id, seq = sp->seq;
    px_->backend_->get(sp->key, sp->d, this, [this, cid, seq](bool hit, CacheValue v) {
      on_cache(cid, seq, hit, std::move(v));
    });
  } else {
    forward(c, sp);
  }
}

void Reactor::on_cache(uint64_t cid, uint64_t seq, bool hit, CacheValue v) {
  Client* c = find_client(cid);
  if (!c) return;
  Slot* s = find_slot(c, seq);
  if (!s || s->ready) return;
  if (hit && v.data && is_vary_marker(v.data->view())) {
    // the URL's responses Vary: look the variant of this request up under its own key
    // (a marker found by a variant lookup, or without the request, counts as a miss)
    if (cfg_.policy == "rfc" && !s->vary_probe && s->req) {
      s->key = vary_key(s->base_key, marker_names(v.data->view()), s->req->headers());
      s->d = digest_bytes(reinterpret_cast<const uint8_t*>(s->key.data()), s->key.size());
      s->vary_probe = true;
      px_->backend_->get(s->key, s->d, this, [this, cid, seq](bool h2, CacheValue v2) {
        on_cache(cid, seq, h2, std::move(v2));
      });
      return;
    }
    hit = false;
  }
  if (hit && v.data) {
    hits++;
    if (s->vary_probe) vary_hits++;
    deliver(c, s, v.data);
    return;
  }
  misses++;
  auto it = inflight_.find(s->key);
  if (it != inflight_.end()) {  // same object already being fetched: wait for it
    collapsed++;
    it->second.emplace_back(cid, seq);
    return;
  }
  inflight_[s->key];  // this request leads the fetch
  forward(c, s);
}

// The last response on a connection announces the close (cached objects carry
// "Connection: keep-alive" from the fill, Server.py:414-415).
static Bytes with_connection_close(const Bytes& obj) {
  const std::string_view ov = obj.view();
  const size_t eoh = ov.find("\r\n\r\n");
  if (eoh == std::string::npos) return obj;
  std::string head(ov.substr(0, eoh + 2));
  std::string out;
  out.reserve(obj->size() + 8);
  size_t pos = 0;
  while (pos < head.size()) {
    size_t e = head.find("\r\n", pos);
    if (e == std::string::npos) e = head.size();
    const std::string line = head.substr(pos, e - pos);
    const std::string low = to_lower(line.substr(0, line.find(':')));
    if (pos == 0 || (low != "connection" && low != "keep-alive")) {
      out += line;
      out += "\r\n";
    }
    pos = e + 2;
  }
  out += "Connection: close\r\n\r\n";
  out.append(ov.substr(eoh + 4));
  return std::make_shared<const std::string>(std::move(out));
}

// A cached (or just fetched) object to one client: under policy rfc a gzip-coded object
// goes to a client without `Accept-Encoding: gzip` as its identity variant.
void Reactor::deliver(Client* c, Slot* s, Bytes obj) {
  if (obj && !s->client_gzip && !s->head && cfg_.policy == "rfc" && object_is_gzip(obj->view())) {
    if (px_->gzip_ && px_->gzip_->can_inflate()) {
      // the GPU gzip service inflates it in a batch (zlib on its thread as the fallback);
      // the slot completes on this reactor when it returns, if the client is still there
      auto rp = std::make_shared<HttpParser>(false);
      rp->parse(obj->data(), obj->size());
      if (rp->message_complete() || rp->finish()) {
        std::string member = std::move(rp->mutable_body());
        const uint64_t cid = c->id, seq = s->seq;
        px_->gzip_->submit_inflate(
            std::move(member), cfg_.max_inflate_bytes,
            [this, rp, cid, seq](bool ok, std::string out) {
              post([this, rp, cid, seq, ok, out = std::move(out)]() mutable {
                Client* c2 = find_client(cid);
                Slot* s2 = c2 ? find_slot(c2, seq) : nullptr;
                if (!s2 || s2->ready) return;
                if (!ok) {
                  errors++;
                  complete_slot(c2, s2, std::make_shared<const std::string>(simple_response(
                                            502, "Bad Gateway", cfg_.server_name,
                                            "undecodable gzip object\n")));
                  return;
                }
                rp->remove_header("content-encoding");
                rp->mutable_body() = std::move(out);
                identity_decoded++;
                gzip_gpu_inflated++;
                complete_slot(c2, s2, std::make_shared<const std::string>(rp->serialize()));
              });
            });
        return;
      }
    }
    Bytes id = identity_variant(obj, cfg_.max_inflate_bytes);
    if (!id) {
      errors++;
      complete_slot(c, s, std::make_shared<const std::string>(simple_response(
                              502, "Bad Gateway", cfg_.server_name, "undecodable gzip object\n")));
      return;
    }
    identity_decoded++;
    obj = std::move(id);
  }
  complete_slot(c, s, std::move(obj));
}

void Reactor::complete_slot(Client* c, Slot* s, Bytes data) {
  if (s->req) give_parser(std::move(s->req));
  if (s->close_after && data) data = with_connection_close(data);
  s->out.write_shared(std::move(data));
  s->out.close();
  s->ready = true;
  const double us = (now_s() - s->t0) * 1e6;
  const int b = us < 1 ? 0 : std::min(kHistBuckets - 1, 1 + (int)std::log2(us));
  hist[b]++;
  flush_client(c);
}

void Reactor::flush_client(Client* c) {
  // Head-of-line ordered write of every *ready* response slot (Server.py:236-239),
  // many pipelined responses per writev.
  if (c->dead) return;
  for (;;) {
    iovec iov[64];
    int cnt = 0;
    size_t want = 0;
    for (auto& s : c->slots) {
      if (!(s->ready || s->streaming) || cnt >= 64) break;
      const int k = s->out.iov(iov + cnt, 64 - cnt);
      for (int j = 0; j < k; ++j) want += iov[cnt + j].iov_len;
      cnt += k;
      if (!s->ready) break;  // a response still streaming holds back its successors
    }
    if (cnt == 0) break;
    const ssize_t w = writev(c->fd, iov, cnt);
    if (w < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        arm(c, true);
        return;
      }
      if (errno == ECONNRESET || errno == EPIPE) client_resets++;
      else errors++;
      close_client(c);
      return;
    }
    bytes_out += (uint64_t)w;
    c->atime = now_s();
    size_t left = (size_t)w;
    while (!c->slots.empty() && (c->slots.front()->ready || c->slots.front()->streaming)) {
      Slot* s = c->slots.front().get();
      const size_t take = std::min<size_t>(left, s->out.pending());
      s->out.ack(take);
      left -= take;
      if (!s->out.complete()) break;
      const bool last = s->close_after;
      if (s->stream_up) resume_stream(s->stream_up);
      c->slots.pop_front();
      if (last) {  // "Connection: close" / max requests reached / bad request
        close_client(c);
        return;
      }
    }
    if (!c->slots.empty()) {
      Slot* f = c->slots.front().get();
      if (f->streaming && f->stream_up && f->out.pending() < cfg_.stream_high_water / 4)
        resume_stream(f->stream_up);
    }
    if ((size_t)w < want) {
      arm(c, true);
      return;
    }
  }
  if (c->eof && c->slots.empty()) {
    close_client(c);
    return;
  }
  arm(c, false);
}

void Reactor::close_client(Client* c) {
  if (c->dead) return;
  c->dead = true;
  epoll_ctl(epfd_, EPOLL_CTL_DEL, c->fd, nullptr);
  close(c->fd);
  conns_.erase(c->id);
  clients--;
  if (c->up) {
    // release the pooled upstream (Server.py:189-192); its in-flight responses
    // still complete and fill the cache
    if (c->up->owner == c) c->up->owner = nullptr;
    c->up = nullptr;
  }
  for (auto& s : c->slots)  // a stream paused for this client drains (and is dropped)
    if (s->stream_up) resume_stream(s->stream_up);
  graveyard_.push_back(c);
}

// ---------------------------------------------------------------------------------
// upstream side
// ---------------------------------------------------------------------------------
int Reactor::choose_server() {
  const int n = (int)cfg_.upstreams.size();
  if (n == 0) return -1;
  const double t = now_s();
  std::vector<int> up;
  for (int i = 0; i < n; ++i)
    if (px_->upstream_up(i, t)) up.push_back(i);
  if (up.empty()) return -1;
  if (cfg_.balance == "roundrobin") return up[(size_t)px_->next_rr() % up.size()];
  if (cfg_.balance == "leastconn") {
    std::vector<int> load(n, 0);
    for (Upstream* u : pool_) load[u->server] += (int)u->pend.size() + (u->owner ? 1 : 0);
    int best = up[0];
    for (int i : up)
      if (load[i] < load[best]) best = i;
    return best;
  }
  return up[std::uniform_int_distribution<size_t>(0, up.size() - 1)(rng_)];  // Server.py:123
}

Upstream* Reactor::pick_upstream(Client* c) {
  const double t = now_s();
  auto valid = [&](Upstream* u) {
    if (u->dead || !px_->upstream_healthy(u->server)) return false;
    if (u->count >= u->ka_max) return false;
    return u->ka_timeout < 0 || t - u->atime < u->ka_timeout;
  };
  if (c->up && valid(c->up)) return c->up;  // affinity (Server.py:94-101)
  if (c->up) {
    if (c->up->owner == c) c->up->owner = nullptr;
    c->up = nullptr;
  }
  for (Upstream* u : pool_) {  // reuse a free pooled connection (Server.py:103-116)
    if (!u->owner && valid(u) && px_->upstream_up(u->server, t)) {
      u->owner = c;
      c->up = u;
      return u;
    }
  }
  for (int attempt = 0; attempt < (int)cfg_.upstreams.size() + 1; ++attempt) {
    const int srv = choose_server();
    if (srv < 0) return nullptr;
    const int fd = connect_nonblock(cfg_.upstreams[srv]);  // non-blocking (ref blocks, :126)
    if (fd < 0) {
      px_->upstream_failed(srv, t);
      upstream_failures++;
      continue;
    }
    auto* u = new Upstream();
    if (server_nka_[srv]) u->ka_max = 1;
    u->fd = fd;
    u->kind = 1;
    u->id = next_id_++;
    u->server = srv;
    u->ctime = u->atime = t;
    conns_[u->id] = u;
    pool_.push_back(u);
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP | EPOLLOUT;
    ev.data.u64 = u->id;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
    u->out_armed = true;
    upstreams++;
    u->owner = c;
    c->up = u;
    return u;
  }
  return nullptr;
}

// The request as forwarded upstream: gzip forced (Server.py:358), hop-by-hop headers
// dropped, the upstream connection kept alive for the pool.
std::string Reactor::upstream_request(HttpParser& q) {
  q.set_header("accept-encoding", "gzip");
  q.remove_header("proxy-connection");
  q.remove_header("keep-alive");
  q.set_header("connection", "keep-alive");
  return q.serialize();
}

std::unique_ptr<HttpParser> Reactor::take_parser() {
  if (parser_pool_.empty()) return std::make_unique<HttpParser>(true);
  auto p = std::move(parser_pool_.back());
  parser_pool_.pop_back();
  return p;
}

void Reactor::give_parser(std::unique_ptr<HttpParser> p) {
  if (!p || parser_pool_.size() >= 4096) return;
  p->reset();
  parser_pool_.push_back(std::move(p));
}

void Reactor::forward(Client* c, Slot* s) {
  s->attempts++;
  if (s->fwd.empty() && s->req) {
    if (s->lookup && cfg_.policy == "rfc")  // a Vary'd response is keyed by these
      s->req_headers = std::make_shared<const std::vector<Header>>(s->req->headers());
    s->fwd = upstream_request(*s->req);
    give_parser(std::move(s->req));
  }
  Upstream* u = pick_upstream(c);
  if (!u) {
    complete_slot(c, s, std::make_shared<const std::string>(simple_response(
                            503, "Service Unavailable", cfg_.server_name, "no upstream available\n")));
    return;
  }
  u->out.write(s->fwd);
  u->pend.push_back(Pend{c->id, s->seq, s->key, s->d, s->lookup, s->head, s->client_gzip,
                        s->base_key, s->req_headers});
  u->count++;
  upstream_reqs++;
  flush_upstream(u);
}

void Reactor::flush_upstream(Upstream* u) {
  if (u->dead) return;
  if (!u->connected) {
    arm(u, true);
    return;
  }
  while (u->out.pending()) {
    iovec iov[64];
    const int cnt = u->out.iov(iov, 64);
    const ssize_t w = writev(u->fd, iov, cnt);
    if (w < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        arm(u, true);
        return;
      }
      close_upstream(u);
      return;
    }
    u->out.ack((uint64_t)w);
    u->atime = now_s();
  }
  u->out.release_acked();
  arm(u, false);
}

void Reactor::release_waiters(const std::string& key, Bytes obj) {
  auto it = inflight_.find(key);
  if (it == inflight_.end()) return;
  std::vector<std::pair<uint64_t, uint64_t>> waiters;
  waiters.swap(it->second);
  inflight_.erase(it);
  for (auto& w : waiters) {
    Client* c = find_client(w.first);
    if (!c) continue;
    Slot* s = find_slot(c, w.second);
    if (!s || s->ready) continue;
    if (obj) {
      hits++;
      deliver(c, s, obj);
    } else {
      forward(c, s);  // uncacheable ("hit-for-pass"): each waiter fetches its own copy
    }
  }
}

void Reactor::fail_pend(Pend& p, int code, const char* reason) {
  if (p.lookup && code != 502) release_waiters(p.key, nullptr);
  Client* c = find_client(p.client_id);
  if (!c) {
    if (p.lookup) release_waiters(p.key, nullptr);
    return;
  }
  Slot* s = find_slot(c, p.seq);
  if (!s || s->ready) return;
  if (s->attempts < 3 && code == 502) {  // idempotent retry on another connection
    retries++;
    if (c->up && c->up->dead) c->up = nullptr;
    forward(c, s);
    return;
  }
  if (p.lookup) release_waiters(p.key, nullptr);
  complete_slot(c, s, std::make_shared<const std::string>(
                          simple_response(code, reason, cfg_.server_name, "upstream failed\n")));
}

void Reactor::on_upstream(Upstream* u, uint32_t ev) {
  if ((ev & EPOLLOUT) && !u->connected) {
    int err = 0;
    socklen_t el = sizeof err;
    getsockopt(u->fd, SOL_SOCKET, SO_ERROR, &err, &el);
    if (err) {
      px_->upstream_failed(u->server, now_s());
      upstream_failures++;
      close_upstream(u);
      return;
    }
    u->connected = true;
  }
  if (ev & EPOLLOUT) flush_upstream(u);
  if (u->dead) return;
  if (!(ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR))) return;
  for (;;) {
    const ssize_t r = recv(u->fd, buf_.data(), buf_.size(), 0);
    if (r > 0) {
      u->atime = now_s();
      const char* p = buf_.data();
      size_t n = (size_t)r;
      while (n > 0 && !u->dead) {
        if (u->pend.empty()) {  // unsolicited bytes: protocol error
          close_upstream(u);
          return;
        }
        if (!u->resp) {
          u->resp = std::make_unique<HttpParser>(cfg_.decode_gzip);
          u->resp->set_max_decoded_bytes(cfg_.max_inflate_bytes);
          u->resp->set_no_body(u->pend.front().head);
          u->resp->set_eof_body(true);
        }
        const size_t used = u->resp->parse(p, n);
        p += used;
        n -= used;
        if (u->resp->error()) {
          close_upstream(u);
          return;
        }
        if (u->resp->message_complete()) {
          on_upstream_response(u);
          if (u->dead) return;
        } else if (u->resp->headers_complete() && maybe_stream(u)) {
          stream_out(u, std::move(u->resp->mutable_body()), false);
          u->resp->mutable_body().clear();
          if (used == 0) break;
        } else if (used == 0) {
          break;
        }
      }
      if ((size_t)r < buf_.size()) return;
      continue;
    }
    if (r == 0) {
      if (u->resp && u->resp->finish() && !u->pend.empty()) on_upstream_response(u);
      close_upstream(u);
      return;
    }
    if (errno == EAGAIN || errno == EWOULDBLOCK) return;
    close_upstream(u);
    return;
  }
}

bool Reactor::cacheable_response(const HttpParser& r, uint32_t* ttl) const {
  *ttl = cfg_.ttl;
  if (cfg_.policy == "reference") return true;  // Server.py:431-432 caches everything
  switch (r.status()) {
    case 200: case 203: case 204: case 300: case 301: case 404: case 405: case 410: case 414:
    case 501:
      break;
    default:
      return false;
  }
  const std::string* cc = r.header("cache-control");
  if (contains_ci(cc, "no-store") || contains_ci(cc, "private") || contains_ci(cc, "no-cache"))
    return false;
  if (r.header("set-cookie")) return false;
  const long ma = cc_max_age(cc);
  if (ma == 0) return false;
  if (ma > 0) *ttl = (uint32_t)ma;
  return true;
}

void Reactor::on_upstream_response(Upstream* u) {
  Pend p = std::move(u->pend.front());
  u->pend.pop_front();
  std::unique_ptr<HttpParser> rp = std::move(u->resp);
  HttpParser& r = *rp;
  const bool ka = r.keep_alive();
  const auto kap = r.keep_alive_params();
  responses++;
  if (u->streaming) {  // tail of a streamed response: nothing is cached
    u->pend.push_front(std::move(p));
    stream_out(u, std::move(r.mutable_body()), true);
    p = std::move(u->pend.front());
    u->pend.pop_front();
    u->streaming = false;
    if (p.lookup) release_waiters(p.key, nullptr);
    if (!ka) {
      server_nka_[u->server] = 1;
      close_upstream(u);
      return;
    }
    server_nka_[u->server] = 0;
    u->ka_timeout = kap.first;
    u->ka_max = kap.second;
    return;
  }
  rewrite_response_headers(r);
  const std::string* ce = r.header("content-encoding");
  bool deferred = false;
  // -z: under rfc the stored variant is gzip whichever client leads the fetch (a client
  // without gzip gets the identity variant from deliver()); the reference policy keeps
  // compressing only for gzip clients
  if (cfg_.compress && !ce && (p.client_gzip || cfg_.policy == "rfc") && r.body().size() >= 256) {
    const std::string* ct = r.header("content-type");
    if (ct && (contains_ci(ct, "text/") || contains_ci(ct, "json") || contains_ci(ct, "javascript") ||
               contains_ci(ct, "xml"))) {
      if (px_->gzip_) {
        // GPU: the body joins the current batch window; the response completes (cache
        // store, client slot, collapsed waiters) on this reactor when the batch returns.
        // Keep-alive bookkeeping of the upstream below does not wait for it.
        std::shared_ptr<HttpParser> rs(std::move(rp));
        auto ps = std::make_shared<Pend>(std::move(p));
        std::string body = std::move(rs->mutable_body());
        px_->gzip_->submit(std::move(body), [this, rs, ps](bool ok, std::string out) {
          post([this, rs, ps, ok, out = std::move(out)]() mutable {
            rs->mutable_body() = std::move(out);
            if (ok) {
              rs->set_header("content-encoding", "gzip");
              rs->set_header("vary", "Accept-Encoding");
              gzip_gpu_bodies++;
            }
            finish_response(*rs, *ps);
          });
        });
        deferred = true;
      } else {
        r.mutable_body() = gzip_compress(r.body(), 6);
        r.set_header("content-encoding", "gzip");
        r.set_header("vary", "Accept-Encoding");
      }
    }
  }
  if (!deferred) finish_response(r, p);
  if (!ka) {
    server_nka_[u->server] = 1;
    close_upstream(u);  // remaining pipelined requests are retried elsewhere
    return;
  }
  server_nka_[u->server] = 0;
  u->ka_timeout = kap.first;
  u->ka_max = kap.second;
}

// Cache store, client slot and collapsed waiters of a complete upstream response.
void Reactor::finish_response(HttpParser& r, const Pend& p) {
  Bytes obj;
  const bool rfc = cfg_.policy == "rfc";
  std::vector<std::string> vnames;
  if (rfc && !p.head) {
    vnames = vary_names(r);
    // one cache entry serves both codings: say so to downstream caches
    if (r.header("content-encoding") && !contains_ci(r.header("vary"), "accept-encoding")) {
      const std::string* v = r.header("vary");
      r.set_header("vary", v ? *v + ", Accept-Encoding" : std::string("Accept-Encoding"));
    }
  }
  if (p.head) {
    const std::string* cl = r.header("content-length");
    const uint64_t len = cl ? std::strtoull(cl->c_str(), nullptr, 10) : 0;
    obj = std::make_shared<const std::string>(r.serialize_head(len, cl != nullptr));
  } else {
    obj = std::make_shared<const std::string>(r.serialize());
  }
  uint32_t ttl = cfg_.ttl;
  bool cached = false, waiters_share = true;
  if (p.lookup && !p.head && cacheable_response(r, &ttl)) {
    if (vnames.empty()) {
      cached = true;
      px_->backend_->set(p.key, p.d, obj, 0, ttl);  // Server.py:432 mc.set(key, obj, time=ttl)
      cache_sets++;
    } else if (vnames[0] != "*" && p.req_headers) {
      // Vary: marker under the URL key, the object under this request's variant key
      const std::string vk = vary_key(p.base_key, vnames, *p.req_headers);
      std::string marker = kVaryMarker;
      for (size_t i = 0; i < vnames.size(); ++i) marker += (i ? "," : "") + vnames[i];
      const Digest bd = digest_bytes(reinterpret_cast<const uint8_t*>(p.base_key.data()),
                                     p.base_key.size());
      const Digest vd = digest_bytes(reinterpret_cast<const uint8_t*>(vk.data()), vk.size());
      px_->backend_->set(p.base_key, bd, std::make_shared<const std::string>(std::move(marker)), 0,
                         ttl);
      px_->backend_->set(vk, vd, obj, 0, ttl);
      cache_sets++;
      vary_stored++;
      cached = true;
      // requests collapsed onto the URL key may carry other header values: they fetch
      // their own variant; those collapsed onto this variant key share it
      waiters_share = p.key == vk;
    }  // Vary: * (or no request headers kept): not cacheable
  }
  if (Client* c = find_client(p.client_id)) {
    if (Slot* s = find_slot(c, p.seq)) {
      if (!s->ready) deliver(c, s, obj);
    }
  }
  if (p.lookup) release_waiters(p.key, cached && waiters_share ? obj : nullptr);
}

void Reactor::rewrite_response_headers(HttpParser& r) {
  // header rewrite (Server.py:412-416)
  r.set_header("server", cfg_.server_name);
  r.set_header("keep-alive", "timeout=5, max=100");
  r.set_header("connection", "keep-alive");
  r.remove_header("accept-ranges");
}

bool Reactor::maybe_stream(Upstream* u) {
  if (u->streaming) return true;
  HttpParser& r = *u->resp;
  const Pend& p = u->pend.front();
  if (p.head || r.body_decoded()) return false;
  const int64_t cl = r.content_length();
  const bool big = (!r.chunked() && cl >= 0 && (uint64_t)cl > cfg_.stream_bytes) ||
                   r.body().size() > cfg_.stream_bytes;
  if (!big) return false;
  Client* c = find_client(p.client_id);
  Slot* s = c ? find_slot(c, p.seq) : nullptr;
  u->streaming = true;
  u->stream_chunked = r.chunked() || cl < 0;
  streamed++;
  rewrite_response_headers(r);
  if (s && s->close_after) r.set_header("connection", "close");
  std::string head;
  if (u->stream_chunked) {
    head = r.serialize_head(0, false);
    head.insert(head.size() - 2, "Transfer-Encoding: chunked\r\n");
  } else {
    head = r.serialize_head((uint64_t)cl, true);
  }
  stream_out(u, std::move(head), false);
  return true;
}

// Append streamed bytes to the front request's client slot (`last` ends the response).
// Body pieces are re-framed as chunks when the length is unknown.
void Reactor::stream_out(Upstream* u, std::string data, bool last) {
  const Pend& p = u->pend.front();
  Client* c = find_client(p.client_id);
  Slot* s = c ? find_slot(c, p.seq) : nullptr;
  if (!s || s->ready) return;  // client gone: drain and drop
  const bool is_head = !s->streaming;
  std::string framed;
  if (!is_head && u->stream_chunked) {
    if (!data.empty()) {
      char hx[24];
      std::snprintf(hx, sizeof hx, "%zx\r\n", data.size());
      framed = hx;
      framed += data;
      framed += "\r\n";
    }
    if (last) framed += "0\r\n\r\n";
  } else {
    framed = std::move(data);
  }
  s->streaming = true;
  s->stream_up = u->id;
  if (!framed.empty()) s->out.write_shared(std::make_shared<const std::string>(std::move(framed)));
  if (last) {
    s->out.close();
    s->ready = true;
    const double us = (now_s() - s->t0) * 1e6;
    const int b = us < 1 ? 0 : std::min(kHistBuckets - 1, 1 + (int)std::log2(us));
    hist[b]++;
  }
  flush_client(c);
  if (!last && !c->dead && s->out.pending() > cfg_.stream_high_water && !u->in_paused) {
    stream_pauses++;
    pause_input(u, true);
  }
}

void Reactor::resume_stream(uint64_t up_id) {
  auto it = conns_.find(up_id);
  if (it != conns_.end() && !it->second->dead && it->second->in_paused)
    pause_input(it->second, false);
}

void Reactor::close_upstream(Upstream* u) {
  if (u->dead) return;
  u->dead = true;
  epoll_ctl(epfd_, EPOLL_CTL_DEL, u->fd, nullptr);
  close(u->fd);
  conns_.erase(u->id);
  upstreams--;
  pool_.erase(std::remove(pool_.begin(), pool_.end(), u), pool_.end());
  if (u->owner && u->owner->up == u) u->owner->up = nullptr;
  u->owner = nullptr;
  std::deque<Pend> pend;
  pend.swap(u->pend);
  graveyard_.push_back(u);
  if (u->streaming && !pend.empty()) {  // bytes already left: the client cannot be answered
    u->streaming = false;
    Pend p = std::move(pend.front());
    pend.pop_front();
    if (p.lookup) release_waiters(p.key, nullptr);
    if (Client* c = find_client(p.client_id)) close_client(c);
  }
  for (auto& p : pend) fail_pend(p, 502, "Bad Gateway");
}

void Reactor::gc() {
  // Client keep-alive policy (Server.py:155-166): idle timeout / max requests.
  const double t = now_s();
  std::vector<Client*> idle;
  std::vector<Upstream*> stale;
  for (auto& kv : conns_) {
    Conn* c = kv.second;
    if (c->dead) continue;
    if (c->kind == 0) {
      auto* cl = static_cast<Client*>(c);
      if (cl->slots.empty() &&
          (t - cl->atime >= cfg_.client_timeout || cl->nreq >= cfg_.client_max_reqs))
        idle.push_back(cl);
    } else {
      auto* u = static_cast<Upstream*>(c);
      if (u->pend.empty() && !u->owner && u->ka_timeout >= 0 &&
          (t - u->atime >= u->ka_timeout || u->count >= u->ka_max))
        stale.push_back(u);
    }
  }
  for (Client* c : idle) {
    gc_closed++;
    close_client(c);
  }
  for (Upstream* u : stale) close_upstream(u);
}

// =====================================================================================
// Proxy
// =====================================================================================
Proxy::Proxy(const ProxyConfig& cfg, std::shared_ptr<CacheBackend> backend)
    : cfg_(cfg), backend_(std::move(backend)) {
  SH_CHECK(!cfg_.upstreams.empty(), "no upstream web servers specified");
  SH_CHECK(cfg_.threads >= 1, "threads >= 1");
  if (cfg_.cache_enabled) SH_CHECK(backend_ != nullptr, "cache enabled without a backend");
  up_down_until_.reset(new std::atomic<double>[cfg_.upstreams.size()]);
  health_down_.reset(new std::atomic<bool>[cfg_.upstreams.size()]);
  for (size_t i = 0; i < cfg_.upstreams.size(); ++i) {
    up_down_until_[i] = 0;
    health_down_[i] = false;
  }
}

Proxy::~Proxy() {
  stop();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  if (health_th_.joinable()) health_th_.join();
}

bool Proxy::upstream_up(int idx, double now) const {
  return !health_down_[idx].load(std::memory_order_relaxed) && now >= up_down_until_[idx].load();
}

// One health probe: connect, `GET path`, read the status line; true for a status < 400
// within the timeout. Blocking I/O with poll() deadlines on the checker thread only.
static bool probe_upstream(const Addr& a, const std::string& path, int timeout_ms) {
  const double deadline = now_s() + timeout_ms * 1e-3;
  auto left_ms = [&] { return std::max(0, (int)((deadline - now_s()) * 1e3)); };
  const int fd = connect_nonblock(a);
  if (fd < 0) return false;
  bool ok = false;
  pollfd pfd{fd, POLLOUT, 0};
  if (poll(&pfd, 1, left_ms()) == 1 && (pfd.revents & POLLOUT)) {
    int err = 0;
    socklen_t el = sizeof err;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el);
    const std::string req = "GET " + path + " HTTP/1.1\r\nHost: " + a.host +
                            "\r\nUser-Agent: shellac-health\r\nConnection: close\r\n\r\n";
    if (!err && send(fd, req.data(), req.size(), MSG_NOSIGNAL) == (ssize_t)req.size()) {
      std::string head;
      char buf[512];
      while (head.find("\r\n") == std::string::npos && left_ms() > 0) {
        pfd = pollfd{fd, POLLIN, 0};
        if (poll(&pfd, 1, left_ms()) != 1) break;
        const ssize_t k = recv(fd, buf, sizeof buf, 0);
        if (k <= 0) break;
        head.append(buf, (size_t)k);
      }
      // "HTTP/1.x SSS ..."
      if (head.size() >= 12 && head.compare(0, 5, "HTTP/") == 0) {
        const int status = std::atoi(head.c_str() + 9);
        ok = status >= 100 && status < 400;
      }
    }
  }
  close(fd);
  return ok;
}

void Proxy::health_loop() {
  const size_t n = cfg_.upstreams.size();
  std::vector<int> fails(n, 0), passes(n, 0);
  while (running_) {
    for (size_t i = 0; i < n && running_; ++i) {
      const bool ok = probe_upstream(cfg_.upstreams[i], cfg_.health_path, cfg_.health_timeout_ms);
      health_checks_++;
      if (ok) {
        fails[i] = 0;
        if (health_down_[i] && ++passes[i] >= cfg_.health_passes) {
          health_down_[i] = false;
          health_transitions_++;
        }
      } else {
        passes[i] = 0;
        if (!health_down_[i] && ++fails[i] >= cfg_.health_fails) {
          health_down_[i] = true;
          health_transitions_++;
        }
      }
    }
    // sleep in small slices so stop() is prompt
    const double until = now_s() + cfg_.health_interval_ms * 1e-3;
    while (running_ && now_s() < until)
      std::this_thread::sleep_for(std::chrono::milliseconds(
          std::min(20, std::max(1, (int)((until - now_s()) * 1e3)))));
  }
}

void Proxy::upstream_failed(int idx, double now) {
  up_down_until_[idx] = now + cfg_.upstream_retry_s;
}

void Proxy::start() {
  SH_CHECK(!running_, "already running");
  reserve_fd_table(cfg_.max_fds);
  start_time_ = now_s();
  const int first = listen_tcp(cfg_.bind, cfg_.port, cfg_.threads > 1, cfg_.backlog);
  port_ = local_port(first);
  running_ = true;
  for (int i = 0; i < cfg_.threads; ++i) {
    const int fd = i == 0 ? first : listen_tcp(cfg_.bind, port_, true, cfg_.backlog);
    reactors_.emplace_back(new Reactor(this, i, fd));
  }
  for (size_t i = 0; i < reactors_.size(); ++i) {
    Reactor* rp = reactors_[i].get();
    threads_.emplace_back([this, rp, i] {
      pin_thread(cfg_.cpus, i);
      const std::string nm = "shellac-rx" + std::to_string(i);  // per-thread CPU accounting
      pthread_setname_np(pthread_self(), nm.c_str());
      rp->loop();
    });
  }
  if (!cfg_.health_path.empty()) health_th_ = std::thread([this] { health_loop(); });
}

void Proxy::wait() {
  for (auto& t : threads_)
    if (t.joinable()) t.join();
}

void Proxy::stop() {
  running_ = false;
  for (auto& r : reactors_) r->wake();
}

namespace {
// A minimal reader of the stats JSON above (objects, arrays, numbers, strings; no escapes
// beyond \" are ever produced), flattened into Prometheus samples: nested keys join with
// '_' under the `shellac_` prefix, array elements become an `i` label, and string fields
// (server, backend) become labels of one `shellac_info` sample.
struct PromFlat {
  const std::string& j;
  size_t p = 0;
  std::ostringstream out;
  std::vector<std::pair<std::string, std::string>> info;
  explicit PromFlat(const std::string& s) : j(s) {}
  void ws() {
    while (p < j.size() && (j[p] == ' ' || j[p] == '\n' || j[p] == '\t' || j[p] == '\r')) ++p;
  }
  std::string str() {
    std::string r;
    ++p;  // opening quote
    while (p < j.size() && j[p] != '"') {
      if (j[p] == '\\' && p + 1 < j.size()) ++p;
      r += j[p++];
    }
    ++p;
    return r;
  }
  static std::string clean(const std::string& k) {
    std::string r;
    for (char c : k) r += (std::isalnum((unsigned char)c) || c == '_') ? c : '_';
    return r;
  }
  void value(const std::string& name, const std::string& label) {
    ws();
    if (p >= j.size()) return;
    const char c = j[p];
    if (c == '{') {
      ++p;
      for (;;) {
        ws();
        if (p < j.size() && j[p] == '}') {
          ++p;
          return;
        }
        const std::string k = str();
        ws();
        ++p;  // ':'
        value(name.empty() ? clean(k) : name + "_" + clean(k), label);
        ws();
        if (p < j.size() && j[p] == ',') ++p;
      }
    } else if (c == '[') {
      ++p;
      for (int i = 0;; ++i) {
        ws();
        if (p < j.size() && j[p] == ']') {
          ++p;
          return;
        }
        value(name, "i=\"" + std::to_string(i) + "\"");
        ws();
        if (p < j.size() && j[p] == ',') ++p;
      }
    } else if (c == '"') {
      info.emplace_back(name, str());
    } else {
      const size_t a = p;
      while (p < j.size() && j[p] != ',' && j[p] != '}' && j[p] != ']' && !std::isspace((unsigned char)j[p])) ++p;
      out << "shellac_" << name;
      if (!label.empty()) out << "{" << label << "}";
      out << " " << j.substr(a, p - a) << "\n";
    }
  }
};
}  // namespace

std::string prometheus_text(const std::string& stats_json) {
  PromFlat f(stats_json);
  f.value("", "");
  std::ostringstream o;
  if (!f.info.empty()) {
    o << "shellac_info{";
    for (size_t i = 0; i < f.info.size(); ++i) {
      std::string v;
      for (char c : f.info[i].second) v += (c == '"' || c == '\\') ? '_' : c;
      o << (i ? "," : "") << f.info[i].first << "=\"" << v << "\"";
    }
    o << "} 1\n";
  }
  o << f.out.str();
  return o.str();
}

std::string Proxy::stats_json() {
  uint64_t req = 0, hit = 0, miss = 0, ur = 0, resp = 0, bo = 0, err = 0, cl = 0, up = 0, acc = 0,
           gcc = 0, sets = 0, bad = 0, uf = 0, rt = 0, col = 0, stm = 0, stp = 0, lmax = 0,
           lslow = 0, idd = 0, vst = 0, vh = 0;
  uint64_t pmax[5] = {}, crst = 0;
  uint64_t h[kHistBuckets] = {};
  for (auto& r : reactors_) {
    req += r->requests; hit += r->hits; miss += r->misses; ur += r->upstream_reqs;
    resp += r->responses; bo += r->bytes_out; err += r->errors; cl += r->clients;
    up += r->upstreams; acc += r->accepts; gcc += r->gc_closed; sets += r->cache_sets;
    bad += r->bad_requests; uf += r->upstream_failures; rt += r->retries; col += r->collapsed;
    stm += r->streamed; stp += r->stream_pauses;
    lmax = std::max<uint64_t>(lmax, r->loop_max_us);
    lslow += r->loop_slow;
    crst += r->client_resets;
    idd += r->identity_decoded;
    vst += r->vary_stored;
    vh += r->vary_hits;
    for (int k = 0; k < 5; ++k) pmax[k] = std::max<uint64_t>(pmax[k], r->phase_max_us[k]);
    for (int b = 0; b < kHistBuckets; ++b) h[b] += r->hist[b];
  }
  uint64_t total = 0;
  for (uint64_t v : h) total += v;
  auto pct = [&](double q) -> double {
    if (!total) return 0;
    uint64_t acc2 = 0;
    for (int b = 0; b < kHistBuckets; ++b) {
      acc2 += h[b];
      if (acc2 >= q * total) return b == 0 ? 1.0 : std::pow(2.0, b);  // bucket upper bound (us)
    }
    return std::pow(2.0, kHistBuckets);
  };
  std::ostringstream o;
  o << "{\"server\":\"" << cfg_.server_name << "\",\"uptime_s\":" << (now_s() - start_time_)
    << ",\"threads\":" << cfg_.threads << ",\"requests\":" << req << ",\"cache_hits\":" << hit
    << ",\"cache_misses\":" << miss << ",\"upstream_requests\":" << ur
    << ",\"upstream_responses\":" << resp << ",\"cache_fills\":" << sets
    << ",\"bytes_out\":" << bo << ",\"errors\":" << err << ",\"bad_requests\":" << bad
    << ",\"upstream_failures\":" << uf << ",\"retries\":" << rt << ",\"collapsed\":" << col
    << ",\"streamed\":" << stm << ",\"stream_pauses\":" << stp << ",\"clients\":" << cl
    << ",\"upstream_conns\":" << up << ",\"accepts\":" << acc << ",\"gc_closed\":" << gcc
    << ",\"client_resets\":" << crst << ",\"identity_decoded\":" << idd
    << ",\"vary_stored\":" << vst << ",\"vary_hits\":" << vh
    << ",\"loop_max_us\":" << lmax << ",\"loop_slow\":" << lslow
    << ",\"loop_phase_max_us\":{\"accept\":" << pmax[0] << ",\"client\":" << pmax[1]
    << ",\"upstream\":" << pmax[2] << ",\"posted\":" << pmax[3] << ",\"timer\":" << pmax[4]
    << "}"
    << ",\"latency_us\":{\"p50\":" << pct(0.5) << ",\"p99\":" << pct(0.99) << ",\"samples\":"
    << total << "}";
  if (gzip_) {
    uint64_t gb = 0, gi = 0;
    for (auto& r : reactors_) {
      gb += r->gzip_gpu_bodies;
      gi += r->gzip_gpu_inflated;
    }
    StatList gs;
    gzip_->stats(&gs);
    o << ",\"gzip_gpu\":{\"completed\":" << gb << ",\"identity_served\":" << gi;
    for (const auto& kv : gs) o << ",\"" << kv.first << "\":" << kv.second;
    o << "}";
  }
  o << ",\"health_checks\":" << health_checks_.load()
    << ",\"health_transitions\":" << health_transitions_.load() << ",\"upstreams_up\":[";
  const double tn = now_s();
  for (size_t i = 0; i < cfg_.upstreams.size(); ++i) o << (i ? "," : "") << (upstream_up((int)i, tn) ? 1 : 0);
  o << "]";
  if (backend_) {
    StatList st;
    backend_->stats(&st);
    o << ",\"backend\":\"" << backend_->name() << "\",\"cache\":{";
    for (size_t i = 0; i < st.size(); ++i)
      o << (i ? "," : "") << "\"" << st[i].first << "\":" << st[i].second;
    o << "}";
  }
  o << "}";
  return o.str();
}

}  // namespace shellac
