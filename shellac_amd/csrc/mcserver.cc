// memcached binary protocol server over a CacheBackend (see mcserver.h).
#include "mcserver.h"

#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/uio.h>

#include <ctime>
#include <deque>
#include <unordered_map>

#include "mcproto.h"

namespace shellac {

namespace {
constexpr uint64_t kListen = 1, kEvent = 2, kFirst = 16;

struct McSlot {
  std::string data;
  bool ready = false;
  bool close_after = false;
};

struct McClient {
  int fd = -1;
  uint64_t id = 0;
  std::string in;
  std::deque<std::unique_ptr<McSlot>> slots;
  bool dead = false, out_armed = false, quit = false;
};

uint32_t unix_now() { return (uint32_t)time(nullptr); }

Digest key_digest(const std::string& k) {
  return digest_bytes(reinterpret_cast<const uint8_t*>(k.data()), k.size());
}
}  // namespace

class McReactor : public Executor {
 public:
  McReactor(CacheServer* srv, int listen_fd) : srv_(srv), lfd_(listen_fd) {
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    ev_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event e{};
    e.events = EPOLLIN;
    e.data.u64 = kListen;
    epoll_ctl(ep_, EPOLL_CTL_ADD, lfd_, &e);
    e.data.u64 = kEvent;
    epoll_ctl(ep_, EPOLL_CTL_ADD, ev_, &e);
  }
  ~McReactor() override {
    for (auto& kv : clients_) {
      close(kv.second->fd);
      delete kv.second;
    }
    for (auto* c : dead_) delete c;
    close(lfd_);
    close(ev_);
    close(ep_);
  }
  void post(std::function<void()> fn) override {
    bool was_empty;
    {
      std::lock_guard<std::mutex> lk(mu_);
      was_empty = posted_.empty();
      posted_.push_back(std::move(fn));
    }
    if (was_empty) wake();  // a non-empty queue already has a wake-up pending
  }
  void post_batch(std::vector<std::function<void()>>& fns) override {
    if (fns.empty()) return;
    bool was_empty;
    {
      std::lock_guard<std::mutex> lk(mu_);
      was_empty = posted_.empty();
      for (auto& f : fns) posted_.push_back(std::move(f));
    }
    fns.clear();
    if (was_empty) wake();
  }
  void wake() {
    uint64_t one = 1;
    (void)!write(ev_, &one, 8);
  }
  void loop();
  std::atomic<uint64_t> ops{0};

 private:
  void on_readable(McClient* c);
  void handle(McClient* c, const mc::Frame& f);
  void flush(McClient* c);
  void close_client(McClient* c);
  McClient* find(uint64_t id) {
    auto it = clients_.find(id);
    return it == clients_.end() || it->second->dead ? nullptr : it->second;
  }
  McSlot* new_slot(McClient* c) {
    c->slots.emplace_back(new McSlot());
    return c->slots.back().get();
  }
  // complete a slot later (async backends); ids guard against closed clients
  template <typename F>
  void finish(uint64_t cid, McSlot* s, F&& fill) {
    McClient* c = find(cid);
    if (!c) return;
    fill(s);
    s->ready = true;
    flush(c);
  }

  CacheServer* srv_;
  int lfd_, ep_, ev_;
  uint64_t next_ = kFirst;
  std::unordered_map<uint64_t, McClient*> clients_;
  std::vector<McClient*> dead_;
  std::mutex mu_;
  std::vector<std::function<void()>> posted_;
};

void McReactor::loop() {
  epoll_event evs[128];
  char buf[1 << 16];
  while (srv_->running_) {
    const int n = epoll_wait(ep_, evs, 128, 100);
    for (int i = 0; i < n; ++i) {
      const uint64_t id = evs[i].data.u64;
      if (id == kListen) {
        for (;;) {
          const int fd = accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (fd < 0) break;
          set_nodelay(fd);
          auto* c = new McClient();
          c->fd = fd;
          c->id = next_++;
          clients_[c->id] = c;
          epoll_event e{};
          e.events = EPOLLIN | EPOLLRDHUP;
          e.data.u64 = c->id;
          epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
        }
      } else if (id == kEvent) {
        uint64_t v;
        (void)!read(ev_, &v, 8);
      } else {
        McClient* c = find(id);
        if (!c) continue;
        if (evs[i].events & EPOLLOUT) flush(c);
        if (c->dead) continue;
        if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
          bool eof = false;
          for (;;) {
            const ssize_t r = recv(c->fd, buf, sizeof buf, 0);
            if (r > 0) {
              c->in.append(buf, (size_t)r);
              if ((size_t)r < sizeof buf) break;
              continue;
            }
            if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) eof = true;
            break;
          }
          on_readable(c);
          if (eof && !c->dead) {
            if (c->slots.empty()) close_client(c);
            else c->quit = true;
          }
        }
      }
    }
    std::vector<std::function<void()>> fns;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fns.swap(posted_);
    }
    for (auto& f : fns) f();
    for (auto* c : dead_) delete c;
    dead_.clear();
  }
}

void McReactor::on_readable(McClient* c) {
  size_t pos = 0;
  mc::Frame f;
  while (!c->dead) {
    const size_t used = mc::next_frame(reinterpret_cast<const uint8_t*>(c->in.data()) + pos,
                                       c->in.size() - pos, &f);
    if (!used) break;
    if (f.h.magic != mc::kReqMagic) {
      close_client(c);
      return;
    }
    handle(c, f);
    pos += used;
  }
  if (!c->dead && pos) c->in.erase(0, pos);
  if (!c->dead) flush(c);
}

void McReactor::handle(McClient* c, const mc::Frame& f) {
  ops++;
  CacheBackend* be = srv_->backend_.get();
  const uint8_t op = f.h.opcode;
  const uint32_t opaque = f.h.opaque;
  const std::string key = f.key_str();
  const Digest d = key_digest(key);
  const uint64_t cid = c->id;
  McSlot* s = new_slot(c);
  auto reply = [op, opaque](McSlot* sl, uint16_t st, const std::string& k, const std::string& ex,
                            const std::string& val) {
    mc::response(sl->data, op, st, k, ex, val.data(), val.size(), opaque);
  };
  switch (op) {
    case mc::GET: case mc::GETQ: case mc::GETK: case mc::GETKQ: {
      const bool quiet = op == mc::GETQ || op == mc::GETKQ;
      const bool withkey = op == mc::GETK || op == mc::GETKQ;
      be->get(key, d, this, [this, cid, s, quiet, withkey, key, reply](bool hit, CacheValue v) {
        finish(cid, s, [&](McSlot* sl) {
          if (hit && v.data) {
            std::string ex;
            mc::put32(ex, v.flags);
            reply(sl, mc::OK, withkey ? key : std::string(), ex, v.data.str());
          } else if (!quiet) {
            reply(sl, mc::KEY_ENOENT, withkey ? key : std::string(), "", "Not found");
          }
        });
      });
      return;
    }
    case mc::SET: case mc::SETQ: case mc::ADD: case mc::ADDQ: case mc::REPLACE:
    case mc::REPLACEQ: {
      if (f.h.extlen < 8 || key.empty()) {
        reply(s, mc::INVALID_ARGS, "", "", "Invalid arguments");
        s->ready = true;
        return;
      }
      const uint32_t flags = mc::get32(f.extras);
      const uint32_t ttl = mc::exptime_to_relative(mc::get32(f.extras + 4), unix_now());
      auto val = std::make_shared<const std::string>((const char*)f.value, f.vlen);
      const bool quiet = op == mc::SETQ || op == mc::ADDQ || op == mc::REPLACEQ;
      if (op == mc::SET || op == mc::SETQ) {
        be->set(key, d, val, flags, ttl);
        if (!quiet) reply(s, mc::OK, "", "", "");
        s->ready = true;
        return;
      }
      const bool is_add = op == mc::ADD || op == mc::ADDQ;
      be->get(key, d, this, [this, be, cid, s, is_add, quiet, key, d, val, flags, ttl, reply](
                                bool hit, CacheValue) {
        finish(cid, s, [&](McSlot* sl) {
          if (is_add == hit) {
            reply(sl, is_add ? mc::KEY_EEXISTS : mc::KEY_ENOENT, "", "",
                  is_add ? "Data exists for key." : "Not found");
          } else {
            be->set(key, d, val, flags, ttl);
            if (!quiet) reply(sl, mc::OK, "", "", "");
          }
        });
      });
      return;
    }
    case mc::APPEND: case mc::PREPEND: {
      auto val = std::make_shared<const std::string>((const char*)f.value, f.vlen);
      const bool app = op == mc::APPEND;
      be->get(key, d, this, [this, be, cid, s, app, key, d, val, reply](bool hit, CacheValue v) {
        finish(cid, s, [&](McSlot* sl) {
          if (!hit || !v.data) {
            reply(sl, mc::NOT_STORED, "", "", "Not stored.");
            return;
          }
          auto nv = std::make_shared<const std::string>(app ? v.data.str() + *val
                                                            : *val + v.data.str());
          be->set(key, d, nv, v.flags, 0);
          reply(sl, mc::OK, "", "", "");
        });
      });
      return;
    }
    case mc::INCREMENT: case mc::DECREMENT: {
      if (f.h.extlen < 20) {
        reply(s, mc::INVALID_ARGS, "", "", "Invalid arguments");
        s->ready = true;
        return;
      }
      const uint64_t delta = mc::get64(f.extras), initial = mc::get64(f.extras + 8);
      const uint32_t exptime = mc::get32(f.extras + 16);
      const bool inc = op == mc::INCREMENT;
      be->get(key, d, this, [this, be, cid, s, inc, delta, initial, exptime, key, d, reply](
                                bool hit, CacheValue v) {
        finish(cid, s, [&](McSlot* sl) {
          uint64_t nv;
          if (!hit || !v.data) {
            if (exptime == 0xffffffffu) {
              reply(sl, mc::KEY_ENOENT, "", "", "Not found");
              return;
            }
            nv = initial;
          } else {
            char* endp = nullptr;
            const std::string cs = v.data.str();
            const unsigned long long cur = std::strtoull(cs.c_str(), &endp, 10);
            if (v.data->empty() || (endp && *endp)) {
              reply(sl, mc::DELTA_BADVAL, "", "", "Non-numeric server-side value for incr or decr");
              return;
            }
            nv = inc ? cur + delta : (cur > delta ? cur - delta : 0);
          }
          be->set(key, d, std::make_shared<const std::string>(std::to_string(nv)), 0,
                  mc::exptime_to_relative(exptime == 0xffffffffu ? 0 : exptime, unix_now()));
          std::string body;
          mc::put64(body, nv);
          reply(sl, mc::OK, "", "", body);
        });
      });
      return;
    }
    case mc::TOUCH: {
      const uint32_t ttl = f.h.extlen >= 4 ? mc::exptime_to_relative(mc::get32(f.extras), unix_now()) : 0;
      be->get(key, d, this, [this, be, cid, s, key, d, ttl, reply](bool hit, CacheValue v) {
        finish(cid, s, [&](McSlot* sl) {
          if (!hit || !v.data) {
            reply(sl, mc::KEY_ENOENT, "", "", "Not found");
            return;
          }
          be->set(key, d, v.data, v.flags, ttl);
          reply(sl, mc::OK, "", "", "");
        });
      });
      return;
    }
    case mc::DELETE: case mc::DELETEQ: {
      const bool quiet = op == mc::DELETEQ;
      be->del(key, d, this, [this, cid, s, quiet, reply](bool found) {
        finish(cid, s, [&](McSlot* sl) {
          if (!found) reply(sl, mc::KEY_ENOENT, "", "", "Not found");
          else if (!quiet) reply(sl, mc::OK, "", "", "");
        });
      });
      return;
    }
    case mc::NOOP:
      reply(s, mc::OK, "", "", "");
      break;
    case mc::VERSION:
      reply(s, mc::OK, "", "", srv_->cfg_.version);
      break;
    case mc::FLUSH: case mc::FLUSHQ:
      be->flush();
      if (op == mc::FLUSH) reply(s, mc::OK, "", "", "");
      break;
    case mc::STAT: {
      StatList st;
      be->stats(&st);
      st.emplace_back("curr_connections", clients_.size());
      st.emplace_back("server_ops", srv_->ops());
      for (auto& kv : st) reply(s, mc::OK, kv.first, "", std::to_string(kv.second));
      reply(s, mc::OK, "", "", "");
      break;
    }
    case mc::QUIT: case mc::QUITQ:
      if (op == mc::QUIT) reply(s, mc::OK, "", "", "");
      s->close_after = true;
      break;
    default:
      reply(s, mc::UNKNOWN_COMMAND, "", "", "Unknown command");
  }
  s->ready = true;
}

void McReactor::flush(McClient* c) {
  if (c->dead) return;
  for (;;) {
    iovec iov[64];
    int cnt = 0;
    size_t want = 0;
    for (auto& s : c->slots) {
      if (!s->ready || cnt >= 64) break;
      if (s->data.empty()) continue;
      iov[cnt].iov_base = s->data.data();
      iov[cnt].iov_len = s->data.size();
      want += s->data.size();
      ++cnt;
    }
    size_t left = 0;
    if (cnt) {
      const ssize_t w = writev(c->fd, iov, cnt);
      if (w < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        close_client(c);
        return;
      }
      left = (size_t)w;
    }
    bool progressed = false;
    while (!c->slots.empty() && c->slots.front()->ready) {
      McSlot* s = c->slots.front().get();
      const size_t take = std::min(left, s->data.size());
      s->data.erase(0, take);
      left -= take;
      if (!s->data.empty()) break;
      const bool last = s->close_after;
      c->slots.pop_front();
      progressed = true;
      if (last) {
        close_client(c);
        return;
      }
    }
    if (!cnt || !progressed || want == 0) break;
  }
  if (c->quit && c->slots.empty()) {
    close_client(c);
    return;
  }
  bool pending = false;
  for (auto& s : c->slots)
    if (s->ready && !s->data.empty()) pending = true;
  if (pending != c->out_armed) {
    epoll_event e{};
    e.events = EPOLLIN | EPOLLRDHUP | (pending ? EPOLLOUT : 0);
    e.data.u64 = c->id;
    epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &e);
    c->out_armed = pending;
  }
}

void McReactor::close_client(McClient* c) {
  if (c->dead) return;
  c->dead = true;
  epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
  close(c->fd);
  clients_.erase(c->id);
  dead_.push_back(c);
}

// =====================================================================================
CacheServer::CacheServer(const CacheServerConfig& cfg, std::shared_ptr<CacheBackend> backend)
    : cfg_(cfg), backend_(std::move(backend)) {
  SH_CHECK(backend_ != nullptr, "CacheServer needs a backend");
}

CacheServer::~CacheServer() {
  stop();
  wait();
}

void CacheServer::start() {
  SH_CHECK(!running_, "already running");
  const int first = listen_tcp(cfg_.bind, cfg_.port, cfg_.threads > 1, 1024);
  port_ = local_port(first);
  running_ = true;
  for (int i = 0; i < cfg_.threads; ++i) {
    const int fd = i == 0 ? first : listen_tcp(cfg_.bind, port_, true, 1024);
    reactors_.emplace_back(new McReactor(this, fd));
  }
  for (auto& r : reactors_) {
    McReactor* rp = r.get();
    threads_.emplace_back([rp] { rp->loop(); });
  }
}

void CacheServer::stop() {
  running_ = false;
  for (auto& r : reactors_) r->wake();
}

void CacheServer::wait() {
  for (auto& t : threads_)
    if (t.joinable()) t.join();
}

uint64_t CacheServer::ops() const {
  uint64_t n = 0;
  for (auto& r : reactors_) n += r->ops;
  return n;
}

}  // namespace shellac
