// Native origin server; see origin.h.
#include "origin.h"

#include <strings.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <unordered_map>

#include "common.h"
#include "net.h"

namespace shellac {

namespace {

struct Conn {
  std::string in;
  std::string out;
  size_t sent = 0;
  bool close_after = false;
};

std::string gzip_bytes(const std::string& s, int level) {
  z_stream z{};
  SH_CHECK(deflateInit2(&z, level, Z_DEFLATED, 31, 8, Z_DEFAULT_STRATEGY) == Z_OK,
           "deflateInit2 failed");
  std::string out(deflateBound(&z, s.size()) + 32, '\0');
  z.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(s.data()));
  z.avail_in = (uInt)s.size();
  z.next_out = reinterpret_cast<Bytef*>(&out[0]);
  z.avail_out = (uInt)out.size();
  const int rc = deflate(&z, Z_FINISH);
  deflateEnd(&z);
  SH_CHECK(rc == Z_STREAM_END, "deflate failed");
  out.resize(z.total_out);
  return out;
}

// Case-insensitive header lookup inside [head, head + len).
bool header_has(const char* head, size_t len, const char* name, const char* needle) {
  const size_t nl = strlen(name);
  const char* end = head + len;
  for (const char* p = head; p < end;) {
    const char* eol = static_cast<const char*>(memchr(p, '\n', end - p));
    if (!eol) eol = end;
    if ((size_t)(eol - p) > nl && strncasecmp(p, name, nl) == 0 && p[nl] == ':') {
      const std::string v(p + nl + 1, eol);
      if (strcasestr(v.c_str(), needle)) return true;
    }
    p = eol + 1;
  }
  return false;
}

int64_t content_length(const char* head, size_t len) {
  static const char kName[] = "content-length:";
  const char* end = head + len;
  for (const char* p = head; p < end;) {
    const char* eol = static_cast<const char*>(memchr(p, '\n', end - p));
    if (!eol) eol = end;
    if ((size_t)(eol - p) > sizeof kName - 1 && strncasecmp(p, kName, sizeof kName - 1) == 0)
      return strtoll(p + sizeof kName - 1, nullptr, 10);
    p = eol + 1;
  }
  return 0;
}

}  // namespace

NativeOrigin::NativeOrigin(const OriginConfig& cfg) : cfg_(cfg) {
  SH_CHECK(cfg_.threads >= 1, "origin needs at least one thread");
  const int first = listen_tcp(cfg_.host, cfg_.port, true, 4096);
  port_ = local_port(first);
  listen_fds_.push_back(first);
  for (int i = 1; i < cfg_.threads; ++i) listen_fds_.push_back(listen_tcp(cfg_.host, port_, true, 4096));
  wake_fd_ = eventfd(0, EFD_NONBLOCK);
}

NativeOrigin::~NativeOrigin() {
  stop();
  for (int fd : listen_fds_) close(fd);
  if (wake_fd_ >= 0) close(wake_fd_);
}

void NativeOrigin::start() {
  for (int fd : listen_fds_) threads_.emplace_back([this, fd] { loop(fd); });
}

void NativeOrigin::stop() {
  if (stop_.exchange(true)) return;
  uint64_t one = 1;
  if (write(wake_fd_, &one, sizeof one) < 0) {
  }
  for (auto& t : threads_) t.join();
  threads_.clear();
}

void NativeOrigin::loop(int lfd) {
  const int ep = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd;
  epoll_ctl(ep, EPOLL_CTL_ADD, lfd, &ev);
  ev.data.fd = wake_fd_;
  epoll_ctl(ep, EPOLL_CTL_ADD, wake_fd_, &ev);
  std::unordered_map<int, Conn> conns;
  const std::string filler(cfg_.body_bytes, 'x');
  std::vector<epoll_event> evs(256);
  char rbuf[16384];

  auto close_conn = [&](int fd) {
    epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
    close(fd);
    conns.erase(fd);
  };
  // Write what is pending; arm EPOLLOUT only while bytes remain.
  auto flush = [&](int fd, Conn& c) -> bool {
    while (c.sent < c.out.size()) {
      const ssize_t k = send(fd, c.out.data() + c.sent, c.out.size() - c.sent, MSG_NOSIGNAL);
      if (k < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        return false;
      }
      c.sent += (size_t)k;
    }
    epoll_event e{};
    e.data.fd = fd;
    if (c.sent == c.out.size()) {
      c.out.clear();
      c.sent = 0;
      if (c.close_after) return false;
      e.events = EPOLLIN | EPOLLRDHUP;
    } else {
      e.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
    }
    epoll_ctl(ep, EPOLL_CTL_MOD, fd, &e);
    return true;
  };
  auto serve = [&](Conn& c) {
    size_t pos = 0;
    for (;;) {
      const size_t he = c.in.find("\r\n\r\n", pos);
      if (he == std::string::npos) break;
      const char* head = c.in.data() + pos;
      const size_t hlen = he - pos;
      const int64_t clen = content_length(head, hlen);
      if (c.in.size() < he + 4 + (size_t)clen) break;
      const size_t sp1 = c.in.find(' ', pos);
      const size_t sp2 = c.in.find(' ', sp1 + 1);
      const std::string method = c.in.substr(pos, sp1 - pos);
      const std::string path = c.in.substr(sp1 + 1, sp2 - sp1 - 1);
      const bool http10 = c.in.compare(sp2 + 1, 8, "HTTP/1.0") == 0;
      const bool close_req = header_has(head, hlen, "connection", "close") ||
                             (http10 && !header_has(head, hlen, "connection", "keep-alive"));
      std::string body;
      if (cfg_.random_body) {
        body.resize((size_t)cfg_.body_bytes);
        uint64_t x = 0xcbf29ce484222325ull;  // FNV-1a of the path seeds a xorshift stream
        for (unsigned char ch : path) x = (x ^ ch) * 0x100000001b3ull;
        for (size_t k = 0; k < body.size(); k += 8) {
          x ^= x << 13;
          x ^= x >> 7;
          x ^= x << 17;
          std::memcpy(&body[k], &x, std::min<size_t>(8, body.size() - k));
        }
      } else if (cfg_.text_body) {
        static const char* kWords[] = {"<div class=\"item\">", "</div>", "<span>", "</span>",
                                       "<a href=\"/static/obj/", "\">", "</a>", "<li>", "</li>",
                                       "cache", "proxy", "memory", "the", "of", "and", "GPU",
                                       "request", "\n", "  ", "<p>", "</p>", "object"};
        constexpr int kNw = (int)(sizeof(kWords) / sizeof(kWords[0]));
        uint64_t x = 0xcbf29ce484222325ull;
        for (unsigned char ch : path) x = (x ^ ch) * 0x100000001b3ull;
        body = "<html>" + path + " #1 ";
        while ((int)body.size() < cfg_.body_bytes) {
          x ^= x << 13;
          x ^= x >> 7;
          x ^= x << 17;
          body += kWords[x % kNw];
          if ((x >> 20) % 7 == 0) body += std::to_string((x >> 32) % 10000000);
          body += ' ';
        }
        body.resize((size_t)cfg_.body_bytes);
      } else {
        body = "<html>" + path + " #1 " + filler + "</html>\n";
      }
      std::string extra;
      if (path.compare(0, 3, "/gz") == 0 && header_has(head, hlen, "accept-encoding", "gzip")) {
        body = gzip_bytes(body, cfg_.gzip_level);
        extra = "Content-Encoding: gzip\r\n";
      }
      c.out += "HTTP/1.1 200 OK\r\nServer: shellac-origin\r\nContent-Type: text/html\r\n";
      c.out += extra;
      c.out += "Content-Length: " + std::to_string(body.size()) + "\r\n";
      c.out += close_req ? "Connection: close\r\n\r\n" : "Keep-Alive: timeout=5, max=100000\r\n\r\n";
      if (method != "HEAD") c.out += body;
      requests_.fetch_add(1, std::memory_order_relaxed);
      pos = he + 4 + (size_t)clen;
      if (close_req) {
        c.close_after = true;
        break;
      }
    }
    c.in.erase(0, pos);
  };

  while (!stop_.load(std::memory_order_relaxed)) {
    const int n = epoll_wait(ep, evs.data(), (int)evs.size(), 200);
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == wake_fd_) continue;
      if (fd == lfd) {
        for (;;) {
          const int cfd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK);
          if (cfd < 0) break;
          set_nodelay(cfd);
          conns[cfd];
          epoll_event e{};
          e.events = EPOLLIN | EPOLLRDHUP;
          e.data.fd = cfd;
          epoll_ctl(ep, EPOLL_CTL_ADD, cfd, &e);
        }
        continue;
      }
      auto it = conns.find(fd);
      if (it == conns.end()) continue;
      Conn& c = it->second;
      bool ok = true;
      if (evs[i].events & EPOLLIN) {
        for (;;) {
          const ssize_t k = recv(fd, rbuf, sizeof rbuf, 0);
          if (k > 0) {
            c.in.append(rbuf, (size_t)k);
            continue;
          }
          if (k == 0) ok = false;  // peer closed
          else if (errno != EAGAIN && errno != EWOULDBLOCK) ok = false;
          break;
        }
        if (!c.close_after) serve(c);
      }
      if (!c.out.empty()) ok = flush(fd, c) && ok;
      else if (evs[i].events & (EPOLLHUP | EPOLLERR)) ok = false;
      if (!ok) close_conn(fd);
    }
  }
  for (auto& kv : conns) close(kv.first);
  close(ep);
}

}  // namespace shellac
