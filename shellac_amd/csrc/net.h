// Socket helpers shared by the proxy reactor, the memcached client and server.
#pragma once

#include <arpa/inet.h>
#include <fcntl.h>
#include <sys/resource.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sched.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace shellac {

struct Addr {
  std::string host;  // as given (DNS name or dotted quad)
  uint16_t port = 0;
  sockaddr_in sa{};  // resolved IPv4
  std::string str() const { return host + ":" + std::to_string(port); }
};

// Resolve "host" / "host:port" (reference: parse_server_list, Server.py:493-505).
inline Addr resolve(const std::string& spec, uint16_t default_port) {
  Addr a;
  const size_t c = spec.rfind(':');
  a.host = c == std::string::npos ? spec : spec.substr(0, c);
  a.port = c == std::string::npos ? default_port : (uint16_t)std::stoi(spec.substr(c + 1));
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const int rc = getaddrinfo(a.host.c_str(), nullptr, &hints, &res);
  SH_CHECK(rc == 0 && res, "cannot resolve host " + a.host);
  a.sa = *reinterpret_cast<sockaddr_in*>(res->ai_addr);
  a.sa.sin_port = htons(a.port);
  freeaddrinfo(res);
  return a;
}

inline std::vector<Addr> resolve_list(const std::string& csv, uint16_t default_port) {
  std::vector<Addr> out;
  size_t i = 0;
  while (i <= csv.size()) {
    size_t j = csv.find(',', i);
    if (j == std::string::npos) j = csv.size();
    const std::string part = csv.substr(i, j - i);
    if (!part.empty()) out.push_back(resolve(part, default_port));
    i = j + 1;
  }
  return out;
}

inline void set_nonblock(int fd) {
  const int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, fl | O_NONBLOCK);
}

// Pins the calling thread to cpus[i % size] (no-op for an empty list). Event-loop threads
// pinned to distinct cores of one socket keep a request's loopback/NIC, socket-buffer
// and reactor state in one L3 instead of migrating across a two-socket host.
inline void pin_thread(const std::vector<int>& cpus, size_t i) {
  if (cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpus[i % cpus.size()], &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
}

// Grows this process's file-descriptor table to cover `want` descriptors now. The kernel
// grows it by doubling as sockets are opened, and in a multi-threaded process every
// growth waits for an RCU grace period (expand_fdtable -> synchronize_rcu): measured on
// the GPU box at up to ~140 ms per growth, 0.5 s for a burst of 1000 connections. Done
// once at start-up, before the event loops run, the table never grows under load.
inline void reserve_fd_table(int want) {
  rlimit rl{};
  if (getrlimit(RLIMIT_NOFILE, &rl) != 0) return;
  const long top = std::min<long>(want, rl.rlim_cur == RLIM_INFINITY ? want : (long)rl.rlim_cur) - 1;
  if (top < 64) return;
  const int fd = open("/dev/null", O_RDONLY | O_CLOEXEC);
  if (fd < 0) return;
  if (fd < top && dup2(fd, (int)top) == (int)top) close((int)top);
  close(fd);
}

inline void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

// TCP_CORK helpers (reference: cork_socket / flush_socket, Server.py:481-487 —
// defined but unused there; the reactor corks a connection while it appends a
// pipelined batch of responses and flushes once).
inline void cork_socket(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_CORK, &one, sizeof one);
}
inline void flush_socket(int fd) {
  int zero = 0;
  setsockopt(fd, IPPROTO_TCP, TCP_CORK, &zero, sizeof zero);
}

// Listening socket: SO_REUSEADDR (+ SO_REUSEPORT so every reactor thread can own
// one), a real backlog (the reference uses listen(1), Server.py:73), non-blocking.
inline int listen_tcp(const std::string& bind_host, uint16_t port, bool reuseport, int backlog) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  SH_CHECK(fd >= 0, "socket() failed");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (reuseport) setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(port);
  if (inet_pton(AF_INET, bind_host.c_str(), &sa.sin_addr) != 1) sa.sin_addr.s_addr = INADDR_ANY;
  if (bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
    const int e = errno;
    close(fd);
    throw Error("bind(" + bind_host + ":" + std::to_string(port) + ") failed: " + strerror(e));
  }
  SH_CHECK(listen(fd, backlog) == 0, "listen() failed");
  set_nonblock(fd);
  return fd;
}

inline uint16_t local_port(int fd) {
  sockaddr_in sa{};
  socklen_t len = sizeof sa;
  getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &len);
  return ntohs(sa.sin_port);
}

// Non-blocking connect (the reference blocks the reactor in connect(), Server.py:126).
// Returns fd (connection in progress or done) or -1.
inline int connect_nonblock(const Addr& a) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  set_nonblock(fd);
  set_nodelay(fd);
  const int rc = connect(fd, reinterpret_cast<const sockaddr*>(&a.sa), sizeof a.sa);
  if (rc != 0 && errno != EINPROGRESS) {
    close(fd);
    return -1;
  }
  return fd;
}

inline double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

}  // namespace shellac
