// Native HTTP/1.1 origin server for the miss-path benchmark (stands in for the
// reference's Apache upstream, benchmarks/run-baseline.sh). The Python origin
// (utils/origin.py) is the test fixture; this one exists so that the proxy's miss
// throughput is measured against an origin that is not itself the bottleneck.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

namespace shellac {

struct OriginConfig {
  std::string host = "127.0.0.1";
  uint16_t port = 0;     // 0 = ephemeral
  int threads = 2;       // one epoll loop + SO_REUSEPORT listener each
  int body_bytes = 1024; // filler bytes per body, like utils/origin.py
  int gzip_level = 1;    // /gz* paths are gzip-encoded when the client accepts it
  // incompressible bodies: body_bytes of pseudo-random bytes seeded by the path (the same
  // object always has the same body), so cached objects are body_bytes on the wire
  bool random_body = false;
  // compressible text bodies: body_bytes of HTML-like markup built from a small word list
  // by a generator seeded with the path (zlib -6 reaches ~0.3 on it, like real pages)
  bool text_body = false;
};

class NativeOrigin {
 public:
  explicit NativeOrigin(const OriginConfig& cfg);
  ~NativeOrigin();
  void start();
  void stop();
  uint16_t port() const { return port_; }
  uint64_t requests() const { return requests_.load(std::memory_order_relaxed); }

 private:
  void loop(int listen_fd);

  OriginConfig cfg_;
  uint16_t port_ = 0;
  std::vector<int> listen_fds_;
  std::vector<std::thread> threads_;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> requests_{0};
  int wake_fd_ = -1;
};

}  // namespace shellac
