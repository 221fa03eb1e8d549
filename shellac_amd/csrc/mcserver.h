// memcached-binary-protocol server exporting a CacheBackend (HBM or DRAM shards).
//
// With it, a node's GPU shards join the cluster-wide cache exactly the way the
// reference's memcached nodes do (README.md:30; Server.py:81-83): other proxies
// reach it through their ketama ring. Supported: GET/GETQ/GETK/GETKQ, SET/SETQ,
// ADD/ADDQ, REPLACE/REPLACEQ, DELETE/DELETEQ, APPEND/PREPEND, INCREMENT/DECREMENT,
// TOUCH, NOOP, VERSION, STAT, FLUSH/FLUSHQ, QUIT/QUITQ. Responses are returned in
// request order per connection even though backend completions are async.
// ADD/REPLACE/APPEND/INCR are read-modify-write through the backend and are
// atomic per connection, not across connections (documented limitation).
#pragma once

#include <atomic>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "backend.h"

namespace shellac {

struct CacheServerConfig {
  std::string bind = "0.0.0.0";
  uint16_t port = 11211;
  int threads = 1;
  std::string version = "shellac-0.2.0";
};

class McReactor;

class CacheServer {
 public:
  CacheServer(const CacheServerConfig& cfg, std::shared_ptr<CacheBackend> backend);
  ~CacheServer();
  void start();
  void stop();
  void wait();
  uint16_t port() const { return port_; }
  bool running() const { return running_; }
  uint64_t ops() const;

 private:
  friend class McReactor;
  CacheServerConfig cfg_;
  std::shared_ptr<CacheBackend> backend_;
  std::vector<std::unique_ptr<McReactor>> reactors_;
  std::vector<std::thread> threads_;
  std::atomic<bool> running_{false};
  uint16_t port_ = 0;
};

}  // namespace shellac
