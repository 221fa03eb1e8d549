// Native HTTP load generator (ab-compatible knobs); see loadgen.cc.
#pragma once

#include <string>
#include <vector>

#include "net.h"

namespace shellac {

struct LoadConfig {
  std::string host = "127.0.0.1";
  uint16_t port = 8080;
  std::vector<std::string> paths{"/"};
  std::string method = "GET";
  std::vector<std::string> headers;  // "Name: value" (ab -H)
  int64_t requests = 10000;          // ab -n
  int concurrency = 10;              // ab -c
  int depth = 1;                     // pipelined requests per connection
  int threads = 1;
  std::vector<int> cpus;  // worker t runs on cpus[t % size] (empty: unpinned)
  int spin_us = 0;        // > 0: poll epoll without sleeping for this long after an event
  bool keepalive = true;             // ab -k
  double timeout_s = 60;
  // Generated request paths instead of `paths`: object ids 0..objects-1 as
  // path_prefix + id + path_suffix, drawn Zipf(zipf_s) (popularity ranks scattered over
  // ids by a fixed bijection) or, with zipf_s == 0, sequentially (request k -> id k mod
  // objects: a cache-fill pass).
  int64_t objects = 0;
  double zipf_s = 0.99;
  std::string path_prefix = "/obj/";
  std::string path_suffix = ".html";
  uint64_t seed = 1;
};

struct LoadSample {
  double start;    // seconds since the run started
  double latency;  // seconds (send -> complete response)
  int status;
};

struct LoadResult {
  std::vector<LoadSample> samples;
  uint64_t completed = 0, bytes = 0, errors = 0, non2xx = 0, reconnects = 0;
  double elapsed_s = 0;
  double connected_s = 0;  // when the last connection completed its handshake
  std::vector<double> connect_lat;  // per connection: connect() call -> writable (s)
  std::vector<double> connect_call;  // per connection: the connect() syscall itself (s)
  double open_loop_s = 0;            // longest per-thread loop opening its connections
};

LoadResult run_load(const LoadConfig& cfg);

}  // namespace shellac
