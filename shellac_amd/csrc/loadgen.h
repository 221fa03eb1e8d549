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
  bool keepalive = true;             // ab -k
  double timeout_s = 60;
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
};

LoadResult run_load(const LoadConfig& cfg);

}  // namespace shellac
