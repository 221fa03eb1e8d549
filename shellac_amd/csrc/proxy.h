// The caching reverse proxy: native epoll reactors, pipelined client connections,
// pooled upstream connections, asynchronous cache backends.
//
// Reference map (src/python/shellac/server/Server.py):
//   C1 reactor loop            run()                 :442-478   -> Reactor::loop
//   C2 listener / accept       __init__/_new_connection :70-77, :137-153 -> accept_all
//   C3 client table + keep-alive policy (30 s / 1000 req) :22-24, :150-166 -> Client, gc()
//   C4 upstream pool + balancer _get_upstream_fd      :86-134   -> pick_upstream
//   C5 request path            _read_requests        :302-378  -> on_request
//   C6 response path           _read_responses       :380-440  -> on_upstream_response
//   C7 ordered pipelining      _responses/_stream_map :39-43, :342, :369-374 -> Slot FIFO
//   C9 write path              _write_response/_write_request :227-292 -> flush_client/flush_upstream
//   C12 teardown               _close_client/_close_upstream :168-217 -> close_client/close_upstream
// Deliberate fixes: reactor threads with SO_REUSEPORT and a real backlog (ref:
// one thread, listen(1)); non-blocking upstream connect (ref blocks, :126);
// EPOLLOUT armed only while bytes are pending (ref spins on idle upstreams, :439);
// client EOF closes the connection (ref leaks it until GC); atime starts at
// accept (ref starts at 0 so GC may kill fresh clients, :151); a non-keep-alive
// upstream no longer tears down its client (ref :423-425) — pending requests get
// a 502 instead; responses of departed clients still fill the cache.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "backend.h"
#include "net.h"

namespace shellac {

struct ProxyConfig {
  std::string bind = "0.0.0.0";
  uint16_t port = 8080;               // -p (Server.py:512)
  std::vector<Addr> upstreams;        // -s
  int threads = 1;
  std::vector<int> cpus;  // reactor i runs on cpus[i % size] (empty: unpinned)
  // > 0: a reactor that had work within the last spin_us polls epoll without sleeping
  // (a dedicated core: no wake-up IPI or idle-state exit per request under load)
  int spin_us = 0;
  uint32_t ttl = 170;                 // -t (Server.py:514)
  bool compress = false;              // -z: gzip uncompressed text before caching
  // >= 0: that GPU does the -z compression, batched across reactors (deflate.h
  // GzipService, one window of gzip_batch_us; the binding installs it with
  // Proxy::set_compressor); the response completes when it returns
  int gzip_gpu = -1;
  int gzip_batch_us = 200;
  bool cache_enabled = true;
  std::string policy = "rfc";         // "rfc" | "reference" (cache every response)
  bool kill_switch = true;            // GET /kill stops the proxy (Server.py:329-331)
  bool kill_loopback_only = true;
  // cache key = Host + URL (ref: URL only). The Python/CLI layer defaults it on for
  // policy rfc (vhosts must not share entries) and off for policy reference.
  bool key_host = false;
  int client_timeout = 30;            // CLIENT_TIMEOUT (Server.py:23)
  int client_max_reqs = 1000;         // CLIENT_MAX_REQS (Server.py:24)
  std::string balance = "random";     // random (ref :123) | roundrobin | leastconn
  int upstream_retry_s = 2;           // a failed upstream is skipped for this long
  // Active health checks (the reference's "todo: check that servers are responsive",
  // Server.py:532): when `health_path` is set, a checker thread sends
  // `GET <health_path>` to every upstream each `health_interval_ms`; `health_fails`
  // consecutive failures (connect error, timeout, or a status >= 400) take it out of
  // rotation, `health_passes` consecutive successes bring it back.
  std::string health_path;
  int health_interval_ms = 1000;
  int health_timeout_ms = 500;
  int health_fails = 2;
  int health_passes = 1;
  bool decode_gzip = false;           // inflate + re-deflate every miss like the reference
  // cap on any inflate the proxy runs (--decode-gzip bodies, identity variants for
  // clients without gzip): a larger body is a decompression bomb and fails (502)
  uint64_t max_inflate_bytes = 64ull << 20;
  // Responses whose body exceeds this are streamed to the client as they arrive and not
  // cached (the reference buffers every object whole, Server.py:408-421).
  uint64_t stream_bytes = 1 << 20;
  // A streamed response stops reading its upstream while this much waits for the
  // client, and resumes below a quarter of it.
  uint64_t stream_high_water = 8 << 20;
  int backlog = 1024;
  int max_fds = 1 << 16;  // fd table reserved at start (capped by RLIMIT_NOFILE)
  std::string server_name = "Shellac/0.2.0";
};

class Reactor;

class Proxy {
 public:
  Proxy(const ProxyConfig& cfg, std::shared_ptr<CacheBackend> backend);
  ~Proxy();
  void start();               // bind + spawn reactor threads
  void wait();                // block until stop()
  void stop();
  bool running() const { return running_; }
  uint16_t port() const { return port_; }
  std::string stats_json();
  const ProxyConfig& config() const { return cfg_; }
  CacheBackend* backend() { return backend_.get(); }
  // -z compression off the reactor threads (before start(); null = zlib inline)
  void set_compressor(std::shared_ptr<Compressor> c) { gzip_ = std::move(c); }

  // upstream health (shared by all reactors): passive (failed connects) and active
  bool upstream_up(int idx, double now) const;
  bool upstream_healthy(int idx) const { return !health_down_[idx].load(); }
  void upstream_failed(int idx, double now);
  int next_rr() { return rr_++; }

 private:
  friend class Reactor;
  ProxyConfig cfg_;
  std::shared_ptr<CacheBackend> backend_;
  std::vector<std::unique_ptr<Reactor>> reactors_;
  std::vector<std::thread> threads_;
  // declared after reactors_: released before them (a GzipService joins its thread
  // then), so a late completion still posts into a live reactor
  std::shared_ptr<Compressor> gzip_;
  std::atomic<bool> running_{false};
  uint16_t port_ = 0;
  std::unique_ptr<std::atomic<double>[]> up_down_until_;
  std::unique_ptr<std::atomic<bool>[]> health_down_;
  std::atomic<uint64_t> health_checks_{0}, health_transitions_{0};
  std::thread health_th_;
  void health_loop();
  std::atomic<int> rr_{0};
  std::mutex wait_mu_;
  double start_time_ = 0;
};

// The stats JSON (Proxy::stats_json) as Prometheus text-format samples (GET
// /_shellac/metrics): nested keys joined with '_' under `shellac_`, array elements as an
// `i` label, string fields as labels of `shellac_info`.
std::string prometheus_text(const std::string& stats_json);

}  // namespace shellac
