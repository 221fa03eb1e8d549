// pybind11 registration: ketama ring, cache backends, proxy server, memcached server.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <condition_variable>
#include <cstdlib>

#include "backend.h"
#include "bind_parts.h"
#include "ketama.h"
#include "loadgen.h"
#include <pybind11/numpy.h>
#include "mcserver.h"
#include "origin.h"
#include "deflate.h"
#include "proxy.h"

namespace py = pybind11;
using namespace shellac;

namespace {

// Executes posted completions inline on whatever thread completes them.
class InlineExecutor : public Executor {
 public:
  void post(std::function<void()> fn) override { fn(); }
};
InlineExecutor g_inline;

struct BackendHandle {
  std::shared_ptr<CacheBackend> be;
};

py::object blocking_get(CacheBackend* be, const std::string& key, const Digest* forced = nullptr) {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false, hit = false;
  CacheValue val;
  {
    py::gil_scoped_release nogil;
    const Digest d = forced ? *forced
                            : digest_bytes(reinterpret_cast<const uint8_t*>(key.data()), key.size());
    be->get(key, d, &g_inline, [&](bool h, CacheValue v) {
      std::lock_guard<std::mutex> lk(mu);
      hit = h;
      val = std::move(v);
      done = true;
      cv.notify_all();
    });
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
  }
  if (!hit || !val.data) return py::none();
  return py::make_tuple(py::bytes(val.data->data(), val.data->size()), val.flags);
}

bool blocking_del(CacheBackend* be, const std::string& key) {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false, found = false;
  py::gil_scoped_release nogil;
  const Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(key.data()), key.size());
  be->del(key, d, &g_inline, [&](bool f) {
    std::lock_guard<std::mutex> lk(mu);
    found = f;
    done = true;
    cv.notify_all();
  });
  std::unique_lock<std::mutex> lk(mu);
  cv.wait(lk, [&] { return done; });
  return found;
}

}  // namespace

void bind_net(py::module_& m) {
  m.def("run_load", [](const std::string& host, uint16_t port, std::vector<std::string> paths,
                       int64_t requests, int concurrency, int depth, int threads, bool keepalive,
                       std::vector<std::string> headers, const std::string& method,
                       double timeout_s, int64_t objects, double zipf_s,
                       const std::string& path_prefix, const std::string& path_suffix,
                       uint64_t seed, std::vector<int> cpus, int spin_us) {
    LoadConfig c;
    c.spin_us = spin_us;
    c.cpus = std::move(cpus);
    c.objects = objects;
    c.zipf_s = zipf_s;
    c.path_prefix = path_prefix;
    c.path_suffix = path_suffix;
    c.seed = seed;
    c.host = host;
    c.port = port;
    c.paths = std::move(paths);
    c.requests = requests;
    c.concurrency = concurrency;
    c.depth = depth;
    c.threads = threads;
    c.keepalive = keepalive;
    c.headers = std::move(headers);
    c.method = method;
    c.timeout_s = timeout_s;
    LoadResult r;
    {
      py::gil_scoped_release nogil;
      r = run_load(c);
    }
    const size_t n = r.samples.size();
    py::array_t<double> start(n), lat(n);
    py::array_t<int32_t> status(n);
    auto ps = start.mutable_unchecked<1>();
    auto pl = lat.mutable_unchecked<1>();
    auto pst = status.mutable_unchecked<1>();
    for (size_t i = 0; i < n; ++i) {
      ps(i) = r.samples[i].start;
      pl(i) = r.samples[i].latency;
      pst(i) = r.samples[i].status;
    }
    py::dict d;
    d["completed"] = r.completed;
    d["elapsed_s"] = r.elapsed_s;
    d["connected_s"] = r.connected_s;
    d["connect_lat"] = r.connect_lat;
    d["connect_call"] = r.connect_call;
    d["open_loop_s"] = r.open_loop_s;
    d["bytes"] = r.bytes;
    d["errors"] = r.errors;
    d["non2xx"] = r.non2xx;
    d["reconnects"] = r.reconnects;
    d["start"] = start;
    d["latency"] = lat;
    d["status"] = status;
    return d;
  }, py::arg("host"), py::arg("port"), py::arg("paths"), py::arg("requests"),
     py::arg("concurrency"), py::arg("depth") = 1, py::arg("threads") = 1,
     py::arg("keepalive") = true, py::arg("headers") = std::vector<std::string>{},
     py::arg("method") = "GET", py::arg("timeout_s") = 60.0, py::arg("objects") = 0,
     py::arg("zipf_s") = 0.99, py::arg("path_prefix") = "/obj/",
     py::arg("path_suffix") = ".html", py::arg("seed") = 1,
     py::arg("cpus") = std::vector<int>{}, py::arg("spin_us") = 0);

  m.def("md5_hex", [](py::bytes b) { return md5_hex(std::string(b)); });

  py::class_<KetamaRing>(m, "KetamaRing")
      .def(py::init([](const std::vector<std::string>& names, uint32_t ppw) {
             std::vector<KetamaRing::Node> nodes;
             for (const auto& n : names) nodes.push_back(KetamaRing::Node{n, 1, true});
             return new KetamaRing(nodes, ppw);
           }),
           py::arg("names"), py::arg("points_per_weight") = 160)
      .def("pick", [](KetamaRing& r, py::bytes k) { return r.pick(std::string(k)); })
      .def("set_alive", &KetamaRing::set_alive)
      .def("points", &KetamaRing::points)
      .def_static("key_hash", [](py::bytes k) {
        std::string s = k;
        return KetamaRing::key_hash(s.data(), s.size());
      });

  py::class_<BackendHandle>(m, "CacheBackend")
      .def_property_readonly("name", [](BackendHandle& h) { return h.be->name(); })
      .def("get", [](BackendHandle& h, py::bytes key) { return blocking_get(h.be.get(), key); })
      .def("get_with_digest", [](BackendHandle& h, py::bytes key, py::bytes digest_of) {
        // GET `key` but look it up under the digest of `digest_of`: a forged collision
        const std::string o = digest_of;
        const Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(o.data()), o.size());
        return blocking_get(h.be.get(), key, &d);
      })
      .def("set", [](BackendHandle& h, py::bytes key, py::bytes value, uint32_t flags,
                     uint32_t ttl) {
        std::string k = key;
        const Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(k.data()), k.size());
        h.be->set(k, d, std::make_shared<const std::string>(std::string(value)), flags, ttl);
      }, py::arg("key"), py::arg("value"), py::arg("flags") = 0, py::arg("ttl") = 0)
      .def("delete", [](BackendHandle& h, py::bytes key) { return blocking_del(h.be.get(), key); })
      .def("get_many", [](BackendHandle& h, std::vector<std::string> keys) {
        // every GET issued at once (one batch stream, as concurrent clients would), then
        // waited for: [(value, flags) or None]
        const size_t n = keys.size();
        std::vector<CacheValue> vals(n);
        std::vector<uint8_t> hit(n, 0);
        std::mutex mu;
        std::condition_variable cv;
        size_t left = n;
        {
          py::gil_scoped_release nogil;
          for (size_t i = 0; i < n; ++i) {
            const Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(keys[i].data()),
                                          keys[i].size());
            h.be->get(keys[i], d, &g_inline, [&, i](bool ht, CacheValue v) {
              std::lock_guard<std::mutex> lk(mu);
              hit[i] = ht;
              vals[i] = std::move(v);
              if (--left == 0) cv.notify_all();
            });
          }
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return left == 0; });
        }
        py::list out;
        for (size_t i = 0; i < n; ++i) {
          if (hit[i] && vals[i].data)
            out.append(py::make_tuple(py::bytes(vals[i].data->data(), vals[i].data->size()),
                                      vals[i].flags));
          else
            out.append(py::none());
        }
        return out;
      })
      .def("flush", [](BackendHandle& h) { h.be->flush(); })
      .def("stats", [](BackendHandle& h) {
        StatList st;
        h.be->stats(&st);
        py::dict d;
        for (auto& kv : st) d[py::str(kv.first)] = kv.second;
        return d;
      });

  m.def("fault_backend", [](BackendHandle inner, const std::string& spec, uint64_t seed) {
    auto fb = std::make_shared<FaultBackend>(inner.be, parse_fault_spec(spec), seed);
    return BackendHandle{fb};
  }, py::arg("inner"), py::arg("spec") = "", py::arg("seed") = 1);
  m.def("set_fault", [](BackendHandle& h, const std::string& spec) {
    auto* fb = dynamic_cast<FaultBackend*>(h.be.get());
    if (!fb) throw Error("not a fault-injection backend");
    fb->set_spec(parse_fault_spec(spec));
  });
  m.def("dram_backend", [](uint64_t bytes, uint32_t max_item, int stripes) {
    return BackendHandle{std::make_shared<DramBackend>(bytes, max_item, stripes)};
  }, py::arg("bytes"), py::arg("max_item") = 1u << 20, py::arg("stripes") = 16);
  m.def("hbm_backend", [](std::vector<int> devices, uint64_t log_bytes_per_gpu,
                          uint64_t nbuckets_per_gpu, uint32_t max_item, int batch_us,
                          int max_batch, int sweep_interval_s, int spin_us,
                          bool presence_filter, int depth, const std::string& evict,
                          int retry_s, int batch_timeout_ms, bool flush_on_restore,
                          bool warm_restore, const std::string& peer_copy, bool edge_server,
                          std::vector<int> batcher_cpus, int serve_backlog, bool direct,
                          int direct_backlog, int serve_blocks, int hot_objects,
                          int hot_refresh_ms, int hot_sample, uint64_t hot_min_samples,
                          uint64_t hot_fill_budget, double hot_spray_above) {
    HbmBackendConfig c;
    c.devices = std::move(devices);
    c.log_bytes_per_gpu = log_bytes_per_gpu;
    c.nbuckets_per_gpu = nbuckets_per_gpu;
    c.max_item = max_item;
    c.batch_us = batch_us;
    c.max_batch = max_batch;
    c.sweep_interval_s = sweep_interval_s;
    c.spin_us = spin_us;
    c.presence_filter = presence_filter;
    c.depth = depth;
    SH_CHECK(evict == "clock" || evict == "fifo", "evict must be clock or fifo");
    c.evict = evict == "clock" ? 1 : 0;
    c.retry_s = retry_s;
    c.batch_timeout_ms = batch_timeout_ms;
    c.flush_on_restore = flush_on_restore;
    c.warm_restore = warm_restore;
    SH_CHECK(peer_copy == "auto" || peer_copy == "staged", "peer_copy must be auto or staged");
    c.peer_copy = peer_copy;
    c.edge_server = edge_server;
    c.batcher_cpus = std::move(batcher_cpus);
    SH_CHECK(serve_backlog >= 1, "serve_backlog must be >= 1");
    c.serve_backlog = serve_backlog;
    SH_CHECK(direct_backlog >= 1, "direct_backlog must be >= 1");
    c.direct = direct;
    c.direct_backlog = direct_backlog;
    SH_CHECK(serve_blocks >= 1 && serve_blocks <= 8, "serve_blocks must be in 1..8");
    c.serve_blocks = serve_blocks;
    SH_CHECK(hot_objects >= 0 && hot_refresh_ms >= 0, "hot_objects / hot_refresh_ms must be >= 0");
    c.hot_objects = hot_objects;
    c.hot_refresh_ms = hot_refresh_ms;
    c.hot_sample = hot_sample;
    c.hot_min_samples = hot_min_samples;
    c.hot_fill_budget = hot_fill_budget;
    c.hot_spray_above = hot_spray_above;
    py::gil_scoped_release nogil;
    return BackendHandle{std::make_shared<HbmBackend>(c)};
  }, py::arg("devices"), py::arg("log_bytes_per_gpu"), py::arg("nbuckets_per_gpu"),
     py::arg("max_item") = 1u << 20, py::arg("batch_us") = 0, py::arg("max_batch") = 65536,
     py::arg("sweep_interval_s") = 10, py::arg("spin_us") = 50,
     py::arg("presence_filter") = true, py::arg("depth") = 3, py::arg("evict") = "clock",
     py::arg("retry_s") = 2, py::arg("batch_timeout_ms") = 2000,
     py::arg("flush_on_restore") = true, py::arg("warm_restore") = true,
     py::arg("peer_copy") = "auto", py::arg("edge_server") = true,
     py::arg("batcher_cpus") = std::vector<int>{}, py::arg("serve_backlog") = 2,
     py::arg("direct") = true, py::arg("direct_backlog") = 4, py::arg("serve_blocks") = 8,
     py::arg("hot_objects") = 1024, py::arg("hot_refresh_ms") = 1000, py::arg("hot_sample") = 8,
     py::arg("hot_min_samples") = 512, py::arg("hot_fill_budget") = 256ull << 20,
     py::arg("hot_spray_above") = 0.0);
  m.def("hot_refresh", [](BackendHandle& h) {
    StatList st;
    {
      py::gil_scoped_release nogil;
      st = h.be->hot_refresh();
    }
    py::dict d;
    for (auto& kv : st) d[py::str(kv.first)] = kv.second;
    return d;
  }, py::arg("backend"));
  m.def("inject_shard_down", [](BackendHandle& h, int shard, bool down) {
    return h.be->inject_shard_down(shard, down);
  }, py::arg("backend"), py::arg("shard"), py::arg("down") = true);
  m.def("tiered_backend", [](BackendHandle& l1, BackendHandle& l2, uint32_t promote_ttl,
                             uint64_t promote_max) {
    return BackendHandle{std::make_shared<TieredBackend>(l1.be, l2.be, promote_ttl, promote_max)};
  }, py::arg("l1"), py::arg("l2"), py::arg("promote_ttl") = 60,
     py::arg("promote_max") = 32u << 10);
  m.def("memcached_backend", [](const std::string& servers, int retry_s, int op_timeout_ms) {
    MemcachedConfig c;
    c.servers = resolve_list(servers, 11211);
    c.retry_timeout_s = retry_s;
    c.op_timeout_ms = op_timeout_ms;
    return BackendHandle{std::make_shared<MemcachedBackend>(c)};
  }, py::arg("servers"), py::arg("retry_s") = 2, py::arg("op_timeout_ms") = 1000);

  py::class_<Proxy>(m, "Proxy")
      .def(py::init([](const std::string& upstreams, py::object backend, uint16_t port,
                       const std::string& bind, int threads, uint32_t ttl, bool compress,
                       const std::string& policy, bool kill_switch, bool key_host,
                       int client_timeout, int client_max_reqs, const std::string& balance,
                       bool decode_gzip, int upstream_retry_s, uint64_t stream_bytes,
                       uint64_t stream_high_water, const std::string& health_path,
                       int health_interval_ms, int health_timeout_ms, int health_fails,
                       std::vector<int> cpus, int spin_us, int gzip_gpu, int gzip_batch_us,
                       uint64_t max_inflate_bytes, int gzip_workers) {
             ProxyConfig c;
             c.spin_us = spin_us;
             c.gzip_gpu = gzip_gpu;
             c.gzip_batch_us = gzip_batch_us;
             c.upstreams = resolve_list(upstreams, 80);
             c.port = port;
             c.bind = bind;
             c.threads = threads;
             c.ttl = ttl;
             c.compress = compress;
             c.policy = policy;
             c.kill_switch = kill_switch;
             c.key_host = key_host;
             c.client_timeout = client_timeout;
             c.client_max_reqs = client_max_reqs;
             c.balance = balance;
             c.decode_gzip = decode_gzip;
             c.max_inflate_bytes = max_inflate_bytes;
             c.upstream_retry_s = upstream_retry_s;
             c.stream_bytes = stream_bytes;
             c.stream_high_water = stream_high_water;
             c.health_path = health_path;
             c.health_interval_ms = health_interval_ms;
             c.health_timeout_ms = health_timeout_ms;
             c.health_fails = health_fails;
             c.cpus = std::move(cpus);
             std::shared_ptr<CacheBackend> be;
             if (!backend.is_none()) be = backend.cast<BackendHandle&>().be;
             c.cache_enabled = be != nullptr;
             auto* px = new Proxy(c, be);
             if (c.compress && c.gzip_gpu >= 0) {
               // service workers (each its own engine and stream), default 2: with 4 the
               // bodies split into twice as many smaller batches and the per-batch host
               // work grew (49.8K vs 70.6K misses/s, profiles/archive/r2_http_compress_workers_ab.log)
               px->set_compressor(std::make_shared<GzipService>(c.gzip_gpu, c.gzip_batch_us,
                                                                4096, std::max(1, gzip_workers)));
             }
             return px;
           }),
           py::arg("upstreams"), py::arg("backend") = py::none(), py::arg("port") = 8080,
           py::arg("bind") = "0.0.0.0", py::arg("threads") = 1, py::arg("ttl") = 170,
           py::arg("compress") = false, py::arg("policy") = "rfc", py::arg("kill_switch") = true,
           py::arg("key_host") = false, py::arg("client_timeout") = 30,
           py::arg("client_max_reqs") = 1000, py::arg("balance") = "random",
           py::arg("decode_gzip") = false, py::arg("upstream_retry_s") = 2,
           py::arg("stream_bytes") = 1 << 20, py::arg("stream_high_water") = 8 << 20,
           py::arg("health_path") = "", py::arg("health_interval_ms") = 1000,
           py::arg("health_timeout_ms") = 500, py::arg("health_fails") = 2,
           py::arg("cpus") = std::vector<int>{}, py::arg("spin_us") = 0,
           py::arg("gzip_gpu") = -1, py::arg("gzip_batch_us") = 200,
           py::arg("max_inflate_bytes") = 64ull << 20, py::arg("gzip_workers") = 2)
      .def("start", &Proxy::start)
      .def("wait", &Proxy::wait, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Proxy::stop)
      .def_property_readonly("port", &Proxy::port)
      .def_property_readonly("running", &Proxy::running)
      .def("stats_json", &Proxy::stats_json);

  py::class_<CacheServer>(m, "CacheServer")
      .def(py::init([](BackendHandle& be, uint16_t port, const std::string& bind, int threads) {
             CacheServerConfig c;
             c.port = port;
             c.bind = bind;
             c.threads = threads;
             return new CacheServer(c, be.be);
           }),
           py::arg("backend"), py::arg("port") = 11211, py::arg("bind") = "0.0.0.0",
           py::arg("threads") = 1)
      .def("start", &CacheServer::start)
      .def("stop", &CacheServer::stop)
      .def("wait", &CacheServer::wait, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &CacheServer::port)
      .def_property_readonly("running", &CacheServer::running)
      .def("ops", &CacheServer::ops);

  py::class_<NativeOrigin>(m, "NativeOrigin")
      .def(py::init([](uint16_t port, int threads, int body_bytes, int gzip_level,
                       const std::string& host, bool random_body, bool text_body) {
             OriginConfig c;
             c.text_body = text_body;
             c.host = host;
             c.port = port;
             c.threads = threads;
             c.body_bytes = body_bytes;
             c.gzip_level = gzip_level;
             c.random_body = random_body;
             return new NativeOrigin(c);
           }),
           py::arg("port") = 0, py::arg("threads") = 2, py::arg("body_bytes") = 1024,
           py::arg("gzip_level") = 1, py::arg("host") = "127.0.0.1",
           py::arg("random_body") = false, py::arg("text_body") = false)
      .def("start", &NativeOrigin::start)
      .def("stop", &NativeOrigin::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &NativeOrigin::port)
      .def_property_readonly("requests", &NativeOrigin::requests);
}
