// pybind11 bindings for the shellac_amd native core (_shellac_core).
//
// Device-side entry points take raw device pointers and a hipStream_t as Python
// ints (tensor.data_ptr(), torch.cuda.current_stream().cuda_stream) so the core
// does not link against libtorch; the Python layer (shellac_amd/ops) owns
// allocation through PyTorch's caching allocator.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime_api.h>

#include "bind_parts.h"
#include "hbm_cache.h"
#include "host_cache.h"
#include "trace.h"

namespace py = pybind11;
using namespace shellac;

namespace {

template <typename T>
T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::dict counters_dict(const CacheCounters& c) {
  py::dict d;
  d["get_ops"] = c.get_ops;
  d["get_hits"] = c.get_hits;
  d["get_bytes"] = c.get_bytes;
  d["set_ops"] = c.set_ops;
  d["set_bytes"] = c.set_bytes;
  d["set_dropped"] = c.set_dropped;
  d["set_evicted"] = c.set_evicted;
  d["del_ops"] = c.del_ops;
  d["del_hits"] = c.del_hits;
  d["swept"] = c.swept;
  d["get_coalesced"] = c.get_coalesced;
  d["reinserted"] = c.reinserted;
  d["reinsert_bytes"] = c.reinsert_bytes;
  d["reinsert_lost"] = c.reinsert_lost;
  return d;
}

}  // namespace

PYBIND11_MODULE(_shellac_core, m) {
  m.doc() = "shellac_amd native core: HBM/DRAM cache shards, HTTP codec, reactor, protocols";

  m.attr("ENTRY_BYTES") = (int)sizeof(Entry);
  m.attr("BUCKET_BYTES") = (int)kBucketBytes;
  m.attr("ITEM_HEADER_BYTES") = (int)kItemHeaderBytes;
  m.attr("SMALL_GET_MAX") = (int64_t)HbmCache::kSmallGetMax;
  m.attr("LOOKUP_PREFIX_WORDS") = (int64_t)HbmCache::kLookupPrefixWords;
  m.attr("SERVE_KEYS") = (int64_t)HbmCache::kServeKeys;
  m.attr("ITEM_MAGIC") = kItemMagic;
  m.attr("MISS_LOC") = py::int_(kMissLoc);

  m.def("digest", [](py::bytes b) {
    std::string s = b;
    Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    return py::make_tuple(d.lo, d.hi);
  }, "128-bit digest (lo, hi) of a byte string");
  m.def("item_bytes", [](uint32_t vlen) { return item_bytes(vlen); });
  m.def("bucket_pair", [](uint64_t lo, uint64_t hi, uint64_t nbuckets) {
    const Digest d{lo, hi};
    return std::vector<uint64_t>{bucket1(d, nbuckets - 1), bucket2(d, nbuckets - 1)};
  });

  // ---------------- device (HIP) ----------------
  py::class_<HbmCache::StoreGraph>(m, "StoreGraph")
      .def(py::init<>())
      .def_readonly("captures", &HbmCache::StoreGraph::captures)
      .def_readonly("launches", &HbmCache::StoreGraph::launches)
      .def("destroy", [](HbmCache::StoreGraph& g) { HbmCache::destroy_graph(&g); });

  py::class_<HbmCache>(m, "HbmCache")
      .def(py::init([](uint64_t log_bytes, uint64_t nbuckets, uint32_t max_item, int device,
                       int evict, uint64_t reinsert_max, int serve_blocks) {
             ShardConfig c;
             c.log_bytes = log_bytes;
             c.nbuckets = nbuckets;
             c.max_item = max_item;
             c.device = device;
             c.evict = evict;
             c.reinsert_max = reinsert_max;
             c.serve_blocks = serve_blocks;
             return new HbmCache(c);
           }),
           py::arg("log_bytes"), py::arg("nbuckets"), py::arg("max_item"), py::arg("device"),
           py::arg("evict") = (int)kEvictClock, py::arg("reinsert_max") = 0,
           py::arg("serve_blocks") = 8)
      .def_property_readonly("serve_blocks", &HbmCache::serve_blocks)
      .def_property_readonly("reinsert_max", &HbmCache::reinsert_max)
      .def("lookup", [](HbmCache& c, uintptr_t keys, int64_t n, uintptr_t loc, uintptr_t size,
                        uintptr_t off, uint32_t now, uintptr_t s, uint64_t reserve, int slot,
                        uintptr_t first) {
        py::gil_scoped_release nogil;
        c.lookup(P<const Digest>(keys), n, P<uint64_t>(loc), P<uint64_t>(size), P<uint64_t>(off),
                 now, S(s), reserve, slot, P<const uint32_t>(first));
      }, py::arg("keys"), py::arg("n"), py::arg("loc"), py::arg("size"), py::arg("off"),
         py::arg("now"), py::arg("stream"), py::arg("reserve") = 0, py::arg("total_slot") = -1,
         py::arg("first") = 0)
      .def("lookup_coalesced", [](HbmCache& c, uintptr_t keys, int64_t n, uintptr_t table,
                                  int64_t slots, uintptr_t first, uintptr_t loc, uintptr_t size,
                                  uintptr_t off, uint32_t now, uintptr_t s, uint64_t reserve,
                                  int slot, uintptr_t cslot, bool table_clean, uintptr_t prefix,
                                  uintptr_t index_done) {
        py::gil_scoped_release nogil;
        return c.lookup_coalesced(P<const Digest>(keys), n, P<uint32_t>(table), slots,
                                  P<uint32_t>(first), P<uint64_t>(loc), P<uint64_t>(size),
                                  P<uint64_t>(off), now, S(s), reserve, slot, P<uint32_t>(cslot),
                                  table_clean, P<uint64_t>(prefix),
                                  reinterpret_cast<hipEvent_t>(index_done));
      }, py::arg("keys"), py::arg("n"), py::arg("table"), py::arg("slots"), py::arg("first"),
         py::arg("loc"), py::arg("size"), py::arg("off"), py::arg("now"), py::arg("stream"),
         py::arg("reserve") = 0, py::arg("total_slot") = -1, py::arg("cslot") = 0,
         py::arg("table_clean") = false, py::arg("prefix") = 0, py::arg("index_done") = 0)
      .def("small_get", [](HbmCache& c, uintptr_t keys, int64_t n, uintptr_t out,
                           uint64_t out_cap, uintptr_t off, uint32_t now, uintptr_t s,
                           int done_slot) {
        py::gil_scoped_release nogil;
        c.small_get(P<const Digest>(keys), n, P<uint8_t>(out), out_cap, P<uint64_t>(off), now,
                    S(s), done_slot);
      }, py::arg("keys"), py::arg("n"), py::arg("out"), py::arg("out_cap"), py::arg("off"),
         py::arg("now"), py::arg("stream"), py::arg("done_slot") = -1)
      // ordered after `stream` only (the caller's current stream; 0 = the null stream): the
      // resident server runs on no stream, so what the caller queued there to fill `out` /
      // `off` (or SETs queued on that stream) lands before the job is queued; SETs a
      // ShardedCache queued on its own streams need its sync_sets() first
      .def("serve_get", [](HbmCache& c, uintptr_t host_keys, int64_t n, uintptr_t out,
                           uint64_t out_cap, uintptr_t off, uint32_t now, int done_slot,
                           uintptr_t stream) {
        py::gil_scoped_release nogil;
        return c.serve_get_after(S(stream), P<const Digest>(host_keys), n, P<uint8_t>(out),
                                 out_cap, P<uint64_t>(off), now, done_slot);
      }, py::arg("host_keys"), py::arg("n"), py::arg("out"), py::arg("out_cap"), py::arg("off"),
         py::arg("now"), py::arg("done_slot"), py::arg("stream") = 0)
      .def("serve_wait", [](HbmCache& c, int slot, int64_t timeout_ms) {
        py::gil_scoped_release nogil;
        return c.serve_wait(slot, timeout_ms);
      }, py::arg("slot"), py::arg("timeout_ms") = 10000)
      .def("serve_kick", [](HbmCache& c) {
        py::gil_scoped_release nogil;
        c.serve_kick();
      })
      .def("serve_stop", [](HbmCache& c) {
        py::gil_scoped_release nogil;
        c.serve_stop();
      })
      .def("serve_trace", &HbmCache::serve_trace)
      .def_property_readonly("wall_khz", &HbmCache::wall_khz)
      .def_property_readonly("serve_launches", &HbmCache::serve_launches)
      .def_property_readonly("serve_jobs", &HbmCache::serve_jobs)
      .def("host_slot", &HbmCache::host_slot)
      .def("wait_host_slot", [](const HbmCache& c, int i, int64_t timeout_ms) {
        py::gil_scoped_release nogil;
        return c.wait_host_slot(i, timeout_ms);
      }, py::arg("slot"), py::arg("timeout_ms") = 10000)
      .def("gather", [](HbmCache& c, uintptr_t loc, uintptr_t off, int64_t n, uintptr_t out,
                        uintptr_t s, uint64_t out_cap, uintptr_t first, uintptr_t size,
                        uintptr_t out_size, uintptr_t out_off, uintptr_t table, uintptr_t cslot,
                        uintptr_t prefix, int shift) {
        py::gil_scoped_release nogil;
        c.gather(P<const uint64_t>(loc), P<const uint64_t>(off), n, P<uint8_t>(out), S(s),
                 out_cap, P<const uint32_t>(first), P<const uint64_t>(size), P<uint64_t>(out_size),
                 P<uint64_t>(out_off), P<uint32_t>(table), P<const uint32_t>(cslot),
                 P<const uint64_t>(prefix), shift);
      }, py::arg("loc"), py::arg("off"), py::arg("n"), py::arg("out"), py::arg("stream"),
         py::arg("out_cap") = ~0ull, py::arg("first") = 0, py::arg("size") = 0,
         py::arg("out_size") = 0, py::arg("out_off") = 0, py::arg("table") = 0,
         py::arg("cslot") = 0, py::arg("prefix") = 0, py::arg("shift") = 0)
      .def("store_graph", [](HbmCache& c, HbmCache::StoreGraph& g, uintptr_t keys,
                             uintptr_t values, uintptr_t val_off, uintptr_t vlen, uintptr_t flags,
                             uintptr_t expire, int64_t n, uint64_t bytes_bound, uint32_t now,
                             uintptr_t s) {
        py::gil_scoped_release nogil;
        c.store_graph(&g, P<const Digest>(keys), P<const uint8_t>(values),
                      P<const uint64_t>(val_off), P<const uint32_t>(vlen),
                      P<const uint32_t>(flags), P<const uint32_t>(expire), n, bytes_bound, now,
                      S(s));
      })
      .def("store", [](HbmCache& c, uintptr_t keys, uintptr_t values, uintptr_t val_off,
                       uintptr_t vlen, uintptr_t flags, uintptr_t expire, int64_t n,
                       uint64_t bytes_bound, uint32_t now, uintptr_t s, uintptr_t index_after,
                       uintptr_t append_after, uintptr_t append_done, int phase,
                       uintptr_t plan_done, uintptr_t done) {
        py::gil_scoped_release nogil;
        c.store(P<const Digest>(keys), P<const uint8_t>(values), P<const uint64_t>(val_off),
                P<const uint32_t>(vlen), P<const uint32_t>(flags), P<const uint32_t>(expire), n,
                bytes_bound, now, S(s), reinterpret_cast<hipEvent_t>(index_after), true,
                reinterpret_cast<hipEvent_t>(append_after),
                reinterpret_cast<hipEvent_t>(append_done), phase,
                reinterpret_cast<hipEvent_t>(plan_done), reinterpret_cast<hipEvent_t>(done));
      }, py::arg("keys"), py::arg("values"), py::arg("val_off"), py::arg("vlen"),
         py::arg("flags"), py::arg("expire"), py::arg("n"), py::arg("bytes_bound"), py::arg("now"),
         py::arg("stream"), py::arg("index_after") = 0, py::arg("append_after") = 0,
         py::arg("append_done") = 0, py::arg("phase") = 0, py::arg("plan_done") = 0,
         py::arg("done") = 0)
      .def("remove", [](HbmCache& c, uintptr_t keys, int64_t n, uintptr_t found, uint32_t now,
                        uintptr_t s) {
        py::gil_scoped_release nogil;
        c.remove(P<const Digest>(keys), n, P<uint8_t>(found), now, S(s));
      })
      .def("sweep", [](HbmCache& c, uint32_t now, uintptr_t s) {
        uint64_t live = 0, bytes = 0;
        {
          py::gil_scoped_release nogil;
          c.sweep(now, S(s), &live, &bytes);
        }
        return py::make_tuple(live, bytes);
      })
      .def("flush", [](HbmCache& c, uintptr_t s) { c.flush(S(s)); })
      .def("debug_bucket", &HbmCache::debug_bucket)
      .def("debug_hand", &HbmCache::debug_hand)
      .def("debug_set_entry", &HbmCache::debug_set_entry)
      .def("debug_set_hand", &HbmCache::debug_set_hand, py::arg("hand"), py::arg("catch_up") = true)
      .def("retired_bytes", &HbmCache::retired_bytes, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("retired_ever", &HbmCache::retired_ever)
      .def("export_keys", [](HbmCache& c, uintptr_t out, uint64_t cap, uint32_t now, uintptr_t s) {
        py::gil_scoped_release nogil;
        return c.export_keys(P<Digest>(out), cap, now, S(s));
      })
      .def("save", [](HbmCache& c, const std::string& path, std::vector<uint64_t> user, uintptr_t s) {
        user.resize(4);
        py::gil_scoped_release nogil;
        c.save(path, user.data(), S(s));
      })
      .def("load", [](HbmCache& c, const std::string& path, uintptr_t s) {
        std::vector<uint64_t> user(4);
        {
          py::gil_scoped_release nogil;
          c.load(path, user.data(), S(s));
        }
        return user;
      })
      .def("counters", [](HbmCache& c, uintptr_t s) { return counters_dict(c.counters(S(s))); })
      .def("head", [](HbmCache& c, uintptr_t s) { return c.head(S(s)); })
      .def("reserve", &HbmCache::reserve)
      .def("hbm_bytes", &HbmCache::hbm_bytes)
      .def_property_readonly("log_ptr", [](HbmCache& c) { return (uintptr_t)c.log_ptr(); })
      .def_property_readonly("index_ptr", [](HbmCache& c) { return (uintptr_t)c.index_ptr(); })
      .def_property_readonly("head_ptr", [](HbmCache& c) { return (uintptr_t)c.head_ptr(); });

  m.def("scan_tmp_bytes", &device_scan_tmp_bytes);
  m.def("exclusive_scan", [](uintptr_t in, uintptr_t out, int64_t n, uintptr_t tmp,
                             size_t tmp_bytes, uintptr_t s) {
    device_exclusive_scan(P<const uint64_t>(in), P<uint64_t>(out), n, P<void>(tmp), tmp_bytes,
                          S(s));
  });
  m.def("trace_enable", [](bool on) { trace_enable(on); });
  m.def("trace_on", []() { return trace_on(); });
  m.def("trace_push", [](const std::string& name) { trace_push(name.c_str()); });
  m.def("trace_pop", []() { trace_pop(); });
  m.def("trace_mark", [](const std::string& name) { trace_mark(name.c_str()); });
  m.def("segcopy", [](uintptr_t src, uintptr_t src_off, uintptr_t dst_off, int64_t n,
                      uintptr_t dst, uintptr_t s) {
    segcopy(P<const uint8_t>(src), P<const uint64_t>(src_off), P<const uint64_t>(dst_off), n,
            P<uint8_t>(dst), S(s));
  });
  m.def("coalesce_table_slots", &coalesce_table_slots);
  m.def("coalesce_keys", [](uintptr_t keys, int64_t n, uintptr_t table, int64_t slots,
                            uintptr_t first, uintptr_t s, uintptr_t cslot, bool table_clean) {
    coalesce_keys(P<const Digest>(keys), n, P<uint32_t>(table), slots, P<uint32_t>(first), S(s),
                  P<uint32_t>(cslot), table_clean);
  }, py::arg("keys"), py::arg("n"), py::arg("table"), py::arg("slots"), py::arg("first"),
     py::arg("stream"), py::arg("cslot") = 0, py::arg("table_clean") = false);
  m.def("expand_coalesced", [](uintptr_t first, int64_t n, uintptr_t size, uintptr_t off,
                               uintptr_t s) {
    expand_coalesced(P<const uint32_t>(first), n, P<uint64_t>(size), P<uint64_t>(off), S(s));
  });
  m.def("expand_coalesced_out", [](uintptr_t first, int64_t n, uintptr_t size, uintptr_t off,
                                   uintptr_t out_size, uintptr_t out_off, uintptr_t table,
                                   uintptr_t cslot, uintptr_t s) {
    expand_coalesced_out(P<const uint32_t>(first), n, P<const uint64_t>(size),
                         P<const uint64_t>(off), P<uint64_t>(out_size), P<uint64_t>(out_off),
                         P<uint32_t>(table), P<const uint32_t>(cslot), S(s));
  });
  m.def("digest_keys", [](uintptr_t bytes, uintptr_t offs, int64_t n, uintptr_t out,
                          uintptr_t s) {
    digest_keys(P<const uint8_t>(bytes), P<const int64_t>(offs), n, P<Digest>(out), S(s));
  });
  m.def("route_keys", [](uintptr_t keys, int64_t n, uintptr_t pts, uintptr_t owner, int32_t npts,
                         uintptr_t dest, uintptr_t counts, int32_t nranks, uintptr_t s) {
    route_keys(P<const Digest>(keys), n, P<const uint32_t>(pts), P<const int32_t>(owner), npts,
               P<int32_t>(dest), P<int64_t>(counts), nranks, S(s));
  });
  m.def("scatter_by_dest", [](uintptr_t dest, uintptr_t base, int64_t n, int32_t nranks,
                              uintptr_t cursor, uintptr_t perm, uintptr_t s) {
    scatter_by_dest(P<const int32_t>(dest), P<const int64_t>(base), n, nranks, P<int64_t>(cursor),
                    P<int64_t>(perm), S(s));
  });
  m.def("permute_records", [](uintptr_t in, uintptr_t perm, int64_t n, int32_t rec_bytes,
                              uintptr_t out, uintptr_t s) {
    permute_records(P<const void>(in), P<const int64_t>(perm), n, rec_bytes, P<void>(out), S(s));
  });
  m.def("mfma_hello", [](uintptr_t a, uintptr_t b, uintptr_t c, int tiles, uintptr_t s) {
    mfma_hello(P<const uint16_t>(a), P<const uint16_t>(b), P<float>(c), tiles, S(s));
  });
  // Cross-stream ordering with events whose fence scope the caller picks (torch's events
  // use the default: a system-scope release/acquire, i.e. an L2 write-back and invalidate at
  // every record). Two streams of one GPU only need device scope.
  m.attr("EVENT_DISABLE_TIMING") = (unsigned)hipEventDisableTiming;
  m.attr("EVENT_DISABLE_SYSTEM_FENCE") = (unsigned)hipEventDisableSystemFence;
  m.attr("EVENT_RELEASE_TO_DEVICE") = (unsigned)hipEventReleaseToDevice;
  m.def("event_create", [](unsigned flags) {
    hipEvent_t e = nullptr;
    SH_CHECK(hipEventCreateWithFlags(&e, flags) == hipSuccess, "hipEventCreateWithFlags failed");
    return reinterpret_cast<uintptr_t>(e);
  });
  m.def("event_destroy", [](uintptr_t e) { (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e)); });
  m.def("event_elapsed_ms", [](uintptr_t a, uintptr_t b) {
    float ms = 0.f;
    SH_CHECK(hipEventSynchronize(reinterpret_cast<hipEvent_t>(b)) == hipSuccess &&
                 hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(a),
                                     reinterpret_cast<hipEvent_t>(b)) == hipSuccess,
             "hipEventElapsedTime failed");
    return ms;
  });
  m.def("event_query", [](uintptr_t e) {  // true: the work the event marks is complete
    return hipEventQuery(reinterpret_cast<hipEvent_t>(e)) == hipSuccess;
  });
  m.def("event_record", [](uintptr_t e, uintptr_t s) {
    SH_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(e), S(s)) == hipSuccess,
             "hipEventRecord failed");
  });
  m.def("stream_wait_event", [](uintptr_t s, uintptr_t e) {
    SH_CHECK(hipStreamWaitEvent(S(s), reinterpret_cast<hipEvent_t>(e), 0) == hipSuccess,
             "hipStreamWaitEvent failed");
  });
  // raw streams a caller owns (tests: a stream destroyed while a cache still remembers it)
  m.def("stream_create", []() {
    hipStream_t st = nullptr;
    SH_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess,
             "hipStreamCreateWithFlags failed");
    return reinterpret_cast<uintptr_t>(st);
  });
  m.def("stream_destroy", [](uintptr_t s) {
    SH_CHECK(hipStreamSynchronize(S(s)) == hipSuccess && hipStreamDestroy(S(s)) == hipSuccess,
             "hipStreamDestroy failed");
  });
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });

  // ---------------- host (DRAM) ----------------
  py::class_<HostCache>(m, "HostCache")
      .def(py::init<uint64_t, uint64_t, uint32_t, int, uint64_t>(), py::arg("log_bytes"),
           py::arg("nbuckets"), py::arg("max_item"), py::arg("evict") = 1,
           py::arg("reinsert_max") = 0)
      .def_property_readonly("reinsert_max", &HostCache::reinsert_max)
      .def("lookup", [](HostCache& c, uintptr_t keys, int64_t n, uintptr_t loc, uintptr_t size,
                        uintptr_t off, uint32_t now, uint64_t reserve) {
        py::gil_scoped_release nogil;
        c.lookup(P<const Digest>(keys), n, P<uint64_t>(loc), P<uint64_t>(size), P<uint64_t>(off),
                 now, reserve);
      }, py::arg("keys"), py::arg("n"), py::arg("loc"), py::arg("size"), py::arg("off"),
         py::arg("now"), py::arg("reserve") = 0)
      .def("gather", [](HostCache& c, uintptr_t loc, uintptr_t off, int64_t n, uintptr_t out) {
        py::gil_scoped_release nogil;
        c.gather(P<const uint64_t>(loc), P<const uint64_t>(off), n, P<uint8_t>(out));
      })
      .def("store", [](HostCache& c, uintptr_t keys, uintptr_t values, uintptr_t val_off,
                       uintptr_t vlen, uintptr_t flags, uintptr_t expire, int64_t n,
                       uint32_t now, uint64_t bytes_bound) {
        py::gil_scoped_release nogil;
        c.store(P<const Digest>(keys), P<const uint8_t>(values), P<const uint64_t>(val_off),
                P<const uint32_t>(vlen), P<const uint32_t>(flags), P<const uint32_t>(expire), n,
                now, bytes_bound);
      }, py::arg("keys"), py::arg("values"), py::arg("val_off"), py::arg("vlen"), py::arg("flags"),
         py::arg("expire"), py::arg("n"), py::arg("now"), py::arg("bytes_bound") = 0)
      .def("remove", [](HostCache& c, uintptr_t keys, int64_t n, uintptr_t found, uint32_t now) {
        py::gil_scoped_release nogil;
        c.remove(P<const Digest>(keys), n, P<uint8_t>(found), now);
      })
      .def("sweep", [](HostCache& c, uint32_t now) {
        uint64_t live = 0, bytes = 0;
        c.sweep(now, &live, &bytes);
        return py::make_tuple(live, bytes);
      })
      .def("flush", &HostCache::flush)
      .def("debug_bucket", &HostCache::debug_bucket)
      .def("debug_hand", &HostCache::debug_hand)
      .def("debug_set_entry", &HostCache::debug_set_entry)
      .def("debug_set_hand", &HostCache::debug_set_hand, py::arg("hand"), py::arg("catch_up") = true)
      .def("export_keys", [](HostCache& c, uintptr_t out, uint64_t cap, uint32_t now) {
        return c.export_keys(P<Digest>(out), cap, now);
      })
      .def("save", [](HostCache& c, const std::string& path, std::vector<uint64_t> user) {
        user.resize(4);
        c.save(path, user.data());
      })
      .def("load", [](HostCache& c, const std::string& path) {
        std::vector<uint64_t> user(4);
        c.load(path, user.data());
        return user;
      })
      .def("counters", [](HostCache& c) { return counters_dict(c.counters()); })
      .def("head", &HostCache::head)
      .def("get", [](HostCache& c, py::bytes key, uint32_t now) -> py::object {
        std::string k = key;
        Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(k.data()), k.size());
        std::vector<uint8_t> v;
        uint32_t flags = 0;
        if (!c.get_one(d, &v, &flags, now)) return py::none();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def("set", [](HostCache& c, py::bytes key, py::bytes value, uint32_t flags,
                     uint32_t expire, uint32_t now) {
        std::string k = key, v = value;
        Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(k.data()), k.size());
        c.set_one(d, reinterpret_cast<const uint8_t*>(v.data()), (uint32_t)v.size(), flags, expire,
                  now);
      });

  m.def("host_exclusive_scan", [](uintptr_t in, uintptr_t out, int64_t n) {
    host_exclusive_scan(P<const uint64_t>(in), P<uint64_t>(out), n);
  });
  m.def("host_segcopy", [](uintptr_t src, uintptr_t src_off, uintptr_t dst_off, int64_t n,
                           uintptr_t dst) {
    host_segcopy(P<const uint8_t>(src), P<const uint64_t>(src_off), P<const uint64_t>(dst_off), n,
                 P<uint8_t>(dst));
  });
  m.def("host_digest_keys", [](uintptr_t bytes, uintptr_t offs, int64_t n, uintptr_t out) {
    host_digest_keys(P<const uint8_t>(bytes), P<const int64_t>(offs), n, P<Digest>(out));
  });
  m.def("host_route_keys", [](uintptr_t keys, int64_t n, uintptr_t pts, uintptr_t owner,
                              int32_t npts, uintptr_t dest, uintptr_t counts, int32_t nranks) {
    host_route_keys(P<const Digest>(keys), n, P<const uint32_t>(pts), P<const int32_t>(owner),
                    npts, P<int32_t>(dest), P<int64_t>(counts), nranks);
  });
  m.def("host_scatter_by_dest", [](uintptr_t dest, uintptr_t base, int64_t n, int32_t nranks,
                                   uintptr_t cursor, uintptr_t perm) {
    host_scatter_by_dest(P<const int32_t>(dest), P<const int64_t>(base), n, nranks,
                         P<int64_t>(cursor), P<int64_t>(perm));
  });
  m.def("host_permute_records", [](uintptr_t in, uintptr_t perm, int64_t n, int32_t rec_bytes,
                                   uintptr_t out) {
    host_permute_records(P<const void>(in), P<const int64_t>(perm), n, rec_bytes, P<void>(out));
  });

  bind_http(m);
  bind_net(m);
  bind_router(m);
  bind_deflate(m);
}
