// pybind11 bindings of the fused routed-step ops (router.h). Raw device pointers
// and hipStream_t as Python ints, like bind.cc.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bind_parts.h"
#include "hbm_cache.h"
#include "host_router.h"
#include "router.h"
#include "step_comm.h"

namespace py = pybind11;
using namespace shellac;

namespace {
template <typename T>
T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// Collectives of RoutedStep::step implemented by a Python object (tests: several ranks
// sharing one GPU, exchanging through gloo): obj.native_all_gather(out, in, words,
// peer_blocks, stream) and obj.native_all_to_all(rbuf, roff, rbytes, sbuf, soff,
// sbytes, stream), raw device pointers and the HIP stream as ints.
class PyStepComm final : public StepComm {
 public:
  PyStepComm(py::object obj, int world, int rank) : obj_(std::move(obj)), w_(world), r_(rank) {}
  ~PyStepComm() override {
    py::gil_scoped_acquire g;
    obj_ = py::object();
  }
  int world() const override { return w_; }
  int rank() const override { return r_; }
  void all_gather(int64_t* out, const int64_t* in, int64_t words, int peer_blocks, hipStream_t s,
                  int) override {
    py::gil_scoped_acquire g;
    obj_.attr("native_all_gather")((uintptr_t)out, (uintptr_t)in, words, peer_blocks,
                                   (uintptr_t)s);
  }
  void all_to_all(uint8_t* rbuf, const std::vector<int64_t>& roff,
                  const std::vector<int64_t>& rbytes, const uint8_t* sbuf,
                  const std::vector<int64_t>& soff, const std::vector<int64_t>& sbytes,
                  hipStream_t s, int) override {
    py::gil_scoped_acquire g;
    obj_.attr("native_all_to_all")((uintptr_t)rbuf, roff, rbytes, (uintptr_t)sbuf, soff, sbytes,
                                   (uintptr_t)s);
  }

 private:
  py::object obj_;
  int w_, r_;
};
}  // namespace

void bind_router(py::module_& m) {
  m.def("group_ws_words", &group_ws_words);
  m.def("group_rows", [](uintptr_t dest, int64_t n, int32_t nb, uintptr_t rows, int32_t row_bytes,
                         uintptr_t out_rows, uintptr_t perm, uintptr_t counts, uintptr_t ws,
                         uintptr_t s) {
    group_rows(P<const int32_t>(dest), n, nb, P<const void>(rows), row_bytes, P<void>(out_rows),
               P<int64_t>(perm), P<int64_t>(counts), P<uint64_t>(ws), S(s));
  });
  m.def("route_gets", [](uintptr_t keys, int64_t n, uintptr_t rsize, uintptr_t pts,
                         uintptr_t owner, int32_t npts, int32_t w, uintptr_t dest, uintptr_t s) {
    route_gets(P<const Digest>(keys), n, P<const uint64_t>(rsize), P<const uint32_t>(pts),
               P<const int32_t>(owner), npts, w, P<int32_t>(dest), S(s));
  });

  py::class_<StepComm, std::shared_ptr<StepComm>>(m, "StepComm")
      .def_property_readonly("world", &StepComm::world)
      .def_property_readonly("rank", &StepComm::rank);
  m.def("rccl_unique_id", [] { return py::bytes(rccl_unique_id()); });
  m.def("make_rccl_comm", [](int world, int rank, int device, const std::vector<py::bytes>& ids) {
    std::vector<std::string> v;
    for (const auto& b : ids) v.emplace_back(b);
    py::gil_scoped_release nogil;  // collective: blocks until every rank has joined
    return std::shared_ptr<StepComm>(make_rccl_comm(world, rank, device, v));
  });
  m.def("make_mirror_comm", [](int world, int rank) {
    return std::shared_ptr<StepComm>(make_mirror_comm(world, rank));
  });
  m.def("make_python_comm", [](py::object obj, int world, int rank) {
    return std::shared_ptr<StepComm>(std::make_shared<PyStepComm>(std::move(obj), world, rank));
  });
  // synchronous staging copies for the Python-callback comm (after the stream drained)
  m.def("stream_copy_to_host", [](uintptr_t src, int64_t n, uintptr_t s) {
    std::string out((size_t)std::max<int64_t>(n, 0), '\0');
    {
      py::gil_scoped_release nogil;
      if (hipStreamSynchronize(S(s)) != hipSuccess ||
          (n > 0 && hipMemcpy(out.data(), P<const void>(src), (size_t)n, hipMemcpyDeviceToHost) !=
                        hipSuccess))
        throw Error("stream_copy_to_host failed");
    }
    return py::bytes(out);
  });
  m.def("stream_copy_from_host", [](uintptr_t dst, py::bytes data, uintptr_t s) {
    std::string v(data);
    py::gil_scoped_release nogil;
    if (hipStreamSynchronize(S(s)) != hipSuccess ||
        (!v.empty() && hipMemcpy(P<void>(dst), v.data(), v.size(), hipMemcpyHostToDevice) !=
                           hipSuccess))
      throw Error("stream_copy_from_host failed");
  });

  // The host request router (host_router.h); host pointers as ints.
  py::class_<HostRouter>(m, "HostRouter")
      .def(py::init<int, int>(), py::arg("nshards"), py::arg("points_per_shard") = 160)
      .def_property_readonly("nshards", &HostRouter::nshards)
      .def_property_readonly("nhot", &HostRouter::nhot)
      .def_property_readonly("cumulative", &HostRouter::cumulative)
      .def_property("lanes", &HostRouter::lanes, &HostRouter::set_lanes)
      .def_property_readonly("publications", &HostRouter::publications)
      .def("hot_rank", [](const HostRouter& r, uint64_t lo, uint64_t hi) {
        return r.hot_rank(Digest{lo, hi});
      })
      .def("owner", [](const HostRouter& r, uint64_t lo, uint64_t hi) {
        return r.owner(Digest{lo, hi});
      })
      .def("set_hot", [](HostRouter& r, uintptr_t hot, int64_t n, uintptr_t rank,
                         std::vector<double> w) {
        SH_CHECK((int)w.size() == r.nshards(), "one spray weight per shard");
        py::gil_scoped_release nogil;
        r.set_hot(P<const Digest>(hot), n, P<const int32_t>(rank), w.data());
      }, py::arg("hot"), py::arg("n"), py::arg("rank"), py::arg("weights"))
      .def("route_gets", [](const HostRouter& r, uintptr_t keys, int64_t n, uint64_t seq0,
                            uintptr_t dest, uintptr_t counts, int threads) {
        py::gil_scoped_release nogil;
        r.route_gets(P<const Digest>(keys), n, seq0, P<int32_t>(dest), P<int64_t>(counts),
                     threads);
      }, py::arg("keys"), py::arg("n"), py::arg("seq0"), py::arg("dest"), py::arg("counts"),
         py::arg("threads") = 1)
      .def("route_sets", [](const HostRouter& r, uintptr_t keys, int64_t n, uintptr_t dest,
                            uintptr_t counts, int threads) {
        py::gil_scoped_release nogil;
        r.route_sets(P<const Digest>(keys), n, P<int32_t>(dest), P<int64_t>(counts), threads);
      }, py::arg("keys"), py::arg("n"), py::arg("dest"), py::arg("counts"),
         py::arg("threads") = 1);

  // plan_hot (host_router.h) over (lo, hi, count) rows with the router's owners
  m.def("plan_hot", [](const HostRouter& router, std::vector<std::tuple<uint64_t, uint64_t, uint64_t>> rows,
                       int k, uint64_t eligible, double spray_above, uint64_t min_count,
                       std::vector<std::pair<uint64_t, uint64_t>> sticky, double sticky_factor) {
    std::vector<std::pair<Digest, uint64_t>> c;
    c.reserve(rows.size());
    for (auto& t : rows) c.emplace_back(Digest{std::get<0>(t), std::get<1>(t)}, std::get<2>(t));
    std::vector<Digest> st;
    for (auto& x : sticky) st.push_back(Digest{x.first, x.second});
    const std::function<bool(const Digest&)> is_sticky = [&](const Digest& d) {
      for (const Digest& x : st)
        if (x.lo == d.lo && x.hi == d.hi) return true;
      return false;
    };
    const HotPlan p = plan_hot(c, k, router.nshards(), eligible,
                               [&](const Digest& d) { return router.owner(d); }, spray_above,
                               min_count, st.empty() ? nullptr : &is_sticky, sticky_factor);
    py::list hot;
    for (const Digest& d : p.hot) hot.append(py::make_tuple(d.lo, d.hi));
    py::dict out;
    out["hot"] = hot;
    out["rank"] = p.rank;
    out["weights"] = p.weights;
    out["hot_share"] = p.hot_share;
    out["planned"] = p.planned;
    return out;
  }, py::arg("router"), py::arg("rows"), py::arg("k"), py::arg("eligible"),
     py::arg("spray_above"), py::arg("min_count") = 2,
     py::arg("sticky") = std::vector<std::pair<uint64_t, uint64_t>>{},
     py::arg("sticky_factor") = 1.0);

  m.def("step_streams", [](int device) {
    const StepStreams& ss = step_streams(device);
    return std::vector<uintptr_t>{(uintptr_t)ss.plan, (uintptr_t)ss.set, (uintptr_t)ss.asm_};
  });

  py::class_<RoutedStep>(m, "RoutedStep")
      .def(py::init<int, int, int>(), py::arg("world"), py::arg("rank"), py::arg("device"))
      .def("set_ring", [](RoutedStep& r, uintptr_t pts, uintptr_t owner, int32_t npts) {
        r.set_ring(P<const uint32_t>(pts), P<const int32_t>(owner), npts);
      })
      .def("set_probe_keys", [](RoutedStep& r, uintptr_t pkeys, uintptr_t spkeys) {
        r.set_probe_keys(P<const Digest>(pkeys), P<const Digest>(spkeys));
      })
      .def("set_hot", [](RoutedStep& r, uintptr_t hot, int64_t nhot, uintptr_t dir, bool changed) {
        py::gil_scoped_release nogil;
        r.set_hot(P<const Digest>(hot), nhot, P<const int64_t>(dir), changed);
      }, py::arg("hot"), py::arg("nhot"), py::arg("dir") = 0, py::arg("changed") = false)
      .def_property_readonly("row_words", &RoutedStep::row_words)
      .def("caps", &RoutedStep::caps)
      .def("prepare", &RoutedStep::prepare)
      .def("set_caps", &RoutedStep::set_caps)
      .def("set_set_cap_override", &RoutedStep::set_set_cap_override)
      .def("carry_stats", [](RoutedStep& r) {
        py::gil_scoped_release nogil;
        return r.carry_stats();
      })
      .def("take_stats", &RoutedStep::take_stats)
      .def("harvest_all", [](RoutedStep& r) {
        py::gil_scoped_release nogil;
        r.harvest_all();
      })
      .def_property("single_comm", &RoutedStep::single_comm, &RoutedStep::set_single_comm)
      .def("reset_caps", &RoutedStep::reset_caps)
      .def("set_cap_override", &RoutedStep::set_cap_override)
      .def("plan", [](RoutedStep& r, uintptr_t keys, int64_t n, HbmCache* replica, uint32_t now,
                      uintptr_t skeys, uintptr_t svlen, uintptr_t sflags, uintptr_t sexpire,
                      uintptr_t sval_off, uintptr_t svalues, int64_t ns, bool fanout,
                      uintptr_t G, uintptr_t row, uintptr_t s, bool coalesce) {
        py::gil_scoped_release nogil;
        r.plan(P<const Digest>(keys), n, replica, now, P<const Digest>(skeys),
               P<const uint32_t>(svlen), P<const uint32_t>(sflags), P<const uint32_t>(sexpire),
               P<const uint64_t>(sval_off), P<const uint8_t>(svalues), ns, fanout,
               P<uint8_t>(G), P<int64_t>(row), S(s), coalesce);
      }, py::arg("keys"), py::arg("n"), py::arg("replica").none(true), py::arg("now"),
         py::arg("skeys"), py::arg("svlen"), py::arg("sflags"), py::arg("sexpire"),
         py::arg("sval_off"), py::arg("svalues"), py::arg("ns"), py::arg("fanout"),
         py::arg("G"), py::arg("row"), py::arg("stream"), py::arg("coalesce") = false)
      .def("publish", [](RoutedStep& r, uintptr_t mat, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.publish(P<const int64_t>(mat), S(s));
      })
      .def("calibrate_local", [](RoutedStep& r) {
        py::gil_scoped_release nogil;
        r.calibrate_local();
      })
      .def("owner_probe", [](RoutedStep& r, uintptr_t G, HbmCache* shard, uint32_t now,
                             uintptr_t s) {
        py::gil_scoped_release nogil;
        r.owner_probe(P<const uint8_t>(G), shard, now, S(s));
      })
      .def("owner_demand", [](RoutedStep& r, uintptr_t out, uintptr_t s) {
        r.owner_demand(P<int64_t>(out), S(s));
      })
      .def("calibrate_reply", [](RoutedStep& r, uintptr_t dmat) {
        py::gil_scoped_release nogil;
        r.calibrate_reply(P<const int64_t>(dmat));
      })
      .def("owner_reply", [](RoutedStep& r, HbmCache* shard, uintptr_t R, uintptr_t data,
                             uintptr_t s) {
        py::gil_scoped_release nogil;
        r.owner_reply(shard, P<uint8_t>(R), P<uint8_t>(data), S(s));
      })
      .def("gather_local", [](RoutedStep& r, uintptr_t data, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.gather_local(P<uint8_t>(data), S(s));
      })
      .def("set_splits", [](RoutedStep& r) {
        py::gil_scoped_release nogil;
        return r.set_splits();
      })
      .def("pack_sets", [](RoutedStep& r, uintptr_t Sb, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.pack_sets(P<uint8_t>(Sb), S(s));
      })
      .def("store_sets", [](RoutedStep& r, uintptr_t Rs, HbmCache* shard, HbmCache* replica,
                            uint32_t now, uintptr_t s, uintptr_t sset) {
        py::gil_scoped_release nogil;
        r.store_sets(P<const uint8_t>(Rs), shard, replica, now, S(s), S(sset));
      }, py::arg("Rs"), py::arg("shard"), py::arg("replica").none(true), py::arg("now"),
         py::arg("stream"), py::arg("set_stream"))
      .def("assemble", [](RoutedStep& r, uintptr_t data, uintptr_t out_size, uintptr_t out_off,
                          uintptr_t s) {
        py::gil_scoped_release nogil;
        r.assemble(P<const uint8_t>(data), P<uint64_t>(out_size), P<uint64_t>(out_off), S(s));
      })
      .def("join_sets", [](RoutedStep& r, uintptr_t s) { r.join_sets(S(s)); })
      .def("set_comm", &RoutedStep::set_comm)
      .def_property_readonly("has_comm", &RoutedStep::has_comm)
      .def_property_readonly("early_sets", &RoutedStep::early_sets)
      .def("step", [](RoutedStep& r, uintptr_t keys, int64_t n, HbmCache* replica, uint32_t now,
                      uintptr_t skeys, uintptr_t svlen, uintptr_t sflags, uintptr_t sexpire,
                      uintptr_t sval_off, uintptr_t svalues, int64_t ns, bool fanout,
                      bool coalesce, HbmCache* shard, uintptr_t data, uintptr_t out_size,
                      uintptr_t out_off, uintptr_t s, uintptr_t sset, uintptr_t sasm,
                      uintptr_t ready, int64_t svalues_bytes) {
        py::gil_scoped_release nogil;
        return r.step(P<const Digest>(keys), n, replica, now, P<const Digest>(skeys),
                      P<const uint32_t>(svlen), P<const uint32_t>(sflags),
                      P<const uint32_t>(sexpire), P<const uint64_t>(sval_off),
                      P<const uint8_t>(svalues), ns, fanout, coalesce, shard, P<uint8_t>(data),
                      P<uint64_t>(out_size), P<uint64_t>(out_off), S(s), S(sset), S(sasm),
                      reinterpret_cast<hipEvent_t>(ready), svalues_bytes);
      }, py::arg("keys"), py::arg("n"), py::arg("replica").none(true), py::arg("now"),
         py::arg("skeys"), py::arg("svlen"), py::arg("sflags"), py::arg("sexpire"),
         py::arg("sval_off"), py::arg("svalues"), py::arg("ns"), py::arg("fanout"),
         py::arg("coalesce"), py::arg("shard"), py::arg("data"), py::arg("out_size"),
         py::arg("out_off"), py::arg("stream"), py::arg("set_stream"), py::arg("asm_stream"),
         py::arg("inputs_ready") = 0, py::arg("svalues_bytes") = 0)
      .def_property_readonly("sets_pending", &RoutedStep::sets_pending);
}
