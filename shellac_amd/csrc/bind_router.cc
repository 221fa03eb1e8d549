// pybind11 bindings of the fused routed-step ops (router.h). Raw device pointers
// and hipStream_t as Python ints, like bind.cc.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bind_parts.h"
#include "hbm_cache.h"
#include "router.h"

namespace py = pybind11;
using namespace shellac;

namespace {
template <typename T>
T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
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

  py::class_<RoutedStep>(m, "RoutedStep")
      .def(py::init<int, int, int>(), py::arg("world"), py::arg("rank"), py::arg("device"))
      .def("set_ring", [](RoutedStep& r, uintptr_t pts, uintptr_t owner, int32_t npts) {
        r.set_ring(P<const uint32_t>(pts), P<const int32_t>(owner), npts);
      })
      .def("set_hot", [](RoutedStep& r, uintptr_t hot, int64_t nhot, uintptr_t dir) {
        r.set_hot(P<const Digest>(hot), nhot, P<const int64_t>(dir));
      }, py::arg("hot"), py::arg("nhot"), py::arg("dir") = 0)
      .def("plan", [](RoutedStep& r, uintptr_t keys, int64_t n, HbmCache* replica, uint32_t now,
                      uintptr_t skeys, uintptr_t svlen, uintptr_t sflags, uintptr_t sexpire,
                      uintptr_t sval_off, uintptr_t svalues, int64_t ns, bool fanout,
                      uintptr_t table, uintptr_t s, bool coalesce) {
        py::gil_scoped_release nogil;
        r.plan(P<const Digest>(keys), n, replica, now, P<const Digest>(skeys),
               P<const uint32_t>(svlen), P<const uint32_t>(sflags), P<const uint32_t>(sexpire),
               P<const uint64_t>(sval_off), P<const uint8_t>(svalues), ns, fanout,
               P<int64_t>(table), S(s), coalesce);
      }, py::arg("keys"), py::arg("n"), py::arg("replica").none(true), py::arg("now"),
         py::arg("skeys"), py::arg("svlen"), py::arg("sflags"), py::arg("sexpire"),
         py::arg("sval_off"), py::arg("svalues"), py::arg("ns"), py::arg("fanout"),
         py::arg("table"), py::arg("stream"), py::arg("coalesce") = false)
      .def("read_counts", [](RoutedStep& r, uintptr_t rtable, uintptr_t s) {
        py::gil_scoped_release nogil;
        return r.read_counts(P<const int64_t>(rtable), S(s));
      })
      .def("pack", [](RoutedStep& r, uintptr_t send, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.pack(P<uint8_t>(send), S(s));
      })
      .def("owner", [](RoutedStep& r, uintptr_t recv, HbmCache* shard, uint32_t now,
                       uintptr_t sizes_out, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.owner(P<const uint8_t>(recv), shard, now, P<uint64_t>(sizes_out), S(s));
      })
      .def("reply_sizes", [](RoutedStep& r, uintptr_t sizes_in, uintptr_t s) {
        py::gil_scoped_release nogil;
        return r.reply_sizes(P<const uint64_t>(sizes_in), S(s));
      })
      .def("gather_replies", [](RoutedStep& r, HbmCache* shard, uintptr_t reply, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.gather_replies(shard, P<uint8_t>(reply), S(s));
      })
      .def("finish", [](RoutedStep& r, uintptr_t data, uintptr_t recv, int64_t recv_bytes,
                        HbmCache* shard, HbmCache* replica, uint32_t now, uintptr_t out_size,
                        uintptr_t out_off, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.finish(P<uint8_t>(data), P<const uint8_t>(recv), recv_bytes, shard, replica, now,
                 P<uint64_t>(out_size), P<uint64_t>(out_off), S(s));
      }, py::arg("data"), py::arg("recv"), py::arg("recv_bytes"), py::arg("shard"),
         py::arg("replica").none(true), py::arg("now"), py::arg("out_size"), py::arg("out_off"),
         py::arg("stream"))
      .def("join_sets", [](RoutedStep& r, uintptr_t s) { r.join_sets(S(s)); })
      .def("gather_local", [](RoutedStep& r, uintptr_t data, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.gather_local(P<uint8_t>(data), S(s));
      })
      .def("join_local", [](RoutedStep& r, uintptr_t s) { r.join_local(S(s)); })
      .def("set_defer_join", &RoutedStep::set_defer_join)
      .def_property_readonly("sets_pending", &RoutedStep::sets_pending)
      .def_property_readonly("mg", &RoutedStep::mg)
      .def_property_readonly("ms", &RoutedStep::ms)
      .def_property_readonly("n_local", &RoutedStep::n_local);
}
