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
  m.def("plan_sets", [](uintptr_t keys, uintptr_t vlen, uintptr_t flags, uintptr_t expire,
                        uintptr_t val_off, int64_t ns, uintptr_t values_base, uintptr_t pts,
                        uintptr_t owner, int32_t npts, uintptr_t hot, int64_t nhot, int32_t w,
                        bool fanout, uintptr_t dest_ws, uintptr_t owner_ws, uintptr_t ws,
                        uintptr_t srec, uintptr_t sval, uintptr_t spad, uintptr_t counts,
                        uintptr_t s) {
    plan_sets(P<const Digest>(keys), P<const uint32_t>(vlen), P<const uint32_t>(flags),
              P<const uint32_t>(expire), P<const uint64_t>(val_off), ns, values_base,
              P<const uint32_t>(pts), P<const int32_t>(owner), npts, P<const Digest>(hot), nhot,
              w, fanout, P<int32_t>(dest_ws), P<int32_t>(owner_ws), P<uint64_t>(ws),
              P<int64_t>(srec), P<uint64_t>(sval), P<uint64_t>(spad), P<int64_t>(counts), S(s));
  });
  m.def("plan_table", [](uintptr_t cnt_g, uintptr_t cnt_s, uintptr_t vscan, int32_t w,
                         uintptr_t table, uintptr_t s) {
    plan_table(P<const int64_t>(cnt_g), P<const int64_t>(cnt_s), P<const uint64_t>(vscan), w,
               P<int64_t>(table), S(s));
  });
  m.def("send_segments", [](uintptr_t cnt_g, uintptr_t cnt_s, uintptr_t spad, uintptr_t sval,
                            uintptr_t gk_base, uintptr_t srec_base, int32_t w, int64_t ns,
                            uintptr_t seg_len, uintptr_t seg_src, uintptr_t s) {
    send_segments(P<const int64_t>(cnt_g), P<const int64_t>(cnt_s), P<const uint64_t>(spad),
                  P<const uint64_t>(sval), gk_base, srec_base, w, ns, P<uint64_t>(seg_len),
                  P<uint64_t>(seg_src), S(s));
  });
  m.def("recv_segments", [](uintptr_t rtable, uintptr_t recv_base, int32_t w, uintptr_t seg_len,
                            uintptr_t seg_src, uintptr_t s) {
    recv_segments(P<const int64_t>(rtable), recv_base, w, P<uint64_t>(seg_len),
                  P<uint64_t>(seg_src), S(s));
  });
  m.def("recv_sets", [](uintptr_t rrec, int64_t ms, uintptr_t rtable, int32_t w, uintptr_t rpad,
                        uintptr_t rscan, uintptr_t tmp, size_t tmp_bytes, uintptr_t keys,
                        uintptr_t vlen0, uintptr_t vlen1, uintptr_t flags, uintptr_t expire,
                        uintptr_t roff, uintptr_t s) {
    recv_sets(P<const int64_t>(rrec), ms, P<const int64_t>(rtable), w, P<uint64_t>(rpad),
              P<uint64_t>(rscan), P<void>(tmp), tmp_bytes, P<Digest>(keys), P<uint32_t>(vlen0),
              P<uint32_t>(vlen1), P<uint32_t>(flags), P<uint32_t>(expire), P<uint64_t>(roff),
              S(s));
  });
  m.def("reply_bytes", [](uintptr_t lk_off, uintptr_t rtable, uintptr_t gscan, uintptr_t table,
                          int32_t w, uintptr_t bytes, uintptr_t s) {
    reply_bytes(P<const uint64_t>(lk_off), P<const int64_t>(rtable), P<const uint64_t>(gscan),
                P<const int64_t>(table), w, P<int64_t>(bytes), S(s));
  });
  m.def("assemble_response", [](uintptr_t perm, int64_t n, int64_t n_remote, uintptr_t sizes,
                                uintptr_t gscan, uintptr_t rl_size, uintptr_t rl_off,
                                uint64_t local_bytes, uintptr_t size, uintptr_t off, uintptr_t s) {
    assemble_response(P<const int64_t>(perm), n, n_remote, P<const uint64_t>(sizes),
                      P<const uint64_t>(gscan), P<const uint64_t>(rl_size),
                      P<const uint64_t>(rl_off), local_bytes, P<uint64_t>(size), P<uint64_t>(off),
                      S(s));
  });

  py::class_<RoutedStep>(m, "RoutedStep")
      .def(py::init<int, int, int>(), py::arg("world"), py::arg("rank"), py::arg("device"))
      .def("set_ring", [](RoutedStep& r, uintptr_t pts, uintptr_t owner, int32_t npts) {
        r.set_ring(P<const uint32_t>(pts), P<const int32_t>(owner), npts);
      })
      .def("set_hot", [](RoutedStep& r, uintptr_t hot, int64_t nhot) {
        r.set_hot(P<const Digest>(hot), nhot);
      })
      .def("plan", [](RoutedStep& r, uintptr_t keys, int64_t n, HbmCache* replica, uint32_t now,
                      uintptr_t skeys, uintptr_t svlen, uintptr_t sflags, uintptr_t sexpire,
                      uintptr_t sval_off, uintptr_t svalues, int64_t ns, bool fanout,
                      uintptr_t table, uintptr_t s) {
        py::gil_scoped_release nogil;
        r.plan(P<const Digest>(keys), n, replica, now, P<const Digest>(skeys),
               P<const uint32_t>(svlen), P<const uint32_t>(sflags), P<const uint32_t>(sexpire),
               P<const uint64_t>(sval_off), P<const uint8_t>(svalues), ns, fanout,
               P<int64_t>(table), S(s));
      }, py::arg("keys"), py::arg("n"), py::arg("replica").none(true), py::arg("now"),
         py::arg("skeys"), py::arg("svlen"), py::arg("sflags"), py::arg("sexpire"),
         py::arg("sval_off"), py::arg("svalues"), py::arg("ns"), py::arg("fanout"),
         py::arg("table"), py::arg("stream"))
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
      .def_property_readonly("mg", &RoutedStep::mg)
      .def_property_readonly("ms", &RoutedStep::ms)
      .def_property_readonly("n_local", &RoutedStep::n_local);
}
