// pybind11 bindings of the GPU batch gzip engine (deflate.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <string_view>

#include "bind_parts.h"
#include "common.h"
#include "deflate.h"
#include "huffman.h"

namespace py = pybind11;
using namespace shellac;

namespace {
// Views of the callers' bytes objects (immutable, and the argument list keeps them alive
// for the call, so the GIL can be released without copying them).
std::vector<std::string_view> views(const py::list& in) {
  std::vector<std::string_view> v;
  v.reserve(in.size());
  for (const auto& o : in) {
    if (!PyBytes_Check(o.ptr())) throw py::type_error("gzip inputs must be bytes");
    v.emplace_back(PyBytes_AS_STRING(o.ptr()), (size_t)PyBytes_GET_SIZE(o.ptr()));
  }
  return v;
}

py::list to_list(const std::vector<std::string>& out) {
  py::list l(out.size());
  for (size_t i = 0; i < out.size(); ++i) l[i] = py::bytes(out[i]);
  return l;
}
}  // namespace

void bind_deflate(py::module_& m) {
  m.attr("DEFLATE_BLOCK") = kDeflateBlock;
  // host-side DEFLATE planning, exposed for CPU tests (huffman.h)
  m.def("huffman_lengths", [](const std::vector<uint32_t>& freq, int max_len) {
    std::vector<uint8_t> len(freq.size());
    huffman_lengths(freq.data(), (int)freq.size(), max_len, len.data());
    return std::vector<int>(len.begin(), len.end());
  });
  m.def("plan_block", [](const std::vector<uint32_t>& hist, uint32_t n, bool fin) {
    SH_CHECK(hist.size() == (size_t)kHistSyms, "histogram of 316 symbols expected");
    BlockPlan p;
    plan_block(hist.data(), n, fin, &p);
    return py::make_tuple(p.mode, py::bytes(std::string(p.header.begin(), p.header.end())),
                          p.header_bits, std::vector<uint32_t>(p.codes, p.codes + kHistSyms),
                          p.total_bytes);
  });
  m.def("deflate_tokens_cpu", [](const std::vector<uint32_t>& tokens, const py::bytes& data,
                                 bool fin) {
    return py::bytes(deflate_tokens_cpu(tokens, std::string(data), fin));
  });
  py::class_<GzipStats>(m, "GzipStats")
      .def_readonly("inputs", &GzipStats::inputs)
      .def_readonly("blocks", &GzipStats::blocks)
      .def_readonly("in_bytes", &GzipStats::in_bytes)
      .def_readonly("out_bytes", &GzipStats::out_bytes)
      .def_readonly("stored_blocks", &GzipStats::stored_blocks)
      .def_readonly("inflated", &GzipStats::inflated)
      .def_readonly("last_pack_ms", &GzipStats::last_pack_ms)
      .def_readonly("last_gpu_ms", &GzipStats::last_gpu_ms)
      .def_readonly("last_assemble_ms", &GzipStats::last_assemble_ms);
  py::class_<GpuGzip>(m, "GpuGzip")
      .def(py::init<int>(), py::arg("device") = 0)
      .def("compress", [](GpuGzip& g, const py::list& in) {
        auto v = views(in);
        std::vector<std::string> out;
        {
          py::gil_scoped_release nogil;
          out = g.compress(v);
        }
        return to_list(out);
      })
      .def("deflate", [](GpuGzip& g, const py::list& in) {
        auto v = views(in);
        std::vector<std::string> out;
        {
          py::gil_scoped_release nogil;
          out = g.deflate(v);
        }
        return to_list(out);
      })
      .def("inflate", [](GpuGzip& g, const py::list& in, uint64_t max_out) {
        auto v = views(in);
        std::vector<std::string> out;
        std::vector<uint8_t> ok;
        {
          py::gil_scoped_release nogil;
          out = g.inflate(v, &ok, max_out);
        }
        py::list l(out.size());
        for (size_t i = 0; i < out.size(); ++i)
          l[i] = ok[i] ? py::object(py::bytes(out[i])) : py::object(py::none());
        return l;
      }, py::arg("members"), py::arg("max_out") = 64ull << 20)
      .def("stats", &GpuGzip::stats)
      .def_property_readonly("device", &GpuGzip::device);
}
