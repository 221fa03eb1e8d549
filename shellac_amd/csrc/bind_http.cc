// pybind11 registration: native HTTP codec and StreamBuf.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bind_parts.h"
#include "http.h"
#include "stream_buf.h"

namespace py = pybind11;
using namespace shellac;

void bind_http(py::module_& m) {
  py::class_<HttpParser>(m, "NativeHttpParser")
      .def(py::init<bool>(), py::arg("decode_gzip") = true)
      .def("parse", [](HttpParser& p, py::buffer b, int64_t length) -> size_t {
        py::buffer_info info = b.request();
        size_t n = (size_t)info.size * (size_t)info.itemsize;
        if (length >= 0 && (size_t)length < n) n = (size_t)length;
        return p.parse(static_cast<const char*>(info.ptr), n);
      }, py::arg("data"), py::arg("length") = -1)
      .def("finish", &HttpParser::finish)
      .def("reset", &HttpParser::reset)
      .def("set_eof_body", &HttpParser::set_eof_body)
      .def("set_no_body", &HttpParser::set_no_body)
      .def("set_max_header_bytes", &HttpParser::set_max_header_bytes)
      .def("headers_complete", &HttpParser::headers_complete)
      .def("message_complete", &HttpParser::message_complete)
      .def("error", &HttpParser::error)
      .def("error_message", &HttpParser::error_message)
      .def("is_request", &HttpParser::is_request)
      .def("method", [](HttpParser& p) -> py::object {
        if (!p.is_request() || p.method().empty()) return py::none();
        return py::str(p.method());
      })
      .def("url", [](HttpParser& p) -> py::object {
        if (!p.is_request() || p.url().empty()) return py::none();
        return py::str(p.url());
      })
      .def("status", [](HttpParser& p) -> py::object {
        if (p.is_request()) return py::none();
        return py::int_(p.status());
      })
      .def("version", &HttpParser::version)
      .def("version_tuple", [](HttpParser& p) {
        return py::make_tuple(p.version_major(), p.version_minor());
      })
      .def("message", [](HttpParser& p) -> py::object {
        if (p.is_request()) return py::none();
        return py::str(p.message());
      })
      .def("header_list", [](HttpParser& p) {
        py::list out;
        for (const auto& h : p.headers()) out.append(py::make_tuple(h.first, h.second));
        return out;
      })
      .def("set_header_list", [](HttpParser& p, const std::vector<Header>& hs) {
        p.mutable_headers() = hs;
      })
      .def("body_bytes", [](HttpParser& p) { return py::bytes(p.body()); })
      .def("keep_alive", &HttpParser::keep_alive)
      .def("keep_alive_params", &HttpParser::keep_alive_params)
      .def("serialize", [](HttpParser& p) { return py::bytes(p.serialize()); });

  m.def("canonical_header", &canonical_header);
  m.def("gzip_compress", [](py::bytes b, int level) {
    return py::bytes(gzip_compress(std::string(b), level));
  }, py::arg("data"), py::arg("level") = 6);
  m.def("gzip_decompress", [](py::bytes b) -> py::object {
    std::string out;
    if (!gzip_decompress(std::string(b), &out)) return py::none();
    return py::bytes(out);
  });

  py::class_<StreamBuf>(m, "NativeStreamBuf")
      .def(py::init<>())
      .def("write", [](StreamBuf& s, py::bytes b) { s.write(std::string(b)); })
      .def("ack", &StreamBuf::ack)
      .def("seek", &StreamBuf::seek)
      .def("read", [](StreamBuf& s) { return py::bytes(s.read()); })
      .def("close", &StreamBuf::close)
      .def("buffer", [](StreamBuf& s) { return py::bytes(s.buffer()); })
      .def("clear", &StreamBuf::clear)
      .def("complete", &StreamBuf::complete)
      .def("closed", &StreamBuf::closed)
      .def("ready", &StreamBuf::ready)
      .def("size", &StreamBuf::size)
      .def("pending", &StreamBuf::pending)
      .def("release_acked", &StreamBuf::release_acked);
}
