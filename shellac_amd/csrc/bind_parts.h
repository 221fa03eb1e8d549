// Split pybind11 registration units (keeps each translation unit small).
#pragma once
#include <pybind11/pybind11.h>

void bind_http(pybind11::module_& m);  // bind_http.cc: HttpParser, StreamBuf
void bind_net(pybind11::module_& m);   // bind_net.cc: ketama ring, proxy, memcached protocol
void bind_router(pybind11::module_& m);  // bind_router.cc: fused routed-step ops
void bind_deflate(pybind11::module_& m);  // bind_deflate.cc: GPU batch gzip
