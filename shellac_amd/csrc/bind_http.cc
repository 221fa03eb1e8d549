#include "bind_parts.h"
void bind_http(pybind11::module_& m) { (void)m; }
