#include <pybind11/pybind11.h>
#include "suite_kernels.h"
namespace py = pybind11;
void bind_suite(py::module_& m) { (void)m; }
