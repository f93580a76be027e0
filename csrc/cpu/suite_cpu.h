// Native CPU side of the homework suite (OpenMP): bindings registrar.
#pragma once
#include <pybind11/pybind11.h>
namespace cme::cpu {
void bind_suite_cpu(pybind11::module_& m);
}
