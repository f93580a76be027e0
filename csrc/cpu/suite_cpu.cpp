#include "suite_cpu.h"
namespace cme::cpu {
void bind_suite_cpu(pybind11::module_& m) { (void)m; }
}
