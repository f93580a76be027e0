// pybind11 bindings of the native CPU homework suite (module ``_cpu.suite``).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdlib>
#include <cstring>

#include "cpu/suite_cpu.h"

namespace py = pybind11;

namespace cme::cpu {

using namespace cme::cpu::suite;

void bind_suite_cpu(pybind11::module_& m) {
  using u32arr = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>;
  auto sm = m.def_submodule("suite", "CME213 homework algorithms on the CPU (OpenMP) and host oracles");
  sm.def("glibc_rand", [](int64_t n, unsigned seed) {
    // the reference's fixtures and generators use C rand() (hw1code/test_files/input = srand(1) stream)
    py::array_t<uint32_t> out(n);
    std::srand(seed);
    auto* p = out.mutable_data();
    for (int64_t i = 0; i < n; ++i) p[i] = (uint32_t)std::rand();
    return out;
  }, py::arg("n"), py::arg("seed") = 1);
  sm.def("sum_even_odd", [](u32arr v, bool parallel) {
    auto r = parallel ? sum_even_odd_parallel(v.data(), v.size()) : sum_even_odd_serial(v.data(), v.size());
    return py::make_tuple(r.first, r.second);
  }, py::arg("v"), py::arg("parallel") = true);
  sm.def("block_histograms", [](u32arr keys, int num_blocks, int num_buckets, int start_bit, int64_t block_size) {
    auto h = block_histograms(keys.data(), keys.size(), num_blocks, num_buckets, start_bit, block_size);
    return py::array_t<uint32_t>(h.size(), h.data());
  });
  sm.def("reduce_to_global", [](u32arr bh, int num_blocks, int num_buckets) {
    u32vec v(bh.data(), bh.data() + bh.size());
    auto g = reduce_to_global(v, num_blocks, num_buckets);
    return py::array_t<uint32_t>(g.size(), g.data());
  });
  sm.def("scan_global", [](u32arr g) {
    u32vec v(g.data(), g.data() + g.size());
    auto s = exclusive_scan(v);
    return py::array_t<uint32_t>(s.size(), s.data());
  });
  sm.def("block_exscan", [](int num_buckets, int num_blocks, u32arr gscan, u32arr bh) {
    u32vec gs(gscan.data(), gscan.data() + gscan.size()), b(bh.data(), bh.data() + bh.size());
    auto o = block_exscan(num_buckets, num_blocks, gs, b);
    return py::array_t<uint32_t>(o.size(), o.data());
  });
  sm.def("populate", [](u32arr bex, int num_blocks, int num_buckets, int start_bit, int64_t block_size,
                        u32arr keys) {
    u32vec b(bex.data(), bex.data() + bex.size());
    py::array_t<uint32_t> out(keys.size());
    populate(b, num_blocks, num_buckets, start_bit, block_size, keys.data(), keys.size(), out.mutable_data());
    return out;
  });
  sm.def("radix_sort_parallel", [](u32arr keys, int num_bits, int num_blocks) {
    py::array_t<uint32_t> out(keys.size());
    std::memcpy(out.mutable_data(), keys.data(), keys.size() * 4);
    std::vector<uint32_t> tmp(keys.size());
    {
      py::gil_scoped_release r;
      radix_parallel(out.mutable_data(), tmp.data(), keys.size(), num_bits, num_blocks);
    }
    return out;
  }, py::arg("keys"), py::arg("num_bits") = 8, py::arg("num_blocks") = 8);
  sm.def("radix_sort_serial", [](u32arr keys, int num_bits) {
    py::array_t<uint32_t> out(keys.size());
    std::memcpy(out.mutable_data(), keys.data(), keys.size() * 4);
    std::vector<uint32_t> tmp(keys.size());
    radix_serial(out.mutable_data(), tmp.data(), keys.size(), num_bits);
    return out;
  }, py::arg("keys"), py::arg("num_bits") = 16);
  sm.def("radix_sort_lsd", [](u32arr keys) {
    py::array_t<uint32_t> out(keys.size());
    std::memcpy(out.mutable_data(), keys.data(), keys.size() * 4);
    std::vector<uint32_t> tmp(keys.size());
    {
      py::gil_scoped_release r;
      radix_parallel_lsd(out.mutable_data(), tmp.data(), keys.size());
    }
    return out;
  }, py::arg("keys"));
  sm.def("std_sort", [](u32arr keys) {
    py::array_t<uint32_t> out(keys.size());
    std::memcpy(out.mutable_data(), keys.data(), keys.size() * 4);
    {
      py::gil_scoped_release r;
      std_sort(out.mutable_data(), keys.size());
    }
    return out;
  }, py::arg("keys"));
  sm.def("stencil", [](py::array_t<float, py::array::c_style> grid, int order, float xcfl, float ycfl, float scale,
                       int iters) {
    if (grid.ndim() != 2) throw std::invalid_argument("grid must be 2-D [gy][gx]");
    py::array_t<float> out({grid.shape(0), grid.shape(1)});
    std::memcpy(out.mutable_data(), grid.data(), grid.size() * 4);
    {
      py::gil_scoped_release r;
      stencil_cpu(out.mutable_data(), (int)grid.shape(1), (int)grid.shape(0), order, xcfl, ycfl, scale, iters);
    }
    return out;
  });
  sm.def("pagerank", [](u32arr indptr, u32arr edges, py::array_t<float, py::array::c_style | py::array::forcecast> inv,
                        py::array_t<float, py::array::c_style | py::array::forcecast> vals, int iters) {
    py::array_t<float> out(vals.size());
    std::memcpy(out.mutable_data(), vals.data(), vals.size() * 4);
    pagerank_cpu(indptr.data(), edges.data(), inv.data(), out.mutable_data(), (int)vals.size(), iters);
    return out;
  });
}

}  // namespace cme::cpu
