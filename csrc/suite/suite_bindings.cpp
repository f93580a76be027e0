// pybind11 bindings for the homework kernel suite (raw device pointers + stream handles).
#include <pybind11/pybind11.h>

#include "suite_kernels.h"

namespace py = pybind11;

namespace {
template <typename T>
T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace

void bind_suite(py::module_& m) {
  using namespace cme::suite;
  auto sm = m.def_submodule("suite", "CME213 homework kernels on gfx950");
  sm.def("shift_bytes", [](uintptr_t in, uintptr_t out, int64_t n, int shift, int width, int block, int grid_cap,
                           uintptr_t s) {
    shift_bytes(P<const uint8_t>(in), P<uint8_t>(out), n, (uint8_t)shift, width, block, grid_cap, S(s));
  }, py::arg("inp"), py::arg("out"), py::arg("n"), py::arg("shift"), py::arg("width"), py::arg("block") = 256,
     py::arg("grid_cap") = 1 << 20, py::arg("stream") = 0);
  sm.def("pagerank_propagate", [](uintptr_t indptr, uintptr_t edges, uintptr_t in, uintptr_t out, uintptr_t inv,
                                  int n, int variant, uintptr_t s) {
    pagerank_propagate(P<const uint32_t>(indptr), P<const uint32_t>(edges), P<const float>(in), P<float>(out),
                       P<const float>(inv), n, variant, S(s));
  }, py::arg("indptr"), py::arg("edges"), py::arg("inp"), py::arg("out"), py::arg("inv_deg"), py::arg("n"),
     py::arg("variant") = 2, py::arg("stream") = 0);
  sm.def("pagerank_premul", [](uintptr_t in, uintptr_t inv, uintptr_t w, int n, uintptr_t s) {
    pagerank_premul(P<const float>(in), P<const float>(inv), P<float>(w), n, S(s));
  }, py::arg("inp"), py::arg("inv_deg"), py::arg("w"), py::arg("n"), py::arg("stream") = 0);
  sm.def("pagerank_propagate_w", [](uintptr_t indptr, uintptr_t edges, uintptr_t w_in, uintptr_t out, uintptr_t w_out,
                                    uintptr_t inv, int n, int lpn, uintptr_t s) {
    pagerank_propagate_w(P<const uint32_t>(indptr), P<const uint32_t>(edges), P<const float>(w_in), P<float>(out),
                         P<float>(w_out), P<const float>(inv), n, lpn, S(s));
  }, py::arg("indptr"), py::arg("edges"), py::arg("w_in"), py::arg("out"), py::arg("w_out"), py::arg("inv_deg"),
     py::arg("n"), py::arg("lpn"), py::arg("stream") = 0);
  sm.def("stencil_lds_tune", [](uintptr_t next, uintptr_t curr, int gx, int gy, float xcfl, float ycfl, int rows,
                                int ahead, int nt, uintptr_t s) {
    stencil_lds_tune(P<float>(next), P<const float>(curr), gx, gy, xcfl, ycfl, rows, ahead, nt, S(s));
  }, py::arg("next"), py::arg("curr"), py::arg("gx"), py::arg("gy"), py::arg("xcfl"), py::arg("ycfl"),
     py::arg("rows"), py::arg("ahead"), py::arg("nt"), py::arg("stream") = 0);
  sm.def("stencil_step", [](uintptr_t next, uintptr_t curr, int gx, int gy, int order, float xcfl, float ycfl,
                            int variant, uintptr_t s) {
    stencil_step(P<float>(next), P<const float>(curr), gx, gy, order, xcfl, ycfl, variant, S(s));
  }, py::arg("next"), py::arg("curr"), py::arg("gx"), py::arg("gy"), py::arg("order"), py::arg("xcfl"),
     py::arg("ycfl"), py::arg("variant"), py::arg("stream") = 0);
  sm.def("stencil_step_bc", [](uintptr_t next, uintptr_t curr, int gx, int gy, int order, float xcfl, float ycfl,
                               int variant, float scale, uintptr_t s) {
    stencil_step_bc(P<float>(next), P<const float>(curr), gx, gy, order, xcfl, ycfl, variant, scale, true, S(s));
  }, py::arg("next"), py::arg("curr"), py::arg("gx"), py::arg("gy"), py::arg("order"), py::arg("xcfl"),
     py::arg("ycfl"), py::arg("variant"), py::arg("scale"), py::arg("stream") = 0);
  sm.def("stencil_step2_bc", [](uintptr_t next, uintptr_t curr, int gx, int gy, int order, float xcfl, float ycfl,
                                float scale, uintptr_t s, int rows, int ahead) {
    stencil_step2_bc(P<float>(next), P<const float>(curr), gx, gy, order, xcfl, ycfl, scale, S(s), rows, ahead);
  }, py::arg("next"), py::arg("curr"), py::arg("gx"), py::arg("gy"), py::arg("order"), py::arg("xcfl"),
     py::arg("ycfl"), py::arg("scale"), py::arg("stream") = 0, py::arg("rows") = 0, py::arg("ahead") = 0);
  sm.def("stencil_bc", [](uintptr_t next, uintptr_t curr, int gx, int gy, int b, float scale, uintptr_t s) {
    stencil_bc(P<float>(next), P<const float>(curr), gx, gy, b, scale, S(s));
  }, py::arg("next"), py::arg("curr"), py::arg("gx"), py::arg("gy"), py::arg("b"), py::arg("scale"),
     py::arg("stream") = 0);
  sm.def("sum_even_odd", [](uintptr_t v, int64_t n, uintptr_t sums, uintptr_t s) {
    sum_even_odd(P<const uint32_t>(v), n, P<unsigned long long>(sums), S(s));
  }, py::arg("v"), py::arg("n"), py::arg("sums"), py::arg("stream") = 0);
  sm.def("radix_workspace_bytes", &radix_workspace_bytes);
  sm.def("radix_sort_u32", [](uintptr_t keys, uintptr_t tmp, int64_t n, uintptr_t ws, uintptr_t s) {
    radix_sort_u32(P<uint32_t>(keys), P<uint32_t>(tmp), n, P<void>(ws), S(s));
  }, py::arg("keys"), py::arg("tmp"), py::arg("n"), py::arg("workspace"), py::arg("stream") = 0);
  sm.def("radix_pass_u32", [](uintptr_t in, uintptr_t out, int64_t n, int bit, uintptr_t ws, uintptr_t s) {
    radix_pass_u32(P<const uint32_t>(in), P<uint32_t>(out), n, bit, P<void>(ws), S(s));
  }, py::arg("inp"), py::arg("out"), py::arg("n"), py::arg("start_bit"), py::arg("workspace"),
     py::arg("stream") = 0);
  sm.def("cipher_workspace_bytes", &cipher_workspace_bytes);
  sm.def("sanitize_lower", [](uintptr_t in, int64_t n, uintptr_t out, uintptr_t count, uintptr_t ws, uintptr_t s) {
    sanitize_lower(P<const uint8_t>(in), n, P<uint8_t>(out), P<int64_t>(count), P<void>(ws), S(s));
  }, py::arg("inp"), py::arg("n"), py::arg("out"), py::arg("count"), py::arg("workspace"), py::arg("stream") = 0);
  sm.def("vigenere_apply", [](uintptr_t in, uintptr_t out, int64_t n, uintptr_t shifts, int period, int sign,
                              int wrap, uintptr_t s) {
    vigenere_apply(P<const uint8_t>(in), P<uint8_t>(out), n, P<const int>(shifts), period, sign, wrap, S(s));
  }, py::arg("inp"), py::arg("out"), py::arg("n"), py::arg("shifts"), py::arg("period"), py::arg("sign"),
     py::arg("wrap"), py::arg("stream") = 0);
  sm.def("byte_histogram", [](uintptr_t in, int64_t n, uintptr_t hist, uintptr_t s) {
    byte_histogram(P<const uint8_t>(in), n, P<uint32_t>(hist), S(s));
  }, py::arg("inp"), py::arg("n"), py::arg("hist"), py::arg("stream") = 0);
  sm.def("shifted_matches", [](uintptr_t t, int64_t n, int lo, int hi, uintptr_t counts, uintptr_t s) {
    shifted_matches(P<const uint8_t>(t), n, lo, hi, P<unsigned long long>(counts), S(s));
  }, py::arg("text"), py::arg("n"), py::arg("lo"), py::arg("hi"), py::arg("counts"), py::arg("stream") = 0);
  sm.def("residue_histogram", [](uintptr_t t, int64_t n, int period, uintptr_t hist, uintptr_t s) {
    residue_histogram(P<const uint8_t>(t), n, period, P<uint32_t>(hist), S(s));
  }, py::arg("text"), py::arg("n"), py::arg("period"), py::arg("hist"), py::arg("stream") = 0);
}
