// pybind11 bindings for the native CPU runtime (module cme213_sp18_amd._cpu).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <omp.h>

#include <cstring>

#include "cpu/io.h"
#include "cpu/mlp_cpu.h"
#include "cpu/suite_cpu.h"

namespace py = pybind11;
using f64arr = py::array_t<double, py::array::c_style | py::array::forcecast>;
using i32arr = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
using u32arr = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>;

namespace {

double* mut(py::array_t<double>& a) {
  if (!(a.flags() & py::array::c_style)) throw std::invalid_argument("expected C-contiguous float64 array");
  return a.mutable_data();
}

cme::cpu::NetView view(py::array_t<double>& W1, py::array_t<double>& b1, py::array_t<double>& W2,
                       py::array_t<double>& b2) {
  if (W1.ndim() != 2 || W2.ndim() != 2) throw std::invalid_argument("W1, W2 must be 2-D");
  cme::cpu::NetView v{(int)W1.shape(1), (int)W1.shape(0), (int)W2.shape(0), mut(W1), mut(b1), mut(W2), mut(b2)};
  if (W2.shape(1) != v.H || b1.size() != v.H || b2.size() != v.C) throw std::invalid_argument("param shape mismatch");
  return v;
}

void check_x(const f64arr& X, int P) {
  if (X.ndim() != 2 || X.shape(1) != P) throw std::invalid_argument("X must be [n][P] float64");
}

}  // namespace

PYBIND11_MODULE(_cpu, m) {
  m.doc() = "cme213_sp18_amd native CPU runtime (fp64 oracle trainer, IDX/raw_ascii I/O, OpenMP suite)";

  m.def("omp_max_threads", []() { return omp_get_max_threads(); });

  m.def("init_params", [](py::array_t<double> W1, py::array_t<double> b1, py::array_t<double> W2,
                          py::array_t<double> b2) { cme::cpu::init_params(view(W1, b1, W2, b2)); });

  m.def(
      "feedforward",
      [](py::array_t<double> W1, py::array_t<double> b1, py::array_t<double> W2, py::array_t<double> b2, f64arr X,
         bool shift) {
        auto v = view(W1, b1, W2, b2);
        check_x(X, v.P);
        const int n = (int)X.shape(0);
        py::array_t<double> a1({n, v.H}), yc({n, v.C});
        {
          py::gil_scoped_release r;
          cme::cpu::feedforward(v, X.data(), n, a1.mutable_data(), yc.mutable_data(), shift);
        }
        return py::make_tuple(a1, yc);
      },
      py::arg("W1"), py::arg("b1"), py::arg("W2"), py::arg("b2"), py::arg("X"), py::arg("shift") = true);

  m.def(
      "backprop",
      [](py::array_t<double> W1, py::array_t<double> b1, py::array_t<double> W2, py::array_t<double> b2, f64arr X,
         i32arr labels, double reg, f64arr a1, f64arr yc, double scale) {
        auto v = view(W1, b1, W2, b2);
        check_x(X, v.P);
        const int n = (int)X.shape(0);
        py::array_t<double> dW1({v.H, v.P}), db1(v.H), dW2({v.C, v.H}), db2(v.C);
        {
          py::gil_scoped_release r;
          cme::cpu::backprop(v, X.data(), labels.data(), n, reg, a1.data(), yc.data(), scale, dW1.mutable_data(),
                             db1.mutable_data(), dW2.mutable_data(), db2.mutable_data());
        }
        return py::make_tuple(dW1, db1, dW2, db2);
      });

  m.def("loss", [](py::array_t<double> W1, py::array_t<double> b1, py::array_t<double> W2, py::array_t<double> b2,
                   f64arr yc, i32arr labels, double reg) {
    auto v = view(W1, b1, W2, b2);
    return cme::cpu::loss(v, yc.data(), labels.data(), (int)labels.size(), reg);
  });

  m.def(
      "predict",
      [](py::array_t<double> W1, py::array_t<double> b1, py::array_t<double> W2, py::array_t<double> b2, f64arr X,
         bool shift) {
        auto v = view(W1, b1, W2, b2);
        check_x(X, v.P);
        const int n = (int)X.shape(0);
        py::array_t<int32_t> out(n);
        {
          py::gil_scoped_release r;
          cme::cpu::predict(v, X.data(), n, out.mutable_data(), shift);
        }
        return out;
      },
      py::arg("W1"), py::arg("b1"), py::arg("W2"), py::arg("b2"), py::arg("X"), py::arg("shift") = true);

  m.def(
      "numgrad",
      [](py::array_t<double> W1, py::array_t<double> b1, py::array_t<double> W2, py::array_t<double> b2, f64arr X,
         i32arr labels, double reg, bool shift) {
        auto v = view(W1, b1, W2, b2);
        check_x(X, v.P);
        py::array_t<double> dW1({v.H, v.P}), db1(v.H), dW2({v.C, v.H}), db2(v.C);
        cme::cpu::numgrad(v, X.data(), labels.data(), (int)X.shape(0), reg, dW1.mutable_data(), db1.mutable_data(),
                          dW2.mutable_data(), db2.mutable_data(), shift);
        return py::make_tuple(dW1, db1, dW2, db2);
      },
      py::arg("W1"), py::arg("b1"), py::arg("W2"), py::arg("b2"), py::arg("X"), py::arg("labels"),
      py::arg("reg"), py::arg("shift") = true);

  m.def(
      "train",
      [](py::array_t<double> W1, py::array_t<double> b1, py::array_t<double> W2, py::array_t<double> b2, f64arr X,
         i32arr labels, double lr, double reg, int epochs, int batch, int print_every, bool debug,
         std::string outdir, bool shift, int ckpt_precision, int iter0) {
        auto v = view(W1, b1, W2, b2);
        check_x(X, v.P);
        cme::cpu::TrainOpts o;
        o.lr = lr; o.reg = reg; o.epochs = epochs; o.batch = batch; o.print_every = print_every;
        o.debug = debug; o.outdir = outdir; o.shift = shift; o.ckpt_precision = ckpt_precision; o.iter0 = iter0;
        std::vector<double> losses;
        {
          py::gil_scoped_release r;
          losses = cme::cpu::train(v, X.data(), labels.data(), (int)X.shape(0), o);
        }
        return losses;
      },
      py::arg("W1"), py::arg("b1"), py::arg("W2"), py::arg("b2"), py::arg("X"), py::arg("labels"), py::arg("lr"),
      py::arg("reg"), py::arg("epochs"), py::arg("batch"), py::arg("print_every") = 0, py::arg("debug") = false,
      py::arg("outdir") = "Outputs", py::arg("shift") = true, py::arg("ckpt_precision") = 12,
      py::arg("iter0") = 0);

  // ---------------------------------------------------------------- I/O
  m.def(
      "read_idx_images",
      [](const std::string& path, int max_n) {
        int n, r, c;
        auto v = cme::io::read_idx_images(path, &n, &r, &c, max_n);
        py::array_t<uint8_t> a({n, r * c});
        std::memcpy(a.mutable_data(), v.data(), v.size());
        return py::make_tuple(a, r, c);
      },
      py::arg("path"), py::arg("max_n") = -1);
  m.def(
      "read_idx_labels",
      [](const std::string& path, int max_n) {
        int n;
        auto v = cme::io::read_idx_labels(path, &n, max_n);
        py::array_t<uint8_t> a(n);
        std::memcpy(a.mutable_data(), v.data(), v.size());
        return a;
      },
      py::arg("path"), py::arg("max_n") = -1);
  m.def("write_idx_images", [](const std::string& path, py::array_t<uint8_t, py::array::c_style> px, int rows,
                               int cols) {
    cme::io::write_idx_images(path, px.data(), (int)(px.size() / ((size_t)rows * cols)), rows, cols);
  });
  m.def("write_idx_labels", [](const std::string& path, py::array_t<uint8_t, py::array::c_style> lab) {
    cme::io::write_idx_labels(path, lab.data(), (int)lab.size());
  });
  m.def(
      "save_raw_ascii",
      [](const std::string& path, f64arr a, int precision) {
        const int64_t rows = a.ndim() >= 1 ? a.shape(0) : 1;
        const int64_t cols = a.ndim() == 2 ? a.shape(1) : 1;
        cme::io::save_raw_ascii(path, a.data(), rows, cols, precision);
      },
      py::arg("path"), py::arg("a"), py::arg("precision") = 12);
  m.def("load_raw_ascii", [](const std::string& path) {
    int64_t r, c;
    auto v = cme::io::load_raw_ascii(path, &r, &c);
    py::array_t<double> a({r, c});
    std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(double));
    return a;
  });
  m.def("save_label", [](const std::string& path, i32arr lab) { cme::io::save_label(path, lab.data(), lab.size()); });

  cme::cpu::bind_suite_cpu(m);
}
