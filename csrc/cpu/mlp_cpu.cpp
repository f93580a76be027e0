#include "mlp_cpu.h"

#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <filesystem>
#include <random>
#include <stdexcept>

#include "io.h"

namespace cme::cpu {

namespace {

inline double dot(const double* __restrict__ a, const double* __restrict__ b, int n) {
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    s0 += a[i] * b[i];
    s1 += a[i + 1] * b[i + 1];
    s2 += a[i + 2] * b[i + 2];
    s3 += a[i + 3] * b[i + 3];
  }
  for (; i < n; ++i) s0 += a[i] * b[i];
  return (s0 + s1) + (s2 + s3);
}

void softmax_row(double* z, int C, bool shift) {
  double m = 0;
  if (shift) {
    m = z[0];
    for (int c = 1; c < C; ++c) m = std::max(m, z[c]);
  }
  double s = 0;
  for (int c = 0; c < C; ++c) {
    z[c] = std::exp(z[c] - m);
    s += z[c];
  }
  for (int c = 0; c < C; ++c) z[c] /= s;
}

}  // namespace

void init_params(NetView net) {
  const int dims[3] = {net.P, net.H, net.C};
  double* W[2] = {net.W1, net.W2};
  double* b[2] = {net.b1, net.b2};
  for (int i = 0; i < 2; ++i) {
    const int rows = dims[i + 1], cols = dims[i];
    std::mt19937_64 engine;
    engine.seed((std::mt19937_64::result_type)i);
    std::normal_distribution<double> nd;
    nd.reset();
    // column-major fill order of an rows x cols Armadillo matrix -> row-major storage
    for (int64_t k = 0; k < (int64_t)rows * cols; ++k) {
      const int64_t r = k % rows, c = k / rows;
      W[i][r * cols + c] = 0.01 * nd(engine);
    }
    std::fill(b[i], b[i] + rows, 0.0);
  }
}

void feedforward(const NetView& net, const double* X, int n, double* a1, double* yc, bool shift) {
  const int P = net.P, H = net.H, C = net.C;
#pragma omp parallel for schedule(static)
  for (int j = 0; j < n; ++j) {
    const double* x = X + (size_t)j * P;
    double* a = a1 + (size_t)j * H;
    for (int h = 0; h < H; ++h) {
      const double z = dot(net.W1 + (size_t)h * P, x, P) + net.b1[h];
      a[h] = 1.0 / (1.0 + std::exp(-z));
    }
    double* y = yc + (size_t)j * C;
    for (int c = 0; c < C; ++c) y[c] = dot(net.W2 + (size_t)c * H, a, H) + net.b2[c];
    softmax_row(y, C, shift);
  }
}

void backprop(const NetView& net, const double* X, const int* labels, int n, double reg, const double* a1,
              const double* yc, double scale, double* dW1, double* db1, double* dW2, double* db2) {
  const int P = net.P, H = net.H, C = net.C;
  std::vector<double> D((size_t)n * C), dZ((size_t)n * H);
#pragma omp parallel for schedule(static)
  for (int j = 0; j < n; ++j) {
    const double* y = yc + (size_t)j * C;
    double* d = D.data() + (size_t)j * C;
    for (int c = 0; c < C; ++c) d[c] = scale * (y[c] - (c == labels[j] ? 1.0 : 0.0));
    const double* a = a1 + (size_t)j * H;
    double* dz = dZ.data() + (size_t)j * H;
    for (int h = 0; h < H; ++h) {
      double da = 0;
      for (int c = 0; c < C; ++c) da += net.W2[(size_t)c * H + h] * d[c];
      dz[h] = da * a[h] * (1.0 - a[h]);
    }
  }
  // dW2 = D a1^T + reg W2 ; db2 = sum D
  for (int c = 0; c < C; ++c) {
    double sb = 0;
    for (int j = 0; j < n; ++j) sb += D[(size_t)j * C + c];
    db2[c] = sb;
    for (int h = 0; h < H; ++h) {
      double s = 0;
      for (int j = 0; j < n; ++j) s += D[(size_t)j * C + c] * a1[(size_t)j * H + h];
      dW2[(size_t)c * H + h] = s + reg * net.W2[(size_t)c * H + h];
    }
  }
  // dW1 = dZ X^T + reg W1 ; db1 = sum dZ
#pragma omp parallel for schedule(static)
  for (int h = 0; h < H; ++h) {
    double* g = dW1 + (size_t)h * P;
    const double* w = net.W1 + (size_t)h * P;
    for (int p = 0; p < P; ++p) g[p] = reg * w[p];
    double sb = 0;
    for (int j = 0; j < n; ++j) {
      const double dz = dZ[(size_t)j * H + h];
      sb += dz;
      const double* x = X + (size_t)j * P;
      for (int p = 0; p < P; ++p) g[p] += dz * x[p];
    }
    db1[h] = sb;
  }
}

double loss(const NetView& net, const double* yc, const int* labels, int n, double reg) {
  double ce = 0;
  for (int j = 0; j < n; ++j) ce -= std::log(yc[(size_t)j * net.C + labels[j]]);
  double nrm = 0;
  for (int64_t i = 0; i < (int64_t)net.H * net.P; ++i) nrm += net.W1[i] * net.W1[i];
  for (int64_t i = 0; i < (int64_t)net.C * net.H; ++i) nrm += net.W2[i] * net.W2[i];
  return ce / n + 0.5 * reg * nrm;
}

void predict(const NetView& net, const double* X, int n, int* out, bool shift) {
  const int chunk = 4096;
  std::vector<double> a1((size_t)chunk * net.H), yc((size_t)chunk * net.C);
  for (int s = 0; s < n; s += chunk) {
    const int m = std::min(chunk, n - s);
    feedforward(net, X + (size_t)s * net.P, m, a1.data(), yc.data(), shift);
    for (int j = 0; j < m; ++j) {
      const double* y = yc.data() + (size_t)j * net.C;
      out[s + j] = (int)(std::max_element(y, y + net.C) - y);
    }
  }
}

void numgrad(NetView net, const double* X, const int* labels, int n, double reg, double* dW1, double* db1,
             double* dW2, double* db2, bool shift) {
  const double h = 1e-5;
  std::vector<double> a1((size_t)n * net.H), yc((size_t)n * net.C);
  auto f = [&]() {
    feedforward(net, X, n, a1.data(), yc.data(), shift);
    return loss(net, yc.data(), labels, n, reg);
  };
  auto fd = [&](double* p, int64_t cnt, double* out) {
    for (int64_t i = 0; i < cnt; ++i) {
      const double old = p[i];
      p[i] = old + h;
      const double fp = f();
      p[i] = old - h;
      const double fm = f();
      out[i] = (fp - fm) / (2 * h);
      p[i] = old;
    }
  };
  fd(net.W1, (int64_t)net.H * net.P, dW1);
  fd(net.W2, (int64_t)net.C * net.H, dW2);
  fd(net.b1, net.H, db1);
  fd(net.b2, net.C, db2);
}

std::vector<double> train(NetView net, const double* X, const int* labels, int N, const TrainOpts& o) {
  const int P = net.P, H = net.H, C = net.C, B = o.batch;
  if (B <= 0) throw std::invalid_argument("batch size must be positive");
  std::vector<double> a1((size_t)B * H), yc((size_t)B * C);
  std::vector<double> dW1((size_t)H * P), db1(H), dW2((size_t)C * H), db2(C);
  std::vector<double> losses;
  if (o.debug) std::filesystem::create_directories(o.outdir + "/CPUmats");
  int iter = o.iter0;
  for (int epoch = 0; epoch < o.epochs; ++epoch) {
    const int nb = (N + B - 1) / B;
    for (int batch = 0; batch < nb; ++batch) {
      const int s = batch * B, n = std::min(B, N - s);
      const double* Xb = X + (size_t)s * P;
      feedforward(net, Xb, n, a1.data(), yc.data(), o.shift);
      backprop(net, Xb, labels + s, n, o.reg, a1.data(), yc.data(), 1.0 / n, dW1.data(), db1.data(), dW2.data(),
               db2.data());
      if (o.print_every > 0 && iter % o.print_every == 0) {
        const double l = loss(net, yc.data(), labels + s, n, o.reg);
        losses.push_back(l);
        std::printf("Loss at iteration %d of epoch %d/%d = %.10g\n", iter, epoch, o.epochs, l);
        std::fflush(stdout);
      }
      for (int64_t i = 0; i < (int64_t)H * P; ++i) net.W1[i] -= o.lr * dW1[i];
      for (int64_t i = 0; i < (int64_t)C * H; ++i) net.W2[i] -= o.lr * dW2[i];
      for (int i = 0; i < H; ++i) net.b1[i] -= o.lr * db1[i];
      for (int i = 0; i < C; ++i) net.b2[i] -= o.lr * db2[i];
      const bool print_flag = o.print_every <= 0 ? batch == 0 : iter % o.print_every == 0;
      if (o.debug && print_flag) {
        const std::string d = o.outdir + "/CPUmats/Sequential";
        const std::string it = std::to_string(iter) + ".mat";
        io::save_raw_ascii(d + "W0-" + it, net.W1, H, P, o.ckpt_precision);
        io::save_raw_ascii(d + "W1-" + it, net.W2, C, H, o.ckpt_precision);
        io::save_raw_ascii(d + "b0-" + it, net.b1, H, 1, o.ckpt_precision);
        io::save_raw_ascii(d + "b1-" + it, net.b2, C, 1, o.ckpt_precision);
      }
      ++iter;
    }
  }
  return losses;
}

}  // namespace cme::cpu
