// Native test driver for the C++ CPU runtime (no Python): the fp64 MLP oracle,
// file I/O and the OpenMP homework algorithms.  Built by CMake (target
// `native_tests`) and by tests/test_native.py, normally with
// -fsanitize=address,undefined so host-side memory errors fail the run.
//
//   ./native_tests [filter]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "cpu/io.h"
#include "cpu/mlp_cpu.h"
#include "cpu/suite_cpu.h"
#include "test_macros.h"

using namespace cme;

namespace {

std::string tmpdir() {
  const char* t = std::getenv("TMPDIR");
  return t ? t : "/tmp";
}

struct Net {
  int P, H, C;
  std::vector<double> W1, b1, W2, b2;
  Net(int p, int h, int c) : P(p), H(h), C(c), W1(h * p), b1(h), W2(c * h), b2(c) {}
  cpu::NetView view() { return {P, H, C, W1.data(), b1.data(), W2.data(), b2.data()}; }
};

std::vector<double> random_X(int n, int P, unsigned seed) {
  std::mt19937 g(seed);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<double> X((size_t)n * P);
  for (auto& x : X) x = u(g);
  return X;
}

std::vector<int> random_labels(int n, int C, unsigned seed) {
  std::mt19937 g(seed);
  std::vector<int> y(n);
  for (auto& v : y) v = (int)(g() % C);
  return y;
}

double max_rel(const std::vector<double>& a, const std::vector<double>& b) {
  double m = 0;
  for (size_t i = 0; i < a.size(); ++i)
    m = std::max(m, std::fabs(a[i] - b[i]) / std::max(1.0, std::max(std::fabs(a[i]), std::fabs(b[i]))));
  return m;
}

std::vector<uint32_t> rand_keys(size_t n, unsigned seed) {
  std::mt19937 g(seed);
  std::vector<uint32_t> k(n);
  for (auto& x : k) x = g();
  return k;
}

}  // namespace

// ------------------------------------------------------------------ MLP oracle
CME_TEST(mlp_init_is_seeded_and_deterministic) {
  Net a(20, 7, 3), b(20, 7, 3);
  cpu::init_params(a.view());
  cpu::init_params(b.view());
  EXPECT_VECTOR_EQ(a.W1, b.W1);
  EXPECT_VECTOR_EQ(a.W2, b.W2);
  EXPECT_TRUE(std::all_of(a.b1.begin(), a.b1.end(), [](double v) { return v == 0.0; }));
  double s = 0;
  for (double w : a.W1) s += w * w;
  EXPECT_NEAR(std::sqrt(s / a.W1.size()), 0.01, 0.004);  // 0.01 * randn
}

CME_TEST(mlp_softmax_rows_sum_to_one) {
  Net net(12, 5, 4);
  cpu::init_params(net.view());
  const int n = 9;
  auto X = random_X(n, 12, 1);
  std::vector<double> a1(n * 5), yc(n * 4);
  cpu::feedforward(net.view(), X.data(), n, a1.data(), yc.data(), true);
  for (int i = 0; i < n; ++i) EXPECT_NEAR(yc[i * 4] + yc[i * 4 + 1] + yc[i * 4 + 2] + yc[i * 4 + 3], 1.0, 1e-12);
  for (double v : a1) EXPECT_TRUE(v > 0.0 && v < 1.0);
}

CME_TEST(mlp_backprop_matches_numgrad) {
  Net net(10, 6, 3);
  cpu::init_params(net.view());
  for (auto& w : net.W1) w *= 30;  // leave the linear regime
  for (auto& w : net.W2) w *= 30;
  const int n = 8;
  auto X = random_X(n, 10, 2);
  auto y = random_labels(n, 3, 3);
  const double reg = 1e-3;
  std::vector<double> a1(n * 6), yc(n * 3);
  cpu::feedforward(net.view(), X.data(), n, a1.data(), yc.data(), true);
  std::vector<double> dW1(60), db1(6), dW2(18), db2(3), nW1(60), nb1(6), nW2(18), nb2(3);
  cpu::backprop(net.view(), X.data(), y.data(), n, reg, a1.data(), yc.data(), 1.0 / n, dW1.data(), db1.data(),
                dW2.data(), db2.data());
  cpu::numgrad(net.view(), X.data(), y.data(), n, reg, nW1.data(), nb1.data(), nW2.data(), nb2.data(), true);
  EXPECT_TRUE(max_rel(dW1, nW1) < 1e-7);
  EXPECT_TRUE(max_rel(db1, nb1) < 1e-7);
  EXPECT_TRUE(max_rel(dW2, nW2) < 1e-7);
  EXPECT_TRUE(max_rel(db2, nb2) < 1e-7);
}

CME_TEST(mlp_train_reduces_loss) {
  Net net(16, 8, 4);
  cpu::init_params(net.view());
  const int N = 400;
  auto y = random_labels(N, 4, 5);
  std::vector<double> X((size_t)N * 16, 0.0);
  std::mt19937 g(6);
  std::normal_distribution<double> nd(0.0, 0.3);
  for (int i = 0; i < N; ++i)
    for (int p = 0; p < 16; ++p) X[(size_t)i * 16 + p] = (p % 4 == y[i] ? 1.0 : 0.0) + nd(g);
  cpu::TrainOpts o;
  o.lr = 0.5;
  o.reg = 1e-4;
  o.epochs = 30;
  o.batch = 50;
  o.print_every = 1;
  o.outdir = tmpdir();
  auto losses = cpu::train(net.view(), X.data(), y.data(), N, o);
  EXPECT_TRUE(losses.size() > 2);
  if (losses.size() > 2) EXPECT_TRUE(losses.back() < 0.5 * losses.front());
  std::vector<int> pred(N);
  cpu::predict(net.view(), X.data(), N, pred.data(), true);
  int ok = 0;
  for (int i = 0; i < N; ++i) ok += pred[i] == y[i];
  EXPECT_TRUE(ok > N * 9 / 10);
}

// ------------------------------------------------------------------ I/O
CME_TEST(io_raw_ascii_roundtrip) {
  std::vector<double> a = {1.0, -2.5e-7, 3.14159265358979, 0.0, 1e300, -1e-300};
  const std::string p = tmpdir() + "/cme_native_raw.mat";
  io::save_raw_ascii(p, a.data(), 2, 3, 17);
  int64_t r = 0, c = 0;
  auto b = io::load_raw_ascii(p, &r, &c);
  EXPECT_EQ(r, 2);
  EXPECT_EQ(c, 3);
  EXPECT_VECTOR_EQ(a, b);
}

CME_TEST(io_idx_roundtrip) {
  std::vector<uint8_t> px(3 * 4 * 5), lab = {7, 0, 9};
  std::iota(px.begin(), px.end(), 0);
  const std::string pi = tmpdir() + "/cme_native_img.idx", pl = tmpdir() + "/cme_native_lab.idx";
  io::write_idx_images(pi, px.data(), 3, 4, 5);
  io::write_idx_labels(pl, lab.data(), 3);
  int n = 0, rows = 0, cols = 0, nl = 0;
  auto px2 = io::read_idx_images(pi, &n, &rows, &cols);
  auto lab2 = io::read_idx_labels(pl, &nl);
  EXPECT_EQ(n, 3);
  EXPECT_EQ(rows, 4);
  EXPECT_EQ(cols, 5);
  EXPECT_VECTOR_EQ(px, px2);
  EXPECT_VECTOR_EQ(lab, lab2);
}

// ------------------------------------------------------------------ hw1
CME_TEST(hw1_sum_even_odd) {
  std::vector<uint32_t> v(1000003);
  std::mt19937 g(7);
  for (auto& x : v) x = g() % 101;
  uint64_t e = 0, o = 0;
  for (auto x : v) (x % 2 ? o : e) += x;
  auto s = cpu::suite::sum_even_odd_serial(v.data(), v.size());
  auto p = cpu::suite::sum_even_odd_parallel(v.data(), v.size());
  EXPECT_EQ(s.first, e);
  EXPECT_EQ(s.second, o);
  EXPECT_EQ(p.first, e);
  EXPECT_EQ(p.second, o);
}

CME_TEST(hw1_radix_stages_compose_to_stable_pass) {
  auto keys = rand_keys(40000, 8);
  const int nb = 8, buckets = 256;
  const int64_t bs = 5000;
  auto bh = cpu::suite::block_histograms(keys.data(), keys.size(), nb, buckets, 0, bs);
  auto gh = cpu::suite::reduce_to_global(bh, nb, buckets);
  EXPECT_EQ(std::accumulate(gh.begin(), gh.end(), 0u), 40000u);
  auto gs = cpu::suite::exclusive_scan(gh);
  auto bex = cpu::suite::block_exscan(buckets, nb, gs, bh);
  std::vector<uint32_t> out(keys.size());
  cpu::suite::populate(bex, nb, buckets, 0, bs, keys.data(), keys.size(), out.data());
  auto exp = keys;
  std::stable_sort(exp.begin(), exp.end(), [](uint32_t a, uint32_t b) { return (a & 255) < (b & 255); });
  EXPECT_VECTOR_EQ(out, exp);
}

CME_TEST(hw1_radix_sorts) {
  for (size_t n : {size_t(0), size_t(1), size_t(17), size_t(100000)}) {
    auto keys = rand_keys(n, 9 + (unsigned)n);
    auto exp = keys;
    std::sort(exp.begin(), exp.end());
    std::vector<uint32_t> tmp(n);
    auto a = keys;
    cpu::suite::radix_serial(a.data(), tmp.data(), n, 16);
    EXPECT_VECTOR_EQ(a, exp);
    for (int blocks : {1, 3, 8, 64}) {
      auto b = keys;
      cpu::suite::radix_parallel(b.data(), tmp.data(), n, 8, blocks);
      EXPECT_VECTOR_EQ(b, exp);
    }
  }
}

// ------------------------------------------------------------------ hw2 / hw3
CME_TEST(hw2_pagerank_conserves_mass_on_regular_graph) {
  // ring where every node has in-degree = out-degree = 2: the uniform vector is a fixed point
  const int n = 1000;
  std::vector<uint32_t> indptr(n + 1), edges(2 * n);
  for (int i = 0; i <= n; ++i) indptr[i] = 2 * i;
  for (int i = 0; i < n; ++i) {
    edges[2 * i] = (i + 1) % n;
    edges[2 * i + 1] = (i + n - 1) % n;
  }
  std::vector<float> inv(n, 0.5f), v(n, 1.0f / n);
  cpu::suite::pagerank_cpu(indptr.data(), edges.data(), inv.data(), v.data(), n, 7);
  for (float x : v) EXPECT_NEAR(x, 1.0 / n, 1e-9);
}

CME_TEST(hw3_stencil_linear_field_is_steady) {
  // the discrete Laplacian of a linear field is zero: with a fixed border (scale 1) the field must not change
  for (int order : {2, 4, 8}) {
    const int gx = 40, gy = 30;
    const float cfl = order == 2 ? 0.1f : order == 4 ? 0.1f / 12 : 0.1f / 5040;
    std::vector<float> g((size_t)gx * gy);
    for (int y = 0; y < gy; ++y)
      for (int x = 0; x < gx; ++x) g[(size_t)y * gx + x] = 0.25f * x + 0.5f * y;
    auto g0 = g;
    cpu::suite::stencil_cpu(g.data(), gx, gy, order, cfl, cfl, 1.0f, 3);
    for (size_t i = 0; i < g.size(); ++i) EXPECT_NEAR(g[i], g0[i], 1e-3);
    auto h = g0;
    cpu::suite::stencil_cpu(h.data(), gx, gy, order, cfl, cfl, 0.5f, 3);
    EXPECT_NEAR(h[gx - 1], g0[gx - 1] * 0.125f, 1e-5);  // border decays by scale^iters
  }
}

int main(int argc, char** argv) { return cme::test::run_all(argc > 1 ? argv[1] : nullptr); }
