// Native fp64 CPU reference trainer -- the correctness oracle.
//
// Reproduces the reference's sequential Armadillo trainer
// (fpcode/neural_network.cpp:91-279, fpcode/utils/common.cpp:7-18) without
// Armadillo: hand-written OpenMP loops over raw arrays.
//
// Storage (all row-major, C order):
//   X   [N][P]   one sample per row  (== Armadillo's P x N column-major matrix)
//   W1  [H][P]   b1 [H]   W2 [C][H]   b2 [C]
//   yc  [N][C]   softmax output
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace cme::cpu {

struct NetView {
  int P, H, C;
  double *W1, *b1, *W2, *b2;
};

// Armadillo-compatible seeded init (neural_network.h:25-29):
//   layer i: seed(i); W[i] = 0.01 * randn(H[i+1], H[i]) filled column-major; b[i] = 0.
// Uses std::mt19937_64 + std::normal_distribution<double> as Armadillo's C++11
// RNG does; byte-parity with a real Armadillo build is unverified here.
void init_params(NetView net);

// Forward: a1 [n][H] (sigmoid), yc [n][C] (softmax). shift: max-shifted softmax.
void feedforward(const NetView& net, const double* X, int n, double* a1, double* yc, bool shift);

// Gradients for one batch; scale = 1/N_batch (reference), reg added to dW only.
void backprop(const NetView& net, const double* X, const int* labels, int n, double reg, const double* a1,
              const double* yc, double scale, double* dW1, double* db1, double* dW2, double* db2);

// Cross-entropy + 0.5*reg*(|W1|^2 + |W2|^2)   (neural_network.cpp:144-154)
double loss(const NetView& net, const double* yc, const int* labels, int n, double reg);

void predict(const NetView& net, const double* X, int n, int* labels_out, bool shift);

// Central-difference numerical gradient, h = 1e-5 (neural_network.cpp:174-214).
void numgrad(NetView net, const double* X, const int* labels, int n, double reg, double* dW1, double* db1,
             double* dW2, double* db2, bool shift);

struct TrainOpts {
  double lr = 1e-3, reg = 1e-4;
  int epochs = 1, batch = 800, print_every = 0;
  bool debug = false, shift = true;
  std::string outdir = "Outputs";
  int ckpt_precision = 12;  // raw_ascii format, see io.h
  int iter0 = 0;            // iteration counter at the start (a resumed run continues the numbering)
};

// Minibatch SGD (neural_network.cpp:219-279): ceil(N/B) batches per epoch, the
// last one partial; debug snapshots to <outdir>/CPUmats/Sequential{W0,W1,b0,b1}-<iter>.mat.
// Returns the loss values printed (one per print_every iteration).
std::vector<double> train(NetView net, const double* X, const int* labels, int N, const TrainOpts& o);

}  // namespace cme::cpu
