// Native file I/O: MNIST IDX reader, Armadillo raw_ascii matrices, label files.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace cme::io {

// IDX image file (magic 2051): returns n images of rows*cols uint8 pixels,
// image-major (== the reference's one-column-per-image P x N matrix,
// fpcode/utils/mnist.cpp:9-36, pixel index r*cols + c).  max_n < 0: all.
std::vector<uint8_t> read_idx_images(const std::string& path, int* n, int* rows, int* cols, int max_n = -1);
// IDX label file (magic 2049), fpcode/utils/mnist.cpp:38-57.
std::vector<uint8_t> read_idx_labels(const std::string& path, int* n, int max_n = -1);
void write_idx_images(const std::string& path, const uint8_t* px, int n, int rows, int cols);
void write_idx_labels(const std::string& path, const uint8_t* lab, int n);

// Armadillo raw_ascii text matrix: one matrix ROW per line, each element
// written as ' ' + std::setw(20) scientific with `precision` digits (Armadillo
// diskio::prepare_stream for real types).  precision = 12 reproduces that
// writer; 17 gives an exact fp64 round trip.  `a` is row-major rows x cols.
void save_raw_ascii(const std::string& path, const double* a, int64_t rows, int64_t cols, int precision = 12);
std::vector<double> load_raw_ascii(const std::string& path, int64_t* rows, int64_t* cols);

// Digits concatenated without separators (fpcode/utils/common.cpp:82-94).
void save_label(const std::string& path, const int* labels, int64_t n);

}  // namespace cme::io
