#include "io.h"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace cme::io {

namespace {

uint32_t be32(const unsigned char* b) {
  return (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | uint32_t(b[3]);
}
void put_be32(std::ofstream& f, uint32_t v) {
  unsigned char b[4] = {(unsigned char)(v >> 24), (unsigned char)(v >> 16), (unsigned char)(v >> 8),
                        (unsigned char)v};
  f.write(reinterpret_cast<char*>(b), 4);
}

std::ifstream open_in(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  return f;
}

}  // namespace

std::vector<uint8_t> read_idx_images(const std::string& path, int* n, int* rows, int* cols, int max_n) {
  auto f = open_in(path);
  unsigned char h[16];
  if (!f.read(reinterpret_cast<char*>(h), 16)) throw std::runtime_error("short IDX header: " + path);
  if (be32(h) != 2051) throw std::runtime_error("not an IDX image file (magic != 2051): " + path);
  int cnt = (int)be32(h + 4);
  *rows = (int)be32(h + 8);
  *cols = (int)be32(h + 12);
  if (max_n >= 0 && max_n < cnt) cnt = max_n;
  *n = cnt;
  std::vector<uint8_t> px((size_t)cnt * (*rows) * (*cols));
  if (!f.read(reinterpret_cast<char*>(px.data()), (std::streamsize)px.size()))
    throw std::runtime_error("truncated IDX image payload: " + path);
  return px;
}

std::vector<uint8_t> read_idx_labels(const std::string& path, int* n, int max_n) {
  auto f = open_in(path);
  unsigned char h[8];
  if (!f.read(reinterpret_cast<char*>(h), 8)) throw std::runtime_error("short IDX header: " + path);
  if (be32(h) != 2049) throw std::runtime_error("not an IDX label file (magic != 2049): " + path);
  int cnt = (int)be32(h + 4);
  if (max_n >= 0 && max_n < cnt) cnt = max_n;
  *n = cnt;
  std::vector<uint8_t> lab((size_t)cnt);
  if (!f.read(reinterpret_cast<char*>(lab.data()), (std::streamsize)lab.size()))
    throw std::runtime_error("truncated IDX label payload: " + path);
  return lab;
}

void write_idx_images(const std::string& path, const uint8_t* px, int n, int rows, int cols) {
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot write " + path);
  put_be32(f, 2051);
  put_be32(f, (uint32_t)n);
  put_be32(f, (uint32_t)rows);
  put_be32(f, (uint32_t)cols);
  f.write(reinterpret_cast<const char*>(px), (std::streamsize)n * rows * cols);
}

void write_idx_labels(const std::string& path, const uint8_t* lab, int n) {
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot write " + path);
  put_be32(f, 2049);
  put_be32(f, (uint32_t)n);
  f.write(reinterpret_cast<const char*>(lab), n);
}

void save_raw_ascii(const std::string& path, const double* a, int64_t rows, int64_t cols, int precision) {
  FILE* fp = std::fopen(path.c_str(), "w");
  if (!fp) throw std::runtime_error("cannot write " + path);
  // Armadillo: f.put(' '); f.width(20); f << x  (scientific, precision 12)
  char fmt[16];
  std::snprintf(fmt, sizeof(fmt), " %%%d.%de", precision + 8, precision);
  std::vector<char> line;
  for (int64_t r = 0; r < rows; ++r) {
    for (int64_t c = 0; c < cols; ++c) std::fprintf(fp, fmt, a[r * cols + c]);
    std::fputc('\n', fp);
  }
  std::fclose(fp);
}

std::vector<double> load_raw_ascii(const std::string& path, int64_t* rows, int64_t* cols) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::vector<double> out;
  std::string line;
  int64_t r = 0, c = -1;
  while (std::getline(f, line)) {
    const char* p = line.c_str();
    char* end = nullptr;
    int64_t k = 0;
    for (;;) {
      double v = std::strtod(p, &end);
      if (end == p) break;
      out.push_back(v);
      ++k;
      p = end;
    }
    if (k == 0) continue;  // blank line
    if (c < 0) c = k;
    else if (k != c) throw std::runtime_error("ragged raw_ascii matrix: " + path);
    ++r;
  }
  *rows = r;
  *cols = c < 0 ? 0 : c;
  return out;
}

void save_label(const std::string& path, const int* labels, int64_t n) {
  std::ofstream f(path);
  if (!f) throw std::runtime_error("cannot write " + path);
  for (int64_t i = 0; i < n; ++i) f << labels[i];
}

}  // namespace cme::io
