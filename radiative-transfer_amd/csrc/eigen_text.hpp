// eigen_text.hpp -- text output byte-compatible with `os << matrix` under
// Eigen's default IOFormat (Eigen/src/Core/IO.h print_matrix): stream
// precision (6 significant digits), columns right-aligned to the widest
// coefficient, " " between coefficients, "\n" between rows.  A rank-3
// Tensor prints as a dim0 x (rest) ColMajor matrix (main.cc:37-46,119).
#pragma once

#include <algorithm>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace rtamd {

// `os << matrix` for data ColMajor rows x cols (no trailing newline)
inline void write_eigen_text(std::ostream &os, const double *data, size_t rows, size_t cols) {
  size_t width = 0;
  for (size_t k = 0; k < rows * cols; ++k) {
    std::stringstream ss;
    ss.copyfmt(os);
    ss << data[k];
    width = std::max(width, ss.str().size());
  }
  for (size_t i = 0; i < rows; ++i) {
    if (i) os << "\n";
    for (size_t j = 0; j < cols; ++j) {
      if (j) os << " ";
      os.width(static_cast<std::streamsize>(width));
      os << data[i + rows * j];
    }
  }
}

// print_to_file (main.cc:37-57): the matrix followed by std::endl
inline bool write_eigen_text(const std::string &path, const double *data, size_t rows, size_t cols) {
  std::ofstream file(path);
  if (!file.is_open()) return false;
  write_eigen_text(file, data, rows, cols);
  file << std::endl;
  return true;
}

inline bool write_eigen_text(const std::string &path, const std::vector<double> &v, size_t rows, size_t cols) {
  return write_eigen_text(path, v.data(), rows, cols);
}

}  // namespace rtamd
