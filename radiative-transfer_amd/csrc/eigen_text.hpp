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

// data is ColMajor rows x cols; writes the matrix followed by std::endl
inline bool write_eigen_text(const std::string &path, const double *data, size_t rows, size_t cols) {
  std::ofstream file(path);
  if (!file.is_open()) return false;
  size_t width = 0;
  for (size_t k = 0; k < rows * cols; ++k) {
    std::stringstream ss;
    ss.copyfmt(file);
    ss << data[k];
    width = std::max(width, ss.str().size());
  }
  for (size_t i = 0; i < rows; ++i) {
    if (i) file << "\n";
    for (size_t j = 0; j < cols; ++j) {
      if (j) file << " ";
      file.width(static_cast<std::streamsize>(width));
      file << data[i + rows * j];
    }
  }
  file << std::endl;
  return true;
}

inline bool write_eigen_text(const std::string &path, const std::vector<double> &v, size_t rows, size_t cols) {
  return write_eigen_text(path, v.data(), rows, cols);
}

}  // namespace rtamd
