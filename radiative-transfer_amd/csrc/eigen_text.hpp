// eigen_text.hpp -- text output byte-compatible with `os << matrix` under
// Eigen's default IOFormat (Eigen/src/Core/IO.h print_matrix): stream
// precision (6 significant digits), columns right-aligned to the widest
// coefficient, " " between coefficients, "\n" between rows.  A rank-3
// Tensor prints as a dim0 x (rest) ColMajor matrix (main.cc:37-46,119).
#pragma once

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace rtamd {

// `os << matrix` for data ColMajor rows x cols (no trailing newline).  Under the stream's
// default flags `os << double` is printf's "%.*g" at the stream's precision (libstdc++
// num_put), so each coefficient is formatted once into one buffer, the widest sets the column
// width, and the rows go out in one write: ~30x faster than a stringstream per coefficient
// (llnl_slab_test's eight files 10.7 ms -> 0.3 ms, profiles/r06_cold_start.json), the same bytes
// (tests/test_cli.py).  Other flags take the stream path.
inline void write_eigen_text(std::ostream &os, const double *data, size_t rows, size_t cols) {
  const size_t n = rows * cols;
  if (os.flags() != (std::ios_base::dec | std::ios_base::skipws) || os.precision() > 17) {
    size_t width = 0;
    for (size_t k = 0; k < n; ++k) {
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
    return;
  }
  const int prec = static_cast<int>(os.precision());
  std::vector<char> txt(n * 32);
  std::vector<unsigned char> len(n);
  size_t width = 0;
  for (size_t k = 0; k < n; ++k) {  // ColMajor order, as stored
    const int w = std::snprintf(txt.data() + 32 * k, 32, "%.*g", prec, data[k]);
    len[k] = static_cast<unsigned char>(w);
    width = std::max(width, static_cast<size_t>(w));
  }
  std::string out;
  out.reserve(rows * cols * (width + 1) + rows);
  for (size_t i = 0; i < rows; ++i) {
    if (i) out += '\n';
    for (size_t j = 0; j < cols; ++j) {
      const size_t k = i + rows * j;
      if (j) out += ' ';
      out.append(width - len[k], ' ');
      out.append(txt.data() + 32 * k, len[k]);
    }
  }
  os.write(out.data(), static_cast<std::streamsize>(out.size()));
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
