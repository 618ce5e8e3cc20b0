// prm.cpp -- see prm.hpp.
#include "prm.hpp"

#include "eigen_text.hpp"

#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>

namespace rtamd {

KeyValueFile::KeyValueFile(const std::string &path) {
  std::ifstream in(path);
  if (!in) {
    std::cerr << "Could not open file " << path << std::endl;  // param.h:55
    return;
  }
  opened_ = true;
  std::string line;
  while (std::getline(in, line)) {
    if (!line.empty() && line.front() == '#') continue;
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    kv_.emplace(line.substr(0, eq), line.substr(eq + 1));  // emplace keeps the first key
  }
}

// std::stoi (param.cpp:30): strtol base 10; throws invalid_argument when nothing
// converts and out_of_range on ERANGE or a value outside int -- a parse error here
int KeyValueFile::get_int(const std::string &key, int fallback) {
  auto it = kv_.find(key);
  if (it == kv_.end()) return fallback;
  const char *s = it->second.c_str();
  char *end = nullptr;
  errno = 0;
  const long v = std::strtol(s, &end, 10);
  if (end == s || errno == ERANGE || v > 2147483647L || v < -2147483647L - 1) {
    status_ = RT_ERR_PARSE;
    return fallback;
  }
  return static_cast<int>(v);
}

// std::stod (param.cpp:44): strtod; invalid_argument when nothing converts,
// out_of_range on ERANGE (overflow, and underflow to a subnormal or zero)
double KeyValueFile::get_double(const std::string &key, double fallback) {
  auto it = kv_.find(key);
  if (it == kv_.end()) return fallback;
  const char *s = it->second.c_str();
  char *end = nullptr;
  errno = 0;
  const double v = std::strtod(s, &end);
  if (end == s || errno == ERANGE) {
    status_ = RT_ERR_PARSE;
    return fallback;
  }
  return v;
}

bool KeyValueFile::get_bool(const std::string &key, bool fallback) const {
  auto it = kv_.find(key);
  if (it == kv_.end()) return fallback;
  const std::string &v = it->second;
  return v == "yes" || v == "Yes" || v == "true" || v == "True";
}

std::string KeyValueFile::get_string(const std::string &key, const std::string &fallback) const {
  auto it = kv_.find(key);
  return it == kv_.end() ? fallback : it->second;
}

// `while (is >> d)` over text (ParameterHandler.cpp:122-128 psi_source, :152 and
// :184 tables), as libstdc++'s num_get<char> in the C locale does it: skip
// whitespace; take [+-], digits with at most one '.', then 'e'/'E' (only after a
// digit) with an optional sign and digits; the token must convert in full
// (strtod) and not overflow, else the extraction fails and the loop ends.  So
// "inf", "nan", "0x..", "1e" stop it, "0x10" yields 0, "1.2.3" yields 1.2, 0.3,
// and an underflow yields the subnormal / zero.
std::vector<double> stream_doubles(const std::string &text) {
  std::vector<double> out;
  const char *p = text.c_str();
  std::string tok;
  for (;;) {
    while (*p && std::isspace(static_cast<unsigned char>(*p))) ++p;
    tok.clear();
    if (*p == '+' || *p == '-') tok += *p++;
    bool mant = false, dec = false, sci = false;
    for (;; ++p) {
      const char c = *p;
      if (c >= '0' && c <= '9') {
        tok += c;
        mant = true;
      } else if (c == '.' && !dec && !sci) {
        tok += c;
        dec = true;
      } else if ((c == 'e' || c == 'E') && !sci && mant) {
        tok += 'e';
        sci = true;
        if (p[1] == '+' || p[1] == '-') tok += *++p;
      } else {
        break;
      }
    }
    if (tok.empty()) break;
    char *end = nullptr;
    const double v = std::strtod(tok.c_str(), &end);
    if (end == tok.c_str() || *end != '\0' || std::isinf(v)) break;
    out.push_back(v);
  }
  return out;
}

void ParameterHandler::fail(rt_status st, const std::string &msg) {
  if (status_ == RT_OK) {
    status_ = st;
    error_ = msg;
  }
}

int ParameterHandler::read_table(const std::string &path, size_t expect, std::vector<double> &out) {
  std::ifstream in(path);
  if (!in) {
    fail(RT_ERR_IO, "could not open table " + path);
    return 1;
  }
  std::stringstream ss;
  ss << in.rdbuf();
  out = stream_doubles(ss.str());
  if (out.size() != expect) {
    fail(RT_ERR_PARAM, "table " + path + " holds " + std::to_string(out.size()) + " values, expected " +
                           std::to_string(expect));
    return 2;
  }
  return 0;
}

// ParameterHandler::get_parameters (ParameterHandler.cpp:100-212)
ParameterHandler::ParameterHandler(const std::string &filename, const std::string &table_dir) {
  KeyValueFile kv(filename);
  prm_found_ = kv.opened();
  if (!prm_found_) std::cerr << "Error in reading file.\n" << std::endl;  // :13-15, continues
  M_ = kv.get_int("M", 2);
  G_ = kv.get_int("G", 1);
  efirst_ = kv.get_double("efirst", .1);
  elast_ = kv.get_double("elast", 10.);
  X_ = kv.get_double("X", 1.);
  N_ = kv.get_int("N", 100);
  dx_ = X_ / N_;
  bc_left_ = kv.get_int("bc_left_indicator", 2);
  bc_right_ = kv.get_int("bc_right_indicator", 1);
  use_mg_equilib_ = kv.get_bool("use_mg_equilib", false);
  if (kv.status() != RT_OK) fail(kv.status(), "a numeric .prm value has no numeric prefix");
  if (M_ <= 0 || G_ <= 0 || N_ <= 0) {
    fail(RT_ERR_PARAM, "M, G and N must be positive");
    return;
  }

  psi_source_.assign(static_cast<size_t>(M_) * G_, 0.0);
  if (!use_mg_equilib_) {
    const std::vector<double> v = stream_doubles(kv.get_string("psi_source", "no_sources_provided"));
    if (v.size() > psi_source_.size()) {
      fail(RT_ERR_PARAM, "psi_source holds more than M*G values");
    } else {
      for (size_t k = 0; k < v.size(); ++k) psi_source_[(k / G_) * G_ + (k % G_)] = v[k];
    }
  }

  const std::string dir = table_dir.empty() ? std::string("../prm/") : table_dir;
  have_group_bounds_ = kv.get_bool("have_group_bounds", false);
  if (have_group_bounds_) {
    filename_group_bounds_ = dir + kv.get_string("filename_group_bounds", "NA");
    if (read_table(filename_group_bounds_, static_cast<size_t>(G_) + 1, group_bounds_) == 0)  // after :162's assert
      load_log_ += "specified group bounds: " + filename_group_bounds_ + "\n";
  }
  have_group_kappa_ = kv.get_bool("have_group_absorption_opacities", false);
  if (have_group_kappa_) {
    filename_group_kappa_ = dir + kv.get_string("filename_group_kappa", "NA");
    const int r = read_table(filename_group_kappa_, static_cast<size_t>(G_), group_kappa_);
    if (r != 1) load_log_ += "group_kappa size: " + std::to_string(G_) + "\n";  // :191, before the assert
    if (r == 0) load_log_ += "specified group opacities filename: " + filename_group_kappa_ + "\n";
  }
  rho_ = kv.get_double("rho", 1.);
  kappa_grey_ = kv.get_double("kappa_grey", 1.);
  T_ = kv.get_double("T", 1.);
  V_ = kv.get_double("V", 0.);
  use_correction_ = kv.get_bool("use_correction", false);
  ts_method_ = kv.get_int("ts_method", 3);
  dt_ = kv.get_double("dt", 0.00001);
  max_timesteps_ = kv.get_int("max_timesteps", 1000);
  include_validation_ = kv.get_bool("include_validation", true);
  if (kv.status() != RT_OK) fail(kv.status(), "a numeric .prm value has no numeric prefix");
}

static const char *bc_name(int bc) {
  switch (bc) {
    case 0: return "vacuum";
    case 1: return "source";
    case 2: return "reflective";
    default: return nullptr;
  }
}

void ParameterHandler::display_input_quantities(std::ostream &os) const {
  os << "\n--- Input Parameters ---\n";
  os << "Angle quadrature order: " << M_ << "\n";
  os << "Number of energy groups: " << G_ << "\n";
  if (have_group_bounds_)
    os << "Group bounds (keV) specified in file: " << filename_group_bounds_ << "\n";
  else
    os << "Group bounds (keV) will be computed logarithmically, with first group edge at " << efirst_
       << " and last group edge at " << elast_ << "\n";
  os << "Slab thickness (cm): " << X_ << "\n";
  os << "Number of cells: " << N_ << "\n";
  os << "Material density (g/cm^3): " << rho_ << "\n";
  if (have_group_kappa_)
    os << "Group opacities (cm^2/g) specified in file: " << filename_group_kappa_ << "\n";
  else
    os << "Group opacities will be set to the constant grey opacity (cm^2/g): " << kappa_grey_ << "\n";
  os << "Material temperature (keV): " << T_ << "\n";
  os << "Material velocity (cm/shake): " << V_ << "\n";
  os << "Beta: " << V_ / 299.79245800 << "\n";
  const char *r = bc_name(bc_right_), *l = bc_name(bc_left_);
  os << "Right boundary condition: " << (r ? r : "Incorrect boundary conditions provided.") << "\n";
  if (!r) return;
  os << "Left boundary condition: " << (l ? l : "Incorrect boundary conditions provided.") << "\n\n";
  if (!l) return;
  os << "Psi_source: \n";  // `cout << psi_source << endl`: an Eigen MatrixXd (M, G)
  std::vector<double> colmajor(psi_source_.size());
  for (int m = 0; m < M_; ++m)
    for (int g = 0; g < G_; ++g) colmajor[m + static_cast<size_t>(M_) * g] = psi_source_[static_cast<size_t>(m) * G_ + g];
  write_eigen_text(os, colmajor.data(), M_, G_);
  os << std::endl;
}

rt_params ParameterHandler::as_params() const {
  rt_params p{};
  p.M = M_;
  p.G = G_;
  p.N = N_;
  p.efirst = efirst_;
  p.elast = elast_;
  p.X = X_;
  p.bc_left_indicator = bc_left_;
  p.bc_right_indicator = bc_right_;
  p.use_mg_equilib = use_mg_equilib_;
  p.rho = rho_;
  p.kappa_grey = kappa_grey_;
  p.T = T_;
  p.V = V_;
  p.use_correction = use_correction_;
  p.ts_method = ts_method_;
  p.dt = dt_;
  p.max_timesteps = max_timesteps_;
  p.include_validation = include_validation_;
  p.psi_source = psi_source_.empty() ? nullptr : psi_source_.data();
  p.group_bounds = have_group_bounds_ ? group_bounds_.data() : nullptr;
  p.group_kappa = have_group_kappa_ ? group_kappa_.data() : nullptr;
  return p;
}

}  // namespace rtamd
