// prm.hpp -- the reference's .prm input surface, re-implemented.
//
// ParameterHandler (include/ParameterHandler.h:11-99, src/ParameterHandler.cpp)
// over a key=value reader with the semantics of the vendored kaityo256/param
// (include/param.h:62-75, src/param.cpp:4-66):
//   * a line is a comment only when its column 0 is '#';
//   * key = the exact text before the first '=', value = the rest;
//   * the first occurrence of a key wins (std::map::insert);
//   * int/double parse a numeric prefix (std::stoi/std::stod), so trailing
//     "# comments" are ignored; a value with no numeric prefix is an error;
//   * bool is true only for the exact strings yes/Yes/true/True.
#pragma once

#include <map>
#include <ostream>
#include <string>
#include <vector>

#include "../../include/rtsn.h"

namespace rtamd {

class KeyValueFile {
 public:
  explicit KeyValueFile(const std::string &path);
  bool opened() const { return opened_; }
  bool has(const std::string &key) const { return kv_.count(key) != 0; }
  int get_int(const std::string &key, int fallback);
  double get_double(const std::string &key, double fallback);
  bool get_bool(const std::string &key, bool fallback) const;
  std::string get_string(const std::string &key, const std::string &fallback) const;
  rt_status status() const { return status_; }

 private:
  std::map<std::string, std::string> kv_;
  bool opened_ = false;
  rt_status status_ = RT_OK;
};

// The numbers `while (stream >> d)` extracts from a text under libstdc++'s
// num_get (ParameterHandler.cpp:126,152,184): see prm.cpp.
std::vector<double> stream_doubles(const std::string &text);

class ParameterHandler {
 public:
  // table_dir "" means the reference's "../prm/" relative to the CWD.
  explicit ParameterHandler(const std::string &filename, const std::string &table_dir = "");

  rt_status status() const { return status_; }
  const std::string &error() const { return error_; }
  bool prm_found() const { return prm_found_; }

  // getters of include/ParameterHandler.h:73-98
  int get_M() const { return M_; }
  int get_G() const { return G_; }
  double get_efirst() const { return efirst_; }
  double get_elast() const { return elast_; }
  bool get_have_group_bounds() const { return have_group_bounds_; }
  double get_kappa_grey() const { return kappa_grey_; }
  double get_X() const { return X_; }
  int get_N() const { return N_; }
  double get_dx() const { return dx_; }
  int get_bc_left_indicator() const { return bc_left_; }
  int get_bc_right_indicator() const { return bc_right_; }
  bool get_use_mg_equilib() const { return use_mg_equilib_; }
  double get_rho() const { return rho_; }
  bool get_have_group_absorption_opacities() const { return have_group_kappa_; }
  double get_T() const { return T_; }
  double get_V() const { return V_; }
  bool get_use_correction() const { return use_correction_; }
  int get_ts_method() const { return ts_method_; }
  double get_dt() const { return dt_; }
  int get_max_timesteps() const { return max_timesteps_; }
  bool get_validation() const { return include_validation_; }
  const std::vector<double> &psi_source() const { return psi_source_; }   // M*G, m*G+g
  const std::vector<double> &group_bounds() const { return group_bounds_; }
  const std::vector<double> &group_kappa() const { return group_kappa_; }

  // ParameterHandler::display_input_quantities (ParameterHandler.cpp:20-96)
  void display_input_quantities(std::ostream &os) const;
  // what get_parameters itself prints while reading the tables (ParameterHandler.cpp:165,
  // 191, 195): "specified group bounds: ...", "group_kappa size: G", "specified group
  // opacities filename: ..." -- kept here for the CLI to print, never by the library
  const std::string &load_log() const { return load_log_; }

  // Borrowed view for rt_create_from_params (valid while *this lives).
  rt_params as_params() const;

 private:
  void fail(rt_status st, const std::string &msg);
  // 0: read, 1: could not open, 2: opened but holds another count
  int read_table(const std::string &path, size_t expect, std::vector<double> &out);

  rt_status status_ = RT_OK;
  std::string error_;
  std::string load_log_;
  bool prm_found_ = false;
  int M_ = 2, G_ = 1, N_ = 100;
  double efirst_ = .1, elast_ = 10., X_ = 1., dx_ = .01;
  int bc_left_ = 2, bc_right_ = 1;
  bool use_mg_equilib_ = false;
  bool have_group_bounds_ = false, have_group_kappa_ = false;
  std::string filename_group_bounds_, filename_group_kappa_;
  double rho_ = 1., kappa_grey_ = 1., T_ = 1., V_ = 0.;
  bool use_correction_ = false;
  int ts_method_ = 3;
  double dt_ = 0.00001;
  int max_timesteps_ = 1000;
  bool include_validation_ = true;
  std::vector<double> psi_source_, group_bounds_, group_kappa_;
};

}  // namespace rtamd
