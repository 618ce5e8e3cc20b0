// ref_param_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Drives the reference's own .prm reader -- kaityo256/param as vendored in
// Helblindi/radiative-transfer (include/param.h, src/param.cpp), compiled
// UNMODIFIED from /root/reference by oracle/Makefile into oracle/_ref/ -- through
// exactly the get<T>(key, default) calls, in the same order, that
// ParameterHandler::get_parameters makes (src/ParameterHandler.cpp:100-212).
// ParameterHandler.cpp itself needs Eigen (absent here), so the few lines of it
// that post-process values are restated below and marked as such.
//
// Output (stdout, after whatever param prints itself): one "@key<TAB>value"
// line per value, doubles as %.17g; psi_source as the values the reference's
// `stringstream >> double` loop extracts (:119-129); "@status<TAB>ok" at the
// end.  When std::stoi / std::stod throws the process terminates, as the
// reference does (no handler: the calls resolve to param.cpp's explicit
// specialisations at link time, which the compiler saw as non-throwing
// primary templates).  Used by tests/test_ref_param.py to pin
// radiative-transfer_amd/csrc/prm.cpp and oracle/rt_oracle.c's parser.
#include <cstdio>
#include <sstream>
#include <string>

#include "param.h"

static void put(const char *k, double v) { std::printf("@%s\t%.17g\n", k, v); }
static void put(const char *k, const std::string &v) { std::printf("@%s\t%s\n", k, v.c_str()); }

int main(int argc, char **argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: ref_param <file.prm>\n");
    return 2;
  }
  std::setvbuf(stdout, nullptr, _IONBF, 0);  // keep what was printed if a throw terminates
  parameter::parameter param(argv[1]);       // ParameterHandler.cpp:10
  std::printf("@found\t%d\n", static_cast<bool>(param) ? 1 : 0);
  {
    const int M = param.get<int>("M", 2);
    put("M", M);
    const int G = param.get<int>("G", 1);
    put("G", G);
    put("efirst", param.get<double>("efirst", .1));
    put("elast", param.get<double>("elast", 10.));
    put("X", param.get<double>("X", 1.));
    put("N", param.get<int>("N", 100));
    put("bc_left_indicator", param.get<int>("bc_left_indicator", 2));
    put("bc_right_indicator", param.get<int>("bc_right_indicator", 1));
    const bool eq = param.get<bool>("use_mg_equilib", false);
    put("use_mg_equilib", eq);
    if (!eq) {
      // restated from ParameterHandler.cpp:119-129 (the Eigen matrix write omitted)
      std::stringstream ss(param.get<std::string>("psi_source", "no_sources_provided"));
      double d;
      int counter = 0;
      while (ss >> d) {
        std::printf("@psi_source[%d]\t%.17g\n", counter, d);
        ++counter;
      }
      put("psi_source_count", counter);
    }
    const bool hb = param.get<bool>("have_group_bounds", false);
    put("have_group_bounds", hb);
    if (hb) put("filename_group_bounds", param.get<std::string>("filename_group_bounds", "NA"));
    const bool hk = param.get<bool>("have_group_absorption_opacities", false);
    put("have_group_absorption_opacities", hk);
    if (hk) put("filename_group_kappa", param.get<std::string>("filename_group_kappa", "NA"));
    put("rho", param.get<double>("rho", 1.));
    put("kappa_grey", param.get<double>("kappa_grey", 1.));
    put("T", param.get<double>("T", 1.));
    put("V", param.get<double>("V", 0.));
    put("use_correction", param.get<bool>("use_correction", false));
    put("ts_method", param.get<int>("ts_method", 3));
    put("dt", param.get<double>("dt", 0.00001));
    put("max_timesteps", param.get<int>("max_timesteps", 1000));
    put("include_validation", param.get<bool>("include_validation", true));
  }
  std::printf("@status\tok\n");
  return 0;
}
