// transfer -- the reference's CLI (src/main.cc:60-136) on the MI355X solver.
//   transfer [file.prm]
// Writes phi.csv phi_plus.csv psi.csv x.csv F.csv e_ave.csv left_ends.csv
// right_ends.csv to the working directory in Eigen's default text format.
// Group tables are read from "../prm/" relative to the working directory, as
// in the reference (RT_TABLE_DIR overrides).  With no argument the default
// file is $TRANSFER_DIR/prm/default.prm (TRANSFER_DIR as in
// config/var-config.h.in; default: <repo>/tests/golden/).
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "eigen_text.hpp"
#include "prm.hpp"
#include "solver.hpp"
#include "transfer_dir.hpp"

int main(int argc, char **argv) {
  std::string filename;
  if (argc == 2) {
    filename = argv[1];
  } else if (argc == 1) {
    filename = rtamd::transfer_dir() + "prm/default.prm";
  } else {
    std::cerr << "Too many command line arguments passed in.\n";
  }
  std::cout << "filename: " << filename << std::endl;
  const char *tdir = std::getenv("RT_TABLE_DIR");
  rtamd::ParameterHandler parameter_handler(filename, tdir ? tdir : "");
  std::cout << parameter_handler.load_log();  // get_parameters' own prints (ParameterHandler.cpp:165-195)
  if (parameter_handler.status() != RT_OK) {
    std::cerr << parameter_handler.error() << std::endl;
    return 1;
  }
  parameter_handler.display_input_quantities(std::cout);

  const int M = parameter_handler.get_M(), N = parameter_handler.get_N(), G = parameter_handler.get_G();
  std::vector<double> psi_mat, phi, F, x(N);
  for (int i = 0; i < N; i++) x[i] = (i + 0.5) * parameter_handler.get_dx();

  try {
    // the reference prints as it goes; RTSN_QUIET=1 keeps only the CLI's own lines
    std::ostream *log = std::getenv("RTSN_QUIET") ? nullptr : &std::cout;
    rt::Solver solver(parameter_handler, psi_mat, phi, F, 0, log);
    solver.solve();
    solver.compute_angle_integrated_intensity();
    solver.compute_radiative_flux();
    solver.compute_balance();
    std::vector<double> phi_plus;
    solver.compute_positive_angle_integrated_intensity();
    solver.get_phi_plus(phi_plus);

    rtamd::write_eigen_text("phi.csv", phi, G, N);
    rtamd::write_eigen_text("phi_plus.csv", phi_plus, G, N);
    rtamd::write_eigen_text("psi.csv", psi_mat, M, static_cast<size_t>(G) * N);
    rtamd::write_eigen_text("x.csv", x, N, 1);
    rtamd::write_eigen_text("F.csv", F, G, N);
    std::vector<double> e_ave, left_ends, right_ends;
    solver.get_e_ave(e_ave);
    rtamd::write_eigen_text("e_ave.csv", e_ave, G, 1);
    solver.compute_group_ends();
    solver.get_ends("left", left_ends);
    solver.get_ends("right", right_ends);
    rtamd::write_eigen_text("left_ends.csv", left_ends, G, 1);
    rtamd::write_eigen_text("right_ends.csv", right_ends, G, 1);
  } catch (const rt::SolverError &e) {
    std::cerr << e.what() << std::endl;
    return 2;
  }
  return 0;
}
