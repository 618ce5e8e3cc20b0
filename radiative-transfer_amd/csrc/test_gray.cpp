// test_gray -- the reference's GrayTest (tests/test_gray.cpp:47-101) on the
// MI355X solver: $TRANSFER_DIR/prm/single_group.prm, pass iff |max_c F| < 1e-6 (the signed
// maximum, as written at :89).
#include <cmath>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "eigen_text.hpp"
#include "prm.hpp"
#include "solver.hpp"
#include "transfer_dir.hpp"

int main(int argc, char **argv) {
  const std::string filename = argc > 1 ? argv[1] : rtamd::transfer_dir() + "prm/single_group.prm";
  rtamd::ParameterHandler parameter_handler(filename);
  if (parameter_handler.status() != RT_OK) {
    std::cerr << parameter_handler.error() << std::endl;
    return 1;
  }
  const int N = parameter_handler.get_N(), G = parameter_handler.get_G();
  std::vector<double> psi_mat, phi, F, x(N);
  for (int i = 0; i < N; i++) x[i] = (i + 0.5) * parameter_handler.get_dx();
  double maxF = 0.0;
  try {
    // the reference prints as it goes; RTSN_QUIET=1 keeps only the CLI's own lines
    std::ostream *log = std::getenv("RTSN_QUIET") ? nullptr : &std::cout;
    rt::Solver solver(parameter_handler, psi_mat, phi, F, 0, log);
    solver.solve();
    solver.compute_angle_integrated_intensity();
    solver.compute_radiative_flux();
    solver.compute_balance();
    maxF = F[0];
    for (double f : F) maxF = f > maxF ? f : maxF;
  } catch (const rt::SolverError &e) {
    std::cerr << e.what() << std::endl;
    return 2;
  }
  std::cout << "max F: " << maxF << std::endl;
  rtamd::write_eigen_text("gray-test-phi.csv", phi, G, N);
  rtamd::write_eigen_text("gray-test-x.csv", x, N, 1);
  rtamd::write_eigen_text("gray-test-F.csv", F, G, N);
  if (std::fabs(maxF) < 1.E-6) {
    std::cout << "Gray test passed.\n";
    return 0;
  }
  std::cout << "Gray test failed.\n";
  return 1;
}
