// solver_rtsn.cpp -- drop-in replacement of Helblindi/radiative-transfer's src/solver.cpp over
// librtsn (include/rtsn.h).  It implements the reference's rt::Solver exactly as its header
// declares it (include/solver.h:79-97, UNMODIFIED): the reference's main.cc, ParameterHandler
// and .prm files stay as they are; correction.cpp, GLQuad.cpp and Planck.cpp are no longer
// linked (the library computes the group table, quadrature and Planck integrals itself).
//
// The header declares no member for the device handle and no destructor, so the handle of
// each Solver object lives in a process-wide table keyed by the object and is released with
// the table at exit (main.cc builds one Solver).  Results go straight into the caller's
// storage: psi_mat (M, G, N), phi / F (G, N) are the ABI's ColMajor layouts.
//
// Build (src/CMakeLists.txt):
//   add_library(rtsn SHARED IMPORTED)
//   set_target_properties(rtsn PROPERTIES IMPORTED_LOCATION ${RTSN_ROOT}/radiative-transfer_amd/lib/librtsn.so
//                                         INTERFACE_INCLUDE_DIRECTORIES ${RTSN_ROOT}/include)
//   add_executable(transfer main.cc param.cpp ParameterHandler.cpp solver_rtsn.cpp)
//   target_link_libraries(transfer rtsn)
// Checked by tests/test_adapter.py: g++ -fsyntax-only against the reference's headers.
#include "solver.h"

#include <cassert>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "rtsn.h"

namespace {

struct Handles {
  std::mutex m;
  std::map<const rt::Solver *, rt_solver *> of;
  ~Handles() {
    for (auto &kv : of) rt_destroy(kv.second);
  }
};

Handles &handles() {
  static Handles h;
  return h;
}

rt_solver *handle(const rt::Solver *s) {
  Handles &H = handles();
  std::lock_guard<std::mutex> lk(H.m);
  auto it = H.of.find(s);
  if (it == H.of.end()) throw std::runtime_error("rt::Solver: no librtsn handle");
  return it->second;
}

// Where the reference asserts or exit(1)s, the library returns a status: surface it as the
// reference's failure would be (an exception the caller's main does not catch).
void ok(rt_status st, rt_solver *h, const char *what) {
  if (st != RT_OK) throw std::runtime_error(std::string(what) + ": " + rt_last_error(h));
}

}  // namespace

namespace rt {

// solver.cpp:46-188: the configuration from the ParameterHandler, psi = B_g
Solver::Solver(ParameterHandler &parameter_handler, Eigen::Tensor<double, 3> &psi_mat,
               Eigen::Ref<Eigen::MatrixXd> phi, Eigen::Ref<Eigen::MatrixXd> F)
    : ph(parameter_handler), psi_mat_ref(psi_mat), phi_ref(phi), F_ref(F) {
  M = ph.get_M();
  N = ph.get_N();
  num_groups = ph.get_G();
  dx = ph.get_dx();
  dt = ph.get_dt();
  efirst = ph.get_efirst();
  elast = ph.get_elast();
  const int G = num_groups;
  psi_source.resize(M, G);
  ph.get_psi_source(psi_source);  // (m, g) -> the ABI's m * G + g
  std::vector<double> psrc(static_cast<size_t>(M) * G);
  for (int m = 0; m < M; ++m)
    for (int g = 0; g < G; ++g) psrc[static_cast<size_t>(m) * G + g] = psi_source(m, g);
  Eigen::VectorXd bounds(G + 1), kappa(G);
  rt_params p;
  rt_params_default(&p);
  p.M = M;
  p.G = G;
  p.N = N;
  p.efirst = efirst;
  p.elast = elast;
  p.X = ph.get_X();
  p.bc_left_indicator = ph.get_bc_left_indicator();
  p.bc_right_indicator = ph.get_bc_right_indicator();
  p.use_mg_equilib = ph.get_use_mg_equilib();
  p.rho = ph.get_rho();
  p.kappa_grey = ph.get_kappa_grey();
  p.T = ph.get_T();
  p.V = ph.get_V();
  p.use_correction = ph.get_use_correction();
  p.ts_method = ph.get_ts_method();
  p.dt = dt;
  p.max_timesteps = ph.get_max_timesteps();
  p.include_validation = ph.get_validation();
  p.psi_source = psrc.data();
  if (ph.get_have_group_bounds()) {
    ph.get_group_bounds(bounds);
    p.group_bounds = bounds.data();
  }
  if (ph.get_have_group_absorption_opacities()) {
    ph.get_group_kappa(kappa);
    p.group_kappa = kappa.data();
  }
  rt_solver *h = nullptr;
  ok(rt_create_from_params(&p, 0, 0, /*device=*/0, &h), nullptr, "rt_create_from_params");
  {
    Handles &H = handles();
    std::lock_guard<std::mutex> lk(H.m);
    H.of[this] = h;
  }
  e_edge.resize(G + 1);
  e_ave.resize(G);
  de_ave.resize(G);
  energy_discretization.resize(G, 2);
  generate_group_edges();
  generate_group_averages();
  fill_energy_bound_arrays();
  ok(rt_get_psi(h, psi_mat_ref.data()), h, "rt_get_psi");  // psi = B_g (solver.cpp:165-181)
}

// solver.cpp:6-43: the group grid is the library's (log grid or the .prm's bounds table)
void Solver::generate_group_edges() {
  ok(rt_get_group_data(handle(this), e_edge.data(), nullptr, nullptr, nullptr), handle(this), "rt_get_group_data");
}

void Solver::generate_group_averages() {
  ok(rt_get_e_ave(handle(this), e_ave.data()), handle(this), "rt_get_e_ave");
  for (int g = 0; g < num_groups; g++) de_ave(g) = e_edge(g + 1) - e_edge(g);
}

void Solver::fill_energy_bound_arrays() {
  for (int g = 0; g < num_groups; g++) {
    energy_discretization(g, 0) = e_edge(g);
    energy_discretization(g, 1) = e_edge(g + 1);
  }
}

// solver.cpp:590-823: max_timesteps full steps (BDF2: four substeps each) on the device
void Solver::solve() {
  rt_solver *h = handle(this);
  ok(rt_solve(h), h, "rt_solve");  // RT_ERR_VALIDATION where assert(validate_correction()) fired
  ok(rt_get_psi(h, psi_mat_ref.data()), h, "rt_get_psi");
}

// solver.cpp:191-237 (the caller's MatrixXd(G, N) is contiguous; a strided block goes through
// a temporary)
void Solver::compute_angle_integrated_intensity() {
  rt_solver *h = handle(this);
  if (phi_ref.outerStride() == num_groups) {
    ok(rt_get_moments(h, phi_ref.data(), nullptr, nullptr), h, "rt_get_moments");
  } else {
    Eigen::MatrixXd tmp(num_groups, N);
    ok(rt_get_moments(h, tmp.data(), nullptr, nullptr), h, "rt_get_moments");
    phi_ref = tmp;
  }
}

void Solver::compute_radiative_flux() {
  rt_solver *h = handle(this);
  if (F_ref.outerStride() == num_groups) {
    ok(rt_get_moments(h, nullptr, F_ref.data(), nullptr), h, "rt_get_moments");
  } else {
    Eigen::MatrixXd tmp(num_groups, N);
    ok(rt_get_moments(h, nullptr, tmp.data(), nullptr), h, "rt_get_moments");
    F_ref = tmp;
  }
}

void Solver::compute_positive_angle_integrated_intensity() {
  rt_solver *h = handle(this);
  phi_plus.resize(num_groups, N);
  ok(rt_get_moments(h, nullptr, nullptr, phi_plus.data()), h, "rt_get_moments");
}

// solver.cpp:240-284
void Solver::compute_balance() {
  rt_solver *h = handle(this);
  balance.resize(num_groups);
  ok(rt_get_balance(h, balance.data()), h, "rt_get_balance");
}

// solver.cpp:826-850
void Solver::compute_group_ends() {
  rt_solver *h = handle(this);
  left_ends.resize(num_groups);
  right_ends.resize(num_groups);
  ok(rt_get_group_ends(h, left_ends.data(), right_ends.data()), h, "rt_get_group_ends");
}

// solver.cpp:853-864
void Solver::get_ends(const string side, Eigen::Ref<Eigen::VectorXd> group_ends) {
  assert((side == "left" || side == "right") && "Invalid option for 'side'.");
  if (side == "left")
    group_ends = left_ends;
  else
    group_ends = right_ends;
}

}  // namespace rt
