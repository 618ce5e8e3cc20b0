// solver.cpp -- see solver.hpp.
#include "solver.hpp"

namespace rt {

void Solver::check(rt_status st, const char *what) const {
  if (st != RT_OK)
    throw SolverError(st, std::string(what) + ": " + rt_status_string(st) + " (" + rt_last_error(h_) + ")");
}

Solver::Solver(rtamd::ParameterHandler &parameter_handler, std::vector<double> &psi_mat, std::vector<double> &phi,
               std::vector<double> &F, int device)
    : ph_(parameter_handler), psi_(psi_mat), phi_(phi), F_(F) {
  if (ph_.status() != RT_OK) throw SolverError(ph_.status(), "ParameterHandler: " + ph_.error());
  M_ = ph_.get_M();
  G_ = ph_.get_G();
  N_ = ph_.get_N();
  const rt_params p = ph_.as_params();
  check(rt_create_from_params(&p, 0, 0, device, &h_), "rt_create_from_params");
  psi_.assign(static_cast<size_t>(M_) * G_ * N_, 0.0);
  phi_.assign(static_cast<size_t>(G_) * N_, 0.0);
  F_.assign(static_cast<size_t>(G_) * N_, 0.0);
  refresh_psi();  // psi = B_g (solver.cpp:165-181)
}

Solver::~Solver() { rt_destroy(h_); }

void Solver::refresh_psi() { check(rt_get_psi(h_, psi_.data()), "rt_get_psi"); }

void Solver::solve() {
  check(rt_solve(h_), "rt_solve");
  refresh_psi();
}

void Solver::compute_angle_integrated_intensity() {
  check(rt_get_moments(h_, phi_.data(), nullptr, nullptr), "rt_get_moments");
}

void Solver::compute_positive_angle_integrated_intensity() {
  phi_plus_.assign(static_cast<size_t>(G_) * N_, 0.0);
  check(rt_get_moments(h_, nullptr, nullptr, phi_plus_.data()), "rt_get_moments");
}

void Solver::compute_radiative_flux() { check(rt_get_moments(h_, nullptr, F_.data(), nullptr), "rt_get_moments"); }

void Solver::compute_balance() {
  balance_.assign(G_, 0.0);
  check(rt_get_balance(h_, balance_.data()), "rt_get_balance");
}

void Solver::compute_group_ends() {
  left_ends_.assign(G_, 0.0);
  right_ends_.assign(G_, 0.0);
  check(rt_get_group_ends(h_, left_ends_.data(), right_ends_.data()), "rt_get_group_ends");
}

void Solver::get_e_ave(std::vector<double> &e_ave) const {
  e_ave.assign(G_, 0.0);
  check(rt_get_e_ave(h_, e_ave.data()), "rt_get_e_ave");
}

void Solver::get_ends(const std::string &side, std::vector<double> &group_ends) const {
  if (side != "left" && side != "right") throw SolverError(RT_ERR_ARG, "Invalid option for 'side'.");
  group_ends = side == "left" ? left_ends_ : right_ends_;
}

}  // namespace rt
