// solver.cpp -- see solver.hpp.
#include "solver.hpp"

#include <cmath>
#include <cstdlib>
#include <iomanip>
#include <iostream>

#include "eigen_text.hpp"
#include "physics.hpp"

namespace rt {

void Solver::check(rt_status st, const char *what) const {
  if (st != RT_OK) {
    const char *detail = comm_ && std::string(what).rfind("rt_comm", 0) == 0 ? rt_comm_last_error(comm_) : rt_last_error(h_);
    throw SolverError(st, std::string(what) + ": " + rt_status_string(st) + " (" + detail + ")");
  }
}

Solver::Solver(rtamd::ParameterHandler &parameter_handler, std::vector<double> &psi_mat, std::vector<double> &phi,
               std::vector<double> &F, int device, std::ostream *log)
    : ph_(parameter_handler), psi_(psi_mat), phi_(phi), F_(F), log_(log) {
  create(device, Ranks{});
}

Solver::Solver(rtamd::ParameterHandler &parameter_handler, std::vector<double> &psi_mat, std::vector<double> &phi,
               std::vector<double> &F, int device, std::ostream *log, const Ranks &ranks)
    : ph_(parameter_handler), psi_(psi_mat), phi_(phi), F_(F), log_(log) {
  create(device, ranks);
}

// The rank's shard: groups [r G / n, (r + 1) G / n) -- every rank at least one
// group when G >= n -- else all groups and direction pairs [r H / n, (r + 1) H / n).
void Solver::create(int device, const Ranks &ranks) {
  if (ph_.status() != RT_OK) throw SolverError(ph_.status(), "ParameterHandler: " + ph_.error());
  M_ = ph_.get_M();
  G_ = ph_.get_G();
  N_ = ph_.get_N();
  rank_ = ranks.rank;
  const rt_params p = ph_.as_params();
  const int n = ranks.nranks, r = ranks.rank, H = M_ / 2;
  if (n <= 1) {
    check(rt_create_from_params(&p, 0, 0, device, &h_), "rt_create_from_params");
  } else {
    if (!ranks.comm_id || r < 0 || r >= n) throw SolverError(RT_ERR_ARG, "Solver: bad rank / communicator id");
    if (G_ >= n) {
      const int lo = static_cast<int>(static_cast<long long>(r) * G_ / n);
      const int hi = static_cast<int>(static_cast<long long>(r + 1) * G_ / n);
      check(rt_create_from_params(&p, lo, hi, device, &h_), "rt_create_from_params");
    } else if (H >= n) {
      check(rt_create_direction_shard(&p, 0, G_, r * H / n, (r + 1) * H / n, device, &h_), "rt_create_direction_shard");
    } else {
      throw SolverError(RT_ERR_PARAM, "Solver: more ranks than groups and than direction pairs");
    }
    check(rt_comm_init(n, r, ranks.comm_id, device, &comm_), "rt_comm_init");
  }
  if (rank_ == 0) psi_.assign(static_cast<size_t>(M_) * G_ * N_, 0.0);
  phi_.assign(static_cast<size_t>(G_) * N_, 0.0);
  F_.assign(static_cast<size_t>(G_) * N_, 0.0);
  refresh_psi();  // psi = B_g (solver.cpp:165-181)
  if (log_) print_constructor();
}

// solver.cpp:55-187 (and the Correction constructor's line, correction.cpp:301)
void Solver::print_constructor() const {
  std::ostream &os = *log_;
  os << "Solver constructor.\n";
  std::vector<double> mu(M_), wt(M_);
  check(rt_quadrature(M_, mu.data(), wt.data()), "rt_quadrature");  // all M (a direction shard holds a subset)
  os << std::setw(16) << std::left << "Mu" << std::setw(16) << std::left << "Wt" << std::endl
     << std::setw(16) << std::left << "--" << std::setw(16) << std::left << "--" << std::endl;
  for (int i = 0; i < M_; ++i)
    os << std::showpos << std::setw(16) << std::left << mu[i] << std::setw(16) << std::left << wt[i] << std::endl;
  os << std::noshowpos << std::endl;
  std::vector<double> edge(G_ + 1), B(G_), e_ave(G_);
  check(rt_get_group_data(h_, edge.data(), B.data(), nullptr, nullptr), "rt_get_group_data");
  check(rt_get_e_ave(h_, e_ave.data()), "rt_get_e_ave");
  os << std::left << std::setw(13) << "Group Index" << std::left << std::setw(16) << "Average Energy" << std::left
     << std::setw(14) << "Upper Energy" << std::left << std::setw(13) << "Group Width" << std::endl;
  os << std::left << std::setw(13) << "-----------" << std::left << std::setw(16) << "(keV)---------" << std::left
     << std::setw(14) << "(keV)-------" << std::left << std::setw(13) << "(keV)------" << std::endl;
  for (int g = 0; g < G_; ++g)
    os << std::left << std::setw(13) << g << std::left << std::setw(16) << e_ave[g] << std::left << std::setw(14)
       << edge[g + 1] << std::left << std::setw(13) << (edge[g + 1] - edge[g]) << std::endl;  // de_ave (:26-32)
  os << "\n" << std::endl;
  os << "Correction constructor.\n";
  os << "B: ";
  rtamd::write_eigen_text(os, B.data(), G_, 1);
  os << std::endl;
  os << "psi_mat_ref: ";
  rtamd::write_eigen_text(os, psi_.data(), M_, static_cast<size_t>(G_) * N_);
  os << std::endl;
  os << "end solver constructor\n";
}

// Correction::validate_correction (correction.cpp:39-63, 100-122, 366-369) with its prints
bool Solver::validation_report() const {
  std::vector<double> edge(G_ + 1), B(G_), dBdT(G_), kappa(G_);
  check(rt_get_group_data(h_, edge.data(), B.data(), dBdT.data(), kappa.data()), "rt_get_group_data");
  const double ac = rtamd::phys::kRadA * rtamd::phys::kLight, T = ph_.get_T();
  double bsum = 0., dbsum = 0.;
  for (int g = 0; g < G_; ++g) {
    bsum += B[g];
    dbsum += dBdT[g];
  }
  const double acT4 = ac * std::pow(T, 4), dacT4 = 4.0 * ac * std::pow(T, 3);
  if (std::fabs(acT4 - bsum) > rtamd::phys::kValidationTol || std::fabs(dacT4 - dbsum) > rtamd::phys::kValidationTol) {
    if (log_) {
      *log_ << "acT^4 = " << acT4 << " B sum = " << bsum << std::endl;
      *log_ << "4acT^3 = " << dacT4 << " dBdT sum = " << dbsum << "\n" << std::endl;
    }
    return false;
  }
  const double sigacT4 = ph_.get_kappa_grey() * acT4;
  double emis_tot = 0.0;
  for (int g = 0; g < G_; ++g) emis_tot += kappa[g] * B[g];
  if (std::fabs(emis_tot - sigacT4) > rtamd::phys::kValidationTol) {
    if (log_) *log_ << "Total Emission = " << emis_tot << " kappa_ref*acT^4 = " << sigacT4 << "\n" << std::endl;
    return false;
  }
  return true;
}

Solver::~Solver() {
  rt_comm_destroy(comm_);
  rt_destroy(h_);
}

void Solver::refresh_psi() {
  if (comm_)
    check(rt_comm_gather_psi(comm_, h_, 0, rank_ == 0 ? psi_.data() : nullptr), "rt_comm_gather_psi");
  else
    check(rt_get_psi(h_, psi_.data()), "rt_get_psi");
}

void Solver::moments(double *phi, double *F, double *phi_plus) {
  if (comm_)
    check(rt_comm_gather_moments(comm_, h_, phi, F, phi_plus), "rt_comm_gather_moments");
  else
    check(rt_get_moments(h_, phi, F, phi_plus), "rt_get_moments");
}

void Solver::solve() {
  if (log_ && ph_.get_validation() && (ph_.get_use_mg_equilib() || ph_.get_max_timesteps() > 0) &&
      !validation_report()) {
    // assert(validate_correction()) in computeEquilibriumSources / solve (solver.cpp:290-293, 609-612)
    log_->flush();
    std::cerr << "transfer: solver.cpp:610: void rt::Solver::solve(): Assertion `correction->validate_correction() "
                 "&& \"Invalid Correction Terms\\n\"' failed." << std::endl;
    std::abort();
  }
  check(rt_solve(h_), "rt_solve");
  refresh_psi();
  if (!log_ && !(comm_ && ph_.get_use_mg_equilib())) return;
  if (ph_.get_use_mg_equilib()) {  // computeEquilibriumSources (solver.cpp:296-312); collective with ranks
    std::vector<double> mu(M_), wt(M_), src(static_cast<size_t>(M_) * G_);
    check(rt_quadrature(M_, mu.data(), wt.data()), "rt_quadrature");
    if (comm_)
      check(rt_comm_gather_psi_source(comm_, h_, src.data()), "rt_comm_gather_psi_source");
    else
      check(rt_get_psi_source(h_, src.data()), "rt_get_psi_source");
    if (!log_) return;
    std::ostream &os = *log_;
    for (int i = 0; i < M_; ++i)
      for (int g = 0; g < G_; ++g)
        os << "source condition for mu: " << mu[i] << " and group " << g << ": " << src[static_cast<size_t>(i) * G_ + g]
           << std::endl;
  }
  std::ostream &os = *log_;
  const int ts = ph_.get_ts_method();
  const long long its = static_cast<long long>(ph_.get_max_timesteps()) * (ts == 3 ? 4 : 1);
  for (long long it = 0; it < its; ++it)  // solver.cpp:620-625
    if (ts != 3 || it % 4 == 0) os << "============= Timestep: " << it << " =============" << std::endl;
}

void Solver::compute_angle_integrated_intensity() { moments(phi_.data(), nullptr, nullptr); }

void Solver::compute_positive_angle_integrated_intensity() {
  phi_plus_.assign(static_cast<size_t>(G_) * N_, 0.0);
  moments(nullptr, nullptr, phi_plus_.data());
}

void Solver::compute_radiative_flux() { moments(nullptr, F_.data(), nullptr); }

void Solver::compute_balance() {
  balance_.assign(G_, 0.0);
  std::vector<double> sources(G_), sinks(G_);
  if (comm_)
    check(rt_comm_gather_balance(comm_, h_, balance_.data(), sources.data(), sinks.data()), "rt_comm_gather_balance");
  else
    check(rt_get_balance_terms(h_, balance_.data(), sources.data(), sinks.data()), "rt_get_balance_terms");
  if (log_)
    for (int g = 0; g < G_; ++g)  // solver.cpp:278-282
      *log_ << "sources: " << sources[g] << std::endl
            << "sinks: " << sinks[g] << std::endl
            << "balance at (" << g << "): " << balance_[g] << std::endl;
}

void Solver::compute_group_ends() {
  left_ends_.assign(G_, 0.0);
  right_ends_.assign(G_, 0.0);
  if (comm_)
    check(rt_comm_gather_group_ends(comm_, h_, left_ends_.data(), right_ends_.data()), "rt_comm_gather_group_ends");
  else
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
