// physics.hpp -- per-run host constants of the S_n path.
//
// Everything here is O(G) or O(M) work that the reference recomputes on the
// host (T is a constant scalar, solver.cpp:157, so every quantity is the same
// in every substep).  It is evaluated once, on the host, in the reference's
// own arithmetic -- including the 80-bit long double Gauss-Legendre nodes of
// Planck.cpp:231-337 -- so the group emission B_g matches the reference
// bit for bit on the same machine.  The O(M G N) work happens on the GPU.
#pragma once

#include <functional>
#include <vector>

#include "../../include/rtsn.h"

namespace rtamd {
namespace phys {

// include/Constants.h:9-23
constexpr double kPlanck = 4.141895e-10;      // keV-sh
constexpr double kBoltzmann = 1.0;            // keV/keV
constexpr double kBoltzmannJPK = 1.601558e-25;  // jk/keV
constexpr double kLight = 299.79245800;       // cm/sh
constexpr double kPi = 3.1415926546;          // not M_PI
constexpr double kFourPi = 4.0 * kPi;
constexpr double kRadA = 1.3653104e-2;        // jk/(cm^3-keV^4)
constexpr double kValidationTol = 1.E-6;
double rad_a_long();                          // Constants.h:22-23

// Host setup loops on the process's persistent workers (physics.cpp): fn(i) for i in [0, n),
// the caller taking a share; host_workers() threads in all (the caller included).
int host_workers();
void parallel_for(int n, const std::function<void(int)> &fn);

// GLQuad::build (GLQuad.cpp:4-44): mu ascending, weights scaled to `norm`.
void gauss_legendre(int M, double norm, double *mu, double *wt);

// Planck group integrals (Planck.cpp:44-337).
class PlanckIntegrator {
 public:
  PlanckIntegrator();
  // Planck::get_Planck: groups [edge[g], edge[g+1]]; the last group receives
  // the remainder of the grey total only when it is positive -- otherwise B /
  // dBdT keep whatever the caller stored (Planck.cpp:73-76).
  void group_integrals(double T, int G, const double *e_lo, const double *e_hi, double *B, double *dBdT) const;
  double integral_B(double T, double e_min, double e_max) const;
  double integral_dBdT(double T, double e_min, double e_max) const;
  // the Gauss-Legendre nodes and weights rounded to double (device copy)
  void nodes(double *x, double *w) const {
    for (int r = 0; r < 12; ++r) {
      x[r] = static_cast<double>(node_[r]);
      w[r] = static_cast<double>(weight_[r]);
    }
  }

 private:
  // Bose-series terms f(n, z), n = 1 .. size - 1, of one bound z (B and dB/dT), kept so that
  // adjacent groups, whose shared edge is one group's z2 and the next one's z1, evaluate them
  // once (group_integrals)
  struct Terms {
    double z = -1.0;
    std::vector<double> b, d;
  };
  double gauss(double T, double mid, double half_width, bool dBdT) const;
  int series_terms(double z1, bool dBdT) const;
  static double series_term(int n, double z, bool dBdT);
  const std::vector<double> &terms(Terms &c, double z, int n, bool dBdT) const;
  double tail_series(double z1, double z2, bool dBdT, Terms *c1 = nullptr, Terms *c2 = nullptr) const;
  double integral(double T, double e_min, double e_max, bool dBdT, Terms *c1, Terms *c2) const;
  long double node_[12];
  long double weight_[12];
  double accuracy_;
};

// Per-group tables of one run (all G groups).
struct GroupTable {
  int G = 0;
  std::vector<double> e_edge, e_ave, de_ave;   // solver.cpp:6-43 (or the bounds table)
  std::vector<double> kappa, rho;              // solver.cpp:145-156
  std::vector<double> B, dBdT;                 // correction.cpp:25-36 (x kcon)
  std::vector<double> kappa_edge;              // correction.cpp:125-159
  std::vector<double> dEB, dsigEdE, dkapEB;    // correction.cpp:162-277
  std::vector<double> cor1, cor2, cor3;        // correction.cpp:328-340
};

rt_status build_group_table(const rt_params &p, GroupTable &out);
// Correction::validate_correction (correction.cpp:39-63, 100-122)
bool validate_correction(const rt_params &p, const GroupTable &t);
// Solver-owned psi_source after construction (solver.cpp:67-73; left
// uninitialised by the reference unless a BC is "source": defined 0 here)
// and, with use_mg_equilib, computeEquilibriumSources (solver.cpp:287-315).
void solver_psi_source(const rt_params &p, const GroupTable &t, const double *mu, std::vector<double> &out);

}  // namespace phys
}  // namespace rtamd
