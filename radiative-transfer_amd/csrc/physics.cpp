// physics.cpp -- see physics.hpp.  Host code, compiled without FMA
// contraction so that the reference's expression order is the arithmetic.
#include "physics.hpp"

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <limits>
#include <mutex>
#include <thread>
#include <vector>

namespace rtamd {
namespace phys {

// Threads for host-side setup work: the process's CPU affinity (the lease's share on a
// shared machine, not hardware_concurrency), at most 8.
static int host_threads() {
  cpu_set_t set;
  int n = 1;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
  return std::max(1, std::min(n, 8));
}

// Persistent host workers for rt_create's setup loops: started on first use and kept for the
// process (a thread start costs 30-40 us, which the per-create work of a .prm-sized handle
// does not amortise); a job wakes them, the caller takes a share, and run() returns when
// every index is done.  One job at a time.
namespace {
class HostPool {
 public:
  static HostPool &get() {
    static HostPool *pool = new HostPool(host_threads() - 1);  // never destroyed: workers sleep at exit
    return *pool;
  }
  int size() const { return static_cast<int>(workers_.size()) + 1; }
  void run(int n, const std::function<void(int)> &fn) {
    // a forked child has the pool's bookkeeping but none of its threads: it works alone
    if (getpid() != pid_) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> one(job_m_);
    if (workers_.empty() || n <= 1) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(m_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      busy_ = static_cast<int>(workers_.size());
      ++gen_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  explicit HostPool(int workers) : pid_(getpid()) {
    for (int w = 0; w < workers; ++w) workers_.emplace_back([this] { loop(); });
    for (std::thread &t : workers_) t.detach();
  }
  void drain() {
    for (int i = next_.fetch_add(1); i < n_; i = next_.fetch_add(1)) (*fn_)(i);
  }
  void loop() {
    unsigned long long seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
      }
      drain();
      std::lock_guard<std::mutex> lk(m_);
      if (--busy_ == 0) done_.notify_one();
    }
  }
  const pid_t pid_;  // the process the workers run in
  std::vector<std::thread> workers_;
  std::mutex job_m_, m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)> *fn_ = nullptr;
  int n_ = 0, busy_ = 0;
  std::atomic<int> next_{0};
  unsigned long long gen_ = 0;
};
}  // namespace

int host_workers() { return HostPool::get().size(); }
void parallel_for(int n, const std::function<void(int)> &fn) { HostPool::get().run(n, fn); }

double rad_a_long() {
  return (8.0 * std::pow(kPi, 5) * std::pow(kBoltzmann, 4)) /
         (15.0 * std::pow(kPlanck, 3) * std::pow(kLight, 3));
}

void gauss_legendre(int M, double norm, double *mu, double *wt) {
  const double tol = 1.0e-12;
  const double x1 = -1.0, x2 = 1.0;
  const double xm = 0.5 * (x2 + x1), xl = 0.5 * (x2 - x1);
  const double n = static_cast<double>(M);
  for (int r = 1; r <= (M + 1) / 2; ++r) {
    double z = std::cos(kPi * (static_cast<double>(r) - 0.25) / (n + 0.5));
    double zprev, dP;
    do {
      double P = 1.0, Pm1 = 0.0;  // Legendre recursion P_j(z)
      for (int j = 1; j <= M; ++j) {
        const double dj = static_cast<double>(j);
        const double Pm2 = Pm1;
        Pm1 = P;
        P = ((2.0 * dj - 1.0) * z * Pm1 - (dj - 1.0) * Pm2) / dj;
      }
      dP = n * (z * P - Pm1) / (z * z - 1.0);
      zprev = z;
      z = zprev - P / dP;
    } while (std::fabs(z - zprev) > tol);
    mu[r - 1] = xm - xl * z;
    mu[M - r] = xm + xl * z;
    wt[r - 1] = norm * xl / ((1.0 - z * z) * dP * dP);
    wt[M - r] = wt[r - 1];
  }
}

// ---------------------------------------------------------------------------
// Planck
// ---------------------------------------------------------------------------
static bool nearly_equal(double a, double b) {  // Planck.h:84-90, 2 ulps
  const double d = std::fabs(a - b);
  return d <= DBL_EPSILON * std::fabs(a + b) * 2 || d < DBL_MIN;
}

static double planck_density(double T, double E) {  // Planck.h:96-111
  if (nearly_equal(T, 0.0)) return 0.0;
  return 2.0 * std::pow(E, 3.0) * std::pow(kPlanck, -3.0) * std::pow(kLight, -2.0) /
         (std::exp(E / (kBoltzmann * T)) - 1.0);
}

static double planck_density_dT(double T, double E) {  // Planck.h:113-125
  if (nearly_equal(T, 0.0)) return 0.0;
  return 2.0 * std::pow(kPlanck, -3.0) * std::pow(kLight, -2.0) * std::pow(kBoltzmann, -1.0) *
         std::pow(E, 4.0) * std::pow(T, -2.0) * std::exp(E / (kBoltzmann * T)) *
         std::pow(std::exp(E / (kBoltzmann * T)) - 1.0, -2.0);
}

// 12-point Gauss-Legendre on [-1, 1] in long double (Planck.cpp:231-337).
// The Newton derivative uses the loop counter after the recursion, i.e.
// order + 1 (as the reference does); the final weight normalisation to 2
// removes the constant factor this introduces.
PlanckIntegrator::PlanckIntegrator() : accuracy_(std::numeric_limits<double>::epsilon()) {
  const unsigned short order = 12;
  long double wsum = 0;
  for (unsigned short r = 0; r < (order + 1) / 2; ++r) {
    long double x = std::cos(kPi * (r + 0.75) / (order + 0.5));
    long double deriv = 0;
    for (;;) {
      long double P = 1, Pm1 = 0, Pm2;
      unsigned short j;
      for (j = 1; j <= order; ++j) {
        Pm2 = Pm1;
        Pm1 = P;
        P = ((2 * j - 1) * x * Pm1 - (j - 1) * Pm2) / (j);
      }
      deriv = j * (x * P - Pm1) / (x * x - 1);
      const long double x_old = x;
      x = x_old - P / deriv;
      if (std::fabs(x - x_old) < accuracy_) break;
    }
    node_[r] = -x;
    node_[order - 1 - r] = x;
    weight_[r] = 1 / ((1 - x * x) * deriv * deriv);
    weight_[order - 1 - r] = weight_[r];
    wsum += weight_[r] + weight_[order - 1 - r];
  }
  for (unsigned short r = 0; r < order; ++r) weight_[r] *= 2 / wsum;
}

double PlanckIntegrator::gauss(double T, double mid, double half_width, bool dT) const {
  double acc = 0.0;  // double accumulator, long double products (Planck.cpp:136-137)
  for (int r = 0; r < 12; ++r) {
    const double E = static_cast<double>(mid + half_width * node_[r]);
    const double f = dT ? planck_density_dT(T, E) : planck_density(T, E);
    acc = static_cast<double>(acc + half_width * weight_[r] * f);
  }
  return acc;
}

// Bose series of the integral from z1 to z2 (Planck.cpp:94-118, 170-193):
// the number of terms is the first n > 32 whose next term drops below the
// accuracy relative to the leading term.
int PlanckIntegrator::series_terms(double z1, bool dT) const {
  int n_terms = 32;
  double lead = dT ? std::exp(-z1) * (std::pow(z1, 4.0) + 4.0 * std::pow(z1, 3.0) + 12.0 * z1 * z1 + 24.0 * z1 + 24.0)
                   : std::exp(-z1) * (z1 * z1 * z1 + 3.0 * z1 * z1 + 6.0 * z1 + 6.0);
  lead = std::max(lead, std::numeric_limits<double>::epsilon());
  for (;;) {
    const double np1 = n_terms + 1.0;
    const double next =
        dT ? std::exp(-np1 * z1) / (1.0 - std::exp(-z1)) * std::pow(np1, -4.0) *
                 (std::pow(np1 * z1, 4.0) + 4.0 * std::pow(np1 * z1, 3.0) + 12.0 * std::pow(np1 * z1, 2.0) +
                  24.0 * np1 * z1 + 24.0) / lead
           : std::exp(-np1 * z1) / (1.0 - std::exp(-z1)) * std::pow(np1, -4.0) *
                 (std::pow(np1 * z1, 3.0) + 3.0 * std::pow(np1 * z1, 2.0) + 6.0 * np1 * z1 + 6.0) / lead;
    if (next > accuracy_)
      ++n_terms;
    else
      break;
  }
  return n_terms;
}

// Term n of the series at z, the reference's expression.  pow(n, 4.0) of an integer
// n < 2^13 is exact (n^4 < 2^53 and libm's pow errs by < 1 ulp, so it returns the
// representable exact value): the product n n n n, bitwise the same.
double PlanckIntegrator::series_term(int n, double z, bool dT) {
  const double dn = n, n4 = dn * dn * dn * dn;
  if (dT)
    return std::exp(-n * z) / n4 *
           (std::pow(n * z, 4.0) + 4.0 * std::pow(n * z, 3.0) + 12.0 * std::pow(n * z, 2.0) + 24.0 * n * z + 24.0);
  return std::exp(-n * z) / n4 * (std::pow(n * z, 3.0) + 3.0 * std::pow(n * z, 2.0) + 6.0 * n * z + 6.0);
}

// The terms 1 .. n at z from the cache c (recomputed when it holds another z, extended when
// it holds fewer).
const std::vector<double> &PlanckIntegrator::terms(Terms &c, double z, int n, bool dT) const {
  if (c.z != z) {
    c.z = z;
    c.b.assign(1, 0.0);
    c.d.assign(1, 0.0);
  }
  std::vector<double> &t = dT ? c.d : c.b;
  for (int k = static_cast<int>(t.size()); k <= n; ++k) t.push_back(series_term(k, z, dT));
  return t;
}

double PlanckIntegrator::tail_series(double z1, double z2, bool dT, Terms *c1, Terms *c2) const {
  const int n_terms = series_terms(z1, dT);
  Terms l1, l2;
  const std::vector<double> &t1 = terms(c1 ? *c1 : l1, z1, n_terms, dT);
  const std::vector<double> &t2 = terms(c2 ? *c2 : l2, z2, n_terms, dT);
  double s1 = 0.0, s2 = 0.0;
  for (int n = n_terms; n > 0; --n) {  // the reference's order: n descending
    s1 += t1[n];
    s2 += t2[n];
  }
  return s1 - s2;
}

// Planck.cpp:85-154 (B) and :161-229 (dB/dT): Gauss below z = 0.7, series above z = 0.5,
// split at 0.6.  c1 / c2: term caches of the bounds (NULL: none).
double PlanckIntegrator::integral(double T, double e_min, double e_max, bool dT, Terms *c1, Terms *c2) const {
  if (nearly_equal(T, 0.0) || nearly_equal(e_min, e_max)) return 0.0;
  const double kT = kBoltzmann * T;
  double z1 = e_min / kT;
  const double z2 = e_max / kT;
  // the series part in the reference's expression order (B: Planck.cpp:100-103, dB/dT: :176-179)
  const auto series = [&](double a, Terms *ca) {
    return dT ? 2.0 * std::pow(kBoltzmann, 4.0) * std::pow(T, 3.0) * tail_series(a, z2, true, ca, c2) /
                    (std::pow(kPlanck, 3.0) * std::pow(kLight, 2.0))
              : 2.0 * std::pow(kBoltzmann * T, 4.0) * tail_series(a, z2, false, ca, c2) /
                    (std::pow(kPlanck, 3.0) * std::pow(kLight, 2.0));
  };
  double value;
  if (z2 <= 0.7) {
    value = gauss(T, 0.5 * (e_max + e_min), 0.5 * (e_max - e_min), dT);
  } else if (z1 >= 0.5) {
    value = series(z1, c1);
  } else {
    z1 = 0.6;
    const double lo = gauss(T, 0.5 * (z1 * kBoltzmann * T + e_min), 0.5 * (z1 * kBoltzmann * T - e_min), dT);
    value = lo + series(z1, nullptr);
  }
  return value * 4.0 * kPi;
}

double PlanckIntegrator::integral_B(double T, double e_min, double e_max) const {
  return integral(T, e_min, e_max, false, nullptr, nullptr);
}

double PlanckIntegrator::integral_dBdT(double T, double e_min, double e_max) const {
  return integral(T, e_min, e_max, true, nullptr, nullptr);
}

// The G - 1 integral pairs are independent; only the remainder group's running
// subtraction is ordered.  With many groups they are evaluated on host threads (each
// group's arithmetic unchanged, so the table is bitwise the serial one): the Bose series
// takes >= 32 terms of exp / pow per bound, ~9 us per group on one core, which was most of
// llnl_slab_test's rt_create (124 groups: 1.1 ms on one core of the build container).
void PlanckIntegrator::group_integrals(double T, int G, const double *e_lo, const double *e_hi, double *B,
                                       double *dBdT) const {
  double rest_B = rad_a_long() * kLight * std::pow(T, 4.0);
  double rest_dB = 4.0 * rad_a_long() * kLight * std::pow(T, 3.0);
  const auto work = [&](int g0, int g1) {
    Terms lo, hi;  // the terms at z1 and z2 of the group; a group's z2 is the next group's z1
    for (int g = g0; g < g1; ++g) {
      B[g] = integral(T, e_lo[g], e_hi[g], false, &lo, &hi);
      dBdT[g] = integral(T, e_lo[g], e_hi[g], true, &lo, &hi);
      std::swap(lo, hi);
    }
  };
  const int n = G - 1;
  const int nt = n < 32 ? 1 : std::min(HostPool::get().size(), (n + 15) / 16);
  if (nt <= 1)
    work(0, n);
  else
    HostPool::get().run(nt, [&](int t) { work(n * t / nt, n * (t + 1) / nt); });
  for (int g = 0; g < n; ++g) {
    rest_B -= B[g];
    rest_dB -= dBdT[g];
  }
  if (rest_B > 0.0) B[G - 1] = rest_B;
  if (rest_dB > 0.0) dBdT[G - 1] = rest_dB;
}

// ---------------------------------------------------------------------------
// Group table: edges, opacities, Planck, correction coefficients
// ---------------------------------------------------------------------------
static double planck_kernel_jk(double E, double T) {  // Correction::pf (correction.cpp:11-22)
  const double denom = std::pow(kPlanck, 3) * std::pow(kLight, 2) * (std::exp(E / T) - 1.0);
  return kBoltzmannJPK * std::pow(E, 3) / denom;
}

rt_status build_group_table(const rt_params &p, GroupTable &t) {
  const int G = p.G;
  if (G <= 0) return RT_ERR_PARAM;
  t.G = G;
  t.e_edge.assign(G + 1, 0.0);
  t.e_ave.assign(G, 0.0);
  t.de_ave.assign(G, 0.0);
  if (p.group_bounds) {
    std::copy(p.group_bounds, p.group_bounds + G + 1, t.e_edge.begin());
  } else {  // solver.cpp:6-19: e_edge(0) = 0, log spacing from efirst to elast
    double ratio = std::exp((std::log(p.elast) - std::log(p.efirst)) / (G - 1.0));
    if (G == 1) ratio = 1.;
    t.e_edge[0] = 0.0;
    t.e_edge[1] = p.efirst;
    for (int g = 1; g < G; ++g) t.e_edge[g + 1] = t.e_edge[g] * ratio;
  }
  for (int g = 0; g < G; ++g) {  // solver.cpp:22-32
    t.e_ave[g] = 0.5 * (t.e_edge[g] + t.e_edge[g + 1]);
    t.de_ave[g] = t.e_edge[g + 1] - t.e_edge[g];
  }
  for (int g = 0; g + 1 <= G; ++g) {
    if (!(t.e_edge[g + 1] > t.e_edge[g])) return RT_ERR_PARAM;  // Planck.cpp:89 assert(E_max > E_min)
  }
  t.kappa.assign(G, p.kappa_grey);
  if (p.group_kappa) std::copy(p.group_kappa, p.group_kappa + G, t.kappa.begin());
  t.rho.assign(G, p.rho);

  // Planck integrals x kcon (correction.cpp:25-36)
  t.B.assign(G, 0.0);
  t.dBdT.assign(G, 0.0);
  {
    std::vector<double> lo(t.e_edge.begin(), t.e_edge.end() - 1), hi(t.e_edge.begin() + 1, t.e_edge.end());
    PlanckIntegrator planck;
    planck.group_integrals(p.T, G, lo.data(), hi.data(), t.B.data(), t.dBdT.data());
  }
  for (int g = 0; g < G; ++g) {
    t.B[g] = kBoltzmannJPK * t.B[g];
    t.dBdT[g] = kBoltzmannJPK * t.dBdT[g];
  }

  // edge opacities: linear interpolation in group-average energy (correction.cpp:125-159)
  t.kappa_edge.assign(G + 1, 0.0);
  t.kappa_edge[0] = t.kappa[0];
  for (int g = 1; g < G; ++g) {
    const double span = t.e_ave[g] - t.e_ave[g - 1];
    const double wl = (t.e_ave[g] - t.e_edge[g]) / span;
    const double wr = (t.e_edge[g] - t.e_ave[g - 1]) / span;
    t.kappa_edge[g] = t.kappa[g - 1] * wl + t.kappa[g] * wr;
  }
  t.kappa_edge[G] = t.kappa[G - 1];

  // energy differences (correction.cpp:162-277). The last entries of dEB and
  // dkapEB use edge G-1 (not G), exactly as the reference writes them.
  const double T = p.T;
  const std::vector<double> &E = t.e_edge, &KE = t.kappa_edge;
  auto EB = [&](int k) { return E[k] * planck_kernel_jk(E[k], T); };
  auto KEB = [&](int k) { return KE[k] * E[k] * planck_kernel_jk(E[k], T); };
  t.dEB.assign(G, 0.0);
  t.dsigEdE.assign(G, 0.0);
  t.dkapEB.assign(G, 0.0);
  t.dEB[0] = EB(1);
  t.dkapEB[0] = KEB(1);
  if (G > 1) {
    for (int g = 1; g < G - 1; ++g) {
      t.dEB[g] = EB(g + 1) - EB(g);
      t.dkapEB[g] = KEB(g + 1) - KEB(g);
    }
    t.dEB[G - 1] = -E[G - 1] * planck_kernel_jk(E[G - 1], T);
    t.dkapEB[G - 1] = -KE[G - 1] * E[G - 1] * planck_kernel_jk(E[G - 1], T);
  }
  t.dsigEdE[0] = KE[1] * E[1] / t.de_ave[0];
  for (int g = 1; g < G - 1; ++g) t.dsigEdE[g] = (KE[g + 1] * E[g + 1] - KE[g] * E[g]) / t.de_ave[g];
  t.dsigEdE[G - 1] = -KE[G] * E[G] / t.de_ave[G - 1];

  // correction coefficients (correction.cpp:328-340; cor1(g) at :338 is the
  // linear index of a ColMajor G x N matrix, i.e. cor1(g, 0) = dsigEdE(g))
  t.cor1.assign(G, 0.0);
  t.cor2.assign(G, 0.0);
  t.cor3.assign(G, 0.0);
  for (int g = 0; g < G; ++g) {
    t.cor1[g] = t.dsigEdE[g];
    t.cor2[g] = 3.0 * t.rho[g] * t.kappa[g] * t.B[g] - t.dkapEB[g];
    t.cor3[g] = t.cor1[g] * (4.0 * t.B[g] - t.dEB[g]);
  }
  return RT_OK;
}

bool validate_correction(const rt_params &p, const GroupTable &t) {
  const double ac = kRadA * kLight;
  double bsum = 0., dbsum = 0., emis = 0.;
  for (int g = 0; g < t.G; ++g) {
    bsum += t.B[g];
    dbsum += t.dBdT[g];
  }
  const double acT4 = ac * std::pow(p.T, 4), dacT4 = 4.0 * ac * std::pow(p.T, 3);
  if (std::fabs(acT4 - bsum) > kValidationTol || std::fabs(dacT4 - dbsum) > kValidationTol) return false;
  for (int g = 0; g < t.G; ++g) emis += t.kappa[g] * t.B[g];
  return std::fabs(emis - p.kappa_grey * acT4) <= kValidationTol;
}

void solver_psi_source(const rt_params &p, const GroupTable &t, const double *mu, std::vector<double> &out) {
  const int M = p.M, G = p.G;
  out.assign(static_cast<size_t>(M) * G, 0.0);
  if ((p.bc_left_indicator == 1 || p.bc_right_indicator == 1) && p.psi_source)
    std::copy(p.psi_source, p.psi_source + static_cast<size_t>(M) * G, out.begin());
  if (p.use_mg_equilib) {
    for (int i = 0; i < M; ++i)
      for (int g = 0; g < G; ++g) {
        double v = 4 * t.B[g] - t.dEB[g];
        v *= mu[i] * p.V / kLight;
        v += t.B[g];
        out[static_cast<size_t>(i) * G + g] = v;
      }
  }
}

}  // namespace phys
}  // namespace rtamd
