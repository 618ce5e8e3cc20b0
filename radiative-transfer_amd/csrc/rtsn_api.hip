// rtsn_api.hip -- the C ABI (include/rtsn.h): solver lifecycle, device
// state, per-line setup, launches and result reductions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/rtsn.h"
#include "cell.hpp"
#include "kernels.hpp"
#include "physics.hpp"
#include "prm.hpp"

using namespace rtamd;

namespace {

thread_local std::string g_last_error;

// ---------------------------------------------------------------------------
// Handle resource cache.  A handle's lifetime allocates ~20 device buffers, two pinned
// staging buffers, a stream and events, and hipFree / hipHostFree synchronise the device:
// together ~1 ms per Solver(ph) ... ~Solver() pair on the box, more than the reference's
// own configurations take to solve (llnl_slab_test's 2 steps: 21 us).  rt_destroy (and
// the getters' temporaries) hand them to this process-wide cache -- blocks of at most
// kPoolMaxBlock, RTSN_POOL_MB in all (default 512; 0 turns the cache off), only after the
// owning stream is idle -- and the next allocation of the same kind, device and size class
// takes them back.  A failed device allocation empties that device's cache and retries.
// The cache is never destroyed (no HIP call after the runtime's teardown at exit).
// ---------------------------------------------------------------------------
constexpr size_t kPoolMaxBlock = size_t(64) << 20;

class ResourcePool {
 public:
  static ResourcePool &get() {
    static ResourcePool *pool = new ResourcePool();
    return *pool;
  }
  // device (host = false) or pinned host (host = true) memory: *cap receives the block's size
  hipError_t alloc(bool host, size_t bytes, void **out, size_t *cap) {
    const size_t want = round(bytes);
    int dev = 0;
    if (!host) (void)hipGetDevice(&dev);
    if (cap_ && want <= kPoolMaxBlock) {
      std::lock_guard<std::mutex> lk(m_);
      auto it = blocks_.lower_bound(std::make_tuple(host, host ? 0 : dev, want));
      if (it != blocks_.end() && std::get<0>(it->first) == host && std::get<1>(it->first) == (host ? 0 : dev) &&
          std::get<2>(it->first) <= 2 * want) {  // the smallest cached block that fits, if not twice too big
        *cap = std::get<2>(it->first);
        *out = it->second;
        cached_ -= *cap;
        blocks_.erase(it);
        return hipSuccess;
      }
    }
    *cap = want;
    hipError_t e = host ? hipHostMalloc(out, want, hipHostMallocDefault) : hipMalloc(out, want);
    if (e != hipSuccess) {  // memory held by the cache first
      (void)hipGetLastError();
      trim(host, dev);
      e = host ? hipHostMalloc(out, want, hipHostMallocDefault) : hipMalloc(out, want);
    }
    return e;
  }
  // p must not be in use by any queued work (its stream synchronised)
  void release(bool host, void *p, size_t cap, int dev) {
    if (!p) return;
    if (cap_ && cap <= kPoolMaxBlock) {
      std::lock_guard<std::mutex> lk(m_);
      if (cached_ + cap <= cap_) {
        blocks_.emplace(std::make_tuple(host, host ? 0 : dev, cap), p);
        cached_ += cap;
        return;
      }
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (!host && cur != dev) (void)hipSetDevice(dev);
    (void)(host ? hipHostFree(p) : hipFree(p));
    if (!host && cur != dev) (void)hipSetDevice(cur);
  }
  hipError_t stream(hipStream_t *out) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (cap_) {
      std::lock_guard<std::mutex> lk(m_);
      for (size_t i = 0; i < streams_.size(); ++i)
        if (streams_[i].first == dev) {
          *out = streams_[i].second;
          streams_.erase(streams_.begin() + static_cast<long>(i));
          return hipSuccess;
        }
    }
    return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
  }
  void release_stream(hipStream_t st, int dev) {  // st idle
    if (!st) return;
    if (cap_) {
      std::lock_guard<std::mutex> lk(m_);
      if (streams_.size() < 64) {
        streams_.emplace_back(dev, st);
        return;
      }
    }
    (void)hipStreamDestroy(st);
  }
  hipError_t event(bool timing, hipEvent_t *out) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (cap_) {
      std::lock_guard<std::mutex> lk(m_);
      auto it = events_.find(std::make_pair(dev, timing));
      if (it != events_.end()) {
        *out = it->second;
        events_.erase(it);
        return hipSuccess;
      }
    }
    return timing ? hipEventCreate(out) : hipEventCreateWithFlags(out, hipEventDisableTiming);
  }
  void release_event(hipEvent_t ev, bool timing, int dev) {
    if (!ev) return;
    if (cap_) {
      std::lock_guard<std::mutex> lk(m_);
      if (events_.size() < 4096) {
        events_.emplace(std::make_pair(dev, timing), ev);
        return;
      }
    }
    (void)hipEventDestroy(ev);
  }

 private:
  ResourcePool() {
    cap_ = size_t(512) << 20;
    if (const char *env = std::getenv("RTSN_POOL_MB")) cap_ = static_cast<size_t>(std::max(0L, std::atol(env))) << 20;
  }
  static size_t round(size_t bytes) {  // size classes: 256 B up to 64 KiB, then 64 KiB
    const size_t q = bytes <= (size_t(64) << 10) ? 256 : (size_t(64) << 10);
    return (std::max<size_t>(bytes, 16) + q - 1) / q * q;
  }
  void trim(bool host, int dev) {
    std::lock_guard<std::mutex> lk(m_);
    for (auto it = blocks_.begin(); it != blocks_.end();) {
      if (std::get<0>(it->first) == host && (host || std::get<1>(it->first) == dev)) {
        (void)(host ? hipHostFree(it->second) : hipFree(it->second));
        cached_ -= std::get<2>(it->first);
        it = blocks_.erase(it);
      } else {
        ++it;
      }
    }
  }
  std::mutex m_;
  size_t cap_ = 0, cached_ = 0;
  std::multimap<std::tuple<bool, int, size_t>, void *> blocks_;  // (pinned host, device, size) -> block
  std::vector<std::pair<int, hipStream_t>> streams_;
  std::multimap<std::pair<int, bool>, hipEvent_t> events_;      // (device, timing) -> event
};

struct DeviceBuf {
  void *p = nullptr;
  size_t bytes = 0, cap = 0;
  int dev = 0;
  DeviceBuf() = default;
  DeviceBuf(const DeviceBuf &) = delete;  // owns p
  DeviceBuf &operator=(const DeviceBuf &) = delete;
  ~DeviceBuf() { reset(); }
  void reset() {  // the owner's stream must be idle
    ResourcePool::get().release(false, p, cap, dev);
    p = nullptr;
    bytes = cap = 0;
  }
};

}  // namespace

struct rt_solver {
  // configuration (owned copies)
  rt_params p{};
  std::vector<double> prm_psi_source, prm_bounds, prm_kappa;
  phys::GroupTable gt;
  std::vector<double> mu, wt;
  std::vector<double> psi_source;  // solver-owned, M*G
  bool equilibrium_done = false;
  int g_lo = 0, g_hi = 0, Gl = 0, H = 0, Lh = 0, Lpad = 0, Q = 0, J = 0;
  int scheme = SCHEME_BDF2, K = 5;
  int T = 1;                     // full steps fused per pass (time block)
  int Tp = 0;                    // steps of the pass whose correction is pending
  int Sg = 1, Ls = 16;           // segments per line and cells per segment
  int seg_T = 0;                 // the time block the segments were sized for (0: none)
  int seg_w = 0;                 // ... and the workgroups per CU they were sized for
  bool T_set = false;            // the caller chose the time block (rt_set_time_block / RTSN_TIME_BLOCK)
  int level_waves = 0;           // pipelined BDF2 passes: 0 auto (level_waves_of), 1 one wave, 2 levels shared by two
  bool lw_set = false;           // the caller chose the waves per segment (rt_set_level_waves)
  int seg_wgs = 0;               // segments sized for this many workgroups per CU (0: the pass's occupancy)
  bool seg_set = false;          // the caller chose the segmentation (rt_set_segmentation)
  bool planned = false;          // rt_solve planned the schedule (plan_schedule): pipelined from one pass
  int d_lo = 0, d_hi = 0;        // direction-pair shard [d_lo, d_hi) of the M/2 pairs (d_hi = 0: all)
  int M_full = 0;                // the configuration's M (p.M is the handle's own direction count)
  int device = 0, cus = 0;
  hipStream_t stream = nullptr;
  // device state
  DeviceBuf E, map, lc, prop[kMaxAlignedBlock + 1], bdry, agg[2], yseg, yrefl, lineB, muwt, mom, rows, sigma;
  std::vector<double> map_host;  // [2][WN][Lpad], kept for the lazily built propagators
  bool prop_ready[kMaxAlignedBlock + 1] = {};
  int agg_cur = 0;               // aggregates of the last pass live in agg[agg_cur ^ 1]
  bool pending = false;          // E holds provisional segments (correction outstanding)
  // every launch that writes E bumps state_version; the moments kernel's phi, F, phi_plus
  // in `mom` are reused by every read-out (moments, balance, absorption) of the same state
  unsigned long long state_version = 1, mom_version = 0;
  // pipelined schedule (rt_set_pipeline): chain positions (segments; half 0 then
  // half 1 when the left boundary is reflective) at staggered time levels
  int pipe = 1;                  // 0 off, 1 auto (runs long enough to fill), 2 always
  bool pipe_set = false;         // the caller chose the schedule (rt_set_pipeline)
  int wave = 1;                  // short lines, one launch per advance (rt_set_wavefront): 0 off, 1 auto, 2 on
  int wave_max = kWaveMaxWaves;  // waves a wavefront chain may span (rt_set_wavefront_waves)
  std::vector<long long> tau;    // full steps completed per chain position
  long long target = 0;          // full steps every position must reach
  long long pipe_base = 0;       // tau of every position when the pipeline started
  int queued = 0;                // requested steps not yet enqueued (< T)
  int Tpipe = 0;                 // time block of the running pipeline (0: positions aligned)
  // material-temperature coupling (rt_material_enable)
  bool material = false;
  double rho_cv = 0.0, wsum = 0.0;
  DeviceBuf Tcell, Bcell, qbuf, edges, map_unit, lc_unit, phi_part;
  DeviceBuf corr_pow;            // A^Lsub per line for phi_correction_kernel's sub-segments
  int corr_pow_L = 0;            // the Lsub it holds (0: none)
  DeviceBuf corr_rows;           // BDF2: rows b A^j and A^64 per line (phi_correction_rows_kernel)
  bool phi_fused = false;        // angular sums fused into the coupled pass (M/2 divides 64)
  PlanckCells pc{};
  // profiling
  bool profiling = false;
  std::vector<hipEvent_t> ev_pool;   // (start, stop) pairs of profiled launches
  size_t ev_used = 0;
  double sweep_ms = 0.0;             // folded-in time of earlier pairs
  long long launches = 0, profiled = 0;
  // chunked host transfers (rt_get_psi / rt_get_ends / rt_set_ends): pinned staging
  void *staging[2] = {nullptr, nullptr};
  size_t staging_bytes = 0, staging_cap[2] = {0, 0};
  hipEvent_t staging_ev[2] = {nullptr, nullptr};
  std::string err;

  ~rt_solver() {  // everything goes back to the resource cache once the stream is idle
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);  // no kernel may outlive the buffers it uses
    ResourcePool &pool = ResourcePool::get();
    for (int k = 0; k < 2; ++k) pool.release(true, staging[k], staging_cap[k], 0);
    for (hipEvent_t e : staging_ev) pool.release_event(e, false, device);
    for (hipEvent_t e : ev_pool) pool.release_event(e, true, device);
    pool.release_stream(stream, device);
  }
};

// Waves per segment of the pipelined pass: the caller's choice, or by default two waves
// (sweep_split_kernel) where measured faster -- BDF2 at T = 20, whose one-wave kernel
// needs 126 AGPRs beside 256 VGPRs (9% extra moves; split 8.29-8.31 vs 8.52-8.53 ms/step
// on SL, profiles/r02b_split20.jsonl) -- and one wave otherwise (T = 16: 4% faster).
static bool split_block(int T);

static int level_waves_of(const rt_solver *s, int T) {
  if (s->scheme != SCHEME_BDF2 || !split_block(T)) return 1;  // the split kernel is BDF2's
  if (T > 20) return 4;                                         // one or two waves would spill
  int lw = s->level_waves ? s->level_waves : (T == 20 ? 2 : 1);
  if (lw == 4 && T % 4) lw = 2;
  return lw;
}

// Waves per segment of one pipelined launch of `grid` workgroups.  The segments are sized
// so that a full launch (every chain position active) fills the chip; the pipeline's fill
// and drain launches hold fewer positions, and with the default level_waves (0) their
// segments are split over 2 or 4 waves (sweep_split_kernel) as long as the launch stays
// within the full launch's wave count -- the lines are then traversed 2-4x faster while
// the chip would otherwise idle (BDF2 time blocks the split kernel has: 8, 10, 12, 16, 20).
static bool split_block(int T) {
  return T == 8 || T == 10 || T == 12 || T == 16 || T == 20 || T == 24 || T == 32 || T == 40;
}

static int fill_level_waves(const rt_solver *s, int grid) {
  const int base = level_waves_of(s, s->Tpipe);
  if (s->level_waves || s->scheme != SCHEME_BDF2 || !split_block(s->Tpipe)) return base;
  const long long full = 2LL * s->Q * s->Sg * base;  // waves of a launch with every position active
  int k = base;
  while (k < 4 && s->Tpipe % (2 * k) == 0 && static_cast<long long>(grid) * 2 * k <= full) k *= 2;
  return k;
}

// Chain positions of the pipelined schedule: the Sg segments of a line (both
// halves in step), or 2 Sg when the mu > 0 lines continue the mu < 0 ones.
static int chain_positions(const rt_solver *s) {
  return s->p.bc_left_indicator == 2 ? 2 * s->Sg : s->Sg;
}

static rt_status fail(rt_solver *s, rt_status st, const std::string &msg) {
  if (s) s->err = msg;
  g_last_error = msg;
  return st;
}

#define HIP_TRY(s, expr)                                                                        \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail((s), RT_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

// Full steps fused per HBM pass by default (rt_set_time_block changes it).
// Measured on SL (pipelined schedule, profiles/): BDF2 43.0 / 21.7 / 14.5 / 12.3 /
// 9.5 / 9.0 / 8.4 ms per step at T = 1 / 2 / 3 / 4 / 8 / 12 / 16.
static int default_time_block(int) { return 16; }

// rt_set_time_block's domain: the instantiated sweep kernels (kernels.hip launch_s)
static bool supported_time_block(int T) {
  return (T >= 1 && T <= 8) || T == 10 || T == 12 || T == 16 || T == 20 || T == 24 || T == 32 || T == 40;
}

static int map_count_of(int scheme) {
  switch (scheme) {
    case SCHEME_BE: return map_count<SCHEME_BE>();
    case SCHEME_CN: return map_count<SCHEME_CN>();
    default: return map_count<SCHEME_BDF2>();
  }
}

static hipError_t dalloc(DeviceBuf &b, size_t bytes) {  // b empty
  b.bytes = bytes;
  (void)hipGetDevice(&b.dev);
  return ResourcePool::get().alloc(false, bytes, &b.p, &b.cap);
}

// ---------------------------------------------------------------------------
// host-only configuration
// ---------------------------------------------------------------------------
extern "C" void rt_params_default(rt_params *out) {
  if (!out) return;
  *out = rt_params{};
  out->M = 2;
  out->G = 1;
  out->N = 100;
  out->efirst = .1;
  out->elast = 10.;
  out->X = 1.;
  out->bc_left_indicator = 2;
  out->bc_right_indicator = 1;
  out->use_mg_equilib = 0;
  out->rho = 1.;
  out->kappa_grey = 1.;
  out->T = 1.;
  out->V = 0.;
  out->use_correction = 0;
  out->ts_method = 3;
  out->dt = 0.00001;
  out->max_timesteps = 1000;
  out->include_validation = 1;
}

extern "C" rt_status rt_params_load(const char *prm_path, const char *table_dir, rt_params *out, int *prm_found) {
  if (!prm_path || !out) return fail(nullptr, RT_ERR_ARG, "rt_params_load: NULL argument");
  ParameterHandler ph(prm_path, table_dir ? table_dir : "");
  if (prm_found) *prm_found = ph.prm_found();
  if (ph.status() != RT_OK) return fail(nullptr, ph.status(), ph.error());
  *out = ph.as_params();
  auto dup = [](const std::vector<double> &v) -> double * {
    if (v.empty()) return nullptr;
    double *d = static_cast<double *>(std::malloc(sizeof(double) * v.size()));
    std::memcpy(d, v.data(), sizeof(double) * v.size());
    return d;
  };
  out->psi_source = dup(ph.psi_source());
  out->group_bounds = ph.get_have_group_bounds() ? dup(ph.group_bounds()) : nullptr;
  out->group_kappa = ph.get_have_group_absorption_opacities() ? dup(ph.group_kappa()) : nullptr;
  return RT_OK;
}

extern "C" void rt_params_free(rt_params *p) {
  if (!p) return;
  std::free(const_cast<double *>(p->psi_source));
  std::free(const_cast<double *>(p->group_bounds));
  std::free(const_cast<double *>(p->group_kappa));
  p->psi_source = p->group_bounds = p->group_kappa = nullptr;
}

extern "C" rt_status rt_quadrature(int M, double *mu, double *wt) {
  if (M <= 0 || !mu || !wt) return fail(nullptr, RT_ERR_ARG, "rt_quadrature: bad argument");
  phys::gauss_legendre(M, phys::kFourPi, mu, wt);
  return RT_OK;
}

extern "C" rt_status rt_planck_groups(double T, int G, const double *e_edge, double *B, double *dBdT) {
  if (G <= 0 || !e_edge || !B || !dBdT) return fail(nullptr, RT_ERR_ARG, "rt_planck_groups: bad argument");
  std::vector<double> lo(e_edge, e_edge + G), hi(e_edge + 1, e_edge + G + 1);
  std::fill(B, B + G, 0.0);
  std::fill(dBdT, dBdT + G, 0.0);
  phys::PlanckIntegrator().group_integrals(T, G, lo.data(), hi.data(), B, dBdT);
  for (int g = 0; g < G; ++g) {
    B[g] *= phys::kBoltzmannJPK;
    dBdT[g] *= phys::kBoltzmannJPK;
  }
  return RT_OK;
}

// ---------------------------------------------------------------------------
// per-line setup
// ---------------------------------------------------------------------------
// Line l of half h: direction i = H-1-i' (h = 0, mu < 0) or H+i' (h = 1),
// local group gl, with l = i' + H*gl; both halves share (i', gl) numbering so
// a reflective mu > 0 line and its mirror have the same l.
static int line_direction(int H, int half, int ip) { return half == 0 ? H - 1 - ip : H + ip; }

// unit_B: the source for B_g = 1 (material coupling scales it per cell)
static LineConst line_constants(const rt_solver &s, int i, int g, bool unit_B = false) {
  const rt_params &p = s.p;
  const double c = phys::kLight;
  const double dx = p.X / p.N;
  const double dt = p.dt;
  const double tau = (p.ts_method == 3) ? dt / 2.0 : dt;
  const double mu = s.mu[i], m = std::fabs(mu);
  const double sigma = s.gt.rho[g] * s.gt.kappa[g];
  LineConst L{};
  const double half = 0.5 * c * tau * dx;
  // S = 1/2 c tau dx (sigma B_g + total_correction), psi = (e_in + e_out)/2
  L.c[LC_SC] = half * sigma * (unit_B ? 1.0 : s.gt.B[g]);
  L.c[LC_SL] = 0.0;
  if (p.use_correction) {
    const double beta = p.V / c;
    L.c[LC_SC] += half * ((s.gt.cor2[g] * mu) * beta - s.gt.cor3[g] * (mu * mu) * (beta * beta));
    L.c[LC_SL] = half * s.gt.cor1[g] * mu * beta * 0.5;
  }
  auto inverse = [](double d, double o, double &i0, double &i1) {
    const double det = d * d + o * o;
    i0 = d / det;
    i1 = o / det;
  };
  {  // BE(tau)
    const double a = 1.0 + c * tau * sigma, b = c * tau * m;
    L.c[LC_BE_B] = b;
    inverse((a * dx + b) / 2.0, b / 2.0, L.c[LC_BE_I0], L.c[LC_BE_I1]);
  }
  {  // CN(tau)
    const double t = 0.5 * c * tau * sigma, A = 0.5 * c * m * tau;
    const double Bp = 1.0 + t, Cp = 1.0 - t;
    L.c[LC_CN_A] = A;
    L.c[LC_CN_K1] = 0.5 * (Cp * dx - A);
    L.c[LC_CN_K2] = 0.5 * A;
    inverse(0.5 * (A + Bp * dx), A / 2.0, L.c[LC_CN_I0], L.c[LC_CN_I1]);
  }
  {  // BDF(tau) with const_B from the full dt
    const double t = c * sigma * tau / 6.0, Ab = 1.0 + t, Bc = c * m * dt / 6.0, Cb = 1.0 - 4.0 * t, D = t;
    L.c[LC_BD_BC] = Bc;
    L.c[LC_BD_Q1] = 0.5 * (Cb * dx - 4.0 * Bc);
    L.c[LC_BD_Q2] = 2.0 * Bc;
    L.c[LC_BD_Q3] = 0.5 * (Bc + D * dx);
    L.c[LC_BD_Q4] = 0.5 * Bc;
    inverse(0.5 * (Ab * dx + Bc), 0.5 * Bc, L.c[LC_BD_I0], L.c[LC_BD_I1]);
  }
  return L;
}

// The per-line affine cell map (cell.hpp, map_apply): coefficients from
// cell_step<S> on unit inputs (constants and data zeroed), constants from
// cell_step<S> on zero inputs.  Every coefficient outside the structural
// pattern must come out exactly zero; false otherwise.
template <int S>
static bool cell_map(const LineConst &Lin, double hd, bool neg, double *W) {
  constexpr int K = SchemeDim<S>::K;
  double dense[K + 1][K + 3];  // [row][input 0..K+1, constant K+2]
  for (int col = 0; col <= K + 2; ++col) {
    LineConst L = Lin;
    if (col != K + 2) L.c[LC_SC] = 0.0;
    double X[K] = {};
    double pin = 0.0, pout = 0.0;
    if (col < K) X[col] = 1.0;
    if (col == K) pin = 1.0;
    if (col == K + 1) pout = 1.0;
    double oi, oo;
    cell_step<S>(L, hd, neg, pin, pout, X, oi, oo);
    for (int r = 0; r < K; ++r) dense[r][col] = X[r];
    dense[K][col] = oi;
    if (X[K - 1] != oo) return false;  // oout is X'[K-1]
  }
  for (int r = 0; r <= K; ++r)
    for (int col = 0; col <= K + 2; ++col) {
      const bool copy = map_copy_row0<S>() && r == 0;
      const bool used = !copy && (col == K + 2 || map_dep<S>(r, col));
      if (used) {
        W[map_slot<S>(r, col)] = dense[r][col];
      } else if (dense[r][col] != (copy && col == K + 1 ? 1.0 : 0.0)) {
        return false;
      }
    }
  return true;
}

// Linear part of the T-level combined map on the carried state (X_0..X_{T-1}):
// level t's outputs are level t+1's data (KC x KC row-major, lower triangular).
template <int S>
static void combined_linear(const double *W, int T, double *A) {
  constexpr int K = SchemeDim<S>::K;
  const int KC = T * K;
  for (int col = 0; col < KC; ++col) {
    double di = 0.0, dd = 0.0;
    for (int t = 0; t < T; ++t) {
      double X[K] = {}, Xn[K], a, e;
      if (col / K == t) X[col % K] = 1.0;
      map_apply<S, false>(W, X, di, dd, Xn, a, e);
      for (int r = 0; r < K; ++r) A[(t * K + r) * KC + col] = Xn[r];
      di = a;
      dd = e;
    }
  }
}

static void matmul(int K, const double *A, const double *B, double *C) {
  for (int r = 0; r < K; ++r)
    for (int c = 0; c < K; ++c) {
      double acc = 0.0;
      for (int m = 0; m < K; ++m) acc += A[r * K + m] * B[m * K + c];
      C[r * K + c] = acc;
    }
}

// A^n by binary exponentiation
static void matpow(int K, const double *A, long long n, double *out) {
  std::vector<double> base(A, A + K * K), acc(K * K, 0.0), tmp(K * K);
  for (int r = 0; r < K; ++r) acc[r * K + r] = 1.0;
  while (n > 0) {
    if (n & 1) {
      matmul(K, acc.data(), base.data(), tmp.data());
      acc.swap(tmp);
    }
    n >>= 1;
    if (n) {
      matmul(K, base.data(), base.data(), tmp.data());
      base.swap(tmp);
    }
  }
  std::copy(acc.begin(), acc.end(), out);
}

static rt_status upload(rt_solver *s, DeviceBuf &b, const void *src, size_t bytes) {
  HIP_TRY(s, hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s->stream));
  return RT_OK;
}

// boundary inflow per line (solver.cpp:635-692) from the solver's psi_source
static void line_inflow(const rt_solver &s, std::vector<double> &bd) {
  const int M = s.p.M, G = s.p.G;
  bd.assign(static_cast<size_t>(2) * s.Lpad, 0.0);
  for (int half = 0; half < 2; ++half) {
    const int bc = half == 0 ? s.p.bc_right_indicator : s.p.bc_left_indicator;
    for (int gl = 0; gl < s.Gl; ++gl)
      for (int ip = 0; ip < s.H; ++ip) {
        const int i = line_direction(s.H, half, ip), g = s.g_lo + gl;
        double v = 0.0;
        if (half == 0 && bc == 1) v = s.psi_source[static_cast<size_t>(i) * G + g];
        if (half == 1 && (bc == 0 || bc == 1)) v = s.psi_source[static_cast<size_t>(i) * G + g];
        bd[static_cast<size_t>(half) * s.Lpad + ip + s.H * gl] = v;
      }
  }
  (void)M;
}

// Per-line maps and constants into (map, lc); unit_B: sources for B_g = 1
// (material coupling), leaving map_host (the propagators' source) alone.
template <int S>
static rt_status line_maps_s(rt_solver *s, bool unit_B, DeviceBuf &map_dev, DeviceBuf &lc_dev) {
  constexpr int WN = map_count<S>();
  const double hd = 0.5 * (s->p.X / s->p.N);
  const size_t Lp = s->Lpad;
  std::vector<double> lc(2 * LC_COUNT * Lp, 0.0), unit_map;
  std::vector<double> &map = unit_B ? unit_map : s->map_host;
  map.assign(2 * WN * Lp, 0.0);
  double W[WN];
  for (int half = 0; half < 2; ++half)
    for (int gl = 0; gl < s->Gl; ++gl)
      for (int ip = 0; ip < s->H; ++ip) {
        const int i = line_direction(s->H, half, ip), g = s->g_lo + gl;
        const size_t ell = ip + static_cast<size_t>(s->H) * gl;
        const LineConst L = line_constants(*s, i, g, unit_B);
        for (int n = 0; n < LC_COUNT; ++n) lc[(half * LC_COUNT + n) * Lp + ell] = L.c[n];
        if (!cell_map<S>(L, hd, half == 0, W))
          return fail(s, RT_ERR_PARAM, "cell map: a structurally zero coefficient is not zero");
        for (int n = 0; n < WN; ++n) map[(half * WN + n) * Lp + ell] = W[n];
      }
  rt_status st;
  if ((st = upload(s, lc_dev, lc.data(), lc.size() * sizeof(double)))) return st;
  if ((st = upload(s, map_dev, map.data(), map.size() * sizeof(double)))) return st;
  HIP_TRY(s, hipStreamSynchronize(s->stream));  // host vectors die at return
  return RT_OK;
}

template <int S>
static rt_status setup_lines_s(rt_solver *s) {
  const size_t Lp = s->Lpad;
  rt_status st;
  if ((st = line_maps_s<S>(s, false, s->map, s->lc))) return st;
  std::vector<double> lineB(2 * Lp, 0.0);
  for (int half = 0; half < 2; ++half)
    for (int gl = 0; gl < s->Gl; ++gl)
      for (int ip = 0; ip < s->H; ++ip) lineB[half * Lp + ip + static_cast<size_t>(s->H) * gl] = s->gt.B[s->g_lo + gl];
  if ((st = upload(s, s->lineB, lineB.data(), lineB.size() * sizeof(double)))) return st;
  std::vector<double> sig(s->Gl);
  for (int gl = 0; gl < s->Gl; ++gl) sig[gl] = s->gt.rho[s->g_lo + gl] * s->gt.kappa[s->g_lo + gl];
  if ((st = upload(s, s->sigma, sig.data(), sig.size() * sizeof(double)))) return st;
  std::vector<double> muwt(2 * s->p.M);
  std::copy(s->mu.begin(), s->mu.end(), muwt.begin());
  std::copy(s->wt.begin(), s->wt.end(), muwt.begin() + s->p.M);
  if ((st = upload(s, s->muwt, muwt.data(), muwt.size() * sizeof(double)))) return st;
  HIP_TRY(s, hipStreamSynchronize(s->stream));  // host vectors die at return
  return RT_OK;
}

// Segment propagators A_T^Ls, A_T^Llast of every line for the aligned schedule
// (fold_kernel), built on first use of a time block T: the pipelined schedule
// never needs them.  Lines are independent: host threads split them.
template <int S>
static rt_status build_propagators_s(rt_solver *s, int T) {
  constexpr int K = SchemeDim<S>::K, WN = map_count<S>();
  const int KC = T * K, NTC = KC * (KC + 1) / 2;
  const long long L_last = s->p.N - static_cast<long long>(s->Sg - 1) * s->Ls;
  const size_t Lp = s->Lpad, lines = 2 * Lp;
  std::vector<double> pr(2 * prop_count(K, T) * Lp, 0.0);
  auto work = [&](size_t l0, size_t l1) {
    std::vector<double> A(KC * KC), Aseg(KC * KC), Alast(KC * KC);
    double W[WN];
    for (size_t idx = l0; idx < l1; ++idx) {
      const size_t half = idx / Lp, ell = idx % Lp;
      for (int n = 0; n < WN; ++n) W[n] = s->map_host[(half * WN + n) * Lp + ell];
      std::fill(A.begin(), A.end(), 0.0);
      combined_linear<S>(W, T, A.data());
      matpow(KC, A.data(), s->Ls, Aseg.data());
      matpow(KC, A.data(), L_last, Alast.data());
      double *dst = pr.data() + half * prop_count(K, T) * Lp + ell;
      for (int r = 0; r < KC; ++r)
        for (int c = 0; c <= r; ++c) {
          dst[tri(r, c) * Lp] = Aseg[r * KC + c];
          dst[(NTC + tri(r, c)) * Lp] = Alast[r * KC + c];
        }
    }
  };
  const size_t nt = std::max<size_t>(1, std::min<size_t>(16, std::thread::hardware_concurrency()));
  std::vector<std::thread> pool;
  for (size_t t = 0; t < nt; ++t) pool.emplace_back(work, lines * t / nt, lines * (t + 1) / nt);
  for (std::thread &th : pool) th.join();
  rt_status st = upload(s, s->prop[T], pr.data(), pr.size() * sizeof(double));
  if (st) return st;
  HIP_TRY(s, hipStreamSynchronize(s->stream));  // pr dies at return
  s->prop_ready[T] = true;
  return RT_OK;
}

static rt_status ensure_propagators(rt_solver *s, int T) {
  if (s->prop_ready[T]) return RT_OK;
  switch (s->scheme) {
    case SCHEME_BE: return build_propagators_s<SCHEME_BE>(s, T);
    case SCHEME_CN: return build_propagators_s<SCHEME_CN>(s, T);
    default: return build_propagators_s<SCHEME_BDF2>(s, T);
  }
}

static rt_status setup_lines(rt_solver *s) {
  switch (s->scheme) {
    case SCHEME_BE: return setup_lines_s<SCHEME_BE>(s);
    case SCHEME_CN: return setup_lines_s<SCHEME_CN>(s);
    default: return setup_lines_s<SCHEME_BDF2>(s);
  }
}

static rt_status upload_inflow(rt_solver *s) {
  std::vector<double> bd;
  line_inflow(*s, bd);
  rt_status st = upload(s, s->bdry, bd.data(), bd.size() * sizeof(double));
  if (st) return st;
  HIP_TRY(s, hipStreamSynchronize(s->stream));
  return RT_OK;
}

static Geometry geometry(const rt_solver *s) { return Geometry{s->p.M, s->Gl, s->p.N, s->J * kSweepTile, s->Lpad}; }

// Segments per line: enough waves (2 Q Sg) to fill the chip at the sweep
// kernel's occupancy, Ls a multiple of the register chunk.
static void segment_lines(rt_solver *h, int waves_per_cu) {
  waves_per_cu = std::max(1, std::min(waves_per_cu, 64));
  const long long target = static_cast<long long>(h->cus) * waves_per_cu;
  long long sg = std::max<long long>(1, target / (2LL * h->Q));
  const long long max_sg = (h->p.N + kSweepCells - 1) / kSweepCells;
  sg = std::min(sg, max_sg);
  long long ls = (h->p.N + sg - 1) / sg;
  ls = ((ls + kSweepCells - 1) / kSweepCells) * kSweepCells;
  h->Ls = static_cast<int>(ls);
  h->Sg = static_cast<int>((h->p.N + ls - 1) / ls);
}

// Per-segment buffers (aggregates, folded incoming states), zeroed; the
// segment propagators are rebuilt on their next use.
static hipError_t alloc_segments(rt_solver *h) {
  const size_t Lp = h->Lpad;
  const int K = h->K;
  if (h->agg[0].p || h->agg[1].p || h->yseg.p) (void)hipStreamSynchronize(h->stream);  // before the cache may hand them out
  for (DeviceBuf *b : {&h->agg[0], &h->agg[1], &h->yseg}) b->reset();
  hipError_t e = dalloc(h->agg[0], sizeof(double) * 2 * h->Sg * kMaxTimeBlock * K * Lp);
  if (!e) e = dalloc(h->agg[1], sizeof(double) * 2 * h->Sg * kMaxTimeBlock * K * Lp);
  if (!e) e = dalloc(h->yseg, sizeof(double) * 2 * (h->Sg + 1) * kMaxAlignedBlock * K * Lp);
  if (!e) e = hipMemsetAsync(h->agg[0].p, 0, h->agg[0].bytes, h->stream);
  if (!e) e = hipMemsetAsync(h->agg[1].p, 0, h->agg[1].bytes, h->stream);
  for (bool &r : h->prop_ready) r = false;
  return e;
}

// Segments sized for the pipelined pass of the current time block (its occupancy: one
// wave per SIMD at T = 16 and 20, two at T = 10, ...), applied only while every chain
// position is at the same time with no correction outstanding -- the state rows do not
// depend on the segmentation, only the aggregates and propagators do.  Called by
// rt_set_time_block and again before the next pipelined or aligned pass, so a handle
// always runs its passes with segments for the time block it runs.
static rt_status segment_target(rt_solver *h, int *w_out);

static rt_status resegment(rt_solver *h) {
  if (h->material || h->pending || h->Tpipe) return RT_OK;
  int w = 0;
  if (rt_status st = segment_target(h, &w)) return st;
  if (h->seg_T == h->T && h->seg_w == w) return RT_OK;
  const int sg0 = h->Sg, ls0 = h->Ls;
  segment_lines(h, w);
  h->seg_T = h->T;
  h->seg_w = w;
  if (h->Sg == sg0 && h->Ls == ls0) return RT_OK;
  if (2LL * h->Q * h->Sg >= (1LL << 31)) return fail(h, RT_ERR_PARAM, "too many lines for one handle: shard the groups");
  HIP_TRY(h, alloc_segments(h));
  h->tau.assign(chain_positions(h), h->target);  // every position at the same, requested time
  return RT_OK;
}

// Workgroups per CU the segments of the current time block are sized for: the caller's
// (rt_set_segmentation, or the schedule rt_solve planned), else the pipelined pass's
// occupancy (RTSN_WAVES_PER_CU overrides, for experiments).
static rt_status segment_target(rt_solver *h, int *w_out) {
  int w = h->seg_wgs;
  if (!w) HIP_TRY(h, sweep_occupancy(h->scheme, h->T, level_waves_of(h, h->T), &w));
  if (const char *env = std::getenv("RTSN_WAVES_PER_CU")) w = std::atoi(env);  // experiments
  *w_out = std::max(1, std::min(w, 64));
  return RT_OK;
}

// ---------------------------------------------------------------------------
// lifecycle
// ---------------------------------------------------------------------------
// Direction-pair shard [d_lo, d_hi) of the M/2 pairs (i' counted from mu = 0 outward):
// the handle holds M_l = 2 (d_hi - d_lo) directions, global i in [H - d_hi, H - d_lo) and
// [H + d_lo, H + d_hi) (ascending mu, mirror pairs together for the reflective BC), with
// the full quadrature's nodes and weights and the prm psi_source rows of those directions.
static rt_status create_impl(const rt_params *pin, int g_lo, int g_hi, int d_lo, int d_hi, int device,
                             rt_solver **out);

extern "C" rt_status rt_create_from_params(const rt_params *pin, int g_lo, int g_hi, int device, rt_solver **out) {
  return create_impl(pin, g_lo, g_hi, 0, 0, device, out);
}

extern "C" rt_status rt_create_direction_shard(const rt_params *pin, int g_lo, int g_hi, int d_lo, int d_hi,
                                               int device, rt_solver **out) {
  if (!pin || !out) return fail(nullptr, RT_ERR_ARG, "rt_create_direction_shard: NULL argument");
  if (pin->M > 0 && (d_lo < 0 || d_lo >= d_hi || d_hi > pin->M / 2))
    return fail(nullptr, RT_ERR_PARAM, "bad direction-pair range (0 <= d_lo < d_hi <= M/2)");
  return create_impl(pin, g_lo, g_hi, d_lo, d_hi, device, out);
}

static rt_status create_impl(const rt_params *pin, int g_lo, int g_hi, int d_lo, int d_hi, int device,
                             rt_solver **out) {
  if (!pin || !out) return fail(nullptr, RT_ERR_ARG, "rt_create_from_params: NULL argument");
  *out = nullptr;
  const rt_params &q = *pin;
  if (q.M <= 0 || (q.M % 2) != 0) return fail(nullptr, RT_ERR_PARAM, "M must be positive and even (mu = 0 asserts, solver.cpp:402)");
  if (q.G <= 0 || q.N <= 0) return fail(nullptr, RT_ERR_PARAM, "G and N must be positive");
  if (q.ts_method < 1 || q.ts_method > 3) return fail(nullptr, RT_ERR_PARAM, "ts_method must be 1, 2 or 3 (solver.cpp:755)");
  if (q.bc_left_indicator < 0 || q.bc_left_indicator > 2 || q.bc_right_indicator < 0 || q.bc_right_indicator > 2)
    return fail(nullptr, RT_ERR_PARAM, "boundary indicators must be 0, 1 or 2 (solver.cpp:658-690)");
  if (!(q.X > 0.0) || !(q.dt > 0.0)) return fail(nullptr, RT_ERR_PARAM, "X and dt must be positive");
  if (g_hi <= 0) g_hi = q.G;
  if (g_lo < 0 || g_lo >= g_hi || g_hi > q.G) return fail(nullptr, RT_ERR_PARAM, "bad group range");

  std::unique_ptr<rt_solver> s(new rt_solver());
  s->p = q;
  const size_t MG = static_cast<size_t>(q.M) * q.G;
  if (q.psi_source) s->prm_psi_source.assign(q.psi_source, q.psi_source + MG);
  if (q.group_bounds) s->prm_bounds.assign(q.group_bounds, q.group_bounds + q.G + 1);
  if (q.group_kappa) s->prm_kappa.assign(q.group_kappa, q.group_kappa + q.G);
  s->p.psi_source = s->prm_psi_source.empty() ? nullptr : s->prm_psi_source.data();
  s->p.group_bounds = s->prm_bounds.empty() ? nullptr : s->prm_bounds.data();
  s->p.group_kappa = s->prm_kappa.empty() ? nullptr : s->prm_kappa.data();

  rt_status st = phys::build_group_table(s->p, s->gt);
  if (st) return fail(nullptr, st, "group table: group edges must increase");
  s->mu.resize(q.M);
  s->wt.resize(q.M);
  phys::gauss_legendre(q.M, phys::kFourPi, s->mu.data(), s->wt.data());
  s->M_full = q.M;
  if (d_hi > 0 && !(d_lo == 0 && d_hi == q.M / 2)) {  // direction-pair shard: keep its directions
    const int H = q.M / 2, n = d_hi - d_lo;
    std::vector<int> keep;
    for (int i = H - d_hi; i < H - d_lo; ++i) keep.push_back(i);
    for (int i = H + d_lo; i < H + d_hi; ++i) keep.push_back(i);
    std::vector<double> mu(2 * n), wt(2 * n), src;
    for (int k = 0; k < 2 * n; ++k) {
      mu[k] = s->mu[keep[k]];
      wt[k] = s->wt[keep[k]];
    }
    if (!s->prm_psi_source.empty())  // rows m of the prm's (M, G) table, index m G + g
      for (int k = 0; k < 2 * n; ++k)
        src.insert(src.end(), s->prm_psi_source.begin() + static_cast<size_t>(keep[k]) * q.G,
                   s->prm_psi_source.begin() + static_cast<size_t>(keep[k] + 1) * q.G);
    s->mu.swap(mu);
    s->wt.swap(wt);
    s->prm_psi_source.swap(src);
    s->p.psi_source = s->prm_psi_source.empty() ? nullptr : s->prm_psi_source.data();
    s->p.M = 2 * n;
    s->d_lo = d_lo;
    s->d_hi = d_hi;
  }
  phys::solver_psi_source(s->p, s->gt, s->mu.data(), s->psi_source);
  if (q.use_mg_equilib) {  // only the ph copy until solve() (solver.cpp:601-604)
    rt_params pre = s->p;
    pre.use_mg_equilib = 0;
    phys::solver_psi_source(pre, s->gt, s->mu.data(), s->psi_source);
  }

  s->g_lo = g_lo;
  s->g_hi = g_hi;
  s->Gl = g_hi - g_lo;
  s->H = s->p.M / 2;
  s->Lh = s->H * s->Gl;
  s->Q = (s->Lh + 63) / 64;
  s->Lpad = 64 * s->Q;
  s->J = (q.N + kSweepTile - 1) / kSweepTile;
  s->scheme = q.ts_method;
  s->K = q.ts_method == 1 ? 1 : (q.ts_method == 2 ? 2 : 5);
  s->device = device;

  rt_solver *h = s.get();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0)
    return fail(nullptr, RT_ERR_DEVICE, "no HIP device " + std::to_string(device));
  HIP_TRY(h, hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(h, hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
    return fail(nullptr, RT_ERR_DEVICE, std::string("librtsn is built for gfx950, device is ") + prop.gcnArchName);
  HIP_TRY(h, ResourcePool::get().stream(&h->stream));
  for (hipEvent_t &ev : h->staging_ev) HIP_TRY(h, ResourcePool::get().event(false, &ev));

  // segments: enough waves to fill the chip (occupancy x CUs), Ls a multiple of the chunk
  int waves_per_cu = 0;
  h->T = default_time_block(h->scheme);
  if (const char *t = std::getenv("RTSN_TIME_BLOCK"))  // experiments: the segment count follows
    if (supported_time_block(std::atoi(t))) {
      h->T = std::atoi(t);
      h->T_set = true;
    }
  if (const char *wv = std::getenv("RTSN_WAVEFRONT"))  // experiments: "0" off, "2" on for every short line
    if (!std::strcmp(wv, "0") || !std::strcmp(wv, "2")) h->wave = wv[0] - '0';
  if (const char *ww = std::getenv("RTSN_WAVE_WAVES"))  // experiments: waves per wavefront chain, 1..8
    if (std::atoi(ww) >= 1 && std::atoi(ww) <= kWaveMaxWaves) h->wave_max = std::atoi(ww);
  if (const char *lw = std::getenv("RTSN_LEVEL_WAVES"))  // experiments: only "1", "2" or "4" are read
    if (!std::strcmp(lw, "1") || !std::strcmp(lw, "2") || !std::strcmp(lw, "4")) h->level_waves = lw[0] - '0';
  h->cus = prop.multiProcessorCount;
  if ((st = segment_target(h, &waves_per_cu))) return st;
  segment_lines(h, waves_per_cu);
  h->seg_T = h->T;
  h->seg_w = waves_per_cu;
  if (2LL * h->Q * h->Sg >= (1LL << 31)) return fail(nullptr, RT_ERR_PARAM, "too many lines for one handle: shard the groups");
  // a chunk's rows are addressed through one buffer descriptor with 32-bit offsets
  if (16LL * 16 * h->Lpad >= (1LL << 31)) return fail(nullptr, RT_ERR_PARAM, "too many lines per row: shard the groups");

  const size_t Lp = h->Lpad;
  const int K = h->K;
  hipError_t e = hipSuccess;
  const size_t Nrow = static_cast<size_t>(h->J) * kSweepTile;  // cells padded to whole tiles
  if (!e) e = dalloc(h->E, sizeof(double2) * 2 * Nrow * Lp);
  if (!e) e = dalloc(h->lc, sizeof(double) * 2 * LC_COUNT * Lp);
  if (!e) e = dalloc(h->map, sizeof(double) * 2 * map_count_of(h->scheme) * Lp);
  for (int T = 1; T <= kMaxAlignedBlock; ++T)
    if (!e) e = dalloc(h->prop[T], sizeof(double) * 2 * prop_count(K, T) * Lp);
  if (!e) e = dalloc(h->bdry, sizeof(double) * 2 * Lp);
  if (!e) e = alloc_segments(h);
  if (!e) e = dalloc(h->yrefl, sizeof(double) * kMaxAlignedBlock * K * Lp);
  if (!e) e = dalloc(h->lineB, sizeof(double) * 2 * Lp);
  if (!e) e = dalloc(h->muwt, sizeof(double) * 2 * h->p.M);
  if (!e) e = dalloc(h->mom, sizeof(double) * 3 * h->Gl * static_cast<size_t>(q.N));
  if (!e) e = dalloc(h->rows, sizeof(double2) * 4 * Lp);
  if (!e) e = dalloc(h->sigma, sizeof(double) * h->Gl);
  if (e) return fail(nullptr, RT_ERR_NOMEM, std::string("device allocation: ") + hipGetErrorString(e));

  h->tau.assign(chain_positions(h), 0);
  if ((st = setup_lines(h))) return st;
  if ((st = upload_inflow(h))) return st;
  HIP_TRY(h, launch_init_state(static_cast<double2 *>(h->E.p), static_cast<const double *>(h->lineB.p), geometry(h),
                               h->stream));
  ++h->state_version;

  HIP_TRY(h, hipStreamSynchronize(h->stream));
  *out = s.release();
  return RT_OK;
}

extern "C" rt_status rt_create(const char *prm_path, const char *table_dir, int device, rt_solver **out) {
  if (!prm_path || !out) return fail(nullptr, RT_ERR_ARG, "rt_create: NULL argument");
  ParameterHandler ph(prm_path, table_dir ? table_dir : "");
  if (ph.status() != RT_OK) return fail(nullptr, ph.status(), ph.error());
  const rt_params p = ph.as_params();
  return rt_create_from_params(&p, 0, 0, device, out);
}

extern "C" void rt_destroy(rt_solver *s) { delete s; }

// ---------------------------------------------------------------------------
// stepping
// ---------------------------------------------------------------------------
static rt_status check_validation(rt_solver *s) {
  if (s->p.include_validation && !phys::validate_correction(s->p, s->gt))
    return fail(s, RT_ERR_VALIDATION, "validate_correction() fails (correction.cpp:39-63,100-122)");
  return RT_OK;
}

static rt_status ensure_equilibrium(rt_solver *s) {
  if (!s->p.use_mg_equilib || s->equilibrium_done) return RT_OK;
  rt_status st = check_validation(s);  // solver.cpp:290-293
  if (st) return st;
  phys::solver_psi_source(s->p, s->gt, s->mu.data(), s->psi_source);
  s->equilibrium_done = true;
  return upload_inflow(s);
}

// Sum the elapsed time of the recorded (start, stop) event pairs.
static rt_status fold_events(rt_solver *s) {
  for (size_t k = 0; k + 1 < s->ev_used; k += 2) {
    HIP_TRY(s, hipEventSynchronize(s->ev_pool[k + 1]));
    float ms = 0.f;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev_pool[k], s->ev_pool[k + 1]));
    s->sweep_ms += ms;
  }
  s->ev_used = 0;
  return RT_OK;
}

static SegArgs seg_args(rt_solver *s) {
  SegArgs a{};
  a.E = static_cast<double2 *>(s->E.p);
  a.map = static_cast<const double *>(s->map.p);
  a.lc = static_cast<const double *>(s->lc.p);
  a.bdry = static_cast<const double *>(s->bdry.p);
  a.yseg = static_cast<const double *>(s->yseg.p);
  a.yrefl = static_cast<const double *>(s->yrefl.p);
  a.agg_cur = static_cast<double *>(s->agg[s->agg_cur].p);
  a.N = s->p.N;
  a.Nrow = s->J * kSweepTile;
  a.Lpad = s->Lpad;
  a.Q = s->Q;
  a.Sg = s->Sg;
  a.Ls = s->Ls;
  a.half0 = 0;
  a.reflective = s->p.bc_left_indicator == 2;
  a.pending = s->pending ? 1 : 0;
  a.hd = 0.5 * (s->p.X / s->p.N);
  a.level_waves = level_waves_of(s, s->T);
  return a;
}

// Fold segment aggregates of a T-step pass into true incoming states:
// previous pass (agg_prev) -> yseg for the pending correction, or this pass's
// mu < 0 half (agg_cur) -> yrefl for the reflective mu > 0 heads.
static rt_status enqueue_fold(rt_solver *s, int T, bool reflective_outflow) {
  if (rt_status st = ensure_propagators(s, T)) return st;
  FoldArgs f{};
  const int slot = reflective_outflow ? s->agg_cur : (s->agg_cur ^ 1);
  f.agg = static_cast<const double *>(s->agg[slot].p);
  f.prop = static_cast<const double *>(s->prop[T].p);
  f.y = static_cast<double *>(reflective_outflow ? s->yrefl.p : s->yseg.p);
  f.prop_half = prop_count(s->K, T);
  f.Sg = s->Sg;
  f.Lpad = s->Lpad;
  f.half0 = 0;
  f.nhalf = reflective_outflow ? 1 : 2;
  f.last_short = (s->p.N - (s->Sg - 1) * s->Ls) != s->Ls;
  f.only_last = reflective_outflow ? 1 : 0;
  HIP_TRY(s, launch_fold(T * s->K, f, s->stream));
  return RT_OK;
}

// Apply the outstanding cross-segment correction in place (before any read,
// or before a pass with a different time block).
static rt_status apply_correction(rt_solver *s) {
  if (!s->pending) return RT_OK;
  rt_status st = enqueue_fold(s, s->Tp, false);
  if (st) return st;
  SegArgs a = seg_args(s);
  HIP_TRY(s, launch_sweep(s->scheme, s->Tp, SWEEP_FINALIZE, a, 2 * s->Q * s->Sg, s->stream));
  ++s->state_version;
  s->pending = false;
  return RT_OK;
}

static rt_status event_begin(rt_solver *s, hipEvent_t *e1) {
  *e1 = nullptr;
  if (!s->profiling) return RT_OK;
  if (s->ev_used + 2 > s->ev_pool.size()) {
    rt_status st = fold_events(s);  // drain the pool when it is full
    if (st) return st;
  }
  hipEvent_t e0 = s->ev_pool[s->ev_used++];
  *e1 = s->ev_pool[s->ev_used++];
  HIP_TRY(s, hipEventRecord(e0, s->stream));
  return RT_OK;
}

static rt_status event_end(rt_solver *s, hipEvent_t e1) {
  if (e1) {
    HIP_TRY(s, hipEventRecord(e1, s->stream));
    ++s->profiled;
  }
  ++s->launches;
  return RT_OK;
}

// One pass of T full steps, every segment at the same time level.
// coupled: the material-coupled sweep (T = 1, per-cell emission).
static rt_status enqueue_pass(rt_solver *s, int T, bool coupled = false) {
  if (s->pending && s->Tp != T) {
    rt_status st = apply_correction(s);
    if (st) return st;
  }
  const int per_half = s->Q * s->Sg;
  SegArgs a = seg_args(s);
  if (coupled) {
    a.map = static_cast<const double *>(s->map_unit.p);
    a.lc = static_cast<const double *>(s->lc_unit.p);
    a.bcell = static_cast<const double *>(s->Bcell.p);
    a.Gl = s->Gl;
    a.H = s->H;
    a.phi = s->phi_fused ? static_cast<double *>(s->phi_part.p) : nullptr;
    a.wt = static_cast<const double *>(s->muwt.p) + s->p.M;
  }
  hipEvent_t e1;
  rt_status st = event_begin(s, &e1);
  if (st) return st;
  if (s->pending && (st = enqueue_fold(s, T, false))) return st;
  if (a.reflective) {  // mu > 0 heads need this pass's mu < 0 outflow: two launches
    a.half0 = 0;
    HIP_TRY(s, launch_sweep(s->scheme, T, SWEEP_PASS, a, per_half, s->stream));
    if ((st = enqueue_fold(s, T, true))) return st;
    a.half0 = 1;
    HIP_TRY(s, launch_sweep(s->scheme, T, SWEEP_PASS, a, per_half, s->stream));
  } else {
    HIP_TRY(s, launch_sweep(s->scheme, T, SWEEP_PASS, a, 2 * per_half, s->stream));
  }
  if ((st = event_end(s, e1))) return st;
  ++s->state_version;
  s->pending = s->Sg > 1;
  s->Tp = T;
  s->agg_cur ^= 1;
  for (long long &t : s->tau) t += T;
  s->target += T;
  return RT_OK;
}

// nsteps full steps in aligned passes of at most T (and kMaxAlignedBlock) steps.
static rt_status enqueue_steps(rt_solver *s, int nsteps) {
  if (rt_status st = resegment(s)) return st;
  const int T = std::min(s->T, kMaxAlignedBlock);
  while (nsteps > 0) {
    const int n = std::min(T, nsteps);
    rt_status st = enqueue_pass(s, n);
    if (st) return st;
    nsteps -= n;
  }
  return RT_OK;
}

// ---------------------------------------------------------------------------
// Pipelined schedule.  Chain position c (segment s of half 0, or of half 1:
// c = s for both halves, or c = Sg + s when the mu > 0 heads take the mu < 0
// outflow) runs one pass behind position c-1: in every launch each position
// that can advance T steps does, starting from the exit state position c-1
// published in the previous launch for exactly those steps.  Every segment
// starts exact, so no provisional state and no correction.  The first
// launches fill the pipeline (position c starts in launch c), the last ones
// drain it; both happen once per run of advances, and the drain only when a
// read-out needs the state (finalize).
// ---------------------------------------------------------------------------
static rt_status pipe_launch(rt_solver *s) {
  const int P = chain_positions(s), T = s->Tpipe;
  int lo = -1, hi = -1;
  for (int c = 0; c < P; ++c) {
    const bool ready = s->tau[c] < s->target && (c == 0 || s->tau[c - 1] >= s->tau[c] + T);
    if (!ready) continue;
    if (lo < 0) lo = c;
    if (hi >= 0 && hi != c - 1) return fail(s, RT_ERR_PARAM, "pipeline: active positions not contiguous");
    hi = c;
  }
  if (lo < 0) return fail(s, RT_ERR_PARAM, "pipeline: no position can advance");  // loops below rely on progress
  for (int c = lo; c <= hi; ++c)
    if (s->tau[c] != s->tau[lo] - static_cast<long long>(c - lo) * T)
      return fail(s, RT_ERR_PARAM, "pipeline: positions out of step");
  SegArgs a = seg_args(s);
  a.aggs[0] = static_cast<double *>(s->agg[0].p);
  a.aggs[1] = static_cast<double *>(s->agg[1].p);
  a.pending = 0;
  a.pos_lo = lo;
  a.npos = hi - lo + 1;
  a.pass_lo = static_cast<int>(((s->tau[lo] - s->pipe_base) / T) & 1);
  const int grid = (a.reflective ? 1 : 2) * a.npos * s->Q;
  a.level_waves = fill_level_waves(s, grid);
  hipEvent_t e1;
  rt_status st = event_begin(s, &e1);
  if (st) return st;
  HIP_TRY(s, launch_sweep(s->scheme, T, SWEEP_PIPELINED, a, grid, s->stream));
  ++s->state_version;
  if ((st = event_end(s, e1))) return st;
  for (int c = lo; c <= hi; ++c) s->tau[c] += T;
  return RT_OK;
}

// rt_set_pipeline(1): the fewest whole passes an advance must bring for the pipelined
// schedule.  A pipelined run of n passes over P chain positions takes P + n - 1 launches;
// with the fill/drain launches split over 4 waves (fill_level_waves: BDF2 blocks with a
// split kernel) a launch of at most P/4 positions costs a quarter of a pass, so from
// n >= P/8 passes the run beats aligned passes (at most 4 steps each, the correction doubling
// the FP64 work: 20.0 vs 8.3 ms per step on SL).  Without the split, n >= P.
static int auto_pipeline_passes(const rt_solver *s) {
  const int P = chain_positions(s);
  if (s->planned) return 1;  // the planned schedule's model is the pipelined run
  if (s->scheme == SCHEME_BDF2 && !s->level_waves && split_block(s->T)) return std::max(1, (P + 7) / 8);
  return P;
}

// Queue nsteps; launch whole passes while the chain head is behind.
static rt_status pipe_advance(rt_solver *s, int nsteps) {
  s->queued += nsteps;
  const int T = s->T;
  rt_status st;
  if (s->Tpipe && s->Tpipe != T) {  // a lagged pipeline of another block size: let it drain
    while (s->tau.back() < s->target)
      if ((st = pipe_launch(s))) return st;
    s->Tpipe = 0;
  }
  const long long passes = s->queued / T;
  if (passes == 0) return RT_OK;
  if (!s->Tpipe) {
    if (s->pipe == 1 && passes < auto_pipeline_passes(s)) {
      // too few passes to fill the pipeline (it would run its segments nearly one
      // at a time): aligned passes of at most kMaxAlignedBlock steps instead
      s->queued -= static_cast<int>(passes * T);
      return enqueue_steps(s, static_cast<int>(passes * T));
    }
    // start from aligned positions with an exact state, segments sized for this T
    if ((st = apply_correction(s))) return st;
    if ((st = resegment(s))) return st;
    s->Tpipe = T;
    s->pipe_base = s->tau[0];
  }
  s->queued -= static_cast<int>(passes * T);
  s->target += passes * T;
  while (s->tau[0] < s->target)
    if ((st = pipe_launch(s))) return st;
  return RT_OK;
}

// Bring every position to the target (drain) and run the queued remainder.
static rt_status complete(rt_solver *s) {
  rt_status st;
  if (s->Tpipe) {
    while (s->tau.back() < s->target)
      if ((st = pipe_launch(s))) return st;
    s->Tpipe = 0;
  }
  if (s->queued) {
    const int r = s->queued;
    s->queued = 0;
    if ((st = enqueue_steps(s, r))) return st;
  }
  return RT_OK;
}

// The state at the requested time, exact: before any read-out.
static rt_status finalize(rt_solver *s) {
  rt_status st = complete(s);
  if (st) return st;
  return apply_correction(s);
}

// Short lines (kernels_wave.hip): every step of an advance in one launch per chunk of
// steps, lanes over cells -- by default (rt_set_wavefront 1) when the line fits a
// workgroup's chain and the caller chose neither a time block nor a schedule, always with
// rt_set_wavefront 2.
static WavePlan wave_plan(const rt_solver *s) {
  return wavefront_plan(s->p.N, s->p.bc_left_indicator == 2, s->wave_max);
}

// Auto (mode 1) takes a chain of several waves while the chains need at most two waves per
// SIMD: mid-length lines run 4-7x faster as chains than as segment passes there (1000 BDF2
// steps, N = 600-4000 cells: 4 groups 0.46-1.5 ms vs 2.7-6.6 ms, 124 groups, i.e. 1984 waves,
// 0.67-1.7 ms vs 4.0-8.1 ms; profiles/r03ai_mid.jsonl).  Beyond, the chains time-share the
// SIMDs, and the segment pipeline's full-chip passes (28 FMAs per cell and level at ~90% of
// the FP64 issue rate) carry the same work with less overhead per cell.
static bool use_wavefront(const rt_solver *s) {
  if (s->material || s->wave == 0) return false;
  const WavePlan p = wave_plan(s);
  if (p.C == 0) return false;
  if (s->wave == 2) return true;
  if (s->T_set || s->pipe_set) return false;
  const long long chains = static_cast<long long>(s->H) * s->Gl * (s->p.bc_left_indicator == 2 ? 1 : 2);
  return p.waves == 1 || chains * p.waves <= 8LL * s->cus;
}

constexpr int kWaveMaxSteps = 1 << 16;  // steps per wavefront launch (bounds one launch's length)

static rt_status wave_advance(rt_solver *s, int nsteps) {
  if (rt_status st = finalize(s)) return st;  // the stored state exact at the requested time
  SegArgs a = seg_args(s);
  a.Gl = s->Gl;
  a.H = s->H;
  while (nsteps > 0) {
    const int m = std::min(nsteps, kWaveMaxSteps);
    hipEvent_t e1;
    rt_status st = event_begin(s, &e1);
    if (st) return st;
    HIP_TRY(s, launch_wavefront(s->scheme, wave_plan(s), a, m, s->stream));
    if ((st = event_end(s, e1))) return st;
    ++s->state_version;
    for (long long &t : s->tau) t += m;
    s->target += m;
    nsteps -= m;
  }
  return RT_OK;
}

extern "C" rt_status rt_advance(rt_solver *s, int nsteps) {
  if (!s || nsteps < 0) return fail(s, RT_ERR_ARG, "rt_advance: bad argument");
  if (s->material) return fail(s, RT_ERR_STATE, "material coupling is on: step with rt_material_step / rt_material_sweep");
  HIP_TRY(s, hipSetDevice(s->device));
  rt_status st = check_validation(s);
  if (st) return st;
  if ((st = ensure_equilibrium(s))) return st;
  if (use_wavefront(s)) return wave_advance(s, nsteps);
  return s->pipe ? pipe_advance(s, nsteps) : enqueue_steps(s, nsteps);
}

extern "C" rt_status rt_finish(rt_solver *s) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_finish: NULL handle");
  HIP_TRY(s, hipSetDevice(s->device));
  return finalize(s);
}

extern "C" rt_status rt_synchronize(rt_solver *s) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_synchronize: NULL handle");
  HIP_TRY(s, hipStreamSynchronize(s->stream));
  return RT_OK;
}

// rt_solve knows the run's length.  Unless the caller chose the schedule (time block, waves
// per segment, segmentation), a BDF2 run takes the pipelined schedule with the least
// estimated whole-run time (plan_schedule): time block T of 8-40 steps, four waves per
// segment (sweep_split_kernel<3, T, 4>, every launch of the run) and segments sized for w of
// 4-32 workgroups per CU.  The model (fitted to the finite-state whole-run
// grids profiles/r03l_grid{16,128}.jsonl: mean error 3%): a run of n steps is P = n / T
// passes over a chain of C segment positions, launched as P + C - 1 launches whose active
// positions form a band (ramp up, plateau of min(P, C), ramp down); a launch of W workgroups
// runs in rounds of the resident 2 per CU, and a round's time is one segment's Ls x T / 4
// cell-levels per wave at the per-level cost of its block (t_T) times the workgroups the
// busiest CU holds (ceil(W / CUs): a wave per SIMD each).  n mod T steps more run as aligned
// passes with the cross-segment correction (~3 steps' cost each, ~30 ms of folds).
struct RunGeom {
  long long N;
  int M, Gl, cus;
  bool reflective;
};

static double level_ns(int T) {  // per cell-level and wave, a SIMD's issue shared by its waves
  switch (T) {
    case 8: return 76.7;
    case 16: return 71.0;
    case 20: return 67.6;
    case 24: return 70.4;
    case 32: return 66.7;
    default: return 64.7;  // 40
  }
}

static void model_segments(const RunGeom &g, int w, long long *Sg, long long *Ls) {
  const long long Q = (static_cast<long long>(g.M / 2) * g.Gl + 63) / 64;
  long long sg = std::max<long long>(1, static_cast<long long>(g.cus) * w / (2 * Q));
  sg = std::min(sg, (g.N + kSweepCells - 1) / kSweepCells);
  long long ls = (g.N + sg - 1) / sg;
  ls = (ls + kSweepCells - 1) / kSweepCells * kSweepCells;
  *Ls = ls;
  *Sg = (g.N + ls - 1) / ls;
}

static double run_ms_model(const RunGeom &g, long long n, int T, int w) {
  constexpr int kw = 4, occ = 2;
  long long Sg, Ls;
  model_segments(g, w, &Sg, &Ls);
  const long long Q = (static_cast<long long>(g.M / 2) * g.Gl + 63) / 64;
  const long long C = g.reflective ? 2 * Sg : Sg, R = g.reflective ? Q : 2 * Q;
  const long long P = n / T, rem = n % T;
  if (P == 0) return 1e300;
  const double tf = level_ns(T) * 1e-9, tl = 0.99 * tf, unit = static_cast<double>(Ls) * T / kw;
  const long long S = static_cast<long long>(occ) * g.cus;
  auto launch = [&](long long a) {  // seconds
    const long long W = a * R, full = W / S, part = W % S;
    double t = full * unit * tf * occ;
    if (part) {
      const long long per_cu = (part + g.cus - 1) / g.cus;  // workgroups on the busiest CU
      t += unit * (per_cu <= 1 ? tl : tf * per_cu);
    }
    return t + 5e-6;  // + launch
  };
  const long long m = std::min(P, C);
  double s = 0.0;
  for (long long a = 1; a < m; ++a) s += 2.0 * launch(a);  // fill and drain ramps
  s += static_cast<double>(std::max(P, C) - m + 1) * launch(m);
  if (rem) {
    const double step = static_cast<double>(R) * g.N * tf / (4.0 * g.cus);  // one step, every line, full load
    s += rem * 3.0 * step + 0.03;
  }
  return 1e3 * s;
}

struct Schedule {
  int T = 0, w = 0;
  double ms = 0.0;
};

static Schedule plan_schedule(const RunGeom &g, long long nsteps) {
  static const int kBlocks[] = {40, 32, 24, 20, 16, 8}, kWgs[] = {4, 8, 16, 32};
  Schedule best;
  for (int T : kBlocks)
    for (int w : kWgs) {
      const double ms = run_ms_model(g, nsteps, T, w);
      if (ms < 1e300 && (!best.T || ms < best.ms)) best = {T, w, ms};
    }
  return best;
}

static RunGeom run_geom(const rt_solver *s) {
  return RunGeom{s->p.N, s->p.M, s->Gl, s->cus, s->p.bc_left_indicator == 2};
}

extern "C" rt_status rt_plan_time_block(int ts_method, long long nsteps, int *steps_per_pass) {
  if (!steps_per_pass || nsteps < 0 || ts_method < 1 || ts_method > 3)
    return fail(nullptr, RT_ERR_ARG, "rt_plan_time_block: bad argument");
  *steps_per_pass = default_time_block(ts_method);
  if (ts_method == SCHEME_BDF2) {  // the SL slab's geometry on one MI355X: N = 1e6, S64, 128 groups, 256 CUs
    const Schedule sc = plan_schedule(RunGeom{1000000, 64, 128, 256, false}, nsteps);
    if (sc.T) *steps_per_pass = sc.T;
  }
  return RT_OK;
}

extern "C" rt_status rt_plan_schedule(rt_solver *s, long long nsteps, int *steps_per_pass, int *level_waves,
                                      int *wgs_per_cu, double *estimated_ms) {
  if (!s || nsteps < 0) return fail(s, RT_ERR_ARG, "rt_plan_schedule: bad argument");
  Schedule sc;
  if (s->scheme == SCHEME_BDF2) sc = plan_schedule(run_geom(s), nsteps);
  if (steps_per_pass) *steps_per_pass = sc.T ? sc.T : s->T;
  if (level_waves) *level_waves = sc.T ? 4 : s->level_waves;
  if (wgs_per_cu) *wgs_per_cu = sc.T ? sc.w : s->seg_wgs;
  if (estimated_ms) *estimated_ms = sc.T ? sc.ms : 0.0;
  return RT_OK;
}

static void solve_time_block(rt_solver *s) {
  if (s->scheme != SCHEME_BDF2 || s->Tpipe || s->queued || use_wavefront(s)) return;
  if (s->T_set || s->lw_set || s->seg_set) return;  // the caller chose (part of) the schedule
  const Schedule sc = plan_schedule(run_geom(s), s->p.max_timesteps);
  if (!sc.T) return;
  s->T = sc.T;
  s->level_waves = 4;
  s->seg_wgs = sc.w;
  s->planned = true;
}

extern "C" rt_status rt_solve(rt_solver *s) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_solve: NULL handle");
  solve_time_block(s);
  rt_status st = rt_advance(s, s->p.max_timesteps);
  if (st) return st;
  if ((st = complete(s))) return st;
  return rt_synchronize(s);
}

extern "C" void *rt_stream(rt_solver *s) { return s ? static_cast<void *>(s->stream) : nullptr; }

// ---------------------------------------------------------------------------
// material-temperature coupling (include/rtsn.h)
// ---------------------------------------------------------------------------
static rt_status compute_moments(rt_solver *s);

template <int S>
static rt_status unit_maps_s(rt_solver *s) {
  return line_maps_s<S>(s, true, s->map_unit, s->lc_unit);
}

static rt_status material_planck(rt_solver *s) {
  HIP_TRY(s, launch_planck_cells(s->pc, static_cast<const double *>(s->Tcell.p), static_cast<double *>(s->Bcell.p),
                                 s->stream));
  return RT_OK;
}

// dt W sum_g rho kappa_g dB_g/dT(T_max) / rho_cv over all G groups (rt_material_stability)
static double material_stability_number(const rt_solver *s, double T_max) {
  const int G = s->p.G;
  std::vector<double> lo(s->gt.e_edge.begin(), s->gt.e_edge.begin() + G), hi(s->gt.e_edge.begin() + 1,
                                                                             s->gt.e_edge.begin() + G + 1);
  std::vector<double> B(G, 0.0), dB(G, 0.0), mu(s->M_full), wt(s->M_full);
  if (T_max > 0.0) phys::PlanckIntegrator().group_integrals(T_max, G, lo.data(), hi.data(), B.data(), dB.data());
  phys::gauss_legendre(s->M_full, phys::kFourPi, mu.data(), wt.data());
  double W = 0.0, sum = 0.0;
  for (double w : wt) W += w;
  for (int g = 0; g < G; ++g) sum += s->gt.rho[g] * s->gt.kappa[g] * dB[g] * phys::kBoltzmannJPK;
  return s->p.dt * W * sum / s->rho_cv;
}

extern "C" rt_status rt_material_stability(rt_solver *s, double *number) {
  if (!s || !number) return fail(s, RT_ERR_ARG, "rt_material_stability: bad argument");
  if (!s->material) return fail(s, RT_ERR_STATE, "rt_material_stability: material coupling is off");
  HIP_TRY(s, hipSetDevice(s->device));
  std::vector<double> T(s->p.N);
  HIP_TRY(s, hipMemcpyAsync(T.data(), s->Tcell.p, sizeof(double) * T.size(), hipMemcpyDeviceToHost, s->stream));
  HIP_TRY(s, hipStreamSynchronize(s->stream));
  double T_max = 0.0;
  for (double t : T)
    if (std::isfinite(t)) T_max = std::max(T_max, t);
  *number = material_stability_number(s, T_max);
  return RT_OK;
}

extern "C" rt_status rt_material_enable(rt_solver *s, double rho_cv, const double *T_cells) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_material_enable: NULL handle");
  if (!(rho_cv > 0.0) || !std::isfinite(rho_cv)) return fail(s, RT_ERR_ARG, "rt_material_enable: rho_cv must be > 0");
  if (s->p.use_correction && s->p.V != 0.0)
    return fail(s, RT_ERR_PARAM, "material coupling needs the v/c correction off (V = 0 or use_correction = 0)");
  HIP_TRY(s, hipSetDevice(s->device));
  rt_status st = finalize(s);  // the state at the requested time, exact
  if (st) return st;
  const size_t N = s->p.N, NG = N * s->Gl;
  if (!s->Tcell.p) {
    hipError_t e = dalloc(s->Tcell, sizeof(double) * N);
    if (!e) e = dalloc(s->Bcell, sizeof(double) * NG);
    if (!e) e = dalloc(s->qbuf, sizeof(double) * N);
    if (!e) e = dalloc(s->edges, sizeof(double) * (s->p.G + 1));
    if (!e) e = dalloc(s->map_unit, s->map.bytes);
    if (!e) e = dalloc(s->lc_unit, s->lc.bytes);
    s->phi_fused = 64 % s->H == 0;  // a group's lines never straddle a wave
    if (!e && s->phi_fused) e = dalloc(s->phi_part, sizeof(double) * 4 * NG);  // [half sums, corrections][half]
    if (e) return fail(s, RT_ERR_NOMEM, std::string("material buffers: ") + hipGetErrorString(e));
  }
  switch (s->scheme) {
    case SCHEME_BE: st = unit_maps_s<SCHEME_BE>(s); break;
    case SCHEME_CN: st = unit_maps_s<SCHEME_CN>(s); break;
    default: st = unit_maps_s<SCHEME_BDF2>(s); break;
  }
  if (st) return st;
  {  // coupled passes are single steps: segments for the coupled kernel's occupancy
     // (measured on SL: 16 waves per CU instead is slower for BE, even for BDF2)
    int w = 0;
    HIP_TRY(s, coupled_occupancy(s->scheme, &w));
    if (const char *env = std::getenv("RTSN_WAVES_PER_CU")) w = std::atoi(env);
    const int sg0 = s->Sg;
    segment_lines(s, w);
    s->seg_T = 0;  // sized for the coupled pass
    s->seg_w = 0;
    if (s->Sg != sg0) {
      if (2LL * s->Q * s->Sg >= (1LL << 31)) return fail(s, RT_ERR_PARAM, "too many segments");
      HIP_TRY(s, alloc_segments(s));
      s->tau.assign(chain_positions(s), s->target);  // every position at the same, requested time
    }
  }
  std::vector<double> T0(N, s->p.T);
  if (T_cells) std::copy(T_cells, T_cells + N, T0.begin());
  if (s->phi_fused)  // the correction sums of segment-0 cells are never written: zero
    HIP_TRY(s, hipMemsetAsync(s->phi_part.p, 0, s->phi_part.bytes, s->stream));
  if ((st = upload(s, s->Tcell, T0.data(), N * sizeof(double)))) return st;
  if ((st = upload(s, s->edges, s->gt.e_edge.data(), (s->p.G + 1) * sizeof(double)))) return st;
  PlanckCells &pc = s->pc;
  phys::PlanckIntegrator().nodes(pc.node, pc.weight);
  pc.e_edge = static_cast<const double *>(s->edges.p);
  pc.G = s->p.G;
  pc.g_lo = s->g_lo;
  pc.Gl = s->Gl;
  pc.N = s->p.N;
  pc.a_c = phys::rad_a_long() * phys::kLight;
  pc.kcon = phys::kBoltzmannJPK;
  pc.accuracy = std::numeric_limits<double>::epsilon();
  s->wsum = 0.0;
  for (double w : s->wt) s->wsum += w;
  s->rho_cv = rho_cv;
  if ((st = material_planck(s))) return st;
  HIP_TRY(s, hipStreamSynchronize(s->stream));  // T0 dies at return
  s->material = true;
  double T_max = 0.0;
  for (double t : T0)
    if (std::isfinite(t)) T_max = std::max(T_max, t);
  const double number = material_stability_number(s, T_max);
  if (number > 2.0) {
    char msg[160];
    std::snprintf(msg, sizeof(msg), "explicit emission stability number %.4g > 2 at T_max = %.4g keV: "
                                    "reduce dt or raise rho_cv", number, T_max);
    return fail(s, RT_WARN_UNSTABLE, msg);
  }
  return RT_OK;
}

extern "C" rt_status rt_material_sweep(rt_solver *s, double *d_q) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_material_sweep: NULL handle");
  if (!s->material) return fail(s, RT_ERR_STATE, "rt_material_sweep: call rt_material_enable first");
  HIP_TRY(s, hipSetDevice(s->device));
  rt_status st = check_validation(s);
  if (st) return st;
  if ((st = ensure_equilibrium(s))) return st;
  double *q = d_q ? d_q : static_cast<double *>(s->qbuf.p);
  const double *B = static_cast<const double *>(s->Bcell.p), *sig = static_cast<const double *>(s->sigma.p);
  if (s->phi_fused) {
    // one pass over the state: the pass sums w psi of its provisional cells, the
    // correction kernel adds the cross-segment correction's share (no state
    // traffic) and the stored state keeps its correction pending for the next pass
    if ((st = complete(s))) return st;
    if ((st = enqueue_pass(s, 1, true))) return st;
    if (s->pending) {
      if ((st = enqueue_fold(s, 1, false))) return st;
      SegArgs a = seg_args(s);
      a.Gl = s->Gl;
      a.H = s->H;
      a.phic = static_cast<double *>(s->phi_part.p) + 2 * static_cast<size_t>(s->p.N) * s->Gl;
      a.wt = static_cast<const double *>(s->muwt.p) + s->p.M;
      // BE, CN: closed form, lanes over cells (phi_correction_geo_kernel); RTSN_PHI_WALK=1
      // keeps the walk for comparison
      const char *walk = std::getenv("RTSN_PHI_WALK");
      if (phi_correction_geo_supported(s->scheme, a) && !(walk && !std::strcmp(walk, "1"))) {
        HIP_TRY(s, launch_phi_correction_geo(s->scheme, a, s->stream));
        HIP_TRY(s, launch_material_q(static_cast<const double *>(s->phi_part.p), 4, B, sig, s->wsum, q, s->Gl,
                                     s->p.N, s->stream));
        return RT_OK;
      }
      // BDF2: closed form by tabulated rows (phi_correction_rows_kernel)
      if (phi_correction_rows_supported(s->scheme, a) && !(walk && !std::strcmp(walk, "1"))) {
        if (!s->corr_rows.p) {
          HIP_TRY(s, dalloc(s->corr_rows, sizeof(double) * corr_rows_doubles(s->scheme, s->Lpad)));
          HIP_TRY(s, launch_corr_rows(s->scheme, static_cast<const double *>(s->map.p),
                                      static_cast<double *>(s->corr_rows.p), s->Lpad, s->stream));
        }
        HIP_TRY(s, launch_phi_correction_rows(s->scheme, a, static_cast<const double *>(s->corr_rows.p), s->stream));
        HIP_TRY(s, launch_material_q(static_cast<const double *>(s->phi_part.p), 4, B, sig, s->wsum, q, s->Gl,
                                     s->p.N, s->stream));
        return RT_OK;
      }
      // the walk along a segment is a dependent chain: cut each segment into sub-segments
      // (multiples of 16 cells) until the grid holds ~8 waves per SIMD
      const long long segs = 2LL * s->Q * s->Sg;
      const int nsub = static_cast<int>(
          std::max<long long>(1, std::min<long long>((32LL * s->cus + segs - 1) / segs, s->Ls / 16)));
      const int Lsub = ((s->Ls + nsub - 1) / nsub + 15) / 16 * 16;
      if (nsub > 1 && s->corr_pow_L != Lsub) {
        if (!s->corr_pow.p) HIP_TRY(s, dalloc(s->corr_pow, sizeof(double) * 2 * tri_count(s->K) * s->Lpad));
        HIP_TRY(s, launch_correction_power(s->scheme, static_cast<const double *>(s->map.p),
                                           static_cast<double *>(s->corr_pow.p), Lsub, s->Lpad, s->stream));
        s->corr_pow_L = Lsub;
      }
      HIP_TRY(s, launch_phi_correction(s->scheme, a, nsub, Lsub, static_cast<const double *>(s->corr_pow.p),
                                       s->stream));
    }
    HIP_TRY(s, launch_material_q(static_cast<const double *>(s->phi_part.p), s->pending ? 4 : 2, B, sig, s->wsum, q,
                                 s->Gl, s->p.N, s->stream));
    return RT_OK;
  }
  if ((st = finalize(s))) return st;
  if ((st = enqueue_pass(s, 1, true))) return st;
  if ((st = compute_moments(s))) return st;  // finalizes the pass
  HIP_TRY(s, launch_material_q(static_cast<const double *>(s->mom.p), 1, B, sig, s->wsum, q, s->Gl, s->p.N,
                               s->stream));
  return RT_OK;
}

extern "C" rt_status rt_material_update(rt_solver *s, const double *d_q) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_material_update: NULL handle");
  if (!s->material) return fail(s, RT_ERR_STATE, "rt_material_update: call rt_material_enable first");
  HIP_TRY(s, hipSetDevice(s->device));
  HIP_TRY(s, launch_material_update(static_cast<double *>(s->Tcell.p), d_q ? d_q : static_cast<const double *>(s->qbuf.p),
                                    s->p.dt, s->rho_cv, s->p.N, s->stream));
  return material_planck(s);
}

extern "C" rt_status rt_material_step(rt_solver *s, int nsteps) {
  if (!s || nsteps < 0) return fail(s, RT_ERR_ARG, "rt_material_step: bad argument");
  if (s->g_lo != 0 || s->g_hi != s->p.G || s->d_hi > 0)
    return fail(s, RT_ERR_STATE, "rt_material_step: the handle holds a group or direction-pair shard; sum q "
                                 "over the shards (rt_material_sweep, all-reduce, rt_material_update)");
  for (int n = 0; n < nsteps; ++n) {
    rt_status st = rt_material_sweep(s, nullptr);
    if (st) return st;
    if ((st = rt_material_update(s, nullptr))) return st;
  }
  return RT_OK;
}

// which: 0 T(x), 1 B per cell
static rt_status material_fetch(rt_solver *s, int which, double *out, const char *what) {
  if (!s || !out) return fail(s, RT_ERR_ARG, std::string(what) + ": bad argument");
  if (!s->material) return fail(s, RT_ERR_STATE, std::string(what) + ": material coupling is off");
  HIP_TRY(s, hipSetDevice(s->device));
  const size_t count = which == 0 ? s->p.N : static_cast<size_t>(s->p.N) * s->Gl;
  const void *src = which == 0 ? s->Tcell.p : s->Bcell.p;
  HIP_TRY(s, hipMemcpyAsync(out, src, sizeof(double) * count, hipMemcpyDeviceToHost, s->stream));
  HIP_TRY(s, hipStreamSynchronize(s->stream));
  return RT_OK;
}

extern "C" rt_status rt_get_temperature(rt_solver *s, double *T_cells) {
  return material_fetch(s, 0, T_cells, "rt_get_temperature");
}

extern "C" rt_status rt_get_cell_planck(rt_solver *s, double *B) { return material_fetch(s, 1, B, "rt_get_cell_planck"); }

// ---------------------------------------------------------------------------
// results
// ---------------------------------------------------------------------------
extern "C" rt_status rt_get_dims(rt_solver *s, int *M, int *G_local, int *N, int *g_lo, int *g_hi) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_dims: NULL handle");
  if (M) *M = s->p.M;
  if (G_local) *G_local = s->Gl;
  if (N) *N = s->p.N;
  if (g_lo) *g_lo = s->g_lo;
  if (g_hi) *g_hi = s->g_hi;
  return RT_OK;
}

extern "C" rt_status rt_get_shard(rt_solver *s, int *G_total, int *M_total, int *g_lo, int *g_hi, int *d_lo,
                                  int *d_hi) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_shard: NULL handle");
  if (G_total) *G_total = s->p.G;
  if (M_total) *M_total = s->M_full;
  if (g_lo) *g_lo = s->g_lo;
  if (g_hi) *g_hi = s->g_hi;
  if (d_lo) *d_lo = s->d_hi > 0 ? s->d_lo : 0;
  if (d_hi) *d_hi = s->d_hi > 0 ? s->d_hi : s->M_full / 2;
  return RT_OK;
}

// The reference-layout transfers go through a bounded device buffer, a chunk of cells
// at a time (the layout's slowest index is the cell): kExportChunk doubles per node
// block, so rt_get_psi / rt_get_ends / rt_set_ends need ~0.5 GB of device memory beside
// the state instead of a full copy of it (65 / 131 GB on SL).
constexpr size_t kExportChunk = size_t(1) << 25;  // doubles

static int chunk_cells(const rt_solver *s) {
  const size_t per_cell = static_cast<size_t>(s->p.M) * s->Gl;
  size_t chunk = kExportChunk;
  if (const char *env = std::getenv("RTSN_EXPORT_CHUNK")) chunk = std::max(1L, std::atol(env));  // tests
  return static_cast<int>(std::max<size_t>(1, std::min<size_t>(s->p.N, chunk / per_cell)));
}

// Host side of the chunked transfers: two pinned staging buffers (the DMA engine reaches
// PCIe rate only from page-locked memory -- pageable copies measured 0.73 GB/s for psi)
// and the copy between staging and the caller's buffer split over host threads, so the
// copy of chunk i overlaps the device's export + DMA of chunk i + 1.
static rt_status ensure_staging(rt_solver *s, size_t bytes) {
  if (s->staging_bytes >= bytes) return RT_OK;
  (void)hipStreamSynchronize(s->stream);  // no transfer may still use the old pair
  for (int k = 0; k < 2; ++k) {
    ResourcePool::get().release(true, s->staging[k], s->staging_cap[k], 0);
    s->staging[k] = nullptr;
    s->staging_cap[k] = 0;
  }
  s->staging_bytes = 0;
  for (int k = 0; k < 2; ++k) HIP_TRY(s, ResourcePool::get().alloc(true, bytes, &s->staging[k], &s->staging_cap[k]));
  s->staging_bytes = std::min(s->staging_cap[0], s->staging_cap[1]);
  return RT_OK;
}

static void parallel_copy(double *dst, const double *src, size_t n) {
  const size_t nt = n < (size_t(1) << 20) ? 1 : std::max<size_t>(1, std::min<size_t>(16, std::thread::hardware_concurrency()));
  if (nt == 1) {
    std::memcpy(dst, src, n * sizeof(double));
    return;
  }
  std::vector<std::thread> pool;
  for (size_t t = 0; t < nt; ++t)
    pool.emplace_back([=] {
      const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
      std::memcpy(dst + lo, src + lo, (hi - lo) * sizeof(double));
    });
  for (std::thread &th : pool) th.join();
}

// Device -> pageable host through the pinned staging pair, kStagedPiece doubles at a time:
// the DMA of piece i + 1 overlaps the host copy of piece i.
constexpr size_t kStagedPiece = size_t(1) << 21;  // 16 MB
static rt_status staged_d2h(rt_solver *s, double *host, const double *dev, size_t count) {
  if (rt_status st = ensure_staging(s, sizeof(double) * std::min(count, kStagedPiece))) return st;
  size_t piece = std::min(kStagedPiece, s->staging_bytes / sizeof(double));
  if (const char *env = std::getenv("RTSN_EXPORT_CHUNK")) piece = std::min(piece, size_t(std::max(1L, std::atol(env))));  // tests
  hipError_t e = hipSuccess;
  size_t k = 0, prev = 0, prev_n = 0;
  for (size_t o = 0; o < count && e == hipSuccess; o += piece, ++k) {
    const size_t n = std::min(piece, count - o);
    e = hipMemcpyAsync(s->staging[k & 1], dev + o, sizeof(double) * n, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipEventRecord(s->staging_ev[k & 1], s->stream);
    if (e == hipSuccess && k > 0) {
      e = hipEventSynchronize(s->staging_ev[(k - 1) & 1]);
      if (e == hipSuccess) parallel_copy(host + prev, static_cast<const double *>(s->staging[(k - 1) & 1]), prev_n);
    }
    prev = o;
    prev_n = n;
  }
  if (e == hipSuccess && k > 0) {
    e = hipEventSynchronize(s->staging_ev[(k - 1) & 1]);
    if (e == hipSuccess) parallel_copy(host + prev, static_cast<const double *>(s->staging[(k - 1) & 1]), prev_n);
  }
  if (e != hipSuccess) return fail(s, RT_ERR_DEVICE, std::string("result transfer: ") + hipGetErrorString(e));
  return RT_OK;
}

// nodes: 1 (psi) or 2 (ends, node 0 then node 1 in the host layout, MGN apart)
template <typename F>
static rt_status export_chunks(rt_solver *s, int nodes, double *host, F &&launch) {
  const size_t MG = static_cast<size_t>(s->p.M) * s->Gl, MGN = MG * s->p.N;
  const int cc = chunk_cells(s);
  const size_t cap = static_cast<size_t>(nodes) * MG * cc;  // doubles per chunk
  if (rt_status st = ensure_staging(s, sizeof(double) * cap)) return st;
  DeviceBuf dbuf;
  HIP_TRY(s, dalloc(dbuf, sizeof(double) * cap));
  double *d = static_cast<double *>(dbuf.p);
  hipError_t e = hipSuccess;
  int prev_c0 = -1, prev_nc = 0, k = 0;
  auto drain = [&](int c0, int nc, const double *h) {  // staging -> caller, node blocks MGN apart
    const size_t n = MG * nc;
    for (int b = 0; b < nodes; ++b) parallel_copy(host + b * MGN + MG * c0, h + b * n, n);
  };
  for (int c0 = 0; c0 < s->p.N && e == hipSuccess; c0 += cc, ++k) {
    const int nc = std::min(cc, s->p.N - c0);
    double *h = static_cast<double *>(s->staging[k & 1]);
    e = launch(d, c0, nc);  // stream order: after the previous chunk's DMA out of d
    if (e == hipSuccess)
      e = hipMemcpyAsync(h, d, sizeof(double) * nodes * MG * nc, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipEventRecord(s->staging_ev[k & 1], s->stream);
    if (e == hipSuccess && prev_c0 >= 0) {  // the previous chunk, while this one is in flight
      e = hipEventSynchronize(s->staging_ev[(k - 1) & 1]);
      if (e == hipSuccess) drain(prev_c0, prev_nc, static_cast<const double *>(s->staging[(k - 1) & 1]));
    }
    prev_c0 = c0;
    prev_nc = nc;
  }
  if (e == hipSuccess && prev_c0 >= 0) {
    e = hipEventSynchronize(s->staging_ev[(k - 1) & 1]);
    if (e == hipSuccess) drain(prev_c0, prev_nc, static_cast<const double *>(s->staging[(k - 1) & 1]));
  }
  (void)hipStreamSynchronize(s->stream);  // d is released below
  dbuf.reset();
  if (e != hipSuccess) return fail(s, RT_ERR_DEVICE, std::string("result transfer: ") + hipGetErrorString(e));
  return RT_OK;
}

extern "C" rt_status rt_get_psi(rt_solver *s, double *psi) {
  if (!s || !psi) return fail(s, RT_ERR_ARG, "rt_get_psi: bad argument");
  HIP_TRY(s, hipSetDevice(s->device));
  if (rt_status st = finalize(s)) return st;
  const Geometry g = geometry(s);
  return export_chunks(s, 1, psi, [&](double *d, int c0, int nc) {
    return launch_export_psi(static_cast<const double2 *>(s->E.p), d, g, c0, nc, s->stream);
  });
}

extern "C" rt_status rt_get_ends(rt_solver *s, double *ends) {
  if (!s || !ends) return fail(s, RT_ERR_ARG, "rt_get_ends: bad argument");
  HIP_TRY(s, hipSetDevice(s->device));
  if (rt_status st = finalize(s)) return st;
  const Geometry g = geometry(s);
  return export_chunks(s, 2, ends, [&](double *d, int c0, int nc) {
    return launch_export_ends(static_cast<const double2 *>(s->E.p), d, g, c0, nc, s->stream);
  });
}

extern "C" rt_status rt_set_ends(rt_solver *s, const double *ends) {
  if (!s || !ends) return fail(s, RT_ERR_ARG, "rt_set_ends: bad argument");
  HIP_TRY(s, hipSetDevice(s->device));
  if (rt_status st = complete(s)) return st;  // requested steps happen before the state is replaced
  const Geometry g = geometry(s);
  const size_t MG = static_cast<size_t>(g.M) * g.Gl, MGN = MG * g.N;
  const int cc = chunk_cells(s);
  if (rt_status st = ensure_staging(s, sizeof(double) * 2 * MG * cc)) return st;
  DeviceBuf dbuf;
  HIP_TRY(s, dalloc(dbuf, sizeof(double) * 2 * MG * cc));
  double *d = static_cast<double *>(dbuf.p);
  hipError_t e = hipSuccess;
  int k = 0;
  for (int c0 = 0; c0 < g.N && e == hipSuccess; c0 += cc, ++k) {
    const int nc = std::min(cc, g.N - c0);
    const size_t n = MG * nc;
    double *h = static_cast<double *>(s->staging[k & 1]);
    if (k >= 2) e = hipEventSynchronize(s->staging_ev[k & 1]);  // its previous upload has left h
    for (int b = 0; b < 2 && e == hipSuccess; ++b) parallel_copy(h + b * n, ends + b * MGN + MG * c0, n);
    if (e == hipSuccess) e = hipMemcpyAsync(d, h, sizeof(double) * 2 * n, hipMemcpyHostToDevice, s->stream);
    if (e == hipSuccess) e = hipEventRecord(s->staging_ev[k & 1], s->stream);
    if (e == hipSuccess) e = launch_import_ends(static_cast<double2 *>(s->E.p), d, g, c0, nc, s->stream);
  }
  (void)hipStreamSynchronize(s->stream);  // d is released below
  dbuf.reset();
  ++s->state_version;
  if (e != hipSuccess)  // some chunks may hold the new cells, the rest the old ones
    return fail(s, RT_ERR_DEVICE, std::string("rt_set_ends: ") + hipGetErrorString(e) +
                                      " (the handle's state is undefined: load it again or destroy the handle)");
  s->pending = false;  // the loaded state is exact
  return RT_OK;
}

static rt_status compute_moments(rt_solver *s) {
  if (rt_status st = finalize(s)) return st;
  if (s->mom_version == s->state_version) return RT_OK;  // `mom` holds this state's moments
  const Geometry g = geometry(s);
  const size_t GN = static_cast<size_t>(s->Gl) * s->p.N;
  double *m = static_cast<double *>(s->mom.p);
  const double *muwt = static_cast<const double *>(s->muwt.p);
  HIP_TRY(s, launch_moments(static_cast<const double2 *>(s->E.p), muwt, muwt + s->p.M, m, m + GN, m + 2 * GN, g,
                            s->stream));
  s->mom_version = s->state_version;
  return RT_OK;
}

extern "C" rt_status rt_get_moments(rt_solver *s, double *phi, double *F, double *phi_plus) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_moments: NULL handle");
  HIP_TRY(s, hipSetDevice(s->device));
  rt_status st = compute_moments(s);
  if (st) return st;
  const size_t GN = static_cast<size_t>(s->Gl) * s->p.N;
  const double *m = static_cast<const double *>(s->mom.p);
  double *dst[3] = {phi, F, phi_plus};
  for (int k = 0; k < 3; ++k)
    if (dst[k])
      if (rt_status st2 = staged_d2h(s, dst[k], m + k * GN, GN)) return st2;
  return RT_OK;
}

extern "C" rt_status rt_get_moments_device(rt_solver *s, double *d_phi, double *d_F, double *d_phi_plus) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_moments_device: NULL handle");
  HIP_TRY(s, hipSetDevice(s->device));
  rt_status st = compute_moments(s);
  if (st) return st;
  const size_t GN = static_cast<size_t>(s->Gl) * s->p.N;
  const double *m = static_cast<const double *>(s->mom.p);
  double *dst[3] = {d_phi, d_F, d_phi_plus};
  for (int k = 0; k < 3; ++k)
    if (dst[k]) HIP_TRY(s, hipMemcpyAsync(dst[k], m + k * GN, sizeof(double) * GN, hipMemcpyDeviceToDevice, s->stream));
  return RT_OK;
}

// boundary rows: [0] half0 k=0, [1] half0 k=N-1, [2] half1 k=0, [3] half1 k=N-1
static rt_status fetch_rows(rt_solver *s, std::vector<double> &rows) {
  if (rt_status st = finalize(s)) return st;
  const Geometry g = geometry(s);
  rows.resize(static_cast<size_t>(8) * s->Lpad);
  HIP_TRY(s, launch_boundary_rows(static_cast<const double2 *>(s->E.p), static_cast<double2 *>(s->rows.p), g,
                                  s->stream));
  HIP_TRY(s, hipMemcpyAsync(rows.data(), s->rows.p, sizeof(double) * rows.size(), hipMemcpyDeviceToHost, s->stream));
  HIP_TRY(s, hipStreamSynchronize(s->stream));
  return RT_OK;
}

// physical ends(i, g, c, node) for c in {0, N-1} from the boundary rows
static double bnode(const rt_solver *s, const std::vector<double> &rows, int i, int gl, bool last_cell, int node) {
  const int H = s->H;
  if (i < H) {  // mu < 0: physical c = N-1-k; node 0 (left) = e_out
    const int ell = (H - 1 - i) + H * gl;
    const int which = last_cell ? 0 : 1;  // c = N-1 -> k = 0
    const double *r = rows.data() + static_cast<size_t>(2) * (static_cast<size_t>(which) * s->Lpad + ell);
    return node == 0 ? r[1] : r[0];
  }
  const int ell = (i - H) + H * gl;
  const int which = last_cell ? 3 : 2;
  const double *r = rows.data() + static_cast<size_t>(2) * (static_cast<size_t>(which) * s->Lpad + ell);
  return node == 0 ? r[0] : r[1];
}

extern "C" rt_status rt_get_group_ends(rt_solver *s, double *left, double *right) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_group_ends: NULL handle");
  HIP_TRY(s, hipSetDevice(s->device));
  std::vector<double> rows;
  rt_status st = fetch_rows(s, rows);
  if (st) return st;
  for (int gl = 0; gl < s->Gl; ++gl) {  // solver.cpp:826-850
    double l = 0., r = 0.;
    for (int i = 0; i < s->p.M; ++i) {
      if (s->mu[i] < 0.)
        l += bnode(s, rows, i, gl, false, 0);
      else
        r += bnode(s, rows, i, gl, true, 1);
    }
    const double den = s->gt.de_ave[s->g_lo + gl] * phys::kLight;
    if (left) left[gl] = l / den;
    if (right) right[gl] = r / den;
  }
  return RT_OK;
}

// compute_balance's absorption and emission sums per group (solver.cpp:262-272) on the
// device from the moments kernel's phi (N x Gl, g fastest): sequential within contiguous
// cell ranges, then over the ranges (balance_partials_kernel, balance_sums_kernel).
static rt_status balance_sums(rt_solver *s, std::vector<double> &ab, std::vector<double> &sr) {
  if (rt_status st = compute_moments(s)) return st;
  const int N = s->p.N, Gl = s->Gl;
  const double ac = phys::kRadA * phys::kLight, dx = s->p.X / N;
  std::vector<double> host(4 * static_cast<size_t>(Gl));  // rk, src | ab, sr
  for (int gl = 0; gl < Gl; ++gl) {
    host[gl] = s->gt.rho[s->g_lo + gl] * s->gt.kappa[s->g_lo + gl];
    host[Gl + gl] = host[gl] * ac * std::pow(s->p.T, 4) * dx;
  }
  DeviceBuf dbuf;
  HIP_TRY(s, dalloc(dbuf, sizeof(double) * (host.size() + balance_scratch_doubles(Gl))));
  double *d = static_cast<double *>(dbuf.p);
  hipError_t e = hipMemcpyAsync(d, host.data(), sizeof(double) * 2 * Gl, hipMemcpyHostToDevice, s->stream);
  if (e == hipSuccess)
    e = launch_balance_sums(static_cast<const double *>(s->mom.p), d, d + Gl, dx, d + host.size(), d + 2 * Gl,
                            d + 3 * Gl, Gl, N, s->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(host.data() + 2 * Gl, d + 2 * Gl, sizeof(double) * 2 * Gl, hipMemcpyDeviceToHost, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  (void)hipStreamSynchronize(s->stream);
  dbuf.reset();
  if (e != hipSuccess) return fail(s, RT_ERR_DEVICE, std::string("balance sums: ") + hipGetErrorString(e));
  ab.assign(host.begin() + 2 * Gl, host.begin() + 3 * Gl);
  sr.assign(host.begin() + 3 * Gl, host.end());
  return RT_OK;
}

extern "C" rt_status rt_get_balance_terms(rt_solver *s, double *balance, double *sources_out, double *sinks_out) {
  if (!s) return fail(s, RT_ERR_ARG, "rt_get_balance_terms: NULL handle");
  if (s->d_hi > 0)  // its emission/absorption terms need phi over all directions
    return fail(s, RT_ERR_PARAM, "rt_get_balance_terms: a direction shard holds part of phi; sum the shards' "
                                 "moments and group ends, then balance on the totals");
  HIP_TRY(s, hipSetDevice(s->device));
  const int Gl = s->Gl;
  std::vector<double> ab, sr, rows;
  rt_status st = balance_sums(s, ab, sr);
  if (st) return st;
  if ((st = fetch_rows(s, rows))) return st;
  for (int gl = 0; gl < Gl; ++gl) {  // solver.cpp:240-284
    double jhm = 0., jhp = 0., jNm = 0., jNp = 0.;
    for (int i = 0; i < s->p.M; ++i) {
      const double mu = s->mu[i];
      if (mu < 0.) {
        jhm -= bnode(s, rows, i, gl, false, 0) * mu * s->wt[i];
        jNm -= bnode(s, rows, i, gl, true, 0) * mu * s->wt[i];
      } else {
        jhp += bnode(s, rows, i, gl, false, 1) * mu * s->wt[i];
        jNp += bnode(s, rows, i, gl, true, 1) * mu * s->wt[i];
      }
    }
    const double sources = jhp + jNm + sr[gl], sinks = jNp + jhm + ab[gl];
    if (balance) balance[gl] = std::fabs(sinks - sources) / sources;
    if (sources_out) sources_out[gl] = sources;
    if (sinks_out) sinks_out[gl] = sinks;
  }
  return RT_OK;
}

// compute_balance's terms split by how they add over direction-pair shards: the
// boundary inflow currents (jhp + jNm), the outflow currents plus absorption (jNp + jhm
// + sum rho kappa phi dx: linear in psi, so the shards' partials sum to the total) and
// the emission sum (sum rho kappa a c T^4 dx: the same on every shard)
extern "C" rt_status rt_get_balance_partials(rt_solver *s, double *inflow, double *outflow_absorption,
                                             double *emission) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_balance_partials: NULL handle");
  HIP_TRY(s, hipSetDevice(s->device));
  const int Gl = s->Gl;
  std::vector<double> ab, sr, rows;
  rt_status st = balance_sums(s, ab, sr);
  if (st) return st;
  if ((st = fetch_rows(s, rows))) return st;
  for (int gl = 0; gl < Gl; ++gl) {
    double jin = 0., jout = 0.;
    for (int i = 0; i < s->p.M; ++i) {
      const double mu = s->mu[i];
      if (mu < 0.) {
        jout -= bnode(s, rows, i, gl, false, 0) * mu * s->wt[i];
        jin -= bnode(s, rows, i, gl, true, 0) * mu * s->wt[i];
      } else {
        jin += bnode(s, rows, i, gl, false, 1) * mu * s->wt[i];
        jout += bnode(s, rows, i, gl, true, 1) * mu * s->wt[i];
      }
    }
    if (inflow) inflow[gl] = jin;
    if (outflow_absorption) outflow_absorption[gl] = jout + ab[gl];
    if (emission) emission[gl] = sr[gl];
  }
  return RT_OK;
}

extern "C" rt_status rt_get_balance(rt_solver *s, double *balance) {
  if (!s || !balance) return fail(s, RT_ERR_ARG, "rt_get_balance: bad argument");
  return rt_get_balance_terms(s, balance, nullptr, nullptr);
}

extern "C" rt_status rt_get_e_ave(rt_solver *s, double *e_ave) {
  if (!s || !e_ave) return fail(s, RT_ERR_ARG, "rt_get_e_ave: bad argument");
  std::copy(s->gt.e_ave.begin(), s->gt.e_ave.end(), e_ave);
  return RT_OK;
}

extern "C" rt_status rt_get_group_data(rt_solver *s, double *e_edge, double *B, double *dBdT, double *kappa) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_group_data: NULL handle");
  if (e_edge) std::copy(s->gt.e_edge.begin(), s->gt.e_edge.end(), e_edge);
  if (B) std::copy(s->gt.B.begin(), s->gt.B.end(), B);
  if (dBdT) std::copy(s->gt.dBdT.begin(), s->gt.dBdT.end(), dBdT);
  if (kappa) std::copy(s->gt.kappa.begin(), s->gt.kappa.end(), kappa);
  return RT_OK;
}

extern "C" rt_status rt_get_quadrature(rt_solver *s, double *mu, double *wt) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_quadrature: NULL handle");
  if (mu) std::copy(s->mu.begin(), s->mu.end(), mu);
  if (wt) std::copy(s->wt.begin(), s->wt.end(), wt);
  return RT_OK;
}

extern "C" rt_status rt_get_psi_source(rt_solver *s, double *out) {
  if (!s || !out) return fail(s, RT_ERR_ARG, "rt_get_psi_source: bad argument");
  std::copy(s->psi_source.begin(), s->psi_source.end(), out);
  return RT_OK;
}

extern "C" rt_status rt_group_absorption_device(rt_solver *s, double *d_out) {
  if (!s || !d_out) return fail(s, RT_ERR_ARG, "rt_group_absorption_device: bad argument");
  HIP_TRY(s, hipSetDevice(s->device));
  rt_status st = compute_moments(s);
  if (st) return st;
  HIP_TRY(s, launch_group_absorption(static_cast<const double *>(s->mom.p), static_cast<const double *>(s->sigma.p),
                                     d_out, geometry(s), s->stream));
  return RT_OK;
}

extern "C" rt_status rt_state_finite(rt_solver *s, int *finite) {
  if (!s || !finite) return fail(s, RT_ERR_ARG, "rt_state_finite: bad argument");
  HIP_TRY(s, hipSetDevice(s->device));
  rt_status st = finalize(s);  // the state at the requested time, exact
  if (st) return st;
  int *flag = static_cast<int *>(s->rows.p);  // scratch: the boundary-row buffer
  HIP_TRY(s, hipMemsetAsync(flag, 0, sizeof(int), s->stream));
  HIP_TRY(s, launch_finite_scan(static_cast<const double2 *>(s->E.p), flag, geometry(s), s->stream));
  int h = 0;
  HIP_TRY(s, hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, s->stream));
  HIP_TRY(s, hipStreamSynchronize(s->stream));
  *finite = h ? 0 : 1;
  return RT_OK;
}

extern "C" rt_status rt_set_profiling(rt_solver *s, int on) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_profiling: NULL handle");
  rt_status st = fold_events(s);
  if (st) return st;
  s->profiling = on != 0;
  s->sweep_ms = 0.0;
  s->profiled = 0;
  if (s->profiling && s->ev_pool.empty()) {
    HIP_TRY(s, hipSetDevice(s->device));
    s->ev_pool.resize(256, nullptr);
    for (hipEvent_t &e : s->ev_pool) HIP_TRY(s, ResourcePool::get().event(true, &e));
  }
  return RT_OK;
}

extern "C" rt_status rt_get_sweep_time(rt_solver *s, double *total_ms, long long *launches) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_sweep_time: NULL handle");
  rt_status st = fold_events(s);
  if (st) return st;
  if (total_ms) *total_ms = s->sweep_ms;
  if (launches) *launches = s->profiled;
  return RT_OK;
}

extern "C" rt_status rt_sweep_traffic(rt_solver *s, double *bytes_per_launch, double *updates_per_step) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_sweep_traffic: NULL handle");
  const double lines_cells = static_cast<double>(s->p.M) * s->Gl * s->p.N;
  // one pass (of T steps): read (e_in, e_out) and write them back, per cell x line
  if (bytes_per_launch) *bytes_per_launch = 32.0 * lines_cells;
  if (updates_per_step) *updates_per_step = (s->p.ts_method == 3 ? 4.0 : 1.0) * lines_cells;
  return RT_OK;
}

extern "C" rt_status rt_sweep_flops(rt_solver *s, double *flops_per_launch) {
  if (!s || !flops_per_launch) return fail(s, RT_ERR_ARG, "rt_sweep_flops: bad argument");
  // one FMA per structural coefficient of the cell map (cell.hpp): the
  // affine constants are the accumulators' initial values, not extra ops
  const int rows = s->K + 1 - (s->scheme == SCHEME_BE ? 0 : 1);
  const double fma = static_cast<double>(map_count_of(s->scheme) - rows);
  *flops_per_launch = 2.0 * fma * s->T * static_cast<double>(s->p.M) * s->Gl * s->p.N;
  return RT_OK;
}

extern "C" rt_status rt_set_pipeline(rt_solver *s, int on) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_pipeline: NULL handle");
  HIP_TRY(s, hipSetDevice(s->device));
  if (on < 0 || on > 2) return fail(s, RT_ERR_ARG, "rt_set_pipeline: 0 (off), 1 (auto) or 2 (always)");
  if (!on && s->pipe) {
    if (rt_status st = complete(s)) return st;  // leave the positions aligned
  }
  s->pipe = on;
  s->pipe_set = true;
  s->planned = false;
  return RT_OK;
}

extern "C" rt_status rt_set_wavefront(rt_solver *s, int mode) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_wavefront: NULL handle");
  if (mode < 0 || mode > 2) return fail(s, RT_ERR_ARG, "rt_set_wavefront: 0 (off), 1 (auto) or 2 (on)");
  s->wave = mode;
  return RT_OK;
}

extern "C" rt_status rt_get_wavefront(rt_solver *s, int *mode, int *active, int *cells_per_lane) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_wavefront: NULL handle");
  if (mode) *mode = s->wave;
  if (active) *active = use_wavefront(s) ? 1 : 0;
  if (cells_per_lane) *cells_per_lane = wave_plan(s).C;
  return RT_OK;
}

extern "C" rt_status rt_set_wavefront_waves(rt_solver *s, int max_waves) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_wavefront_waves: NULL handle");
  if (max_waves < 1 || max_waves > kWaveMaxWaves) return fail(s, RT_ERR_ARG, "rt_set_wavefront_waves: 1..8 waves");
  s->wave_max = max_waves;
  return RT_OK;
}

extern "C" rt_status rt_get_wavefront_waves(rt_solver *s, int *max_waves, int *waves_per_chain) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_get_wavefront_waves: NULL handle");
  if (max_waves) *max_waves = s->wave_max;
  if (waves_per_chain) *waves_per_chain = wave_plan(s).waves;
  return RT_OK;
}

extern "C" rt_status rt_pipeline_state(rt_solver *s, long long *lag_steps, int *queued_steps, int *pending) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_pipeline_state: NULL handle");
  if (lag_steps) *lag_steps = s->tau.front() - s->tau.back();
  if (queued_steps) *queued_steps = s->queued;
  if (pending) *pending = s->pending ? 1 : 0;
  return RT_OK;
}

extern "C" rt_status rt_get_pipeline(rt_solver *s, int *on) {
  if (!s || !on) return fail(s, RT_ERR_ARG, "rt_get_pipeline: bad argument");
  *on = s->pipe;
  return RT_OK;
}

extern "C" rt_status rt_set_time_block(rt_solver *s, int steps_per_pass) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_time_block: NULL handle");
  if (!supported_time_block(steps_per_pass))
    return fail(s, RT_ERR_ARG, "rt_set_time_block: steps per pass must be 1..8, 10, 12, 16, 20, 24, 32 or 40");
  HIP_TRY(s, hipSetDevice(s->device));
  s->T = steps_per_pass;
  s->T_set = true;
  s->planned = false;
  return resegment(s);  // now if the positions are aligned, else when they next are
}

extern "C" rt_status rt_get_time_block(rt_solver *s, int *steps_per_pass) {
  if (!s || !steps_per_pass) return fail(s, RT_ERR_ARG, "rt_get_time_block: bad argument");
  *steps_per_pass = s->T;
  return RT_OK;
}

extern "C" rt_status rt_set_level_waves(rt_solver *s, int waves) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_level_waves: NULL handle");
  if (waves < 0 || waves > 4 || waves == 3) return fail(s, RT_ERR_PARAM, "rt_set_level_waves: 0 (auto), 1, 2 or 4");
  s->level_waves = waves;  // segments re-sized for its occupancy before the next pass (the schedule is exact
  s->lw_set = true;        // for any segmentation)
  s->planned = false;
  if (rt_status st = resegment(s)) return st;
  return RT_OK;
}

extern "C" rt_status rt_set_segmentation(rt_solver *s, int wgs_per_cu) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_segmentation: NULL handle");
  if (wgs_per_cu < 0 || wgs_per_cu > 64) return fail(s, RT_ERR_ARG, "rt_set_segmentation: 0 (occupancy) .. 64");
  HIP_TRY(s, hipSetDevice(s->device));
  s->seg_wgs = wgs_per_cu;
  s->seg_set = true;
  s->planned = false;
  return resegment(s);  // now if the positions are aligned, else before the next pass
}

extern "C" rt_status rt_get_level_waves(rt_solver *s, int *waves) {
  if (!s || !waves) return fail(s, RT_ERR_ARG, "rt_get_level_waves: bad argument");
  *waves = level_waves_of(s, s->T);  // the effective choice for the current time block
  return RT_OK;
}

extern "C" rt_status rt_sweep_geometry(rt_solver *s, int *workgroups, long long *tiles) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_sweep_geometry: NULL handle");
  if (workgroups) *workgroups = 2 * s->Q * s->Sg;  // one 64-lane wave per (line group, segment)
  if (tiles) *tiles = s->Sg;                        // segments per line
  return RT_OK;
}

extern "C" const char *rt_status_string(rt_status st) {
  switch (st) {
    case RT_OK: return "ok";
    case RT_ERR_IO: return "io error";
    case RT_ERR_PARSE: return "parse error";
    case RT_ERR_PARAM: return "invalid parameter";
    case RT_ERR_VALIDATION: return "correction validation failed";
    case RT_ERR_NOMEM: return "out of memory";
    case RT_ERR_DEVICE: return "device error";
    case RT_ERR_TIMEOUT: return "timeout (reserved)";
    case RT_ERR_ARG: return "bad argument";
    case RT_ERR_STATE: return "not valid in the handle's mode";
    case RT_WARN_UNSTABLE: return "warning: explicit emission above its stability limit";
  }
  return "unknown";
}

extern "C" const char *rt_last_error(rt_solver *s) { return s ? s->err.c_str() : g_last_error.c_str(); }
