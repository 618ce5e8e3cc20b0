// rtsn_api.hip -- the C ABI entry points of include/rtsn.h that configure a handle: parameters,
// lifecycle (rt_create* / rt_destroy), schedule setters and getters, status strings and
// the last-error text.  Stepping lives in rtsn_schedule.hip, per-line setup in
// rtsn_lines.hip, read-outs in rtsn_readout.hip, the material coupling in rtsn_material.hip,
// the handle resource cache in rtsn_internal.hpp.

#include "rtsn_internal.hpp"

using namespace rtamd;
using namespace rtsn_detail;

namespace {
thread_local std::string g_last_error;
}  // namespace

rt_status rtsn_detail::fail(rt_solver *s, rt_status st, const std::string &msg) {
  if (s) s->err = msg;
  g_last_error = msg;
  return st;
}

// for the host-only units (comm_layout.cpp): the thread's last-error text (rt_last_error(NULL))
void rtsn_detail::set_last_error(const char *msg) { g_last_error = msg ? msg : ""; }

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
  // the time block, wavefront use, waves per chain and level split are the caller's (rt_set_*);
  // no environment variable changes them (round 5: the experiment overrides were removed)
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
  if (!e) e = dalloc(h->hmap, sizeof(double) * map_count_of(h->scheme) * Lp);
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
  // no host wait: the setup copies leave from the handle's pinned arena and every later call
  // is ordered after them on the stream (round 5: the create of llnl_slab_test made five
  // host round trips here and in the uploads)
  HIP_TRY(h, hipGetLastError());
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

extern "C" rt_status rt_set_pipeline(rt_solver *s, int on) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_pipeline: NULL handle");
  HIP_TRY(s, hipSetDevice(s->device));
  if (on < 0 || on > 2) return fail(s, RT_ERR_ARG, "rt_set_pipeline: 0 (off), 1 (auto) or 2 (always)");
  if (!on && s->pipe) {
    if (rt_status st = complete(s)) return st;  // leave the positions aligned
  }
  s->pipe = on;
  s->pipe_set = true;
  end_plan(s);  // a planned run's schedule gives way to the caller's
  return RT_OK;
}

extern "C" rt_status rt_set_wavefront(rt_solver *s, int mode) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_wavefront: NULL handle");
  if (mode < 0 || mode > 2) return fail(s, RT_ERR_ARG, "rt_set_wavefront: 0 (off), 1 (auto) or 2 (on)");
  if (s->wqueued) {  // steps queued for the current chain plan run on it first
    HIP_TRY(s, hipSetDevice(s->device));
    if (rt_status st = wave_flush(s)) return st;
  }
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
  if (s->wqueued) {  // steps queued for the current chain plan run on it first
    HIP_TRY(s, hipSetDevice(s->device));
    if (rt_status st = wave_flush(s)) return st;
  }
  s->wave_max = max_waves;
  return RT_OK;
}

extern "C" rt_status rt_set_wavefront_cells(rt_solver *s, int cells_per_lane) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_wavefront_cells: NULL handle");
  if (cells_per_lane != 0 && cells_per_lane != 1 && cells_per_lane != 2 && cells_per_lane != 4 && cells_per_lane != 8)
    return fail(s, RT_ERR_ARG, "rt_set_wavefront_cells: 0 (the plan's), 1, 2, 4 or 8");
  if (s->wqueued) {  // steps queued for the current chain plan run on it first
    HIP_TRY(s, hipSetDevice(s->device));
    if (rt_status st = wave_flush(s)) return st;
  }
  s->wave_cells = cells_per_lane;
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
  if (queued_steps)  // s->tail: a remainder block still owed by an interrupted drain (complete)
    *queued_steps = static_cast<int>(std::min<long long>(s->queued + s->wqueued + s->tail, INT32_MAX));
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
  end_plan(s);  // a planned run's schedule gives way to the caller's
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
  HIP_TRY(s, hipSetDevice(s->device));
  s->level_waves = waves;  // segments re-sized for its occupancy before the next pass (the schedule is exact
  s->lw_set = true;        // for any segmentation)
  end_plan(s);  // a planned run's schedule gives way to the caller's
  if (rt_status st = resegment(s)) return st;
  return RT_OK;
}

extern "C" rt_status rt_set_segmentation(rt_solver *s, int wgs_per_cu) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_segmentation: NULL handle");
  if (wgs_per_cu < 0 || wgs_per_cu > 64) return fail(s, RT_ERR_ARG, "rt_set_segmentation: 0 (occupancy) .. 64");
  HIP_TRY(s, hipSetDevice(s->device));
  s->seg_wgs = wgs_per_cu;
  s->seg_set = true;
  end_plan(s);  // a planned run's schedule gives way to the caller's
  return resegment(s);  // now if the positions are aligned, else before the next pass
}

extern "C" rt_status rt_get_level_waves(rt_solver *s, int *waves) {
  if (!s || !waves) return fail(s, RT_ERR_ARG, "rt_get_level_waves: bad argument");
  *waves = level_waves_of(s, s->T);  // the effective choice for the current time block
  return RT_OK;
}

extern "C" rt_status rt_set_moments_form(rt_solver *s, int form) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_moments_form: NULL handle");
  if (form != 0 && form != 1) return fail(s, RT_ERR_ARG, "rt_set_moments_form: 0 (one wave) or 1 (producer/consumer)");
  s->moments_form = form;
  s->mom_version = 0;  // the next read-out runs the chosen kernel
  return RT_OK;
}

extern "C" rt_status rt_set_phi_correction_form(rt_solver *s, int form) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_set_phi_correction_form: NULL handle");
  if (form != 0 && form != 1) return fail(s, RT_ERR_ARG, "rt_set_phi_correction_form: 0 (closed forms) or 1 (walk)");
  s->phi_corr_form = form;
  return RT_OK;
}

extern "C" rt_status rt_debug_fail_launch(rt_solver *s, int after) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_debug_fail_launch: NULL handle");
  if (after < -1) return fail(s, RT_ERR_ARG, "rt_debug_fail_launch: -1 (off) or launches before the failure");
  s->fail_launch_after = after;
  return RT_OK;
}

extern "C" rt_status rt_debug_set_transfer_chunk(rt_solver *s, long long doubles) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_debug_set_transfer_chunk: NULL handle");
  if (doubles < 0) return fail(s, RT_ERR_ARG, "rt_debug_set_transfer_chunk: 0 (default) or doubles per piece");
  s->transfer_chunk = doubles;
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
    case RT_ERR_TIMEOUT: return "timeout (communicator aborted)";
    case RT_ERR_ARG: return "bad argument";
    case RT_ERR_STATE: return "not valid in the handle's mode";
    case RT_WARN_UNSTABLE: return "warning: explicit emission above its stability limit";
  }
  return "unknown";
}

extern "C" const char *rt_last_error(rt_solver *s) { return s ? s->err.c_str() : g_last_error.c_str(); }
