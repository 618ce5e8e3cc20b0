// rtsn_material.hip -- material-temperature coupling (include/rtsn.h "material"):
// per-cell Planck emission and its T derivative, the coupled sweep with fused angular sums,
// the T update implicit in the material's own emission and the owed emission it implies.

#include "rtsn_internal.hpp"

using namespace rtamd;
using namespace rtsn_detail;

// ---------------------------------------------------------------------------
// material-temperature coupling (include/rtsn.h)
// ---------------------------------------------------------------------------

template <int S>
static rt_status unit_maps_s(rt_solver *s) {
  return line_maps_s<S>(s, true, s->map_unit, s->hmap_unit);
}

static rt_status material_planck(rt_solver *s) {
  HIP_TRY(s, launch_planck_cells(s->pc, static_cast<const double *>(s->Tcell.p), static_cast<double *>(s->Bcell.p),
                                 s->stream));
  return RT_OK;
}

// dt W sum_g rho kappa_g dB_g/dT(T_max) / rho_cv over all G groups (rt_material_stability): the
// emission's stiffness at the hottest cell, 1 / (1 + number) the Fleck factor there
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
    if (!e) e = dalloc(s->Beff, sizeof(double) * NG);
    if (!e) e = dalloc(s->owed, sizeof(double) * NG);
    if (!e) e = dalloc(s->dBcell, sizeof(double) * NG);
    if (!e) e = dalloc(s->dTlast, sizeof(double) * N);
    if (!e) e = dalloc(s->bpart, sizeof(double) * N);
    if (!e) e = dalloc(s->qbuf, sizeof(double) * 2 * N);
    if (!e) e = dalloc(s->edges, sizeof(double) * (s->p.G + 1));
    if (!e) e = dalloc(s->sigma_all, sizeof(double) * s->p.G);
    if (!e) e = dalloc(s->map_unit, s->map.bytes);
    if (!e) e = dalloc(s->hmap_unit, s->hmap.bytes);
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
     // (measured on SL: 16 waves per CU instead is slower for BE, even for BDF2), or the
     // caller's rt_set_segmentation
    int w = 0;
    HIP_TRY(s, coupled_occupancy(s->scheme, &w));
    if (s->seg_set && s->seg_wgs) w = s->seg_wgs;
    const int sg0 = s->Sg;
    segment_lines(s, w);
    s->seg_T = 0;  // sized for the coupled pass
    s->seg_w = 0;
    if (s->Sg != sg0) {
      if (2LL * s->Q * s->Sg >= (1LL << 31)) return fail(s, RT_ERR_PARAM, "too many segments");
      HIP_TRY(s, alloc_segments(s));
      s->tau.assign(chain_positions(s), s->target);  // every position at the same, requested time
      s->resume_lo = s->resume_hi = -1;
    }
  }
  std::vector<double> T0(N, s->p.T);
  if (T_cells) std::copy(T_cells, T_cells + N, T0.begin());
  if (s->phi_fused)  // the correction sums of segment-0 cells are never written: zero
    HIP_TRY(s, hipMemsetAsync(s->phi_part.p, 0, s->phi_part.bytes, s->stream));
  if ((st = upload(s, s->Tcell, T0.data(), N * sizeof(double)))) return st;
  HIP_TRY(s, hipMemsetAsync(s->dTlast.p, 0, sizeof(double) * N, s->stream));  // nothing owed yet
  HIP_TRY(s, hipMemsetAsync(s->owed.p, 0, sizeof(double) * NG, s->stream));
  HIP_TRY(s, hipMemsetAsync(s->dBcell.p, 0, sizeof(double) * NG, s->stream));
  if ((st = upload(s, s->edges, s->gt.e_edge.data(), (s->p.G + 1) * sizeof(double)))) return st;
  {
    std::vector<double> sig(s->p.G);
    for (int g = 0; g < s->p.G; ++g) sig[g] = s->gt.rho[g] * s->gt.kappa[g];
    if ((st = upload(s, s->sigma_all, sig.data(), sig.size() * sizeof(double)))) return st;
  }
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
  pc.sigma = static_cast<const double *>(s->sigma.p);
  pc.dTlast = static_cast<const double *>(s->dTlast.p);
  pc.owed = static_cast<double *>(s->owed.p);
  pc.dB = static_cast<double *>(s->dBcell.p);
  pc.Beff = static_cast<double *>(s->Beff.p);
  pc.bpart = static_cast<double *>(s->bpart.p);
  pc.b_scale = s->d_lo == 0 ? 1.0 : 0.0;  // direction shards: every one holds all groups, count b once
  pc.sigma_all = static_cast<const double *>(s->sigma_all.p);
  pc.Bcell = static_cast<const double *>(s->Bcell.p);
  s->wsum = 0.0;
  for (double w : s->wt) s->wsum += w;
  {
    std::vector<double> mu_all(s->M_full), wt_all(s->M_full);
    phys::gauss_legendre(s->M_full, phys::kFourPi, mu_all.data(), wt_all.data());
    s->wsum_all = 0.0;
    for (double w : wt_all) s->wsum_all += w;
  }
  s->rho_cv = rho_cv;
  if ((st = material_planck(s))) return st;
  HIP_TRY(s, hipStreamSynchronize(s->stream));  // T0 dies at return
  s->material = true;
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
  const double *bp = static_cast<const double *>(s->bpart.p);
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
      // BE, CN: closed form, lanes over cells (phi_correction_geo_kernel); rt_set_phi_correction_form
      // 1 keeps the walk for comparison
      const bool walk = s->phi_corr_form == 1;
      if (phi_correction_geo_supported(s->scheme, a) && !walk) {
        HIP_TRY(s, launch_phi_correction_geo(s->scheme, a, s->stream));
        HIP_TRY(s, launch_material_q(static_cast<const double *>(s->phi_part.p), 4, B, sig, s->wsum, bp, q, s->Gl,
                                     s->p.N, s->stream));
        return RT_OK;
      }
      // BDF2: closed form by tabulated rows (phi_correction_rows_kernel)
      if (phi_correction_rows_supported(s->scheme, a) && !walk) {
        if (!s->corr_rows.p) {
          HIP_TRY(s, dalloc(s->corr_rows, sizeof(double) * corr_rows_doubles(s->scheme, s->Lpad)));
          HIP_TRY(s, launch_corr_rows(s->scheme, static_cast<const double *>(s->map.p),
                                      static_cast<double *>(s->corr_rows.p), s->Lpad, s->stream));
        }
        HIP_TRY(s, launch_phi_correction_rows(s->scheme, a, static_cast<const double *>(s->corr_rows.p), s->stream));
        HIP_TRY(s, launch_material_q(static_cast<const double *>(s->phi_part.p), 4, B, sig, s->wsum, bp, q, s->Gl,
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
    HIP_TRY(s, launch_material_q(static_cast<const double *>(s->phi_part.p), s->pending ? 4 : 2, B, sig, s->wsum, bp,
                                 q, s->Gl, s->p.N, s->stream));
    return RT_OK;
  }
  if ((st = finalize(s))) return st;
  if ((st = enqueue_pass(s, 1, true))) return st;
  if ((st = compute_moments(s))) return st;  // finalizes the pass
  HIP_TRY(s, launch_material_q(static_cast<const double *>(s->mom.p), 1, B, sig, s->wsum, bp, q, s->Gl, s->p.N,
                               s->stream));
  return RT_OK;
}

extern "C" rt_status rt_material_update(rt_solver *s, const double *d_q) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_material_update: NULL handle");
  if (!s->material) return fail(s, RT_ERR_STATE, "rt_material_update: call rt_material_enable first");
  HIP_TRY(s, hipSetDevice(s->device));
  HIP_TRY(s, launch_material_update(s->pc, static_cast<double *>(s->Tcell.p),
                                    d_q ? d_q : static_cast<const double *>(s->qbuf.p),
                                    static_cast<double *>(s->dTlast.p), s->p.dt, s->rho_cv, s->wsum_all, s->p.N,
                                    s->stream));
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

// which: 0 T(x), 1 B per cell, 2 the next step's emission per cell
static rt_status material_fetch(rt_solver *s, int which, double *out, const char *what) {
  if (!s || !out) return fail(s, RT_ERR_ARG, std::string(what) + ": bad argument");
  if (!s->material) return fail(s, RT_ERR_STATE, std::string(what) + ": material coupling is off");
  HIP_TRY(s, hipSetDevice(s->device));
  const size_t count = which == 0 ? s->p.N : static_cast<size_t>(s->p.N) * s->Gl;
  const void *src = which == 0 ? s->Tcell.p : (which == 1 ? s->Bcell.p : s->Beff.p);
  HIP_TRY(s, hipMemcpyAsync(out, src, sizeof(double) * count, hipMemcpyDeviceToHost, s->stream));
  HIP_TRY(s, hipStreamSynchronize(s->stream));
  return RT_OK;
}

extern "C" rt_status rt_get_temperature(rt_solver *s, double *T_cells) {
  return material_fetch(s, 0, T_cells, "rt_get_temperature");
}

extern "C" rt_status rt_get_cell_planck(rt_solver *s, double *B) { return material_fetch(s, 1, B, "rt_get_cell_planck"); }

extern "C" rt_status rt_get_cell_emission(rt_solver *s, double *Beff) {
  return material_fetch(s, 2, Beff, "rt_get_cell_emission");
}

extern "C" rt_status rt_get_material_transit(rt_solver *s, double *E) {
  if (!s || !E) return fail(s, RT_ERR_ARG, "rt_get_material_transit: bad argument");
  if (!s->material) return fail(s, RT_ERR_STATE, "rt_get_material_transit: material coupling is off");
  HIP_TRY(s, hipSetDevice(s->device));
  DeviceBuf d;
  HIP_TRY(s, dalloc(d, sizeof(double) * s->p.N));
  hipError_t e = launch_material_transit(static_cast<const double *>(s->Bcell.p), static_cast<const double *>(s->Beff.p),
                                         static_cast<const double *>(s->owed.p), static_cast<const double *>(s->sigma.p),
                                         s->p.dt * s->wsum, static_cast<double *>(d.p), s->Gl, s->p.N, s->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(E, d.p, sizeof(double) * s->p.N, hipMemcpyDeviceToHost, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  (void)hipStreamSynchronize(s->stream);
  d.reset();
  if (e != hipSuccess) return fail(s, RT_ERR_DEVICE, std::string("rt_get_material_transit: ") + hipGetErrorString(e));
  return RT_OK;
}
