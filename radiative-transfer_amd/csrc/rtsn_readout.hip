// rtsn_readout.hip -- read-outs in the reference's layouts (psi, ends, moments, group ends,
// compute_balance), the chunked pinned-staging transfers, the finite scan and profiling.

#include "rtsn_internal.hpp"

using namespace rtamd;
using namespace rtsn_detail;

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
  if (s->transfer_chunk > 0) chunk = static_cast<size_t>(s->transfer_chunk);  // rt_debug_set_transfer_chunk
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
  if (s->transfer_chunk > 0) piece = std::min(piece, static_cast<size_t>(s->transfer_chunk));  // rt_debug_set_transfer_chunk
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

rt_status rtsn_detail::compute_moments(rt_solver *s) {
  if (rt_status st = finalize(s)) return st;
  if (s->mom_version == s->state_version) return RT_OK;  // `mom` holds this state's moments
  const Geometry g = geometry(s);
  const size_t GN = static_cast<size_t>(s->Gl) * s->p.N;
  double *m = static_cast<double *>(s->mom.p);
  const double *muwt = static_cast<const double *>(s->muwt.p);
  HIP_TRY(s, launch_moments(static_cast<const double2 *>(s->E.p), muwt, muwt + s->p.M, m, m + GN, m + 2 * GN, g,
                            s->moments_form, s->stream));
  s->mom_version = s->state_version;
  ++s->mom_serial;
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
  if (3 * GN <= kStagedPiece && s->transfer_chunk == 0) {  // the three fields ([3][GN] in `mom`) in one transfer, once per state
    if (s->mom_host_serial != s->mom_serial) {
      if (s->mom_host_cap < sizeof(double) * 3 * GN) {
        ResourcePool::get().release(true, s->mom_host, s->mom_host_cap, 0);
        s->mom_host = nullptr;
        s->mom_host_cap = 0;
        HIP_TRY(s, ResourcePool::get().alloc(true, sizeof(double) * 3 * GN, &s->mom_host, &s->mom_host_cap));
      }
      HIP_TRY(s, hipMemcpyAsync(s->mom_host, m, sizeof(double) * 3 * GN, hipMemcpyDeviceToHost, s->stream));
      HIP_TRY(s, hipEventRecord(s->staging_ev[0], s->stream));
      HIP_TRY(s, hipEventSynchronize(s->staging_ev[0]));
      s->mom_host_serial = s->mom_serial;
    }
    for (int k = 0; k < 3; ++k)
      if (dst[k]) std::memcpy(dst[k], static_cast<const double *>(s->mom_host) + k * GN, sizeof(double) * GN);
    return RT_OK;
  }
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
// (through the pinned staging pair: a copy into pageable memory makes the runtime pin a
// staging buffer of its own, ~18 ms on the first read-out of a process, r06g)
static rt_status fetch_rows(rt_solver *s, std::vector<double> &rows) {
  if (rt_status st = finalize(s)) return st;
  const Geometry g = geometry(s);
  rows.resize(static_cast<size_t>(8) * s->Lpad);
  HIP_TRY(s, launch_boundary_rows(static_cast<const double2 *>(s->E.p), static_cast<double2 *>(s->rows.p), g,
                                  s->stream));
  return staged_d2h(s, rows.data(), static_cast<const double *>(s->rows.p), rows.size());
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
