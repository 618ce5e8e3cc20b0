// rtsn_lines.hip -- per-line setup of a handle: the line constants of the reference algebra,
// the per-line affine cell map (cell.hpp) and the reflective head cell's own map (probed from
// the same algebra), the aligned schedule's segment propagators,
// boundary inflows, and the segmentation of the lines (segment_lines / resegment).

#include <atomic>
#include <cstring>

#include "rtsn_internal.hpp"

using namespace rtamd;
using namespace rtsn_detail;

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

// Host -> device, asynchronous: `src` may be freed at return.  Up to kArenaMax bytes go
// through the handle's pinned upload arena (a DMA from page-locked memory, no host wait):
// the setup of a handle -- line maps and constants, inflows, sources -- is a handful of small
// copies that a pageable hipMemcpyAsync + stream synchronisation each made a host round trip
// (round 5, profiles/r05a_*: ~100 us of llnl_slab_test's create).  The arena restarts from
// its beginning after a stream synchronisation once full; larger copies (the aligned
// schedule's propagators) go from `src` and wait.
constexpr size_t kArenaMax = size_t(16) << 20;
rt_status rtsn_detail::upload(rt_solver *s, DeviceBuf &b, const void *src, size_t bytes) {
  if (bytes > kArenaMax) {
    HIP_TRY(s, hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));  // src dies at return
    return RT_OK;
  }
  const size_t need = (bytes + 255) & ~size_t(255);
  if (s->up_used + need > s->up_cap) {
    if (s->up_used) HIP_TRY(s, hipStreamSynchronize(s->stream));  // earlier uploads have left the arena
    s->up_used = 0;
    if (need > s->up_cap) {
      ResourcePool::get().release(true, s->up_arena, s->up_cap, 0);
      s->up_arena = nullptr;
      s->up_cap = 0;
      HIP_TRY(s, ResourcePool::get().alloc(true, std::max(need, size_t(1) << 20), &s->up_arena, &s->up_cap));
    }
  }
  char *h = static_cast<char *>(s->up_arena) + s->up_used;
  std::memcpy(h, src, bytes);
  HIP_TRY(s, hipMemcpyAsync(b.p, h, bytes, hipMemcpyHostToDevice, s->stream));
  s->up_used += need;
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

// Per-line maps into map_dev, and the mu > 0 lines' head-cell maps into hmap_dev (used by
// reflective chains only); unit_B: sources for B_g = 1 (material coupling), leaving
// map_host (the propagators' source) alone.
template <int S>
rt_status rtsn_detail::line_maps_s(rt_solver *s, bool unit_B, DeviceBuf &map_dev, DeviceBuf &hmap_dev) {
  constexpr int WN = map_count<S>();
  const double hd = 0.5 * (s->p.X / s->p.N);
  const size_t Lp = s->Lpad;
  std::vector<double> hmap(WN * Lp, 0.0), unit_map;
  std::vector<double> &map = unit_B ? unit_map : s->map_host;
  map.assign(2 * WN * Lp, 0.0);
  // lines are independent: chunks of them on the host workers (phys::parallel_for)
  const long long lines = 2LL * s->Gl * s->H;
  const int chunks = static_cast<int>(std::min<long long>(phys::host_workers(), (lines + 63) / 64));
  std::atomic<bool> bad{false};
  phys::parallel_for(chunks, [&](int t) {
    double W[WN];
    for (long long x = lines * t / chunks; x < lines * (t + 1) / chunks; ++x) {
      const int half = static_cast<int>(x / (static_cast<long long>(s->Gl) * s->H));
      const int rem = static_cast<int>(x % (static_cast<long long>(s->Gl) * s->H));
      const int gl = rem / s->H, ip = rem % s->H;
      const int i = line_direction(s->H, half, ip), g = s->g_lo + gl;
      const size_t ell = ip + static_cast<size_t>(s->H) * gl;
      const LineConst L = line_constants(*s, i, g, unit_B);
      if (!cell_map<S>(L, hd, half == 0, W)) bad = true;
      for (int n = 0; n < WN; ++n) map[(half * WN + n) * Lp + ell] = W[n];
      if (half == 1) {
        double Wh[WN];
        if (!cell_map<S, true>(L, hd, false, Wh)) bad = true;
        for (int n = 0; n < head_map_first<S>(); ++n)  // the kernels keep only the rest apart
          if (Wh[n] != W[n]) bad = true;
        for (int n = 0; n < WN; ++n) hmap[n * Lp + ell] = Wh[n];
      }
    }
  });
  if (bad) return fail(s, RT_ERR_PARAM, "cell map: a structurally zero coefficient is not zero (or a head-cell row differs from its line map)");
  rt_status st;
  if ((st = upload(s, hmap_dev, hmap.data(), hmap.size() * sizeof(double)))) return st;
  if ((st = upload(s, map_dev, map.data(), map.size() * sizeof(double)))) return st;
  return RT_OK;
}

template <int S>
static rt_status setup_lines_s(rt_solver *s) {
  const size_t Lp = s->Lpad;
  rt_status st;
  if ((st = line_maps_s<S>(s, false, s->map, s->hmap))) return st;
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
  s->prop_ready[T] = true;
  return RT_OK;
}

rt_status rtsn_detail::ensure_propagators(rt_solver *s, int T) {
  if (s->prop_ready[T]) return RT_OK;
  switch (s->scheme) {
    case SCHEME_BE: return build_propagators_s<SCHEME_BE>(s, T);
    case SCHEME_CN: return build_propagators_s<SCHEME_CN>(s, T);
    default: return build_propagators_s<SCHEME_BDF2>(s, T);
  }
}

rt_status rtsn_detail::setup_lines(rt_solver *s) {
  switch (s->scheme) {
    case SCHEME_BE: return setup_lines_s<SCHEME_BE>(s);
    case SCHEME_CN: return setup_lines_s<SCHEME_CN>(s);
    default: return setup_lines_s<SCHEME_BDF2>(s);
  }
}

rt_status rtsn_detail::upload_inflow(rt_solver *s) {
  std::vector<double> bd;
  line_inflow(*s, bd);
  return upload(s, s->bdry, bd.data(), bd.size() * sizeof(double));
}

// Segments per line: enough waves (2 Q Sg) to fill the chip at the sweep
// kernel's occupancy, Ls a multiple of the register chunk; at most max_sg segments.
void rtsn_detail::segment_lines(rt_solver *h, int waves_per_cu, long long max_sg) {
  waves_per_cu = std::max(1, std::min(waves_per_cu, 64));
  const long long target = static_cast<long long>(h->cus) * waves_per_cu;
  long long sg = std::max<long long>(1, target / (2LL * h->Q));
  sg = std::min(sg, std::max<long long>(1, max_sg));
  sg = std::min<long long>(sg, (h->p.N + kSweepCells - 1) / kSweepCells);
  long long ls = (h->p.N + sg - 1) / sg;
  ls = ((ls + kSweepCells - 1) / kSweepCells) * kSweepCells;
  h->Ls = static_cast<int>(ls);
  h->Sg = static_cast<int>((h->p.N + ls - 1) / ls);
}

// Segments of an aligned pass.  The pass sweeps every segment at once (Ls cells x Ta
// levels per wave) and the fold walks the Sg segments one after another, so beyond the
// chip's occupancy more segments only lengthen the walk: Sg balances Ls Ta t_cell against
// Sg t_fold, with t_cell ~ 145 ns per cell-level and wave (the aligned T = 4 pass with its
// correction, SL: 72.3 ms for 62500 x 4 cell-levels per wave at two waves per SIMD) and
// t_fold ~ 200 ns + 4 ns per propagator coefficient (fold_kernel's step, LDS-resident
// propagator).  On the SL slab the occupancy's 16 segments stay (the balance is ~900);
// few long lines get ~100-200 segments instead of the pipeline's hundreds or thousands.
long long rtsn_detail::aligned_segments(const rt_solver *h) {
  const int Ta = std::min(h->T, kMaxAlignedBlock), KC = Ta * h->K;
  const double t_cell = 145.0, t_fold = 200.0 + 4.0 * KC * (KC + 1) / 2;
  return std::max(1LL, std::llround(std::sqrt(static_cast<double>(h->p.N) * Ta * t_cell / t_fold)));
}

// Per-segment buffers (aggregates, folded incoming states), zeroed; the
// segment propagators are rebuilt on their next use.
hipError_t rtsn_detail::alloc_segments(rt_solver *h) {
  // the handle's device, whatever the caller's current one (dalloc records the device)
  if (hipError_t e = hipSetDevice(h->device)) return e;
  const size_t Lp = h->Lpad;
  const int K = h->K;
  if (h->agg[0].p || h->agg[1].p || h->yseg.p) (void)hipStreamSynchronize(h->stream);  // before the cache may hand them out
  for (DeviceBuf *b : {&h->agg[0], &h->agg[1], &h->yseg}) b->reset();
  hipError_t e = dalloc(h->agg[0], sizeof(double) * 2 * h->Sg * kMaxTimeBlock * K * Lp);
  if (!e) e = dalloc(h->agg[1], sizeof(double) * 2 * h->Sg * kMaxTimeBlock * K * Lp);
  if (!e) e = dalloc(h->yseg, sizeof(double) * 2 * (h->Sg + 1) * kMaxAlignedBlock * K * Lp);
  h->agg_zero_pending = true;  // zeroed before the first segment pass (ensure_segments): a
                               // wavefront-only handle never touches them
  for (bool &r : h->prop_ready) r = false;
  return e;
}

rt_status rtsn_detail::ensure_segments(rt_solver *s) {
  if (!s->agg_zero_pending) return RT_OK;
  HIP_TRY(s, hipMemsetAsync(s->agg[0].p, 0, s->agg[0].bytes, s->stream));
  HIP_TRY(s, hipMemsetAsync(s->agg[1].p, 0, s->agg[1].bytes, s->stream));
  s->agg_zero_pending = false;
  return RT_OK;
}

// Segments sized for the pipelined pass of the current time block (its occupancy: one
// wave per SIMD at T = 16 and 20, two at T = 10, ...), applied only while every chain
// position is at the same time with no correction outstanding -- the state rows do not
// depend on the segmentation, only the aggregates and propagators do.  Called by
// rt_set_time_block and again before the next pipelined or aligned pass (aligned: at
// most aligned_segments), so a handle always runs its passes with segments for the time
// block and the kind of pass it runs.

rt_status rtsn_detail::resegment(rt_solver *h, bool aligned) {
  if (h->material || h->pending || h->Tpipe) return RT_OK;
  int w = 0;
  if (rt_status st = segment_target(h, &w)) return st;
  const int key = aligned ? -w : w;  // which kind of pass the segments were sized for
  if (h->seg_T == h->T && h->seg_w == key) return RT_OK;
  const int sg0 = h->Sg, ls0 = h->Ls;
  segment_lines(h, w, aligned ? aligned_segments(h) : (1LL << 40));
  h->seg_T = h->T;
  h->seg_w = key;
  if (h->Sg == sg0 && h->Ls == ls0) return RT_OK;
  if (2LL * h->Q * h->Sg >= (1LL << 31)) return fail(h, RT_ERR_PARAM, "too many lines for one handle: shard the groups");
  HIP_TRY(h, alloc_segments(h));
  h->tau.assign(chain_positions(h), h->target);  // every position at the same, requested time
  h->resume_lo = h->resume_hi = -1;
  return RT_OK;
}

// Workgroups per CU the segments of the current time block are sized for: the caller's
// (rt_set_segmentation, or the schedule rt_solve planned), else the pipelined pass's
// occupancy.
rt_status rtsn_detail::segment_target(rt_solver *h, int *w_out) {
  int w = h->seg_wgs;
  if (!w) HIP_TRY(h, sweep_occupancy(h->scheme, h->T, level_waves_of(h, h->T), &w));
  *w_out = std::max(1, std::min(w, 64));
  return RT_OK;
}

template rt_status rtsn_detail::line_maps_s<SCHEME_BE>(rt_solver *, bool, DeviceBuf &, DeviceBuf &);
template rt_status rtsn_detail::line_maps_s<SCHEME_CN>(rt_solver *, bool, DeviceBuf &, DeviceBuf &);
template rt_status rtsn_detail::line_maps_s<SCHEME_BDF2>(rt_solver *, bool, DeviceBuf &, DeviceBuf &);
