// kernels.hip -- CDNA4 (gfx950) kernels of the S_n path.
//
// Hot path: sweep_segment_kernel<S, MODE> -- one full time step (BE, CN or the
// fused 4-substep BDF2 cycle, cell.hpp) of every (direction, group) line.
//
// Layout in HBM:
//   E[half][k][l]  double2 (e_in, e_out), half 0 = mu < 0 lines, half 1 = mu > 0,
//                  k = cell in the line's upwind frame, l = line = i' + (M/2) g,
//                  padded to Lpad = 64 Q lines and Nrow = 64 J rows.  A wave
//                  moves one 1 KiB row per instruction.
//
// Parallelisation without in-step synchronisation.  Within a step, a line
// is the affine recurrence X_{k+1} = A X_k + B d_k + c over its cells, and the
// step-end state of cell k is R X_k + (data terms), with A, R constant per
// line (cell.hpp).  Each line is cut into Sg segments of Ls cells; one wave
// (64 lines) sweeps one segment in a single pass, streaming 16-row chunks
// through registers with a rolling prefetch.  Segment 0 starts from the true
// inflow; segment s > 0 starts from X = 0, so its stored state is
// *provisional*: exact up to the term R A^(k - k_s) X_s, where X_s is the
// segment's true incoming state.  Every wave publishes its final carried
// state (its aggregate).  The next step -- or a finalize launch before any
// read-out -- rebuilds X_s = fold of the previous segments' aggregates with
// the segment propagator A^Ls and adds the correction while it loads the
// rows.  No workgroup ever waits for another, so there is nothing to
// deadlock and nothing to stall; the cost is ~20 FMA per cell for the
// correction instead of a second compute pass.
//
// Reflective left boundary (solver.cpp:677-684): the mu > 0 heads need the
// mu < 0 outflow of the SAME step, so the two halves go in two launches and
// the mu > 0 head folds the mu < 0 aggregates of this step.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cell.hpp"
#include "kernels.hpp"

namespace rtamd {

// A wave's 16 rows of one chunk are addressed through a buffer descriptor
// built from wave-uniform values: base (SGPR) + row offset (SGPR soffset) +
// lane*16 (one VGPR), instead of a 64-bit VGPR address per row.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const double2 *base, int row_bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double2 *>(base), 0, kSweepCells * row_bytes, 0x00020000);
}
__device__ __forceinline__ double2 row_load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void row_store(__amdgpu_buffer_rsrc_t r, int voff, int soff, double x, double y) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(x, y)), r, voff, soff, 0);
}

// y = A x with A packed lower-triangular, one entry per stride in memory
template <int K>
__device__ __forceinline__ void matvec_lt_g(const double *A, size_t stride, const double *x, double *y) {
#pragma unroll
  for (int r = 0; r < K; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c <= r; ++c) acc += A[tri(r, c) * stride] * x[c];
    y[r] = acc;
  }
}

// X_s of segment s (its true incoming carried state) from the aggregates of
// segments 0..s-1: X_1 = agg_0 (segment 0 starts from the true inflow),
// X_{s'+1} = P_{s'} X_{s'} + agg_{s'}, with P = A^Ls, or A^Llast for the last
// segment (last_short).
template <int K>
__device__ __forceinline__ void fold_segments(const double *agg, size_t seg_stride, size_t stride, int s,
                                              const double *Aseg, const double *Alast, bool last_short,
                                              double *X) {
#pragma unroll
  for (int r = 0; r < K; ++r) X[r] = agg[r * stride];
  for (int sp = 1; sp < s; ++sp) {
    double t[K];
    const double *P = (last_short && sp == s - 1) ? Alast : Aseg;
    matvec_lt_g<K>(P, stride, X, t);
#pragma unroll
    for (int r = 0; r < K; ++r) X[r] = t[r] + agg[sp * seg_stride + r * stride];
  }
}

// One 16-row chunk: correct the loaded rows by the pending term R Y (Y <- A Y
// per cell), sweep them (MODE 0), store, and prefetch the next chunk's rows
// into the registers just consumed.  PARTIAL: only the first nv cells are
// real; the carried state after cell nv-1 is returned in Xcap.
template <int S, int MODE, bool PARTIAL>
__device__ __forceinline__ void sweep_chunk(const LineConst &L, double hd, bool neg, double (&ein)[kSweepCells],
                                            double (&eout)[kSweepCells], double *X, bool corr, double *Y,
                                            const double *A1, const double *Rm, bool head, double b3,
                                            __amdgpu_buffer_rsrc_t Rw, __amdgpu_buffer_rsrc_t Rn, int voff,
                                            int row_bytes, int nv, double *Xcap) {
  constexpr int K = SchemeDim<S>::K;
#pragma unroll
  for (int c = 0; c < kSweepCells; ++c) {
    double pin = ein[c], pout = eout[c];
    if (corr) {  // e += R Y ; Y <- A Y   (deferred cross-segment correction)
#pragma unroll
      for (int r = 0; r < K; ++r) {
        pin += Rm[r] * Y[r];
        pout += Rm[K + r] * Y[r];
      }
      double t[K];
#pragma unroll
      for (int r = 0; r < K; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int cc = 0; cc <= r; ++cc) acc += A1[tri(r, cc)] * Y[cc];
        t[r] = acc;
      }
#pragma unroll
      for (int r = 0; r < K; ++r) Y[r] = t[r];
    }
    double oi = pin, oo = pout;
    if constexpr (MODE == 0) {
      if (c == 0)
        cell_step_maybe_head<S>(L, hd, neg, pin, pout, X, head, b3, oi, oo);
      else
        cell_step<S>(L, hd, neg, pin, pout, X, oi, oo);
    }
    row_store(Rw, voff, c * row_bytes, oi, oo);
    const double2 v = row_load(Rn, voff, c * row_bytes);
    ein[c] = v.x;
    eout[c] = v.y;
    if constexpr (PARTIAL) {
      if (c == nv - 1) {
#pragma unroll
        for (int r = 0; r < K; ++r) Xcap[r] = X[r];
      }
    }
  }
}

template <int S, int MODE>
__global__ __launch_bounds__(64) void sweep_segment_kernel(SegArgs a) {
  constexpr int K = SchemeDim<S>::K;
  constexpr int NT = K * (K + 1) / 2;
  const int lane = threadIdx.x;
  const size_t stride = static_cast<size_t>(a.Lpad);
  const int per_half = a.Q * a.Sg;
  const int half = a.half0 + static_cast<int>(blockIdx.x) / per_half;
  const int rem = static_cast<int>(blockIdx.x) % per_half;
  const int s = rem / a.Q;  // segment (wave-uniform)
  const int q = rem - s * a.Q;
  const int ell = q * 64 + lane;
  const bool neg = half == 0;
  const int k_begin = s * a.Ls;
  const int k_end = min(a.N, k_begin + a.Ls);
  if (k_begin >= k_end) return;
  const bool last_short = (a.N - (a.Sg - 1) * a.Ls) != a.Ls;

  // per-line propagators: A1 (one cell), R (state -> step-end nodes), A^Ls, A^Llast
  const double *pr = a.prop + static_cast<size_t>(half) * kPropCount<K> * stride + ell;
  const double *pA1 = pr;
  const double *pR = pr + NT * stride;
  const double *pAseg = pr + (NT + 2 * K) * stride;
  const double *pAlast = pr + (2 * NT + 2 * K) * stride;
  const size_t seg_stride = static_cast<size_t>(K) * stride;

  // ---- pending correction of the previous step: Y = true incoming state ----
  const bool corr = a.pending && s > 0;
  double Y[K], A1[NT], Rm[2 * K];
#pragma unroll
  for (int r = 0; r < K; ++r) Y[r] = 0.0;
  if (corr) {
    const double *ag = a.agg_prev + static_cast<size_t>(half) * a.Sg * seg_stride + ell;
    fold_segments<K>(ag, seg_stride, stride, s, pAseg, pAlast, false, Y);
  }
#pragma unroll
  for (int e = 0; e < NT; ++e) A1[e] = pA1[e * stride];
#pragma unroll
  for (int e = 0; e < 2 * K; ++e) Rm[e] = pR[e * stride];

  // ---- line constants, inflow ----
  LineConst L;
#pragma unroll
  for (int n = 0; n < LC_COUNT; ++n) L.c[n] = a.lc[(static_cast<size_t>(half) * LC_COUNT + n) * stride + ell];
  double X[K];
  double b[4];
  const bool head_seg = (s == 0);
  {
    const double v = a.bdry[static_cast<size_t>(half) * stride + ell];
    b[0] = b[1] = b[2] = b[3] = v;
  }
  if (MODE == 0 && head_seg && !neg && a.reflective) {
    // solver.cpp:677-684: mu > 0 inflow = the mirror mu < 0 line's outflow of this
    // step, folded from that line's segment aggregates (previous launch)
    const double *ag = a.agg_cur + ell;  // half 0, same l
    const double *pr0 = a.prop + ell;    // half 0 propagators
    double Xo[K];
    fold_segments<K>(ag, seg_stride, stride, a.Sg, pr0 + (NT + 2 * K) * stride,
                     pr0 + (2 * NT + 2 * K) * stride, last_short, Xo);
    if constexpr (S == SCHEME_BDF2) {
      b[0] = Xo[1];
      b[1] = Xo[2];
      b[2] = Xo[3];
      b[3] = Xo[4];
    } else {
      b[0] = b[1] = b[2] = b[3] = Xo[K - 1];
    }
  }
  if (head_seg) {
    head_state<S>(b, X);
  } else {
#pragma unroll
    for (int r = 0; r < K; ++r) X[r] = 0.0;
  }

  // ---- stream the segment in 16-row chunks ----
  const int row_bytes = a.Lpad * static_cast<int>(sizeof(double2));
  const int voff = lane * static_cast<int>(sizeof(double2));
  const double2 *Eh = a.E + static_cast<size_t>(half) * a.Nrow * stride + q * 64;
  auto rows = [&](int k0) { return rows_rsrc(Eh + static_cast<size_t>(k0) * stride, row_bytes); };
  double ein[kSweepCells], eout[kSweepCells];
  {
    const __amdgpu_buffer_rsrc_t R0 = rows(k_begin);
#pragma unroll
    for (int c = 0; c < kSweepCells; ++c) {
      const double2 v = row_load(R0, voff, c * row_bytes);
      ein[c] = v.x;
      eout[c] = v.y;
    }
  }
  double Xcap[K];
  int k0 = k_begin;
  for (; k0 + kSweepCells < k_end; k0 += kSweepCells) {  // full chunks with a successor
    sweep_chunk<S, MODE, false>(L, a.hd, neg, ein, eout, X, corr, Y, A1, Rm, head_seg && k0 == 0, b[3], rows(k0),
                                rows(k0 + kSweepCells), voff, row_bytes, kSweepCells, Xcap);
  }
  {  // last chunk (possibly partial); its "prefetch" re-reads its own rows (harmless)
    const int nv = k_end - k0;
    const __amdgpu_buffer_rsrc_t Rl = rows(k0);
    if (nv == kSweepCells) {
      sweep_chunk<S, MODE, false>(L, a.hd, neg, ein, eout, X, corr, Y, A1, Rm, head_seg && k0 == 0, b[3], Rl, Rl,
                                  voff, row_bytes, nv, Xcap);
#pragma unroll
      for (int r = 0; r < K; ++r) Xcap[r] = X[r];
    } else {
      sweep_chunk<S, MODE, true>(L, a.hd, neg, ein, eout, X, corr, Y, A1, Rm, head_seg && k0 == 0, b[3], Rl, Rl,
                                 voff, row_bytes, nv, Xcap);
    }
  }
  if constexpr (MODE == 0) {
    double *ag = a.agg_cur + static_cast<size_t>(half) * a.Sg * seg_stride + static_cast<size_t>(s) * seg_stride + ell;
#pragma unroll
    for (int r = 0; r < K; ++r) ag[r * stride] = Xcap[r];
  }
}

// ------------------------------------------------------------------------
// Non-hot kernels: state initialisation, layout conversion, moments
// ------------------------------------------------------------------------
// psi = ends = B_g (solver.cpp:165-181); padding rows k >= N are zero
__global__ void init_state_kernel(double2 *E, const double *lineB, int N, int Nrow, int Lpad) {
  const size_t total = static_cast<size_t>(2) * Nrow * Lpad;
  for (size_t idx = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; idx < total;
       idx += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const size_t row = idx / Lpad;
    const size_t half = row / Nrow;
    const int k = static_cast<int>(row - half * Nrow);
    const int ell = static_cast<int>(idx % Lpad);
    const double v = k < N ? lineB[half * Lpad + ell] : 0.0;
    E[idx] = make_double2(v, v);
  }
}

struct LineMap {
  int M, H, Gl, N, Nrow, Lpad;
  // reference (i, g, c) -> (half, ell, k) and node swap for mu < 0
  __device__ __forceinline__ void map(int i, int g, int c, int &half, int &ell, int &k) const {
    if (i < H) {
      half = 0;
      ell = (H - 1 - i) + H * g;
      k = N - 1 - c;
    } else {
      half = 1;
      ell = (i - H) + H * g;
      k = c;
    }
  }
  __device__ __forceinline__ size_t at(int half, int k, int ell) const {
    return (static_cast<size_t>(half) * Nrow + k) * Lpad + ell;
  }
};

// psi (M, Gl, N) ColMajor = mean of the nodes (solver.cpp:352,389)
__global__ void export_psi_kernel(const double2 *E, double *psi, LineMap m) {
  const size_t total = static_cast<size_t>(m.M) * m.Gl * m.N;
  for (size_t o = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; o < total;
       o += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const int i = static_cast<int>(o % m.M);
    const int g = static_cast<int>((o / m.M) % m.Gl);
    const int c = static_cast<int>(o / (static_cast<size_t>(m.M) * m.Gl));
    int half, ell, k;
    m.map(i, g, c, half, ell, k);
    const double2 v = E[m.at(half, k, ell)];
    psi[o] = 0.5 * (v.x + v.y);
  }
}

// ends (M, Gl, N, 2) ColMajor <-> E; node 0 = left, 1 = right
__global__ void export_ends_kernel(const double2 *E, double *ends, LineMap m) {
  const size_t mgn = static_cast<size_t>(m.M) * m.Gl * m.N;
  for (size_t o = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; o < mgn;
       o += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const int i = static_cast<int>(o % m.M);
    const int g = static_cast<int>((o / m.M) % m.Gl);
    const int c = static_cast<int>(o / (static_cast<size_t>(m.M) * m.Gl));
    int half, ell, k;
    m.map(i, g, c, half, ell, k);
    const double2 v = E[m.at(half, k, ell)];
    ends[o] = half == 0 ? v.y : v.x;
    ends[o + mgn] = half == 0 ? v.x : v.y;
  }
}

__global__ void import_ends_kernel(double2 *E, const double *ends, LineMap m) {
  const size_t mgn = static_cast<size_t>(m.M) * m.Gl * m.N;
  for (size_t o = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; o < mgn;
       o += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const int i = static_cast<int>(o % m.M);
    const int g = static_cast<int>((o / m.M) % m.Gl);
    const int c = static_cast<int>(o / (static_cast<size_t>(m.M) * m.Gl));
    int half, ell, k;
    m.map(i, g, c, half, ell, k);
    const double l = ends[o], r = ends[o + mgn];
    E[m.at(half, k, ell)] = half == 0 ? make_double2(r, l) : make_double2(l, r);
  }
}

// phi, F, phi_plus (Gl, N) ColMajor: sequential sums over i in the
// reference's order (solver.cpp:191-237), no FMA contraction.
__global__ void moments_kernel(const double2 *E, const double *mu, const double *wt, double *phi, double *F,
                               double *phi_plus, LineMap m) {
#pragma clang fp contract(off)
  const size_t total = static_cast<size_t>(m.Gl) * m.N;
  for (size_t o = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; o < total;
       o += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(o % m.Gl);
    const int c = static_cast<int>(o / m.Gl);
    double a = 0.0, f = 0.0, p = 0.0;
    for (int i = 0; i < m.M; ++i) {
      int half, ell, k;
      m.map(i, g, c, half, ell, k);
      const double2 v = E[m.at(half, k, ell)];
      const double psi = 0.5 * (v.x + v.y);
      a += wt[i] * psi;
      f += mu[i] * wt[i] * psi;
      if (i >= m.M / 2) p += wt[i] * psi;
    }
    phi[o] = a;
    F[o] = f;
    phi_plus[o] = p;
  }
}

// Boundary rows k = 0 and k = N-1 of both halves (for group ends / balance)
__global__ void boundary_rows_kernel(const double2 *E, double2 *rows, int N, int Nrow, int Lpad) {
  const int total = 4 * Lpad;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int which = o / Lpad;  // 0: half0 k=0, 1: half0 k=N-1, 2: half1 k=0, 3: half1 k=N-1
    const int ell = o % Lpad;
    const int half = which / 2;
    const int k = (which & 1) ? N - 1 : 0;
    rows[o] = E[(static_cast<size_t>(half) * Nrow + k) * Lpad + ell];
  }
}

// A(x_c) = sum_g rho kappa_g phi_g(c) over the handle's groups
__global__ void group_absorption_kernel(const double *phi, const double *sigma, double *out, int Gl, int N) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < N; c += gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int g = 0; g < Gl; ++g) s += sigma[g] * phi[static_cast<size_t>(c) * Gl + g];
    out[c] = s;
  }
}

// ------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------
template <int S, int MODE>
static hipError_t launch_seg_t(const SegArgs &a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((sweep_segment_kernel<S, MODE>), dim3(grid), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_sweep(int scheme, bool finalize, const SegArgs &a, int grid, hipStream_t st) {
  switch (scheme) {
    case SCHEME_BE: return finalize ? launch_seg_t<SCHEME_BE, 1>(a, grid, st) : launch_seg_t<SCHEME_BE, 0>(a, grid, st);
    case SCHEME_CN: return finalize ? launch_seg_t<SCHEME_CN, 1>(a, grid, st) : launch_seg_t<SCHEME_CN, 0>(a, grid, st);
    default:
      return finalize ? launch_seg_t<SCHEME_BDF2, 1>(a, grid, st) : launch_seg_t<SCHEME_BDF2, 0>(a, grid, st);
  }
}

hipError_t sweep_occupancy(int scheme, int *waves_per_cu) {
  switch (scheme) {
    case SCHEME_BE:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(waves_per_cu, sweep_segment_kernel<SCHEME_BE, 0>, 64, 0);
    case SCHEME_CN:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(waves_per_cu, sweep_segment_kernel<SCHEME_CN, 0>, 64, 0);
    default:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(waves_per_cu, sweep_segment_kernel<SCHEME_BDF2, 0>, 64, 0);
  }
}

static int grid_for(size_t total, int block) {
  size_t g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

hipError_t launch_init_state(double2 *E, const double *lineB, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(init_state_kernel, dim3(grid_for(static_cast<size_t>(2) * g.Nrow * g.Lpad, 256)), dim3(256), 0, st,
                     E, lineB, g.N, g.Nrow, g.Lpad);
  return hipGetLastError();
}

static LineMap make_map(const Geometry &g) { return LineMap{g.M, g.M / 2, g.Gl, g.N, g.Nrow, g.Lpad}; }

hipError_t launch_export_psi(const double2 *E, double *psi, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(export_psi_kernel, dim3(grid_for(static_cast<size_t>(g.M) * g.Gl * g.N, 256)), dim3(256), 0, st,
                     E, psi, make_map(g));
  return hipGetLastError();
}

hipError_t launch_export_ends(const double2 *E, double *ends, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(export_ends_kernel, dim3(grid_for(static_cast<size_t>(g.M) * g.Gl * g.N, 256)), dim3(256), 0, st,
                     E, ends, make_map(g));
  return hipGetLastError();
}

hipError_t launch_import_ends(double2 *E, const double *ends, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(import_ends_kernel, dim3(grid_for(static_cast<size_t>(g.M) * g.Gl * g.N, 256)), dim3(256), 0, st,
                     E, ends, make_map(g));
  return hipGetLastError();
}

hipError_t launch_moments(const double2 *E, const double *mu, const double *wt, double *phi, double *F,
                          double *phi_plus, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(moments_kernel, dim3(grid_for(static_cast<size_t>(g.Gl) * g.N, 256)), dim3(256), 0, st, E, mu, wt,
                     phi, F, phi_plus, make_map(g));
  return hipGetLastError();
}

hipError_t launch_boundary_rows(const double2 *E, double2 *rows, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(boundary_rows_kernel, dim3(grid_for(static_cast<size_t>(4) * g.Lpad, 256)), dim3(256), 0, st, E,
                     rows, g.N, g.Nrow, g.Lpad);
  return hipGetLastError();
}

hipError_t launch_group_absorption(const double *phi, const double *sigma, double *out, const Geometry &g,
                                   hipStream_t st) {
  hipLaunchKernelGGL(group_absorption_kernel, dim3(grid_for(static_cast<size_t>(g.N), 256)), dim3(256), 0, st, phi,
                     sigma, out, g.Gl, g.N);
  return hipGetLastError();
}

}  // namespace rtamd
