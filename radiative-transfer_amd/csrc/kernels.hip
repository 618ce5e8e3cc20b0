// kernels.hip -- CDNA4 (gfx950) kernels of the S_n path.
//
// Hot path: sweep_step_kernel<S> -- one full time step (BE, CN or the fused
// 4-substep BDF2 cycle) of every (direction, group) line, cell-parallel.
//
// Layout in HBM:
//   E[half][k][l]  double2 (e_in, e_out), half 0 = mu < 0 lines, half 1 = mu > 0,
//                  k = cell in the line's upwind frame, l = line = i' + (M/2) g
//                  padded to Lpad = 64 * Q.  One wave reads/writes a 1 KiB row.
//
// Parallelisation: a line is an affine recurrence X_{k+1} = A X_k + b_k over
// its cells (cell.hpp).  A tile = 64 lines x 64 cells is owned by one
// 256-thread workgroup; each of its 4 waves holds 16 cells x 64 lines in
// registers.  Phase 1 sweeps each wave's cells from X = 0 (its aggregate);
// the waves' aggregates are chained with A^16 through LDS; wave 0 publishes
// the tile aggregate, resolves the tile's incoming X by a decoupled look-back
// over its predecessors' records (A^64 powers), publishes the inclusive
// prefix, and phase 2 re-sweeps the register-resident cells with the true X
// and streams the step-end state out.  HBM traffic per cell x line x step:
// 16 B read + 16 B write (+ 2 x 40 B of look-back records per 64 cells).
//
// Scheduling: a persistent grid of P resident workgroups walks the tiles in
// the static order t = b, b + P, ...; tiles are ordered [half][j][q] (q = line
// group fastest), so a tile only ever waits on lower-numbered tiles, which
// resident workgroups own: no deadlock for any dispatch order (every spin is
// also bounded by a wall-clock timeout that sets an error word).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cell.hpp"
#include "kernels.hpp"

namespace rtamd {

// ------------------------------------------------------------------------
// inter-workgroup hand-off helpers (MI355X_MICROARCH.md "Valid forms":
// 8-byte agent-scope atomic stores/loads both sides, drained before an
// agent-scope flag store; relaxed polls)
// ------------------------------------------------------------------------
__device__ __forceinline__ void store_sc1(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double *p) {
  const unsigned long long v = __hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
  return __longlong_as_double(static_cast<long long>(v));
}
__device__ __forceinline__ void store_flag(unsigned *p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned load_flag(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Poll *flag until it reaches >= want; returns the value, or 0 after the
// timeout (error word set).  Wave-uniform: every lane polls the same word.
__device__ __forceinline__ unsigned wait_flag(const unsigned *flag, unsigned want, unsigned *err) {
  unsigned v = load_flag(flag);
  if (v >= want) return v;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  for (;;) {
    __builtin_amdgcn_s_sleep(2);
    v = load_flag(flag);
    if (v >= want) return v;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {  // 20 s
      atomicOr(err, 1u);
      return 0;
    }
  }
}

// A wave's 16 rows of one tile are addressed through a buffer descriptor built
// from wave-uniform values: base (SGPR) + row offset (SGPR soffset) + lane*16
// (one VGPR), instead of a 64-bit VGPR address per row.
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

template <int K>
__device__ __forceinline__ void matvec_lt(const double *Asm, int lane, const double *x, double *y) {
  // y = A x, A packed lower-triangular in LDS as [tri][64]
#pragma unroll
  for (int r = 0; r < K; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c <= r; ++c) acc += Asm[tri(r, c) * 64 + lane] * x[c];
    y[r] = acc;
  }
}

// ------------------------------------------------------------------------
// The sweep kernel
// ------------------------------------------------------------------------
// Phase-2 sweep of one wave's 16 cells: write the step-end state and
// prefetch the same row of the workgroup's next tile into the registers just
// consumed.  Rows are padded to whole tiles, so no access needs a bound check.
// CAPTURE: also return the carried state after cell c_last (a mu < 0 line's
// outflow, for reflective partners).
template <int S, bool CAPTURE>
__device__ __forceinline__ void sweep_phase2(const LineConst &L, double hd, bool neg, double (&ein)[kSweepCells],
                                             double (&eout)[kSweepCells], double *X, bool head, double b3,
                                             __amdgpu_buffer_rsrc_t Rw, __amdgpu_buffer_rsrc_t Rn, int voff,
                                             int row_bytes, int c_last, double *Xcap) {
  constexpr int K = SchemeDim<S>::K;
#pragma unroll
  for (int c = 0; c < kSweepCells; ++c) {
    double oi, oo;
#if RT_PIN_CELLS
    asm volatile("" : "+v"(ein[c]), "+v"(eout[c]));
#endif
    if (c == 0)
      cell_step_maybe_head<S>(L, hd, neg, ein[0], eout[0], X, head, b3, oi, oo);
    else
      cell_step<S>(L, hd, neg, ein[c], eout[c], X, oi, oo);
    row_store(Rw, voff, c * row_bytes, oi, oo);
    const double2 v = row_load(Rn, voff, c * row_bytes);
    ein[c] = v.x;
    eout[c] = v.y;
    // keep the prefetch in the registers it replaces: no hoisting across cells
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (CAPTURE) {
      if (c == c_last) {
#pragma unroll
        for (int r = 0; r < K; ++r) Xcap[r] = X[r];
      }
    }
  }
}

template <int S>
__global__ __launch_bounds__(kSweepThreads, RT_SWEEP_MIN_WAVES) void sweep_step_kernel(SweepArgs a) {
  constexpr int K = SchemeDim<S>::K;
  constexpr int NT = K * (K + 1) / 2;
  __shared__ double sm_agg[kSweepWaves][K][64];
  __shared__ double sm_xin[K][64];
  __shared__ double sm_A16[NT * 64];
  __shared__ double sm_A64[NT * 64];
  __shared__ double sm_lc[LC_COUNT * 64];  // this line group's constants
  __shared__ double sm_bdry[64];           // and inflow values

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int tiles_per_half = a.J * a.Q;  // host guarantees 2 J Q < 2^31
  const int total_tiles = static_cast<int>(a.total_tiles);
  const size_t stride = static_cast<size_t>(a.Lpad);
  int cached_key = -1;
  LineConst L;

  // tile t -> (half, j, q) and the address of this wave's first row
  auto decode = [&](int t, int &half, int &j, int &q) {
    half = t >= tiles_per_half ? 1 : 0;
    const int rem = t - half * tiles_per_half;
    j = static_cast<int>(static_cast<unsigned>(rem) / static_cast<unsigned>(a.Q));
    q = rem - j * a.Q;
  };
  const int row_bytes = a.Lpad * static_cast<int>(sizeof(double2));
  const int voff = lane * static_cast<int>(sizeof(double2));
  auto rows = [&](int half, int j, int q) {  // wave-uniform descriptor of this wave's 16 rows
    const int k0 = j * kSweepTile + w * kSweepCells;
    return rows_rsrc(a.E + (static_cast<size_t>(half) * a.Nrow + k0) * stride + q * 64, row_bytes);
  };

  int t = blockIdx.x;
  if (t >= total_tiles) return;
  int half, j, q;
  decode(t, half, j, q);
  double ein[kSweepCells], eout[kSweepCells];
  {  // prologue: this workgroup's first tile
    const __amdgpu_buffer_rsrc_t R = rows(half, j, q);
#pragma unroll
    for (int c = 0; c < kSweepCells; ++c) {
      const double2 v = row_load(R, voff, c * row_bytes);
      ein[c] = v.x;
      eout[c] = v.y;
    }
  }

  for (;;) {
    const int ell = q * 64 + lane;
    const bool neg = (half == 0);
    const int key = half * a.Q + q;
    if (key != cached_key) {
      // a new line group: constants, inflows and propagator powers -> LDS.
      // Every global load of this block is drained here, so the prefetched
      // rows still in flight are never waited for on the common path.
      __syncthreads();  // previous tile's LDS readers are done
      const double *lc = a.lc + static_cast<size_t>(half) * LC_COUNT * stride;
      const double *A16 = a.Apow + static_cast<size_t>(half * 2 + 0) * NT * stride;
      const double *A64 = a.Apow + static_cast<size_t>(half * 2 + 1) * NT * stride;
      for (int e = w; e < LC_COUNT; e += kSweepWaves) sm_lc[e * 64 + lane] = lc[e * stride + ell];
      for (int e = w; e < NT; e += kSweepWaves) {
        sm_A16[e * 64 + lane] = A16[e * stride + ell];
        sm_A64[e * 64 + lane] = A64[e * stride + ell];
      }
      if (w == 0) sm_bdry[lane] = a.bdry[static_cast<size_t>(half) * stride + ell];
      __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
      __syncthreads();
      cached_key = key;
    }
#pragma unroll
    for (int n = 0; n < LC_COUNT; ++n) L.c[n] = sm_lc[n * 64 + lane];

    // ---- inflow values for the line head (tile 0, wave 0) ----
    const bool head = (j == 0 && w == 0);
    double b[4];
    {
      const double v = sm_bdry[lane];
      b[0] = b[1] = b[2] = b[3] = v;
    }
    if (head && !neg && a.reflective) {
      // solver.cpp:677-684: the mu > 0 line reads its mirror's outflow at cell 0,
      // produced by the same substep of the mu < 0 sweep (earlier tiles)
      wait_flag(a.outflow_flag + q, 1u, a.error);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int nsub = (S == SCHEME_BDF2) ? 4 : 1;
      for (int s = 0; s < nsub; ++s) b[s] = load_sc1(a.outflow + static_cast<size_t>(s) * stride + ell);
      __builtin_amdgcn_s_waitcnt(0);
    }

    // ---- phase 1: aggregate from X = 0 (the head starts from its inflow) ----
    double X[K];
    if (head) {
      head_state<S>(b, X);
    } else {
#pragma unroll
      for (int r = 0; r < K; ++r) X[r] = 0.0;
    }
    if (!(a.debug_flags & 2)) {
      double oi, oo;
      cell_step_maybe_head<S>(L, a.hd, neg, ein[0], eout[0], X, head, b[3], oi, oo);
#pragma unroll
      for (int c = 1; c < kSweepCells; ++c) {
        // pin each cell's inputs to this point: no X-independent work of later
        // cells is hoisted ahead (bounded live ranges -> occupancy)
#if RT_PIN_CELLS
        asm volatile("" : "+v"(ein[c]), "+v"(eout[c]));
#endif
        cell_step<S>(L, a.hd, neg, ein[c], eout[c], X, oi, oo);
      }
    }
#pragma unroll
    for (int r = 0; r < K; ++r) sm_agg[w][r][lane] = X[r];
    __syncthreads();

    // ---- wave 0: tile aggregate, publish, look-back, publish prefix ----
    if (w == 0) {
      const size_t rec = static_cast<size_t>(t) * K * 64;
      double T[K], tmp[K];
#pragma unroll
      for (int r = 0; r < K; ++r) T[r] = sm_agg[0][r][lane];
      for (int ww = 1; ww < kSweepWaves; ++ww) {
        matvec_lt<K>(sm_A16, lane, T, tmp);
#pragma unroll
        for (int r = 0; r < K; ++r) T[r] = tmp[r] + sm_agg[ww][r][lane];
      }
      if (j == 0) {
        // the head made this an inclusive prefix already
#pragma unroll
        for (int r = 0; r < K; ++r) store_sc1(a.pref + rec + r * 64 + lane, T[r]);
        drain_stores();
        if (lane == 0) store_flag(a.status + t, 2u);
      } else if (a.debug_flags & 1) {
#pragma unroll
        for (int r = 0; r < K; ++r) sm_xin[r][lane] = 0.0;
      } else {
#pragma unroll
        for (int r = 0; r < K; ++r) store_sc1(a.agg + rec + r * 64 + lane, T[r]);
        drain_stores();
        if (lane == 0) store_flag(a.status + t, 1u);
#if RT_LOOKBACK_PARALLEL
        // decoupled look-back.  The 64 lanes poll the status words of the 64
        // nearest predecessors of this line group (t - Q, t - 2Q, ...) in one
        // go; the nearest one holding an inclusive prefix, with aggregates
        // published by everything in between, closes the look-back:
        //   X_in = A64 (... (A64 pref[t - dQ] + agg[t - (d-1)Q]) ...) + agg[t - Q]
        // (published records are immutable, so they are re-read safely).
        const int window = min(j, 64);
        int d = 0;
        {
          const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
          for (;;) {
            unsigned st = 0;
            if (lane < window) st = load_flag(a.status + (t - (lane + 1) * a.Q));
            const unsigned long long pm = __ballot(st >= 2u);
            const unsigned long long rm = __ballot(st >= 1u);
            if (pm) {
              d = __builtin_ctzll(pm) + 1;  // distance of the nearest prefix
              const unsigned long long need = (d == 64) ? ~0ull : ((1ull << d) - 1);
              if ((rm & need) == need) break;
            }
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t_start > 2000000000ull) {  // 20 s
              if (lane == 0) atomicOr(a.error, 1u);
              d = 1;
              break;
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double acc[K];
        {
          const double *pr = a.pref + static_cast<size_t>(t - d * a.Q) * K * 64 + lane;
#pragma unroll
          for (int r = 0; r < K; ++r) acc[r] = load_sc1(pr + r * 64);
        }
        for (int m = d - 1; m >= 1; m -= 2) {  // fold the aggregates, 2 records per batch
          double v[2][K];
#pragma unroll
          for (int u = 0; u < 2; ++u)
            if (m - u >= 1) {
              const double *ag = a.agg + static_cast<size_t>(t - (m - u) * a.Q) * K * 64 + lane;
#pragma unroll
              for (int r = 0; r < K; ++r) v[u][r] = load_sc1(ag + r * 64);
            }
#pragma unroll
          for (int u = 0; u < 2; ++u)
            if (m - u >= 1) {
              matvec_lt<K>(sm_A64, lane, acc, tmp);
#pragma unroll
              for (int r = 0; r < K; ++r) acc[r] = tmp[r] + v[u][r];
            }
        }
#else
        // decoupled look-back (serial): walk back over the predecessors of this
        // line group (t - Q, t - 2Q, ...) until one has published its inclusive
        // prefix, then fold forward from it:
        //   X_in = A64 (... (A64 pref[t - dQ] + agg[t - (d-1)Q]) ...) + agg[t - Q]
        // (published records are immutable, so they are re-read safely).
        int s = t - a.Q;
        for (;;) {
          const unsigned st = wait_flag(a.status + s, 1u, a.error);
          if (st >= 2u || st == 0u) break;
          s -= a.Q;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double acc[K];
#pragma unroll
        for (int r = 0; r < K; ++r) acc[r] = load_sc1(a.pref + static_cast<size_t>(s) * K * 64 + r * 64 + lane);
        for (s += a.Q; s < t; s += a.Q) {
          matvec_lt<K>(sm_A64, lane, acc, tmp);
#pragma unroll
          for (int r = 0; r < K; ++r) acc[r] = tmp[r] + load_sc1(a.agg + static_cast<size_t>(s) * K * 64 + r * 64 + lane);
        }
#endif
        // inclusive prefix = A64 X_in + T
        matvec_lt<K>(sm_A64, lane, acc, tmp);
#pragma unroll
        for (int r = 0; r < K; ++r) store_sc1(a.pref + rec + r * 64 + lane, tmp[r] + T[r]);
        drain_stores();
        if (lane == 0) store_flag(a.status + t, 2u);
#pragma unroll
        for (int r = 0; r < K; ++r) sm_xin[r][lane] = acc[r];
      }
    }
    __syncthreads();

    // ---- phase 2: true incoming X, re-sweep, stream out; prefetch the next tile ----
    // Re-derive every X-independent term from the data rather than keeping
    // phase 1's copies live (register pressure / occupancy over FLOPs).
#if RT_PHASE_BARRIER
#pragma unroll
    for (int c = 0; c < kSweepCells; ++c) asm volatile("" : "+v"(ein[c]), "+v"(eout[c]));
#endif
    const int tn = t + static_cast<int>(gridDim.x);
    const bool more = tn < total_tiles;
    int half_n = half, j_n = j, q_n = q;
    if (more) decode(tn, half_n, j_n, q_n);
    {
      double tmp[K];
      int first_wave;
      if (head) {
        head_state<S>(b, X);
        first_wave = 1;
      } else if (j == 0) {
#pragma unroll
        for (int r = 0; r < K; ++r) X[r] = sm_agg[0][r][lane];
        first_wave = 1;
      } else {
#pragma unroll
        for (int r = 0; r < K; ++r) X[r] = sm_xin[r][lane];
        first_wave = 0;
      }
      for (int ww = first_wave; ww < w; ++ww) {
        matvec_lt<K>(sm_A16, lane, X, tmp);
#pragma unroll
        for (int r = 0; r < K; ++r) X[r] = tmp[r] + sm_agg[ww][r][lane];
      }
    }
    const __amdgpu_buffer_rsrc_t Rw = rows(half, j, q);
    const __amdgpu_buffer_rsrc_t Rn = rows(half_n, j_n, q_n);
    const int k0 = j * kSweepTile + w * kSweepCells;
    const int c_last = a.N - 1 - k0;  // this wave holds the line's last cell iff 0 <= c_last < 16
    if (neg && a.reflective && c_last >= 0 && c_last < kSweepCells) {
      double Xo[K];
      sweep_phase2<S, true>(L, a.hd, neg, ein, eout, X, head, b[3], Rw, Rn, voff, row_bytes, c_last, Xo);
      // publish the per-substep outflows for the reflective mu > 0 partners
      if constexpr (S == SCHEME_BDF2) {
#pragma unroll
        for (int s = 0; s < 4; ++s) store_sc1(a.outflow + static_cast<size_t>(s) * stride + ell, Xo[1 + s]);
      } else {
        store_sc1(a.outflow + ell, Xo[K - 1]);
      }
      drain_stores();
      if (lane == 0) store_flag(a.outflow_flag + q, 1u);
    } else {
      sweep_phase2<S, false>(L, a.hd, neg, ein, eout, X, head, b[3], Rw, Rn, voff, row_bytes, 0, nullptr);
    }
    if (!more) break;
    t = tn;
    half = half_n;
    j = j_n;
    q = q_n;
    __syncthreads();  // LDS (sm_agg, sm_xin) is reused by the next tile
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
template <int S>
static hipError_t launch_sweep_t(const SweepArgs &a, int grid, hipStream_t st) {
  hipLaunchKernelGGL(sweep_step_kernel<S>, dim3(grid), dim3(kSweepThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_sweep(int scheme, const SweepArgs &a, int grid, hipStream_t st) {
  switch (scheme) {
    case SCHEME_BE: return launch_sweep_t<SCHEME_BE>(a, grid, st);
    case SCHEME_CN: return launch_sweep_t<SCHEME_CN>(a, grid, st);
    default: return launch_sweep_t<SCHEME_BDF2>(a, grid, st);
  }
}

hipError_t sweep_occupancy(int scheme, int *blocks_per_cu) {
  switch (scheme) {
    case SCHEME_BE:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, sweep_step_kernel<SCHEME_BE>, kSweepThreads, 0);
    case SCHEME_CN:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, sweep_step_kernel<SCHEME_CN>, kSweepThreads, 0);
    default:
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, sweep_step_kernel<SCHEME_BDF2>, kSweepThreads,
                                                          0);
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
