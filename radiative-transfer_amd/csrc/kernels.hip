// kernels.hip -- CDNA4 (gfx950) kernels of the S_n path.
//
// Hot path: sweep_block_kernel<S, T, MODE> -- T full time steps (BE, CN or the
// fused 4-substep BDF2 cycle) of every (direction, group) line in one pass
// over HBM, each cell step evaluated as the line's affine map (cell.hpp).
//
// Layout in HBM:
//   E[half][k][l]  double2 (e_in, e_out), half 0 = mu < 0 lines, half 1 = mu > 0,
//                  k = cell in the line's upwind frame, l = line = i' + (M/2) g,
//                  padded to Lpad = 64 Q lines and Nrow = 64 J rows.  A wave
//                  moves one 1 KiB row per instruction.
//
// Parallelisation over cells.  Each line is cut into Sg segments of Ls cells;
// one wave (64 lines) sweeps one segment, streaming C-row chunks through
// registers with a rolling prefetch, carrying T states (one per fused step;
// level t's step-end nodes are level t+1's data).  The state entering
// segment s > 0 comes from one of two schedules, neither with any
// inter-workgroup wait:
//   MODE 2 (pipelined): segments run at staggered time levels, one pass
//     apart; segment s starts from the exit state segment s-1 published in
//     the previous launch -- exact, nothing to correct.
//   MODE 0 (aligned): segment s starts from X = 0, so its stored state is
//     provisional, exact up to R_T A_T^(k - k_s) Y_s (Y_s its true incoming
//     state).  fold_kernel rebuilds Y_s from the segments' exit states; the
//     next pass (or MODE 1, finalize) adds the correction while it loads the
//     rows, by running the linear part of the map on Y.
//
// Reflective left boundary (solver.cpp:677-684): the mu > 0 heads need the
// mu < 0 outflow of the same steps: the next chain position (MODE 2), or a
// second launch after a fold of the mu < 0 exit states (MODE 0).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "cell.hpp"
#include "kernels.hpp"
#include "sweep_device.hpp"

namespace rtamd {

// True incoming carried state of every segment from the aggregates of one
// pass (each segment swept from X = 0):  Y_1 = agg_0,
// Y_{s+1} = P_s Y_s + agg_s with P = A^Ls, or A^Llast for the last segment;
// Y_Sg is the state after the whole line (the reflective outflow); only_last: write
// Y_Sg alone, to y[KC][Lpad].  One wave per (half, 64-line group), lane = line.  The
// chain is a dependent walk over the segments, so what bounds it is the latency of each
// step: the line's propagator A^Ls (the same for every segment but the last) is staged in
// LDS once -- [NTC/2][64 lanes] double pairs, a lane reading only its own column, so one
// ds_read_b128 fetches its next two coefficients and no barrier is needed -- and the next
// segment's aggregate is prefetched while the current step runs.  (The first version
// re-read the propagator from memory at every segment: ~23 us per segment on few long
// lines, 1.4-4.5 s for 1000 aligned steps of 4000-50000 cells, profiles/archive/r03ao_solve_mid.jsonl.)
constexpr int kFoldChunk = 8;  // LDS pairs per read chunk of fold_kernel's walk

// fold_kernel's memory traffic: a buffer descriptor over a wave-uniform base, the row as a
// scalar byte offset and the lane as the one VGPR offset -- a 64-bit VGPR address per row
// would hold 2 NTC registers for the propagator alone (spills at KC = 20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fold_rsrc(const double *base, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base), 0,
                                           static_cast<int>(bytes < 0x7fffffffULL ? bytes : 0x7fffffffULL), 0x00020000);
}
__device__ __forceinline__ double fold_load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void fold_store(__amdgpu_buffer_rsrc_t r, int voff, int soff, double v) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, 0);
}

template <int KC>
__global__ __launch_bounds__(64) void fold_kernel(FoldArgs f) {
  constexpr int NTC = KC * (KC + 1) / 2, NP = (NTC + 1) / 2;
  __shared__ double2 lds_p[NP * 64];
  const int lane = threadIdx.x;
  const int groups = f.Lpad / 64;
  const int half = f.half0 + static_cast<int>(blockIdx.x) / groups;
  const int ell0 = (static_cast<int>(blockIdx.x) % groups) * 64;  // the wave's first line
  const size_t stride = f.Lpad, seg_stride = static_cast<size_t>(KC) * stride;
  const int rb = static_cast<int>(stride * sizeof(double));      // bytes per row (a coefficient, a component)
  const int voff = lane * static_cast<int>(sizeof(double));
  const double *ag = f.agg + static_cast<size_t>(half) * f.Sg * seg_stride + ell0;
  const double *pr = f.prop + static_cast<size_t>(half) * f.prop_half * stride + ell0;
  double *y = f.y + static_cast<size_t>(half) * (f.Sg + 1) * seg_stride + ell0;
  const auto seg = [&](const double *base, long long s) {  // segment s's KC rows
    return fold_rsrc(base + static_cast<size_t>(s) * seg_stride, static_cast<size_t>(KC) * rb);
  };
  // a propagator (at coefficient offset o) into LDS, kFoldChunk pairs at a time; each pair of
  // coefficient rows through its own descriptor (64-bit base), so no offset exceeds 2 rows --
  // 2 NTC rows of a whole propagator overflow a 32-bit offset from ~640k lines on (KC = 20)
  const auto stage = [&](int o) {
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      if (q % kFoldChunk == 0) __builtin_amdgcn_sched_barrier(0);
      const __amdgpu_buffer_rsrc_t Rq = fold_rsrc(pr + static_cast<size_t>(o + 2 * q) * stride, 2 * static_cast<size_t>(rb));
      lds_p[q * 64 + lane] = make_double2(fold_load(Rq, voff, 0), 2 * q + 1 < NTC ? fold_load(Rq, voff, rb) : 0.0);
    }
  };
  if (f.Sg > 1) stage(0);
  double X[KC], nx[KC];
  {
    const __amdgpu_buffer_rsrc_t R0 = seg(ag, 0);
#pragma unroll
    for (int r = 0; r < KC; ++r) X[r] = fold_load(R0, voff, r * rb);
  }
  if (f.Sg > 1) {
    const __amdgpu_buffer_rsrc_t R1 = seg(ag, 1);
#pragma unroll
    for (int r = 0; r < KC; ++r) nx[r] = fold_load(R1, voff, r * rb);
  }
  for (int s = 1; s <= f.Sg; ++s) {
    if (!f.only_last) {
      const __amdgpu_buffer_rsrc_t Ry = seg(y, s);
#pragma unroll
      for (int r = 0; r < KC; ++r) fold_store(Ry, voff, r * rb, X[r]);
    }
    if (s == f.Sg) break;
    double cur[KC];
#pragma unroll
    for (int r = 0; r < KC; ++r) cur[r] = nx[r];
    if (s + 1 < f.Sg) {  // the next segment's aggregate, in flight during this step
      const __amdgpu_buffer_rsrc_t Rn = seg(ag, s + 1);
#pragma unroll
      for (int r = 0; r < KC; ++r) nx[r] = fold_load(Rn, voff, r * rb);
    }
    if (f.last_short && s == f.Sg - 1) stage(NTC);  // A^Llast for the last step: over P, no longer needed
    // coefficients in tri order = LDS pair order, read in chunks of kFoldChunk pairs: the
    // next chunk's reads are issued before the current chunk's FMAs (two buffers), with a
    // scheduling barrier at each chunk so the compiler cannot hoist every read to the top.
    // An opaque copy of the lane index keeps the loop-invariant reads inside the walk.
    constexpr int CH = kFoldChunk;
    int lo = lane;
    asm volatile("" : "+v"(lo));
    double2 buf[2][CH];
#pragma unroll
    for (int j = 0; j < CH; ++j)
      if (j < NP) buf[0][j] = lds_p[j * 64 + lo];
    double t[KC];
#pragma unroll
    for (int r = 0; r < KC; ++r) {
      double acc = cur[r];
#pragma unroll
      for (int c = 0; c <= r; ++c) {
        const int i = tri(r, c), k = i / (2 * CH), j = (i % (2 * CH)) / 2;
        if (i % (2 * CH) == 0) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int jj = 0; jj < CH; ++jj)
            if ((k + 1) * CH + jj < NP) buf[(k + 1) & 1][jj] = lds_p[((k + 1) * CH + jj) * 64 + lo];
        }
        const double2 pq = buf[k & 1][j];
        acc += ((i & 1) ? pq.y : pq.x) * X[c];
      }
      t[r] = acc;
    }
#pragma unroll
    for (int r = 0; r < KC; ++r) X[r] = t[r];
  }
  if (f.only_last) {
    const __amdgpu_buffer_rsrc_t Ry = fold_rsrc(f.y + ell0, static_cast<size_t>(KC) * rb);
#pragma unroll
    for (int r = 0; r < KC; ++r) fold_store(Ry, voff, r * rb, X[r]);
  }
}

// One chunk of C rows of a T-step pass: correct the loaded rows by the
// pending term of the previous pass (the linear part of the T-level map run
// on the correction state Z), advance every cell through T full steps with
// the per-line affine map W (level t's outputs are level t+1's inputs),
// store, and prefetch the next chunk's rows into the registers just
// consumed.  LAST: the segment's final chunk -- no prefetch, and only its
// first nv cells are real (X is left after cell nv-1).  CB: the map constants
// are scaled by the cell's B_g(T(x)) (bv, prefetched with the rows by bload),
// and phisum accumulates the cell's psi into the fused angular sums.
template <int S, int T, int MODE, int C, bool LAST, bool CB, typename BL, typename PS>
__device__ __forceinline__ void sweep_chunk(const double *W, double (&ein)[C], double (&eout)[C], double (&bv)[C],
                                            double (&X)[T][SchemeDim<S>::K], bool corr,
                                            double (&Z)[T][SchemeDim<S>::K], bool head, double h_oi, double h_oo,
                                            __amdgpu_buffer_rsrc_t Rw, __amdgpu_buffer_rsrc_t Rn, int voff,
                                            int row_bytes, int nv, int k0, const BL &bload, const PS &phisum) {
  constexpr int K = SchemeDim<S>::K;
  double pv[C];  // CB: the chunk's psi, for the fused angular sums
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (LAST && c >= nv) continue;  // wave-uniform: past the end of the segment
    double pin = ein[c], pout = eout[c];
    if (corr) {  // e += (R' A'^k Y): the linear T-level chain on Z, zero data delta at level 0
      double di = 0.0, dd = 0.0;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        double Zn[K], a, e;
        if (t == 0)  // zero data delta at level 0 (resolved at compile time once unrolled)
          map_apply<S, false, true>(W, Z[t], di, dd, Zn, a, e);
        else
          map_apply<S, false>(W, Z[t], di, dd, Zn, a, e);
#pragma unroll
        for (int r = 0; r < K; ++r) Z[t][r] = Zn[r];
        di = a;
        dd = e;
      }
      pin += di;
      pout += dd;
    }
    double oi = pin, oo = pout;
    if constexpr (MODE != 1) {
      if (c == 0 && head) {  // reflective head cell, computed in the prologue
        oi = h_oi;
        oo = h_oo;
      } else {
#pragma unroll
        for (int t = 0; t < T; ++t) {
          double Xn[K], a, e;
          map_apply<S, true>(W, X[t], oi, oo, Xn, a, e, CB ? bv[c] : 1.0);
#pragma unroll
          for (int r = 0; r < K; ++r) X[t][r] = Xn[r];
          oi = a;
          oo = e;
        }
      }
    }
    if constexpr (CB) pv[c] = 0.5 * (oi + oo);
    row_store(Rw, voff, c * row_bytes, oi, oo);
    if constexpr (!LAST) {
      const double2 v = row_load(Rn, voff, c * row_bytes);
      ein[c] = v.x;
      eout[c] = v.y;
      if constexpr (CB) bv[c] = bload(k0 + C + c);
    }
  }
  if constexpr (CB) phisum(pv, LAST ? nv : C, k0);
}

// Fused angular sums of one chunk: vals[c] is this lane's psi in chunk cell c
// (rows k0 + c, c < nv); w psi goes through LDS (one row of 64 lines per
// cell) and each (cell, group) sum over the group's H lines (H divides 64)
// is taken by one lane as four interleaved partial sums (the material path is
// held to a tolerance: the per-half split already departs from the
// reference's single sequential sum), then stored to dst[x][g], x the
// physical cell.  gw0: the wave's first local group.
// LDS tile of group_sums: per cell a row of 64/H groups of H + 1 slots (+1):
// the summing lanes then read from different banks.
constexpr int group_tile_row(int H) { return (64 / H) * (H + 1) + 1; }
constexpr int kGroupTileMax = 16 * 129;  // C = 16 rows, H = 1 (the widest row)

template <int C>
__device__ __forceinline__ void group_sums(const double (&vals)[C], double w, int nv, double *tile, int lane, int H,
                                           int gw0, int Gl, bool neg, int N, int k0, double *dst) {
  const int ngw = 64 / H, RS = group_tile_row(H);
  const int slot = (lane / H) * (H + 1) + lane % H;
#pragma unroll
  for (int c = 0; c < C; ++c) tile[c * RS + slot] = w * vals[c];
  __syncthreads();  // one-wave workgroup: orders the LDS writes before the reads
  const int tasks = ngw * nv;
  for (int t = lane; t < tasks; t += 64) {
    const int c = t / ngw, j = t - c * ngw;
    const double *r = tile + c * RS + j * (H + 1);
    // four interleaved partial sums: a quarter of the dependent-add chain
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int i = 0;
    for (; i + 4 <= H; i += 4) {
      a0 += r[i];
      a1 += r[i + 1];
      a2 += r[i + 2];
      a3 += r[i + 3];
    }
    for (; i < H; ++i) a0 += r[i];
    const double acc = (a0 + a1) + (a2 + a3);
    const int g = gw0 + j, k = k0 + c;
    if (g < Gl) dst[static_cast<size_t>(neg ? N - 1 - k : k) * Gl + g] = acc;
  }
  __syncthreads();  // the tile is rewritten by the next chunk
}

// One pass of T full steps over every line (MODE 0), only the pending
// correction of a T-step pass (MODE 1, finalize before a read-out), or one
// launch of the pipelined schedule (MODE 2): segments at staggered time
// levels, each one pass behind its upwind neighbour, so every segment starts
// from the exact incoming state that neighbour published in the previous
// launch -- no provisional state, no correction.
template <int S, int T, int MODE, bool CB = false>
__global__ __launch_bounds__(64) void sweep_block_kernel(SegArgs a) {
  constexpr int K = SchemeDim<S>::K;
  constexpr int KC = T * K;
  constexpr int WN = map_count<S>();
  constexpr int C = chunk_cells(S, T);
  const int lane = threadIdx.x;
  const size_t stride = static_cast<size_t>(a.Lpad);
  int half, s, q, slot = 0;
  if constexpr (MODE == 2) {
    // active chain positions [pos_lo, pos_lo + npos): two chains of Sg segments
    // (one per half), or one chain of 2 Sg (half 0 then half 1) when reflective
    int pos;
    if (a.reflective) {
      pos = a.pos_lo + static_cast<int>(blockIdx.x) / a.Q;
      q = static_cast<int>(blockIdx.x) % a.Q;
      half = pos / a.Sg;
      s = pos % a.Sg;
    } else {
      const int per_half = a.Q * a.npos;
      half = static_cast<int>(blockIdx.x) / per_half;
      const int rem = static_cast<int>(blockIdx.x) % per_half;
      pos = a.pos_lo + rem / a.Q;
      q = rem % a.Q;
      s = pos;
    }
    slot = (a.pass_lo - (pos - a.pos_lo)) & 1;  // aggregates of pass p live in slot p & 1
  } else {
    const int per_half = a.Q * a.Sg;
    half = a.half0 + static_cast<int>(blockIdx.x) / per_half;
    const int rem = static_cast<int>(blockIdx.x) % per_half;
    s = rem / a.Q;  // segment (wave-uniform)
    q = rem - s * a.Q;
  }
  const int ell = q * 64 + lane;
  const bool neg = half == 0;
  const int k_begin = s * a.Ls;
  const int k_end = min(a.N, k_begin + a.Ls);
  if (k_begin >= k_end) return;
  if (MODE == 1 && s == 0) return;  // segment 0 is never provisional
  const size_t seg_stride = static_cast<size_t>(KC) * stride;
  const size_t half_stride = static_cast<size_t>(a.Sg) * seg_stride;

  // ---- pending correction of the previous pass: Z = true incoming state ----
  const bool corr = MODE != 2 && a.pending && s > 0;
  double Z[T][K];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int r = 0; r < K; ++r) Z[t][r] = 0.0;
  if (corr) {  // folded by fold_kernel from the previous pass's aggregates
    const double *y = a.yseg + (static_cast<size_t>(half) * (a.Sg + 1) + s) * seg_stride + ell;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int r = 0; r < K; ++r) Z[t][r] = y[(t * K + r) * stride];
  }

  // ---- inflow and carried state ----
  const bool head_seg = (s == 0);
  double b[T][4];
  {
    const double v = a.bdry[static_cast<size_t>(half) * stride + ell];
#pragma unroll
    for (int t = 0; t < T; ++t) b[t][0] = b[t][1] = b[t][2] = b[t][3] = v;
  }
  const bool refl_head = MODE != 1 && head_seg && !neg && a.reflective;
  if (refl_head) {
    // solver.cpp:677-684: mu > 0 inflow = the mirror mu < 0 line's outflow of the
    // same steps: folded by fold_kernel from that line's aggregates of this pass
    // (MODE 0), or the aggregate its last segment published (MODE 2)
    const double *src = MODE == 2 ? a.aggs[slot] + (a.Sg - 1) * seg_stride + ell : a.yrefl + ell;
    double Xo[KC];
#pragma unroll
    for (int r = 0; r < KC; ++r) Xo[r] = src[r * stride];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if constexpr (S == SCHEME_BDF2) {
        b[t][0] = Xo[t * K + 1];
        b[t][1] = Xo[t * K + 2];
        b[t][2] = Xo[t * K + 3];
        b[t][3] = Xo[t * K + 4];
      } else {
        b[t][0] = b[t][1] = b[t][2] = b[t][3] = Xo[t * K + K - 1];
      }
    }
  }
  double X[T][K];
  if (head_seg) {
#pragma unroll
    for (int t = 0; t < T; ++t) head_state<S>(b[t], X[t]);
  } else if (MODE == 2) {  // exact: the upwind segment's exit state, published last launch
    const double *up = a.aggs[slot] + half * half_stride + (s - 1) * seg_stride + ell;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int r = 0; r < K; ++r) X[t][r] = up[(t * K + r) * stride];
  } else {
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int r = 0; r < K; ++r) X[t][r] = 0.0;
  }
  const double *hmp = a.hmap + ell;  // the head cell's map (refl_head only)

  // ---- stream the segment in C-row chunks ----
  const int row_bytes = a.Lpad * static_cast<int>(sizeof(double2));
  const int voff = lane * static_cast<int>(sizeof(double2));
  const double2 *Eh = a.E + static_cast<size_t>(half) * a.Nrow * stride + q * 64;
  auto rows = [&](int k0) { return rows_rsrc<C>(Eh + static_cast<size_t>(k0) * stride, row_bytes); };
  // material coupling: B_g(T(x)) of row k (physical cell N-1-k for mu < 0);
  // padding lanes and rows read a clamped, unused value
  const double *bl = nullptr;
  if constexpr (CB) bl = a.bcell + min(ell / a.H, a.Gl - 1);
  auto bload = [&](int k) -> double {
    if constexpr (CB) {
      const int kk = min(k, a.N - 1);
      return bl[static_cast<size_t>(neg ? a.N - 1 - kk : kk) * a.Gl];
    } else {
      return 1.0;
    }
  };
  // material coupling, fused angular sums (group_sums): w_i psi summed over
  // the lines of each group into phi[half][x][g]
  static_assert(C <= 16, "group_sums tile holds 16 rows");
  __shared__ double ptile[CB ? kGroupTileMax : 1];
  double wl = 0.0;
  if constexpr (CB) {
    if (a.phi) {
      const int ip = ell % a.H;
      wl = a.wt[neg ? a.H - 1 - ip : a.H + ip];
    }
  }
  auto phisum = [&](const double (&pv)[C], int nv, int k0) {
    if constexpr (CB) {
      if (a.phi)  // wave-uniform
        group_sums<C>(pv, wl, nv, ptile, lane, a.H, q * 64 / a.H, a.Gl, neg, a.N, k0,
                      a.phi + static_cast<size_t>(half) * a.N * a.Gl);
    }
  };
  double ein[C], eout[C], bv[C];
  {
    const __amdgpu_buffer_rsrc_t R0 = rows(k_begin);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const double2 v = row_load(R0, voff, c * row_bytes);
      ein[c] = v.x;
      eout[c] = v.y;
      bv[c] = bload(k_begin + c);
    }
  }
  // reflective head cell (cell 0 of segment 0, distinct per-substep inflows)
  double h_oi = 0.0, h_oo = 0.0;
  if (refl_head) {
    h_oi = ein[0];
    h_oo = eout[0];
    head_cell<S, T>(hmp, stride, X, h_oi, h_oo, bv[0]);
  }

  // ---- the line's cell map ----
  double W[WN];
#pragma unroll
  for (int n = 0; n < WN; ++n) W[n] = a.map[(static_cast<size_t>(half) * WN + n) * stride + ell];

  int k0 = k_begin;
  for (; k0 + C < k_end; k0 += C) {  // full chunks with a successor
    sweep_chunk<S, T, MODE, C, false, CB>(W, ein, eout, bv, X, corr, Z, refl_head && k0 == 0, h_oi, h_oo, rows(k0),
                                          rows(k0 + C), voff, row_bytes, C, k0, bload, phisum);
  }
  sweep_chunk<S, T, MODE, C, true, CB>(W, ein, eout, bv, X, corr, Z, refl_head && k0 == 0, h_oi, h_oo, rows(k0),
                                       rows(k0), voff, row_bytes, k_end - k0, k0, bload, phisum);
  if constexpr (MODE != 1) {
    double *ag = (MODE == 2 ? a.aggs[slot] : a.agg_cur) + half * half_stride + static_cast<size_t>(s) * seg_stride + ell;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int r = 0; r < K; ++r) ag[(t * K + r) * stride] = X[t][r];
  }
}

// ------------------------------------------------------------------------
// Non-hot kernels: state initialisation, layout conversion, moments
// ------------------------------------------------------------------------
// psi = ends = B_g (solver.cpp:165-181); padding rows k >= N are zero
// E = B_g on every node of every line (solver.cpp:165-181), zero on padding rows:
// a block per row (no 64-bit index division), nt stores (written once, read next pass)
__global__ void init_state_kernel(double2 *E, const double *lineB, int N, int Nrow, int Lpad) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  for (int row = blockIdx.x; row < 2 * Nrow; row += gridDim.x) {
    const int half = row / Nrow, k = row - half * Nrow;
    d2v *dst = reinterpret_cast<d2v *>(E) + static_cast<size_t>(row) * Lpad;
    const double *b = lineB + static_cast<size_t>(half) * Lpad;
    for (int ell = threadIdx.x; ell < Lpad; ell += blockDim.x) {
      const double v = k < N ? b[ell] : 0.0;
      __builtin_nontemporal_store(d2v{v, v}, dst + ell);
    }
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

// The reference-layout exports / import work on a chunk of cells [c0, c0 + nc) so the
// device buffer stays small (rtsn_api.hip: kExportChunk doubles); chunk index
// o = i + M (g + Gl (c - c0)) < M Gl nc < 2^31.

// psi (M, Gl, N) ColMajor = mean of the nodes (solver.cpp:352,389)
__global__ void export_psi_kernel(const double2 *E, double *psi, LineMap m, int c0, int nc) {
  const int MG = m.M * m.Gl, total = MG * nc;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int cl = o / MG, r = o - cl * MG, g = r / m.M, i = r - g * m.M;
    int half, ell, k;
    m.map(i, g, c0 + cl, half, ell, k);
    const double2 v = E[m.at(half, k, ell)];
    psi[o] = 0.5 * (v.x + v.y);
  }
}

// ends (M, Gl, N, 2) ColMajor <-> E; node 0 = left, 1 = right; the chunk buffer
// holds node 0 of the chunk's cells, then node 1
__global__ void export_ends_kernel(const double2 *E, double *ends, LineMap m, int c0, int nc) {
  const int MG = m.M * m.Gl, total = MG * nc;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int cl = o / MG, r = o - cl * MG, g = r / m.M, i = r - g * m.M;
    int half, ell, k;
    m.map(i, g, c0 + cl, half, ell, k);
    const double2 v = E[m.at(half, k, ell)];
    ends[o] = half == 0 ? v.y : v.x;
    ends[o + total] = half == 0 ? v.x : v.y;
  }
}

__global__ void import_ends_kernel(double2 *E, const double *ends, LineMap m, int c0, int nc) {
  const int MG = m.M * m.Gl, total = MG * nc;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int cl = o / MG, r = o - cl * MG, g = r / m.M, i = r - g * m.M;
    int half, ell, k;
    m.map(i, g, c0 + cl, half, ell, k);
    const double l = ends[o], rr = ends[o + total];
    E[m.at(half, k, ell)] = half == 0 ? make_double2(rr, l) : make_double2(l, rr);
  }
}

// phi, F, phi_plus (Gl, N) ColMajor: sequential sums over i in the
// reference's order (solver.cpp:191-237), no FMA contraction.
// One wave per task (cell c, 64 groups): lane = group, running the three sums
// side by side.  The task's rows (row k = N-1-c of half 0 walked with i'
// descending, i = 0..H-1; row k = c of half 1, i = H..M-1) are read in chunks
// of MOM_W directions: each group's MOM_W nodes are one contiguous 128 B run
// (l = i' + H g), so an instruction covers 8 whole cache lines; the chunk is
// transposed through LDS (lane g then reads its MOM_W values), and the next
// chunk's loads are in flight while the current one is summed.  The weights
// are wave-uniform (scalar loads).
// MOM_W directions per chunk: 8 x 16 B = one 128 B line per group, 16 = two (16 KB of the
// state in flight per wave instead of 8: round 4).  23.0 ms on SL (5.7 TB/s of the 131 GB
// state, profiles/archive/r04q_*).  Round 4 measured and removed, all within +-5% of this kernel on
// one box while a plain scan of the same state runs at 6.9 TB/s: 32-direction chunks; a
// register ring of 2-4 chunks in flight per wave; LDS-DMA rings (global_load_lds) of 2-3
// 32 KB units; two passes in row order (half 0's partial sums through the outputs); whole
// rows per 256-thread workgroup loaded like the scan, in two passes and in one.
// FAST: H % MOM_W == 0, so every chunk is 64 groups x MOM_W directions and lane
// (gr, col) = (lane / MOM_W, lane % MOM_W) loads group gr + (64 / MOM_W) r, direction col.
template <bool FAST, int MOM_W>
__global__ void __launch_bounds__(64) moments_kernel(const double2 *__restrict__ E, const double *__restrict__ mu,
                                                     const double *__restrict__ wt, double *phi, double *F,
                                                     double *phi_plus, LineMap m) {
#pragma clang fp contract(off)
  __shared__ double tile[64 * (MOM_W + 1)];
  const int lane = threadIdx.x;
  const int H = m.H;
  const int nchunks = (m.Gl + 63) / 64;
  const int nj = (H + MOM_W - 1) / MOM_W;  // chunks per half
  const size_t tasks = static_cast<size_t>(m.N) * nchunks;
  double2 v[MOM_W];
  // chunk `step` of a task: half 0 chunks j = nj-1 .. 0 (i' descending), then half 1 j = 0 .. nj-1
  auto load = [&](size_t task, int step) {
    const int c = static_cast<int>(task / nchunks);
    const int g0 = static_cast<int>(task % nchunks) * 64;
    const int ng = min(64, m.Gl - g0);
    const int half = step < nj ? 0 : 1;
    const int i0 = (half == 0 ? nj - 1 - step : step - nj) * MOM_W;
    const double2 *row = E + m.at(half, half == 0 ? m.N - 1 - c : c, H * g0 + i0);
    if constexpr (FAST) {
      // descriptor over the chunk's ng groups: groups >= ng read as 0 (bounds-checked), never stored
      const __amdgpu_buffer_rsrc_t R =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<double2 *>(row), 0, ng * H * 16, 0x00020000);
      const int voff = (H * (lane / MOM_W) + lane % MOM_W) * 16;
#pragma unroll
      for (int r = 0; r < MOM_W; ++r) v[r] = row_load(R, voff, r * (64 / MOM_W) * H * 16);
    } else {
      const int w = min(MOM_W, H - i0);
#pragma unroll
      for (int r = 0; r < MOM_W; ++r) {
        const int e = lane + 64 * r;
        if (e < ng * w) v[r] = row[static_cast<size_t>(H) * (e / w) + e % w];
      }
    }
  };
  size_t task = blockIdx.x;
  if (task < tasks) load(task, 0);
  for (; task < tasks; task += gridDim.x) {
    const int c = static_cast<int>(task / nchunks);
    const int g0 = static_cast<int>(task % nchunks) * 64;
    const int ng = min(64, m.Gl - g0);
    double sphi = 0.0, sF = 0.0, splus = 0.0;
    for (int step = 0; step < 2 * nj; ++step) {
      const int half = step < nj ? 0 : 1;
      const int i0 = (half == 0 ? nj - 1 - step : step - nj) * MOM_W;
      const int w = FAST ? MOM_W : min(MOM_W, H - i0);
      if constexpr (FAST) {
        const int gr = lane / MOM_W, col = lane % MOM_W;
#pragma unroll
        for (int r = 0; r < MOM_W; ++r)
          if (gr + (64 / MOM_W) * r < ng) tile[(gr + (64 / MOM_W) * r) * (MOM_W + 1) + col] = 0.5 * (v[r].x + v[r].y);
      } else {
#pragma unroll
        for (int r = 0; r < MOM_W; ++r) {
          const int e = lane + 64 * r;
          if (e < ng * w) tile[(e / w) * (MOM_W + 1) + e % w] = 0.5 * (v[r].x + v[r].y);
        }
      }
      __syncthreads();
      // next chunk (of this task or the next one) in flight during the sums
      if (step + 1 < 2 * nj) load(task, step + 1);
      else if (task + gridDim.x < tasks) load(task + gridDim.x, 0);
      // the chunk's weights, ascending in i (wave-uniform: one scalar load each)
      const int ib = half == 0 ? H - i0 - w : H + i0;  // lowest i of the chunk
      double wv[MOM_W], xv[MOM_W];
#pragma unroll
      for (int k = 0; k < MOM_W; ++k) {
        wv[k] = k < w ? wt[ib + k] : 0.0;
        xv[k] = k < w ? mu[ib + k] : 0.0;
      }
      if (lane < ng) {
        const double *t = tile + lane * (MOM_W + 1);
        if (half == 0) {  // i = H-1-(i0+ii) = ib + (w-1-ii)
#pragma unroll
          for (int ii = MOM_W - 1; ii >= 0; --ii) {
            if (ii < w) {
              const int k = w - 1 - ii;
              const double q = t[ii];
              sphi += wv[k] * q;
              sF += xv[k] * wv[k] * q;
            }
          }
        } else {  // i = H + i0 + ii = ib + ii
#pragma unroll
          for (int ii = 0; ii < MOM_W; ++ii) {
            if (ii < w) {
              const double q = t[ii];
              sphi += wv[ii] * q;
              sF += xv[ii] * wv[ii] * q;
              splus += wv[ii] * q;
            }
          }
        }
      }
      __syncthreads();
    }
    if (lane < ng) {
      const size_t o = static_cast<size_t>(c) * m.Gl + g0 + lane;
      phi[o] = sphi;
      F[o] = sF;
      phi_plus[o] = splus;
    }
  }
}

// Producer/consumer moments (round 5): the same sums, bitwise, from a workgroup of five
// waves with fixed roles.  An item is (cell c, 64 groups): half 0's row k = N-1-c and half
// 1's row k = c, each a contiguous run of 64 H lines (l = i' + H g).  Four loader waves
// (two per half, half the run's 1 KiB load instructions each) stream the runs with
// lane-contiguous 16-byte nt loads, as the state scan reads, into a register ring two items
// deep: while item p's values are converted to psi = (e_in + e_out) / 2 and written to an LDS
// slot [half][group][i'] (row stride H + 1 doubles: conflict-free), the loads of items p + 1
// and p + 2 are in flight, and a loader's only waits are on its own oldest load.  The
// summing wave (lane = group) takes the previous item's slot and runs the three sums over
// i = 0 .. M-1 in the reference's order (solver.cpp:191-237, no FMA contraction; w psi
// computed once for phi and phi_plus, mu w as one product, as moments_kernel).  The five
// waves meet at one barrier per item (LDS traffic drained, lgkmcnt(0); the barrier does not
// wait for the loads in flight), two slots alternating.
// Bytes in flight per CU (two workgroups: 68.6 KB of LDS each, <= 168 VGPRs for three waves
// per SIMD): 4 x 2 x 32 KB = 256 KB -- the first form (one loader per half, one item deep,
// 128 KB) read at 5.94 TB/s (22.1 ms on SL, profiles/r05b_*), the state scan at 6.86.
constexpr int kMomLoadersPerHalf = 2;  // loader waves per half
template <int H>
__global__ void __launch_bounds__(64 * (2 * kMomLoadersPerHalf + 1)) moments_pc_kernel(const double2 *__restrict__ E, const double *__restrict__ mu,
                                                         const double *__restrict__ wt, double *phi, double *F,
                                                         double *phi_plus, LineMap m) {
#pragma clang fp contract(off)
  constexpr int NL = kMomLoadersPerHalf;
  static_assert(64 % H == 0 && H % NL == 0 && H >= 8, "a load of 64 lines covers whole groups");
  constexpr int R = H / NL;             // loads per item of one loader
  constexpr int ST = H + 1;             // doubles per group row in a slot
  constexpr int SLOT = 2 * 64 * ST;     // one item: [half][64 groups][ST]
  __shared__ double lds[2 * SLOT + 4 * H];  // two slots, then (w_i, mu_i w_i) for i < 2H
  double *const wl = lds + 2 * SLOT;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int nchunks = (m.Gl + 63) / 64;
  const long long items = static_cast<long long>(m.N) * nchunks;
  const long long first = blockIdx.x, step = gridDim.x;
  const long long mine = first < items ? (items - 1 - first) / step + 1 : 0;  // this workgroup's items
  const long long phases = (mine + 1) & ~1LL;  // loaders run whole pairs of items (a zero item pads)
  for (int i = threadIdx.x; i < 2 * H; i += blockDim.x) {
    wl[2 * i] = wt[i];
    wl[2 * i + 1] = mu[i] * wt[i];
  }
  __syncthreads();
  const auto sync = [] {  // LDS traffic drained, then the workgroup barrier (loads stay in flight)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
  };
  if (wave < 2 * NL) {  // loader `part` of half h: the run's loads r = part R .. part R + R - 1
    const int h = wave / NL, part = wave % NL;
    typedef double d2v __attribute__((ext_vector_type(2)));
    // item p's run in half h and its lines; lines past them (a partial group chunk) re-read
    // the run's last line, and an item past the workgroup's last reads line 0 of the state:
    // the slot rows they fill belong to no summed group or item
    const auto run = [&](long long p, int &lim) -> const d2v * {
      if (p >= mine) {
        lim = 1;
        return reinterpret_cast<const d2v *>(E);
      }
      const long long it = first + p * step;
      const int c = static_cast<int>(it / nchunks), g0 = static_cast<int>(it % nchunks) * 64;
      lim = min(64, m.Gl - g0) * H;
      return reinterpret_cast<const d2v *>(E + m.at(h, h == 0 ? m.N - 1 - c : c, H * g0));
    };
    // global (not buffer) loads, nt: the buffer form kept the texture addresser busy for the
    // whole kernel (TA_BUSY 4.28e7 cycles per dispatch against 1.98e7 for the state scan's
    // global loads of the same bytes and requests, profiles/r05d_moments_pmc.json)
    const auto load = [&](const d2v *row, int lim, int r) {
      const d2v v = __builtin_nontemporal_load(row + min(lane + 64 * (part * R + r), lim - 1));
      return make_double2(v.x, v.y);
    };
    double2 v0[R], v1[R];  // the ring: items p (v0) and p + 1 (v1), p even
    {
      int l0, l1;
      const d2v *r0 = run(0, l0), *r1 = run(1, l1);
#pragma unroll
      for (int r = 0; r < R; ++r) {  // in ring order (the loop's waits count on it)
        v0[r] = load(r0, l0, r);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        v1[r] = load(r1, l1, r);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // line lane + 64 (part R + r): group lane / H + (64 / H)(part R + r), i' = lane % H
    double *const base = lds + h * 64 * ST + (lane / H) * ST + lane % H + (64 / H) * part * R * ST;
    const auto consume = [&](double2 (&v)[R], long long p) {  // item p in, item p + 2 issued
      double *const slot = base + (p & 1) * SLOT;
      int ln;
      const d2v *rn = run(p + 2, ln);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        slot[(64 / H) * r * ST] = 0.5 * (v[r].x + v[r].y);
        v[r] = load(rn, ln, r);
        __builtin_amdgcn_sched_barrier(0);  // a rolling ring: each load waits only for the oldest
      }
    };
    for (long long p = 0; p < phases; p += 2) {
      consume(v0, p);
      sync();
      consume(v1, p + 1);
      sync();
    }
    sync();  // the summing wave's last item
  } else {  // the summing wave: lane = group of the item
    for (long long p = 0; p <= phases; ++p) {
      if (p > 0 && p - 1 < mine) {
        const long long it = first + (p - 1) * step;
        const int c = static_cast<int>(it / nchunks), g0 = static_cast<int>(it % nchunks) * 64;
        const double *s0 = lds + ((p - 1) & 1) * SLOT + lane * ST;
        const double *s1 = s0 + 64 * ST;
        double sphi = 0.0, sF = 0.0, splus = 0.0;
#pragma unroll 8
        for (int i = 0; i < H; ++i) {  // mu < 0: i' = H - 1 - i
          const double q = s0[H - 1 - i];
          const double wq = wl[2 * i] * q;
          sphi += wq;
          sF += wl[2 * i + 1] * q;
        }
#pragma unroll 8
        for (int i = 0; i < H; ++i) {  // mu > 0: i = H + i'
          const double q = s1[i];
          const double wq = wl[2 * (H + i)] * q;
          sphi += wq;
          sF += wl[2 * (H + i) + 1] * q;
          splus += wq;
        }
        if (g0 + lane < m.Gl) {
          const size_t o = static_cast<size_t>(c) * m.Gl + g0 + lane;
          __builtin_nontemporal_store(sphi, phi + o);
          __builtin_nontemporal_store(sF, F + o);
          __builtin_nontemporal_store(splus, phi_plus + o);
        }
      }
      sync();
    }
  }
}

// NaN/Inf scan of the state: a block per row of the real cells (padding rows and
// lanes hold zeros), one ballot per wave, one flag store per offending wave.
__global__ void finite_scan_kernel(const double2 *E, int *flag, int N, int Nrow, int Lpad) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  for (int r = blockIdx.x; r < 2 * N; r += gridDim.x) {
    const int half = r / N, k = r - half * N;
    const d2v *row = reinterpret_cast<const d2v *>(E) + (static_cast<size_t>(half) * Nrow + k) * Lpad;
    bool bad = false;
    for (int ell = threadIdx.x; ell < Lpad; ell += blockDim.x) {
      const d2v v = __builtin_nontemporal_load(row + ell);
      bad |= !isfinite(v.x) || !isfinite(v.y);
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) *flag = 1;
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

// compute_balance's absorption and emission sums (solver.cpp:262-272) per group:
// ab = sum_c (rho kappa phi_c) dx, sr = sum_c src.  The reference adds sequentially over
// the N cells; here kBalanceParts contiguous cell ranges are summed sequentially (one
// lane per (range, group): a wave's loads of one cell are contiguous), then the ranges'
// partial sums in range order -- a two-level sum, so the result differs from the
// reference's by rounding only (the balance is compared at 1e-9; one lane per group
// over 1e6 cells took 62 ms on SL, latency-bound on its loads).
constexpr int kBalanceParts = 512;

__global__ void balance_partials_kernel(const double *phi, const double *rk, const double *src, double dx,
                                        double *part, int Gl, int N) {
  const long long t = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= static_cast<long long>(kBalanceParts) * Gl) return;
  const int g = static_cast<int>(t % Gl), rp = static_cast<int>(t / Gl);
  const int c0 = static_cast<int>(static_cast<long long>(N) * rp / kBalanceParts);
  const int c1 = static_cast<int>(static_cast<long long>(N) * (rp + 1) / kBalanceParts);
  const double r = rk[g], q = src[g];
  double a = 0.0, e = 0.0;
  const double *col = phi + g;
  for (int c = c0; c < c1; ++c) {
    a = fma(r * col[static_cast<size_t>(c) * Gl], dx, a);
    e += q;
  }
  part[(static_cast<size_t>(rp) * Gl + g) * 2] = a;
  part[(static_cast<size_t>(rp) * Gl + g) * 2 + 1] = e;
}

__global__ void balance_sums_kernel(const double *part, double *ab, double *sr, int Gl) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= Gl) return;
  double a = 0.0, e = 0.0;
  for (int rp = 0; rp < kBalanceParts; ++rp) {
    a += part[(static_cast<size_t>(rp) * Gl + g) * 2];
    e += part[(static_cast<size_t>(rp) * Gl + g) * 2 + 1];
  }
  ab[g] = a;
  sr[g] = e;
}

// ------------------------------------------------------------------------
// Material coupling: Planck group integrals per cell, exchange term, T update
// ------------------------------------------------------------------------
// Planck.h:84-90 (2 ulps)
__device__ __forceinline__ bool nearly_equal(double a, double b) {
  const double d = fabs(a - b);
  return d <= 2.220446049250313e-16 * fabs(a + b) * 2 || d < 2.2250738585072014e-308;
}

// Bose series of the normalised integrals from z1 to z2 of B (Planck.cpp:94-118) and of
// dB/dT (:170-193), side by side: each series' n_terms is the first n >= 32 whose next term
// falls below the accuracy relative to its leading one (capped so a bad input cannot spin).
// The powers e^{-k z} come from one exp and a running product shared by both, and
// P(k z) / k^4 = r (z^3 + r (3 z^2 + r (6 z + 6 r))), P4(k z) / k^4 = z^4 + r (4 z^3 +
// r (12 z^2 + r (24 z + 24 r))) with r = 1/k (rk: a table for k <= 64); the terms are summed
// in ascending k (the reference sums descending): the same values to a few ulps, for two
// exps per pair of series instead of two per term.  Each sum stops at its own n_terms, so
// the pair equals the two series evaluated one after the other, bit for bit.
struct PlanckPair {
  double b, db;
};

__device__ PlanckPair planck_series_pair(double z1, double z2, double accuracy, const double *rk) {
  const double e1 = exp(-z1), f1 = exp(-z2);
  const double a1 = z1 * z1 * z1, b1 = 3.0 * (z1 * z1), c1 = 6.0 * z1;
  const double a2 = z2 * z2 * z2, b2 = 3.0 * (z2 * z2), c2 = 6.0 * z2;
  const double qa1 = (z1 * z1) * (z1 * z1), qb1 = 4.0 * (z1 * z1 * z1), qc1 = 12.0 * (z1 * z1), qd1 = 24.0 * z1;
  const double qa2 = (z2 * z2) * (z2 * z2), qb2 = 4.0 * (z2 * z2 * z2), qc2 = 12.0 * (z2 * z2), qd2 = 24.0 * z2;
  auto pr = [](double r, double a, double b, double c) { return r * (a + r * (b + r * (c + 6.0 * r))); };
  auto pq = [](double r, double a, double b, double c, double d) { return a + r * (b + r * (c + r * (d + 24.0 * r))); };
  auto recip = [rk](int k) { return k <= 64 ? rk[k] : 1.0 / k; };
  const double lead = fmax(e1 * (a1 + b1 + c1 + 6.0), 2.220446049250313e-16);
  const double qlead = fmax(e1 * (qa1 + qb1 + qc1 + qd1 + 24.0), 2.220446049250313e-16);
  const double stop = accuracy * (1.0 - e1) * lead;  // next term <= accuracy, without the divisions
  const double qstop = accuracy * (1.0 - e1) * qlead;
  int n = 32, qn = 32;
  for (double em = exp(-33.0 * z1); n < 4096; ++n, em *= e1)
    if (!(em * pr(recip(n + 1), a1, b1, c1) > stop)) break;
  for (double em = exp(-33.0 * z1); qn < 4096; ++qn, em *= e1)
    if (!(em * pq(recip(qn + 1), qa1, qb1, qc1, qd1) > qstop)) break;
  const int nmax = n > qn ? n : qn;
  double s1 = 0.0, s2 = 0.0, t1 = 0.0, t2 = 0.0, p1 = 1.0, p2 = 1.0;
  for (int k = 1; k <= nmax; ++k) {
    p1 *= e1;
    p2 *= f1;
    if (p1 == 0.0) break;  // e^{-k z1} underflowed: so has every later term
    const double r = recip(k);
    if (k <= n) {
      s1 += p1 * pr(r, a1, b1, c1);
      s2 += p2 * pr(r, a2, b2, c2);
    }
    if (k <= qn) {
      t1 += p1 * pq(r, qa1, qb1, qc1, qd1);
      t2 += p2 * pq(r, qa2, qb2, qc2, qd2);
    }
  }
  return PlanckPair{s1 - s2, t1 - t2};
}

// 12-point Gauss-Legendre of the Planck density and of its temperature derivative over
// [mid - hw, mid + hw] (Planck.cpp:129-140, Planck.h:113-125; k_B = 1 keV/keV), one exp per
// node for both
__device__ PlanckPair planck_gauss_pair(const PlanckCells &pc, double inv_T, double mid, double hw, double pre) {
  double acc = 0.0, dacc = 0.0;
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    const double E = mid + hw * pc.node[r];
    const double ex = exp(E * inv_T), em1 = ex - 1.0;
    acc += hw * pc.weight[r] * (pre * (E * E * E) / em1);
    dacc += hw * pc.weight[r] * (pre * ((E * E) * (E * E)) * (inv_T * inv_T) * ex / (em1 * em1));
  }
  return PlanckPair{acc, dacc};
}

// Planck::integrate_B (Planck.cpp:85-154) and integrate_dBdT (:161-229) for T > 0, the same
// branches: Gauss below z = 0.7, series above z = 0.5, split at z = 0.6; x 4 pi.
// pre = 2 / (h^3 c^2).
__device__ PlanckPair planck_integral_pair(const PlanckCells &pc, double T, double e_min, double e_max, double pre,
                                           const double *rk) {
  if (nearly_equal(e_min, e_max)) return PlanckPair{0.0, 0.0};
  const double inv_T = 1.0 / T;
  const double z1 = e_min * inv_T, z2 = e_max * inv_T;
  const double t3 = (T * T) * T, t4 = (T * T) * (T * T);
  PlanckPair v;
  if (z2 <= 0.7) {
    v = planck_gauss_pair(pc, inv_T, 0.5 * (e_max + e_min), 0.5 * (e_max - e_min), pre);
  } else if (z1 >= 0.5) {
    const PlanckPair sv = planck_series_pair(z1, z2, pc.accuracy, rk);
    v = PlanckPair{pre * t4 * sv.b, pre * t3 * sv.db};
  } else {
    const double e6 = 0.6 * T;
    const PlanckPair gv = planck_gauss_pair(pc, inv_T, 0.5 * (e6 + e_min), 0.5 * (e6 - e_min), pre);
    const PlanckPair sv = planck_series_pair(0.6, z2, pc.accuracy, rk);
    v = PlanckPair{gv.b + pre * t4 * sv.b, gv.db + pre * t3 * sv.db};
  }
  return PlanckPair{v.b * 4.0 * 3.1415926546, v.db * 4.0 * 3.1415926546};
}

// kcon B_g(T) and kcon dB_g/dT(T) of group g (0 .. G-1): the integral over the group, the last
// group the grey remainder a c T^4 - (the integral over groups 0..G-2 as one) and its
// derivative, each only where positive; T <= 0 (or nearly 0, Planck.h:84-90) or not finite: 0
__device__ PlanckPair cell_group_planck(const PlanckCells &pc, double T, int g, double pre, const double *rk) {
  if (!(T > 0.0 && isfinite(T) && !nearly_equal(T, 0.0))) return PlanckPair{0.0, 0.0};
  if (g < pc.G - 1) {
    const PlanckPair v = planck_integral_pair(pc, T, pc.e_edge[g], pc.e_edge[g + 1], pre, rk);
    return PlanckPair{pc.kcon * v.b, pc.kcon * v.db};
  }
  const PlanckPair v = planck_integral_pair(pc, T, pc.e_edge[0], pc.e_edge[pc.G - 1], pre, rk);
  const double rest = pc.a_c * ((T * T) * (T * T)) - v.b;
  const double drest = 4.0 * pc.a_c * ((T * T) * T) - v.db;
  return PlanckPair{rest > 0.0 ? pc.kcon * rest : 0.0, drest > 0.0 ? pc.kcon * drest : 0.0};
}

constexpr double kPlanckPre = 2.0 / ((4.141895e-10 * 4.141895e-10 * 4.141895e-10) * (299.792458 * 299.792458));

// B[x][gl] = kcon * integral over group g_lo + gl at T(x); the last group takes
// the grey remainder a c T^4 - (integral over groups 0..G-2) when positive
// (Planck.cpp:73-76; the sum of the other groups as one integral over their
// joint range, so no shard needs another shard's groups).  T <= 0 (or
// nearly 0, Planck.h:84-90) or not finite: 0.  With the same branches dB/dT
// (the last group 4 a c T^3 - the joint integral).  The coupling's owed emission
// (include/rtsn.h "material", rt_oracle.c material_planck): owed grows by the old
// dB/dT times the last update's dT[x], the next sweep pays pay = max(owed, -B) of it,
// Beff[x][gl] = B + pay, and bpart[x] = b_scale sum_gl sigma_gl dB/dT.  owed and dB/dT
// are the kernel's own, group-major [gl][x] (a wave's 64 cells contiguous).
//
// A block owns 64 cells (one per lane) and walks the groups wave by wave, so
// a wave evaluates ONE group at 64 temperatures -- the branch (Gauss / series
// / split) and the series length are then nearly uniform across the wave --
// and stages the tiles in LDS to write them back as contiguous [x][g] rows.  Four waves
// per SIMD (127 VGPRs, 36 KB of LDS per block, 32-group tiles): the exp and series chains
// are latency-bound at two (SL coupled step: 5.95 -> 4.52 ms, profiles/r06t_material_kernels.json).
constexpr int kPlanckCells = 64, kPlanckGroups = 32, kPlanckThreads = 256;
__global__ __launch_bounds__(kPlanckThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void planck_cells_kernel(PlanckCells pc, const double *Tc, double *B) {
  __shared__ double tile[2][kPlanckCells * (kPlanckGroups + 1)];
  __shared__ double bsum[kPlanckThreads / 64][kPlanckCells];
  __shared__ double rk[65];
  const double pre = kPlanckPre;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  if (threadIdx.x <= 64) rk[threadIdx.x] = threadIdx.x ? 1.0 / threadIdx.x : 0.0;
  const int ntiles = (pc.N + kPlanckCells - 1) / kPlanckCells;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int x0 = t * kPlanckCells, nx = min(kPlanckCells, pc.N - x0);
    const double T = lane < nx ? Tc[x0 + lane] : 0.0;
    const double dT = lane < nx ? pc.dTlast[x0 + lane] : 0.0;
    const bool hot = T > 0.0 && isfinite(T) && !nearly_equal(T, 0.0);
    double bacc = 0.0;  // this wave's groups of sigma_g dB_g/dT at cell lane
    for (int g0 = 0; g0 < pc.Gl; g0 += kPlanckGroups) {
      const int ng = min(kPlanckGroups, pc.Gl - g0);
      __syncthreads();  // rk ready; the previous chunk's tiles written out
      for (int j = wave; j < ng; j += nwave) {
        const int g = pc.g_lo + g0 + j;
        double b = 0.0, db = 0.0;
        if (hot) {
          const PlanckPair v = cell_group_planck(pc, T, g, pre, rk);
          b = v.b;
          db = v.db;
        }
        double pay = 0.0;
        if (lane < nx) {
#pragma clang fp contract(off)
          const size_t o = static_cast<size_t>(g0 + j) * pc.N + x0 + lane;
          const double owed = pc.owed[o] + pc.dB[o] * dT;
          pay = owed > -b ? owed : -b;
          pc.owed[o] = owed - pay;
          pc.dB[o] = db;
        }
        tile[0][lane * (kPlanckGroups + 1) + j] = b;
        tile[1][lane * (kPlanckGroups + 1) + j] = b + pay;
        bacc += pc.sigma[g0 + j] * db;
      }
      __syncthreads();
      for (int i = threadIdx.x; i < nx * ng; i += blockDim.x) {
        const int xl = i / ng, j = i - xl * ng;
        const size_t o = static_cast<size_t>(x0 + xl) * pc.Gl + g0 + j;
        B[o] = tile[0][xl * (kPlanckGroups + 1) + j];
        pc.Beff[o] = tile[1][xl * (kPlanckGroups + 1) + j];
      }
    }
    bsum[wave][lane] = bacc;
    __syncthreads();
    if (wave == 0 && lane < nx) {
      double b = 0.0;
      for (int w = 0; w < nwave; ++w) b += bsum[w][lane];
      pc.bpart[x0 + lane] = pc.b_scale * b;
    }
  }
}

// The cross-segment correction's share of the fused angular sums after a
// coupled pass (T = 1) whose segments s > 0 started from X = 0: the linear
// chain of the map on the true incoming state Z = Y_s (fold_kernel) gives
// each cell's correction (d_in, d_out) -- no state traffic -- and
// group_sums stores the sums of w (d_in + d_out)/2 to phic[half][x][g]
// (segment 0 cells, exact, are never written: zero).  The stored state keeps
// its correction pending (the next pass or a finalize applies it).
// A^L of every line's correction propagator (the map's linear X -> X' block, lower
// triangular: X'_r reads X_0..X_r), packed lower triangle [half][tri_count(K)][Lpad],
// by binary powering; one thread per (half, line).
template <int S>
__global__ void correction_power_kernel(const double *map, double *pow, int L, int Lpad) {
  constexpr int K = SchemeDim<S>::K;
  constexpr int WN = map_count<S>();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 2 * Lpad) return;
  const int half = idx / Lpad, ell = idx % Lpad;
  const size_t stride = static_cast<size_t>(Lpad);
  double W[WN];
#pragma unroll
  for (int n = 0; n < WN; ++n) W[n] = map[(static_cast<size_t>(half) * WN + n) * stride + ell];
  double A[tri_count(K)], P[tri_count(K)];
#pragma unroll
  for (int c = 0; c < K; ++c) {  // column c of A: the map's linear part on unit input c
    double e[K], Zn[K], di, dd;
#pragma unroll
    for (int r = 0; r < K; ++r) e[r] = r == c ? 1.0 : 0.0;
    map_apply<S, false>(W, e, 0.0, 0.0, Zn, di, dd);
#pragma unroll
    for (int r = c; r < K; ++r) A[tri(r, c)] = Zn[r];
  }
#pragma unroll
  for (int r = 0; r < K; ++r)
#pragma unroll
    for (int c = 0; c <= r; ++c) P[tri(r, c)] = r == c ? 1.0 : 0.0;
  auto mul = [&](double (&X)[tri_count(K)], const double (&Y)[tri_count(K)]) {  // X = X Y
    double R[tri_count(K)];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int c = 0; c <= r; ++c) {
        double acc = 0.0;
#pragma unroll
        for (int m = c; m <= r; ++m) acc = fma(X[tri(r, m)], Y[tri(m, c)], acc);
        R[tri(r, c)] = acc;
      }
#pragma unroll
    for (int n = 0; n < tri_count(K); ++n) X[n] = R[n];
  };
  for (int e = L; e > 0; e >>= 1) {
    if (e & 1) mul(P, A);
    if (e > 1) mul(A, A);
  }
  double *out = pow + static_cast<size_t>(half) * tri_count(K) * stride + ell;
#pragma unroll
  for (int n = 0; n < tri_count(K); ++n) out[n * stride] = P[n];
}

// cells per LDS tile of the correction's sums (the tile bounds the waves a CU holds)
constexpr int kPhiChunk = 16;

template <int S>
__global__ __launch_bounds__(64) void phi_correction_kernel(SegArgs a, int nsub, int Lsub, const double *pow) {
  constexpr int K = SchemeDim<S>::K;
  constexpr int WN = map_count<S>();
  constexpr int C = kPhiChunk;
  extern __shared__ double tile[];  // C rows of group_tile_row(H) (launch_phi_correction)
  const int lane = threadIdx.x;
  const size_t stride = static_cast<size_t>(a.Lpad);
  // block -> (piece t = (half, segment, sub-segment), line group q).  Workgroups go to the
  // 8 XCDs round-robin by block index; all Q line groups of a piece share blockIdx % 8,
  // so a cell's row of group sums (written by Q waves) is assembled in one XCD's L2.
  const int xr = static_cast<int>(blockIdx.x) % kXcds, rest = static_cast<int>(blockIdx.x) / kXcds;
  const int q = rest % a.Q;
  const int t = (rest / a.Q) * kXcds + xr;
  if (t >= 2 * a.Sg * nsub) return;  // padding of the piece count to a multiple of kXcds
  const int half = t / (a.Sg * nsub);
  const int j = t % nsub, s = (t / nsub) % a.Sg;
  const int ell = q * 64 + lane;
  const bool neg = half == 0;
  const int seg_end = min(a.N, s * a.Ls + a.Ls);
  const int k_begin = s * a.Ls + j * Lsub, k_end = min(seg_end, k_begin + Lsub);
  if (s == 0 || k_begin >= k_end) return;  // segment 0 starts exact
  double Z[K];
  const double *y = a.yseg + (static_cast<size_t>(half) * (a.Sg + 1) + s) * K * stride + ell;
#pragma unroll
  for (int r = 0; r < K; ++r) Z[r] = y[r * stride];
  if (j > 0) {  // the state entering sub-segment j: (A^Lsub)^j Z (pow: packed lower triangle)
    const double *pw = pow + static_cast<size_t>(half) * tri_count(K) * stride + ell;
    double P[tri_count(K)];
#pragma unroll
    for (int n = 0; n < tri_count(K); ++n) P[n] = pw[n * stride];
    for (int i = 0; i < j; ++i) {
#pragma unroll
      for (int r = K - 1; r >= 0; --r) {  // in place, rows from the bottom (lower triangular)
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m <= r; ++m) acc = fma(P[tri(r, m)], Z[m], acc);
        Z[r] = acc;
      }
    }
  }
  double W[WN];
#pragma unroll
  for (int n = 0; n < WN; ++n) W[n] = a.map[(static_cast<size_t>(half) * WN + n) * stride + ell];
  const int ip = ell % a.H;
  const double wl = a.wt[neg ? a.H - 1 - ip : a.H + ip];
  double *dst = a.phic + static_cast<size_t>(half) * a.N * a.Gl;
  // CN / BDF2: row 0 copies d_out = 0, so X[0] is 0 after the segment's first cell (and at
  // every sub-segment start): that cell runs the full linear map, the rest skip column 0
  constexpr bool Z0 = map_copy_row0<S>();
  double d_first = 0.0;
  if (Z0 && j == 0) {
    double Zn[K], di, dd;
    map_apply<S, false, true>(W, Z, 0.0, 0.0, Zn, di, dd);
#pragma unroll
    for (int r = 0; r < K; ++r) Z[r] = Zn[r];
    d_first = 0.5 * (di + dd);
  }
  for (int k0 = k_begin; k0 < k_end; k0 += C) {
    const int nv = min(C, k_end - k0);
    double d[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      d[c] = 0.0;
      if (c >= nv) continue;  // wave-uniform
      if (Z0 && j == 0 && c == 0 && k0 == k_begin) {  // wave-uniform: done above
        d[c] = d_first;
        continue;
      }
      double Zn[K], di, dd;
      map_apply<S, false, true, Z0>(W, Z, 0.0, 0.0, Zn, di, dd);
#pragma unroll
      for (int r = 0; r < K; ++r) Z[r] = Zn[r];
      d[c] = 0.5 * (di + dd);
    }
    group_sums<C>(d, wl, nv, tile, lane, a.H, q * 64 / a.H, a.Gl, neg, a.N, k0, dst);
  }
}

// The correction's share for BE and CN, in closed form.  The map's linear part moves the
// correction state Z with no data delta (d_in = d_out = 0): BE carries one scalar, and
// CN's first component is the copied d_out = 0 after one cell, so from the second cell of
// a segment on both carry one live scalar y with y' = lambda y and the cell's share
// (d_in + d_out)/2 = mu y (lambda, mu: the map's linear part on the unit live component).
// At cell m of a segment the line adds
//   m = 0:  w f,                       f = (d_in + d_out)/2 of Z = z (the segment's
//                                      incoming correction state, yseg)
//   m >= 1: w mu y1 lambda^(m-1),      y1 = the live component after cell 0
// Instead of walking each line cell by cell and reducing over the group's lines per
// cell, lanes run over cells: wave w of a workgroup owns group g = 8 gb + w, keeps
// p_i = lambda_i^(m-1) for its H <= 32 lines in registers (by binary powering at the
// workgroup's start, then times lambda_i^64 per 64-cell chunk) and sums c_i p_i; the 8
// waves' rows go through LDS to [x][g] stores of 8 consecutive groups.  2 FP64
// operations per cell and line against the walk's map application plus an LDS tile
// reduction.
constexpr int kGeoLines = 32;   // lines per group and half held in registers (H <= 32)
constexpr int kGeoWaves = 8;    // groups (waves) per workgroup
constexpr int kGeoRange = 2048; // cells per workgroup (32 chunks of 64)

__device__ __forceinline__ double pow_u(double x, unsigned e) {
  double r = 1.0;
  for (; e; e >>= 1) {
    if (e & 1) r *= x;
    x *= x;
  }
  return r;
}

template <int S>
__global__ __launch_bounds__(64 * kGeoWaves) void phi_correction_geo_kernel(SegArgs a, int ranges, int gblocks) {
  static_assert(S == SCHEME_BE || S == SCHEME_CN, "one live scalar after the first cell");
  constexpr int K = SchemeDim<S>::K;
  constexpr int WN = map_count<S>();
  // per wave and line: w mu y1, lambda, lambda^64, lambda^e0 (e0 = m0 - 1, or 0), w f
  __shared__ double uni[kGeoWaves][5][kGeoLines];
  __shared__ double tile[64][kGeoWaves + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const size_t stride = static_cast<size_t>(a.Lpad);
  int b = blockIdx.x;
  const int gb = b % gblocks;
  b /= gblocks;
  const int r = b % ranges;
  b /= ranges;
  const int s = 1 + b % (a.Sg - 1), half = b / (a.Sg - 1);  // segment 0 starts exact
  const bool neg = half == 0;
  const int k_seg = s * a.Ls, seg_len = min(a.Ls, a.N - k_seg);
  const int m0 = r * kGeoRange, m_end = min(seg_len, m0 + kGeoRange);
  if (m0 >= m_end) return;  // workgroup-uniform
  const int g = gb * kGeoWaves + w, H = a.H;
  const bool gv = g < a.Gl;  // wave-uniform
  if (gv && lane < H) {
    const int ell = g * H + lane;
    double W[WN];
#pragma unroll
    for (int n = 0; n < WN; ++n) W[n] = a.map[(static_cast<size_t>(half) * WN + n) * stride + ell];
    double z[K], zn[K], di, dd, u[K], un[K], ui, ud;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      z[k] = a.yseg[((static_cast<size_t>(half) * (a.Sg + 1) + s) * K + k) * stride + ell];
      u[k] = k == K - 1 ? 1.0 : 0.0;
    }
    map_apply<S, false>(W, z, 0.0, 0.0, zn, di, dd);  // cell 0
    map_apply<S, false>(W, u, 0.0, 0.0, un, ui, ud);  // the live component's propagator
    const double wl = a.wt[neg ? H - 1 - lane : H + lane];
    const double lam = un[K - 1];
    uni[w][0][lane] = wl * (0.5 * (ui + ud)) * zn[K - 1];
    uni[w][1][lane] = lam;
    uni[w][2][lane] = pow_u(lam, 64);
    uni[w][3][lane] = pow_u(lam, static_cast<unsigned>(m0 > 0 ? m0 - 1 : 0));
    uni[w][4][lane] = wl * (0.5 * (di + dd));
  }
  __syncthreads();
  double c[kGeoLines], a64[kGeoLines], p[kGeoLines];
  double f0 = 0.0;  // cell 0 of the segment (m0 = 0, lane 0): the sum of w f over the lines
  const unsigned el = static_cast<unsigned>(m0 > 0 ? lane : (lane > 0 ? lane - 1 : 0));
#pragma unroll
  for (int i = 0; i < kGeoLines; ++i) {
    c[i] = 0.0;
    a64[i] = 0.0;
    p[i] = 0.0;
    if (gv && i < H) {  // wave-uniform
      c[i] = uni[w][0][i];
      a64[i] = uni[w][2][i];
      p[i] = uni[w][3][i] * pow_u(uni[w][1][i], el);  // lambda_i^(m0 + lane - 1)
      f0 += uni[w][4][i];
    }
  }
  const int t_cell = threadIdx.x / kGeoWaves, t_g = threadIdx.x % kGeoWaves, t_gg = gb * kGeoWaves + t_g;
  for (int m = m0; m < m_end; m += 64) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < kGeoLines; ++i) {
      acc = fma(c[i], p[i], acc);
      p[i] *= a64[i];
    }
    if (m == 0 && lane == 0) {  // cell 0 (its Z is the incoming state itself); cell 64 next
      acc = f0;
#pragma unroll
      for (int i = 0; i < kGeoLines; ++i)
        if (gv && i < H) p[i] = pow_u(uni[w][1][i], 63);
    }
    tile[lane][w] = acc;
    __syncthreads();
    // 512 threads store 64 cells x 8 groups: each cell's 8 groups are one 64-byte run
    if (t_gg < a.Gl && m + t_cell < m_end) {
      const int k = k_seg + m + t_cell;
      a.phic[(static_cast<size_t>(half) * a.N + (neg ? a.N - 1 - k : k)) * a.Gl + t_gg] = tile[t_cell][t_g];
    }
    __syncthreads();
  }
}

// The correction's share for BDF2 (any scheme whose map copies a zero d_out into X[0]),
// lanes over cells.  After a segment's cell 0 the correction state lives in the KL = K-1
// components X[1..K-1] and moves by the lower-triangular A (the map's linear part on
// them); the share of cell m >= 1 is b A^(m-1) Z1 (b: (d_in + d_out)/2 on a unit
// component, Z1 the state after cell 0).  corr_rows_kernel tabulates per line the row
// vectors R_j = b A^j (j < 64) and A^64 once per handle; phi_correction_rows_kernel gives
// lane j of a 64-cell chunk starting at cell m the share R_j . v with v = w A^(m-1) Z1
// (one vector per line, broadcast through LDS, advanced by A^64 per chunk): KL FMAs per
// cell and line, no walk along the segment and no per-cell reduction across lanes.
constexpr int kRowsRep = 1;                // cells per lane and chunk (v read once for them)
constexpr int kRowsLen = 64 * kRowsRep;    // R_j per line: one per cell of a chunk
constexpr int kRowsLines = 16;             // lines per wave (R_j of each held in registers)
constexpr int kRowsWaves = 8;              // waves per workgroup
constexpr int kRowsSquarings = 6;          // A^kRowsLen = A^(2^6)
constexpr int kRowsBatch = 4;              // chunks per barrier round (their v staged together)
static_assert(kRowsLen == 1 << kRowsSquarings, "chunk length");

template <int S>
__global__ void corr_rows_kernel(const double *map, double *rows, double *a64, int Lpad) {
  constexpr int K = SchemeDim<S>::K, KL = K - 1, WN = map_count<S>();
  static_assert(map_copy_row0<S>(), "X[0] is the copied zero d_out after one cell");
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 2 * Lpad) return;
  const int half = idx / Lpad, ell = idx % Lpad;
  const size_t stride = static_cast<size_t>(Lpad);
  double W[WN];
#pragma unroll
  for (int n = 0; n < WN; ++n) W[n] = map[(static_cast<size_t>(half) * WN + n) * stride + ell];
  double A[tri_count(KL)], b[KL];
#pragma unroll
  for (int c = 0; c < KL; ++c) {  // live component c = X[c + 1]
    double e[K], Zn[K], di, dd;
#pragma unroll
    for (int r = 0; r < K; ++r) e[r] = r == c + 1 ? 1.0 : 0.0;
    map_apply<S, false, true>(W, e, 0.0, 0.0, Zn, di, dd);
#pragma unroll
    for (int r = c; r < KL; ++r) A[tri(r, c)] = Zn[r + 1];
    b[c] = 0.5 * (di + dd);
  }
  double *out = rows + (static_cast<size_t>(half) * stride + ell) * KL * kRowsLen;
  for (int j = 0; j < kRowsLen; ++j) {  // R_j, then R_{j+1} = R_j A
#pragma unroll
    for (int c = 0; c < KL; ++c) out[c * kRowsLen + j] = b[c];
    double Rn[KL];
#pragma unroll
    for (int c = 0; c < KL; ++c) {
      double acc = 0.0;
#pragma unroll
      for (int r = c; r < KL; ++r) acc = fma(b[r], A[tri(r, c)], acc);
      Rn[c] = acc;
    }
#pragma unroll
    for (int c = 0; c < KL; ++c) b[c] = Rn[c];
  }
#pragma unroll
  for (int sq = 0; sq < kRowsSquarings; ++sq) {  // A^kRowsLen by squaring
    double Rm[tri_count(KL)];
#pragma unroll
    for (int r = 0; r < KL; ++r)
#pragma unroll
      for (int c = 0; c <= r; ++c) {
        double acc = 0.0;
#pragma unroll
        for (int m = c; m <= r; ++m) acc = fma(A[tri(r, m)], A[tri(m, c)], acc);
        Rm[tri(r, c)] = acc;
      }
#pragma unroll
    for (int n = 0; n < tri_count(KL); ++n) A[n] = Rm[n];
  }
#pragma unroll
  for (int n = 0; n < tri_count(KL); ++n) a64[(static_cast<size_t>(half) * tri_count(KL) + n) * stride + ell] = A[n];
}

template <int KL>
__device__ __forceinline__ void tri_apply(const double (&P)[tri_count(KL)], double (&v)[KL]) {
#pragma unroll
  for (int r = KL - 1; r >= 0; --r) {  // in place, rows from the bottom (lower triangular)
    double acc = 0.0;
#pragma unroll
    for (int m = 0; m <= r; ++m) acc = fma(P[tri(r, m)], v[m], acc);
    v[r] = acc;
  }
}

// grid: [half][segment 1..Sg-1][cell range][block of 8 groups].  The workgroup takes its 8
// groups in rounds of gpw = 8 / wpg groups: wave w takes group w / wpg of the round, lines
// (w % wpg) * 16 .. +16 of it (LW = kRowsLines = 16, wpg = ceil(H / 16) <= 2 for H <= 32);
// lane j of a chunk starting at cell m
// gives cells m + j + 64 c (c < kRowsRep) with R_(j + 64 c); each chunk's sums leave as
// runs of gpw groups per cell.
// Range r covers cells 1 + r * kRowsRange .. (r + 1) * kRowsRange; range 0 also cell 0.
constexpr int kRowsRange = 8192;

template <int S>
__global__ __launch_bounds__(64 * kRowsWaves) void phi_correction_rows_kernel(SegArgs a, int ranges, int gblocks,
                                                                              int wpg, const double *rows,
                                                                              const double *a64) {
  constexpr int K = SchemeDim<S>::K, KL = K - 1, WN = map_count<S>(), LW = kRowsLines, NG = kRowsWaves;
  constexpr int NB = kRowsBatch;
  __shared__ double vsh[kRowsWaves][NB][LW][KL];  // v of the round's NB chunks
  __shared__ double fsh[kRowsWaves][LW];
  __shared__ double tile[NB * kRowsLen][kRowsWaves + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const size_t stride = static_cast<size_t>(a.Lpad);
  int b = blockIdx.x;
  const int gb = b % gblocks;
  b /= gblocks;
  const int r = b % ranges;
  b /= ranges;
  const int s = 1 + b % (a.Sg - 1), half = b / (a.Sg - 1);
  const bool neg = half == 0;
  const int k_seg = s * a.Ls, seg_len = min(a.Ls, a.N - k_seg);
  const int base = r * kRowsRange, c0 = base + 1, c_end = min(seg_len, c0 + kRowsRange);
  const int gpw = kRowsWaves / wpg, H = a.H, rounds = (NG + gpw - 1) / gpw;
  const int i0 = (w % wpg) * LW, nl = min(LW, H - i0);
  const int t_cell = threadIdx.x / kRowsWaves, t_g = threadIdx.x % kRowsWaves;
  constexpr int kCellsPerPass = 64;  // the 512 threads store 64 cells x 8 groups per pass
  auto cell_index = [&](int m, int gl) {
    const int k = k_seg + m;
    return (static_cast<size_t>(half) * a.N + (neg ? a.N - 1 - k : k)) * a.Gl + gb * NG + gl;
  };
  for (int round = 0; round < rounds; ++round) {
    const int gloc = round * gpw + w / wpg, g = gb * NG + gloc;
    const bool gv = w < gpw * wpg && gloc < NG && g < a.Gl;  // wave-uniform
    double v[KL], P[tri_count(KL)];
#pragma unroll
    for (int c = 0; c < KL; ++c) v[c] = 0.0;
#pragma unroll
    for (int n = 0; n < tri_count(KL); ++n) P[n] = 0.0;
    double f = 0.0;
    if (gv && lane < nl) {
      const int ell = g * H + i0 + lane;
      double W[WN], z[K], Z1[K], di, dd;
#pragma unroll
      for (int n = 0; n < WN; ++n) W[n] = a.map[(static_cast<size_t>(half) * WN + n) * stride + ell];
#pragma unroll
      for (int k = 0; k < K; ++k)
        z[k] = a.yseg[((static_cast<size_t>(half) * (a.Sg + 1) + s) * K + k) * stride + ell];
      map_apply<S, false, true>(W, z, 0.0, 0.0, Z1, di, dd);  // cell 0 (its share from z itself)
      const double wl = a.wt[neg ? H - 1 - i0 - lane : H + i0 + lane];
      f = wl * (0.5 * (di + dd));
#pragma unroll
      for (int c = 0; c < KL; ++c) v[c] = Z1[c + 1];
#pragma unroll
      for (int n = 0; n < tri_count(KL); ++n)
        P[n] = a64[(static_cast<size_t>(half) * tri_count(KL) + n) * stride + ell];
      // v = A^(c0 - 1) Z1 = (A^L)^(base / L) Z1 (L = kRowsLen), binary powering of A^L
      double Q[tri_count(KL)];
#pragma unroll
      for (int n = 0; n < tri_count(KL); ++n) Q[n] = P[n];
      for (unsigned e = static_cast<unsigned>(base / kRowsLen); e; e >>= 1) {
        if (e & 1) tri_apply<KL>(Q, v);
        if (e > 1) {
          double Rm[tri_count(KL)];
#pragma unroll
          for (int rr = 0; rr < KL; ++rr)
#pragma unroll
            for (int c = 0; c <= rr; ++c) {
              double acc = 0.0;
#pragma unroll
              for (int m = c; m <= rr; ++m) acc = fma(Q[tri(rr, m)], Q[tri(m, c)], acc);
              Rm[tri(rr, c)] = acc;
            }
#pragma unroll
          for (int n = 0; n < tri_count(KL); ++n) Q[n] = Rm[n];
        }
      }
#pragma unroll
      for (int c = 0; c < KL; ++c) v[c] *= wl;
    }
    if (lane < LW) {
      fsh[w][lane] = f;
#pragma unroll
      for (int c = 0; c < KL; ++c) vsh[w][0][lane][c] = v[c];
#pragma unroll
      for (int qb = 1; qb < NB; ++qb) {
        tri_apply<KL>(P, v);
#pragma unroll
        for (int c = 0; c < KL; ++c) vsh[w][qb][lane][c] = v[c];
      }
    }
    double R[kRowsRep][LW][KL];  // R_(lane + 64 c) of each of the wave's lines (0 for absent lines)
#pragma unroll
    for (int cc = 0; cc < kRowsRep; ++cc)
#pragma unroll
      for (int i = 0; i < LW; ++i)
#pragma unroll
        for (int c = 0; c < KL; ++c) {
          R[cc][i][c] = 0.0;
          if (gv && i < nl)  // wave-uniform
            R[cc][i][c] =
                rows[((static_cast<size_t>(half) * stride + g * H + i0 + i) * KL + c) * kRowsLen + 64 * cc + lane];
        }
    __syncthreads();
    const bool t_store = t_g < gpw && round * gpw + t_g < NG && gb * NG + round * gpw + t_g < a.Gl;
    if (r == 0 && t_cell == 0 && t_store) {  // cell 0 of the segment
      double acc = 0.0;
      for (int p = 0; p < wpg; ++p)
        for (int i = 0; i < LW; ++i) acc += fsh[t_g * wpg + p][i];
      a.phic[cell_index(0, round * gpw + t_g)] = acc;
    }
    for (int m = c0; m < c_end; m += NB * kRowsLen) {
#pragma unroll
      for (int qb = 0; qb < NB; ++qb) {
        double acc[kRowsRep];
#pragma unroll
        for (int cc = 0; cc < kRowsRep; ++cc) acc[cc] = 0.0;
#pragma unroll
        for (int i = 0; i < LW; ++i)
#pragma unroll
          for (int c = 0; c < KL; ++c) {
            const double vv = vsh[w][qb][i][c];
#pragma unroll
            for (int cc = 0; cc < kRowsRep; ++cc) acc[cc] = fma(R[cc][i][c], vv, acc[cc]);
          }
#pragma unroll
        for (int cc = 0; cc < kRowsRep; ++cc) tile[qb * kRowsLen + 64 * cc + lane][w] = acc[cc];
      }
      __syncthreads();
#pragma unroll
      for (int cc = 0; cc < NB * kRowsLen / kCellsPerPass; ++cc) {
        const int mc = cc * kCellsPerPass + t_cell;
        if (t_store && m + mc < c_end) {
          double sum = tile[mc][t_g * wpg];
          for (int p = 1; p < wpg; ++p) sum += tile[mc][t_g * wpg + p];
          a.phic[cell_index(m + mc, round * gpw + t_g)] = sum;
        }
      }
      if (lane < LW) {  // the next round's chunks: v = A^kRowsLen v, NB times
#pragma unroll
        for (int qb = 0; qb < NB; ++qb) {
          tri_apply<KL>(P, v);
#pragma unroll
          for (int c = 0; c < KL; ++c) vsh[w][qb][lane][c] = v[c];
        }
      }
      __syncthreads();
    }
    // the next round rewrites fsh / vsh: a range with no chunk (c0 >= c_end, e.g. range 0 of a
    // one-cell last segment) has passed no barrier since the cell-0 sum read fsh above
    __syncthreads();
  }
}

// q(x) = sum_g sigma_g (phi_g(x) - W B_g(x)), phi the sum of nparts arrays
// [part][x][g] (the fused halves and their corrections, or one full phi):
// one wave per cell, lanes over groups, then a butterfly over the wave
__global__ void material_q_kernel(const double *phi, int nparts, const double *B, const double *sigma, double W,
                                  const double *bpart, double *q, int Gl, int N) {
  const int lane = threadIdx.x & 63;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  const size_t NG = static_cast<size_t>(N) * Gl;
  for (int x = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; x < N; x += nw) {
    const size_t o = static_cast<size_t>(x) * Gl;
    double acc = 0.0;
    for (int g = lane; g < Gl; g += 64) {
      double ph = phi[o + g];
      for (int p = 1; p < nparts; ++p) ph += phi[p * NG + o + g];
      acc += sigma[g] * (ph - W * B[o + g]);
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) {
      q[x] = acc;
      q[N + x] = bpart[x];  // the exchange buffer's second half: this handle's sum sigma dB/dT
    }
  }
}

// dT = dt q / (rho_cv + dt W b), T += dT (rt_oracle.c orc_material_update, the same
// expressions unfused); dT kept for the next Planck pass's owed emission
// S(T) = sum over ALL G groups of sigma_g B_g(T) and its derivative (rt_oracle.c
// material_emission_all)
__device__ PlanckPair material_emission_all(const PlanckCells &pc, double T, const double *rk) {
  double a = 0.0, d = 0.0;
  for (int g = 0; g < pc.G; ++g) {
    const PlanckPair v = cell_group_planck(pc, T, g, kPlanckPre, rk);
    a += pc.sigma_all[g] * v.b;
    d += pc.sigma_all[g] * v.db;
  }
  return PlanckPair{a, d};
}

// dT = dt q / (rho_cv + dt W b), T += dT (rt_oracle.c orc_material_update, the same
// expressions unfused); dT kept for the next Planck pass's owed emission.  Where dT > T / 4
// the tangent of the convex B under-counts the emission at the new T (heating a cold cell
// beside hot ones, the linear update overshot by 10^3 and diverged; cooling it only lags):
// the cell solves rho_cv (T' - T) = dt (A - W S(T')),
// A = q + W S(T), S over all groups -- increasing, 0 for T' <= 0: one root, bracketed in
// [0, T + dt A / rho_cv] -- by Newton's method with bisection (rt_oracle.c material_solve_cell);
// its owed emission grows by B_g(T') - B_g(T) here and dTlast is 0 (no dB/dT dT term).
constexpr double kNewtonFrac = 0.25;
__global__ void material_update_kernel(PlanckCells pc, double *T, const double *qb, double *dTlast, double dt,
                                       double rho_cv, double W, int N) {
  __shared__ double rk[65];
  if (threadIdx.x <= 64) rk[threadIdx.x] = threadIdx.x ? 1.0 / threadIdx.x : 0.0;
  __syncthreads();
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < N; x += gridDim.x * blockDim.x) {
    const double q = qb[x], b = qb[N + x], T0 = T[x];
    double dT;
    {
#pragma clang fp contract(off)
      dT = dt * q / (rho_cv + dt * W * b);
    }
    if (dT <= kNewtonFrac * T0) {
#pragma clang fp contract(off)
      T[x] = T0 + dT;
      dTlast[x] = dT;
      continue;
    }
    const PlanckPair s0 = material_emission_all(pc, T0, rk);
    const double A = q + W * s0.b;
    const double hi0 = T0 + dt * A / rho_cv;  // f(hi0) = dt W S(hi0) >= 0
    double Tn = hi0;
    if (hi0 > 0.0) {
      double lo = 0.0, hi = hi0, t = T0 > 0.0 && T0 < hi0 ? T0 : 0.5 * hi0;
      if (T0 > 0.0 && s0.b > 0.0) {
        // start at the root of the grey model S(T') ~ S(T0) (T'/T0)^4 (no Planck terms; from
        // the linear update, above it: Newton on the convex model converges from the right)
        const double k = dt * W * s0.b / (T0 * T0 * T0 * T0);
        double m = fmin(T0 + dT, hi0);
        for (int it = 0; it < 60; ++it) {
          const double m2 = m * m, fm = rho_cv * (m - T0) + k * m2 * m2 - dt * A;
          const double mn = m - fm / (rho_cv + 4.0 * k * m2 * m);
          if (!(mn > 0.0) || fabs(mn - m) <= 1e-3 * m) {
            m = mn > 0.0 ? mn : m;
            break;
          }
          m = mn;
        }
        if (m > lo && m < hi) t = m;
      }
      Tn = t;
      for (int it = 0; it < 200; ++it) {
        const PlanckPair sv = material_emission_all(pc, t, rk);
        const double f = rho_cv * (t - T0) + dt * W * sv.b - dt * A;
        if (f > 0.0) hi = t; else lo = t;
        double tn = t - f / (rho_cv + dt * W * sv.db);
        if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
        Tn = tn;
        if (fabs(tn - t) <= 1e-15 * fabs(tn) || hi - lo <= 1e-15 * hi) break;
        t = tn;
      }
    }
    // the material emitted B_g(T') - B_g(T0) beyond the sweep's B: owed now, no dT term next
    for (int gl = 0; gl < pc.Gl; ++gl) {
#pragma clang fp contract(off)
      const size_t o = static_cast<size_t>(gl) * N + x;
      pc.owed[o] = pc.owed[o] + (cell_group_planck(pc, Tn, pc.g_lo + gl, kPlanckPre, rk).b -
                                 pc.Bcell[static_cast<size_t>(x) * pc.Gl + gl]);
    }
    T[x] = Tn;
    dTlast[x] = 0.0;
  }
}

// E[x] = dt W sum_gl sigma_gl ((Beff - B) + owed): the energy per volume the material owes
// the radiation (rt_get_material_transit); one wave per cell, lanes over groups
__global__ void material_transit_kernel(const double *B, const double *Beff, const double *owed, const double *sigma,
                                        double scale, double *E, int Gl, int N) {
  const int lane = threadIdx.x & 63;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  for (int x = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; x < N; x += nw) {
    const size_t o = static_cast<size_t>(x) * Gl;
    double acc = 0.0;
    for (int g = lane; g < Gl; g += 64)
      acc += sigma[g] * ((Beff[o + g] - B[o + g]) + owed[static_cast<size_t>(g) * N + x]);
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) E[x] = scale * acc;
  }
}

// ------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------
template <int S, int T>
static hipError_t launch_t(int mode, const SegArgs &a, int grid, hipStream_t st) {
  if (a.bcell) {  // material coupling: one full step per aligned pass
    if constexpr (T == 1) {
      if (mode == SWEEP_PASS) {
        hipLaunchKernelGGL((sweep_block_kernel<S, 1, 0, true>), dim3(grid), dim3(64), 0, st, a);
        return hipGetLastError();
      }
    }
    if (mode != SWEEP_FINALIZE) return hipErrorInvalidValue;  // the correction has no source term
  }
  if (mode == SWEEP_PIPELINED) {
    if (a.level_waves != 1) {  // level-split pass (kernels_split.hip)
      if constexpr (level_split_supported(S, T)) return launch_split(T, a.level_waves, a, grid, st);
      return hipErrorInvalidValue;
    }
    if constexpr (one_wave_block(S, T)) {
      hipLaunchKernelGGL((sweep_block_kernel<S, T, 2>), dim3(grid), dim3(64), 0, st, a);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if constexpr (T <= kMaxAlignedBlock) {
    if (mode == SWEEP_PASS)
      hipLaunchKernelGGL((sweep_block_kernel<S, T, 0>), dim3(grid), dim3(64), 0, st, a);
    else if (mode == SWEEP_FINALIZE)
      hipLaunchKernelGGL((sweep_block_kernel<S, T, 1>), dim3(grid), dim3(64), 0, st, a);
    else
      return hipErrorInvalidValue;
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

template <int S>
static hipError_t launch_s(int T, int mode, const SegArgs &a, int grid, hipStream_t st) {
  switch (T) {
    case 1: return launch_t<S, 1>(mode, a, grid, st);
    case 2: return launch_t<S, 2>(mode, a, grid, st);
    case 3: return launch_t<S, 3>(mode, a, grid, st);
    case 4: return launch_t<S, 4>(mode, a, grid, st);
    case 5: return launch_t<S, 5>(mode, a, grid, st);
    case 6: return launch_t<S, 6>(mode, a, grid, st);
    case 7: return launch_t<S, 7>(mode, a, grid, st);
    case 8: return launch_t<S, 8>(mode, a, grid, st);
    case 10: return launch_t<S, 10>(mode, a, grid, st);
    case 12: return launch_t<S, 12>(mode, a, grid, st);
    case 16: return launch_t<S, 16>(mode, a, grid, st);
    case 20: return launch_t<S, 20>(mode, a, grid, st);
    case 24: return launch_t<S, 24>(mode, a, grid, st);
    case 32: return launch_t<S, 32>(mode, a, grid, st);
    case 40: return launch_t<S, 40>(mode, a, grid, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_sweep(int scheme, int T, int mode, const SegArgs &a, int grid, hipStream_t st) {
  switch (scheme) {
    case SCHEME_BE: return launch_s<SCHEME_BE>(T, mode, a, grid, st);
    case SCHEME_CN: return launch_s<SCHEME_CN>(T, mode, a, grid, st);
    default: return launch_s<SCHEME_BDF2>(T, mode, a, grid, st);
  }
}

hipError_t launch_fold(int KC, const FoldArgs &f, hipStream_t st) {
  if (f.Lpad % 64) return hipErrorInvalidValue;  // one wave per 64-line group
  const dim3 grid(f.nhalf * (f.Lpad / 64)), block(64);
  switch (KC) {
#define RT_FOLD_CASE(n) \
  case n: hipLaunchKernelGGL(fold_kernel<n>, grid, block, 0, st, f); break;
    RT_FOLD_CASE(1) RT_FOLD_CASE(2) RT_FOLD_CASE(3) RT_FOLD_CASE(4) RT_FOLD_CASE(5) RT_FOLD_CASE(6)
    RT_FOLD_CASE(8) RT_FOLD_CASE(10) RT_FOLD_CASE(15) RT_FOLD_CASE(20)
#undef RT_FOLD_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int S>
static hipError_t occupancy_s(int T, int level_waves, int *w) {
  if constexpr (level_split_supported(S, 16)) {  // workgroups (segments) per CU of the level-split pass
    if (level_waves > 1) return split_occupancy(T, level_waves, w);
  }
  switch (T) {
    case 1: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 1, 0>, 64, 0);
    case 2: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 2, 0>, 64, 0);
    case 3: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 3, 0>, 64, 0);
    case 4: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 4, 0>, 64, 0);
    case 5: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 5, 2>, 64, 0);
    case 6: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 6, 2>, 64, 0);
    case 7: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 7, 2>, 64, 0);
    case 8: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 8, 2>, 64, 0);
    case 10: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 10, 2>, 64, 0);
    case 12: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 12, 2>, 64, 0);
    case 16: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 16, 2>, 64, 0);
    case 20: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 20, 2>, 64, 0);
    case 24:
      if constexpr (one_wave_block(S, 24)) return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 24, 2>, 64, 0);
      return hipErrorInvalidValue;
    case 32:
      if constexpr (one_wave_block(S, 32)) return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 32, 2>, 64, 0);
      return hipErrorInvalidValue;
    case 40:
      if constexpr (one_wave_block(S, 40)) return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<S, 40, 2>, 64, 0);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

hipError_t sweep_occupancy(int scheme, int T, int level_waves, int *waves_per_cu) {
  switch (scheme) {
    case SCHEME_BE: return occupancy_s<SCHEME_BE>(T, level_waves, waves_per_cu);
    case SCHEME_CN: return occupancy_s<SCHEME_CN>(T, level_waves, waves_per_cu);
    default: return occupancy_s<SCHEME_BDF2>(T, level_waves, waves_per_cu);
  }
}

hipError_t coupled_occupancy(int scheme, int *w) {
  switch (scheme) {
    case SCHEME_BE: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<SCHEME_BE, 1, 0, true>, 64, 0);
    case SCHEME_CN: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<SCHEME_CN, 1, 0, true>, 64, 0);
    default: return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_block_kernel<SCHEME_BDF2, 1, 0, true>, 64, 0);
  }
}

static int grid_for(size_t total, int block) {
  size_t g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

hipError_t launch_init_state(double2 *E, const double *lineB, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(init_state_kernel, dim3(grid_for(static_cast<size_t>(2) * g.Nrow * 256, 256)), dim3(256), 0, st,
                     E, lineB, g.N, g.Nrow, g.Lpad);  // one block per row
  return hipGetLastError();
}

// blocks of `threads` the device keeps resident at once (occupancy x CUs)
template <typename K>
static size_t resident_blocks(K kernel, int threads) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || cus * per_cu <= 0)
    return 4096;
  return static_cast<size_t>(cus) * per_cu;
}

static LineMap make_map(const Geometry &g) { return LineMap{g.M, g.M / 2, g.Gl, g.N, g.Nrow, g.Lpad}; }

hipError_t launch_export_psi(const double2 *E, double *psi, const Geometry &g, int c0, int nc, hipStream_t st) {
  hipLaunchKernelGGL(export_psi_kernel, dim3(grid_for(static_cast<size_t>(g.M) * g.Gl * nc, 256)), dim3(256), 0, st,
                     E, psi, make_map(g), c0, nc);
  return hipGetLastError();
}

hipError_t launch_export_ends(const double2 *E, double *ends, const Geometry &g, int c0, int nc, hipStream_t st) {
  hipLaunchKernelGGL(export_ends_kernel, dim3(grid_for(static_cast<size_t>(g.M) * g.Gl * nc, 256)), dim3(256), 0, st,
                     E, ends, make_map(g), c0, nc);
  return hipGetLastError();
}

hipError_t launch_import_ends(double2 *E, const double *ends, const Geometry &g, int c0, int nc, hipStream_t st) {
  hipLaunchKernelGGL(import_ends_kernel, dim3(grid_for(static_cast<size_t>(g.M) * g.Gl * nc, 256)), dim3(256), 0, st,
                     E, ends, make_map(g), c0, nc);
  return hipGetLastError();
}

// The moments form where M/2 is 8, 16 or 32 (rt_set_moments_form, for A/B timing and the bitwise
// test of the forms): 0 the one-wave moments_kernel, 1 (the default) moments_pc_kernel.  A
// two-pass form (each half's rows in one ascending stream, the partial sums through the
// outputs) was measured slower and removed: 11.4 + 12.3 ms against 22.4 on one box
// (profiles/r05g_*), refuting the two-address-stream explanation of the gap to the scan.
hipError_t launch_moments(const double2 *E, const double *mu, const double *wt, double *phi, double *F,
                          double *phi_plus, const Geometry &g, int form, hipStream_t st) {
  const LineMap m = make_map(g);
  const size_t tasks = static_cast<size_t>(g.N) * ((g.Gl + 63) / 64);
  // as many waves as the chip holds at once; each walks its tasks with a one-chunk prefetch:
  // 16-direction chunks where the half's directions come in whole ones, else 8
  constexpr int W = 16;
  static const size_t resident[3] = {resident_blocks(moments_kernel<false, 8>, 64),
                                     resident_blocks(moments_kernel<true, 8>, 64),
                                     resident_blocks(moments_kernel<true, W>, 64)};
  if (form >= 1 && (m.H == 8 || m.H == 16 || m.H == 32)) {  // producer/consumer form
    constexpr int TH = 64 * (2 * kMomLoadersPerHalf + 1);
    static const size_t pc[3] = {resident_blocks(moments_pc_kernel<8>, TH), resident_blocks(moments_pc_kernel<16>, TH),
                                 resident_blocks(moments_pc_kernel<32>, TH)};
    const int k = m.H == 8 ? 0 : (m.H == 16 ? 1 : 2);
    const dim3 g(static_cast<unsigned>(tasks < pc[k] ? tasks : pc[k]));
    if (m.H == 8)
      hipLaunchKernelGGL((moments_pc_kernel<8>), g, dim3(TH), 0, st, E, mu, wt, phi, F, phi_plus, m);
    else if (m.H == 16)
      hipLaunchKernelGGL((moments_pc_kernel<16>), g, dim3(TH), 0, st, E, mu, wt, phi, F, phi_plus, m);
    else
      hipLaunchKernelGGL((moments_pc_kernel<32>), g, dim3(TH), 0, st, E, mu, wt, phi, F, phi_plus, m);
    return hipGetLastError();
  }
  const int kind = m.H % W == 0 ? 2 : (m.H % 8 == 0 ? 1 : 0);
  const dim3 grid(static_cast<unsigned>(tasks < resident[kind] ? tasks : resident[kind]));
  if (kind == 2)
    hipLaunchKernelGGL((moments_kernel<true, W>), grid, dim3(64), 0, st, E, mu, wt, phi, F, phi_plus, m);
  else if (kind == 1)
    hipLaunchKernelGGL((moments_kernel<true, 8>), grid, dim3(64), 0, st, E, mu, wt, phi, F, phi_plus, m);
  else
    hipLaunchKernelGGL((moments_kernel<false, 8>), grid, dim3(64), 0, st, E, mu, wt, phi, F, phi_plus, m);
  return hipGetLastError();
}

hipError_t launch_finite_scan(const double2 *E, int *flag, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(finite_scan_kernel, dim3(grid_for(static_cast<size_t>(2) * g.N * 256, 256)), dim3(256), 0, st, E,
                     flag, g.N, g.Nrow, g.Lpad);
  return hipGetLastError();
}

hipError_t launch_boundary_rows(const double2 *E, double2 *rows, const Geometry &g, hipStream_t st) {
  hipLaunchKernelGGL(boundary_rows_kernel, dim3(grid_for(static_cast<size_t>(4) * g.Lpad, 256)), dim3(256), 0, st, E,
                     rows, g.N, g.Nrow, g.Lpad);
  return hipGetLastError();
}

size_t balance_scratch_doubles(int Gl) { return static_cast<size_t>(kBalanceParts) * Gl * 2; }

hipError_t launch_balance_sums(const double *phi, const double *rk, const double *src, double dx, double *part,
                               double *ab, double *sr, int Gl, int N, hipStream_t st) {
  const long long lanes = static_cast<long long>(kBalanceParts) * Gl;
  hipLaunchKernelGGL(balance_partials_kernel, dim3(static_cast<unsigned>((lanes + 255) / 256)), dim3(256), 0, st, phi,
                     rk, src, dx, part, Gl, N);
  hipLaunchKernelGGL(balance_sums_kernel, dim3((Gl + 63) / 64), dim3(64), 0, st, part, ab, sr, Gl);
  return hipGetLastError();
}

hipError_t launch_group_absorption(const double *phi, const double *sigma, double *out, const Geometry &g,
                                   hipStream_t st) {
  hipLaunchKernelGGL(group_absorption_kernel, dim3(grid_for(static_cast<size_t>(g.N), 256)), dim3(256), 0, st, phi,
                     sigma, out, g.Gl, g.N);
  return hipGetLastError();
}

hipError_t launch_planck_cells(const PlanckCells &pc, const double *T, double *B, hipStream_t st) {
  hipLaunchKernelGGL(planck_cells_kernel, dim3(grid_for(static_cast<size_t>(pc.N), kPlanckCells)), dim3(256), 0, st,
                     pc, T, B);
  return hipGetLastError();
}

hipError_t launch_correction_power(int scheme, const double *map, double *pow, int L, int Lpad, hipStream_t st) {
  const dim3 grid((2 * Lpad + 255) / 256), block(256);
  switch (scheme) {
    case SCHEME_BE: hipLaunchKernelGGL(correction_power_kernel<SCHEME_BE>, grid, block, 0, st, map, pow, L, Lpad); break;
    case SCHEME_CN: hipLaunchKernelGGL(correction_power_kernel<SCHEME_CN>, grid, block, 0, st, map, pow, L, Lpad); break;
    default: hipLaunchKernelGGL(correction_power_kernel<SCHEME_BDF2>, grid, block, 0, st, map, pow, L, Lpad); break;
  }
  return hipGetLastError();
}

hipError_t launch_phi_correction(int scheme, const SegArgs &a, int nsub, int Lsub, const double *pow, hipStream_t st) {
  const long long pieces = (2LL * a.Sg * nsub + kXcds - 1) / kXcds * kXcds;
  const dim3 grid(static_cast<unsigned>(pieces * a.Q)), block(64);
  const size_t lds = sizeof(double) * kPhiChunk * group_tile_row(a.H);
  switch (scheme) {
    case SCHEME_BE: hipLaunchKernelGGL(phi_correction_kernel<SCHEME_BE>, grid, block, lds, st, a, nsub, Lsub, pow); break;
    case SCHEME_CN: hipLaunchKernelGGL(phi_correction_kernel<SCHEME_CN>, grid, block, lds, st, a, nsub, Lsub, pow); break;
    default: hipLaunchKernelGGL(phi_correction_kernel<SCHEME_BDF2>, grid, block, lds, st, a, nsub, Lsub, pow); break;
  }
  return hipGetLastError();
}

bool phi_correction_geo_supported(int scheme, const SegArgs &a) {
  return (scheme == SCHEME_BE || scheme == SCHEME_CN) && a.H >= 1 && a.H <= kGeoLines && a.Sg > 1;
}

hipError_t launch_phi_correction_geo(int scheme, const SegArgs &a, hipStream_t st) {
  if (!phi_correction_geo_supported(scheme, a)) return hipErrorInvalidValue;
  const int ranges = (a.Ls + kGeoRange - 1) / kGeoRange, gblocks = (a.Gl + kGeoWaves - 1) / kGeoWaves;
  const dim3 grid(static_cast<unsigned>(2LL * (a.Sg - 1) * ranges * gblocks)), block(64 * kGeoWaves);
  if (scheme == SCHEME_BE)
    hipLaunchKernelGGL(phi_correction_geo_kernel<SCHEME_BE>, grid, block, 0, st, a, ranges, gblocks);
  else
    hipLaunchKernelGGL(phi_correction_geo_kernel<SCHEME_CN>, grid, block, 0, st, a, ranges, gblocks);
  return hipGetLastError();
}

bool phi_correction_rows_supported(int scheme, const SegArgs &a) {
  return scheme == SCHEME_BDF2 && a.H >= 1 && a.H <= kGeoLines && a.Sg > 1;
}

size_t corr_rows_doubles(int scheme, int Lpad) {
  const int KL = (scheme == SCHEME_BDF2 ? SchemeDim<SCHEME_BDF2>::K : 1) - 1;
  return 2ULL * Lpad * (static_cast<size_t>(KL) * kRowsLen + tri_count(KL));
}

hipError_t launch_corr_rows(int scheme, const double *map, double *rows, int Lpad, hipStream_t st) {
  if (scheme != SCHEME_BDF2) return hipErrorInvalidValue;
  constexpr int KL = SchemeDim<SCHEME_BDF2>::K - 1;
  double *a64 = rows + 2ULL * Lpad * KL * kRowsLen;
  hipLaunchKernelGGL(corr_rows_kernel<SCHEME_BDF2>, dim3((2 * Lpad + 255) / 256), dim3(256), 0, st, map, rows, a64,
                     Lpad);
  return hipGetLastError();
}

hipError_t launch_phi_correction_rows(int scheme, const SegArgs &a, const double *rows, hipStream_t st) {
  if (!phi_correction_rows_supported(scheme, a)) return hipErrorInvalidValue;
  constexpr int KL = SchemeDim<SCHEME_BDF2>::K - 1;
  const int wpg = (a.H + kRowsLines - 1) / kRowsLines;
  const int ranges = std::max(1, (a.Ls - 1 + kRowsRange - 1) / kRowsRange), gblocks = (a.Gl + kRowsWaves - 1) / kRowsWaves;
  const dim3 grid(static_cast<unsigned>(2LL * (a.Sg - 1) * ranges * gblocks)), block(64 * kRowsWaves);
  const double *a64 = rows + 2ULL * a.Lpad * KL * kRowsLen;
  hipLaunchKernelGGL(phi_correction_rows_kernel<SCHEME_BDF2>, grid, block, 0, st, a, ranges, gblocks, wpg, rows, a64);
  return hipGetLastError();
}

hipError_t launch_material_q(const double *phi, int nparts, const double *B, const double *sigma, double W,
                             const double *bpart, double *q, int Gl, int N, hipStream_t st) {
  hipLaunchKernelGGL(material_q_kernel, dim3(grid_for(static_cast<size_t>(N) * 64, 256)), dim3(256), 0, st, phi, nparts,
                     B, sigma, W, bpart, q, Gl, N);
  return hipGetLastError();
}

hipError_t launch_material_update(const PlanckCells &pc, double *T, const double *qb, double *dTlast, double dt,
                                  double rho_cv, double W, int N, hipStream_t st) {
  hipLaunchKernelGGL(material_update_kernel, dim3(grid_for(static_cast<size_t>(N), 256)), dim3(256), 0, st, pc, T,
                     qb, dTlast, dt, rho_cv, W, N);
  return hipGetLastError();
}

hipError_t launch_material_transit(const double *B, const double *Beff, const double *owed, const double *sigma,
                                   double scale, double *E, int Gl, int N, hipStream_t st) {
  hipLaunchKernelGGL(material_transit_kernel, dim3(grid_for(static_cast<size_t>(N) * 64, 256)), dim3(256), 0, st, B,
                     Beff, owed, sigma, scale, E, Gl, N);
  return hipGetLastError();
}

}  // namespace rtamd
