// cell.hpp -- the per-cell algebra of the S_n sweep in the upwind frame.
//
// Shared by the sweep kernels (device) and the host-side setup that derives
// each line's linear propagator (host), so both see one definition.
//
// Upwind frame: a (direction, group) "line" is stored with cell k = 0 at its
// inflow boundary (physical cell N-1-k for mu < 0) and each cell's two nodes
// as (e_in, e_out) = (upwind node, downwind node).  With m = |mu| the three
// 2x2 cell systems of the reference are then sign-free:
//   BE   solver.cpp:319-404   [[d, b/2], [-b/2, d]] u = (S + b x + dx/2 e_in, S + dx/2 e_out)
//   CN   solver.cpp:407-490   rhs adds the explicit half of the step and A (x_prev + x_half)
//   BDF  solver.cpp:493-587   BDF2 corrector from the half (H) and previous (P) states,
//                             const_B built from the FULL dt (:501)
// The source S = 1/2 c tau dx (sigma B_g + total_correction) with the v/c
// correction (correction.cpp:393-395) linear in psi = (e_in + e_out)/2:
//   S = Sc + Sl (e_in + e_out).
// Each matrix is [[d, o], [-o, d]], whose inverse is [[i0, -i1], [i1, i0]]
// with i0 = d/(d^2+o^2), i1 = o/(d^2+o^2): precomputed once per line.
//
// Fused step.  One full step is swept in ONE pass over the cells: BE (1
// substep, X = x), CN (1 substep, X = (p_up, x_half)) or the 4-substep BDF2
// cycle BE -> CN -> BE -> BDF (solver.cpp:721-753), carrying
//   X = (p_up, x0, xh, x2, x3)
// p_up = step-start downwind node of the upwind cell (prev_ends, :449/:483/
// :542/:581), x0/xh/x2/x3 = the four substeps' upwind scalars.  Within the
// step the half state H (solver.cpp:733) is the CN result for mu < 0 lines
// and the BE-predictor result for mu > 0 lines.  X after a cell is an affine
// function of X before it with a cell-independent linear part A -- the basis
// of the cell-parallel scan (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace rtamd {

enum LineConstIndex {
  LC_SC = 0, LC_SL,
  LC_BE_B, LC_BE_I0, LC_BE_I1,
  LC_CN_A, LC_CN_K1, LC_CN_K2, LC_CN_I0, LC_CN_I1,
  LC_BD_BC, LC_BD_Q1, LC_BD_Q2, LC_BD_Q3, LC_BD_Q4, LC_BD_I0, LC_BD_I1,
  LC_COUNT
};

enum Scheme { SCHEME_BE = 1, SCHEME_CN = 2, SCHEME_BDF2 = 3 };

template <int S> struct SchemeDim;
template <> struct SchemeDim<SCHEME_BE> { static constexpr int K = 1; };
template <> struct SchemeDim<SCHEME_CN> { static constexpr int K = 2; };
template <> struct SchemeDim<SCHEME_BDF2> { static constexpr int K = 5; };

struct LineConst {
  double c[LC_COUNT];
};

__host__ __device__ __forceinline__ double src(const LineConst &L, double ein, double eout) {
  return L.c[LC_SC] + L.c[LC_SL] * (ein + eout);
}

// Backward Euler cell (solver.cpp:319-404)
__host__ __device__ __forceinline__ void cell_be(const LineConst &L, double hd, double ein, double eout, double x,
                                                 double &uin, double &uout) {
  const double S = src(L, ein, eout);
  const double rin = S + L.c[LC_BE_B] * x + hd * ein;
  const double rout = S + hd * eout;
  uin = L.c[LC_BE_I0] * rin - L.c[LC_BE_I1] * rout;
  uout = L.c[LC_BE_I1] * rin + L.c[LC_BE_I0] * rout;
}

// Crank-Nicolson cell (solver.cpp:407-490): xp = prev_ends of the upwind cell, xh = half_local_bdry
__host__ __device__ __forceinline__ void cell_cn(const LineConst &L, double hd, double ein, double eout, double xp,
                                                 double xh, double &uin, double &uout) {
  const double S = src(L, ein, eout);
  const double rin = S + L.c[LC_CN_K1] * ein - L.c[LC_CN_K2] * eout + L.c[LC_CN_A] * (xp + xh);
  const double rout = S + L.c[LC_CN_K2] * ein + L.c[LC_CN_K1] * eout;
  uin = L.c[LC_CN_I0] * rin - L.c[LC_CN_I1] * rout;
  uout = L.c[LC_CN_I1] * rin + L.c[LC_CN_I0] * rout;
}

// BDF corrector cell (solver.cpp:493-587); (ein, eout) = state at substep start (source only)
__host__ __device__ __forceinline__ void cell_bdf(const LineConst &L, double ein, double eout, double hin,
                                                  double hout, double pin, double pout, double x, double xh,
                                                  double xp, double &uin, double &uout) {
  const double S = src(L, ein, eout);
  const double rin = S + L.c[LC_BD_Q1] * hin - L.c[LC_BD_Q2] * hout - L.c[LC_BD_Q3] * pin - L.c[LC_BD_Q4] * pout +
                     L.c[LC_BD_BC] * (x + 4.0 * xh + xp);
  const double rout = S + L.c[LC_BD_Q2] * hin + L.c[LC_BD_Q1] * hout + L.c[LC_BD_Q4] * pin - L.c[LC_BD_Q3] * pout;
  uin = L.c[LC_BD_I0] * rin - L.c[LC_BD_I1] * rout;
  uout = L.c[LC_BD_I1] * rin + L.c[LC_BD_I0] * rout;
}

// One BDF2 full step of one cell with explicit upwind inputs.
// x0/xh/x2/x3: the substeps' carried scalars; xp1/xp3: prev-state upwind node
// seen by CN / BDF; hup: half-state upwind node seen by BDF.
__host__ __device__ __forceinline__ void cell_bdf2_explicit(const LineConst &L, double hd, bool neg, double pin,
                                                            double pout, double x0, double xh, double x2, double x3,
                                                            double xp1, double xp3, double hup, double &e1out,
                                                            double &e2out, double &e3out, double &oin,
                                                            double &oout) {
  double e1in, e2in, e3in;
  cell_be(L, hd, pin, pout, x0, e1in, e1out);                    // substep 0: BE predictor
  cell_cn(L, hd, e1in, e1out, xp1, xh, e2in, e2out);             // substep 1: CN corrector
  const double hin = neg ? e2in : e1in, hout = neg ? e2out : e1out;  // half_ends (:733)
  cell_be(L, hd, e2in, e2out, x2, e3in, e3out);                  // substep 2: BE predictor
  cell_bdf(L, e3in, e3out, hin, hout, pin, pout, x3, hup, xp3, oin, oout);  // substep 3: BDF
}

// Generic interior cell: X -> X' for scheme S; (pin, pout) = step-start state,
// (oin, oout) = step-end state.  neg selects the mu < 0 half-state rule.
template <int S>
__host__ __device__ __forceinline__ void cell_step(const LineConst &L, double hd, bool neg, double pin, double pout,
                                                   double *X, double &oin, double &oout) {
  if constexpr (S == SCHEME_BE) {
    cell_be(L, hd, pin, pout, X[0], oin, oout);
    X[0] = oout;
  } else if constexpr (S == SCHEME_CN) {
    cell_cn(L, hd, pin, pout, X[0], X[1], oin, oout);
    X[0] = pout;
    X[1] = oout;
  } else {
    double a, b, c;
    const double hup = neg ? X[2] : X[1];
    cell_bdf2_explicit(L, hd, neg, pin, pout, X[1], X[2], X[3], X[4], X[0], X[0], hup, a, b, c, oin, oout);
    X[0] = pout;
    X[1] = a;
    X[2] = b;
    X[3] = c;
    X[4] = oout;
  }
}

// Carried state entering the first cell of a line from per-substep inflow
// values b[0..3] (solver.cpp:695-697: local_bdry = half_local_bdry =
// local_bdry_prev_it = bdry_cond).
template <int S>
__host__ __device__ __forceinline__ void head_state(const double *b, double *X) {
  if constexpr (S == SCHEME_BE) {
    X[0] = b[0];
  } else if constexpr (S == SCHEME_CN) {
    X[0] = b[0];
    X[1] = b[0];
  } else {
    X[0] = b[1];
    X[1] = b[0];
    X[2] = b[1];
    X[3] = b[2];
    X[4] = b[3];
  }
}

// cell_step for a cell that may be a line head (head_state already applied):
// in the BDF substep the head sees b[3] as both prev and half upwind node.
// With equal inflows (non-reflective boundaries) this equals cell_step.
template <int S>
__host__ __device__ __forceinline__ void cell_step_maybe_head(const LineConst &L, double hd, bool neg, double pin,
                                                              double pout, double *X, bool head, double b3,
                                                              double &oin, double &oout) {
  if constexpr (S == SCHEME_BDF2) {
    double a, b, c;
    const double hup = head ? b3 : (neg ? X[2] : X[1]);
    const double xp3 = head ? b3 : X[0];
    cell_bdf2_explicit(L, hd, neg, pin, pout, X[1], X[2], X[3], X[4], X[0], xp3, hup, a, b, c, oin, oout);
    X[0] = pout;
    X[1] = a;
    X[2] = b;
    X[3] = c;
    X[4] = oout;
  } else {
    cell_step<S>(L, hd, neg, pin, pout, X, oin, oout);
  }
}

// Index of (r, c), c <= r, in a packed lower triangle.
__host__ __device__ __forceinline__ constexpr int tri(int r, int c) { return r * (r + 1) / 2 + c; }
__host__ __device__ __forceinline__ constexpr int tri_count(int K) { return K * (K + 1) / 2; }

// ---------------------------------------------------------------------------
// The cell step as a per-line affine map.
//
// Because sigma, B_g and the correction constants do not vary along a line
// (T and rho are constant, solver.cpp:157), one full step of one cell is an
// affine map with line-constant coefficients from the inputs
//   u = (X[0..K-1], pin, pout)            (carried state, step-start nodes)
// to the outputs
//   row r < K : X'[r]      row K : oin      (oout == X'[K-1] for every scheme).
// The coefficients are derived on the host by evaluating cell_step<S> above
// (the reference's algebra) on unit inputs, so the map is the same
// arithmetic up to rounding.  Rows keep only their structural non-zeros:
//   BE   X=(x)                     X'0=oout: x,pin,pout      oin: x,pin,pout
//   CN   X=(p_up,xh)               X'0=pout (copy)           X'1=oout, oin: all
//   BDF2 X=(p_up,x0,xh,x2,x3)      X'0=pout (copy)  X'1=e1out: x0,pin,pout
//        X'2=e2out: p_up,x0,xh,pin,pout   X'3=e3out: + x2   X'4=oout, oin: all
// (the host checks every other coefficient is exactly zero).
// ---------------------------------------------------------------------------
template <int S>
__host__ __device__ constexpr bool map_copy_row0() {
  return S != SCHEME_BE;
}

// does output row r (0..K) depend on input c (0..K+1)?
template <int S>
__host__ __device__ constexpr bool map_dep(int r, int c) {
  constexpr int K = SchemeDim<S>::K;
  if (map_copy_row0<S>() && r == 0) return false;
  if (c >= K) return true;  // pin, pout feed every computed row
  if constexpr (S == SCHEME_BDF2) {
    if (r == 1) return c == 1;
    if (r == 2) return c <= 2;
    if (r == 3) return c <= 3;
    return true;
  }
  return true;
}

// slot of coefficient (r, c) in the packed map; the constant of row r follows its coefficients
template <int S>
__host__ __device__ constexpr int map_slot(int r, int c) {
  constexpr int K = SchemeDim<S>::K;
  int n = 0;
  for (int rr = 0; rr <= K; ++rr) {
    if (map_copy_row0<S>() && rr == 0) continue;
    for (int cc = 0; cc < K + 2; ++cc) {
      if (!map_dep<S>(rr, cc)) continue;
      if (rr == r && cc == c) return n;
      ++n;
    }
    if (rr == r && c == K + 2) return n;  // constant
    ++n;
  }
  return -1;
}

template <int S>
__host__ __device__ constexpr int map_count() {
  constexpr int K = SchemeDim<S>::K;
  return map_slot<S>(K, K + 2) + 1;
}

// The reflective mu > 0 head cell's map (cell_step_maybe_head probed the same way) differs
// from its line's map only from this slot on: BDF2's last two rows (the BDF substep reads the
// mirror's last-substep outflow as its prev and half upwind nodes); BE / CN: nowhere.
template <int S>
__host__ __device__ constexpr int head_map_first() {
  return S == SCHEME_BDF2 ? map_slot<S>(SchemeDim<S>::K - 1, 0) : map_count<S>();
}

// Apply the map (CONST: with the affine constants; otherwise its linear part).
// cs scales the constants: the material-coupled sweep stores them for B = 1
// and passes the cell's B_g(T(x)) (with the correction off they are linear in
// the source); 1.0 elsewhere, which the compiler folds away.  For the correction
// walks, which move a state with no data delta: NODATA skips the din/dout columns
// (both 0.0; fma(w, 0.0, acc) is not folded by the compiler), ZERO0 also skips X[0]
// (0.0 after one cell where row 0 copies dout: CN, BDF2) -- the same values.  ROW_LO > 0:
// only rows ROW_LO .. K (Xn below ROW_LO untouched), each the same FMA sequence as in the
// whole map -- the reflective head lane redoing the rows where its map differs.
template <int S, bool CONST, bool NODATA = false, bool ZERO0 = false, int ROW_LO = 0>
__host__ __device__ __forceinline__ void map_apply(const double *W, const double *X, double din, double dout,
                                                   double *Xn, double &oin, double &oout, double cs = 1.0) {
  constexpr int K = SchemeDim<S>::K;
  static_assert(!ZERO0 || (NODATA && map_copy_row0<S>()), "X[0] vanishes only where row 0 copies a zero dout");
#pragma unroll
  for (int r = ROW_LO; r <= K; ++r) {
    if (map_copy_row0<S>() && r == 0) {
      Xn[0] = dout;
      continue;
    }
    double acc = CONST ? W[map_slot<S>(r, K + 2)] * cs : 0.0;
#pragma unroll
    for (int c = 0; c < K + 2; ++c) {
      if (!map_dep<S>(r, c)) continue;
      if ((NODATA && c >= K) || (ZERO0 && c == 0)) continue;
      const double u = c < K ? X[c] : (c == K ? din : dout);
      acc = fma(W[map_slot<S>(r, c)], u, acc);
    }
    if (r < K)
      Xn[r] = acc;
    else
      oin = acc;
  }
  oout = Xn[K - 1];
}

// The per-line affine cell map (cell.hpp, map_apply): coefficients from
// cell_step<S> on unit inputs (constants and data zeroed), constants from
// cell_step<S> on zero inputs.  Every coefficient outside the structural
// pattern must come out exactly zero; false otherwise.
// (host code: rtsn_lines.hip builds every line's maps with it, tools/cell_map_check.cpp tests it.)
// HEAD: the reflective mu > 0 head cell's map instead (cell_step_maybe_head with the
// mirror's last-substep outflow b3 = X[K-1], the carried state being head_state(b): a map
// of the same structure, so the kernels run the head cell as the same FMA rows as every
// other cell -- no divergent per-tick branch into the reference's algebra).
template <int S, bool HEAD = false>
inline bool cell_map(const LineConst &Lin, double hd, bool neg, double *W) {
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
    if constexpr (HEAD)
      cell_step_maybe_head<S>(L, hd, neg, pin, pout, X, true, X[K - 1], oi, oo);
    else
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

}  // namespace rtamd
