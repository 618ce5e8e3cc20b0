// kernels.hpp -- launch interface of kernels.hip (host side of the C ABI).
#pragma once

#include <hip/hip_runtime.h>

namespace rtamd {

// Register-tiling constants (the measured best).
constexpr int kSweepCells = 16;  // cells per wave held in registers; segment lengths are multiples of this
// rows per chunk held in registers (prefetch depth) for scheme S fusing T steps:
// measured on SL, BDF2 T = 16: 4 rows 8.67, 8 rows 8.33, 16 rows 8.15 ms/step;
// T = 20: 16 rows spill to scratch, 8 rows fit 256 VGPRs + 126 AGPRs
constexpr int chunk_cells(int S, int T) {
  return S == 3 && T >= 20 ? 8 : S == 3 && T >= 12 ? 16 : (S == 3 && T >= 2 ? 8 : kSweepCells);
}
// pipelined passes whose T levels two waves can share (sweep_split_kernel):
// BDF2, where the carried states (5 per level) are what overflows 256 registers
constexpr bool level_split_supported(int S, int T) {
  return S == 3 && (T == 4 || T == 8 || T == 10 || T == 12 || T == 16 || T == 20 || T == 24 || T == 32 || T == 40);
}
// pipelined passes with a one-wave kernel: all but BDF2 beyond 20 levels (its carried
// states would spill; those run split over four waves)
constexpr bool one_wave_block(int S, int T) { return S != 3 || T <= 20; }
// rows per chunk of the level-split pass (16 rows with T/2 = 8 levels spill past 256 registers)
constexpr int split_chunk_cells() { return 8; }
constexpr int kXcds = 8;                                // gfx950: workgroups are dealt to 8 XCDs round-robin
constexpr int kSweepTile = 64;                          // cells are padded to whole tiles of 64 rows

constexpr int kMaxTimeBlock = 40;                       // full steps fused per pipelined pass (template range)
constexpr int kMaxAlignedBlock = 4;                     // ... per aligned pass (carries a T K correction state)

// Segment propagators of the T-level combined state (KC = T K, packed lower
// triangle of NTC = KC (KC + 1) / 2 entries each): A_T^Ls, A_T^Llast.
constexpr int prop_count(int K, int T) { return (T * K) * (T * K + 1); }

struct SegArgs {
  double2 *E;                 // [2][Nrow][Lpad] (e_in, e_out)
  const double *map;          // [2][map_count<S>][Lpad] per-line affine cell map (cell.hpp)
  const double *hmap;         // [map_count<S>][Lpad] the reflective mu > 0 head cell's map (half 1 lines)
  const double *bdry;         // [2][Lpad] inflow value per line (non-reflective)
  const double *yseg;         // [2][Sg+1][T K][Lpad] true incoming state per segment (fold_kernel)
  const double *yrefl;        // [T K][Lpad] this pass's mu < 0 line outflow state (reflective)
  double *agg_cur;            // [2][Sg][T K][Lpad] segment aggregates of this pass
  double *aggs[2];            // pipelined: aggregates of pass p in aggs[p & 1], [2][Sg][T K][Lpad]
  int N, Nrow, Lpad, Q;
  int Sg, Ls;                 // segments per line, cells per segment (multiple of 16)
  int half0;                  // first half swept by this launch (grid covers 1 or 2 halves)
  int reflective;             // bc_left == 2
  int pending;                // the stored state is provisional: apply the correction
  int pos_lo, npos, pass_lo;  // pipelined: active chain positions and the pass of the first
  int level_waves;            // pipelined: waves per segment, 1 (sweep_block_kernel) or 2, 4 (sweep_split_kernel)
  int tail_levels;            // pipelined (launch_split_tail): position pos_lo runs this many (< T) levels
  double hd;                  // dx / 2
  // material coupling (SWEEP_PASS, T = 1 only): per-cell emission B_g(T(x)),
  // [N][Gl] (g fastest), scaling the map constants stored for B = 1
  const double *bcell;        // nullptr: line-constant source (the reference's constant T)
  int Gl, H;                  // local groups, lines per half per group (line l = i' + H g)
  // ... with the angular sums fused (H divides 64): the pass writes
  // phi[half][x][g] = sum over the half's directions of w_i psi (provisional
  // state), phi_correction_kernel adds the cross-segment correction's share
  double *phi;                // nullptr: not fused (phi from moments_kernel after a finalize)
  double *phic;               // [half][x][g] the correction's share (phi_correction_kernel)
  const double *wt;           // [M] quadrature weights
};

struct FoldArgs {
  const double *agg;          // [2][Sg][KC][Lpad]
  const double *prop;         // [2][prop_half][Lpad]: A^Ls then A^Llast (packed)
  double *y;                  // [2][Sg+1][KC][Lpad], or [KC][Lpad] when only_last
  int prop_half, Sg, Lpad, half0, nhalf, last_short, only_last;
};

struct Geometry {
  int M, Gl, N, Nrow, Lpad;
};

enum SweepMode {
  SWEEP_PASS = 0,       // one pass of T full steps, every segment at the same time level
  SWEEP_FINALIZE = 1,   // only the pending correction of a T-step pass
  SWEEP_PIPELINED = 2   // one launch of the staggered (pipelined) schedule
};
hipError_t launch_sweep(int scheme, int T, int mode, const SegArgs &a, int grid, hipStream_t st);
// the level-split pipelined BDF2 pass (kernels_split.hip): T levels over `waves` waves
hipError_t launch_split(int T, int waves, const SegArgs &a, int grid, hipStream_t st);
hipError_t split_occupancy(int T, int waves, int *workgroups_per_cu);
// a pipelined launch whose position pos_lo runs a.tail_levels < T levels (the run's n mod T
// remainder; vacuum lines), the rest T: (T, waves) pairs split_tail_supported
bool split_tail_supported(int T, int waves);
hipError_t launch_split_tail(int T, int waves, const SegArgs &a, int grid, hipStream_t st);
// segments resident per CU (workgroups of the pass: one wave, or two with level_waves 2)
hipError_t sweep_occupancy(int scheme, int T, int level_waves, int *waves_per_cu);
hipError_t coupled_occupancy(int scheme, int *waves_per_cu);  // the material-coupled pass (T = 1)
hipError_t launch_fold(int KC, const FoldArgs &f, hipStream_t st);
// short lines (kernels_wave.hip): nsteps full steps of every line in one launch, lanes over
// cells (a.Gl, a.H set: lines ell < H Gl).  A line (reflective: a line pair) is a chain of
// `lanes` lanes per line holding C cells each, on `waves` waves of one workgroup (C = 0: too
// long for kWaveMaxWaves waves); waves > 1 hand the chain over through LDS once per tick
// and meet at a barrier every kWaveBlockTicks ticks
constexpr int kWaveMaxWaves = 8;
constexpr int kWaveBlockTicks = 8;
struct WavePlan {
  int C, waves, lanes;
};
WavePlan wavefront_plan(int N, bool reflective, int max_waves);
hipError_t launch_wavefront(int scheme, const WavePlan &p, const SegArgs &a, int nsteps, hipStream_t st);
hipError_t launch_init_state(double2 *E, const double *lineB, const Geometry &g, hipStream_t st);
// reference-layout psi / ends of the cells [c0, c0 + nc) (ends: node 0 block, then node 1)
hipError_t launch_export_psi(const double2 *E, double *psi, const Geometry &g, int c0, int nc, hipStream_t st);
hipError_t launch_export_ends(const double2 *E, double *ends, const Geometry &g, int c0, int nc, hipStream_t st);
hipError_t launch_import_ends(double2 *E, const double *ends, const Geometry &g, int c0, int nc, hipStream_t st);
// form (rt_set_moments_form): 1 the producer/consumer moments_pc_kernel where M/2 is 8, 16 or
// 32, 0 the one-wave moments_kernel; bitwise-identical results
hipError_t launch_moments(const double2 *E, const double *mu, const double *wt, double *phi, double *F,
                          double *phi_plus, const Geometry &g, int form, hipStream_t st);
hipError_t launch_boundary_rows(const double2 *E, double2 *rows, const Geometry &g, hipStream_t st);
// *flag |= 1 if any node of the N real rows of either half is not finite (flag zeroed by the caller)
hipError_t launch_finite_scan(const double2 *E, int *flag, const Geometry &g, hipStream_t st);
// per group: ab = sum_c (rk phi) dx, sr = sum_c src (compute_balance), as a two-level sum
// over contiguous cell ranges; part: balance_scratch_doubles(Gl) doubles of scratch
size_t balance_scratch_doubles(int Gl);
hipError_t launch_balance_sums(const double *phi, const double *rk, const double *src, double dx, double *part,
                               double *ab, double *sr, int Gl, int N, hipStream_t st);
hipError_t launch_group_absorption(const double *phi, const double *sigma, double *out, const Geometry &g,
                                   hipStream_t st);

// Planck group integrals per cell (material coupling): the algorithm of
// Planck.cpp:44-337 in double precision on the device.
struct PlanckCells {
  double node[12], weight[12];  // Gauss-Legendre on [-1, 1] (Planck.cpp:231-337, rounded to double)
  const double *e_edge;         // [G+1] all groups' edges (device)
  int G, g_lo, Gl, N;
  double a_c;                   // rad_a_long() * c (Constants.h:22-23)
  double kcon;                  // jk per keV (correction.cpp:25-36)
  double accuracy;              // series tolerance (Planck.h:96, DBL_EPSILON)
  // the coupling's owed emission (rtsn_material.hip): the last update's dT per cell in;
  // owed and dB (group-major [Gl][N], the kernel's own) updated; Beff = B + the paid share
  // and bpart = b_scale sum_gl sigma[gl] dB/dT out
  const double *sigma;          // [Gl] rho kappa of the handle's groups
  const double *dTlast;         // [N]
  double *owed, *dB;            // [Gl][N]
  double *Beff;                 // [N][Gl]
  double *bpart;                // [N]
  double b_scale;               // 1, or 0 on a direction shard without pair 0 (b counted once)
  const double *sigma_all;      // [G] rho kappa of every group (the update's S(T), all groups)
  const double *Bcell;          // [N][Gl] B_g(T^n) (the update's full-emission cells: owed += B(T') - B(T^n))
};
// B[N][Gl] = B_g(T(x)) and the fields above
hipError_t launch_planck_cells(const PlanckCells &pc, const double *T, double *B, hipStream_t st);
// the correction's share of the fused angular sums (SegArgs.phi) after a
// coupled pass with segments started from X = 0 (T = 1; each segment walked as
// sub-segments, enough to fill the chip)
// nsub sub-segments of Lsub cells per segment (Lsub a multiple of 16), each started from
// pow^j applied to the segment's correction state, pow = A^Lsub (launch_correction_power)
hipError_t launch_phi_correction(int scheme, const SegArgs &a, int nsub, int Lsub, const double *pow, hipStream_t st);
// pow[half][K (K + 1) / 2][Lpad] = A^L, A the map's linear X -> X' block (lower triangular)
// BE, CN: the correction's share in closed form (lanes over cells, H <= 32 lines per group-half)
bool phi_correction_geo_supported(int scheme, const SegArgs &a);
hipError_t launch_phi_correction_geo(int scheme, const SegArgs &a, hipStream_t st);
// BDF2: the correction's share by tabulated rows b A^j (lanes over cells, H <= 32);
// launch_corr_rows fills the table (corr_rows_doubles) once per handle from the map
bool phi_correction_rows_supported(int scheme, const SegArgs &a);
size_t corr_rows_doubles(int scheme, int Lpad);
hipError_t launch_corr_rows(int scheme, const double *map, double *rows, int Lpad, hipStream_t st);
hipError_t launch_phi_correction_rows(int scheme, const SegArgs &a, const double *rows, hipStream_t st);
hipError_t launch_correction_power(int scheme, const double *map, double *pow, int L, int Lpad, hipStream_t st);
// q[x] = sum_g sigma_g (phi_g(x) - W B_g(x)) over the handle's groups, phi the
// sum of nparts [N][Gl] arrays at phi (the fused parts, or one full phi); q[N + x] = bpart[x]
hipError_t launch_material_q(const double *phi, int nparts, const double *B, const double *sigma, double W,
                             const double *bpart, double *q, int Gl, int N, hipStream_t st);
// from qb = [q, b] summed over all groups: dT = dt q / (rho_cv + dt W b), T(x) += dT, dTlast = dT
// T += dt q / (rho_cv + dt W b), or the root of the full emission where dT > T / 4 (its owed
// emission added there, dT 0): rt_oracle.c orc_material_update
hipError_t launch_material_update(const PlanckCells &pc, double *T, const double *qb, double *dTlast, double dt,
                                  double rho_cv, double W, int N, hipStream_t st);
// E[x] = scale sum_gl sigma[gl] ((Beff - B) + owed[gl][x]) (rt_get_material_transit)
hipError_t launch_material_transit(const double *B, const double *Beff, const double *owed, const double *sigma,
                                   double scale, double *E, int Gl, int N, hipStream_t st);

}  // namespace rtamd
