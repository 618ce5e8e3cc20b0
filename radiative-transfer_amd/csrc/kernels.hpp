// kernels.hpp -- launch interface of kernels.hip (host side of the C ABI).
#pragma once

#include <hip/hip_runtime.h>

namespace rtamd {

// Build-time tunables (defaults are the measured best).
#ifndef RT_SWEEP_CELLS
#define RT_SWEEP_CELLS 16     // cells per wave held in registers
#endif
#ifndef RT_PIN_CELLS
#define RT_PIN_CELLS 0        // 1: asm-pin each cell's inputs (bounded live ranges)
#endif
#ifndef RT_PHASE_BARRIER
#define RT_PHASE_BARRIER 1    // 1: phase 2 re-derives X-independent terms (no cross-phase CSE)
#endif
#ifndef RT_LOOKBACK_PARALLEL
#define RT_LOOKBACK_PARALLEL 0  // 1: poll 64 predecessors at once
#endif
#ifndef RT_SWEEP_MIN_WAVES
#define RT_SWEEP_MIN_WAVES 1  // __launch_bounds__ minimum waves per SIMD
#endif

constexpr int kSweepWaves = 4;                          // waves per workgroup
constexpr int kSweepThreads = 64 * kSweepWaves;         // 256
constexpr int kSweepCells = RT_SWEEP_CELLS;             // cells per wave (registers)
constexpr int kSweepTile = kSweepWaves * kSweepCells;   // 64 cells per tile

struct SweepArgs {
  double2 *E;                 // [2][N][Lpad] (e_in, e_out)
  const double *lc;           // [2][LC_COUNT][Lpad] line constants
  const double *Apow;         // [2 half][2 (A^16, A^64)][K(K+1)/2][Lpad]
  const double *bdry;         // [2][Lpad] inflow value per line (non-reflective)
  double *outflow;            // [4][Lpad] mu<0 outflows per substep (reflective)
  unsigned *outflow_flag;     // [Q]
  unsigned *status;           // [total_tiles]  0 none / 1 aggregate / 2 inclusive prefix
  double *agg;                // [total_tiles][K][64]
  double *pref;               // [total_tiles][K][64]
  unsigned *error;            // [1] timeout word
  long long total_tiles;      // 2 * J * Q
  int N, Nrow, Lpad, Q, J;    // Nrow = 64 J rows per half (cells padded to whole tiles)
  int reflective;             // bc_left == 2
  int debug_flags;            // timing experiments only (RTSN_DEBUG_FLAGS): 1 = skip the look-back
                              // wait, 2 = skip phase 1; results are wrong when set
  double hd;                  // dx / 2
};

struct Geometry {
  int M, Gl, N, Nrow, Lpad;
};

hipError_t launch_sweep(int scheme, const SweepArgs &a, int grid, hipStream_t st);
hipError_t sweep_occupancy(int scheme, int *blocks_per_cu);
hipError_t launch_init_state(double2 *E, const double *lineB, const Geometry &g, hipStream_t st);
hipError_t launch_export_psi(const double2 *E, double *psi, const Geometry &g, hipStream_t st);
hipError_t launch_export_ends(const double2 *E, double *ends, const Geometry &g, hipStream_t st);
hipError_t launch_import_ends(double2 *E, const double *ends, const Geometry &g, hipStream_t st);
hipError_t launch_moments(const double2 *E, const double *mu, const double *wt, double *phi, double *F,
                          double *phi_plus, const Geometry &g, hipStream_t st);
hipError_t launch_boundary_rows(const double2 *E, double2 *rows, const Geometry &g, hipStream_t st);
hipError_t launch_group_absorption(const double *phi, const double *sigma, double *out, const Geometry &g,
                                   hipStream_t st);

}  // namespace rtamd
