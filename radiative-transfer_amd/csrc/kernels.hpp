// kernels.hpp -- launch interface of kernels.hip (host side of the C ABI).
#pragma once

#include <hip/hip_runtime.h>

namespace rtamd {

// Build-time tunables (defaults are the measured best).
#ifndef RT_SWEEP_CELLS
#define RT_SWEEP_CELLS 16     // cells per wave held in registers
#endif

constexpr int kSweepCells = RT_SWEEP_CELLS;             // rows per chunk held in registers
constexpr int kSweepTile = 64;                          // cells are padded to whole tiles of 64 rows

// Per-line propagator block: A (one cell, packed lower-triangular), R (2 x K,
// state -> step-end nodes), A^Ls and A^Llast (segment propagators).
template <int K>
constexpr int kPropCount = 3 * (K * (K + 1) / 2) + 2 * K;

struct SegArgs {
  double2 *E;                 // [2][Nrow][Lpad] (e_in, e_out)
  const double *lc;           // [2][LC_COUNT][Lpad] line constants
  const double *prop;         // [2][kPropCount<K>][Lpad] propagators
  const double *bdry;         // [2][Lpad] inflow value per line (non-reflective)
  const double *agg_prev;     // [2][Sg][K][Lpad] segment aggregates of the previous step
  double *agg_cur;            // [2][Sg][K][Lpad] segment aggregates of this step
  int N, Nrow, Lpad, Q;
  int Sg, Ls;                 // segments per line, cells per segment (multiple of 16)
  int half0;                  // first half swept by this launch (grid covers 1 or 2 halves)
  int reflective;             // bc_left == 2
  int pending;                // the stored state is provisional: apply the correction
  double hd;                  // dx / 2
};

struct Geometry {
  int M, Gl, N, Nrow, Lpad;
};

hipError_t launch_sweep(int scheme, bool finalize, const SegArgs &a, int grid, hipStream_t st);
hipError_t sweep_occupancy(int scheme, int *waves_per_cu);
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
