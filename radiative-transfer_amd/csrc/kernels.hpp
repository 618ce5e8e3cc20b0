// kernels.hpp -- launch interface of kernels.hip (host side of the C ABI).
#pragma once

#include <hip/hip_runtime.h>

namespace rtamd {

constexpr int kSweepWaves = 4;                          // waves per workgroup
constexpr int kSweepThreads = 64 * kSweepWaves;         // 256
constexpr int kSweepCells = 16;                         // cells per wave (registers)
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
