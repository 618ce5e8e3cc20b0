// comm_layout.hpp -- where every rank's shard data lands in the reference's result arrays.
//
// The multi-GPU gathers (rtsn_comm.hip) move per-rank blocks through RCCL and then place
// them into the reference's layouts (main.cc:88-133): phi / F / phi_plus (G, N) ColMajor
// (g + G c), psi (M, G, N) (i + M (g + G c)), psi_source (M x G, m G + g) and per-group
// vectors.  The placement is pure index arithmetic, so it lives here as host code with no
// device calls: each step is a *copy plan* -- a list of strided 2-D copies over doubles --
// that rtsn_comm.hip runs with hipMemcpy2DAsync and the C ABI's rt_layout_* functions run
// on host memory (callers with their own collectives, and the CPU tests, which check every
// plan against one handle's arrays at world sizes 2, 3 and 8).
#pragma once

#include <cstddef>
#include <vector>

#include "../../include/rtsn.h"

namespace rtamd::layout {

// dst[dst + r * dpitch + j] = src[src + r * spitch + j] for r < height, j < width (doubles)
struct Copy2D {
  size_t dst, dpitch, src, spitch, width, height;
};

inline int groups_of(const rt_shard &a) { return a.g_hi - a.g_lo; }
inline int dirs_of(const rt_shard &a) { return 2 * (a.d_hi - a.d_lo); }

// How the shards tile the problem: 0 = group shards tiling [0, G) in rank order (every
// shard all M/2 direction pairs), 1 = direction-pair shards tiling [0, M/2) in rank order
// over all G groups, -1 = neither (or the shards disagree on G, M or N).
int shard_mode(const rt_shard *sh, int n);
// the largest shard's group count: every rank's block is padded to it on the wire
int max_groups(const rt_shard *sh, int n);

// moments: a rank's local arrays (phi, F, phi_plus back to back, each N x Gl, g fastest)
// -> its wire block [3][N][Gmax] (the caller zeroes the padding first)
std::vector<Copy2D> moments_pack(const rt_shard *sh, int n, int rank);
// the gathered buffer -- group shards: the all-gather [rank][3][N][Gmax]; direction
// shards: the all-reduced sum [3][N][Gmax] -> field k (0 phi, 1 F, 2 phi_plus) as (G, N)
std::vector<Copy2D> moments_unpack(const rt_shard *sh, int n, int field);
// k per-group vectors: rank's block [k][Gmax]; gathered [rank][k][Gmax] (group shards) or
// the sum [k][Gmax] (direction shards) -> vector j as G values
std::vector<Copy2D> vectors_pack(const rt_shard *sh, int n, int rank, int k, int j);
std::vector<Copy2D> vectors_unpack(const rt_shard *sh, int n, int k, int j);
// one shard's psi (M_l, Gl, N) ColMajor (its directions in ascending mu: i' in
// [H - d_hi, H - d_lo) then [H + d_lo, H + d_hi)) -> its rows of psi (M, G, N)
std::vector<Copy2D> psi_place(const rt_shard &a);
// one shard's psi_source rows (M_l x G, ascending mu) -> rows of the (M x G) table
std::vector<Copy2D> psi_source_place(const rt_shard &a);

// run a plan on host memory
void apply(const std::vector<Copy2D> &plan, const double *src, double *dst);

}  // namespace rtamd::layout
