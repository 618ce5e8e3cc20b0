// sweep_device.hpp -- device helpers shared by the sweep kernels (kernels.hip) and the
// level-split pass (kernels_split.hip): buffer-descriptor row streaming and the
// reflective head cell.
#pragma once

#include <hip/hip_runtime.h>

#include "cell.hpp"
#include "kernels.hpp"

namespace rtamd {

// A wave's C rows of one chunk are addressed through a buffer descriptor
// built from wave-uniform values: base (SGPR) + row offset (SGPR soffset) +
// lane*16 (one VGPR), instead of a 64-bit VGPR address per row.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Descriptor word 3 = 0x00020000: DATA_FORMAT (bits 15-18) = 4, 32-bit, as for raw
// dword buffers on gfx9-family parts; num_records = the chunk's bytes (bounds-checked).
template <int C>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const double2 *base, int row_bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double2 *>(base), 0, C * row_bytes, 0x00020000);
}
// Cache policy of the state stream (the buffer aux operand): nt (2).  Every row is
// read and written once per pass and the state (131 GB on SL) is far beyond L2 and
// MALL: nt loads and stores measured 1.8% faster on the HBM-bound T = 1 pass (41.9 vs
// 42.7 ms) and 0.2-0.8% on the T = 16 pass.
constexpr int kRowAuxNT = 2;
__device__ __forceinline__ double2 row_load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kRowAuxNT));
}
__device__ __forceinline__ void row_store(__amdgpu_buffer_rsrc_t r, int voff, int soff, double x, double y) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(x, y)), r, voff, soff, kRowAuxNT);
}

// Reflective mu > 0 head cell (cell 0 of segment 0) with distinct per-substep
// inflows, level by level: the head cell's own affine map (the host's probe of the
// reference's algebra, cell_step_maybe_head, cell.hpp cell_map<S, true>) on the
// carried state head_state(b), whose last component is the mirror's last-substep outflow --
// the same FMA rows the wavefront kernels run for it.  Rare (one cell per line per pass):
// the map is read from memory here instead of being kept in registers.  bs scales the map's
// constants (material coupling: the cell's B_g(T(x)); 1 otherwise).
template <int S, int T>
__device__ __forceinline__ void head_cell(const double *hmp, size_t stride, double (&X)[T][SchemeDim<S>::K],
                                          double &oi, double &oo, double bs) {
  constexpr int K = SchemeDim<S>::K, WN = map_count<S>();
  double Wh[WN];
#pragma unroll
  for (int n = 0; n < WN; ++n) Wh[n] = hmp[n * stride];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    double Xn[K], a, c;
    map_apply<S, true>(Wh, X[t], oi, oo, Xn, a, c, bs);
#pragma unroll
    for (int r = 0; r < K; ++r) X[t][r] = Xn[r];
    oi = a;
    oo = c;
  }
}

}  // namespace rtamd
