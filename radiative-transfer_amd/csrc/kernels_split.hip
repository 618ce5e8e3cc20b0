// kernels_split.hip -- the level-split pipelined pass (sweep_split_kernel): a BDF2
// segment's T levels shared by 2 or 4 waves of a workgroup.  Its own translation unit
// (the kernel is instantiated for 14 (T, waves) pairs, the tail variant for 9) so it compiles beside kernels.hip.
#include <hip/hip_runtime.h>

#include "cell.hpp"
#include "kernels.hpp"
#include "sweep_device.hpp"

namespace rtamd {

// ------------------------------------------------------------------------
// Level-split pipelined pass: the same launch as sweep_block_kernel<S, T, 2>
// with its T levels shared by KW waves of one workgroup (KW = 2 or 4), wave w
// running levels [w T/KW, (w + 1) T/KW).  Wave 0 streams the rows in from HBM,
// the last wave stores them, and each wave hands its chunk's nodes at its last
// level to the next wave through LDS (two buffers per link, one barrier per
// chunk interval): in interval I wave w computes chunk I - 2w from registers
// while it refills them with chunk I - 2w + 1 (written by wave w - 1 in
// interval I - 1) and writes chunk I - 2w into its outgoing buffer (I - 2w) & 1.
// Same arithmetic in the same order per (cell, level) as the one-wave kernel:
// bitwise equal.
//   KW = 2: each wave holds half the carried states (X), so a SIMD runs two
//     waves instead of one: at T = 20 (one-wave kernel: 126 AGPRs beside 256
//     VGPRs) 8.29-8.31 vs 8.52-8.53 ms per step on SL, the default there; at
//     T = 16 4% slower than one wave (140.6 vs 134.6 ms per pass).
//   KW = 2, 4 in the pipeline's fill and drain: a launch with few active chain
//     positions runs each segment on more waves, so the lines' traversal takes
//     1/KW of the time while the chip would otherwise idle (rtsn_api.hip
//     pipe_launch).
// ------------------------------------------------------------------------
// TAIL: the wave runs only its first nl of the TW levels (wave-uniform), the rest pass the
// nodes through unchanged -- the run's last n mod T steps as a pipelined block (tail_levels).
template <int S, int TW, int C, bool IN_HBM, bool OUT_HBM, bool LASTCH, bool TAIL>
__device__ __forceinline__ void split_chunk(const double *W, double (&ein)[C], double (&eout)[C],
                                            double (&X)[TW][SchemeDim<S>::K], bool head, double h_oi, double h_oo,
                                            const double2 *lin, double2 *lout, __amdgpu_buffer_rsrc_t Rw,
                                            __amdgpu_buffer_rsrc_t Rn, int voff, int row_bytes, int nv, int lane,
                                            int nl) {
  constexpr int K = SchemeDim<S>::K;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (LASTCH && c >= nv) continue;  // wave-uniform: past the end of the segment
    double oi = ein[c], oo = eout[c];
    if (c == 0 && head) {  // reflective head cell, computed in the prologue
      oi = h_oi;
      oo = h_oo;
    } else {
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        if constexpr (TAIL)
          if (t >= nl) break;
        double Xn[K], a, e;
        map_apply<S, true>(W, X[t], oi, oo, Xn, a, e);
#pragma unroll
        for (int r = 0; r < K; ++r) X[t][r] = Xn[r];
        oi = a;
        oo = e;
      }
    }
    if constexpr (OUT_HBM)
      row_store(Rw, voff, c * row_bytes, oi, oo);
    else  // hand the nodes at this wave's last level to the next wave
      lout[c * 64 + lane] = make_double2(oi, oo);
    if constexpr (IN_HBM) {
      // refill from HBM one cell late: row c - 1 with the next chunk's (row C - 1 of THIS
      // chunk at cell 0).  The upwind node of cell c - 1 (row c - 1's e_out) is the carried
      // state's component 0 until cell c's first level, so an earlier load could not reuse
      // its registers: the allocator copied the loaded rows at the loop head, whose wait for
      // the chunk's last loads, issued just before, stalled every chunk's start
      const bool load = LASTCH ? (c == 0 && C - 1 < nv) : true;
      if (load) {
        const int rr = c == 0 ? C - 1 : c - 1;
        const double2 v = row_load(c == 0 ? Rw : Rn, voff, rr * row_bytes);
        ein[rr] = v.x;
        eout[rr] = v.y;
      }
      // each load after its cell's FMAs (left alone, the scheduler sinks them to the end)
      __builtin_amdgcn_sched_group_barrier(0x002, TW * 28, 0);  // VALU
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);        // VMEM read
    } else if constexpr (!LASTCH) {  // refill with the next chunk from the previous wave
      const double2 v = lin[c * 64 + lane];
      ein[c] = v.x;
      eout[c] = v.y;
    }
  }
}

// Wave w of KW runs levels [split_t0, split_t0 + split_tw) of the T: split_role and the choice
// of its TAIL body (split_role_of) take both from here.
template <int T, int KW, int w>
__device__ __forceinline__ constexpr int split_t0() {
  return w * (T / KW);
}
template <int T, int KW, int w>
__device__ __forceinline__ constexpr int split_tw() {
  return T / KW;
}

// Wave w's role (compile time: with the role a runtime branch inside one body the
// allocation measured ~340 registers, each role alone ~215).
template <int S, int T, int KW, int w, bool TAIL>
__device__ __forceinline__ void split_role(const SegArgs &a, double2 (*hand)[2][split_chunk_cells() * 64],
                                           double2 *hhead) {
  constexpr int K = SchemeDim<S>::K;
  constexpr int TW = split_tw<T, KW, w>();  // levels [t0, t0 + TW)
  constexpr int WN = map_count<S>();
  constexpr int C = split_chunk_cells();
  constexpr bool IN = w == 0, OUT = w == KW - 1;
  const int lane = threadIdx.x & 63;
  constexpr int t0 = split_t0<T, KW, w>();  // this wave's first level
  const size_t stride = static_cast<size_t>(a.Lpad);
  int half, s, q, pos;
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
  const int slot = (a.pass_lo - (pos - a.pos_lo)) & 1;
  // TAIL: position pos_lo's block is a.tail_levels < T levels (layout and carried states
  // still T's); every other position runs all T
  const int nl = TAIL && pos == a.pos_lo ? min(max(a.tail_levels - t0, 0), TW) : TW;
  const int ell = q * 64 + lane;
  const bool neg = half == 0;
  const int k_begin = s * a.Ls;
  const int k_end = min(a.N, k_begin + a.Ls);
  if (k_begin >= k_end) return;  // workgroup-uniform
  const size_t seg_stride = static_cast<size_t>(T * K) * stride;
  const size_t half_stride = static_cast<size_t>(a.Sg) * seg_stride;

  // ---- inflow and carried state of this wave's levels ----
  const bool head_seg = (s == 0);
  double b[TW][4];
  {
    const double v = a.bdry[static_cast<size_t>(half) * stride + ell];
#pragma unroll
    for (int t = 0; t < TW; ++t) b[t][0] = b[t][1] = b[t][2] = b[t][3] = v;
  }
  const bool refl_head = head_seg && !neg && a.reflective;
  if (refl_head) {  // solver.cpp:677-684, as in sweep_block_kernel (MODE 2)
    const double *src = a.aggs[slot] + (a.Sg - 1) * seg_stride + ell;
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      if constexpr (S == SCHEME_BDF2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) b[t][r] = src[((t0 + t) * K + 1 + r) * stride];
      } else {
        b[t][0] = b[t][1] = b[t][2] = b[t][3] = src[((t0 + t) * K + K - 1) * stride];
      }
    }
  }
  double X[TW][K];
  if (head_seg) {
#pragma unroll
    for (int t = 0; t < TW; ++t) head_state<S>(b[t], X[t]);
  } else {
    const double *up = a.aggs[slot] + half * half_stride + (s - 1) * seg_stride + ell;
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int r = 0; r < K; ++r) X[t][r] = up[((t0 + t) * K + r) * stride];
  }

  // ---- rows: wave 0 streams them in, the last wave stores them ----
  const int row_bytes = a.Lpad * static_cast<int>(sizeof(double2));
  const int voff = lane * static_cast<int>(sizeof(double2));
  const double2 *Eh = a.E + static_cast<size_t>(half) * a.Nrow * stride + q * 64;
  auto rows = [&](int k0) { return rows_rsrc<C>(Eh + static_cast<size_t>(k0) * stride, row_bytes); };
  double ein[C], eout[C];
  if constexpr (IN) {
    const __amdgpu_buffer_rsrc_t R0 = rows(k_begin);
#pragma unroll
    for (int c = 0; c < C; ++c) {  // (row C - 1 comes with the first chunk's cell 0)
      const double2 v = c + 1 < C ? row_load(R0, voff, c * row_bytes) : make_double2(0.0, 0.0);
      ein[c] = v.x;
      eout[c] = v.y;
    }
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c) ein[c] = eout[c] = 0.0;
  }
  // reflective head cell: wave r runs its levels on wave r - 1's result, in turn
  double h_oi = 0.0, h_oo = 0.0;
  if (refl_head) {  // workgroup-uniform: every wave passes the KW - 1 barriers
    const double *hmp = a.hmap + ell;
    if constexpr (IN) {
      h_oi = ein[0];
      h_oo = eout[0];
    }
#pragma unroll
    for (int r = 0; r < KW - 1; ++r) {
      if (r == w) {  // compile-time after unrolling
        if constexpr (!IN) {
          const double2 v = hhead[lane];
          h_oi = v.x;
          h_oo = v.y;
        }
        head_cell<S, TW>(hmp, stride, X, h_oi, h_oo, 1.0);
        hhead[lane] = make_double2(h_oi, h_oo);
      }
      __syncthreads();
    }
    if constexpr (OUT) {
      const double2 v = hhead[lane];
      h_oi = v.x;
      h_oo = v.y;
      head_cell<S, TW>(hmp, stride, X, h_oi, h_oo, 1.0);
    }
  }

  double W[WN];
#pragma unroll
  for (int n = 0; n < WN; ++n) W[n] = a.map[(static_cast<size_t>(half) * WN + n) * stride + ell];
  // every prologue load (map, carried states, chunk 0) complete before the chunks start:
  // the wait-count pass merges the loop's entry into its head, and a map load still
  // pending there made EVERY chunk start wait for all loads in flight (vmcnt(0)) -- the
  // next chunk's rows, issued just before
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)

  // ---- chunk intervals: nch + 2 (KW - 1) of them, one barrier after each, for every wave ----
  const int nch = (k_end - k_begin + C - 1) / C;
  const double2 *lin = hand[w > 0 ? w - 1 : 0][0];  // (wave 0 reads HBM, the last wave writes it:
  double2 *lout = hand[w < KW - 1 ? w : 0][0];       //  their unused link pointer is never touched)
  constexpr int LB = split_chunk_cells() * 64;  // one buffer of a link
  if constexpr (!IN) {
    for (int I = 0; I < 2 * w - 1; ++I) __syncthreads();  // the previous waves fill the pipeline
    // interval 2w - 1: chunk 0 of the previous wave (written in interval 2w - 2)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const double2 v = lin[c * 64 + lane];
      ein[c] = v.x;
      eout[c] = v.y;
    }
    __syncthreads();
  }
  int k0 = k_begin;
  for (int m = 0; m + 1 < nch; ++m, k0 += C) {
    split_chunk<S, TW, C, IN, OUT, false, TAIL>(W, ein, eout, X, refl_head && m == 0, h_oi, h_oo,
                                                lin + ((m + 1) & 1) * LB, lout + (m & 1) * LB, rows(k0), rows(k0 + C),
                                                voff, row_bytes, C, lane, nl);
    __syncthreads();
  }
  split_chunk<S, TW, C, IN, OUT, true, TAIL>(W, ein, eout, X, refl_head && nch == 1, h_oi, h_oo, lin,
                                             lout + ((nch - 1) & 1) * LB, rows(k0), rows(k0), voff, row_bytes,
                                             k_end - k0, lane, nl);
  __syncthreads();
  double *ag = a.aggs[slot] + half * half_stride + static_cast<size_t>(s) * seg_stride + ell;
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int r = 0; r < K; ++r) ag[((t0 + t) * K + r) * stride] = X[t][r];
  for (int I = 0; I < 2 * (KW - 1 - w); ++I) __syncthreads();  // the later waves drain it
}

constexpr int kSplitPrioWave = 0;  // the wave given issue priority 1 (wave 0 streams the rows in)
// Wave w's role; with `tail`, the waves whose levels reach past the tail's take the TAIL body,
// the others the plain one -- correct only when wave 0's levels all lie inside the tail
// (tail_levels >= split_tw of wave 0), which launch_split_tail enforces.
template <int S, int T, int KW, int w>
__device__ __forceinline__ void split_role_of(const SegArgs &a, double2 (*hand)[2][split_chunk_cells() * 64],
                                              double2 *hhead, bool tail) {
  if (tail && a.tail_levels < split_t0<T, KW, w>() + split_tw<T, KW, w>())
    split_role<S, T, KW, w, true>(a, hand, hhead);
  else
    split_role<S, T, KW, w, false>(a, hand, hhead);
}

template <int S, int T, int KW, bool TAIL>
__device__ __forceinline__ void split_roles(const SegArgs &a, double2 (*hand)[2][split_chunk_cells() * 64],
                                            double2 *hhead, int w) {
  bool tail = false;  // workgroup-uniform: this workgroup is position pos_lo's, which runs the tail
  if constexpr (TAIL) tail = (static_cast<int>(blockIdx.x) % (a.Q * a.npos)) / a.Q == 0;
  if constexpr (KW == 2) {
    if (w == 0)
      split_role_of<S, T, 2, 0>(a, hand, hhead, tail);
    else
      split_role_of<S, T, 2, 1>(a, hand, hhead, tail);
  } else {
    if (w == 0)
      split_role_of<S, T, 4, 0>(a, hand, hhead, tail);
    else if (w == 1)
      split_role_of<S, T, 4, 1>(a, hand, hhead, tail);
    else if (w == 2)
      split_role_of<S, T, 4, 2>(a, hand, hhead, tail);
    else
      split_role_of<S, T, 4, 3>(a, hand, hhead, tail);
  }
}

template <int S, int T, int KW>
__global__ __launch_bounds__(64 * KW) __attribute__((amdgpu_waves_per_eu(2, 2))) void sweep_split_kernel(SegArgs a) {
  static_assert(T % KW == 0 && (KW == 2 || KW == 4), "levels split evenly over 2 or 4 waves");
  __shared__ double2 hand[KW - 1][2][split_chunk_cells() * 64];  // link w: wave w -> w + 1, chunk m in [m & 1]
  __shared__ double2 hhead[64];                                    // reflective head cell, wave to wave
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Static issue priority for wave 0 (it streams the rows in and runs the first levels; the
  // SIMD it shares with another workgroup's wave gives it the issue slot first): the T = 20
  // pass 8.42-8.46 vs 8.61-8.65 ms/step, priority for wave 1 instead 8.52-8.57
  // (profiles/archive/r03ap_prio.jsonl); on another box 8.17-8.18 vs 8.36-8.41, and the four-wave
  // T = 40 pass 7.85-7.88 vs 7.90-7.91 (r03aq_prio.jsonl; MI355X_MICROARCH.md, two waves per
  // SIMD, item 4).
  if (w == kSplitPrioWave) __builtin_amdgcn_s_setprio(1);
  split_roles<S, T, KW, false>(a, hand, hhead, w);
}

// A pipelined launch whose first active position (pos_lo, vacuum lines only) runs the
// run's last a.tail_levels < T steps while the positions behind it run whole T blocks: the
// n mod T remainder rides the drain (one extra launch, for the last position) instead of
// aligned passes with the cross-segment correction after it.  The tail positions keep T's
// aggregate layout, so the two kinds share the aggs ring.  Same arithmetic per (cell,
// level) as every other schedule.
template <int S, int T, int KW>
__global__ __launch_bounds__(64 * KW) __attribute__((amdgpu_waves_per_eu(2, 2))) void sweep_split_tail_kernel(
    SegArgs a) {
  __shared__ double2 hand[KW - 1][2][split_chunk_cells() * 64];
  __shared__ double2 hhead[64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w == kSplitPrioWave) __builtin_amdgcn_s_setprio(1);
  // The waves that run all their levels take the plain body: with the tail's level count a
  // runtime bound in the level loop the workgroup ran ~55% slower (the loop's pinned loads
  // lose their place), which set every drain launch's time (16-group shard, 100 steps: 237
  // vs 150 ms for 96 steps, gpurun r04ac)
  split_roles<S, T, KW, true>(a, hand, hhead, w);
}

template <int T, int KW>
static hipError_t launch_split_t(const SegArgs &a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((sweep_split_kernel<SCHEME_BDF2, T, KW>), dim3(grid), dim3(64 * KW), 0, st, a);
  return hipGetLastError();
}

template <int T, int KW>
static hipError_t launch_split_tail_t(const SegArgs &a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((sweep_split_tail_kernel<SCHEME_BDF2, T, KW>), dim3(grid), dim3(64 * KW), 0, st, a);
  return hipGetLastError();
}

template <int T, int KW>
static hipError_t occupancy_split_t(int *w) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(w, sweep_split_kernel<SCHEME_BDF2, T, KW>, 64 * KW, 0);
}

// (T, waves) pairs with a split kernel: 2 waves up to 20 levels (beyond, 12 or more
// levels per wave spill), 4 waves for T divisible by 4 up to 40.  T = 4 over 4 waves (one
// level per wave): short planned runs, whose time is the line's traversal (rt_plan_schedule).
#define RT_SPLIT_PAIRS(X) X(4, 2) X(8, 2) X(10, 2) X(12, 2) X(16, 2) X(20, 2) \
  X(4, 4) X(8, 4) X(12, 4) X(16, 4) X(20, 4) X(24, 4) X(32, 4) X(40, 4)

hipError_t launch_split(int T, int waves, const SegArgs &a, int grid, hipStream_t st) {
#define RT_SPLIT_LAUNCH(t, k) \
  if (T == t && waves == k) return launch_split_t<t, k>(a, grid, st);
  RT_SPLIT_PAIRS(RT_SPLIT_LAUNCH)
#undef RT_SPLIT_LAUNCH
  return hipErrorInvalidValue;
}

// the planned schedules' blocks (four waves) and two waves up to 16 levels; not (20, 2) and
// (40, 4): 10 levels per wave with the tail's exit spill (416 B of scratch per lane)
#define RT_SPLIT_TAIL_PAIRS(X) X(8, 2) X(12, 2) X(16, 2) \
  X(8, 4) X(12, 4) X(16, 4) X(20, 4) X(24, 4) X(32, 4)

bool split_tail_supported(int T, int waves) {
#define RT_SPLIT_HAS(t, k) \
  if (T == t && waves == k) return true;
  RT_SPLIT_TAIL_PAIRS(RT_SPLIT_HAS)
#undef RT_SPLIT_HAS
  return false;
}

hipError_t launch_split_tail(int T, int waves, const SegArgs &a, int grid, hipStream_t st) {
  // the tail must cover wave 0's levels: its plain body runs them all (split_role_of)
  if (a.reflective || waves < 1 || a.tail_levels < T / waves || a.tail_levels >= T) return hipErrorInvalidValue;
#define RT_SPLIT_TAIL_LAUNCH(t, k) \
  if (T == t && waves == k) return launch_split_tail_t<t, k>(a, grid, st);
  RT_SPLIT_TAIL_PAIRS(RT_SPLIT_TAIL_LAUNCH)
#undef RT_SPLIT_TAIL_LAUNCH
  return hipErrorInvalidValue;
}

hipError_t split_occupancy(int T, int waves, int *w) {
#define RT_SPLIT_OCC(t, k) \
  if (T == t && waves == k) return occupancy_split_t<t, k>(w);
  RT_SPLIT_PAIRS(RT_SPLIT_OCC)
#undef RT_SPLIT_OCC
  return hipErrorInvalidValue;
}

}  // namespace rtamd
