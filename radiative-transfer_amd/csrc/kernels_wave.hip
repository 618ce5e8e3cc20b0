// kernels_wave.hip -- short lines: a wavefront over (cell, time level), lanes over cells,
// every step of an advance in one launch (wavefront_kernel).
//
// The segment pipeline (kernels.hip) parallelises a line over segments that hand their
// exit states from one launch to the next, so a line's traversal costs a launch per
// segment and time block -- for the reference's own configurations (llnl_slab_test: 50
// cells, single_group / multi_group_equilibrium: 100) that is microseconds of dependent
// latency per step on a handful of workgroups.  Here a line (or, with the reflective left
// boundary, a mu < 0 line followed by its mu > 0 mirror) lives in ONE wave: lane j holds
// C consecutive cells of the chain in registers and, at tick tau, runs time level
// t = tau - j of its cells -- the upwind recurrence x_{k+1} = A x_k + b_k of every level is
// carried across lanes by one DPP lane shift of the carried state per tick (wave_shr:1), so
// level t of lane j starts from lane j - 1's exit state of the same level, produced one tick
// earlier.  n steps of an L-lane chain take n + L - 1 ticks of C cell maps each; the state
// is read once and written once per launch.
//
// Same arithmetic per (cell, level) as the pipelined segment pass (the per-line affine map
// of cell.hpp, exact carries; the reflective mu > 0 head cell by the reference's algebra
// with the mirror's per-substep outflows, sweep_device.hpp head_cell): bitwise equal to it.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "cell.hpp"
#include "kernels.hpp"

namespace rtamd {

// DPP wave_shr:1 (gfx9 family): lane l receives lane l - 1's value; lane 0 has no source and
// keeps `old` -- the chain head's inflow state, loop-carried in the same registers, so the
// head needs no per-tick select or copy.
__device__ __forceinline__ double lane_shift_up(double old, double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned long long o = __builtin_bit_cast(unsigned long long, old);
  const int lo = __builtin_amdgcn_update_dpp(static_cast<int>(o & 0xffffffffu), static_cast<int>(b & 0xffffffffu),
                                             0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(static_cast<int>(o >> 32), static_cast<int>(b >> 32), 0x138, 0xf, 0xf,
                                             false);
  return __builtin_bit_cast(double, (static_cast<unsigned long long>(static_cast<unsigned int>(hi)) << 32) |
                                        static_cast<unsigned int>(lo));
}

// grid: one wave per line (mu < 0 lines then mu > 0 lines, ell < H Gl) -- or, PAIR (the
// reflective left boundary), one wave per line pair ell (lanes [0, Lw) the mu < 0 line,
// [Lw, 2 Lw) its mirror).  Lw = lanes per line = ceil(N / C) <= 64 (PAIR: 32).  nsteps full
// steps from the stored state.  Padding cells (the last lane of a line holds N mod C real
// cells) feed nothing real -- except, with PAIR and N mod C != 0 (PAD), those of the mu < 0
// line, whose exit state is the mirror head's inflow: there they pass X through by a select
// (a per-lane branch would make every tick divergent).
template <int S, int C, bool PAIR, bool PAD>
__global__ __launch_bounds__(64) void wavefront_kernel(SegArgs a, int nsteps, int Lw) {
  constexpr int K = SchemeDim<S>::K, WN = map_count<S>();
  const int lane = threadIdx.x;
  const int nl = a.H * a.Gl;
  int half, ell, j;
  if (PAIR) {
    ell = blockIdx.x;
    half = lane < Lw ? 0 : 1;
    j = lane - half * Lw;
  } else {
    half = static_cast<int>(blockIdx.x) / nl;
    ell = static_cast<int>(blockIdx.x) % nl;
    j = lane;
  }
  const int used = PAIR ? 2 * Lw : Lw;  // lanes holding cells; the chain's lane index is `lane`
  const bool real = lane < used;
  const size_t stride = static_cast<size_t>(a.Lpad);
  double2 *Eh = a.E + static_cast<size_t>(half) * a.Nrow * stride + ell;

  double ein[C], eout[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int k = j * C + c;
    ein[c] = eout[c] = 0.0;
    if (real && k < a.N) {
      const double2 v = Eh[static_cast<size_t>(k) * stride];
      ein[c] = v.x;
      eout[c] = v.y;
    }
  }
  double W[WN];
#pragma unroll
  for (int n = 0; n < WN; ++n) W[n] = a.map[(static_cast<size_t>(half) * WN + n) * stride + ell];
  // a wave-uniform line map would live in SGPRs, and gfx9's one scalar operand per VALU op
  // then costs an accumulator copy per row and cell: keep it in VGPRs (after all the loads
  // are issued, so that they are in flight together)
#pragma unroll
  for (int n = 0; n < WN; ++n) asm volatile("" : "+v"(W[n]));
  const bool refl_head = PAIR && half == 1 && j == 0;  // one lane of a pair wave
  LineConst L{};
  if (refl_head) {
    const double *lcp = a.lc + static_cast<size_t>(half) * LC_COUNT * stride + ell;
#pragma unroll
    for (int n = 0; n < LC_COUNT; ++n) L.c[n] = lcp[n * stride];
  }

  // Xin: the state each lane receives at its tick -- lane - 1's exit state of the same level;
  // lane 0's stays the chain head's inflow state (solver.cpp:695-697), the mu < 0 line's
  // with PAIR.  Every lane runs its cells every tick (no divergent branch, no register
  // shuffling at a join); only lanes at a level in [0, nsteps) commit their nodes, and
  // an idle lane's exit state only ever reaches idle lanes.
  double Xin[K], X[K];
  {
    const double bv = a.bdry[static_cast<size_t>(PAIR ? 0 : half) * stride + ell];
    const double b[4] = {bv, bv, bv, bv};
    head_state<S>(b, Xin);
#pragma unroll
    for (int r = 0; r < K; ++r) X[r] = Xin[r];
  }
  // ticks [used, nsteps) have every lane of the chain at a level in [1, nsteps): that
  // stretch (all but the chain's fill and drain) runs without the commit masks, and there
  // component 0 of the received state (the upwind cell's node before level t, which the
  // map copies from dout) is not shifted in: it is the upwind cell's output node of level
  // t - 1, which this lane received one tick earlier as component K - 1 (CN, BDF2; the
  // chain head's inflow state has equal components) -- one DPP lane shift fewer per tick
  const auto run = [&](int tick0, int tick1, auto masked) {
    const auto body = [&](int tick) {
      if constexpr (K > 1 && !decltype(masked)::value) {
        // the shift of component K - 1 keeps Xin[0] as its `old` (lane 0: the head's
        // inflow state, all of whose components are equal), so the two registers trade
        // roles each tick and two ticks per iteration need no copy
        const double x0 = Xin[K - 1];
        Xin[K - 1] = lane_shift_up(Xin[0], X[K - 1]);
#pragma unroll
        for (int r = 1; r < K - 1; ++r) Xin[r] = lane_shift_up(Xin[r], X[r]);
        Xin[0] = x0;
      } else {
#pragma unroll
        for (int r = 0; r < K; ++r) Xin[r] = lane_shift_up(Xin[r], X[r]);
      }
      bool active = true;
      if constexpr (decltype(masked)::value) {
        const int t = tick - lane;
        active = real && t >= 0 && t < nsteps;
      }
#pragma unroll
      for (int r = 0; r < K; ++r) X[r] = Xin[r];
      if (PAIR && refl_head) {
        // solver.cpp:677-684: the mirror's outflow after each substep is the inflow b of the
        // same substep; head_state(b) differs from the received state in component 0 only
        if constexpr (S == SCHEME_BDF2) X[0] = X[2];
        if constexpr (S == SCHEME_CN) X[0] = X[1];
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        double Xn[K], oi, oo;
        if (PAIR && c == 0 && refl_head) {  // reflective head: the reference's algebra, distinct inflows
          cell_step_maybe_head<S>(L, a.hd, false, ein[0], eout[0], X, true, X[K - 1], oi, oo);
#pragma unroll
          for (int r = 0; r < K; ++r) Xn[r] = X[r];
        } else {
          map_apply<S, true>(W, X, ein[c], eout[c], Xn, oi, oo);
        }
        if constexpr (PAD) {
          const bool pad = j * C + c >= a.N;
#pragma unroll
          for (int r = 0; r < K; ++r) X[r] = pad ? X[r] : Xn[r];
        } else {
#pragma unroll
          for (int r = 0; r < K; ++r) X[r] = Xn[r];
        }
        ein[c] = active ? oi : ein[c];
        eout[c] = active ? oo : eout[c];
      }
    };
    // two ticks per iteration: the loop-carried renames of X, ein and eout then cancel
    int tick = tick0;
    for (; tick + 1 < tick1; tick += 2) {
      body(tick);
      body(tick + 1);
    }
    if (tick < tick1) body(tick);
  };
  const int ticks = nsteps + used - 1;
  if (nsteps > used) {
    run(0, used, std::true_type{});
    run(used, nsteps, std::false_type{});
    run(nsteps, ticks, std::true_type{});
  } else {
    run(0, ticks, std::true_type{});
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int k = j * C + c;
    if (real && k < a.N) Eh[static_cast<size_t>(k) * stride] = make_double2(ein[c], eout[c]);
  }
}

template <int S, bool PAIR>
static hipError_t launch_wave_s(int C, const SegArgs &a, int nsteps, int Lw, int grid, hipStream_t st) {
  const bool pad = PAIR && a.N % C != 0;
  switch (C) {
#define RT_WAVE_CASE(c)                                                                                      \
  case c:                                                                                                    \
    if (pad)                                                                                                 \
      hipLaunchKernelGGL((wavefront_kernel<S, c, PAIR, PAIR && (c > 1)>), dim3(grid), dim3(64), 0, st, a, nsteps, \
                         Lw);                                                                                \
    else                                                                                                     \
      hipLaunchKernelGGL((wavefront_kernel<S, c, PAIR, false>), dim3(grid), dim3(64), 0, st, a, nsteps, Lw); \
    break;
    RT_WAVE_CASE(1) RT_WAVE_CASE(2) RT_WAVE_CASE(4) RT_WAVE_CASE(8)
#undef RT_WAVE_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// lanes of a chain: 64, a reflective pair 2 x 32
int wavefront_cells_per_lane(int N, bool reflective) {
  const int lanes = reflective ? 32 : 64;
  const int c = (N + lanes - 1) / lanes;
  for (int C : {1, 2, 4, 8})
    if (c <= C) return C;
  return 0;  // too long: the segment pipeline
}

hipError_t launch_wavefront(int scheme, const SegArgs &a, int nsteps, hipStream_t st) {
  const bool pair = a.reflective != 0;
  const int C = wavefront_cells_per_lane(a.N, pair);
  const int nl = a.H * a.Gl;
  if (C == 0 || nl <= 0 || nsteps < 0) return hipErrorInvalidValue;
  if (nsteps == 0) return hipSuccess;
  const int Lw = (a.N + C - 1) / C;
  const int grid = pair ? nl : 2 * nl;
  switch (scheme) {
    case SCHEME_BE:
      return pair ? launch_wave_s<SCHEME_BE, true>(C, a, nsteps, Lw, grid, st)
                  : launch_wave_s<SCHEME_BE, false>(C, a, nsteps, Lw, grid, st);
    case SCHEME_CN:
      return pair ? launch_wave_s<SCHEME_CN, true>(C, a, nsteps, Lw, grid, st)
                  : launch_wave_s<SCHEME_CN, false>(C, a, nsteps, Lw, grid, st);
    default:
      return pair ? launch_wave_s<SCHEME_BDF2, true>(C, a, nsteps, Lw, grid, st)
                  : launch_wave_s<SCHEME_BDF2, false>(C, a, nsteps, Lw, grid, st);
  }
}

}  // namespace rtamd
