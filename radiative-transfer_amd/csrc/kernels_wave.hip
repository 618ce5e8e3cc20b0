// kernels_wave.hip -- short lines: a wavefront over (cell, time level), lanes over cells,
// every step of an advance in one launch (wavefront_kernel).
//
// The segment pipeline (kernels.hip) parallelises a line over segments that hand their
// exit states from one launch to the next, so a line's traversal costs a launch per
// segment and time block -- for the reference's own configurations (llnl_slab_test: 50
// cells, single_group / multi_group_equilibrium: 100) that is microseconds of dependent
// latency per step on a handful of workgroups.  Here a line (or, with the reflective left
// boundary, a mu < 0 line followed by its mu > 0 mirror) is a CHAIN of lanes of one
// workgroup: chain lane g holds C consecutive cells in registers and, at tick tau, runs
// time level t = tau - g of its cells -- the upwind recurrence x_{k+1} = A x_k + b_k of
// every level is carried across lanes by one DPP lane shift of the carried state per tick
// (wave_shr:1), so level t of lane g starts from lane g - 1's exit state of the same level,
// produced one tick earlier.  n steps of an L-lane chain take n + L - 1 ticks of C cell
// maps each; the state is read once and written once per launch.
//
// A chain longer than one wave (up to kWaveMaxWaves waves, 4096 cells) runs on chain_kernel
// below: the waves of one workgroup hand the carried state over through an LDS ring and meet
// at a barrier every kChainBlock ticks.  Which lines take one wave and which a chain is
// wavefront_plan's choice, from measured tick costs (profiles/r05*_plan.jsonl).
//
// Same arithmetic per (cell, level) as the pipelined segment pass (the per-line affine map
// of cell.hpp, exact carries; the reflective mu > 0 head cell by its own map of the
// reference's head algebra, as sweep_device.hpp head_cell runs it): bitwise equal to it,
// whatever the cells per lane and waves per chain.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "cell.hpp"
#include "kernels.hpp"

namespace rtamd {

// DPP wave_shr:1 (gfx9 family): lane l receives lane l - 1's value; lane 0 has no source and
// keeps `old` -- the chain head's inflow state, loop-carried in the same registers (or the
// previous wave's exit state from LDS), so the head needs no per-tick select or copy.
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

// Ticks per loop iteration of the single-wave kernel (even)
constexpr int kWaveUnroll = 8;
static_assert(kWaveUnroll >= 2 && kWaveUnroll % 2 == 0, "renames cancel over an even number of ticks");


// The lane's cell maps.  A pair chain's mu > 0 head lane runs its cell 0 on the head cell's
// own map (cell.hpp cell_map<S, true>: the reference's head algebra with the mirror's
// per-substep outflows, probed into the same FMA rows), so every lane runs the same
// instructions every tick -- round 4 branched into the reference's algebra there, and the
// exec-mask divergence roughly doubled a reflective chain's tick.  The head map differs from
// the line's only from slot head_map_first on (BDF2: the BDF substep's output and oin, which
// read the mirror's last-substep outflow; the host checks the others are bitwise the line's;
// BE / CN: nowhere), so a lane holds just those: W gets them on the head lane where a lane has
// one cell; with 2-4 cells, cell 0 reads W0 = W with them replaced (the rest are W's own
// registers).  In the 5-8-wave chains at 8 cells per lane (which spilled already) the head
// lane instead redoes those rows for its cell 0 with the head map's coefficients,
// wave-uniform in Wh (the pair's line is the workgroup's): 16 FMAs under an exec mask in the
// head's wave only -- 927-1046 ns per tick at 5-8 waves against 1032-1113 with W0, while up to
// 4 waves W0 is 0-8% the faster (profiles/r05t_chain_plan_c8.jsonl).
template <int S, int C, bool WIDE>
__device__ __forceinline__ constexpr bool head_redo() {
  return WIDE && C >= 8 && head_map_first<S>() < map_count<S>();
}

template <int S, int C, bool PAIR, bool REDO>
__device__ __forceinline__ void head_maps(const SegArgs &a, int half, int ell, size_t stride, bool refl_head,
                                          double (&W)[map_count<S>()], double (&W0)[map_count<S>()],
                                          double (&Wh)[map_count<S>()]) {
  constexpr int WN = map_count<S>(), F = head_map_first<S>();
#pragma unroll
  for (int n = 0; n < WN; ++n) W[n] = a.map[(static_cast<size_t>(half) * WN + n) * stride + ell];
  double T[WN - F > 0 ? WN - F : 1];
#pragma unroll
  for (int n = 0; n < WN; ++n) Wh[n] = 0.0;  // (REDO reads slots >= F only)
  if constexpr (PAIR) {
#pragma unroll
    for (int n = F; n < WN; ++n) {
      const double h = a.hmap[n * stride + ell];  // every lane (ell < Lpad): a select, no branch
      if constexpr (REDO)
        Wh[n] = h;  // a wave-uniform address: scalar loads
      else
        T[n - F] = refl_head ? h : W[n];
    }
    if constexpr (C == 1) {
#pragma unroll
      for (int n = F; n < WN; ++n) W[n] = T[n - F];
    }
  }
  // a wave-uniform line map would live in SGPRs, and gfx9's one scalar operand per VALU op
  // then costs an accumulator copy per row and cell: keep it in VGPRs (after all the loads
  // are issued, so that they are in flight together)
#pragma unroll
  for (int n = 0; n < WN; ++n) asm volatile("" : "+v"(W[n]));
#pragma unroll
  for (int n = 0; n < WN; ++n) W0[n] = (PAIR && C > 1 && !REDO && n >= F) ? T[n - F] : W[n];
}

// Cell c of a lane: the map (W0 for a pair chain's cell 0), and with REDO the head lane's
// redo of the rows where its map differs (head_maps).
template <int S, int C, bool PAIR, bool REDO>
__device__ __forceinline__ void lane_cell(int c, bool refl_head, const double (&W)[map_count<S>()],
                                          const double (&W0)[map_count<S>()], const double (&Wh)[map_count<S>()],
                                          const double *X, double din, double dout, double *Xn, double &oi,
                                          double &oo) {
  constexpr int K = SchemeDim<S>::K;
  map_apply<S, true>(PAIR && C > 1 && c == 0 ? W0 : W, X, din, dout, Xn, oi, oo);
  if constexpr (PAIR && REDO) {
    if (c == 0 && refl_head) map_apply<S, true, false, false, K - 1>(Wh, X, din, dout, Xn, oi, oo);
  }
}

// grid: one workgroup per line (mu < 0 lines then mu > 0 lines, ell < H Gl) -- or, PAIR (the
// reflective left boundary), one per line pair ell (chain lanes [0, Lw) the mu < 0 line,
// [Lw, 2 Lw) its mirror).  Lw = lanes per line = ceil(N / C); the chain fills one wave.
// nsteps full steps from the stored state.  Padding cells (the last lane of a line holds
// N mod C real cells) feed nothing real -- except, with PAIR and N mod C != 0 (PAD), those of the mu < 0 line, whose exit
// state is the mirror head's inflow: there they pass X through by a select (a per-lane
// branch would make every tick divergent).
template <int S, int C, bool PAIR, bool PAD>
__global__ __launch_bounds__(64) void wavefront_kernel(SegArgs a, int nsteps, int Lw) {
  constexpr int K = SchemeDim<S>::K, WN = map_count<S>();
  const int g = threadIdx.x & 63;  // chain lane
  const int nl = a.H * a.Gl;
  int half, ell, j;
  if (PAIR) {
    ell = blockIdx.x;
    half = g < Lw ? 0 : 1;
    j = g - half * Lw;
  } else {
    half = static_cast<int>(blockIdx.x) / nl;
    ell = static_cast<int>(blockIdx.x) % nl;
    j = g;
  }
  const int used = PAIR ? 2 * Lw : Lw;  // chain lanes holding cells
  const bool real = g < used;
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
  const bool refl_head = PAIR && half == 1 && j == 0;  // one lane of a pair chain
  double W[WN], W0[WN], Wh[WN];
  head_maps<S, C, PAIR, false>(a, half, ell, stride, refl_head, W, W0, Wh);

  // Xin: the state each lane receives at its tick -- lane - 1's exit state of the same level;
  // chain lane 0's is the chain head's inflow state (solver.cpp:695-697), the mu < 0 line's
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
  // the ticks between the chain's fill and drain (every lane of this wave at a level in
  // [1, nsteps)) run without the commit masks, and there component 0 of the received state
  // (the upwind cell's node before level t, which the map copies from dout) is not shifted
  // in: it is the upwind cell's output node of level t - 1, which this lane received one
  // tick earlier as component K - 1 (CN, BDF2; the chain head's inflow state has equal
  // components) -- one DPP lane shift fewer per tick
  const auto run = [&](int tick0, int tick1, auto masked) {
    const auto body = [&](int tick) {
      double o[K];
#pragma unroll
      for (int r = 0; r < K; ++r) o[r] = Xin[r];
      if constexpr (K > 1 && !decltype(masked)::value) {
        // the shift of component K - 1 keeps Xin[0] as its `old` (lane 0 of the chain: the
        // head's inflow state, all of whose components are equal), so the two registers trade
        // roles each tick and two ticks per iteration need no copy
        const double x0 = Xin[K - 1];
        Xin[K - 1] = lane_shift_up(Xin[0], X[K - 1]);
#pragma unroll
        for (int r = 1; r < K - 1; ++r) Xin[r] = lane_shift_up(o[r], X[r]);
        Xin[0] = x0;
      } else {
#pragma unroll
        for (int r = 0; r < K; ++r) Xin[r] = lane_shift_up(o[r], X[r]);
      }
      bool active = true;
      if constexpr (decltype(masked)::value) {
        const int t = tick - g;
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
        lane_cell<S, C, PAIR, false>(c, refl_head, W, W0, Wh, X, ein[c], eout[c], Xn, oi, oo);
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
    // kWaveUnroll (even) ticks per iteration: the loop-carried renames of X, ein and eout
    // then cancel
    int tick = tick0;
    for (; tick + kWaveUnroll - 1 < tick1; tick += kWaveUnroll) {
#pragma unroll
      for (int u = 0; u < kWaveUnroll; ++u) body(tick + u);
    }
    for (; tick < tick1; ++tick) body(tick);
  };
  const int ticks = nsteps + used - 1;
  // the unmasked ticks: every real lane at a level in [1, nsteps)
  const int u_lo = min(63, used - 1) + 1, u_hi = max(u_lo, nsteps);
  if (u_lo < u_hi && u_hi <= ticks) {
    run(0, u_lo, std::true_type{});
    run(u_lo, u_hi, std::false_type{});
    run(u_hi, ticks, std::true_type{});
  } else {
    run(0, ticks, std::true_type{});
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int k = j * C + c;
    if (real && k < a.N) Eh[static_cast<size_t>(k) * stride] = make_double2(ein[c], eout[c]);
  }
}

// ---------------------------------------------------------------------------
// Chains over several waves (chain_kernel, round 4).  Round 3's chain (a multi-wave path of
// wavefront_kernel, removed in round 5) ran ~75 instructions per tick against the single
// wave's 37: runtime ring indices, a per-tick barrier test, the writer's branch and rotating
// prefetch registers became SALU address arithmetic, exec-mask branches and register moves
// (DESIGN.md §2.7).  Here every wave runs
// its tick stream in blocks of kChainBlock wall ticks that end in the barrier, so inside a
// block every ring slot is a compile-time offset from one per-block base: wave w runs
// kChainSkew = 2 blocks of chain ticks behind wave w - 1, so the chain tick of a block's
// first wall tick is a multiple of the block (mod the ring) for every wave.  Slot s of
// boundary w holds what lane 0 of wave w receives at chain tick s (lane 63 of wave w - 1's
// exit state of tick s - 1: written at wall tick s - 1 + 16 (w - 1), read one tick ahead,
// at wall tick s - 1 + 16 w: two barriers later; overwritten 32 chain ticks on, after the
// read and a barrier).  Components 1..K-1 sit first in a slot (two 16-byte pairs for BDF2,
// the whole unmasked exchange), component 0 after them: lane 0 needs it from the ring only
// while it is at level 0 (at levels >= 1 it is the component K-1 lane 0 received one tick
// earlier, as in the single wave), so the writer's unmasked ticks store components 1..K-1.  Region
// 0 holds the chain head's inflow state in every slot, so wave 0 reads the same way.  Writer
// stores go two ticks at a time (one exec-mask branch per pair).  Same arithmetic per (cell,
// level) as wavefront_kernel: bitwise the pipelined schedule.
constexpr int kChainBlock = 8;                 // wall ticks per barrier block
constexpr int kChainSkew = 2 * kChainBlock;    // chain ticks wave w runs behind wave w - 1
constexpr int kChainRing = 4 * kChainBlock;    // slots per boundary (and region 0)
constexpr int kChainSlot = 6;                  // doubles per slot (48 B: 16-byte aligned)
// masked blocks (a wave's fill and drain ramps) are unrolled too (2-6%: r04r); scheduling
// fences at each tick's start (4-8 cells per lane) and after its ring read
static_assert(kChainSkew >= kChainBlock + 2 && kChainSkew + kChainBlock <= kChainRing, "ring too short for the skew");
static_assert(kChainSkew % kChainBlock == 0 && kChainRing % kChainBlock == 0, "blocks align with the ring");

template <int K>
__device__ __forceinline__ constexpr int slot_pos(int r) {  // component r's double in a slot
  return r == 0 ? K - 1 : r - 1;
}

// WIDE: more than 4 waves (two share a SIMD: 256 registers per lane); up to 4 waves a lane
// has the SIMD's 512 (VGPRs + AGPRs), which the reflective pair at 8 cells per lane needs
// (256 VGPRs + 376 B of scratch under the 8-wave bound).
template <int S, int C, bool PAIR, bool PAD, bool WIDE>
__global__ __launch_bounds__(64 * (WIDE ? kWaveMaxWaves : 4)) void chain_kernel(SegArgs a, int nsteps, int Lw) {
  constexpr int K = SchemeDim<S>::K, WN = map_count<S>();
  static_assert(K <= kChainSlot - 1, "a slot holds the carried state");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int nw = static_cast<int>(blockDim.x >> 6);
  const int g = w * 64 + lane;  // chain lane
  const int nl = a.H * a.Gl;
  int half, ell, j;
  if (PAIR) {
    ell = blockIdx.x;
    half = g < Lw ? 0 : 1;
    j = g - half * Lw;
  } else {
    half = static_cast<int>(blockIdx.x) / nl;
    ell = static_cast<int>(blockIdx.x) % nl;
    j = g;
  }
  const int used = PAIR ? 2 * Lw : Lw;
  const bool real = g < used;
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
  const bool refl_head = PAIR && half == 1 && j == 0;
  constexpr bool REDO = head_redo<S, C, WIDE>();
  double W[WN], W0[WN], Wh[WN];
  head_maps<S, C, PAIR, REDO>(a, half, ell, stride, refl_head, W, W0, Wh);  // VGPR-resident maps
  double Xin[K], X[K];
  {
    const double bv = a.bdry[static_cast<size_t>(PAIR ? 0 : half) * stride + ell];
    const double b[4] = {bv, bv, bv, bv};
    head_state<S>(b, Xin);
#pragma unroll
    for (int r = 0; r < K; ++r) X[r] = Xin[r];
  }
  // ring: [nw][kChainRing][kChainSlot] doubles, 16-byte aligned; region 0 the head's state
  extern __shared__ double2 ring2[];
  double *ring = reinterpret_cast<double *>(ring2);
  {
    const int n = nw * kChainRing * kChainSlot;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int p = i % kChainSlot;
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < K; ++r)
        if (p == slot_pos<K>(r)) v = Xin[r];
      ring[i] = i < kChainRing * kChainSlot ? v : 0.0;
    }
  }
  __syncthreads();
  double *const rd_region = ring + static_cast<size_t>(w) * kChainRing * kChainSlot;
  double *const wr_region = ring + static_cast<size_t>(w + 1) * kChainRing * kChainSlot;  // unused by the last wave
  const bool writer = lane == 63 && w < nw - 1;
  constexpr int RM = kChainRing - 1;

  // one tick's cells: X (received state, the shifts done) through the lane's C cells
  const auto cells = [&](bool active) {
    if (PAIR && refl_head) {
      if constexpr (S == SCHEME_BDF2) X[0] = X[2];
      if constexpr (S == SCHEME_CN) X[0] = X[1];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      double Xn[K], oi, oo;
      lane_cell<S, C, PAIR, REDO>(c, refl_head, W, W0, Wh, X, ein[c], eout[c], Xn, oi, oo);
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
  const auto read_slot = [&](const double *sl, double (&o)[K], bool all) {
    if constexpr (K == 5) {
      const double2 p0 = *reinterpret_cast<const double2 *>(sl), p1 = *reinterpret_cast<const double2 *>(sl + 2);
      o[1] = p0.x;
      o[2] = p0.y;
      o[3] = p1.x;
      o[4] = p1.y;
      if (all) o[0] = sl[4];
    } else {
#pragma unroll
      for (int r = 0; r < K; ++r)
        if (all || r > 0) o[r] = sl[slot_pos<K>(r)];
    }
  };
  const auto write_slot = [&](double *sl, const double (&x)[K], bool all) {
    if constexpr (K == 5) {
      *reinterpret_cast<double2 *>(sl) = make_double2(x[1], x[2]);
      *reinterpret_cast<double2 *>(sl + 2) = make_double2(x[3], x[4]);
      if (all) sl[4] = x[0];
    } else {
#pragma unroll
      for (int r = 0; r < K; ++r)
        if (all || r > 0) sl[slot_pos<K>(r)] = x[r];
    }
  };

  const int wsk = w * kChainSkew;
  const int ticks = nsteps + used - 1;
  const int nblocks = (ticks + (nw - 1) * kChainSkew + kChainBlock - 1) / kChainBlock;  // every wave: same barriers
  // this wave's unmasked chain ticks: its real lanes all at a level in [1, nsteps)
  const int u_lo = min(64 * w + 63, used - 1) + 1, u_hi = max(u_lo, nsteps + 64 * w);
  double nx[K];  // the ring values lane 0 receives at the next tick
#pragma unroll
  for (int r = 0; r < K; ++r) nx[r] = 0.0;
  read_slot(rd_region, nx, true);  // chain tick 0 (slot 0)
  for (int b = 0; b < nblocks; ++b) {
    const int t0 = b * kChainBlock - wsk;  // chain tick of the block's first wall tick (= 0 mod the block)
    if (K > 1 && t0 >= u_lo && t0 + kChainBlock <= u_hi) {
      // unmasked block: ring offsets fixed relative to the block's slot base
      const int base = t0 & RM, nbase = (t0 + kChainBlock) & RM;
      const double *rb = rd_region + base * kChainSlot, *rn = rd_region + nbase * kChainSlot;
      double *wb = wr_region + base * kChainSlot, *wn = wr_region + nbase * kChainSlot;
      double prev[K];
#pragma unroll
      for (int i = 0; i < kChainBlock; ++i) {
        // ticks are not interleaved: at 8 cells per lane an 8-tick block would not fit
        // the registers
        if (C >= 4) __builtin_amdgcn_sched_barrier(0);
        const double x0 = Xin[K - 1];
        Xin[K - 1] = lane_shift_up(nx[K - 1], X[K - 1]);
#pragma unroll
        for (int r = 1; r < K - 1; ++r) Xin[r] = lane_shift_up(nx[r], X[r]);
        Xin[0] = x0;
        // the ring traffic of this tick goes out before its FMAs: the stores of the exit
        // states computed so far in the block (the previous tick's, or the previous two in
        // one branch below 4 cells per lane), then the read of slot t + 1.  The next tick's
        // lgkmcnt wait then finds them complete; issued at the end of the tick (the
        // compiler's placement otherwise) every tick began by waiting out their latency.
        if constexpr (C >= 4) {
          if (i > 0 && writer) write_slot(wb + i * kChainSlot, X, false);
        } else if (i > 0 && !(i & 1)) {
          if (writer) {
            write_slot(wb + (i - 1) * kChainSlot, prev, false);
            write_slot(wb + i * kChainSlot, X, false);
          }
        } else if (i & 1) {
#pragma unroll
          for (int r = 0; r < K; ++r) prev[r] = X[r];
        }
        read_slot(i + 1 < kChainBlock ? rb + (i + 1) * kChainSlot : rn, nx, false);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < K; ++r) X[r] = Xin[r];
        cells(true);
        if (i == kChainBlock - 1 && writer) {  // the block's last exit state(s), before the barrier
          if constexpr (C < 4) write_slot(wb + i * kChainSlot, prev, false);
          write_slot(wn, X, false);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < kChainBlock; ++i) {
        const int t = t0 + i;
        if (t < 0 || t >= ticks) continue;  // wall ticks before or after this wave's chain
        // lane 0's component 0: the ring's only where lane 0 is at level 0 or idle -- at a
        // level >= 1 it is the component K - 1 lane 0 received one tick earlier (the unmasked
        // stretch's rule), since the writer's unmasked ticks store components 1..K-1 only
        const double old0 = (K > 1 && t - 64 * w >= 1) ? Xin[K - 1] : nx[0];
        Xin[0] = lane_shift_up(old0, X[0]);
#pragma unroll
        for (int r = 1; r < K; ++r) Xin[r] = lane_shift_up(nx[r], X[r]);
        read_slot(rd_region + ((t + 1) & RM) * kChainSlot, nx, true);
        const int lv = t - g;
#pragma unroll
        for (int r = 0; r < K; ++r) X[r] = Xin[r];
        cells(real && lv >= 0 && lv < nsteps);
        if (writer) write_slot(wr_region + ((t + 1) & RM) * kChainSlot, X, true);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int k = j * C + c;
    if (real && k < a.N) Eh[static_cast<size_t>(k) * stride] = make_double2(ein[c], eout[c]);
  }
}

template <int S, bool PAIR>
static hipError_t launch_wave_s(const WavePlan &p, const SegArgs &a, int nsteps, int grid, hipStream_t st) {
  const bool pad = PAIR && a.N % p.C != 0;
  const int Lw = p.lanes;
  if (p.waves > 1) {
    const size_t lds = sizeof(double) * kChainSlot * kChainRing * static_cast<size_t>(p.waves);
    switch (p.C) {
#define RT_CHAIN_LAUNCH(c, pd, wide)                                                                             \
  hipLaunchKernelGGL((chain_kernel<S, c, PAIR, pd, wide>), dim3(grid), dim3(64 * p.waves), lds, st, a, nsteps, Lw)
#define RT_CHAIN_CASE(c)                                                                                         \
  case c:                                                                                                        \
    if (pad && p.waves > 4)                                                                                      \
      RT_CHAIN_LAUNCH(c, PAIR && (c > 1), true);                                                                 \
    else if (pad)                                                                                                \
      RT_CHAIN_LAUNCH(c, PAIR && (c > 1), false);                                                                \
    else if (p.waves > 4)                                                                                        \
      RT_CHAIN_LAUNCH(c, false, true);                                                                           \
    else                                                                                                         \
      RT_CHAIN_LAUNCH(c, false, false);                                                                          \
    break;
      RT_CHAIN_CASE(1) RT_CHAIN_CASE(2) RT_CHAIN_CASE(4) RT_CHAIN_CASE(8)
#undef RT_CHAIN_CASE
#undef RT_CHAIN_LAUNCH
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (p.C) {
#define RT_WAVE_CASE(c)                                                                                          \
  case c:                                                                                                        \
    if (pad)                                                                                                     \
      hipLaunchKernelGGL((wavefront_kernel<S, c, PAIR, PAIR && (c > 1)>), dim3(grid), dim3(64), 0, st, a, nsteps, \
                         Lw);                                                                                    \
    else                                                                                                         \
      hipLaunchKernelGGL((wavefront_kernel<S, c, PAIR, false>), dim3(grid), dim3(64), 0, st, a, nsteps, Lw);      \
    break;
    RT_WAVE_CASE(1) RT_WAVE_CASE(2) RT_WAVE_CASE(4) RT_WAVE_CASE(8)
#undef RT_WAVE_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Which (cells per lane C, waves) a chain takes: the least estimated time of a 1000-step
// advance, (1000 + L - 1) ticks x the measured cost of one tick at (C, waves), L the chain's
// lanes.  Tick costs (ns, medians) from tools/chain_plan.py on chain_kernel / wavefront_kernel
// (round 5, profiles/r05d_chain_plan.jsonl: 1000 BDF2 steps, 8 lines, every feasible C at
// N = 16 .. 2048, vacuum and reflective; * = interpolated, no length measured there; the
// reflective rows re-measured after the head cell took its own map, r05p_chain_plan_refl.jsonl:
// N = 32 .. 2048 in steps filling each wave count).  A
// reflective pair whose N is not a multiple of C runs the padded kernel (the mu < 0 line's
// padding cells pass the state through by a select): ~1.3x the tick (C = 4: 430 vs 346 ns at
// one wave).  A chain's tick is ~2x a single wave's at the same C (the hand-over through LDS
// and the per-block barrier), and beyond 4 waves two share a SIMD, so round 3's rule -- one
// wave up to 4 cells per lane -- lost to 3 waves at C = 1 by 18% at 129 cells, and by 35% on
// a reflective 65-cell pair.
static const float kTickVacuum[4][kWaveMaxWaves] = {
    {79, 141, 166, 185, 225, 248, 259, 272},     // C = 1
    {126, 194, 217, 238, 306, 343, 356, 368},    // C = 2 (7 waves *)
    {220, 300, 323, 341, 441, 541, 560, 579},    // C = 4 (5, 7 waves *)
    {410, 500, 532, 555, 800, 880, 910, 943}};   // C = 8 (5-8 waves *: only C = 8 fits there)
static const float kTickReflective[4][kWaveMaxWaves] = {  // N a multiple of C
    {83, 156, 173, 191, 230, 255, 266, 278},     // C = 1 (round 5 before the head map: 201 .. 354)
    {131, 203, 222, 244, 321, 349, 363, 388},    // C = 2
    {227, 307, 330, 351, 515, 551, 570, 587},    // C = 4
    {421, 529, 559, 579, 927, 977, 1001, 1046}};  // C = 8 (5-8 waves: the head's redo, r05t_chain_plan_c8)
constexpr double kTickPadded = 1.3;
WavePlan wavefront_plan(int N, bool reflective, int max_waves) {
  max_waves = max_waves < 1 ? 1 : (max_waves > kWaveMaxWaves ? kWaveMaxWaves : max_waves);
  if (N < 1) return WavePlan{0, 0, 0};
  WavePlan best{0, 0, 0};
  double best_cost = 0.0;
  for (int ci = 0; ci < 4; ++ci) {
    const int C = 1 << ci, Lw = (N + C - 1) / C;
    const int used = reflective ? 2 * Lw : Lw, waves = (used + 63) / 64;
    if (waves > max_waves) continue;
    double cost = (1000.0 + used - 1) * (reflective ? kTickReflective : kTickVacuum)[ci][waves - 1];
    if (reflective && N % C) cost *= kTickPadded;
    if (!best.C || cost < best_cost) {
      best = WavePlan{C, waves, Lw};
      best_cost = cost;
    }
  }
  return best;  // C = 0: too long for max_waves waves (the segment pipeline)
}

hipError_t launch_wavefront(int scheme, const WavePlan &p, const SegArgs &a, int nsteps, hipStream_t st) {
  const bool pair = a.reflective != 0;
  const int nl = a.H * a.Gl;
  if (p.C == 0 || p.waves < 1 || p.waves > kWaveMaxWaves || nl <= 0 || nsteps < 0) return hipErrorInvalidValue;
  // the chain must fit the plan's waves: checked here, since the kernel indexes by it
  const int used = pair ? 2 * p.lanes : p.lanes;
  if (p.lanes * p.C < a.N || used > 64 * p.waves || used <= 64 * (p.waves - 1)) return hipErrorInvalidValue;
  if (nsteps == 0) return hipSuccess;
  const int grid = pair ? nl : 2 * nl;
  switch (scheme) {
    case SCHEME_BE:
      return pair ? launch_wave_s<SCHEME_BE, true>(p, a, nsteps, grid, st)
                  : launch_wave_s<SCHEME_BE, false>(p, a, nsteps, grid, st);
    case SCHEME_CN:
      return pair ? launch_wave_s<SCHEME_CN, true>(p, a, nsteps, grid, st)
                  : launch_wave_s<SCHEME_CN, false>(p, a, nsteps, grid, st);
    default:
      return pair ? launch_wave_s<SCHEME_BDF2, true>(p, a, nsteps, grid, st)
                  : launch_wave_s<SCHEME_BDF2, false>(p, a, nsteps, grid, st);
  }
}

}  // namespace rtamd
