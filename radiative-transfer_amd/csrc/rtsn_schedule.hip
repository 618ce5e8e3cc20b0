// rtsn_schedule.hip -- stepping: aligned passes with the cross-segment correction, the
// pipelined segment schedule, the short-line wavefront, rt_advance / rt_finish / rt_solve
// and the run planner (rt_plan_schedule).

#include "rtsn_internal.hpp"

using namespace rtamd;
using namespace rtsn_detail;

// ---------------------------------------------------------------------------
// stepping
// ---------------------------------------------------------------------------
rt_status rtsn_detail::check_validation(rt_solver *s) {
  if (s->p.include_validation && !phys::validate_correction(s->p, s->gt))
    return fail(s, RT_ERR_VALIDATION, "validate_correction() fails (correction.cpp:39-63,100-122)");
  return RT_OK;
}

rt_status rtsn_detail::ensure_equilibrium(rt_solver *s) {
  if (!s->p.use_mg_equilib || s->equilibrium_done) return RT_OK;
  rt_status st = check_validation(s);  // solver.cpp:290-293
  if (st) return st;
  phys::solver_psi_source(s->p, s->gt, s->mu.data(), s->psi_source);
  s->equilibrium_done = true;
  return upload_inflow(s);
}

// Sum the elapsed time of the recorded (start, stop) event pairs.
rt_status rtsn_detail::fold_events(rt_solver *s) {
  for (size_t k = 0; k + 1 < s->ev_used; k += 2) {
    HIP_TRY(s, hipEventSynchronize(s->ev_pool[k + 1]));
    float ms = 0.f;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev_pool[k], s->ev_pool[k + 1]));
    s->sweep_ms += ms;
  }
  s->ev_used = 0;
  return RT_OK;
}

SegArgs rtsn_detail::seg_args(rt_solver *s) {
  SegArgs a{};
  a.E = static_cast<double2 *>(s->E.p);
  a.map = static_cast<const double *>(s->map.p);
  a.hmap = static_cast<const double *>(s->hmap.p);
  a.bdry = static_cast<const double *>(s->bdry.p);
  a.yseg = static_cast<const double *>(s->yseg.p);
  a.yrefl = static_cast<const double *>(s->yrefl.p);
  a.agg_cur = static_cast<double *>(s->agg[s->agg_cur].p);
  a.N = s->p.N;
  a.Nrow = s->J * kSweepTile;
  a.Lpad = s->Lpad;
  a.Q = s->Q;
  a.Sg = s->Sg;
  a.Ls = s->Ls;
  a.half0 = 0;
  a.reflective = s->p.bc_left_indicator == 2;
  a.pending = s->pending ? 1 : 0;
  a.hd = 0.5 * (s->p.X / s->p.N);
  a.level_waves = level_waves_of(s, s->T);
  return a;
}

// Fold segment aggregates of a T-step pass into true incoming states:
// previous pass (agg_prev) -> yseg for the pending correction, or this pass's
// mu < 0 half (agg_cur) -> yrefl for the reflective mu > 0 heads.
rt_status rtsn_detail::enqueue_fold(rt_solver *s, int T, bool reflective_outflow) {
  if (rt_status st = ensure_segments(s)) return st;
  if (rt_status st = ensure_propagators(s, T)) return st;
  FoldArgs f{};
  const int slot = reflective_outflow ? s->agg_cur : (s->agg_cur ^ 1);
  f.agg = static_cast<const double *>(s->agg[slot].p);
  f.prop = static_cast<const double *>(s->prop[T].p);
  f.y = static_cast<double *>(reflective_outflow ? s->yrefl.p : s->yseg.p);
  f.prop_half = prop_count(s->K, T);
  f.Sg = s->Sg;
  f.Lpad = s->Lpad;
  f.half0 = 0;
  f.nhalf = reflective_outflow ? 1 : 2;
  f.last_short = (s->p.N - (s->Sg - 1) * s->Ls) != s->Ls;
  f.only_last = reflective_outflow ? 1 : 0;
  HIP_TRY(s, launch_fold(T * s->K, f, s->stream));
  return RT_OK;
}

// Apply the outstanding cross-segment correction in place (before any read,
// or before a pass with a different time block).
rt_status rtsn_detail::apply_correction(rt_solver *s) {
  if (!s->pending) return RT_OK;
  rt_status st = enqueue_fold(s, s->Tp, false);
  if (st) return st;
  SegArgs a = seg_args(s);
  HIP_TRY(s, launch_sweep(s->scheme, s->Tp, SWEEP_FINALIZE, a, 2 * s->Q * s->Sg, s->stream));
  ++s->state_version;
  s->pending = false;
  return RT_OK;
}

static rt_status event_begin(rt_solver *s, hipEvent_t *e1) {
  *e1 = nullptr;
  if (!s->profiling) return RT_OK;
  if (s->ev_used + 2 > s->ev_pool.size()) {
    rt_status st = fold_events(s);  // drain the pool when it is full
    if (st) return st;
  }
  hipEvent_t e0 = s->ev_pool[s->ev_used++];
  *e1 = s->ev_pool[s->ev_used++];
  HIP_TRY(s, hipEventRecord(e0, s->stream));
  return RT_OK;
}

// a launch that failed after event_begin: its pair is returned unused (e1 never recorded)
static void event_abort(rt_solver *s, hipEvent_t e1) {
  if (e1) s->ev_used -= 2;
}

static rt_status event_end(rt_solver *s, hipEvent_t e1) {
  if (e1) {
    HIP_TRY(s, hipEventRecord(e1, s->stream));
    ++s->profiled;
  }
  ++s->launches;
  return RT_OK;
}

// One pass of T full steps, every segment at the same time level.
// coupled: the material-coupled sweep (T = 1, per-cell emission).
rt_status rtsn_detail::enqueue_pass(rt_solver *s, int T, bool coupled) {
  if (rt_status st = ensure_segments(s)) return st;
  if (s->pending && s->Tp != T) {
    rt_status st = apply_correction(s);
    if (st) return st;
  }
  const int per_half = s->Q * s->Sg;
  SegArgs a = seg_args(s);
  if (coupled) {
    a.map = static_cast<const double *>(s->map_unit.p);
    a.hmap = static_cast<const double *>(s->hmap_unit.p);
    a.bcell = static_cast<const double *>(s->Beff.p);  // the step's linearised emission
    a.Gl = s->Gl;
    a.H = s->H;
    a.phi = s->phi_fused ? static_cast<double *>(s->phi_part.p) : nullptr;
    a.wt = static_cast<const double *>(s->muwt.p) + s->p.M;
  }
  hipEvent_t e1;
  rt_status st = event_begin(s, &e1);
  if (st) return st;
  if (s->pending && (st = enqueue_fold(s, T, false))) return st;
  if (a.reflective) {  // mu > 0 heads need this pass's mu < 0 outflow: two launches
    a.half0 = 0;
    HIP_TRY(s, launch_sweep(s->scheme, T, SWEEP_PASS, a, per_half, s->stream));
    if ((st = enqueue_fold(s, T, true))) return st;
    a.half0 = 1;
    HIP_TRY(s, launch_sweep(s->scheme, T, SWEEP_PASS, a, per_half, s->stream));
  } else {
    HIP_TRY(s, launch_sweep(s->scheme, T, SWEEP_PASS, a, 2 * per_half, s->stream));
  }
  if ((st = event_end(s, e1))) return st;
  ++s->state_version;
  s->pending = s->Sg > 1;
  s->Tp = T;
  s->agg_cur ^= 1;
  for (long long &t : s->tau) t += T;
  s->target += T;
  return RT_OK;
}

// nsteps full steps in aligned passes of at most T (and kMaxAlignedBlock) steps.
static rt_status enqueue_steps(rt_solver *s, int nsteps) {
  if (rt_status st = resegment(s, true)) return st;
  const int T = std::min(s->T, kMaxAlignedBlock);
  while (nsteps > 0) {
    const int n = std::min(T, nsteps);
    rt_status st = enqueue_pass(s, n);
    if (st) return st;
    nsteps -= n;
  }
  return RT_OK;
}

// ---------------------------------------------------------------------------
// Pipelined schedule.  Chain position c (segment s of half 0, or of half 1:
// c = s for both halves, or c = Sg + s when the mu > 0 heads take the mu < 0
// outflow) runs one pass behind position c-1: in every launch each position
// that can advance T steps does, starting from the exit state position c-1
// published in the previous launch for exactly those steps.  Every segment
// starts exact, so no provisional state and no correction.  The first
// launches fill the pipeline (position c starts in launch c), the last ones
// drain it; both happen once per run of advances, and the drain only when a
// read-out needs the state (finalize).
// ---------------------------------------------------------------------------
//
// The run's n mod T last steps (complete: the queued remainder) can ride the drain as a
// final block of `tail` < T steps per position (launch_split_tail: vacuum lines, BDF2 split
// blocks): position c runs it once position c - 1 has, in the launch where position c + 1
// runs its last whole block -- one launch more than the drain, instead of aligned passes
// with the cross-segment correction after it.
// Positions per launch of the fill and drain ramps (round 5).  A ramp launch of k < P
// positions takes four waves per segment (fill_level_waves), and at two 4-wave workgroups per
// CU the chip holds the workgroups of m = resident / (workgroups per position) positions:
// beyond m (the SL slab's T = 20 pipeline: m = 4 of 8 positions) the rest ran as a second
// round on half the SIMDs (k = 5 / 6: 149 / 151 ms against shares of 104 / 125 ms,
// profiles/archive/r04ag_trace_summary.json).  Positions of one launch never exchange data (each
// reads what its predecessor published in the previous launch), so such a launch is cut into
// consecutive launches of at most m positions, each with its own waves per segment.  The
// full launch (k = P), a caller-set level split and other schemes keep one launch.
static int ramp_chunk(const rt_solver *s, int k, int grid_per_pos) {
  const int T = s->Tpipe, P = chain_positions(s);
  if (k >= P || s->level_waves || s->scheme != SCHEME_BDF2 || !split_block(T) || T % 4) return k;
  int wpc = 0;
  if (split_occupancy(T, 4, &wpc) != hipSuccess || wpc < 1) return k;
  const long long m = static_cast<long long>(wpc) * s->cus / grid_per_pos;
  return m >= 1 && m < k ? static_cast<int>(m) : k;
}

// One pipelined launch: every position that can advance a block does.  A launch cut into
// sub-launches (ramp_chunk) commits each sub-launch's positions (tau, state_version) as soon as
// it is in the stream, and until the whole launch is, the handle remembers the positions still
// owed (resume_lo..resume_hi): a call after a failed sub-launch (a non-sticky launch error, or
// the profiling pool's event wait) runs exactly those, never a position twice.
static rt_status pipe_launch(rt_solver *s) {
  if (rt_status st = ensure_segments(s)) return st;
  const int P = chain_positions(s), T = s->Tpipe;
  const long long end = s->target + s->tail;
  auto block = [&](int c) { return s->tau[c] < s->target ? T : s->tail; };
  auto ready = [&](int c) { return s->tau[c] < end && (c == 0 || s->tau[c - 1] >= s->tau[c] + block(c)); };
  int lo = -1, hi = -1;
  if (s->resume_lo >= 0) {  // the rest of an interrupted launch
    lo = s->resume_lo;
    hi = s->resume_hi;
    if (hi >= P || lo > hi) return fail(s, RT_ERR_STATE, "pipeline: interrupted launch out of range");
    for (int c = lo; c <= hi; ++c)
      if (!ready(c)) return fail(s, RT_ERR_STATE, "pipeline: interrupted launch no longer ready");
  } else {
    for (int c = 0; c < P; ++c) {
      if (!ready(c)) continue;
      if (lo < 0) lo = c;
      if (hi >= 0 && hi != c - 1) return fail(s, RT_ERR_PARAM, "pipeline: active positions not contiguous");
      hi = c;
    }
  }
  if (lo < 0) return fail(s, RT_ERR_PARAM, "pipeline: no position can advance");  // loops below rely on progress
  for (int c = lo; c <= hi; ++c)
    if (s->tau[c] != s->tau[lo] - static_cast<long long>(c - lo) * T || (c > lo && block(c) != T))
      return fail(s, RT_ERR_PARAM, "pipeline: positions out of step");
  const int per_pos = (s->p.bc_left_indicator == 2 ? 1 : 2) * s->Q;  // workgroups per position
  const int m = ramp_chunk(s, hi - lo + 1, per_pos);
  for (int c0 = lo; c0 <= hi; c0 += m) {
    const int c1 = std::min(hi, c0 + m - 1);
    s->resume_lo = c0;  // owed until this sub-launch is in the stream
    s->resume_hi = hi;
    SegArgs a = seg_args(s);
    a.aggs[0] = static_cast<double *>(s->agg[0].p);
    a.aggs[1] = static_cast<double *>(s->agg[1].p);
    a.pending = 0;
    a.pos_lo = c0;
    a.npos = c1 - c0 + 1;
    a.pass_lo = static_cast<int>(((s->tau[c0] - s->pipe_base) / T) & 1);
    const int grid = a.npos * per_pos;
    a.level_waves = fill_level_waves(s, grid);
    a.tail_levels = block(c0) == T ? 0 : s->tail;  // only the first position can run the tail
    hipEvent_t e1;
    rt_status st = event_begin(s, &e1);
    if (st) return st;
    hipError_t e = hipSuccess;
    if (s->fail_launch_after == 0) {  // test hook (rt_debug_fail_launch): this launch fails, nothing runs
      s->fail_launch_after = -1;
      e = hipErrorLaunchFailure;
    } else {
      if (s->fail_launch_after > 0) --s->fail_launch_after;
      if (a.tail_levels) {
        a.level_waves = tail_waves(s, T);  // (complete: wave 0 runs whole levels)
        e = launch_split_tail(T, a.level_waves, a, grid, s->stream);
      } else {
        e = launch_sweep(s->scheme, T, SWEEP_PIPELINED, a, grid, s->stream);
      }
    }
    if (e != hipSuccess) {
      event_abort(s, e1);
      return fail(s, RT_ERR_DEVICE, std::string("pipelined launch: ") + hipGetErrorString(e));
    }
    for (int c = c0; c <= c1; ++c) s->tau[c] += block(c);
    ++s->state_version;
    s->resume_lo = c1 < hi ? c1 + 1 : -1;
    s->resume_hi = c1 < hi ? hi : -1;
    if ((st = event_end(s, e1))) return st;
  }
  return RT_OK;
}

// rt_set_pipeline(1): the fewest whole passes an advance must bring for the pipelined
// schedule.  A pipelined run of n passes over P chain positions takes P + n - 1 launches;
// with the fill/drain launches split over 4 waves (fill_level_waves: BDF2 blocks with a
// split kernel) a launch of at most P/4 positions costs a quarter of a pass, so from
// n >= P/8 passes the run beats aligned passes (at most 4 steps each, the correction doubling
// the FP64 work: 20.0 vs 8.3 ms per step on SL).  Without the split, n >= P.
static int auto_pipeline_passes(const rt_solver *s) {
  const int P = chain_positions(s);
  if (s->planned) return 1;  // the planned schedule's model is the pipelined run
  if (s->scheme == SCHEME_BDF2 && !s->level_waves && split_block(s->T)) return std::max(1, (P + 7) / 8);
  return P;
}

static bool plan_allowed(const rt_solver *s);
static bool plan_for_advance(rt_solver *s);

// Queue nsteps; launch whole passes while the chain head is behind.  A run not yet
// pipelined starts its pipeline only once it has queued enough passes for one
// (auto_pipeline_passes; for an unplanned BDF2 run, once rt_solve's plan for the .prm's run
// length would pipeline them: plan_for_advance); until then the steps stay queued, and a
// read-out (finalize) runs them as aligned passes.  So a run advanced in chunks pipelines
// through its chunks -- the same launches as one rt_solve -- while a short advance followed
// by a read-out costs aligned passes, not a pipeline fill and drain.
static rt_status pipe_advance(rt_solver *s, int nsteps) {
  s->queued += nsteps;
  rt_status st;
  if (s->Tpipe && s->Tpipe != s->T) {  // a lagged pipeline of another block size: let it drain
    while (s->tau.back() < s->target)
      if ((st = pipe_launch(s))) return st;
    s->Tpipe = 0;
  }
  if (!s->Tpipe) {
    if (s->pipe == 1) {  // auto: deferred until enough passes are queued for a pipeline
      if (plan_allowed(s)) {
        if (!plan_for_advance(s)) return RT_OK;
      } else if (s->queued / s->T < auto_pipeline_passes(s)) {
        return RT_OK;
      }
    }
    if (s->queued / s->T == 0) return RT_OK;
    // start from aligned positions with an exact state, segments sized for this T
    if ((st = apply_correction(s))) return st;
    if ((st = resegment(s))) return st;
    s->Tpipe = s->T;
    s->pipe_base = s->tau[0];
  }
  const int T = s->T;
  const long long passes = s->queued / T;
  if (passes == 0) return RT_OK;
  s->queued -= static_cast<int>(passes * T);
  s->target += passes * T;
  while (s->tau[0] < s->target)
    if ((st = pipe_launch(s))) return st;
  return RT_OK;
}

// Bring every position to the target (drain) and run the queued remainder.  A planned
// schedule ends with its run's pipeline.
rt_status rtsn_detail::complete(rt_solver *s) {
  rt_status st;
  if (s->wqueued && (st = wave_flush(s))) return st;
  if (s->Tpipe) {
    const int kw = tail_waves(s, s->Tpipe);
    // the remainder as every position's last block; a tail already set is a drain a failed
    // launch interrupted, which a later call resumes (rt_pipeline_state counts it as queued)
    if (!s->tail && s->queued && kw && s->queued >= s->Tpipe / kw) {
      s->tail = s->queued;
      s->queued = 0;
    }
    while (s->tau.back() < s->target + s->tail)
      if ((st = pipe_launch(s))) return st;
    s->target += s->tail;
    s->tail = 0;
    s->Tpipe = 0;
  }
  end_plan(s);
  if (s->queued) {
    const int r = s->queued;
    s->queued = 0;
    if ((st = enqueue_steps(s, r))) return st;
  }
  return RT_OK;
}

// The state at the requested time, exact: before any read-out.
rt_status rtsn_detail::finalize(rt_solver *s) {
  rt_status st = complete(s);
  if (st) return st;
  return apply_correction(s);
}

// Short lines (kernels_wave.hip): every step of an advance in one launch per chunk of
// steps, lanes over cells -- by default (rt_set_wavefront 1) when the line fits a
// workgroup's chain and the caller chose neither a time block nor a schedule, always with
// rt_set_wavefront 2.
WavePlan rtsn_detail::wave_plan(const rt_solver *s) {
  const bool refl = s->p.bc_left_indicator == 2;
  if (s->wave_cells) {  // the caller's cells per lane, where the chain then fits wave_max waves
    const int C = s->wave_cells, lanes = (s->p.N + C - 1) / C;
    const int waves = ((refl ? 2 * lanes : lanes) + 63) / 64;
    if (waves <= s->wave_max) return WavePlan{C, waves, lanes};
  }
  return wavefront_plan(s->p.N, refl, s->wave_max);
}

// Auto (mode 1) takes a chain of several waves while the chains need at most two waves per
// SIMD: mid-length lines run 4-7x faster as chains than as segment passes there (1000 BDF2
// steps, N = 600-4000 cells: 4 groups 0.46-1.5 ms vs 2.7-6.6 ms, 124 groups, i.e. 1984 waves,
// 0.67-1.7 ms vs 4.0-8.1 ms; profiles/archive/r03ai_mid.jsonl).  Beyond, the chains time-share the
// SIMDs, and the segment pipeline's full-chip passes (28 FMAs per cell and level at ~90% of
// the FP64 issue rate) carry the same work with less overhead per cell.
bool rtsn_detail::use_wavefront(const rt_solver *s) {
  if (s->material || s->wave == 0) return false;
  const WavePlan p = wave_plan(s);
  if (p.C == 0) return false;
  if (s->wave == 2) return true;
  if (s->T_set || s->pipe_set) return false;
  const long long chains = static_cast<long long>(s->H) * s->Gl * (s->p.bc_left_indicator == 2 ? 1 : 2);
  return p.waves == 1 || chains * p.waves <= 8LL * s->cus;
}

constexpr int kWaveMaxSteps = 1 << 16;  // steps per wavefront launch (bounds one launch's length)

// A wavefront launch of m steps runs m + L - 1 ticks (L lanes in the chain), so an advance
// of a few steps is mostly the chain's fill and drain: 7-step advances of a 4000-cell line
// (500 lanes) would cost 506 ticks for 7 steps' work.  The steps are queued instead and
// launched together once they hold 8 (L - 1) -- the fill and drain then at most 1/8 of the
// launch -- or when anything needs the state (complete: every read-out, rt_finish, the
// setters that align the schedule, a switch to the segment schedules).  The arithmetic per
// (cell, level) does not depend on how the steps are cut into launches: bitwise the same.
static long long wave_defer_steps(const rt_solver *s) {
  const WavePlan p = wave_plan(s);
  const long long used = s->p.bc_left_indicator == 2 ? 2LL * p.lanes : p.lanes;
  return std::max<long long>(1, 8 * (used - 1));
}

rt_status rtsn_detail::wave_flush(rt_solver *s) {
  SegArgs a = seg_args(s);
  a.Gl = s->Gl;
  a.H = s->H;
  while (s->wqueued > 0) {
    const int m = static_cast<int>(std::min<long long>(s->wqueued, kWaveMaxSteps));
    hipEvent_t e1;
    rt_status st = event_begin(s, &e1);
    if (st) return st;
    HIP_TRY(s, launch_wavefront(s->scheme, wave_plan(s), a, m, s->stream));
    if ((st = event_end(s, e1))) return st;
    ++s->state_version;
    for (long long &t : s->tau) t += m;
    s->target += m;
    s->wqueued -= m;
  }
  return RT_OK;
}

static rt_status wave_advance(rt_solver *s, int nsteps) {
  if (!s->wqueued)
    if (rt_status st = finalize(s)) return st;  // the stored state exact at the requested time
  s->wqueued += nsteps;
  return s->wqueued >= wave_defer_steps(s) ? wave_flush(s) : RT_OK;
}

extern "C" rt_status rt_advance(rt_solver *s, int nsteps) {
  if (!s || nsteps < 0) return fail(s, RT_ERR_ARG, "rt_advance: bad argument");
  if (s->material) return fail(s, RT_ERR_STATE, "material coupling is on: step with rt_material_step / rt_material_sweep");
  HIP_TRY(s, hipSetDevice(s->device));
  rt_status st = check_validation(s);
  if (st) return st;
  if ((st = ensure_equilibrium(s))) return st;
  if (use_wavefront(s)) return wave_advance(s, nsteps);
  if (s->wqueued && (st = wave_flush(s))) return st;  // the path changed: queued wavefront steps first
  return s->pipe ? pipe_advance(s, nsteps) : enqueue_steps(s, nsteps);
}

extern "C" rt_status rt_finish(rt_solver *s) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_finish: NULL handle");
  HIP_TRY(s, hipSetDevice(s->device));
  return finalize(s);
}

extern "C" rt_status rt_synchronize(rt_solver *s) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_synchronize: NULL handle");
  HIP_TRY(s, hipStreamSynchronize(s->stream));
  return RT_OK;
}

// rt_solve knows the run's length.  Unless the caller chose the schedule (time block, waves
// per segment, segmentation), a BDF2 run takes the pipelined schedule with the least
// estimated whole-run time (plan_schedule): time block T of 8-40 steps, four waves per
// segment (sweep_split_kernel<3, T, 4>, every launch of the run) and segments sized for w of
// 1-32 workgroups per CU (1 and 2 only when clearly ahead, plan_schedule).  The model
// (fitted to the finite-state whole-run grids
// profiles/archive/r03l_grid{16,128}.jsonl, mean error 3%, and refit in round 5 on few-group
// long lines, profiles/r05zf_* / r05zg_*, 4% over 120 forced runs): a run of n steps is P = n / T
// passes over a chain of C segment positions, launched as P + C - 1 launches whose active
// positions form a band (ramp up, plateau of min(P, C), ramp down); a launch of W workgroups
// runs in rounds of the resident 2 per CU, and a round's time is one segment's Ls x T / 4
// cell-levels per wave at the per-level cost of its block (t_T) times the workgroups the
// busiest CU holds (ceil(W / CUs): a wave per SIMD each), stretched by the workgroup's own
// wave pipeline fill over a short segment.  n mod T steps more ride the drain as
// every position's last block (one launch more, pipe_launch) when they are at least T / 4;
// else, on reflective chains and at T = 40 (whose tail kernel would spill) they run
// as aligned passes with the cross-segment correction (~3 steps' cost each, ~3 ms of folds
// and the finalize on the aligned segmentation).
struct RunGeom {
  long long N;
  int M, Gl, cus;
  bool reflective;
};

static double level_ns(int T) {  // per cell-level and wave, a SIMD's issue shared by its waves
  switch (T) {
    case 8: return 76.7;
    case 16: return 71.0;
    case 20: return 67.6;
    case 24: return 70.4;
    case 32: return 66.7;
    default: return 64.7;  // 40
  }
}

static void model_segments(const RunGeom &g, int w, long long *Sg, long long *Ls) {
  const long long Q = (static_cast<long long>(g.M / 2) * g.Gl + 63) / 64;
  long long sg = std::max<long long>(1, static_cast<long long>(g.cus) * w / (2 * Q));
  sg = std::min(sg, (g.N + kSweepCells - 1) / kSweepCells);
  long long ls = (g.N + sg - 1) / sg;
  ls = (ls + kSweepCells - 1) / kSweepCells * kSweepCells;
  *Ls = ls;
  *Sg = (g.N + ls - 1) / ls;
}

static double run_ms_model(const RunGeom &g, long long n, int T, int w) {
  constexpr int kw = 4, occ = 2;
  long long Sg, Ls;
  model_segments(g, w, &Sg, &Ls);
  const long long Q = (static_cast<long long>(g.M / 2) * g.Gl + 63) / 64;
  const long long C = g.reflective ? 2 * Sg : Sg, R = g.reflective ? Q : 2 * Q;
  const long long P = n / T, rem = n % T;
  if (P == 0) return 1e300;
  // a segment's cell-levels per wave, and the workgroup's own pipeline fill: wave w of kw
  // starts 2 w chunk intervals after wave 0 (kernels_split.hip), which short segments feel
  // (round 5, late: 48-cell segments ran ~2x the model without it, profiles/r05zf_*)
  const long long nch = (Ls + split_chunk_cells() - 1) / split_chunk_cells();
  const double fill = static_cast<double>(nch + 2 * (kw - 1)) / static_cast<double>(nch);
  const double tf = level_ns(T) * 1e-9, tl = 0.99 * tf, unit = static_cast<double>(Ls) * T / kw * fill;
  const long long S = static_cast<long long>(occ) * g.cus;
  auto launch = [&](long long a) {  // seconds
    const long long W = a * R, full = W / S, part = W % S;
    double t = full * unit * tf * occ;
    if (part) {
      const long long per_cu = (part + g.cus - 1) / g.cus;  // workgroups on the busiest CU
      t += unit * (per_cu <= 1 ? tl : tf * per_cu);
    }
    return t + 5e-6;  // + launch
  };
  // launch l holds the positions c with 0 <= l - c < P (whole blocks) and, with a remainder
  // riding the drain, the one at l - c == P (its tail block, counted as a whole position)
  const bool tail = rem >= T / kw && !g.reflective && split_tail_supported(T, kw);
  double s = 0.0;
  for (long long l = 0; l < P + C - 1 + (tail ? 1 : 0); ++l) {
    long long a = std::min(l + 1, C) - std::max<long long>(0, l - P + 1);
    if (tail && l >= P && l - P < C) ++a;
    s += launch(a);
  }
  if (rem && !tail) {
    const double step = static_cast<double>(R) * g.N * tf / (4.0 * g.cus);  // one step, every line, full load
    s += rem * 3.0 * step + 0.003;  // + the folds and the finalize (aligned segmentation, LDS fold)
  }
  return 1e3 * s;
}

struct Schedule {
  int T = 0, w = 0;
  double ms = 0.0;
};

constexpr double kPlanFewGuard = 0.97;  // 1-2 workgroups per CU must beat the best of 4-32 by this factor
static Schedule plan_schedule(const RunGeom &g, long long nsteps) {
  // T = 4 over four waves (no remainder for n % 4 == 0) measured slower than T = 8 with its
  // aligned remainder (16-group shard, 100 steps: 181 vs 167 ms, profiles/archive/r04d_solve_plan.jsonl)
  // Segments for 1 or 2 workgroups per CU (round 5, late) serve lines too few to fill the chip
  // at any segmentation (few groups, long lines: 4 groups x 5000 cells, 1000 steps, 4.6 ms at
  // one workgroup per CU against 7.3 at the old plan's four, profiles/r05zf_*); they are taken
  // only when the model puts them 3% ahead of the best of 4-32 (its error on these runs), so
  // that chip-filling runs (the SL slab: < 1% either way) keep the measured schedules.
  static const int kBlocks[] = {40, 32, 24, 20, 16, 8}, kWgs[] = {1, 2, 4, 8, 16, 32};
  Schedule best, few;
  for (int T : kBlocks)
    for (int w : kWgs) {
      const double ms = run_ms_model(g, nsteps, T, w);
      Schedule &b = w >= 4 ? best : few;
      if (ms < 1e300 && (!b.T || ms < b.ms)) b = {T, w, ms};
    }
  if (few.T && (!best.T || few.ms < kPlanFewGuard * best.ms)) return few;
  return best;
}

static RunGeom run_geom(const rt_solver *s) {
  return RunGeom{s->p.N, s->p.M, s->Gl, s->cus, s->p.bc_left_indicator == 2};
}

extern "C" rt_status rt_plan_time_block(int ts_method, long long nsteps, int *steps_per_pass) {
  if (!steps_per_pass || nsteps < 0 || ts_method < 1 || ts_method > 3)
    return fail(nullptr, RT_ERR_ARG, "rt_plan_time_block: bad argument");
  *steps_per_pass = default_time_block(ts_method);
  if (ts_method == SCHEME_BDF2) {  // the SL slab's geometry on one MI355X: N = 1e6, S64, 128 groups, 256 CUs
    const Schedule sc = plan_schedule(RunGeom{1000000, 64, 128, 256, false}, nsteps);
    if (sc.T) *steps_per_pass = sc.T;
  }
  return RT_OK;
}

extern "C" rt_status rt_plan_schedule(rt_solver *s, long long nsteps, int *steps_per_pass, int *level_waves,
                                      int *wgs_per_cu, double *estimated_ms) {
  if (!s || nsteps < 0) return fail(s, RT_ERR_ARG, "rt_plan_schedule: bad argument");
  Schedule sc;
  if (s->scheme == SCHEME_BDF2) sc = plan_schedule(run_geom(s), nsteps);
  if (steps_per_pass) *steps_per_pass = sc.T ? sc.T : s->T;
  if (level_waves) *level_waves = sc.T ? 4 : s->level_waves;
  if (wgs_per_cu) *wgs_per_cu = sc.T ? sc.w : s->seg_wgs;
  if (estimated_ms) *estimated_ms = sc.T ? sc.ms : 0.0;
  return RT_OK;
}

// The planned schedule for a run (time block, four waves per segment, segmentation),
// over the handle's own choices, which end_plan restores: the plan holds for one run's
// pipeline (rt_solve, or a run of advances) and a later run plans again.
static void begin_plan(rt_solver *s, const Schedule &sc) {
  s->plan_T0 = s->T;
  s->plan_lw0 = s->level_waves;
  s->plan_w0 = s->seg_wgs;
  s->T = sc.T;
  s->level_waves = 4;
  s->seg_wgs = sc.w;
  s->planned = true;
}

void rtsn_detail::end_plan(rt_solver *s) {
  if (!s->planned) return;
  s->T = s->plan_T0;
  s->level_waves = s->plan_lw0;
  s->seg_wgs = s->plan_w0;
  s->planned = false;
}

static bool plan_allowed(const rt_solver *s) {
  if (s->scheme != SCHEME_BDF2 || s->planned || s->Tpipe || use_wavefront(s)) return false;
  return !(s->T_set || s->lw_set || s->seg_set || s->pipe_set);  // the caller chose (part of) the schedule
}

static void solve_time_block(rt_solver *s) {
  if (s->queued || !plan_allowed(s)) return;
  const Schedule sc = plan_schedule(run_geom(s), s->p.max_timesteps);
  if (sc.T) begin_plan(s, sc);
}

// An unplanned BDF2 run of advances: rt_solve's plan for the .prm's run length (at least the
// steps queued), taken -- and its pipeline started -- once the queued steps hold 1/8 of the
// planned chain's depth in passes (the rule of auto_pipeline_passes, on the planned
// segments) or the whole run (max_timesteps, which rt_solve would pipeline with this plan).
// True when the plan is in place.
static bool plan_for_advance(rt_solver *s) {
  if (s->planned) return true;
  if (!plan_allowed(s)) return false;
  const RunGeom g = run_geom(s);
  const long long run = std::max<long long>(s->p.max_timesteps, s->queued);
  const Schedule sc = plan_schedule(g, run);
  if (!sc.T) return false;
  long long Sg = 0, Ls = 0;
  model_segments(g, sc.w, &Sg, &Ls);
  const long long depth = g.reflective ? 2 * Sg : Sg;
  const long long need = std::min(std::max<long long>(1, (depth + 7) / 8) * sc.T, std::max<long long>(sc.T, run / sc.T * sc.T));
  if (s->queued < need) return false;
  begin_plan(s, sc);
  return true;
}

// The planned schedule holds for this run only: afterwards the handle's time block, waves
// per segment and segmentation are the caller's (or the defaults) again, so a later
// rt_advance is scheduled as if rt_solve had not run (the segments are re-sized at its
// first pass).
extern "C" rt_status rt_solve(rt_solver *s) {
  if (!s) return fail(nullptr, RT_ERR_ARG, "rt_solve: NULL handle");
  solve_time_block(s);
  rt_status st = rt_advance(s, s->p.max_timesteps);
  if (!st) st = complete(s);
  end_plan(s);
  if (st) return st;
  return rt_synchronize(s);
}

extern "C" void *rt_stream(rt_solver *s) { return s ? static_cast<void *>(s->stream) : nullptr; }
