/*
 * rtsn.h -- C ABI of the MI355X-native S_n radiative-transfer solver
 * (librtsn.so).  Drop-in for the Solver / ParameterHandler surface of
 * Helblindi/radiative-transfer; plain pointers and sizes, no C++/torch types.
 *
 * The reference has no C ABI: its boundary is the C++ classes
 *   ParameterHandler(const string)                 include/ParameterHandler.h:67
 *   Solver(ParameterHandler&, Tensor3& psi, Ref<MatrixXd> phi, Ref<MatrixXd> F)
 *                                                  include/solver.h:79-83
 *   void solve()                                   include/solver.h:92
 *   compute_angle_integrated_intensity / compute_positive_angle_integrated_intensity /
 *   compute_radiative_flux / compute_balance       include/solver.h:85-88
 *   get_balance / get_phi_plus / get_e_ave / compute_group_ends / get_ends
 *                                                  include/solver.h:89-97
 * Each entry point below names the member it replaces.  Where the reference
 * asserts or exit(1)s, these functions return an rt_status instead.
 *
 * Array layouts are the reference's Eigen ColMajor layouts:
 *   psi  (M, G, N)    index i + M*(g + G*c)          main.cc:88
 *   ends (M, G, N, 2) index i + M*(g + G*(c + N*s))  solver.h:36
 *   phi / F / phi_plus (G, N) index g + G*c          main.cc:91-92, solver.h:31-33
 * where G is the number of groups held by the handle (all groups, or the
 * [g_lo, g_hi) shard given to rt_create_from_params).
 *
 * Threading: one handle per host thread; every call on a handle is ordered on
 * the handle's own HIP stream (rt_stream).  Host-buffer getters synchronise.
 */
#ifndef RTSN_H
#define RTSN_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  RT_OK = 0,
  RT_ERR_IO = 1,          /* a group table could not be opened (ParameterHandler.cpp:146-149 exit(1)) */
  RT_ERR_PARSE = 2,       /* std::stoi / std::stod would throw (param.cpp:30,44) */
  RT_ERR_PARAM = 3,       /* invalid configuration (odd M -> mu = 0 assert solver.cpp:402, bad BC :660, ...) */
  RT_ERR_VALIDATION = 4,  /* assert(validate_correction()) would fire (solver.cpp:609-612) */
  RT_ERR_NOMEM = 5,       /* host or device allocation failed */
  RT_ERR_DEVICE = 6,      /* HIP runtime error / no usable gfx950 device */
  RT_ERR_TIMEOUT = 7,     /* an rt_comm wait passed RTSN_COMM_TIMEOUT_S: the communicator was aborted */
  RT_ERR_ARG = 8,         /* NULL handle / bad argument */
  RT_ERR_STATE = 9,       /* call not valid in the handle's mode (e.g. rt_advance with material coupling on) */
  RT_WARN_UNSTABLE = 10   /* not returned since round 6 (the coupling's T update is implicit in its emission);
                             kept so that the values of the codes do not change */
} rt_status;

/* Every .prm key (ParameterHandler.cpp:100-212) with the reference's meaning.
 * Pointer members are borrowed (caller-owned) and may be NULL. */
typedef struct {
  int M;                         /* angle quadrature order (even) */
  int G;                         /* energy groups */
  int N;                         /* cells */
  double efirst, elast;          /* log group grid (solver.cpp:6-19) when no bounds table */
  double X;                      /* slab thickness; dx = X / N */
  int bc_left_indicator;         /* 0 vacuum (falls through to source, solver.cpp:668), 1 source, 2 reflective */
  int bc_right_indicator;        /* 0 vacuum, 1 source, 2 reflective (= vacuum in the reference) */
  int use_mg_equilib;            /* psi_source from computeEquilibriumSources (solver.cpp:287-315) */
  double rho, kappa_grey, T, V;
  int use_correction;
  int ts_method;                 /* 1 BE, 2 CN, 3 BDF2 (4 substeps per step) */
  double dt;
  int max_timesteps;
  int include_validation;
  const double *psi_source;      /* M*G, element (m, g) at m*G + g (ParameterHandler.cpp:126-132); NULL = zeros */
  const double *group_bounds;    /* G+1 edges (have_group_bounds) or NULL */
  const double *group_kappa;     /* G opacities (have_group_absorption_opacities) or NULL */
} rt_params;

typedef struct rt_solver rt_solver;

/* ---- host-only configuration (no device calls) ------------------------- */

/* ParameterHandler(filename) (ParameterHandler.cpp:12-17, 100-212): parses the
 * .prm with the kaityo256/param semantics.  Tables are read from
 * table_dir + name; table_dir NULL means the reference's "../prm/" relative
 * to the working directory.  A missing .prm yields the defaults (as in the
 * reference) and *prm_found = 0.  The returned arrays are owned by the
 * library: release with rt_params_free. */
rt_status rt_params_load(const char *prm_path, const char *table_dir, rt_params *out, int *prm_found);
void rt_params_free(rt_params *p);
void rt_params_default(rt_params *out); /* defaults of get_parameters, no arrays */

/* Host physics the solver is built from (per-run constants; T is constant).
 * GLQuad(M, 4 pi).mu()/wt() (GLQuad.cpp:4-44). */
rt_status rt_quadrature(int M, double *mu, double *wt);
/* Planck::get_Planck(T, edges) (Planck.cpp:50-77) times kcon -- the group
 * emission B_g [jk/cm^2/sh] and dB/dT_g (correction.cpp:25-36). */
rt_status rt_planck_groups(double T, int G, const double *e_edge, double *B, double *dBdT);

/* ---- solver lifecycle --------------------------------------------------- */

/* ParameterHandler(prm_path) + Solver ctor (solver.cpp:46-188): psi = B_g. */
rt_status rt_create(const char *prm_path, const char *table_dir, int device, rt_solver **out);
/* Same from an explicit configuration.  Only groups [g_lo, g_hi) get device
 * state (energy groups are independent for the whole run because T is
 * constant); all G groups' coefficients are still computed (the last Planck
 * group is a remainder, Planck.cpp:73-76).  g_hi <= 0 means G. */
rt_status rt_create_from_params(const rt_params *p, int g_lo, int g_hi, int device, rt_solver **out);
/* Direction-pair shard (SURVEY §8e fallback when there are fewer groups than GPUs):
 * the handle sweeps only the direction pairs [d_lo, d_hi) of the M/2 (pair d = the
 * directions mu_{H-1-d} < 0 and mu_{H+d} > 0, H = M/2; a line and its reflective
 * mirror stay together), with the full quadrature's nodes and weights.  Its psi/ends
 * cover M_l = 2 (d_hi - d_lo) directions in ascending mu; its moments and group ends
 * are the partial sums over them (sum them over the shards: the reference's
 * sequential sum over i then differs only by rounding); rt_get_balance* returns
 * RT_ERR_PARAM.  Lines are independent given their inflow, so each line's psi is
 * bitwise that of a full handle. */
rt_status rt_create_direction_shard(const rt_params *p, int g_lo, int g_hi, int d_lo, int d_hi, int device,
                                    rt_solver **out);
/* ~Solver.  Waits for the handle's queued work, then returns its device buffers (up to
 * 64 MB each), pinned staging, stream and events to a process-wide cache that the next
 * rt_create* on the device draws from (RTSN_POOL_MB, default 512, caps it; 0 frees
 * everything at once, as before); a failed device allocation empties the cache first. */
void rt_destroy(rt_solver *s);

/* Solver::solve (solver.cpp:590-823): max_timesteps full steps (x4 substeps
 * for BDF2), preceded by computeEquilibriumSources when use_mg_equilib.
 * Synchronous.  Short lines take the wavefront (rt_set_wavefront); a BDF2 run of longer
 * lines whose caller chose no time block, waves per segment or segmentation takes the
 * schedule rt_plan_schedule returns (results equal to rounding). */
rt_status rt_solve(rt_solver *s);
/* The pipelined schedule rt_solve picks for a BDF2 run of nsteps on this handle's lines:
 * the time block (8..40 steps), waves per segment (4) and segments sized for wgs_per_cu
 * workgroups per CU (4..32) with the least estimated whole-run time -- a model of the run
 * as P = n / T passes over the chain of segments (fill ramp, plateau, drain ramp; each
 * launch in rounds of the resident workgroups) plus the n mod T remainder (on vacuum
 * lines, at least T / 4 steps: a tail block riding the drain, one launch more; else aligned
 * passes) -- and that estimate.  Host arithmetic only; any NULL skipped. */
rt_status rt_plan_schedule(rt_solver *s, long long nsteps, int *steps_per_pass, int *level_waves, int *wgs_per_cu,
                           double *estimated_ms);
/* The time block rt_plan_schedule picks on the SL slab's geometry (N = 1e6 cells, S64, 128
 * groups, 256 CUs) for a BDF2 run of nsteps (host only, no handle), e.g. 20 for 300 steps,
 * 40 for 1000; the default block for BE / CN. */
rt_status rt_plan_time_block(int ts_method, long long nsteps, int *steps_per_pass);
/* Asynchronous: request nsteps full steps on the handle's stream.  Steps may stay queued
 * on the host until enough accumulate for an efficient launch -- a pipelined schedule
 * starts once its run would pipeline (a remainder of fewer than T steps waits for the
 * next read-out), the wavefront kernel launches once 8 times its chain's fill is queued --
 * and rt_finish or any read-out launches whatever is queued.  Results do not depend on how
 * a run is cut into rt_advance calls. */
rt_status rt_advance(rt_solver *s, int nsteps);
/* Enqueue what brings the stored state exactly to the requested time --
 * pipeline drain (with the queued remainder as each position's last block where the
 * pipeline can: vacuum lines, at least T / 4 steps), queued remainder steps as aligned
 * passes otherwise, pending correction.  Every
 * read-out does this implicitly; asynchronous. */
rt_status rt_finish(rt_solver *s);
rt_status rt_synchronize(rt_solver *s);
/* hipStream_t of the handle, as void*. */
void *rt_stream(rt_solver *s);

/* ---- results (host buffers, reference layouts) ------------------------- */
/* The host buffers may be pageable: psi / ends / moments move through two pinned
 * staging buffers of the handle (one export chunk each, up to 2 x 512 MB for ends;
 * allocated on the first transfer, freed by rt_destroy) with the host-side copy
 * split over up to 16 threads -- about 49 GB/s D2H on the SL state. */
rt_status rt_get_dims(rt_solver *s, int *M, int *G_local, int *N, int *g_lo, int *g_hi);
rt_status rt_get_psi(rt_solver *s, double *psi);                /* psi_mat_ref */
rt_status rt_get_ends(rt_solver *s, double *ends);              /* Solver::ends */
rt_status rt_set_ends(rt_solver *s, const double *ends);        /* load a state: checkpoint resume, tests */
/* compute_angle_integrated_intensity, compute_radiative_flux,
 * compute_positive_angle_integrated_intensity (solver.cpp:191-237); any NULL skipped */
rt_status rt_get_moments(rt_solver *s, double *phi, double *F, double *phi_plus);
/* compute_group_ends + get_ends("left"/"right") (solver.cpp:826-864) */
rt_status rt_get_group_ends(rt_solver *s, double *left, double *right);
/* compute_balance + get_balance (solver.cpp:240-284) */
rt_status rt_get_balance(rt_solver *s, double *balance);
/* ... with the sources and sinks it is built from (printed by the reference,
 * solver.cpp:278-279); any NULL skipped */
rt_status rt_get_balance_terms(rt_solver *s, double *balance, double *sources, double *sinks);
/* get_e_ave (solver.h:95): all G groups */
rt_status rt_get_e_ave(rt_solver *s, double *e_ave);
/* The shard a handle holds: the configuration's G and M, its groups [g_lo, g_hi) and
 * its direction pairs [d_lo, d_hi) of the M/2 (all pairs unless a direction shard). */
rt_status rt_get_shard(rt_solver *s, int *G_total, int *M_total, int *g_lo, int *g_hi, int *d_lo, int *d_hi);
/* compute_balance's terms (solver.cpp:240-284) split by how they add over direction-pair
 * shards, per local group: boundary inflow currents (jhp + jNm), outflow currents plus
 * absorption (jNp + jhm + sum_c rho kappa phi dx) -- both sums over the handle's
 * directions -- and the emission sum_c rho kappa a c T^4 dx (direction-independent).
 * sources = inflow + emission, sinks = outflow_absorption.  Any NULL skipped. */
rt_status rt_get_balance_partials(rt_solver *s, double *inflow, double *outflow_absorption, double *emission);
/* Group data of all G groups: e_edge (G+1), B, dBdT, kappa (G); any NULL skipped. */
rt_status rt_get_group_data(rt_solver *s, double *e_edge, double *B, double *dBdT, double *kappa);
rt_status rt_get_quadrature(rt_solver *s, double *mu, double *wt);
/* Solver-owned psi_source (M*G, m*G+g) after construction / equilibrium sources. */
rt_status rt_get_psi_source(rt_solver *s, double *psi_source);

/* ---- device-side hooks (multi-GPU, measurement) ------------------------- */
/* rt_get_moments into DEVICE buffers of G_local*N doubles (g + G_local*c), on
 * the handle's stream, asynchronous: the per-rank blocks of the end-of-run
 * gather; any NULL skipped. */
rt_status rt_get_moments_device(rt_solver *s, double *d_phi, double *d_F, double *d_phi_plus);
/* Group-summed absorption rate A(x_c) = sum_{g local} rho kappa_g phi_g(c),
 * written to a DEVICE buffer of N doubles on the handle's stream: the per-rank
 * partial of the group-sum all-reduce (north_star; the reference has no
 * material-temperature update, so nothing consumes it in the solve). */
rt_status rt_group_absorption_device(rt_solver *s, double *d_out);
/* NaN/Inf scan of the state (failure detection): *finite = 1 when
 * every node value of every line and cell is finite at the requested time
 * (queued steps are completed first), else 0.  One read of the state on the
 * device; blocks until the answer is on the host. */
rt_status rt_state_finite(rt_solver *s, int *finite);
/* Per-launch timing of the sweep kernel with HIP events on the handle's
 * stream (off by default). */
rt_status rt_set_profiling(rt_solver *s, int on);
rt_status rt_get_sweep_time(rt_solver *s, double *total_ms, long long *launches);
/* Algorithmic HBM bytes of one sweep pass (one profiled launch: T full steps,
 * the state is read and written once) and updates (cell x angle x group x
 * substep) per full step, for the handle's groups. */
rt_status rt_sweep_traffic(rt_solver *s, double *bytes_per_launch, double *updates_per_step);
/* Algorithmic FP64 flops of one pass: 2 per coefficient of the per-line
 * affine cell map (BDF2 28, CN 8, BE 6 FMAs per cell x line x step) times T
 * steps; the cross-segment correction is parallelisation overhead, not counted. */
rt_status rt_sweep_flops(rt_solver *s, double *flops_per_launch);
/* Time blocking: full steps advanced per pass over HBM: 1..8, 10, 12, 16, 20, 24,
 * 32 or 40 (default 16; aligned passes take at most 4; BDF2 beyond 20 runs the
 * level-split pass over four waves -- on SL T = 40 is the fastest per step, 7.5 vs
 * 8.2 ms at T = 16).  Results do not depend on it beyond rounding.  The segments of a line are re-sized for the new block's
 * pipelined kernel (its occupancy) as soon as every segment is at the same time
 * with no correction outstanding (now, or before the next pass). */
rt_status rt_set_time_block(rt_solver *s, int steps_per_pass);
/* Pipelined schedule: the segments of a line run at staggered time levels,
 * one pass apart, so each starts from its upwind neighbour's exact exit state
 * -- no cross-segment correction.  Steps are queued and launched as whole
 * passes; the pipeline fills over the first launches (one per segment) and
 * drains when a result is read (or rt_solve returns); those launches split
 * their segments over 2-4 waves (BDF2).  0: off -- every pass moves all
 * segments together (at most 4 steps) and corrects them in the next pass;
 * 1 (default): pipelined once the queued steps bring enough whole passes (BDF2 with
 * the split fill: at least 1/8 of the pipeline's depth, or rt_solve's plan for the run;
 * otherwise its depth) -- until then an advance's steps stay queued, and a read-out runs
 * them as aligned passes; 2: always pipelined. */
rt_status rt_set_pipeline(rt_solver *s, int on);
rt_status rt_get_pipeline(rt_solver *s, int *on);
/* Schedule state: steps the chain head is ahead of the tail (0 = aligned),
 * steps queued but not launched (segment schedules and the wavefront kernel's queue),
 * whether a correction is pending; any NULL skipped. */
rt_status rt_pipeline_state(rt_solver *s, long long *lag_steps, int *queued_steps, int *pending);
rt_status rt_get_time_block(rt_solver *s, int *steps_per_pass);
/* Short and mid-length lines: a wavefront over (cell, time level) with lanes over cells -- a
 * line (with the reflective left boundary: a mu < 0 line and its mirror) is a chain of lanes
 * of one workgroup, C cells per lane in registers, every step of an advance in one launch (up
 * to 65536 steps per launch), the upwind recurrence carried lane to lane by a DPP shift each
 * tick: C cells per lane (1, 2, 4, 8) on ceil(lanes / 64) waves -- one wave, or a chain of up
 * to rt_set_wavefront_waves' waves (default 8, lines of up to 4096 cells, reflective 2048)
 * handing the carried state from wave to wave through LDS -- with C the least estimated time
 * of a 1000-step advance from measured tick costs (kernels_wave.hip wavefront_plan;
 * rt_set_wavefront_cells overrides).  Results are bitwise those of the pipelined segment
 * schedule, whatever C and the waves per chain.  mode 0: off; 1 (default): used when the line
 * fits, the caller set neither a time block (rt_set_time_block) nor a schedule
 * (rt_set_pipeline), and -- for a chain of several waves -- the chains need at most two waves
 * per SIMD; 2: used whenever the line fits. */
rt_status rt_set_wavefront(rt_solver *s, int mode);
/* *mode as set; *active: the next rt_advance takes the wavefront; *cells_per_lane: C for
 * this handle's lines (0: too long for a wave).  Any NULL skipped. */
rt_status rt_get_wavefront(rt_solver *s, int *mode, int *active, int *cells_per_lane);
/* Waves a wavefront chain may span, 1..8 (default 8; 1 = one wave per chain, lines of up to
 * 512 cells).  The chain's lanes per line are ceil(N / C); replaces nothing in the reference
 * (its sweep is serial, solver.cpp:700-717). */
rt_status rt_set_wavefront_waves(rt_solver *s, int max_waves);
/* Cells per lane of the chain (1, 2, 4, 8; 0 = wavefront_plan's choice, the default): the
 * chain then spans ceil(lanes / 64) waves, and a choice whose chain would exceed max_waves
 * falls back to the plan's.  For measuring the plan's crossovers (tools/chain_plan.py);
 * bitwise-identical results. */
rt_status rt_set_wavefront_cells(rt_solver *s, int cells_per_lane);
/* *max_waves as set; *waves_per_chain: this handle's chain (0: too long).  NULLs skipped. */
rt_status rt_get_wavefront_waves(rt_solver *s, int *max_waves, int *waves_per_chain);
/* Waves per segment of a pipelined BDF2 pass of 8, 10, 12, 16 or 20 steps: 1 runs
 * all levels in one wave; 2 (or 4, T divisible by 4) shares them between the waves of
 * a workgroup through LDS; 0 (default) = 2 at T = 20 (its one-wave kernel leans on
 * AGPRs; the split one measured 2.7% faster on SL), 1 otherwise (at T = 16 one wave is
 * 4% faster), and with 0 the pipeline's fill and drain launches split
 * further (up to 4 waves) while the chip would idle.  T = 24, 32, 40 always run 4
 * waves.  rt_get_level_waves reports the effective choice for the current time block.
 * The choice covers whole blocks: a run's remainder block riding the drain (rt_plan_schedule)
 * always takes the tail kernel with the most waves for T (4, else 2), whatever is set here.
 * Bitwise-identical results.  Other schemes always use one wave. */
rt_status rt_set_level_waves(rt_solver *s, int waves);
/* Segments per line: sized so a pipelined launch with every segment active holds
 * wgs_per_cu workgroups per CU (1..64), or 0 (default) for the pass kernel's occupancy.
 * More segments than resident workgroups shorten the pipeline's fill and drain (the line
 * traversal per launch) at a small cost per segment: a 1000-step run of a 16-group SL
 * shard 1270 -> 1017 ms at 16 per CU (profiles/archive/r03g_grid16.jsonl).  Applied now if the
 * positions are aligned, else before the next pass; results bitwise independent of it in
 * the pipelined schedule. */
rt_status rt_set_segmentation(rt_solver *s, int wgs_per_cu);
rt_status rt_get_level_waves(rt_solver *s, int *waves);
/* Sweep geometry actually used: waves launched per step (one per line group
 * and segment) and segments per line. */
rt_status rt_sweep_geometry(rt_solver *s, int *workgroups, long long *tiles);

/* ---- test and A/B hooks -------------------------------------------------
 * Kernel forms the tests compare bitwise and the measurements time against each other
 * (the library reads no environment variable to pick a kernel or a schedule; the variables
 * read are RTSN_COMM_TIMEOUT_S, RTSN_POOL_MB and, in
 * bin/transfer and bin/test_gray, TRANSFER_DIR, RT_TABLE_DIR, RTSN_QUIET and the rank
 * variables RTSN_RANKS, RTSN_DEVICE_BASE and RTSN_FAULT_STALL_RANK, a test hook).
 * Moments kernel where M/2 is 8, 16 or 32: 1 (default) the producer/consumer
 * moments_pc_kernel, 0 the one-wave moments_kernel; bitwise-identical results. */
rt_status rt_set_moments_form(rt_solver *s, int form);
/* The material coupling's cross-segment correction of the fused angular sums: 0 (default)
 * the closed forms (phi_correction_geo_kernel for BE / CN, phi_correction_rows_kernel for
 * BDF2), 1 the cell-by-cell walk; equal to rounding. */
rt_status rt_set_phi_correction_form(rt_solver *s, int form);
/* Fault injection: the pipelined sub-launch after `after` more successful ones fails with
 * RT_ERR_DEVICE without starting a kernel (-1: off, the default).  A launch cut into
 * sub-launches commits each sub-launch's chain positions as soon as it is in the stream, so
 * the next call (rt_advance, rt_finish, a read-out) runs exactly the positions still owed. */
rt_status rt_debug_fail_launch(rt_solver *s, int after);
/* Host transfers in pieces of at most `doubles` doubles (0: the defaults, 256 MB device
 * chunks and 16 MB pinned pieces; moments then come in one transfer per state): the chunk
 * edges of rt_get_psi / rt_get_ends / rt_set_ends and the staged moments, for testing. */
rt_status rt_debug_set_transfer_chunk(rt_solver *s, long long doubles);

/* ---- material-temperature coupling (beyond the reference) ---------------
 * The reference holds T constant (solver.cpp:157).  With coupling enabled the
 * handle carries a cell temperature T(x) and, per full time step n (duration
 * dt; ts_method 3's four substeps form one step), with sigma_g = rho kappa_g and
 * W = sum_i w_i over all directions:
 *   1. sweep with the per-cell emission Beff_g = B_g(T^n) + p_g (Planck group
 *      integrals on the device, Planck.cpp:44-337's algorithm; the last group is
 *      the grey remainder a c T^4 - integral over groups 0..G-2, when positive),
 *      p_g the share of the owed emission (below) paid in this sweep;
 *   2. q(x) = sum_g sigma_g (phi_g^{n+1} - W B_g(T^n)) and b(x) = sum_g sigma_g
 *      dB_g/dT(T^n): this handle's groups only -- with sharded groups the callers
 *      sum both over the ranks (ONE all-reduce of 2N doubles per step, e.g. RCCL);
 *   3. T^{n+1} = T^n + dT with dT = dt q / (rho_cv + dt W b): the update implicit
 *      in the material's own emission (B(T^{n+1}) linearised about T^n), which
 *      relaxes T toward the radiation's temperature at any dt / rho_cv (linear grey
 *      analysis; the explicit dT = dt q / rho_cv of rounds 1-5 needed
 *      dt W b / rho_cv < 2 + sigma c dt) and keeps T > 0 for BE (dT > -T since
 *      B_g <= T dB_g/dT).  Where dT > T / 4 the tangent of the convex B under-counts
 *      the emission at the new T (a cold cell beside hot ones absorbs many times its
 *      energy in a step: the linear update overshoots, then diverges; cooling, it only
 *      lags): the cell solves rho_cv (T' - T) = dt (A - W S(T'))
 *      instead, A = q + W S(T^n), S(T) = sum over ALL groups of sigma_g B_g(T) --
 *      every handle holds every group's edges and opacity, so no second reduction;
 *      one root (S increases), by Newton's method with bisection;
 *   4. the material thereby emitted dt W sigma_g dB_g/dT dT per group beyond the
 *      sweep's B (B_g(T^{n+1}) - B_g(T^n) where it solved the full emission): it joins
 *      the group's owed emission, paid in the next sweeps as p_g = max(owed_g, -B_g)
 *      (Beff >= 0; all of it unless the material cooled by a large fraction of T).
 * With ts_method 1 (BE) radiation + material + owed energy,
 * sum_x dx (sum_g phi_g / c + rho_cv T + rt_get_material_transit), changes by
 * exactly -dt x (net boundary outflow) per step (up to rounding).  Requires the
 * v/c correction to be inactive (V == 0 or use_correction == 0). */
/* Turn coupling on: rho_cv > 0 (material energy per volume per keV), T_cells
 * (N, host) the initial T(x), NULL for the uniform p.T.  The state psi is kept; nothing
 * is owed.  (RT_WARN_UNSTABLE is no longer returned: the update is implicit in T.) */
rt_status rt_material_enable(rt_solver *s, double rho_cv, const double *T_cells);
/* The emission's stiffness at the current T(x): number = dt W sum_g rho kappa_g
 * dB_g/dT(T_max) / rho_cv over ALL G groups (a shard reports the whole configuration's
 * number); the implicit update scales the explicit change by 1 / (1 + number) at the
 * hottest cell, and number < 2 was the explicit emission's limit.  Blocks (reads T(x)). */
rt_status rt_material_stability(rt_solver *s, double *number);
/* Steps 1-2: one coupled sweep, then this handle's [q, b] into d_q (DEVICE, 2N
 * doubles: q(x) then b(x); NULL: an internal buffer), on the handle's stream,
 * asynchronous. */
rt_status rt_material_sweep(rt_solver *s, double *d_q);
/* Steps 3-4 from the group-summed [q, b] in d_q (DEVICE, 2N; NULL: the internal
 * buffer), then B_g, dB_g/dT, the owed emission and Beff_g at the new T(x) for the next
 * step; handle's stream, asynchronous. */
rt_status rt_material_update(rt_solver *s, const double *d_q);
/* nsteps x (sweep + update) for a handle that holds all G groups. */
rt_status rt_material_step(rt_solver *s, int nsteps);
/* T(x) (N), the per-cell B_g(T(x)) and the next step's emission Beff (G_local*N each,
 * g + G_local*c) to host memory. */
rt_status rt_get_temperature(rt_solver *s, double *T_cells);
rt_status rt_get_cell_planck(rt_solver *s, double *B);
rt_status rt_get_cell_emission(rt_solver *s, double *Beff);
/* Energy per volume the material owes the radiation, per cell (N, host): dt W sum over
 * the handle's groups of sigma_g (p_g + owed_g) -- the next sweep's payment and the rest;
 * sum it over group shards. */
rt_status rt_get_material_transit(rt_solver *s, double *E);

/* ---- multi-GPU: RCCL behind the ABI (one process per GPU, xGMI) -----------
 * The reference is single-process (main.cc:79-133).  Energy groups are independent for
 * the whole run (T constant), so a job gives every rank a contiguous group shard
 * (rt_create_from_params(p, g_lo, g_hi, device)), or -- with fewer groups than ranks --
 * a direction-pair shard of all groups (rt_create_direction_shard); time stepping needs
 * no exchange.  An rt_comm joins the ranks' handles for the collectives after (or
 * between) the steps: every call below is collective (all ranks, same order), runs on
 * the handle's stream (RCCL over xGMI) and, where it returns host arrays, synchronises.
 * Shards must be all group shards that tile [0, G) in rank order, or all direction
 * shards of the same groups that tile [0, M/2) in rank order (else RT_ERR_PARAM).
 * No wait on a peer is unbounded: the communicator is non-blocking and every wait on it
 * (the init, a collective call in progress, the host synchronisations of the gathers) has
 * a deadline of RTSN_COMM_TIMEOUT_S seconds (default 300) per collective, clocked from the
 * moment the stream reaches that collective: the handle's own work queued before it (a long
 * rt_advance, the sweeps of rt_comm_material_step) is waited for without the deadline.  On
 * expiry -- a rank missing or stalled -- the communicator is aborted, the call returns
 * RT_ERR_TIMEOUT and later collectives on it RT_ERR_STATE.  The stream-ordered collectives
 * (rt_comm_allreduce_absorption, rt_comm_material_step) return before their all-reduces ran:
 * retire them with rt_comm_synchronize before any other host wait on the handle (a host
 * read-out such as rt_get_temperature, rt_synchronize, an upload that waits for the stream),
 * whose own waits carry no deadline -- only then does the bound hold for a missing peer. */
typedef struct rt_comm rt_comm;
#define RT_COMM_ID_BYTES 128
/* ncclGetUniqueId: on one rank, then handed to every rank (file, pipe, MPI, ...). */
rt_status rt_comm_unique_id(void *id);
/* ncclCommInitRankConfig (non-blocking) on `device` (the device of the rank's handle),
 * waited for up to RTSN_COMM_TIMEOUT_S: RT_ERR_TIMEOUT if the other ranks do not join. */
rt_status rt_comm_init(int nranks, int rank, const void *id, int device, rt_comm **out);
void rt_comm_destroy(rt_comm *c);
rt_status rt_comm_rank(rt_comm *c, int *nranks, int *rank);
/* ncclCommCount: the number of ranks RCCL itself reports for the communicator (equal to
 * rt_comm_init's nranks once it formed). */
rt_status rt_comm_count(rt_comm *c, int *count);
/* phi, F, phi_plus of ALL groups (G x N each, g + G c; NULL skipped; host, every rank):
 * group shards are gathered, direction shards summed (the reference's sequential sum
 * over i regrouped by shard: rounding only). */
rt_status rt_comm_gather_moments(rt_comm *c, rt_solver *s, double *phi, double *F, double *phi_plus);
/* compute_group_ends + get_ends of all G groups (host, every rank). */
rt_status rt_comm_gather_group_ends(rt_comm *c, rt_solver *s, double *left, double *right);
/* compute_balance of all G groups with its sources and sinks (host, every rank; NULL
 * skipped): group shards gather their own terms (bitwise the single-handle values);
 * direction shards sum rt_get_balance_partials and add the emission once. */
rt_status rt_comm_gather_balance(rt_comm *c, rt_solver *s, double *balance, double *sources, double *sinks);
/* psi_mat (M, G, N) of all groups and directions into host `psi` on `root` (other ranks
 * may pass NULL); moves M G_local N doubles per rank through the device, so meant for
 * .prm-sized runs (ψ of large runs stays sharded: rt_get_psi per rank). */
rt_status rt_comm_gather_psi(rt_comm *c, rt_solver *s, int root, double *psi);
/* Solver-owned psi_source (M*G, m*G+g) of all directions on every rank (direction shards
 * hold their rows only; rt_get_psi_source). */
rt_status rt_comm_gather_psi_source(rt_comm *c, rt_solver *s, double *psi_source);
/* The group-summed absorption A(x) = sum over ALL groups of rho kappa_g phi_g(x): each
 * rank's rt_group_absorption_device, then one ncclAllReduce(sum) of N doubles into the
 * DEVICE buffer d_out, stream-ordered, no host synchronisation. */
rt_status rt_comm_allreduce_absorption(rt_comm *c, rt_solver *s, double *d_out);
/* nsteps coupled steps (rt_material_*) across the shards: per step the shard's sweep and
 * [q, b], one ncclAllReduce(sum) of those 2N doubles on the handle's stream, then the T
 * update -- stream-ordered, no host synchronisation; every rank ends with the same T(x). */
rt_status rt_comm_material_step(rt_comm *c, rt_solver *s, int nsteps);
/* Host wait for everything enqueued on the handle's stream (its sweeps and c's stream-
 * ordered collectives), bounded by RTSN_COMM_TIMEOUT_S like the gathers: the replacement
 * for rt_synchronize after rt_comm_material_step / rt_comm_allreduce_absorption. */
rt_status rt_comm_synchronize(rt_comm *c, rt_solver *s);
const char *rt_comm_last_error(rt_comm *c);
/* The RCCL this library's collectives run on (host only, no device call): ncclGetVersion
 * (e.g. 22707 for 2.27.7) and the file the process resolved ncclGetVersion from.  librtsn
 * links librccl.so.1; a process that loaded another library of that name first (torch's
 * bundled RCCL, when torch is imported before librtsn) runs rt_comm on that one -- the same
 * RCCL as torch.distributed's process group in that process.  path may be NULL. */
rt_status rt_comm_version(int *version, char *path, size_t path_len);

/* ---- multi-GPU: host-side layout of the gathered shard blocks ----------------------
 * The placement steps of the rt_comm gathers as host functions (no device calls, valid
 * without a GPU) for callers that run their own collectives (MPI, torch.distributed, ...).
 * rt_comm_* runs exactly these copy plans on the device (hipMemcpy2DAsync).  A shard is
 * groups [g_lo, g_hi) and direction pairs [d_lo, d_hi) of the M/2 of a (G, M, N)
 * configuration (rt_get_shard, rt_get_dims); the ranks' shards must be group shards
 * tiling [0, G) in rank order or direction shards tiling [0, M/2) over all groups
 * (else RT_ERR_PARAM).  Wire blocks are padded to the largest shard's Gmax groups. */
typedef struct {
  int G, M;         /* the configuration's groups and directions */
  int g_lo, g_hi;   /* the shard's groups */
  int d_lo, d_hi;   /* its direction pairs of the M/2 (all: 0, M/2) */
  int N;            /* cells */
  int reserved;     /* 0 */
} rt_shard;
/* *mode: 0 group shards, 1 direction shards; *max_groups: Gmax.  Any NULL skipped. */
rt_status rt_layout_mode(const rt_shard *shards, int nranks, int *mode, int *max_groups);
/* rank's phi, F, phi_plus (local: 3 arrays of N x G_local back to back, g fastest, as
 * rt_get_moments_device writes them; NULL for an empty shard) -> its wire block
 * [3][N][Gmax], padding zeroed */
rt_status rt_layout_pack_moments(const rt_shard *shards, int nranks, int rank, const double *local, double *block);
/* gathered: group shards the all-gather of every rank's block [rank][3][N][Gmax];
 * direction shards their sum [3][N][Gmax] -> phi, F, phi_plus (G x N, g + G c); NULL skipped */
rt_status rt_layout_unpack_moments(const rt_shard *shards, int nranks, const double *gathered, double *phi,
                                   double *F, double *phi_plus);
/* k per-group vectors (G_local each) -> the rank's block [k][Gmax]; in[j] NULL leaves zeros */
rt_status rt_layout_pack_vectors(const rt_shard *shards, int nranks, int rank, int k, const double *const *in,
                                 double *block);
/* gathered [rank][k][Gmax] (group shards) or their sum [k][Gmax] (direction shards) -> k
 * vectors of G; out[j] NULL skipped */
rt_status rt_layout_unpack_vectors(const rt_shard *shards, int nranks, int k, const double *gathered,
                                   double *const *out);
/* one shard's psi (M_l, G_local, N) as rt_get_psi returns it -> its entries of the (M, G, N) psi */
rt_status rt_layout_place_psi(const rt_shard *shard, const double *block, double *psi);
/* one shard's psi_source rows (M_l x G, as rt_get_psi_source returns them) -> its rows of (M x G) */
rt_status rt_layout_place_psi_source(const rt_shard *shard, const double *rows, double *psi_source);

const char *rt_status_string(rt_status st);
/* Last error message recorded on the handle (or the global one for s == NULL). */
const char *rt_last_error(rt_solver *s);

#ifdef __cplusplus
}
#endif
#endif /* RTSN_H */
