// rtsn_internal.hpp -- what the translation units behind the C ABI share: the handle
// (struct rt_solver), the device-buffer / stream / event cache, error reporting and the
// small schedule helpers.  Not installed; include/rtsn.h is the interface.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/rtsn.h"
#include "cell.hpp"
#include "kernels.hpp"
#include "physics.hpp"
#include "prm.hpp"

namespace rtsn_detail {
using namespace rtamd;

// ---------------------------------------------------------------------------
// Handle resource cache.  A handle's lifetime allocates ~20 device buffers, two pinned
// staging buffers, a stream and events, and hipFree / hipHostFree synchronise the device:
// together ~1 ms per Solver(ph) ... ~Solver() pair on the box, more than the reference's
// own configurations take to solve (llnl_slab_test's 2 steps: 21 us).  rt_destroy (and
// the getters' temporaries) hand them to this process-wide cache -- blocks of at most
// kPoolMaxBlock, RTSN_POOL_MB in all (default 512; 0 turns the cache off), only after the
// owning stream is idle -- and the next allocation of the same kind, device and size class
// takes them back.  A failed device allocation empties that device's cache and retries.
// The cache is never destroyed (no HIP call after the runtime's teardown at exit).
// ---------------------------------------------------------------------------
constexpr size_t kPoolMaxBlock = size_t(64) << 20;

class ResourcePool {
 public:
  static ResourcePool &get() {
    static ResourcePool *pool = new ResourcePool();
    return *pool;
  }
  // device (host = false) or pinned host (host = true) memory: *cap receives the block's size
  hipError_t alloc(bool host, size_t bytes, void **out, size_t *cap) {
    const size_t want = round(bytes);
    int dev = 0;
    if (!host) (void)hipGetDevice(&dev);
    if (cap_ && want <= kPoolMaxBlock) {
      std::lock_guard<std::mutex> lk(m_);
      auto it = blocks_.lower_bound(std::make_tuple(host, host ? 0 : dev, want));
      if (it != blocks_.end() && std::get<0>(it->first) == host && std::get<1>(it->first) == (host ? 0 : dev) &&
          std::get<2>(it->first) <= 2 * want) {  // the smallest cached block that fits, if not twice too big
        *cap = std::get<2>(it->first);
        *out = it->second;
        cached_ -= *cap;
        blocks_.erase(it);
        return hipSuccess;
      }
    }
    *cap = want;
    hipError_t e = host ? hipHostMalloc(out, want, hipHostMallocDefault) : hipMalloc(out, want);
    if (e != hipSuccess) {  // memory held by the cache first
      (void)hipGetLastError();
      trim(host, dev);
      e = host ? hipHostMalloc(out, want, hipHostMallocDefault) : hipMalloc(out, want);
    }
    return e;
  }
  // p must not be in use by any queued work (its stream synchronised)
  void release(bool host, void *p, size_t cap, int dev) {
    if (!p) return;
    if (cap_ && cap <= kPoolMaxBlock) {
      std::lock_guard<std::mutex> lk(m_);
      if (cached_ + cap <= cap_) {
        blocks_.emplace(std::make_tuple(host, host ? 0 : dev, cap), p);
        cached_ += cap;
        return;
      }
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (!host && cur != dev) (void)hipSetDevice(dev);
    (void)(host ? hipHostFree(p) : hipFree(p));
    if (!host && cur != dev) (void)hipSetDevice(cur);
  }
  hipError_t stream(hipStream_t *out) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (cap_) {
      std::lock_guard<std::mutex> lk(m_);
      for (size_t i = 0; i < streams_.size(); ++i)
        if (streams_[i].first == dev) {
          *out = streams_[i].second;
          streams_.erase(streams_.begin() + static_cast<long>(i));
          return hipSuccess;
        }
    }
    return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
  }
  void release_stream(hipStream_t st, int dev) {  // st idle
    if (!st) return;
    if (cap_) {
      std::lock_guard<std::mutex> lk(m_);
      if (streams_.size() < 64) {
        streams_.emplace_back(dev, st);
        return;
      }
    }
    (void)hipStreamDestroy(st);
  }
  hipError_t event(bool timing, hipEvent_t *out) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (cap_) {
      std::lock_guard<std::mutex> lk(m_);
      auto it = events_.find(std::make_pair(dev, timing));
      if (it != events_.end()) {
        *out = it->second;
        events_.erase(it);
        return hipSuccess;
      }
    }
    return timing ? hipEventCreate(out) : hipEventCreateWithFlags(out, hipEventDisableTiming);
  }
  void release_event(hipEvent_t ev, bool timing, int dev) {
    if (!ev) return;
    if (cap_) {
      std::lock_guard<std::mutex> lk(m_);
      if (events_.size() < 4096) {
        events_.emplace(std::make_pair(dev, timing), ev);
        return;
      }
    }
    (void)hipEventDestroy(ev);
  }

 private:
  ResourcePool() {
    cap_ = size_t(512) << 20;
    if (const char *env = std::getenv("RTSN_POOL_MB")) cap_ = static_cast<size_t>(std::max(0L, std::atol(env))) << 20;
  }
  static size_t round(size_t bytes) {  // size classes: 256 B up to 64 KiB, then 64 KiB
    const size_t q = bytes <= (size_t(64) << 10) ? 256 : (size_t(64) << 10);
    return (std::max<size_t>(bytes, 16) + q - 1) / q * q;
  }
  void trim(bool host, int dev) {
    std::lock_guard<std::mutex> lk(m_);
    for (auto it = blocks_.begin(); it != blocks_.end();) {
      if (std::get<0>(it->first) == host && (host || std::get<1>(it->first) == dev)) {
        (void)(host ? hipHostFree(it->second) : hipFree(it->second));
        cached_ -= std::get<2>(it->first);
        it = blocks_.erase(it);
      } else {
        ++it;
      }
    }
  }
  std::mutex m_;
  size_t cap_ = 0, cached_ = 0;
  std::multimap<std::tuple<bool, int, size_t>, void *> blocks_;  // (pinned host, device, size) -> block
  std::vector<std::pair<int, hipStream_t>> streams_;
  std::multimap<std::pair<int, bool>, hipEvent_t> events_;      // (device, timing) -> event
};

struct DeviceBuf {
  void *p = nullptr;
  size_t bytes = 0, cap = 0;
  int dev = 0;
  DeviceBuf() = default;
  DeviceBuf(const DeviceBuf &) = delete;  // owns p
  DeviceBuf &operator=(const DeviceBuf &) = delete;
  ~DeviceBuf() { reset(); }
  void reset() {  // the owner's stream must be idle
    ResourcePool::get().release(false, p, cap, dev);
    p = nullptr;
    bytes = cap = 0;
  }
};

}  // namespace rtsn_detail

using namespace rtamd;  // the handle's members are rtamd types

struct rt_solver {
  // configuration (owned copies)
  rt_params p{};
  std::vector<double> prm_psi_source, prm_bounds, prm_kappa;
  phys::GroupTable gt;
  std::vector<double> mu, wt;
  std::vector<double> psi_source;  // solver-owned, M*G
  bool equilibrium_done = false;
  int g_lo = 0, g_hi = 0, Gl = 0, H = 0, Lh = 0, Lpad = 0, Q = 0, J = 0;
  int scheme = SCHEME_BDF2, K = 5;
  int T = 1;                     // full steps fused per pass (time block)
  int Tp = 0;                    // steps of the pass whose correction is pending
  int Sg = 1, Ls = 16;           // segments per line and cells per segment
  int seg_T = 0;                 // the time block the segments were sized for (0: none)
  int seg_w = 0;                 // ... and the workgroups per CU they were sized for
  bool T_set = false;            // the caller chose the time block (rt_set_time_block)
  int level_waves = 0;           // pipelined BDF2 passes: 0 auto (level_waves_of), 1 one wave, 2 levels shared by two
  bool lw_set = false;           // the caller chose the waves per segment (rt_set_level_waves)
  int seg_wgs = 0;               // segments sized for this many workgroups per CU (0: the pass's occupancy)
  bool seg_set = false;          // the caller chose the segmentation (rt_set_segmentation)
  bool planned = false;          // the run's schedule was planned (plan_schedule): pipelined from one pass
  int plan_T0 = 0, plan_lw0 = 0, plan_w0 = 0;  // ... over the handle's own T, level_waves, seg_wgs (end_plan)
  int d_lo = 0, d_hi = 0;        // direction-pair shard [d_lo, d_hi) of the M/2 pairs (d_hi = 0: all)
  int M_full = 0;                // the configuration's M (p.M is the handle's own direction count)
  int device = 0, cus = 0;
  hipStream_t stream = nullptr;
  // device state
  rtsn_detail::DeviceBuf E, map, hmap, prop[kMaxAlignedBlock + 1], bdry, agg[2], yseg, yrefl, lineB, muwt, mom, rows, sigma;
  std::vector<double> map_host;  // [2][WN][Lpad], kept for the lazily built propagators
  bool prop_ready[kMaxAlignedBlock + 1] = {};
  int agg_cur = 0;               // aggregates of the last pass live in agg[agg_cur ^ 1]
  bool pending = false;          // E holds provisional segments (correction outstanding)
  // every launch that writes E bumps state_version; the moments kernel's phi, F, phi_plus
  // in `mom` are reused by every read-out (moments, balance, absorption) of the same state
  unsigned long long state_version = 1, mom_version = 0;
  unsigned long long mom_serial = 0;  // moments kernel launches; mom_host holds launch mom_host_serial's
  // pipelined schedule (rt_set_pipeline): chain positions (segments; half 0 then
  // half 1 when the left boundary is reflective) at staggered time levels
  int pipe = 1;                  // 0 off, 1 auto (runs long enough to fill), 2 always
  bool pipe_set = false;         // the caller chose the schedule (rt_set_pipeline)
  int wave = 1;                  // short lines, one launch per advance (rt_set_wavefront): 0 off, 1 auto, 2 on
  int wave_max = kWaveMaxWaves;  // waves a wavefront chain may span (rt_set_wavefront_waves)
  int wave_cells = 0;            // cells per lane of the chain: 0 the plan's, else 1, 2, 4, 8 (rt_set_wavefront_cells)
  std::vector<long long> tau;    // full steps completed per chain position
  long long target = 0;          // full steps every position must reach
  long long pipe_base = 0;       // tau of every position when the pipeline started
  int queued = 0;                // requested steps not yet enqueued (< T)
  long long wqueued = 0;         // requested steps queued for the wavefront kernel (wave_advance)
  int Tpipe = 0;                 // time block of the running pipeline (0: positions aligned)
  int tail = 0;                  // draining: the run's last steps (< Tpipe), each position's final block
  int resume_lo = -1, resume_hi = -1;  // positions a failed sub-launch still owes (pipe_launch)
  int fail_launch_after = -1;    // test hook (rt_debug_fail_launch): pipelined sub-launches before one fails
  long long transfer_chunk = 0;  // test hook (rt_debug_set_transfer_chunk): doubles per host transfer piece, 0 default
  int moments_form = 1;          // rt_set_moments_form: 1 producer/consumer, 0 one-wave (bitwise equal)
  int phi_corr_form = 0;         // rt_set_phi_correction_form: 0 closed forms, 1 the cell-by-cell walk
  // material-temperature coupling (rt_material_enable)
  bool material = false;
  double rho_cv = 0.0, wsum = 0.0;  // wsum: this handle's quadrature weights (its q share)
  double wsum_all = 0.0;              // all M directions' weights (W of the T update)
  // Tcell [N]; Bcell [N][Gl] B_g(T); Beff [N][Gl] the step's emission B + the owed share paid;
  // owed, dBcell [Gl][N] the owed emission and dB_g/dT; dTlast [N] the last update's dT; bpart
  // [N] sum_gl sigma dB/dT; qbuf [2N] the exchange buffer (q, b)
  rtsn_detail::DeviceBuf Tcell, Bcell, Beff, owed, dBcell, dTlast, bpart, qbuf, edges, map_unit, hmap_unit, phi_part;
  rtsn_detail::DeviceBuf sigma_all;  // [G] rho kappa of every group (the update's full-emission cells)
  rtsn_detail::DeviceBuf corr_pow;            // A^Lsub per line for phi_correction_kernel's sub-segments
  int corr_pow_L = 0;            // the Lsub it holds (0: none)
  rtsn_detail::DeviceBuf corr_rows;           // BDF2: rows b A^j and A^64 per line (phi_correction_rows_kernel)
  bool phi_fused = false;        // angular sums fused into the coupled pass (M/2 divides 64)
  PlanckCells pc{};
  // profiling
  bool profiling = false;
  std::vector<hipEvent_t> ev_pool;   // (start, stop) pairs of profiled launches
  size_t ev_used = 0;
  double sweep_ms = 0.0;             // folded-in time of earlier pairs
  long long launches = 0, profiled = 0;
  // chunked host transfers (rt_get_psi / rt_get_ends / rt_set_ends): pinned staging
  void *staging[2] = {nullptr, nullptr};
  size_t staging_bytes = 0, staging_cap[2] = {0, 0};
  hipEvent_t staging_ev[2] = {nullptr, nullptr};
  // pinned host copy of `mom` ([3][GN], when it fits one staged piece): every moments read-out
  // of one state after the first is a host copy (a D2H after the rows' small copies stalled
  // the first phi_plus read-out of a process ~8 ms, r06j)
  void *mom_host = nullptr;
  size_t mom_host_cap = 0;
  unsigned long long mom_host_serial = 0;
  // host -> device uploads of the per-line setup (upload()): a pinned arena the copies leave
  // from asynchronously; reused from its start after a stream synchronisation
  void *up_arena = nullptr;
  size_t up_cap = 0, up_used = 0;
  bool agg_zero_pending = false;  // the aggregates are zeroed before the first segment pass
  std::string err;

  ~rt_solver() {  // everything goes back to the resource cache once the stream is idle
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);  // no kernel may outlive the buffers it uses
    rtsn_detail::ResourcePool &pool = rtsn_detail::ResourcePool::get();
    for (int k = 0; k < 2; ++k) pool.release(true, staging[k], staging_cap[k], 0);
    pool.release(true, mom_host, mom_host_cap, 0);
    pool.release(true, up_arena, up_cap, 0);
    for (hipEvent_t e : staging_ev) pool.release_event(e, false, device);
    for (hipEvent_t e : ev_pool) pool.release_event(e, true, device);
    pool.release_stream(stream, device);
  }
};

namespace rtsn_detail {

// the handle's (and the thread's) last error; returns st
rt_status fail(rt_solver *s, rt_status st, const std::string &msg);
void set_last_error(const char *msg);  // the thread's error text alone (host-only units)

inline bool split_block(int T) { return level_split_supported(SCHEME_BDF2, T); }

// Waves per segment of the pipelined pass: the caller's choice, or by default two waves
// (sweep_split_kernel) where measured faster -- BDF2 at T = 20, whose one-wave kernel
// needs 126 AGPRs beside 256 VGPRs (9% extra moves; split 8.29-8.31 vs 8.52-8.53 ms/step
// on SL, profiles/archive/r02b_split20.jsonl) -- and one wave otherwise (T = 16: 4% faster).
inline int level_waves_of(const rt_solver *s, int T) {
  if (s->scheme != SCHEME_BDF2 || !split_block(T)) return 1;  // the split kernel is BDF2's
  if (T > 20) return 4;                                         // one or two waves would spill
  int lw = s->level_waves ? s->level_waves : (T == 20 ? 2 : 1);
  if (lw == 4 && T % 4) lw = 2;
  return lw;
}


// Waves per segment of one pipelined launch of `grid` workgroups.  The segments are sized
// so that a full launch (every chain position active) fills the chip; the pipeline's fill
// and drain launches hold fewer positions, and with the default level_waves (0) their
// segments are split over 2 or 4 waves (sweep_split_kernel; BDF2 time blocks the split
// kernel has) -- the lines are then traversed 2-4x faster while the chip would otherwise
// idle.  The pick minimises the levels the busiest SIMD runs (a workgroup's k waves take
// one SIMD each; T / k levels per wave): e.g. 5 of 8 positions of the driver's T = 20 window
// as four waves run 3 x 5 levels per SIMD instead of 2 x 10 (round 3 had kept two waves
// beyond the full launch's wave count: 133 of the full launch's 164 ms for 5/8 of its work,
// profiles/archive/r03ar_trace_summary.json).  Ties go to the most waves within that count.
inline int fill_level_waves(const rt_solver *s, int grid) {
  const int base = level_waves_of(s, s->Tpipe);
  if (s->level_waves || s->scheme != SCHEME_BDF2 || !split_block(s->Tpipe)) return base;
  const int T = s->Tpipe;
  const long long full = 2LL * s->Q * s->Sg * base;  // waves of a launch with every position active
  int within = base;                                 // the most waves per segment within `full`
  while (within < 4 && T % (2 * within) == 0 && static_cast<long long>(grid) * 2 * within <= full) within *= 2;
  const long long per_cu = (static_cast<long long>(grid) + s->cus - 1) / s->cus;  // workgroups on the busiest CU
  const auto cost = [&](int k) { return (per_cu * k + 3) / 4 * (T / k); };       // levels on its busiest SIMD
  int best = base;
  for (int k = 2 * base; k <= 4 && T % k == 0; k *= 2) {
    const long long c = cost(k), cb = cost(best);
    if (c < cb || (c == cb && k <= within)) best = k;
  }
  return best;
}

// Waves of the tail launch (launch_split_tail): the most waves with a tail kernel for T,
// whatever rt_set_level_waves fixed for the whole blocks -- the split of the shortest tails
// that can ride the drain (T / waves levels), and a layout the whole blocks share; 0 when
// the pipeline cannot carry a tail: reflective chains (the mu > 0 heads take the mu < 0
// outflow), other schemes, blocks without a tail kernel.  complete() takes a tail of at
// least T / waves steps, so that wave 0 (which streams the rows in) runs the plain body.
inline int tail_waves(const rt_solver *s, int T) {
  if (s->scheme != SCHEME_BDF2 || s->p.bc_left_indicator == 2) return 0;
  for (int k : {4, 2})
    if (split_tail_supported(T, k)) return k;
  return 0;
}

// Chain positions of the pipelined schedule: the Sg segments of a line (both
// halves in step), or 2 Sg when the mu > 0 lines continue the mu < 0 ones.
inline int chain_positions(const rt_solver *s) {
  return s->p.bc_left_indicator == 2 ? 2 * s->Sg : s->Sg;
}


#define HIP_TRY(s, expr)                                                                        \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail((s), RT_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

// Full steps fused per HBM pass by default (rt_set_time_block changes it).
// Measured on SL (pipelined schedule, profiles/): BDF2 43.0 / 21.7 / 14.5 / 12.3 /
// 9.5 / 9.0 / 8.4 ms per step at T = 1 / 2 / 3 / 4 / 8 / 12 / 16.
inline int default_time_block(int) { return 16; }

// rt_set_time_block's domain: the instantiated sweep kernels (kernels.hip launch_s)
inline bool supported_time_block(int T) {
  return (T >= 1 && T <= 8) || T == 10 || T == 12 || T == 16 || T == 20 || T == 24 || T == 32 || T == 40;
}

inline int map_count_of(int scheme) {
  switch (scheme) {
    case SCHEME_BE: return map_count<SCHEME_BE>();
    case SCHEME_CN: return map_count<SCHEME_CN>();
    default: return map_count<SCHEME_BDF2>();
  }
}

inline hipError_t dalloc(DeviceBuf &b, size_t bytes) {  // b empty
  b.bytes = bytes;
  (void)hipGetDevice(&b.dev);
  return ResourcePool::get().alloc(false, bytes, &b.p, &b.cap);
}
inline Geometry geometry(const rt_solver *s) { return Geometry{s->p.M, s->Gl, s->p.N, s->J * kSweepTile, s->Lpad}; }

// rtsn_lines.hip
rt_status upload(rt_solver *s, DeviceBuf &b, const void *src, size_t bytes);
template <int S>
rt_status line_maps_s(rt_solver *s, bool unit_B, DeviceBuf &map_dev, DeviceBuf &hmap_dev);
rt_status ensure_propagators(rt_solver *s, int T);
rt_status setup_lines(rt_solver *s);
rt_status upload_inflow(rt_solver *s);
void segment_lines(rt_solver *h, int waves_per_cu, long long max_sg = 1LL << 40);
long long aligned_segments(const rt_solver *h);
hipError_t alloc_segments(rt_solver *h);
rt_status segment_target(rt_solver *h, int *w_out);
rt_status resegment(rt_solver *h, bool aligned = false);

// rtsn_schedule.hip
rt_status check_validation(rt_solver *s);
rt_status ensure_equilibrium(rt_solver *s);
rt_status fold_events(rt_solver *s);
SegArgs seg_args(rt_solver *s);
// zero the segment aggregates if a (re)allocation left them pending: before any segment pass
rt_status ensure_segments(rt_solver *s);
rt_status enqueue_fold(rt_solver *s, int T, bool reflective_outflow);
rt_status apply_correction(rt_solver *s);
rt_status enqueue_pass(rt_solver *s, int T, bool coupled = false);
rt_status complete(rt_solver *s);
rt_status finalize(rt_solver *s);
rt_status wave_flush(rt_solver *s);
WavePlan wave_plan(const rt_solver *s);
void end_plan(rt_solver *s);  // the planned schedule gives way to the handle's own
bool use_wavefront(const rt_solver *s);

// rtsn_readout.hip
rt_status compute_moments(rt_solver *s);

}  // namespace rtsn_detail
