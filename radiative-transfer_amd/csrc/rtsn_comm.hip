// rtsn_comm.hip -- RCCL behind the C ABI (include/rtsn.h, "multi-GPU").
//
// The reference runs one process (main.cc:79-133).  Here a job runs one process per
// GPU, each holding a shard handle; groups never exchange data while stepping (T is
// constant, solver.cpp:157), so the only collectives are the end-of-run reductions of
// the reference's result arrays and, in the material-coupled mode, one all-reduce of
// [q(x), b(x)] (2N doubles) per step.  Every collective is enqueued on the handle's own stream, so it is
// ordered after the sweeps that produce its input without a host synchronisation.
//
// Layouts on the wire (one all-gather per result, each rank's block padded to the
// largest shard so the counts agree):
//   moments  [3][N][Gmax]   (phi, F, phi_plus; g fastest, as rt_get_moments_device)
//   vectors  [k][Gmax]      (group ends, balance terms)
// and the assembly into the (G, N) / (G) arrays is the copy plans of comm_layout.cpp --
// host code shared with the rt_layout_* entry points, which the CPU tests check at world
// sizes 2, 3 and 8 -- run here with hipMemcpy2DAsync (device blocks) or on the host.
//
// No wait on a peer can hang a job: the communicator is created non-blocking
// (ncclCommInitRankConfig, blocking = 0) and every wait on it -- the init, a collective call
// that reports ncclInProgress, and each host synchronisation after collectives -- polls with a
// deadline of RTSN_COMM_TIMEOUT_S seconds (default 300).  The deadline runs only while a
// collective is executing: every collective is bracketed by two events on the stream
// (Mark), and a host wait clocks the collective whose opening event has completed and whose
// closing one has not.  The local work queued before it (a long rt_advance, the sweeps of
// rt_comm_material_step) is the handle's own and is waited for without that deadline.  On
// expiry the communicator is aborted (ncclCommAbort: RCCL stops the kernels still waiting on
// a peer) and the call returns RT_ERR_TIMEOUT; the handle then refuses further collectives
// (RT_ERR_STATE).  Scratch buffers are stream-ordered (hipMallocAsync / hipFreeAsync), so an
// error path never blocks the host on the stream to free them.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtsn.h"
#include "comm_layout.hpp"

namespace layout = rtamd::layout;

// One enqueued collective: `pre` completes when the stream reaches it (the local work before
// it is done), `post` when the collective has finished.  `since` is when a host wait first
// saw `pre` complete and `post` not: the collective's deadline runs from there.
struct Mark {
  hipStream_t st = nullptr;
  hipEvent_t pre = nullptr, post = nullptr;
  std::chrono::steady_clock::time_point since{};
  bool started = false;
};

struct rt_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
  bool aborted = false;  // a wait expired: the communicator was aborted
  double timeout_s = 300.0;
  double *q = nullptr;  // material coupling: [q(x), b(x)] of the running step (2N doubles)
  size_t q_len = 0;
  std::vector<Mark> marks;         // collectives enqueued since the last completed host wait
  std::vector<hipEvent_t> events;  // recycled event pool
  std::string err;
  ~rt_comm() {
    if (q) (void)hipFree(q);
    for (Mark &m : marks) {
      events.push_back(m.pre);
      events.push_back(m.post);
    }
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    if (nc) {  // non-blocking: finalize, wait (bounded) for quiescence, then free
      const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
      ncclResult_t st = ncclCommFinalize(nc);
      while (st == ncclInProgress && std::chrono::steady_clock::now() < end) {
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        if (ncclCommGetAsyncError(nc, &st) != ncclSuccess) break;
      }
      if (st == ncclSuccess)
        (void)ncclCommDestroy(nc);
      else
        (void)ncclCommAbort(nc);
    }
  }
};

namespace {

thread_local std::string g_comm_error;

rt_status cfail(rt_comm *c, rt_status st, const std::string &msg) {
  if (c) c->err = msg;
  g_comm_error = msg;
  return st;
}

double comm_timeout_s() {
  const char *env = std::getenv("RTSN_COMM_TIMEOUT_S");
  const double t = env ? std::atof(env) : 300.0;
  return t > 0.0 ? t : 300.0;
}

// The deadline expired or RCCL reported an error: abort the communicator (RCCL stops the
// kernels still waiting on a peer), after which the handle refuses collectives.
rt_status abort_comm(rt_comm *c, rt_status st, const std::string &msg) {
  if (c->nc) (void)ncclCommAbort(c->nc);
  c->nc = nullptr;
  c->aborted = true;
  return cfail(c, st, msg);
}

// A non-blocking call's result: ncclInProgress is polled (ncclCommGetAsyncError) until it
// settles or the deadline passes.
rt_status nc_settle(rt_comm *c, ncclResult_t r, const char *what) {
  if (r == ncclSuccess) return RT_OK;
  if (r != ncclInProgress || !c || !c->nc)
    return c && c->nc ? abort_comm(c, RT_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r))
                      : cfail(c, RT_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    ncclResult_t st = ncclInProgress;
    const ncclResult_t q = ncclCommGetAsyncError(c->nc, &st);
    if (q != ncclSuccess) st = q;
    if (st == ncclSuccess) return RT_OK;
    if (st != ncclInProgress) return abort_comm(c, RT_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(st));
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > c->timeout_s)
      return abort_comm(c, RT_ERR_TIMEOUT, std::string(what) + ": no progress within RTSN_COMM_TIMEOUT_S = " +
                                               std::to_string(c->timeout_s) + " s (a rank is missing or stalled); "
                                               "communicator aborted");
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

hipEvent_t take_event(rt_comm *c) {
  if (!c->events.empty()) {
    hipEvent_t e = c->events.back();
    c->events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  return hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess ? e : nullptr;
}

// The collectives of stream st have completed (or were aborted): their events go back to the pool.
void retire_marks(rt_comm *c, hipStream_t st) {
  std::vector<Mark> keep;
  for (Mark &m : c->marks) {
    if (m.st != st) {
      keep.push_back(m);
      continue;
    }
    c->events.push_back(m.pre);
    c->events.push_back(m.post);
  }
  c->marks.swap(keep);
}

// A collective enqueued on st between two events (Mark): the host waits clock it from the
// moment the stream reaches it, not from the moment they start.
template <class F>
rt_status enqueue_collective(rt_comm *c, hipStream_t st, const char *what, F &&call) {
  {  // collectives already finished (a caller that never waits through rt_comm) leave the list
    std::vector<Mark> live;
    for (Mark &m : c->marks) {
      if (hipEventQuery(m.post) == hipSuccess) {
        c->events.push_back(m.pre);
        c->events.push_back(m.post);
      } else {
        live.push_back(m);
      }
    }
    c->marks.swap(live);
  }
  Mark m;
  m.st = st;
  m.pre = take_event(c);
  m.post = take_event(c);
  if (!m.pre || !m.post) {
    if (m.pre) c->events.push_back(m.pre);
    if (m.post) c->events.push_back(m.post);
    return cfail(c, RT_ERR_DEVICE, std::string(what) + ": hipEventCreate failed");
  }
  if (hipEventRecord(m.pre, st) != hipSuccess) {
    c->events.push_back(m.pre);
    c->events.push_back(m.post);
    return cfail(c, RT_ERR_DEVICE, std::string(what) + ": hipEventRecord failed");
  }
  rt_status r = nc_settle(c, call(), what);
  if (r == RT_OK && hipEventRecord(m.post, st) != hipSuccess)
    r = cfail(c, RT_ERR_DEVICE, std::string(what) + ": hipEventRecord failed");
  if (r != RT_OK) {
    c->events.push_back(m.pre);
    c->events.push_back(m.post);
    return r;
  }
  c->marks.push_back(m);
  return RT_OK;
}

// Host wait for the collectives enqueued on st.  Only a collective in flight is clocked:
// the first Mark of st whose `pre` has completed and `post` has not has RTSN_COMM_TIMEOUT_S
// from the moment a poll first saw it running; a peer that never joins leaves RCCL's kernel
// spinning, which the abort ends.  Local work ahead of a collective (or after the last) is
// the handle's own and is not clocked.
rt_status comm_sync(rt_comm *c, hipStream_t st, const char *what) {
  for (;;) {
    const hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) {
      retire_marks(c, st);
      return RT_OK;
    }
    if (e != hipErrorNotReady) return cfail(c, RT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
    ncclResult_t as = ncclSuccess;
    if (c->nc && ncclCommGetAsyncError(c->nc, &as) == ncclSuccess && as != ncclSuccess && as != ncclInProgress)
      return abort_comm(c, RT_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(as));
    const auto now = std::chrono::steady_clock::now();
    for (Mark &m : c->marks) {
      if (m.st != st || hipEventQuery(m.post) == hipSuccess) continue;
      if (hipEventQuery(m.pre) != hipSuccess) break;  // local work ahead of this collective
      if (!m.started) {
        m.started = true;
        m.since = now;
      }
      if (std::chrono::duration<double>(now - m.since).count() > c->timeout_s) {
        (void)abort_comm(c, RT_ERR_TIMEOUT, "");
        (void)hipStreamSynchronize(st);  // the aborted kernels have returned; only local work remains
        retire_marks(c, st);
        return cfail(c, RT_ERR_TIMEOUT, std::string(what) + ": a collective did not complete within "
                                            "RTSN_COMM_TIMEOUT_S = " + std::to_string(c->timeout_s) +
                                            " s of starting (a rank is missing or stalled); communicator aborted");
      }
      break;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

#define NC_TRY(c, expr)                                          \
  do {                                                           \
    if (rt_status st_ = nc_settle((c), (expr), #expr)) return st_; \
  } while (0)
#define CO_TRY(c, st, expr)                                                                     \
  do {                                                                                          \
    if (rt_status st_ = enqueue_collective((c), (st), #expr, [&] { return (expr); })) return st_; \
  } while (0)
#define CS_TRY(c, st)                                                         \
  do {                                                                        \
    if (rt_status e_ = comm_sync((c), (st), __func__)) return e_;             \
  } while (0)
// every collective entry point: the communicator must be live
#define LIVE(c, what)                                                                                     \
  do {                                                                                                    \
    if ((c)->aborted) return cfail((c), RT_ERR_STATE, std::string(what) + ": the communicator was aborted " \
                                                      "after a timeout or an RCCL error; create a new one"); \
  } while (0)
#define HC_TRY(c, expr)                                                                                    \
  do {                                                                                                     \
    hipError_t e_ = (expr);                                                                                \
    if (e_ != hipSuccess) return cfail((c), RT_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_));  \
  } while (0)
#define RT_TRY(c, s, expr)                                                                                 \
  do {                                                                                                     \
    rt_status st_ = (expr);                                                                                \
    if (st_ != RT_OK) return cfail((c), st_, std::string(#expr ": ") + rt_last_error(s));                \
  } while (0)

// Device scratch, stream-ordered: allocated on the handle's stream and freed on it at scope
// exit (no host wait).
struct Scratch {
  void *p = nullptr;
  hipStream_t st = nullptr;
  hipError_t alloc(size_t bytes) { return hipMallocAsync(&p, bytes, st); }
  ~Scratch() {
    if (p) (void)hipFreeAsync(p, st);
  }
};

// Every rank's shard, and how the shards tile the problem (layout::shard_mode): 0 = group
// shards covering [0, G) in rank order (all directions each), 1 = direction shards covering
// [0, M/2) in rank order over the same groups.
rt_status all_shards(rt_comm *c, rt_solver *s, std::vector<rt_shard> &out, int &mode) {
  rt_shard me{};
  int G_total = 0, M_total = 0;
  RT_TRY(c, s, rt_get_shard(s, &G_total, &M_total, &me.g_lo, &me.g_hi, &me.d_lo, &me.d_hi));
  RT_TRY(c, s, rt_get_dims(s, nullptr, nullptr, &me.N, nullptr, nullptr));
  me.G = G_total;
  me.M = M_total;
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  constexpr int kInts = sizeof(rt_shard) / sizeof(int);
  static_assert(sizeof(rt_shard) == kInts * sizeof(int), "rt_shard is ints only");
  Scratch buf;
  buf.st = st;
  HC_TRY(c, buf.alloc(sizeof(int) * kInts * (c->nranks + 1)));
  int *d = static_cast<int *>(buf.p);
  HC_TRY(c, hipMemcpyAsync(d, &me, sizeof(rt_shard), hipMemcpyHostToDevice, st));
  CO_TRY(c, st, ncclAllGather(d, d + kInts, kInts, ncclInt32, c->nc, st));
  out.resize(c->nranks);
  HC_TRY(c, hipMemcpyAsync(out.data(), d + kInts, sizeof(rt_shard) * c->nranks, hipMemcpyDeviceToHost, st));
  CS_TRY(c, st);
  mode = layout::shard_mode(out.data(), c->nranks);
  if (mode < 0)
    return cfail(c, RT_ERR_PARAM, "shards must be group shards tiling [0, G) or direction shards tiling [0, M/2), "
                                  "in rank order, of one configuration");
  return RT_OK;
}

// A copy plan between device buffers, or from a device buffer to host memory.
rt_status run_plan(rt_comm *c, const std::vector<layout::Copy2D> &plan, const double *src, double *dst,
                   hipMemcpyKind kind, hipStream_t st) {
  for (const layout::Copy2D &p : plan)
    HC_TRY(c, hipMemcpy2DAsync(dst + p.dst, sizeof(double) * p.dpitch, src + p.src, sizeof(double) * p.spitch,
                               sizeof(double) * p.width, p.height, kind, st));
  return RT_OK;
}

// k host vectors of this rank's Gl groups -> all G groups on every rank: gathered (mode 0)
// or summed (mode 1).  in[j] / out[j] may be NULL (out NULL: not wanted).
rt_status combine_vectors(rt_comm *c, rt_solver *s, const std::vector<rt_shard> &sh, int mode,
                          const std::vector<const double *> &in, const std::vector<double *> &out) {
  const int k = static_cast<int>(in.size()), n = c->nranks, Gm = layout::max_groups(sh.data(), n);
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  const size_t cnt = static_cast<size_t>(k) * Gm;
  std::vector<double> block(cnt, 0.0);
  for (int j = 0; j < k; ++j)
    if (in[j]) layout::apply(layout::vectors_pack(sh.data(), n, c->rank, k, j), in[j], block.data());
  Scratch buf;
  buf.st = st;
  HC_TRY(c, buf.alloc(sizeof(double) * cnt * (n + 1)));
  double *d = static_cast<double *>(buf.p);
  HC_TRY(c, hipMemcpyAsync(d, block.data(), sizeof(double) * cnt, hipMemcpyHostToDevice, st));
  std::vector<double> all(mode == 0 ? cnt * n : cnt);
  if (mode == 0) {
    CO_TRY(c, st, ncclAllGather(d, d + cnt, cnt, ncclFloat64, c->nc, st));
    HC_TRY(c, hipMemcpyAsync(all.data(), d + cnt, sizeof(double) * all.size(), hipMemcpyDeviceToHost, st));
  } else {
    CO_TRY(c, st, ncclAllReduce(d, d, cnt, ncclFloat64, ncclSum, c->nc, st));
    HC_TRY(c, hipMemcpyAsync(all.data(), d, sizeof(double) * cnt, hipMemcpyDeviceToHost, st));
  }
  CS_TRY(c, st);
  for (int j = 0; j < k; ++j)
    if (out[j]) layout::apply(layout::vectors_unpack(sh.data(), n, k, j), all.data(), out[j]);
  return RT_OK;
}

}  // namespace

extern "C" rt_status rt_comm_unique_id(void *id) {
  if (!id) return cfail(nullptr, RT_ERR_ARG, "rt_comm_unique_id: NULL id");
  static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "unique id size");
  ncclUniqueId u;
  NC_TRY(nullptr, ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return RT_OK;
}

extern "C" rt_status rt_comm_init(int nranks, int rank, const void *id, int device, rt_comm **out) {
  if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks)
    return cfail(nullptr, RT_ERR_ARG, "rt_comm_init: bad argument");
  *out = nullptr;
  HC_TRY(nullptr, hipSetDevice(device));
  rt_comm *c = new rt_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  c->timeout_s = comm_timeout_s();
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;  // returns at once; the wait below is bounded
  const ncclResult_t r = ncclCommInitRankConfig(&c->nc, nranks, u, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) c->nc = nullptr;
  if (rt_status st = nc_settle(c, r, "ncclCommInitRankConfig")) {
    const std::string msg = c->err;
    delete c;  // aborted (nc cleared) or never created
    return cfail(nullptr, st, msg);
  }
  *out = c;
  return RT_OK;
}

extern "C" void rt_comm_destroy(rt_comm *c) { delete c; }

extern "C" rt_status rt_comm_rank(rt_comm *c, int *nranks, int *rank) {
  if (!c) return cfail(nullptr, RT_ERR_ARG, "rt_comm_rank: NULL comm");
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank;
  return RT_OK;
}

extern "C" rt_status rt_comm_count(rt_comm *c, int *count) {
  if (!c || !count) return cfail(c, RT_ERR_ARG, "rt_comm_count: NULL argument");
  LIVE(c, "rt_comm_count");
  NC_TRY(c, ncclCommCount(c->nc, count));
  return RT_OK;
}

extern "C" const char *rt_comm_last_error(rt_comm *c) { return c ? c->err.c_str() : g_comm_error.c_str(); }

extern "C" rt_status rt_comm_gather_moments(rt_comm *c, rt_solver *s, double *phi, double *F, double *phi_plus) {
  if (!c || !s) return cfail(c, RT_ERR_ARG, "rt_comm_gather_moments: NULL argument");
  LIVE(c, "rt_comm_gather_moments");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<rt_shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const int n = c->nranks;
  const rt_shard &me = sh[c->rank];
  const int N = me.N, Gl = layout::groups_of(me), Gm = layout::max_groups(sh.data(), n);
  const size_t blk = static_cast<size_t>(N) * Gm;  // one field of one rank, padded
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  Scratch buf;
  buf.st = st;
  HC_TRY(c, buf.alloc(sizeof(double) * 3 * blk * (mode == 0 ? n + 1 : 1)));
  double *d = static_cast<double *>(buf.p);
  if (Gl == Gm) {  // the local arrays are the wire block (layout::moments_pack is one contiguous copy)
    RT_TRY(c, s, rt_get_moments_device(s, d, d + blk, d + 2 * blk));
  } else {  // a short shard: its (N, Gl) blocks into the padded (N, Gm) rows
    Scratch tmp;
    tmp.st = st;
    const size_t gn = static_cast<size_t>(N) * Gl;
    HC_TRY(c, tmp.alloc(sizeof(double) * 3 * gn));
    double *t = static_cast<double *>(tmp.p);
    RT_TRY(c, s, rt_get_moments_device(s, t, t + gn, t + 2 * gn));
    HC_TRY(c, hipMemsetAsync(d, 0, sizeof(double) * 3 * blk, st));
    if (rt_status e = run_plan(c, layout::moments_pack(sh.data(), n, c->rank), t, d, hipMemcpyDeviceToDevice, st))
      return e;
  }
  double *want[3] = {phi, F, phi_plus};
  const double *gathered = d;
  if (mode == 1) {  // every rank holds partial sums over its directions of all G groups
    CO_TRY(c, st, ncclAllReduce(d, d, 3 * blk, ncclFloat64, ncclSum, c->nc, st));
  } else {
    CO_TRY(c, st, ncclAllGather(d, d + 3 * blk, 3 * blk, ncclFloat64, c->nc, st));  // [rank][3][N][Gm]
    gathered = d + 3 * blk;
  }
  for (int k = 0; k < 3; ++k)
    if (want[k])
      if (rt_status e = run_plan(c, layout::moments_unpack(sh.data(), n, k), gathered, want[k],
                                 hipMemcpyDeviceToHost, st))
        return e;
  CS_TRY(c, st);
  return RT_OK;
}

extern "C" rt_status rt_comm_gather_group_ends(rt_comm *c, rt_solver *s, double *left, double *right) {
  if (!c || !s) return cfail(c, RT_ERR_ARG, "rt_comm_gather_group_ends: NULL argument");
  LIVE(c, "rt_comm_gather_group_ends");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<rt_shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const int Gl = layout::groups_of(sh[c->rank]);
  std::vector<double> l(Gl), r(Gl);
  RT_TRY(c, s, rt_get_group_ends(s, l.data(), r.data()));
  return combine_vectors(c, s, sh, mode, {l.data(), r.data()}, {left, right});
}

extern "C" rt_status rt_comm_gather_balance(rt_comm *c, rt_solver *s, double *balance, double *sources,
                                            double *sinks) {
  if (!c || !s) return cfail(c, RT_ERR_ARG, "rt_comm_gather_balance: NULL argument");
  LIVE(c, "rt_comm_gather_balance");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<rt_shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const int G = sh[0].G, Gl = layout::groups_of(sh[c->rank]);
  if (mode == 0) {  // each shard's own terms, exactly as one handle computes them
    std::vector<double> b(Gl), so(Gl), si(Gl);
    RT_TRY(c, s, rt_get_balance_terms(s, b.data(), so.data(), si.data()));
    return combine_vectors(c, s, sh, mode, {b.data(), so.data(), si.data()}, {balance, sources, sinks});
  }
  // direction shards: currents and absorption add over directions, the emission is once
  std::vector<double> in(Gl), oa(Gl), em(Gl), jin(G), jout(G);
  RT_TRY(c, s, rt_get_balance_partials(s, in.data(), oa.data(), em.data()));
  if (rt_status st = combine_vectors(c, s, sh, mode, {in.data(), oa.data()}, {jin.data(), jout.data()})) return st;
  for (int g = 0; g < G; ++g) {  // solver.cpp:274-281
    const double so = jin[g] + em[g], si = jout[g];
    if (balance) balance[g] = std::fabs(si - so) / so;
    if (sources) sources[g] = so;
    if (sinks) sinks[g] = si;
  }
  return RT_OK;
}

extern "C" rt_status rt_comm_gather_psi(rt_comm *c, rt_solver *s, int root, double *psi) {
  if (!c || !s || root < 0 || root >= c->nranks || (c->rank == root && !psi))
    return cfail(c, RT_ERR_ARG, "rt_comm_gather_psi: bad argument");
  LIVE(c, "rt_comm_gather_psi");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<rt_shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const rt_shard &me = sh[c->rank];
  auto block = [&](const rt_shard &a) {  // (M_l, Gl, N): i + M_l (g + Gl c)
    return static_cast<size_t>(layout::dirs_of(a)) * layout::groups_of(a) * a.N;
  };
  size_t big = 0;
  for (const rt_shard &a : sh) big = std::max(big, block(a));
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  std::vector<double> mine(block(me));
  RT_TRY(c, s, rt_get_psi(s, mine.data()));
  Scratch buf;
  buf.st = st;
  HC_TRY(c, buf.alloc(sizeof(double) * big * (c->rank == root ? 2 : 1)));
  double *d = static_cast<double *>(buf.p);
  HC_TRY(c, hipMemcpyAsync(d, mine.data(), sizeof(double) * mine.size(), hipMemcpyHostToDevice, st));
  if (c->rank != root) {
    CO_TRY(c, st, ncclSend(d, block(me), ncclFloat64, root, c->nc, st));
    CS_TRY(c, st);
    return RT_OK;
  }
  double *rx = d + big;
  for (int r = 0; r < c->nranks; ++r) {
    const double *src = d;
    if (r != root) {  // one rank's block at a time through the receive buffer
      CO_TRY(c, st, ncclRecv(rx, block(sh[r]), ncclFloat64, r, c->nc, st));
      src = rx;
    }
    if (rt_status e = run_plan(c, layout::psi_place(sh[r]), src, psi, hipMemcpyDeviceToHost, st)) return e;
    CS_TRY(c, st);  // rx is reused by the next rank
  }
  return RT_OK;
}

extern "C" rt_status rt_comm_gather_psi_source(rt_comm *c, rt_solver *s, double *out) {
  if (!c || !s || !out) return cfail(c, RT_ERR_ARG, "rt_comm_gather_psi_source: bad argument");
  LIVE(c, "rt_comm_gather_psi_source");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<rt_shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const int G = sh[0].G;
  if (mode == 0) {  // every group shard holds all M x G rows (the table covers all groups)
    RT_TRY(c, s, rt_get_psi_source(s, out));
    return RT_OK;
  }
  // direction shards: rows m of the shard's (M_l, G) table, ascending mu, into the (M, G) table
  int Hm = 0;
  for (const rt_shard &a : sh) Hm = std::max(Hm, a.d_hi - a.d_lo);
  const size_t cnt = static_cast<size_t>(2) * Hm * G;
  std::vector<double> mine(cnt, 0.0);
  RT_TRY(c, s, rt_get_psi_source(s, mine.data()));
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  Scratch buf;
  buf.st = st;
  HC_TRY(c, buf.alloc(sizeof(double) * cnt * (c->nranks + 1)));
  double *d = static_cast<double *>(buf.p);
  HC_TRY(c, hipMemcpyAsync(d, mine.data(), sizeof(double) * cnt, hipMemcpyHostToDevice, st));
  CO_TRY(c, st, ncclAllGather(d, d + cnt, cnt, ncclFloat64, c->nc, st));
  std::vector<double> all(cnt * c->nranks);
  HC_TRY(c, hipMemcpyAsync(all.data(), d + cnt, sizeof(double) * all.size(), hipMemcpyDeviceToHost, st));
  CS_TRY(c, st);
  for (int r = 0; r < c->nranks; ++r) layout::apply(layout::psi_source_place(sh[r]), all.data() + cnt * r, out);
  return RT_OK;
}

extern "C" rt_status rt_comm_allreduce_absorption(rt_comm *c, rt_solver *s, double *d_out) {
  if (!c || !s || !d_out) return cfail(c, RT_ERR_ARG, "rt_comm_allreduce_absorption: bad argument");
  LIVE(c, "rt_comm_allreduce_absorption");
  HC_TRY(c, hipSetDevice(c->device));
  int N = 0;
  RT_TRY(c, s, rt_get_dims(s, nullptr, nullptr, &N, nullptr, nullptr));
  RT_TRY(c, s, rt_group_absorption_device(s, d_out));
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  CO_TRY(c, st, ncclAllReduce(d_out, d_out, N, ncclFloat64, ncclSum, c->nc, st));
  return RT_OK;
}

extern "C" rt_status rt_comm_material_step(rt_comm *c, rt_solver *s, int nsteps) {
  if (!c || !s || nsteps < 0) return cfail(c, RT_ERR_ARG, "rt_comm_material_step: bad argument");
  LIVE(c, "rt_comm_material_step");
  HC_TRY(c, hipSetDevice(c->device));
  int N = 0;
  RT_TRY(c, s, rt_get_dims(s, nullptr, nullptr, &N, nullptr, nullptr));
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  const size_t len = 2 * static_cast<size_t>(N);  // q and b: one all-reduce per step
  if (c->q_len < len) {
    if (c->q) {
      CS_TRY(c, st);
      HC_TRY(c, hipFree(c->q));
      c->q = nullptr;
    }
    HC_TRY(c, hipMalloc(&c->q, sizeof(double) * len));
    c->q_len = len;
  }
  for (int n = 0; n < nsteps; ++n) {
    RT_TRY(c, s, rt_material_sweep(s, c->q));
    CO_TRY(c, st, ncclAllReduce(c->q, c->q, len, ncclFloat64, ncclSum, c->nc, st));
    RT_TRY(c, s, rt_material_update(s, c->q));
  }
  return RT_OK;
}

extern "C" rt_status rt_comm_synchronize(rt_comm *c, rt_solver *s) {
  if (!c || !s) return cfail(c, RT_ERR_ARG, "rt_comm_synchronize: NULL argument");
  LIVE(c, "rt_comm_synchronize");
  HC_TRY(c, hipSetDevice(c->device));
  CS_TRY(c, static_cast<hipStream_t>(rt_stream(s)));
  return RT_OK;
}

extern "C" rt_status rt_comm_version(int *version, char *path, size_t path_len) {
  if (!version) return cfail(nullptr, RT_ERR_ARG, "rt_comm_version: NULL version");
  NC_TRY(nullptr, ncclGetVersion(version));
  if (path && path_len) {
    Dl_info info{};
    const char *f = dladdr(reinterpret_cast<void *>(&ncclGetVersion), &info) && info.dli_fname ? info.dli_fname : "";
    std::strncpy(path, f, path_len - 1);
    path[path_len - 1] = '\0';
  }
  return RT_OK;
}
