// rtsn_comm.hip -- RCCL behind the C ABI (include/rtsn.h, "multi-GPU").
//
// The reference runs one process (main.cc:79-133).  Here a job runs one process per
// GPU, each holding a shard handle; groups never exchange data while stepping (T is
// constant, solver.cpp:157), so the only collectives are the end-of-run reductions of
// the reference's result arrays and, in the material-coupled mode, one all-reduce of
// q(x) per step.  Every collective is enqueued on the handle's own stream, so it is
// ordered after the sweeps that produce its input without a host synchronisation.
//
// Layouts on the wire (one all-gather per result, each rank's block padded to the
// largest shard so the counts agree):
//   moments  [3][N][Gmax]   (phi, F, phi_plus; g fastest, as rt_get_moments_device)
//   vectors  [k][Gmax]      (group ends, balance terms)
// and the assembly into the (G, N) / (G) arrays is a strided copy per rank.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtsn.h"

struct rt_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
  double *q = nullptr;  // material coupling: q(x) of the running step (N doubles)
  size_t q_len = 0;
  std::string err;
  ~rt_comm() {
    if (q) (void)hipFree(q);
    if (nc) (void)ncclCommDestroy(nc);
  }
};

namespace {

thread_local std::string g_comm_error;

rt_status cfail(rt_comm *c, rt_status st, const std::string &msg) {
  if (c) c->err = msg;
  g_comm_error = msg;
  return st;
}

#define NC_TRY(c, expr)                                                                                    \
  do {                                                                                                     \
    ncclResult_t r_ = (expr);                                                                              \
    if (r_ != ncclSuccess) return cfail((c), RT_ERR_DEVICE, std::string(#expr ": ") + ncclGetErrorString(r_)); \
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

// Device scratch freed on scope exit (after the stream has drained it).
struct Scratch {
  void *p = nullptr;
  hipStream_t st = nullptr;
  ~Scratch() {
    if (p) {
      (void)hipStreamSynchronize(st);
      (void)hipFree(p);
    }
  }
};

struct Shard {
  int G, M, g_lo, g_hi, d_lo, d_hi, N, Gl;
};

// Every rank's shard, and how the shards tile the problem: 0 = group shards covering
// [0, G) in rank order (all directions each), 1 = direction shards covering [0, M/2) in
// rank order over the same groups.
rt_status all_shards(rt_comm *c, rt_solver *s, std::vector<Shard> &out, int &mode) {
  Shard me{};
  RT_TRY(c, s, rt_get_shard(s, &me.G, &me.M, &me.g_lo, &me.g_hi, &me.d_lo, &me.d_hi));
  RT_TRY(c, s, rt_get_dims(s, nullptr, &me.Gl, &me.N, nullptr, nullptr));
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  constexpr int kInts = sizeof(Shard) / sizeof(int);
  Scratch buf;
  buf.st = st;
  HC_TRY(c, hipMalloc(&buf.p, sizeof(int) * kInts * (c->nranks + 1)));
  int *d = static_cast<int *>(buf.p);
  HC_TRY(c, hipMemcpyAsync(d, &me, sizeof(Shard), hipMemcpyHostToDevice, st));
  NC_TRY(c, ncclAllGather(d, d + kInts, kInts, ncclInt32, c->nc, st));
  out.resize(c->nranks);
  HC_TRY(c, hipMemcpyAsync(out.data(), d + kInts, sizeof(Shard) * c->nranks, hipMemcpyDeviceToHost, st));
  HC_TRY(c, hipStreamSynchronize(st));
  const int H = me.M / 2;
  bool groups = true, dirs = true;
  for (int r = 0; r < c->nranks; ++r) {
    const Shard &a = out[r];
    if (a.G != me.G || a.M != me.M || a.N != me.N) return cfail(c, RT_ERR_PARAM, "ranks hold different configurations");
    groups = groups && a.d_lo == 0 && a.d_hi == H && a.g_lo == (r ? out[r - 1].g_hi : 0);
    dirs = dirs && a.g_lo == me.g_lo && a.g_hi == me.g_hi && a.d_lo == (r ? out[r - 1].d_hi : 0);
  }
  groups = groups && out.back().g_hi == me.G;
  dirs = dirs && out.back().d_hi == H && me.g_lo == 0 && me.g_hi == me.G;
  if (groups) {
    mode = 0;
  } else if (dirs) {
    mode = 1;
  } else {
    return cfail(c, RT_ERR_PARAM, "shards must be group shards tiling [0, G) or direction shards tiling [0, M/2), "
                                  "in rank order");
  }
  return RT_OK;
}

int max_groups(const std::vector<Shard> &sh) {
  int m = 0;
  for (const Shard &a : sh) m = std::max(m, a.g_hi - a.g_lo);
  return m;
}

// k host vectors of this rank's Gl groups -> all G groups on every rank: gathered (mode 0)
// or summed (mode 1).  in[j] / out[j] may be NULL (out NULL: not wanted).
rt_status combine_vectors(rt_comm *c, rt_solver *s, const std::vector<Shard> &sh, int mode,
                          const std::vector<const double *> &in, const std::vector<double *> &out) {
  const int k = static_cast<int>(in.size()), G = sh[0].G, Gl = sh[c->rank].Gl, Gm = max_groups(sh);
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  std::vector<double> block(static_cast<size_t>(k) * Gm, 0.0);
  for (int j = 0; j < k; ++j)
    if (in[j]) std::copy(in[j], in[j] + Gl, block.begin() + static_cast<size_t>(j) * Gm);
  Scratch buf;
  buf.st = st;
  const size_t cnt = static_cast<size_t>(k) * Gm;
  HC_TRY(c, hipMalloc(&buf.p, sizeof(double) * cnt * (c->nranks + 1)));
  double *d = static_cast<double *>(buf.p);
  HC_TRY(c, hipMemcpyAsync(d, block.data(), sizeof(double) * cnt, hipMemcpyHostToDevice, st));
  std::vector<double> all;
  if (mode == 0) {
    NC_TRY(c, ncclAllGather(d, d + cnt, cnt, ncclFloat64, c->nc, st));
    all.resize(cnt * c->nranks);
    HC_TRY(c, hipMemcpyAsync(all.data(), d + cnt, sizeof(double) * all.size(), hipMemcpyDeviceToHost, st));
  } else {
    NC_TRY(c, ncclAllReduce(d, d, cnt, ncclFloat64, ncclSum, c->nc, st));
    all.resize(cnt);
    HC_TRY(c, hipMemcpyAsync(all.data(), d, sizeof(double) * cnt, hipMemcpyDeviceToHost, st));
  }
  HC_TRY(c, hipStreamSynchronize(st));
  for (int j = 0; j < k; ++j) {
    if (!out[j]) continue;
    if (mode == 1) {
      std::copy(all.begin() + static_cast<size_t>(j) * Gm, all.begin() + static_cast<size_t>(j) * Gm + G, out[j]);
      continue;
    }
    for (int r = 0; r < c->nranks; ++r) {
      const double *src = all.data() + cnt * r + static_cast<size_t>(j) * Gm;
      std::copy(src, src + sh[r].Gl, out[j] + sh[r].g_lo);
    }
  }
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
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->nc, nranks, u, rank);
  if (r != ncclSuccess) {
    c->nc = nullptr;
    delete c;
    return cfail(nullptr, RT_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
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

extern "C" const char *rt_comm_last_error(rt_comm *c) { return c ? c->err.c_str() : g_comm_error.c_str(); }

extern "C" rt_status rt_comm_gather_moments(rt_comm *c, rt_solver *s, double *phi, double *F, double *phi_plus) {
  if (!c || !s) return cfail(c, RT_ERR_ARG, "rt_comm_gather_moments: NULL argument");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<Shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const Shard &me = sh[c->rank];
  const int N = me.N, G = me.G, Gm = max_groups(sh);
  const size_t blk = static_cast<size_t>(N) * Gm;  // one field of one rank, padded
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  Scratch buf;
  buf.st = st;
  HC_TRY(c, hipMalloc(&buf.p, sizeof(double) * 3 * blk * (mode == 0 ? c->nranks + 1 : 1)));
  double *d = static_cast<double *>(buf.p);
  if (me.Gl == Gm) {
    RT_TRY(c, s, rt_get_moments_device(s, d, d + blk, d + 2 * blk));
  } else {  // a short shard: its (N, Gl) blocks into the padded (N, Gm) rows
    Scratch tmp;
    tmp.st = st;
    const size_t gn = static_cast<size_t>(N) * me.Gl;
    HC_TRY(c, hipMalloc(&tmp.p, sizeof(double) * 3 * gn));
    double *t = static_cast<double *>(tmp.p);
    RT_TRY(c, s, rt_get_moments_device(s, t, t + gn, t + 2 * gn));
    HC_TRY(c, hipMemsetAsync(d, 0, sizeof(double) * 3 * blk, st));
    for (int k = 0; k < 3; ++k)
      HC_TRY(c, hipMemcpy2DAsync(d + k * blk, sizeof(double) * Gm, t + k * gn, sizeof(double) * me.Gl,
                                 sizeof(double) * me.Gl, N, hipMemcpyDeviceToDevice, st));
  }
  double *want[3] = {phi, F, phi_plus};
  if (mode == 1) {  // every rank holds partial sums over its directions of all G groups
    NC_TRY(c, ncclAllReduce(d, d, 3 * blk, ncclFloat64, ncclSum, c->nc, st));
    for (int k = 0; k < 3; ++k)
      if (want[k]) HC_TRY(c, hipMemcpyAsync(want[k], d + k * blk, sizeof(double) * blk, hipMemcpyDeviceToHost, st));
  } else {
    double *all = d + 3 * blk;  // [rank][3][N][Gm]
    NC_TRY(c, ncclAllGather(d, all, 3 * blk, ncclFloat64, c->nc, st));
    for (int r = 0; r < c->nranks; ++r)
      for (int k = 0; k < 3; ++k)
        if (want[k] && sh[r].Gl > 0)
          HC_TRY(c, hipMemcpy2DAsync(want[k] + sh[r].g_lo, sizeof(double) * G, all + (3 * r + k) * blk,
                                     sizeof(double) * Gm, sizeof(double) * sh[r].Gl, N, hipMemcpyDeviceToHost, st));
  }
  HC_TRY(c, hipStreamSynchronize(st));
  return RT_OK;
}

extern "C" rt_status rt_comm_gather_group_ends(rt_comm *c, rt_solver *s, double *left, double *right) {
  if (!c || !s) return cfail(c, RT_ERR_ARG, "rt_comm_gather_group_ends: NULL argument");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<Shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const int Gl = sh[c->rank].Gl;
  std::vector<double> l(Gl), r(Gl);
  RT_TRY(c, s, rt_get_group_ends(s, l.data(), r.data()));
  return combine_vectors(c, s, sh, mode, {l.data(), r.data()}, {left, right});
}

extern "C" rt_status rt_comm_gather_balance(rt_comm *c, rt_solver *s, double *balance, double *sources,
                                            double *sinks) {
  if (!c || !s) return cfail(c, RT_ERR_ARG, "rt_comm_gather_balance: NULL argument");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<Shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const int G = sh[0].G, Gl = sh[c->rank].Gl;
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
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<Shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const Shard &me = sh[c->rank];
  const int N = me.N, G = me.G, M = me.M, H = M / 2;
  auto Ml = [&](const Shard &a) { return 2 * (a.d_hi - a.d_lo); };  // directions a shard holds
  auto block = [&](const Shard &a) { return static_cast<size_t>(Ml(a)) * a.Gl * N; };
  size_t big = 0;
  for (const Shard &a : sh) big = std::max(big, block(a));
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  std::vector<double> mine(block(me));
  RT_TRY(c, s, rt_get_psi(s, mine.data()));  // (Ml, Gl, N): i + Ml (g + Gl c)
  Scratch buf;
  buf.st = st;
  HC_TRY(c, hipMalloc(&buf.p, sizeof(double) * big * (c->rank == root ? 2 : 1)));
  double *d = static_cast<double *>(buf.p);
  HC_TRY(c, hipMemcpyAsync(d, mine.data(), sizeof(double) * mine.size(), hipMemcpyHostToDevice, st));
  if (c->rank != root) {
    NC_TRY(c, ncclSend(d, block(me), ncclFloat64, root, c->nc, st));
    HC_TRY(c, hipStreamSynchronize(st));
    return RT_OK;
  }
  double *rx = d + big;
  for (int r = 0; r < c->nranks; ++r) {
    const Shard &a = sh[r];
    const double *src = d;
    if (r != root) {  // one rank's block at a time through the receive buffer
      NC_TRY(c, ncclRecv(rx, block(a), ncclFloat64, r, c->nc, st));
      src = rx;
    }
    const int ml = Ml(a), n = a.d_hi - a.d_lo;
    // rows (g, c) of the shard's block hold its directions i' in [H - d_hi, H - d_lo) then
    // [H + d_lo, H + d_hi): two strided copies into the (M, G, N) rows i + M (g + G c)
    const size_t rows = static_cast<size_t>(a.Gl) * N;
    if (mode == 0) {  // all directions, groups [g_lo, g_hi): one contiguous run of M Gl per cell
      HC_TRY(c, hipMemcpy2DAsync(psi + static_cast<size_t>(M) * a.g_lo, sizeof(double) * M * G, src,
                                 sizeof(double) * M * a.Gl, sizeof(double) * M * a.Gl, N, hipMemcpyDeviceToHost, st));
    } else {
      HC_TRY(c, hipMemcpy2DAsync(psi + (H - a.d_hi), sizeof(double) * M, src, sizeof(double) * ml, sizeof(double) * n,
                                 rows, hipMemcpyDeviceToHost, st));
      HC_TRY(c, hipMemcpy2DAsync(psi + (H + a.d_lo), sizeof(double) * M, src + n, sizeof(double) * ml,
                                 sizeof(double) * n, rows, hipMemcpyDeviceToHost, st));
    }
    HC_TRY(c, hipStreamSynchronize(st));  // rx is reused by the next rank
  }
  return RT_OK;
}

extern "C" rt_status rt_comm_gather_psi_source(rt_comm *c, rt_solver *s, double *out) {
  if (!c || !s || !out) return cfail(c, RT_ERR_ARG, "rt_comm_gather_psi_source: bad argument");
  HC_TRY(c, hipSetDevice(c->device));
  std::vector<Shard> sh;
  int mode = 0;
  if (rt_status st = all_shards(c, s, sh, mode)) return st;
  const Shard &me = sh[c->rank];
  const int G = me.G, M = me.M, H = M / 2;
  if (mode == 0) {  // every group shard holds all M x G rows (the table covers all groups)
    RT_TRY(c, s, rt_get_psi_source(s, out));
    return RT_OK;
  }
  // direction shards: rows m of the shard's (M_l, G) table, ascending mu, into the (M, G) table
  int Hm = 0;
  for (const Shard &a : sh) Hm = std::max(Hm, a.d_hi - a.d_lo);
  const size_t cnt = static_cast<size_t>(2) * Hm * G;
  std::vector<double> mine(cnt, 0.0);
  RT_TRY(c, s, rt_get_psi_source(s, mine.data()));
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  Scratch buf;
  buf.st = st;
  HC_TRY(c, hipMalloc(&buf.p, sizeof(double) * cnt * (c->nranks + 1)));
  double *d = static_cast<double *>(buf.p);
  HC_TRY(c, hipMemcpyAsync(d, mine.data(), sizeof(double) * cnt, hipMemcpyHostToDevice, st));
  NC_TRY(c, ncclAllGather(d, d + cnt, cnt, ncclFloat64, c->nc, st));
  std::vector<double> all(cnt * c->nranks);
  HC_TRY(c, hipMemcpyAsync(all.data(), d + cnt, sizeof(double) * all.size(), hipMemcpyDeviceToHost, st));
  HC_TRY(c, hipStreamSynchronize(st));
  for (int r = 0; r < c->nranks; ++r) {
    const Shard &a = sh[r];
    const int n = a.d_hi - a.d_lo;
    const double *src = all.data() + cnt * r;
    for (int k = 0; k < 2 * n; ++k) {  // shard row k -> global direction (see rt_create_direction_shard)
      const int i = k < n ? H - a.d_hi + k : H + a.d_lo + (k - n);
      std::copy(src + static_cast<size_t>(k) * G, src + static_cast<size_t>(k + 1) * G, out + static_cast<size_t>(i) * G);
    }
  }
  return RT_OK;
}

extern "C" rt_status rt_comm_allreduce_absorption(rt_comm *c, rt_solver *s, double *d_out) {
  if (!c || !s || !d_out) return cfail(c, RT_ERR_ARG, "rt_comm_allreduce_absorption: bad argument");
  HC_TRY(c, hipSetDevice(c->device));
  int N = 0;
  RT_TRY(c, s, rt_get_dims(s, nullptr, nullptr, &N, nullptr, nullptr));
  RT_TRY(c, s, rt_group_absorption_device(s, d_out));
  NC_TRY(c, ncclAllReduce(d_out, d_out, N, ncclFloat64, ncclSum, c->nc, static_cast<hipStream_t>(rt_stream(s))));
  return RT_OK;
}

extern "C" rt_status rt_comm_material_step(rt_comm *c, rt_solver *s, int nsteps) {
  if (!c || !s || nsteps < 0) return cfail(c, RT_ERR_ARG, "rt_comm_material_step: bad argument");
  HC_TRY(c, hipSetDevice(c->device));
  int N = 0;
  RT_TRY(c, s, rt_get_dims(s, nullptr, nullptr, &N, nullptr, nullptr));
  hipStream_t st = static_cast<hipStream_t>(rt_stream(s));
  if (c->q_len < static_cast<size_t>(N)) {
    if (c->q) {
      HC_TRY(c, hipStreamSynchronize(st));
      HC_TRY(c, hipFree(c->q));
      c->q = nullptr;
    }
    HC_TRY(c, hipMalloc(&c->q, sizeof(double) * N));
    c->q_len = N;
  }
  for (int n = 0; n < nsteps; ++n) {
    RT_TRY(c, s, rt_material_sweep(s, c->q));
    NC_TRY(c, ncclAllReduce(c->q, c->q, N, ncclFloat64, ncclSum, c->nc, st));
    RT_TRY(c, s, rt_material_update(s, c->q));
  }
  return RT_OK;
}
