// comm_layout.cpp -- see comm_layout.hpp.  Host code only (no HIP): built into librtsn
// with the host objects, so the rt_layout_* entry points work without a GPU.
#include "comm_layout.hpp"

#include <algorithm>
#include <cstring>
#include <string>

namespace rtamd::layout {

namespace {

// one copy; rows that are contiguous on both sides become a single row
void push(std::vector<Copy2D> &plan, Copy2D c) {
  if (c.width == 0 || c.height == 0) return;
  if (c.height > 1 && c.width == c.dpitch && c.width == c.spitch) {
    c.width *= c.height;
    c.dpitch = c.spitch = c.width;
    c.height = 1;
  }
  if (c.height == 1) c.dpitch = c.spitch = c.width;
  plan.push_back(c);
}

}  // namespace

int shard_mode(const rt_shard *sh, int n) {
  if (!sh || n < 1) return -1;
  const rt_shard &f = sh[0];
  if (f.M <= 0 || f.M % 2 || f.G <= 0 || f.N <= 0) return -1;
  const int H = f.M / 2;
  bool groups = true, dirs = true;
  for (int r = 0; r < n; ++r) {
    const rt_shard &a = sh[r];
    if (a.G != f.G || a.M != f.M || a.N != f.N) return -1;
    groups = groups && a.d_lo == 0 && a.d_hi == H && a.g_lo == (r ? sh[r - 1].g_hi : 0) && a.g_lo <= a.g_hi;
    dirs = dirs && a.g_lo == 0 && a.g_hi == f.G && a.d_lo == (r ? sh[r - 1].d_hi : 0) && a.d_lo < a.d_hi;
  }
  groups = groups && sh[n - 1].g_hi == f.G;
  dirs = dirs && sh[n - 1].d_hi == H;
  return groups ? 0 : (dirs ? 1 : -1);
}

int max_groups(const rt_shard *sh, int n) {
  int m = 0;
  for (int r = 0; r < n; ++r) m = std::max(m, groups_of(sh[r]));
  return m;
}

std::vector<Copy2D> moments_pack(const rt_shard *sh, int n, int rank) {
  std::vector<Copy2D> plan;
  const rt_shard &me = sh[rank];
  const size_t N = me.N, Gl = groups_of(me), Gm = max_groups(sh, n);
  for (size_t k = 0; k < 3; ++k) push(plan, {k * N * Gm, Gm, k * N * Gl, Gl, Gl, N});
  return plan;
}

std::vector<Copy2D> moments_unpack(const rt_shard *sh, int n, int field) {
  std::vector<Copy2D> plan;
  const int mode = shard_mode(sh, n);
  const size_t N = sh[0].N, G = sh[0].G, Gm = max_groups(sh, n), k = field;
  if (mode == 1) {  // every rank holds partial sums over its directions of all G groups
    push(plan, {0, G, k * N * Gm, Gm, G, N});
  } else if (mode == 0) {
    for (int r = 0; r < n; ++r)
      push(plan, {static_cast<size_t>(sh[r].g_lo), G, (3 * static_cast<size_t>(r) + k) * N * Gm, Gm,
                  static_cast<size_t>(groups_of(sh[r])), N});
  }
  return plan;
}

std::vector<Copy2D> vectors_pack(const rt_shard *sh, int n, int rank, int k, int j) {
  std::vector<Copy2D> plan;
  (void)k;
  const size_t Gm = max_groups(sh, n), Gl = groups_of(sh[rank]);
  push(plan, {j * Gm, Gl, 0, Gl, Gl, 1});
  return plan;
}

std::vector<Copy2D> vectors_unpack(const rt_shard *sh, int n, int k, int j) {
  std::vector<Copy2D> plan;
  const int mode = shard_mode(sh, n);
  const size_t G = sh[0].G, Gm = max_groups(sh, n);
  if (mode == 1) {
    push(plan, {0, G, j * Gm, G, G, 1});
  } else if (mode == 0) {
    for (int r = 0; r < n; ++r) {
      const size_t Gl = groups_of(sh[r]);
      push(plan, {static_cast<size_t>(sh[r].g_lo), Gl, (static_cast<size_t>(r) * k + j) * Gm, Gl, Gl, 1});
    }
  }
  return plan;
}

std::vector<Copy2D> psi_place(const rt_shard &a) {
  std::vector<Copy2D> plan;
  const size_t M = a.M, G = a.G, N = a.N, H = M / 2, Gl = groups_of(a), nd = a.d_hi - a.d_lo, Ml = 2 * nd;
  if (nd == H) {  // all directions: each cell's M Gl values are one run of the (M, G, N) array
    push(plan, {M * a.g_lo, M * G, 0, M * Gl, M * Gl, N});
  } else if (Gl == G) {  // all groups: the block's rows (g, c) are the array's rows, its directions two runs
    push(plan, {H - a.d_hi, M, 0, Ml, nd, G * N});
    push(plan, {H + a.d_lo, M, nd, Ml, nd, G * N});
  } else {  // a group range of some directions (no rt_comm layout makes these): per cell
    for (size_t c = 0; c < N; ++c) {
      push(plan, {H - a.d_hi + M * (a.g_lo + G * c), M, Ml * Gl * c, Ml, nd, Gl});
      push(plan, {H + a.d_lo + M * (a.g_lo + G * c), M, nd + Ml * Gl * c, Ml, nd, Gl});
    }
  }
  return plan;
}

std::vector<Copy2D> psi_source_place(const rt_shard &a) {
  std::vector<Copy2D> plan;
  const size_t G = a.G, H = a.M / 2, nd = a.d_hi - a.d_lo;
  push(plan, {(H - a.d_hi) * G, nd * G, 0, nd * G, nd * G, 1});   // mu < 0 rows, ascending mu
  push(plan, {(H + a.d_lo) * G, nd * G, nd * G, nd * G, nd * G, 1});
  return plan;
}

void apply(const std::vector<Copy2D> &plan, const double *src, double *dst) {
  for (const Copy2D &c : plan)
    for (size_t r = 0; r < c.height; ++r)
      std::memcpy(dst + c.dst + r * c.dpitch, src + c.src + r * c.spitch, sizeof(double) * c.width);
}

}  // namespace rtamd::layout

// ---------------------------------------------------------------------------
// C ABI (include/rtsn.h "host-side layout of the gathered shard blocks")
// ---------------------------------------------------------------------------
using namespace rtamd::layout;

// rtsn_api.hip: the text rt_last_error(NULL) returns (weak: the plans also build alone, e.g.
// under the host sanitizer, tools/layout_sanitize.cpp)
namespace rtsn_detail {
__attribute__((weak)) void set_last_error(const char *msg);
}

namespace {
rt_status lfail(rt_status st, const char *msg) {
  if (rtsn_detail::set_last_error) rtsn_detail::set_last_error(msg);
  return st;
}
constexpr const char *kBadTiling =
    "shards must be group shards tiling [0, G) in rank order (each d_lo = 0, d_hi = M/2) or direction-pair "
    "shards tiling [0, M/2) (each g_lo = 0, g_hi = G), with equal G, M, N > 0 and M even";
}  // namespace

extern "C" rt_status rt_layout_mode(const rt_shard *shards, int nranks, int *mode, int *max_groups_out) {
  if (!shards || nranks < 1) return lfail(RT_ERR_ARG, "rt_layout_mode: NULL shards or nranks < 1");
  const int m = shard_mode(shards, nranks);
  if (mode) *mode = m;
  if (max_groups_out) *max_groups_out = max_groups(shards, nranks);
  return m < 0 ? lfail(RT_ERR_PARAM, kBadTiling) : RT_OK;
}

extern "C" rt_status rt_layout_pack_moments(const rt_shard *shards, int nranks, int rank, const double *local,
                                            double *block) {
  if (!shards || nranks < 1 || rank < 0 || rank >= nranks || !block)
    return lfail(RT_ERR_ARG, "rt_layout_pack_moments: NULL argument or rank outside [0, nranks)");
  if (shard_mode(shards, nranks) < 0) return lfail(RT_ERR_PARAM, kBadTiling);
  if (!local && groups_of(shards[rank]) > 0)
    return lfail(RT_ERR_ARG, "rt_layout_pack_moments: NULL local moments for a non-empty shard");  // an empty shard has no local arrays
  std::fill(block, block + 3 * static_cast<size_t>(shards[0].N) * max_groups(shards, nranks), 0.0);
  apply(moments_pack(shards, nranks, rank), local, block);
  return RT_OK;
}

extern "C" rt_status rt_layout_unpack_moments(const rt_shard *shards, int nranks, const double *gathered,
                                              double *phi, double *F, double *phi_plus) {
  if (!shards || nranks < 1 || !gathered) return lfail(RT_ERR_ARG, "rt_layout_unpack_moments: NULL argument");
  if (shard_mode(shards, nranks) < 0) return lfail(RT_ERR_PARAM, kBadTiling);
  double *want[3] = {phi, F, phi_plus};
  for (int k = 0; k < 3; ++k)
    if (want[k]) apply(moments_unpack(shards, nranks, k), gathered, want[k]);
  return RT_OK;
}

extern "C" rt_status rt_layout_pack_vectors(const rt_shard *shards, int nranks, int rank, int k,
                                            const double *const *in, double *block) {
  if (!shards || nranks < 1 || rank < 0 || rank >= nranks || k < 1 || !in || !block)
    return lfail(RT_ERR_ARG, "rt_layout_pack_vectors: NULL argument, k < 1 or rank outside [0, nranks)");
  if (shard_mode(shards, nranks) < 0) return lfail(RT_ERR_PARAM, kBadTiling);
  std::fill(block, block + static_cast<size_t>(k) * max_groups(shards, nranks), 0.0);
  for (int j = 0; j < k; ++j)
    if (in[j]) apply(vectors_pack(shards, nranks, rank, k, j), in[j], block);
  return RT_OK;
}

extern "C" rt_status rt_layout_unpack_vectors(const rt_shard *shards, int nranks, int k, const double *gathered,
                                              double *const *out) {
  if (!shards || nranks < 1 || k < 1 || !gathered || !out)
    return lfail(RT_ERR_ARG, "rt_layout_unpack_vectors: NULL argument or k < 1");
  if (shard_mode(shards, nranks) < 0) return lfail(RT_ERR_PARAM, kBadTiling);
  for (int j = 0; j < k; ++j)
    if (out[j]) apply(vectors_unpack(shards, nranks, k, j), gathered, out[j]);
  return RT_OK;
}

extern "C" rt_status rt_layout_place_psi(const rt_shard *shard, const double *block, double *psi) {
  if (!shard || !block || !psi) return lfail(RT_ERR_ARG, "rt_layout_place_psi: NULL argument");
  const rt_shard &a = *shard;
  if (a.M <= 0 || a.M % 2 || a.g_lo < 0 || a.g_lo >= a.g_hi || a.g_hi > a.G || a.d_lo < 0 || a.d_lo >= a.d_hi ||
      a.d_hi > a.M / 2 || a.N <= 0)
    return lfail(RT_ERR_PARAM, "rt_layout_place_psi: the shard needs M > 0 even, 0 <= g_lo < g_hi <= G, "
                               "0 <= d_lo < d_hi <= M/2 and N > 0");
  apply(psi_place(a), block, psi);
  return RT_OK;
}

extern "C" rt_status rt_layout_place_psi_source(const rt_shard *shard, const double *rows, double *psi_source) {
  if (!shard || !rows || !psi_source) return lfail(RT_ERR_ARG, "rt_layout_place_psi_source: NULL argument");
  const rt_shard &a = *shard;
  if (a.M <= 0 || a.M % 2 || a.G <= 0 || a.d_lo < 0 || a.d_lo >= a.d_hi || a.d_hi > a.M / 2)
    return lfail(RT_ERR_PARAM, "rt_layout_place_psi_source: the shard needs M > 0 even, G > 0 and 0 <= d_lo < d_hi <= M/2");
  apply(psi_source_place(a), rows, psi_source);
  return RT_OK;
}
