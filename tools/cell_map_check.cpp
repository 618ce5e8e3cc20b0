// cell_map_check -- host check of the per-line affine cell maps (cell.hpp cell_map), which the
// kernels run instead of the reference's cell algebra: for random line constants and every
// scheme, (1) the probe finds the map's structural pattern (every other coefficient exactly
// zero), (2) the reflective mu > 0 head cell's own map (cell_map<S, true>) equals the line's
// map bitwise before head_map_first<S>() -- the rows the wavefront kernels share between the
// head lane and the others -- and (3) both maps reproduce the algebra they were probed from
// (cell_step, cell_step_maybe_head with the mirror's last-substep outflow X[K-1]) on random
// inputs to rounding.  Host code only; tests/test_host.py builds it under ASan + UBSan.
//   g++ -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I radiative-transfer_amd/csrc \
//       tools/cell_map_check.cpp -o /tmp/cell_map_check && /tmp/cell_map_check
#include <cmath>
#include <cstdio>
#include <random>

#include "cell.hpp"

using namespace rtamd;

namespace {

std::mt19937_64 rng(20261015);
double uni(double a, double b) { return std::uniform_real_distribution<double>(a, b)(rng); }

int fails = 0;
double worst = 0.0;

void expect_close(double a, double b, const char *what, int S) {
  const double d = std::fabs(a - b) / (1.0 + std::fabs(b));
  if (d > worst) worst = d;
  if (!(d <= 1e-12)) {
    if (fails < 10) std::printf("scheme %d %s: map %.17g vs algebra %.17g\n", S, what, a, b);
    ++fails;
  }
}

template <int S>
void check(int lines) {
  constexpr int K = SchemeDim<S>::K, WN = map_count<S>(), F = head_map_first<S>();
  for (int n = 0; n < lines; ++n) {
    LineConst L;
    for (double &c : L.c) c = uni(0.1, 2.0);
    const double hd = uni(1e-4, 0.5);
    for (int neg = 0; neg < 2; ++neg) {
      double W[WN];
      if (!cell_map<S>(L, hd, neg != 0, W)) {
        if (fails++ < 10) std::printf("scheme %d: line map not of the structural pattern\n", S);
        continue;
      }
      double X[K], Xc[K], Xn[K], oi, oo, ai, ao;
      for (int r = 0; r < K; ++r) X[r] = Xc[r] = uni(-1.0, 1.0);
      const double pin = uni(-1.0, 1.0), pout = uni(-1.0, 1.0);
      map_apply<S, true>(W, X, pin, pout, Xn, oi, oo);
      cell_step<S>(L, hd, neg != 0, pin, pout, Xc, ai, ao);
      for (int r = 0; r < K; ++r) expect_close(Xn[r], Xc[r], "line map X'", S);
      expect_close(oi, ai, "line map oin", S);
      expect_close(oo, ao, "line map oout", S);
      if (neg) continue;
      // the head cell of a reflective pair (mu > 0 only)
      double Wh[WN];
      if (!cell_map<S, true>(L, hd, false, Wh)) {
        if (fails++ < 10) std::printf("scheme %d: head map not of the structural pattern\n", S);
        continue;
      }
      for (int s = 0; s < F; ++s)
        if (Wh[s] != W[s]) {
          if (fails++ < 10) std::printf("scheme %d: head map slot %d differs from the line map\n", S, s);
        }
      for (int r = 0; r < K; ++r) X[r] = Xc[r] = uni(-1.0, 1.0);
      if constexpr (S == SCHEME_BDF2) X[0] = Xc[0] = X[2];  // head_state: p_up = the half inflow
      if constexpr (S == SCHEME_CN) X[0] = Xc[0] = X[1];
      map_apply<S, true>(Wh, X, pin, pout, Xn, oi, oo);
      cell_step_maybe_head<S>(L, hd, false, pin, pout, Xc, true, Xc[K - 1], ai, ao);
      for (int r = 0; r < K; ++r) expect_close(Xn[r], Xc[r], "head map X'", S);
      expect_close(oi, ai, "head map oin", S);
      expect_close(oo, ao, "head map oout", S);
    }
  }
}

}  // namespace

int main() {
  const int lines = 2000;
  check<SCHEME_BE>(lines);
  check<SCHEME_CN>(lines);
  check<SCHEME_BDF2>(lines);
  std::printf("%d random lines per scheme, %d failures, worst relative difference %.3g\n", lines, fails, worst);
  return fails ? 1 : 0;
}
