// Host Planck group table timing (tools/, not the product): llnl_slab_test's 124 groups,
// PlanckIntegrator::group_integrals as the library runs it, against the same integrals on
// one thread, and the cost of starting k threads that do nothing.  Build:
//   g++ -O2 -std=c++17 -ffp-contract=off -Iradiative-transfer_amd/csrc -Iinclude tools/planck_host.cpp \
//       radiative-transfer_amd/csrc/physics.cpp -o tools/planck_host -lpthread
#include <chrono>
#include <cstdio>
#include <fstream>
#include <thread>
#include <vector>

#include "physics.hpp"

using namespace rtamd::phys;
using clk = std::chrono::steady_clock;

static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

int main(int argc, char **argv) {
  std::vector<double> e;
  double x;
  std::ifstream f(argc > 1 ? argv[1] : "tests/golden/prm/llnl_slab_test_group_bounds.txt");
  while (f >> x) e.push_back(x);
  const int G = static_cast<int>(e.size()) - 1;
  std::vector<double> lo(e.begin(), e.end() - 1), hi(e.begin() + 1, e.end()), B(G), dB(G);
  PlanckIntegrator P;
  double best_lib = 1e9, best_serial = 1e9;
  for (int r = 0; r < 20; ++r) {
    auto t0 = clk::now();
    P.group_integrals(1.0, G, lo.data(), hi.data(), B.data(), dB.data());
    auto t1 = clk::now();
    for (int g = 0; g < G - 1; ++g) {
      volatile double b = P.integral_B(1.0, lo[g], hi[g]);
      volatile double d = P.integral_dBdT(1.0, lo[g], hi[g]);
      (void)b;
      (void)d;
    }
    auto t2 = clk::now();
    best_lib = std::min(best_lib, us(t0, t1));
    best_serial = std::min(best_serial, us(t1, t2));
  }
  std::printf("{\"groups\": %d, \"group_integrals_us\": %.1f, \"serial_us\": %.1f", G, best_lib, best_serial);
  for (int k : {1, 2, 4, 8}) {
    double best = 1e9;
    for (int r = 0; r < 20; ++r) {
      auto t0 = clk::now();
      std::vector<std::thread> pool;
      for (int t = 0; t < k; ++t) pool.emplace_back([] {});
      for (auto &th : pool) th.join();
      best = std::min(best, us(t0, clk::now()));
    }
    std::printf(", \"spawn_join_%d_us\": %.1f", k, best);
  }
  std::printf(", \"hardware_concurrency\": %u}\n", std::thread::hardware_concurrency());
}
