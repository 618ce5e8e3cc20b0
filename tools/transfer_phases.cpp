// transfer_phases -- bin/transfer's run (src/main.cc:60-136 on librtsn) with its cold start
// split into phases, as one JSON line on stdout:
//   exec_to_main  the process start to main(): the dynamic loader, librtsn's and the HIP
//                 runtime's static initialisers (the fat-binary registration) -- from the
//                 launcher's CLOCK_MONOTONIC stamp passed as argv[2] (tools/transfer_phases.py)
//   hip_init      the first HIP call and the device context (hipInit, hipSetDevice, hipFree(0))
//   create        rt::Solver's constructor (Planck table, uploads, init_state: the first
//                 kernel launches, i.e. the code objects' load where it is deferred)
//   solve         the .prm's run (the wavefront kernels' first launch)
//   results       moments, flux, balance, phi_plus, group ends (the read-out kernels)
//   csv           the eight CSV files, into the working directory
//   warm_*        the same create / solve / results a second time in the process
//   teardown      from the end of main to the process's exit (destructors, runtime
//                 teardown): measured by the launcher
// usage: transfer_phases file.prm [t_launch_ns]
#include <hip/hip_runtime.h>
#include <time.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../radiative-transfer_amd/csrc/eigen_text.hpp"
#include "../radiative-transfer_amd/csrc/prm.hpp"
#include "../radiative-transfer_amd/csrc/solver.hpp"

static long long now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

int main(int argc, char **argv) {
  const long long t_main = now_ns();
  if (argc < 2) {
    std::fprintf(stderr, "usage: transfer_phases file.prm [t_launch_ns]\n");
    return 2;
  }
  const long long t_launch = argc > 2 ? std::atoll(argv[2]) : t_main;
  const std::string filename = argv[1];
  const char *tdir = std::getenv("RT_TABLE_DIR");
  rtamd::ParameterHandler ph(filename, tdir ? tdir : "");
  if (ph.status() != RT_OK) {
    std::fprintf(stderr, "%s\n", ph.error().c_str());
    return 1;
  }
  const long long t_prm = now_ns();
  if (hipInit(0) != hipSuccess || hipSetDevice(0) != hipSuccess || hipFree(nullptr) != hipSuccess) {
    std::fprintf(stderr, "no HIP device\n");
    return 1;
  }
  const long long t_hip = now_ns();
  // (PHASES_NO_PROBE unset) the runtime's first-use costs the library pays on its first calls, timed apart: a stream
  // (its hardware queue), the first copy host -> device and device -> host between pinned
  // buffers (the runtime's blit kernels), and a device -> pageable copy (its staging buffer)
  hipStream_t st0;
  double *dbuf = nullptr, *hbuf = nullptr, pageable[8];
  const bool probe = std::getenv("PHASES_NO_PROBE") == nullptr;
  long long t_probe[5] = {t_hip, t_hip, t_hip, t_hip, t_hip};
  if (probe) {
    if (hipStreamCreateWithFlags(&st0, hipStreamNonBlocking) != hipSuccess) return 1;
    t_probe[1] = now_ns();
    if (hipMalloc(&dbuf, 64) != hipSuccess || hipHostMalloc(&hbuf, 64, hipHostMallocDefault) != hipSuccess) return 1;
    if (hipMemcpyAsync(dbuf, hbuf, 64, hipMemcpyHostToDevice, st0) != hipSuccess || hipStreamSynchronize(st0)) return 1;
    t_probe[2] = now_ns();
    if (hipMemcpyAsync(hbuf, dbuf, 64, hipMemcpyDeviceToHost, st0) != hipSuccess || hipStreamSynchronize(st0)) return 1;
    t_probe[3] = now_ns();
    if (hipMemcpyAsync(pageable, dbuf, 64, hipMemcpyDeviceToHost, st0) != hipSuccess || hipStreamSynchronize(st0)) return 1;
    t_probe[4] = now_ns();
  }
  const int M = ph.get_M(), N = ph.get_N(), G = ph.get_G();
  std::vector<double> x(N);
  for (int i = 0; i < N; i++) x[i] = (i + 0.5) * ph.get_dx();
  long long t[2][4], tr[4] = {0, 0, 0, 0};  // tr: the first read-outs one by one
  std::vector<double> psi, phi, F, phi_plus, e_ave, left, right;
  for (int rep = 0; rep < 2; ++rep) {
    t[rep][0] = now_ns();
    rt::Solver solver(ph, psi, phi, F, 0, nullptr);
    t[rep][1] = now_ns();
    solver.solve();
    t[rep][2] = now_ns();
    solver.compute_angle_integrated_intensity();
    if (rep == 0) tr[0] = now_ns();
    solver.compute_radiative_flux();
    if (rep == 0) tr[1] = now_ns();
    solver.compute_balance();
    if (rep == 0) tr[2] = now_ns();
    solver.compute_positive_angle_integrated_intensity();
    solver.get_phi_plus(phi_plus);
    solver.get_e_ave(e_ave);
    if (rep == 0) tr[3] = now_ns();
    solver.compute_group_ends();
    solver.get_ends("left", left);
    solver.get_ends("right", right);
    t[rep][3] = now_ns();
  }
  const long long t_csv0 = now_ns();
  rtamd::write_eigen_text("phi.csv", phi, G, N);
  rtamd::write_eigen_text("phi_plus.csv", phi_plus, G, N);
  rtamd::write_eigen_text("psi.csv", psi, M, static_cast<size_t>(G) * N);
  rtamd::write_eigen_text("x.csv", x, N, 1);
  rtamd::write_eigen_text("F.csv", F, G, N);
  rtamd::write_eigen_text("e_ave.csv", e_ave, G, 1);
  rtamd::write_eigen_text("left_ends.csv", left, G, 1);
  rtamd::write_eigen_text("right_ends.csv", right, G, 1);
  const long long t_csv1 = now_ns();
  auto ms = [](long long a, long long b) { return 1e-6 * static_cast<double>(b - a); };
  std::printf(
      "{\"prm\": \"%s\", \"exec_to_main_ms\": %.4f, \"prm_ms\": %.4f, \"hip_init_ms\": %.4f, \"create_ms\": %.4f, "
      "\"solve_ms\": %.4f, \"results_ms\": %.4f, \"csv_ms\": %.4f, \"warm_create_ms\": %.4f, \"warm_solve_ms\": %.4f, "
      "\"warm_results_ms\": %.4f, \"stream_ms\": %.4f, \"first_h2d_ms\": %.4f, \"first_d2h_ms\": %.4f, "
      "\"first_d2h_pageable_ms\": %.4f, \"first_phi_ms\": %.4f, \"first_F_ms\": %.4f, \"first_balance_ms\": %.4f, "
      "\"first_phi_plus_ms\": %.4f, \"first_group_ends_ms\": %.4f, \"t_end_ns\": %lld}\n",
      filename.c_str(), ms(t_launch, t_main), ms(t_main, t_prm), ms(t_prm, t_hip), ms(t[0][0], t[0][1]),
      ms(t[0][1], t[0][2]), ms(t[0][2], t[0][3]), ms(t_csv0, t_csv1), ms(t[1][0], t[1][1]), ms(t[1][1], t[1][2]),
      ms(t[1][2], t[1][3]), ms(t_probe[0], t_probe[1]), ms(t_probe[1], t_probe[2]), ms(t_probe[2], t_probe[3]),
      ms(t_probe[3], t_probe[4]), ms(t[0][2], tr[0]), ms(tr[0], tr[1]), ms(tr[1], tr[2]), ms(tr[2], tr[3]),
      ms(tr[3], t[0][3]), now_ns());
  std::fflush(stdout);
  return 0;
}
