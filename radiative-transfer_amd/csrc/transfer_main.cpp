// transfer -- the reference's CLI (src/main.cc:60-136) on the MI355X solver.
//   transfer [file.prm]
// Writes phi.csv phi_plus.csv psi.csv x.csv F.csv e_ave.csv left_ends.csv
// right_ends.csv to the working directory in Eigen's default text format.
// Group tables are read from "../prm/" relative to the working directory, as
// in the reference (RT_TABLE_DIR overrides).  With no argument the default
// file is $TRANSFER_DIR/prm/default.prm (TRANSFER_DIR as in
// config/var-config.h.in; default: <repo>/tests/golden/).
//
// Multi-GPU (beyond the reference): RTSN_RANKS=n runs n ranks, one per GPU (device =
// rank + RTSN_DEVICE_BASE), as n child processes forked before any device call.  Each
// holds a shard (rt::Ranks: contiguous groups, or direction pairs when G < n) joined by
// an RCCL communicator whose unique id rank 0 makes and hands to the others through
// pipes; rank 0 prints and writes the CSV files (of all groups), the others are quiet.
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <csignal>

#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "eigen_text.hpp"
#include "prm.hpp"
#include "solver.hpp"
#include "transfer_dir.hpp"

namespace {

struct RankSetup {
  int nranks = 1, rank = 0, device = 0;
  char comm_id[RT_COMM_ID_BYTES] = {};
};

bool write_all(int fd, const char *p, size_t n) {
  while (n) {
    const ssize_t k = write(fd, p, n);
    if (k <= 0) return false;
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

bool read_all(int fd, char *p, size_t n) {
  while (n) {
    const ssize_t k = read(fd, p, n);
    if (k <= 0) return false;
    p += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

// Parent: fork the ranks and reap them (returns main's exit code: 0 when every rank
// succeeded).  Child: returns -1 with *rs filled in.  All pipes exist before the first
// fork; rank 0 makes the communicator id and writes it into the pipe of every rank > 0.
// A rank that fails after the hand-off (no device, a bad .prm, ...) would leave the others
// blocked in ncclCommInitRank or a collective: the parent reaps whichever rank ends first
// and, on the first failure, stops the rest (SIGTERM, SIGKILL after a grace period).
// Fault injection (tests): RTSN_FAULT_STALL_RANK=r makes rank r block right after the fork,
// standing in for a rank stuck in a collective.
int spawn_ranks(int n, RankSetup *rs) {
  const char *base = std::getenv("RTSN_DEVICE_BASE");
  const int dev0 = base ? std::atoi(base) : 0;
  const char *stall = std::getenv("RTSN_FAULT_STALL_RANK");
  const int stall_rank = stall ? std::atoi(stall) : -1;
  std::vector<int> rd(n, -1), wr(n, -1);
  for (int r = 1; r < n; ++r) {
    int fds[2];
    if (pipe(fds) != 0) return 1;
    rd[r] = fds[0];
    wr[r] = fds[1];
  }
  std::cout.flush();
  std::vector<pid_t> kids;
  for (int r = 0; r < n; ++r) {
    const pid_t pid = fork();
    if (pid < 0) {
      for (pid_t k : kids) kill(k, SIGKILL);
      for (pid_t k : kids) waitpid(k, nullptr, 0);
      return 1;
    }
    if (pid > 0) {
      kids.push_back(pid);
      continue;
    }
    rs->nranks = n;
    rs->rank = r;
    rs->device = dev0 + r;
    for (int q = 1; q < n; ++q) {
      if (q != r) close(rd[q]);
      if (r != 0) close(wr[q]);
    }
    if (r == stall_rank)
      for (;;) pause();
    if (r == 0) {
      const bool ok = rt_comm_unique_id(rs->comm_id) == RT_OK;
      if (!ok) std::cerr << "rt_comm_unique_id: " << rt_comm_last_error(nullptr) << std::endl;
      for (int q = 1; q < n; ++q) {
        if (ok) write_all(wr[q], rs->comm_id, RT_COMM_ID_BYTES);
        close(wr[q]);  // a failed rank 0 leaves the others at end of file
      }
      if (!ok) std::exit(2);
    } else {
      const bool ok = read_all(rd[r], rs->comm_id, RT_COMM_ID_BYTES);
      close(rd[r]);
      if (!ok) std::exit(2);
    }
    return -1;
  }
  for (int q = 1; q < n; ++q) {
    close(rd[q]);
    close(wr[q]);
  }
  int code = 0;
  size_t live = kids.size();
  auto forget = [&](pid_t k) {
    for (pid_t &x : kids)
      if (x == k) x = 0;
  };
  while (live) {
    int st = 0;
    const pid_t k = waitpid(-1, &st, 0);
    if (k < 0) {
      if (errno == EINTR) continue;
      code = code ? code : 1;
      break;
    }
    bool known = false;
    for (pid_t x : kids) known = known || x == k;
    if (!known) continue;
    forget(k);
    --live;
    if (WIFEXITED(st) && WEXITSTATUS(st) == 0) continue;
    if (!code) code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
    // first failure: the remaining ranks cannot complete their collectives
    for (pid_t x : kids)
      if (x) kill(x, SIGTERM);
    for (int tick = 0; tick < 50 && live; ++tick) {  // 5 s grace, then SIGKILL
      for (pid_t &x : kids)
        if (x && waitpid(x, nullptr, WNOHANG) == x) {
          x = 0;
          --live;
        }
      if (live) usleep(100000);
    }
    for (pid_t &x : kids)
      if (x) {
        kill(x, SIGKILL);
        waitpid(x, nullptr, 0);
        x = 0;
        --live;
      }
  }
  return code;
}

}  // namespace

int main(int argc, char **argv) {
  RankSetup rs;
  if (const char *nr = std::getenv("RTSN_RANKS")) {
    const int n = std::atoi(nr);
    if (n >= 1) {  // 1: one rank through the communicator path (the one-GPU check of it)
      const int code = spawn_ranks(n, &rs);
      if (code >= 0) return code;  // the parent
    }
  }
  // ranks > 0 run quietly: rank 0 prints what the reference prints and writes the files
  std::ostream quiet(nullptr);
  std::ostream &out = rs.rank == 0 ? std::cout : quiet;
  std::string filename;
  if (argc == 2) {
    filename = argv[1];
  } else if (argc == 1) {
    filename = rtamd::transfer_dir() + "prm/default.prm";
  } else {
    std::cerr << "Too many command line arguments passed in.\n";
  }
  out << "filename: " << filename << std::endl;
  const char *tdir = std::getenv("RT_TABLE_DIR");
  rtamd::ParameterHandler parameter_handler(filename, tdir ? tdir : "");
  out << parameter_handler.load_log();  // get_parameters' own prints (ParameterHandler.cpp:165-195)
  if (parameter_handler.status() != RT_OK) {
    std::cerr << parameter_handler.error() << std::endl;
    return 1;
  }
  parameter_handler.display_input_quantities(out);

  const int M = parameter_handler.get_M(), N = parameter_handler.get_N(), G = parameter_handler.get_G();
  std::vector<double> psi_mat, phi, F, x(N);
  for (int i = 0; i < N; i++) x[i] = (i + 0.5) * parameter_handler.get_dx();

  try {
    // the reference prints as it goes; RTSN_QUIET=1 keeps only the CLI's own lines
    std::ostream *log = std::getenv("RTSN_QUIET") || rs.rank ? nullptr : &std::cout;
    const rt::Ranks ranks{rs.nranks, rs.rank, rs.comm_id};
    rt::Solver solver(parameter_handler, psi_mat, phi, F, rs.device, log, ranks);
    solver.solve();
    solver.compute_angle_integrated_intensity();
    solver.compute_radiative_flux();
    solver.compute_balance();
    std::vector<double> phi_plus;
    solver.compute_positive_angle_integrated_intensity();
    solver.get_phi_plus(phi_plus);

    std::vector<double> e_ave, left_ends, right_ends;
    solver.get_e_ave(e_ave);
    solver.compute_group_ends();  // collective with ranks
    solver.get_ends("left", left_ends);
    solver.get_ends("right", right_ends);
    if (rs.rank == 0) {
      rtamd::write_eigen_text("phi.csv", phi, G, N);
      rtamd::write_eigen_text("phi_plus.csv", phi_plus, G, N);
      rtamd::write_eigen_text("psi.csv", psi_mat, M, static_cast<size_t>(G) * N);
      rtamd::write_eigen_text("x.csv", x, N, 1);
      rtamd::write_eigen_text("F.csv", F, G, N);
      rtamd::write_eigen_text("e_ave.csv", e_ave, G, 1);
      rtamd::write_eigen_text("left_ends.csv", left_ends, G, 1);
      rtamd::write_eigen_text("right_ends.csv", right_ends, G, 1);
    }
  } catch (const rt::SolverError &e) {
    std::cerr << e.what() << std::endl;
    return 2;
  }
  // Every handle is destroyed (its stream drained), the files are closed: leave without the
  // HIP runtime's teardown at exit (~25-35 ms of a ~200 ms llnl_slab_test process,
  // profiles/r06_cold_start.json); the kernel driver reclaims the device state as for any exit.
  std::cout.flush();
  std::cerr.flush();
  _exit(0);
}
