// solver.hpp -- the reference's Solver class surface (include/solver.h:18-98)
// over the C ABI (include/rtsn.h).  Caller-owned psi/phi/F buffers are
// written through, as Solver writes through its Eigen references
// (solver.cpp:50-53); here they are std::vector<double> in the reference's
// ColMajor layouts (psi: i + M(g + G c); phi, F: g + G c).
#pragma once

#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rtsn.h"
#include "prm.hpp"

namespace rt {

class SolverError : public std::runtime_error {
 public:
  SolverError(rt_status st, const std::string &what) : std::runtime_error(what), status(st) {}
  rt_status status;
};

// One rank of a multi-GPU job (one process per GPU): the ranks split the groups into
// contiguous shards (or, with fewer groups than ranks, the direction pairs) and join
// their handles with an RCCL communicator (include/rtsn.h, rt_comm_*).  comm_id is the
// RT_COMM_ID_BYTES unique id rt_comm_unique_id made on one rank, handed to all.
struct Ranks {
  int nranks = 1, rank = 0;
  const void *comm_id = nullptr;
};

class Solver {
 public:
  // log: where the reference's solver-side messages go (its cout prints:
  // solver.cpp:55-187, 278-282, 310, 623; correction.cpp:56-57, 115-116, 301),
  // in the reference's formats; nullptr = quiet.
  Solver(rtamd::ParameterHandler &parameter_handler, std::vector<double> &psi_mat, std::vector<double> &phi,
         std::vector<double> &F, int device = 0, std::ostream *log = nullptr);
  // Multi-GPU: this rank's shard on `device`.  Every member below is then collective
  // (all ranks call it, in the same order); the result arrays (phi, F, phi_plus,
  // balance, group ends) hold ALL groups on every rank, psi_mat only on rank 0.
  Solver(rtamd::ParameterHandler &parameter_handler, std::vector<double> &psi_mat, std::vector<double> &phi,
         std::vector<double> &F, int device, std::ostream *log, const Ranks &ranks);
  ~Solver();
  Solver(const Solver &) = delete;
  Solver &operator=(const Solver &) = delete;

  void solve();                                          // solver.cpp:590-823
  void compute_angle_integrated_intensity();             // :191-204
  void compute_positive_angle_integrated_intensity();    // :207-221
  void compute_radiative_flux();                         // :224-237
  void compute_balance();                                // :240-284
  void compute_group_ends();                             // :826-850
  void get_balance(std::vector<double> &balance) const { balance = balance_; }
  void get_phi_plus(std::vector<double> &phi_plus) const { phi_plus = phi_plus_; }
  void get_e_ave(std::vector<double> &e_ave) const;
  void get_ends(const std::string &side, std::vector<double> &group_ends) const;  // :853-864

  rt_solver *handle() { return h_; }
  rt_comm *comm() { return comm_; }

 private:
  void check(rt_status st, const char *what) const;
  void create(int device, const Ranks &ranks);
  void moments(double *phi, double *F, double *phi_plus);
  void refresh_psi();
  void print_constructor() const;
  bool validation_report() const;  // Correction::validate_correction with its prints
  rtamd::ParameterHandler &ph_;
  std::vector<double> &psi_, &phi_, &F_;
  std::vector<double> phi_plus_, balance_, left_ends_, right_ends_;
  int M_, G_, N_;
  std::ostream *log_ = nullptr;
  rt_solver *h_ = nullptr;
  rt_comm *comm_ = nullptr;  // multi-GPU only
  int rank_ = 0;
};

}  // namespace rt
