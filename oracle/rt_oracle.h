/*
 * rt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of Helblindi/radiative-transfer's S_n solver
 * (src/solver.cpp, src/correction.cpp, src/Planck.cpp, src/GLQuad.cpp,
 * src/ParameterHandler.cpp, include/param.h), used as the parity checker for
 * the MI355X product path and as the CPU baseline in bench.py.  Nothing in the
 * product (radiative-transfer_amd/) links, loads or calls this code; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may.
 *
 * Pinning status (see DESIGN.md "Oracle"): the reference cannot be compiled in
 * this image (Eigen3 is absent, and headers include "constants.h" while the
 * file is Constants.h), and it ships no golden vectors.  This restatement is
 * pinned against every known-answer check the reference owns: GrayTest
 * (tests/test_gray.cpp:89, |max F| < 1e-6), Correction::validate_correction
 * (correction.cpp:39-63,100-122), GLQuad symmetry / 4pi weight sum.  Bitwise
 * agreement with Eigen's rounding is NOT pinned ("parity unpinned" at the ulp
 * level); Eigen's PartialPivLU 2x2 inverse is restated from its published
 * algorithm (Eigen 3.3/3.4, LU/PartialPivLU.h unblocked_lu +
 * TriangularSolverMatrix.h small-panel kernel).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Mirrors ParameterHandler's members (include/ParameterHandler.h:11-62) and
 * the defaults of ParameterHandler::get_parameters (ParameterHandler.cpp:100-212). */
typedef struct {
  int M, G, N;
  double efirst, elast, X, dx;
  int bc_left, bc_right;
  int use_mg_equilib;
  int have_group_bounds, have_group_kappa;
  double rho, kappa_grey, T, V;
  int use_correction;
  int ts_method;
  double dt;
  int max_timesteps;
  int include_validation;
  int prm_found;          /* 0 when the .prm could not be opened (ref continues with defaults) */
  double *psi_source;     /* M*G, row m major index m*G+g as parsed (ParameterHandler.cpp:126-132) */
  double *group_bounds;   /* G+1 when have_group_bounds */
  double *group_kappa;    /* G   when have_group_kappa */
} orc_params;

/* Error codes (the reference asserts / exit(1)s instead). */
enum { ORC_OK = 0, ORC_ERR_IO = 1, ORC_ERR_PARSE = 2, ORC_ERR_PARAM = 3, ORC_ERR_VALIDATION = 4, ORC_ERR_NOMEM = 5 };

/* Parse a .prm with the kaityo256/param semantics (param.h:62-75, param.cpp:4-66).
 * Table files are opened at table_dir + name; table_dir NULL means the
 * reference's "../prm/" relative to the CWD (ParameterHandler.cpp:141,172). */
int orc_parse_prm(const char *path, const char *table_dir, orc_params *out);
/* Fill defaults only (the reference's behaviour for a missing .prm). */
void orc_default_params(orc_params *p);
void orc_free_params(orc_params *p);

typedef struct orc_solver orc_solver;

/* half_copy_literal = 1 reproduces solver.cpp:733's per-cell full copy
 * half_ends = ends (quadratic); 0 takes the one copy whose value survives
 * (after the last mu<0 cell of the CN substep) -- identical results.
 * Groups [g_lo, g_hi) are swept; all G groups' coefficients are computed.
 * g_hi <= 0 means G. */
orc_solver *orc_create(const orc_params *p, int half_copy_literal, int g_lo, int g_hi, int *status);
/* OpenMP threads over the lines of one direction (default 1; results do not depend on it) */
void orc_set_threads(orc_solver *s, int threads);
/* CPU baseline only: 1 = the whole-array prev/half snapshot copies (solver.cpp:620-625,
 * 733) split over the OpenMP threads instead of one serial memcpy; results identical.
 * 0 (default) = serial copies, as the reference. */
void orc_set_parallel_copies(orc_solver *s, int on);
void orc_destroy(orc_solver *s);
/* Solver::solve (solver.cpp:590-823). Returns ORC_ERR_VALIDATION where the
 * reference would hit assert(validate_correction()). */
int orc_solve(orc_solver *s);
/* Run `substeps` iterations of solve()'s _it loop starting at _it = it0
 * (used by tests to compare intermediate states). */
int orc_run_substeps(orc_solver *s, int it0, int substeps);

int orc_num_groups_local(const orc_solver *s);
/* psi (M, Gl, N) ColMajor: i + M*(g + Gl*c) -- Eigen::Tensor default (main.cc:88). */
void orc_get_psi(const orc_solver *s, double *out);
/* ends (M, Gl, N, 2) ColMajor. */
void orc_get_ends(const orc_solver *s, double *out);
void orc_set_ends(orc_solver *s, const double *in); /* also sets psi = mean of ends */
/* solver.cpp:191-237, phi/F/phi_plus as (Gl, N) ColMajor g + Gl*c. */
void orc_moments(const orc_solver *s, double *phi, double *F, double *phi_plus);
/* solver.cpp:826-850 */
void orc_group_ends(const orc_solver *s, double *left, double *right);
/* solver.cpp:240-284 (needs phi from orc_moments) */
void orc_balance(const orc_solver *s, const double *phi, double *balance);
/* Quadrature and group data (all G groups). */
void orc_get_quad(const orc_solver *s, double *mu, double *wt);
void orc_get_groups(const orc_solver *s, double *e_edge, double *e_ave, double *de_ave,
                    double *B, double *dBdT, double *kappa);
/* Correction terms per group (correction.cpp:162-277,328-363) */
void orc_get_correction_coeffs(const orc_solver *s, double *dEB, double *dsigEdE,
                               double *dkapEB, double *cor1, double *cor2, double *cor3);
/* Solver-owned psi_source after construction / equilibrium sources (M*G, m*G+g). */
void orc_get_psi_source(const orc_solver *s, double *out);
/* validate_correction() (correction.cpp:366-369): 1 pass, 0 fail. */
int orc_validate(orc_solver *s);

/* Material-temperature coupling (NOT in the reference: the product's
 * rt_material_* of include/rtsn.h restated on the CPU): T updated implicitly in
 * the material's own emission, the emission change carried into the next sweep.
 * Per full step: orc_material_sweep runs the step with the per-cell emission
 * Beff_g = B_g(T^n) + dB_g/dT(T^{n-1}) dT^{n-1} and writes this solver's
 * q(c) = sum_g sigma_g (phi_g - W B_g(T^n)) and b(c) = sum_g sigma_g dB_g/dT(T^n)
 * (2N: q then b); the caller sums both over group shards and calls
 * orc_material_update (dT = dt q / (rho_cv + dt W b), T += dT, the Planck terms
 * at the new T).  Requires the v/c correction off. */
int orc_material_enable(orc_solver *s, double rho_cv, const double *T_cells /* N or NULL */);
int orc_material_sweep(orc_solver *s, double *qb /* 2N */);
void orc_material_update(orc_solver *s, const double *qb /* 2N */);
/* energy per volume the material owes the radiation (dt W sum_g sigma_g owed_g, this solver's groups) */
void orc_get_material_transit(const orc_solver *s, double *E);
void orc_get_temperature(const orc_solver *s, double *T);
void orc_get_cell_planck(const orc_solver *s, double *B);     /* N x Gl, c*Gl + gl: B_g(T(c)) */
void orc_get_cell_emission(const orc_solver *s, double *Beff); /* N x Gl: the next step's emission */
/* kcon x B_g(T) / kcon x dB_g/dT(T) of one group, the last one the grey remainder (see .c) */
double orc_planck_cell(double T, int G, const double *e_edge, int g);
double orc_planck_cell_dBdT(double T, int G, const double *e_edge, int g);

/* Stand-alone building blocks exposed for unit tests. */
void orc_glquad(int M, double norm, double *mu, double *wt);
void orc_planck_groups(double T, int G, const double *e_lo, const double *e_hi,
                       double *B, double *dBdT); /* raw Planck::get_Planck, no kcon */
void orc_eigen_inverse2(const double m[4], double inv[4]); /* row-major in/out */

#ifdef __cplusplus
}
#endif
#endif
