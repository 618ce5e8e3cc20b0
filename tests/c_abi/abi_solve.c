/* C client of the solve path through include/rtsn.h, as a maintainer's C/C++ host would
 * drive it in place of Solver (solver.h:79-97): rt_create from a .prm (tables from the
 * given directory), rt_solve, then the reference's result arrays -- psi, phi / F / phi_plus,
 * group ends, balance, e_ave -- through the host getters, written as raw doubles to
 * argv[3] in that order for the test to compare with the oracle.
 * usage: abi_solve file.prm table_dir/ out.bin */
#include <stdio.h>
#include <stdlib.h>

#include "rtsn.h"

static int put(FILE *f, const double *a, size_t n) { return fwrite(a, sizeof(double), n, f) == n ? 0 : 1; }

int main(int argc, char **argv) {
  rt_solver *s = NULL;
  rt_status st;
  int M, G, N, lo, hi, bad = 0;
  size_t GN, MGN;
  double *psi, *phi, *F, *pp, *left, *right, *bal, *e_ave;
  FILE *f;
  if (argc != 4) return 64;
  st = rt_create(argv[1], argv[2], 0, &s);
  if (st != RT_OK) {
    fprintf(stderr, "rt_create: %s (%s)\n", rt_status_string(st), rt_last_error(NULL));
    return 2;
  }
  if (rt_get_dims(s, &M, &G, &N, &lo, &hi) != RT_OK) return 3;
  if ((st = rt_solve(s)) != RT_OK) {
    fprintf(stderr, "rt_solve: %s (%s)\n", rt_status_string(st), rt_last_error(s));
    return 4;
  }
  GN = (size_t)G * N;
  MGN = (size_t)M * GN;
  psi = malloc(sizeof(double) * MGN);
  phi = malloc(sizeof(double) * GN);
  F = malloc(sizeof(double) * GN);
  pp = malloc(sizeof(double) * GN);
  left = malloc(sizeof(double) * G);
  right = malloc(sizeof(double) * G);
  bal = malloc(sizeof(double) * G);
  e_ave = malloc(sizeof(double) * G);
  if (!psi || !phi || !F || !pp || !left || !right || !bal || !e_ave) return 5;
  bad |= rt_get_psi(s, psi) != RT_OK;
  bad |= rt_get_moments(s, phi, F, pp) != RT_OK;
  bad |= rt_get_group_ends(s, left, right) != RT_OK;
  bad |= rt_get_balance(s, bal) != RT_OK;
  bad |= rt_get_e_ave(s, e_ave) != RT_OK;
  if (bad) {
    fprintf(stderr, "getter failed: %s\n", rt_last_error(s));
    return 6;
  }
  f = fopen(argv[3], "wb");
  if (!f) return 7;
  bad |= put(f, psi, MGN) | put(f, phi, GN) | put(f, F, GN) | put(f, pp, GN);
  bad |= put(f, left, G) | put(f, right, G) | put(f, bal, G) | put(f, e_ave, G);
  fclose(f);
  printf("M=%d G=%d N=%d\n", M, G, N);
  rt_destroy(s);
  free(psi), free(phi), free(F), free(pp), free(left), free(right), free(bal), free(e_ave);
  return bad ? 8 : 0;
}
