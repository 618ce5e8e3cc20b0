/* C (not C++) client of include/rtsn.h: the header is plain C and the library
 * links from C.  Host-only entry points run anywhere; rt_create_from_params
 * reports the device status (RT_ERR_DEVICE without a gfx950). */
#include <math.h>
#include <stdio.h>

#include "rtsn.h"

int main(void) {
  rt_params p;
  double mu[8], wt[8], e[4] = {0.0, 0.1, 1.0, 10.0}, B[3], dB[3], sum = 0.0;
  rt_solver *s = NULL;
  rt_status st;
  int i;
  rt_params_default(&p);
  if (p.M != 2 || p.ts_method != 3) return 1;
  if (rt_quadrature(8, mu, wt) != RT_OK) return 2;
  for (i = 0; i < 8; ++i) sum += wt[i];
  if (fabs(sum - 4.0 * 3.1415926546) > 1e-9 || mu[0] >= 0.0 || fabs(mu[0] + mu[7]) > 1e-15) return 3;
  if (rt_planck_groups(1.0, 3, e, B, dB) != RT_OK || !(B[0] > 0.0)) return 4;
  if (rt_quadrature(0, mu, wt) != RT_ERR_ARG) return 5;
  st = rt_create_from_params(&p, 0, 0, 0, &s);
  printf("rt_create_from_params: %s (%s)\n", rt_status_string(st), st == RT_OK ? "" : rt_last_error(NULL));
  if (st == RT_OK) {
    int M, G, N, lo, hi;
    if (rt_get_dims(s, &M, &G, &N, &lo, &hi) != RT_OK || M != 2 || N != 100) return 6;
    rt_destroy(s);
  } else if (st != RT_ERR_DEVICE) {
    return 7;
  }
  puts("ok");
  return 0;
}
