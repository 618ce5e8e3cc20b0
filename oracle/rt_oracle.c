/*
 * rt_oracle.c -- TEST INFRASTRUCTURE ONLY (see rt_oracle.h for the contract).
 *
 * A plain-C restatement of Helblindi/radiative-transfer's S_n hot path.  Every
 * function follows the reference's loop order and floating-point expression
 * order so that the restatement reproduces the reference's arithmetic; each
 * block cites the reference file:line it restates.  x86-64 baseline build
 * (no FMA contraction), like the reference's default CMake build.
 */
#define _GNU_SOURCE /* madvise(MADV_HUGEPAGE) */
#include "rt_oracle.h"

#include <ctype.h>
#include <errno.h>
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

/* ---- include/Constants.h:9-23 ------------------------------------------- */
#define C_PLANCK      4.141895e-10   /* keV-sh */
#define C_BOLTZMANN   1.0            /* keV/keV */
#define C_BOLTZ_JPK   1.601558e-25   /* jk/keV */
#define C_LIGHT       299.79245800   /* cm/sh */
#define C_PI          3.1415926546
#define C_FOUR_PI     (4.0 * C_PI)
#define C_RAD_A       1.3653104e-2
#define C_VALID_TOL   1.E-6

static double rad_a_long(void) {
  /* Constants.h:22-23: (8 pi^5 k^4)/(15 h^3 c^3), evaluated with pow at startup */
  return (8.0 * pow(C_PI, 5) * pow(C_BOLTZMANN, 4)) /
         (15.0 * pow(C_PLANCK, 3) * pow(C_LIGHT, 3));
}

/* ======================================================================== */
/* kaityo256/param (include/param.h:62-75, src/param.cpp:4-66)               */
/* ======================================================================== */
typedef struct { char *key; char *val; } kv_t;
typedef struct { kv_t *kv; int n, cap; } kvmap_t;

static const char *kv_find(const kvmap_t *m, const char *key) {
  for (int i = 0; i < m->n; ++i)
    if (strcmp(m->kv[i].key, key) == 0) return m->kv[i].val;
  return NULL;
}

static void kv_insert(kvmap_t *m, const char *key, size_t klen, const char *val) {
  char *k = (char *)malloc(klen + 1);
  memcpy(k, key, klen);
  k[klen] = 0;
  if (kv_find(m, k)) { free(k); return; } /* std::map::insert keeps the first */
  if (m->n == m->cap) {
    m->cap = m->cap ? 2 * m->cap : 32;
    m->kv = (kv_t *)realloc(m->kv, sizeof(kv_t) * m->cap);
  }
  m->kv[m->n].key = k;
  m->kv[m->n].val = strdup(val);
  m->n++;
}

static void kv_free(kvmap_t *m) {
  for (int i = 0; i < m->n; ++i) { free(m->kv[i].key); free(m->kv[i].val); }
  free(m->kv);
  m->kv = NULL;
  m->n = m->cap = 0;
}

/* param.h:62-75: getline; skip lines whose column 0 is '#'; key = text before
 * the first '=', value = everything after it (no trimming). */
static int kv_load(kvmap_t *m, const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return 0;
  size_t cap = 256, len = 0;
  char *line = (char *)malloc(cap);
  int c;
  for (;;) {
    c = fgetc(f);
    if (c == EOF || c == '\n') {
      if (c == EOF && len == 0) break;
      line[len] = 0;
      if (!(len > 0 && line[0] == '#')) {
        char *eq = strchr(line, '=');
        if (eq) kv_insert(m, line, (size_t)(eq - line), eq + 1);
      }
      len = 0;
      if (c == EOF) break;
      continue;
    }
    if (len + 1 >= cap) { cap *= 2; line = (char *)realloc(line, cap); }
    line[len++] = (char)c;
  }
  free(line);
  fclose(f);
  return 1;
}

/* std::stoi (param.cpp:30): strtol base 10; invalid_argument when nothing
 * converts, out_of_range on ERANGE or outside int (the reference terminates). */
static int kv_get_int(const kvmap_t *m, const char *key, int def, int *err) {
  const char *v = kv_find(m, key);
  if (!v) return def;
  char *end;
  errno = 0;
  long x = strtol(v, &end, 10);
  if (end == v || errno == ERANGE || x > INT_MAX || x < INT_MIN) { *err = ORC_ERR_PARSE; return def; }
  return (int)x;
}
/* std::stod (param.cpp:44): strtod; invalid_argument when nothing converts,
 * out_of_range on ERANGE (overflow, or underflow to a subnormal / zero). */
static double kv_get_double(const kvmap_t *m, const char *key, double def, int *err) {
  const char *v = kv_find(m, key);
  if (!v) return def;
  char *end;
  errno = 0;
  double x = strtod(v, &end);
  if (end == v || errno == ERANGE) { *err = ORC_ERR_PARSE; return def; }
  return x;
}
/* param.cpp:5-18: true only for the exact strings yes/Yes/true/True. */
static int kv_get_bool(const kvmap_t *m, const char *key, int def) {
  const char *v = kv_find(m, key);
  if (!v) return def;
  return strcmp(v, "yes") == 0 || strcmp(v, "Yes") == 0 || strcmp(v, "true") == 0 ||
         strcmp(v, "True") == 0;
}

/* `while (stream >> d)` over text (ParameterHandler.cpp:122-128, :152, :184)
 * as libstdc++'s num_get<char> does it in the C locale: skip whitespace; take
 * [+-], digits with at most one '.', then 'e'/'E' (only after a digit) with an
 * optional sign and digits; the token must convert in full (strtod) and must
 * not overflow, else the extraction fails and the loop ends ("inf", "nan",
 * "1e" stop it; "0x10" yields 0; "1.2.3" yields 1.2 and 0.3). */
static int read_doubles(const char *s, double **out, int *n) {
  int cap = 16;
  *n = 0;
  *out = (double *)malloc(sizeof(double) * cap);
  char *tok = (char *)malloc(strlen(s) + 2);
  const char *p = s;
  for (;;) {
    while (*p && isspace((unsigned char)*p)) ++p;
    size_t t = 0;
    if (*p == '+' || *p == '-') tok[t++] = *p++;
    int mant = 0, dec = 0, sci = 0;
    for (;; ++p) {
      const char c = *p;
      if (c >= '0' && c <= '9') { tok[t++] = c; mant = 1; }
      else if (c == '.' && !dec && !sci) { tok[t++] = c; dec = 1; }
      else if ((c == 'e' || c == 'E') && !sci && mant) {
        tok[t++] = 'e';
        sci = 1;
        if (p[1] == '+' || p[1] == '-') tok[t++] = *++p;
      } else break;
    }
    tok[t] = 0;
    if (t == 0) break;
    char *end;
    double d = strtod(tok, &end);
    if (end == tok || *end != 0 || isinf(d)) break;
    if (*n == cap) { cap *= 2; *out = (double *)realloc(*out, sizeof(double) * cap); }
    (*out)[(*n)++] = d;
  }
  free(tok);
  return *n;
}

static char *slurp(const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *buf = (char *)malloc((size_t)sz + 1);
  size_t rd = fread(buf, 1, (size_t)sz, f);
  buf[rd] = 0;
  fclose(f);
  return buf;
}

void orc_default_params(orc_params *p) {
  memset(p, 0, sizeof(*p));
  /* ParameterHandler.cpp:102-211 defaults */
  p->M = 2; p->G = 1; p->efirst = .1; p->elast = 10.; p->X = 1.; p->N = 100;
  p->dx = p->X / p->N;
  p->bc_left = 2; p->bc_right = 1; p->use_mg_equilib = 0;
  p->rho = 1.; p->kappa_grey = 1.; p->T = 1.; p->V = 0.;
  p->use_correction = 0; p->ts_method = 3; p->dt = 0.00001; p->max_timesteps = 1000;
  p->include_validation = 1;
  p->psi_source = (double *)calloc((size_t)p->M * p->G, sizeof(double));
}

void orc_free_params(orc_params *p) {
  free(p->psi_source); free(p->group_bounds); free(p->group_kappa);
  p->psi_source = p->group_bounds = p->group_kappa = NULL;
}

static int read_table(const char *dir, const char *name, int expect, double **out) {
  char path[4096];
  snprintf(path, sizeof path, "%s%s", dir, name);
  char *txt = slurp(path);
  if (!txt) return ORC_ERR_IO; /* ParameterHandler.cpp:146-149: exit(1) */
  double *v; int n;
  read_doubles(txt, &v, &n);
  free(txt);
  if (n != expect) { free(v); return ORC_ERR_PARAM; } /* :163 / :195 asserts */
  *out = v;
  return ORC_OK;
}

/* ParameterHandler::get_parameters (ParameterHandler.cpp:100-212). */
int orc_parse_prm(const char *path, const char *table_dir, orc_params *p) {
  kvmap_t m = {0};
  int err = ORC_OK;
  memset(p, 0, sizeof(*p));
  p->prm_found = kv_load(&m, path); /* param.h:53-60 sets valid=false and goes on */
  p->M = kv_get_int(&m, "M", 2, &err);
  p->G = kv_get_int(&m, "G", 1, &err);
  p->efirst = kv_get_double(&m, "efirst", .1, &err);
  p->elast = kv_get_double(&m, "elast", 10., &err);
  p->X = kv_get_double(&m, "X", 1., &err);
  p->N = kv_get_int(&m, "N", 100, &err);
  p->dx = p->X / p->N;
  p->bc_left = kv_get_int(&m, "bc_left_indicator", 2, &err);
  p->bc_right = kv_get_int(&m, "bc_right_indicator", 1, &err);
  p->use_mg_equilib = kv_get_bool(&m, "use_mg_equilib", 0);
  if (err || p->M <= 0 || p->G <= 0) { kv_free(&m); return err ? err : ORC_ERR_PARAM; }

  p->psi_source = (double *)calloc((size_t)p->M * p->G, sizeof(double));
  if (!p->use_mg_equilib) {
    const char *s = kv_find(&m, "psi_source");
    if (s) {
      double *v; int n;
      read_doubles(s, &v, &n);
      if (n > p->M * p->G) { free(v); kv_free(&m); return ORC_ERR_PARAM; } /* Eigen index assert */
      for (int k = 0; k < n; ++k) {
        int mm = k / p->G, gg = k % p->G;
        p->psi_source[mm * p->G + gg] = v[k];
      }
      free(v);
    }
  }
  const char *dir = table_dir ? table_dir : "../prm/";
  p->have_group_bounds = kv_get_bool(&m, "have_group_bounds", 0);
  if (p->have_group_bounds) {
    const char *name = kv_find(&m, "filename_group_bounds");
    int st = read_table(dir, name ? name : "NA", p->G + 1, &p->group_bounds);
    if (st) { kv_free(&m); return st; }
  }
  p->have_group_kappa = kv_get_bool(&m, "have_group_absorption_opacities", 0);
  if (p->have_group_kappa) {
    const char *name = kv_find(&m, "filename_group_kappa");
    int st = read_table(dir, name ? name : "NA", p->G, &p->group_kappa);
    if (st) { kv_free(&m); return st; }
  }
  p->rho = kv_get_double(&m, "rho", 1., &err);
  p->kappa_grey = kv_get_double(&m, "kappa_grey", 1., &err);
  p->T = kv_get_double(&m, "T", 1., &err);
  p->V = kv_get_double(&m, "V", 0., &err);
  p->use_correction = kv_get_bool(&m, "use_correction", 0);
  p->ts_method = kv_get_int(&m, "ts_method", 3, &err);
  p->dt = kv_get_double(&m, "dt", 0.00001, &err);
  p->max_timesteps = kv_get_int(&m, "max_timesteps", 1000, &err);
  p->include_validation = kv_get_bool(&m, "include_validation", 1);
  kv_free(&m);
  return err;
}

/* ======================================================================== */
/* GLQuad::build (src/GLQuad.cpp:4-44)                                       */
/* ======================================================================== */
void orc_glquad(int M, double norm, double *mu, double *wt) {
  const double tolerance = 1.0e-12; /* GLQuad.h:11 default */
  double x1 = -1.0, x2 = 1.0;
  double xm = 0.5 * (x2 + x1);
  double xl = 0.5 * (x2 - x1);
  double dnp = (double)M;
  int m = (M + 1) / 2;
  for (int i = 1; i <= m; ++i) {
    double di = (double)i;
    double z1, pp, z = cos(C_PI * (di - 0.25) / (dnp + 0.5));
    do {
      double p1 = 1.0, p2 = 0.0;
      for (int j = 1; j <= M; ++j) {
        double dj = (double)j;
        double p3 = p2;
        p2 = p1;
        p1 = ((2.0 * dj - 1.0) * z * p2 - (dj - 1.0) * p3) / dj;
      }
      pp = dnp * (z * p1 - p2) / (z * z - 1.0);
      z1 = z;
      z = z1 - p1 / pp;
    } while (fabs(z - z1) > tolerance);
    mu[i - 1] = xm - xl * z;
    mu[M - i] = xm + xl * z;
    wt[i - 1] = norm * xl / ((1.0 - z * z) * pp * pp);
    wt[M - i] = wt[i - 1];
  }
}

/* ======================================================================== */
/* Planck (src/Planck.cpp:44-337, include/Planck.h:71-125)                  */
/* ======================================================================== */
typedef struct {
  double accuracy;
  long double pts[12], wts[12];
} planck_t;

/* Planck.cpp:231-337 (long double; note j == order+1 in p_deriv, as written) */
static void planck_setup(planck_t *P) {
  const unsigned short order = 12;
  unsigned short midpoint = (order + 1) / 2;
  long double weight_sum = 0;
  long double p_j, p_jm1, p_jm2, p_deriv = 0, mu, old_mu;
  unsigned short i, j;
  P->accuracy = DBL_EPSILON; /* Planck.h:96 default */
  for (i = 0; i < midpoint; i++) {
    mu = cos(C_PI * (i + 0.75) / (order + 0.5));
    int converged = 0;
    while (!converged) {
      p_jm1 = 0;
      p_j = 1;
      for (j = 1; j <= order; j++) {
        p_jm2 = p_jm1;
        p_jm1 = p_j;
        p_j = ((2 * j - 1) * mu * p_jm1 - (j - 1) * p_jm2) / (j);
      }
      p_deriv = j * (mu * p_j - p_jm1) / (mu * mu - 1);
      old_mu = mu;
      mu = old_mu - p_j / p_deriv;
      if (fabsl(mu - old_mu) < P->accuracy) converged = 1;
    }
    P->pts[i] = -mu;
    P->pts[order - 1 - i] = mu;
    P->wts[i] = 1 / ((1 - mu * mu) * p_deriv * p_deriv);
    P->wts[order - 1 - i] = P->wts[i];
    weight_sum += P->wts[i] + P->wts[order - 1 - i];
    if (i == order - 1 - i) weight_sum -= P->wts[i];
  }
  for (i = 0; i < order; i++) P->wts[i] *= 2 / weight_sum;
}

/* Planck.h:84-90 */
static int p_equal(double l, double r) {
  return fabs(l - r) <= DBL_EPSILON * fabs(l + r) * 2 || fabs(l - r) < DBL_MIN;
}

/* Planck.h:96-111 */
static double planck_get_B(double T, double E) {
  if (p_equal(T, 0.0)) return 0.0;
  const double h = C_PLANCK, k = C_BOLTZMANN, c = C_LIGHT;
  return 2.0 * pow(E, 3.0) * pow(h, -3.0) * pow(c, -2.0) / (exp(E / (k * T)) - 1.0);
}

/* Planck.h:113-125 */
static double planck_get_dBdT(double T, double E) {
  if (p_equal(T, 0.0)) return 0.0;
  const double h = C_PLANCK, k = C_BOLTZMANN, c = C_LIGHT;
  return 2.0 * pow(h, -3.0) * pow(c, -2.0) * pow(k, -1.0) * pow(E, 4.0) * pow(T, -2.0) *
         exp(E / (k * T)) * pow(exp(E / (k * T)) - 1.0, -2.0);
}

/* Planck.cpp:94-118 lambda */
static double series_B(const planck_t *P, double z1, double z2) {
  int N = 32;
  double sum1 = exp(-z1) * (z1 * z1 * z1 + 3.0 * z1 * z1 + 6.0 * z1 + 6.0);
  sum1 = sum1 > DBL_EPSILON ? sum1 : DBL_EPSILON; /* std::max(sum1, eps) */
  for (;;) {
    double val = exp(-(N + 1.0) * z1) / (1.0 - exp(-z1)) * pow(N + 1.0, -4.0) *
                 (pow((N + 1.0) * z1, 3.0) + 3.0 * pow((N + 1.0) * z1, 2.0) +
                  6.0 * (N + 1.0) * z1 + 6.0) / sum1;
    if (val > P->accuracy) ++N; else break;
  }
  sum1 = 0.0;
  double sum2 = 0.0;
  for (int n = N; n != 0; --n) {
    sum1 += exp(-n * z1) / pow(n, 4.0) * (pow(n * z1, 3.0) + 3.0 * pow(n * z1, 2.0) + 6.0 * n * z1 + 6.0);
    sum2 += exp(-n * z2) / pow(n, 4.0) * (pow(n * z2, 3.0) + 3.0 * pow(n * z2, 2.0) + 6.0 * n * z2 + 6.0);
  }
  return sum1 - sum2;
}

/* Planck.cpp:170-193 lambda */
static double series_dBdT(const planck_t *P, double z1, double z2) {
  int N = 32;
  double sum1 = exp(-z1) * (pow(z1, 4.0) + 4.0 * pow(z1, 3.0) + 12.0 * z1 * z1 + 24.0 * z1 + 24.0);
  sum1 = sum1 > DBL_EPSILON ? sum1 : DBL_EPSILON;
  for (;;) {
    double val = exp(-(N + 1.0) * z1) / (1.0 - exp(-z1)) * pow(N + 1.0, -4.0) *
                 (pow((N + 1.0) * z1, 4.0) + 4.0 * pow((N + 1.0) * z1, 3.0) +
                  12.0 * pow((N + 1.0) * z1, 2.0) + 24.0 * (N + 1.0) * z1 + 24.0) / sum1;
    if (val > P->accuracy) ++N; else break;
  }
  sum1 = 0.0;
  double sum2 = 0.0;
  for (int n = N; n > 0; --n) {
    sum1 += exp(-n * z1) / pow(n, 4.0) *
            (pow(n * z1, 4.0) + 4.0 * pow(n * z1, 3.0) + 12.0 * pow(n * z1, 2.0) + 24.0 * n * z1 + 24.0);
    sum2 += exp(-n * z2) / pow(n, 4.0) *
            (pow(n * z2, 4.0) + 4.0 * pow(n * z2, 3.0) + 12.0 * pow(n * z2, 2.0) + 24.0 * n * z2 + 24.0);
  }
  return sum1 - sum2;
}

/* gauss += g_map * m_weights[i] * f(T, g_mid + g_map*m_points[i]) with the
 * long-double promotion of Planck.cpp:136-137 / 148-149 / 211-212 / 223-224 */
static double gauss_sum(const planck_t *P, double T, double g_mid, double g_map, int dbdt) {
  double gauss = 0.0;
  for (int i = 0; i < 12; ++i) {
    double E = (double)(g_mid + g_map * P->pts[i]);
    double f = dbdt ? planck_get_dBdT(T, E) : planck_get_B(T, E);
    gauss = (double)(gauss + g_map * P->wts[i] * f);
  }
  return gauss;
}

/* Planck.cpp:85-154 */
static double planck_integrate_B(const planck_t *P, double T, double E_min, double E_max) {
  if (p_equal(T, 0.0) || p_equal(E_min, E_max)) return 0.0;
  const double h = C_PLANCK, k = C_BOLTZMANN, c = C_LIGHT;
  double z1 = E_min / (k * T);
  double z2 = E_max / (k * T);
  double Bg;
  if (z2 <= 0.7) {
    double g_mid = 0.5 * (E_max + E_min);
    double g_map = 0.5 * (E_max - E_min);
    Bg = gauss_sum(P, T, g_mid, g_map, 0);
  } else if (z1 >= 0.5) {
    Bg = 2.0 * pow(k * T, 4.0) * series_B(P, z1, z2) / (pow(h, 3.0) * pow(c, 2.0));
  } else {
    z1 = 0.6;
    double g_mid = 0.5 * (z1 * k * T + E_min);
    double g_map = 0.5 * (z1 * k * T - E_min);
    double gauss = gauss_sum(P, T, g_mid, g_map, 0);
    Bg = gauss + 2.0 * pow(k * T, 4.0) * series_B(P, z1, z2) / (pow(h, 3.0) * pow(c, 2.0));
  }
  return Bg * 4.0 * C_PI;
}

/* Planck.cpp:161-229 */
static double planck_integrate_dBdT(const planck_t *P, double T, double E_min, double E_max) {
  if (p_equal(T, 0.0) || p_equal(E_min, E_max)) return 0.0;
  const double h = C_PLANCK, k = C_BOLTZMANN, c = C_LIGHT;
  double z1 = E_min / (k * T);
  double z2 = E_max / (k * T);
  double dBgdT;
  if (z2 <= 0.7) {
    double g_mid = 0.5 * (E_max + E_min);
    double g_map = 0.5 * (E_max - E_min);
    dBgdT = gauss_sum(P, T, g_mid, g_map, 1);
  } else if (z1 >= 0.5) {
    dBgdT = 2.0 * pow(k, 4.0) * pow(T, 3.0) * series_dBdT(P, z1, z2) / (pow(h, 3.0) * pow(c, 2.0));
  } else {
    z1 = 0.6;
    double g_mid = 0.5 * (z1 * k * T + E_min);
    double g_map = 0.5 * (z1 * k * T - E_min);
    double gauss = gauss_sum(P, T, g_mid, g_map, 1);
    dBgdT = gauss + 2.0 * pow(k, 4.0) * pow(T, 3.0) * series_dBdT(P, z1, z2) / (pow(h, 3.0) * pow(c, 2.0));
  }
  return dBgdT * 4.0 * C_PI;
}

/* Planck.cpp:50-77: B, dBdT keep their last-group value when the remainder
 * is not positive (caller-owned storage). */
static void planck_get(const planck_t *P, double T, int G, const double *e_lo, const double *e_hi,
                       double *B, double *dBdT) {
  double B_sum = rad_a_long() * C_LIGHT * pow(T, 4.0);            /* :79-83 */
  double dBdT_sum = 4.0 * rad_a_long() * C_LIGHT * pow(T, 3.0);   /* :156-159 */
  for (int g = 0; g < G - 1; ++g) {
    double integral = planck_integrate_B(P, T, e_lo[g], e_hi[g]);
    B[g] = integral;
    B_sum -= integral;
    integral = planck_integrate_dBdT(P, T, e_lo[g], e_hi[g]);
    dBdT[g] = integral;
    dBdT_sum -= integral;
  }
  if (B_sum > 0.0) B[G - 1] = B_sum;
  if (dBdT_sum > 0.0) dBdT[G - 1] = dBdT_sum;
}

void orc_planck_groups(double T, int G, const double *e_lo, const double *e_hi, double *B, double *dBdT) {
  planck_t P;
  planck_setup(&P);
  memset(B, 0, sizeof(double) * G);
  memset(dBdT, 0, sizeof(double) * G);
  planck_get(&P, T, G, e_lo, e_hi, B, dBdT);
}

/* ======================================================================== */
/* Eigen: MatrixXd(2,2).inverse() then MatrixXd * VectorXd                   */
/* (Eigen 3.3/3.4 InverseImpl.h compute_inverse<Dynamic> -> PartialPivLU;    */
/*  PartialPivLU.h unblocked_lu; TriangularSolverMatrix.h small-panel loop) */
/* ======================================================================== */
void orc_eigen_inverse2(const double m[4], double inv[4]) {
  /* LU with partial pivoting, k = 0: pivot iff |m10| > |m00| (maxCoeff keeps the first max) */
  double m00 = m[0], m01 = m[1], m10 = m[2], m11 = m[3];
  int swap = fabs(m10) > fabs(m00);
  double u00, u01, l10, u11;
  if (swap) { u00 = m10; u01 = m11; l10 = m00; u11 = m01; }
  else { u00 = m00; u01 = m01; l10 = m10; u11 = m11; }
  if (u00 != 0.0) l10 = l10 / u00;      /* lu.col(k).tail(rrows) /= lu(k,k) */
  u11 = u11 - l10 * u01;                /* bottomRightCorner -= col * row */
  /* dst = P * I */
  double d00, d01, d10, d11;
  if (swap) { d00 = 0.0; d01 = 1.0; d10 = 1.0; d11 = 0.0; }
  else { d00 = 1.0; d01 = 0.0; d10 = 0.0; d11 = 1.0; }
  /* UnitLower solve in place: row1 -= row0 * l10 */
  d10 = d10 - d00 * l10;
  d11 = d11 - d01 * l10;
  /* Upper solve: i = 1 then i = 0; a = 1/tri(i,i); other(i,j) *= a; rows above -= b * tri(s,i) */
  double a1 = 1.0 / u11;
  d10 *= a1;
  d11 *= a1;
  d00 = d00 - d10 * u01;
  d01 = d01 - d11 * u01;
  double a0 = 1.0 / u00;
  d00 *= a0;
  d01 *= a0;
  inv[0] = d00; inv[1] = d01; inv[2] = d10; inv[3] = d11;
}

/* _res = _mat_inverse * _rhs (col-major GEMV: res(i) = A(i,0) x0 + A(i,1) x1) */
static inline void solve2(const double mat[4], const double rhs[2], double res[2]) {
  double inv[4];
  orc_eigen_inverse2(mat, inv);
  res[0] = inv[0] * rhs[0] + inv[1] * rhs[1];
  res[1] = inv[2] * rhs[0] + inv[3] * rhs[1];
}

/* ======================================================================== */
/* Solver + Correction state                                                 */
/* ======================================================================== */
struct orc_solver {
  orc_params p;       /* deep copy */
  int M, G, N, g_lo, Gl;
  double dx, dt;
  int literal_half;
  int threads;        /* OpenMP threads over the lines of a same-sign direction run (orc_set_threads); 1 = serial */
  int par_copies;     /* CPU baseline: the whole-array snapshot copies split over the threads */
  double ac;          /* RADIATION_CONSTANT_A * c (solver.h:29, correction.h:25) */
  double *mu, *wt;
  double *e_edge, *e_ave, *de_ave;
  double *kappa, *rho, *temperature;
  double *B;          /* Solver::B */
  double *dEB_s;      /* Solver::dEB */
  double *psi_source; /* Solver-owned M x G, (i, g) -> i*G + g */
  /* Correction members */
  planck_t planck;
  double *cB, *cdBdT, *kappa_edge, *dEB, *dsigEdE, *dkapEB, *cor1, *cor2, *cor3;
  double *total_correction; /* M x Gl x N ColMajor */
  /* state */
  double *psi, *ends, *prev_ends, *half_ends;
  /* material-temperature coupling (not in the reference; orc_material_*) */
  double *Tcell;      /* N */
  double *Bcell;      /* N x Gl, c*Gl + gl: B_g(T(c)); NULL = the reference's constant-T B_g */
  double *dBcell;     /* N x Gl: dB_g/dT(T(c)) */
  double *Beff;       /* N x Gl: the step's emission B_g(T^n) + the owed emission paid in it */
  double *owed;       /* N x Gl: emission the material owes the radiation, not yet paid (B units) */
  double *dTlast;     /* N: the last update's temperature change (0 before the first) */
  double *bpart;      /* N: sum over the local groups of sigma_g dB_g/dT(T(c)) */
  double rho_cv, wsum;
  int mat_it;         /* substep counter of the coupled steps (_it of solve()) */
  int equil_done;
};

/* emission of cell c, local group gl: per cell when coupled, else B_g (solver.cpp:338,...) */
#define SRC_B(s, gl, c) ((s)->Beff ? (s)->Beff[(size_t)(c) * (s)->Gl + (size_t)(gl)] : (s)->B[(s)->g_lo + (gl)])
#define PSI(s, i, g, c) ((s)->psi[(size_t)(i) + (size_t)(s)->M * ((size_t)(g) + (size_t)(s)->Gl * (size_t)(c))])
#define TC(s, i, g, c) ((s)->total_correction[(size_t)(i) + (size_t)(s)->M * ((size_t)(g) + (size_t)(s)->Gl * (size_t)(c))])
#define E4(arr, s, i, g, c, k) \
  ((arr)[(size_t)(i) + (size_t)(s)->M * ((size_t)(g) + (size_t)(s)->Gl * ((size_t)(c) + (size_t)(s)->N * (size_t)(k)))])

/* Correction::pf (correction.cpp:11-22) */
static double corr_pf(double E, double T) {
  double h = C_PLANCK, c = C_LIGHT, k = C_BOLTZ_JPK;
  double denom = pow(h, 3) * pow(c, 2) * (exp(E / T) - 1.0);
  double val = k * pow(E, 3) / denom;
  return val;
}

/* Correction::generate_planck_integrals (correction.cpp:25-36) */
static void corr_planck(orc_solver *s) {
  int G = s->G;
  double *lo = (double *)malloc(sizeof(double) * G), *hi = (double *)malloc(sizeof(double) * G);
  for (int g = 0; g < G; ++g) { lo[g] = s->e_edge[g]; hi[g] = s->e_edge[g + 1]; }
  planck_get(&s->planck, s->p.T, G, lo, hi, s->cB, s->cdBdT);
  const double kcon = C_BOLTZ_JPK;
  for (int g = 0; g < G; ++g) {
    s->cB[g] = kcon * s->cB[g];
    s->cdBdT[g] = kcon * s->cdBdT[g];
  }
  free(lo);
  free(hi);
}

/* correction.cpp:125-159 */
static void corr_edge_opacities(orc_solver *s) {
  int G = s->G;
  s->kappa_edge[0] = s->kappa[0];
  for (int g = 1; g < G; ++g) {
    double wgt_L = (s->e_ave[g] - s->e_edge[g]) / (s->e_ave[g] - s->e_ave[g - 1]);
    double wgt_R = (s->e_edge[g] - s->e_ave[g - 1]) / (s->e_ave[g] - s->e_ave[g - 1]);
    s->kappa_edge[g] = s->kappa[g - 1] * wgt_L + s->kappa[g] * wgt_R;
  }
  s->kappa_edge[G] = s->kappa[G - 1];
}

/* correction.cpp:162-277 (sums that are only printed are omitted) */
static void corr_components(orc_solver *s) {
  int G = s->G;
  double T = s->p.T;
  const double *ee = s->e_edge, *ke = s->kappa_edge;
  s->dEB[0] = ee[1] * corr_pf(ee[1], T);
  if (G > 1) {
    for (int g = 1; g < G - 1; ++g)
      s->dEB[g] = ee[g + 1] * corr_pf(ee[g + 1], T) - ee[g] * corr_pf(ee[g], T);
    s->dEB[G - 1] = -ee[G - 1] * corr_pf(ee[G - 1], T); /* index G-1, as written (:173) */
  }
  s->dsigEdE[0] = ke[1] * ee[1] / s->de_ave[0];
  for (int g = 1; g < G - 1; ++g)
    s->dsigEdE[g] = (ke[g + 1] * ee[g + 1] - ke[g] * ee[g]) / s->de_ave[g];
  s->dsigEdE[G - 1] = -ke[G] * ee[G] / s->de_ave[G - 1];
  s->dkapEB[0] = ke[1] * ee[1] * corr_pf(ee[1], T);
  if (G > 1) {
    for (int g = 1; g < G - 1; ++g)
      s->dkapEB[g] = ke[g + 1] * ee[g + 1] * corr_pf(ee[g + 1], T) - ke[g] * ee[g] * corr_pf(ee[g], T);
    s->dkapEB[G - 1] = -ke[G - 1] * ee[G - 1] * corr_pf(ee[G - 1], T); /* :248 */
  }
}

/* correction.cpp:328-340: cor1(g) at :338 is a linear index = cor1(g, 0) = dsigEdE(g) */
static void corr_terms(orc_solver *s) {
  for (int g = 0; g < s->G; ++g) {
    s->cor1[g] = s->dsigEdE[g];
    s->cor2[g] = 3.0 * s->rho[g] * s->kappa[g] * s->cB[g] - s->dkapEB[g];
    s->cor3[g] = s->cor1[g] * (4.0 * s->cB[g] - s->dEB[g]);
  }
}

/* Correction::compute_correction (correction.cpp:372-401), local groups only */
static void corr_compute(orc_solver *s) {
  corr_planck(s);
  corr_edge_opacities(s);
  corr_components(s);
  corr_terms(s);
  double beta = s->p.V / C_LIGHT;
#pragma omp parallel for collapse(2) schedule(static) num_threads(s->threads) if (s->threads > 1)
  for (int i = 0; i < s->M; ++i) {
    for (int gl = 0; gl < s->Gl; ++gl) {
      double mu = s->mu[i];
      int g = s->g_lo + gl;
      for (int c = 0; c < s->N; ++c) {
        double val = (s->cor1[g] * PSI(s, i, gl, c) + s->cor2[g]) * mu * beta;
        val -= s->cor3[g] * pow(mu, 2) * pow(beta, 2);
        TC(s, i, gl, c) = val;
      }
    }
  }
}

/* correction.cpp:39-63, 100-122 */
static int corr_validate(orc_solver *s) {
  double bsum = 0., dbsum = 0.;
  for (int g = 0; g < s->G; ++g) { bsum += s->cB[g]; dbsum += s->cdBdT[g]; }
  double acT4 = s->ac * pow(s->p.T, 4);
  double dacT4 = 4.0 * s->ac * pow(s->p.T, 3);
  if (fabs(acT4 - bsum) > C_VALID_TOL || fabs(dacT4 - dbsum) > C_VALID_TOL) return 0;
  double sigacT4 = s->p.kappa_grey * acT4;
  double emis_tot = 0.0;
  for (int g = 0; g < s->G; ++g) emis_tot += s->kappa[g] * s->cB[g];
  if (fabs(emis_tot - sigacT4) > C_VALID_TOL) return 0;
  return 1;
}

int orc_validate(orc_solver *s) { return corr_validate(s); }

/* Zeroed arrays; the large ones (the MGN state arrays) 2 MiB-aligned and marked for
 * transparent huge pages: the reference layout walks a line with a stride of M G doubles,
 * one 4 KiB page per cell on SL-sized arrays, so with 4 KiB pages nearly every access is
 * a TLB miss (CPU-baseline speed only; values unaffected). */
static void *xcalloc(size_t n, size_t sz, int *ok) {
  const size_t bytes = (n ? n : 1) * sz, huge = (size_t)2 << 20;
  void *p = NULL;
  if (bytes >= huge) {
    if (posix_memalign(&p, huge, bytes) != 0) p = NULL;
    if (p) {
#ifdef MADV_HUGEPAGE
      (void)madvise(p, (bytes + huge - 1) / huge * huge, MADV_HUGEPAGE);
#endif
      memset(p, 0, bytes);
    }
  } else {
    p = calloc(n ? n : 1, sz);
  }
  if (!p) *ok = 0;
  return p;
}

/* Solver::Solver (solver.cpp:46-188) */
void orc_set_threads(orc_solver *s, int threads) { s->threads = threads > 0 ? threads : 1; }
void orc_set_parallel_copies(orc_solver *s, int on) { s->par_copies = on; }

orc_solver *orc_create(const orc_params *pin, int half_copy_literal, int g_lo, int g_hi, int *status) {
  *status = ORC_OK;
  if (pin->M <= 0 || (pin->M % 2) != 0 || pin->G <= 0 || pin->N <= 0 ||
      pin->ts_method < 1 || pin->ts_method > 3 || pin->bc_left < 0 || pin->bc_left > 2 ||
      pin->bc_right < 0 || pin->bc_right > 2) {
    *status = ORC_ERR_PARAM;
    return NULL;
  }
  if (g_hi <= 0) g_hi = pin->G;
  if (g_lo < 0 || g_lo >= g_hi || g_hi > pin->G) { *status = ORC_ERR_PARAM; return NULL; }
  orc_solver *s = (orc_solver *)calloc(1, sizeof(orc_solver));
  if (s) s->threads = 1;
  int ok = 1;
  s->p = *pin;
  int M = pin->M, G = pin->G, N = pin->N;
  s->p.psi_source = (double *)xcalloc((size_t)M * G, sizeof(double), &ok);
  if (pin->psi_source) memcpy(s->p.psi_source, pin->psi_source, sizeof(double) * M * G);
  s->p.group_bounds = s->p.group_kappa = NULL;
  s->M = M; s->G = G; s->N = N; s->g_lo = g_lo; s->Gl = g_hi - g_lo;
  s->dx = pin->dx; s->dt = pin->dt;
  s->literal_half = half_copy_literal;
  s->ac = C_RAD_A * C_LIGHT;

  /* :67-73  psi_source is uninitialised unless a BC is "source" -- defined as 0 here */
  s->psi_source = (double *)xcalloc((size_t)M * G, sizeof(double), &ok);
  if (pin->bc_left == 1 || pin->bc_right == 1)
    for (int i = 0; i < M; ++i)
      for (int g = 0; g < G; ++g) s->psi_source[i * G + g] = pin->psi_source ? pin->psi_source[i * G + g] : 0.0;

  /* :76-78 */
  s->mu = (double *)xcalloc(M, sizeof(double), &ok);
  s->wt = (double *)xcalloc(M, sizeof(double), &ok);
  orc_glquad(M, C_FOUR_PI, s->mu, s->wt);

  /* :90-104 group grid */
  s->e_edge = (double *)xcalloc(G + 1, sizeof(double), &ok);
  s->e_ave = (double *)xcalloc(G, sizeof(double), &ok);
  s->de_ave = (double *)xcalloc(G, sizeof(double), &ok);
  if (pin->have_group_bounds && pin->group_bounds) {
    memcpy(s->e_edge, pin->group_bounds, sizeof(double) * (G + 1));
  } else { /* generate_group_edges :6-19 */
    double logfac = (log(pin->elast) - log(pin->efirst)) / (G - 1.0);
    logfac = exp(logfac);
    if (G == 1) logfac = 1.; /* assert(logfac = 1.) assigns */
    s->e_edge[0] = 0.0;
    s->e_edge[1] = pin->efirst;
    for (int g = 1; g < G; ++g) s->e_edge[g + 1] = s->e_edge[g] * logfac;
  }
  s->e_ave[0] = 0.5 * (s->e_edge[0] + s->e_edge[1]); /* :22-32 */
  s->de_ave[0] = s->e_edge[1] - s->e_edge[0];
  for (int g = 1; g < G; ++g) {
    s->e_ave[g] = 0.5 * (s->e_edge[g] + s->e_edge[g + 1]);
    s->de_ave[g] = s->e_edge[g + 1] - s->e_edge[g];
  }

  /* :145-157 */
  s->kappa = (double *)xcalloc(G, sizeof(double), &ok);
  s->rho = (double *)xcalloc(G, sizeof(double), &ok);
  s->temperature = (double *)xcalloc(G, sizeof(double), &ok);
  for (int g = 0; g < G; ++g) {
    s->kappa[g] = (pin->have_group_kappa && pin->group_kappa) ? pin->group_kappa[g] : pin->kappa_grey;
    s->rho[g] = pin->rho;
    s->temperature[g] = pin->T;
  }
  s->B = (double *)xcalloc(G, sizeof(double), &ok);
  s->dEB_s = (double *)xcalloc(G, sizeof(double), &ok);

  /* Correction ctor (correction.cpp:280-325) */
  planck_setup(&s->planck);
  s->cB = (double *)xcalloc(G, sizeof(double), &ok);
  s->cdBdT = (double *)xcalloc(G, sizeof(double), &ok);
  s->kappa_edge = (double *)xcalloc(G + 1, sizeof(double), &ok);
  s->dEB = (double *)xcalloc(G, sizeof(double), &ok);
  s->dsigEdE = (double *)xcalloc(G, sizeof(double), &ok);
  s->dkapEB = (double *)xcalloc(G, sizeof(double), &ok);
  s->cor1 = (double *)xcalloc(G, sizeof(double), &ok);
  s->cor2 = (double *)xcalloc(G, sizeof(double), &ok);
  s->cor3 = (double *)xcalloc(G, sizeof(double), &ok);
  size_t mgn = (size_t)M * s->Gl * N;
  s->total_correction = (double *)xcalloc(mgn, sizeof(double), &ok);
  s->psi = (double *)xcalloc(mgn, sizeof(double), &ok);
  s->ends = (double *)xcalloc(2 * mgn, sizeof(double), &ok);
  s->prev_ends = (double *)xcalloc(2 * mgn, sizeof(double), &ok);
  s->half_ends = (double *)xcalloc(2 * mgn, sizeof(double), &ok);
  if (!ok) { orc_destroy(s); *status = ORC_ERR_NOMEM; return NULL; }
  corr_planck(s);

  /* :165-181 psi = ends = B_g */
  memcpy(s->B, s->cB, sizeof(double) * G);
  for (int i = 0; i < M; ++i)
    for (int gl = 0; gl < s->Gl; ++gl) {
      double val = s->B[g_lo + gl];
      for (int c = 0; c < N; ++c) {
        PSI(s, i, gl, c) = val;
        E4(s->ends, s, i, gl, c, 0) = val;
        E4(s->ends, s, i, gl, c, 1) = val;
      }
    }
  return s;
}

void orc_destroy(orc_solver *s) {
  if (!s) return;
  free(s->p.psi_source);
  free(s->psi_source); free(s->mu); free(s->wt); free(s->e_edge); free(s->e_ave); free(s->de_ave);
  free(s->kappa); free(s->rho); free(s->temperature); free(s->B); free(s->dEB_s);
  free(s->cB); free(s->cdBdT); free(s->kappa_edge); free(s->dEB); free(s->dsigEdE); free(s->dkapEB);
  free(s->cor1); free(s->cor2); free(s->cor3); free(s->total_correction);
  free(s->psi); free(s->ends); free(s->prev_ends); free(s->half_ends);
  free(s->Tcell); free(s->Bcell); free(s->dBcell); free(s->Beff); free(s->owed); free(s->dTlast); free(s->bpart);
  free(s);
}

/* Per-sweep scratch mirroring Solver's members (solver.h:45-53) */
typedef struct { double local_bdry, half_local_bdry, local_bdry_prev_it; } sweep_t;

/* Solver::backwardEuler (solver.cpp:319-404) */
static void cell_be(orc_solver *s, sweep_t *w, int cell, int i, int gl, double timestep, double mu) {
  int g = s->g_lo + gl;
  const double c = C_LIGHT, dx = s->dx;
  double const_A = 1. + c * timestep * s->rho[g] * s->kappa[g];
  double const_B = c * timestep * mu;
  double mat[4], rhs[2], res[2];
  double tv;
  if (mu < 0) {
    tv = (const_A * dx - const_B) / 2.;
    mat[0] = tv; mat[1] = const_B / 2.; mat[2] = -const_B / 2.; mat[3] = tv;
    tv = 0.5 * c * timestep * dx * s->rho[g] * s->kappa[g] * SRC_B(s, gl, cell);
    if (s->p.use_correction) tv += 0.5 * c * timestep * dx * TC(s, i, gl, cell);
    rhs[0] = tv + dx * E4(s->ends, s, i, gl, cell, 0) / 2.;
    rhs[1] = tv - (const_B * w->local_bdry) + dx * E4(s->ends, s, i, gl, cell, 1) / 2.;
    solve2(mat, rhs, res);
    PSI(s, i, gl, cell) = 0.5 * (res[0] + res[1]);
    E4(s->ends, s, i, gl, cell, 0) = res[0];
    E4(s->ends, s, i, gl, cell, 1) = res[1];
    w->local_bdry = res[0];
  } else {
    tv = (const_A * dx + const_B) / 2.;
    mat[0] = tv; mat[1] = const_B / 2.; mat[2] = -const_B / 2.; mat[3] = tv;
    tv = 0.5 * c * timestep * dx * s->rho[g] * s->kappa[g] * SRC_B(s, gl, cell);
    if (s->p.use_correction) tv += 0.5 * c * timestep * dx * TC(s, i, gl, cell);
    rhs[0] = tv + (const_B * w->local_bdry) + dx * E4(s->ends, s, i, gl, cell, 0) / 2.;
    rhs[1] = tv + dx * E4(s->ends, s, i, gl, cell, 1) / 2.;
    solve2(mat, rhs, res);
    PSI(s, i, gl, cell) = 0.5 * (res[0] + res[1]);
    E4(s->ends, s, i, gl, cell, 0) = res[0];
    E4(s->ends, s, i, gl, cell, 1) = res[1];
    w->local_bdry = res[1];
  }
}

/* Solver::crankNicolson (solver.cpp:407-490) */
static void cell_cn(orc_solver *s, sweep_t *w, int cell, int i, int gl, double timestep, double mu) {
  int g = s->g_lo + gl;
  const double c = C_LIGHT, dx = s->dx;
  double tv = 0.5 * c * timestep * s->rho[g] * s->kappa[g];
  double const_A = 0.5 * c * mu * timestep;
  double const_B = 1 + tv;
  double const_C = 1 - tv;
  double mat[4], rhs[2], res[2];
  double e0 = E4(s->ends, s, i, gl, cell, 0), e1 = E4(s->ends, s, i, gl, cell, 1);
  if (mu < 0) {
    tv = 0.5 * (const_B * dx - const_A);
    mat[0] = tv; mat[1] = 0.5 * const_A; mat[2] = -0.5 * const_A; mat[3] = tv;
    tv = 0.5 * c * timestep * dx * s->rho[g] * s->kappa[g] * SRC_B(s, gl, cell);
    if (s->p.use_correction) tv += 0.5 * c * timestep * dx * TC(s, i, gl, cell);
    rhs[0] = tv + 0.5 * (const_C * dx + const_A) * e0 - 0.5 * const_A * e1;
    rhs[1] = tv + 0.5 * const_A * e0 + 0.5 * (const_C * dx + const_A) * e1 -
             const_A * (w->local_bdry_prev_it + w->half_local_bdry);
    solve2(mat, rhs, res);
    PSI(s, i, gl, cell) = 0.5 * (res[0] + res[1]);
    E4(s->ends, s, i, gl, cell, 0) = res[0];
    E4(s->ends, s, i, gl, cell, 1) = res[1];
    w->local_bdry_prev_it = E4(s->prev_ends, s, i, gl, cell, 0);
    w->half_local_bdry = res[0];
  } else {
    tv = 0.5 * (const_A + const_B * dx);
    mat[0] = tv; mat[1] = const_A / 2.; mat[2] = -const_A / 2.; mat[3] = tv;
    tv = 0.5 * c * timestep * dx * s->rho[g] * s->kappa[g] * SRC_B(s, gl, cell);
    if (s->p.use_correction) tv += 0.5 * c * timestep * dx * TC(s, i, gl, cell);
    rhs[0] = tv + 0.5 * (const_C * dx - const_A) * e0 - 0.5 * const_A * e1 +
             const_A * (w->local_bdry_prev_it + w->half_local_bdry);
    rhs[1] = tv + 0.5 * const_A * e0 + 0.5 * (const_C * dx - const_A) * e1;
    solve2(mat, rhs, res);
    PSI(s, i, gl, cell) = 0.5 * (res[0] + res[1]);
    E4(s->ends, s, i, gl, cell, 0) = res[0];
    E4(s->ends, s, i, gl, cell, 1) = res[1];
    w->local_bdry_prev_it = E4(s->prev_ends, s, i, gl, cell, 1);
    w->half_local_bdry = res[1];
  }
}

/* Solver::bdf (solver.cpp:493-587): const_B uses the member dt (:501) */
static void cell_bdf(orc_solver *s, sweep_t *w, int cell, int i, int gl, double timestep, double mu) {
  int g = s->g_lo + gl;
  const double c = C_LIGHT, dx = s->dx;
  double tv = c * s->rho[g] * s->kappa[g] * timestep / 6.;
  double const_A = 1. + tv;
  double const_B = c * mu * s->dt / 6.;
  double const_C = 1. - 4. * tv;
  double const_D = tv;
  double mat[4], rhs[2], res[2];
  double h0 = E4(s->half_ends, s, i, gl, cell, 0), h1 = E4(s->half_ends, s, i, gl, cell, 1);
  double p0 = E4(s->prev_ends, s, i, gl, cell, 0), p1 = E4(s->prev_ends, s, i, gl, cell, 1);
  if (mu < 0) {
    tv = 0.5 * (const_A * dx - const_B);
    mat[0] = tv; mat[1] = 0.5 * const_B; mat[2] = -0.5 * const_B; mat[3] = tv;
    tv = 0.5 * c * timestep * dx * s->rho[g] * s->kappa[g] * SRC_B(s, gl, cell);
    if (s->p.use_correction) tv += 0.5 * c * timestep * dx * TC(s, i, gl, cell);
    rhs[0] = tv + 0.5 * (const_C * dx + 4. * const_B) * h0 - 2. * const_B * h1;
    rhs[0] += 0.5 * (const_B - const_D * dx) * p0 - 0.5 * const_B * p1;
    rhs[1] = tv + 2. * const_B * h0 + 0.5 * (const_C * dx + 4. * const_B) * h1;
    rhs[1] += 0.5 * const_B * p0 + 0.5 * (const_B - const_D * dx) * p1;
    rhs[1] -= const_B * (w->local_bdry + 4. * w->half_local_bdry + w->local_bdry_prev_it);
    solve2(mat, rhs, res);
    PSI(s, i, gl, cell) = 0.5 * (res[0] + res[1]);
    E4(s->ends, s, i, gl, cell, 0) = res[0];
    E4(s->ends, s, i, gl, cell, 1) = res[1];
    w->local_bdry = res[0];
    w->half_local_bdry = h0;
    w->local_bdry_prev_it = p0;
  } else {
    tv = 0.5 * (const_A * dx + const_B);
    mat[0] = tv; mat[1] = 0.5 * const_B; mat[2] = -0.5 * const_B; mat[3] = tv;
    tv = 0.5 * c * timestep * dx * s->rho[g] * s->kappa[g] * SRC_B(s, gl, cell);
    if (s->p.use_correction) tv += 0.5 * c * timestep * dx * TC(s, i, gl, cell);
    rhs[0] = tv + 0.5 * (const_C * dx - 4. * const_B) * h0 - 2. * const_B * h1;
    rhs[0] -= 0.5 * (const_B + const_D * dx) * p0 + 0.5 * const_B * p1;
    rhs[0] += const_B * (w->local_bdry + 4. * w->half_local_bdry + w->local_bdry_prev_it);
    rhs[1] = tv + 2. * const_B * h0 + 0.5 * (const_C * dx - 4. * const_B) * h1;
    rhs[1] += 0.5 * const_B * p0 - 0.5 * (const_B + const_D * dx) * p1;
    solve2(mat, rhs, res);
    PSI(s, i, gl, cell) = 0.5 * (res[0] + res[1]);
    E4(s->ends, s, i, gl, cell, 0) = res[0];
    E4(s->ends, s, i, gl, cell, 1) = res[1];
    w->local_bdry = res[1];
    w->half_local_bdry = h1;
    w->local_bdry_prev_it = p1;
  }
}

/* Solver::computeEquilibriumSources (solver.cpp:287-315) */
static int equilibrium_sources(orc_solver *s) {
  corr_compute(s);
  if (s->p.include_validation && !corr_validate(s)) return ORC_ERR_VALIDATION;
  memcpy(s->B, s->cB, sizeof(double) * s->G);
  memcpy(s->dEB_s, s->dEB, sizeof(double) * s->G);
  for (int i = 0; i < s->M; ++i)
    for (int g = 0; g < s->G; ++g) {
      double val = 4 * s->B[g] - s->dEB_s[g];
      double mult = s->mu[i] * s->p.V / C_LIGHT;
      val *= mult;
      val += s->B[g];
      s->psi_source[i * s->G + g] = val;
    }
  return ORC_OK;
}

static size_t ends_bytes(const orc_solver *s) { return sizeof(double) * 2 * (size_t)s->M * s->Gl * s->N; }

/* One iteration _it of Solver::solve's time loop (solver.cpp:606-819) */
/* One line (i, g) of one substep: boundary value (solver.cpp:635-697) and the
 * cell sweep (:699-816).  *half_pending: a mu<0 CN cell ran (lazy :733 copy). */
static int sweep_line(orc_solver *s, int it, int i, int gl, int *half_pending) {
  const int M = s->M, N = s->N, ts = s->p.ts_method;
  const double dt = s->dt, mu = s->mu[i];
  const int g = s->g_lo + gl;
  double bdry = 0.;
  if (mu < 0.) {
    switch (s->p.bc_right) {
      case 0: bdry = 0.; break;
      case 2: bdry = 0.; break; /* TODO in the reference */
      case 1: bdry = s->psi_source[i * s->G + g]; break;
      default: return ORC_ERR_PARAM;
    }
  } else {
    switch (s->p.bc_left) {
      case 0: /* falls through to source (:668-676) */
      case 1: bdry = s->psi_source[i * s->G + g]; break;
      case 2: {
        int diff = i - (M / 2);
        int m_neg = (M / 2) - 1 - diff;
        bdry = E4(s->ends, s, m_neg, gl, 0, 0);
        break;
      }
      default: return ORC_ERR_PARAM;
    }
  }
  sweep_t w = {bdry, bdry, bdry};
  for (int j = 0; j < N; ++j) {
    int cell = mu < 0 ? N - j - 1 : j;
    switch (ts) {
      case 1: cell_be(s, &w, cell, i, gl, dt, mu); break;
      case 2: cell_cn(s, &w, cell, i, gl, dt, mu); break;
      case 3:
        switch (it % 4) {
          case 0: cell_be(s, &w, cell, i, gl, dt / 2., mu); break;
          case 1:
            cell_cn(s, &w, cell, i, gl, dt / 2., mu);
            if (mu < 0) {
              if (s->literal_half) memcpy(s->half_ends, s->ends, ends_bytes(s));
              else *half_pending = 1;
            }
            break;
          case 2: cell_be(s, &w, cell, i, gl, dt / 2., mu); break;
          case 3: cell_bdf(s, &w, cell, i, gl, dt / 2., mu); break;
        }
        break;
      default: return ORC_ERR_PARAM;
    }
  }
  return ORC_OK;
}

/* memcpy split over the OpenMP threads (same bytes, same result) */
static void par_copy(void *dst, const void *src, size_t bytes, int threads) {
  if (threads <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int t = 0; t < threads; ++t) {
    size_t lo = bytes * (size_t)t / (size_t)threads, hi = bytes * (size_t)(t + 1) / (size_t)threads;
    memcpy((char *)dst + lo, (const char *)src + lo, hi - lo);
  }
}

static int solve_iteration(orc_solver *s, int it) {
  const int M = s->M, ts = s->p.ts_method;
  corr_compute(s);                                           /* :608 */
  if (s->p.include_validation && !corr_validate(s)) return ORC_ERR_VALIDATION; /* :609-612 */
  memcpy(s->B, s->cB, sizeof(double) * s->G);                /* :614 */
  if (ts != 3 || it % 4 == 0) par_copy(s->prev_ends, s->ends, ends_bytes(s), s->par_copies ? s->threads : 1); /* :620-625 */

  int half_copy_pending = 0;
  for (int i = 0; i < M;) {
    const int neg = s->mu[i] < 0.;
    /* Lazy form of :733: the surviving copy is the one after the last mu<0 CN cell. */
    if (half_copy_pending && !neg) {
      par_copy(s->half_ends, s->ends, ends_bytes(s), s->par_copies ? s->threads : 1);
      half_copy_pending = 0;
    }
    /* A run [i, i1) of directions of one sign: its lines (i, g) are independent --
     * groups never couple (T constant), a mu<0 line reads only the right BC, a mu>0
     * line at most the mu<0 outflow of this substep (reflective left BC, :677-684),
     * final before the run starts, and the lazy :733 copy falls between runs. */
    int i1 = i + 1;
    while (i1 < M && (s->mu[i1] < 0.) == neg) ++i1;
    int err = 0, pend = 0;
    const int nl = (i1 - i) * s->Gl;
#pragma omp parallel for schedule(static) num_threads(s->threads) reduction(| : err, pend) if (s->threads > 1 && !s->literal_half)
    for (int l = 0; l < nl; ++l) {
      int hp = 0;
      err |= sweep_line(s, it, i + l / s->Gl, l % s->Gl, &hp);
      pend |= hp;
    }
    if (err) return ORC_ERR_PARAM;
    if (pend) half_copy_pending = 1;
    i = i1;
  }
  if (half_copy_pending) par_copy(s->half_ends, s->ends, ends_bytes(s), s->par_copies ? s->threads : 1);
  return ORC_OK;
}

int orc_run_substeps(orc_solver *s, int it0, int substeps) {
  for (int it = it0; it < it0 + substeps; ++it) {
    int st = solve_iteration(s, it);
    if (st) return st;
  }
  return ORC_OK;
}

/* Solver::solve (solver.cpp:590-605) */
int orc_solve(orc_solver *s) {
  int steps = s->p.max_timesteps;
  if (s->p.ts_method == 3) steps *= 4;
  if (s->p.use_mg_equilib) {
    int st = equilibrium_sources(s);
    if (st) return st;
  }
  return orc_run_substeps(s, 0, steps);
}

/* ======================================================================== */
/* Material-temperature coupling (beyond the reference; include/rtsn.h)      */
/* ======================================================================== */
/* B_g(T) x kcon for one group g: Planck::integrate_B (Planck.cpp:85-154) for
 * g < G-1; the last group is the grey remainder a c T^4 minus the integral
 * over groups 0..G-2 taken as ONE integral over [e_0, e_{G-1}], assigned only
 * when positive (Planck.cpp:73-76), else 0.  T <= 0 or not finite: 0. */
static double planck_cell(const planck_t *P, double T, int G, const double *e_edge, int g) {
  if (!(T > 0.0) || !isfinite(T)) return 0.0;
  if (g < G - 1) return C_BOLTZ_JPK * planck_integrate_B(P, T, e_edge[g], e_edge[g + 1]);
  double rest = rad_a_long() * C_LIGHT * pow(T, 4.0) - planck_integrate_B(P, T, e_edge[0], e_edge[G - 1]);
  return rest > 0.0 ? C_BOLTZ_JPK * rest : 0.0;
}

double orc_planck_cell(double T, int G, const double *e_edge, int g) {
  planck_t P;
  planck_setup(&P);
  return planck_cell(&P, T, G, e_edge, g);
}

/* kcon dB_g/dT(T) for one group g: Planck::integrate_dBdT (Planck.cpp:161-229) for g < G-1;
 * the last group the remainder 4 a c T^3 minus the integral over [e_0, e_{G-1}] (the
 * derivative of planck_cell's remainder, Planck.cpp:156-159), when positive, else 0. */
static double planck_cell_dBdT(const planck_t *P, double T, int G, const double *e_edge, int g) {
  if (!(T > 0.0) || !isfinite(T)) return 0.0;
  if (g < G - 1) return C_BOLTZ_JPK * planck_integrate_dBdT(P, T, e_edge[g], e_edge[g + 1]);
  double rest = 4.0 * rad_a_long() * C_LIGHT * pow(T, 3.0) - planck_integrate_dBdT(P, T, e_edge[0], e_edge[G - 1]);
  return rest > 0.0 ? C_BOLTZ_JPK * rest : 0.0;
}

double orc_planck_cell_dBdT(double T, int G, const double *e_edge, int g) {
  planck_t P;
  planck_setup(&P);
  return planck_cell_dBdT(&P, T, G, e_edge, g);
}

/* Per cell at the new T(c), per local group: the owed emission grows by dB_g/dT(T_old) dT
 * (what the last implicit update let the material emit beyond the sweep's B; a cell whose
 * update solved the full emission added B_g(T) - B_g(T_old) there and left dT 0); B_g(T); the
 * next sweep pays p_g = max(owed_g, -B_g) of it -- Beff_g = B_g + p_g >= 0 -- and owed_g
 * keeps the rest; then dB_g/dT(T) and bpart(c) = sum over the local groups (ascending) of
 * sigma_g dB_g/dT. */
static void material_planck(orc_solver *s) {
#pragma omp parallel for schedule(static) num_threads(s->threads) if (s->threads > 1)
  for (int c = 0; c < s->N; ++c) {
    double b = 0.0;
    for (int gl = 0; gl < s->Gl; ++gl) {
      const int g = s->g_lo + gl;
      const size_t o = (size_t)c * s->Gl + gl;
      const double owed = s->owed[o] + s->dBcell[o] * s->dTlast[c];
      const double B = planck_cell(&s->planck, s->Tcell[c], s->G, s->e_edge, g);
      const double dB = planck_cell_dBdT(&s->planck, s->Tcell[c], s->G, s->e_edge, g);
      const double pay = owed > -B ? owed : -B;
      s->Bcell[o] = B;
      s->Beff[o] = B + pay;
      s->owed[o] = owed - pay;
      s->dBcell[o] = dB;
      b = b + s->rho[g] * s->kappa[g] * dB;
    }
    s->bpart[c] = b;
  }
}

/* The coupling (include/rtsn.h "material"): the temperature update implicit in the
 * material's own emission, the emission change it implies paid to the radiation in the
 * following sweeps.  Per full step, with W = sum_i w_i and sigma_g = rho kappa_g:
 *   sweep with the emission Beff_g = B_g(T^n) + p_g (p_g: the owed emission paid now);
 *   q = sum_g sigma_g (phi_g^{n+1} - W B_g(T^n)) and b = sum_g sigma_g dB_g/dT(T^n) over ALL
 *     groups (the callers sum both over the shards: one all-reduce of 2N doubles);
 *   dT = dt q / (rho_cv + dt W b) -- rho_cv dT = dt sum_g sigma_g (phi_g - W B_g(T^{n+1})) with
 *     B(T^{n+1}) linearised about T^n -- and T^{n+1} = T^n + dT;
 *   the material thereby emitted dt W sum_g sigma_g dB_g/dT dT beyond the sweep's B: each
 *     group's share joins its owed emission, paid in the next sweeps as far as the emission
 *     stays >= 0 (all of it unless the material cooled by a large fraction of T).
 * Radiation + material + owed energy changes only by the boundary flows (BE: to rounding;
 * orc_get_material_transit).  Linear grey analysis: stable at any dt / rho_cv;
 * BE keeps T > 0 (dT > -T when phi >= 0, since B_g / dB_g/dT <= T). */
int orc_material_enable(orc_solver *s, double rho_cv, const double *T_cells) {
  if (!(rho_cv > 0.0)) return ORC_ERR_PARAM;
  if (s->p.use_correction && s->p.V != 0.0) return ORC_ERR_PARAM;
  int ok = 1;
  if (!s->Tcell) s->Tcell = (double *)xcalloc(s->N, sizeof(double), &ok);
  if (!s->dTlast) s->dTlast = (double *)xcalloc(s->N, sizeof(double), &ok);
  if (!s->bpart) s->bpart = (double *)xcalloc(s->N, sizeof(double), &ok);
  if (!s->Bcell) s->Bcell = (double *)xcalloc((size_t)s->N * s->Gl, sizeof(double), &ok);
  if (!s->dBcell) s->dBcell = (double *)xcalloc((size_t)s->N * s->Gl, sizeof(double), &ok);
  if (!s->Beff) s->Beff = (double *)xcalloc((size_t)s->N * s->Gl, sizeof(double), &ok);
  if (!s->owed) s->owed = (double *)xcalloc((size_t)s->N * s->Gl, sizeof(double), &ok);
  if (!ok) return ORC_ERR_NOMEM;
  for (int c = 0; c < s->N; ++c) {
    s->Tcell[c] = T_cells ? T_cells[c] : s->p.T;
    s->dTlast[c] = 0.0;
    for (int gl = 0; gl < s->Gl; ++gl) s->owed[(size_t)c * s->Gl + gl] = 0.0;
  }
  s->rho_cv = rho_cv;
  s->wsum = 0.0;
  for (int i = 0; i < s->M; ++i) s->wsum += s->wt[i];
  material_planck(s);
  return ORC_OK;
}

/* One full step with the per-cell emission Beff (ts 3: four substeps), then into qb (2N):
 * q(c) = sum_gl sigma_g (phi_g(c) - W B_g(c)) and b(c) = bpart(c), local groups. */
int orc_material_sweep(orc_solver *s, double *qb) {
  if (!s->Beff) return ORC_ERR_PARAM;
  if (s->p.use_mg_equilib && !s->equil_done) {
    int st = equilibrium_sources(s);
    if (st) return st;
    s->equil_done = 1;
  }
  const int sub = s->p.ts_method == 3 ? 4 : 1;
  int st = orc_run_substeps(s, s->mat_it, sub);
  if (st) return st;
  s->mat_it += sub;
  const size_t GN = (size_t)s->Gl * s->N;
  double *phi = (double *)malloc(sizeof(double) * (GN ? GN : 1));
  if (!phi) return ORC_ERR_NOMEM;
  orc_moments(s, phi, NULL, NULL);
  for (int c = 0; c < s->N; ++c) {
    double acc = 0.0;
    for (int gl = 0; gl < s->Gl; ++gl) {
      int g = s->g_lo + gl;
      double sigma = s->rho[g] * s->kappa[g];
      acc += sigma * (phi[(size_t)c * s->Gl + gl] - s->wsum * s->Bcell[(size_t)c * s->Gl + gl]);
    }
    qb[c] = acc;
    qb[(size_t)s->N + c] = s->bpart[c];
  }
  free(phi);
  return ORC_OK;
}

/* S(T) = sum over ALL G groups of sigma_g B_g(T), and its derivative (planck_cell's groups) */
static void material_emission_all(const orc_solver *s, double T, double *S, double *dS) {
  double a = 0.0, d = 0.0;
  for (int g = 0; g < s->G; ++g) {
    const double sigma = s->rho[g] * s->kappa[g];
    a += sigma * planck_cell(&s->planck, T, s->G, s->e_edge, g);
    d += sigma * planck_cell_dBdT(&s->planck, T, s->G, s->e_edge, g);
  }
  *S = a;
  *dS = d;
}

/* A cell whose linearised update would heat it by more than MAT_NEWTON_FRAC of T (B is convex
 * in T, so its tangent at T^n under-counts the emission at T^{n+1}: heating, the linear update
 * overshoots -- a cold cell beside hot ones absorbs many times its energy in one step and
 * overshoots by orders of magnitude, then diverges; cooling, it only lags, T staying above the
 * full solution) solves the full emission instead:
 *   rho_cv (T' - T) = dt (A - W S(T')),  A = q + W S(T) = sum_g sigma_g phi_g (all groups),
 * S over ALL groups (every handle holds every group's edges and opacity, so a shard needs no
 * second reduction).  S is increasing and 0 for T' <= 0, so the root is unique: in
 * [0, T + dt A / rho_cv] when the material keeps a positive energy, else T + dt A / rho_cv.
 * Newton's method, bisection where a step leaves the bracket. */
#define MAT_NEWTON_FRAC 0.25
static double material_solve_cell(const orc_solver *s, double T, double q) {
  const double W = s->wsum, dt = s->dt, rc = s->rho_cv;
  double S0, dS0;
  material_emission_all(s, T, &S0, &dS0);
  const double A = q + W * S0;
  const double hi0 = T + dt * A / rc; /* f(hi0) = dt W S(hi0) >= 0 */
  if (!(hi0 > 0.0)) return hi0;       /* no emission left to balance: the linear root, <= 0 */
  double lo = 0.0, hi = hi0, x = T > 0.0 && T < hi0 ? T : 0.5 * hi0;
  for (int it = 0; it < 200; ++it) {
    double S, dS;
    material_emission_all(s, x, &S, &dS);
    const double f = rc * (x - T) + dt * W * S - dt * A;
    if (f > 0.0) hi = x; else lo = x;
    const double fp = rc + dt * W * dS;
    double xn = x - f / fp;
    if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
    if (fabs(xn - x) <= 1e-15 * fabs(xn) || hi - lo <= 1e-15 * hi) return xn;
    x = xn;
  }
  return x;
}

/* From qb (2N: q and b summed over all groups): dT = dt q / (rho_cv + dt W b), T += dT --
 * or, where dT > MAT_NEWTON_FRAC T, the root of the full emission (material_solve_cell) --
 * then the Planck terms at the new T and the next emission (see orc_material_enable). */
void orc_material_update(orc_solver *s, const double *qb) {
  const double W = s->wsum, dt = s->dt, rc = s->rho_cv;
  for (int c = 0; c < s->N; ++c) {
    const double q = qb[c], b = qb[(size_t)s->N + c];
    const double T = s->Tcell[c];
    const double dT = dt * q / (rc + dt * W * b);
    if (dT <= MAT_NEWTON_FRAC * T) {
      s->Tcell[c] = T + dT;
      s->dTlast[c] = dT;
    } else {
      /* the material emitted B_g(T') - B_g(T) beyond the sweep's B: owed now, no dT term */
      const double Tn = material_solve_cell(s, T, q);
      for (int gl = 0; gl < s->Gl; ++gl) {
        const size_t o = (size_t)c * s->Gl + gl;
        s->owed[o] = s->owed[o] + (planck_cell(&s->planck, Tn, s->G, s->e_edge, s->g_lo + gl) - s->Bcell[o]);
      }
      s->Tcell[c] = Tn;
      s->dTlast[c] = 0.0;
    }
  }
  material_planck(s);
}

/* Energy per volume the material owes the radiation, per cell: dt W sum_gl sigma_g (p_g +
 * owed_g) -- the next sweep's payment and the rest (this solver's groups). */
void orc_get_material_transit(const orc_solver *s, double *E) {
  for (int c = 0; c < s->N; ++c) {
    double e = 0.0;
    if (s->owed)
      for (int gl = 0; gl < s->Gl; ++gl) {
        const int g = s->g_lo + gl;
        const size_t o = (size_t)c * s->Gl + gl;
        e += s->rho[g] * s->kappa[g] * ((s->Beff[o] - s->Bcell[o]) + s->owed[o]);
      }
    E[c] = s->dt * s->wsum * e;
  }
}

void orc_get_temperature(const orc_solver *s, double *T) {
  for (int c = 0; c < s->N; ++c) T[c] = s->Tcell ? s->Tcell[c] : s->p.T;
}

void orc_get_cell_planck(const orc_solver *s, double *B) {
  if (s->Bcell) memcpy(B, s->Bcell, sizeof(double) * (size_t)s->N * s->Gl);
}

void orc_get_cell_emission(const orc_solver *s, double *Beff) {
  if (s->Beff) memcpy(Beff, s->Beff, sizeof(double) * (size_t)s->N * s->Gl);
}

int orc_num_groups_local(const orc_solver *s) { return s->Gl; }

void orc_get_psi(const orc_solver *s, double *out) {
  memcpy(out, s->psi, sizeof(double) * (size_t)s->M * s->Gl * s->N);
}
void orc_get_ends(const orc_solver *s, double *out) { memcpy(out, s->ends, ends_bytes(s)); }
void orc_set_ends(orc_solver *s, const double *in) {
  memcpy(s->ends, in, ends_bytes(s));
  for (int c = 0; c < s->N; ++c)
    for (int gl = 0; gl < s->Gl; ++gl)
      for (int i = 0; i < s->M; ++i)
        PSI(s, i, gl, c) = 0.5 * (E4(s->ends, s, i, gl, c, 0) + E4(s->ends, s, i, gl, c, 1));
}

/* solver.cpp:191-237 */
void orc_moments(const orc_solver *s, double *phi, double *F, double *phi_plus) {
  const int M = s->M, Gl = s->Gl, N = s->N;
  for (int g = 0; g < Gl; ++g)
    for (int c = 0; c < N; ++c) {
      double a = 0., f = 0., pp = 0.;
      for (int i = 0; i < M; ++i) a += s->wt[i] * PSI(s, i, g, c);
      for (int i = 0; i < M; ++i) f += s->mu[i] * s->wt[i] * PSI(s, i, g, c);
      for (int i = M / 2; i < M; ++i) pp += s->wt[i] * PSI(s, i, g, c);
      if (phi) phi[g + Gl * c] = a;
      if (F) F[g + Gl * c] = f;
      if (phi_plus) phi_plus[g + Gl * c] = pp;
    }
}

/* solver.cpp:826-850 */
void orc_group_ends(const orc_solver *s, double *left, double *right) {
  for (int gl = 0; gl < s->Gl; ++gl) {
    int g = s->g_lo + gl;
    double l = 0., r = 0.;
    for (int i = 0; i < s->M; ++i) {
      if (s->mu[i] < 0.) l += E4(s->ends, s, i, gl, 0, 0);
      else r += E4(s->ends, s, i, gl, s->N - 1, 1);
    }
    left[gl] = l / (s->de_ave[g] * C_LIGHT);
    right[gl] = r / (s->de_ave[g] * C_LIGHT);
  }
}

/* solver.cpp:240-284 */
void orc_balance(const orc_solver *s, const double *phi, double *balance) {
  const int M = s->M, N = s->N, Gl = s->Gl;
  for (int gl = 0; gl < Gl; ++gl) {
    int g = s->g_lo + gl;
    double jhm = 0., jhp = 0., jNm = 0., jNp = 0., ab = 0., src = 0.;
    for (int i = 0; i < M; ++i) {
      double mu = s->mu[i];
      if (mu < 0.) {
        jhm -= E4(s->ends, s, i, gl, 0, 0) * mu * s->wt[i];
        jNm -= E4(s->ends, s, i, gl, N - 1, 0) * mu * s->wt[i];
      } else {
        jhp += E4(s->ends, s, i, gl, 0, 1) * mu * s->wt[i];
        jNp += E4(s->ends, s, i, gl, N - 1, 1) * mu * s->wt[i];
      }
    }
    for (int c = 0; c < N; ++c) {
      ab += s->rho[g] * s->kappa[g] * phi[gl + Gl * c] * s->dx;
      src += s->rho[g] * s->kappa[g] * s->ac * pow(s->temperature[g], 4) * s->dx;
    }
    double sources = jhp + jNm + src;
    double sinks = jNp + jhm + ab;
    balance[gl] = fabs(sinks - sources) / sources;
  }
}

void orc_get_quad(const orc_solver *s, double *mu, double *wt) {
  memcpy(mu, s->mu, sizeof(double) * s->M);
  memcpy(wt, s->wt, sizeof(double) * s->M);
}

void orc_get_groups(const orc_solver *s, double *e_edge, double *e_ave, double *de_ave, double *B,
                    double *dBdT, double *kappa) {
  int G = s->G;
  if (e_edge) memcpy(e_edge, s->e_edge, sizeof(double) * (G + 1));
  if (e_ave) memcpy(e_ave, s->e_ave, sizeof(double) * G);
  if (de_ave) memcpy(de_ave, s->de_ave, sizeof(double) * G);
  if (B) memcpy(B, s->cB, sizeof(double) * G);
  if (dBdT) memcpy(dBdT, s->cdBdT, sizeof(double) * G);
  if (kappa) memcpy(kappa, s->kappa, sizeof(double) * G);
}

void orc_get_correction_coeffs(const orc_solver *s, double *dEB, double *dsigEdE, double *dkapEB,
                               double *cor1, double *cor2, double *cor3) {
  /* refresh (compute_correction is what fills them; T is constant) */
  orc_solver *m = (orc_solver *)s;
  corr_edge_opacities(m);
  corr_components(m);
  corr_terms(m);
  int G = s->G;
  if (dEB) memcpy(dEB, s->dEB, sizeof(double) * G);
  if (dsigEdE) memcpy(dsigEdE, s->dsigEdE, sizeof(double) * G);
  if (dkapEB) memcpy(dkapEB, s->dkapEB, sizeof(double) * G);
  if (cor1) memcpy(cor1, s->cor1, sizeof(double) * G);
  if (cor2) memcpy(cor2, s->cor2, sizeof(double) * G);
  if (cor3) memcpy(cor3, s->cor3, sizeof(double) * G);
}

void orc_get_psi_source(const orc_solver *s, double *out) {
  memcpy(out, s->psi_source, sizeof(double) * (size_t)s->M * s->G);
}
