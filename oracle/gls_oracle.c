/* gls_oracle.c — CPU restatement of Lethe's GLS Navier–Stokes assembly.
 *
 * TEST INFRASTRUCTURE ONLY (see gls_oracle.h). Every function cites the
 * reference lines it restates. Finite-element machinery that the reference
 * takes from deal.II 9.2 (FE_Q on Gauss–Lobatto support points, QGauss,
 * affine mapping, shape Hessians) is restated here from its published
 * definitions; it is pinned only end-to-end by the reference's goldens.
 */
#include "gls_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXN 8 /* max 1D points */
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ---------------- scheme predicates: time_integration_utilities.h:12-141 ---------------- */
static int is_bdf(int s) { return s == OR_BDF1 || s == OR_BDF2 || s == OR_BDF3; }
static int is_sdirk(int s) { return s >= OR_SDIRK2 && s <= OR_SDIRK3_3; }
static int is_sdirk2(int s) { return s == OR_SDIRK2 || s == OR_SDIRK2_1 || s == OR_SDIRK2_2; }
static int is_sdirk3(int s) { return s == OR_SDIRK3 || s == OR_SDIRK3_1 || s == OR_SDIRK3_2 || s == OR_SDIRK3_3; }
static int is_sdirk_step1(int s) { return s == OR_SDIRK2_1 || s == OR_SDIRK3_1; }
static int is_sdirk_step2(int s) { return s == OR_SDIRK2_2 || s == OR_SDIRK3_2; }
static int is_sdirk_step3(int s) { return s == OR_SDIRK3_3; }
static int has_two_stages(int s) { return s == OR_BDF2 || s == OR_BDF3 || is_sdirk(s); }
static int has_three_stages(int s) { return s == OR_BDF3 || is_sdirk3(s); }

/* ---------------- time coefficients ---------------- */
/* delta(p, n, j, times): bdf.cc:23-43 (recursive divided differences) */
static void bdf_delta(int p, int n, int j, const double *times, double *out) {
  if (j == 0) {
    for (int i = 0; i <= p; ++i) out[i] = 0.;
    out[n] = 1.;
    return;
  }
  double d1[8], d2[8];
  bdf_delta(p, n, j - 1, times, d1);
  bdf_delta(p, n + 1, j - 1, times, d2);
  for (int i = 0; i <= p; ++i) out[i] = (d1[i] - d2[i]) / (times[n] - times[n + j]);
}

/* bdf_coefficients(p, dt): bdf.cc:45-75 */
int gls_oracle_bdf_coefficients(int p, const double *dt, int n_dt, double *alpha) {
  if (p < 1 || p > 5 || n_dt < p) return -1;
  double times[8];
  for (int i = 0; i <= p; ++i) {
    times[i] = 0.;
    for (int j = 0; j < i; ++j) times[i] -= dt[j];
  }
  for (int i = 0; i <= p; ++i) alpha[i] = 0.;
  for (int j = 1; j <= p; ++j) {
    double factor = 1.;
    for (int i = 1; i < j; ++i) factor *= times[0] - times[i];
    double d[8];
    bdf_delta(p, 0, j, times, d);
    for (int i = 0; i <= p; ++i) alpha[i] += factor * d[i];
  }
  return 0;
}

/* sdirk_coefficients(order, dt): sdirk.cc:11-44, row-major [order][order+1] */
int gls_oracle_sdirk_coefficients(int order, double dt, double *c) {
  const double sdt = 1. / dt;
  if (order == 2) {
    const double a = (2. - sqrt(2.)) / 2.;
    for (int i = 0; i < 6; ++i) c[i] = 0.;
    c[0 * 3 + 0] = 1. / a * sdt;
    c[0 * 3 + 1] = -1. / a * sdt;
    c[1 * 3 + 0] = 1. / a * sdt;
    c[1 * 3 + 1] = -(2 * a - 1) / a / a * sdt;
    c[1 * 3 + 2] = -(1 - a) / a / a * sdt;
    return 0;
  }
  if (order == 3) {
    for (int i = 0; i < 12; ++i) c[i] = 0.;
    c[0 * 4 + 0] = 2.29428036027904 * sdt;
    c[0 * 4 + 1] = -2.29428036027904 * sdt;
    c[1 * 4 + 0] = 2.29428036027904 * sdt;
    c[1 * 4 + 1] = -0.809559354637498 * sdt;
    c[1 * 4 + 2] = -1.48472100564154 * sdt;
    c[2 * 4 + 0] = 2.29428036027904 * sdt;
    c[2 * 4 + 1] = 2.87009860433106 * sdt;
    c[2 * 4 + 2] = -8.55612780155264 * sdt;
    c[2 * 4 + 3] = 3.39174883694255 * sdt;
    return 0;
  }
  return -1;
}

/* ---------------- 1D FE machinery (deal.II FE_Q / QGauss semantics) ---------------- */
static void legendre(int n, double x, double *P, double *dP) {
  double p0 = 1., p1 = x;
  if (n == 0) { *P = 1.; *dP = 0.; return; }
  for (int m = 2; m <= n; ++m) {
    double p2 = ((2. * m - 1.) * x * p1 - (m - 1.) * p0) / m;
    p0 = p1; p1 = p2;
  }
  *P = p1;
  *dP = n * (x * p1 - p0) / (x * x - 1.);
}

/* QGauss(n) on [0,1] */
static void gauss_1d(int n, double *x, double *w) {
  for (int i = 0; i < n; ++i) {
    double z = cos(M_PI * (i + 0.75) / (n + 0.5)), P, dP;
    for (int it = 0; it < 100; ++it) {
      legendre(n, z, &P, &dP);
      double dz = P / dP;
      z -= dz;
      if (fabs(dz) < 1e-17) break;
    }
    legendre(n, z, &P, &dP);
    /* ascending order on [0,1] */
    x[n - 1 - i] = 0.5 * (1. + z);
    w[n - 1 - i] = 1. / ((1. - z * z) * dP * dP);
  }
}

/* FE_Q(k) support points: Gauss–Lobatto on [0,1] (endpoints + roots of P'_k) */
static void lobatto_1d(int k, double *x) {
  x[0] = 0.; x[k] = 1.;
  for (int i = 1; i < k; ++i) {
    double z = -cos(M_PI * i / k);
    for (int it = 0; it < 100; ++it) {
      /* roots of P'_k: Newton on f = P'_k with f' from Legendre ODE */
      double P, dP;
      legendre(k, z, &P, &dP);
      double d2P = (2. * z * dP - k * (k + 1.) * P) / (1. - z * z);
      double dz = dP / d2P;
      z -= dz;
      if (fabs(dz) < 1e-17) break;
    }
    x[i] = 0.5 * (1. + z);
  }
  if (k == 2) x[1] = 0.5;
}

/* Lagrange polynomial i on nodes xn[0..k], value / first / second derivative at s */
static double lag(int k, const double *xn, int i, double s) {
  double v = 1.;
  for (int j = 0; j <= k; ++j) if (j != i) v *= (s - xn[j]) / (xn[i] - xn[j]);
  return v;
}
static double lag_d(int k, const double *xn, int i, double s) {
  double sum = 0.;
  for (int m = 0; m <= k; ++m) {
    if (m == i) continue;
    double t = 1. / (xn[i] - xn[m]);
    for (int j = 0; j <= k; ++j) if (j != i && j != m) t *= (s - xn[j]) / (xn[i] - xn[j]);
    sum += t;
  }
  return sum;
}
static double lag_dd(int k, const double *xn, int i, double s) {
  double sum = 0.;
  for (int m = 0; m <= k; ++m) {
    if (m == i) continue;
    for (int l = 0; l <= k; ++l) {
      if (l == i || l == m) continue;
      double t = 1. / ((xn[i] - xn[m]) * (xn[i] - xn[l]));
      for (int j = 0; j <= k; ++j) if (j != i && j != m && j != l) t *= (s - xn[j]) / (xn[i] - xn[j]);
      sum += t;
    }
  }
  return sum;
}

static int ipow(int b, int e) { int r = 1; while (e--) r *= b; return r; }

int gls_oracle_n_dofs(const gls_oracle_problem *p) { return p->dim * p->n_vnodes + p->n_pnodes; }
int gls_oracle_dofs_per_cell(const gls_oracle_problem *p) {
  return p->dim * ipow(p->k + 1, p->dim) + ipow(p->kp + 1, p->dim);
}

/* local DoF order of this restatement: velocity (node a, comp c) -> a*dim+c, then pressure nodes */
int gls_oracle_cell_dofs(const gls_oracle_problem *p, int cell, int *dofs) {
  const int dim = p->dim, nv = ipow(p->k + 1, dim), np = ipow(p->kp + 1, dim);
  for (int a = 0; a < nv; ++a)
    for (int c = 0; c < dim; ++c) dofs[a * dim + c] = p->cell_vnodes[(long)cell * nv + a] * dim + c;
  for (int a = 0; a < np; ++a) dofs[dim * nv + a] = dim * p->n_vnodes + p->cell_pnodes[(long)cell * np + a];
  return dim * nv + np;
}

/* MappingQ(md) at reference point xi of one cell: x, J[i][a] = dx_i/dxi_a, Hx[k][a][b] */
static void map_eval(const gls_oracle_problem *p, int cell, const double *xi, double *x, double J[3][3],
                     double Hx[3][3][3]) {
  const int dim = p->dim, md = p->map_degree, m1 = md + 1, ns = ipow(m1, dim);
  double xn[4];
  for (int i = 0; i <= md; ++i) xn[i] = (double)i / md;
  const double *S = p->cell_support + (size_t)cell * ns * dim;
  for (int i = 0; i < 3; ++i) {
    x[i] = 0.;
    for (int a = 0; a < 3; ++a) {
      J[i][a] = 0.;
      for (int b = 0; b < 3; ++b) Hx[i][a][b] = 0.;
    }
  }
  for (int s = 0; s < ns; ++s) {
    const int si[3] = {s % m1, (s / m1) % m1, s / (m1 * m1)};
    double L[3], dL[3], ddL[3];
    for (int d = 0; d < dim; ++d) {
      L[d] = lag(md, xn, si[d], xi[d]);
      dL[d] = lag_d(md, xn, si[d], xi[d]);
      ddL[d] = lag_dd(md, xn, si[d], xi[d]);
    }
    for (int i = 0; i < dim; ++i) {
      const double X = S[s * dim + i];
      double v = X;
      for (int d = 0; d < dim; ++d) v *= L[d];
      x[i] += v;
      for (int a = 0; a < dim; ++a) {
        double g = X;
        for (int d = 0; d < dim; ++d) g *= d == a ? dL[d] : L[d];
        J[i][a] += g;
        for (int b = 0; b < dim; ++b) {
          double h = X;
          for (int d = 0; d < dim; ++d) h *= (d == a && d == b) ? ddL[d] : ((d == a || d == b) ? dL[d] : L[d]);
          Hx[i][a][b] += h;
        }
      }
    }
  }
}

/* deal.II cell->measure(): exact volume of the multilinear cell through its corner vertices */
static double cell_measure(const gls_oracle_problem *p, int cell) {
  const int dim = p->dim;
  if (!p->map_degree) {
    double m = 1.;
    for (int d = 0; d < dim; ++d) m *= p->cell_h[cell * dim + d];
    return m;
  }
  const int md = p->map_degree, m1 = md + 1, ns = ipow(m1, dim);
  const double *S = p->cell_support + (size_t)cell * ns * dim;
  /* corner vertices -> Q1 map, integrated with the 2-point Gauss rule (exact) */
  double V[8][3];
  for (int v = 0; v < (1 << dim); ++v) {
    int s = 0, st = 1;
    for (int d = 0; d < dim; ++d) { s += ((v >> d) & 1) * md * st; st *= m1; }
    for (int i = 0; i < dim; ++i) V[v][i] = S[s * dim + i];
  }
  double xg[2], wg[2];
  gauss_1d(2, xg, wg);
  double vol = 0.;
  for (int q = 0; q < (1 << dim); ++q) {
    double xi[3] = {xg[q & 1], xg[(q >> 1) & 1], xg[(q >> 2) & 1]}, w = 1.;
    for (int d = 0; d < dim; ++d) w *= wg[(q >> d) & 1];
    double J[3][3] = {{0}};
    for (int v = 0; v < (1 << dim); ++v)
      for (int a = 0; a < dim; ++a) {
        double g = ((v >> a) & 1) ? 1. : -1.;
        for (int d = 0; d < dim; ++d)
          if (d != a) g *= ((v >> d) & 1) ? xi[d] : 1. - xi[d];
        for (int i = 0; i < dim; ++i) J[i][a] += g * V[v][i];
      }
    const double det = dim == 2 ? J[0][0] * J[1][1] - J[0][1] * J[1][0]
                                : J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                                      J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                                      J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
    vol += w * det;
  }
  return vol;
}

int gls_oracle_qpoints(const gls_oracle_problem *p, int nq1d, int cell, double *out) {
  double xq[MAXN], wq[MAXN];
  gauss_1d(nq1d, xq, wq);
  const int dim = p->dim, nq = ipow(nq1d, dim);
  if (p->map_degree) {
    for (int q = 0; q < nq; ++q) {
      int qi[3] = {q % nq1d, (q / nq1d) % nq1d, q / (nq1d * nq1d)};
      double xi[3] = {0, 0, 0}, x[3], J[3][3], Hx[3][3][3];
      for (int d = 0; d < dim; ++d) xi[d] = xq[qi[d]];
      map_eval(p, cell, xi, x, J, Hx);
      for (int d = 0; d < dim; ++d) out[q * dim + d] = x[d];
    }
    return nq;
  }
  for (int q = 0; q < nq; ++q) {
    int qi[3] = {q % nq1d, (q / nq1d) % nq1d, q / (nq1d * nq1d)};
    for (int d = 0; d < dim; ++d)
      out[q * dim + d] = p->cell_x0[cell * dim + d] + p->cell_h[cell * dim + d] * xq[qi[d]];
  }
  return nq;
}

/* Scalar Qk shape function (lexicographic multi-index) on an axis-aligned cell:
 * value, physical gradient, physical Laplacian (affine map: gradient scaled by 1/h_d,
 * Hessian by 1/(h_d h_e); deal.II FEValues with MappingQ on a straight-sided box). */
static void shape_eval(int dim, int k, const double *xn, int a, const double *xi, const double *h,
                       double *val, double *grad, double *lap) {
  int ai[3] = {a % (k + 1), (a / (k + 1)) % (k + 1), a / ((k + 1) * (k + 1))};
  double L[3], dL[3], ddL[3];
  for (int d = 0; d < dim; ++d) {
    L[d] = lag(k, xn, ai[d], xi[d]);
    dL[d] = lag_d(k, xn, ai[d], xi[d]);
    ddL[d] = lag_dd(k, xn, ai[d], xi[d]);
  }
  double v = 1.;
  for (int d = 0; d < dim; ++d) v *= L[d];
  *val = v;
  double lp = 0.;
  for (int d = 0; d < dim; ++d) {
    double g = dL[d], s = ddL[d];
    for (int e = 0; e < dim; ++e)
      if (e != d) { g *= L[e]; s *= L[e]; }
    grad[d] = g / h[d];
    lp += s / (h[d] * h[d]);
  }
  *lap = lp;
}

typedef struct {
  int dim, nv, np, nd, nq;
  double *phi_u;   /* [nq][nd][3] */
  double *grad_u;  /* [nq][nd][3][3] */
  double *lap_u;   /* [nq][nd][3] */
  double *div_u;   /* [nq][nd] */
  double *phi_p;   /* [nq][nd] */
  double *grad_p;  /* [nq][nd][3] */
  double *JxW;     /* [nq] */
  double *xq;      /* [nq][3] */
  /* reference-cell tables (FEValues' precomputed shape data; affine cells scale them by 1/h):
   * per (q, scalar shape a): value, d/dxi_d, d2/dxi_d2 of the velocity (k) and pressure (kp) bases */
  double *rv, *rg, *rs;   /* [nq][nv], [nq][nv][3], [nq][nv][3] */
  double *rpv, *rpg;      /* [nq][np], [nq][np][3] */
} cell_tab;

/* timing path only (gls_oracle_time_local_systems): 1 = reference-cell tables, as deal.II's FEValues
 * precomputes them; the values are bit-identical to the per-cell tabulation */
static int g_fast_tables = 0;
void gls_oracle_set_fast_tables(int on) { g_fast_tables = on; }

static void tab_alloc(cell_tab *t, const gls_oracle_problem *p) {
  t->dim = p->dim;
  t->nv = ipow(p->k + 1, p->dim);
  t->np = ipow(p->kp + 1, p->dim);
  t->nd = p->dim * t->nv + t->np;
  t->nq = ipow(p->nq1d, p->dim);
  size_t nqd = (size_t)t->nq * t->nd;
  t->phi_u = calloc(nqd * 3, sizeof(double));
  t->grad_u = calloc(nqd * 9, sizeof(double));
  t->lap_u = calloc(nqd * 3, sizeof(double));
  t->div_u = calloc(nqd, sizeof(double));
  t->phi_p = calloc(nqd, sizeof(double));
  t->grad_p = calloc(nqd * 3, sizeof(double));
  t->JxW = calloc(t->nq, sizeof(double));
  t->xq = calloc((size_t)t->nq * 3, sizeof(double));
  t->rv = t->rg = t->rs = t->rpv = t->rpg = NULL;
  if (g_fast_tables && !p->map_degree) {
    const int dim = p->dim, nq1 = p->nq1d;
    double xq1[MAXN], wq1[MAXN], xnv[MAXN], xnp[MAXN];
    gauss_1d(nq1, xq1, wq1);
    lobatto_1d(p->k, xnv);
    lobatto_1d(p->kp, xnp);
    t->rv = calloc((size_t)t->nq * t->nv, sizeof(double));
    t->rg = calloc((size_t)t->nq * t->nv * 3, sizeof(double));
    t->rs = calloc((size_t)t->nq * t->nv * 3, sizeof(double));
    t->rpv = calloc((size_t)t->nq * t->np, sizeof(double));
    t->rpg = calloc((size_t)t->nq * t->np * 3, sizeof(double));
    for (int q = 0; q < t->nq; ++q) {
      int qi[3] = {q % nq1, (q / nq1) % nq1, q / (nq1 * nq1)};
      double xi[3] = {0, 0, 0};
      for (int d = 0; d < dim; ++d) xi[d] = xq1[qi[d]];
      for (int pass = 0; pass < 2; ++pass) {
        const int kk = pass ? p->kp : p->k, na = pass ? t->np : t->nv;
        const double *xn = pass ? xnp : xnv;
        for (int a = 0; a < na; ++a) {
          int ai[3] = {a % (kk + 1), (a / (kk + 1)) % (kk + 1), a / ((kk + 1) * (kk + 1))};
          double L[3], dL[3], ddL[3];
          for (int d = 0; d < dim; ++d) {
            L[d] = lag(kk, xn, ai[d], xi[d]);
            dL[d] = lag_d(kk, xn, ai[d], xi[d]);
            ddL[d] = lag_dd(kk, xn, ai[d], xi[d]);
          }
          double v = 1.;
          for (int d = 0; d < dim; ++d) v *= L[d];
          (pass ? t->rpv : t->rv)[(size_t)q * na + a] = v;
          for (int d = 0; d < dim; ++d) {
            double g = dL[d], ss = ddL[d];
            for (int e = 0; e < dim; ++e)
              if (e != d) { g *= L[e]; ss *= L[e]; }
            (pass ? t->rpg : t->rg)[((size_t)q * na + a) * 3 + d] = g;
            if (!pass) t->rs[((size_t)q * na + a) * 3 + d] = ss;
          }
        }
      }
    }
  }
}
static void tab_free(cell_tab *t) {
  free(t->phi_u); free(t->grad_u); free(t->lap_u); free(t->div_u);
  free(t->phi_p); free(t->grad_p); free(t->JxW); free(t->xq);
  free(t->rv); free(t->rg); free(t->rs); free(t->rpv); free(t->rpg);
}

/* scalar Qk shape function on the reference cell: value, gradient, Hessian (d/dxi) */
static void shape_ref(int dim, int k, const double *xn, int a, const double *xi, double *val, double g[3],
                      double H[3][3]) {
  int ai[3] = {a % (k + 1), (a / (k + 1)) % (k + 1), a / ((k + 1) * (k + 1))};
  double L[3], dL[3], ddL[3];
  for (int d = 0; d < dim; ++d) {
    L[d] = lag(k, xn, ai[d], xi[d]);
    dL[d] = lag_d(k, xn, ai[d], xi[d]);
    ddL[d] = lag_dd(k, xn, ai[d], xi[d]);
  }
  double v = 1.;
  for (int d = 0; d < dim; ++d) v *= L[d];
  *val = v;
  for (int e = 0; e < dim; ++e) {
    g[e] = 1.;
    for (int d = 0; d < dim; ++d) g[e] *= d == e ? dL[d] : L[d];
    for (int f = 0; f < dim; ++f) {
      H[e][f] = 1.;
      for (int d = 0; d < dim; ++d) H[e][f] *= (d == e && d == f) ? ddL[d] : ((d == e || d == f) ? dL[d] : L[d]);
    }
  }
}

static void invert(int dim, double J[3][3], double Ji[3][3], double *det) {
  if (dim == 2) {
    *det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    Ji[0][0] = J[1][1] / *det; Ji[0][1] = -J[0][1] / *det;
    Ji[1][0] = -J[1][0] / *det; Ji[1][1] = J[0][0] / *det;
    return;
  }
  *det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
         J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
  Ji[0][0] = (J[1][1] * J[2][2] - J[1][2] * J[2][1]) / *det;
  Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / *det;
  Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / *det;
  Ji[1][0] = (J[1][2] * J[2][0] - J[1][0] * J[2][2]) / *det;
  Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / *det;
  Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / *det;
  Ji[2][0] = (J[1][0] * J[2][1] - J[1][1] * J[2][0]) / *det;
  Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / *det;
  Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / *det;
}

/* mapped scalar shape function: physical gradient and Laplacian (trace of the pushed-forward Hessian) */
static void shape_mapped(int dim, int k, const double *xn, int a, const double *xi, double Ji[3][3],
                         double Hx[3][3][3], double *val, double *grad, double *lap) {
  double g[3], H[3][3];
  shape_ref(dim, k, xn, a, xi, val, g, H);
  for (int i = 0; i < dim; ++i) {  /* grad_i = sum_a dxi_a/dx_i g_a, Ji[a][i] = dxi_a/dx_i (J^-1 = Ji) */
    grad[i] = 0.;
    for (int e = 0; e < dim; ++e) grad[i] += Ji[e][i] * g[e];
  }
  double Hc[3][3];  /* H_ref - sum_k grad_k d2x_k */
  for (int e = 0; e < dim; ++e)
    for (int f = 0; f < dim; ++f) {
      Hc[e][f] = H[e][f];
      for (int kk = 0; kk < dim; ++kk) Hc[e][f] -= grad[kk] * Hx[kk][e][f];
    }
  double lp = 0.;
  for (int i = 0; i < dim; ++i) {
    double hii = 0.;
    for (int e = 0; e < dim; ++e)
      for (int f = 0; f < dim; ++f) hii += Ji[e][i] * Hc[e][f] * Ji[f][i];
    lp += hii;
  }
  *lap = lp;
}

/* fe_values.reinit(cell) + the per-q shape tabulation of gls_navier_stokes.cc:412-423 */
static void tab_fill(cell_tab *t, const gls_oracle_problem *p, int cell) {
  const int dim = p->dim, nq1 = p->nq1d;
  double xq1[MAXN], wq1[MAXN], xnv[MAXN], xnp[MAXN];
  gauss_1d(nq1, xq1, wq1);
  lobatto_1d(p->k, xnv);
  lobatto_1d(p->kp, xnp);
  const double *h = p->cell_h + (long)cell * dim;
  const double *x0 = p->cell_x0 + (long)cell * dim;
  double meas = 1.;
  for (int d = 0; d < dim; ++d) meas *= h[d];
  for (int q = 0; q < t->nq; ++q) {
    int qi[3] = {q % nq1, (q / nq1) % nq1, q / (nq1 * nq1)};
    double xi[3] = {0, 0, 0}, w = 1.;
    for (int d = 0; d < dim; ++d) { xi[d] = xq1[qi[d]]; w *= wq1[qi[d]]; }
    double Ji[3][3] = {{0}}, Hx[3][3][3];
    if (p->map_degree) {
      double x[3], J[3][3], det;
      map_eval(p, cell, xi, x, J, Hx);
      invert(dim, J, Ji, &det);
      t->JxW[q] = w * det;
      for (int d = 0; d < dim; ++d) t->xq[q * 3 + d] = x[d];
    } else {
      t->JxW[q] = w * meas;
      for (int d = 0; d < dim; ++d) t->xq[q * 3 + d] = x0[d] + h[d] * xi[d];
    }
    for (int kk = 0; kk < t->nd; ++kk) {
      size_t o = (size_t)q * t->nd + kk;
      for (int d = 0; d < 3; ++d) { t->phi_u[o * 3 + d] = 0.; t->lap_u[o * 3 + d] = 0.; t->grad_p[o * 3 + d] = 0.; }
      for (int d = 0; d < 9; ++d) t->grad_u[o * 9 + d] = 0.;
      t->div_u[o] = 0.;
      t->phi_p[o] = 0.;
      double val, grad[3], lap;
      if (t->rv && kk < dim * t->nv) {  /* reference-cell tables scaled to the box (shape_eval's order) */
        int a = kk / dim, c = kk % dim;
        const size_t ra = (size_t)q * t->nv + a;
        t->phi_u[o * 3 + c] = t->rv[ra];
        double lp = 0.;
        for (int e = 0; e < dim; ++e) {
          const double ge = t->rg[ra * 3 + e] / h[e];
          t->grad_u[o * 9 + c * 3 + e] = ge;
          lp += t->rs[ra * 3 + e] / (h[e] * h[e]);
        }
        t->lap_u[o * 3 + c] = lp;
        t->div_u[o] = t->grad_u[o * 9 + c * 3 + c];
      } else if (t->rv) {
        int a = kk - dim * t->nv;
        const size_t ra = (size_t)q * t->np + a;
        t->phi_p[o] = t->rpv[ra];
        for (int e = 0; e < dim; ++e) t->grad_p[o * 3 + e] = t->rpg[ra * 3 + e] / h[e];
      } else if (kk < dim * t->nv) {
        int a = kk / dim, c = kk % dim;
        if (p->map_degree) shape_mapped(dim, p->k, xnv, a, xi, Ji, Hx, &val, grad, &lap);
        else shape_eval(dim, p->k, xnv, a, xi, h, &val, grad, &lap);
        t->phi_u[o * 3 + c] = val;
        for (int e = 0; e < dim; ++e) t->grad_u[o * 9 + c * 3 + e] = grad[e];
        t->lap_u[o * 3 + c] = lap;
        t->div_u[o] = grad[c];
      } else {
        int a = kk - dim * t->nv;
        if (p->map_degree) shape_mapped(dim, p->kp, xnp, a, xi, Ji, Hx, &val, grad, &lap);
        else shape_eval(dim, p->kp, xnp, a, xi, h, &val, grad, &lap);
        t->phi_p[o] = val;
        for (int e = 0; e < dim; ++e) t->grad_p[o * 3 + e] = grad[e];
      }
    }
  }
}

/* The per-cell body of assembleGLS, gls_navier_stokes.cc:338-749. */
static void local_system(const gls_oracle_problem *p, cell_tab *t, int cell,
                         const double *U, const double *U1, const double *U2, const double *U3,
                         double *Ke, double *Fe, int *dofs) {
  const int dim = p->dim, nd = t->nd, nq = t->nq, scheme = p->scheme;
  const double viscosity = p->viscosity;
  tab_fill(t, p, cell);
  gls_oracle_cell_dofs(p, cell, dofs);

  /* time coefficients, gls_navier_stokes.cc:295-329 */
  const double dt = p->time_steps[0], sdt = 1. / dt;
  double bdf[5] = {0, 0, 0, 0, 0}, sd[12];
  memset(sd, 0, sizeof(sd));
  if (scheme == OR_BDF1) gls_oracle_bdf_coefficients(1, p->time_steps, 4, bdf);
  if (scheme == OR_BDF2) gls_oracle_bdf_coefficients(2, p->time_steps, 4, bdf);
  if (scheme == OR_BDF3) gls_oracle_bdf_coefficients(3, p->time_steps, 4, bdf);
  int sc = 0;
  if (is_sdirk2(scheme)) { gls_oracle_sdirk_coefficients(2, dt, sd); sc = 3; }
  if (is_sdirk3(scheme)) { gls_oracle_sdirk_coefficients(3, dt, sd); sc = 4; }
#define SD(r, c) sd[(r) * sc + (c)]
  double omega[3] = {p->omega[0], p->omega[1], dim == 3 ? p->omega[2] : 0.};
  const double omega_z = p->omega[2];

  /* element size, :340-345 (cell->measure(): Q1 volume through the vertices) */
  const double meas = cell_measure(p, cell);
  double h = dim == 2 ? sqrt(4. * meas / M_PI) / p->k : pow(6 * meas / M_PI, 1. / 3.) / p->k;

  if (Ke) memset(Ke, 0, sizeof(double) * nd * nd);
  memset(Fe, 0, sizeof(double) * nd);

  for (int q = 0; q < nq; ++q) {
    const double *phi_u = t->phi_u + (size_t)q * nd * 3;
    const double *grad_phi_u = t->grad_u + (size_t)q * nd * 9;
    const double *lap_phi_u = t->lap_u + (size_t)q * nd * 3;
    const double *div_phi_u = t->div_u + (size_t)q * nd;
    const double *phi_p = t->phi_p + (size_t)q * nd;
    const double *grad_phi_p = t->grad_p + (size_t)q * nd * 3;

    /* gather, :351-384 (get_function_values / gradients / laplacians) */
    double uq[3] = {0, 0, 0}, G[3][3] = {{0}}, Lu[3] = {0, 0, 0}, pq = 0., gp[3] = {0, 0, 0};
    double u1q[3] = {0, 0, 0}, u2q[3] = {0, 0, 0}, u3q[3] = {0, 0, 0};
    for (int kk = 0; kk < nd; ++kk) {
      const double val = U[dofs[kk]];
      for (int d = 0; d < dim; ++d) {
        uq[d] += val * phi_u[kk * 3 + d];
        Lu[d] += val * lap_phi_u[kk * 3 + d];
        for (int e = 0; e < dim; ++e) G[d][e] += val * grad_phi_u[kk * 9 + d * 3 + e];
        gp[d] += val * grad_phi_p[kk * 3 + d];
      }
      pq += val * phi_p[kk];
      if (scheme != OR_STEADY)
        for (int d = 0; d < dim; ++d) u1q[d] += U1[dofs[kk]] * phi_u[kk * 3 + d];
      if (has_two_stages(scheme))
        for (int d = 0; d < dim; ++d) u2q[d] += U2[dofs[kk]] * phi_u[kk * 3 + d];
      if (has_three_stages(scheme))
        for (int d = 0; d < dim; ++d) u3q[d] += U3[dofs[kk]] * phi_u[kk * 3 + d];
    }
    double force[3] = {0, 0, 0};
    if (p->force_q)
      for (int d = 0; d < dim; ++d) force[d] = p->force_q[((size_t)cell * nq + q) * dim + d];
    const double *xq = t->xq + q * 3;

    /* :391-408 */
    double unorm = 0.;
    for (int d = 0; d < dim; ++d) unorm += uq[d] * uq[d];
    const double u_mag = fmax(sqrt(unorm), 1e-12 * 1.0 /* GLS_u_scale */);
    const double JxW = t->JxW[q];
    const double tau = scheme == OR_STEADY
                           ? 1. / sqrt(pow(2. * u_mag / h, 2) + 9 * pow(4 * viscosity / (h * h), 2))
                           : 1. / sqrt(pow(sdt, 2) + pow(2. * u_mag / h, 2) + 9 * pow(4 * viscosity / (h * h), 2));

    /* :434-441 */
    double divu = 0.;
    for (int d = 0; d < dim; ++d) divu += G[d][d];
    double R[3] = {0, 0, 0};
    for (int d = 0; d < dim; ++d) {
      double Gu = 0.;
      for (int e = 0; e < dim; ++e) Gu += G[d][e] * uq[e];
      R[d] = Gu + gp[d] - viscosity * Lu[d] - force[d];
    }
    /* SRF, :443-467 */
    double srf_cor[3] = {0, 0, 0}, srf_cen[3] = {0, 0, 0};
    if (p->srf) {
      if (dim == 2) {
        /* cross_product_2d(a) = (a1, -a0) */
        srf_cor[0] = 2 * omega_z * (-1.) * uq[1];
        srf_cor[1] = 2 * omega_z * (-1.) * (-uq[0]);
        double t0 = omega_z * (-1.) * xq[1], t1 = omega_z * (-1.) * (-xq[0]);
        srf_cen[0] = omega_z * (-1.) * t1;
        srf_cen[1] = omega_z * (-1.) * (-t0);
      } else {
        double c0[3] = {omega[1] * uq[2] - omega[2] * uq[1], omega[2] * uq[0] - omega[0] * uq[2],
                        omega[0] * uq[1] - omega[1] * uq[0]};
        double ox[3] = {omega[1] * xq[2] - omega[2] * xq[1], omega[2] * xq[0] - omega[0] * xq[2],
                        omega[0] * xq[1] - omega[1] * xq[0]};
        for (int d = 0; d < 3; ++d) srf_cor[d] = 2 * c0[d];
        srf_cen[0] = omega[1] * ox[2] - omega[2] * ox[1];
        srf_cen[1] = omega[2] * ox[0] - omega[0] * ox[2];
        srf_cen[2] = omega[0] * ox[1] - omega[1] * ox[0];
      }
      for (int d = 0; d < dim; ++d) R[d] += srf_cor[d];
      for (int d = 0; d < dim; ++d) R[d] += srf_cen[d];
    }
    /* time terms, :477-516 */
    for (int d = 0; d < dim; ++d) {
      if (scheme == OR_BDF1) R[d] += bdf[0] * uq[d] + bdf[1] * u1q[d];
      if (scheme == OR_BDF2) R[d] += bdf[0] * uq[d] + bdf[1] * u1q[d] + bdf[2] * u2q[d];
      if (scheme == OR_BDF3) R[d] += bdf[0] * uq[d] + bdf[1] * u1q[d] + bdf[2] * u2q[d] + bdf[3] * u3q[d];
      if (is_sdirk_step1(scheme)) R[d] += SD(0, 0) * uq[d] + SD(0, 1) * u1q[d];
      if (is_sdirk_step2(scheme)) R[d] += SD(1, 0) * uq[d] + SD(1, 1) * u1q[d] + SD(1, 2) * u2q[d];
      if (is_sdirk_step3(scheme))
        R[d] += SD(2, 0) * uq[d] + SD(2, 1) * u1q[d] + SD(2, 2) * u2q[d] + SD(2, 3) * u3q[d];
    }

    /* matrix, :519-625 */
    if (Ke) {
      for (int j = 0; j < nd; ++j) {
        const double *pj = phi_u + j * 3, *gj = grad_phi_u + j * 9;
        double S[3];
        for (int d = 0; d < dim; ++d) {
          double a = 0., b = 0.;
          for (int e = 0; e < dim; ++e) { a += G[d][e] * pj[e]; b += gj[d * 3 + e] * uq[e]; }
          S[d] = a + b + grad_phi_p[j * 3 + d] - viscosity * lap_phi_u[j * 3 + d];
        }
        if (is_bdf(scheme)) for (int d = 0; d < dim; ++d) S[d] += pj[d] * bdf[0];
        if (is_sdirk(scheme)) for (int d = 0; d < dim; ++d) S[d] += pj[d] * SD(0, 0);
        double cj[3] = {0, 0, 0}; /* 2 omega x phi_j (3D) / 2 omega_z (-1) cross2d(phi_j) (2D) */
        if (p->srf) {
          if (dim == 2) { cj[0] = 2 * omega_z * (-1.) * pj[1]; cj[1] = 2 * omega_z * (-1.) * (-pj[0]); }
          else {
            cj[0] = 2 * (omega[1] * pj[2] - omega[2] * pj[1]);
            cj[1] = 2 * (omega[2] * pj[0] - omega[0] * pj[2]);
            cj[2] = 2 * (omega[0] * pj[1] - omega[1] * pj[0]);
          }
          for (int d = 0; d < dim; ++d) S[d] += cj[d];
        }
        double Gpj[3], gju[3];
        for (int d = 0; d < dim; ++d) {
          Gpj[d] = 0.; gju[d] = 0.;
          for (int e = 0; e < dim; ++e) { Gpj[d] += G[d][e] * pj[e]; gju[d] += gj[d * 3 + e] * uq[e]; }
        }
        for (int i = 0; i < nd; ++i) {
          const double *pi = phi_u + i * 3, *gi = grad_phi_u + i * 9;
          double sp = 0., a1 = 0., a2 = 0., mass = 0.;
          for (int d = 0; d < dim; ++d) {
            for (int e = 0; e < dim; ++e) sp += gj[d * 3 + e] * gi[d * 3 + e];
            a1 += Gpj[d] * pi[d];
            a2 += gju[d] * pi[d];
            mass += pj[d] * pi[d];
          }
          double Kij = (viscosity * sp + a1 + a2 - div_phi_u[i] * phi_p[j] + phi_p[i] * div_phi_u[j]) * JxW;
          if (is_bdf(scheme)) Kij += mass * bdf[0] * JxW;
          if (is_sdirk(scheme)) Kij += mass * SD(0, 0) * JxW;
          double sgp = 0.;
          for (int d = 0; d < dim; ++d) sgp += S[d] * grad_phi_p[i * 3 + d];
          Kij += tau * sgp * JxW;
          if (p->srf) {
            double c = 0.;
            for (int d = 0; d < dim; ++d) c += cj[d] * pi[d];
            Kij += c * JxW;
          }
          /* SUPG (SUPG == true, gls_navier_stokes.h:137) */
          double giu[3], gipj[3];
          for (int d = 0; d < dim; ++d) {
            giu[d] = 0.; gipj[d] = 0.;
            for (int e = 0; e < dim; ++e) { giu[d] += gi[d * 3 + e] * uq[e]; gipj[d] += gi[d * 3 + e] * pj[e]; }
          }
          double s1 = 0., s2 = 0.;
          for (int d = 0; d < dim; ++d) { s1 += S[d] * giu[d]; s2 += R[d] * gipj[d]; }
          Kij += tau * (s1 + s2) * JxW;
          Ke[(size_t)i * nd + j] += Kij;
        }
      }
    }

    /* rhs, :628-748 */
    double Gu[3];
    for (int d = 0; d < dim; ++d) {
      Gu[d] = 0.;
      for (int e = 0; e < dim; ++e) Gu[d] += G[d][e] * uq[e];
    }
    for (int i = 0; i < nd; ++i) {
      const double *pi = phi_u + i * 3, *gi = grad_phi_u + i * 9;
      double sp = 0., gup = 0., fp = 0., up = 0., u1p = 0., u2p = 0., u3p = 0., dup = 0.;
      for (int d = 0; d < dim; ++d) {
        for (int e = 0; e < dim; ++e) sp += G[d][e] * gi[d * 3 + e];
        gup += Gu[d] * pi[d];
        fp += force[d] * pi[d];
        up += uq[d] * pi[d];
        u1p += u1q[d] * pi[d];
        u2p += u2q[d] * pi[d];
        u3p += u3q[d] * pi[d];
        dup += (uq[d] - u1q[d]) * pi[d];
      }
      double F = (-viscosity * sp - gup + pq * div_phi_u[i] + fp - divu * phi_p[i]) * JxW;
      if (scheme == OR_BDF1) F -= bdf[0] * dup * JxW;
      if (scheme == OR_BDF2) F -= (bdf[0] * up + bdf[1] * u1p + bdf[2] * u2p) * JxW;
      if (scheme == OR_BDF3) F -= (bdf[0] * up + bdf[1] * u1p + bdf[2] * u2p + bdf[3] * u3p) * JxW;
      if (is_sdirk_step1(scheme)) F -= (SD(0, 0) * up + SD(0, 1) * u1p) * JxW;
      if (is_sdirk_step2(scheme)) F -= (SD(1, 0) * up + SD(1, 1) * u1p + SD(1, 2) * u2p) * JxW;
      if (is_sdirk_step3(scheme)) F -= (SD(2, 0) * up + SD(2, 1) * u1p + SD(2, 2) * u2p + SD(2, 3) * u3p) * JxW;
      if (p->srf) {
        double a = 0., b = 0.;
        for (int d = 0; d < dim; ++d) { a += srf_cor[d] * pi[d]; b += srf_cen[d] * pi[d]; }
        F += -a * JxW;
        F += -b * JxW;
      }
      double rg = 0.;
      for (int d = 0; d < dim; ++d) rg += R[d] * grad_phi_p[i * 3 + d];
      F += -tau * rg * JxW;
      double giu = 0.;
      for (int d = 0; d < dim; ++d) {
        double g = 0.;
        for (int e = 0; e < dim; ++e) g += gi[d * 3 + e] * uq[e];
        giu += R[d] * g;
      }
      F += -tau * giu * JxW;
      Fe[i] += F;
    }
  }
#undef SD
}

int gls_oracle_local_system(const gls_oracle_problem *p, int cell,
                            const double *u, const double *u1, const double *u2, const double *u3,
                            double *Ke, double *Fe) {
  cell_tab t;
  tab_alloc(&t, p);
  int *dofs = malloc(sizeof(int) * t.nd);
  local_system(p, &t, cell, u, u1, u2, u3, Ke, Fe, dofs);
  free(dofs);
  tab_free(&t);
  return 0;
}

/* where local DoF row/column g of an element lands in the condensed system: itself when
 * unconstrained, its unconstrained masters (weights) when hanging, nowhere when Dirichlet */
#define MAXT 64
static int dof_targets(const gls_oracle_problem *p, int g, int *tg, double *tw) {
  if (!p->constrained[g]) {
    tg[0] = g;
    tw[0] = 1.0;
    return 1;
  }
  if (!p->hang_off) return 0;
  int n = 0;
  for (int j = p->hang_off[g]; j < p->hang_off[g + 1] && n < MAXT; ++j) {
    const int m = p->hang_master[j];
    if (p->constrained[m]) continue;
    tg[n] = m;
    tw[n] = p->hang_w[j];
    ++n;
  }
  return n;
}

int gls_oracle_assemble_rhs(const gls_oracle_problem *p,
                            const double *u, const double *u1, const double *u2, const double *u3,
                            double *rhs) {
  cell_tab t;
  tab_alloc(&t, p);
  const int nd = t.nd, N = gls_oracle_n_dofs(p);
  int *dofs = malloc(sizeof(int) * nd);
  double *Fe = malloc(sizeof(double) * nd);
  for (int i = 0; i < N; ++i) rhs[i] = 0.;
  for (int c = 0; c < p->n_cells; ++c) {
    local_system(p, &t, c, u, u1, u2, u3, NULL, Fe, dofs);
    /* zero_constraints.distribute_local_to_global(local_rhs, ...), :767-771 */
    for (int i = 0; i < nd; ++i) {
      int tg[MAXT];
      double tw[MAXT];
      const int nt = dof_targets(p, dofs[i], tg, tw);
      for (int a = 0; a < nt; ++a) rhs[tg[a]] += tw[a] * Fe[i];
    }
  }
  free(Fe); free(dofs); tab_free(&t);
  return 0;
}

/* deal.II 9.2 AffineConstraints diagonal rule for eliminated rows */
static double constrained_diag(const double *Ke, int nd, int i) {
  double a = fabs(Ke[(size_t)i * nd + i]);
  if (a != 0.) return a;
  double avg = 0.;
  for (int j = 0; j < nd; ++j) avg += fabs(Ke[(size_t)j * nd + j]);
  return avg / nd;
}

/* number of COO triplets gls_oracle_assemble_coo will emit (hanging rows/cols expand onto masters) */
long long gls_oracle_coo_size(const gls_oracle_problem *p) {
  const int nd = gls_oracle_dofs_per_cell(p);
  int *dofs = malloc(sizeof(int) * nd);
  int *cnt = malloc(sizeof(int) * nd);
  long long n = 0;
  for (int c = 0; c < p->n_cells; ++c) {
    gls_oracle_cell_dofs(p, c, dofs);
    long long row = 0;
    for (int i = 0; i < nd; ++i) {
      int tg[MAXT];
      double tw[MAXT];
      cnt[i] = dof_targets(p, dofs[i], tg, tw);
      row += cnt[i];
      if (p->constrained[dofs[i]]) ++n;
    }
    for (int i = 0; i < nd; ++i) n += (long long)cnt[i] * row;
  }
  free(cnt); free(dofs);
  return n;
}

int gls_oracle_assemble_coo(const gls_oracle_problem *p,
                            const double *u, const double *u1, const double *u2, const double *u3,
                            int *rows, int *cols, double *vals, long long *nnz, double *rhs) {
  cell_tab t;
  tab_alloc(&t, p);
  const int nd = t.nd, N = gls_oracle_n_dofs(p);
  int *dofs = malloc(sizeof(int) * nd);
  double *Fe = malloc(sizeof(double) * nd);
  double *Ke = malloc(sizeof(double) * nd * nd);
  long long n = 0;
  for (int i = 0; i < N; ++i) rhs[i] = 0.;
  for (int c = 0; c < p->n_cells; ++c) {
    local_system(p, &t, c, u, u1, u2, u3, Ke, Fe, dofs);
    for (int i = 0; i < nd; ++i) {
      const int gi = dofs[i];
      if (p->constrained[gi]) { rows[n] = gi; cols[n] = gi; vals[n] = constrained_diag(Ke, nd, i); ++n; }
      int ti[MAXT], tj[MAXT];
      double wi[MAXT], wj[MAXT];
      const int ni = dof_targets(p, gi, ti, wi);
      for (int a = 0; a < ni; ++a) rhs[ti[a]] += wi[a] * Fe[i];
      for (int j = 0; j < nd; ++j) {
        const int nj = dof_targets(p, dofs[j], tj, wj);
        for (int a = 0; a < ni; ++a)
          for (int b = 0; b < nj; ++b) {
            rows[n] = ti[a]; cols[n] = tj[b]; vals[n] = wi[a] * wj[b] * Ke[(size_t)i * nd + j]; ++n;
          }
      }
    }
  }
  *nnz = n;
  free(Ke); free(Fe); free(dofs); tab_free(&t);
  return 0;
}

int gls_oracle_jacobian_apply(const gls_oracle_problem *p,
                              const double *u, const double *u1, const double *u2, const double *u3,
                              const double *v, double *y) {
  cell_tab t;
  tab_alloc(&t, p);
  const int nd = t.nd, N = gls_oracle_n_dofs(p);
  int *dofs = malloc(sizeof(int) * nd);
  double *Fe = malloc(sizeof(double) * nd);
  double *Ke = malloc(sizeof(double) * nd * nd);
  double *vloc = malloc(sizeof(double) * nd);
  for (int i = 0; i < N; ++i) y[i] = 0.;
  for (int c = 0; c < p->n_cells; ++c) {
    local_system(p, &t, c, u, u1, u2, u3, Ke, Fe, dofs);
    for (int j = 0; j < nd; ++j) {  /* (C v) at the element's DoFs */
      int tj[MAXT];
      double wj[MAXT];
      const int nj = dof_targets(p, dofs[j], tj, wj);
      double x = 0.;
      for (int b = 0; b < nj; ++b) x += wj[b] * v[tj[b]];
      vloc[j] = x;
    }
    for (int i = 0; i < nd; ++i) {
      const int gi = dofs[i];
      if (p->constrained[gi]) y[gi] += constrained_diag(Ke, nd, i) * v[gi];
      double s = 0.;
      for (int j = 0; j < nd; ++j) s += Ke[(size_t)i * nd + j] * vloc[j];
      int ti[MAXT];
      double wi[MAXT];
      const int ni = dof_targets(p, gi, ti, wi);
      for (int a = 0; a < ni; ++a) y[ti[a]] += wi[a] * s;
    }
  }
  free(vloc); free(Ke); free(Fe); free(dofs); tab_free(&t);
  return 0;
}

int gls_oracle_jacobian_diagonal(const gls_oracle_problem *p,
                                 const double *u, const double *u1, const double *u2, const double *u3,
                                 double *dg) {
  cell_tab t;
  tab_alloc(&t, p);
  const int nd = t.nd, N = gls_oracle_n_dofs(p);
  int *dofs = malloc(sizeof(int) * nd);
  double *Fe = malloc(sizeof(double) * nd);
  double *Ke = malloc(sizeof(double) * nd * nd);
  for (int i = 0; i < N; ++i) dg[i] = 0.;
  for (int c = 0; c < p->n_cells; ++c) {
    local_system(p, &t, c, u, u1, u2, u3, Ke, Fe, dofs);
    for (int i = 0; i < nd; ++i) {
      const int gi = dofs[i];
      if (p->constrained[gi]) dg[gi] += constrained_diag(Ke, nd, i);
      if (!p->hang_off) {
        if (!p->constrained[gi]) dg[gi] += Ke[(size_t)i * nd + i];
        continue;
      }
      int ti[MAXT], tj[MAXT];  /* exact diagonal of C^T K C */
      double wi[MAXT], wj[MAXT];
      const int ni = dof_targets(p, gi, ti, wi);
      for (int j = 0; j < nd; ++j) {
        const int nj = dof_targets(p, dofs[j], tj, wj);
        for (int a = 0; a < ni; ++a)
          for (int b = 0; b < nj; ++b)
            if (ti[a] == tj[b]) dg[ti[a]] += wi[a] * wj[b] * Ke[(size_t)i * nd + j];
      }
    }
  }
  free(Ke); free(Fe); free(dofs); tab_free(&t);
  return 0;
}

/* calculate_L2_error, navier_stokes_base.cc:253-380 (mean-free pressure) */
int gls_oracle_l2_error(const gls_oracle_problem *p, int nq1d_err, const double *sol,
                        const double *exact_q, double *err_u, double *err_p) {
  gls_oracle_problem pe = *p;
  pe.nq1d = nq1d_err;
  cell_tab t;
  tab_alloc(&t, &pe);
  const int dim = p->dim, nd = t.nd, nq = t.nq;
  int *dofs = malloc(sizeof(int) * nd);
  double p_int = 0., pex_int = 0., vol = 0.;
  for (int c = 0; c < p->n_cells; ++c) {
    tab_fill(&t, &pe, c);
    gls_oracle_cell_dofs(&pe, c, dofs);
    for (int q = 0; q < nq; ++q) {
      double pq = 0.;
      for (int kk = 0; kk < nd; ++kk) pq += sol[dofs[kk]] * t.phi_p[(size_t)q * nd + kk];
      p_int += pq * t.JxW[q];
      pex_int += exact_q[((size_t)c * nq + q) * (dim + 1) + dim] * t.JxW[q];
    }
    vol += cell_measure(p, c);  /* GridTools::volume(triangulation): the Q1 volume */
  }
  const double pavg = p_int / vol, pexavg = pex_int / vol;
  double eu = 0., ep = 0.;
  for (int c = 0; c < p->n_cells; ++c) {
    tab_fill(&t, &pe, c);
    gls_oracle_cell_dofs(&pe, c, dofs);
    for (int q = 0; q < nq; ++q) {
      double uq[3] = {0, 0, 0}, pq = 0.;
      for (int kk = 0; kk < nd; ++kk) {
        const double val = sol[dofs[kk]];
        for (int d = 0; d < dim; ++d) uq[d] += val * t.phi_u[((size_t)q * nd + kk) * 3 + d];
        pq += val * t.phi_p[(size_t)q * nd + kk];
      }
      const double *ex = exact_q + ((size_t)c * nq + q) * (dim + 1);
      for (int d = 0; d < dim; ++d) eu += (uq[d] - ex[d]) * (uq[d] - ex[d]) * t.JxW[q];
      const double ps = pq - pavg, pe_ = ex[dim] - pexavg;
      ep += (ps - pe_) * (ps - pe_) * t.JxW[q];
    }
  }
  *err_u = sqrt(eu);
  *err_p = sqrt(ep);
  free(dofs); tab_free(&t);
  return 0;
}


/* assemble_L2_projection, gls_navier_stokes.cc:830-914: velocity + pressure mass matrix and
 * rhs = (phi_u . u0 + phi_p p0) JxW; uvwp_q[n_cells*nq*(dim+1)] at the assembly q-points.
 * Written as COO (n_cells*ndofs*ndofs capacity); constraints are applied by the caller. */
int gls_oracle_l2_projection_coo(const gls_oracle_problem *p, const double *uvwp_q,
                                 int *rows, int *cols, double *vals, long long *nnz, double *rhs) {
  cell_tab t;
  tab_alloc(&t, p);
  const int dim = p->dim, nd = t.nd, nq = t.nq, N = gls_oracle_n_dofs(p);
  int *dofs = malloc(sizeof(int) * nd);
  double *Ke = malloc(sizeof(double) * nd * nd), *Fe = malloc(sizeof(double) * nd);
  long long n = 0;
  for (int i = 0; i < N; ++i) rhs[i] = 0.;
  for (int c = 0; c < p->n_cells; ++c) {
    tab_fill(&t, p, c);
    gls_oracle_cell_dofs(p, c, dofs);
    memset(Ke, 0, sizeof(double) * nd * nd);
    memset(Fe, 0, sizeof(double) * nd);
    for (int q = 0; q < nq; ++q) {
      const double *phi_u = t.phi_u + (size_t)q * nd * 3, *phi_p = t.phi_p + (size_t)q * nd;
      const double *ic = uvwp_q + ((size_t)c * nq + q) * (dim + 1);
      for (int i = 0; i < nd; ++i) {
        for (int j = 0; j < nd; ++j) {
          double m = 0.;
          for (int d = 0; d < dim; ++d) m += phi_u[j * 3 + d] * phi_u[i * 3 + d];
          Ke[(size_t)i * nd + j] += m * t.JxW[q];
          Ke[(size_t)i * nd + j] += (phi_p[j] * phi_p[i]) * t.JxW[q];
        }
        double f = 0.;
        for (int d = 0; d < dim; ++d) f += phi_u[i * 3 + d] * ic[d];
        Fe[i] += (f + phi_p[i] * ic[dim]) * t.JxW[q];
      }
    }
    for (int i = 0; i < nd; ++i) {
      rhs[dofs[i]] += Fe[i];
      for (int j = 0; j < nd; ++j) { rows[n] = dofs[i]; cols[n] = dofs[j]; vals[n] = Ke[(size_t)i * nd + j]; ++n; }
    }
  }
  *nnz = n;
  free(Ke); free(Fe); free(dofs); tab_free(&t);
  return 0;
}

double gls_oracle_time_local_systems(const gls_oracle_problem *p,
                                     const double *u, const double *u1, const double *u2, const double *u3,
                                     int c0, int count, int with_matrix, int nthreads) {
  double checksum = 0.;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(+ : checksum)
#endif
  {
    cell_tab t;
    tab_alloc(&t, p);
    const int nd = t.nd;
    int *dofs = malloc(sizeof(int) * nd);
    double *Fe = malloc(sizeof(double) * nd);
    double *Ke = with_matrix ? malloc(sizeof(double) * nd * nd) : NULL;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (int c = c0; c < c0 + count; ++c) {
      local_system(p, &t, c % p->n_cells, u, u1, u2, u3, Ke, Fe, dofs);
      checksum += Fe[0] + (Ke ? Ke[nd + 1] : 0.);
    }
    free(Ke); free(Fe); free(dofs); tab_free(&t);
  }
  return checksum;
}

/* ------------------------------------------------------------------------------------------------
 * One complete CPU Newton iteration on the assembled system (bench.py's cpu_baseline; baseline /
 * test infrastructure, never the product): NewtonNonLinearSolver::solve's loop body
 * (newton_non_linear_solver.h:90-137) with
 *   assemble_matrix_and_rhs into CSR (gls_navier_stokes.cc:916-1022; zero_constraints elimination,
 *     deal.II's |K_e(i,i)| on constrained rows), cells in parallel on `nthreads` (atomic adds);
 *   setup_ILU = Ifpack ILU(0) (:1161-1176; diagonal rthresh * a + sign(a) * athresh), serial as
 *     Ifpack's factorisation of a rank's rows is;
 *   solve_system_GMRES (:1242-1289): GMRES(restart) right-preconditioned from x0 = 0 to
 *     max(rel * ||rhs||, minres), modified Gram-Schmidt, serial ILU triangular solves, threaded
 *     SpMV and vector operations;
 *   the alpha line search with assemble_rhs (alpha = 1, 1/2, ... while not 0.9 * ||r0||).
 * Dirichlet constraints only (no hanging lines). x is updated in place.
 * ------------------------------------------------------------------------------------------------ */
static int csr_find(const int *col, int b, int e, int j) {
  while (b < e) {
    const int m = (b + e) >> 1;
    if (col[m] < j) b = m + 1;
    else e = m;
  }
  return b;
}
static void csr_spmv(int n, const int *rp, const int *ci, const double *v, const double *x, double *y) {
#pragma omp parallel for schedule(static) if (n >= (1 << 15))
  for (int i = 0; i < n; ++i) {
    double s = 0.;
    for (int e = rp[i]; e < rp[i + 1]; ++e) s += v[e] * x[ci[e]];
    y[i] = s;
  }
}
#define PAR_N (1 << 20) /* vector operations below this length run on one thread (team start-up costs more) */
static double vdot(int n, const double *a, const double *b) {
  double s = 0.;
#pragma omp parallel for reduction(+ : s) schedule(static) if (n >= PAR_N)
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}
static void ilu_solve(int n, const int *rp, const int *ci, const double *lu, const int *dg, const double *b, double *x) {
  for (int i = 0; i < n; ++i) {  /* L y = b (unit lower) */
    double s = b[i];
    for (int e = rp[i]; e < dg[i]; ++e) s -= lu[e] * x[ci[e]];
    x[i] = s;
  }
  for (int i = n - 1; i >= 0; --i) {  /* U x = y */
    double s = x[i];
    for (int e = dg[i] + 1; e < rp[i + 1]; ++e) s -= lu[e] * x[ci[e]];
    x[i] = s / lu[dg[i]];
  }
}
static void assemble_csr(const gls_oracle_problem *p, const double *u, const double *u1, const double *u2,
                         const double *u3, const int *rp, const int *ci, const int *dg, double *val, double *rhs,
                         int with_matrix) {
  const int N = gls_oracle_n_dofs(p);
  if (with_matrix) memset(val, 0, sizeof(double) * (size_t)rp[N]);
  memset(rhs, 0, sizeof(double) * (size_t)N);
#pragma omp parallel
  {
    cell_tab t;
    tab_alloc(&t, p);
    const int nd = t.nd;
    int *dofs = malloc(sizeof(int) * nd);
    double *Fe = malloc(sizeof(double) * nd);
    double *Ke = with_matrix ? malloc(sizeof(double) * nd * nd) : NULL;
#pragma omp for schedule(dynamic, 64)
    for (int c = 0; c < p->n_cells; ++c) {
      local_system(p, &t, c, u, u1, u2, u3, Ke, Fe, dofs);
      for (int i = 0; i < nd; ++i) {
        const int gi = dofs[i];
        if (p->constrained[gi]) {
          if (with_matrix) {
            const double d = constrained_diag(Ke, nd, i);
#pragma omp atomic
            val[dg[gi]] += d;
          }
          continue;
        }
#pragma omp atomic
        rhs[gi] += Fe[i];
        if (!with_matrix) continue;
        for (int j = 0; j < nd; ++j) {
          const int gj = dofs[j];
          if (p->constrained[gj]) continue;
          const int e = csr_find(ci, rp[gi], rp[gi + 1], gj);
#pragma omp atomic
          val[e] += Ke[(size_t)i * nd + j];
        }
      }
    }
    free(Ke); free(Fe); free(dofs); tab_free(&t);
  }
}

int gls_oracle_newton_csr(const gls_oracle_problem *p, double *x, const double *u1, const double *u2,
                          const double *u3, int nthreads, int restart, double rel, double minres, int max_its,
                          double athresh, double rthresh, gls_oracle_newton_stats *st) {
  if (p->hang_off) return -1;
  if (nthreads > 0) omp_set_num_threads(nthreads);
  memset(st, 0, sizeof(*st));
  const int N = gls_oracle_n_dofs(p), nd = gls_oracle_dofs_per_cell(p);
  double t0 = omp_get_wtime();
  /* sparsity (setup_dofs' make_sparsity_pattern with the constraints, keep_constrained = false) */
  int *dcnt = calloc((size_t)N + 1, sizeof(int)), *dofs = malloc(sizeof(int) * nd);
  for (int c = 0; c < p->n_cells; ++c) {
    gls_oracle_cell_dofs(p, c, dofs);
    for (int i = 0; i < nd; ++i) ++dcnt[dofs[i] + 1];
  }
  for (int i = 0; i < N; ++i) dcnt[i + 1] += dcnt[i];
  int *dcell = malloc(sizeof(int) * (size_t)dcnt[N]), *fillp = malloc(sizeof(int) * (size_t)N);
  memcpy(fillp, dcnt, sizeof(int) * (size_t)N);
  for (int c = 0; c < p->n_cells; ++c) {
    gls_oracle_cell_dofs(p, c, dofs);
    for (int i = 0; i < nd; ++i) dcell[fillp[dofs[i]]++] = c;
  }
  int *rp = malloc(sizeof(int) * ((size_t)N + 1)), *mark = malloc(sizeof(int) * (size_t)N);
  for (int i = 0; i < N; ++i) mark[i] = -1;
  long long nnz = 0;
  int *ci = NULL;
  for (int pass = 0; pass < 2; ++pass) {  /* count, then fill */
    nnz = 0;
    rp[0] = 0;
    for (int r = 0; r < N; ++r) {
      const long long b = nnz;
      if (pass) ci[nnz] = r;
      ++nnz;
      mark[r] = r;
      if (!p->constrained[r])
        for (int t = dcnt[r]; t < dcnt[r + 1]; ++t) {
          gls_oracle_cell_dofs(p, dcell[t], dofs);
          for (int i = 0; i < nd; ++i) {
            const int j = dofs[i];
            if (p->constrained[j] || mark[j] == r) continue;
            mark[j] = r;
            if (pass) ci[nnz] = j;
            ++nnz;
          }
        }
      if (pass) { /* sort the row (insertion: short rows) */
        for (long long a = b + 1; a < nnz; ++a) {
          const int v = ci[a];
          long long q = a - 1;
          while (q >= b && ci[q] > v) { ci[q + 1] = ci[q]; --q; }
          ci[q + 1] = v;
        }
      }
      rp[r + 1] = (int)nnz;
    }
    for (int i = 0; i < N; ++i) mark[i] = -1;
    if (!pass) ci = malloc(sizeof(int) * (size_t)nnz);
  }
  int *dg = malloc(sizeof(int) * (size_t)N);
  for (int r = 0; r < N; ++r) dg[r] = csr_find(ci, rp[r], rp[r + 1], r);
  st->nnz = nnz;
  st->t_pattern = omp_get_wtime() - t0;
  double *val = malloc(sizeof(double) * (size_t)nnz), *lu = malloc(sizeof(double) * (size_t)nnz);
  double *rhs = malloc(sizeof(double) * (size_t)N), *dx = calloc((size_t)N, sizeof(double));
  const int m = restart > 0 ? restart : 30;
  double *V = malloc(sizeof(double) * (size_t)N * (size_t)(m + 1)), *Z = malloc(sizeof(double) * (size_t)N * (size_t)m);
  double *w = malloc(sizeof(double) * (size_t)N), *H = calloc((size_t)(m + 1) * m, sizeof(double));
  double *g = malloc(sizeof(double) * (size_t)(m + 1)), *cs = malloc(sizeof(double) * (size_t)m), *sn = malloc(sizeof(double) * (size_t)m);
  double *yv = malloc(sizeof(double) * (size_t)m), *xt = malloc(sizeof(double) * (size_t)N);
  /* assemble_matrix_and_rhs */
  t0 = omp_get_wtime();
  assemble_csr(p, x, u1, u2, u3, rp, ci, dg, val, rhs, 1);
  st->t_assemble = omp_get_wtime() - t0;
  const double res0 = sqrt(vdot(N, rhs, rhs));
  st->res0 = res0;
  /* setup_ILU: ILU(0) */
  t0 = omp_get_wtime();
  memcpy(lu, val, sizeof(double) * (size_t)nnz);
  for (int r = 0; r < N; ++r) {
    const double a = lu[dg[r]];
    lu[dg[r]] = rthresh * a + (a < 0 ? -athresh : athresh);
  }
  for (int i = 0; i < N; ++i) {
    for (int e = rp[i]; e < rp[i + 1]; ++e) mark[ci[e]] = e;
    for (int e = rp[i]; e < dg[i]; ++e) {
      const int k = ci[e];
      const double lik = lu[e] / lu[dg[k]];
      lu[e] = lik;
      for (int f = dg[k] + 1; f < rp[k + 1]; ++f) {
        const int q = mark[ci[f]];
        if (q >= 0) lu[q] -= lik * lu[f];
      }
    }
    for (int e = rp[i]; e < rp[i + 1]; ++e) mark[ci[e]] = -1;
  }
  st->t_ilu = omp_get_wtime() - t0;
  /* solve_system_GMRES: right-preconditioned GMRES(m), x0 = 0 */
  t0 = omp_get_wtime();
  const double tol = fmax(rel * res0, minres);
  double beta = res0;
  int its = 0;
  memset(dx, 0, sizeof(double) * (size_t)N);
  memcpy(w, rhs, sizeof(double) * (size_t)N);
  while (beta > tol && its < max_its) {
#pragma omp parallel for schedule(static) if (N >= PAR_N)
    for (int i = 0; i < N; ++i) V[i] = w[i] / beta;
    for (int i = 0; i <= m; ++i) g[i] = 0.;
    g[0] = beta;
    int j = 0;
    for (; j < m && its < max_its; ++j) {
      double *zj = Z + (size_t)j * N, *vj = V + (size_t)j * N, *vn = V + (size_t)(j + 1) * N;
      ilu_solve(N, rp, ci, lu, dg, vj, zj);
      csr_spmv(N, rp, ci, val, zj, vn);
      for (int i = 0; i <= j; ++i) {  /* modified Gram-Schmidt */
        const double *vi = V + (size_t)i * N;
        const double h = vdot(N, vn, vi);
        H[(size_t)i * m + j] = h;
#pragma omp parallel for schedule(static) if (N >= PAR_N)
        for (int q = 0; q < N; ++q) vn[q] -= h * vi[q];
      }
      const double hn = sqrt(vdot(N, vn, vn));
      H[(size_t)(j + 1) * m + j] = hn;
      if (hn > 0) {
#pragma omp parallel for schedule(static) if (N >= PAR_N)
        for (int q = 0; q < N; ++q) vn[q] /= hn;
      }
      for (int i = 0; i < j; ++i) {
        const double a = H[(size_t)i * m + j], b = H[(size_t)(i + 1) * m + j];
        H[(size_t)i * m + j] = cs[i] * a + sn[i] * b;
        H[(size_t)(i + 1) * m + j] = -sn[i] * a + cs[i] * b;
      }
      const double a = H[(size_t)j * m + j], b = H[(size_t)(j + 1) * m + j], rr = hypot(a, b);
      cs[j] = rr > 0 ? a / rr : 1.;
      sn[j] = rr > 0 ? b / rr : 0.;
      H[(size_t)j * m + j] = rr;
      H[(size_t)(j + 1) * m + j] = 0.;
      g[j + 1] = -sn[j] * g[j];
      g[j] *= cs[j];
      ++its;
      if (fabs(g[j + 1]) <= tol) { ++j; break; }
    }
    for (int i = j - 1; i >= 0; --i) {
      double s = g[i];
      for (int l = i + 1; l < j; ++l) s -= H[(size_t)i * m + l] * yv[l];
      yv[i] = H[(size_t)i * m + i] != 0. ? s / H[(size_t)i * m + i] : 0.;
    }
    for (int i = 0; i < j; ++i) {
      const double *zi = Z + (size_t)i * N;
#pragma omp parallel for schedule(static) if (N >= PAR_N)
      for (int q = 0; q < N; ++q) dx[q] += yv[i] * zi[q];
    }
    csr_spmv(N, rp, ci, val, dx, w);  /* true residual at the restart */
#pragma omp parallel for schedule(static) if (N >= PAR_N)
    for (int q = 0; q < N; ++q) w[q] = rhs[q] - w[q];
    beta = sqrt(vdot(N, w, w));
  }
  st->gmres_its = its;
  st->t_gmres = omp_get_wtime() - t0;
  /* line search with assemble_rhs (zero_constraints: the update vanishes on constrained rows) */
  t0 = omp_get_wtime();
  double res = res0;
  for (double alpha = 1.0; alpha > 1e-3; alpha *= 0.5) {
#pragma omp parallel for schedule(static) if (N >= PAR_N)
    for (int q = 0; q < N; ++q) xt[q] = x[q] + (p->constrained[q] ? 0. : alpha * dx[q]);
    assemble_csr(p, xt, u1, u2, u3, rp, ci, dg, NULL, rhs, 0);
    ++st->line_search_rhs;
    res = sqrt(vdot(N, rhs, rhs));
    if (res < 0.9 * res0) break;
  }
  memcpy(x, xt, sizeof(double) * (size_t)N);
  st->res1 = res;
  st->t_linesearch = omp_get_wtime() - t0;
  free(dcnt); free(dofs); free(dcell); free(fillp); free(rp); free(mark); free(ci); free(dg); free(val); free(lu);
  free(rhs); free(dx); free(V); free(Z); free(w); free(H); free(g); free(cs); free(sn); free(yv); free(xt);
  return 0;
}
