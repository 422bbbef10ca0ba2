// gls_common.hpp — shared host/device definitions of the MI355X GLS Navier–Stokes path.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace gls {

constexpr int kMaxNodes1D = 4;  // k <= 3
constexpr int kMaxQ1D = 5;      // QGauss(n) with n <= 5

constexpr int ipow(int b, int e) { return e == 0 ? 1 : b * ipow(b, e - 1); }

// MODE_LIN / MODE_JVQ (brick kernels only): MODE_LIN stores the linearization at every quadrature
// point (u, grad u, tau, R_s: kQData doubles) once per state; MODE_JVQ applies J.v from it.
enum Mode { MODE_RESIDUAL = 0, MODE_JV = 1, MODE_DIAG = 2, MODE_LIN = 3, MODE_JVQ = 4,
            MODE_RESLIN = 5 /* pencil kernel: residual + linearization + diagonal in one pass */ };
constexpr int kQData = 16;  // u[3], grad u[3][3], tau, R_s[3]

// Reference-cell 1D tables on [0,1] (deal.II unit cell): Lagrange basis on Gauss–Lobatto
// support points evaluated at QGauss points. [q][node].
struct Tables1D {
  double V[kMaxQ1D][kMaxNodes1D];   // velocity basis value
  double D[kMaxQ1D][kMaxNodes1D];   // d/dxi
  double S[kMaxQ1D][kMaxNodes1D];   // d2/dxi2
  double Vp[kMaxQ1D][kMaxNodes1D];  // pressure basis value
  double Dp[kMaxQ1D][kMaxNodes1D];  // pressure d/dxi
  double w[kMaxQ1D];                // Gauss weights on [0,1]
  double xi[kMaxQ1D];               // Gauss points on [0,1]
};

// General (mapped) cells: per quadrature point geometry, [n_cells][nq][kGeo] doubles:
//   x_q (3), JxW, J^-1 [a][i] = d xi_a / d x_i (9, row-major), G = J^-1 J^-T (6: 00 11 22 01 02 12),
//   c_k = sum_ab G_ab d2 x_k / d xi_a d xi_b (3): grad phi = J^-T grad_ref phi and
//   lap phi = sum_ab G_ab d2_ref phi - c . grad phi (FEValues hessians on MappingQ cells)
constexpr int kGeo = 22;
constexpr int kGeoX = 0, kGeoJxW = 3, kGeoJI = 4, kGeoG = 13, kGeoC = 19;

// Per-launch operator parameters (device pointers).
struct OpParams {
  int n_cells;
  int n_vnodes;
  int n_pnodes;
  int n_hist;                 // history vectors read by this scheme (0..3)
  const int32_t *cell_vnodes;
  const int32_t *cell_pnodes; // nullptr -> use cell_vnodes (kp == k)
  const double *geo;          // [n_cells][4]: h_x, h_y, h_z, h_stab
  const double *x0;           // [n_cells][3] (SRF only)
  const double *gq;           // [n_cells][nq][kGeo] mapped-cell geometry, nullptr = axis-aligned boxes
  const double *force_q;      // [n_cells][nq][dim] or nullptr
  const uint8_t *vmask;       // [n_vnodes] zero_constraints bits, nullptr = none
  const uint8_t *hmask;       // [n_vnodes] hanging velocity components (MODE_DIAG: |K_ii| per cell)
  // pencil kernel on the complete sibling groups of an adapted forest: first cell of each (compact)
  // brick; the launch writes element vectors (ev) instead of node sums
  const int32_t *brick_cell0;
  const int32_t *cell_list;  // per-cell kernels: the cells to run (NULL: all), e.g. those outside forest bricks
  int cell_list_n;
  const double *u;
  const double *h1, *h2, *h3; // history (solution_m1..m3)
  const double *v;            // JV input
  double *qd;                 // MODE_LIN output / MODE_JVQ input (brick wave-major layout)
  float *qdf;                 // FP32 copy of qd (MODE_JVQ in FP32: the multigrid smoother's J.v)
  int n_probe;                // MODE_JVQ probing: > 0 -> block b computes J e_(probe_base + b / n_bricks)
  int64_t probe_base;         //   into y + (b / n_bricks) * n_dofs (v unused)
  double *y;                  // output (brick-interior nodes: plain stores; others: slab or atomics)
  const int32_t *subset;      // brick kernels: launch only bricks subset[0 .. subset_n) (slab scheme), nullptr = all
  int subset_n;
  double *ev;                 // per-cell kernels: element vectors [n_cells][NV*dim + NP] instead of atomics
                              //   into y (summed per node in a fixed order by gather_element_vectors)
  int64_t bv_stride;          // per-cell MODE_JV batch (probing): blockIdx.y = vector, v / ev at these strides;
  int64_t bev_stride;         //   cell batches on which the vector vanishes skip their element vectors and
  uint8_t *bact;              //   exit, flagged 0 in bact[vector * gridDim.x + block] (1 = computed)
  const int32_t *work;        //   or: the (vector, block) pairs known to be active, one block each (bact read only)
  int n_work;
  double *slab;               // brick path: [n_bricks][NBND][4] partial sums of brick-boundary nodes
                              //   (nullptr -> FP64 atomics into y, which the caller zeroes)
  float *slabf;               // FP32 kernels: the same slab in FP32 when set (takes precedence)
  // fused damped-Jacobi sweep (MODE_JVQ brick kernel, interior nodes; the slab sum does the rest):
  // instead of y = A v, jx <- jx + jomega (jb - y) / jd with y = jd * jx on zero_constraints rows
  // (jx aliases v: a brick's interior nodes are read and written by that brick only)
  double *jx;
  const double *jb, *jd;
  double jomega;
  // residual form (MODE_JVQ brick kernels, no jx): y = rb - A v instead of y = A v (nullptr: off)
  const double *rb;
  // with rb (pencil J.v, hyper_cube slab sum): the first damped-Jacobi sweep from x = 0 fused in front of
  // the residual: v = 0 + jomega rb / jd is formed in the gather and stored to jx0 (interior nodes here,
  // surface nodes by the slab sum), y = rb - A v
  double *jx0;
  // MODE_RESLIN: the residual's node sums (brick-interior nodes, and the brick-surface slab summed by
  // the slab sum) next to the diagonal's in y / slab
  double *res_y;
  double *res_slab;
  // colored brick launches (replace the slab + k_slab_sum): bricks are launched one color at a time
  // (no two bricks of a color share a node); a brick-surface node's running sum lives in acc[] and
  // is carried across colors in color order (deterministic): the node's first-color brick writes,
  // later ones add, its last-color brick completes it (plain / residual / fused-Jacobi store)
  const int32_t *bricks;      // brick ids sorted by color (nullptr: no coloring)
  const uint16_t *ncolor;     // [n_vnodes] bit c set: a brick of color c holds the node
  double *acc;                // running sums of surface nodes (y itself unless the fused Jacobi sweep)
  int n_colors;
  int color;                  // color of this launch (set by the launcher)
  int color_off[17];          // bricks[color_off[c] .. color_off[c+1]) have color c
  double nu;
  double alpha[4];            // time coefficients applied to (u, u1, u2, u3) in R_s / rhs
  double alpha_jac;           // mass coefficient of the Jacobian (bdf[0] / sdirk[0][0])
  double sdt2;                // (1/dt)^2 for transient tau, 0 when steady
  int srf;
  double omega[3];
  // FP32 smoother J.v on the cube's bricks: the Oseen (Picard) linearization instead of Newton's, i.e. without
  // the (grad u) v terms and the SUPG term tau (v . grad phi) R_s (the multigrid smoother's operator,
  // gls_mg_params.smoother_operator = 1); the outer GMRES operator is never affected
  int oseen;
  // per-cell kernels: the linearization cache [cell][NCQ][NQ] (u, grad u, tau, R_s at every quadrature point,
  // NCQ = dim + dim^2 + 1 + dim): cq_mode 1 = MODE_DIAG writes it, 2 = MODE_JV reads it instead of re-deriving
  // u, its derivatives, the history terms and R_s from the state (same values: the diagonal pass computes them
  // with the same code)
  double *cq;
  int cq_mode;
};

}  // namespace gls
