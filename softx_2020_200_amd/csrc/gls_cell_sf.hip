// gls_cell_sf.hip — sum-factorized per-cell GLS Jacobian action for 3D Q2-Qk' cells (k' = 1, 2) on
// mapped (MappingQ, curved / unstructured) and axis-aligned cells, from the per-cell linearization cache.
//
// Replaces the dense thread-per-(cell, q) contraction of gls_cell_kernel<3, 2, kp, 3, MODE_JV, GEN, 256, true>
// (gls_cell_kernels.hip) for the J.v that GMRES and the multigrid smoother call: same inputs (the cache P.cq
// written by the diagonal pass at this state, P.gq mapped geometry, the constraint mask), same output (element
// vectors P.ev, summed per node in a fixed order by gather_element_vectors), same arithmetic per quadrature
// point (gls_navier_stokes.cc:548-622 restated: the Jacobian of the strong residual, SUPG and PSPG terms,
// grad-div omitted as in the reference).
//
// Dataflow: one wave = one workgroup = 2 cells, lane (cell, i, j, k) with i + 3 j + 9 k < 27 (54 of 64 lanes).
//   gather  : v at the cell's 27 velocity nodes (Dirichlet columns masked) and its pressure nodes -> LDS
//   forward : x sweep (V, D, S of the 1D Q2 basis at the Gauss points), y sweep (6 products), z sweep in
//             registers at the lane's quadrature point: value, reference gradient and the 6 reference second
//             derivatives of each velocity component (27 x (3 + 6 + 10) x 3 FMAs per component instead of the
//             dense 27 x 27 x 10); the pressure (Q1: 8 nodes, Q2: 27) by value and gradient sweeps
//   pointwise: MappingQ -- physical gradient J^-T g, Laplacian sum_ab G_ab H_ab - c . grad -- or the box map;
//             the cached u, grad u, tau, R_s; the test coefficients turned back to the reference cell (J^-1)
//   backward: the transposed z, y and x sweeps for the 3 velocity test fields (and the pressure test field on
//             Q2-Q2; Q2-Q1's 8 pressure test functions are integrated densely)
// LDS hand-offs are wave-local (one wave per workgroup, gls_brick_common.hpp wave_sync): no workgroup barrier.
#include "gls_brick_common.hpp"
#include "gls_launch.hpp"

#include <cstdlib>

namespace gls {
namespace {

constexpr int kSfCells = 2;   // cells per wave
constexpr int kSfR1 = 324;    // per-cell LDS doubles: forward x stage (3 x 3 + 2) x 27, backward z stage 4 x 3 x 27
constexpr int kSfR2 = 567;    // forward y stage (3 x 6 + 3) x 27, test coefficients 16 x 27, backward y 4 x 2 x 27

// The J.v's pointwise part at quadrature point q = i + 3 j + 9 k of `cell` (gls_navier_stokes.cc:548-622):
// v's value, reference gradient and reference Hessian (xx yy zz xy xz yz) per velocity component, the pressure
// value and reference gradient in; the 16 test coefficients out (velocity c: value and reference-gradient
// coefficients at 4c, pressure at 12), with the MappingQ (GEN) or box geometry and the linearization cache.
template <bool GEN>
__device__ __forceinline__ void jv_point(const OpParams &P, int64_t cell, int q, int i, int j, int k, const double *sW,
                                         double (&v)[3], double (&gv)[3][3], const double (&H)[3][6], double vp,
                                         double (&gvp)[3], double (&tc)[16]) {
  // geometry
  double JI[3][3], JxW, lv[3];
  double ih[3] = {1.0, 1.0, 1.0};
  if constexpr (GEN) {
    const double *g = P.gq + (cell * 27 + q) * kGeo;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int e = 0; e < 3; ++e) JI[a][e] = g[kGeoJI + 3 * a + e];
    double Gm[6], cg[3];
#pragma unroll
    for (int t = 0; t < 6; ++t) Gm[t] = g[kGeoG + t];
#pragma unroll
    for (int t = 0; t < 3; ++t) cg[t] = g[kGeoC + t];
    JxW = g[kGeoJxW];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double L = Gm[0] * H[c][0] + Gm[1] * H[c][1] + 2 * Gm[3] * H[c][3] + Gm[2] * H[c][2] + 2 * Gm[4] * H[c][4] +
                 2 * Gm[5] * H[c][5];
      double o[3];
#pragma unroll
      for (int e = 0; e < 3; ++e) o[e] = JI[0][e] * gv[c][0] + JI[1][e] * gv[c][1] + JI[2][e] * gv[c][2];
#pragma unroll
      for (int e = 0; e < 3; ++e) gv[c][e] = o[e];
#pragma unroll
      for (int e = 0; e < 3; ++e) L -= cg[e] * gv[c][e];
      lv[c] = L;
    }
    double o[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) o[e] = JI[0][e] * gvp[0] + JI[1][e] * gvp[1] + JI[2][e] * gvp[2];
#pragma unroll
    for (int e = 0; e < 3; ++e) gvp[e] = o[e];
  } else {
    const double hx = P.geo[cell * 4 + 0], hy = P.geo[cell * 4 + 1], hz = P.geo[cell * 4 + 2];
    ih[0] = 1.0 / hx;
    ih[1] = 1.0 / hy;
    ih[2] = 1.0 / hz;
    JxW = sW[i] * sW[j] * sW[k] * hx * hy * hz;
    const double wy = (hx * hx) / (hy * hy), wz = (hx * hx) / (hz * hz), il2 = ih[0] * ih[0];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      lv[c] = (H[c][0] + wy * H[c][1] + wz * H[c][2]) * il2;
#pragma unroll
      for (int e = 0; e < 3; ++e) gv[c][e] *= ih[e];
    }
#pragma unroll
    for (int e = 0; e < 3; ++e) gvp[e] *= ih[e];
  }
  // the linearization cache of this point (u, grad u, tau, R_s)
  const double *cq = P.cq + cell * 16 * 27 + q;
  double u[3], gu[3][3], R[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) u[c] = cq[c * 27];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int e = 0; e < 3; ++e) gu[c][e] = cq[(3 + 3 * c + e) * 27];
  const double tau = cq[12 * 27];
#pragma unroll
  for (int c = 0; c < 3; ++c) R[c] = cq[(13 + c) * 27];

  const double nu = P.nu, aj = P.alpha_jac;
  double S[3], A[3], divv = 0.;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double gvu = 0., guv = 0.;
#pragma unroll
    for (int e = 0; e < 3; ++e) { guv += gu[c][e] * v[e]; gvu += gv[c][e] * u[e]; }
    A[c] = guv + gvu + aj * v[c];
    S[c] = guv + gvu + gvp[c] - nu * lv[c] + aj * v[c];
    divv += gv[c][c];
  }
  if (P.srf) {
    const double *om = P.omega;
    const double cj[3] = {2 * (om[1] * v[2] - om[2] * v[1]), 2 * (om[2] * v[0] - om[0] * v[2]),
                          2 * (om[0] * v[1] - om[1] * v[0])};
#pragma unroll
    for (int c = 0; c < 3; ++c) { A[c] += cj[c]; S[c] += cj[c]; }
  }
  auto to_ref = [&](double (&t)[3]) {
    if constexpr (GEN) {
      double o[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) o[a] = JI[a][0] * t[0] + JI[a][1] * t[1] + JI[a][2] * t[2];
#pragma unroll
      for (int a = 0; a < 3; ++a) t[a] = o[a];
    } else {
#pragma unroll
      for (int a = 0; a < 3; ++a) t[a] *= ih[a];
    }
  };
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    tc[4 * c] = JxW * A[c];
    double t[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) t[e] = JxW * (nu * gv[c][e] - (c == e ? vp : 0.0) + tau * S[c] * u[e] + tau * R[c] * v[e]);
    to_ref(t);
#pragma unroll
    for (int e = 0; e < 3; ++e) tc[4 * c + 1 + e] = t[e];
  }
  tc[12] = JxW * divv;
  {
    double t[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) t[e] = JxW * tau * S[e];
    to_ref(t);
#pragma unroll
    for (int e = 0; e < 3; ++e) tc[13 + e] = t[e];
  }
}

template <int KP, bool GEN>
__global__ void __launch_bounds__(64) k_cell_sf_jv(const OpParams P, const Tables1D T) {
  constexpr int NV = 27, NQ = 27, NP = (KP + 1) * (KP + 1) * (KP + 1);
  constexpr bool PSF = KP == 2;  // pressure through the sweeps too
  __shared__ double sV[3][3], sD[3][3], sS[3][3], sW[3];  // [q][node] Q2 tables, Gauss weights
  __shared__ double sVp[3][KP + 1], sDp[3][KP + 1];
  __shared__ __attribute__((aligned(16))) double sv[kSfCells][4][NV];  // v per field at the nodes
  __shared__ __attribute__((aligned(16))) double r1[kSfCells][kSfR1];
  __shared__ __attribute__((aligned(16))) double r2[kSfCells][kSfR2];

  const int lane = threadIdx.x;
  if (lane < 9) {
    const int q = lane / 3, a = lane % 3;
    sV[q][a] = T.V[q][a];
    sD[q][a] = T.D[q][a];
    sS[q][a] = T.S[q][a];
    if (a == 0) sW[q] = T.w[q];
  }
  if (lane < 3 * (KP + 1)) {
    const int q = lane / (KP + 1), a = lane % (KP + 1);
    sVp[q][a] = T.Vp[q][a];
    sDp[q][a] = T.Dp[q][a];
  }
  const int n_run = P.cell_list ? P.cell_list_n : P.n_cells;
  const int nblk = (n_run + kSfCells - 1) / kSfCells;
  // batched ILU probing from the recorded work list: block = one (probe vector, 2-cell batch) pair known active
  const bool listed = P.work != nullptr;
  const int wb = xcd_swizzle((int)blockIdx.x, listed ? P.n_work : nblk);  // XCD-aware: neighbouring cells share an L2
  const int blk = listed ? P.work[2 * wb + 1] : wb;
  const double *Pv = listed ? P.v + (int64_t)P.work[2 * wb] * P.bv_stride : P.v;
  double *Pev = listed ? P.ev + (int64_t)P.work[2 * wb] * P.bev_stride : P.ev;
  const int cl = lane / 27, id = lane % 27;
  const int crun = blk * kSfCells + cl;
  const bool act = cl < kSfCells && crun < n_run;
  const int64_t cell = act ? (P.cell_list ? (int64_t)P.cell_list[crun] : (int64_t)crun) : 0;
  const int i = id % 3, j = (id / 3) % 3, k = id / 9;
  const int64_t voff = 3 * (int64_t)P.n_vnodes;
  double *R1 = r1[cl < kSfCells ? cl : 0];
  double *R2 = r2[cl < kSfCells ? cl : 0];
  double(*V3)[NV] = sv[cl < kSfCells ? cl : 0];

  // ---- gather: lane = node id
  if (act) {
    const int node = P.cell_vnodes[cell * NV + id];
    const unsigned m = P.vmask ? P.vmask[node] : 0u;
    const double *pv = Pv + (int64_t)node * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) V3[c][id] = ((m >> c) & 1u) ? 0.0 : pv[c];
    if (id < NP) {
      const int pn = P.cell_pnodes ? P.cell_pnodes[cell * NP + id] : node;
      V3[3][id] = Pv[voff + pn];
    }
  }
  wave_sync();

  // ---- forward x sweep: lane (qx = i, node y = j, node z = k)
  if (act) {
    const double v0 = sV[i][0], v1 = sV[i][1], v2 = sV[i][2];
    const double d0 = sD[i][0], d1 = sD[i][1], d2 = sD[i][2];
    const double s0 = sS[i][0], s1 = sS[i][1], s2 = sS[i][2];
    const int b = 3 * j + 9 * k;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double x0 = V3[c][b], x1 = V3[c][b + 1], x2 = V3[c][b + 2];
      R1[(3 * c + 0) * 27 + id] = v0 * x0 + v1 * x1 + v2 * x2;
      R1[(3 * c + 1) * 27 + id] = d0 * x0 + d1 * x1 + d2 * x2;
      R1[(3 * c + 2) * 27 + id] = s0 * x0 + s1 * x1 + s2 * x2;
    }
    if constexpr (PSF) {
      const double x0 = V3[3][b], x1 = V3[3][b + 1], x2 = V3[3][b + 2];
      R1[9 * 27 + id] = v0 * x0 + v1 * x1 + v2 * x2;
      R1[10 * 27 + id] = d0 * x0 + d1 * x1 + d2 * x2;
    }
  }
  wave_sync();
  // ---- forward y sweep: lane (qx = i, qy = j, node z = k); products [xop][yop]: VV VD VS DV DD SV
  if (act) {
    const double v0 = sV[j][0], v1 = sV[j][1], v2 = sV[j][2];
    const double d0 = sD[j][0], d1 = sD[j][1], d2 = sD[j][2];
    const double s0 = sS[j][0], s1 = sS[j][1], s2 = sS[j][2];
    const int b = i + 9 * k;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double *XV = R1 + (3 * c + 0) * 27 + b, *XD = R1 + (3 * c + 1) * 27 + b, *XS = R1 + (3 * c + 2) * 27 + b;
      const double a0 = XV[0], a1 = XV[3], a2 = XV[6];
      const double e0 = XD[0], e1 = XD[3], e2 = XD[6];
      const double f0 = XS[0], f1 = XS[3], f2 = XS[6];
      double *Y = R2 + 6 * c * 27 + id;
      Y[0 * 27] = v0 * a0 + v1 * a1 + v2 * a2;
      Y[1 * 27] = d0 * a0 + d1 * a1 + d2 * a2;
      Y[2 * 27] = s0 * a0 + s1 * a1 + s2 * a2;
      Y[3 * 27] = v0 * e0 + v1 * e1 + v2 * e2;
      Y[4 * 27] = d0 * e0 + d1 * e1 + d2 * e2;
      Y[5 * 27] = v0 * f0 + v1 * f1 + v2 * f2;
    }
    if constexpr (PSF) {
      const double *XV = R1 + 9 * 27 + b, *XD = R1 + 10 * 27 + b;
      const double a0 = XV[0], a1 = XV[3], a2 = XV[6];
      const double e0 = XD[0], e1 = XD[3], e2 = XD[6];
      double *Y = R2 + 18 * 27 + id;
      Y[0 * 27] = v0 * a0 + v1 * a1 + v2 * a2;
      Y[1 * 27] = d0 * a0 + d1 * a1 + d2 * a2;
      Y[2 * 27] = v0 * e0 + v1 * e1 + v2 * e2;
    }
  }
  wave_sync();

  // ---- forward z sweep + pointwise: lane = quadrature point q = i + 3 j + 9 k
  double tc[16];  // test coefficients: velocity c: (value, d/dxi_0..2) at 4c, pressure at 12
#pragma unroll
  for (int t = 0; t < 16; ++t) tc[t] = 0.0;
  if (act) {
    const double v0 = sV[k][0], v1 = sV[k][1], v2 = sV[k][2];
    const double d0 = sD[k][0], d1 = sD[k][1], d2 = sD[k][2];
    const double s0 = sS[k][0], s1 = sS[k][1], s2 = sS[k][2];
    const int b = i + 3 * j;
    double v[3], gv[3][3], H[3][6];  // H: xx yy zz xy xz yz (reference)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double *Y = R2 + 6 * c * 27 + b;
      double y[6][3];
#pragma unroll
      for (int o = 0; o < 6; ++o) {
        y[o][0] = Y[o * 27];
        y[o][1] = Y[o * 27 + 9];
        y[o][2] = Y[o * 27 + 18];
      }
      v[c] = v0 * y[0][0] + v1 * y[0][1] + v2 * y[0][2];
      gv[c][0] = v0 * y[3][0] + v1 * y[3][1] + v2 * y[3][2];
      gv[c][1] = v0 * y[1][0] + v1 * y[1][1] + v2 * y[1][2];
      gv[c][2] = d0 * y[0][0] + d1 * y[0][1] + d2 * y[0][2];
      H[c][0] = v0 * y[5][0] + v1 * y[5][1] + v2 * y[5][2];
      H[c][1] = v0 * y[2][0] + v1 * y[2][1] + v2 * y[2][2];
      H[c][2] = s0 * y[0][0] + s1 * y[0][1] + s2 * y[0][2];
      H[c][3] = v0 * y[4][0] + v1 * y[4][1] + v2 * y[4][2];
      H[c][4] = d0 * y[3][0] + d1 * y[3][1] + d2 * y[3][2];
      H[c][5] = d0 * y[1][0] + d1 * y[1][1] + d2 * y[1][2];
    }
    double vp = 0., gvp[3] = {0., 0., 0.};
    if constexpr (PSF) {
      const double *Y = R2 + 18 * 27 + b;
      double y[3][3];
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        y[o][0] = Y[o * 27];
        y[o][1] = Y[o * 27 + 9];
        y[o][2] = Y[o * 27 + 18];
      }
      vp = v0 * y[0][0] + v1 * y[0][1] + v2 * y[0][2];
      gvp[0] = v0 * y[2][0] + v1 * y[2][1] + v2 * y[2][2];
      gvp[1] = v0 * y[1][0] + v1 * y[1][1] + v2 * y[1][2];
      gvp[2] = d0 * y[0][0] + d1 * y[0][1] + d2 * y[0][2];
    } else {  // Q1 pressure: 8 nodes, dense
#pragma unroll
      for (int az = 0; az < 2; ++az)
#pragma unroll
        for (int ay = 0; ay < 2; ++ay)
#pragma unroll
          for (int ax = 0; ax < 2; ++ax) {
            const double w = V3[3][ax + 2 * ay + 4 * az];
            const double vx = sVp[i][ax], vy = sVp[j][ay], vz = sVp[k][az];
            vp += w * vx * vy * vz;
            gvp[0] += w * sDp[i][ax] * vy * vz;
            gvp[1] += w * vx * sDp[j][ay] * vz;
            gvp[2] += w * vx * vy * sDp[k][az];
          }
    }
    jv_point<GEN>(P, cell, id, i, j, k, sW, v, gv, H, vp, gvp, tc);
  }
  wave_sync();  // every lane's y-stage reads are done before the coefficients overwrite that area
  if (act) {
#pragma unroll
    for (int t = 0; t < 16; ++t) R2[t * 27 + id] = tc[t];
  }
  wave_sync();

  // ---- backward z sweep: lane (qx = i, qy = j, node z = k): ZA = sum_qz V T0 + D T3, ZB = V T1, ZC = V T2
  constexpr int NFB = PSF ? 4 : 3;
  double outp = 0.;
  if (act) {
    const double v0 = sV[0][k], v1 = sV[1][k], v2 = sV[2][k];
    const double d0 = sD[0][k], d1 = sD[1][k], d2 = sD[2][k];
    const int b = i + 3 * j;
#pragma unroll
    for (int f = 0; f < NFB; ++f) {
      const double *Tt = R2 + 4 * f * 27 + b;
      double t[4][3];
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        t[o][0] = Tt[o * 27];
        t[o][1] = Tt[o * 27 + 9];
        t[o][2] = Tt[o * 27 + 18];
      }
      R1[(3 * f + 0) * 27 + id] = v0 * t[0][0] + v1 * t[0][1] + v2 * t[0][2] + d0 * t[3][0] + d1 * t[3][1] + d2 * t[3][2];
      R1[(3 * f + 1) * 27 + id] = v0 * t[1][0] + v1 * t[1][1] + v2 * t[1][2];
      R1[(3 * f + 2) * 27 + id] = v0 * t[2][0] + v1 * t[2][1] + v2 * t[2][2];
    }
    if constexpr (!PSF) {  // Q1 pressure test functions: lanes id < 8, dense over the 27 points
      if (id < 8) {
        const int ax = id & 1, ay = (id >> 1) & 1, az = id >> 2;
        const double *Tp = R2 + 12 * 27;
#pragma unroll 3
        for (int q = 0; q < NQ; ++q) {
          const int qx = q % 3, qy = (q / 3) % 3, qz = q / 9;
          const double vx = sVp[qx][ax], vy = sVp[qy][ay], vz = sVp[qz][az];
          outp += vx * vy * vz * Tp[q] + sDp[qx][ax] * vy * vz * Tp[27 + q] + vx * sDp[qy][ay] * vz * Tp[54 + q] +
                  vx * vy * sDp[qz][az] * Tp[81 + q];
        }
      }
    }
  }
  wave_sync();
  // ---- backward y sweep: lane (qx = i, node y = j, node z = k): YA = sum_qy V ZA + D ZC, YB = V ZB
  if (act) {
    const double v0 = sV[0][j], v1 = sV[1][j], v2 = sV[2][j];
    const double d0 = sD[0][j], d1 = sD[1][j], d2 = sD[2][j];
    const int b = i + 9 * k;
#pragma unroll
    for (int f = 0; f < NFB; ++f) {
      const double *Z = R1 + 3 * f * 27 + b;
      double z[3][3];
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        z[o][0] = Z[o * 27];
        z[o][1] = Z[o * 27 + 3];
        z[o][2] = Z[o * 27 + 6];
      }
      R2[(2 * f + 0) * 27 + id] = v0 * z[0][0] + v1 * z[0][1] + v2 * z[0][2] + d0 * z[2][0] + d1 * z[2][1] + d2 * z[2][2];
      R2[(2 * f + 1) * 27 + id] = v0 * z[1][0] + v1 * z[1][1] + v2 * z[1][2];
    }
  }
  wave_sync();
  // ---- backward x sweep: lane = node (i, j, k): out = sum_qx V YA + D YB; element vector store
  if (act) {
    const double v0 = sV[0][i], v1 = sV[1][i], v2 = sV[2][i];
    const double d0 = sD[0][i], d1 = sD[1][i], d2 = sD[2][i];
    const int b = 3 * j + 9 * k;
    double out[4];
#pragma unroll
    for (int f = 0; f < NFB; ++f) {
      const double *Y = R2 + 2 * f * 27 + b;
      out[f] = v0 * Y[0] + v1 * Y[1] + v2 * Y[2] + d0 * Y[27] + d1 * Y[28] + d2 * Y[29];
    }
    double *e = Pev + cell * (NV * 3 + NP);
#pragma unroll
    for (int c = 0; c < 3; ++c) e[id * 3 + c] = out[c];
    if constexpr (PSF) e[NV * 3 + id] = out[3];
    else if (id < 8) e[NV * 3 + id] = outp;
  }
}


// ---------------------------------------------------------------------------------------------------------------
// The same J.v with the dense per-cell contractions on the matrix cores (A/B against the sweeps above; selected by
// GLS_CELL_SF=2). v_mfma_f64_16x16x4f64: D[16 x 16] += A[16 x 4] B[4 x 16], lane l holds A[l & 15][l >> 4],
// B[l >> 4][l & 15] and D rows (l >> 4) + 4 r, column l & 15 (cdna_hip_programming.md, the f64 map).
// One wave = 5 cells; the 16 columns of every product are (cell, velocity component) pairs (15 used).
//   evaluate : per quadrature point q, E[op][col] = sum_a B_op(q, a) V[a][col] over the 27 nodes (7 k-steps of 4):
//              the 10 rows op = value, 3 reference derivatives, 6 reference second derivatives (16 padded);
//              the A operand (the basis product) is formed per lane from the 1D tables
//   pointwise: jv_point per (cell, q), 9 points of a chunk at a time
//   integrate: Y[a][col] = sum_(q, t) N_t(q, a) T[(q, t)][col] over 108 = 27 q x 4 (value, 3 derivatives)
//              k-steps of 4 (one q each), 2 row tiles of nodes
// The Q1 / Q2 pressure value, gradient and test integration stay on the VALU (dense, small).
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int kMfCells = 5;

template <int KP, bool GEN>
__global__ void __launch_bounds__(64) k_cell_mfma_jv(const OpParams P, const Tables1D T) {
  constexpr int NV = 27, NQ = 27, NP = (KP + 1) * (KP + 1) * (KP + 1), QC = 9;
  __shared__ double sTab[3][3][3], sW[3];  // [V, D, S][q][node]
  double(*sV)[3] = sTab[0];
  double(*sD)[3] = sTab[1];
  double(*sS)[3] = sTab[2];
  __shared__ double sVp[3][KP + 1], sDp[3][KP + 1];
  __shared__ double sB[28][16];                 // node values [node][cell * 3 + component], node 27 / column 15: 0
  __shared__ double sPv[kMfCells][NP];          // pressure node values
  __shared__ double sE[QC][10][16];             // evaluations of a chunk of 9 points
  __shared__ double sT[NQ][4][16];              // velocity test coefficients [q][value, d0, d1, d2][column]
  __shared__ double sTp[kMfCells][NQ][4];       // pressure test coefficients
  const int lane = threadIdx.x;
  if (lane < 9) {
    const int q = lane / 3, a = lane % 3;
    sV[q][a] = T.V[q][a];
    sD[q][a] = T.D[q][a];
    sS[q][a] = T.S[q][a];
    if (a == 0) sW[q] = T.w[q];
  }
  if (lane < 3 * (KP + 1)) {
    const int q = lane / (KP + 1), a = lane % (KP + 1);
    sVp[q][a] = T.Vp[q][a];
    sDp[q][a] = T.Dp[q][a];
  }
  const int n_run = P.cell_list ? P.cell_list_n : P.n_cells;
  const int nblk = (n_run + kMfCells - 1) / kMfCells;
  const int blk = xcd_swizzle((int)blockIdx.x, nblk);
  auto cell_of = [&](int cl) -> int64_t {
    const int cr = blk * kMfCells + cl;
    return cr >= n_run ? -1 : (P.cell_list ? (int64_t)P.cell_list[cr] : (int64_t)cr);
  };
  const int64_t voff = 3 * (int64_t)P.n_vnodes;
  // ---- gather
  for (int t = lane; t < 28 * 16; t += 64) (&sB[0][0])[t] = 0.0;
  wave_sync();
  for (int t = lane; t < kMfCells * NV; t += 64) {
    const int cl = t / NV, a = t % NV;
    const int64_t cell = cell_of(cl);
    if (cell < 0) continue;
    const int node = P.cell_vnodes[cell * NV + a];
    const unsigned m = P.vmask ? P.vmask[node] : 0u;
#pragma unroll
    for (int c = 0; c < 3; ++c) sB[a][cl * 3 + c] = ((m >> c) & 1u) ? 0.0 : P.v[(int64_t)node * 3 + c];
    if (a < NP) sPv[cl][a] = P.v[voff + (P.cell_pnodes ? P.cell_pnodes[cell * NP + a] : node)];
  }
  wave_sync();
  // the lane's evaluation row: op = lane & 15 -> (x, y, z) 1D operator: 0 V, 1 D, 2 S
  const int op = lane & 15, kq = lane >> 4;
  constexpr int OPX[10] = {0, 1, 0, 0, 2, 0, 0, 1, 1, 0}, OPY[10] = {0, 0, 1, 0, 0, 2, 0, 1, 0, 1},
                OPZ[10] = {0, 0, 0, 1, 0, 0, 2, 0, 1, 1};
  const int ox = op < 10 ? OPX[op] : 0, oy = op < 10 ? OPY[op] : 0, oz = op < 10 ? OPZ[op] : 0;
  for (int q0 = 0; q0 < NQ; q0 += QC) {
    for (int qi = 0; qi < QC; ++qi) {  // ---- evaluate: one 16 x 16 tile per point
      const int q = q0 + qi, qx = q % 3, qy = (q / 3) % 3, qz = q / 9;
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 7; ++ks) {
        const int a = 4 * ks + kq;
        const int ax = a % 3, ay = (a / 3) % 3, az = a / 9;
        const double av = (op < 10 && a < NV) ? sTab[ox][qx][ax] * sTab[oy][qy][ay] * sTab[oz][qz][az] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, sB[a][op], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = kq + 4 * r;
        if (row < 10) sE[qi][row][op] = acc[r];
      }
    }
    wave_sync();
    if (lane < kMfCells * QC) {  // ---- pointwise, lane = (cell, point of the chunk)
      const int cl = lane / QC, qi = lane % QC, q = q0 + qi;
      const int64_t cell = cell_of(cl);
      double tc[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) tc[t] = 0.0;
      if (cell >= 0) {
        const int i = q % 3, j = (q / 3) % 3, k = q / 9;
        double v[3], gv[3][3], H[3][6];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int col = cl * 3 + c;
          v[c] = sE[qi][0][col];
#pragma unroll
          for (int e = 0; e < 3; ++e) gv[c][e] = sE[qi][1 + e][col];
#pragma unroll
          for (int h = 0; h < 6; ++h) H[c][h] = sE[qi][4 + h][col];
        }
        double vp = 0., gvp[3] = {0., 0., 0.};
        for (int b = 0; b < NP; ++b) {
          const int bx = b % (KP + 1), by = (b / (KP + 1)) % (KP + 1), bz = b / ((KP + 1) * (KP + 1));
          const double w = sPv[cl][b];
          const double vx = sVp[i][bx], vy = sVp[j][by], vz = sVp[k][bz];
          vp += w * vx * vy * vz;
          gvp[0] += w * sDp[i][bx] * vy * vz;
          gvp[1] += w * vx * sDp[j][by] * vz;
          gvp[2] += w * vx * vy * sDp[k][bz];
        }
        jv_point<GEN>(P, cell, q, i, j, k, sW, v, gv, H, vp, gvp, tc);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int t = 0; t < 4; ++t) sT[q][t][cl * 3 + c] = tc[4 * c + t];
#pragma unroll
      for (int t = 0; t < 4; ++t) sTp[cl][q][t] = tc[12 + t];
    }
    if (q0 == 0)
      for (int t = lane; t < NQ * 4; t += 64) sT[t / 4][t % 4][15] = 0.0;  // the padding column
    wave_sync();
  }
  // ---- integrate (velocity test functions): node rows 16 mt + (lane & 15), k = the point's 4 test operators
  for (int mt = 0; mt < 2; ++mt) {
    const int a = 16 * mt + op;
    const int ax = a % 3, ay = (a / 3) % 3, az = a / 9;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < NQ; ++q) {
      const int qx = q % 3, qy = (q / 3) % 3, qz = q / 9;
      double av = 0.0;
      if (a < NV) {
        const double vx = sV[qx][ax], vy = sV[qy][ay], vz = sV[qz][az];
        av = kq == 0 ? vx * vy * vz : kq == 1 ? sD[qx][ax] * vy * vz : kq == 2 ? vx * sD[qy][ay] * vz : vx * vy * sD[qz][az];
      }
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, sT[q][kq][op], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int node = 16 * mt + kq + 4 * r, col = op, cl = col / 3;
      const int64_t cell = col < 15 ? cell_of(cl) : -1;
      if (node < NV && cell >= 0) P.ev[cell * (NV * 3 + NP) + node * 3 + col % 3] = acc[r];
    }
  }
  // ---- pressure test functions (VALU): lane -> (cell, pressure node)
  for (int t = lane; t < kMfCells * NP; t += 64) {
    const int cl = t / NP, b = t % NP;
    const int64_t cell = cell_of(cl);
    if (cell < 0) continue;
    const int bx = b % (KP + 1), by = (b / (KP + 1)) % (KP + 1), bz = b / ((KP + 1) * (KP + 1));
    double o = 0.;
    for (int q = 0; q < NQ; ++q) {
      const int qx = q % 3, qy = (q / 3) % 3, qz = q / 9;
      const double vx = sVp[qx][bx], vy = sVp[qy][by], vz = sVp[qz][bz];
      o += vx * vy * vz * sTp[cl][q][0] + sDp[qx][bx] * vy * vz * sTp[cl][q][1] + vx * sDp[qy][by] * vz * sTp[cl][q][2] +
           vx * vy * sDp[qz][bz] * sTp[cl][q][3];
    }
    P.ev[cell * (NV * 3 + NP) + NV * 3 + b] = o;
  }
}

}  // namespace

// GLS_CELL_SF (read per launch: tests compare the kernels in one process): unset / 1 = the sweeps (default),
// 0 = the dense thread-per-(cell, q) kernel, 2 = the MFMA contractions (A/B)
static int cell_sf_mode() {
  const char *e = std::getenv("GLS_CELL_SF");
  return e ? std::atoi(e) : 1;
}
bool cell_sf_enabled() { return cell_sf_mode() != 0; }

// J.v from the linearization cache (P.cq, cq_mode 2) into element vectors (P.ev); hipErrorNotSupported when the
// launch is not the sum-factorized kernel's (2D, other degrees, probing batches, no cache, atomics)
hipError_t launch_cell_sf_jv(int dim, int k, int kp, int nq1d, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (!cell_sf_enabled() || dim != 3 || k != 2 || nq1d != 3 || (kp != 1 && kp != 2)) return hipErrorNotSupported;
  if (!P.cq || P.cq_mode != 2 || (P.bv_stride && !P.work) || !P.ev || P.oseen) return hipErrorNotSupported;
  if (P.work && P.cell_list) return hipErrorNotSupported;  // probes run over all cells
  const int n_run = P.cell_list ? P.cell_list_n : P.n_cells;
  if (n_run <= 0 || (P.work && P.n_work <= 0)) return hipSuccess;
  if (P.work) {  // listed (probe vector, 2-cell batch) blocks: the dense probe kernel's batches of 64 / 27 = 2 cells
    static_assert(kSfCells == 2, "work-list batches are the 64-thread dense kernel's 2-cell batches");
    if (cell_sf_mode() == 2) return hipErrorNotSupported;
    if (kp == 1) {
      if (P.gq) hipLaunchKernelGGL((k_cell_sf_jv<1, true>), dim3((unsigned)P.n_work), dim3(64), 0, s, P, T);
      else hipLaunchKernelGGL((k_cell_sf_jv<1, false>), dim3((unsigned)P.n_work), dim3(64), 0, s, P, T);
    } else {
      if (P.gq) hipLaunchKernelGGL((k_cell_sf_jv<2, true>), dim3((unsigned)P.n_work), dim3(64), 0, s, P, T);
      else hipLaunchKernelGGL((k_cell_sf_jv<2, false>), dim3((unsigned)P.n_work), dim3(64), 0, s, P, T);
    }
    return hipGetLastError();
  }
  if (cell_sf_mode() == 2) {
    const unsigned mb = (unsigned)((n_run + kMfCells - 1) / kMfCells);
    if (kp == 1) {
      if (P.gq) hipLaunchKernelGGL((k_cell_mfma_jv<1, true>), dim3(mb), dim3(64), 0, s, P, T);
      else hipLaunchKernelGGL((k_cell_mfma_jv<1, false>), dim3(mb), dim3(64), 0, s, P, T);
    } else {
      if (P.gq) hipLaunchKernelGGL((k_cell_mfma_jv<2, true>), dim3(mb), dim3(64), 0, s, P, T);
      else hipLaunchKernelGGL((k_cell_mfma_jv<2, false>), dim3(mb), dim3(64), 0, s, P, T);
    }
    return hipGetLastError();
  }
  const unsigned blocks = (unsigned)((n_run + kSfCells - 1) / kSfCells);
  if (kp == 1) {
    if (P.gq) hipLaunchKernelGGL((k_cell_sf_jv<1, true>), dim3(blocks), dim3(64), 0, s, P, T);
    else hipLaunchKernelGGL((k_cell_sf_jv<1, false>), dim3(blocks), dim3(64), 0, s, P, T);
  } else {
    if (P.gq) hipLaunchKernelGGL((k_cell_sf_jv<2, true>), dim3(blocks), dim3(64), 0, s, P, T);
    else hipLaunchKernelGGL((k_cell_sf_jv<2, false>), dim3(blocks), dim3(64), 0, s, P, T);
  }
  return hipGetLastError();
}

}  // namespace gls
