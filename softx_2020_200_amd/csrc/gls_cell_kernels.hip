// gls_cell_kernels.hip — per-cell GLS (SUPG/PSPG) Navier–Stokes operators for gfx950.
//
// One workgroup = a batch of CB cells (CB*NQ <= 256 threads: Q2 3D -> 9 cells x 27 q).
// Phases (all in one launch):
//   1. gather   : cell->node index rows (coalesced int32 reads) -> DoF values of u, history,
//                 and v (JV) into LDS, Dirichlet columns masked (P v).
//   2. evaluate : one thread per (cell, q): dense basis x coefficient contraction over the
//                 cell's nodes; the Qk basis is formed from 1D tables staged in LDS
//                 (tensor product), so no n_dofs x n_q table is read from memory.
//   3. pointwise: tau, strong residual R_s, S(v) and the test-function coefficients
//                 (restated from gls_navier_stokes.cc:387-748, Appendix A of SURVEY.md).
//   4. integrate: one thread per (cell, node): transposed contraction sum_q B^T coef.
//   5. scatter  : element vectors stored per cell, then summed per node in a fixed (cell, local node)
//                 order by gather_element_vectors (bit-reproducible); FP64 global atomics into the
//                 output vector only when no element-vector buffer is given.
//
// Modes: residual (assemble_rhs), Jacobian action (matrix-free assembleGLS<true> . v),
// Jacobian diagonal (for the Jacobi preconditioner and the deal.II constrained-row diagonal).
// GEN: mapped (curved / unstructured) cells. The contractions stay on the reference cell; the
// per-q geometry (P.gq: J^-1, JxW, G = J^-1 J^-T, the Hessian correction c, x_q) turns reference
// gradients into physical ones (J^-T), the reference Hessian into the physical Laplacian
// (sum G_ab H_ab - c . grad), and physical test coefficients back to reference ones (J^-1) —
// FEValues with MappingQ (gls_navier_stokes.cc:245-252) restated per quadrature point.
#include "gls_common.hpp"
#include "gls_launch.hpp"

namespace gls {

template <int DIM, int K, int KP, int NQ1, int TPB = 256>
struct Cfg {
  static constexpr int NV = ipow(K + 1, DIM);
  static constexpr int NP = ipow(KP + 1, DIM);
  static constexpr int NQ = ipow(NQ1, DIM);
  static constexpr int CB = TPB / NQ;  // cells per workgroup (TPB = 64: the batched probe launches)
  static constexpr int NT = DIM * (DIM + 1) + DIM + 1;  // test coefficients per q
  static constexpr int K1 = K + 1, KP1 = KP + 1;
  static constexpr int TABN = 5 * kMaxQ1D * kMaxNodes1D + 2 * kMaxQ1D;
};

// CQ: J.v from the linearization cache the diagonal pass wrote (P.cq, cq_mode 2) -- its own instantiation, so the
// state-field sums drop out at compile time and the evaluation rows unroll at the old register count (198 / 248
// VGPRs on boxes / mapped cells; profiles/r05_ab_cell_cache_instantiation.txt: taylorcouette3d -7 % per Newton step)
template <int DIM, int K, int KP, int NQ1, int MODE, bool GEN = false, int TPB = 256, bool CQ = false>
__global__ void __launch_bounds__(TPB) gls_cell_kernel(const OpParams P, const Tables1D T) {
  static_assert(!CQ || MODE == MODE_JV, "the cache feeds J.v only");
  using C = Cfg<DIM, K, KP, NQ1, TPB>;
  constexpr int NV = C::NV, NP = C::NP, NQ = C::NQ, CB = C::CB, NT = C::NT;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double *sTab = smem;                              // Tables1D copy
  double *sU = sTab + ((C::TABN + 1) & ~1);         // [CB][NV][DIM]
  double *sP = sU + CB * NV * DIM;                  // [CB][NP]
  double *sH = sP + CB * NP;                        // [n_hist][CB][NV][DIM]
  double *sV = sH + 3 * CB * NV * DIM;              // [CB][NV][DIM]   (JV)
  double *sVP = sV + CB * NV * DIM;                 // [CB][NP]        (JV)
  double *sT = sVP + CB * NP;                       // [CB][NQ][NT]

  const double(*tV)[kMaxNodes1D] = reinterpret_cast<const double(*)[kMaxNodes1D]>(sTab);
  const double(*tD)[kMaxNodes1D] = tV + kMaxQ1D;
  const double(*tS)[kMaxNodes1D] = tD + kMaxQ1D;
  const double(*tVp)[kMaxNodes1D] = tS + kMaxQ1D;
  const double(*tDp)[kMaxNodes1D] = tVp + kMaxQ1D;
  const double *tW = sTab + 5 * kMaxQ1D * kMaxNodes1D;
  const double *tXi = tW + kMaxQ1D;

  const int tid = threadIdx.x;
  // batched probing from a recorded work list: this block's (vector, cell batch) pair, known active
  const bool listed = MODE == MODE_JV && P.work != nullptr;
  const int bx = listed ? P.work[2 * blockIdx.x + 1] : (int)blockIdx.x;
  const int by = listed ? P.work[2 * blockIdx.x] : (int)blockIdx.y;
  const int c0 = bx * CB;
  // cell list (adapted forests: the cells outside the pencil's sibling-group bricks), else all cells
  const int ncb = min(CB, (P.cell_list ? P.cell_list_n : P.n_cells) - c0);
  auto cid = [&](int cl) -> int64_t { return P.cell_list ? (int64_t)P.cell_list[c0 + cl] : (int64_t)(c0 + cl); };
  const int64_t voff = (int64_t)DIM * P.n_vnodes;  // first pressure DoF
  constexpr int NCQ = DIM + DIM * DIM + 1 + DIM;    // linearization cache values per q (u, grad u, tau, R_s)
  constexpr bool cqr = CQ;                                      // J.v from the cache (launch_cell_g picks it)
  const bool cqw = MODE == MODE_DIAG && P.cq && P.cq_mode == 1;  // the diagonal pass fills it

  // batched J.v (probing): this block's vector; J is linear, so a batch of cells on which the vector
  // vanishes has zero element vectors (most (probe, cell batch) pairs of a distance-2 colored probe set)
  const double *Pv = P.v;
  double *Pev = P.ev;
  if constexpr (MODE == MODE_JV) {
    if (P.bv_stride) {
      Pv += (int64_t)by * P.bv_stride;
      Pev += (int64_t)by * P.bev_stride;
    }
    if (P.bv_stride && !listed) {
      int any = 0;
      for (int i = tid; i < ncb * NV; i += blockDim.x) {
        const int64_t b = (int64_t)P.cell_vnodes[cid(i / NV) * NV + i % NV] * DIM;
#pragma unroll
        for (int c = 0; c < DIM; ++c) any |= Pv[b + c] != 0.0;
      }
      for (int i = tid; i < ncb * NP; i += blockDim.x) {
        const int pn = P.cell_pnodes ? P.cell_pnodes[cid(i / NP) * NP + i % NP] : P.cell_vnodes[cid(i / NV) * NV + i % NV];
        any |= Pv[voff + pn] != 0.0;
      }
      const int act = __syncthreads_or(any);
      if (tid == 0) P.bact[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = act ? 1 : 0;
      if (!act) return;  // the batched gather reads these element vectors as zero
    }
  }
  // ---- stage tables
  {
    const double *src = reinterpret_cast<const double *>(&T);
    for (int i = tid; i < C::TABN; i += blockDim.x) sTab[i] = src[i];
  }
  // ---- 1. gather (velocity-type fields)
  for (int i = tid; i < ncb * NV; i += blockDim.x) {
    const int node = P.cell_vnodes[cid(i / NV) * NV + i % NV];
    const int64_t b = (int64_t)node * DIM;
    if constexpr (MODE == MODE_JV) {
      const unsigned m = P.vmask ? P.vmask[node] : 0u;
#pragma unroll
      for (int c = 0; c < DIM; ++c) sV[i * DIM + c] = ((m >> c) & 1u) ? 0.0 : Pv[b + c];
      if (cqr) continue;  // u and its history come from the cache
    }
#pragma unroll
    for (int c = 0; c < DIM; ++c) sU[i * DIM + c] = P.u[b + c];
    if (P.n_hist > 0) {
#pragma unroll
      for (int c = 0; c < DIM; ++c) sH[i * DIM + c] = P.h1[b + c];
    }
    if (P.n_hist > 1) {
#pragma unroll
      for (int c = 0; c < DIM; ++c) sH[CB * NV * DIM + i * DIM + c] = P.h2[b + c];
    }
    if (P.n_hist > 2) {
#pragma unroll
      for (int c = 0; c < DIM; ++c) sH[2 * CB * NV * DIM + i * DIM + c] = P.h3[b + c];
    }
  }
  for (int i = tid; i < ncb * NP; i += blockDim.x) {
    const int pn = P.cell_pnodes ? P.cell_pnodes[cid(i / NP) * NP + i % NP] : P.cell_vnodes[cid(i / NV) * NV + i % NV];
    if (!cqr) sP[i] = P.u[voff + pn];
    if constexpr (MODE == MODE_JV) sVP[i] = Pv[voff + pn];
  }
  __syncthreads();

  // ---- 2./3. evaluate + pointwise, one thread per (cell, q)
  if (tid < ncb * NQ) {
    const int cl = tid / NQ, q = tid % NQ;
    const int cell = (int)cid(cl);
    const int qx = q % NQ1, qy = (q / NQ1) % NQ1, qz = DIM == 3 ? q / (NQ1 * NQ1) : 0;
    const double hx = P.geo[cell * 4 + 0], hy = P.geo[cell * 4 + 1], hz = DIM == 3 ? P.geo[cell * 4 + 2] : 1.0;
    const double hst = P.geo[cell * 4 + 3];
    const double ih[3] = {1.0 / hx, 1.0 / hy, 1.0 / hz};
    // mapped cells: this q's geometry (J^-1 [a][i], G, c, JxW, x_q)
    const double *gqq = GEN ? P.gq + ((int64_t)cell * NQ + q) * kGeo : nullptr;
    double JI[3][3] = {}, Gm[6] = {}, cg[3] = {};
    if constexpr (GEN) {
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int i = 0; i < 3; ++i) JI[a][i] = gqq[kGeoJI + 3 * a + i];
#pragma unroll
      for (int i = 0; i < 6; ++i) Gm[i] = gqq[kGeoG + i];
#pragma unroll
      for (int i = 0; i < 3; ++i) cg[i] = gqq[kGeoC + i];
    }
    const double JxW = GEN ? gqq[kGeoJxW]
                           : tW[qx] * tW[qy] * (DIM == 3 ? tW[qz] : 1.0) * hx * hy * (DIM == 3 ? hz : 1.0);
    // Laplacian weights relative to x (1 for cubes)
    const double wy = (hx * hx) / (hy * hy), wz = (hx * hx) / (hz * hz);
    // reference gradient -> physical (J^-T), physical test coefficient -> reference (J^-1)
    auto to_phys = [&](double (&g)[DIM]) {
      double o[DIM];
#pragma unroll
      for (int i = 0; i < DIM; ++i) {
        double s = 0.;
#pragma unroll
        for (int a = 0; a < DIM; ++a) s += JI[a][i] * g[a];
        o[i] = s;
      }
#pragma unroll
      for (int i = 0; i < DIM; ++i) g[i] = o[i];
    };
    auto to_ref = [&](double (&t)[DIM]) {
      double o[DIM];
#pragma unroll
      for (int a = 0; a < DIM; ++a) {
        double s = 0.;
#pragma unroll
        for (int i = 0; i < DIM; ++i) s += JI[a][i] * t[i];
        o[a] = s;
      }
#pragma unroll
      for (int a = 0; a < DIM; ++a) t[a] = o[a];
    };

    double u[DIM] = {}, gu[DIM][DIM] = {}, lu[DIM] = {}, pq = 0., gp[DIM] = {};
    double h1[DIM] = {}, h2[DIM] = {}, h3[DIM] = {};
    double v[DIM] = {}, gv[DIM][DIM] = {}, lv[DIM] = {}, vp = 0., gvp[DIM] = {};
    const double *cu = sU + cl * NV * DIM;
    const double *cv = sV + cl * NV * DIM;
    const double *ch = sH + cl * NV * DIM;
    const int nh = P.n_hist;
    auto eval_row = [&](int az, int ay) {
      const double vz = DIM == 3 ? tV[qz][az] : 1.0, dz = DIM == 3 ? tD[qz][az] : 0.0,
                   sz = DIM == 3 ? tS[qz][az] : 0.0;
      {
        const double vy = tV[qy][ay], dy = tD[qy][ay], sy = tS[qy][ay];
#pragma unroll
        for (int ax = 0; ax < C::K1; ++ax) {
          const double vx = tV[qx][ax], dx = tD[qx][ax], sx = tS[qx][ax];
          const int a = ax + C::K1 * (ay + C::K1 * az);
          const double N = vx * vy * vz;
          const double g0 = dx * vy * vz, g1 = vx * dy * vz, g2 = vx * vy * dz;
          // box: x-scaled Laplacian; mapped: sum_ab G_ab d2_ref (the -c . grad part comes after)
          const double L = GEN ? (Gm[0] * sx * vy * vz + Gm[1] * vx * sy * vz + 2 * Gm[3] * dx * dy * vz +
                                  (DIM == 3 ? Gm[2] * vx * vy * sz + 2 * Gm[4] * dx * vy * dz + 2 * Gm[5] * vx * dy * dz
                                            : 0.0))
                               : sx * vy * vz + wy * vx * sy * vz + (DIM == 3 ? wz * vx * vy * sz : 0.0);
          const double gr[3] = {g0, g1, g2};
#pragma unroll
          for (int c = 0; c < DIM; ++c) {
            if (!cqr) {
              const double val = cu[a * DIM + c];
              u[c] += val * N;
              lu[c] += val * L;
#pragma unroll
              for (int e = 0; e < DIM; ++e) gu[c][e] += val * gr[e];
            }
            if constexpr (MODE == MODE_JV) {
              const double vv = cv[a * DIM + c];
              v[c] += vv * N;
              lv[c] += vv * L;
#pragma unroll
              for (int e = 0; e < DIM; ++e) gv[c][e] += vv * gr[e];
            }
            if (!cqr) {
              if (nh > 0) h1[c] += ch[a * DIM + c] * N;
              if (nh > 1) h2[c] += ch[CB * NV * DIM + a * DIM + c] * N;
              if (nh > 2) h3[c] += ch[2 * CB * NV * DIM + a * DIM + c] * N;
            }
          }
        }
      }
    };
    if constexpr (CQ) {  // v only: a plane's rows unroll (their table and node loads in flight together)
#pragma nounroll
      for (int az = 0; az < (DIM == 3 ? C::K1 : 1); ++az)
#pragma unroll
        for (int ay = 0; ay < C::K1; ++ay) eval_row(az, ay);
    } else {
#pragma nounroll
      for (int az = 0; az < (DIM == 3 ? C::K1 : 1); ++az)
#pragma nounroll
        for (int ay = 0; ay < C::K1; ++ay) eval_row(az, ay);
    }
    {
      const double *cp = sP + cl * NP;
      const double *cvp = sVP + cl * NP;
#pragma nounroll
      for (int az = 0; az < (DIM == 3 ? C::KP1 : 1); ++az) {
        const double vz = DIM == 3 ? tVp[qz][az] : 1.0, dz = DIM == 3 ? tDp[qz][az] : 0.0;
#pragma nounroll
        for (int ay = 0; ay < C::KP1; ++ay) {
          const double vy = tVp[qy][ay], dy = tDp[qy][ay];
#pragma unroll
          for (int ax = 0; ax < C::KP1; ++ax) {
            const double vx = tVp[qx][ax], dx = tDp[qx][ax];
            const int a = ax + C::KP1 * (ay + C::KP1 * az);
            const double N = vx * vy * vz;
            const double gr[3] = {dx * vy * vz, vx * dy * vz, vx * vy * dz};
            if (!cqr) {
              const double pv = cp[a];
              if constexpr (MODE == MODE_RESIDUAL) pq += pv * N;
#pragma unroll
              for (int e = 0; e < DIM; ++e) gp[e] += pv * gr[e];
            }
            if constexpr (MODE == MODE_JV) {
              const double w = cvp[a];
              vp += w * N;
#pragma unroll
              for (int e = 0; e < DIM; ++e) gvp[e] += w * gr[e];
            }
          }
        }
      }
    }
    if constexpr (GEN) {  // reference -> physical derivatives (MappingQ)
#pragma unroll
      for (int c = 0; c < DIM; ++c) {
        to_phys(gu[c]);
        to_phys(gv[c]);
#pragma unroll
        for (int k = 0; k < DIM; ++k) { lu[c] -= cg[k] * gu[c][k]; lv[c] -= cg[k] * gv[c][k]; }
      }
      to_phys(gp);
      to_phys(gvp);
    } else {  // reference -> physical derivatives (affine box map)
      const double il2 = ih[0] * ih[0];
#pragma unroll
      for (int c = 0; c < DIM; ++c) {
        lu[c] *= il2;
        lv[c] *= il2;
#pragma unroll
        for (int e = 0; e < DIM; ++e) { gu[c][e] *= ih[e]; gv[c][e] *= ih[e]; }
      }
#pragma unroll
      for (int e = 0; e < DIM; ++e) { gp[e] *= ih[e]; gvp[e] *= ih[e]; }
    }

    const int64_t cqb = ((int64_t)cell * NCQ) * NQ + q;  // cache entry k of this point at cqb + k * NQ
    if (cqr) {
#pragma unroll
      for (int c = 0; c < DIM; ++c) u[c] = P.cq[cqb + (int64_t)c * NQ];
#pragma unroll
      for (int c = 0; c < DIM; ++c)
#pragma unroll
        for (int e = 0; e < DIM; ++e) gu[c][e] = P.cq[cqb + (int64_t)(DIM + DIM * c + e) * NQ];
    }
    // ---- pointwise (gls_navier_stokes.cc:391-516)
    const double nu = P.nu;
    double un2 = 0.;
#pragma unroll
    for (int c = 0; c < DIM; ++c) un2 += u[c] * u[c];
    const double u_mag = fmax(sqrt(un2), 1e-12);
    const double t1 = 2. * u_mag / hst, t2 = 4 * nu / (hst * hst);
    double tau = 1. / sqrt(P.sdt2 + t1 * t1 + 9 * (t2 * t2));
    double f[DIM] = {};
    if (P.force_q) {
#pragma unroll
      for (int c = 0; c < DIM; ++c) f[c] = P.force_q[((int64_t)cell * NQ + q) * DIM + c];
    }
    double Gu[DIM], R[DIM], srf_cor[DIM] = {}, srf_cen[DIM] = {};
#pragma unroll
    for (int c = 0; c < DIM; ++c) {
      double s = 0.;
#pragma unroll
      for (int e = 0; e < DIM; ++e) s += gu[c][e] * u[e];
      Gu[c] = s;
      R[c] = s + gp[c] - nu * lu[c] - f[c];
    }
    double om[3] = {P.omega[0], P.omega[1], P.omega[2]};
    if (P.srf) {
      double xq[3];
      if constexpr (GEN) {
        xq[0] = gqq[kGeoX];
        xq[1] = gqq[kGeoX + 1];
        xq[2] = DIM == 3 ? gqq[kGeoX + 2] : 0.0;
      } else {
        xq[0] = P.x0[cell * 3 + 0] + hx * tXi[qx];
        xq[1] = P.x0[cell * 3 + 1] + hy * tXi[qy];
        xq[2] = DIM == 3 ? P.x0[cell * 3 + 2] + hz * tXi[qz] : 0.0;
      }
      if constexpr (DIM == 2) {
        const double wz_ = om[2];
        srf_cor[0] = 2 * wz_ * (-1.) * u[1];
        srf_cor[1] = 2 * wz_ * (-1.) * (-u[0]);
        const double a0 = wz_ * (-1.) * xq[1], a1 = wz_ * (-1.) * (-xq[0]);
        srf_cen[0] = wz_ * (-1.) * a1;
        srf_cen[1] = wz_ * (-1.) * (-a0);
      } else {
        const double cx[3] = {om[1] * u[2] - om[2] * u[1], om[2] * u[0] - om[0] * u[2], om[0] * u[1] - om[1] * u[0]};
        const double ox[3] = {om[1] * xq[2] - om[2] * xq[1], om[2] * xq[0] - om[0] * xq[2],
                              om[0] * xq[1] - om[1] * xq[0]};
        srf_cor[0] = 2 * cx[0]; srf_cor[1] = 2 * cx[1]; srf_cor[DIM - 1] = 2 * cx[DIM - 1];
        const double cc[3] = {om[1] * ox[2] - om[2] * ox[1], om[2] * ox[0] - om[0] * ox[2], om[0] * ox[1] - om[1] * ox[0]};
#pragma unroll
        for (int c = 0; c < DIM; ++c) srf_cen[c] = cc[c];
      }
#pragma unroll
      for (int c = 0; c < DIM; ++c) R[c] += srf_cor[c] + srf_cen[c];
    }
    double Tt[DIM];  // time term sum_k alpha_k u^(k)
#pragma unroll
    for (int c = 0; c < DIM; ++c) {
      double s = P.alpha[0] * u[c];
      if (nh > 0) s += P.alpha[1] * h1[c];
      if (nh > 1) s += P.alpha[2] * h2[c];
      if (nh > 2) s += P.alpha[3] * h3[c];
      Tt[c] = s;
      R[c] += s;
    }
    if (cqr) {  // tau and R_s as the diagonal pass computed them (the state's gathers were skipped)
      tau = P.cq[cqb + (int64_t)(DIM + DIM * DIM) * NQ];
#pragma unroll
      for (int c = 0; c < DIM; ++c) R[c] = P.cq[cqb + (int64_t)(DIM + DIM * DIM + 1 + c) * NQ];
    }
    if (cqw) {
#pragma unroll
      for (int c = 0; c < DIM; ++c) P.cq[cqb + (int64_t)c * NQ] = u[c];
#pragma unroll
      for (int c = 0; c < DIM; ++c)
#pragma unroll
        for (int e = 0; e < DIM; ++e) P.cq[cqb + (int64_t)(DIM + DIM * c + e) * NQ] = gu[c][e];
      P.cq[cqb + (int64_t)(DIM + DIM * DIM) * NQ] = tau;
#pragma unroll
      for (int c = 0; c < DIM; ++c) P.cq[cqb + (int64_t)(DIM + DIM * DIM + 1 + c) * NQ] = R[c];
    }

    double *Tq = sT + (cl * NQ + q) * NT;
    if constexpr (MODE == MODE_RESIDUAL) {
      double divu = 0.;
#pragma unroll
      for (int c = 0; c < DIM; ++c) divu += gu[c][c];
#pragma unroll
      for (int c = 0; c < DIM; ++c) {
        Tq[c * (DIM + 1)] = JxW * (-Gu[c] + f[c] - Tt[c] - srf_cor[c] - srf_cen[c]);
        double t[DIM];
#pragma unroll
        for (int e = 0; e < DIM; ++e) t[e] = JxW * (-nu * gu[c][e] + (c == e ? pq : 0.0) - tau * R[c] * u[e]);
        if constexpr (GEN) to_ref(t);
#pragma unroll
        for (int e = 0; e < DIM; ++e) Tq[c * (DIM + 1) + 1 + e] = GEN ? t[e] : t[e] * ih[e];
      }
      Tq[DIM * (DIM + 1)] = -JxW * divu;
      {
        double t[DIM];
#pragma unroll
        for (int e = 0; e < DIM; ++e) t[e] = -JxW * tau * R[e];
        if constexpr (GEN) to_ref(t);
#pragma unroll
        for (int e = 0; e < DIM; ++e) Tq[DIM * (DIM + 1) + 1 + e] = GEN ? t[e] : t[e] * ih[e];
      }
    } else if constexpr (MODE == MODE_JV) {
      const double aj = P.alpha_jac;
      double S[DIM], A[DIM], divv = 0.;
#pragma unroll
      for (int c = 0; c < DIM; ++c) {
        double gvu = 0., guv = 0.;
#pragma unroll
        for (int e = 0; e < DIM; ++e) { guv += gu[c][e] * v[e]; gvu += gv[c][e] * u[e]; }
        A[c] = guv + gvu + aj * v[c];
        S[c] = guv + gvu + gvp[c] - nu * lv[c] + aj * v[c];
        divv += gv[c][c];
      }
      if (P.srf) {
        double cj[DIM];
        if constexpr (DIM == 2) {
          cj[0] = 2 * om[2] * (-1.) * v[1];
          cj[1] = 2 * om[2] * (-1.) * (-v[0]);
        } else {
          cj[0] = 2 * (om[1] * v[2] - om[2] * v[1]);
          cj[1] = 2 * (om[2] * v[0] - om[0] * v[2]);
          cj[DIM - 1] = 2 * (om[0] * v[1] - om[1] * v[0]);
        }
#pragma unroll
        for (int c = 0; c < DIM; ++c) { A[c] += cj[c]; S[c] += cj[c]; }
      }
#pragma unroll
      for (int c = 0; c < DIM; ++c) {
        Tq[c * (DIM + 1)] = JxW * A[c];
        double t[DIM];
#pragma unroll
        for (int e = 0; e < DIM; ++e) t[e] = JxW * (nu * gv[c][e] - (c == e ? vp : 0.0) + tau * S[c] * u[e] + tau * R[c] * v[e]);
        if constexpr (GEN) to_ref(t);
#pragma unroll
        for (int e = 0; e < DIM; ++e) Tq[c * (DIM + 1) + 1 + e] = GEN ? t[e] : t[e] * ih[e];
      }
      Tq[DIM * (DIM + 1)] = JxW * divv;
      {
        double t[DIM];
#pragma unroll
        for (int e = 0; e < DIM; ++e) t[e] = JxW * tau * S[e];
        if constexpr (GEN) to_ref(t);
#pragma unroll
        for (int e = 0; e < DIM; ++e) Tq[DIM * (DIM + 1) + 1 + e] = GEN ? t[e] : t[e] * ih[e];
      }
    } else {  // MODE_DIAG: per-q state for the diagonal
      Tq[0] = JxW;
      Tq[1] = tau;
#pragma unroll
      for (int c = 0; c < DIM; ++c) {
        Tq[2 + c] = u[c];
        Tq[2 + DIM + c] = gu[c][c];
        Tq[2 + 2 * DIM + c] = R[c];
      }
    }
  }
  __syncthreads();

  // ---- 4./5. integrate + scatter, one thread per (cell, node)
  for (int i = tid; i < ncb * NV; i += blockDim.x) {
    const int cl = i / NV, a = i % NV;
    const int ax = a % C::K1, ay = (a / C::K1) % C::K1, az = DIM == 3 ? a / (C::K1 * C::K1) : 0;
    const double *Tc = sT + cl * NQ * NT;
    const int node = P.cell_vnodes[cid(i / NV) * NV + i % NV];
    if constexpr (MODE != MODE_DIAG) {
      double out[DIM] = {};
      // unrolled by 3: three points' table and coefficient loads in flight (same VGPRs and occupancy; the small
      // latency-bound leaf launches of forests 2.5 % faster per Newton step, profiles/r05_ab_cell_unroll.txt)
#pragma unroll 3
      for (int q = 0; q < NQ; ++q) {
        const int qx = q % NQ1, qy = (q / NQ1) % NQ1, qz = DIM == 3 ? q / (NQ1 * NQ1) : 0;
        const double vx = tV[qx][ax], vy = tV[qy][ay], vz = DIM == 3 ? tV[qz][az] : 1.0;
        const double N = vx * vy * vz;
        const double gr[3] = {tD[qx][ax] * vy * vz, vx * tD[qy][ay] * vz, DIM == 3 ? vx * vy * tD[qz][az] : 0.0};
        const double *Tq = Tc + q * NT;
#pragma unroll
        for (int c = 0; c < DIM; ++c) {
          double s = N * Tq[c * (DIM + 1)];
#pragma unroll
          for (int e = 0; e < DIM; ++e) s += gr[e] * Tq[c * (DIM + 1) + 1 + e];
          out[c] += s;
        }
      }
      if (Pev) {
        double *e = Pev + cid(cl) * (NV * DIM + NP) + a * DIM;
#pragma unroll
        for (int c = 0; c < DIM; ++c) e[c] = out[c];
      } else {
#pragma unroll
        for (int c = 0; c < DIM; ++c) atomicAdd(&P.y[(int64_t)node * DIM + c], out[c]);
      }
    } else {
      const int cell = (int)cid(cl);
      const double hx = P.geo[cell * 4 + 0], hy = P.geo[cell * 4 + 1], hz = DIM == 3 ? P.geo[cell * 4 + 2] : 1.0;
      const double ih[3] = {1.0 / hx, 1.0 / hy, 1.0 / hz};
      const double nu = P.nu, aj = P.alpha_jac;
      double out[DIM] = {};
#pragma nounroll
      for (int q = 0; q < NQ; ++q) {
        const int qx = q % NQ1, qy = (q / NQ1) % NQ1, qz = DIM == 3 ? q / (NQ1 * NQ1) : 0;
        const double vx = tV[qx][ax], vy = tV[qy][ay], vz = DIM == 3 ? tV[qz][az] : 1.0;
        const double N = vx * vy * vz;
        double g[3] = {tD[qx][ax] * vy * vz * ih[0], vx * tD[qy][ay] * vz * ih[1],
                       DIM == 3 ? vx * vy * tD[qz][az] * ih[2] : 0.0};
        double L = tS[qx][ax] * vy * vz * ih[0] * ih[0] + vx * tS[qy][ay] * vz * ih[1] * ih[1] +
                   (DIM == 3 ? vx * vy * tS[qz][az] * ih[2] * ih[2] : 0.0);
        if constexpr (GEN) {  // physical gradient / Laplacian of the test function on the mapped cell
          const double *gg = P.gq + ((int64_t)cell * NQ + q) * kGeo;
          const double dxv = tD[qx][ax], dyv = tD[qy][ay], dzv = DIM == 3 ? tD[qz][az] : 0.0;
          const double gr[3] = {dxv * vy * vz, vx * dyv * vz, vx * vy * dzv};
          const double sx = tS[qx][ax], sy = tS[qy][ay], sz = DIM == 3 ? tS[qz][az] : 0.0;
          L = gg[kGeoG] * sx * vy * vz + gg[kGeoG + 1] * vx * sy * vz + 2 * gg[kGeoG + 3] * dxv * dyv * vz +
              (DIM == 3 ? gg[kGeoG + 2] * vx * vy * sz + 2 * gg[kGeoG + 4] * dxv * vy * dzv + 2 * gg[kGeoG + 5] * vx * dyv * dzv
                        : 0.0);
#pragma unroll
          for (int i = 0; i < DIM; ++i) {
            double s = 0.;
#pragma unroll
            for (int a = 0; a < DIM; ++a) s += gg[kGeoJI + 3 * a + i] * gr[a];
            g[i] = s;
          }
#pragma unroll
          for (int i = 0; i < DIM; ++i) L -= gg[kGeoC + i] * g[i];
        }
        const double *Tq = Tc + q * NT;
        const double JxW = Tq[0], tau = Tq[1];
        double ug = 0., gg = 0.;
#pragma unroll
        for (int e = 0; e < DIM; ++e) { ug += Tq[2 + e] * g[e]; gg += g[e] * g[e]; }
#pragma unroll
        for (int c = 0; c < DIM; ++c) {
          const double Gcc = Tq[2 + DIM + c], Rc = Tq[2 + 2 * DIM + c];
          const double Sc = Gcc * N + ug - nu * L + aj * N;
          out[c] += JxW * (nu * gg + Gcc * N * N + ug * N + aj * N * N + tau * Sc * ug + tau * Rc * g[c] * N);
        }
      }
      // constrained rows (Dirichlet or hanging) get deal.II's |K_e(i,i)| per cell
      const unsigned m = (P.vmask ? P.vmask[node] : 0u) | (P.hmask ? P.hmask[node] : 0u);
      if (Pev) {
        double *e = Pev + cid(cl) * (NV * DIM + NP) + a * DIM;
#pragma unroll
        for (int c = 0; c < DIM; ++c) e[c] = ((m >> c) & 1u) ? fabs(out[c]) : out[c];
      } else {
#pragma unroll
        for (int c = 0; c < DIM; ++c) atomicAdd(&P.y[(int64_t)node * DIM + c], ((m >> c) & 1u) ? fabs(out[c]) : out[c]);
      }
    }
  }
  for (int i = tid; i < ncb * NP; i += blockDim.x) {
    const int cl = i / NP, a = i % NP;
    const int ax = a % C::KP1, ay = (a / C::KP1) % C::KP1, az = DIM == 3 ? a / (C::KP1 * C::KP1) : 0;
    const double *Tc = sT + cl * NQ * NT;
    const int pn = P.cell_pnodes ? P.cell_pnodes[cid(i / NP) * NP + i % NP] : P.cell_vnodes[cid(i / NV) * NV + i % NV];
    double out = 0.;
    if constexpr (MODE != MODE_DIAG) {
#pragma unroll 3
      for (int q = 0; q < NQ; ++q) {
        const int qx = q % NQ1, qy = (q / NQ1) % NQ1, qz = DIM == 3 ? q / (NQ1 * NQ1) : 0;
        const double vx = tVp[qx][ax], vy = tVp[qy][ay], vz = DIM == 3 ? tVp[qz][az] : 1.0;
        const double *Tq = Tc + q * NT + DIM * (DIM + 1);
        double s = vx * vy * vz * Tq[0];
        s += tDp[qx][ax] * vy * vz * Tq[1];
        s += vx * tDp[qy][ay] * vz * Tq[2];
        if (DIM == 3) s += vx * vy * tDp[qz][az] * Tq[DIM];
        out += s;
      }
    } else {
      const int cell = (int)cid(cl);
      const double hx = P.geo[cell * 4 + 0], hy = P.geo[cell * 4 + 1], hz = DIM == 3 ? P.geo[cell * 4 + 2] : 1.0;
#pragma nounroll
      for (int q = 0; q < NQ; ++q) {
        const int qx = q % NQ1, qy = (q / NQ1) % NQ1, qz = DIM == 3 ? q / (NQ1 * NQ1) : 0;
        const double vx = tVp[qx][ax], vy = tVp[qy][ay], vz = DIM == 3 ? tVp[qz][az] : 1.0;
        double g0 = tDp[qx][ax] * vy * vz / hx, g1 = vx * tDp[qy][ay] * vz / hy,
               g2 = DIM == 3 ? vx * vy * tDp[qz][az] / hz : 0.0;
        if constexpr (GEN) {
          const double *gg = P.gq + ((int64_t)cell * NQ + q) * kGeo;
          const double gr[3] = {tDp[qx][ax] * vy * vz, vx * tDp[qy][ay] * vz, DIM == 3 ? vx * vy * tDp[qz][az] : 0.0};
          double ph[3] = {0., 0., 0.};
#pragma unroll
          for (int i = 0; i < DIM; ++i)
#pragma unroll
            for (int a = 0; a < DIM; ++a) ph[i] += gg[kGeoJI + 3 * a + i] * gr[a];
          g0 = ph[0];
          g1 = ph[1];
          g2 = ph[2];
        }
        const double *Tq = Tc + q * NT;
        out += Tq[0] * Tq[1] * (g0 * g0 + g1 * g1 + g2 * g2);
      }
    }
    if (Pev) Pev[cid(cl) * (NV * DIM + NP) + NV * DIM + a] = out;
    else atomicAdd(&P.y[voff + pn], out);
  }
}

template <int DIM, int K, int KP, int NQ1, int TPB = 256>
size_t cell_kernel_lds_bytes() {
  using C = Cfg<DIM, K, KP, NQ1, TPB>;
  size_t n = ((C::TABN + 1) & ~1) + C::CB * C::NV * DIM + C::CB * C::NP + 3 * C::CB * C::NV * DIM +
             C::CB * C::NV * DIM + C::CB * C::NP + C::CB * C::NQ * C::NT;
  return n * sizeof(double);
}

template <int DIM, int K, int KP, int NQ1, bool GEN>
hipError_t launch_cell_g(int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  using C = Cfg<DIM, K, KP, NQ1>;
  const int blocks = ((P.cell_list ? P.cell_list_n : P.n_cells) + C::CB - 1) / C::CB;
  const size_t lds = cell_kernel_lds_bytes<DIM, K, KP, NQ1>();
  static bool attr_set = false;  // allow > 64 KiB dynamic LDS (gfx950 has 160 KiB per CU)
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void *)gls_cell_kernel<DIM, K, KP, NQ1, MODE_RESIDUAL, GEN>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void *)gls_cell_kernel<DIM, K, KP, NQ1, MODE_JV, GEN>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void *)gls_cell_kernel<DIM, K, KP, NQ1, MODE_JV, GEN, 256, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void *)gls_cell_kernel<DIM, K, KP, NQ1, MODE_DIAG, GEN>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  switch (mode) {
    case MODE_RESIDUAL:
      hipLaunchKernelGGL((gls_cell_kernel<DIM, K, KP, NQ1, MODE_RESIDUAL, GEN>), dim3(blocks), dim3(256), lds, s, P, T);
      break;
    case MODE_JV:
      if (P.bv_stride) {  // batched probes: small workgroups, so that more (probe, cell batch) pairs skip
        using C64 = Cfg<DIM, K, KP, NQ1, 64>;
        if constexpr (C64::CB >= 1) {
          const dim3 grid = P.work ? dim3((unsigned)P.n_work) : dim3((P.n_cells + C64::CB - 1) / C64::CB, P.n_probe);
          if (P.work && P.cq && P.cq_mode == 2)  // listed blocks from the linearization cache
            hipLaunchKernelGGL((gls_cell_kernel<DIM, K, KP, NQ1, MODE_JV, GEN, 64, true>), grid, dim3(64),
                               (cell_kernel_lds_bytes<DIM, K, KP, NQ1, 64>()), s, P, T);
          else
            hipLaunchKernelGGL((gls_cell_kernel<DIM, K, KP, NQ1, MODE_JV, GEN, 64>), grid, dim3(64),
                               (cell_kernel_lds_bytes<DIM, K, KP, NQ1, 64>()), s, P, T);
          break;
        }
        if (P.work) return hipErrorNotSupported;  // work lists pair with the 64-lane batches only
      }
      if (P.cq && P.cq_mode == 2 && !P.bv_stride)  // from the linearization cache
        hipLaunchKernelGGL((gls_cell_kernel<DIM, K, KP, NQ1, MODE_JV, GEN, 256, true>), dim3(blocks), dim3(256), lds, s,
                           P, T);
      else
        hipLaunchKernelGGL((gls_cell_kernel<DIM, K, KP, NQ1, MODE_JV, GEN>), dim3(blocks, P.bv_stride ? P.n_probe : 1),
                           dim3(256), lds, s, P, T);
      break;
    default:
      hipLaunchKernelGGL((gls_cell_kernel<DIM, K, KP, NQ1, MODE_DIAG, GEN>), dim3(blocks), dim3(256), lds, s, P, T);
  }
  return hipGetLastError();
}
template <int DIM, int K, int KP, int NQ1>
hipError_t launch_cell_t(int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (P.n_cells <= 0 || (P.cell_list && P.cell_list_n <= 0)) return hipSuccess;
  if (P.cell_list && P.bv_stride) return hipErrorNotSupported;  // probes run over all cells
  if (P.gq) return launch_cell_g<DIM, K, KP, NQ1, true>(mode, P, T, s);
  return launch_cell_g<DIM, K, KP, NQ1, false>(mode, P, T, s);
}

// Supported element families (dim, k, kp) with the reference quadrature QGauss(k+1).
hipError_t launch_cell_kernel(int dim, int k, int kp, int nq1d, int mode, const OpParams &P, const Tables1D &T,
                              hipStream_t s) {
  if (mode == MODE_JV && !(P.cell_list && P.cell_list_n <= 0)) {  // sum-factorized J.v where it applies
    const hipError_t e = launch_cell_sf_jv(dim, k, kp, nq1d, P, T, s);
    if (e != hipErrorNotSupported) return e;
  }
#define GLS_CASE(D, KK, KKP)                                                         \
  if (dim == D && k == KK && kp == KKP && nq1d == KK + 1) return launch_cell_t<D, KK, KKP, KK + 1>(mode, P, T, s);
  GLS_CASE(2, 1, 1)
  GLS_CASE(2, 2, 1)
  GLS_CASE(2, 2, 2)
  GLS_CASE(2, 3, 3)
  GLS_CASE(3, 1, 1)
  GLS_CASE(3, 2, 1)
  GLS_CASE(3, 2, 2)
#undef GLS_CASE
  return hipErrorNotSupported;
}

int cell_kernel_cells_per_block(int dim, int k, int nq1d, bool probe) {
  (void)k;
  int nq = 1;
  for (int d = 0; d < dim; ++d) nq *= nq1d;
  return probe && nq <= 64 ? 64 / nq : 256 / nq;  // Cfg<>::CB of the launch launch_cell_g picks
}

bool cell_kernel_supported(int dim, int k, int kp, int nq1d) {
  if (nq1d != k + 1) return false;
  return (dim == 2 && ((k == 1 && kp == 1) || (k == 2 && (kp == 1 || kp == 2)) || (k == 3 && kp == 3))) ||
         (dim == 3 && ((k == 1 && kp == 1) || (k == 2 && (kp == 1 || kp == 2))));
}

}  // namespace gls
