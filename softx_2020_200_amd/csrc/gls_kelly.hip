// gls_kelly.hip — Kelly error indicator on Qk meshes: conforming axis-aligned boxes,
// octree meshes with hanging faces, and mapped (MappingQ) unstructured meshes with hanging faces.
//
// Restates KellyErrorEstimator<dim>::estimate as refine_mesh_kelly calls it
// (navier_stokes_base.cc:612-652: QGauss<dim-1>(n_q + 1) on the faces, no Neumann boundaries, the
// velocity or the pressure component mask, deal.II's default cell_diameter_over_24 strategy):
//   eta_K^2 = sum over the interior faces F of K of  diam(K)/24 * int_F sum_c [d u_c / dn]^2.
// One thread per cell; each face integral is evaluated from both sides' nodal values (the
// neighbour's face quadrature points coincide on a conforming box mesh), so no atomics are needed.
#include "gls_launch.hpp"

namespace gls {

namespace {

template <int DIM, int M>
__global__ void __launch_bounds__(256) k_kelly(const int32_t *__restrict__ cell_nodes, const int32_t *__restrict__ nbr,
                                               const double *__restrict__ geo, const double *__restrict__ sol,
                                               int n_cells, int ncomp, int64_t base, int stride, KellyTables T,
                                               double *__restrict__ eta) {
  constexpr int M1 = M + 1;
  constexpr int NN = DIM == 3 ? M1 * M1 * M1 : M1 * M1;
  const int cell = blockIdx.x * blockDim.x + threadIdx.x;
  if (cell >= n_cells) return;
  const int nqf = T.nq;
  double h[3] = {geo[cell * 4 + 0], geo[cell * 4 + 1], DIM == 3 ? geo[cell * 4 + 2] : 1.0};
  const double diam = sqrt(h[0] * h[0] + h[1] * h[1] + (DIM == 3 ? h[2] * h[2] : 0.0));
  double acc = 0.0;
  for (int d = 0; d < DIM; ++d) {
    for (int s = 0; s < 2; ++s) {
      const int nb = nbr[(int64_t)cell * 2 * DIM + 2 * d + s];
      if (nb < 0) continue;  // boundary face: no jump (no Neumann map)
      const double hn[3] = {geo[nb * 4 + 0], geo[nb * 4 + 1], DIM == 3 ? geo[nb * 4 + 2] : 1.0};
      // tangential directions
      int t0 = -1, t1 = -1;
      for (int e = 0; e < DIM; ++e)
        if (e != d) {
          if (t0 < 0) t0 = e;
          else t1 = e;
        }
      const double area = h[t0] * (DIM == 3 ? h[t1] : 1.0);
      const int nq1 = DIM == 3 ? nqf : 1;
      double integral = 0.0;
      for (int qa = 0; qa < nqf; ++qa)
        for (int qb = 0; qb < nq1; ++qb) {
          const double w = T.w[qa] * (DIM == 3 ? T.w[qb] : 1.0) * area;
          double jump2 = 0.0;
          for (int c = 0; c < ncomp; ++c) {
            double g[2] = {0.0, 0.0};
            for (int side = 0; side < 2; ++side) {  // 0: this cell (face at xi_d = s), 1: neighbour (1 - s)
              const int cc = side ? nb : cell;
              const int end = side ? 1 - s : s;
              const double inv = 1.0 / (side ? hn[d] : h[d]);
              double sum = 0.0;
              for (int a = 0; a < NN; ++a) {
                int ai[3] = {a % M1, (a / M1) % M1, DIM == 3 ? a / (M1 * M1) : 0};
                double phi = T.De[end][ai[d]] * inv;
                phi *= T.V[qa][ai[t0]];
                if (DIM == 3) phi *= T.V[qb][ai[t1]];
                const int node = cell_nodes[(int64_t)cc * NN + a];
                sum += phi * sol[base + (int64_t)node * stride + c];
              }
              g[side] = sum;
            }
            const double j = g[0] - g[1];
            jump2 += j * j;
          }
          integral += w * jump2;
        }
      acc += diam / 24.0 * integral;
    }
  }
  eta[cell] = sqrt(acc);
}

// Lagrange basis a of degree M on the support points xn, and its derivative, at x
template <int M>
__device__ __forceinline__ void lagr(const double *xn, int a, double x, double &v, double &dv) {
  v = 1.0;
  dv = 0.0;
  for (int b = 0; b <= M; ++b) {
    if (b == a) continue;
    const double inv = 1.0 / (xn[a] - xn[b]);
    dv = dv * (x - xn[b]) * inv + v * inv;
    v *= (x - xn[b]) * inv;
  }
}

// one thread per face piece (non-conforming meshes): the jump of the normal derivative between
// cell a (face xi_d = 1) and cell b (face xi_d = 0) integrated over the piece
template <int DIM, int M>
__global__ void __launch_bounds__(256) k_kelly_faces(const int32_t *__restrict__ cell_nodes, const double *__restrict__ geo,
                                                     const double *__restrict__ sol, int64_t n_faces,
                                                     const int32_t *__restrict__ fa, const int32_t *__restrict__ fb,
                                                     const int32_t *__restrict__ fdir, const double *__restrict__ ra,
                                                     const double *__restrict__ rb, int ncomp, int64_t base, int stride,
                                                     KellyTables T, double *__restrict__ fint) {
  constexpr int M1 = M + 1;
  constexpr int NN = DIM == 3 ? M1 * M1 * M1 : M1 * M1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_faces) return;
  const int d = fdir[e];
  int t[2] = {-1, -1}, nt = 0;
  for (int k = 0; k < DIM; ++k)
    if (k != d) t[nt++] = k;
  const int cells[2] = {fa[e], fb[e]};
  const double *rect[2] = {ra + e * 4, rb + e * 4};
  const double ha[3] = {geo[cells[0] * 4 + 0], geo[cells[0] * 4 + 1], DIM == 3 ? geo[cells[0] * 4 + 2] : 1.0};
  double area = 1.0;
  for (int j = 0; j < DIM - 1; ++j) area *= (rect[0][2 * j + 1] - rect[0][2 * j]) * ha[t[j]];
  const int nq1 = DIM == 3 ? T.nq : 1;
  double integral = 0.0;
  for (int qa = 0; qa < T.nq; ++qa)
    for (int qb = 0; qb < nq1; ++qb) {
      const double w = T.w[qa] * (DIM == 3 ? T.w[qb] : 1.0) * area;
      double g[2][3] = {{0, 0, 0}, {0, 0, 0}};
      for (int side = 0; side < 2; ++side) {
        const int c = cells[side];
        const double hd = geo[c * 4 + d];
        double xi[3];
        xi[d] = side == 0 ? 1.0 : 0.0;
        xi[t[0]] = rect[side][0] + (rect[side][1] - rect[side][0]) * T.xq[qa];
        if (DIM == 3) xi[t[1]] = rect[side][2] + (rect[side][3] - rect[side][2]) * T.xq[qb];
        for (int a = 0; a < NN; ++a) {
          const int ai[3] = {a % M1, (a / M1) % M1, DIM == 3 ? a / (M1 * M1) : 0};
          double v, dv, phi = 1.0;
          lagr<M>(T.xn, ai[d], xi[d], v, dv);
          phi = dv / hd;
          lagr<M>(T.xn, ai[t[0]], xi[t[0]], v, dv);
          phi *= v;
          if (DIM == 3) {
            lagr<M>(T.xn, ai[t[1]], xi[t[1]], v, dv);
            phi *= v;
          }
          const int64_t node = cell_nodes[(int64_t)c * NN + a];
          for (int cc = 0; cc < ncomp; ++cc) g[side][cc] += phi * sol[base + node * stride + cc];
        }
      }
      double j2 = 0.0;
      for (int cc = 0; cc < ncomp; ++cc) j2 += (g[0][cc] - g[1][cc]) * (g[0][cc] - g[1][cc]);
      integral += w * j2;
    }
  fint[e] = integral;
}

// one thread per face piece of a mapped (MappingQ) mesh: the host lists, per face quadrature point,
// both sides' reference coordinates xi, the vectors g = J^-1 n (n: the unit normal of the piece)
// and JxW, so that n . grad u = g . grad_xi u on each side; fint[e] = sum_q JxW sum_c jump_c^2
template <int DIM, int M>
__global__ void __launch_bounds__(256) k_kelly_mapped(const int32_t *__restrict__ cell_nodes, const double *__restrict__ sol,
                                                      int64_t n_pieces, int nqf, const int32_t *__restrict__ ca,
                                                      const int32_t *__restrict__ cb, const double *__restrict__ xi,
                                                      const double *__restrict__ gv, const double *__restrict__ jxw,
                                                      int ncomp, int64_t base, int stride, KellyTables T,
                                                      double *__restrict__ fint) {
  constexpr int M1 = M + 1;
  constexpr int NN = DIM == 3 ? M1 * M1 * M1 : M1 * M1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_pieces) return;
  const int cells[2] = {ca[e], cb[e]};
  double integral = 0.0;
  for (int q = 0; q < nqf; ++q) {
    double dn[2][3] = {{0, 0, 0}, {0, 0, 0}};
    for (int side = 0; side < 2; ++side) {
      const double *x = xi + ((e * nqf + q) * 2 + side) * DIM;
      const double *g = gv + ((e * nqf + q) * 2 + side) * DIM;
      double v[3][M1], dv[3][M1];
      for (int d = 0; d < DIM; ++d)
        for (int a = 0; a <= M; ++a) lagr<M>(T.xn, a, x[d], v[d][a], dv[d][a]);
      for (int a = 0; a < NN; ++a) {
        const int ai[3] = {a % M1, (a / M1) % M1, DIM == 3 ? a / (M1 * M1) : 0};
        double phi_n = 0.0;  // g . grad_xi phi_a
        for (int d = 0; d < DIM; ++d) {
          double t = g[d] * dv[d][ai[d]];
          for (int o = 0; o < DIM; ++o)
            if (o != d) t *= v[o][ai[o]];
          phi_n += t;
        }
        const int64_t node = cell_nodes[(int64_t)cells[side] * NN + a];
        for (int c = 0; c < ncomp; ++c) dn[side][c] += phi_n * sol[base + node * stride + c];
      }
    }
    double j2 = 0.0;
    for (int c = 0; c < ncomp; ++c) j2 += (dn[0][c] - dn[1][c]) * (dn[0][c] - dn[1][c]);
    integral += jxw[e * nqf + q] * j2;
  }
  fint[e] = integral;
}

}  // namespace

hipError_t launch_kelly_faces(int dim, int m, const int32_t *cell_nodes, const double *geo, const double *sol,
                              int64_t n_faces, const int32_t *fa, const int32_t *fb, const int32_t *fdir,
                              const double *rect_a, const double *rect_b, int ncomp, int64_t base, int stride,
                              const KellyTables &T, double *fint, hipStream_t s) {
  if (n_faces <= 0) return hipSuccess;
  const dim3 g((unsigned)((n_faces + 255) / 256)), b(256);
#define GLS_KELLYF_CASE(D, MM)                                                                                        \
  if (dim == D && m == MM) {                                                                                          \
    hipLaunchKernelGGL((k_kelly_faces<D, MM>), g, b, 0, s, cell_nodes, geo, sol, n_faces, fa, fb, fdir, rect_a, rect_b, \
                       ncomp, base, stride, T, fint);                                                                \
    return hipGetLastError();                                                                                         \
  }
  GLS_KELLYF_CASE(2, 1)
  GLS_KELLYF_CASE(2, 2)
  GLS_KELLYF_CASE(3, 1)
  GLS_KELLYF_CASE(3, 2)
#undef GLS_KELLYF_CASE
  return hipErrorNotSupported;
}

hipError_t launch_kelly_mapped(int dim, int m, const int32_t *cell_nodes, const double *sol, int64_t n_pieces, int nqf,
                               const int32_t *ca, const int32_t *cb, const double *xi, const double *g,
                               const double *jxw, int ncomp, int64_t base, int stride, const KellyTables &T,
                               double *fint, hipStream_t s) {
  if (n_pieces <= 0) return hipSuccess;
  const dim3 gr((unsigned)((n_pieces + 255) / 256)), b(256);
#define GLS_KELLYM_CASE(D, MM)                                                                                     if (dim == D && m == MM) {                                                                                         hipLaunchKernelGGL((k_kelly_mapped<D, MM>), gr, b, 0, s, cell_nodes, sol, n_pieces, nqf, ca, cb, xi, g, jxw,                        ncomp, base, stride, T, fint);                                                               return hipGetLastError();                                                                                      }
  GLS_KELLYM_CASE(2, 1)
  GLS_KELLYM_CASE(2, 2)
  GLS_KELLYM_CASE(3, 1)
  GLS_KELLYM_CASE(3, 2)
#undef GLS_KELLYM_CASE
  return hipErrorNotSupported;
}

hipError_t launch_kelly(int dim, int m, const int32_t *cell_nodes, const int32_t *nbr, const double *geo,
                        const double *sol, int n_cells, int ncomp, int64_t base, int stride, const KellyTables &T,
                        double *eta, hipStream_t s) {
  if (n_cells <= 0) return hipSuccess;
  const dim3 g((unsigned)((n_cells + 255) / 256)), b(256);
#define GLS_KELLY_CASE(D, MM)                                                                                 \
  if (dim == D && m == MM) {                                                                                \
    hipLaunchKernelGGL((k_kelly<D, MM>), g, b, 0, s, cell_nodes, nbr, geo, sol, n_cells, ncomp, base, stride, \
                       T, eta);                                                                             \
    return hipGetLastError();                                                                               \
  }
  GLS_KELLY_CASE(2, 1)
  GLS_KELLY_CASE(2, 2)
  GLS_KELLY_CASE(2, 3)
  GLS_KELLY_CASE(3, 1)
  GLS_KELLY_CASE(3, 2)
#undef GLS_KELLY_CASE
  return hipErrorNotSupported;
}

}  // namespace gls
