// gls_brick_kernels.hip — sum-factorized GLS operators on 2x2x2 cell bricks (3D, Qk-Qk).
//
// Why this shape (MI355X-first): on gfx950 FP64 MFMA (v_mfma_f64_16x16x4) and FP64 VALU share
// one ~62 TF budget (profiles/r01_microbench_fp64.txt: 61.3 / 63.5 / 59.1 TF mixed), so the lever
// is FLOPs, not the pipe. Tensor-product sum factorization does the basis x coefficient work
// in ~24 kFLOP per Q2 cell (dense n_dofs x n_q contraction: ~86 kFLOP). The 1D matrices are
// uniform across the wave and indexed with compile-time constants, so they live in SGPRs.
//
// Work unit: one Morton brick = 8 consecutive cells forming a 2x2x2 block (the hyper_cube
// builder emits cells in p4est z-order). Per brick the unique (2k+1)^3 nodes are gathered once
// into LDS (u, p, history combination H = sum_k alpha_k u^(k), and v / v_p for J.v),
// the cells' contributions are summed in LDS in a fixed order (deterministic), brick-interior
// nodes are written with plain stores and brick-boundary nodes with FP64 atomics.
//
// Per-cell pipeline (all LDS line sweeps, one task = one 1D line of one array):
//   state  : x/y/z sweeps of u (value, grad, Laplacian), grad p (+p), H (value)   -> pointwise
//   v      : x/y/z sweeps of v (value, grad, Laplacian), v_p (value, grad)        -> pointwise (J.v)
//   test   : transposed z/y/x sweeps of the 4 x (value, grad) test coefficients  -> node sums
// The pointwise algebra restates gls_navier_stokes.cc:387-748.
#include "gls_common.hpp"
#include "gls_launch.hpp"

namespace gls {

template <int K>
struct BrickCfg {
  static constexpr int K1 = K + 1;           // nodes per direction per cell == QGauss points (k+1)
  static constexpr int N3 = K1 * K1 * K1;    // per-cell array length
  static constexpr int L2 = K1 * K1;         // lines per array
  static constexpr int BN = 2 * K + 1;       // brick nodes per direction
  static constexpr int BN3 = BN * BN * BN;
  static constexpr int NB = K == 1 ? 2 : 1;  // bricks per workgroup
  static constexpr int NC = 8 * NB;          // cells per workgroup
  static constexpr int THREADS = NC * N3;
  static constexpr int R1N = 18, R2N = 22;   // per-cell LDS array slots
};

// offset of element e of line l in a [K1][K1][K1] array ([z][y][x], x fastest), sweep dim D
template <int D, int K1>
__device__ __forceinline__ int loff(int l, int e) {
  if constexpr (D == 0) return e + K1 * l;
  else if constexpr (D == 1) return (l % K1) + K1 * e + K1 * K1 * (l / K1);
  else return l + K1 * K1 * e;
}

// forward 1D contraction: out[j] = sum_i M[j][i] in[i]   (nodes -> quadrature)
template <int K1>
__device__ __forceinline__ void fwd(const double (&M)[kMaxQ1D][kMaxNodes1D], const double *in, double *out,
                                    double scale = 1.0) {
#pragma unroll
  for (int j = 0; j < K1; ++j) {
    double s = 0.;
#pragma unroll
    for (int i = 0; i < K1; ++i) s += M[j][i] * in[i];
    out[j] = s * scale;
  }
}
// transposed: out[i] += sum_j M[j][i] in[j]   (quadrature -> nodes)
template <int K1>
__device__ __forceinline__ void bwd_add(const double (&M)[kMaxQ1D][kMaxNodes1D], const double *in, double *out) {
#pragma unroll
  for (int i = 0; i < K1; ++i) {
    double s = out[i];
#pragma unroll
    for (int j = 0; j < K1; ++j) s += M[j][i] * in[j];
    out[i] = s;
  }
}

template <int K, int MODE>
__global__ void __launch_bounds__(BrickCfg<K>::THREADS) gls_brick_kernel(const OpParams P, const Tables1D T) {
  using C = BrickCfg<K>;
  constexpr int K1 = C::K1, N3 = C::N3, L2 = C::L2, BN = C::BN, BN3 = C::BN3, NB = C::NB, NC = C::NC;
  constexpr int R1N = C::R1N, R2N = C::R2N;
  constexpr bool JV = MODE == MODE_JV;
  constexpr int NF = JV ? 11 : 7;  // brick fields: u0 u1 u2 p H0 H1 H2 [v0 v1 v2 vp]
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double *sB = smem;                         // [NB][NF][BN3]
  double *sR1 = sB + NB * NF * BN3;          // [NC][R1N][N3]
  double *sR2 = sR1 + NC * R1N * N3;         // [NC][R2N][N3]
  int *sNode = reinterpret_cast<int *>(sR2 + NC * R2N * N3);  // [NB][BN3]
  auto A1 = [&](int c, int s) { return sR1 + (c * R1N + s) * N3; };
  auto A2 = [&](int c, int s) { return sR2 + (c * R2N + s) * N3; };
  auto BF = [&](int b, int f) { return sB + (b * NF + f) * BN3; };

  const int tid = threadIdx.x;
  const int n_bricks = P.n_cells / 8;
  const int b0 = blockIdx.x * NB;
  const int nb = min(NB, n_bricks - b0);
  const int ncell = 8 * nb;
  const int64_t voff = (int64_t)3 * P.n_vnodes;

  // ---------------- gather brick nodes
  for (int t = tid; t < nb * BN3; t += blockDim.x) {
    const int b = t / BN3, n = t % BN3;
    const int X = n % BN, Y = (n / BN) % BN, Z = n / (BN * BN);
    const int cx = min(X / K, 1), cy = min(Y / K, 1), cz = min(Z / K, 1);
    const int a = (X - K * cx) + K1 * ((Y - K * cy) + K1 * (Z - K * cz));
    const int cell = (b0 + b) * 8 + cx + 2 * cy + 4 * cz;
    const int node = P.cell_vnodes[(int64_t)cell * N3 + a];
    sNode[b * BN3 + n] = node;
    const int64_t i3 = (int64_t)node * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      BF(b, c)[n] = P.u[i3 + c];
      double h = 0.;
      if (P.n_hist > 0) h += P.alpha[1] * P.h1[i3 + c];
      if (P.n_hist > 1) h += P.alpha[2] * P.h2[i3 + c];
      if (P.n_hist > 2) h += P.alpha[3] * P.h3[i3 + c];
      BF(b, 4 + c)[n] = h;
    }
    BF(b, 3)[n] = P.u[voff + node];
    if constexpr (JV) {
      const unsigned m = P.vmask ? P.vmask[node] : 0u;
#pragma unroll
      for (int c = 0; c < 3; ++c) BF(b, 7 + c)[n] = ((m >> c) & 1u) ? 0.0 : P.v[i3 + c];
      BF(b, 10)[n] = P.v[voff + node];
    }
  }
  __syncthreads();

  // per-cell geometry (cell of this thread in the pointwise phases)
  auto cell_h = [&](int ci, double &hx, double &hy, double &hz) {
    const int cell = b0 * 8 + ci;
    hx = P.geo[cell * 4 + 0];
    hy = P.geo[cell * 4 + 1];
    hz = P.geo[cell * 4 + 2];
  };

  // ---------------- x sweep from the brick: field f of brick -> R2 slots (phase A: f=0..6, phase B: f=7..10)
  auto sweep_x = [&](int f0, int nvel, int out_vel, int out_p, int out_h, int nh) {
    // jobs: [0,nvel): velocity comps (B,D,S); nvel: pressure (B,D); then nh value-only fields
    const int jobs = nvel + 1 + nh;
    for (int t = tid; t < ncell * jobs * L2; t += blockDim.x) {
      const int ci = t / (jobs * L2), r = t % (jobs * L2), job = r / L2, l = r % L2;
      const int b = ci / 8, cc = ci % 8, cx = cc & 1, cy = (cc >> 1) & 1, cz = cc >> 2;
      const int i1 = l % K1, i2 = l / K1;
      const int base = K * cx + BN * (K * cy + i1) + BN * BN * (K * cz + i2);
      const int f = job < nvel ? f0 + job : (job == nvel ? f0 + nvel : f0 + nvel + 1 + (job - nvel - 1));
      double in[K1], o[K1];
      const double *src = BF(b, f) + base;
#pragma unroll
      for (int e = 0; e < K1; ++e) in[e] = src[e];
      if (job < nvel) {
        double *d0 = A2(ci, out_vel + 3 * job), *d1 = d0 + N3, *d2 = d1 + N3;
        fwd<K1>(T.V, in, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) d0[loff<0, K1>(l, e)] = o[e];
        fwd<K1>(T.D, in, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) d1[loff<0, K1>(l, e)] = o[e];
        fwd<K1>(T.S, in, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) d2[loff<0, K1>(l, e)] = o[e];
      } else if (job == nvel) {
        double *d0 = A2(ci, out_p), *d1 = d0 + N3;
        fwd<K1>(T.V, in, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) d0[loff<0, K1>(l, e)] = o[e];
        fwd<K1>(T.D, in, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) d1[loff<0, K1>(l, e)] = o[e];
      } else {
        double *d0 = A2(ci, out_h + (job - nvel - 1));
        fwd<K1>(T.V, in, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) d0[loff<0, K1>(l, e)] = o[e];
      }
    }
  };

  // ---------------- y sweep R2 -> R1: velocity comps (X_B,X_D,X_S -> BB,BD,DB,L), pressure (BB,BD,DB), H (BB)
  auto sweep_y = [&](int nvel, int in_p, int in_h, int nh) {
    const int jobs = nvel + 1 + nh;
    for (int t = tid; t < ncell * jobs * L2; t += blockDim.x) {
      const int ci = t / (jobs * L2), r = t % (jobs * L2), job = r / L2, l = r % L2;
      double hx, hy, hz;
      cell_h(ci, hx, hy, hz);
      double a[K1], bq[K1], o[K1], o2[K1];
      if (job < nvel) {
        const double *xb = A2(ci, 3 * job), *xd = xb + N3, *xs = xd + N3;
        double *dbb = A1(ci, 4 * job), *dbd = dbb + N3, *ddb = dbd + N3, *dl = ddb + N3;
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = xb[loff<1, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dbb[loff<1, K1>(l, e)] = o[e];
        fwd<K1>(T.D, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dbd[loff<1, K1>(l, e)] = o[e];
        fwd<K1>(T.S, a, o, 1.0 / (hy * hy));
#pragma unroll
        for (int e = 0; e < K1; ++e) bq[e] = xs[loff<1, K1>(l, e)];
        fwd<K1>(T.V, bq, o2, 1.0 / (hx * hx));
#pragma unroll
        for (int e = 0; e < K1; ++e) dl[loff<1, K1>(l, e)] = o[e] + o2[e];
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = xd[loff<1, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) ddb[loff<1, K1>(l, e)] = o[e];
      } else if (job == nvel) {
        const double *xb = A2(ci, in_p), *xd = xb + N3;
        double *dbb = A1(ci, 12), *dbd = dbb + N3, *ddb = dbd + N3;
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = xb[loff<1, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dbb[loff<1, K1>(l, e)] = o[e];
        fwd<K1>(T.D, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dbd[loff<1, K1>(l, e)] = o[e];
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = xd[loff<1, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) ddb[loff<1, K1>(l, e)] = o[e];
      } else {
        const int hcmp = job - nvel - 1;
        const double *xb = A2(ci, in_h + hcmp);
        double *dbb = A1(ci, 15 + hcmp);
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = xb[loff<1, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dbb[loff<1, K1>(l, e)] = o[e];
      }
    }
  };

  // ---------------- z sweep R1 -> R2: velocity -> (val,gx,gy,gz,L) at 5c; pressure -> (gx,gy,gz,val) at 15..18; H -> 19..
  auto sweep_z = [&](int nvel, int nh) {
    const int jobs = nvel + 1 + nh;
    for (int t = tid; t < ncell * jobs * L2; t += blockDim.x) {
      const int ci = t / (jobs * L2), r = t % (jobs * L2), job = r / L2, l = r % L2;
      double hx, hy, hz;
      cell_h(ci, hx, hy, hz);
      double a[K1], o[K1], o2[K1];
      if (job < nvel) {
        const double *ybb = A1(ci, 4 * job), *ybd = ybb + N3, *ydb = ybd + N3, *yl = ydb + N3;
        double *dv = A2(ci, 5 * job), *dgx = dv + N3, *dgy = dgx + N3, *dgz = dgy + N3, *dl = dgz + N3;
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = ybb[loff<2, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dv[loff<2, K1>(l, e)] = o[e];
        fwd<K1>(T.D, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dgz[loff<2, K1>(l, e)] = o[e];
        fwd<K1>(T.S, a, o, 1.0 / (hz * hz));
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = yl[loff<2, K1>(l, e)];
        fwd<K1>(T.V, a, o2);
#pragma unroll
        for (int e = 0; e < K1; ++e) dl[loff<2, K1>(l, e)] = o[e] + o2[e];
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = ydb[loff<2, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dgx[loff<2, K1>(l, e)] = o[e];
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = ybd[loff<2, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dgy[loff<2, K1>(l, e)] = o[e];
      } else if (job == nvel) {
        const double *ybb = A1(ci, 12), *ybd = ybb + N3, *ydb = ybd + N3;
        double *dgx = A2(ci, 15), *dgy = dgx + N3, *dgz = dgy + N3, *dv = dgz + N3;
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = ybb[loff<2, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dv[loff<2, K1>(l, e)] = o[e];
        fwd<K1>(T.D, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dgz[loff<2, K1>(l, e)] = o[e];
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = ydb[loff<2, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dgx[loff<2, K1>(l, e)] = o[e];
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = ybd[loff<2, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dgy[loff<2, K1>(l, e)] = o[e];
      } else {
        const int hcmp = job - nvel - 1;
        const double *ybb = A1(ci, 15 + hcmp);
        double *dv = A2(ci, 19 + hcmp);
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = ybb[loff<2, K1>(l, e)];
        fwd<K1>(T.V, a, o);
#pragma unroll
        for (int e = 0; e < K1; ++e) dv[loff<2, K1>(l, e)] = o[e];
      }
    }
  };

  // ---------------- phase A: state at quadrature points
  sweep_x(0, 3, 0, 9, 11, 3);
  __syncthreads();
  sweep_y(3, 9, 11, 3);
  __syncthreads();
  sweep_z(3, 3);
  __syncthreads();

  const bool active = tid < ncell * N3;
  const int ci = tid / N3, q = tid % N3;
  double hx = 1, hy = 1, hz = 1;
  double u[3] = {}, gu[3][3] = {}, R[3] = {}, tau = 0., JxW = 0.;
  double Tc[16];
  if (active) {
    cell_h(ci, hx, hy, hz);
    const int cell = b0 * 8 + ci;
    const int qx = q % K1, qy = (q / K1) % K1, qz = q / (K1 * K1);
    const double ih[3] = {1.0 / hx, 1.0 / hy, 1.0 / hz};
    const double hst = P.geo[cell * 4 + 3];
    JxW = T.w[qx] * T.w[qy] * T.w[qz] * hx * hy * hz;
    double lu[3], gp[3], Hq[3], pq;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      u[c] = A2(ci, 5 * c)[q];
#pragma unroll
      for (int e = 0; e < 3; ++e) gu[c][e] = A2(ci, 5 * c + 1 + e)[q] * ih[e];
      lu[c] = A2(ci, 5 * c + 4)[q];
      gp[c] = A2(ci, 15 + c)[q] * ih[c];
      Hq[c] = A2(ci, 19 + c)[q];
    }
    pq = A2(ci, 18)[q];
    const double nu = P.nu;
    const double un2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
    const double u_mag = fmax(sqrt(un2), 1e-12);
    const double t1 = 2. * u_mag / hst, t2 = 4 * nu / (hst * hst);
    tau = 1. / sqrt(P.sdt2 + t1 * t1 + 9 * (t2 * t2));
    double f[3] = {0., 0., 0.};
    if (P.force_q) {
#pragma unroll
      for (int c = 0; c < 3; ++c) f[c] = P.force_q[((int64_t)cell * N3 + q) * 3 + c];
    }
    double Gu[3], srf[3] = {0., 0., 0.};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      Gu[c] = gu[c][0] * u[0] + gu[c][1] * u[1] + gu[c][2] * u[2];
      R[c] = Gu[c] + gp[c] - nu * lu[c] - f[c];
    }
    if (P.srf) {
      const double *om = P.omega;
      const double xq[3] = {P.x0[cell * 3 + 0] + hx * T.xi[qx], P.x0[cell * 3 + 1] + hy * T.xi[qy],
                            P.x0[cell * 3 + 2] + hz * T.xi[qz]};
      const double cx_[3] = {om[1] * u[2] - om[2] * u[1], om[2] * u[0] - om[0] * u[2], om[0] * u[1] - om[1] * u[0]};
      const double ox[3] = {om[1] * xq[2] - om[2] * xq[1], om[2] * xq[0] - om[0] * xq[2], om[0] * xq[1] - om[1] * xq[0]};
      const double cc[3] = {om[1] * ox[2] - om[2] * ox[1], om[2] * ox[0] - om[0] * ox[2], om[0] * ox[1] - om[1] * ox[0]};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        srf[c] = 2 * cx_[c] + cc[c];
        R[c] += srf[c];
      }
    }
    double Tt[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      Tt[c] = P.alpha[0] * u[c] + Hq[c];
      R[c] += Tt[c];
    }
    if constexpr (!JV) {  // residual test coefficients (rhs = -R)
      const double divu = gu[0][0] + gu[1][1] + gu[2][2];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        Tc[4 * c] = JxW * (-Gu[c] + f[c] - Tt[c] - srf[c]);
#pragma unroll
        for (int e = 0; e < 3; ++e)
          Tc[4 * c + 1 + e] = JxW * (-nu * gu[c][e] + (c == e ? pq : 0.0) - tau * R[c] * u[e]) * ih[e];
      }
      Tc[12] = -JxW * divu;
#pragma unroll
      for (int e = 0; e < 3; ++e) Tc[13 + e] = -JxW * tau * R[e] * ih[e];
    }
  }
  __syncthreads();  // R1/R2 reusable

  if constexpr (JV) {
    // ---------------- phase B: trial function v at quadrature points
    sweep_x(7, 3, 0, 9, 0, 0);
    __syncthreads();
    sweep_y(3, 9, 0, 0);
    __syncthreads();
    sweep_z(3, 0);
    __syncthreads();
    if (active) {
      const double ih[3] = {1.0 / hx, 1.0 / hy, 1.0 / hz};
      const double nu = P.nu, aj = P.alpha_jac;
      double v[3], gv[3][3], lv[3], gvp[3], vp;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        v[c] = A2(ci, 5 * c)[q];
#pragma unroll
        for (int e = 0; e < 3; ++e) gv[c][e] = A2(ci, 5 * c + 1 + e)[q] * ih[e];
        lv[c] = A2(ci, 5 * c + 4)[q];
        gvp[c] = A2(ci, 15 + c)[q] * ih[c];
      }
      vp = A2(ci, 18)[q];
      double S[3], A[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const double guv = gu[c][0] * v[0] + gu[c][1] * v[1] + gu[c][2] * v[2];
        const double gvu = gv[c][0] * u[0] + gv[c][1] * u[1] + gv[c][2] * u[2];
        A[c] = guv + gvu + aj * v[c];
        S[c] = guv + gvu + gvp[c] - nu * lv[c] + aj * v[c];
      }
      if (P.srf) {
        const double *om = P.omega;
        const double cj[3] = {2 * (om[1] * v[2] - om[2] * v[1]), 2 * (om[2] * v[0] - om[0] * v[2]),
                              2 * (om[0] * v[1] - om[1] * v[0])};
#pragma unroll
        for (int c = 0; c < 3; ++c) { A[c] += cj[c]; S[c] += cj[c]; }
      }
      const double divv = gv[0][0] + gv[1][1] + gv[2][2];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        Tc[4 * c] = JxW * A[c];
#pragma unroll
        for (int e = 0; e < 3; ++e)
          Tc[4 * c + 1 + e] =
              JxW * (nu * gv[c][e] - (c == e ? vp : 0.0) + tau * S[c] * u[e] + tau * R[c] * v[e]) * ih[e];
      }
      Tc[12] = JxW * divv;
#pragma unroll
      for (int e = 0; e < 3; ++e) Tc[13 + e] = JxW * tau * S[e] * ih[e];
    }
    __syncthreads();
  }

  // ---------------- test coefficients -> R1 slots 4f + {val, gx, gy, gz}
  if (active) {
#pragma unroll
    for (int s = 0; s < 16; ++s) A1(ci, s)[q] = Tc[s];
  }
  __syncthreads();
  // transposed z: Z0 = B^T Tv + D^T Tz, Z1 = B^T Tx, Z2 = B^T Ty  -> R2 3f+{0,1,2}
  for (int t = tid; t < ncell * 4 * L2; t += blockDim.x) {
    const int c_ = t / (4 * L2), r = t % (4 * L2), fld = r / L2, l = r % L2;
    const double *tv = A1(c_, 4 * fld), *tx = tv + N3, *ty = tx + N3, *tz = ty + N3;
    double a[K1], o[K1];
    double *z0 = A2(c_, 3 * fld), *z1 = z0 + N3, *z2 = z1 + N3;
#pragma unroll
    for (int e = 0; e < K1; ++e) o[e] = 0.;
#pragma unroll
    for (int e = 0; e < K1; ++e) a[e] = tv[loff<2, K1>(l, e)];
    bwd_add<K1>(T.V, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) a[e] = tz[loff<2, K1>(l, e)];
    bwd_add<K1>(T.D, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) z0[loff<2, K1>(l, e)] = o[e];
#pragma unroll
    for (int e = 0; e < K1; ++e) { a[e] = tx[loff<2, K1>(l, e)]; o[e] = 0.; }
    bwd_add<K1>(T.V, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) z1[loff<2, K1>(l, e)] = o[e];
#pragma unroll
    for (int e = 0; e < K1; ++e) { a[e] = ty[loff<2, K1>(l, e)]; o[e] = 0.; }
    bwd_add<K1>(T.V, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) z2[loff<2, K1>(l, e)] = o[e];
  }
  __syncthreads();
  // transposed y: W0 = B^T Z0 + D^T Z2, W1 = B^T Z1 -> R1 2f+{0,1}
  for (int t = tid; t < ncell * 4 * L2; t += blockDim.x) {
    const int c_ = t / (4 * L2), r = t % (4 * L2), fld = r / L2, l = r % L2;
    const double *z0 = A2(c_, 3 * fld), *z1 = z0 + N3, *z2 = z1 + N3;
    double *w0 = A1(c_, 2 * fld), *w1 = w0 + N3;
    double a[K1], o[K1];
#pragma unroll
    for (int e = 0; e < K1; ++e) { a[e] = z0[loff<1, K1>(l, e)]; o[e] = 0.; }
    bwd_add<K1>(T.V, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) a[e] = z2[loff<1, K1>(l, e)];
    bwd_add<K1>(T.D, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) w0[loff<1, K1>(l, e)] = o[e];
#pragma unroll
    for (int e = 0; e < K1; ++e) { a[e] = z1[loff<1, K1>(l, e)]; o[e] = 0.; }
    bwd_add<K1>(T.V, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) w1[loff<1, K1>(l, e)] = o[e];
  }
  __syncthreads();
  // transposed x: out = B^T W0 + D^T W1 -> R2 slot 12+f (node-indexed)
  for (int t = tid; t < ncell * 4 * L2; t += blockDim.x) {
    const int c_ = t / (4 * L2), r = t % (4 * L2), fld = r / L2, l = r % L2;
    const double *w0 = A1(c_, 2 * fld), *w1 = w0 + N3;
    double *out = A2(c_, 12 + fld);
    double a[K1], o[K1];
#pragma unroll
    for (int e = 0; e < K1; ++e) { a[e] = w0[loff<0, K1>(l, e)]; o[e] = 0.; }
    bwd_add<K1>(T.V, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) a[e] = w1[loff<0, K1>(l, e)];
    bwd_add<K1>(T.D, a, o);
#pragma unroll
    for (int e = 0; e < K1; ++e) out[loff<0, K1>(l, e)] = o[e];
  }
  __syncthreads();

  // ---------------- brick reduction (fixed order) + scatter
  for (int t = tid; t < nb * BN3 * 4; t += blockDim.x) {
    const int b = t / (BN3 * 4), r = t % (BN3 * 4), n = r / 4, fld = r % 4;
    const int X = n % BN, Y = (n / BN) % BN, Z = n / (BN * BN);
    double s = 0.;
#pragma unroll
    for (int cz = 0; cz < 2; ++cz) {
      const int az = Z - K * cz;
      if (az < 0 || az > K) continue;
#pragma unroll
      for (int cy = 0; cy < 2; ++cy) {
        const int ay = Y - K * cy;
        if (ay < 0 || ay > K) continue;
#pragma unroll
        for (int cx = 0; cx < 2; ++cx) {
          const int ax = X - K * cx;
          if (ax < 0 || ax > K) continue;
          s += A2(b * 8 + cx + 2 * cy + 4 * cz, 12 + fld)[ax + K1 * (ay + K1 * az)];
        }
      }
    }
    const int node = sNode[b * BN3 + n];
    const int64_t gi = fld < 3 ? (int64_t)node * 3 + fld : voff + node;
    const bool interior = X > 0 && X < BN - 1 && Y > 0 && Y < BN - 1 && Z > 0 && Z < BN - 1;
    if (interior) P.y[gi] = s;
    else atomicAdd(&P.y[gi], s);
  }
}

template <int K>
size_t brick_lds_bytes(int mode) {
  using C = BrickCfg<K>;
  const int NF = mode == MODE_JV ? 11 : 7;
  return sizeof(double) * ((size_t)C::NB * NF * C::BN3 + (size_t)C::NC * (C::R1N + C::R2N) * C::N3) +
         sizeof(int) * (size_t)C::NB * C::BN3;
}

template <int K>
hipError_t launch_brick_t(int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  using C = BrickCfg<K>;
  const int n_bricks = P.n_cells / 8;
  if (n_bricks <= 0) return hipSuccess;
  const int blocks = (n_bricks + C::NB - 1) / C::NB;
  const size_t lds = brick_lds_bytes<K>(mode);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void *)gls_brick_kernel<K, MODE_RESIDUAL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)brick_lds_bytes<K>(MODE_JV));
    (void)hipFuncSetAttribute((const void *)gls_brick_kernel<K, MODE_JV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)brick_lds_bytes<K>(MODE_JV));
    attr = true;
  }
  if (mode == MODE_JV)
    hipLaunchKernelGGL((gls_brick_kernel<K, MODE_JV>), dim3(blocks), dim3(C::THREADS), lds, s, P, T);
  else
    hipLaunchKernelGGL((gls_brick_kernel<K, MODE_RESIDUAL>), dim3(blocks), dim3(C::THREADS), lds, s, P, T);
  return hipGetLastError();
}

hipError_t launch_brick_kernel(int k, int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (mode == MODE_DIAG) return hipErrorNotSupported;
  if (k == 1) return launch_brick_t<1>(mode, P, T, s);
  if (k == 2) return launch_brick_t<2>(mode, P, T, s);
  return hipErrorNotSupported;
}

}  // namespace gls
