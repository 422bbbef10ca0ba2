// gls_brick_kernels.hip — sum-factorized GLS operators on 2x2x2 cell bricks (3D, Qk-Qk).
//
// Why this shape (MI355X-first): on gfx950 FP64 MFMA (v_mfma_f64_16x16x4) and FP64 VALU share
// one ~62 TF budget (profiles/r01_microbench_fp64.txt: 61.3 / 63.5 / 59.1 TF mixed), so the lever
// is FLOPs and latency, not the pipe. Tensor-product sum factorization does the basis x
// coefficient work in ~24 kFLOP per Q2 cell (a dense n_dofs x n_q contraction: ~86 kFLOP). The 1D
// matrices are uniform across the wave and indexed with compile-time constants (SGPR operands).
//
// Work unit: one workgroup = one Morton brick = 8 consecutive cells forming a 2x2x2 block (the
// hyper_cube builder emits p4est z-order). The brick's unique (2k+1)^3 nodes are gathered once
// into LDS (u, p, the history combination H = sum_k alpha_k u^(k), and v / v_p for J.v); each
// wave then owns 2 cells and runs its whole per-cell pipeline wave-locally (LDS exchanges ordered
// by in-order LDS execution within a wave: no workgroup barriers); the cells' node contributions
// are summed per brick node in a fixed order (deterministic), brick-interior nodes are written
// with plain stores and brick-boundary nodes with FP64 atomics.
//
// Per-cell pipeline, one field at a time (keeps ~3 KB of LDS per cell -> 4 workgroups per CU):
//   x sweep (brick -> X), y sweep (X -> Y), z sweep fused into the pointwise read (Y -> registers)
//   state  : u (value, grad, Laplacian) x 3 comps, then {p (value, grad), H (value) x 3}
//   J.v    : v (value, grad, Laplacian) x 3 comps, then v_p (value, grad)
//   test   : per test field, transposed z/y/x sweeps of (value, grad) coefficients -> node array
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
  static constexpr int CPW = 64 / N3 >= 2 ? 2 : 1;  // cells per wave (Q1: 8 q -> could be 8; keep 2)
  static constexpr int WAVES = 8 / CPW;      // waves per workgroup (one brick)
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int NX = 5, NY = 6, NO = 4;  // per-cell LDS arrays: X, Y, out
  static constexpr int PER_CELL = NX + NY + NO;
};

// offset of element e of line l in a [K1][K1][K1] array ([z][y][x], x fastest), sweep dim D
template <int D, int K1>
__device__ __forceinline__ int loff(int l, int e) {
  if constexpr (D == 0) return e + K1 * l;
  else if constexpr (D == 1) return (l % K1) + K1 * e + K1 * K1 * (l / K1);
  else return l + K1 * K1 * e;
}

// forward: out[j] = sum_i M[j][i] in[i] (nodes -> q);  transposed: out[i] = sum_j M[j][i] in[j]
template <int K1>
__device__ __forceinline__ void fwd(const double (&M)[kMaxQ1D][kMaxNodes1D], const double *in, double *out) {
#pragma unroll
  for (int j = 0; j < K1; ++j) {
    double s = 0.;
#pragma unroll
    for (int i = 0; i < K1; ++i) s += M[j][i] * in[i];
    out[j] = s;
  }
}
template <int K1>
__device__ __forceinline__ void bwd(const double (&M)[kMaxQ1D][kMaxNodes1D], const double *in, double *out) {
#pragma unroll
  for (int i = 0; i < K1; ++i) {
    double s = 0.;
#pragma unroll
    for (int j = 0; j < K1; ++j) s += M[j][i] * in[j];
    out[i] = s;
  }
}
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

// LDS hand-off between lanes of ONE wave: LDS ops of a wave execute in order; the asm keeps the
// compiler from moving LDS accesses across this point.
__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <int K, int MODE>
__global__ void __launch_bounds__(BrickCfg<K>::THREADS) gls_brick_kernel(const OpParams P, const Tables1D T) {
  using C = BrickCfg<K>;
  constexpr int K1 = C::K1, N3 = C::N3, L2 = C::L2, BN = C::BN, BN3 = C::BN3, CPW = C::CPW;
  constexpr bool JV = MODE == MODE_JV;
  constexpr int NF = JV ? 11 : 7;  // brick fields: u0 u1 u2 p H0 H1 H2 [v0 v1 v2 vp]
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double *sB = smem;                                   // [NF][BN3]
  double *sC = sB + NF * BN3;                          // [8][PER_CELL][N3]
  int *sNode = reinterpret_cast<int *>(sC + 8 * C::PER_CELL * N3);  // [BN3]
  auto BF = [&](int f) { return sB + f * BN3; };

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int brick = blockIdx.x;
  const int64_t voff = (int64_t)3 * P.n_vnodes;

  // ---------------- gather the brick's nodes (all waves)
  for (int t = tid; t < 3 * BN3; t += blockDim.x) {
    const int g = t / BN3, n = t % BN3;
    const int X = n % BN, Y = (n / BN) % BN, Z = n / (BN * BN);
    const int cx = min(X / K, 1), cy = min(Y / K, 1), cz = min(Z / K, 1);
    const int a = (X - K * cx) + K1 * ((Y - K * cy) + K1 * (Z - K * cz));
    const int node = P.cell_vnodes[((int64_t)brick * 8 + cx + 2 * cy + 4 * cz) * N3 + a];
    const int64_t i3 = (int64_t)node * 3;
    if (g == 0) {
      sNode[n] = node;
      BF(0)[n] = P.u[i3];
      BF(1)[n] = P.u[i3 + 1];
      BF(2)[n] = P.u[i3 + 2];
      BF(3)[n] = P.u[voff + node];
    } else if (g == 1) {
      double h[3] = {0., 0., 0.};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        if (P.n_hist > 0) h[c] += P.alpha[1] * P.h1[i3 + c];
        if (P.n_hist > 1) h[c] += P.alpha[2] * P.h2[i3 + c];
        if (P.n_hist > 2) h[c] += P.alpha[3] * P.h3[i3 + c];
      }
      BF(4)[n] = h[0];
      BF(5)[n] = h[1];
      BF(6)[n] = h[2];
    } else if (JV) {
      const unsigned m = P.vmask ? P.vmask[node] : 0u;
      BF(7)[n] = (m & 1u) ? 0.0 : P.v[i3];
      BF(8)[n] = (m & 2u) ? 0.0 : P.v[i3 + 1];
      BF(9)[n] = (m & 4u) ? 0.0 : P.v[i3 + 2];
      BF(10)[n] = P.v[voff + node];
    }
  }
  __syncthreads();

  // ---------------- per-wave: cells 2*wave, 2*wave+1 of the brick
  auto X = [&](int ci, int s) { return sC + (ci * C::PER_CELL + s) * N3; };
  auto Yr = [&](int ci, int s) { return sC + (ci * C::PER_CELL + C::NX + s) * N3; };
  auto Out = [&](int ci, int f) { return sC + (ci * C::PER_CELL + C::NX + C::NY + f) * N3; };
  const int cbase = wave * CPW;
  // pointwise lane mapping: lane -> (cell, q)
  const bool pact = lane < CPW * N3;
  const int pci = cbase + (pact ? lane / N3 : 0);
  const int q = pact ? lane % N3 : 0;
  const int qx = q % K1, qy = (q / K1) % K1, qz = q / (K1 * K1);
  const int gcell = brick * 8 + pci;
  const double hx = P.geo[gcell * 4 + 0], hy = P.geo[gcell * 4 + 1], hz = P.geo[gcell * 4 + 2];
  const double ih[3] = {1.0 / hx, 1.0 / hy, 1.0 / hz};
  const double wx = ih[0] * ih[0], wy = ih[1] * ih[1], wz = ih[2] * ih[2];
  // this lane's rows of the z matrices (q-dependent -> registers)
  double Bz[K1], Dz[K1], Sz[K1];
#pragma unroll
  for (int i = 0; i < K1; ++i) { Bz[i] = T.V[qz][i]; Dz[i] = T.D[qz][i]; Sz[i] = T.S[qz][i]; }

  // brick-array line base for (cell-in-brick, line (i1,i2)) in an x sweep
  auto bline = [&](int ci, int l) {
    const int cx = ci & 1, cy = (ci >> 1) & 1, cz = ci >> 2;
    return K * cx + BN * (K * cy + l % K1) + BN * BN * (K * cz + l / K1);
  };

  // velocity-type field (value, grad, Laplacian): brick field f -> (val, g0, g1, g2, lap) for this lane
  auto vel_field = [&](int f, double &val, double (&g)[3], double &lap) {
    // x sweep: tasks (cell, line, mat) = CPW*L2*3
    for (int t = lane; t < CPW * L2 * 3; t += 64) {
      const int ci = cbase + t / (L2 * 3), r = t % (L2 * 3), l = r / 3, m = r % 3;
      const double *src = BF(f) + bline(ci, l);
      double in[K1], o[K1];
#pragma unroll
      for (int e = 0; e < K1; ++e) in[e] = src[e];
      if (m == 0) fwd<K1>(T.V, in, o);
      else if (m == 1) fwd<K1>(T.D, in, o);
      else fwd<K1>(T.S, in, o);
      double *dst = X(ci, m);
#pragma unroll
      for (int e = 0; e < K1; ++e) dst[loff<0, K1>(l, e)] = o[e];
    }
    wave_sync();
    // y sweep: tasks (cell, line, type): 0: X_B -> BB, BD; 1: X_D -> DB; 2: L = wx B(X_S) + wy S(X_B)
    for (int t = lane; t < CPW * L2 * 3; t += 64) {
      const int ci = cbase + t / (L2 * 3), r = t % (L2 * 3), l = r / 3, m = r % 3;
      double a[K1], o[K1];
      if (m == 0) {
        const double *s = X(ci, 0);
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = s[loff<1, K1>(l, e)];
        fwd<K1>(T.V, a, o);
        double *d = Yr(ci, 0);
#pragma unroll
        for (int e = 0; e < K1; ++e) d[loff<1, K1>(l, e)] = o[e];
        fwd<K1>(T.D, a, o);
        d = Yr(ci, 1);
#pragma unroll
        for (int e = 0; e < K1; ++e) d[loff<1, K1>(l, e)] = o[e];
      } else if (m == 1) {
        const double *s = X(ci, 1);
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = s[loff<1, K1>(l, e)];
        fwd<K1>(T.V, a, o);
        double *d = Yr(ci, 2);
#pragma unroll
        for (int e = 0; e < K1; ++e) d[loff<1, K1>(l, e)] = o[e];
      } else {
        const int cg = brick * 8 + ci;
        const double hx_ = P.geo[cg * 4 + 0], hy_ = P.geo[cg * 4 + 1];
        const double wxx = 1.0 / (hx_ * hx_), wyy = 1.0 / (hy_ * hy_);
        const double *s0 = X(ci, 0), *s2 = X(ci, 2);
        double b[K1], o2[K1];
#pragma unroll
        for (int e = 0; e < K1; ++e) { a[e] = s0[loff<1, K1>(l, e)]; b[e] = s2[loff<1, K1>(l, e)]; }
        fwd<K1>(T.S, a, o);
        fwd<K1>(T.V, b, o2);
        double *d = Yr(ci, 3);
#pragma unroll
        for (int e = 0; e < K1; ++e) d[loff<1, K1>(l, e)] = wyy * o[e] + wxx * o2[e];
      }
    }
    wave_sync();
    // z sweep fused into the pointwise read
    if (pact) {
      const int l = qx + K1 * qy;
      double bb[K1], bd[K1], db[K1], ll[K1];
#pragma unroll
      for (int e = 0; e < K1; ++e) {
        bb[e] = Yr(pci, 0)[loff<2, K1>(l, e)];
        bd[e] = Yr(pci, 1)[loff<2, K1>(l, e)];
        db[e] = Yr(pci, 2)[loff<2, K1>(l, e)];
        ll[e] = Yr(pci, 3)[loff<2, K1>(l, e)];
      }
      double v = 0., gz = 0., zz = 0., gx = 0., gy = 0., lp = 0.;
#pragma unroll
      for (int e = 0; e < K1; ++e) {
        v += Bz[e] * bb[e];
        gz += Dz[e] * bb[e];
        zz += Sz[e] * bb[e];
        gx += Bz[e] * db[e];
        gy += Bz[e] * bd[e];
        lp += Bz[e] * ll[e];
      }
      val = v;
      g[0] = gx * ih[0];
      g[1] = gy * ih[1];
      g[2] = gz * ih[2];
      lap = lp + wz * zz;
    }
    wave_sync();  // Y is rewritten by the next field's y sweep
  };

  // pressure-type field (value, grad) [+ up to 3 value-only fields]: fp -> (pv, pg); fh.. -> hv[]
  auto scal_fields = [&](int fp, int nh, int fh0, double &pv, double (&pg)[3], double (&hv)[3]) {
    // x: tasks (cell, line, job): job 0: p (B -> X0, D -> X1); job 1..nh: H comp (B -> X2+j)
    const int nj = 1 + nh;
    for (int t = lane; t < CPW * L2 * nj; t += 64) {
      const int ci = cbase + t / (L2 * nj), r = t % (L2 * nj), l = r / nj, j = r % nj;
      const double *src = BF(j == 0 ? fp : fh0 + j - 1) + bline(ci, l);
      double in[K1], o[K1];
#pragma unroll
      for (int e = 0; e < K1; ++e) in[e] = src[e];
      fwd<K1>(T.V, in, o);
      double *d = X(ci, j == 0 ? 0 : 1 + j);
#pragma unroll
      for (int e = 0; e < K1; ++e) d[loff<0, K1>(l, e)] = o[e];
      if (j == 0) {
        fwd<K1>(T.D, in, o);
        d = X(ci, 1);
#pragma unroll
        for (int e = 0; e < K1; ++e) d[loff<0, K1>(l, e)] = o[e];
      }
    }
    wave_sync();
    // y: job 0: X0 -> BB (Y0), BD (Y1); job 1: X1 -> DB (Y2); job 1+j: X(1+j) -> Y(2+j)
    const int ny = 2 + nh;
    for (int t = lane; t < CPW * L2 * ny; t += 64) {
      const int ci = cbase + t / (L2 * ny), r = t % (L2 * ny), l = r / ny, j = r % ny;
      const double *s = X(ci, j == 0 ? 0 : j);
      double a[K1], o[K1];
#pragma unroll
      for (int e = 0; e < K1; ++e) a[e] = s[loff<1, K1>(l, e)];
      fwd<K1>(T.V, a, o);
      double *d = Yr(ci, j == 0 ? 0 : 1 + j);
#pragma unroll
      for (int e = 0; e < K1; ++e) d[loff<1, K1>(l, e)] = o[e];
      if (j == 0) {
        fwd<K1>(T.D, a, o);
        d = Yr(ci, 1);
#pragma unroll
        for (int e = 0; e < K1; ++e) d[loff<1, K1>(l, e)] = o[e];
      }
    }
    wave_sync();
    if (pact) {
      const int l = qx + K1 * qy;
      double bb[K1], bd[K1], db[K1];
#pragma unroll
      for (int e = 0; e < K1; ++e) {
        bb[e] = Yr(pci, 0)[loff<2, K1>(l, e)];
        bd[e] = Yr(pci, 1)[loff<2, K1>(l, e)];
        db[e] = Yr(pci, 2)[loff<2, K1>(l, e)];
      }
      double v = 0., gz = 0., gx = 0., gy = 0.;
#pragma unroll
      for (int e = 0; e < K1; ++e) {
        v += Bz[e] * bb[e];
        gz += Dz[e] * bb[e];
        gx += Bz[e] * db[e];
        gy += Bz[e] * bd[e];
      }
      pv = v;
      pg[0] = gx * ih[0];
      pg[1] = gy * ih[1];
      pg[2] = gz * ih[2];
      for (int j = 0; j < nh; ++j) {
        double s = 0.;
#pragma unroll
        for (int e = 0; e < K1; ++e) s += Bz[e] * Yr(pci, 3 + j)[loff<2, K1>(l, e)];
        hv[j] = s;
      }
    }
    wave_sync();
  };

  // ---------------- phase A: state at this lane's quadrature point
  double u[3] = {0., 0., 0.}, gu[3][3] = {}, lu[3] = {0., 0., 0.};
#pragma unroll
  for (int c = 0; c < 3; ++c) vel_field(c, u[c], gu[c], lu[c]);
  double pq = 0., gp[3] = {0., 0., 0.}, Hq[3] = {0., 0., 0.};
  scal_fields(3, 3, 4, pq, gp, Hq);

  const double nu = P.nu;
  const double JxW = T.w[qx] * T.w[qy] * T.w[qz] * hx * hy * hz;
  const double hst = P.geo[gcell * 4 + 3];
  const double un2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
  const double u_mag = fmax(sqrt(un2), 1e-12);
  const double t1 = 2. * u_mag / hst, t2 = 4 * nu / (hst * hst);
  const double tau = 1. / sqrt(P.sdt2 + t1 * t1 + 9 * (t2 * t2));
  double f[3] = {0., 0., 0.};
  if (P.force_q && pact) {
#pragma unroll
    for (int c = 0; c < 3; ++c) f[c] = P.force_q[((int64_t)gcell * N3 + q) * 3 + c];
  }
  double Gu[3], R[3], srf[3] = {0., 0., 0.};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    Gu[c] = gu[c][0] * u[0] + gu[c][1] * u[1] + gu[c][2] * u[2];
    R[c] = Gu[c] + gp[c] - nu * lu[c] - f[c];
  }
  if (P.srf) {
    const double *om = P.omega;
    const double xq[3] = {P.x0[gcell * 3 + 0] + hx * T.xi[qx], P.x0[gcell * 3 + 1] + hy * T.xi[qy],
                          P.x0[gcell * 3 + 2] + hz * T.xi[qz]};
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

  double Tc[16];
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
  } else {
    // ---------------- phase B: the trial function v at this lane's quadrature point
    double v[3] = {0., 0., 0.}, gv[3][3] = {}, lv[3] = {0., 0., 0.};
#pragma unroll
    for (int c = 0; c < 3; ++c) vel_field(7 + c, v[c], gv[c], lv[c]);
    double vp = 0., gvp[3] = {0., 0., 0.}, dummy[3];
    scal_fields(10, 0, 0, vp, gvp, dummy);
    const double aj = P.alpha_jac;
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
        Tc[4 * c + 1 + e] = JxW * (nu * gv[c][e] - (c == e ? vp : 0.0) + tau * S[c] * u[e] + tau * R[c] * v[e]) * ih[e];
    }
    Tc[12] = JxW * divv;
#pragma unroll
    for (int e = 0; e < 3; ++e) Tc[13 + e] = JxW * tau * S[e] * ih[e];
  }

  // ---------------- integration, one test field at a time (wave-local)
#pragma unroll
  for (int fld = 0; fld < 4; ++fld) {
    if (pact) {
      X(pci, 0)[q] = Tc[4 * fld];
      X(pci, 1)[q] = Tc[4 * fld + 1];
      X(pci, 2)[q] = Tc[4 * fld + 2];
      X(pci, 3)[q] = Tc[4 * fld + 3];
    }
    wave_sync();
    // transposed z: Z0 = B^T Tv + D^T Tz -> Y0; Z1 = B^T Tx -> Y1; Z2 = B^T Ty -> Y2
    for (int t = lane; t < CPW * L2 * 3; t += 64) {
      const int ci = cbase + t / (L2 * 3), r = t % (L2 * 3), l = r / 3, m = r % 3;
      double a[K1], o[K1];
      const double *s = X(ci, m == 0 ? 0 : m);
#pragma unroll
      for (int e = 0; e < K1; ++e) a[e] = s[loff<2, K1>(l, e)];
      bwd<K1>(T.V, a, o);
      if (m == 0) {
        const double *s3 = X(ci, 3);
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = s3[loff<2, K1>(l, e)];
        bwd_add<K1>(T.D, a, o);
      }
      double *d = Yr(ci, m);
#pragma unroll
      for (int e = 0; e < K1; ++e) d[loff<2, K1>(l, e)] = o[e];
    }
    wave_sync();
    // transposed y: W0 = B^T Z0 + D^T Z2 -> X0; W1 = B^T Z1 -> X1
    for (int t = lane; t < CPW * L2 * 2; t += 64) {
      const int ci = cbase + t / (L2 * 2), r = t % (L2 * 2), l = r / 2, m = r % 2;
      double a[K1], o[K1];
      const double *s = Yr(ci, m);
#pragma unroll
      for (int e = 0; e < K1; ++e) a[e] = s[loff<1, K1>(l, e)];
      bwd<K1>(T.V, a, o);
      if (m == 0) {
        const double *s2 = Yr(ci, 2);
#pragma unroll
        for (int e = 0; e < K1; ++e) a[e] = s2[loff<1, K1>(l, e)];
        bwd_add<K1>(T.D, a, o);
      }
      double *d = X(ci, m);
#pragma unroll
      for (int e = 0; e < K1; ++e) d[loff<1, K1>(l, e)] = o[e];
    }
    wave_sync();
    // transposed x: out = B^T W0 + D^T W1 (node-indexed)
    for (int t = lane; t < CPW * L2; t += 64) {
      const int ci = cbase + t / L2, l = t % L2;
      double a[K1], o[K1];
      const double *s0 = X(ci, 0), *s1 = X(ci, 1);
#pragma unroll
      for (int e = 0; e < K1; ++e) a[e] = s0[loff<0, K1>(l, e)];
      bwd<K1>(T.V, a, o);
#pragma unroll
      for (int e = 0; e < K1; ++e) a[e] = s1[loff<0, K1>(l, e)];
      bwd_add<K1>(T.D, a, o);
      double *d = Out(ci, fld);
#pragma unroll
      for (int e = 0; e < K1; ++e) d[loff<0, K1>(l, e)] = o[e];
    }
    wave_sync();
  }
  __syncthreads();

  // ---------------- brick reduction (fixed order) + scatter
  for (int t = tid; t < BN3 * 4; t += blockDim.x) {
    const int n = t >> 2, fld = t & 3;
    const int Xn = n % BN, Yn = (n / BN) % BN, Zn = n / (BN * BN);
    double s = 0.;
#pragma unroll
    for (int cz = 0; cz < 2; ++cz) {
      const int az = Zn - K * cz;
      if (az < 0 || az > K) continue;
#pragma unroll
      for (int cy = 0; cy < 2; ++cy) {
        const int ay = Yn - K * cy;
        if (ay < 0 || ay > K) continue;
#pragma unroll
        for (int cx = 0; cx < 2; ++cx) {
          const int ax = Xn - K * cx;
          if (ax < 0 || ax > K) continue;
          s += Out(cx + 2 * cy + 4 * cz, fld)[ax + K1 * (ay + K1 * az)];
        }
      }
    }
    const int node = sNode[n];
    const int64_t gi = fld < 3 ? (int64_t)node * 3 + fld : voff + node;
    const bool interior = Xn > 0 && Xn < BN - 1 && Yn > 0 && Yn < BN - 1 && Zn > 0 && Zn < BN - 1;
    if (interior) P.y[gi] = s;
    else atomicAdd(&P.y[gi], s);
  }
}

template <int K>
size_t brick_lds_bytes(int mode) {
  using C = BrickCfg<K>;
  const int NF = mode == MODE_JV ? 11 : 7;
  return sizeof(double) * ((size_t)NF * C::BN3 + (size_t)8 * C::PER_CELL * C::N3) + sizeof(int) * (size_t)C::BN3;
}

template <int K>
hipError_t launch_brick_t(int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  using C = BrickCfg<K>;
  const int n_bricks = P.n_cells / 8;
  if (n_bricks <= 0) return hipSuccess;
  const size_t lds = brick_lds_bytes<K>(mode);
  if (mode == MODE_JV)
    hipLaunchKernelGGL((gls_brick_kernel<K, MODE_JV>), dim3(n_bricks), dim3(C::THREADS), lds, s, P, T);
  else
    hipLaunchKernelGGL((gls_brick_kernel<K, MODE_RESIDUAL>), dim3(n_bricks), dim3(C::THREADS), lds, s, P, T);
  return hipGetLastError();
}

hipError_t launch_brick_kernel(int k, int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (mode == MODE_DIAG) return hipErrorNotSupported;
  if (k == 1) return launch_brick_t<1>(mode, P, T, s);
  if (k == 2) return launch_brick_t<2>(mode, P, T, s);
  return hipErrorNotSupported;
}

}  // namespace gls
