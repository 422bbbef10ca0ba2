// gls_brick_jvq.hip — J.v from the cached linearization (MODE_JVQ) on 2x2x2 Morton bricks, with
// the sum-factorized sweeps of two fields interleaved per stage.
//
// Same arithmetic as gls_brick_kernels.hip's MODE_JVQ (gls_navier_stokes.cc:519-625 as a matrix-free
// action), re-scheduled for latency: the per-field pipeline there runs
// 4 trial + 4 test fields x 3 dependent LDS stages = 28 wave-syncs per cell pair, each exposing an
// LDS round trip with one chain in flight. Here two fields share every stage (two independent
// chains per wave, half the round trips):
//   trial : X(v0,v1) | Y(v0,v1) | Z(v0,v1) + X(v2,p) | Y(v2,p) | Z(v2,p)             5 stages
//   test  : W(0,1) | Z(0,1) | Y(0,1) | X(0,1) + W(2,3) | Z(2,3) | Y(2,3) | X(2,3)    7 stages
// in two ping-pong LDS regions of 8 arrays per cell (R0, R1). A cell's node contributions go into
// the brick accumulator with LDS float atomics (no per-cell output arrays, no reduction pass); the
// brick's sums leave as plain stores (interior nodes) and slab stores (surface nodes, summed per
// node by k_slab_sum) — deterministic, no global atomics.
// One workgroup = one brick = 4 waves x 2 cells (lane <-> (cell, q), 54 of 64 lanes for Q2).
// Real = double: the outer GMRES operator; Real = float: the mixed-precision V-cycle's smoother.
#include "gls_common.hpp"
#include "gls_launch.hpp"

#include <type_traits>

namespace gls {
namespace {

template <int K>
struct JCfg {
  static constexpr int K1 = K + 1;
  static constexpr int N3 = K1 * K1 * K1;
  static constexpr int BN = 2 * K + 1;
  static constexpr int BN3 = BN * BN * BN;
  static constexpr int NBND = BN3 - (BN - 2) * (BN - 2) * (BN - 2);
  static constexpr int CPW = 2;             // cells per wave
  static constexpr int WAVES = 8 / CPW;
  static constexpr int QW = CPW * N3;       // active lanes
  static constexpr int NR = 8;              // arrays per ping-pong region
};
constexpr int kTab = 5 * 16 + 8;

template <int K, typename Real>
constexpr size_t jvq_lds_bytes() {
  using C = JCfg<K>;
  return sizeof(Real) * ((size_t)kTab + 4 * C::BN3 + 4 * C::BN3 + (size_t)8 * 2 * C::NR * C::N3) +
         sizeof(int) * C::BN3;
}

__device__ __forceinline__ void wsync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <int BN>
__device__ __forceinline__ int surf_rank(int X, int Y, int Z) {
  constexpr int I = BN - 2;
  const int n = X + BN * (Y + BN * Z);
  int before = min(max(Z - 1, 0), I) * I * I;
  if (Z >= 1 && Z <= I) {
    before += min(max(Y - 1, 0), I) * I;
    if (Y >= 1 && Y <= I) before += min(max(X - 1, 0), I);
  }
  return n - before;
}

__device__ __forceinline__ int swz(int orig, int n) {
  const int q = n / 8, r = n % 8, x = orig % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8;
}

template <int K, typename Real>
__global__ void __launch_bounds__(64 * JCfg<K>::WAVES, 4) gls_brick_jvq_kernel(const OpParams P, const Tables1D T) {
  using C = JCfg<K>;
  constexpr int K1 = C::K1, N3 = C::N3, BN = C::BN, BN3 = C::BN3, QW = C::QW, NR = C::NR;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Real *const sM = reinterpret_cast<Real *>(smem_raw);
  Real *const sB = sM + kTab;          // [4][BN3] v0 v1 v2 vp
  Real *const sAcc = sB + 4 * BN3;     // [4][BN3]
  Real *const sC = sAcc + 4 * BN3;     // [8 cells][2 regions][NR][N3]
  int *const sNode = reinterpret_cast<int *>(sC + 8 * 2 * NR * N3);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_bricks = P.n_cells / 8;
  const int brick = swz((int)blockIdx.x, n_bricks);
  const int64_t voff = (int64_t)3 * P.n_vnodes;

  if (tid < 5 * 16) {
    const int mat = tid >> 4, r = (tid >> 2) & 3, c = tid & 3;
    double v = 0.;
    if (r < K1 && c < K1) {
      if (mat == 0) v = T.V[r][c];
      else if (mat == 1) v = T.D[r][c];
      else if (mat == 2) v = T.S[r][c];
      else if (mat == 3) v = T.V[c][r];
      else v = T.D[c][r];
    }
    sM[tid] = (Real)v;
  } else if (tid < kTab) {
    const int j = (tid - 80) & 3;
    sM[tid] = (Real)(j < K1 ? (tid < 84 ? T.w[j] : T.xi[j]) : 0.0);
  }
  for (int t = tid; t < 4 * BN3; t += blockDim.x) sAcc[t] = Real(0);
  // ---------------- gather v (masked by zero_constraints) at the brick's nodes
  for (int n = tid; n < BN3; n += blockDim.x) {
    const int Xn = n % BN, Yn = (n / BN) % BN, Zn = n / (BN * BN);
    const int cx = min(Xn / K, 1), cy = min(Yn / K, 1), cz = min(Zn / K, 1);
    const int a = (Xn - K * cx) + K1 * ((Yn - K * cy) + K1 * (Zn - K * cz));
    const int node = P.cell_vnodes[((int64_t)brick * 8 + cx + 2 * cy + 4 * cz) * N3 + a];
    const int64_t i3 = (int64_t)node * 3;
    const unsigned m = P.vmask ? P.vmask[node] : 0u;
    const double v0 = P.v[i3], v1 = P.v[i3 + 1], v2 = P.v[i3 + 2], vp = P.v[voff + node];
    sNode[n] = node;
    sB[n] = (m & 1u) ? Real(0) : (Real)v0;
    sB[BN3 + n] = (m & 2u) ? Real(0) : (Real)v1;
    sB[2 * BN3 + n] = (m & 4u) ? Real(0) : (Real)v2;
    sB[3 * BN3 + n] = (Real)vp;
  }
  __syncthreads();

  // ---------------- per wave: cells 2*wave, 2*wave+1; lane <-> (cell, q)
  const bool pact = lane < QW;
  const int lc = pact ? lane / N3 : 0;
  const int pci = wave * C::CPW + lc;
  const int q = pact ? lane % N3 : 0;
  const int i0 = q % K1, i1 = (q / K1) % K1, i2 = q / (K1 * K1), me = q;
  const int cxb = pci & 1, cyb = (pci >> 1) & 1, czb = pci >> 2;
  const int bx_base = K * cxb + BN * (K * cyb + i1) + BN * BN * (K * czb + i2);
  const int bn_me = (K * cxb + i0) + BN * ((K * cyb + i1) + BN * (K * czb + i2));
  const int gcell = brick * 8 + pci;
  const Real hx = (Real)P.geo[gcell * 4 + 0], hy = (Real)P.geo[gcell * 4 + 1], hz = (Real)P.geo[gcell * 4 + 2];
  const Real ih[3] = {Real(1) / hx, Real(1) / hy, Real(1) / hz};
  const Real JxW = sM[80 + i0] * sM[80 + i1] * sM[80 + i2] * hx * hy * hz;
  const Real nu = (Real)P.nu;
  Real *const R0 = sC + (pci * 2 + 0) * NR * N3;
  Real *const R1 = sC + (pci * 2 + 1) * NR * N3;
  auto A0 = [&](int s) { return R0 + s * N3; };
  auto A1 = [&](int s) { return R1 + s * N3; };
  auto row = [&](int mat, int r, Real (&o)[K1]) {
    const Real *m = sM + mat * 16 + r * 4;
#pragma unroll
    for (int k = 0; k < K1; ++k) o[k] = m[k];
  };
  auto dot = [&](const Real (&a)[K1], const Real (&b)[K1]) {
    Real s = 0;
#pragma unroll
    for (int k = 0; k < K1; ++k) s += a[k] * b[k];
    return s;
  };
  auto line0 = [&](const Real *A, Real (&o)[K1]) {
#pragma unroll
    for (int e = 0; e < K1; ++e) o[e] = A[e + K1 * (i1 + K1 * i2)];
  };
  auto line1 = [&](const Real *A, Real (&o)[K1]) {
#pragma unroll
    for (int e = 0; e < K1; ++e) o[e] = A[i0 + K1 * (e + K1 * i2)];
  };
  auto line2 = [&](const Real *A, Real (&o)[K1]) {
#pragma unroll
    for (int e = 0; e < K1; ++e) o[e] = A[i0 + K1 * (i1 + K1 * e)];
  };
  // trial stages; velocity field: X -> 3 arrays (B, D, S), Y -> 4 (BB, BD, DB, L); pressure: 2, 3
  auto xvel = [&](int f, Real *o) {  // o[0..2]
    Real in[K1], r[K1];
#pragma unroll
    for (int e = 0; e < K1; ++e) in[e] = sB[f * BN3 + bx_base + e];
    row(0, i0, r);
    o[0 * N3 + me] = dot(r, in);
    row(1, i0, r);
    o[1 * N3 + me] = dot(r, in);
    row(2, i0, r);
    o[2 * N3 + me] = dot(r, in);
  };
  auto xpre = [&](Real *o) {  // o[0..1]
    Real in[K1], r[K1];
#pragma unroll
    for (int e = 0; e < K1; ++e) in[e] = sB[3 * BN3 + bx_base + e];
    row(0, i0, r);
    o[0 * N3 + me] = dot(r, in);
    row(1, i0, r);
    o[1 * N3 + me] = dot(r, in);
  };
  auto yvel = [&](const Real *x, Real *o) {  // x[0..2] -> o[0..3]
    Real xb[K1], xd[K1], xs[K1], rb[K1], rd[K1], rs[K1];
    line1(x, xb);
    line1(x + N3, xd);
    line1(x + 2 * N3, xs);
    row(0, i1, rb);
    row(1, i1, rd);
    row(2, i1, rs);
    o[0 * N3 + me] = dot(rb, xb);
    o[1 * N3 + me] = dot(rd, xb);
    o[2 * N3 + me] = dot(rb, xd);
    o[3 * N3 + me] = ih[1] * ih[1] * dot(rs, xb) + ih[0] * ih[0] * dot(rb, xs);
  };
  auto ypre = [&](const Real *x, Real *o) {  // x[0..1] -> o[0..2]
    Real a[K1], rb[K1], rd[K1];
    row(0, i1, rb);
    row(1, i1, rd);
    line1(x, a);
    o[0 * N3 + me] = dot(rb, a);
    o[1 * N3 + me] = dot(rd, a);
    line1(x + N3, a);
    o[2 * N3 + me] = dot(rb, a);
  };
  Real Bz[K1], Dz[K1], Sz[K1];
  row(0, i2, Bz);
  row(1, i2, Dz);
  row(2, i2, Sz);
  auto zvel = [&](const Real *y, Real &val, Real (&g)[3], Real &lap) {
    Real bb[K1], bd[K1], db[K1], ll[K1];
    line2(y, bb);
    line2(y + N3, bd);
    line2(y + 2 * N3, db);
    line2(y + 3 * N3, ll);
    val = dot(Bz, bb);
    g[0] = dot(Bz, db) * ih[0];
    g[1] = dot(Bz, bd) * ih[1];
    g[2] = dot(Dz, bb) * ih[2];
    lap = dot(Bz, ll) + ih[2] * ih[2] * dot(Sz, bb);
  };
  auto zpre = [&](const Real *y, Real &pv, Real (&pg)[3]) {
    Real bb[K1], bd[K1], db[K1];
    line2(y, bb);
    line2(y + N3, bd);
    line2(y + 2 * N3, db);
    pv = dot(Bz, bb);
    pg[0] = dot(Bz, db) * ih[0];
    pg[1] = dot(Bz, bd) * ih[1];
    pg[2] = dot(Dz, bb) * ih[2];
  };

  Real v[3] = {0, 0, 0}, gv[3][3] = {}, lv[3] = {0, 0, 0}, vp = 0, gvp[3] = {0, 0, 0};
  // trial stage 1: X(v0), X(v1) -> R0[0..5]
  if (pact) { xvel(0, A0(0)); xvel(1, A0(3)); }
  wsync();
  // stage 2: Y(v0), Y(v1) -> R1[0..7]
  if (pact) { yvel(A0(0), A1(0)); yvel(A0(3), A1(4)); }
  wsync();
  // stage 3: Z(v0), Z(v1) from R1; X(v2) -> R0[0..2], X(p) -> R0[3..4]
  if (pact) {
    zvel(A1(0), v[0], gv[0], lv[0]);
    zvel(A1(4), v[1], gv[1], lv[1]);
    xvel(2, A0(0));
    xpre(A0(3));
  }
  wsync();
  // stage 4: Y(v2) -> R1[0..3], Y(p) -> R1[4..6]
  if (pact) { yvel(A0(0), A1(0)); ypre(A0(3), A1(4)); }
  wsync();
  // linearization at this q (u, grad u, tau, R_s), streamed once per call
  Real u[3] = {0, 0, 0}, gu[3][3] = {}, R[3] = {0, 0, 0}, tau = 0;
  const Real *qdw = nullptr;
  if constexpr (std::is_same<Real, double>::value) qdw = P.qd + ((int64_t)brick * C::WAVES + wave) * kQData * QW + lane;
  else qdw = P.qdf + ((int64_t)brick * C::WAVES + wave) * kQData * QW + lane;
  if (pact) {
#pragma unroll
    for (int c = 0; c < 3; ++c) u[c] = __builtin_nontemporal_load(qdw + c * QW);
#pragma unroll
    for (int c = 0; c < 9; ++c) gu[c / 3][c % 3] = __builtin_nontemporal_load(qdw + (3 + c) * QW);
    tau = __builtin_nontemporal_load(qdw + 12 * QW);
#pragma unroll
    for (int c = 0; c < 3; ++c) R[c] = __builtin_nontemporal_load(qdw + (13 + c) * QW);
  }
  // stage 5: Z(v2), Z(p) from R1
  if (pact) {
    zvel(A1(0), v[2], gv[2], lv[2]);
    zpre(A1(4), vp, gvp);
  }

  // ---------------- pointwise (gls_navier_stokes.cc:525-606 applied to v)
  Real Tc[16];
  {
    const Real aj = (Real)P.alpha_jac;
    Real S[3], A[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const Real guv = gu[c][0] * v[0] + gu[c][1] * v[1] + gu[c][2] * v[2];
      const Real gvu = gv[c][0] * u[0] + gv[c][1] * u[1] + gv[c][2] * u[2];
      A[c] = guv + gvu + aj * v[c];
      S[c] = guv + gvu + gvp[c] - nu * lv[c] + aj * v[c];
    }
    if (P.srf) {
      const Real om[3] = {(Real)P.omega[0], (Real)P.omega[1], (Real)P.omega[2]};
      const Real cj[3] = {2 * (om[1] * v[2] - om[2] * v[1]), 2 * (om[2] * v[0] - om[0] * v[2]),
                          2 * (om[0] * v[1] - om[1] * v[0])};
#pragma unroll
      for (int c = 0; c < 3; ++c) { A[c] += cj[c]; S[c] += cj[c]; }
    }
    const Real divv = gv[0][0] + gv[1][1] + gv[2][2];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      Tc[4 * c] = JxW * A[c];
#pragma unroll
      for (int e = 0; e < 3; ++e)
        Tc[4 * c + 1 + e] =
            JxW * (nu * gv[c][e] - (c == e ? vp : Real(0)) + tau * S[c] * u[e] + tau * R[c] * v[e]) * ih[e];
    }
    Tc[12] = JxW * divv;
#pragma unroll
    for (int e = 0; e < 3; ++e) Tc[13 + e] = JxW * tau * S[e] * ih[e];
  }

  // ---------------- test integration, two test fields per stage
  Real cb2[K1], cd2[K1], cb1[K1], cd1[K1], cb0[K1], cd0[K1];
  row(3, i2, cb2);
  row(4, i2, cd2);
  row(3, i1, cb1);
  row(4, i1, cd1);
  row(3, i0, cb0);
  row(4, i0, cd0);
  auto tz = [&](const Real *w, Real *o) {  // w[0..3] (value, x, y, z coefficients) -> o[0..2]
    Real tv[K1], tx[K1], ty[K1], tzz[K1];
    line2(w, tv);
    line2(w + N3, tx);
    line2(w + 2 * N3, ty);
    line2(w + 3 * N3, tzz);
    o[0 * N3 + me] = dot(cb2, tv) + dot(cd2, tzz);
    o[1 * N3 + me] = dot(cb2, tx);
    o[2 * N3 + me] = dot(cb2, ty);
  };
  auto ty_ = [&](const Real *z, Real *o) {  // z[0..2] -> o[0..1]
    Real z0[K1], z1[K1], z2[K1];
    line1(z, z0);
    line1(z + N3, z1);
    line1(z + 2 * N3, z2);
    o[0 * N3 + me] = dot(cb1, z0) + dot(cd1, z2);
    o[1 * N3 + me] = dot(cb1, z1);
  };
  auto tx_ = [&](const Real *y, int fld) {  // y[0..1] -> brick accumulator
    Real w0[K1], w1[K1];
    line0(y, w0);
    line0(y + N3, w1);
    atomicAdd(&sAcc[fld * BN3 + bn_me], dot(cb0, w0) + dot(cd0, w1));
  };
  auto wr = [&](int fld, Real *o) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j * N3 + me] = Tc[4 * fld + j];
  };
  wsync();  // R0 (stage-4 reads) and R1 (stage-5 reads) are free from here on
  if (pact) { wr(0, A0(0)); wr(1, A0(4)); }                      // W(0,1) -> R0
  wsync();
  if (pact) { tz(A0(0), A1(0)); tz(A0(4), A1(3)); }              // Z(0,1) -> R1[0..5]
  wsync();
  if (pact) { ty_(A1(0), A0(0)); ty_(A1(3), A0(2)); }            // Y(0,1) -> R0[0..3]
  wsync();
  if (pact) { tx_(A0(0), 0); tx_(A0(2), 1); wr(2, A1(0)); wr(3, A1(4)); }  // X(0,1); W(2,3) -> R1
  wsync();
  if (pact) { tz(A1(0), A0(0)); tz(A1(4), A0(3)); }              // Z(2,3) -> R0[0..5]
  wsync();
  if (pact) { ty_(A0(0), A1(0)); ty_(A0(3), A1(2)); }            // Y(2,3) -> R1[0..3]
  wsync();
  if (pact) { tx_(A1(0), 2); tx_(A1(2), 3); }                    // X(2,3)
  __syncthreads();

  // ---------------- brick sums -> HBM (interior: plain stores; surface: slab)
  for (int t = tid; t < 4 * BN3; t += blockDim.x) {
    const int n = t >> 2, fld = t & 3;
    const Real s = sAcc[fld * BN3 + n];
    const int Xn = n % BN, Yn = (n / BN) % BN, Zn = n / (BN * BN);
    const int node = sNode[n];
    const int64_t gi = fld < 3 ? (int64_t)node * 3 + fld : voff + node;
    const bool interior = Xn > 0 && Xn < BN - 1 && Yn > 0 && Yn < BN - 1 && Zn > 0 && Zn < BN - 1;
    if (interior) P.y[gi] = (double)s;
    else if (P.slab) P.slab[((int64_t)brick * C::NBND + surf_rank<BN>(Xn, Yn, Zn)) * 4 + fld] = (double)s;
    else atomicAdd(&P.y[gi], (double)s);
  }
}

template <int K, typename Real>
hipError_t launch_jvq_t(const OpParams &P, const Tables1D &T, hipStream_t s) {
  const int n_bricks = P.n_cells / 8;
  if (n_bricks <= 0) return hipSuccess;
  constexpr size_t lds = jvq_lds_bytes<K, Real>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(gls_brick_jvq_kernel<K, Real>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((gls_brick_jvq_kernel<K, Real>), dim3(n_bricks), dim3(64 * JCfg<K>::WAVES), lds, s, P, T);
  return hipGetLastError();
}

}  // namespace

// J.v (MODE_JVQ, no probing) with the interleaved-stage kernel; Real = double reads P.qd, float P.qdf
// (same wave-major layout as gls_brick_kernels.hip: [brick][wave][kQData][2 cells x N3])
hipError_t launch_brick_jvq2(int k, bool f32, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (P.n_probe > 0) return hipErrorInvalidValue;
  if (k == 2) return f32 ? launch_jvq_t<2, float>(P, T, s) : launch_jvq_t<2, double>(P, T, s);
  return hipErrorNotSupported;
}

}  // namespace gls
