// gls_brick_wave.hip — persistent wave-per-brick GLS operators (3D Qk-Qk, k = 1, 2).
//
// Same arithmetic as gls_brick_kernels.hip (sum-factorized sweeps on 2x2x2 Morton bricks, the
// pointwise algebra of gls_navier_stokes.cc:387-748), re-cut for latency hiding on gfx950:
//
//   * one WAVE owns a whole brick at a time and walks a contiguous range of bricks (persistent
//     grid, XCD-contiguous ranges so neighbouring bricks share an L2). No workgroup barrier
//     after the one-time table load: a wave never waits for another wave, and the other waves on
//     the SIMD cover its gather and LDS latencies.
//   * per brick: gather the (2k+1)^3 brick nodes into the wave's LDS (all 64 lanes, loads issued
//     together), then ROUNDS rounds of CPR cells (Q2: 4 rounds of 2 cells = 54 of 64 lanes,
//     lane <-> (cell, q); Q1: 1 round of 8 cells = 64 lanes), each running the x / y / z sweeps,
//     the pointwise GLS algebra and the transposed sweeps wave-locally (in-order LDS);
//   * a cell's node contributions are added into the wave's brick accumulator with LDS float
//     atomics (ds_add), so no per-cell output arrays and no reduction pass; the brick's sums go out
//     as plain stores (brick-interior nodes) and slab stores (surface nodes, summed per node by
//     k_slab_sum in a fixed order) — no global atomics except in probing mode;
//   * setup (tables, lane <-> (cell, q) indices, z-matrix rows) once per wave, not per brick.
#include "gls_common.hpp"
#include "gls_launch.hpp"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>

namespace gls {
namespace {

template <int K>
struct WaveCfg {
  static constexpr int K1 = K + 1;
  static constexpr int N3 = K1 * K1 * K1;
  static constexpr int BN = 2 * K + 1;
  static constexpr int BN3 = BN * BN * BN;
  static constexpr int NBND = BN3 - (BN - 2) * (BN - 2) * (BN - 2);
  static constexpr int CPR = 64 / N3 >= 8 ? 8 : (64 / N3 >= 2 ? 2 : 1);  // cells per round
  static constexpr int ROUNDS = 8 / CPR;
  static constexpr int QW = CPR * N3;        // active lanes per round
  static constexpr int GS = (BN3 + 63) / 64;  // gather slots per lane
  static constexpr int NX = 5, NY = 6;       // per-cell LDS scratch arrays
};

constexpr int kWaves = 4;  // waves per workgroup (independent after the table load)

template <int MODE>
constexpr int n_fields() { return MODE == MODE_JVQ ? 4 : (MODE == MODE_JV ? 11 : 7); }

// A brick is owned by a group of WPB waves (1: a wave walks bricks alone, no barriers; 4: the
// workgroup shares the brick, each wave runs ROUNDS/4 rounds, three barriers per brick).
// LDS: tables | per group: brick fields [NF][BN3], accumulator [4][BN3], geometry [8][4] |
//      per wave: cell scratch [CPR][NX+NY][N3] | per group: brick node ids [BN3] (int)
template <int K, int MODE>
constexpr int group_reals() { return n_fields<MODE>() * WaveCfg<K>::BN3 + 4 * WaveCfg<K>::BN3 + 8 * 4; }
template <int K>
constexpr int scratch_reals() { return WaveCfg<K>::CPR * (WaveCfg<K>::NX + WaveCfg<K>::NY) * WaveCfg<K>::N3; }
constexpr int kTableReals = 5 * 16 + 8;

template <int K, int MODE, int WPB, typename Real>
constexpr size_t wave_lds_bytes() {
  constexpr int NG = kWaves / WPB;
  return sizeof(Real) * ((size_t)kTableReals + (size_t)NG * group_reals<K, MODE>() + (size_t)kWaves * scratch_reals<K>()) +
         sizeof(int) * (size_t)NG * WaveCfg<K>::BN3;
}

__device__ __forceinline__ void wsync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <typename Real>
__device__ __forceinline__ Real recip(Real h) {
  if constexpr (std::is_same<Real, double>::value) {
    double r = __builtin_amdgcn_rcp(h);  // v_rcp_f64, refined by two Newton steps (<= 1 ulp)
    r = fma(r, fma(-h, r, 1.0), r);
    r = fma(r, fma(-h, r, 1.0), r);
    return r;
  } else {
    return 1.0f / h;
  }
}

template <int BN>
__device__ __forceinline__ int bnd_rank(int X, int Y, int Z) {
  constexpr int I = BN - 2;
  const int n = X + BN * (Y + BN * Z);
  int before = min(max(Z - 1, 0), I) * I * I;
  if (Z >= 1 && Z <= I) {
    before += min(max(Y - 1, 0), I) * I;
    if (Y >= 1 && Y <= I) before += min(max(X - 1, 0), I);
  }
  return n - before;
}

template <int K, int MODE, int WPB, typename Real>
__global__ void __launch_bounds__(64 * kWaves, (sizeof(Real) == 8 && WPB == 1) ? 3 : 4)
    gls_brick_wave_kernel(const OpParams P, const Tables1D T) {
  using C = WaveCfg<K>;
  static_assert(WPB == 1 || WPB == kWaves, "a brick is owned by one wave or by the whole workgroup");
  static_assert(C::ROUNDS % WPB == 0, "rounds must split evenly over the brick's waves");
  constexpr int NGRP = kWaves / WPB, GT = 64 * WPB;  // groups per workgroup, threads per group
  constexpr int GS = (C::BN3 + GT - 1) / GT;         // gather slots per thread
  constexpr int K1 = C::K1, N3 = C::N3, BN = C::BN, BN3 = C::BN3, CPR = C::CPR, QW = C::QW;
  constexpr bool JV = MODE == MODE_JV || MODE == MODE_JVQ;
  constexpr bool CACHED = MODE == MODE_JVQ;
  constexpr bool LIN = MODE == MODE_LIN;
  constexpr int NF = n_fields<MODE>();
  constexpr int FV = CACHED ? 0 : 7;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Real *const sM = reinterpret_cast<Real *>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: item math in SGPRs
  const int grpw = wave / WPB, sub = wave % WPB, gtid = sub * 64 + lane;
  Real *const gbase = sM + kTableReals + grpw * group_reals<K, MODE>();
  Real *const sB = gbase;                   // [NF][BN3]
  Real *const sAcc = sB + NF * BN3;         // [4][BN3]
  Real *const sGeo = sAcc + 4 * BN3;        // [8][4]
  Real *const sC = sM + kTableReals + NGRP * group_reals<K, MODE>() + wave * scratch_reals<K>();  // [CPR][NX+NY][N3]
  int *const sNode = reinterpret_cast<int *>(sM + kTableReals + NGRP * group_reals<K, MODE>() + kWaves * scratch_reals<K>()) +
                     grpw * BN3;
  auto gsync = [&]() {
    if constexpr (WPB > 1) __syncthreads();
    else wsync();
  };
  auto BF = [&](int f) { return sB + f * BN3; };

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
  } else if (tid < kTableReals) {
    const int j = (tid - 80) & 3;
    sM[tid] = (Real)(j < K1 ? (tid < 84 ? T.w[j] : T.xi[j]) : 0.0);
  }
  for (int t = gtid; t < 4 * BN3; t += GT) sAcc[t] = Real(0);
  __syncthreads();  // tables visible to every wave (WPB == 1: the only workgroup barrier)

  // ---- this wave's range of work items (item = probe column x brick), XCD-contiguous
  const int n_bricks = P.n_cells / 8;
  const bool probing = CACHED && P.n_probe > 0;
  const int64_t n_items = (int64_t)n_bricks * (probing ? P.n_probe : 1);
  const int G = gridDim.x;                 // multiple of 8 (host)
  const int grp = blockIdx.x % 8, slot = blockIdx.x / 8;
  const int64_t glo = n_items * grp / 8, ghi = n_items * (grp + 1) / 8;
  const int64_t W = (int64_t)(G / 8) * NGRP, w = (int64_t)slot * NGRP + grpw;
  const int64_t ilo = glo + (ghi - glo) * w / W, ihi = glo + (ghi - glo) * (w + 1) / W;
  const int64_t voff = (int64_t)3 * P.n_vnodes;
  const int64_t ndofs = voff + P.n_vnodes;
  const bool use_slab = P.slab != nullptr && !probing;

  // ---- per-lane constants (once per wave)
  const bool pact = lane < QW;
  const int lc = pact ? lane / N3 : 0;  // cell slot within the round
  const int q = pact ? lane % N3 : 0;
  const int qx = q % K1, qy = (q / K1) % K1, qz = q / (K1 * K1);
  const int i0 = qx, i1 = qy, i2 = qz, me = q;
  Real Bz[K1], Dz[K1], Sz[K1];
#pragma unroll
  for (int i = 0; i < K1; ++i) { Bz[i] = sM[qz * 4 + i]; Dz[i] = sM[16 + qz * 4 + i]; Sz[i] = sM[32 + qz * 4 + i]; }
  const Real wq = sM[80 + qx] * sM[80 + qy] * sM[80 + qz];
  const Real nu = (Real)P.nu;

  auto X = [&](int s) { return sC + (lc * (C::NX + C::NY) + s) * N3; };
  auto Yr = [&](int s) { return sC + (lc * (C::NX + C::NY) + C::NX + s) * N3; };
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
  auto lineD0 = [&](const Real *A, Real (&o)[K1]) {
#pragma unroll
    for (int e = 0; e < K1; ++e) o[e] = A[e + K1 * (i1 + K1 * i2)];
  };
  auto lineD1 = [&](const Real *A, Real (&o)[K1]) {
#pragma unroll
    for (int e = 0; e < K1; ++e) o[e] = A[i0 + K1 * (e + K1 * i2)];
  };
  auto lineD2 = [&](const Real *A, Real (&o)[K1]) {
#pragma unroll
    for (int e = 0; e < K1; ++e) o[e] = A[i0 + K1 * (i1 + K1 * e)];
  };

  for (int64_t item = ilo; item < ihi; ++item) {
    const int pj = probing ? (int)(item / n_bricks) : 0;
    const int brick = probing ? (int)(item % n_bricks) : (int)item;
    const int64_t unit_dof = probing ? P.probe_base + pj : -1;
    double *const Yout = probing ? P.y + (int64_t)pj * ndofs : P.y;

    // ---------------- gather the brick (all loads of a lane in flight together)
    {
      int nd[GS];
#pragma unroll
      for (int s = 0; s < GS; ++s) {
        const int n = gtid + GT * s;
        nd[s] = 0;
        if (n < BN3) {
          const int Xn = n % BN, Yn = (n / BN) % BN, Zn = n / (BN * BN);
          const int cx = min(Xn / K, 1), cy = min(Yn / K, 1), cz = min(Zn / K, 1);
          const int a = (Xn - K * cx) + K1 * ((Yn - K * cy) + K1 * (Zn - K * cz));
          nd[s] = P.cell_vnodes[((int64_t)brick * 8 + cx + 2 * cy + 4 * cz) * N3 + a];
        }
      }
      if (gtid < 32) sGeo[gtid] = (Real)P.geo[(int64_t)brick * 32 + gtid];
#pragma unroll
      for (int s = 0; s < GS; ++s) {
        const int n = gtid + GT * s;
        if (n >= BN3) continue;
        const int node = nd[s];
        const int64_t i3 = (int64_t)node * 3;
        sNode[n] = node;
        if constexpr (!CACHED) {
          const double u0 = P.u[i3], u1 = P.u[i3 + 1], u2 = P.u[i3 + 2], up = P.u[voff + node];
          double h[3] = {0., 0., 0.};
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            if (P.n_hist > 0) h[c] += P.alpha[1] * P.h1[i3 + c];
            if (P.n_hist > 1) h[c] += P.alpha[2] * P.h2[i3 + c];
            if (P.n_hist > 2) h[c] += P.alpha[3] * P.h3[i3 + c];
          }
          BF(0)[n] = (Real)u0;
          BF(1)[n] = (Real)u1;
          BF(2)[n] = (Real)u2;
          BF(3)[n] = (Real)up;
          BF(4)[n] = (Real)h[0];
          BF(5)[n] = (Real)h[1];
          BF(6)[n] = (Real)h[2];
        }
        if constexpr (JV) {
          const unsigned m = P.vmask ? P.vmask[node] : 0u;
          double v0, v1, v2, vp;
          if (probing) {
            v0 = i3 == unit_dof ? 1.0 : 0.0;
            v1 = i3 + 1 == unit_dof ? 1.0 : 0.0;
            v2 = i3 + 2 == unit_dof ? 1.0 : 0.0;
            vp = voff + node == unit_dof ? 1.0 : 0.0;
          } else {
            v0 = P.v[i3];
            v1 = P.v[i3 + 1];
            v2 = P.v[i3 + 2];
            vp = P.v[voff + node];
          }
          BF(FV)[n] = (m & 1u) ? Real(0) : (Real)v0;
          BF(FV + 1)[n] = (m & 2u) ? Real(0) : (Real)v1;
          BF(FV + 2)[n] = (m & 4u) ? Real(0) : (Real)v2;
          BF(FV + 3)[n] = (Real)vp;
        }
      }
    }
    gsync();

    const bool integrate = !(LIN && P.y == nullptr);
#pragma unroll 1
    for (int r = sub * (C::ROUNDS / WPB); r < (sub + 1) * (C::ROUNDS / WPB); ++r) {
      const int pci = r * CPR + lc;
      const int cxb = pci & 1, cyb = (pci >> 1) & 1, czb = pci >> 2;
      const int bx_base = K * cxb + BN * (K * cyb + i1) + BN * BN * (K * czb + i2);
      const int bn_me = (K * cxb + i0) + BN * ((K * cyb + i1) + BN * (K * czb + i2));
      const int gcell = brick * 8 + pci;
      const Real hx = sGeo[pci * 4 + 0], hy = sGeo[pci * 4 + 1], hz = sGeo[pci * 4 + 2];
      const Real ih[3] = {recip(hx), recip(hy), recip(hz)};
      const Real wz = ih[2] * ih[2];
      const Real JxW = wq * hx * hy * hz;

      // velocity-type field: value, gradient, Laplacian at this lane's q
      auto vel_field = [&](int f, Real &val, Real (&g)[3], Real &lap) {
        if (pact) {
          Real in[K1], rr[K1];
#pragma unroll
          for (int e = 0; e < K1; ++e) in[e] = BF(f)[bx_base + e];
          row(0, i0, rr);
          X(0)[me] = dot(rr, in);
          row(1, i0, rr);
          X(1)[me] = dot(rr, in);
          row(2, i0, rr);
          X(2)[me] = dot(rr, in);
        }
        wsync();
        if (pact) {
          Real xb[K1], xd[K1], xs[K1], rb[K1], rd[K1], rs[K1];
          lineD1(X(0), xb);
          lineD1(X(1), xd);
          lineD1(X(2), xs);
          row(0, i1, rb);
          row(1, i1, rd);
          row(2, i1, rs);
          Yr(0)[me] = dot(rb, xb);
          Yr(1)[me] = dot(rd, xb);
          Yr(2)[me] = dot(rb, xd);
          Yr(3)[me] = ih[1] * ih[1] * dot(rs, xb) + ih[0] * ih[0] * dot(rb, xs);
        }
        wsync();
        if (pact) {
          Real bb[K1], bd[K1], db[K1], ll[K1];
          lineD2(Yr(0), bb);
          lineD2(Yr(1), bd);
          lineD2(Yr(2), db);
          lineD2(Yr(3), ll);
          val = dot(Bz, bb);
          g[0] = dot(Bz, db) * ih[0];
          g[1] = dot(Bz, bd) * ih[1];
          g[2] = dot(Dz, bb) * ih[2];
          lap = dot(Bz, ll) + wz * dot(Sz, bb);
        }
        wsync();
      };
      // pressure-type field (value, grad) [+ nh value-only fields]
      auto scal_fields = [&](int fp, int nh, int fh0, Real &pv, Real (&pg)[3], Real (&hv)[3]) {
        if (pact) {
          Real in[K1], rb[K1], rd[K1];
          row(0, i0, rb);
          row(1, i0, rd);
#pragma unroll
          for (int e = 0; e < K1; ++e) in[e] = BF(fp)[bx_base + e];
          X(0)[me] = dot(rb, in);
          X(1)[me] = dot(rd, in);
          for (int j = 0; j < nh; ++j) {
#pragma unroll
            for (int e = 0; e < K1; ++e) in[e] = BF(fh0 + j)[bx_base + e];
            X(2 + j)[me] = dot(rb, in);
          }
        }
        wsync();
        if (pact) {
          Real a[K1], rb[K1], rd[K1];
          row(0, i1, rb);
          row(1, i1, rd);
          lineD1(X(0), a);
          Yr(0)[me] = dot(rb, a);
          Yr(1)[me] = dot(rd, a);
          lineD1(X(1), a);
          Yr(2)[me] = dot(rb, a);
          for (int j = 0; j < nh; ++j) {
            lineD1(X(2 + j), a);
            Yr(3 + j)[me] = dot(rb, a);
          }
        }
        wsync();
        if (pact) {
          Real bb[K1], bd[K1], db[K1];
          lineD2(Yr(0), bb);
          lineD2(Yr(1), bd);
          lineD2(Yr(2), db);
          pv = dot(Bz, bb);
          pg[0] = dot(Bz, db) * ih[0];
          pg[1] = dot(Bz, bd) * ih[1];
          pg[2] = dot(Dz, bb) * ih[2];
          for (int j = 0; j < nh; ++j) {
            lineD2(Yr(3 + j), bb);
            hv[j] = dot(Bz, bb);
          }
        }
        wsync();
      };

      // ---------------- phase A: linearization state at this lane's q
      Real u[3] = {0, 0, 0}, gu[3][3] = {}, R[3] = {0, 0, 0}, tau = 0;
      Real pq = 0, f[3] = {0, 0, 0}, Tt[3] = {0, 0, 0}, srf[3] = {0, 0, 0};
      Real *qdw = nullptr;
      if constexpr (std::is_same<Real, double>::value) {
        if (P.qd) qdw = P.qd + ((int64_t)brick * C::ROUNDS + r) * kQData * QW + lane;
      } else {
        if (P.qdf) qdw = P.qdf + ((int64_t)brick * C::ROUNDS + r) * kQData * QW + lane;
      }
      // linearization stream (JVQ), loaded after the v sweeps: short live ranges, no spills
      auto load_qd = [&]() {
        if (pact) {
#pragma unroll
          for (int c = 0; c < 3; ++c) u[c] = __builtin_nontemporal_load(qdw + c * QW);
#pragma unroll
          for (int c = 0; c < 9; ++c) gu[c / 3][c % 3] = __builtin_nontemporal_load(qdw + (3 + c) * QW);
          tau = __builtin_nontemporal_load(qdw + 12 * QW);
#pragma unroll
          for (int c = 0; c < 3; ++c) R[c] = __builtin_nontemporal_load(qdw + (13 + c) * QW);
        }
      };
      if constexpr (!CACHED) {
        Real lu[3] = {0, 0, 0};
#pragma unroll
        for (int c = 0; c < 3; ++c) vel_field(c, u[c], gu[c], lu[c]);
        Real gp[3] = {0, 0, 0}, Hq[3] = {0, 0, 0};
        scal_fields(3, 3, 4, pq, gp, Hq);
        const Real hst = sGeo[pci * 4 + 3];
        const Real un2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
        const Real u_mag = fmax(sqrt(un2), 1e-12);
        const Real t1 = 2. * u_mag / hst, t2 = 4 * nu / (hst * hst);
        tau = 1. / sqrt(P.sdt2 + t1 * t1 + 9 * (t2 * t2));
        if (P.force_q && pact) {
#pragma unroll
          for (int c = 0; c < 3; ++c) f[c] = P.force_q[((int64_t)gcell * N3 + q) * 3 + c];
        }
#pragma unroll
        for (int c = 0; c < 3; ++c)
          R[c] = gu[c][0] * u[0] + gu[c][1] * u[1] + gu[c][2] * u[2] + gp[c] - nu * lu[c] - f[c];
        if (P.srf) {
          const double *om = P.omega;
          const Real xq[3] = {P.x0[gcell * 3 + 0] + hx * sM[84 + qx], P.x0[gcell * 3 + 1] + hy * sM[84 + qy],
                              P.x0[gcell * 3 + 2] + hz * sM[84 + qz]};
          const Real cx_[3] = {om[1] * u[2] - om[2] * u[1], om[2] * u[0] - om[0] * u[2], om[0] * u[1] - om[1] * u[0]};
          const Real ox[3] = {om[1] * xq[2] - om[2] * xq[1], om[2] * xq[0] - om[0] * xq[2],
                              om[0] * xq[1] - om[1] * xq[0]};
          const Real cc[3] = {om[1] * ox[2] - om[2] * ox[1], om[2] * ox[0] - om[0] * ox[2],
                              om[0] * ox[1] - om[1] * ox[0]};
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            srf[c] = 2 * cx_[c] + cc[c];
            R[c] += srf[c];
          }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          Tt[c] = P.alpha[0] * u[c] + Hq[c];
          R[c] += Tt[c];
        }
      }

      if constexpr (LIN) {
        if (pact) {
#pragma unroll
          for (int c = 0; c < 3; ++c) qdw[c * QW] = u[c];
#pragma unroll
          for (int c = 0; c < 9; ++c) qdw[(3 + c) * QW] = gu[c / 3][c % 3];
          qdw[12 * QW] = tau;
#pragma unroll
          for (int c = 0; c < 3; ++c) qdw[(13 + c) * QW] = R[c];
        }
        if (!integrate) continue;  // linearization only (uniform)
        // Jacobian diagonal from the same linearization (gls_navier_stokes.cc:548-622, v = phi_i e_c):
        //   J_ii(c) = sum_q JxW [A phi + nu |grad phi|^2 + tau (A - nu lap phi) a + tau R_c phi d_c phi],
        //   A = (du_c/dx_c + alpha_jac) phi + a, a = u . grad phi;  J_ii(p) = sum_q JxW tau |grad psi|^2,
        // deal.II's |K_e(i,i)| on constrained rows. Lane <-> node i of its cell, loop over q.
        if (pact) {
          X(0)[me] = u[0];
          X(1)[me] = u[1];
          X(2)[me] = u[2];
          X(3)[me] = gu[0][0] + P.alpha_jac;
          X(4)[me] = gu[1][1] + P.alpha_jac;
          Yr(0)[me] = gu[2][2] + P.alpha_jac;
          Yr(1)[me] = tau;
          Yr(2)[me] = R[0];
          Yr(3)[me] = R[1];
          Yr(4)[me] = R[2];
          Yr(5)[me] = JxW;
        }
        wsync();
        if (pact) {
          Real V0[K1], D0[K1], S0[K1];
#pragma unroll
          for (int t = 0; t < K1; ++t) {
            V0[t] = sM[t * 4 + i0];
            D0[t] = sM[16 + t * 4 + i0] * ih[0];
            S0[t] = sM[32 + t * 4 + i0] * ih[0] * ih[0];
          }
          Real acc[4] = {0, 0, 0, 0};
#pragma nounroll
          for (int a2 = 0; a2 < K1; ++a2) {
            const Real b2 = sM[a2 * 4 + i2], d2 = sM[16 + a2 * 4 + i2] * ih[2];
            const Real s2 = sM[32 + a2 * 4 + i2] * ih[2] * ih[2];
#pragma nounroll
            for (int a1 = 0; a1 < K1; ++a1) {
              const Real b1 = sM[a1 * 4 + i1], d1 = sM[16 + a1 * 4 + i1] * ih[1];
              const Real s1 = sM[32 + a1 * 4 + i1] * ih[1] * ih[1];
#pragma unroll
              for (int a0 = 0; a0 < K1; ++a0) {
                const int qq = a0 + K1 * (a1 + K1 * a2);
                const Real b0 = V0[a0];
                const Real phi = b0 * b1 * b2;
                const Real g[3] = {D0[a0] * b1 * b2, b0 * d1 * b2, b0 * b1 * d2};
                const Real lap = S0[a0] * b1 * b2 + b0 * s1 * b2 + b0 * b1 * s2;
                const Real uq[3] = {X(0)[qq], X(1)[qq], X(2)[qq]};
                const Real gc[3] = {X(3)[qq], X(4)[qq], Yr(0)[qq]};
                const Real tq = Yr(1)[qq], jw = Yr(5)[qq];
                const Real Rq[3] = {Yr(2)[qq], Yr(3)[qq], Yr(4)[qq]};
                const Real av = uq[0] * g[0] + uq[1] * g[1] + uq[2] * g[2];
                const Real g2 = g[0] * g[0] + g[1] * g[1] + g[2] * g[2];
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                  const Real A = gc[c] * phi + av;
                  acc[c] += jw * (A * phi + nu * g2 + tq * (A - nu * lap) * av + tq * Rq[c] * phi * g[c]);
                }
                acc[3] += jw * tq * g2;
              }
            }
          }
          const unsigned msk = P.vmask ? P.vmask[sNode[bn_me]] : 0u;
#pragma unroll
          for (int c = 0; c < 3; ++c) atomicAdd(&sAcc[c * BN3 + bn_me], (msk >> c) & 1u ? fabs(acc[c]) : acc[c]);
          atomicAdd(&sAcc[3 * BN3 + bn_me], acc[3]);
        }
        wsync();
      } else {
        Real Tc[16];
        if constexpr (!JV) {  // residual test coefficients (rhs = -R)
          const Real divu = gu[0][0] + gu[1][1] + gu[2][2];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const Real Gu = gu[c][0] * u[0] + gu[c][1] * u[1] + gu[c][2] * u[2];
            Tc[4 * c] = JxW * (-Gu + f[c] - Tt[c] - srf[c]);
#pragma unroll
            for (int e = 0; e < 3; ++e)
              Tc[4 * c + 1 + e] = JxW * (-nu * gu[c][e] + (c == e ? pq : Real(0)) - tau * R[c] * u[e]) * ih[e];
          }
          Tc[12] = -JxW * divu;
#pragma unroll
          for (int e = 0; e < 3; ++e) Tc[13 + e] = -JxW * tau * R[e] * ih[e];
        } else {
          // ---------------- phase B: the trial function v at this lane's q
          Real v[3] = {0, 0, 0}, gv[3][3] = {}, lv[3] = {0, 0, 0};
#pragma unroll
          for (int c = 0; c < 3; ++c) vel_field(FV + c, v[c], gv[c], lv[c]);
          Real vp = 0, gvp[3] = {0, 0, 0}, dummy[3];
          scal_fields(FV + 3, 0, 0, vp, gvp, dummy);
          if constexpr (CACHED) load_qd();
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

        // ---------------- integration: per test field transposed z / y / x sweeps -> brick accumulator
        Real cb2[K1], cd2[K1], cb1[K1], cd1[K1], cb0[K1], cd0[K1];
        row(3, i2, cb2);
        row(4, i2, cd2);
        row(3, i1, cb1);
        row(4, i1, cd1);
        row(3, i0, cb0);
        row(4, i0, cd0);
#pragma unroll
        for (int fld = 0; fld < 4; ++fld) {
          if (pact) {
            X(0)[me] = Tc[4 * fld];
            X(1)[me] = Tc[4 * fld + 1];
            X(2)[me] = Tc[4 * fld + 2];
            X(3)[me] = Tc[4 * fld + 3];
          }
          wsync();
          if (pact) {
            Real tv[K1], tx[K1], ty[K1], tz[K1];
            lineD2(X(0), tv);
            lineD2(X(1), tx);
            lineD2(X(2), ty);
            lineD2(X(3), tz);
            Yr(0)[me] = dot(cb2, tv) + dot(cd2, tz);
            Yr(1)[me] = dot(cb2, tx);
            Yr(2)[me] = dot(cb2, ty);
          }
          wsync();
          if (pact) {
            Real z0[K1], z1[K1], z2[K1];
            lineD1(Yr(0), z0);
            lineD1(Yr(1), z1);
            lineD1(Yr(2), z2);
            X(0)[me] = dot(cb1, z0) + dot(cd1, z2);
            X(1)[me] = dot(cb1, z1);
          }
          wsync();
          if (pact) {
            Real w0[K1], w1[K1];
            lineD0(X(0), w0);
            lineD0(X(1), w1);
            atomicAdd(&sAcc[fld * BN3 + bn_me], dot(cb0, w0) + dot(cd0, w1));
          }
          wsync();
        }
      }
    }  // rounds
    if (!integrate) {
      gsync();  // sB / sNode are rewritten by the next gather
      continue;
    }
    gsync();  // the brick accumulator is complete

    // ---------------- brick sums -> HBM (interior: plain stores; surface: slab / atomics)
#pragma unroll 1
    for (int t = gtid; t < 4 * BN3; t += GT) {
      const int n = t >> 2, fld = t & 3;
      const Real s = sAcc[fld * BN3 + n];
      sAcc[fld * BN3 + n] = Real(0);
      const int Xn = n % BN, Yn = (n / BN) % BN, Zn = n / (BN * BN);
      const int node = sNode[n];
      const int64_t gi = fld < 3 ? (int64_t)node * 3 + fld : voff + node;
      const bool interior = Xn > 0 && Xn < BN - 1 && Yn > 0 && Yn < BN - 1 && Zn > 0 && Zn < BN - 1;
      if (interior) Yout[gi] = (double)s;
      else if (use_slab) P.slab[((int64_t)brick * C::NBND + bnd_rank<BN>(Xn, Yn, Zn)) * 4 + fld] = (double)s;
      else atomicAdd(&Yout[gi], (double)s);
    }
    gsync();
  }  // items
}

int g_num_cu = 0;
std::once_flag g_cu_once;

template <int K, int MODE, int WPB, typename Real>
hipError_t launch_wave_wpb(const OpParams &P, const Tables1D &T, hipStream_t s) {
  const int n_bricks = P.n_cells / 8;
  const int64_t n_items = (int64_t)n_bricks * (MODE == MODE_JVQ && P.n_probe > 0 ? P.n_probe : 1);
  if (n_items <= 0) return hipSuccess;
  std::call_once(g_cu_once, [] {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_num_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_num_cu <= 0) g_num_cu = 256;
  });
  constexpr size_t lds = wave_lds_bytes<K, MODE, WPB, Real>();
  static int per_cu = 0;
  if (per_cu == 0) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(gls_brick_wave_kernel<K, MODE, WPB, Real>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gls_brick_wave_kernel<K, MODE, WPB, Real>, 64 * kWaves,
                                                     lds) != hipSuccess || nb <= 0)
      nb = 1;
    per_cu = nb;
  }
  constexpr int NGRP = kWaves / WPB;
  int64_t G = std::min<int64_t>((int64_t)g_num_cu * per_cu, (n_items + NGRP - 1) / NGRP);
  G = std::max<int64_t>(8, (G + 7) / 8 * 8);
  hipLaunchKernelGGL((gls_brick_wave_kernel<K, MODE, WPB, Real>), dim3((unsigned)G), dim3(64 * kWaves), lds, s, P, T);
  return hipGetLastError();
}

// waves per brick: Q1 (one round of 8 cells) -> 1; Q2 (four rounds of 2 cells) -> 4, the
// workgroup shares the brick (LDS per wave would otherwise cap occupancy at 3 waves / SIMD).
template <int K, int MODE, typename Real>
hipError_t launch_wave_t(const OpParams &P, const Tables1D &T, hipStream_t s) {
  if constexpr (K == 2 && WaveCfg<K>::ROUNDS % 4 == 0) return launch_wave_wpb<K, MODE, 4, Real>(P, T, s);
  return launch_wave_wpb<K, MODE, 1, Real>(P, T, s);
}

template <int K>
hipError_t launch_wave_mode(int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  switch (mode) {
    case MODE_RESIDUAL: return launch_wave_t<K, MODE_RESIDUAL, double>(P, T, s);
    case MODE_JV: return launch_wave_t<K, MODE_JV, double>(P, T, s);
    case MODE_LIN: return launch_wave_t<K, MODE_LIN, double>(P, T, s);
    case MODE_JVQ: return launch_wave_t<K, MODE_JVQ, double>(P, T, s);
    default: return hipErrorNotSupported;
  }
}

}  // namespace

hipError_t launch_brick_wave(int k, int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (k == 1) return launch_wave_mode<1>(mode, P, T, s);
  if (k == 2) return launch_wave_mode<2>(mode, P, T, s);
  return hipErrorNotSupported;
}
hipError_t launch_brick_wave_jv_f32(int k, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (!P.qdf || P.n_probe > 0) return hipErrorInvalidValue;
  if (k == 1) return launch_wave_t<1, MODE_JVQ, float>(P, T, s);
  if (k == 2) return launch_wave_t<2, MODE_JVQ, float>(P, T, s);
  return hipErrorNotSupported;
}
hipError_t launch_brick_wave_probe(int k, const OpParams &P0, const Tables1D &T, int64_t j0, int nprobe,
                                   hipStream_t s) {
  if (nprobe <= 0) return hipSuccess;
  OpParams P = P0;
  P.n_probe = nprobe;
  P.probe_base = j0;
  P.slab = nullptr;
  if (k == 1) return launch_wave_t<1, MODE_JVQ, double>(P, T, s);
  if (k == 2) return launch_wave_t<2, MODE_JVQ, double>(P, T, s);
  return hipErrorNotSupported;
}
size_t brick_wave_qdata_size(int k, int n_cells) {
  const size_t nb = (size_t)(n_cells / 8);
  if (k == 1) return nb * WaveCfg<1>::ROUNDS * kQData * WaveCfg<1>::QW;
  if (k == 2) return nb * WaveCfg<2>::ROUNDS * kQData * WaveCfg<2>::QW;
  return 0;
}

}  // namespace gls
