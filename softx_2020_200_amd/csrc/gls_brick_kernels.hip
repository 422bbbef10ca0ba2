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
// with plain stores (or updated in place by a fused damped-Jacobi sweep) and brick-boundary nodes
// go to the brick's slab, summed per node in a fixed order by k_slab_sum (no atomics).
// (A float2 field-pair variant of the FP32 J.v — half the LDS instructions — measured slower:
// 2.55 vs 2.19 ms at 128^3, and was removed.)
//
// Per-cell pipeline, one field at a time (keeps ~3 KB of LDS per cell -> 4 workgroups per CU):
//   x sweep (brick -> X), y sweep (X -> Y), z sweep fused into the pointwise read (Y -> registers)
//   state  : u (value, grad, Laplacian) x 3 comps, then {p (value, grad), H (value) x 3}
//   J.v    : v (value, grad, Laplacian) x 3 comps, then v_p (value, grad)
//   test   : per test field, transposed z/y/x sweeps of (value, grad) coefficients -> node array
// The pointwise algebra restates gls_navier_stokes.cc:387-748.
#include "gls_brick_common.hpp"
#include "gls_common.hpp"
#include "gls_launch.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#ifndef GLS_ABL
#define GLS_ABL 0  // timing-only ablations: 1 no global gather, 2 no scatter, 4 no sweeps, 8 no qd loads
#endif
#ifndef GLS_ROWS_REG
#define GLS_ROWS_REG 1  // bit 0: FP32 kernels keep the x/y matrix rows in registers; bit 1: FP64
#endif
#ifndef GLS_BRICK_WAVES_PER_EU
#define GLS_BRICK_WAVES_PER_EU 4
#endif
#ifndef GLS_BRICK_WPE_F32
#define GLS_BRICK_WPE_F32 6  // FP32 kernels: 80 VGPRs, 6 waves/SIMD (1.96 -> 1.92 ms; 7 waves spill, 2.45 ms)
#endif

#ifndef GLS_QD_LITE
// 1: the cached J.v linearization holds tau and R_s only (4 values per quadrature point); MODE_JVQ
// gathers u with v and re-derives u and grad u by value + gradient sweeps (bit-identical to the
// values MODE_LIN computes). 0: u, grad u, tau, R_s cached (16 values, the round-1 layout).
#define GLS_QD_LITE 0
#endif

#ifndef GLS_STAGE_LAYOUT
// stage-array layout per kernel (StageLayout): bit 0 FP64 J.v from the cache, bit 1 FP32 J.v, bit 2
// residual, bit 3 linearization / recompute J.v; set = oriented lines read with ds_read_b128, clear =
// natural [z][y][x] arrays read element-wise. Measured at Q2 128^3 (profiles/r02_stage_layout_ab.txt):
// FP64 J.v 3.16 -> 3.00 ms; FP32 J.v 2.01 -> 2.17 ms and residual 3.48 -> 3.74 ms (spills), so 1.
#define GLS_STAGE_LAYOUT 1
#endif

#ifndef GLS_QD_PREFETCH
// 1: the cached J.v issues its linearization loads before the v sweeps (in flight during them,
// 16 VGPRs live across the sweeps); 0: after the sweeps (short live ranges)
#define GLS_QD_PREFETCH 0
#endif

#ifndef GLS_TEST_PAIR
#define GLS_TEST_PAIR 1  // StageLayout bits (1 FP64 cached J.v, 2 FP32): two test fields per integration pass
                         // (FP64 J.v 2.96 -> 2.89 ms at 128^3; FP32 no change, profiles/r03_ab_test_pair.txt)
#endif

#ifndef GLS_REDUCE_NODE
#define GLS_REDUCE_NODE 1  // brick reduction: one thread per node (4 fields) instead of per (node, field)
#endif

#ifndef GLS_SLAB_INFLIGHT
#ifndef GLS_SLAB_NT
#define GLS_SLAB_NT 0  // 1: slab entries read non-temporally (0.55 vs 0.31 ms at 128^3: a slab line serves up to 4 nodes)
#endif
#ifndef GLS_SLAB_XCD
#define GLS_SLAB_XCD 0  // 1: consecutive slab-sum blocks on one XCD (measured no gain, 0.31 vs 0.32 ms)
#endif
#define GLS_SLAB_INFLIGHT 1  // k_slab_sum: every slot of a node loaded at once (0.583 -> 0.548 ms at 128^3, profiles/r03_ab_reduce_node.txt)
#endif

#ifndef GLS_LDS_SPLIT
#define GLS_LDS_SPLIT 0  // 1 asm / 2 masked: FP64 LDS reads as single ds_read_b64 -- measured slower (profiles/r02_lds_split_ab.txt)
#endif

namespace gls {

constexpr bool kQdLite = GLS_QD_LITE != 0;
constexpr int kQDataBrick = kQdLite ? 4 : kQData;  // values per quadrature point in the brick layout

// One LDS read that the backend may not pair with another (GLS_LDS_SPLIT): ds_read2_b64 moves 16 B
// per lane in 8 LDS cycles (4 x 16-lane groups per access, MI355X_MICROARCH.md §LDS) where two
// ds_read_b64 take 2 + 2. Splitting every pair cuts SQ_LDS_IDX_ACTIVE of the cached J.v 37 % and
// its bank conflicts 64 %, but costs one or two VALU address ops per load and spills at 4 waves /
// SIMD: 3.18 -> 4.17 ms (4 waves, spills) / 3.50 ms (3 waves) at 128^3
// (profiles/r02_lds_split_ab.txt), so the default keeps the compiler's pairing.
template <typename T>
__device__ __forceinline__ T lds(const T *p, unsigned zm) {
  if constexpr (sizeof(T) == 8 && GLS_LDS_SPLIT) {
    typedef __attribute__((address_space(3))) const T lds_t;
    unsigned a = (unsigned)(uintptr_t)(lds_t *)p;
    if constexpr (GLS_LDS_SPLIT == 1) asm volatile("" : "+v"(a));
    else a += a & zm;
    return *(lds_t *)(uintptr_t)a;
  } else {
    return *p;
  }
}

template <int K>
struct BrickCfg {
  static constexpr int K1 = K + 1;           // nodes per direction per cell == QGauss points (k+1)
  static constexpr int N3 = K1 * K1 * K1;    // per-cell array length
  static constexpr int L2 = K1 * K1;         // lines per array
  static constexpr int BN = 2 * K + 1;       // brick nodes per direction
  static constexpr int BN3 = BN * BN * BN;
  static constexpr int NBND = BN3 - (BN - 2) * (BN - 2) * (BN - 2);  // brick-boundary nodes
  static constexpr int CPW = 64 / N3 >= 2 ? 2 : 1;  // cells per wave (Q1: 8 q -> could be 8; keep 2)
  static constexpr int WAVES = 8 / CPW;      // waves per workgroup (one brick)
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int BN3P = (BN3 + 3) & ~3;  // brick field stride (keeps the stage arrays 16-B aligned)
  static constexpr int NO = 4;  // per-cell test-field outputs (natural [z][y][x] order, N3 each)
};

// Per-cell sweep-stage arrays in LDS. Each array is stored in the orientation its reader sweeps:
// the lane's K1-element line along that dim is contiguous and 16-B aligned, so it is read with
// ds_read_b128 (4 LDS cycles per 16 B per wave) instead of K1 scalar reads that the backend pairs
// into ds_read2_b64 (8 cycles per 16 B; MI355X_MICROARCH.md §LDS).
//  * FP64, K1 = 3 ("pair" layout): arrays come in pairs (slots 2p, 2p+1); a pair block holds the
//    (e0, e1) halves of both arrays' 9 lines (16 B each, at 0 and A0) and one half-plane at H1 whose
//    line L holds (e2 of slot 2p, e2 of slot 2p+1): a line costs 1.5 ds_read_b128 and no padding.
//  * FP32 K1 = 3 (lines padded to 4 floats) and K1 = 2: one vector read per line.
// The cell stride puts the two cells of a wave on disjoint banks (conflict-free b128 reads under
// the lane-group model of MI355X_MICROARCH.md §LDS; checked offline for every orientation).
template <int K, typename Real, int MODE>
struct StageLayout {
  static constexpr bool CACHED = MODE == MODE_JVQ;
  static constexpr int K1 = K + 1, N3 = K1 * K1 * K1;
  static constexpr int BIT = CACHED ? (sizeof(Real) == 8 ? 1 : 2) : (MODE == MODE_RESIDUAL ? 4 : 8);
  static constexpr bool ORIENTED = (GLS_STAGE_LAYOUT & BIT) != 0;  // else natural arrays
  static constexpr bool PAIR = ORIENTED && sizeof(Real) == 8 && K1 == 3;
  // two test fields integrated side by side (their z / y / x stages share the LDS round trips)
  static constexpr bool TPAIR = CACHED && (GLS_TEST_PAIR & BIT) != 0;
  static constexpr int LP = K1 == 3 ? 4 : K1;            // padded line length (non-pair layouts)
  static constexpr int NXA = CACHED ? (TPAIR ? 8 : 4) : 5, NYA = CACHED ? (TPAIR ? 6 : 4) : 6;  // X / Y arrays
  static constexpr int XP = (NXA + 1) / 2, YP = (NYA + 1) / 2;
  static constexpr int YB = PAIR ? 2 * XP : NXA;        // slot of Y array 0
  static constexpr int A0 = 18, H1 = 44, PB = 62;       // pair block: halves at 0 / A0, e2 plane at H1
  static constexpr int AS = ORIENTED ? K1 * K1 * LP : N3;  // array size (non-pair layouts)
  static constexpr int SR0 = PAIR ? (XP + YP) * PB : (NXA + NYA) * AS;
  static constexpr int SR = (!CACHED && SR0 < 11 * N3) ? 11 * N3 : SR0;  // MODE_LIN's diagonal: 11 plain arrays
  static constexpr int stride(int v) {
    if (PAIR) { while (v % 32 != 18) ++v; }
    else if (ORIENTED && K1 == 3) { while (v % 64 != 40) ++v; }
    return v;
  }
  static constexpr int CS = stride(SR);  // per-cell stride (elements)
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

template <int K, int MODE, typename Real = double>
__global__ void __launch_bounds__(BrickCfg<K>::THREADS,
                                  (std::is_same<Real, float>::value ? GLS_BRICK_WPE_F32 : GLS_BRICK_WAVES_PER_EU))
    gls_brick_kernel(const OpParams P, const Tables1D T) {
  const unsigned zm = (unsigned)(P.n_cells >> 31);  // 0 (n_cells >= 0), opaque to the compiler
  using C = BrickCfg<K>;
  constexpr int K1 = C::K1, N3 = C::N3, BN = C::BN, BN3 = C::BN3, CPW = C::CPW;
  constexpr bool JV = MODE == MODE_JV || MODE == MODE_JVQ;
  constexpr bool CACHED = MODE == MODE_JVQ;  // linearization read from P.qd (no state sweeps)
  constexpr bool LIN = MODE == MODE_LIN;     // store the linearization to P.qd, no integration
  // brick fields: u0 u1 u2 p H0 H1 H2 [v0 v1 v2 vp]; JVQ: [u0 u1 u2] v0 v1 v2 vp
  constexpr int NF = CACHED ? (kQdLite ? 7 : 4) : (JV ? 11 : 7);
  constexpr int FV = CACHED ? (kQdLite ? 3 : 0) : 7;  // first v field
  using SL = StageLayout<K, Real, MODE>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Real *const smem = reinterpret_cast<Real *>(smem_raw);
  Real *sB = smem;                                   // [NF][BN3P]
  Real *sC = sB + NF * C::BN3P;                      // [8][CS] stage arrays (StageLayout)
  Real *sO = sC + 8 * SL::CS;                        // [8][NO][N3]
  // 1D tables [V, D, S, V^T, D^T][4][4], w[4], xi[4] in a SEPARATE shared object: the compiler then
  // knows table reads never alias the stage arrays, so it can issue them ahead of a stage's stores
  // (in the dynamic array every row read after an X store waited for it: serialized LDS latency)
  __shared__ Real sTab[5 * 16 + 8];
  Real *const sM = sTab;
  int *sNode = reinterpret_cast<int *>(sO + 8 * C::NO * N3);  // [BN3]
  auto BF = [&](int f) { return sB + f * C::BN3P; };

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int n_bricks = P.n_cells / 8;
  // probing (MODE_JVQ): block -> (unit vector, brick); v = e_j, output column j of the batch
  const int pj = (CACHED && P.n_probe > 0) ? (int)(blockIdx.x / n_bricks) : 0;
  // XCD-aware order (blocks b, b+8, b+16, ... share an XCD): each XCD walks a contiguous Morton
  // range of bricks, so the nodes neighbouring bricks share stay in that XCD's L2
#ifdef GLS_BRICK_COLORS_BUILD
  const bool colored = P.bricks != nullptr && !(CACHED && P.n_probe > 0);
#else
  // colored brick launches (the measured-slower experiment, profiles/r02_brick_colors_ab.txt) are
  // compiled only with -DGLS_BRICK_COLORS_BUILD: their scatter branch costs the FP32 smoother kernel
  // 4 extra VGPR spills (2.13 -> 2.80 ms at 128^3)
  constexpr bool colored = false;
#endif
  const int brick = (CACHED && P.n_probe > 0) ? (int)(blockIdx.x % n_bricks)
                    : colored ? P.bricks[P.color_off[P.color] +
                                         xcd_swizzle((int)blockIdx.x, P.color_off[P.color + 1] - P.color_off[P.color])]
                    : (std::is_same<Real, double>::value && P.subset) ? P.subset[xcd_swizzle((int)blockIdx.x, P.subset_n)]
                              : xcd_swizzle((int)blockIdx.x, n_bricks);
  const int64_t unit_dof = (CACHED && P.n_probe > 0) ? P.probe_base + pj : -1;
  double *const Yout = (CACHED && P.n_probe > 0)
                           ? P.y + (int64_t)pj * ((int64_t)3 * P.n_vnodes + P.n_vnodes) : P.y;
  const int64_t voff = (int64_t)3 * P.n_vnodes;
  const bool use_slab = !colored && P.slab != nullptr && !(CACHED && P.n_probe > 0);

  if (tid < 5 * 16) {
    const int mat = tid >> 4, r = (tid >> 2) & 3, c = tid & 3;
    Real v = 0.;
    if (r < K1 && c < K1) {
      if (mat == 0) v = T.V[r][c];
      else if (mat == 1) v = T.D[r][c];
      else if (mat == 2) v = T.S[r][c];
      else if (mat == 3) v = T.V[c][r];
      else v = T.D[c][r];
    }
    sM[tid] = v;
  } else if (tid < 5 * 16 + 8) {
    const int j = (tid - 80) & 3;
    sM[tid] = j < K1 ? (tid < 84 ? T.w[j] : T.xi[j]) : 0.0;
  }
  // ---------------- gather the brick's nodes (all waves)
  // gather groups: state (u, p) | history | v;  JVQ: [u (no p)] | v
  constexpr int NG = CACHED ? (kQdLite ? 2 : 1) : (JV ? 3 : 2);
  for (int t = tid; t < NG * BN3; t += blockDim.x) {
    const int g = CACHED ? ((kQdLite && t < BN3) ? 0 : 2) : t / BN3, n = t % BN3;
    if (GLS_ABL & 1) {
      for (int f = 0; f < NF; ++f) BF(f)[n] = 0.001 * (n + f);
      if (g == 0 || CACHED) sNode[n] = (brick * 37 + n) % P.n_vnodes;
      continue;
    }
    const int X = n % BN, Y = (n / BN) % BN, Z = n / (BN * BN);
    const int cx = min(X / K, 1), cy = min(Y / K, 1), cz = min(Z / K, 1);
    const int a = (X - K * cx) + K1 * ((Y - K * cy) + K1 * (Z - K * cz));
    const int node = P.cell_vnodes[((int64_t)brick * 8 + cx + 2 * cy + 4 * cz) * N3 + a];
    const int64_t i3 = (int64_t)node * 3;
    if (g == 0 || CACHED) sNode[n] = node;
    if (g == 0) {
      BF(0)[n] = P.u[i3];
      BF(1)[n] = P.u[i3 + 1];
      BF(2)[n] = P.u[i3 + 2];
      if (!CACHED) BF(3)[n] = P.u[voff + node];
    } else if (g == 1) {
      Real h[3] = {0., 0., 0.};
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
      if (unit_dof >= 0) {
        const unsigned m = P.vmask ? P.vmask[node] : 0u;
        BF(FV)[n] = (m & 1u) ? 0.0 : (i3 == unit_dof ? 1.0 : 0.0);
        BF(FV + 1)[n] = (m & 2u) ? 0.0 : (i3 + 1 == unit_dof ? 1.0 : 0.0);
        BF(FV + 2)[n] = (m & 4u) ? 0.0 : (i3 + 2 == unit_dof ? 1.0 : 0.0);
        BF(FV + 3)[n] = voff + node == unit_dof ? 1.0 : 0.0;
      } else {  // v and the mask loaded together (all in flight: one round trip), masked afterwards
        const double v0 = P.v[i3], v1 = P.v[i3 + 1], v2 = P.v[i3 + 2], vp = P.v[voff + node];
        const unsigned m = P.vmask ? P.vmask[node] : 0u;
        BF(FV)[n] = (m & 1u) ? 0.0 : v0;
        BF(FV + 1)[n] = (m & 2u) ? 0.0 : v1;
        BF(FV + 2)[n] = (m & 4u) ? 0.0 : v2;
        BF(FV + 3)[n] = vp;
      }
    }
  }
  __syncthreads();
  // ---------------- per-wave: cells 2*wave, 2*wave+1 of the brick
  auto Out = [&](int ci, int f) { return sO + (ci * C::NO + f) * N3; };
  const int cbase = wave * CPW;
  // pointwise lane mapping: lane -> (cell, q)
  const bool pact = lane < CPW * N3;
  const int pci = cbase + (pact ? lane / N3 : 0);
  const int q = pact ? lane % N3 : 0;
  const int qx = q % K1, qy = (q / K1) % K1, qz = q / (K1 * K1);
  const int gcell = brick * 8 + pci;
  const Real hx = P.geo[gcell * 4 + 0], hy = P.geo[gcell * 4 + 1], hz = P.geo[gcell * 4 + 2];
  const Real ih[3] = {Real(1) / hx, Real(1) / hy, Real(1) / hz};
  const Real wz = ih[2] * ih[2];
  // this lane's rows of the z matrices (q-dependent -> registers; tables staged in LDS above)
  Real Bz[K1], Dz[K1], Sz[K1];
#pragma unroll
  for (int i = 0; i < K1; ++i) { Bz[i] = sM[0 * 16 + qz * 4 + i]; Dz[i] = sM[1 * 16 + qz * 4 + i]; Sz[i] = sM[2 * 16 + qz * 4 + i]; }

  // Lane <-> output element: every stage computes entry [i2][i1][i0] of its output arrays for the
  // lane's cell (the same lanes as the pointwise (cell, q) mapping), reading one 1D line of each
  // input array; per-lane matrix rows come from the LDS copy of the 1D tables. No divergence.
  const int i0 = qx, i1 = qy, i2 = qz;
  const int me = q;  // offset of this lane's element in a per-cell array
  // brick x-line base of this lane's (cell, y=i1, z=i2) line
  const int cxb = pci & 1, cyb = (pci >> 1) & 1, czb = pci >> 2;
  const int bx_base = K * cxb + BN * (K * cyb + i1) + BN * BN * (K * czb + i2);
  auto row = [&](int mat, int r, Real (&o)[K1]) {  // o[k] = M[r][k], mat: 0 V, 1 D, 2 S, 3 V^T, 4 D^T
    const Real *m = sM + mat * 16 + r * 4;
#pragma unroll
    for (int k = 0; k < K1; ++k) o[k] = lds(m + k, zm);
  };
  // this lane's rows of the x / y 1D matrices (V, D, S at i0 and i1): registers when GLS_ROWS_REG
  // is set for this precision (the sweeps are LDS-bound), else one LDS read per use
  constexpr bool RREG = std::is_same<Real, float>::value ? (GLS_ROWS_REG & 1) : (GLS_ROWS_REG & 2);
  Real rr[RREG ? 6 : 1][K1];
  if constexpr (RREG) {
    row(0, i0, rr[0]);
    row(1, i0, rr[1]);
    row(2, i0, rr[2]);
    row(0, i1, rr[3]);
    row(1, i1, rr[4]);
    row(2, i1, rr[5]);
  }
  auto rowq = [&](int mat, int which, Real (&o)[K1]) {  // which: 0 -> row i0, 1 -> row i1
    if constexpr (RREG) {
#pragma unroll
      for (int k = 0; k < K1; ++k) o[k] = rr[which * 3 + mat][k];
    } else {
      row(mat, which ? i1 : i0, o);
    }
  };
  auto dot = [&](const Real (&a)[K1], const Real (&b)[K1]) {
    Real s = 0.;
#pragma unroll
    for (int k = 0; k < K1; ++k) s += a[k] * b[k];
    return s;
  };
  // Stage arrays (StageLayout): slot g (X arrays 0.., Y arrays SL::YB..) stored d-oriented: the
  // lane's line along dim d (index ln[d], element = the lane's coordinate along d) is contiguous.
  Real *const cellS = sC + pci * SL::CS;
  const int ln[3] = {i1 + K1 * i2, i0 + K1 * i2, i0 + K1 * i1};
  const int co[3] = {i0, i1, i2};
  auto wr = [&](int g, int d, Real val) {  // this lane's element of slot g in the d-oriented layout
    if constexpr (SL::PAIR) {
      // one store per lane at a selected offset (no divergent store pair)
      const int off = co[d] < 2 ? (g & 1) * SL::A0 + 2 * ln[d] + co[d] : SL::H1 + 2 * ln[d] + (g & 1);
      cellS[(g >> 1) * SL::PB + off] = val;
    } else if constexpr (SL::ORIENTED) {
      cellS[g * SL::AS + ln[d] * SL::LP + co[d]] = val;
    } else {
      cellS[g * SL::AS + me] = val;
    }
  };
  auto rdl = [&](int g, int d, Real (&o)[K1]) {  // the lane's whole line of slot g along dim d
    if constexpr (SL::PAIR) {
      typedef double v2 __attribute__((ext_vector_type(2)));
      const Real *b = cellS + (g >> 1) * SL::PB;
      const v2 a = *reinterpret_cast<const v2 *>(b + (g & 1) * SL::A0 + 2 * ln[d]);
      const v2 t = *reinterpret_cast<const v2 *>(b + SL::H1 + 2 * ln[d]);
      o[0] = a.x;
      o[1] = a.y;
      o[2] = (g & 1) ? t.y : t.x;
      return;
    }
    if constexpr (!SL::ORIENTED) {  // natural [z][y][x]: K1 element reads along dim d
      const Real *a = cellS + g * SL::AS;
      const int st = d == 0 ? 1 : (d == 1 ? K1 : K1 * K1);
      const int b0 = me - co[d] * st;
#pragma unroll
      for (int e = 0; e < K1; ++e) o[e] = lds(a + b0 + e * st, zm);
      return;
    }
    const Real *p = cellS + g * SL::AS + ln[d] * SL::LP;
    if constexpr (std::is_same<Real, double>::value) {
      typedef double v2 __attribute__((ext_vector_type(2)));
      const v2 a = *reinterpret_cast<const v2 *>(p);
      o[0] = a.x;
      o[1] = a.y;
    } else if constexpr (K1 == 3) {
      typedef float v4 __attribute__((ext_vector_type(4)));
      const v4 a = *reinterpret_cast<const v4 *>(p);
      o[0] = a.x;
      o[1] = a.y;
      o[2] = a.z;
    } else {
      typedef float v2 __attribute__((ext_vector_type(2)));
      const v2 a = *reinterpret_cast<const v2 *>(p);
      o[0] = a.x;
      o[1] = a.y;
    }
  };

  // velocity-type field (value, grad, Laplacian): brick field f -> (val, g0, g1, g2, lap) for this lane
  auto vel_field = [&](int f, Real &val, Real (&g)[3], Real &lap) {
    if (GLS_ABL & 4) { val = BF(f)[bx_base]; g[0] = g[1] = g[2] = val; lap = val; return; }
    if (pact) {  // x sweep: X_B, X_D, X_S at [i2][i1][i0]
      Real in[K1], r0[K1], r1[K1], r2[K1];  // every load of the stage before its stores
#pragma unroll
      for (int e = 0; e < K1; ++e) in[e] = lds(BF(f) + bx_base + e, zm);
      rowq(0, 0, r0);
      rowq(1, 0, r1);
      rowq(2, 0, r2);
      const Real o0 = dot(r0, in), o1 = dot(r1, in), o2 = dot(r2, in);
      wr(0, 1, o0);
      wr(1, 1, o1);
      wr(2, 1, o2);
    }
    wave_sync();
    if (pact) {  // y sweep: BB, BD, DB, L = wy S_y(X_B) + wx B_y(X_S)
      Real xb[K1], xd[K1], xs[K1], rb[K1], rd[K1], rs[K1];
      rdl(0, 1, xb);
      rdl(1, 1, xd);
      rdl(2, 1, xs);
      rowq(0, 1, rb);
      rowq(1, 1, rd);
      rowq(2, 1, rs);
      wr(SL::YB + 0, 2, dot(rb, xb));
      wr(SL::YB + 1, 2, dot(rd, xb));
      wr(SL::YB + 2, 2, dot(rb, xd));
      wr(SL::YB + 3, 2, ih[1] * ih[1] * dot(rs, xb) + ih[0] * ih[0] * dot(rb, xs));
    }
    wave_sync();
    if (pact) {  // z sweep fused into the pointwise read
      Real bb[K1], bd[K1], db[K1], ll[K1];
      rdl(SL::YB + 0, 2, bb);
      rdl(SL::YB + 1, 2, bd);
      rdl(SL::YB + 2, 2, db);
      rdl(SL::YB + 3, 2, ll);
      val = dot(Bz, bb);
      g[0] = dot(Bz, db) * ih[0];
      g[1] = dot(Bz, bd) * ih[1];
      g[2] = dot(Dz, bb) * ih[2];
      lap = dot(Bz, ll) + wz * dot(Sz, bb);
    }
    wave_sync();  // Y is rewritten by the next field's y sweep
  };

  // pressure-type field (value, grad) [+ up to 3 value-only fields]: fp -> (pv, pg); fh.. -> hv[]
  auto scal_fields = [&](int fp, int nh, int fh0, Real &pv, Real (&pg)[3], Real (&hv)[3]) {
    if (GLS_ABL & 4) { pv = BF(fp)[bx_base]; pg[0] = pg[1] = pg[2] = pv; for (int j = 0; j < nh; ++j) hv[j] = pv; return; }
    if (pact) {  // x: p -> X0 (B), X1 (D); H_j -> X(2+j) (B)
      Real in[K1], rb[K1], rd[K1], ih_[3][K1];
      rowq(0, 0, rb);
      rowq(1, 0, rd);
#pragma unroll
      for (int e = 0; e < K1; ++e) in[e] = lds(BF(fp) + bx_base + e, zm);
      for (int j = 0; j < nh; ++j)
#pragma unroll
        for (int e = 0; e < K1; ++e) ih_[j][e] = lds(BF(fh0 + j) + bx_base + e, zm);
      wr(0, 1, dot(rb, in));
      wr(1, 1, dot(rd, in));
      for (int j = 0; j < nh; ++j) wr(2 + j, 1, dot(rb, ih_[j]));
    }
    wave_sync();
    if (pact) {  // y: X0 -> BB (Y0), BD (Y1); X1 -> DB (Y2); X(2+j) -> Y(3+j)
      Real a[K1], a1[K1], rb[K1], rd[K1], ah[3][K1];
      rowq(0, 1, rb);
      rowq(1, 1, rd);
      rdl(0, 1, a);
      rdl(1, 1, a1);
      for (int j = 0; j < nh; ++j) rdl(2 + j, 1, ah[j]);
      wr(SL::YB + 0, 2, dot(rb, a));
      wr(SL::YB + 1, 2, dot(rd, a));
      wr(SL::YB + 2, 2, dot(rb, a1));
      for (int j = 0; j < nh; ++j) wr(SL::YB + 3 + j, 2, dot(rb, ah[j]));
    }
    wave_sync();
    if (pact) {
      Real bb[K1], bd[K1], db[K1];
      rdl(SL::YB + 0, 2, bb);
      rdl(SL::YB + 1, 2, bd);
      rdl(SL::YB + 2, 2, db);
      pv = dot(Bz, bb);
      pg[0] = dot(Bz, db) * ih[0];
      pg[1] = dot(Bz, bd) * ih[1];
      pg[2] = dot(Dz, bb) * ih[2];
      for (int j = 0; j < nh; ++j) {
        rdl(SL::YB + 3 + j, 2, bb);
        hv[j] = dot(Bz, bb);
      }
    }
    wave_sync();
  };

  const Real nu = P.nu;
  const Real JxW = sM[80 + qx] * sM[80 + qy] * sM[80 + qz] * hx * hy * hz;
  // linearization storage: per wave CPW*N3 lanes x kQDataBrick values, value-major (coalesced)
  constexpr int QW = CPW * N3;
  // K = 2: the pencil layout (qdp_base, gls_brick_common.hpp: the pencil J.v's rows; value stride 54 =
  // QW); K = 1: wave-major per brick
  static_assert(K != 2 || (QW == kQdpRow && !kQdLite), "pencil layout: 54-entry rows, full linearization");
  const int64_t qoff = K == 2 ? qdp_base(brick, pci, q) : ((int64_t)brick * C::WAVES + wave) * kQDataBrick * QW + lane;
  Real *qdw = nullptr;
  if constexpr (std::is_same<Real, double>::value) {
    if (P.qd) qdw = P.qd + qoff;
  } else {
    if (P.qdf) qdw = P.qdf + qoff;
  }

  // ---------------- phase A: state at this lane's quadrature point
  Real u[3] = {0., 0., 0.}, gu[3][3] = {}, R[3] = {0., 0., 0.}, tau = 0.;
  Real pq = 0., f[3] = {0., 0., 0.}, Tt[3] = {0., 0., 0.}, srf[3] = {0., 0., 0.};
  // JVQ: the linearization is loaded after the v sweeps (short live ranges: no spills)
  auto load_qd = [&]() {
    if (GLS_ABL & 8) {  // timing-only: no linearization stream
      if (!kQdLite) {
#pragma unroll
        for (int c = 0; c < 3; ++c) u[c] = JxW * (c + 1);
#pragma unroll
        for (int c = 0; c < 9; ++c) gu[c / 3][c % 3] = hx * c;
      }
      tau = JxW;
#pragma unroll
      for (int c = 0; c < 3; ++c) R[c] = hy * c;
      return;
    }
    if (pact && kQdLite) {  // u, grad u come from the u sweeps
      tau = __builtin_nontemporal_load(qdw);
#pragma unroll
      for (int c = 0; c < 3; ++c) R[c] = __builtin_nontemporal_load(qdw + (1 + c) * QW);
    } else if (pact) {
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
  Real lu[3] = {0., 0., 0.};
#pragma unroll
  for (int c = 0; c < 3; ++c) vel_field(c, u[c], gu[c], lu[c]);
  Real gp[3] = {0., 0., 0.}, Hq[3] = {0., 0., 0.};
  scal_fields(3, 3, 4, pq, gp, Hq);

  const Real hst = P.geo[gcell * 4 + 3];
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
    const Real *om = P.omega;
    const Real xq[3] = {P.x0[gcell * 3 + 0] + hx * sM[84 + qx], P.x0[gcell * 3 + 1] + hy * sM[84 + qy],
                          P.x0[gcell * 3 + 2] + hz * sM[84 + qz]};
    const Real cx_[3] = {om[1] * u[2] - om[2] * u[1], om[2] * u[0] - om[0] * u[2], om[0] * u[1] - om[1] * u[0]};
    const Real ox[3] = {om[1] * xq[2] - om[2] * xq[1], om[2] * xq[0] - om[0] * xq[2], om[0] * xq[1] - om[1] * xq[0]};
    const Real cc[3] = {om[1] * ox[2] - om[2] * ox[1], om[2] * ox[0] - om[0] * ox[2], om[0] * ox[1] - om[1] * ox[0]};
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
  }  // !CACHED

  if constexpr (LIN) {  // store the linearization; the integration below is J.v's (MODE_JVQ)
    if (pact && kQdLite) {
      qdw[0] = tau;
#pragma unroll
      for (int c = 0; c < 3; ++c) qdw[(1 + c) * QW] = R[c];
      if constexpr (std::is_same<Real, double>::value) {
        if (P.qdf) {  // the mixed-precision smoother's FP32 copy, written from registers
          float *qf = P.qdf + (qdw - P.qd);
          __builtin_nontemporal_store((float)tau, qf);
#pragma unroll
          for (int c = 0; c < 3; ++c) __builtin_nontemporal_store((float)R[c], qf + (1 + c) * QW);
        }
      }
    } else if (pact) {
#pragma unroll
      for (int c = 0; c < 3; ++c) qdw[c * QW] = u[c];
#pragma unroll
      for (int c = 0; c < 9; ++c) qdw[(3 + c) * QW] = gu[c / 3][c % 3];
      qdw[12 * QW] = tau;
#pragma unroll
      for (int c = 0; c < 3; ++c) qdw[(13 + c) * QW] = R[c];
      if constexpr (std::is_same<Real, double>::value) {
        if (P.qdf) {  // the mixed-precision smoother's FP32 copy, written from registers
          float *qf = P.qdf + (qdw - P.qd);
#pragma unroll
          for (int c = 0; c < 3; ++c) __builtin_nontemporal_store((float)u[c], qf + c * QW);
#pragma unroll
          for (int c = 0; c < 9; ++c) __builtin_nontemporal_store((float)gu[c / 3][c % 3], qf + (3 + c) * QW);
          __builtin_nontemporal_store((float)tau, qf + 12 * QW);
#pragma unroll
          for (int c = 0; c < 3; ++c) __builtin_nontemporal_store((float)R[c], qf + (13 + c) * QW);
        }
      }
    }
    if (P.y == nullptr) return;  // linearization only (uniform over the block)
    // Jacobian diagonal from the same linearization (replaces the dense MODE_DIAG kernel): for the
    // trial/test pair phi_i e_c (gls_navier_stokes.cc:548-622 with v = phi_i e_c)
    //   J_ii(c) = sum_q JxW [A phi + nu |grad phi|^2 + tau (A - nu lap phi) a + tau R_c phi d_c phi],
    //   A = (du_c/dx_c + alpha_jac) phi + a,  a = u . grad phi;   J_ii(p) = sum_q JxW tau |grad psi|^2
    // with deal.II's |K_e(i,i)| on constrained rows. Lane <-> node i of its cell, loop over q.
    auto Nat = [&](int s) { return cellS + s * N3; };  // plain [z][y][x] arrays over the stage region
    if (pact) {
      Nat(0)[me] = u[0];
      Nat(1)[me] = u[1];
      Nat(2)[me] = u[2];
      Nat(3)[me] = gu[0][0] + P.alpha_jac;
      Nat(4)[me] = gu[1][1] + P.alpha_jac;
      Nat(5)[me] = gu[2][2] + P.alpha_jac;
      Nat(6)[me] = tau;
      Nat(7)[me] = R[0];
      Nat(8)[me] = R[1];
      Nat(9)[me] = R[2];
      Nat(10)[me] = JxW;
    }
    wave_sync();
    if (pact) {
      Real V0[K1], D0[K1], S0[K1];  // x-direction table column of this lane's node (registers)
#pragma unroll
      for (int t = 0; t < K1; ++t) {
        V0[t] = sM[0 * 16 + t * 4 + i0];
        D0[t] = sM[1 * 16 + t * 4 + i0] * ih[0];
        S0[t] = sM[2 * 16 + t * 4 + i0] * ih[0] * ih[0];
      }
      Real acc[4] = {0., 0., 0., 0.};
#pragma nounroll
      for (int a2 = 0; a2 < K1; ++a2) {
        const Real b2 = sM[0 * 16 + a2 * 4 + i2], d2 = sM[16 + a2 * 4 + i2] * ih[2];
        const Real s2 = sM[32 + a2 * 4 + i2] * ih[2] * ih[2];
#pragma nounroll
        for (int a1 = 0; a1 < K1; ++a1) {
          const Real b1 = sM[0 * 16 + a1 * 4 + i1], d1 = sM[16 + a1 * 4 + i1] * ih[1];
          const Real s1 = sM[32 + a1 * 4 + i1] * ih[1] * ih[1];
#pragma unroll
          for (int a0 = 0; a0 < K1; ++a0) {
            const int qq = a0 + K1 * (a1 + K1 * a2);
            const Real b0 = V0[a0];
            const Real phi = b0 * b1 * b2;
            const Real g[3] = {D0[a0] * b1 * b2, b0 * d1 * b2, b0 * b1 * d2};
            const Real lap = S0[a0] * b1 * b2 + b0 * s1 * b2 + b0 * b1 * s2;
            const Real uq[3] = {lds(Nat(0) + qq, zm), lds(Nat(1) + qq, zm), lds(Nat(2) + qq, zm)};
            const Real gc[3] = {lds(Nat(3) + qq, zm), lds(Nat(4) + qq, zm), lds(Nat(5) + qq, zm)};
            const Real tq = lds(Nat(6) + qq, zm), jw = lds(Nat(10) + qq, zm);
            const Real Rq[3] = {lds(Nat(7) + qq, zm), lds(Nat(8) + qq, zm), lds(Nat(9) + qq, zm)};
            const Real av = uq[0] * g[0] + uq[1] * g[1] + uq[2] * g[2];
            const Real g2 = g[0] * g[0] + g[1] * g[1] + g[2] * g[2];
            // the same sum with the component-independent part factored out (A = gc_c phi + av):
            // jw [av phi + nu g2 + tq av (av - nu lap)] + gc_c jw phi (phi + tq av) + Rq_c g_c jw tq phi
            const Real jt = jw * tq;
            const Real c0 = jw * (av * phi + nu * g2) + jt * av * (av - nu * lap);
            const Real k1 = jw * phi * (phi + tq * av), k2 = jt * phi;
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c] += c0 + gc[c] * k1 + k2 * Rq[c] * g[c];
            acc[3] += jt * g2;
          }
        }
      }
      // deal.II's constrained-row rule: |K_e(i,i)| summed over cells
      const int bn = (K * cxb + i0) + BN * ((K * cyb + i1) + BN * (K * czb + i2));
      const unsigned msk = P.vmask ? P.vmask[sNode[bn]] : 0u;
#pragma unroll
      for (int c = 0; c < 3; ++c) Out(pci, c)[me] = (msk >> c) & 1u ? fabs(acc[c]) : acc[c];
      Out(pci, 3)[me] = acc[3];
    }
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
        Tc[4 * c + 1 + e] = JxW * (-nu * gu[c][e] + (c == e ? pq : 0.0) - tau * R[c] * u[e]) * ih[e];
    }
    Tc[12] = -JxW * divu;
#pragma unroll
    for (int e = 0; e < 3; ++e) Tc[13 + e] = -JxW * tau * R[e] * ih[e];
  } else {
    // ---------------- phase B: the trial function v at this lane's quadrature point
    if constexpr (CACHED && GLS_QD_PREFETCH && !kQdLite) load_qd();
    Real v[3] = {0., 0., 0.}, gv[3][3] = {}, lv[3] = {0., 0., 0.};
#pragma unroll
    for (int c = 0; c < 3; ++c) vel_field(FV + c, v[c], gv[c], lv[c]);
    Real vp = 0., gvp[3] = {0., 0., 0.}, dummy[3];
    scal_fields(FV + 3, 0, 0, vp, gvp, dummy);
    if constexpr (CACHED && kQdLite) {  // u, grad u: value + gradient sweeps of the gathered u
#pragma unroll
      for (int c = 0; c < 3; ++c) scal_fields(c, 0, 0, u[c], gu[c], dummy);
    }
    if constexpr (CACHED && !(GLS_QD_PREFETCH && !kQdLite)) load_qd();
    const Real aj = P.alpha_jac;
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
        Tc[4 * c + 1 + e] = JxW * (nu * gv[c][e] - (c == e ? vp : Real(0)) + tau * S[c] * u[e] + tau * R[c] * v[e]) * ih[e];
    }
    Tc[12] = JxW * divv;
#pragma unroll
    for (int e = 0; e < 3; ++e) Tc[13 + e] = JxW * tau * S[e] * ih[e];
  }

  // ---------------- integration, one test field at a time (wave-local, lane <-> output element)
  Real cb2[K1], cd2[K1], cb1[K1], cd1[K1], cb0[K1], cd0[K1];  // columns of V, D (transposed rows)
  row(3, i2, cb2);
  row(4, i2, cd2);
  row(3, i1, cb1);
  row(4, i1, cd1);
  row(3, i0, cb0);
  row(4, i0, cd0);
  // FS test fields per pass (SL::TPAIR: 2, slots 4u.., YB + 3u.., 2u.. for field f0 + u)
  constexpr int FS = SL::TPAIR ? 2 : 1;
#pragma unroll
  for (int f0 = 0; f0 < 4; f0 += FS) {
    if (GLS_ABL & 4) {
      for (int u = 0; u < FS; ++u) {
        const int fld = f0 + u;
        if (pact) Out(pci, fld)[me] = Tc[4 * fld] + Tc[4 * fld + 1] + Tc[4 * fld + 2] + Tc[4 * fld + 3];
      }
      continue;
    }
    if (pact) {
#pragma unroll
      for (int u = 0; u < FS; ++u) {
        const int fld = f0 + u;
        wr(4 * u + 0, 2, Tc[4 * fld]);
        wr(4 * u + 1, 2, Tc[4 * fld + 1]);
        wr(4 * u + 2, 2, Tc[4 * fld + 2]);
        wr(4 * u + 3, 2, Tc[4 * fld + 3]);
      }
    }
    wave_sync();
    if (pact) {  // transposed z (output index az = i2): Z0 = B^T Tv + D^T Tz, Z1 = B^T Tx, Z2 = B^T Ty
#pragma unroll
      for (int u = 0; u < FS; ++u) {
        Real tv[K1], tx[K1], ty[K1], tz[K1];
        rdl(4 * u + 0, 2, tv);
        rdl(4 * u + 1, 2, tx);
        rdl(4 * u + 2, 2, ty);
        rdl(4 * u + 3, 2, tz);
        wr(SL::YB + 3 * u + 0, 1, dot(cb2, tv) + dot(cd2, tz));
        wr(SL::YB + 3 * u + 1, 1, dot(cb2, tx));
        wr(SL::YB + 3 * u + 2, 1, dot(cb2, ty));
      }
    }
    wave_sync();
    if (pact) {  // transposed y (ay = i1): W0 = B^T Z0 + D^T Z2, W1 = B^T Z1
#pragma unroll
      for (int u = 0; u < FS; ++u) {
        Real z0[K1], z1[K1], z2[K1];
        rdl(SL::YB + 3 * u + 0, 1, z0);
        rdl(SL::YB + 3 * u + 1, 1, z1);
        rdl(SL::YB + 3 * u + 2, 1, z2);
        wr(2 * u + 0, 0, dot(cb1, z0) + dot(cd1, z2));
        wr(2 * u + 1, 0, dot(cb1, z1));
      }
    }
    wave_sync();
    if (pact) {  // transposed x (ax = i0): out = B^T W0 + D^T W1
#pragma unroll
      for (int u = 0; u < FS; ++u) {
        Real w0[K1], w1[K1];
        rdl(2 * u + 0, 0, w0);
        rdl(2 * u + 1, 0, w1);
        Out(pci, f0 + u)[me] = dot(cb0, w0) + dot(cd0, w1);
      }
    }
    wave_sync();
  }
  }  // !LIN
  __syncthreads();

  // ---------------- brick reduction (fixed order) + scatter
#if GLS_REDUCE_NODE && !defined(GLS_BRICK_COLORS_BUILD)
  // one thread per brick node, all 4 fields: the node's cell / offset bookkeeping is done once, the
  // slab entry goes out as one vector store. Same cell order per field as the per-(node, field) loop.
  {
    if (!(GLS_ABL & 2)) {
      for (int n = tid; n < BN3; n += blockDim.x) {
        const int Xn = n % BN, Yn = (n / BN) % BN, Zn = n / (BN * BN);
        Real s[4] = {0., 0., 0., 0.};
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
              const Real *o = Out(cx + 2 * cy + 4 * cz, 0) + ax + K1 * (ay + K1 * az);
#pragma unroll
              for (int f = 0; f < 4; ++f) s[f] += lds(o + f * N3, zm);
            }
          }
        }
        const int node = sNode[n];
        const int64_t gi[4] = {(int64_t)node * 3, (int64_t)node * 3 + 1, (int64_t)node * 3 + 2, voff + node};
        const bool interior = Xn > 0 && Xn < BN - 1 && Yn > 0 && Yn < BN - 1 && Zn > 0 && Zn < BN - 1;
        if (interior) {
          if (MODE == MODE_JVQ && P.jx) {  // fused damped-Jacobi sweep
            const unsigned m = P.vmask ? P.vmask[node] : 0u;
#pragma unroll
            for (int f = 0; f < 4; ++f) {
              const bool con = f < 3 && ((m >> f) & 1u);
              const double x = P.jx[gi[f]], dd = P.jd[gi[f]];
              P.jx[gi[f]] = x + P.jomega * (P.jb[gi[f]] - (con ? dd * x : (double)s[f])) / dd;
            }
          } else if (MODE == MODE_JVQ && P.rb) {
#pragma unroll
            for (int f = 0; f < 4; ++f) Yout[gi[f]] = P.rb[gi[f]] - (double)s[f];
          } else {
#pragma unroll
            for (int f = 0; f < 4; ++f) Yout[gi[f]] = s[f];
          }
        } else if (use_slab) {  // this brick's partial sums of a brick-boundary node (k_slab_sum)
          const int64_t si = ((int64_t)brick * C::NBND + bnd_index<BN>(Xn, Yn, Zn)) * 4;
          if (std::is_same<Real, float>::value && P.slabf) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<f4 *>(P.slabf + si) = f4{(float)s[0], (float)s[1], (float)s[2], (float)s[3]};
          } else {
            typedef double d2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<d2 *>(P.slab + si) = d2{(double)s[0], (double)s[1]};
            *reinterpret_cast<d2 *>(P.slab + si + 2) = d2{(double)s[2], (double)s[3]};
          }
        } else {
#pragma unroll
          for (int f = 0; f < 4; ++f) atomicAdd(&Yout[gi[f]], (double)s[f]);
        }
      }
      return;
    }
  }
#endif
  for (int t = tid; t < BN3 * 4; t += blockDim.x) {
    const int n = t >> 2, fld = t & 3;
    const int Xn = n % BN, Yn = (n / BN) % BN, Zn = n / (BN * BN);
    Real s = 0.;
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
          s += lds(Out(cx + 2 * cy + 4 * cz, fld) + ax + K1 * (ay + K1 * az), zm);
        }
      }
    }
    const int node = sNode[n];
    const int64_t gi = fld < 3 ? (int64_t)node * 3 + fld : voff + node;
    const bool interior = Xn > 0 && Xn < BN - 1 && Yn > 0 && Yn < BN - 1 && Zn > 0 && Zn < BN - 1;
    auto complete = [&](double tot) {  // the node's full row: store it (or the fused update)
      if (MODE == MODE_JVQ && P.jx) {  // fused damped-Jacobi sweep: no other brick reads this x later
        const bool con = fld < 3 && P.vmask && ((P.vmask[node] >> fld) & 1u);
        const double x = P.jx[gi], dd = P.jd[gi];
        P.jx[gi] = x + P.jomega * (P.jb[gi] - (con ? dd * x : tot)) / dd;
      } else if (MODE == MODE_JVQ && P.rb) {
        Yout[gi] = P.rb[gi] - tot;
      } else {
        Yout[gi] = tot;
      }
    };
    if (GLS_ABL & 2) {
      if (s == Real(123.5)) Yout[gi] = s;
    } else if (interior) {
      if (MODE == MODE_JVQ && (P.jx || P.rb)) complete((double)s);
      else Yout[gi] = s;
#ifdef GLS_BRICK_COLORS_BUILD
    } else if (colored) {  // running sum across colors, in color order
      const unsigned cm = P.ncolor[node];
      const bool first = (cm & ((1u << P.color) - 1u)) == 0u, last = (cm >> (P.color + 1)) == 0u;
      double tot = (double)s;
      if (!first) tot += P.acc[gi];
      if (last) complete(tot);
      else P.acc[gi] = tot;
#endif
    } else if (use_slab) {  // brick-boundary node: this brick's partial sum, summed per node by k_slab_sum
      const int64_t si = ((int64_t)brick * C::NBND + bnd_index<BN>(Xn, Yn, Zn)) * 4 + fld;
      if (std::is_same<Real, float>::value && P.slabf) P.slabf[si] = (float)s;
      else P.slab[si] = (double)s;
    } else {
      atomicAdd(&Yout[gi], (double)s);
    }
  }
}

template <int K, typename Real = double>
size_t brick_lds_bytes(int mode) {
  using C = BrickCfg<K>;
  const bool cached = mode == MODE_JVQ;
  const int NF = cached ? (kQdLite ? 7 : 4) : (mode == MODE_JV ? 11 : 7);
  const size_t cs = mode == MODE_JVQ ? StageLayout<K, Real, MODE_JVQ>::CS
                    : (mode == MODE_RESIDUAL ? StageLayout<K, Real, MODE_RESIDUAL>::CS
                                             : StageLayout<K, Real, MODE_LIN>::CS);
  return sizeof(Real) * ((size_t)NF * C::BN3P + (size_t)8 * cs + (size_t)8 * C::NO * C::N3) + sizeof(int) * (size_t)C::BN3;
}

template <int K>
size_t brick_qdata_doubles(int n_cells) {
  using C = BrickCfg<K>;
  if (K == 2) return (size_t)((n_cells / 8 + 2) / 3) * kQdpTriple;  // pencil layout: whole brick triples
  return (size_t)(n_cells / 8) * C::WAVES * kQDataBrick * C::CPW * C::N3;
}

template <int K>
hipError_t launch_brick_t(int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  using C = BrickCfg<K>;
  const int n_bricks = P.n_cells / 8;
  if (n_bricks <= 0) return hipSuccess;
  const size_t lds = brick_lds_bytes<K>(mode);
  const bool colored = P.bricks != nullptr && P.y != nullptr;  // MODE_LIN without y stores no rows
  const int nc = colored ? P.n_colors : 1;
  OpParams Q = P;
  if (!colored) Q.bricks = nullptr;
  // the Q2 J.v from the linearization: the pencil-dataflow kernel (gls_brick_pencil.hip)
  if (K == 2 && (mode == MODE_JVQ || mode == MODE_RESIDUAL || mode == MODE_LIN) && !colored && pencil_enabled()) {
    const hipError_t e = mode == MODE_JVQ ? launch_pencil_jv(Q, T, s, false)
                         : mode == MODE_RESIDUAL ? launch_pencil_residual(Q, T, s) : launch_pencil_lin(Q, T, s);
    if (e != hipErrorNotSupported) return e;
  }
  for (int col = 0; col < nc; ++col) {
    Q.color = col;
    const int nb = colored ? P.color_off[col + 1] - P.color_off[col] : P.subset ? P.subset_n : n_bricks;
    if (nb <= 0) continue;
    if (mode == MODE_JV)
      hipLaunchKernelGGL((gls_brick_kernel<K, MODE_JV>), dim3(nb), dim3(C::THREADS), lds, s, Q, T);
    else if (mode == MODE_JVQ)
      hipLaunchKernelGGL((gls_brick_kernel<K, MODE_JVQ>), dim3(nb), dim3(C::THREADS), lds, s, Q, T);
    else if (mode == MODE_LIN)
      hipLaunchKernelGGL((gls_brick_kernel<K, MODE_LIN>), dim3(nb), dim3(C::THREADS), lds, s, Q, T);
    else
      hipLaunchKernelGGL((gls_brick_kernel<K, MODE_RESIDUAL>), dim3(nb), dim3(C::THREADS), lds, s, Q, T);
  }
  return hipGetLastError();
}

// J e_j for j in [j0, j0 + nprobe) into Y[(j - j0) * n_dofs + :] (Y zeroed by the caller)
template <int K>
hipError_t launch_brick_probe_t(const OpParams &P0, const Tables1D &T, int64_t j0, int nprobe, hipStream_t s) {
  using C = BrickCfg<K>;
  const int n_bricks = P0.n_cells / 8;
  if (n_bricks <= 0 || nprobe <= 0) return hipSuccess;
  OpParams P = P0;
  P.n_probe = nprobe;
  P.probe_base = j0;
  P.bricks = nullptr;
  hipLaunchKernelGGL((gls_brick_kernel<K, MODE_JVQ>), dim3((unsigned)((int64_t)n_bricks * nprobe)), dim3(C::THREADS),
                     brick_lds_bytes<K>(MODE_JVQ), s, P, T);
  return hipGetLastError();
}
// Kernel choice per element order (measured at 128^3, profiles/r01_jv_kernel_ab.txt):
//   Q1: the persistent wave-per-brick kernel (gls_brick_wave.hip: one round of 8 cells fills all
//       64 lanes) for every mode;
//   Q2: the workgroup-per-brick kernel here (the wave kernel at 3 waves / SIMD, and a variant
//       interleaving two fields per sweep stage, both measured slower: LDS-issue bound).
// The Q2 linearization layout is the same in all three kernels.
static int brick_impl(int k) { return k == 1 ? 1 : 0; }  // 0 this file, 1 wave kernel

hipError_t launch_brick_probe(int k, const OpParams &P, const Tables1D &T, int64_t j0, int nprobe, hipStream_t s) {
  if (brick_impl(k) == 1) return launch_brick_wave_probe(k, P, T, j0, nprobe, s);
  if (k == 1) return launch_brick_probe_t<1>(P, T, j0, nprobe, s);
  if (k == 2) return launch_brick_probe_t<2>(P, T, j0, nprobe, s);
  return hipErrorNotSupported;
}

// FP32 J.v from the FP32 copy of the linearization (P.qdf): the multigrid smoother's operator
// (mixed-precision preconditioner; v and y stay FP64 vectors, arithmetic and LDS in FP32)
template <int K>
hipError_t launch_brick_jv_f32_t(const OpParams &P, const Tables1D &T, hipStream_t s) {
  using C = BrickCfg<K>;
  const int n_bricks = P.n_cells / 8;
  if (n_bricks <= 0) return hipSuccess;
  if (!P.qdf || P.n_probe > 0) return hipErrorInvalidValue;
  if (K == 2 && !P.bricks && pencil_enabled()) {
    const hipError_t e = launch_pencil_jv(P, T, s, true);
    if (e != hipErrorNotSupported) return e;
  }
  const int nc = P.bricks ? P.n_colors : 1;
  OpParams Q = P;
  for (int col = 0; col < nc; ++col) {
    Q.color = col;
    const int nb = P.bricks ? P.color_off[col + 1] - P.color_off[col] : n_bricks;
    if (nb <= 0) continue;
    hipLaunchKernelGGL((gls_brick_kernel<K, MODE_JVQ, float>), dim3(nb), dim3(C::THREADS),
                       (brick_lds_bytes<K, float>(MODE_JVQ)), s, Q, T);
  }
  return hipGetLastError();
}
hipError_t launch_brick_jv_f32(int k, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (brick_impl(k) == 1) return launch_brick_wave_jv_f32(k, P, T, s);
  if (k == 1) return launch_brick_jv_f32_t<1>(P, T, s);
  if (k == 2) return launch_brick_jv_f32_t<2>(P, T, s);
  return hipErrorNotSupported;
}

__global__ void k_to_f32(const double *__restrict__ a, float *__restrict__ b, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    b[i] = (float)__builtin_nontemporal_load(a + i);
}
hipError_t vec_to_f32(const double *a, float *b, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(k_to_f32, dim3((unsigned)blocks), dim3(256), 0, s, a, b, n);
  return hipGetLastError();
}

__global__ void k_from_f32(const float *__restrict__ a, double *__restrict__ b, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = (double)a[i];
}
hipError_t vec_from_f32(const float *a, double *b, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(k_from_f32, dim3((unsigned)blocks), dim3(256), 0, s, a, b, n);
  return hipGetLastError();
}

int brick_boundary_nodes(int k) { return k == 1 ? BrickCfg<1>::NBND : (k == 2 ? BrickCfg<2>::NBND : 0); }

// y[node] (4 fields) = sum of the bricks' partial sums over the node's slab slots (fixed order:
// deterministic, no atomics). One thread per brick-boundary node.
// S = double / float (FP32 smoother slabs, summed in FP64). With J (fused Jacobi sweep) the node's
// row of y = A v is not stored: x <- x + omega (b - y) / d, y = d x on zero_constraints components.
template <typename S>
struct SlabQuad;
template <>
struct SlabQuad<double> {
  typedef double d2 __attribute__((ext_vector_type(2)));
  __device__ static void load(const double *p, double &a, double &b, double &c, double &d) {
    const d2 *e = reinterpret_cast<const d2 *>(p);
#if GLS_SLAB_NT
    const d2 u = __builtin_nontemporal_load(e), v = __builtin_nontemporal_load(e + 1);
#else
    const d2 u = e[0], v = e[1];
#endif
    a = u.x, b = u.y, c = v.x, d = v.y;
  }
};
template <>
struct SlabQuad<float> {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __device__ static void load(const float *p, double &a, double &b, double &c, double &d) {
#if GLS_SLAB_NT
    const f4 u = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(p));
#else
    const f4 u = *reinterpret_cast<const f4 *>(p);
#endif
    a = u.x, b = u.y, c = u.z, d = u.w;
  }
};
template <typename S, bool J>
__global__ void k_slab_sum(const S *__restrict__ slab, const int32_t *__restrict__ nodes,
                           const int32_t *__restrict__ off, const int32_t *__restrict__ slots, int64_t n_sum,
                           int64_t voff, double *__restrict__ y, const uint8_t *__restrict__ vmask,
                           const double *__restrict__ jb, const double *__restrict__ jd, double jomega,
                           const double *__restrict__ rb) {
  const int blk = GLS_SLAB_XCD ? xcd_swizzle((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const int64_t i = (int64_t)blk * blockDim.x + threadIdx.x;
  if (i >= n_sum) return;
  double s[4] = {0., 0., 0., 0.};
#if GLS_SLAB_INFLIGHT
  // a hex-mesh node lies in at most 8 bricks: all slot indices, then all slab entries in flight at
  // once (one dependent-load round trip instead of one per slot); summed in the same slot order
  const int j0 = off[i], cnt = off[i + 1] - j0;
  int sl[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) sl[t] = t < cnt ? slots[j0 + t] : 0;
  double e[8][4];
#pragma unroll
  for (int t = 0; t < 8; ++t)
    if (t < cnt) SlabQuad<S>::load(slab + (int64_t)sl[t] * 4, e[t][0], e[t][1], e[t][2], e[t][3]);
#pragma unroll
  for (int t = 0; t < 8; ++t)
    if (t < cnt) {
      s[0] += e[t][0];
      s[1] += e[t][1];
      s[2] += e[t][2];
      s[3] += e[t][3];
    }
  for (int j = j0 + 8; j < j0 + cnt; ++j) {  // not reached on hex meshes
    double a, b, c, d;
    SlabQuad<S>::load(slab + (int64_t)slots[j] * 4, a, b, c, d);
    s[0] += a;
    s[1] += b;
    s[2] += c;
    s[3] += d;
  }
#else
  for (int j = off[i]; j < off[i + 1]; ++j) {
    double a, b, c, d;
    SlabQuad<S>::load(slab + (int64_t)slots[j] * 4, a, b, c, d);
    s[0] += a;
    s[1] += b;
    s[2] += c;
    s[3] += d;
  }
#endif
  const int64_t node = nodes[i];
  const int64_t gi[4] = {node * 3, node * 3 + 1, node * 3 + 2, voff + node};
  if constexpr (J) {
    const unsigned m = vmask ? vmask[node] : 0u;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const double x = y[gi[f]], dd = jd[gi[f]];
      y[gi[f]] = x + jomega * (jb[gi[f]] - ((f < 3 && ((m >> f) & 1u)) ? dd * x : s[f])) / dd;
    }
  } else {
    if (rb) {
#pragma unroll
      for (int f = 0; f < 4; ++f) y[gi[f]] = rb[gi[f]] - s[f];
    } else {
#pragma unroll
      for (int f = 0; f < 4; ++f) y[gi[f]] = s[f];
    }
  }
}
hipError_t brick_slab_sum(const double *slab, const int32_t *nodes, const int32_t *off, const int32_t *slots,
                          int64_t n_sum, int64_t n_vnodes, double *y, hipStream_t s) {
  if (n_sum <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_slab_sum<double, false>), dim3((unsigned)((n_sum + 255) / 256)), dim3(256), 0, s, slab, nodes,
                     off, slots, n_sum, 3 * n_vnodes, y, nullptr, nullptr, nullptr, 0.0, nullptr);
  return hipGetLastError();
}
hipError_t brick_slab_sum_ex(const double *slab, const float *slabf, const int32_t *nodes, const int32_t *off,
                             const int32_t *slots, int64_t n_sum, int64_t n_vnodes, double *y, const uint8_t *vmask,
                             const double *jb, const double *jd, double jomega, hipStream_t s, const double *rb) {
  if (n_sum <= 0) return hipSuccess;
  const dim3 g((unsigned)((n_sum + 255) / 256)), b(256);
  const int64_t voff = 3 * n_vnodes;
  if (slabf) {
    if (jb) hipLaunchKernelGGL((k_slab_sum<float, true>), g, b, 0, s, slabf, nodes, off, slots, n_sum, voff, y, vmask, jb, jd, jomega, rb);
    else hipLaunchKernelGGL((k_slab_sum<float, false>), g, b, 0, s, slabf, nodes, off, slots, n_sum, voff, y, vmask, jb, jd, jomega, rb);
  } else {
    if (jb) hipLaunchKernelGGL((k_slab_sum<double, true>), g, b, 0, s, slab, nodes, off, slots, n_sum, voff, y, vmask, jb, jd, jomega, rb);
    else hipLaunchKernelGGL((k_slab_sum<double, false>), g, b, 0, s, slab, nodes, off, slots, n_sum, voff, y, vmask, jb, jd, jomega, rb);
  }
  return hipGetLastError();
}
// The same node sums on the uniform hyper_cube (structured lattice: lexicographic nodes, Morton
// bricks, no periodic wrap; checked by the host, build_slab_map): no node / offset / slot arrays. A
// thread's node follows from its (plane, index) and its slots from the node's lattice coordinates:
// per direction the brick(s) whose surface holds it (two where the coordinate is a brick boundary),
// slot = brick * NBND + bnd_index(local coordinates). The <= 8 slots are sorted so that the sum runs
// in ascending slot order, exactly the order of the CSR map (bitwise equal results). One dependent
// load round (the slab entries) instead of three, and y stored row by row.
__device__ __forceinline__ uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
  uint32_t m = 0;
  for (int b = 0; b < 10; ++b)
    m |= (((x >> b) & 1u) << (3 * b)) | (((y >> b) & 1u) << (3 * b + 1)) | (((z >> b) & 1u) << (3 * b + 2));
  return m;
}
template <typename S, bool J, int K>
__global__ void __launch_bounds__(256) k_slab_sum_cube(const S *__restrict__ slab, int nb1, int64_t voff,
                                                       double *__restrict__ y, const uint8_t *__restrict__ vmask,
                                                       const double *__restrict__ jb, const double *__restrict__ jd,
                                                       double jomega, const double *__restrict__ rb,
                                                       double *__restrict__ x0) {
  constexpr int BN = 2 * K + 1, P2 = 2 * K, NBND = BN * BN * BN - (BN - 2) * (BN - 2) * (BN - 2);
  const int NX = P2 * nb1 + 1;
  int bx = blockIdx.x, Z = blockIdx.y;
  if (GLS_SLAB_XCD) {  // XCD-aware: each XCD walks a contiguous range of planes
    const int lin = xcd_swizzle((int)(blockIdx.x + gridDim.x * blockIdx.y), (int)(gridDim.x * gridDim.y));
    bx = lin % (int)gridDim.x;
    Z = lin / (int)gridDim.x;
  }
  const bool zs = Z % P2 == 0;
  const int64_t t = (int64_t)bx * blockDim.x + threadIdx.x;
  // surface nodes of plane Z: all of it when Z is a brick boundary, else the full rows Y % 2K == 0
  // followed by the brick-boundary columns X % 2K == 0 of the other rows
  int X, Y;
  const int ns = nb1 + 1;  // brick-boundary coordinates per direction
  if (zs) {
    if (t >= (int64_t)NX * NX) return;
    X = (int)(t % NX);
    Y = (int)(t / NX);
  } else {
    const int64_t full = (int64_t)ns * NX, sparse = (int64_t)(NX - ns) * ns;
    if (t >= full + sparse) return;
    if (t < full) {
      X = (int)(t % NX);
      Y = (int)(t / NX) * P2;
    } else {
      const int64_t u = t - full;
      const int r = (int)(u / ns);  // r-th row that is not a brick boundary
      X = (int)(u % ns) * P2;
      Y = (r / (P2 - 1)) * P2 + 1 + r % (P2 - 1);
    }
  }
  // per direction: (brick coordinate, local coordinate) pairs holding the lattice coordinate
  int bc[3][2], lc[3][2], nc[3];
  const int co[3] = {X, Y, Z};
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int x = co[d];
    if (x % P2 == 0 && x > 0 && x < NX - 1) {
      nc[d] = 2;
      bc[d][0] = x / P2 - 1;
      lc[d][0] = P2;
      bc[d][1] = x / P2;
      lc[d][1] = 0;
    } else {
      nc[d] = 1;
      bc[d][0] = min(x / P2, nb1 - 1);
      lc[d][0] = x - P2 * bc[d][0];
      bc[d][1] = bc[d][0];
      lc[d][1] = lc[d][0];
    }
  }
  int64_t sl[8];
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool on = i < nc[0] && j < nc[1] && k < nc[2];
        const int64_t s = (int64_t)morton3(bc[0][i], bc[1][j], bc[2][k]) * NBND + bnd_index<BN>(lc[0][i], lc[1][j], lc[2][k]);
        sl[i + 2 * j + 4 * k] = on ? s : INT64_MAX;
        cnt += on;
      }
  // ascending slot order (sorting network on 8 keys; absent slots sort last)
  auto cs = [&](int a, int b) {
    const int64_t lo = min(sl[a], sl[b]), hi = max(sl[a], sl[b]);
    sl[a] = lo;
    sl[b] = hi;
  };
  cs(0, 1); cs(2, 3); cs(4, 5); cs(6, 7);
  cs(0, 2); cs(1, 3); cs(4, 6); cs(5, 7);
  cs(1, 2); cs(5, 6); cs(0, 4); cs(3, 7);
  cs(1, 5); cs(2, 6);
  cs(1, 4); cs(3, 6);
  cs(2, 4); cs(3, 5);
  cs(3, 4);
  double e[8][4];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (q < cnt) SlabQuad<S>::load(slab + sl[q] * 4, e[q][0], e[q][1], e[q][2], e[q][3]);
  double s[4] = {0., 0., 0., 0.};
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (q < cnt) {
      s[0] += e[q][0];
      s[1] += e[q][1];
      s[2] += e[q][2];
      s[3] += e[q][3];
    }
  const int64_t node = X + (int64_t)NX * (Y + (int64_t)NX * Z);
  const int64_t gi[4] = {node * 3, node * 3 + 1, node * 3 + 2, voff + node};
  if constexpr (J) {
    const unsigned m = vmask ? vmask[node] : 0u;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const double x = y[gi[f]], dd = jd[gi[f]];
      y[gi[f]] = x + jomega * (jb[gi[f]] - ((f < 3 && ((m >> f) & 1u)) ? dd * x : s[f])) / dd;
    }
  } else if (rb) {
#pragma unroll
    for (int f = 0; f < 4; ++f) y[gi[f]] = rb[gi[f]] - s[f];
    if (x0) {  // the fused first Jacobi sweep's x at this surface node (pencil J.v, OpParams::jx0)
#pragma unroll
      for (int f = 0; f < 4; ++f) x0[gi[f]] = 0.0 + jomega * rb[gi[f]] / jd[gi[f]];
    }
  } else {
#pragma unroll
    for (int f = 0; f < 4; ++f) y[gi[f]] = s[f];
  }
}
// nb1 > 0: the structured form (nb1 bricks per direction) instead of the node / offset / slot map
hipError_t brick_slab_sum_cube(int k, int nb1, const double *slab, const float *slabf, int64_t n_vnodes, double *y,
                               const uint8_t *vmask, const double *jb, const double *jd, double jomega, hipStream_t s,
                               const double *rb, double *x0) {
  if (nb1 <= 0 || (k != 1 && k != 2)) return hipErrorInvalidValue;
  if (x0 && (!rb || !jd || jb)) return hipErrorInvalidValue;
  const int NX = 2 * k * nb1 + 1;
  const dim3 g((unsigned)(((int64_t)NX * NX + 255) / 256), (unsigned)NX), b(256);
  const int64_t voff = 3 * n_vnodes;
#define GLS_SLAB_CUBE(KK)                                                                                                   \
  if (slabf) {                                                                                                              \
    if (jb) hipLaunchKernelGGL((k_slab_sum_cube<float, true, KK>), g, b, 0, s, slabf, nb1, voff, y, vmask, jb, jd, jomega, rb, x0);  \
    else hipLaunchKernelGGL((k_slab_sum_cube<float, false, KK>), g, b, 0, s, slabf, nb1, voff, y, vmask, jb, jd, jomega, rb, x0);   \
  } else {                                                                                                                  \
    if (jb) hipLaunchKernelGGL((k_slab_sum_cube<double, true, KK>), g, b, 0, s, slab, nb1, voff, y, vmask, jb, jd, jomega, rb, x0); \
    else hipLaunchKernelGGL((k_slab_sum_cube<double, false, KK>), g, b, 0, s, slab, nb1, voff, y, vmask, jb, jd, jomega, rb, x0);  \
  }
  if (k == 1) {
    GLS_SLAB_CUBE(1)
  } else {
    GLS_SLAB_CUBE(2)
  }
#undef GLS_SLAB_CUBE
  return hipGetLastError();
}

bool brick_fused_jacobi_supported(int k) { return brick_impl(k) == 0 && (k == 1 || k == 2); }
#ifdef GLS_BRICK_COLORS_BUILD
bool brick_colors_supported(int k) { return brick_impl(k) == 0 && (k == 1 || k == 2); }
#else
bool brick_colors_supported(int) { return false; }
#endif
bool brick_subset_supported(int k) { return brick_impl(k) == 0 && (k == 1 || k == 2); }

size_t brick_qdata_size(int k, int n_cells) {
  if (brick_impl(k) == 1) return brick_wave_qdata_size(k, n_cells);
  return k == 1 ? brick_qdata_doubles<1>(n_cells) : (k == 2 ? brick_qdata_doubles<2>(n_cells) : 0);
}

hipError_t launch_brick_kernel(int k, int mode, const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (mode == MODE_DIAG) return hipErrorNotSupported;
  if (brick_impl(k) == 1) return launch_brick_wave(k, mode, P, T, s);
  if (k == 1) return launch_brick_t<1>(mode, P, T, s);
  if (k == 2) return launch_brick_t<2>(mode, P, T, s);
  return hipErrorNotSupported;
}

}  // namespace gls
