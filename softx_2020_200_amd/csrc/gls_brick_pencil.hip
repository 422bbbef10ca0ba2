// gls_brick_pencil.hip — the Q2 brick J.v (MODE_JVQ, FP64 outer operator and FP32 smoother) in the
// "pencil" dataflow: one lane holds a line of 3 values along z for every field it works on.
//
// Why: the lane-per-point brick kernel (gls_brick_kernels.hip) is bound by its LDS
// stream -- every stage array is written once (ds_write_b64, ~6 LDS cycles per wave instruction) and
// read three times (each lane reads the whole line its output needs). Here a lane owns the z-line of
// its (qx, qy) column of a cell (9 lanes per cell, 6 cells per wave, 54 of 64 lanes):
//   forward : x sweep from the brick array (uniform coefficients; per lane one x-line of the node
//             lattice, all 3 qx outputs) -> LDS -> y sweep (each lane reads its qx slab, 9 values per
//             array) -> kept in REGISTERS -> z sweep in registers at each qz;
//   backward: z-transposed contraction accumulated in registers while the pointwise runs over qz ->
//             LDS -> y-transposed -> LDS -> x-transposed -> per-cell node values (Out) -> brick sums.
// The Y stage (4 arrays per velocity field) and the test coefficients (16 values per point) never go
// through LDS, and no element is read three times: per cell ~945 LDS element writes and ~1540 reads
// against ~1780 and ~5350 for the lane-per-point kernel. The sweeps' coefficients are uniform over the
// wave except in the y sweep (row of the lane's qy, from an LDS table).
//
// Workgroup = 3 consecutive (XCD-swizzled) bricks = 24 cells, 4 waves of 6 cells; the brick-interior
// nodes are stored directly, brick-surface nodes go to the brick's slab (k_slab_sum), exactly as the
// lane-per-point kernel does (same slab slots, same fixed per-node summation order: bitwise equal
// sums per brick node). The linearization is read from the pencil layout (qdp_base) that MODE_LIN
// writes: per (qz, value) one contiguous row of 54 entries per wave.
//
// The pointwise algebra restates gls_navier_stokes.cc:548-622 (the Jacobian's action, SURVEY.md
// Appendix A) with the same operation order per term as gls_brick_kernels.hip MODE_JVQ.
#include "gls_brick_common.hpp"
#include "gls_common.hpp"
#include "gls_launch.hpp"

#include <cstdlib>
#include <type_traits>

#ifndef GLS_PENCIL_WPE64
#define GLS_PENCIL_WPE64 2  // FP64: ~230 VGPRs -> 2 waves / SIMD (2 workgroups per CU)
#endif
#ifndef GLS_PENCIL_PIPE
#define GLS_PENCIL_PIPE 1  // J.v linearization batches requested one component ahead: bit 0 FP64, bit 1 FP32
#endif
#ifndef GLS_PENCIL_NT
#define GLS_PENCIL_NT 0  // 1: J.v linearization rows read non-temporally (measured slower: 2.61 / 1.36 ms FP64 / FP32 plain vs 2.65 / 1.44 NT)
#endif
#ifndef GLS_PENCIL_WPE32
#define GLS_PENCIL_WPE32 4  // FP32: <= 128 VGPRs -> 4 waves / SIMD
#endif

namespace gls {

template <typename Real, bool JV>
struct PencilCfg {
  static constexpr int K1 = 3, N3 = 27, BN = 5, BN3 = 125, BN3P = 128, NBND = 98;
  static constexpr int CPW = 6, WAVES = 4, THREADS = 256, CPG = 24, BPG = 3;
  static constexpr bool F64 = sizeof(Real) == 8;
  // LDS layout (strides in Reals). The J.v's (JV) are chosen against bank conflicts by
  // tools/lds_bank_sim.py (the MI355X_MICROARCH.md §LDS lane groups; modelled LDS-array cycles per wave
  // J.v FP64 2296 -> 1594, FP32 1282 -> 1043, conflict-free 1049 / 601: J.v 2.61 -> 2.53 ms, FP32
  // 1.37 -> 1.35 ms). The residual / linearization keep the first layout: the model's best within the
  // 80 KB of 2 workgroups per CU (2554 -> 1828) measured no faster (profiles/r04_ab_lds_layout.txt).
  // brick arrays: node (X, Y, Z) at X + SY Y + SZ Z, field stride FB
  static constexpr int SY = 5, SZ = 25, FB = JV ? (F64 ? 131 : 129) : 128;
  // forward X arrays: [arr * XA + qx * XS + j + 3 k] (slabs 16-B aligned: read as one slab per lane)
  static constexpr int XS = JV ? (F64 ? 12 : 16) : 10, XA = 3 * XS;
  // backward Z arrays [m * ZA + qx * ZS + az * ZAZ + qy], W arrays at WB: [m * WA + az * WAZ + 3 ay + qx]
  static constexpr int ZS = JV ? (F64 ? 12 : 10) : 10, ZAZ = 3, ZA = 3 * ZS, WB = 3 * ZA, WAZ = 9,
                       WA = 28;
  static constexpr int CSF = 3 * XA, CSB = WB + 2 * WA;
  static constexpr int CS0 = CSF > CSB ? CSF : CSB;
  static constexpr int CS = JV ? (F64 ? 190 : 164) : CS0 + 4;  // per-cell stage stride
  static constexpr int NO = 4;                                 // test fields
  static constexpr int OF = 27, OC = JV ? 123 : NO * OF;  // cell node values: [cell * OC + f * OF + 9 az + 3 ay + ax]
  static_assert(CS >= CS0 && OC >= NO * OF && FB >= 4 * SZ + 4 * SY + 5, "pencil LDS layout");
};

// brick fields gathered per brick: J.v: v (3) + v_p; residual: u (3), p, the history H = sum_k alpha_k u^(k) (3)
constexpr int pencil_fields(int mode) { return mode == MODE_JVQ ? 4 : 7; }
template <typename Real, bool JV>
size_t pencil_lds_bytes_t(int mode) {
  using C = PencilCfg<Real, JV>;
  return sizeof(Real) * ((size_t)C::BPG * pencil_fields(mode) * C::FB + (size_t)C::WAVES * C::CPW * C::CS +
                         (size_t)C::CPG * C::OC) +
         sizeof(int) * (size_t)C::BPG * C::BN3P;
}
template <typename Real>
size_t pencil_lds_bytes(int mode) {
  return mode == MODE_JVQ ? pencil_lds_bytes_t<Real, true>(mode) : pencil_lds_bytes_t<Real, false>(mode);
}

// the Q2 1D tables in the kernel's precision (kernel argument -> scalar registers): [q][node]
template <typename Real>
struct PencilTab {
  Real V[3][3], D[3][3], S[3][3], w[3], xi[3];
};

// GEN: the forcing term and the SRF source are compiled in (an instantiation without them is the hot
// path: their per-point loads and terms cost the residual ~50 VGPRs of spills)
// FOREST: an FP32 launch on forest bricks (subset list); OS: the Oseen (Picard) operator of the FP32 smoother
// (MODE_JVQ: no (grad u) v terms, no tau (v . grad phi) R_s term; reads u and tau of the linearization only)
template <typename Real, int MODE, bool GEN, bool FOREST = false, bool OS = false>
__global__ void __launch_bounds__(256, (std::is_same<Real, float>::value ? GLS_PENCIL_WPE32 : GLS_PENCIL_WPE64))
    gls_pencil_kernel(const OpParams P, const PencilTab<Real> T) {
  static_assert(!OS || (MODE == MODE_JVQ && std::is_same<Real, float>::value), "Oseen operator: FP32 J.v only");
  using C = PencilCfg<Real, MODE == MODE_JVQ>;
  // MODE_RESLIN = MODE_RESIDUAL + MODE_LIN at one state (assemble_matrix_and_rhs); else MODE_JVQ
  constexpr bool RL = MODE == MODE_RESLIN, RES = MODE == MODE_RESIDUAL || RL, LIN = MODE == MODE_LIN || RL;
  constexpr bool ST = RES || LIN;  // state sweeps (u, p, H) instead of the cached linearization
  constexpr int BN = C::BN, BN3 = C::BN3, BN3P = C::BN3P, NF = pencil_fields(MODE);
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  constexpr int FB = C::FB, SY = C::SY, SZ = C::SZ;
  Real *const sB = reinterpret_cast<Real *>(smem_raw);            // [3 bricks][NF fields][FB]
  Real *const sS = sB + C::BPG * NF * FB;                          // [4 waves][6 cells][CS] stage arrays
  constexpr int CS = C::CS;
  Real *const sO = sS + C::WAVES * C::CPW * CS;                    // [24 cells][OC] cell node values
  int *const sNode = reinterpret_cast<int *>(sO + C::CPG * C::OC);  // [3][BN3P]
  __shared__ Real sRow[3 * 16];  // V, D, S rows [mat][q][4] for the y sweep's per-lane coefficients

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n_bricks = P.n_cells / 8;
  // brick-subset launches (the distributed split: interior / boundary bricks) for the FP64 operator,
  // as the lane-per-point kernel honours them
  const int32_t *const subset = (std::is_same<Real, double>::value || FOREST) ? P.subset : nullptr;
  const int n_items = subset ? P.subset_n : n_bricks;       // bricks of this launch
  const int n_groups = (n_items + 2) / 3;
  const int g = xcd_swizzle((int)blockIdx.x, n_groups);      // XCD-aware: contiguous Morton triples per XCD
  const int nbg = min(3, n_items - 3 * g);                   // bricks in this group (last one may be short)
  auto brick_of = [&](int bi) { return subset ? subset[3 * g + bi] : 3 * g + bi; };
  // first cell of a brick: 8 b on the cube; the listed cell on an adapted forest's sibling groups
  auto cell0 = [&](int b) -> int64_t { return P.brick_cell0 ? (int64_t)P.brick_cell0[b] : (int64_t)b * 8; };
  const int64_t voff = (int64_t)3 * P.n_vnodes;

  if (tid < 48) {
    const int mat = tid >> 4, r = (tid >> 2) & 3, cc = tid & 3;
    Real v = 0;
    if (r < 3 && cc < 3) v = mat == 0 ? T.V[r][cc] : mat == 1 ? T.D[r][cc] : T.S[r][cc];
    sRow[tid] = v;
  }
  // ---------------- per lane: cell c of this wave, (a, b) position in the cell's 3 x 3 pencil grid
  const bool act = lane < 9 * C::CPW;
  const int c = act ? lane / 9 : 0, rr = act ? lane % 9 : 0, pa = rr % 3, pb = rr / 3;
  const int cw = wave * C::CPW + c, bi = cw >> 3, ci = cw & 7;
  const bool valid = act && bi < nbg;
  const int brick = brick_of(valid ? bi : 0);
  const int cx = ci & 1, cy = (ci >> 1) & 1, cz = ci >> 2;
  const int64_t gcell = cell0(brick) + (valid ? ci : 0);
  const Real hx = (Real)P.geo[gcell * 4 + 0], hy = (Real)P.geo[gcell * 4 + 1], hz = (Real)P.geo[gcell * 4 + 2];
  const Real ihx = Real(1) / hx, ihy = Real(1) / hy, ihz = Real(1) / hz;
  const Real wxx = ihx * ihx, wyy = ihy * ihy, wzz = ihz * ihz;
  Real *const cellS = sS + (wave * C::CPW + c) * CS;
  // J.v: the lane's linearization rows (loaded in batches below)
  const Real *qrow = nullptr;
  if constexpr (!ST) {
    const Real *base = std::is_same<Real, double>::value ? reinterpret_cast<const Real *>(P.qd)
                                                          : reinterpret_cast<const Real *>(P.qdf);
    qrow = base + qdp_base(brick, valid ? ci : 0, pa + 3 * pb);
  }
  // ---------------- gather the group's brick nodes: v (masked: P v) or u, p, H, and the node ids
  for (int t = tid; t < C::BPG * BN3; t += C::THREADS) {
    const int bi = t / BN3, n = t % BN3;
    if (bi >= nbg) break;
    const int brick = brick_of(bi);
    const int X = n % BN, Y = (n / BN) % BN, Z = n / (BN * BN);
    const int cx = min(X / 2, 1), cy = min(Y / 2, 1), cz = min(Z / 2, 1);
    const int a = (X - 2 * cx) + 3 * ((Y - 2 * cy) + 3 * (Z - 2 * cz));
    const int node = P.cell_vnodes[(cell0(brick) + cx + 2 * cy + 4 * cz) * 27 + a];
    const int64_t i3 = (int64_t)node * 3;
    Real *b = sB + bi * NF * FB + X + SY * Y + SZ * Z;
    if constexpr (ST) {
      double h[3] = {0., 0., 0.};
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        if (P.n_hist > 0) h[cc] += P.alpha[1] * P.h1[i3 + cc];
        if (P.n_hist > 1) h[cc] += P.alpha[2] * P.h2[i3 + cc];
        if (P.n_hist > 2) h[cc] += P.alpha[3] * P.h3[i3 + cc];
      }
      b[0] = (Real)P.u[i3];
      b[FB] = (Real)P.u[i3 + 1];
      b[2 * FB] = (Real)P.u[i3 + 2];
      b[3 * FB] = (Real)P.u[voff + node];
      b[4 * FB] = (Real)h[0];
      b[5 * FB] = (Real)h[1];
      b[6 * FB] = (Real)h[2];
    } else {
      double v0, v1, v2, vp;
      if (P.jx0) {  // the first Jacobi sweep from 0: v = 0 + omega b / d (mg_jacobi_update's arithmetic)
        v0 = 0.0 + P.jomega * P.rb[i3] / P.jd[i3];
        v1 = 0.0 + P.jomega * P.rb[i3 + 1] / P.jd[i3 + 1];
        v2 = 0.0 + P.jomega * P.rb[i3 + 2] / P.jd[i3 + 2];
        vp = 0.0 + P.jomega * P.rb[voff + node] / P.jd[voff + node];
      } else {
        v0 = P.v[i3], v1 = P.v[i3 + 1], v2 = P.v[i3 + 2], vp = P.v[voff + node];
      }
      const unsigned m = P.vmask ? P.vmask[node] : 0u;
      b[0] = (m & 1u) ? Real(0) : (Real)v0;
      b[FB] = (m & 2u) ? Real(0) : (Real)v1;
      b[2 * FB] = (m & 4u) ? Real(0) : (Real)v2;
      b[3 * FB] = (Real)vp;
    }
    sNode[bi * BN3P + n] = node;
  }
  __syncthreads();


  // ---------------- forward sweeps of brick field f into Y registers ([k]: BB, BD, DB, L). kind 0: the
  // value only (BB); 1: value and gradient (BB, BD, DB; pressure); 2: velocity (+ L for the Laplacian)
  auto xsweep = [&](int f, int kind, int base) {
    const bool grad = kind >= 1, vel = kind == 2;
    // x sweep, lane (a, b) = (y node j, z node k): the brick's x-line of this cell at (j, k)
    const Real *F = sB + (bi < 3 ? bi : 0) * NF * FB + f * FB + 2 * cx + SY * (2 * cy + pa) + SZ * (2 * cz + pb);
    const Real f0 = F[0], f1 = F[1], f2 = F[2];
    Real *const X = cellS + base;
#pragma unroll
    for (int qx = 0; qx < 3; ++qx) {
      const Real xb = T.V[qx][0] * f0 + T.V[qx][1] * f1 + T.V[qx][2] * f2;
      const Real xd = grad ? T.D[qx][0] * f0 + T.D[qx][1] * f1 + T.D[qx][2] * f2 : Real(0);
      const int o = qx * C::XS + pa + 3 * pb;  // slab qx, entry (j, k) at j + 3 k
      const Real xs = vel ? T.S[qx][0] * f0 + T.S[qx][1] * f1 + T.S[qx][2] * f2 : Real(0);
      if (act) {  // lanes 54..63 mirror lane 0 and store nothing
        X[0 * C::XA + o] = xb;
        if (grad) X[1 * C::XA + o] = xd;
        if (vel) X[2 * C::XA + o] = xs;
      }
    }
  };
  // y sweep, lane (a, b) = (qx, qy): slab qx of each X array, all (j, k); the lane's V / D / S rows
  auto ysweep = [&](int kind, int base, Real (&BB)[3], Real (&BD)[3], Real (&DB)[3], Real (&LL)[3]) {
    const bool grad = kind >= 1, vel = kind == 2;
    const Real *rowp = sRow + pb * 4;
    const Real v0 = rowp[0], v1 = rowp[1], v2 = rowp[2];
    const Real d0 = rowp[16], d1 = rowp[17], d2 = rowp[18];
    const Real s0 = rowp[32], s1 = rowp[33], s2 = rowp[34];
    Real xb[9], xd[9], xs[9];
    const Real *sl = cellS + base + pa * C::XS;
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      xb[e] = sl[e];
      if (grad) xd[e] = sl[C::XA + e];
      if (vel) xs[e] = sl[2 * C::XA + e];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const Real b0 = xb[3 * k], b1 = xb[3 * k + 1], b2 = xb[3 * k + 2];
      BB[k] = v0 * b0 + v1 * b1 + v2 * b2;
      if (grad) {
        BD[k] = d0 * b0 + d1 * b1 + d2 * b2;
        DB[k] = v0 * xd[3 * k] + v1 * xd[3 * k + 1] + v2 * xd[3 * k + 2];
      }
      if (vel)
        LL[k] = wyy * (s0 * b0 + s1 * b1 + s2 * b2) + wxx * (v0 * xs[3 * k] + v1 * xs[3 * k + 1] + v2 * xs[3 * k + 2]);
    }
  };
  // forward sweeps of brick field f into Y registers ([k]: BB, BD, DB, L). kind 0: the value only (BB);
  // 1: value and gradient (BB, BD, DB; pressure); 2: velocity (+ L for the Laplacian)
  auto forward = [&](int f, int kind, Real (&BB)[3], Real (&BD)[3], Real (&DB)[3], Real (&LL)[3]) {
    xsweep(f, kind, 0);
    wave_sync();
    ysweep(kind, 0, BB, BD, DB, LL);
    wave_sync();  // the X arrays are rewritten by the next field
  };

  // z sweep helpers (uniform coefficients: qz, k are compile-time after unrolling)
  auto zval = [&](const Real (&y)[3], int qz) { return T.V[qz][0] * y[0] + T.V[qz][1] * y[1] + T.V[qz][2] * y[2]; };
  auto zder = [&](const Real (&y)[3], int qz) { return T.D[qz][0] * y[0] + T.D[qz][1] * y[1] + T.D[qz][2] * y[2]; };
  auto zsec = [&](const Real (&y)[3], int qz) { return T.S[qz][0] * y[0] + T.S[qz][1] * y[1] + T.S[qz][2] * y[2]; };

  const Real nu = (Real)P.nu, aj = (Real)P.alpha_jac;
  auto wsel = [&](int i) { return i == 0 ? T.w[0] : i == 1 ? T.w[1] : T.w[2]; };  // lane-varying index
  const Real wxy = wsel(pa) * wsel(pb) * hx * hy * hz;  // JxW / w[qz]
  const Real ihv[3] = {ihx, ihy, ihz};
  Real om[3] = {0, 0, 0};
  if (GEN && P.srf) { om[0] = (Real)P.omega[0]; om[1] = (Real)P.omega[1]; om[2] = (Real)P.omega[2]; }

  // backward stages of test field f from its z-transposed sums Z[m][az] (lane (qx, qy)):
  // LDS -> y-transposed (lane (qx, az)) -> LDS -> x-transposed (lane (ay, az)) -> Out
  Real *const outc = sO + cw * C::OC;
  // Z[m][az] -> Zs at cellS + zb: [m][qx][az][qy] = m * ZA + qx * ZS + 3 az + qy
  auto bwd_z = [&](const Real (&Z)[3][3], int zb) {
    if (act) {
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int az = 0; az < 3; ++az) cellS[zb + m * C::ZA + pa * C::ZS + C::ZAZ * az + pb] = Z[m][az];
    }
  };
  // lane (a, b) = (qx, az): y-transposed contraction of Zs (at zb) into Ws at wb: [m][az][ay][qx]
  auto bwd_w = [&](int zb, int wb) {
    const Real *Zs = cellS + zb;
    Real *Ws = cellS + wb;
    Real z[3][3];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int qy = 0; qy < 3; ++qy) z[m][qy] = Zs[m * C::ZA + pa * C::ZS + C::ZAZ * pb + qy];
#pragma unroll
    for (int ay = 0; ay < 3; ++ay) {
      const Real w0 = T.V[0][ay] * z[0][0] + T.V[1][ay] * z[0][1] + T.V[2][ay] * z[0][2] +
                      (T.D[0][ay] * z[2][0] + T.D[1][ay] * z[2][1] + T.D[2][ay] * z[2][2]);
      const Real w1 = T.V[0][ay] * z[1][0] + T.V[1][ay] * z[1][1] + T.V[2][ay] * z[1][2];
      if (act) {
        Ws[0 * C::WA + C::WAZ * pb + 3 * ay + pa] = w0;
        Ws[1 * C::WA + C::WAZ * pb + 3 * ay + pa] = w1;
      }
    }
  };
  // lane (a, b) = (ay, az): x-transposed contraction of Ws (at wb) into the cell's node values of field f
  auto bwd_out = [&](int f, int wb) {
    const Real *Ws = cellS + wb;
    Real w0[3], w1[3];
#pragma unroll
    for (int qx = 0; qx < 3; ++qx) {
      w0[qx] = Ws[C::WAZ * pb + 3 * pa + qx];
      w1[qx] = Ws[C::WA + C::WAZ * pb + 3 * pa + qx];
    }
    if (valid) {
#pragma unroll
      for (int ax = 0; ax < 3; ++ax)
        outc[f * C::OF + 9 * pb + 3 * pa + ax] =
            T.V[0][ax] * w0[0] + T.V[1][ax] * w0[1] + T.V[2][ax] * w0[2] +
            (T.D[0][ax] * w1[0] + T.D[1][ax] * w1[1] + T.D[2][ax] * w1[2]);
    }
  };
  auto backward = [&](int f, const Real (&Z)[3][3]) {
    bwd_z(Z, 0);
    wave_sync();
    bwd_w(0, C::WB);
    wave_sync();
    bwd_out(f, C::WB);
    wave_sync();  // the stage area is rewritten by the next field
  };

  // ---------------- brick reduction (fixed cell order per node) + scatter: one thread per brick node;
  // fused: the launch's damped-Jacobi / residual-form / FP32-slab options apply
  auto reduce_scatter = [&](double *yo, double *slo, bool fused) {
    for (int t = tid; t < C::BPG * BN3; t += C::THREADS) {
      const int rb_ = t / BN3, n = t % BN3;
      if (rb_ >= nbg) break;
      const int bk = brick_of(rb_);
      const int Xn = n % BN, Yn = (n / BN) % BN, Zn = n / (BN * BN);
      Real s[4] = {0, 0, 0, 0};
#pragma unroll
      for (int kz = 0; kz < 2; ++kz) {
        const int az = Zn - 2 * kz;
        if (az < 0 || az > 2) continue;
#pragma unroll
        for (int ky = 0; ky < 2; ++ky) {
          const int ay = Yn - 2 * ky;
          if (ay < 0 || ay > 2) continue;
#pragma unroll
          for (int kx = 0; kx < 2; ++kx) {
            const int ax = Xn - 2 * kx;
            if (ax < 0 || ax > 2) continue;
            const Real *o = sO + (rb_ * 8 + kx + 2 * ky + 4 * kz) * C::OC + ax + 3 * (ay + 3 * az);
#pragma unroll
            for (int f = 0; f < 4; ++f) s[f] += o[f * C::OF];
          }
        }
      }
      const int node = sNode[rb_ * BN3P + n];
      const int64_t gi[4] = {(int64_t)node * 3, (int64_t)node * 3 + 1, (int64_t)node * 3 + 2, voff + node};
      const bool interior = Xn > 0 && Xn < BN - 1 && Yn > 0 && Yn < BN - 1 && Zn > 0 && Zn < BN - 1;
      if (interior) {
        if (fused && P.jx) {  // fused damped-Jacobi sweep (interior nodes: no other brick reads this x)
          const unsigned m = P.vmask ? P.vmask[node] : 0u;
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            const bool con = f < 3 && ((m >> f) & 1u);
            const double x = P.jx[gi[f]], dd = P.jd[gi[f]];
            P.jx[gi[f]] = x + P.jomega * (P.jb[gi[f]] - (con ? dd * x : (double)s[f])) / dd;
          }
        } else if (fused && P.rb) {
#pragma unroll
          for (int f = 0; f < 4; ++f) yo[gi[f]] = P.rb[gi[f]] - (double)s[f];
          if (P.jx0) {
#pragma unroll
            for (int f = 0; f < 4; ++f) P.jx0[gi[f]] = 0.0 + P.jomega * P.rb[gi[f]] / P.jd[gi[f]];
          }
        } else {
#pragma unroll
          for (int f = 0; f < 4; ++f) yo[gi[f]] = s[f];
        }
      } else {  // this brick's partial sums of a brick-boundary node (summed per node by k_slab_sum)
        const int64_t si = ((int64_t)bk * C::NBND + bnd_index<BN>(Xn, Yn, Zn)) * 4;
        if (fused && std::is_same<Real, float>::value && P.slabf) {
          typedef float f4 __attribute__((ext_vector_type(4)));
          *reinterpret_cast<f4 *>(P.slabf + si) = f4{(float)s[0], (float)s[1], (float)s[2], (float)s[3]};
        } else {
          typedef double d2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<d2 *>(slo + si) = d2{(double)s[0], (double)s[1]};
          *reinterpret_cast<d2 *>(slo + si + 2) = d2{(double)s[2], (double)s[3]};
        }
      }
    }
  };

  // element-vector output (adapted forests: the ordered per-node sums of gather_element_vectors include
  // these cells' 27-node vectors with the per-cell kernel's; layout [cell][a * 3 + c | 81 + a])
  auto write_ev = [&]() {
    for (int t = tid; t < nbg * 8 * 27; t += C::THREADS) {
      const int rb_ = t / 216, r = t - rb_ * 216, ci_ = r / 27, a = r - ci_ * 27;
      const Real *o = sO + (rb_ * 8 + ci_) * C::OC + a;
      double *e = P.ev + (cell0(brick_of(rb_)) + ci_) * 108;
      e[a * 3] = (double)o[0];
      e[a * 3 + 1] = (double)o[C::OF];
      e[a * 3 + 2] = (double)o[2 * C::OF];
      e[81 + a] = (double)o[3 * C::OF];
    }
  };

  if constexpr (ST) {
    // ---------------- residual (assemble_rhs, gls_navier_stokes.cc:391-516) / linearization (MODE_LIN:
    // u, grad u, tau, R_s per point into the pencil rows, then the Jacobian diagonal): values of u, H
    // and p, grad p
    Real uq[3][3], Ttq[3][3], pq[3], gp[3][3];
    {
      Real dz[3];
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        Real bb[3], hb[3];
        forward(cc, 0, bb, dz, dz, dz);
        forward(4 + cc, 0, hb, dz, dz, dz);
#pragma unroll
        for (int qz = 0; qz < 3; ++qz) {
          uq[cc][qz] = zval(bb, qz);
          Ttq[cc][qz] = (Real)P.alpha[0] * uq[cc][qz] + zval(hb, qz);  // time term alpha_0 u + H
        }
      }
      Real pb_[3], pbd[3], pdb[3];
      forward(3, 1, pb_, pbd, pdb, dz);
#pragma unroll
      for (int qz = 0; qz < 3; ++qz) {
        pq[qz] = zval(pb_, qz);
        gp[0][qz] = zval(pdb, qz) * ihx;
        gp[1][qz] = zval(pbd, qz) * ihy;
        gp[2][qz] = zder(pb_, qz) * ihz;
      }
    }
    // tau (gls_navier_stokes.cc:401-408), per point
    const Real hst = (Real)P.geo[gcell * 4 + 3];
    Real tauq[3];
#pragma unroll
    for (int qz = 0; qz < 3; ++qz) {
      const Real un2 = uq[0][qz] * uq[0][qz] + uq[1][qz] * uq[1][qz] + uq[2][qz] * uq[2][qz];
      const Real u_mag = fmax(sqrt(un2), Real(1e-12));
      const Real t1 = Real(2) * u_mag / hst, t2 = Real(4) * nu / (hst * hst);
      tauq[qz] = Real(1) / sqrt((Real)P.sdt2 + t1 * t1 + Real(9) * (t2 * t2));
    }
    // MODE_LIN: the lane's linearization rows (pencil layout, qdp_base), FP64 and the FP32 copy
    double *const lrow = LIN && P.qd ? P.qd + qdp_base(brick, valid ? ci : 0, pa + 3 * pb) : nullptr;
    float *const lrowf = LIN && P.qdf ? P.qdf + qdp_base(brick, valid ? ci : 0, pa + 3 * pb) : nullptr;
    const bool f32_all = !P.oseen;  // the Oseen smoother reads only u (0..2) and tau (12) of the FP32 copy
    auto st_lin = [&](int qz, int v, Real x) {
      if (!valid) return;
      if (lrow) lrow[(qz * kQData + v) * kQdpRow] = (double)x;
      if (lrowf && (f32_all || v < 3 || v == 12)) __builtin_nontemporal_store((float)x, lrowf + (qz * kQData + v) * kQdpRow);
    };
    if constexpr (LIN) {
#pragma unroll
      for (int qz = 0; qz < 3; ++qz) {
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) st_lin(qz, cc, uq[cc][qz]);
        st_lin(qz, 12, tauq[qz]);
      }
    }
    Real gcq[3][3];  // MODE_LIN: d u_c / d x_c + alpha_jac per point (the diagonal's mass-like factor)
    // SRF: the lane's point coordinates x0 + h xi (z per point)
    Real xl = 0, yl = 0, zl = 0;
    if (GEN && P.srf) {
      auto xsel = [&](int i) { return i == 0 ? T.xi[0] : i == 1 ? T.xi[1] : T.xi[2]; };
      xl = (Real)P.x0[gcell * 3 + 0] + hx * xsel(pa);
      yl = (Real)P.x0[gcell * 3 + 1] + hy * xsel(pb);
      zl = (Real)P.x0[gcell * 3 + 2];
    }
    Real Rq[3][3], divu[3] = {0, 0, 0};
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) {
      Real Yc[4][3];
      forward(cc, 2, Yc[0], Yc[1], Yc[2], Yc[3]);
      Real Z[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
      for (int qz = 0; qz < 3; ++qz) {
        const Real g0 = zval(Yc[2], qz) * ihx, g1 = zval(Yc[1], qz) * ihy, g2 = zder(Yc[0], qz) * ihz;
        const Real lu = zval(Yc[3], qz) + wzz * zsec(Yc[0], qz);
        const Real u0 = uq[0][qz], u1 = uq[1][qz], u2 = uq[2][qz];
        const Real Gu = g0 * u0 + g1 * u1 + g2 * u2;
        Real f = 0;
        if (GEN && P.force_q && valid) f = (Real)P.force_q[(gcell * 27 + pa + 3 * pb + 9 * qz) * 3 + cc];
        Real R = Gu + gp[cc][qz] - nu * lu - f;
        Real srf = 0;
        if (GEN && P.srf) {
          const Real uu[3] = {u0, u1, u2}, xx[3] = {xl, yl, zl + hz * T.xi[qz]};
          const int c1 = (cc + 1) % 3, c2 = (cc + 2) % 3;
          const Real cxu = om[c1] * uu[c2] - om[c2] * uu[c1];
          const Real ox1 = om[(c1 + 1) % 3] * xx[(c1 + 2) % 3] - om[(c1 + 2) % 3] * xx[(c1 + 1) % 3];
          const Real ox2 = om[(c2 + 1) % 3] * xx[(c2 + 2) % 3] - om[(c2 + 2) % 3] * xx[(c2 + 1) % 3];
          srf = 2 * cxu + (om[c1] * ox2 - om[c2] * ox1);
          R += srf;
        }
        const Real Tt = Ttq[cc][qz];
        R += Tt;
        Rq[cc][qz] = R;
        divu[qz] += cc == 0 ? g0 : cc == 1 ? g1 : g2;
        if constexpr (LIN) {
          st_lin(qz, 3 + 3 * cc + 0, g0);
          st_lin(qz, 3 + 3 * cc + 1, g1);
          st_lin(qz, 3 + 3 * cc + 2, g2);
          st_lin(qz, 13 + cc, R);
          gcq[cc][qz] = (cc == 0 ? g0 : cc == 1 ? g1 : g2) + aj;
          if constexpr (!RES) continue;
        }
        const Real JxW = wxy * T.w[qz], tau = tauq[qz];
        const Real gg[3] = {g0, g1, g2}, uu[3] = {u0, u1, u2};
        Real Te[3];
#pragma unroll
        for (int e = 0; e < 3; ++e)
          Te[e] = JxW * (-nu * gg[e] + (cc == e ? pq[qz] : Real(0)) - tau * R * uu[e]) * ihv[e];
        const Real Tv = JxW * (-Gu + f - Tt - srf);
#pragma unroll
        for (int az = 0; az < 3; ++az) {
          Z[0][az] += T.V[qz][az] * Tv + T.D[qz][az] * Te[2];
          Z[1][az] += T.V[qz][az] * Te[0];
          Z[2][az] += T.V[qz][az] * Te[1];
        }
      }
      if constexpr (RES) backward(cc, Z);
    }
    if constexpr (RES) {  // pressure test field: -JxW div u, -JxW tau R_e / h_e
      Real Z[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
      for (int qz = 0; qz < 3; ++qz) {
        const Real JxW = wxy * T.w[qz], jt = JxW * tauq[qz];
        const Real Tv = -JxW * divu[qz];
        const Real Tx = -jt * Rq[0][qz] * ihx, Ty = -jt * Rq[1][qz] * ihy, Tz = -jt * Rq[2][qz] * ihz;
#pragma unroll
        for (int az = 0; az < 3; ++az) {
          Z[0][az] += T.V[qz][az] * Tv + T.D[qz][az] * Tz;
          Z[1][az] += T.V[qz][az] * Tx;
          Z[2][az] += T.V[qz][az] * Ty;
        }
      }
      backward(3, Z);
    }
    if constexpr (RL) {  // the residual's node sums first; the diagonal then reuses the cell-value area
      __syncthreads();
      reduce_scatter(P.res_y, P.res_slab, false);
      __syncthreads();
    }
    if constexpr (LIN) {
      // ---------------- Jacobian diagonal at this state (the lane-per-point MODE_LIN restated): for
      // the trial / test pair phi_i e_c (gls_navier_stokes.cc:548-622 with v = phi_i e_c)
      //   J_ii(c) = sum_q JxW [A phi + nu |grad phi|^2 + tau (A - nu lap phi) a + tau R_c phi d_c phi],
      //   A = (du_c/dx_c + alpha_jac) phi + a, a = u . grad phi;  J_ii(p) = sum_q JxW tau |grad psi|^2,
      // deal.II's |K_e(i,i)| on constrained rows. Lane (a, b) = node column (ix, iy), nodes iz = 0..2;
      // the points' data go through the stage area one qz plane at a time.
      if (P.y == nullptr && P.ev == nullptr) return;  // linearization only (uniform over the workgroup)
      Real Vx[3], Dx[3], Sx[3], Vy[3], Dy[3], Sy[3];  // the lane's node columns of the 1D tables
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const Real *rx = sRow + q * 4, *ry = sRow + q * 4;
        Vx[q] = rx[pa];
        Dx[q] = rx[16 + pa] * ihx;
        Sx[q] = rx[32 + pa] * wxx;
        Vy[q] = ry[pb];
        Dy[q] = ry[16 + pb] * ihy;
        Sy[q] = ry[32 + pb] * wyy;
      }
      Real acc[3][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int qz = 0; qz < 3; ++qz) {
        // plane qz: [value][qx + 3 qy] = u0 u1 u2 gc0 gc1 gc2 tau R0 R1 R2 JxW
        if (act) {
          const int o = pa + 3 * pb;
          cellS[0 * 9 + o] = uq[0][qz];
          cellS[1 * 9 + o] = uq[1][qz];
          cellS[2 * 9 + o] = uq[2][qz];
          cellS[3 * 9 + o] = gcq[0][qz];
          cellS[4 * 9 + o] = gcq[1][qz];
          cellS[5 * 9 + o] = gcq[2][qz];
          cellS[6 * 9 + o] = tauq[qz];
          cellS[7 * 9 + o] = Rq[0][qz];
          cellS[8 * 9 + o] = Rq[1][qz];
          cellS[9 * 9 + o] = Rq[2][qz];
          cellS[10 * 9 + o] = wxy * T.w[qz];
        }
        wave_sync();
#pragma nounroll
        for (int qy = 0; qy < 3; ++qy) {
#pragma unroll
          for (int qx = 0; qx < 3; ++qx) {
            const int o = qx + 3 * qy;
            const Real u0 = cellS[o], u1 = cellS[9 + o], u2 = cellS[18 + o];
            const Real gc[3] = {cellS[27 + o], cellS[36 + o], cellS[45 + o]};
            const Real tq = cellS[54 + o], jw = cellS[90 + o];
            const Real Rr[3] = {cellS[63 + o], cellS[72 + o], cellS[81 + o]};
            const Real jt = jw * tq;
            const Real bxy = Vx[qx] * Vy[qy], dxy = Dx[qx] * Vy[qy], xdy = Vx[qx] * Dy[qy];
            const Real lxy = Sx[qx] * Vy[qy] + Vx[qx] * Sy[qy];
#pragma unroll
            for (int iz = 0; iz < 3; ++iz) {
              const Real b2 = T.V[qz][iz], d2 = T.D[qz][iz] * ihz, s2 = T.S[qz][iz] * wzz;
              const Real phi = bxy * b2;
              const Real g[3] = {dxy * b2, xdy * b2, bxy * d2};
              const Real lap = lxy * b2 + bxy * s2;
              const Real av = u0 * g[0] + u1 * g[1] + u2 * g[2];
              const Real g2 = g[0] * g[0] + g[1] * g[1] + g[2] * g[2];
              const Real c0 = jw * (av * phi + nu * g2) + jt * av * (av - nu * lap);
              const Real k1 = jw * phi * (phi + tq * av), k2 = jt * phi;
#pragma unroll
              for (int c3 = 0; c3 < 3; ++c3) acc[iz][c3] += c0 + gc[c3] * k1 + k2 * Rr[c3] * g[c3];
              acc[iz][3] += jt * g2;
            }
          }
        }
        wave_sync();  // the plane is rewritten by the next qz
      }
      // deal.II's constrained-row rule: |K_e(i,i)| summed over cells
      if (valid) {
#pragma unroll
        for (int iz = 0; iz < 3; ++iz) {
          const int bn = (2 * cx + pa) + BN * ((2 * cy + pb) + BN * (2 * cz + iz));
          const int nd = sNode[bi * BN3P + bn];  // constrained: Dirichlet or hanging (per-cell kernel's rule)
          const unsigned msk = (P.vmask ? P.vmask[nd] : 0u) | (P.hmask ? P.hmask[nd] : 0u);
#pragma unroll
          for (int c3 = 0; c3 < 3; ++c3)
            outc[c3 * C::OF + 9 * iz + 3 * pb + pa] = (msk >> c3) & 1u ? fabs(acc[iz][c3]) : acc[iz][c3];
          outc[3 * C::OF + 9 * iz + 3 * pb + pa] = acc[iz][3];
        }
      }
    }
  } else {
  // linearization rows of this lane (pencil layout: value v of point qz). Full: u, tau and component 0's
  // grad u_0, R_0 are requested here, behind the gather's loads (vmcnt retires in order, so a load issued
  // before the gather would be waited for at the gather), and component cc + 1's batch while component
  // cc is swept (GLS_PENCIL_PIPE), one batch (12 values) in flight at a time. (Streaming R_s only and
  // re-deriving u, grad u, tau from a u gather was measured slower: DESIGN §4)
  auto ld = [&](int qz, int v) {
#if GLS_PENCIL_NT
    return __builtin_nontemporal_load(qrow + (qz * kQData + v) * kQdpRow);
#else
    return qrow[(qz * kQData + v) * kQdpRow];
#endif
  };
  Real uq[3][3], tauq[3], lnx[3][4];
#pragma unroll
  for (int qz = 0; qz < 3; ++qz) {
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) uq[cc][qz] = ld(qz, cc);
    tauq[qz] = ld(qz, 12);
  }
  auto ld_comp = [&](int cc) {
    if constexpr (!OS) {
#pragma unroll
      for (int qz = 0; qz < 3; ++qz) {
#pragma unroll
        for (int e = 0; e < 3; ++e) lnx[qz][e] = ld(qz, 3 + 3 * cc + e);
        lnx[qz][3] = ld(qz, 13 + cc);
      }
    }
  };
  constexpr bool PIPE = (GLS_PENCIL_PIPE & (std::is_same<Real, double>::value ? 1 : 2)) != 0;
  if (PIPE) ld_comp(0);
  // values of v (all components) and vp, grad vp at the lane's three points: every test field needs
  // them; each velocity component's gradient / Laplacian sweeps run later, next to its test field, so
  // that only one component's Y stage is live at a time
  Real vq[3][3], vpq[3], gvp[3][3];
  {
    Real dz[3];
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) {
      Real bb[3];
      forward(cc, 0, bb, dz, dz, dz);
#pragma unroll
      for (int qz = 0; qz < 3; ++qz) vq[cc][qz] = zval(bb, qz);
    }
    Real pb_[3], pbd[3], pdb[3];
    forward(3, 1, pb_, pbd, pdb, dz);
#pragma unroll
    for (int qz = 0; qz < 3; ++qz) {
      vpq[qz] = zval(pb_, qz);
      gvp[0][qz] = zval(pdb, qz) * ihx;
      gvp[1][qz] = zval(pbd, qz) * ihy;
      gvp[2][qz] = zder(pb_, qz) * ihz;
    }
  }

  // ---------------- pointwise + backward, one velocity test field (= trial component) at a time
  Real Sq[3][3], divv[3] = {0, 0, 0};
#pragma unroll
  for (int cc = 0; cc < 3; ++cc) {
    Real gu[3][3], Rq[3];  // grad u_cc (by e) and R_cc at the lane's three points
    Real Yc[4][3];         // this component's Y stage: BB, BD, DB, L
    {
      if (!PIPE) ld_comp(cc);
#pragma unroll
      for (int qz = 0; qz < 3; ++qz) {
#pragma unroll
        for (int e = 0; e < 3; ++e) gu[e][qz] = OS ? Real(0) : lnx[qz][e];
        Rq[qz] = OS ? Real(0) : lnx[qz][3];
      }
      if (PIPE && cc < 2) ld_comp(cc + 1);
      forward(cc, 2, Yc[0], Yc[1], Yc[2], Yc[3]);
    }
    Real Z[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
    for (int qz = 0; qz < 3; ++qz) {
      const Real gv0 = zval(Yc[2], qz) * ihx, gv1 = zval(Yc[1], qz) * ihy, gv2 = zder(Yc[0], qz) * ihz;
      const Real lv = zval(Yc[3], qz) + wzz * zsec(Yc[0], qz);
      const Real v0 = vq[0][qz], v1 = vq[1][qz], v2 = vq[2][qz];
      const Real u0 = uq[0][qz], u1 = uq[1][qz], u2 = uq[2][qz];
      const Real guv = OS ? Real(0) : gu[0][qz] * v0 + gu[1][qz] * v1 + gu[2][qz] * v2;
      const Real gvu = gv0 * u0 + gv1 * u1 + gv2 * u2;
      Real A = OS ? gvu + aj * vq[cc][qz] : guv + gvu + aj * vq[cc][qz];
      Real S = OS ? gvu + gvp[cc][qz] - nu * lv + aj * vq[cc][qz] : guv + gvu + gvp[cc][qz] - nu * lv + aj * vq[cc][qz];
      if (GEN && P.srf) {
        const Real cj = cc == 0 ? 2 * (om[1] * v2 - om[2] * v1) : cc == 1 ? 2 * (om[2] * v0 - om[0] * v2)
                                                                         : 2 * (om[0] * v1 - om[1] * v0);
        A += cj;
        S += cj;
      }
      Sq[cc][qz] = S;
      divv[qz] += cc == 0 ? gv0 : cc == 1 ? gv1 : gv2;
      const Real JxW = wxy * T.w[qz], tau = tauq[qz];
      const Real gv[3] = {gv0, gv1, gv2}, uu[3] = {u0, u1, u2}, vv[3] = {v0, v1, v2};
      Real Te[3];
#pragma unroll
      for (int e = 0; e < 3; ++e)
        Te[e] = OS ? JxW * (nu * gv[e] - (cc == e ? vpq[qz] : Real(0)) + tau * S * uu[e]) * ihv[e]
                   : JxW * (nu * gv[e] - (cc == e ? vpq[qz] : Real(0)) + tau * S * uu[e] + tau * Rq[qz] * vv[e]) * ihv[e];
      const Real Tv = JxW * A;
#pragma unroll
      for (int az = 0; az < 3; ++az) {
        Z[0][az] += T.V[qz][az] * Tv + T.D[qz][az] * Te[2];
        Z[1][az] += T.V[qz][az] * Te[0];
        Z[2][az] += T.V[qz][az] * Te[1];
      }
    }
    backward(cc, Z);
  }
  {  // pressure test field: Tv = JxW div v, Te = JxW tau S_e / h_e
    Real Z[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
    for (int qz = 0; qz < 3; ++qz) {
      const Real JxW = wxy * T.w[qz], jt = JxW * tauq[qz];
      const Real Tv = JxW * divv[qz];
      const Real Tx = jt * Sq[0][qz] * ihx, Ty = jt * Sq[1][qz] * ihy, Tz = jt * Sq[2][qz] * ihz;
#pragma unroll
      for (int az = 0; az < 3; ++az) {
        Z[0][az] += T.V[qz][az] * Tv + T.D[qz][az] * Tz;
        Z[1][az] += T.V[qz][az] * Tx;
        Z[2][az] += T.V[qz][az] * Ty;
      }
    }
    backward(3, Z);
  }
  }  // MODE_JVQ
  __syncthreads();

  if (P.ev) write_ev();
  else reduce_scatter(P.y, P.slab, true);
}

// (A packed-FP32 variant of the FP32 smoother J.v -- two cells per lane as float2 -- was measured slower than
// the scalar FP32 kernel above, 1.56 vs 1.37 ms per launch at Q2 128^3, profiles/r05_ab_pair_kernel.txt, and was
// removed in round 6.)

// Selection: on by default for the Q2 brick J.v with a slab (the launch contract of the
// lane-per-point kernel); GLS_PENCIL=0 keeps the lane-per-point kernel (A/B, fallback)
bool pencil_enabled() {  // read per launch: tests compare both kernels in one process
  const char *e = std::getenv("GLS_PENCIL");
  return !(e && std::atoi(e) == 0);
}

template <typename Real, int MODE, bool FB = false>
hipError_t launch_pencil_t(const OpParams &P, const Tables1D &T, hipStream_t s) {
  const bool gen = P.srf || (MODE != MODE_JVQ && P.force_q);
  const int n_items = ((std::is_same<Real, double>::value || P.brick_cell0) && P.subset) ? P.subset_n : P.n_cells / 8;
  if (n_items <= 0) return hipSuccess;
  const int n_groups = (n_items + 2) / 3;
  PencilTab<Real> tab;
  for (int q = 0; q < 3; ++q) {
    tab.w[q] = (Real)T.w[q];
    for (int i = 0; i < 3; ++i) {
      tab.V[q][i] = (Real)T.V[q][i];
      tab.D[q][i] = (Real)T.D[q][i];
      tab.S[q][i] = (Real)T.S[q][i];
    }
    tab.xi[q] = (Real)T.xi[q];
  }
  if constexpr (std::is_same<Real, float>::value && MODE == MODE_JVQ && !FB) {
    if (P.oseen) {  // the multigrid smoother's Oseen operator
      if (gen)
        hipLaunchKernelGGL((gls_pencil_kernel<float, MODE_JVQ, true, false, true>), dim3((unsigned)n_groups), dim3(256),
                           pencil_lds_bytes<float>(MODE), s, P, tab);
      else
        hipLaunchKernelGGL((gls_pencil_kernel<float, MODE_JVQ, false, false, true>), dim3((unsigned)n_groups),
                           dim3(256), pencil_lds_bytes<float>(MODE), s, P, tab);
      return hipGetLastError();
    }
  }
  if (gen)
    hipLaunchKernelGGL((gls_pencil_kernel<Real, MODE, true, FB>), dim3((unsigned)n_groups), dim3(256),
                       pencil_lds_bytes<Real>(MODE), s, P, tab);
  else
    hipLaunchKernelGGL((gls_pencil_kernel<Real, MODE, false, FB>), dim3((unsigned)n_groups), dim3(256),
                       pencil_lds_bytes<Real>(MODE), s, P, tab);
  return hipGetLastError();
}
hipError_t launch_pencil_jv(const OpParams &P, const Tables1D &T, hipStream_t s, bool f32) {
  if (P.n_probe > 0 || P.bricks || !(f32 ? (P.slabf != nullptr || P.slab != nullptr) : P.slab != nullptr))
    return hipErrorNotSupported;
  return f32 ? launch_pencil_t<float, MODE_JVQ>(P, T, s) : launch_pencil_t<double, MODE_JVQ>(P, T, s);
}
hipError_t launch_pencil_residual(const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (P.bricks || !P.slab || P.subset) return hipErrorNotSupported;
  return launch_pencil_t<double, MODE_RESIDUAL>(P, T, s);
}
// residual (into res_y / res_slab) + linearization + diagonal (into y / slab) at one state
hipError_t launch_pencil_reslin(const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (P.bricks || P.subset || !P.qd || !P.y || !P.slab || !P.res_y || !P.res_slab) return hipErrorNotSupported;
  return launch_pencil_t<double, MODE_RESLIN>(P, T, s);
}
// adapted forests: the listed sibling-group bricks (P.subset over P.brick_cell0), element-vector output
// (P.ev); mode MODE_JVQ (FP64) or MODE_LIN (linearization rows + the diagonal's element vectors)
hipError_t launch_pencil_ev(int mode, const OpParams &P, const Tables1D &T, hipStream_t s, bool f32) {
  if ((!P.ev && mode != MODE_LIN) || P.y || !P.brick_cell0 || !P.subset || P.subset_n <= 0 || !P.qd || P.slab ||
      P.bricks || P.n_probe > 0 || P.rb || P.jx || P.jx0 || (f32 && (mode != MODE_JVQ || !P.qdf)))
    return hipErrorNotSupported;
  if (mode == MODE_JVQ && f32) return launch_pencil_t<float, MODE_JVQ, true>(P, T, s);
  if (mode == MODE_JVQ) return launch_pencil_t<double, MODE_JVQ>(P, T, s);
  if (mode == MODE_LIN) return launch_pencil_t<double, MODE_LIN>(P, T, s);
  return hipErrorNotSupported;
}
hipError_t launch_pencil_lin(const OpParams &P, const Tables1D &T, hipStream_t s) {
  if (P.bricks || (P.y && !P.slab) || P.subset || !P.qd) return hipErrorNotSupported;
  return launch_pencil_t<double, MODE_LIN>(P, T, s);
}

}  // namespace gls
