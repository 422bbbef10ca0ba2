// gls_ilu_kernels.hip — triangular solves of the assembled ILU in multicolor order (gls_ilu_attach
// with GLS_ILU_ORDER_MULTICOLOR).
//
// In that order the DoFs of one color belong to nodes that share no matrix entry, so inside a color
// a row depends on rows of earlier colors (forward) / later colors (backward) and on the rows of its
// own node only. One launch per color, one or four wavefronts per node group: the group's threads
// stride over its rows' entries of the other colors (a gather-dot), then one thread resolves the
// <= 4 rows of the node in order. The dependency chain of a solve is the number of colors, where the
// general level-scheduled csrsv of a Cuthill-McKee-ordered 3D Q2 matrix waits on thousands of
// levels (profiles/r03_app_cylinder3d_ilu_timing.log vs r03_app_cylinder3d_multicolor_ilu.log).
#include "gls_launch.hpp"

namespace gls {

namespace {

__device__ __forceinline__ double wave_sum(double s) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// One launch per color; WPG wavefronts per node group (1 for short rows, 4 for the ~200-entry rows
// of 3D Q2 matrices, where a single wave would walk each row's other-color entries in several
// dependent load rounds). The rows of a group are contiguous in the CSR, so the group's threads
// stride over its whole entry range at once (all <= 4 rows, kGatherUnroll entries per thread in
// flight) and mask entries outside a row's other-color segment before the x gather. Thread 0 of the
// group loads its serial-part operands (right-hand sides, the <= 3 own-node entries per row, the
// diagonal) before the gather so they are in flight with it, and keeps the rows it has resolved in
// registers: the only dependent global traffic left is the gather.
constexpr int kGatherUnroll = 4;
constexpr int kOwnMax = kMaxGroupRows - 1;  // own-node entries per row besides the diagonal

__device__ __forceinline__ double pick4(const double *a, int j) {
  return j == 0 ? a[0] : j == 1 ? a[1] : j == 2 ? a[2] : a[3];
}

// LOWER: y_i = b_i - sum_{j < i} L_ij y_j (unit lower); entries [rowp_i, sp_i) lie in earlier colors,
//        [sp_i, didx_i) in the row's own node (sp = lsp).
// upper: x_i = (y_i - sum_{j > i} U_ij x_j) / U_ii; entries [sp_i, rowp_{i+1}) lie in later colors,
//        (didx_i, sp_i) in the row's own node (sp = usp).
// In both, the gathered vector is the output (x / y of the other colors, already final).
template <int WPG, bool LOWER>
__global__ void __launch_bounds__(256) k_mc_tri(const int32_t *__restrict__ grow, int g0, int g1,
                                                const int32_t *__restrict__ rowp, const int32_t *__restrict__ col,
                                                const double *__restrict__ val, const int32_t *__restrict__ sp,
                                                const int32_t *__restrict__ didx, const double *__restrict__ rhs,
                                                double *__restrict__ out) {
  constexpr int GPB = 4 / WPG;  // node groups per 256-thread block
  const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const int gl = w / WPG, tig = (w % WPG) * 64 + lane;
  const int g = g0 + (int)blockIdx.x * GPB + gl;
  const bool live = g < g1;
  __shared__ double red[4][kMaxGroupRows];
  int r0 = 0, nr = 0;
  if (live) {
    r0 = grow[g];
    nr = grow[g + 1] - r0;
  }
  int32_t bnd[kMaxGroupRows], lo[kMaxGroupRows], hi[kMaxGroupRows];
#pragma unroll
  for (int t = 0; t < kMaxGroupRows; ++t) {
    const bool in = t < nr;
    bnd[t] = in ? rowp[r0 + t] : INT32_MAX;
    lo[t] = !in ? 0 : LOWER ? rowp[r0 + t] : sp[r0 + t];
    hi[t] = !in ? 0 : LOWER ? sp[r0 + t] : rowp[r0 + t + 1];
  }
  // serial-part operands (thread 0 of the group)
  double rb[kMaxGroupRows] = {0.0, 0.0, 0.0, 0.0}, dg[kMaxGroupRows] = {1.0, 1.0, 1.0, 1.0};
  double ov[kMaxGroupRows][kOwnMax];
  int oc[kMaxGroupRows][kOwnMax];
  if (tig == 0) {
#pragma unroll
    for (int t = 0; t < kMaxGroupRows; ++t) {
      const int i = r0 + t;
      const bool in = t < nr;
      const int d = in ? didx[i] : 0;
      const int ob = !in ? 0 : LOWER ? sp[i] : d + 1, oe = !in ? 0 : LOWER ? d : sp[i];
      rb[t] = in ? rhs[i] : 0.0;
      if (!LOWER) dg[t] = in ? val[d] : 1.0;
#pragma unroll
      for (int k = 0; k < kOwnMax; ++k) {
        const bool ok = ob + k < oe;
        ov[t][k] = ok ? val[ob + k] : 0.0;
        oc[t][k] = ok ? col[ob + k] - r0 : 0;
      }
    }
  }
  // other-color gather-dot
  double acc[kMaxGroupRows] = {0.0, 0.0, 0.0, 0.0};
  const int eb = live ? rowp[r0] : 0, ee = live ? rowp[r0 + nr] : 0;
  for (int e0 = eb + tig; e0 < ee; e0 += 64 * WPG * kGatherUnroll) {
    int c[kGatherUnroll], tt[kGatherUnroll];
    double v[kGatherUnroll], xv[kGatherUnroll];
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const int e = e0 + 64 * WPG * u;
      const int t = (e >= bnd[1]) + (e >= bnd[2]) + (e >= bnd[3]);
      const int l = t == 0 ? lo[0] : t == 1 ? lo[1] : t == 2 ? lo[2] : lo[3];
      const int h = t == 0 ? hi[0] : t == 1 ? hi[1] : t == 2 ? hi[2] : hi[3];
      const bool ok = e < ee && e >= l && e < h;
      tt[u] = ok ? t : -1;
      c[u] = ok ? col[e] : 0;
      v[u] = ok ? val[e] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) xv[u] = tt[u] >= 0 ? out[c[u]] : 0.0;
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const double p = v[u] * xv[u];
#pragma unroll
      for (int r = 0; r < kMaxGroupRows; ++r) acc[r] += tt[u] == r ? p : 0.0;
    }
  }
  double part[kMaxGroupRows];
#pragma unroll
  for (int r = 0; r < kMaxGroupRows; ++r) part[r] = wave_sum(acc[r]);
  if (WPG > 1) {
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < kMaxGroupRows; ++r) red[w][r] = part[r];
    }
    __syncthreads();
    if (tig == 0) {
#pragma unroll
      for (int r = 0; r < kMaxGroupRows; ++r) {
        double sum = 0.0;
#pragma unroll
        for (int k = 0; k < WPG; ++k) sum += red[gl * WPG + k][r];
        part[r] = sum;
      }
    }
  }
  if (tig != 0 || !live) return;
  // the node's own rows (forward in order, backward in reverse), resolved values kept in registers
  double res[kMaxGroupRows] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < kMaxGroupRows; ++q) {
    const int t = LOWER ? q : kMaxGroupRows - 1 - q;
    if (t >= nr) continue;
    double s = rb[t] - part[t];
#pragma unroll
    for (int k = 0; k < kOwnMax; ++k) s -= ov[t][k] * pick4(res, oc[t][k]);
    const double r = LOWER ? s : s / dg[t];
    res[t] = r;
    out[r0 + t] = r;
  }
}

constexpr int kIluPrefetch = 4;
// first position q in [lo, hi) of the sorted column list c with c[q] == j, else -1
__device__ __forceinline__ int lds_find(const int32_t *c, int lo, int hi, int32_t j) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (c[mid] < j) lo = mid + 1;
    else hi = mid;
  }
  return c[lo] == j ? lo : -1;  // c[hi] of the full range is the sentinel: never a column
}

// ILU numeric factorization of one color's node groups in place (IKJ, the order rocSPARSE csrilu0
// and Ifpack use: for every k < i with a_ik in the pattern, a_ik /= u_kk, then a_ij -= a_ik u_kj for
// the pattern's j > k; no fill outside the pattern; pivots with |u_kk| <= boost_tol replaced by
// boost_val as rocsparse_csrilu0_numeric_boost). One workgroup per node group, one wavefront per row:
// the rows of earlier colors are final, so each row's updates from them run in parallel (phase 1, the
// bulk); the couplings inside the node (own-node rows, lower than i) follow row by row (phase 2) from
// the workgroup's LDS copy of the group. Rows of up to kIluMaxRow entries (the caller checks).
__global__ void __launch_bounds__(64 * kMaxGroupRows) k_mc_ilu0(const int32_t *__restrict__ grow, int g0, int g1,
                                                                const int32_t *__restrict__ rowp,
                                                                const int32_t *__restrict__ col, double *__restrict__ val,
                                                                const int32_t *__restrict__ lsp,
                                                                const int32_t *__restrict__ didx, double boost_tol,
                                                                double boost_val) {
  __shared__ int32_t sc[kMaxGroupRows][kIluMaxRow + 1];
  __shared__ double sv[kMaxGroupRows][kIluMaxRow];
  const int g = g0 + (int)blockIdx.x;
  if (g >= g1) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = grow[g], nr = grow[g + 1] - r0;
  const int i = r0 + w;
  const int rp = w < nr ? rowp[i] : 0, len = w < nr ? rowp[i + 1] - rp : 0;
  for (int e = lane; e < len; e += 64) {
    sc[w][e] = col[rp + e];
    sv[w][e] = val[rp + e];
  }
  if (lane == 0) sc[w][len] = 0x7fffffff;  // search sentinel
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
  // phase 1: the pivots of earlier colors (entries [rowp_i, lsp_i)), in ascending column order
  if (w < nr) {
    // software pipeline over the pivot rows k_p = sc[w][p]: while step p updates the row from k_p's
    // upper entries (held in registers), the upper entries of k_{p+1} and the indices of k_{p+2} are in
    // flight. (A two-step-deep rotation of four register stages measured slower, 27 vs 23 ms per
    // factorization at 121 k DoFs: the step is bound by its LDS search chain, and the extra VGPRs cost
    // occupancy.)
    constexpr int PF = kIluPrefetch;  // upper entries per lane held in registers (64 * PF per pivot row)
    const int nl = lsp[i] - rp;
    int dk1 = 0, e11 = 0, dk2 = 0, e12 = 0;  // indices of k_{p+1}, k_{p+2}
    double piv0 = 1.0, piv1 = 1.0, v0[PF], v1[PF];
    int c0[PF], c1[PF];
    auto load_upper = [&](int dk, int e1, double &piv, int (&c)[PF], double (&v)[PF]) {
      piv = val[dk];
#pragma unroll
      for (int t = 0; t < PF; ++t) {
        const int e = dk + 1 + lane + 64 * t;
        c[t] = e < e1 ? col[e] : -1;
        v[t] = e < e1 ? val[e] : 0.0;
      }
    };
    int dk0 = 0, e10 = 0;
    if (nl > 0) {
      dk0 = didx[sc[w][0]];
      e10 = rowp[sc[w][0] + 1];
      load_upper(dk0, e10, piv0, c0, v0);
    }
    if (nl > 1) {
      dk1 = didx[sc[w][1]];
      e11 = rowp[sc[w][1] + 1];
    }
    for (int p = 0; p < nl; ++p) {
      if (p + 1 < nl) load_upper(dk1, e11, piv1, c1, v1);
      if (p + 2 < nl) {
        dk2 = didx[sc[w][p + 2]];
        e12 = rowp[sc[w][p + 2] + 1];
      }
      const double lik = sv[w][p] / piv0;
      {  // PF branchless lower_bound searches in [p+1, len) side by side (the trip count is uniform;
         // an LDS hash of the row's columns measured slower, 47 vs 23 ms: most lookups miss)
        int b[PF], n = len - (p + 1);
#pragma unroll
        for (int t = 0; t < PF; ++t) b[t] = p + 1;
        while (n > 1) {
          const int half = n >> 1;
#pragma unroll
          for (int t = 0; t < PF; ++t) b[t] = sc[w][b[t] + half] < c0[t] ? b[t] + half : b[t];
          n -= half;
        }
        if (n > 0) {
#pragma unroll
          for (int t = 0; t < PF; ++t) {
            const int q = b[t] + (sc[w][b[t]] < c0[t] ? 1 : 0);
            if (c0[t] >= 0 && sc[w][q] == c0[t]) sv[w][q] -= lik * v0[t];  // sc[w][len]: sentinel
          }
        }
      }
      for (int e = dk0 + 1 + lane + 64 * PF; e < e10; e += 64) {  // longer pivot rows: the rest directly
        const int q = lds_find(sc[w], p + 1, len, col[e]);
        if (q >= 0) sv[w][q] -= lik * val[e];
      }
      if (lane == 0) sv[w][p] = lik;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      dk0 = dk1;
      e10 = e11;
      piv0 = piv1;
#pragma unroll
      for (int t = 0; t < PF; ++t) {
        c0[t] = c1[t];
        v0[t] = v1[t];
      }
      dk1 = dk2;
      e11 = e12;
    }
  }
  __syncthreads();
  // phase 2: the own-node pivots (entries [lsp_i, didx_i): rows r0 .. i-1 of this group), row by row
  for (int t = 0; t < nr; ++t) {
    if (w == t) {
      const int pd = didx[i] - rp;
      for (int p = lsp[i] - rp; p < pd; ++p) {
        const int tk = sc[w][p] - r0;  // own-node row, final (phase 2 of row tk done, pivot boosted)
        const int lk = rowp[r0 + tk + 1] - rowp[r0 + tk], dpk = didx[r0 + tk] - rowp[r0 + tk];
        const double lik = sv[w][p] / sv[tk][dpk];
        for (int e = dpk + 1 + lane; e < lk; e += 64) {
          const int q = lds_find(sc[w], p + 1, len, sc[tk][e]);
          if (q >= 0) sv[w][q] -= lik * sv[tk][e];
        }
        if (lane == 0) sv[w][p] = lik;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      }
      if (lane == 0 && fabs(sv[w][pd]) <= boost_tol) sv[w][pd] = boost_val;
    }
    __syncthreads();
  }
  for (int e = lane; e < len; e += 64) val[rp + e] = sv[w][e];
}
}  // namespace

hipError_t ilu_mc_factor(const int32_t *grow, const int32_t *color_groups, int n_colors, const int32_t *rowp,
                         const int32_t *col, double *val, const int32_t *lsp, const int32_t *didx, double boost_tol,
                         double boost_val, hipStream_t s) {
  for (int c = 0; c < n_colors; ++c) {
    const int g0 = color_groups[c], g1 = color_groups[c + 1];
    if (g1 <= g0) continue;
    hipLaunchKernelGGL(k_mc_ilu0, dim3((unsigned)(g1 - g0)), dim3(64 * kMaxGroupRows), 0, s, grow, g0, g1, rowp, col, val,
                       lsp, didx, boost_tol, boost_val);
  }
  return hipGetLastError();
}

hipError_t ilu_mc_solve(const int32_t *grow, const int32_t *color_groups, int n_colors, const int32_t *rowp,
                        const int32_t *col, const double *val, const int32_t *lsp, const int32_t *usp,
                        const int32_t *didx, const double *b, double *y, double *x, int waves_per_group,
                        hipStream_t s) {
  const int wpg = waves_per_group >= 4 ? 4 : 1, gpb = 4 / wpg;
  for (int c = 0; c < n_colors; ++c) {
    const int g0 = color_groups[c], g1 = color_groups[c + 1];
    if (g1 <= g0) continue;
    const unsigned nb = (unsigned)((g1 - g0 + gpb - 1) / gpb);
    if (wpg == 4) hipLaunchKernelGGL((k_mc_tri<4, true>), dim3(nb), dim3(256), 0, s, grow, g0, g1, rowp, col, val, lsp, didx, b, y);
    else hipLaunchKernelGGL((k_mc_tri<1, true>), dim3(nb), dim3(256), 0, s, grow, g0, g1, rowp, col, val, lsp, didx, b, y);
  }
  for (int c = n_colors - 1; c >= 0; --c) {
    const int g0 = color_groups[c], g1 = color_groups[c + 1];
    if (g1 <= g0) continue;
    const unsigned nb = (unsigned)((g1 - g0 + gpb - 1) / gpb);
    if (wpg == 4) hipLaunchKernelGGL((k_mc_tri<4, false>), dim3(nb), dim3(256), 0, s, grow, g0, g1, rowp, col, val, usp, didx, y, x);
    else hipLaunchKernelGGL((k_mc_tri<1, false>), dim3(nb), dim3(256), 0, s, grow, g0, g1, rowp, col, val, usp, didx, y, x);
  }
  return hipGetLastError();
}

}  // namespace gls
