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
// dependent load rounds). The group's threads stride over the concatenation of its rows'
// other-color segments at once (all <= 4 rows, kGatherUnroll entries per thread in flight; no lane
// walks the other triangle's entries). Thread 0 of the
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
// Each node group's row extents come from one 192-byte descriptor (kGroupDesc int64, built at attach:
// r0, nr, entry range, row boundaries, lsp, usp, didx, row ends), so the first dependent load round
// of a launch is the descriptor itself rather than grow -> rowp / lsp / usp / didx.
template <int WPG, bool LOWER>
__global__ void __launch_bounds__(256) k_mc_tri(const int64_t *__restrict__ gdesc, int g0, int g1,
                                                const int32_t *__restrict__ col, const double *__restrict__ val,
                                                const double *__restrict__ rhs, double *__restrict__ out) {
  constexpr int GPB = 4 / WPG;  // node groups per 256-thread block
  const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const int gl = w / WPG, tig = (w % WPG) * 64 + lane;
  const int g = g0 + (int)blockIdx.x * GPB + gl;
  const bool live = g < g1;
  __shared__ double red[4][kMaxGroupRows];
  int64_t dsc[kGroupDesc];
  {
    typedef long long ll2 __attribute__((ext_vector_type(2)));
    const ll2 *d2 = reinterpret_cast<const ll2 *>(gdesc + (int64_t)(live ? g : g0) * kGroupDesc);
#pragma unroll
    for (int k = 0; k < kGroupDesc / 2; ++k) {
      const ll2 q = d2[k];
      dsc[2 * k] = q.x;
      dsc[2 * k + 1] = q.y;
    }
  }
  const int r0 = (int)dsc[0], nr = live ? (int)dsc[1] : 0;
  int64_t bnd[kMaxGroupRows], lo[kMaxGroupRows], hi[kMaxGroupRows], dix[kMaxGroupRows];
#pragma unroll
  for (int t = 0; t < kMaxGroupRows; ++t) {
    const bool in = t < nr;
    bnd[t] = t == 0 ? dsc[2] : dsc[3 + t];
    lo[t] = !in ? 0 : LOWER ? bnd[t] : dsc[12 + t];
    hi[t] = !in ? 0 : LOWER ? dsc[8 + t] : dsc[20 + t];
    dix[t] = dsc[16 + t];
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
      const int64_t d = in ? dix[t] : 0;
      const int64_t ob = !in ? 0 : LOWER ? dsc[8 + t] : d + 1, oe = !in ? 0 : LOWER ? d : dsc[12 + t];
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
  // other-color gather-dot over the rows' segments [lo_t, hi_t) concatenated (virtual index v:
  // row t = number of segment prefix sums <= v), so no lane walks entries of the other triangle
  double acc[kMaxGroupRows] = {0.0, 0.0, 0.0, 0.0};
  const int P1 = (int)(hi[0] - lo[0]), P2 = P1 + (int)(hi[1] - lo[1]), P3 = P2 + (int)(hi[2] - lo[2]),
            tot = P3 + (int)(hi[3] - lo[3]);
  for (int v0 = tig; v0 < tot; v0 += 64 * WPG * kGatherUnroll) {
    int c[kGatherUnroll], tt[kGatherUnroll];
    double v[kGatherUnroll], xv[kGatherUnroll];
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const int vi = v0 + 64 * WPG * u;
      const int t = (vi >= P1) + (vi >= P2) + (vi >= P3);
      const int64_t e = vi + (t == 0 ? lo[0] : t == 1 ? lo[1] - P1 : t == 2 ? lo[2] - P2 : lo[3] - P3);
      const bool ok = vi < tot;
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
// pivot rows in flight in the factorization (template NS): 3; 6 measured the same with the MAP kernel
// (10.5 ms per factorization at 121 k DoFs either way): its step is bound by the wave's own
// instruction stream (loads' address arithmetic, the division, four predicated updates), not by
// the loads
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
//
// MAP: the row positions the upper entries of each pivot row land on (found by the column searches)
// depend on the pattern only; gls_ilu_attach precomputes them once (k_mc_ilu0_map, uint16 per
// (row, pivot, upper entry), 0xffff where the entry is outside the row's pattern, each pivot's
// segment padded to a multiple of 4 so a lane reads its quad of positions in one load), and the
// factorization streams them with the upper values instead of searching: the step's LDS chain
// shrinks to sv[p] / U_kk and one read-modify-write per lane. Same updates in the same order, so the
// factors are bitwise those of the searching kernel.
//
// R: the LDS capacity of a row (entries; its pivots too). Every workgroup holds its group's rows and
// pivot extents in LDS, each pivot's diagonal position (35 bits), upper length (10) and map offset (19) packed
// into one word: 20 bytes per entry, 51 KB at R = kIluMaxRow (three workgroups per CU; unpacked, 72 KB and
// two), 36 KB at R = kIluCompactRow (rows of Q2-Q1 3D cells of valence <= 8: <= 402 entries; four per CU)
// -- waves to hide the step's LDS / division latency chain
constexpr uint16_t kMapMiss = 0xffff;
template <bool MAP, int NS, int R>
__global__ void __launch_bounds__(64 * kMaxGroupRows) k_mc_ilu0(const int32_t *__restrict__ grow, int g0, int g1,
                                                                const int64_t *__restrict__ rowp,
                                                                const int32_t *__restrict__ col, double *__restrict__ val,
                                                                const int64_t *__restrict__ lsp,
                                                                const int64_t *__restrict__ didx, double boost_tol,
                                                                double boost_val, const int64_t *__restrict__ moff,
                                                                const uint16_t *__restrict__ map,
                                                                double *__restrict__ rdiag) {
  static_assert(R < 1024 && R * R < (1 << 19), "packed pivot extents");
  __shared__ int32_t sc[kMaxGroupRows][R + 1];
  __shared__ double sv[kMaxGroupRows][R + 1];  // + a dummy slot for the MAP step's idle lanes
  // pivot-row extents: the diagonal's position, the upper part's length and the map offset in the row, one word
  __shared__ uint64_t sdk[kMaxGroupRows][R];
  const int g = g0 + (int)blockIdx.x;
  if (g >= g1) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = grow[g], nr = grow[g + 1] - r0;
  const int i = r0 + w;
  const int64_t rp = w < nr ? rowp[i] : 0;
  const int len = w < nr ? (int)(rowp[i + 1] - rp) : 0;
  for (int e = lane; e < len; e += 64) {
    sc[w][e] = col[rp + e];
    sv[w][e] = val[rp + e];
  }
  if (lane == 0) sc[w][len] = 0x7fffffff;  // search sentinel
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
  // phase 1: the pivots of earlier colors (entries [rowp_i, lsp_i)), in ascending column order.
  // Every pivot row k_p belongs to an earlier color and is final, so its upper entries can be loaded
  // any number of steps ahead: the extents [didx_k, rowp_{k+1}) of all pivot rows are staged in LDS
  // first (one gather for the row), then a ring of NS register stages keeps the upper
  // entries of k_{p+1} .. k_{p+NS-1} in flight while step p searches and updates the row.
  // The ring is unrolled (stage j serves the pivots p = j mod NS), so no register copies wait
  // on loads in flight. The step itself is the LDS chain: sv[p] / U_kk, the column searches, the
  // updates. (An LDS hash of the row's columns measured slower, 47 vs 23 ms: most lookups miss.)
  if (w < nr) {
    constexpr int PF = kIluPrefetch;  // upper entries per lane held in registers (64 * PF per pivot row)
    const int nl = (int)(lsp[i] - rp);
    int mrun = 0;  // MAP: running offset of the pivot's map segment in the row's
    for (int p0 = 0; p0 < nl; p0 += 64) {
      const int p = p0 + lane;
      int m = 0, ul = 0;
      int64_t dk = 0;
      if (p < nl) {
        const int k = sc[w][p];
        dk = didx[k];
        ul = (int)(rowp[k + 1] - dk - 1);
        m = MAP ? (ul + 3) & ~3 : ul;  // MAP segments are padded to quads
      }
      int mo = 0;
      if (MAP) {  // exclusive prefix sum of the upper-entry counts over the wave
        int x = m;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(x, o, 64);
          if (lane >= o) x += y;
        }
        mo = mrun + x - m;
        mrun += __shfl(x, 63, 64);
      }
      if (p < nl) sdk[w][p] = (uint64_t)dk | ((uint64_t)ul << 35) | ((uint64_t)mo << 45);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int64_t mbase = MAP ? moff[i] : 0;
    struct Stage {
      double rpiv, v[PF];  // rpiv: 1 / U_kk of the pivot row (rdiag, written with the row)
      int64_t dk, e1;
      int c[PF], mo;  // c: the upper entries' columns
      uint64_t mq;            // MAP: the row positions of the lane's quad, 4 x 16 bit (unpacked only
                              // when used: touching a register still in flight waits for its load)
    } S[NS];
    // branchless: every load is issued (clamped to the diagonal entry when out of range) so that the
    // waitcnt pass sees straight-line code and waits for exactly the stage in use, not vmcnt(0)
    auto issue = [&](int p, Stage &st) {
      const bool in = p < nl;
      const uint64_t pk = in ? sdk[w][p] : 0;
      st.dk = in ? (int64_t)(pk & ((uint64_t(1) << 35) - 1)) : rp;
      st.e1 = in ? st.dk + 1 + (int)((pk >> 35) & 1023) : rp;
      st.rpiv = rdiag[in ? sc[w][p] : 0];
      if (MAP) {  // lane l: the quad of upper entries 4l .. 4l+3 (one 8-byte map load, one address
                  // for the values; past the row's end they are masked in the step, and the value
                  // array is padded for the last rows)
        st.mo = in ? (int)(pk >> 45) : 0;
        const bool ok = 4 * lane < st.e1 - st.dk - 1;
        st.mq = reinterpret_cast<const uint64_t *>(map + mbase + st.mo)[ok ? lane : 0];
        const double *vp = val + st.dk + 1 + 4 * lane;
#pragma unroll
        for (int t = 0; t < PF; ++t) st.v[t] = vp[t];
        return;
      }
#pragma unroll
      for (int t = 0; t < PF; ++t) {
        const int64_t e = st.dk + 1 + lane + 64 * t;
        const int64_t ec = e < st.e1 ? e : st.dk;
        // raw; validity (e < e1) is applied where the stage is used, so no instruction touches these
        // registers before the stage's step
        st.c[t] = col[ec];
        st.v[t] = val[ec];
      }
    };
    auto step = [&](int p, const Stage &st) {
      const double lik = sv[w][p] * st.rpiv;  // (a division here sat on the step's dependency chain)
      if (MAP) {  // branchless: all four reads, then all four writes (idle lanes on the dummy slot)
        const int m = (int)(st.e1 - st.dk - 1);
        int qa[PF];
        double r[PF];
#pragma unroll
        for (int t = 0; t < PF; ++t) {
          const int q = (int)((st.mq >> (16 * t)) & 0xffffu);
          qa[t] = 4 * lane + t < m && q != kMapMiss ? q : R;
        }
#pragma unroll
        for (int t = 0; t < PF; ++t) r[t] = sv[w][qa[t]];
#pragma unroll
        for (int t = 0; t < PF; ++t) sv[w][qa[t]] = r[t] - lik * st.v[t];
        for (int e = 4 * 64 + lane; e < m; e += 64) {  // longer pivot rows: the rest directly
          const int q = map[mbase + st.mo + e];
          if (q != kMapMiss) sv[w][q] -= lik * val[st.dk + 1 + e];
        }
        if (lane == 0) sv[w][p] = lik;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        return;
      }
      int cs[PF];
#pragma unroll
      for (int t = 0; t < PF; ++t) cs[t] = st.dk + 1 + lane + 64 * t < st.e1 ? st.c[t] : -1;
      {  // PF branchless lower_bound searches in [p+1, len) side by side (the trip count is uniform)
        int b[PF], n = len - (p + 1);
#pragma unroll
        for (int t = 0; t < PF; ++t) b[t] = p + 1;
        while (n > 1) {
          const int half = n >> 1;
#pragma unroll
          for (int t = 0; t < PF; ++t) b[t] = sc[w][b[t] + half] < cs[t] ? b[t] + half : b[t];
          n -= half;
        }
        if (n > 0) {
#pragma unroll
          for (int t = 0; t < PF; ++t) {
            const int q = b[t] + (sc[w][b[t]] < cs[t] ? 1 : 0);
            if (cs[t] >= 0 && sc[w][q] == cs[t]) sv[w][q] -= lik * st.v[t];  // sc[w][len]: sentinel
          }
        }
      }
      for (int64_t e = st.dk + 1 + lane + 64 * PF; e < st.e1; e += 64) {  // longer pivot rows: the rest directly
        const int q = lds_find(sc[w], p + 1, len, col[e]);
        if (q >= 0) sv[w][q] -= lik * val[e];
      }
      if (lane == 0) sv[w][p] = lik;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    };
#pragma unroll
    for (int j = 0; j < NS; ++j) issue(j, S[j]);
    int p = 0;
    for (; p + NS <= nl; p += NS) {  // full rounds: no branch between the stages
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        step(p + j, S[j]);
        issue(p + j + NS, S[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < NS; ++j)  // the last < NS pivots, already in flight
      if (p + j < nl) step(p + j, S[j]);
  }
  __syncthreads();
  // phase 2: the own-node pivots (entries [lsp_i, didx_i): rows r0 .. i-1 of this group), row by row
  for (int t = 0; t < nr; ++t) {
    if (w == t) {
      const int pd = (int)(didx[i] - rp);
      for (int p = (int)(lsp[i] - rp); p < pd; ++p) {
        const int tk = sc[w][p] - r0;  // own-node row, final (phase 2 of row tk done, pivot boosted)
        const int lk = (int)(rowp[r0 + tk + 1] - rowp[r0 + tk]), dpk = (int)(didx[r0 + tk] - rowp[r0 + tk]);
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
      if (lane == 0) rdiag[i] = 1.0 / sv[w][pd];
    }
    __syncthreads();
  }
  for (int e = lane; e < len; e += 64) val[rp + e] = sv[w][e];
}

// the MAP positions: one wavefront per row, its columns staged in LDS; for every pivot k_p (entries
// [rowp_i, lsp_i)) and every upper entry of row k_p, the position of that column in row i (> p) or
// kMapMiss. Segments follow the pivots in order from moff[i].
__global__ void __launch_bounds__(256) k_mc_ilu0_map(int64_t n, const int64_t *__restrict__ rowp,
                                                     const int32_t *__restrict__ col, const int64_t *__restrict__ lsp,
                                                     const int64_t *__restrict__ didx,
                                                     const int64_t *__restrict__ moff, uint16_t *__restrict__ map) {
  __shared__ int32_t sc[4][kIluMaxRow + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 4 + w;
  if (i >= n) return;
  const int64_t rp = rowp[i];
  const int len = (int)(rowp[i + 1] - rp), nl = (int)(lsp[i] - rp);
  for (int e = lane; e < len; e += 64) sc[w][e] = col[rp + e];
  if (lane == 0) sc[w][len] = 0x7fffffff;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  int64_t o = moff[i];
  for (int p = 0; p < nl; ++p) {
    const int k = sc[w][p];
    const int64_t dk = didx[k];
    const int m = (int)(rowp[k + 1] - dk - 1), mp = (m + 3) & ~3;  // segments padded to quads
    for (int e = lane; e < mp; e += 64) {
      const int q = e < m ? lds_find(sc[w], p + 1, len, col[dk + 1 + e]) : -1;
      map[o + e] = q >= 0 ? (uint16_t)q : kMapMiss;
    }
    o += mp;
  }
}
}  // namespace

hipError_t ilu_mc_factor_map(int64_t n, const int64_t *rowp, const int32_t *col, const int64_t *lsp,
                             const int64_t *didx, const int64_t *moff, uint16_t *map, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mc_ilu0_map, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, n, rowp, col, lsp, didx, moff, map);
  return hipGetLastError();
}

hipError_t ilu_mc_factor(const int32_t *grow, const int32_t *color_groups, int n_colors, const int64_t *rowp,
                         const int32_t *col, double *val, const int64_t *lsp, const int64_t *didx, double boost_tol,
                         double boost_val, const int64_t *moff, const uint16_t *map, bool compact, double *rdiag,
                         hipStream_t s) {
  for (int c = 0; c < n_colors; ++c) {
    const int g0 = color_groups[c], g1 = color_groups[c + 1];
    if (g1 <= g0) continue;
    const dim3 gr((unsigned)(g1 - g0)), bl(64 * kMaxGroupRows);
#define GLS_MC_ILU0(MAP, R)                                                                                 \
  hipLaunchKernelGGL((k_mc_ilu0<MAP, 3, R>), gr, bl, 0, s, grow, g0, g1, rowp, col, val, lsp, didx, boost_tol, \
                     boost_val, moff, map, rdiag)
    if (map && compact) GLS_MC_ILU0(true, kIluCompactRow);
    else if (map) GLS_MC_ILU0(true, kIluMaxRow);
    else if (compact) GLS_MC_ILU0(false, kIluCompactRow);
    else GLS_MC_ILU0(false, kIluMaxRow);
#undef GLS_MC_ILU0
  }
  return hipGetLastError();
}

hipError_t ilu_mc_solve(const int64_t *gdesc, const int32_t *color_groups, int n_colors, const int32_t *col,
                        const double *val, const double *b, double *y, double *x, const uint8_t *waves_lower,
                        const uint8_t *waves_upper, hipStream_t s) {
  for (int c = 0; c < n_colors; ++c) {
    const int g0 = color_groups[c], g1 = color_groups[c + 1];
    if (g1 <= g0) continue;
    if (waves_lower[c] >= 4)
      hipLaunchKernelGGL((k_mc_tri<4, true>), dim3((unsigned)(g1 - g0)), dim3(256), 0, s, gdesc, g0, g1, col, val, b, y);
    else
      hipLaunchKernelGGL((k_mc_tri<1, true>), dim3((unsigned)((g1 - g0 + 3) / 4)), dim3(256), 0, s, gdesc, g0, g1, col,
                         val, b, y);
  }
  for (int c = n_colors - 1; c >= 0; --c) {
    const int g0 = color_groups[c], g1 = color_groups[c + 1];
    if (g1 <= g0) continue;
    if (waves_upper[c] >= 4)
      hipLaunchKernelGGL((k_mc_tri<4, false>), dim3((unsigned)(g1 - g0)), dim3(256), 0, s, gdesc, g0, g1, col, val, y, x);
    else
      hipLaunchKernelGGL((k_mc_tri<1, false>), dim3((unsigned)((g1 - g0 + 3) / 4)), dim3(256), 0, s, gdesc, g0, g1, col,
                         val, y, x);
  }
  return hipGetLastError();
}

}  // namespace gls
