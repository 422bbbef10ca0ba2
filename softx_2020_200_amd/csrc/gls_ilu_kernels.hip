// gls_ilu_kernels.hip — triangular solves of the assembled ILU in multicolor order (gls_ilu_attach
// with GLS_ILU_ORDER_MULTICOLOR).
//
// In that order the DoFs of one color belong to nodes that share no matrix entry, so inside a color
// a row depends on rows of earlier colors (forward) / later colors (backward) and on the rows of its
// own node only. One launch per color, one wavefront per node group: the 64 lanes stride over the
// row's entries of the other colors (a gather-dot, HBM / L2 bound), then lane 0 resolves the <= 4
// rows of the node in order. The dependency chain of a solve is the number of colors, where the
// general level-scheduled csrsv of a Cuthill-McKee-ordered 3D Q2 matrix waits on thousands of
// levels (profiles/r03_ilu_multicolor_ab.txt).
#include "gls_launch.hpp"

namespace gls {

namespace {
constexpr int kGroupsPerBlock = 4;  // 256 threads = 4 wavefronts = 4 node groups

__device__ __forceinline__ double wave_sum(double s) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// forward: y_i = b_i - sum_{j < i} L_ij y_j (unit lower); entries [rowp_i, lsp_i) lie in earlier colors,
// [lsp_i, didx_i) in the row's own node
__global__ void __launch_bounds__(256) k_mc_lower(const int32_t *__restrict__ grow, int g0, int g1,
                                                  const int32_t *__restrict__ rowp, const int32_t *__restrict__ col,
                                                  const double *__restrict__ val, const int32_t *__restrict__ lsp,
                                                  const int32_t *__restrict__ didx, const double *__restrict__ b,
                                                  double *__restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int g = g0 + (int)blockIdx.x * kGroupsPerBlock + (int)(threadIdx.x >> 6);
  if (g >= g1) return;
  const int r0 = grow[g], r1 = grow[g + 1];
  double part[kMaxGroupRows];
#pragma unroll
  for (int t = 0; t < kMaxGroupRows; ++t) {
    double s = 0.0;
    if (r0 + t < r1) {
      const int i = r0 + t;
      for (int e = rowp[i] + lane; e < lsp[i]; e += 64) s += val[e] * y[col[e]];
    }
    part[t] = wave_sum(s);
  }
  if (lane == 0) {
    for (int t = 0; t < r1 - r0; ++t) {
      const int i = r0 + t;
      double s = b[i] - part[t];
      for (int e = lsp[i]; e < didx[i]; ++e) s -= val[e] * y[col[e]];
      y[i] = s;
    }
  }
}

// backward: x_i = (y_i - sum_{j > i} U_ij x_j) / U_ii; entries [usp_i, rowp_{i+1}) lie in later colors,
// (didx_i, usp_i) in the row's own node
__global__ void __launch_bounds__(256) k_mc_upper(const int32_t *__restrict__ grow, int g0, int g1,
                                                  const int32_t *__restrict__ rowp, const int32_t *__restrict__ col,
                                                  const double *__restrict__ val, const int32_t *__restrict__ usp,
                                                  const int32_t *__restrict__ didx, const double *__restrict__ y,
                                                  double *__restrict__ x) {
  const int lane = threadIdx.x & 63;
  const int g = g0 + (int)blockIdx.x * kGroupsPerBlock + (int)(threadIdx.x >> 6);
  if (g >= g1) return;
  const int r0 = grow[g], r1 = grow[g + 1];
  double part[kMaxGroupRows];
#pragma unroll
  for (int t = 0; t < kMaxGroupRows; ++t) {
    double s = 0.0;
    if (r0 + t < r1) {
      const int i = r0 + t;
      for (int e = usp[i] + lane; e < rowp[i + 1]; e += 64) s += val[e] * x[col[e]];
    }
    part[t] = wave_sum(s);
  }
  if (lane == 0) {
    for (int t = r1 - r0 - 1; t >= 0; --t) {
      const int i = r0 + t;
      double s = y[i] - part[t];
      for (int e = didx[i] + 1; e < usp[i]; ++e) s -= val[e] * x[col[e]];
      x[i] = s / val[didx[i]];
    }
  }
}
}  // namespace

hipError_t ilu_mc_solve(const int32_t *grow, const int32_t *color_groups, int n_colors, const int32_t *rowp,
                        const int32_t *col, const double *val, const int32_t *lsp, const int32_t *usp,
                        const int32_t *didx, const double *b, double *y, double *x, hipStream_t s) {
  for (int c = 0; c < n_colors; ++c) {
    const int g0 = color_groups[c], g1 = color_groups[c + 1];
    if (g1 <= g0) continue;
    const unsigned nb = (unsigned)((g1 - g0 + kGroupsPerBlock - 1) / kGroupsPerBlock);
    hipLaunchKernelGGL(k_mc_lower, dim3(nb), dim3(64 * kGroupsPerBlock), 0, s, grow, g0, g1, rowp, col, val, lsp, didx, b, y);
  }
  for (int c = n_colors - 1; c >= 0; --c) {
    const int g0 = color_groups[c], g1 = color_groups[c + 1];
    if (g1 <= g0) continue;
    const unsigned nb = (unsigned)((g1 - g0 + kGroupsPerBlock - 1) / kGroupsPerBlock);
    hipLaunchKernelGGL(k_mc_upper, dim3(nb), dim3(64 * kGroupsPerBlock), 0, s, grow, g0, g1, rowp, col, val, usp, didx, y, x);
  }
  return hipGetLastError();
}

}  // namespace gls
