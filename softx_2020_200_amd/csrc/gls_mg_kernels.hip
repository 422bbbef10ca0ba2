// gls_mg_kernels.hip — grid-transfer kernels of the geometric multigrid preconditioner.
//
// Nested hyper_cube levels: the Qk node lattice of level l+1 (n/2 cells per direction) is every
// second node of level l (k <= 2: Gauss-Lobatto support points are equidistant). Prolongation
// interpolates the coarse Qk field exactly at the fine nodes; restriction is its transpose.
// Both are applied as three separable 1D passes over a [n2][n1][n0][ncomp] lattice array
// (velocity: ncomp 3 interleaved, pressure: ncomp 1), each thread producing one output entry.
// Multi-GPU: each rank works on the box sub-lattice its cells span (box gather / scatter through
// a box -> local node map); nested partitions keep the coarse box the fine box's every-second node.
#include "gls_launch.hpp"

namespace gls {

namespace {

// parent coarse cell and local coordinate of fine lattice index i (k = degree, ncc = coarse cells)
__device__ __forceinline__ void parent(int i, int k, int ncc, int &c, double &xi) {
  const double x = (double)i / (2.0 * k);  // in coarse-cell units
  c = min((int)floor(x), ncc - 1);
  xi = x - c;
}
__device__ __forceinline__ double lag_eq(int k, int a, double xi) {  // equidistant Lagrange on [0,1]
  double L = 1.0;
  for (int b = 0; b <= k; ++b)
    if (b != a) L *= (xi * k - b) / (double)(a - b);
  return L;
}

// one separable pass along `axis`: in dims (d0,d1,d2) -> out dims with d_axis replaced by nout
__global__ void k_transfer_axis(const double *__restrict__ in, double *__restrict__ out, int d0, int d1, int d2,
                                int axis, int nout, int ncomp, int k, int prolong) {
  int od[3] = {d0, d1, d2};
  od[axis] = nout;
  const int64_t total = (int64_t)od[0] * od[1] * od[2] * ncomp;
  const int nin = axis == 0 ? d0 : (axis == 1 ? d1 : d2);
  const int nfine = prolong ? nout : nin;
  const int ncc = (nfine - 1) / (2 * k);  // coarse cells along the axis
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int comp = (int)(t % ncomp);
    int64_t r = t / ncomp;
    int o[3];
    o[0] = (int)(r % od[0]);
    r /= od[0];
    o[1] = (int)(r % od[1]);
    o[2] = (int)(r / od[1]);
    const int oi = o[axis];
    auto in_at = [&](int j) {
      int p[3] = {o[0], o[1], o[2]};
      p[axis] = j;
      return in[(((int64_t)p[2] * d1 + p[1]) * d0 + p[0]) * ncomp + comp];
    };
    double s = 0.;
    if (prolong) {
      int c;
      double xi;
      parent(oi, k, ncc, c, xi);
      for (int a = 0; a <= k; ++a) s += lag_eq(k, a, xi) * in_at(c * k + a);
    } else {
      const int lo = max(0, 2 * oi - (2 * k - 1)), hi = min(nin - 1, 2 * oi + (2 * k - 1));
      for (int i = lo; i <= hi; ++i) {
        int c;
        double xi;
        parent(i, k, ncc, c, xi);
        const int a = oi - c * k;
        if (a >= 0 && a <= k) s += lag_eq(k, a, xi) * in_at(i);
      }
    }
    out[t] = s;
  }
}

// coarse (I,J,K) <- fine (2I,2J,2K) on box lattices, velocity (3 comps) and pressure parts
__global__ void k_inject(const double *__restrict__ fine, double *__restrict__ coarse, int f0, int f1, int f2, int c0,
                         int c1, int c2) {
  const int64_t nvc = (int64_t)c0 * c1 * c2, nvf = (int64_t)f0 * f1 * f2;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nvc; t += (int64_t)gridDim.x * blockDim.x) {
    const int I = (int)(t % c0), J = (int)((t / c0) % c1), K = (int)(t / ((int64_t)c0 * c1));
    const int64_t f = ((int64_t)(2 * K) * f1 + 2 * J) * f0 + 2 * I;
    coarse[3 * t + 0] = fine[3 * f + 0];
    coarse[3 * t + 1] = fine[3 * f + 1];
    coarse[3 * t + 2] = fine[3 * f + 2];
    coarse[3 * nvc + t] = fine[3 * nvf + f];
  }
}

// rank-local vector [vel (3 interleaved) | p] over n_vnodes nodes <-> box lattice vector over nbox
// nodes (box node t is local node map[t]); gather zeroes non-owned nodes when n_owned >= 0
__global__ void k_box_gather(const double *__restrict__ loc, double *__restrict__ box, const int32_t *__restrict__ map,
                             int64_t nbox, int64_t nvl, int64_t n_owned) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nbox; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t li = map[t];
    const bool on = n_owned < 0 || li < n_owned;
    box[3 * t + 0] = on ? loc[3 * li + 0] : 0.0;
    box[3 * t + 1] = on ? loc[3 * li + 1] : 0.0;
    box[3 * t + 2] = on ? loc[3 * li + 2] : 0.0;
    box[3 * nbox + t] = on ? loc[3 * nvl + li] : 0.0;
  }
}
__global__ void k_box_scatter(const double *__restrict__ box, double *__restrict__ loc, const int32_t *__restrict__ map,
                              int64_t nbox, int64_t nvl) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nbox; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t li = map[t];
    loc[3 * li + 0] = box[3 * t + 0];
    loc[3 * li + 1] = box[3 * t + 1];
    loc[3 * li + 2] = box[3 * t + 2];
    loc[3 * nvl + li] = box[3 * nbox + t];
  }
}

// x += omega * (b - y) / d   (damped Jacobi update, y = A x)
__global__ void k_jacobi_update(double *__restrict__ x, const double *__restrict__ b, const double *__restrict__ y,
                                const double *__restrict__ d, double omega, int64_t n, int zero_start) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double r = zero_start ? b[i] : b[i] - y[i];
    x[i] = (zero_start ? 0.0 : x[i]) + omega * r / d[i];
  }
}

int grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (int)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace

// out = T(in) for one Qk vector [vel (3 comps interleaved) | pressure] on a box node lattice
// (dims x, y, z), T = prolongation (nin -> nout = 2 nin - 1 per axis) or restriction (nin -> nout,
// nin = 2 nout - 1); tmp1/tmp2 hold the intermediate passes.
hipError_t mg_transfer(const double *in, double *out, const int nin[3], const int nout[3], int k, int prolong,
                       double *tmp1, double *tmp2, hipStream_t s) {
  const int64_t nvi = (int64_t)nin[0] * nin[1] * nin[2], nvo = (int64_t)nout[0] * nout[1] * nout[2];
  for (int part = 0; part < 2; ++part) {
    const int nc = part == 0 ? 3 : 1;
    const double *src = in + (part == 0 ? 0 : 3 * nvi);
    double *dst = out + (part == 0 ? 0 : 3 * nvo);
    // axis 0: (i0,i1,i2) -> (o0,i1,i2); axis 1 -> (o0,o1,i2); axis 2 -> (o0,o1,o2)
    const int64_t s1 = (int64_t)nout[0] * nin[1] * nin[2] * nc, s2 = (int64_t)nout[0] * nout[1] * nin[2] * nc,
                  s3 = nvo * nc;
    hipLaunchKernelGGL(k_transfer_axis, dim3(grid_for(s1)), dim3(256), 0, s, src, tmp1, nin[0], nin[1], nin[2], 0,
                       nout[0], nc, k, prolong);
    hipLaunchKernelGGL(k_transfer_axis, dim3(grid_for(s2)), dim3(256), 0, s, tmp1, tmp2, nout[0], nin[1], nin[2], 1,
                       nout[1], nc, k, prolong);
    hipLaunchKernelGGL(k_transfer_axis, dim3(grid_for(s3)), dim3(256), 0, s, tmp2, dst, nout[0], nout[1], nin[2], 2,
                       nout[2], nc, k, prolong);
  }
  return hipGetLastError();
}

hipError_t mg_inject(const double *fine, double *coarse, const int nf[3], const int nc[3], hipStream_t s) {
  hipLaunchKernelGGL(k_inject, dim3(grid_for((int64_t)nc[0] * nc[1] * nc[2])), dim3(256), 0, s, fine, coarse, nf[0],
                     nf[1], nf[2], nc[0], nc[1], nc[2]);
  return hipGetLastError();
}

hipError_t mg_box_gather(const double *loc, double *box, const int32_t *map, int64_t nbox, int64_t nvl,
                         int64_t n_owned, hipStream_t s) {
  hipLaunchKernelGGL(k_box_gather, dim3(grid_for(nbox)), dim3(256), 0, s, loc, box, map, nbox, nvl, n_owned);
  return hipGetLastError();
}

hipError_t mg_box_scatter(const double *box, double *loc, const int32_t *map, int64_t nbox, int64_t nvl,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_box_scatter, dim3(grid_for(nbox)), dim3(256), 0, s, box, loc, map, nbox, nvl);
  return hipGetLastError();
}

hipError_t mg_jacobi_update(double *x, const double *b, const double *y, const double *d, double omega, int64_t n,
                            int zero_start, hipStream_t s) {
  hipLaunchKernelGGL(k_jacobi_update, dim3(grid_for(n)), dim3(256), 0, s, x, b, y, d, omega, n, zero_start);
  return hipGetLastError();
}

}  // namespace gls
