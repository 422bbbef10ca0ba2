// gls_mg_kernels.hip — grid-transfer kernels of the geometric multigrid preconditioner.
//
// Nested hyper_cube levels: the Qk node lattice of level l+1 (n/2 cells per direction) is every
// second node of level l (k <= 2: Gauss-Lobatto support points are equidistant). Prolongation
// interpolates the coarse Qk field exactly at the fine nodes; restriction is its transpose. Both
// run as ONE gather pass per transfer (thread per output node, tensor product of per-axis tap
// tables built on the host), velocity and pressure together: the fine vector is read or written
// once (the earlier three separable passes moved ~3.5x the bytes).
// Multi-GPU: each rank works on the box sub-lattice its cells span (box gather / scatter through
// a box -> local node map); nested partitions keep the coarse box the fine box's every-second node.
#include "gls_launch.hpp"

namespace gls {

namespace {

// Direct 3D transfer: out[o] = sum over the tensor product of per-axis taps (<= kMaxTaps each,
// weight 0 pads) of w_x w_y w_z in[i]; velocity (3 interleaved) and pressure in one pass. The tap
// tables are the 1D prolongation (fine <- coarse) or its transpose (restriction) per axis.
constexpr int kMaxTaps = 5;
__global__ void __launch_bounds__(256) k_transfer3d(const double *__restrict__ in, double *__restrict__ out, int i0,
                                                    int i1, int i2, int o0, int o1, int o2,
                                                    const int32_t *__restrict__ tx, const double *__restrict__ wx,
                                                    const int32_t *__restrict__ ty, const double *__restrict__ wy,
                                                    const int32_t *__restrict__ tz, const double *__restrict__ wz) {
  const int64_t nin = (int64_t)i0 * i1 * i2, nout = (int64_t)o0 * o1 * o2;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nout; t += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(t % o0), y = (int)((t / o0) % o1), z = (int)(t / ((int64_t)o0 * o1));
    double s0 = 0., s1 = 0., s2 = 0., sp = 0.;
    for (int c = 0; c < kMaxTaps; ++c) {
      const double az = wz[z * kMaxTaps + c];
      if (az == 0.0) continue;
      const int64_t bz = (int64_t)tz[z * kMaxTaps + c] * i1;
      for (int b = 0; b < kMaxTaps; ++b) {
        const double ay = wy[y * kMaxTaps + b];
        if (ay == 0.0) continue;
        const int64_t by = (bz + ty[y * kMaxTaps + b]) * i0;
        const double ayz = ay * az;
        for (int a = 0; a < kMaxTaps; ++a) {
          const double ax = wx[x * kMaxTaps + a];
          if (ax == 0.0) continue;
          const int64_t n = by + tx[x * kMaxTaps + a];
          const double w = ax * ayz;
          s0 += w * in[3 * n];
          s1 += w * in[3 * n + 1];
          s2 += w * in[3 * n + 2];
          sp += w * in[3 * nin + n];
        }
      }
    }
    out[3 * t] = s0;
    out[3 * t + 1] = s1;
    out[3 * t + 2] = s2;
    out[3 * nout + t] = sp;
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

hipError_t mg_transfer3d(const double *in, double *out, const int nin[3], const int nout[3],
                         const int32_t *const taps[3], const double *const w[3], hipStream_t s) {
  const int64_t n = (int64_t)nout[0] * nout[1] * nout[2];
  const int64_t b = (n + 255) / 256;
  hipLaunchKernelGGL(k_transfer3d, dim3((int)(b < 65536 ? (b > 0 ? b : 1) : 65536)), dim3(256), 0, s, in, out, nin[0],
                     nin[1], nin[2], nout[0], nout[1], nout[2], taps[0], w[0], taps[1], w[1], taps[2], w[2]);
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
