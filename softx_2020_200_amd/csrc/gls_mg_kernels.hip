// gls_mg_kernels.hip — grid-transfer kernels of the geometric multigrid preconditioner.
//
// Nested hyper_cube levels: the Qk node lattice of level l+1 (n/2 cells per direction) is every
// second node of level l (k <= 2: Gauss-Lobatto support points are equidistant). Prolongation
// interpolates the coarse Qk field exactly at the fine nodes; restriction is its transpose. Both
// run as two passes (an LDS-tiled xy pass per plane + a coalesced z pass, per-axis tap tables built
// on the host), velocity and pressure together; the one-pass 125-tap gather remains for lattices
// whose tiles do not fit (it reads the fine vector once but is load-issue bound: 0.45 / 0.72 ms
// for the 128^3 restriction / prolongation).
// Multi-GPU: each rank works on the box sub-lattice its cells span (box gather / scatter through
// a box -> local node map); nested partitions keep the coarse box the fine box's every-second node.
#include "gls_launch.hpp"

namespace gls {

namespace {

// Direct 3D transfer: out[o] = sum over the tensor product of per-axis taps of w_x w_y w_z in[i];
// velocity (3 interleaved) and pressure in one pass. The tap tables are the 1D prolongation
// (fine <- coarse) or its transpose (restriction) per axis: [n_out][kMaxTaps] (index, weight),
// nonzero taps first, their count in cnt[n_out]. 32-bit lattice indices (boxes < 2^31 nodes).
constexpr int kMaxTaps = 5;
// two-pass transfer tiles (outputs per block in x, y) and their input-range bounds
constexpr int kRestrictTile[2] = {16, 8}, kRestrictIn[2] = {36, 20};
constexpr int kProlongTile[2] = {32, 16}, kProlongIn[2] = {20, 12};
__global__ void __launch_bounds__(256) k_transfer3d(const double *__restrict__ in, double *__restrict__ out, int i0,
                                                    int i1, int i2, int o0, int o1, int o2,
                                                    const int32_t *__restrict__ tx, const double *__restrict__ wx,
                                                    const int32_t *__restrict__ cx, const int32_t *__restrict__ ty,
                                                    const double *__restrict__ wy, const int32_t *__restrict__ cy,
                                                    const int32_t *__restrict__ tz, const double *__restrict__ wz,
                                                    const int32_t *__restrict__ cz) {
  const int nin = i0 * i1 * i2, nout = o0 * o1 * o2;
  const int plane = o0 * o1;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nout; t += gridDim.x * blockDim.x) {
    const int z = t / plane, r = t - z * plane, y = r / o0, x = r - y * o0;
    const int nzz = cz[z], nyy = cy[y], nxx = cx[x];
    double s0 = 0., s1 = 0., s2 = 0., sp = 0.;
    for (int c = 0; c < nzz; ++c) {
      const double az = wz[z * kMaxTaps + c];
      const int bz = tz[z * kMaxTaps + c] * i1;
      for (int b = 0; b < nyy; ++b) {
        const double ayz = wy[y * kMaxTaps + b] * az;
        const int by = (bz + ty[y * kMaxTaps + b]) * i0;
        for (int a = 0; a < nxx; ++a) {
          const int n = by + tx[x * kMaxTaps + a];
          const double w = wx[x * kMaxTaps + a] * ayz;
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

// Two-pass transfer (the default where the tiles fit): an xy pass per z plane staged through LDS
// (input tile loaded once, x taps then y taps from LDS) and a 1D z pass over whole planes
// (coalesced). Restriction runs xy first (the fine vector shrinks 4x before the z pass), and
// prolongation z first; the intermediate array is (xy of the smaller lattice) x (z of the larger),
// so the traffic is 1.6x the single-pass bytes with ~8x fewer loads than the 125-tap gather above.
// A tile of OX x OY outputs reads the input x range [min first tap, max last tap] over its outputs,
// <= IXM x IYM (checked on the host when the tables are built).
#ifndef GLS_XFER_NT
#define GLS_XFER_NT 1  // input tiles read non-temporally (neighbouring tiles share only their halo)
#endif
__device__ __forceinline__ double xfer_load(const double *p) {
#if GLS_XFER_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
template <int OX, int OY, int IXM, int IYM>
__global__ void __launch_bounds__(256) k_transfer_xy(const double *__restrict__ in, double *__restrict__ out, int i0,
                                                     int i1, int o0, int o1, int nz, int zb,
                                                     const int32_t *__restrict__ tx, const double *__restrict__ wx,
                                                     const int32_t *__restrict__ cx, const int32_t *__restrict__ ty,
                                                     const double *__restrict__ wy, const int32_t *__restrict__ cy,
                                                     int add) {
  __shared__ double s_in[4][IYM][IXM + 1];
  __shared__ double s_t1[4][IYM][OX + 1];
  __shared__ int s_xi[OX][kMaxTaps], s_yi[OY][kMaxTaps], s_xc[OX], s_yc[OY];
  __shared__ double s_xw[OX][kMaxTaps], s_yw[OY][kMaxTaps];
  __shared__ int s_rng[4];
  const int ntx = (o0 + OX - 1) / OX;
  const int ox0 = (blockIdx.x % ntx) * OX, oy0 = (blockIdx.x / ntx) * OY;
  const int z0 = blockIdx.y * zb, z1 = min(z0 + zb, nz);
  const int nox = min(OX, o0 - ox0), noy = min(OY, o1 - oy0);
  const int tid = threadIdx.x;
  // input range of the tile: min first tap / max last tap over its outputs (each output's taps ascend)
  if (tid < 4) s_rng[tid] = (tid & 1) ? -1 : 0x7fffffff;
  __syncthreads();
  if (tid < nox) {
    atomicMin(&s_rng[0], tx[(ox0 + tid) * kMaxTaps]);
    atomicMax(&s_rng[1], tx[(ox0 + tid) * kMaxTaps + cx[ox0 + tid] - 1]);
  } else if (tid >= 64 && tid - 64 < noy) {
    atomicMin(&s_rng[2], ty[(oy0 + tid - 64) * kMaxTaps]);
    atomicMax(&s_rng[3], ty[(oy0 + tid - 64) * kMaxTaps + cy[oy0 + tid - 64] - 1]);
  }
  for (int e = tid; e < OX * kMaxTaps; e += 256) {
    const int o = e / kMaxTaps, a = e - o * kMaxTaps;
    const bool ok = o < nox;
    s_xi[o][a] = ok ? tx[(ox0 + o) * kMaxTaps + a] : 0;
    s_xw[o][a] = ok ? wx[(ox0 + o) * kMaxTaps + a] : 0.0;
    if (a == 0) s_xc[o] = ok ? cx[ox0 + o] : 0;
  }
  for (int e = tid; e < OY * kMaxTaps; e += 256) {
    const int o = e / kMaxTaps, a = e - o * kMaxTaps;
    const bool ok = o < noy;
    s_yi[o][a] = ok ? ty[(oy0 + o) * kMaxTaps + a] : 0;
    s_yw[o][a] = ok ? wy[(oy0 + o) * kMaxTaps + a] : 0.0;
    if (a == 0) s_yc[o] = ok ? cy[oy0 + o] : 0;
  }
  __syncthreads();
  const int lox = s_rng[0], loy = s_rng[2], nix = s_rng[1] - lox + 1, niy = s_rng[3] - loy + 1;
  const int64_t nin = (int64_t)i0 * i1 * nz, nout = (int64_t)o0 * o1 * nz;
  // per-thread load slots (velocity rows: 3 * nix contiguous doubles; pressure rows: nix), fixed
  // for every plane; plane z+1 is loaded into registers while plane z is computed
  constexpr int NV = (IYM * 3 * IXM + 255) / 256, NP = (IYM * IXM + 255) / 256;
  int offv[NV], offp[NP];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int e = tid + u * 256, yy = e / (3 * nix), r = e - yy * 3 * nix;
    offv[u] = e < niy * 3 * nix ? 3 * ((loy + yy) * i0 + lox) + r : -1;
  }
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int e = tid + u * 256, yy = e / nix, xx = e - yy * nix;
    offp[u] = e < niy * nix ? (loy + yy) * i0 + lox + xx : -1;
  }
  double rv[NV], rp[NP];
  auto load_plane = [&](int z) {
    const double *pv = in + 3 * (int64_t)z * i1 * i0, *pp = in + 3 * nin + (int64_t)z * i1 * i0;
#pragma unroll
    for (int u = 0; u < NV; ++u) rv[u] = offv[u] >= 0 ? xfer_load(pv + offv[u]) : 0.0;
#pragma unroll
    for (int u = 0; u < NP; ++u) rp[u] = offp[u] >= 0 ? xfer_load(pp + offp[u]) : 0.0;
  };
  if (z0 < z1) load_plane(z0);
  for (int z = z0; z < z1; ++z) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int e = tid + u * 256, yy = e / (3 * nix), r = e - yy * 3 * nix;
      if (offv[u] >= 0) s_in[r % 3][yy][r / 3] = rv[u];
    }
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int e = tid + u * 256, yy = e / nix, xx = e - yy * nix;
      if (offp[u] >= 0) s_in[3][yy][xx] = rp[u];
    }
    __syncthreads();
    if (z + 1 < z1) load_plane(z + 1);
    for (int e = tid; e < 4 * niy * OX; e += 256) {
      const int f = e / (niy * OX), r = e - f * niy * OX, yy = r / OX, o = r - yy * OX;
      double s = 0.0;
      for (int a = 0; a < s_xc[o]; ++a) s += s_xw[o][a] * s_in[f][yy][s_xi[o][a] - lox];
      s_t1[f][yy][o] = s;
    }
    __syncthreads();
    const int64_t pout = (int64_t)z * o1 * o0;
    for (int e = tid; e < noy * 3 * OX; e += 256) {
      const int oy = e / (3 * OX), r = e - oy * 3 * OX, o = r / 3, f = r - 3 * o;
      if (o >= nox) continue;
      double s = 0.0;
      for (int b = 0; b < s_yc[oy]; ++b) s += s_yw[oy][b] * s_t1[f][s_yi[oy][b] - loy][o];
      double *o_ = out + 3 * (pout + (int64_t)(oy0 + oy) * o0 + ox0) + r;
      *o_ = add ? *o_ + s : s;
    }
    for (int e = tid; e < noy * OX; e += 256) {
      const int oy = e / OX, o = e - oy * OX;
      if (o >= nox) continue;
      double s = 0.0;
      for (int b = 0; b < s_yc[oy]; ++b) s += s_yw[oy][b] * s_t1[3][s_yi[oy][b] - loy][o];
      double *o_ = out + 3 * nout + pout + (int64_t)(oy0 + oy) * o0 + ox0 + o;
      *o_ = add ? *o_ + s : s;
    }
  }
}

// z pass over whole planes of P nodes: out plane oz = sum_c wz[oz][c] in plane tz[oz][c]
__global__ void __launch_bounds__(256) k_transfer_z(const double *__restrict__ in, double *__restrict__ out, int64_t P,
                                                    int nzi, int nzo, const int32_t *__restrict__ tz,
                                                    const double *__restrict__ wz, const int32_t *__restrict__ cz) {
  const int oz = blockIdx.y;
  const int nc = cz[oz];
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < 4 * P; e += (int64_t)gridDim.x * blockDim.x) {
    const bool vel = e < 3 * P;
    const int64_t base_i = vel ? e : 3 * P * nzi + (e - 3 * P);
    const int64_t pl = vel ? 3 * P : P;
    double v[kMaxTaps];
#pragma unroll
    for (int c = 0; c < kMaxTaps; ++c) v[c] = c < nc ? in[base_i + (int64_t)tz[oz * kMaxTaps + c] * pl] : 0.0;
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < kMaxTaps; ++c) s += c < nc ? wz[oz * kMaxTaps + c] * v[c] : 0.0;
    out[vel ? (int64_t)oz * pl + e : 3 * P * nzo + (int64_t)oz * pl + (e - 3 * P)] = s;
  }
}

template <int OX, int OY, int IXM, int IYM>
hipError_t launch_transfer_xy(const double *in, double *out, int i0, int i1, int o0, int o1, int nz,
                              const int32_t *const taps[3], const double *const w[3], const int32_t *const cnt[3],
                              hipStream_t s, int add = 0) {
  const int nb = ((o0 + OX - 1) / OX) * ((o1 + OY - 1) / OY);
  // planes per block (prefetch pipeline depth): 2 planes (4x the blocks in flight of the former 8: 93.4-93.6 vs 93.8-94.1 ms per Newton step
  // at configs[2], profiles/r04_ab_transfer_planes.txt)
  const int zb = nz >= 16 ? 2 : 1;
  hipLaunchKernelGGL((k_transfer_xy<OX, OY, IXM, IYM>), dim3(nb, (nz + zb - 1) / zb), dim3(256), 0, s, in, out, i0, i1,
                     o0, o1, nz, zb, taps[0], w[0], cnt[0], taps[1], w[1], cnt[1], add);
  return hipGetLastError();
}

hipError_t launch_transfer_z(const double *in, double *out, int64_t P, int nzi, int nzo, const int32_t *tz,
                             const double *wz, const int32_t *cz, hipStream_t s) {
  const int64_t b = (4 * P + 255) / 256;
  hipLaunchKernelGGL(k_transfer_z, dim3((unsigned)std::min<int64_t>(b, 1024), nzo), dim3(256), 0, s, in, out, P, nzi,
                     nzo, tz, wz, cz);
  return hipGetLastError();
}

// Coarsest-level direct solve. The coarse Jacobian A (n <= a few thousand DoFs) is probed
// column by column (Y[j*n + i] = (A e_j)_i) and inverted by Gauss-Jordan with partial pivoting
// on [A | I] in ONE workgroup; each V-cycle then applies x = A^+ b (dense GEMV). A pivot below
// 1e-12 max|A| marks a dependent column (the enclosed-flow Jacobian has the constant-pressure
// null vector): that unknown is dropped (set to 0), which gives a particular solution of the
// consistent part instead of amplifying the null direction. status = number of dropped columns.
constexpr int kGJThreads = 1024;
__global__ void __launch_bounds__(kGJThreads) k_gauss_jordan(const double *__restrict__ Y, double *__restrict__ aug, int n,
                                                          int *status) {
  __shared__ double red_v[kGJThreads];
  __shared__ int red_i[kGJThreads];
  const int tid = threadIdx.x, w = 2 * n;
  double amax = 0.0;
  for (int64_t t = tid; t < (int64_t)n * w; t += kGJThreads) {
    const int i = (int)(t / w), j = (int)(t % w);
    double v;
    if (j < n) {
      v = Y[(int64_t)j * n + i];
      amax = fmax(amax, fabs(v));
    } else {
      v = (j - n == i) ? 1.0 : 0.0;
    }
    aug[t] = v;
  }
  red_v[tid] = amax;
  __syncthreads();
  for (int st = kGJThreads / 2; st > 0; st >>= 1) {
    if (tid < st) red_v[tid] = fmax(red_v[tid], red_v[tid + st]);
    __syncthreads();
  }
  const double tiny = 1e-12 * red_v[0];
  __syncthreads();
  int dropped = 0;
  for (int k = 0; k < n; ++k) {
    // pivot search in column k, rows k..n-1
    double best = -1.0;
    int bi = k;
    for (int i = k + tid; i < n; i += kGJThreads) {
      const double a = fabs(aug[(int64_t)i * w + k]);
      if (a > best) { best = a; bi = i; }
    }
    red_v[tid] = best;
    red_i[tid] = bi;
    __syncthreads();
    for (int st = kGJThreads / 2; st > 0; st >>= 1) {
      if (tid < st && (red_v[tid + st] > red_v[tid] || (red_v[tid + st] == red_v[tid] && red_i[tid + st] < red_i[tid]))) {
        red_v[tid] = red_v[tid + st];
        red_i[tid] = red_i[tid + st];
      }
      __syncthreads();
    }
    const int piv = red_i[0];
    const double pval = red_v[0];
    __syncthreads();
    if (!(pval > tiny)) {  // dependent column: drop unknown k
      for (int i = tid; i < n; i += kGJThreads) aug[(int64_t)i * w + k] = 0.0;
      __syncthreads();
      for (int j = tid; j < w; j += kGJThreads) aug[(int64_t)k * w + j] = (j == k) ? 1.0 : 0.0;
      ++dropped;
      __syncthreads();
      continue;
    }
    if (piv != k)
      for (int j = tid; j < w; j += kGJThreads) {
        const double t0 = aug[(int64_t)k * w + j];
        aug[(int64_t)k * w + j] = aug[(int64_t)piv * w + j];
        aug[(int64_t)piv * w + j] = t0;
      }
    __syncthreads();
    const double inv = 1.0 / aug[(int64_t)k * w + k];
    __syncthreads();
    for (int j = tid; j < w; j += kGJThreads) aug[(int64_t)k * w + j] *= inv;
    __syncthreads();
    // eliminate column k from every other row: a wave per row, lanes along the row; row k is
    // zero left of column k, so only columns > k change
    {
      const int wave = tid >> 6, lane = tid & 63;
      const double *rk = aug + (int64_t)k * w;
      for (int i = wave; i < n; i += kGJThreads / 64) {
        if (i == k) continue;
        double *ri = aug + (int64_t)i * w;
        const double f = ri[k];
        if (f == 0.0) continue;
        for (int j = k + 1 + lane; j < w; j += 64) ri[j] -= f * rk[j];
      }
    }
    __syncthreads();
    for (int i = tid; i < n; i += kGJThreads)
      if (i != k) aug[(int64_t)i * w + k] = 0.0;
    __syncthreads();
  }
  if (tid == 0) *status = dropped;
}

// x = A^-1 b with A^-1 the right half of the Gauss-Jordan result (row stride 2n)
__global__ void k_dense_inv_apply(const double *__restrict__ aug, int n, const double *__restrict__ b,
                                  double *__restrict__ x) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double *row = aug + (int64_t)i * 2 * n + n;
  double s = 0.0;
  for (int j = 0; j < n; ++j) s += row[j] * b[j];
  x[i] = s;
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
                         const int32_t *const taps[3], const double *const w[3], const int32_t *const cnt[3],
                         hipStream_t s) {
  const int64_t n = (int64_t)nout[0] * nout[1] * nout[2];
  const int64_t b = (n + 255) / 256;
  hipLaunchKernelGGL(k_transfer3d, dim3((int)(b < 65536 ? (b > 0 ? b : 1) : 65536)), dim3(256), 0, s, in, out, nin[0],
                     nin[1], nin[2], nout[0], nout[1], nout[2], taps[0], w[0], cnt[0], taps[1], w[1], cnt[1], taps[2],
                     w[2], cnt[2]);
  return hipGetLastError();
}

int mg_transfer_tile_fits(int restrict_, int axis, int n_out, const int32_t *taps, const int32_t *cnt) {
  const int O = restrict_ ? kRestrictTile[axis] : kProlongTile[axis];
  const int IM = restrict_ ? kRestrictIn[axis] : kProlongIn[axis];
  if (O > 64) return 0;  // the kernel's range reduction uses one lane per output
  for (int o0 = 0; o0 < n_out; o0 += O) {
    int lo = 1 << 30, hi = -1;
    for (int o = o0; o < std::min(o0 + O, n_out); ++o) {
      if (cnt[o] < 1 || cnt[o] > kMaxTaps) return 0;
      for (int a = 1; a < cnt[o]; ++a)
        if (taps[o * kMaxTaps + a] <= taps[o * kMaxTaps + a - 1]) return 0;
      lo = std::min(lo, taps[o * kMaxTaps]);
      hi = std::max(hi, taps[o * kMaxTaps + cnt[o] - 1]);
    }
    if (hi - lo + 1 > IM) return 0;
  }
  return 1;
}

hipError_t mg_transfer_2pass(const double *in, double *out, const int nin[3], const int nout[3], int restrict_,
                             const int32_t *const taps[3], const double *const w[3], const int32_t *const cnt[3],
                             double *work, hipStream_t s, int add) {
  if (restrict_) {  // xy (fine planes -> coarse xy), then z
    const hipError_t e = launch_transfer_xy<kRestrictTile[0], kRestrictTile[1], kRestrictIn[0], kRestrictIn[1]>(
        in, work, nin[0], nin[1], nout[0], nout[1], nin[2], taps, w, cnt, s);
    if (e != hipSuccess) return e;
    return launch_transfer_z(work, out, (int64_t)nout[0] * nout[1], nin[2], nout[2], taps[2], w[2], cnt[2], s);
  }
  const hipError_t e = launch_transfer_z(in, work, (int64_t)nin[0] * nin[1], nin[2], nout[2], taps[2], w[2], cnt[2], s);
  if (e != hipSuccess) return e;
  return launch_transfer_xy<kProlongTile[0], kProlongTile[1], kProlongIn[0], kProlongIn[1]>(
      work, out, nin[0], nin[1], nout[0], nout[1], nout[2], taps, w, cnt, s, add);
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

__global__ void k_unit(double *e, int64_t j) {  // e_{j-1} -> e_j (probing)
  if (threadIdx.x == 0) {
    if (j > 0) e[j - 1] = 0.0;
    e[j] = 1.0;
  }
}
hipError_t mg_unit_step(double *e, int64_t j, hipStream_t s) {
  hipLaunchKernelGGL(k_unit, dim3(1), dim3(64), 0, s, e, j);
  return hipGetLastError();
}

__global__ void k_probe_fix(double *Y, int64_t n, int64_t j0, int nprobe, const int64_t *con, int64_t ncon,
                            const double *d) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)nprobe * ncon) return;
  const int64_t j = t / ncon, c = con[t % ncon];
  Y[j * n + c] = (c == j0 + j) ? d[c] : 0.0;
}
hipError_t mg_probe_fix(double *Y, int64_t n, int64_t j0, int nprobe, const int64_t *con, int64_t ncon, const double *d,
                        hipStream_t s) {
  const int64_t tot = (int64_t)nprobe * ncon;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(k_probe_fix, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, Y, n, j0, nprobe, con, ncon, d);
  return hipGetLastError();
}

// column-major A (n x n): row and column `pin` -> identity (fixes the enclosed-flow pressure gauge)
__global__ void k_pin(double *A, int64_t n, int64_t pin) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    A[pin * n + t] = t == pin ? 1.0 : 0.0;  // column pin
    A[t * n + pin] = t == pin ? 1.0 : 0.0;  // row pin
  }
}
hipError_t mg_pin_dof(double *A, int64_t n, int64_t pin, hipStream_t s) {
  hipLaunchKernelGGL(k_pin, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, n, pin);
  return hipGetLastError();
}
__global__ void k_zero_row(double *A, int64_t n, int64_t row) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    A[t * n + row] = 0.0;
}
hipError_t mg_zero_row(double *A, int64_t n, int64_t row, hipStream_t s) {
  hipLaunchKernelGGL(k_zero_row, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, n, row);
  return hipGetLastError();
}

hipError_t mg_dense_invert(const double *Y, double *aug, int n, int *status, hipStream_t s) {
  hipLaunchKernelGGL(k_gauss_jordan, dim3(1), dim3(kGJThreads), 0, s, Y, aug, n, status);
  return hipGetLastError();
}

hipError_t mg_dense_apply(const double *aug, int n, const double *b, double *x, hipStream_t s) {
  hipLaunchKernelGGL(k_dense_inv_apply, dim3((n + 255) / 256), dim3(256), 0, s, aug, n, b, x);
  return hipGetLastError();
}

// ---- dense LU solves of the coarsest level (FP32 factor of rocSOLVER getrf_npvt: column-major, lda = n, unit
// lower L below the diagonal, U on and above it); x overwritten. Block-column steps of kLuB rows: step k has the
// block k solution final; its workgroup 0 applies that block's column to the rows of the next block and solves the
// next diagonal block in LDS (one column at a time), the other workgroups apply it to the rows beyond. 2 n / kLuB
// launches per solve against rocBLAS trsv's 62 ms at n = 25000 (profiles/r06_lu25k.txt).
constexpr int kLuB = 128;
namespace {
// Step k (k < 0: the first diagonal block alone, block 0 forward / the last block backward): workgroup 0 applies
// block column k to the next diagonal block's rows and solves that diagonal block, the others apply block column k
// to the rows beyond. A launch is bound by memory latency, so every global load of it is issued in ONE round before
// anything waits: the right-hand side, block k's solution, and the two 128 x 128 blocks workgroup 0 reads (its rows
// of block column k, the diagonal block), 16-byte loads along the columns, 16 + 16 per thread of 256, staged in LDS.
// (Rounds of dependent loads cost ~2 us each: 128 rounds of one load per thread, 72 / 113 us per forward / backward
// launch; rounds of 32, 21 us; profiles/r06_lu_solve_ab.txt.) The diagonal block is then solved by two wavefronts
// in turn, one column at a time with the column's value broadcast from its lane by v_readlane (no workgroup
// barrier in the sequential part; one hands the first half to the second).
constexpr int kLuT = 256;
template <bool LOWER, bool VEC>
__global__ void __launch_bounds__(kLuT) k_lu_step(const float *__restrict__ A, int n, float *__restrict__ x, int k,
                                                  int rlo) {  // rlo: backward, the first row block the others update
  __shared__ float xk[kLuB], xb[kLuB], rd[kLuB], part[2][kLuB];
  __shared__ float D[kLuB][kLuB + 1], C[kLuB][kLuB + 1];
  const int t = threadIdx.x, nb = (n + kLuB - 1) / kLuB;
  const bool first = k < 0, diag = blockIdx.x == 0;
  const int j0 = first ? 0 : k * kLuB, nj = first ? 1 : min(kLuB, n - j0);
  const int kn = first ? (LOWER ? 0 : nb - 1) : (LOWER ? k + 1 : k - 1);  // the diagonal block solved here
  const int r0 = kn * kLuB, nr = min(kLuB, n - r0);
  const int rb = diag ? r0 : LOWER ? (k + 1 + (int)blockIdx.x) * kLuB : (rlo + (int)blockIdx.x - 1) * kLuB;  // row block
  const int row = t & (kLuB - 1), half = t >> 7;
  const int i = rb + row;
  const bool live = half == 0 && (diag ? row < nr : LOWER ? i < n : i < kn * kLuB);
  // the round of loads
  const float xi = x[min(i, n - 1)];
  const float xkt = first ? 0.f : x[j0 + min(row, nj - 1)];
  const int r4 = t & 31, cq = t >> 5;  // this thread's 4-row slot and column (of 8) in each 16-byte load round
  auto ld = [&](int rbase, int cb, int ncol, int q) {
    const int r = rbase + 4 * r4;
    const int64_t c = (int64_t)(cb + min(q * 8 + cq, ncol - 1)) * n;
    if (VEC && r + 3 < n) return *reinterpret_cast<const float4 *>(A + r + c);
    return make_float4(A[min(r, n - 1) + c], A[min(r + 1, n - 1) + c], A[min(r + 2, n - 1) + c], A[min(r + 3, n - 1) + c]);
  };
  float4 qc[16], qd[16];
  if (!first) {
#pragma unroll
    for (int q = 0; q < 16; ++q) qc[q] = ld(rb, j0, nj, q);
  }
  if (diag) {
#pragma unroll
    for (int q = 0; q < 16; ++q) qd[q] = ld(r0, r0, nr, q);
  }
  if (half == 0) xk[row] = row < nj ? xkt : 0.f;
  if (!first) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = q * 8 + cq;
      C[4 * r4][c] = qc[q].x, C[4 * r4 + 1][c] = qc[q].y, C[4 * r4 + 2][c] = qc[q].z, C[4 * r4 + 3][c] = qc[q].w;
    }
  }
  if (diag) {  // outside the block: identity
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = q * 8 + cq;
      const float e[4] = {qd[q].x, qd[q].y, qd[q].z, qd[q].w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int rr = 4 * r4 + u;
        D[rr][c] = rr < nr && c < nr ? e[u] : (rr == c ? 1.f : 0.f);
      }
    }
  }
  __syncthreads();
  float v = xi;
  if (!first) {  // the block column's product, two threads per row (halves of the columns)
    float sacc = 0.f;
#pragma unroll 16
    for (int c = 0; c < 64; ++c) sacc += C[row][64 * half + c] * xk[64 * half + c];  // (xk = 0 past the block)
    part[half][row] = sacc;
    __syncthreads();
    v = xi - part[0][row] - part[1][row];
  }
  if (!diag) {
    if (live) x[i] = v;
    return;
  }
  const int lane = t & 63, w = t >> 6;
  if (!LOWER && half == 0) {  // (read back by the writing wavefront only)
    rd[t] = 1.f / D[t][t];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  auto bcast = [](float q, int c) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q), c)); };
  auto tri = [&](int cb) {  // the wavefront's own 64 x 64 triangle
    if (LOWER) {
#pragma unroll
      for (int c = 0; c < 64; ++c) {
        const float xc = bcast(v, c), dv = D[t][cb + c];
        v = __builtin_fmaf(lane > c ? -dv : 0.f, xc, v);
      }
    } else {
      float xs = 0.f;
#pragma unroll
      for (int c = 63; c >= 0; --c) {
        const float xc = bcast(v, c) * rd[cb + c], dv = D[t][cb + c];
        xs = lane == c ? xc : xs;
        v = __builtin_fmaf(lane < c ? -dv : 0.f, xc, v);
      }
      v = xs;
    }
  };
  const int wf = LOWER ? 0 : 1;  // the wavefront solved first
  if (w == wf) {
    tri(64 * wf);
    xb[t] = v;
  }
  __syncthreads();
  if (w == 1 - wf) {
    const int cb = 64 * wf;
#pragma unroll 16
    for (int c = 0; c < 64; ++c) v -= D[t][cb + c] * xb[cb + c];
    tri(64 * w);
  }
  if (live) x[i] = v;
}
// bl / bu >= 0: lower / upper bandwidths -- a step updates only the row blocks its block column reaches
template <bool VEC>
void lu_solve(const float *LU, int n, float *x, hipStream_t s, int bl, int bu) {
  const int nb = (n + kLuB - 1) / kLuB;
  hipLaunchKernelGGL((k_lu_step<true, VEC>), dim3(1), dim3(kLuT), 0, s, LU, n, x, -1, 0);
  for (int k = 0; k + 1 < nb; ++k) {
    const int end = bl < 0 ? n : std::min(n, (k + 1) * kLuB + bl);  // rows below reached by block column k
    const int rest = end - (k + 2) * kLuB;
    hipLaunchKernelGGL((k_lu_step<true, VEC>), dim3(1 + (rest > 0 ? (rest + kLuB - 1) / kLuB : 0)), dim3(kLuT), 0, s, LU,
                       n, x, k, 0);
  }
  hipLaunchKernelGGL((k_lu_step<false, VEC>), dim3(1), dim3(kLuT), 0, s, LU, n, x, -1, 0);
  for (int k = nb - 1; k >= 1; --k) {
    const int rlo = bu < 0 ? 0 : std::max(0, k * kLuB - bu) / kLuB;  // rows above reached by block column k
    const int nblk = std::max(0, (k - 1) - rlo);
    hipLaunchKernelGGL((k_lu_step<false, VEC>), dim3(1 + nblk), dim3(kLuT), 0, s, LU, n, x, k, rlo);
  }
}
}  // namespace
hipError_t dense_lu_solve_f32(const float *LU, int n, float *x, hipStream_t s, int bl, int bu) {
  if (n <= 0) return hipSuccess;
  if (n % 4 == 0 && reinterpret_cast<uintptr_t>(LU) % 16 == 0) lu_solve<true>(LU, n, x, s, bl, bu);
  else lu_solve<false>(LU, n, x, s, bl, bu);
  return hipGetLastError();
}

hipError_t mg_jacobi_update(double *x, const double *b, const double *y, const double *d, double omega, int64_t n,
                            int zero_start, hipStream_t s) {
  hipLaunchKernelGGL(k_jacobi_update, dim3(grid_for(n)), dim3(256), 0, s, x, b, y, d, omega, n, zero_start);
  return hipGetLastError();
}

}  // namespace gls
