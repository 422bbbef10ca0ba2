#include <algorithm>
#include <cstdint>
#include <cstdlib>
// gls_vector_kernels.hip — Krylov vector kernels (HBM-bound; 16-byte accesses where aligned).
#include "gls_launch.hpp"

namespace gls {

namespace {
constexpr int kBlock = 256;
constexpr int kMaxBlocks = 2048;  // 256 CUs x 8
constexpr int kDotChunk = 8;      // vectors per multidot pass

inline int grid_for(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  return (int)(b < kMaxBlocks ? (b > 0 ? b : 1) : kMaxBlocks);
}

__global__ void k_fill(double *x, int64_t n, double a) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) x[i] = a;
}
__global__ void k_copy(double *__restrict__ y, const double *__restrict__ x, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) y[i] = x[i];
}
__global__ void k_axpy(double *__restrict__ y, double a, const double *__restrict__ x, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] += a * x[i];
}
// w = y + a x (the copy + k_axpy pair in one pass, same arithmetic)
__global__ void k_waxpy(double *__restrict__ w, const double *__restrict__ y, double a, const double *__restrict__ x,
                        int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    w[i] = y[i] + a * x[i];
}
// y = a x + b y; b == 0 does not read y (a fresh buffer may hold NaN bit patterns: 0 * NaN is NaN)
__global__ void k_axpby(double *__restrict__ y, double a, const double *__restrict__ x, double b, int64_t n) {
  if (b == 0.0) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
      y[i] = a * x[i];
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = a * x[i] + b * y[i];
}
__global__ void k_scale(double *x, double a, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) x[i] *= a;
}
__global__ void k_div(double *__restrict__ y, const double *__restrict__ x, const double *__restrict__ d, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = x[i] / d[i];
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// partial sums of up to kDotChunk dot products per block; work[k*gridDim + block]
// rows are summed over [0, n1) and [off2, off2 + n2) (the owned ranges of a rank-local vector)
template <int NK>
__global__ void __launch_bounds__(kBlock) k_multidot(const double *__restrict__ A, int64_t lda,
                                                     const double *__restrict__ w, int64_t n1, int64_t off2, int64_t n2,
                                                     double *work) {
  double acc[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) acc[k] = 0.;
  const int64_t n = n1 + n2;
  for (int64_t ii = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; ii < n; ii += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = ii < n1 ? ii : off2 + (ii - n1);
    const double wi = w[i];
#pragma unroll
    for (int k = 0; k < NK; ++k) acc[k] += A[k * lda + i] * wi;
  }
  __shared__ double red[NK][kBlock / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const double s = wave_sum(acc[k]);
    if (lane == 0) red[k][wv] = s;
  }
  __syncthreads();
  if (threadIdx.x < NK) {
    double s = 0.;
#pragma unroll
    for (int j = 0; j < kBlock / 64; ++j) s += red[threadIdx.x][j];
    work[threadIdx.x * gridDim.x + blockIdx.x] = s;
  }
}

// out[k] = sum_b work[k*nb + b]; one block per k, deterministic order
__global__ void __launch_bounds__(kBlock) k_reduce_rows(const double *work, int nb, double *out) {
  double s = 0.;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) s += work[blockIdx.x * nb + b];
  __shared__ double red[kBlock / 64];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.;
    for (int j = 0; j < kBlock / 64; ++j) t += red[j];
    out[blockIdx.x] = t;
  }
}

template <int NK>
__global__ void __launch_bounds__(kBlock) k_multiaxpy(double *__restrict__ w, const double *__restrict__ A, int64_t lda,
                                                      const double *__restrict__ h, double sign, int64_t n) {
  double hk[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) hk[k] = sign * h[k];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double s = w[i];
#pragma unroll
    for (int k = 0; k < NK; ++k) s -= hk[k] * A[k * lda + i];
    w[i] = s;
  }
}

// w = scale * (w - sign * sum_k h[k] A[k]); in the same pass the partial sums of A[k] . w_new (DOTS)
// and ||w_new||^2 over the owned rows [0, n1) U [off2, off2 + n2) -> work[d * gridDim + block]
// (the fused classical Gram-Schmidt step: projection + the re-orthogonalisation dots + norm; with
// scale != 1 also the normalisation of the new Krylov vector)
template <int NK, bool DOTS>
__global__ void __launch_bounds__(kBlock) k_multiaxpy_dot(double *__restrict__ w, const double *__restrict__ A,
                                                          int64_t lda, const double *__restrict__ h, double sign,
                                                          int64_t n, int64_t n1, int64_t off2, int64_t n2,
                                                          double scale, double *work) {
  constexpr int ND = (DOTS ? NK : 0) + 1;
  double hk[NK], acc[ND];
#pragma unroll
  for (int k = 0; k < NK; ++k) hk[k] = sign * h[k];
#pragma unroll
  for (int d = 0; d < ND; ++d) acc[d] = 0.;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double a[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) a[k] = A[k * lda + i];
    double s = w[i];
#pragma unroll
    for (int k = 0; k < NK; ++k) s -= hk[k] * a[k];
    s *= scale;
    w[i] = s;
    if (i < n1 || (i >= off2 && i < off2 + n2)) {
      if constexpr (DOTS) {
#pragma unroll
        for (int k = 0; k < NK; ++k) acc[k] += a[k] * s;
      }
      acc[ND - 1] += s * s;
    }
  }
  __shared__ double red[ND][kBlock / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const double t = wave_sum(acc[d]);
    if (lane == 0) red[d][wv] = t;
  }
  __syncthreads();
  if (threadIdx.x < ND) {
    double t = 0.;
#pragma unroll
    for (int j = 0; j < kBlock / 64; ++j) t += red[threadIdx.x][j];
    work[threadIdx.x * gridDim.x + blockIdx.x] = t;
  }
}

// 16-byte variants of the Gram-Schmidt passes (one row pair per thread and trip, double2 loads / stores,
// non-temporal basis loads; single-rank vectors: all rows owned), used when the rows are 16-byte aligned
// (else the 8-byte kernels). Orthogonalisation 11.9 -> 11.0 ms per Newton step at configs[2] (4.9 -> 5.3 TB/s,
// profiles/r05_ab_vec16.txt)
typedef double dbl2 __attribute__((ext_vector_type(2)));
// k_multiaxpy with 16-byte loads / stores (two rows per lane); ZERO: w starts at 0 and is not read
// (same arithmetic as a fill + k_multiaxpy: s = 0.0 - h0 a0 - ...)
template <int NK, bool ZERO>
__global__ void __launch_bounds__(kBlock) k_multiaxpy16(double *__restrict__ w, const double *__restrict__ A, int64_t lda,
                                                        const double *__restrict__ h, double sign, int64_t n) {
  double hk[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) hk[k] = sign * h[k];
  const int64_t np = n / 2;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < np; p += (int64_t)gridDim.x * blockDim.x) {
    dbl2 s = ZERO ? dbl2{0.0, 0.0} : reinterpret_cast<const dbl2 *>(w)[p];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const dbl2 a = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(A + k * lda) + p);
      s.x -= hk[k] * a.x;
      s.y -= hk[k] * a.y;
    }
    reinterpret_cast<dbl2 *>(w)[p] = s;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    double s = ZERO ? 0.0 : w[n - 1];
#pragma unroll
    for (int k = 0; k < NK; ++k) s -= hk[k] * A[k * lda + n - 1];
    w[n - 1] = s;
  }
}

template <int NK>
__global__ void __launch_bounds__(kBlock) k_multidot16(const double *__restrict__ A, int64_t lda,
                                                       const double *__restrict__ w, int64_t n, double *work) {
  double acc[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) acc[k] = 0.;
  const int64_t np = n / 2;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < np; p += (int64_t)gridDim.x * blockDim.x) {
    const dbl2 wi = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(w) + p);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const dbl2 a = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(A + k * lda) + p);
      acc[k] += a.x * wi.x;
      acc[k] += a.y * wi.y;
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NK; ++k) acc[k] += A[k * lda + n - 1] * w[n - 1];
  __shared__ double red[NK][kBlock / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const double t = wave_sum(acc[k]);
    if (lane == 0) red[k][wv] = t;
  }
  __syncthreads();
  if (threadIdx.x < NK) {
    double t = 0.;
#pragma unroll
    for (int j = 0; j < kBlock / 64; ++j) t += red[threadIdx.x][j];
    work[threadIdx.x * gridDim.x + blockIdx.x] = t;
  }
}
template <int NK, bool DOTS>
__global__ void __launch_bounds__(kBlock) k_multiaxpy_dot16(double *__restrict__ w, const double *__restrict__ A,
                                                            int64_t lda, const double *__restrict__ h, double sign,
                                                            int64_t n, double scale, double *work) {
  constexpr int ND = (DOTS ? NK : 0) + 1;
  double hk[NK], acc[ND];
#pragma unroll
  for (int k = 0; k < NK; ++k) hk[k] = sign * h[k];
#pragma unroll
  for (int d = 0; d < ND; ++d) acc[d] = 0.;
  auto row = [&](double wi, const double *a) {
    double s = wi;
#pragma unroll
    for (int k = 0; k < NK; ++k) s -= hk[k] * a[k];
    s *= scale;
    if constexpr (DOTS) {
#pragma unroll
      for (int k = 0; k < NK; ++k) acc[k] += a[k] * s;
    }
    acc[ND - 1] += s * s;
    return s;
  };
  const int64_t np = n / 2;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < np; p += (int64_t)gridDim.x * blockDim.x) {
    double a0[NK], a1[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const dbl2 a = __builtin_nontemporal_load(reinterpret_cast<const dbl2 *>(A + k * lda) + p);
      a0[k] = a.x;
      a1[k] = a.y;
    }
    const dbl2 wi = reinterpret_cast<const dbl2 *>(w)[p];
    const double o0 = row(wi.x, a0), o1 = row(wi.y, a1);
    reinterpret_cast<dbl2 *>(w)[p] = dbl2{o0, o1};
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    double a[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) a[k] = A[k * lda + n - 1];
    w[n - 1] = row(w[n - 1], a);
  }
  __shared__ double red[ND][kBlock / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const double t = wave_sum(acc[d]);
    if (lane == 0) red[d][wv] = t;
  }
  __syncthreads();
  if (threadIdx.x < ND) {
    double t = 0.;
#pragma unroll
    for (int j = 0; j < kBlock / 64; ++j) t += red[threadIdx.x][j];
    work[threadIdx.x * gridDim.x + blockIdx.x] = t;
  }
}
bool vec16(const double *A, int64_t lda, const double *w, int64_t n, int64_t n1, int64_t n2) {
  return n2 == 0 && n1 == n && (lda % 2) == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)w % 16) == 0;
}

// constraint lines: x[dof[i]] = sum_{j in [off[i], off[i+1])} w[j] * src[master[j]]
// (masters are never constrained lines themselves, so src may alias x)
__global__ void k_csr_gather_set(double *x, const double *src, const int64_t *__restrict__ dof,
                                 const int64_t *__restrict__ off, const int64_t *__restrict__ master,
                                 const double *__restrict__ w, int64_t n, int64_t bs = 0) {
  x += blockIdx.y * bs;  // batched (probe) vectors: blockIdx.y selects the vector
  src += blockIdx.y * bs;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.;
    for (int64_t j = off[i]; j < off[i + 1]; ++j) s += w[j] * src[master[j]];
    x[dof[i]] = s;
  }
}
// y = A x (add: y += A x) for a CSR matrix A of n rows: the multigrid transfers of general hierarchies
// (prolongation P and restriction P^T). One thread per row, terms in stored order (deterministic).
__global__ void k_csr_spmv(double *__restrict__ y, const double *__restrict__ x, const int64_t *__restrict__ off,
                           const int32_t *__restrict__ col, const double *__restrict__ w, int64_t n, int add) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.;
    for (int64_t j = off[i]; j < off[i + 1]; ++j) s += w[j] * x[col[j]];
    y[i] = add ? y[i] + s : s;
  }
}
// condensation onto masters: y[tm[i]] += sum_{j in [toff[i], toff[i+1])} tw[j] * y[tdof[j]]
// (one thread per master, fixed order: deterministic)
__global__ void k_csr_condense(double *y, const int64_t *__restrict__ tm, const int64_t *__restrict__ toff,
                               const int64_t *__restrict__ tdof, const double *__restrict__ tw, int64_t n, int64_t bs = 0) {
  y += blockIdx.y * bs;
  constexpr int kIn = 8;  // hanging rows gathered at once: all row ids and weights, then all values, then the sum
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j0 = toff[i], nj = toff[i + 1] - j0;
    double s = 0.;
    if (nj <= kIn) {
      int64_t r[kIn];
      double w[kIn], v[kIn];
#pragma unroll
      for (int t = 0; t < kIn; ++t) {
        r[t] = t < nj ? tdof[j0 + t] : -1;
        w[t] = t < nj ? tw[j0 + t] : 0.;
      }
#pragma unroll
      for (int t = 0; t < kIn; ++t) v[t] = r[t] >= 0 ? y[r[t]] : 0.;
#pragma unroll
      for (int t = 0; t < kIn; ++t)  // the stored order, as the general loop
        if (t < nj) s += w[t] * v[t];
    } else {
      for (int64_t j = j0; j < j0 + nj; ++j) s += tw[j] * y[tdof[j]];
    }
    y[tm[i]] += s;
  }
}

__global__ void k_gather_scale_set(double *y, const double *d, const double *v, const int64_t *idx, int64_t m,
                                   const double *rb, int64_t bs = 0) {
  y += blockIdx.y * bs;
  v += blockIdx.y * bs;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = idx[j];
    y[i] = rb ? rb[i] - d[i] * v[i] : d[i] * v[i];
  }
}
__global__ void k_pack_nodes(const double *__restrict__ x, const int32_t *__restrict__ nodes, int64_t m, int64_t voff,
                             double *__restrict__ buf) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = nodes[j];
    buf[j * 4 + 0] = x[n * 3 + 0];
    buf[j * 4 + 1] = x[n * 3 + 1];
    buf[j * 4 + 2] = x[n * 3 + 2];
    buf[j * 4 + 3] = x[voff + n];
  }
}
__global__ void k_unpack_nodes(double *__restrict__ x, const int32_t *__restrict__ nodes, int64_t m, int64_t voff,
                               const double *__restrict__ buf, int add) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = nodes[j];
    if (add) {
      atomicAdd(&x[n * 3 + 0], buf[j * 4 + 0]);
      atomicAdd(&x[n * 3 + 1], buf[j * 4 + 1]);
      atomicAdd(&x[n * 3 + 2], buf[j * 4 + 2]);
      atomicAdd(&x[voff + n], buf[j * 4 + 3]);
    } else {
      x[n * 3 + 0] = buf[j * 4 + 0];
      x[n * 3 + 1] = buf[j * 4 + 1];
      x[n * 3 + 2] = buf[j * 4 + 2];
      x[voff + n] = buf[j * 4 + 3];
    }
  }
}
__global__ void k_set_indexed(double *y, const int64_t *idx, const double *vals, int64_t m) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x)
    y[idx[j]] = vals ? vals[j] : 0.0;
}
}  // namespace

int multidot_work_size() { return (kDotChunk + 1) * kMaxBlocks; }

// y[node] = sum over the node's element-vector slots in ascending order (deterministic scatter of
// the per-cell kernels): velocity node n, component c: ev[slot + c] for slot in vslot[voff[n]..);
// pressure node q: ev[slot] for slot in pslot[poff[q]..)
__global__ void k_gather_ev(double *__restrict__ y, const double *__restrict__ ev, const int64_t *__restrict__ voff,
                            const int64_t *__restrict__ vslot, int64_t nv, const int64_t *__restrict__ poff,
                            const int64_t *__restrict__ pslot, int64_t np, int dim, int64_t ys = 0, int64_t evs = 0,
                            const uint8_t *__restrict__ act = nullptr, int64_t el = 1, int cb = 1, int nblk = 0) {
  y += blockIdx.y * ys;
  ev += blockIdx.y * evs;
  if (act) act += (int64_t)blockIdx.y * nblk;  // batched probing: cell batches the kernel skipped hold 0
  auto live = [&](int64_t slot) { return !act || act[slot / el / cb]; };
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int kIn = 8;  // incidences gathered at once (all slots, then all activity flags, then all values: one
                          // dependent round each; the batched probes walked them one by one, 160 us per launch at
                          // 1.72 M DoFs)
  if (i < nv && voff[i + 1] - voff[i] <= kIn) {
    const int64_t j0 = voff[i], nj = voff[i + 1] - j0;
    int64_t sl[kIn];
#pragma unroll
    for (int t = 0; t < kIn; ++t) sl[t] = t < nj ? vslot[j0 + t] : -1;
    if (act) {
#pragma unroll
      for (int t = 0; t < kIn; ++t) sl[t] = sl[t] >= 0 && live(sl[t]) ? sl[t] : -1;
    }
    double e[kIn][3];
#pragma unroll
    for (int t = 0; t < kIn; ++t)
#pragma unroll
      for (int c = 0; c < 3; ++c) e[t][c] = (sl[t] >= 0 && c < dim) ? ev[sl[t] + c] : 0.;
    double acc[3] = {0., 0., 0.};
#pragma unroll
    for (int t = 0; t < kIn; ++t)  // ascending slot order, as the general loop below (skipped slots add nothing)
      if (sl[t] >= 0)
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += e[t][c];
    for (int c = 0; c < dim; ++c) y[i * dim + c] = acc[c];
  } else if (i < nv) {
    double acc[3] = {0., 0., 0.};
    for (int64_t j = voff[i]; j < voff[i + 1]; ++j) {
      if (!live(vslot[j])) continue;
      const double *e = ev + vslot[j];
      for (int c = 0; c < dim; ++c) acc[c] += e[c];
    }
    for (int c = 0; c < dim; ++c) y[i * dim + c] = acc[c];
  } else if (i < nv + np && poff[i - nv + 1] - poff[i - nv] <= kIn) {
    const int64_t q = i - nv, j0 = poff[q], nj = poff[q + 1] - j0;
    int64_t sl[kIn];
#pragma unroll
    for (int t = 0; t < kIn; ++t) sl[t] = t < nj ? pslot[j0 + t] : -1;
    if (act) {
#pragma unroll
      for (int t = 0; t < kIn; ++t) sl[t] = sl[t] >= 0 && live(sl[t]) ? sl[t] : -1;
    }
    double e[kIn];
#pragma unroll
    for (int t = 0; t < kIn; ++t) e[t] = sl[t] >= 0 ? ev[sl[t]] : 0.;
    double acc = 0.;
#pragma unroll
    for (int t = 0; t < kIn; ++t)
      if (sl[t] >= 0) acc += e[t];
    y[dim * nv + q] = acc;
  } else if (i < nv + np) {
    const int64_t q = i - nv;
    double acc = 0.;
    for (int64_t j = poff[q]; j < poff[q + 1]; ++j)
      if (live(pslot[j])) acc += ev[pslot[j]];
    y[dim * nv + q] = acc;
  }
}

hipError_t gather_element_vectors(double *y, const double *ev, const int64_t *voff, const int64_t *vslot, int64_t nv,
                                  const int64_t *poff, const int64_t *pslot, int64_t np, int dim, hipStream_t s) {
  const int64_t n = nv + np;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_ev, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, y, ev, voff, vslot, nv, poff,
                     pslot, np, dim);
  return hipGetLastError();
}

hipError_t vec_fill(double *x, int64_t n, double a, hipStream_t s) {
  hipLaunchKernelGGL(k_fill, dim3(grid_for(n)), dim3(kBlock), 0, s, x, n, a);
  return hipGetLastError();
}
hipError_t vec_copy(double *y, const double *x, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_copy, dim3(grid_for(n)), dim3(kBlock), 0, s, y, x, n);
  return hipGetLastError();
}
hipError_t vec_axpy(double *y, double a, const double *x, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_axpy, dim3(grid_for(n)), dim3(kBlock), 0, s, y, a, x, n);
  return hipGetLastError();
}
hipError_t vec_axpby(double *y, double a, const double *x, double b, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_axpby, dim3(grid_for(n)), dim3(kBlock), 0, s, y, a, x, b, n);
  return hipGetLastError();
}
hipError_t vec_scale(double *x, double a, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_scale, dim3(grid_for(n)), dim3(kBlock), 0, s, x, a, n);
  return hipGetLastError();
}
hipError_t vec_div(double *y, const double *x, const double *d, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_div, dim3(grid_for(n)), dim3(kBlock), 0, s, y, x, d, n);
  return hipGetLastError();
}

hipError_t vec_multidot(const double *A, int64_t lda, int nk, const double *w, int64_t n, double *out, double *work,
                        hipStream_t s) {
  return vec_multidot2(A, lda, nk, w, n, 0, 0, out, work, s);
}

hipError_t vec_multidot2(const double *A, int64_t lda, int nk, const double *w, int64_t n1, int64_t off2, int64_t n2,
                         double *out, double *work, hipStream_t s) {
  const int nb = grid_for(n1 + n2);
  const bool v16 = vec16(A, lda, w, n1 + n2, n1, n2);
  for (int k0 = 0; k0 < nk; k0 += kDotChunk) {
    const int m = nk - k0 < kDotChunk ? nk - k0 : kDotChunk;
    const double *Ak = A + (int64_t)k0 * lda;
    switch (m) {
#define MD(M)                                                                                                  \
  case M:                                                                                                      \
    if (v16) hipLaunchKernelGGL(k_multidot16<M>, dim3(nb), dim3(kBlock), 0, s, Ak, lda, w, n1, work);          \
    else hipLaunchKernelGGL(k_multidot<M>, dim3(nb), dim3(kBlock), 0, s, Ak, lda, w, n1, off2, n2, work);      \
    break;
      MD(1) MD(2) MD(3) MD(4) MD(5) MD(6) MD(7) MD(8)
#undef MD
    }
    hipLaunchKernelGGL(k_reduce_rows, dim3(m), dim3(kBlock), 0, s, work, nb, out + k0);
  }
  return hipGetLastError();
}

hipError_t vec_multiaxpy(double *w, const double *A, int64_t lda, int nk, const double *h, double sign, int64_t n,
                         hipStream_t s, bool zero_init) {
  const int nb = grid_for(n);
  const bool v16 = vec16(A, lda, w, n, n, 0);
  if (zero_init && (!v16 || nk <= 0)) {  // nk == 0: w = 0 on both paths (no chunk launch would write it)
    const hipError_t e = vec_fill(w, n, 0.0, s);
    if (e != hipSuccess || nk <= 0) return e;
  }
  for (int k0 = 0; k0 < nk; k0 += kDotChunk) {
    const int m = nk - k0 < kDotChunk ? nk - k0 : kDotChunk;
    const double *Ak = A + (int64_t)k0 * lda;
    const bool z = zero_init && v16 && k0 == 0;
    switch (m) {
#define MA(M)                                                                                                    \
  case M:                                                                                                        \
    if (z)                                                                                                       \
      hipLaunchKernelGGL((k_multiaxpy16<M, true>), dim3(nb), dim3(kBlock), 0, s, w, Ak, lda, h + k0, sign, n);   \
    else if (v16)                                                                                                \
      hipLaunchKernelGGL((k_multiaxpy16<M, false>), dim3(nb), dim3(kBlock), 0, s, w, Ak, lda, h + k0, sign, n);  \
    else                                                                                                         \
      hipLaunchKernelGGL(k_multiaxpy<M>, dim3(nb), dim3(kBlock), 0, s, w, Ak, lda, h + k0, sign, n);             \
    break;
      MA(1) MA(2) MA(3) MA(4) MA(5) MA(6) MA(7) MA(8)
#undef MA
    }
  }
  return hipGetLastError();
}

hipError_t vec_waxpy(double *w, const double *y, double a, const double *x, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_waxpy, dim3(grid_for(n)), dim3(kBlock), 0, s, w, y, a, x, n);
  return hipGetLastError();
}

hipError_t vec_multiaxpy_dots(double *w, const double *A, int64_t lda, int nk, const double *h, double sign, int64_t n,
                              int64_t n1, int64_t off2, int64_t n2, bool dots, double scale, double *out, double *work,
                              hipStream_t s) {
  if (nk < 1 || nk > kDotChunk) return hipErrorInvalidValue;
  const int nb = grid_for(n);
  const bool v16 = vec16(A, lda, w, n, n1, n2);
  switch (nk * 2 + (dots ? 1 : 0)) {
#define MX(M)                                                                                                         \
  case 2 * M:                                                                                                         \
    if (v16)                                                                                                          \
      hipLaunchKernelGGL((k_multiaxpy_dot16<M, false>), dim3(nb), dim3(kBlock), 0, s, w, A, lda, h, sign, n, scale, work); \
    else                                                                                                              \
      hipLaunchKernelGGL((k_multiaxpy_dot<M, false>), dim3(nb), dim3(kBlock), 0, s, w, A, lda, h, sign, n, n1, off2, n2, \
                         scale, work);                                                                                \
    break;                                                                                                            \
  case 2 * M + 1:                                                                                                     \
    if (v16)                                                                                                          \
      hipLaunchKernelGGL((k_multiaxpy_dot16<M, true>), dim3(nb), dim3(kBlock), 0, s, w, A, lda, h, sign, n, scale, work); \
    else                                                                                                              \
      hipLaunchKernelGGL((k_multiaxpy_dot<M, true>), dim3(nb), dim3(kBlock), 0, s, w, A, lda, h, sign, n, n1, off2, n2, \
                         scale, work);                                                                                \
    break;
    MX(1) MX(2) MX(3) MX(4) MX(5) MX(6) MX(7) MX(8)
#undef MX
  }
  hipLaunchKernelGGL(k_reduce_rows, dim3(dots ? nk + 1 : 1), dim3(kBlock), 0, s, work, nb, out);
  return hipGetLastError();
}

// x = C v in one pass: the free DoFs copied, the hanging ones interpolated from their masters' values in v (masters
// are never hanging, so reading them from v equals the copy-then-interpolate order)
__global__ void k_copy_gather_set(double *__restrict__ x, const double *__restrict__ v, const uint8_t *__restrict__ dmask,
                                  int64_t n, const int64_t *__restrict__ dof, const int64_t *__restrict__ off,
                                  const int64_t *__restrict__ master, const double *__restrict__ w, int64_t nl) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n + nl; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n) {
      if (!dmask[i]) x[i] = v[i];
    } else {  // a line: its masters (<= 9 on Q2 faces) and weights first, then their values, then the ordered sum
      const int64_t l = i - n, j0 = off[l], nj = off[l + 1] - j0;
      constexpr int kIn = 9;
      double s = 0.;
      if (nj <= kIn) {
        int64_t m[kIn];
        double wt[kIn], vv[kIn];
#pragma unroll
        for (int t = 0; t < kIn; ++t) {
          m[t] = t < nj ? master[j0 + t] : -1;
          wt[t] = t < nj ? w[j0 + t] : 0.;
        }
#pragma unroll
        for (int t = 0; t < kIn; ++t) vv[t] = m[t] >= 0 ? v[m[t]] : 0.;
#pragma unroll
        for (int t = 0; t < kIn; ++t)
          if (t < nj) s += wt[t] * vv[t];
      } else {
        for (int64_t j = j0; j < j0 + nj; ++j) s += w[j] * v[master[j]];
      }
      x[dof[l]] = s;
    }
  }
}
hipError_t vec_copy_gather_set(double *x, const double *v, const uint8_t *dmask, int64_t n, const int64_t *dof,
                               const int64_t *off, const int64_t *master, const double *w, int64_t nl, hipStream_t s) {
  if (n + nl <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_copy_gather_set, dim3(grid_for(n + nl)), dim3(kBlock), 0, s, x, v, dmask, n, dof, off, master, w,
                     nl);
  return hipGetLastError();
}

hipError_t vec_csr_gather_set(double *x, const double *src, const int64_t *dof, const int64_t *off,
                              const int64_t *master, const double *w, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_csr_gather_set, dim3(grid_for(n)), dim3(kBlock), 0, s, x, src, dof, off, master, w, n);
  return hipGetLastError();
}
// the same with L lanes per row (CSR-vector): lane r of a row sums its entries r, r + L, ... in order, then a
// fixed xor butterfly over the L lanes (deterministic); coalesced col / w reads for long rows (the
// restriction P^T of a Q2 hierarchy: up to 125 terms per coarse row)
template <int L>
__global__ void __launch_bounds__(256) k_csr_spmv_v(double *__restrict__ y, const double *__restrict__ x,
                                                    const int64_t *__restrict__ off, const int32_t *__restrict__ col,
                                                    const double *__restrict__ w, int64_t n, int add) {
  const int r = threadIdx.x % L;
  for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / L; i < n;
       i += (int64_t)gridDim.x * blockDim.x / L) {
    double s = 0.;
    const int64_t e = off[i + 1];
    for (int64_t j = off[i] + r; j < e; j += L) s += w[j] * x[col[j]];
#pragma unroll
    for (int m = L / 2; m > 0; m >>= 1) s += __shfl_xor(s, m, L);
    if (r == 0) y[i] = add ? y[i] + s : s;
  }
}
hipError_t vec_csr_spmv(double *y, const double *x, const int64_t *off, const int32_t *col, const double *w, int64_t n,
                        bool add, hipStream_t s, int lanes) {
  if (n <= 0) return hipSuccess;
  const int a = add ? 1 : 0;
  const int64_t th = n * (lanes < 1 ? 1 : lanes);
  const dim3 g((unsigned)std::min<int64_t>((th + 255) / 256, 65535 * 8)), b(256);
  switch (lanes) {
    case 2: hipLaunchKernelGGL(k_csr_spmv_v<2>, g, b, 0, s, y, x, off, col, w, n, a); break;
    case 4: hipLaunchKernelGGL(k_csr_spmv_v<4>, g, b, 0, s, y, x, off, col, w, n, a); break;
    case 8: hipLaunchKernelGGL(k_csr_spmv_v<8>, g, b, 0, s, y, x, off, col, w, n, a); break;
    case 16: hipLaunchKernelGGL(k_csr_spmv_v<16>, g, b, 0, s, y, x, off, col, w, n, a); break;
    default: hipLaunchKernelGGL(k_csr_spmv, dim3(grid_for(n)), dim3(kBlock), 0, s, y, x, off, col, w, n, a);
  }
  return hipGetLastError();
}
hipError_t vec_csr_condense(double *y, const int64_t *tm, const int64_t *toff, const int64_t *tdof, const double *tw,
                            int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_csr_condense, dim3(grid_for(n)), dim3(kBlock), 0, s, y, tm, toff, tdof, tw, n);
  return hipGetLastError();
}

hipError_t vec_gather_scale_set(double *y, const double *d, const double *v, const int64_t *idx, int64_t m,
                                hipStream_t s, const double *rb) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_scale_set, dim3(grid_for(m)), dim3(kBlock), 0, s, y, d, v, idx, m, rb);
  return hipGetLastError();
}
hipError_t vec_pack_nodes(const double *x, const int32_t *nodes, int64_t m, int64_t voff, double *buf, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack_nodes, dim3(grid_for(m)), dim3(kBlock), 0, s, x, nodes, m, voff, buf);
  return hipGetLastError();
}
hipError_t vec_unpack_nodes(double *x, const int32_t *nodes, int64_t m, int64_t voff, const double *buf, int add,
                            hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_nodes, dim3(grid_for(m)), dim3(kBlock), 0, s, x, nodes, m, voff, buf, add);
  return hipGetLastError();
}
// DoF-level ghost exchange (general meshes): buf[j] = x[dofs[j]]; x[dofs[j]] = buf[j]; and the
// export-add x[u[i]] += sum_{j in [off[i], off[i+1])} buf[slot[j]] in a fixed (neighbour) order
__global__ void k_pack_dofs(const double *__restrict__ x, const int32_t *__restrict__ dofs, int64_t m,
                            double *__restrict__ buf) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x)
    buf[j] = x[dofs[j]];
}
__global__ void k_unpack_dofs(double *__restrict__ x, const int32_t *__restrict__ dofs, int64_t m,
                              const double *__restrict__ buf) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x)
    x[dofs[j]] = buf[j];
}
__global__ void k_add_dofs_ordered(double *__restrict__ x, const int32_t *__restrict__ u, const int32_t *__restrict__ off,
                                   const int32_t *__restrict__ slot, int64_t n, const double *__restrict__ buf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double s = x[u[i]];
    for (int j = off[i]; j < off[i + 1]; ++j) s += buf[slot[j]];
    x[u[i]] = s;
  }
}
hipError_t vec_pack_dofs(const double *x, const int32_t *dofs, int64_t m, double *buf, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack_dofs, dim3(grid_for(m)), dim3(kBlock), 0, s, x, dofs, m, buf);
  return hipGetLastError();
}
hipError_t vec_unpack_dofs(double *x, const int32_t *dofs, int64_t m, const double *buf, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_dofs, dim3(grid_for(m)), dim3(kBlock), 0, s, x, dofs, m, buf);
  return hipGetLastError();
}
hipError_t vec_add_dofs_ordered(double *x, const int32_t *u, const int32_t *off, const int32_t *slot, int64_t n,
                                const double *buf, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_add_dofs_ordered, dim3(grid_for(n)), dim3(kBlock), 0, s, x, u, off, slot, n, buf);
  return hipGetLastError();
}
// node export-add in a fixed order: x[(u[i], c)] += buf[slot[j]*4 + c] for j in [off[i], off[i+1])
// (a corner node of a 4- or 8-rank partition receives from several neighbours; atomics would make
// the sum order, and the last bit, depend on the schedule)
__global__ void k_add_nodes_ordered(double *__restrict__ x, const int32_t *__restrict__ u, const int32_t *__restrict__ off,
                                    const int32_t *__restrict__ slot, int64_t n, int64_t voff,
                                    const double *__restrict__ buf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t nd = u[i];
    double s0 = x[nd * 3 + 0], s1 = x[nd * 3 + 1], s2 = x[nd * 3 + 2], s3 = x[voff + nd];
    for (int j = off[i]; j < off[i + 1]; ++j) {
      const double *b = buf + (int64_t)slot[j] * 4;
      s0 += b[0];
      s1 += b[1];
      s2 += b[2];
      s3 += b[3];
    }
    x[nd * 3 + 0] = s0;
    x[nd * 3 + 1] = s1;
    x[nd * 3 + 2] = s2;
    x[voff + nd] = s3;
  }
}
hipError_t vec_add_nodes_ordered(double *x, const int32_t *u, const int32_t *off, const int32_t *slot, int64_t n,
                                 int64_t voff, const double *buf, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_add_nodes_ordered, dim3(grid_for(n)), dim3(kBlock), 0, s, x, u, off, slot, n, voff, buf);
  return hipGetLastError();
}
hipError_t vec_set_indexed(double *y, const int64_t *idx, const double *vals, int64_t m, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_set_indexed, dim3(grid_for(m)), dim3(kBlock), 0, s, y, idx, vals, m);
  return hipGetLastError();
}

}  // namespace gls

// ---- assembled-ILU preconditioner helpers (gls_api.cpp ilu_*): probe vectors and value extraction
namespace gls {
namespace {
template <typename I>
__global__ void k_set_const_indexed(double *x, const I *idx, int64_t m, double a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) x[idx[i]] = a;
}
// the ILU's remote entries (64-bit positions): x[u[i]] += buf[slot[j]], j in [off[i], off[i+1]) in order
__global__ void k_add_pos_ordered(double *__restrict__ x, const int64_t *__restrict__ u, const int32_t *__restrict__ off,
                                  const int32_t *__restrict__ slot, int64_t n, const double *__restrict__ buf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double s = x[u[i]];
    for (int j = off[i]; j < off[i + 1]; ++j) s += buf[slot[j]];
    x[u[i]] = s;
  }
}
// batched probes p0 .. : V[(pid[e] - p0) * n + dofs[e]] = 1 (V zeroed) and the extraction
// val[ent[e]] = Y[(pid[e] - p0) * n + row[e]]
__global__ void k_probe_set_b(double *V, int64_t n, const int32_t *dofs, const int32_t *pid, int p0, int64_t m) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < m) V[(int64_t)(pid[e] - p0) * n + dofs[e]] = 1.0;
}
__global__ void k_probe_extract_b(double *val, const int64_t *ent, const int32_t *row, const int32_t *pid, int p0,
                                  int64_t m, const double *Y, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < m) val[ent[e]] = Y[(int64_t)(pid[e] - p0) * n + row[e]];
}
// CSR values of the entries whose column belongs to one probe: val[ent[i]] = y[row[i]]
__global__ void k_probe_extract(double *val, const int64_t *ent, const int32_t *row, int64_t m, const double *y,
                                int add) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) val[ent[i]] = add ? val[ent[i]] + y[row[i]] : y[row[i]];
}
// Ifpack-style diagonal perturbation before the factorisation: a_ii <- rthresh a_ii + sign(a_ii) athresh
__global__ void k_diag_perturb(double *val, const int64_t *didx, int64_t n, double athresh, double rthresh) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = val[didx[i]];
  val[didx[i]] = rthresh * a + (a < 0 ? -athresh : athresh);
}
// out[idx[i]] = in[i] (scatter, dir 0) or out[i] = in[idx[i]] (gather, dir 1)
// dense column-major A (A[j * n + i] = A_ij in DoF numbering) from a CSR in a renumbered order (perm: DoF -> CSR
// row, inv: CSR row -> DoF); positions outside the pattern are left as they are (the caller zeroes A)
__global__ void k_csr_to_dense(double *__restrict__ A, const int64_t *__restrict__ rowp, const int32_t *__restrict__ col,
                               const double *__restrict__ val, const int32_t *__restrict__ perm,
                               const int32_t *__restrict__ inv, int64_t n) {
  for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < n; d += (int64_t)gridDim.x * blockDim.x) {
    const int r = perm[d];
    for (int64_t e = rowp[r]; e < rowp[r + 1]; ++e) A[(int64_t)inv[col[e]] * n + d] = val[e];
  }
}
__global__ void k_invert_perm(int32_t *__restrict__ inv, const int32_t *__restrict__ perm, int64_t n) {
  for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < n; d += (int64_t)gridDim.x * blockDim.x)
    inv[perm[d]] = (int32_t)d;
}
__global__ void k_permute(double *out, const double *in, const int32_t *idx, int64_t n, int dir) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (dir == 0) out[idx[i]] = in[i];
  else out[i] = in[idx[i]];
}
}  // namespace
hipError_t csr_to_dense(double *A, const int64_t *rowp, const int32_t *col, const double *val, const int32_t *perm,
                        const int32_t *inv, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_invert_perm, dim3(grid_for(n)), dim3(kBlock), 0, s, const_cast<int32_t *>(inv), perm, n);
  hipLaunchKernelGGL(k_csr_to_dense, dim3(grid_for(n)), dim3(kBlock), 0, s, A, rowp, col, val, perm, inv, n);
  return hipGetLastError();
}
hipError_t vec_permute(double *out, const double *in, const int32_t *idx, int64_t n, int dir, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_permute, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, in, idx, n, dir);
  return hipGetLastError();
}
hipError_t vec_set_const_indexed(double *x, const int32_t *idx, int64_t m, double a, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_set_const_indexed<int32_t>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, x, idx, m, a);
  return hipGetLastError();
}
hipError_t vec_set_const_indexed64(double *x, const int64_t *idx, int64_t m, double a, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_set_const_indexed<int64_t>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, x, idx, m, a);
  return hipGetLastError();
}
hipError_t vec_add_pos_ordered(double *x, const int64_t *u, const int32_t *off, const int32_t *slot, int64_t n,
                               const double *buf, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_add_pos_ordered, dim3(grid_for(n)), dim3(kBlock), 0, s, x, u, off, slot, n, buf);
  return hipGetLastError();
}
hipError_t probe_set_batched(double *V, int64_t n, const int32_t *dofs, const int32_t *pid, int p0, int64_t m,
                             hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_probe_set_b, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, V, n, dofs, pid, p0, m);
  return hipGetLastError();
}
hipError_t probe_extract_batched(double *val, const int64_t *ent, const int32_t *row, const int32_t *pid, int p0,
                                 int64_t m, const double *Y, int64_t n, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_probe_extract_b, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, val, ent, row, pid, p0, m, Y, n);
  return hipGetLastError();
}
hipError_t vec_csr_gather_set_b(double *x, const int64_t *dof, const int64_t *off, const int64_t *master,
                                const double *w, int64_t n, int nb, int64_t bs, hipStream_t s) {
  if (n <= 0 || nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_csr_gather_set, dim3(grid_for(n), nb), dim3(kBlock), 0, s, x, x, dof, off, master, w, n, bs);
  return hipGetLastError();
}
hipError_t vec_csr_condense_b(double *y, const int64_t *tm, const int64_t *toff, const int64_t *tdof, const double *tw,
                              int64_t n, int nb, int64_t bs, hipStream_t s) {
  if (n <= 0 || nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_csr_condense, dim3(grid_for(n), nb), dim3(kBlock), 0, s, y, tm, toff, tdof, tw, n, bs);
  return hipGetLastError();
}
hipError_t vec_gather_scale_set_b(double *y, const double *d, const double *v, const int64_t *idx, int64_t m, int nb,
                                  int64_t bs, hipStream_t s) {
  if (m <= 0 || nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_scale_set, dim3(grid_for(m), nb), dim3(kBlock), 0, s, y, d, v, idx, m, nullptr, bs);
  return hipGetLastError();
}
hipError_t gather_element_vectors_b(double *y, const double *ev, const int64_t *voff, const int64_t *vslot, int64_t nv,
                                    const int64_t *poff, const int64_t *pslot, int64_t np, int dim, int nb, int64_t ys,
                                    int64_t evs, const uint8_t *act, int64_t el, int cb, int nblk, hipStream_t s) {
  const int64_t n = nv + np;
  if (n <= 0 || nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_ev, dim3((unsigned)((n + 255) / 256), nb), dim3(256), 0, s, y, ev, voff, vslot, nv, poff,
                     pslot, np, dim, ys, evs, act, el, cb, nblk);
  return hipGetLastError();
}
hipError_t csr_probe_extract(double *val, const int64_t *ent, const int32_t *row, int64_t m, const double *y,
                             hipStream_t s, bool add) {
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_probe_extract, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, val, ent, row, m, y,
                     add ? 1 : 0);
  return hipGetLastError();
}
hipError_t csr_diag_perturb(double *val, const int64_t *didx, int64_t n, double athresh, double rthresh,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_diag_perturb, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, val, didx, n, athresh, rthresh);
  return hipGetLastError();
}
}  // namespace gls
