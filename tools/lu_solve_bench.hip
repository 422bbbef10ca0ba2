// lu_solve_bench.hip -- timing and correctness of the coarsest level's FP32 dense LU solves
// (gls::dense_lu_solve_f32, csrc/gls_mg_kernels.hip) against a one-barrier-per-column variant kept here
// for the A/B, at the coarse sizes of the configs[4] p-level (n = 25000).
// Build: hipcc -O3 --offload-arch=gfx950 tools/lu_solve_bench.hip -L softx_2020_200_amd -lgls_native
//        -Wl,-rpath,$PWD/softx_2020_200_amd -o tools/lu_solve_bench
// Run:   tools/lu_solve_bench [n ...]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace gls {
hipError_t dense_lu_solve_f32(const float *LU, int n, float *x, hipStream_t s, int bl, int bu);
}

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int B = 128;
// the variant with one workgroup barrier per column of the diagonal block (for the A/B)
template <bool LOWER>
__global__ void __launch_bounds__(B) k_step_barrier(const float *A, int n, float *x, int k) {
  __shared__ float xk[B], xb[B];
  __shared__ float D[B][B + 1];
  const int t = threadIdx.x, nb = (n + B - 1) / B;
  auto diag = [&](int r0, int nr, float v) {
    if (t < nr)
      for (int c = 0; c < nr; ++c) D[t][c] = A[(r0 + t) + (int64_t)(r0 + c) * n];
    __syncthreads();
    if (LOWER) {
      for (int c = 0; c < nr; ++c) {
        if (t == c) xb[c] = v;
        __syncthreads();
        if (t > c && t < nr) v -= D[t][c] * xb[c];
      }
    } else {
      for (int c = nr - 1; c >= 0; --c) {
        if (t == c) xb[c] = v / D[c][c];
        __syncthreads();
        if (t < c) v -= D[t][c] * xb[c];
      }
    }
    __syncthreads();
    if (t < nr) x[r0 + t] = xb[t];
  };
  if (k < 0) {
    const int kb = LOWER ? 0 : nb - 1, r0 = kb * B, nr = min(B, n - r0);
    diag(r0, nr, t < nr ? x[r0 + t] : 0.f);
    return;
  }
  const int j0 = k * B, nj = min(B, n - j0);
  if (t < nj) xk[t] = x[j0 + t];
  __syncthreads();
  auto update = [&](int i) {
    float s = x[i];
    const float *a = A + i + (int64_t)j0 * n;
#pragma unroll 16
    for (int j = 0; j < nj; ++j) s -= a[(int64_t)j * n] * xk[j];
    return s;
  };
  const int kn = LOWER ? k + 1 : k - 1;
  if (blockIdx.x == 0) {
    const int r0 = kn * B, nr = min(B, n - r0);
    diag(r0, nr, t < nr ? update(r0 + t) : 0.f);
    return;
  }
  const int i = LOWER ? (k + 2) * B + ((int)blockIdx.x - 1) * B + t : ((int)blockIdx.x - 1) * B + t;
  if (LOWER ? i < n : i < kn * B) x[i] = update(i);
}
void solve_barrier(const float *LU, int n, float *x, hipStream_t s) {
  const int nb = (n + B - 1) / B;
  hipLaunchKernelGGL(k_step_barrier<true>, dim3(1), dim3(B), 0, s, LU, n, x, -1);
  for (int k = 0; k + 1 < nb; ++k) {
    const int rest = n - (k + 2) * B;
    hipLaunchKernelGGL(k_step_barrier<true>, dim3(1 + (rest > 0 ? (rest + B - 1) / B : 0)), dim3(B), 0, s, LU, n, x, k);
  }
  hipLaunchKernelGGL(k_step_barrier<false>, dim3(1), dim3(B), 0, s, LU, n, x, -1);
  for (int k = nb - 1; k >= 1; --k) hipLaunchKernelGGL(k_step_barrier<false>, dim3(1 + (k - 1)), dim3(B), 0, s, LU, n, x, k);
}

int main(int argc, char **argv) {
  std::vector<int> sizes;
  for (int i = 1; i < argc; ++i) sizes.push_back(std::atoi(argv[i]));
  if (sizes.empty()) sizes = {1000, 25000};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (const int n : sizes) {
    // unit-lower L and upper U in one column-major array: small off-diagonals, U_ii in [1, 2]
    std::vector<float> h((size_t)n * n);
    unsigned r = 12345u;
    auto rnd = [&]() { return (r = r * 1664525u + 1013904223u) / 4294967296.f; };
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) h[(size_t)j * n + i] = i == j ? 1.f + rnd() : (rnd() - 0.5f) * 2.f / n;
    std::vector<float> b(n), ref(n);
    for (int i = 0; i < n; ++i) b[i] = rnd() - 0.5f;
    {  // host reference in FP64: forward (unit lower), backward
      std::vector<double> y(b.begin(), b.end());
      for (int j = 0; j < n; ++j)
        for (int i = j + 1; i < n; ++i) y[i] -= (double)h[(size_t)j * n + i] * y[j];
      for (int j = n - 1; j >= 0; --j) {
        y[j] /= h[(size_t)j * n + j];
        for (int i = 0; i < j; ++i) y[i] -= (double)h[(size_t)j * n + i] * y[j];
      }
      for (int i = 0; i < n; ++i) ref[i] = (float)y[i];
    }
    float *dA, *dx;
    CK(hipMalloc(&dA, sizeof(float) * (size_t)n * n));
    CK(hipMalloc(&dx, sizeof(float) * n));
    CK(hipMemcpy(dA, h.data(), sizeof(float) * (size_t)n * n, hipMemcpyHostToDevice));
    for (int variant = 0; variant < 2; ++variant) {
      auto run = [&]() {
        if (variant == 0) CK(gls::dense_lu_solve_f32(dA, n, dx, s, -1, -1));
        else solve_barrier(dA, n, dx, s);
      };
      CK(hipMemcpy(dx, b.data(), sizeof(float) * n, hipMemcpyHostToDevice));
      run();
      std::vector<float> out(n);
      CK(hipMemcpy(out.data(), dx, sizeof(float) * n, hipMemcpyDeviceToHost));
      double num = 0, den = 0;
      for (int i = 0; i < n; ++i) {
        num += (double)(out[i] - ref[i]) * (out[i] - ref[i]);
        den += (double)ref[i] * ref[i];
      }
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      const int reps = 10;
      CK(hipEventRecord(e0, s));
      for (int q = 0; q < reps; ++q) run();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("n %6d %-22s rel err %.2e  %.3f ms per solve (%d launches)\n", n,
                  variant == 0 ? "dense_lu_solve_f32" : "barrier per column", std::sqrt(num / den), ms / reps,
                  2 * ((n + B - 1) / B));
      CK(hipEventDestroy(e0));
      CK(hipEventDestroy(e1));
    }
    CK(hipFree(dA));
    CK(hipFree(dx));
  }
  return 0;
}
