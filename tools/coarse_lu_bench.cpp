// Times the dense coarsest-level factorization options for an n x n FP64 matrix (n = 2916 is the
// Q2-Q2 4^3 coarsest MG level; n = 25000 the Q1-Q1 p-level of configs[4]'s base mesh): rocSOLVER getrf /
// getrf_npvt / getri / getrs and a plain dgemm, then getrf / getrs in FP32.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { auto e_ = (x); if (e_ != 0) { std::printf("fail %s: %d\n", #x, (int)e_); return 1; } } while (0)
int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2916;
  std::vector<double> A((size_t)n * n);
  srand(1);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) A[(size_t)j * n + i] = (i == j ? n : 0.0) + (double)rand() / RAND_MAX - 0.5;
  double *dA, *dB, *dC;
  int *ipiv, *info;
  CK(hipMalloc(&dA, sizeof(double) * n * n));
  CK(hipMalloc(&dB, sizeof(double) * n * n));
  CK(hipMalloc(&dC, sizeof(double) * n * n));
  CK(hipMalloc(&ipiv, sizeof(int) * n));
  CK(hipMalloc(&info, sizeof(int)));
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  auto now = [] { (void)hipDeviceSynchronize(); return std::chrono::steady_clock::now(); };
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemcpy(dA, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice));
    auto t0 = now();
    CK(rocsolver_dgetrf(h, n, n, dA, n, ipiv, info));
    auto t1 = now();
    CK(rocsolver_dgetri(h, n, dA, n, ipiv, info));
    auto t2 = now();
    CK(hipMemcpy(dA, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice));
    auto t3 = now();
    CK(rocsolver_dgetrf_npvt(h, n, n, dA, n, info));
    auto t4 = now();
    CK(hipMemcpy(dB, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice));
    auto t5 = now();
    CK(rocsolver_dgetrs(h, rocblas_operation_none, n, 1, dA, n, ipiv, dB, n));
    auto t6 = now();
    const double one = 1.0, zero = 0.0;
    CK(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, n, n, n, &one, dA, n, dB, n, &zero, dC, n));
    auto t7 = now();
    CK(rocblas_dgemv(h, rocblas_operation_none, n, n, &one, dA, n, dB, 1, &zero, dC, 1));
    auto t8 = now();
    std::printf("n=%d getrf %.2f ms getri %.2f ms getrf_npvt %.2f ms getrs(1 rhs) %.3f ms dgemm %.3f ms (%.1f TF) dgemv %.3f ms\n",
                n, ms(t0, t1), ms(t1, t2), ms(t3, t4), ms(t5, t6), ms(t6, t7), 2.0 * n * n * (double)n / ms(t6, t7) / 1e9,
                ms(t7, t8));
  }
  // the unpivoted factor applied by two rocBLAS triangular solves (1 RHS), and the triangular inverses
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipMemcpy(dA, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice));
    CK(rocsolver_dgetrf_npvt(h, n, n, dA, n, info));
    CK(hipMemcpy(dB, A.data(), sizeof(double) * n, hipMemcpyHostToDevice));
    auto t0 = now();
    CK(rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_unit, n, dA, n, dB, 1));
    CK(rocblas_dtrsv(h, rocblas_fill_upper, rocblas_operation_none, rocblas_diagonal_non_unit, n, dA, n, dB, 1));
    auto t1 = now();
    CK(hipMemcpy(dC, dA, sizeof(double) * n * n, hipMemcpyDeviceToDevice));
    auto t2 = now();
    CK(rocsolver_dtrtri(h, rocblas_fill_upper, rocblas_diagonal_non_unit, n, dC, n, info));
    auto t3 = now();
    CK(rocsolver_dtrtri(h, rocblas_fill_lower, rocblas_diagonal_unit, n, dC, n, info));
    auto t4 = now();
    std::printf("n=%d dtrsv L+U (1 rhs) %.3f ms, dtrtri upper %.2f ms, dtrtri lower %.2f ms\n", n, ms(t0, t1), ms(t2, t3),
                ms(t3, t4));
  }
  std::vector<float> Af(A.begin(), A.end());
  float *fA, *fB;
  CK(hipMalloc(&fA, sizeof(float) * n * n));
  CK(hipMalloc(&fB, sizeof(float) * n));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemcpy(fA, Af.data(), sizeof(float) * n * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(fB, Af.data(), sizeof(float) * n, hipMemcpyHostToDevice));
    auto t0 = now();
    CK(rocsolver_sgetrf(h, n, n, fA, n, ipiv, info));
    auto t1 = now();
    CK(rocsolver_sgetrs(h, rocblas_operation_none, n, 1, fA, n, ipiv, fB, n));
    auto t2 = now();
    CK(hipMemcpy(fA, Af.data(), sizeof(float) * n * n, hipMemcpyHostToDevice));
    auto t3 = now();
    CK(rocsolver_sgetrf_npvt(h, n, n, fA, n, info));
    auto t4 = now();
    CK(rocblas_strsv(h, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_unit, n, fA, n, fB, 1));
    CK(rocblas_strsv(h, rocblas_fill_upper, rocblas_operation_none, rocblas_diagonal_non_unit, n, fA, n, fB, 1));
    auto t5 = now();
    std::printf("n=%d sgetrf %.2f ms (%.1f TF) sgetrs(1 rhs) %.3f ms sgetrf_npvt %.2f ms strsv L+U %.3f ms\n", n,
                ms(t0, t1), 2.0 / 3.0 * n * (double)n * n / ms(t0, t1) / 1e9, ms(t1, t2), ms(t3, t4), ms(t4, t5));
  }
  return 0;
}
