// Microbenchmarks that size the GLS kernel design on gfx950:
// FP64 VALU FMA rate, FP64 MFMA (v_mfma_f64_16x16x4_f64) rate, f64 global atomic add rate, HBM copy BW.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) valu_fma(double *out, int iters, double s) {
  double a0 = threadIdx.x * 1e-9, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0+4, a5=a0+5, a6=a0+6, a7=a0+7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      a0 = fma(a0, s, 1e-7); a1 = fma(a1, s, 1e-7); a2 = fma(a2, s, 1e-7); a3 = fma(a3, s, 1e-7);
      a4 = fma(a4, s, 1e-7); a5 = fma(a5, s, 1e-7); a6 = fma(a6, s, 1e-7); a7 = fma(a7, s, 1e-7);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ void __launch_bounds__(256) mfma_f64(double *out, int iters) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
  }
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// mixed: half the waves MFMA, half VALU -> do the pipes overlap?
__global__ void __launch_bounds__(256) mixed(double *out, int iters, double sc) {
  int w = threadIdx.x >> 6;
  double r;
  if (w & 1) {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
      }
    }
    d4 s = c0 + c1 + c2 + c3; r = s[0] + s[1] + s[2] + s[3];
  } else {
    double a0 = threadIdx.x * 1e-9, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0+4, a5=a0+5, a6=a0+6, a7=a0+7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        a0 = fma(a0, sc, 1e-7); a1 = fma(a1, sc, 1e-7); a2 = fma(a2, sc, 1e-7); a3 = fma(a3, sc, 1e-7);
        a4 = fma(a4, sc, 1e-7); a5 = fma(a5, sc, 1e-7); a6 = fma(a6, sc, 1e-7); a7 = fma(a7, sc, 1e-7);
      }
    }
    r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void atomics_f64(double *y, const int *idx, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&y[idx[i]], 1.0);
}
__global__ void copy_d2(const double2 *__restrict__ x, double2 *__restrict__ y, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  long st = (long)gridDim.x * blockDim.x;
  for (; i < n; i += st) y[i] = x[i];
}

int main() {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  double *out; CK(hipMalloc(&out, 8l << 24));
  int blocks = 256 * 8;
  int iters = 2000;
  float ms;
  // VALU
  hipLaunchKernelGGL(valu_fma, dim3(blocks), dim3(256), 0, 0, out, 10, 0.999999);
  CK(hipEventRecord(e0)); hipLaunchKernelGGL(valu_fma, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999999);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  double fl = 2.0 * 64 * iters * (double)blocks * 256;
  printf("VALU f64 FMA: %.2f TFLOP/s\n", fl / ms / 1e9);
  // MFMA
  hipLaunchKernelGGL(mfma_f64, dim3(blocks), dim3(256), 0, 0, out, 10);
  CK(hipEventRecord(e0)); hipLaunchKernelGGL(mfma_f64, dim3(blocks), dim3(256), 0, 0, out, iters);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  fl = 2.0 * 16 * 16 * 4 * 16 * (double)iters * blocks * 4;
  printf("MFMA f64 16x16x4: %.2f TFLOP/s\n", fl / ms / 1e9);
  // mixed
  CK(hipEventRecord(e0)); hipLaunchKernelGGL(mixed, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999999);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  fl = 0.5 * (2.0 * 16 * 16 * 4 * 16 * (double)iters * blocks * 4) + 0.5 * (2.0 * 64 * iters * (double)blocks * 256);
  printf("mixed MFMA||VALU: %.2f TFLOP/s (sum of both pipes)\n", fl / ms / 1e9);
  // atomics: 64M adds into 16M doubles, random-ish clustered (27 entries per cell pattern)
  long n = 64l << 20; long ny = 16l << 20;
  std::vector<int> h(n);
  unsigned s = 12345;
  for (long i = 0; i < n; i += 64) { s = s * 1664525u + 1013904223u; long base = (s % (ny - 1024)); for (int j = 0; j < 64 && i + j < n; ++j) h[i + j] = base + (j % 27) * 3 + j / 27; }
  int *didx; double *y; CK(hipMalloc(&didx, n * 4)); CK(hipMalloc(&y, ny * 8));
  CK(hipMemcpy(didx, h.data(), n * 4, hipMemcpyHostToDevice)); CK(hipMemset(y, 0, ny * 8));
  hipLaunchKernelGGL(atomics_f64, dim3((n + 255) / 256), dim3(256), 0, 0, y, didx, n);
  CK(hipEventRecord(e0)); hipLaunchKernelGGL(atomics_f64, dim3((n + 255) / 256), dim3(256), 0, 0, y, didx, n);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("f64 atomicAdd: %.3f G adds/s = %.1f GB/s of added bytes (%.3f ms)\n", n / ms / 1e6, n * 8.0 / ms / 1e6, ms);
  // copy
  long nc = 1l << 27;  // 128M double2 = 2 GiB each
  double2 *x2, *y2; CK(hipMalloc(&x2, nc * 16)); CK(hipMalloc(&y2, nc * 16)); CK(hipMemset(x2, 0, nc * 16));
  hipLaunchKernelGGL(copy_d2, dim3(256 * 16), dim3(256), 0, 0, x2, y2, nc);
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(copy_d2, dim3(256 * 16), dim3(256), 0, 0, x2, y2, nc);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("HBM copy: %.2f TB/s\n", 5 * 2.0 * nc * 16 / ms / 1e9);
  CK(hipDeviceSynchronize());
  return 0;
}
