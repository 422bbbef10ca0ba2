// FP32 MFMA vs VALU for the pencil kernel's 1D contractions (tooling, not product code; VERDICT r4 item 2 asked
// for this A/B before ruling f32 MFMA out for the FP32 smoother).
//
// The pencil sweeps apply 3x3 Q2 operators (values V and derivatives D, stacked: 6 x 3) to lines of 3 node values:
// out[6][L] = B[6][3] x in[3][L]. Best case for each unit, operands resident in registers, no LDS traffic:
//   * VALU: a lane owns lines; 18 FMAs per line (v_fma_f32), dependent chains across iterations;
//   * MFMA: v_mfma_f32_16x16x4_f32 with B padded to 16 x 4 (rows 0-5 used, k 0-2 used) and 16 lines per
//     instruction as the N dimension: 6 x 3 x 16 useful FMAs of the 16 x 4 x 16 issued (28 %).
// Useful FLOPs = 2 x 18 per line in both. Printed: useful TFLOP/s of each over the whole chip.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_f32_ab tools/mfma_f32_ab.hip ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

__global__ void __launch_bounds__(256) k_valu(float *out, float s) {
  // 4 independent lines per lane (ILP), 3 node values each
  float x[4][3];
  for (int l = 0; l < 4; ++l)
    for (int n = 0; n < 3; ++n) x[l][n] = 0.001f * (threadIdx.x + 7 * l + 3 * n);
  const float B[6][3] = {{0.6872f, 0.4000f, -0.0872f}, {0.f, 1.f, 0.f}, {-0.0872f, 0.4000f, 0.6872f},
                         {-2.549f, 3.098f, -0.549f},    {-1.f, 0.f, 1.f}, {0.549f, -3.098f, 2.549f}};
  float acc = 0.f;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      float o[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) o[q] = fmaf(B[q][2], x[l][2], fmaf(B[q][1], x[l][1], B[q][0] * x[l][0]));
      // feed back (the next sweep reads this one's output): keeps the chain dependent
      x[l][0] = fmaf(s, o[0], o[3]);
      x[l][1] = fmaf(s, o[1], o[4]);
      x[l][2] = fmaf(s, o[2], o[5]);
    }
  }
  for (int l = 0; l < 4; ++l) acc += x[l][0] + x[l][1] + x[l][2];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) k_mfma(float *out, float s) {
  const int lane = threadIdx.x & 63;
  // A operand (16 x 4): lane holds A[row = lane % 16][k = lane / 16]; rows 0-5 = V and D, k 0-2
  const float B[6][3] = {{0.6872f, 0.4000f, -0.0872f}, {0.f, 1.f, 0.f}, {-0.0872f, 0.4000f, 0.6872f},
                         {-2.549f, 3.098f, -0.549f},    {-1.f, 0.f, 1.f}, {0.549f, -3.098f, 2.549f}};
  const int ar = lane % 16, ak = lane / 16;
  const float a = (ar < 6 && ak < 3) ? B[ar][ak] : 0.f;
  // B operand (4 x 16): lane holds in[k = lane / 16][line = lane % 16]; 4 independent 16-line groups (ILP)
  float b[4];
  for (int g = 0; g < 4; ++g) b[g] = ak < 3 ? 0.001f * (lane + 5 * g) : 0.f;
  v4f c[4];
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[g], v4f{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      // lane holds C[rows 4 * (lane / 16) .. + 3][line lane % 16]: rows 0-3 for lanes 0-15, 4-7 for 16-31 ...
      // feed back one output per lane into the next input (dependent chain, like the VALU kernel)
      b[g] = ak < 3 ? fmaf(s, c[g][0], c[g][1]) : 0.f;
    }
  }
  float acc = 0.f;
  for (int g = 0; g < 4; ++g) acc += c[g][0] + c[g][1] + c[g][2] + c[g][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = ncu * 8, threads = 256;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
  float *out = nullptr;
  if (hipMalloc(&out, sizeof(float) * blocks * threads) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    float ms_v = 0.f, ms_m = 0.f;
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(threads), 0, 0, out, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms_v, e0, e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(threads), 0, 0, out, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms_m, e0, e1);
    // useful FLOPs: 18 FMAs per line per iteration (the 6 x 3 contraction) + the 3 feedback FMAs counted as
    // overhead in neither; VALU: 4 lines per lane; MFMA: 4 groups of 16 lines per wave
    const double lines_v = (double)blocks * threads * 4 * kIters;
    const double lines_m = (double)blocks * (threads / 64) * 4 * 16 * kIters;
    std::printf("rep %d: VALU %.3f ms, %.1f useful TFLOP/s | MFMA 16x16x4 f32 %.3f ms, %.1f useful TFLOP/s "
                "(%.1f issued)\n", rep, ms_v, lines_v * 36 / (ms_v * 1e-3) / 1e12, ms_m,
                lines_m * 36 / (ms_m * 1e-3) / 1e12, (double)blocks * (threads / 64) * 4 * kIters * 2048 / (ms_m * 1e-3) / 1e12);
  }
  hipFree(out);
  return 0;
}
