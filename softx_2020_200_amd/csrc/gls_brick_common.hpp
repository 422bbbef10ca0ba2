// gls_brick_common.hpp — device helpers shared by the brick kernels (gls_brick_kernels.hip) and the
// pencil-dataflow J.v (gls_brick_pencil.hip).
#pragma once
#include "gls_common.hpp"

namespace gls {

// bijective XCD swizzle of n work items: orig % 8 labels the blocks that share an XCD (blocks b, b+8,
// ... land on one XCD); each XCD then walks a contiguous range of the items
__device__ __forceinline__ int xcd_swizzle(int orig, int n) {
  const int q = n / 8, r = n % 8, x = orig % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8;
}

// rank of brick-lattice node (X, Y, Z) among the brick-boundary nodes (lexicographic, x fastest):
// its index minus the interior nodes that precede it
template <int BN>
__device__ __forceinline__ int bnd_index(int X, int Y, int Z) {
  constexpr int I = BN - 2;
  const int n = X + BN * (Y + BN * Z);
  int before = min(max(Z - 1, 0), I) * I * I;
  if (Z >= 1 && Z <= I) {
    before += min(max(Y - 1, 0), I) * I;
    if (Y >= 1 && Y <= I) before += min(max(X - 1, 0), I);
  }
  return n - before;
}

// LDS hand-off between lanes of ONE wave: LDS ops of a wave execute in order; the asm keeps the
// compiler from moving LDS accesses across this point.
__device__ __forceinline__ void wave_sync() {
#ifdef GLS_WAVE_SYNC_DRAIN
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
  asm volatile("" ::: "memory");
#endif
  __builtin_amdgcn_wave_barrier();
}

// Q2 J.v linearization ("pencil" layout, 16 values per quadrature point): bricks are taken in triples
// (the pencil kernel's workgroup), a triple's 24 cells in 4 groups of 6 (one wave each), and per
// (triple, wave, qz, value) the 6 cells x 9 (qx, qy) points are 54 consecutive entries, lane
// 9 c + 3 qy + qx. A wave of the pencil kernel reads each (qz, value) as one contiguous 432-byte row.
constexpr int kQdpRow = 54;                       // entries per (triple, wave, qz, value) row
constexpr int kQdpTriple = 4 * 3 * kQData * kQdpRow;  // entries per brick triple (10368 = 3 x 3456)
__device__ __forceinline__ int64_t qdp_base(int brick, int ci, int q) {
  const int cw = (brick % 3) * 8 + ci, w = cw / 6, c = cw % 6;
  const int qx = q % 3, qy = (q / 3) % 3, qz = q / 9;
  return (int64_t)(brick / 3) * kQdpTriple + ((w * 3 + qz) * kQData) * kQdpRow + 9 * c + 3 * qy + qx;
}

}  // namespace gls
