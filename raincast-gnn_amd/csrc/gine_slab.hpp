// Fixed-order reduction of split-K partial slabs (deterministic, no float atomics).
//
// Split-row weight-gradient kernels (gine_wgrad.hpp, gine_deepset.hip) leave Z products x
// C chunks of fp32 partials: slab[z * zstride + c * cstride + e], e < per.  out(z, e, v)
// receives sum_c partial in fp64, summed in chunk order within each of kSlabGroups
// interleaved chunk groups and then over the groups in group order -- a function of the
// shapes only, so a rerun is bit-identical.  A workgroup covers 32 float4 quads (128
// elements) x 8 chunk groups; loads are 16-byte and independent (four per loop trip).
#pragma once

#include "gine_common.hpp"

namespace gine {

// Chunk loads in flight per thread: 8 covers the engines' <= 64 chunks (8 groups) in one
// batch (r02_s58: gradient batch 15.1 -> 13.6 us at cfg2; 4 took two memory round trips).
#ifndef GINE_SLAB_UNROLL
#define GINE_SLAB_UNROLL 8
#endif
constexpr int kSlabQuads = 32;   // float4 quads per workgroup
constexpr int kSlabGroups = 8;   // interleaved chunk groups per workgroup

// One workgroup (column block bx of product z); s_part: kSlabGroups x (4*kSlabQuads+1)
// doubles of LDS.
template <bool VEC, class Out>
__device__ __forceinline__ void slab_sum_block(const float* __restrict__ slab, int chunks,
                                               int64_t per, size_t cstride, size_t zstride,
                                               const Out& out, int bx, int z,
                                               double (*s_part)[kSlabQuads * 4 + 1]) {
  const int q = threadIdx.x % kSlabQuads, g = threadIdx.x / kSlabQuads;
  const int64_t e0 = ((int64_t)bx * kSlabQuads + q) * 4;
  const float* base = slab + (size_t)z * zstride;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (e0 < per) {
    if constexpr (VEC) {
#pragma unroll GINE_SLAB_UNROLL
      for (int c = g; c < chunks; c += kSlabGroups) {
        const float4 v = *reinterpret_cast<const float4*>(base + (size_t)c * cstride + e0);
        a0 += (double)v.x;
        a1 += (double)v.y;
        a2 += (double)v.z;
        a3 += (double)v.w;
      }
    } else {
      const int64_t last = per - 1;
#pragma unroll 4
      for (int c = g; c < chunks; c += kSlabGroups) {
        const float* r = base + (size_t)c * cstride;
        a0 += (double)r[e0];
        a1 += (double)r[min(e0 + 1, last)];
        a2 += (double)r[min(e0 + 2, last)];
        a3 += (double)r[min(e0 + 3, last)];
      }
    }
  }
  double* sp = &s_part[g][4 * q];
  sp[0] = a0;
  sp[1] = a1;
  sp[2] = a2;
  sp[3] = a3;
  __syncthreads();
  if (threadIdx.x >= kSlabQuads * 4) return;
  const int j = threadIdx.x;
  const int64_t e = (int64_t)bx * kSlabQuads * 4 + j;
  if (e >= per) return;
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < kSlabGroups; ++k) v += s_part[k][j];
  out(z, e, v);
}

template <bool VEC, class Out>
__global__ __launch_bounds__(256) void k_slab_sum(const float* __restrict__ slab, int chunks,
                                                  int64_t per, size_t cstride, size_t zstride,
                                                  Out out) {
  __shared__ double s_part[kSlabGroups][kSlabQuads * 4 + 1];
  slab_sum_block<VEC, Out>(slab, chunks, per, cstride, zstride, out, blockIdx.x, blockIdx.y,
                           s_part);
}

// Destination of the node-MLP weight-gradient slabs: z = 0 -> dW2 | db2, z = 1 -> dW1 | db1.
struct MlpWgradOut {
  float *dw2, *db2, *dw1, *db1;
  int D;
  __device__ void operator()(int z, int64_t e, double v) const {
    float* w = z == 0 ? dw2 : dw1;
    float* b = z == 0 ? db2 : db1;
    if (e < (int64_t)D * D) {
      if (w) w[e] = (float)v;
    } else if (b) {
      b[e - (int64_t)D * D] = (float)v;
    }
  }
};

// The node-MLP slab reduction run as extra workgroups of another launch (gine_mp_bwd_side):
// block b < nblocks reduces column block b % cols of product b / cols.
struct MlpSlabJob {
  const float* slab;
  int chunks;
  int cols;     // column blocks per product
  int nblocks;  // 2 * cols, or 0 = no job
  MlpWgradOut out;
  __device__ void run(int b, double (*s_part)[kSlabQuads * 4 + 1]) const {
    const int64_t per = (int64_t)out.D * out.D + out.D;
    slab_sum_block<true, MlpWgradOut>(slab, chunks, per, (size_t)per, (size_t)per * chunks, out,
                                      b % cols, b / cols, s_part);
  }
};

template <class Out>
inline int launch_slab_sum(const float* slab, int chunks, int64_t per, size_t cstride,
                           size_t zstride, int Z, const Out& out, hipStream_t s) {
  const dim3 grid((unsigned)ceil_div(per, kSlabQuads * 4), Z);
  const bool vec = per % 4 == 0 && cstride % 4 == 0 && zstride % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(slab) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL((k_slab_sum<true, Out>), grid, dim3(256), 0, s, slab, chunks, per,
                       cstride, zstride, out);
  else
    hipLaunchKernelGGL((k_slab_sum<false, Out>), grid, dim3(256), 0, s, slab, chunks, per,
                       cstride, zstride, out);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

}  // namespace gine
