// Weight-gradient engine: dW[o][i] = sum_n P[n][o] * Q[n][i], db[o] = sum_n P[n][o],
// over MANY rows n (16,000 - 128,000 nodes) into a small [O x I] output (O, I <= 256).
//
// Used by the node-MLP backward (dW2 = do^T r, dW1 = da1^T z; models/gnn.py:21-26 via
// autograd) and by the plain Linears around the GINE stack (DeepSet rho/phi, dim_red,
// aggr: models/gnn.py:48-68,112-123).  P and Q come from "source" policies that load raw
// operands and apply the elementwise prologue (ReLU masks, BatchNorm backward, ...) when
// the tile is staged, so the [N x D] operands are never materialised.
//
// Decomposition: grid = (row chunks, 64x128 output tiles, Z independent products).  A
// 256-thread workgroup owns one 64(o) x 128(i) output tile of one row chunk; wave w holds
// i-columns [32w, 32w+32) for all 64 o-rows as two v_mfma_f32_32x32x2_f32 accumulators
// (one B fragment feeds two MFMAs).  64-row sub-tiles of P and Q are staged through LDS;
// the RAW operands of the next sub-tile are loaded into registers before this sub-tile's
// 64-long MFMA chain and transformed only when staged, so their HBM latency hides under
// the matrix pipe.  Each (chunk, tile) writes an fp32 partial slab; slabs are reduced over
// chunks in fixed order in fp64 (deterministic, no float atomics).
#pragma once

#include "gine_common.hpp"

namespace gine {

typedef float wg_floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWgRows = 64;                           // rows per staged sub-tile
constexpr int kWgTO = 64;                             // o-rows per workgroup tile
constexpr int kWgTI = 128;                            // i-columns per workgroup tile
constexpr int kWgLdP = kWgTO + 4;                     // padded LDS rows (floats)
constexpr int kWgLdQ = kWgTI + 4;
constexpr int kWgPItems = kWgRows * kWgTO / 4 / 256;  // float4 per thread per sub-tile: 4
constexpr int kWgQItems = kWgRows * kWgTI / 4 / 256;  // 8
constexpr int kWgTargetBlocks = 256;                  // one workgroup per CU
constexpr int kWgMinSubtiles = 2;                     // per chunk

struct WgPlan {
  int tiles_o, tiles_i, chunks, rows_per_chunk;
};

// Z products of [O x I] over R rows: about one workgroup per CU, >= 2 sub-tiles per chunk.
inline WgPlan wg_plan(int64_t R, int O, int I, int Z) {
  WgPlan p;
  p.tiles_o = (int)ceil_div(O, kWgTO);
  p.tiles_i = (int)ceil_div(I, kWgTI);
  const int64_t subtiles = ceil_div(R > 0 ? R : 1, kWgRows);
  int64_t chunks = ceil_div(kWgTargetBlocks, (int64_t)Z * p.tiles_o * p.tiles_i);
  const int64_t cap = ceil_div(subtiles, kWgMinSubtiles);
  if (chunks > cap) chunks = cap;
  if (chunks < 1) chunks = 1;
  const int64_t per = ceil_div(subtiles, chunks);
  p.rows_per_chunk = (int)(per * kWgRows);
  p.chunks = (int)ceil_div(R > 0 ? R : 1, p.rows_per_chunk);
  return p;
}

// Src policy (see the users in gine_mlp.hip / gine_linear.hip); every member is a
// template on the product index Z, so each body is free of runtime branches between loads
// (a branch merge makes the compiler drain the memory queue, serialising the prefetch):
//   typename Src::Raw, Src::Col
//   Col p_col<Z>(q4) / q_col<Z>(q4)          per-column constants (q4 = float4 column)
//   Raw p_load<Z>(n, q4) / q_load<Z>(n, q4)  raw operands of row n (n always in range)
//   float4 p_xform<Z>(raw, col) / q_xform<Z> the staged value
template <class Src, int Z>
__device__ __forceinline__ void wgrad_body(const Src& src, int64_t R, int O, int I,
                                           int rows_per_chunk, int tiles_i, size_t zstride,
                                           size_t cstride, float* __restrict__ slab,
                                           float* __restrict__ sP, float* __restrict__ sQ) {
  using Raw = typename Src::Raw;
  using Col = typename Src::Col;

  const int chunk = blockIdx.x;
  const int o0 = (blockIdx.y / tiles_i) * kWgTO, i0 = (blockIdx.y % tiles_i) * kWgTI;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const bool bias_block = (i0 == 0);

  // staging coordinates: a thread always stages the same float4 column of P and of Q
  const int pq = threadIdx.x % (kWgTO / 4), pr = threadIdx.x / (kWgTO / 4);  // rows pr+16k
  const int qq = threadIdx.x % (kWgTI / 4), qr = threadIdx.x / (kWgTI / 4);  // rows qr+8k
  const bool p_ok = o0 + 4 * pq < O, q_ok = i0 + 4 * qq < I;
  const int pqa = p_ok ? o0 / 4 + pq : 0, qqa = q_ok ? i0 / 4 + qq : 0;
  const Col pc = src.template p_col<Z>(pqa);
  const Col qc = src.template q_col<Z>(qqa);

  const int64_t r_begin = (int64_t)chunk * rows_per_chunk;
  const int64_t r_end = min<int64_t>(R, r_begin + rows_per_chunk);

  wg_floatx16 acc0, acc1;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc0[k] = acc1[k] = 0.f;
  double bsum[4] = {0.0, 0.0, 0.0, 0.0};  // bias partials of this thread's P column quad

  Raw rp[kWgPItems], rq[kWgQItems];
  auto load = [&](int64_t n0) {
#pragma unroll
    for (int k = 0; k < kWgPItems; ++k) {
      const int64_t n = n0 + pr + 16 * k;
      rp[k] = src.template p_load<Z>(n < r_end ? n : r_end - 1, pqa);
    }
#pragma unroll
    for (int k = 0; k < kWgQItems; ++k) {
      const int64_t n = n0 + qr + 8 * k;
      rq[k] = src.template q_load<Z>(n < r_end ? n : r_end - 1, qqa);
    }
  };

  if (r_begin < r_end) load(r_begin);
  for (int64_t n0 = r_begin; n0 < r_end; n0 += kWgRows) {
#pragma unroll
    for (int k = 0; k < kWgPItems; ++k) {
      const int r = pr + 16 * k;
      float4 v = src.template p_xform<Z>(rp[k], pc);
      if (n0 + r >= r_end || !p_ok) v = f4_zero();
      *reinterpret_cast<float4*>(&sP[r * kWgLdP + 4 * pq]) = v;
      bsum[0] += (double)v.x;
      bsum[1] += (double)v.y;
      bsum[2] += (double)v.z;
      bsum[3] += (double)v.w;
    }
#pragma unroll
    for (int k = 0; k < kWgQItems; ++k) {
      const int r = qr + 8 * k;
      float4 v = src.template q_xform<Z>(rq[k], qc);
      if (n0 + r >= r_end || !q_ok) v = f4_zero();
      *reinterpret_cast<float4*>(&sQ[r * kWgLdQ + 4 * qq]) = v;
    }
    __syncthreads();
    if (n0 + kWgRows < r_end) load(n0 + kWgRows);  // raw operands of the next sub-tile
    // lane half h contracts rows [32h, 32h+32): the same permutation for A and B
    const float* pa = &sP[(32 * h) * kWgLdP + c32];
    const float* qb = &sQ[(32 * h) * kWgLdQ + 32 * wave + c32];
#pragma unroll
    for (int s = 0; s < kWgRows / 2; ++s) {
      const float a0 = pa[s * kWgLdP];
      const float a1 = pa[s * kWgLdP + 32];
      const float b = qb[s * kWgLdQ];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc1, 0, 0, 0);
    }
    __syncthreads();
  }

  float* out = slab + (size_t)Z * zstride + (size_t)chunk * cstride;
  const int i = i0 + 32 * wave + c32;
  if (i < I) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = o0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (o < O) out[(size_t)o * I + i] = acc0[r];
      if (o + 32 < O) out[(size_t)(o + 32) * I + i] = acc1[r];
    }
  }
  if (bias_block) {  // fixed-order sum of the 16 row groups' partials through LDS
    double* sb = reinterpret_cast<double*>(sQ);  // [16][64], sQ is free after the loop
#pragma unroll
    for (int j = 0; j < 4; ++j) sb[pr * kWgTO + 4 * pq + j] = bsum[j];
    __syncthreads();
    if (threadIdx.x < kWgTO && o0 + (int)threadIdx.x < O) {
      double t = 0.0;
      for (int g = 0; g < 256 / (kWgTO / 4); ++g) t += sb[g * kWgTO + threadIdx.x];
      out[(size_t)O * I + o0 + threadIdx.x] = (float)t;
    }
  }
}

template <class Src>
__global__ __launch_bounds__(256) void k_wgrad_engine(Src src, int64_t R, int O, int I,
                                                      int rows_per_chunk, int tiles_i,
                                                      size_t zstride, size_t cstride,
                                                      float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float sP[kWgRows * kWgLdP];
  __shared__ __attribute__((aligned(16))) float sQ[kWgRows * kWgLdQ];
  if (blockIdx.z == 0)
    wgrad_body<Src, 0>(src, R, O, I, rows_per_chunk, tiles_i, zstride, cstride, slab, sP, sQ);
  else
    wgrad_body<Src, 1>(src, R, O, I, rows_per_chunk, tiles_i, zstride, cstride, slab, sP, sQ);
}

template <class Src>
inline int launch_wgrad_engine(const Src& src, int64_t R, int O, int I, int Z,
                               const WgPlan& p, size_t zstride, size_t cstride, float* slab,
                               hipStream_t s) {
  hipLaunchKernelGGL((k_wgrad_engine<Src>), dim3(p.chunks, p.tiles_o * p.tiles_i, Z),
                     dim3(256), 0, s, src, R, O, I, p.rows_per_chunk, p.tiles_i, zstride,
                     cstride, slab);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

}  // namespace gine
