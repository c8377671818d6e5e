// Shared device/host helpers for the gfx950 GINEConv engine.
// Everything in this directory is compiled with -ffp-contract=off: the message-passing
// kernels reproduce the CPU rounding sequence exactly, so the only fused multiply-adds are
// the explicit __builtin_fmaf calls (CPU Linear(1,D) rounds once, like an fma) and the MFMA
// accumulation chains of the node-MLP GEMMs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gine_hip.h"

#define GINE_RETURN_IF_HIP(expr)                                  \
  do {                                                            \
    hipError_t gine_e_ = (expr);                                  \
    if (gine_e_ != hipSuccess) return GINE_ERR_HIP_BASE + (int)gine_e_; \
  } while (0)

// Every kernel of the library is compiled without the packed-FP32 VALU instructions
// (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32; Makefile: -target-feature -packed-fp32-ops,
// so the compiler emits two-lane VOP3 ops instead).  Measured on MI355X (DESIGN.md 4,
// profiles/r05_s01-s03): in the combined window backward, the low halves of the
// message-passing waves' packed-FP32 results came out wrong and varied from run to run (even
// float columns of dx, ~100 of 16,000 rows) whenever the co-resident engine workgroups ran
// v_mfma_f32_32x32x16_bf16 -- with the message-passing code byte-identical, and correct with
// the fp32 MFMA, without the bf16 MFMAs (at 120 and at 128 VGPRs) and without packed FP32.
// The unpacked form is also as fast or faster here (gather backward at cfg5 87-90 -> 77-79
// us; window backward 13.1 -> 12.3 us at cfg2).  (A `target("no-packed-fp32-ops")` function
// attribute does the same per kernel, but measured 176 instead of 12 bytes of spill in the
// combined window backward, so the switch is the command-line feature.)

#define GINE_LAUNCH_STATUS() \
  do {                                                            \
    hipError_t gine_e_ = hipGetLastError();                       \
    if (gine_e_ != hipSuccess) return GINE_ERR_HIP_BASE + (int)gine_e_; \
  } while (0)

namespace gine {

constexpr int kWave = 64;   // CDNA wavefront width
constexpr int kNumXcd = 8;  // MI355X: 8 XCDs, each with a private 4 MiB L2
constexpr int kNumCu = 256;  // 32 CUs per XCD

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Blocks are dealt round-robin over the 8 XCDs (blocks b and b+8 share one).  Remap the
// hardware block id so that every XCD walks one contiguous range of tiles: neighbouring
// destinations gather neighbouring source rows (graphs are block-diagonal batches of
// station graphs), so a contiguous range keeps those rows in that XCD's L2.  Bijective for
// any grid size (remainder-aware); a placement other than round-robin only costs speed.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int q = nblocks / kNumXcd, r = nblocks % kNumXcd;
  const int xcd = bid % kNumXcd, pos = bid / kNumXcd;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + pos;
}

__device__ __forceinline__ float4 f4_zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// relu with ATen's NaN propagation (clamp_min keeps NaN): IEEE-754-2019 maximum(v, +0)
// propagates NaN and orders -0 < +0 -- one v_maximum3_f32 on gfx950 instead of a compare
// and a select.  A NaN comes out quieted (its payload may differ from the CPU's).
__device__ __forceinline__ float relu_nan(float v) { return __builtin_elementwise_maximum(v, 0.0f); }

// True in every thread when `pred` holds in any thread of the workgroup.  `word`: an int of
// the caller's LDS that nothing else touches during the call (no static LDS of its own,
// unlike __syncthreads_or: kernels that raise their dynamic-LDS ceiling to the whole 160 KiB
// cannot have any).  Four barriers; every thread has read the answer before any returns.
__device__ __forceinline__ bool block_any(bool pred, int* word) {
  __syncthreads();
  if (threadIdx.x == 0) *word = 0;
  __syncthreads();
  if (pred) *word = 1;  // the same value from every writer
  __syncthreads();
  const bool any = *word != 0;
  __syncthreads();
  return any;
}

// Edge Linear(1, D): a*w + b, rounded like the host CPU's PyG path (see gine_hip.h).
template <bool FMA>
__device__ __forceinline__ float edge_lin(float a, float w, float b) {
  if constexpr (FMA) return __builtin_fmaf(a, w, b);
  return a * w + b;  // -ffp-contract=off: two roundings
}

// Double-precision block reduction helper over the 32 lanes of one MFMA column half.
__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  return __shfl_xor(v, m, kWave);
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Non-NaN targets of y [n] as GINE_COUNT_PARTS uint32 partial counts (part p counts the
// contiguous range p * ceil(n / P) ...), written by the workgroups of the calling launch:
// workgroup b writes parts b, b + gridDim.x, ...  Blocks of exactly 256 threads.  Integer
// counts: the consumer's sum is exact whatever the order (gine_crps_fwd_grad).
__device__ __forceinline__ void count_valid_parts(const float* __restrict__ y, int64_t n,
                                                  uint32_t* __restrict__ parts) {
  __shared__ uint32_t s_w[4];
  const int64_t chunk = (n + GINE_COUNT_PARTS - 1) / GINE_COUNT_PARTS;
  for (int p = blockIdx.x; p < GINE_COUNT_PARTS; p += gridDim.x) {
    const int64_t lo = (int64_t)p * chunk, hi = lo + chunk < n ? lo + chunk : n;
    uint32_t c = 0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) c += y[i] == y[i];
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    __syncthreads();  // s_w of the previous part has been read
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) parts[p] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  }
}

}  // namespace gine
