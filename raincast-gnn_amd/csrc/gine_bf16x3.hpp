// fp32-class matrix products on the bf16 matrix cores (three-way split bf16).
//
// gfx950 runs v_mfma_f32_32x32x16_bf16 at 16x the FLOP rate of v_mfma_f32_32x32x2_f32
// (MI355X_MICROARCH.md: 32 vs 64 cycles for 8x the K).  Every fp32 operand is split into
// three bf16 planes, each the round-to-nearest bf16 of what the planes before it leave:
//   x = h + m + l + e,   h = bf16(x), m = bf16(x - h), l = bf16(x - h - m)
// (x - h and x - h - m are exact in fp32; |m| <= 2^-8 |x|, |l| <= 2^-16 |x|, |e| <= 2^-24 |x|)
// and a product is summed from the six partial products above 2^-24 of |a||b|:
//   a.b ~ al.bh + ah.bl + am.bm + am.bh + ah.bm + ah.bh   (smallest first)
// each exact in the fp32 accumulator's products, accumulated in fp32: the dropped terms
// (am.bl, al.bm, al.bl) are below 2^-24 |a||b|, the fp32 rounding of a single product -- an
// fp32 GEMM's accuracy at 6 bf16 MFMAs (192 cycles) per K = 16 instead of 8 fp32 MFMAs (512
// cycles).  The fused and the unfused node-MLP Linear1 (gine_mpmlp.hip matrix role,
// gine_mlp.hip row-tile GEMM) must agree bit for bit: both use these helpers with the same
// k permutation.
//
// Where it is used: every node-MLP product.  The row-tile GEMMs split the weights once per
// workgroup and the A fragment as it is read; the one-launch layers (gine_mpmlp.hip
// k_mp_fwd_layer, gine_mlpbwd.hip k_mlp_bwd_layer) have their A tiles split ONCE into LDS
// planes by the waves that produce them; the weight-gradient engines (gine_wgrad.hpp
// wgrad_body_x3, kMlpEngX3: stand-alone, beside the dz GEMM and inside the window backward)
// have each staged value split once by its stager into column-major planes.  (Round 3's
// engine forms that re-split per wave measured slower than the fp32 engine, profiles/
// r03_s12_*; the stager-split form replaced them in round 4, and round 5 moved the window
// backward's engine onto it too)
#pragma once

#include "gine_common.hpp"

// GINE_GEMM_BF16X3=0 (A/B builds: make fullvariant V=fp32gemm VDEFS=-DGINE_GEMM_BF16X3=0)
// keeps the fp32 chains everywhere.
#ifndef GINE_GEMM_BF16X3
#define GINE_GEMM_BF16X3 1
#endif

namespace gine {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

struct Bf16x3 {
  bf16x8_t h, m, l;
};

// (a, b) -> packed bf16 pair, round to nearest even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t bf16_pk(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

// the three planes of two values, as packed pairs
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = bf16_pk(a, b);
  const float ra = a - __builtin_bit_cast(float, h << 16);
  const float rb = b - __builtin_bit_cast(float, h & 0xffff0000u);
  m = bf16_pk(ra, rb);
  const float sa = ra - __builtin_bit_cast(float, m << 16);
  const float sb = rb - __builtin_bit_cast(float, m & 0xffff0000u);
  l = bf16_pk(sa, sb);
}

// eight consecutive k values (x: k 0-3, y: k 4-7) -> one MFMA fragment per plane
__device__ __forceinline__ Bf16x3 split8(float4 x, float4 y) {
  uint32_t h0, h1, h2, h3, m0, m1, m2, m3, l0, l1, l2, l3;
  split2(x.x, x.y, h0, m0, l0);
  split2(x.z, x.w, h1, m1, l1);
  split2(y.x, y.y, h2, m2, l2);
  split2(y.z, y.w, h3, m3, l3);
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  Bf16x3 r;
  r.h = __builtin_bit_cast(bf16x8_t, (u32x4_t){h0, h1, h2, h3});
  r.m = __builtin_bit_cast(bf16x8_t, (u32x4_t){m0, m1, m2, m3});
  r.l = __builtin_bit_cast(bf16x8_t, (u32x4_t){l0, l1, l2, l3});
  return r;
}

// acc += A.B over one K = 16 block (element j of lane half h: k = 8h + j of the block)
__device__ __forceinline__ f32x16_t mfma_bf16x3(const Bf16x3& a, const Bf16x3& b,
                                                f32x16_t acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, acc, 0, 0, 0);
  return acc;
}

// The exact fp32 form of the same product: acc += A.B over a lane half's KS k values
// (k = h*KS + s), v_mfma_f32_32x32x2_f32, one k per lane half and instruction.
template <int KS>
__device__ __forceinline__ f32x16_t mfma_f32_row(const float* arow, const float (&bf)[KS],
                                                 f32x16_t acc) {
#pragma unroll
  for (int q = 0; q < KS / 4; ++q) {
    const float4 a4 = *reinterpret_cast<const float4*>(&arow[4 * q]);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, bf[4 * q], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, bf[4 * q + 1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, bf[4 * q + 2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, bf[4 * q + 3], acc, 0, 0, 0);
  }
  return acc;
}

// The same with the B fragment read from memory, b[s] = wp[s * ws], four k per step and
// not unrolled: the rare-path form, which keeps its registers to a handful.
template <int KS>
__device__ __forceinline__ f32x16_t mfma_f32_row_mem(const float* arow, const float* wp,
                                                     int64_t ws, f32x16_t acc) {
#pragma unroll 1
  for (int q = 0; q < KS / 4; ++q) {
    const float4 a4 = *reinterpret_cast<const float4*>(&arow[4 * q]);
    const float* w = wp + (int64_t)(4 * q) * ws;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, w[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, w[ws], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, w[2 * ws], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, w[3 * ws], acc, 0, 0, 0);
  }
  return acc;
}

// Non-finite operands: the split of +-inf is (inf, inf - inf = NaN, ...), so a tile with an
// inf (or NaN) operand comes out NaN where the fp32 product gives +-inf.  Such a tile -- the
// wave sees a NaN in any lane's accumulator -- is redone by the fp32 chain from the same
// A fragment rows (still in LDS) and the fp32 weights (mfma_f32_row_mem), so non-finite values propagate
// exactly as in the fp32 GEMM (and in the reference).  Finite tiles never take the branch.
__device__ __forceinline__ bool wave_any_nan(const f32x16_t& acc) {
  bool bad = false;
#pragma unroll
  for (int i = 0; i < 16; ++i) bad = bad || (acc[i] != acc[i]);
  return __any(bad);
}

// The register-resident B operand of the row-tile GEMMs: a lane's KS fp32 weights
// (k = h*KS + s, s < KS: the lane half's contiguous k range) as KS/8 split fragments.
template <int KS>
struct BPlanes {
  Bf16x3 f[KS / 8];
  __device__ __forceinline__ void from(const float (&bf)[KS]) {
#pragma unroll
    for (int s = 0; s < KS / 8; ++s)
      f[s] = split8(make_float4(bf[8 * s], bf[8 * s + 1], bf[8 * s + 2], bf[8 * s + 3]),
                    make_float4(bf[8 * s + 4], bf[8 * s + 5], bf[8 * s + 6], bf[8 * s + 7]));
  }
};

}  // namespace gine
