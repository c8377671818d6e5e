// Folding rho[2] into dim_red for the folded dense chain (gine_chain.hip): the W' / b' /
// W'^T tiles, built by extra workgroups of whichever launch precedes the chain's use of
// them (the first chain kernel, or the DeepSet forward -- gine_deepset_fwd_fold), and the
// small K-split MFMA tile helpers the unfold kernel shares.
#pragma once

#include "gine_common.hpp"

namespace gine {

typedef float chf_floatx16 __attribute__((ext_vector_type(16)));

// W' = [Wdr_x | Wdr_e Wr1] into wfold ([D][F + D]), b' = Wdr_e br1 + bdr ([D]), W'^T
// ([F + D][D]) from the current weights
struct FoldArgs {
  const float *fw_r1, *fb_r1, *fw_dr, *fb_dr;
  float* wfold;
  int F;
};

// v = sum_j sA[r][j] * svec[j] for the 32 rows staged in sA (row stride D + 4): 2D/32
// threads per row, 16 products each, then a shuffle tree; every thread of row
// threadIdx.x / (2D/32) returns that row's total.
template <int D>
__device__ __forceinline__ float rows_dot(const float* sA, const float* svec) {
  constexpr int TPR = 2 * D / 32, LDA = D + 4, J = D / TPR;
  const int r = threadIdx.x / TPR, p = threadIdx.x % TPR;
  float v = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) v = fmaf(sA[r * LDA + p * J + j], svec[p * J + j], v);
#pragma unroll
  for (int o = TPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, TPR);
  return v;
}

// A [32 x 32] tile of a small D x D product, contraction split over the D/32 waves of a
// 2D-thread workgroup: wave w contracts k in [32w, 32w + 32) (lane half h: 16 of them) of
// the 32 A rows staged in sA against its B fragment bf[s] = B[32w + 16h + s][c32]; the
// partial tiles go to sR ([D/32][32 x 33], rows padded for transposed reads), to be summed by
// ksplit_sum after a barrier.
// 16 MFMAs per wave instead of a 64-long chain: these tiles are latency-bound.
__device__ __forceinline__ chf_floatx16 chf_zero16() {
  chf_floatx16 v;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = 0.f;
  return v;
}

constexpr int kSR = 32 * 33;  // floats of one wave's partial tile in sR
template <int D>
__device__ __forceinline__ void ksplit_tile(const float* sA, const float (&bf)[16], float* sR,
                                            int c32, int h) {
  constexpr int LDA = D + 4;
  const int w = threadIdx.x / kWave;
  chf_floatx16 acc = chf_zero16();
  const float* arow = sA + c32 * LDA + w * 32 + h * 16;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 a4 = *reinterpret_cast<const float4*>(&arow[4 * q]);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, bf[4 * q], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, bf[4 * q + 1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, bf[4 * q + 2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, bf[4 * q + 3], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
    sR[w * kSR + rr * 33 + c32] = acc[r];
  }
}
// element (row, col) of the tile (waves summed in order)
template <int D>
__device__ __forceinline__ float ksplit_sum(const float* sR, int row, int col) {
  float v = sR[row * 33 + col];
#pragma unroll
  for (int w = 1; w < D / 32; ++w) v += sR[w * kSR + row * 33 + col];
  return v;
}

// One [32 x 32] tile (rows k0, columns c0 of Wc) of W' = [Wdr_x | Wc], Wc = Wdr_e Wr1, and
// (c0 = 0) the x columns and b' = Wdr_e br1 + bdr of its rows: the folded chain's dim_red
// weight, written as W' [D][F+D], b' [D] and W'^T [F+D][D] (the forward kernel's B
// fragments read W'^T along rows, coalesced).  Run by the fold workgroups of F1.
template <int D>
__device__ void fold_tile(const FoldArgs& a, int ft, float* sA, float* sR, int c32, int h) {
  constexpr int NT = 2 * D, LDA = D + 4, T = D / 32;
  const int F = a.F, LW = a.F + D;
  const int k0 = 32 * (ft / T), c0 = 32 * (ft % T);
  const int w = threadIdx.x / kWave;
  __shared__ float svec[D];
  float bf[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) bf[s] = a.fw_r1[(size_t)(w * 32 + h * 16 + s) * D + c0 + c32];
  // every load of the staging issued before the first wait (unrolled, constant counts)
  constexpr int SI = 32 * D / NT, XI = 32 * 64 / NT;
  float st[SI], xv[XI];
#pragma unroll
  for (int i = 0; i < SI; ++i) {
    const int idx = threadIdx.x + i * NT, r = idx / D, j = idx % D;
    st[i] = a.fw_dr[(size_t)(k0 + r) * LW + F + j];
  }
  if (c0 == 0) {
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int idx = min(threadIdx.x + i * NT, 32 * F - 1), r = idx / F, c = idx % F;
      xv[i] = a.fw_dr[(size_t)(k0 + r) * LW + c];
    }
  }
  const float bv = threadIdx.x < D ? a.fb_r1[threadIdx.x] : 0.f;
  __syncthreads();  // every wave is done with sA / sB
#pragma unroll
  for (int i = 0; i < SI; ++i) {
    const int idx = threadIdx.x + i * NT;
    sA[(idx / D) * LDA + idx % D] = st[i];
  }
  float* wt = a.wfold + (size_t)D * LW + D;  // W'^T
  if (c0 == 0) {
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int idx = threadIdx.x + i * NT;
      if (idx < 32 * F) a.wfold[(size_t)(k0 + idx / F) * LW + idx % F] = xv[i];
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {  // x columns transposed: row r fastest
      const int idx = threadIdx.x + i * NT, r = idx % 32, c = idx / 32;
      if (idx < 32 * F) wt[(size_t)c * D + k0 + r] = a.fw_dr[(size_t)(k0 + r) * LW + c];
    }
  }
  if (threadIdx.x < D) svec[threadIdx.x] = bv;
  __syncthreads();
  ksplit_tile<D>(sA, bf, sR, c32, h);
  if (c0 == 0) {
    const float v = rows_dot<D>(sA, svec);  // (Wdr_e br1)[k0 + r]
    constexpr int TPR = NT / 32;
    if (threadIdx.x % TPR == 0) {
      const int r = threadIdx.x / TPR;
      a.wfold[(size_t)D * LW + k0 + r] = v + a.fb_dr[k0 + r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int o = threadIdx.x + i * NT;
    a.wfold[(size_t)(k0 + o / 32) * LW + F + c0 + o % 32] = ksplit_sum<D>(sR, o / 32, o % 32);
    wt[(size_t)(F + c0 + o / 32) * D + k0 + o % 32] = ksplit_sum<D>(sR, o % 32, o / 32);
  }
}

// The double fold (gine_chain_fwd_folded2): phi[2] is followed by rho[0] with no
// nonlinearity between them either (the member sum sits in between, and a Linear commutes
// with it), so  rho[0](s) = r Wf^T + bf  with  Wf = Wr0 Wp2,  bf = M Wr0 bp2 + br0.
// One [32 x 32] tile (rows k0, columns c0) of Wf into wfold2 ([D][D], then bf [D] by the
// tiles of column 0): A = Wr0's rows staged in sA, B = Wp2's columns.  Run by the second
// set of fold workgroups of gine_deepset_fwd_fold2.
struct Fold2Args {
  const float *w_r0, *b_r0, *w_p2, *b_p2;
  float members;
  float* wfold2;  // NULL: no double fold
};

template <int D>
__device__ void fold2_tile(const Fold2Args& a, int ft, float* sA, float* sR, int c32, int h) {
  constexpr int NT = 2 * D, LDA = D + 4, T = D / 32;
  const int k0 = 32 * (ft / T), c0 = 32 * (ft % T);
  const int w = threadIdx.x / kWave;
  __shared__ float svec2[D];
  float bf[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) bf[s] = a.w_p2[(size_t)(w * 32 + h * 16 + s) * D + c0 + c32];
  constexpr int SI = 32 * D / NT;
  float st[SI];
#pragma unroll
  for (int i = 0; i < SI; ++i) {
    const int idx = threadIdx.x + i * NT;
    st[i] = a.w_r0[(size_t)(k0 + idx / D) * D + idx % D];
  }
  const float bv = threadIdx.x < D ? a.b_p2[threadIdx.x] : 0.f;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < SI; ++i) {
    const int idx = threadIdx.x + i * NT;
    sA[(idx / D) * LDA + idx % D] = st[i];
  }
  if (threadIdx.x < D) svec2[threadIdx.x] = bv;
  __syncthreads();
  ksplit_tile<D>(sA, bf, sR, c32, h);
  if (c0 == 0) {
    const float v = rows_dot<D>(sA, svec2);  // (Wr0 bp2)[k0 + r]
    constexpr int TPR = NT / 32;
    if (threadIdx.x % TPR == 0) {
      const int r = threadIdx.x / TPR;
      a.wfold2[(size_t)D * D + k0 + r] = a.members * v + a.b_r0[k0 + r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int o = threadIdx.x + i * NT;
    a.wfold2[(size_t)(k0 + o / 32) * D + c0 + o % 32] = ksplit_sum<D>(sR, o / 32, o % 32);
  }
}

// F1 of the folded chain launches (D/32)^2 workgroups more than its chain grid: block
// chain_blocks + t folds tile t of W' beside the chain tiles (they fit on the CUs next to
// the one chain workgroup per CU).
template <int D>
constexpr int kFoldBlocks = (D / 32) * (D / 32);


}  // namespace gine
