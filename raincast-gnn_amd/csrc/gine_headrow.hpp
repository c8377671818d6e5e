// Output-head pieces shared by the head kernels (gine_head.hip) and the CRPS pass that runs
// the head backward for a unit loss seed (gine_loss.hip): the PostProcess column roles and
// derivatives (models/model_utils.py:70-113 and ATen's softplus / sigmoid backward), and the
// row-streaming backward of one node row: one 32-lane half-wave per node, lane t holding
// float4 columns t, t+32 of h / dh, workgroup partials of dW and db.
#pragma once

#include "gine_common.hpp"

namespace gine {
namespace head {

constexpr int kThreads = 256;                  // head kernels
constexpr int kRowsPerBlock = kThreads / 32;  // one node per half-wave
constexpr int kMaxK = 5;
constexpr int kMaxChunks = 2;                  // D <= 256: two float4 per lane
constexpr int kHeadBlocks = 256;               // backward grid (partials = one slab row each)

// sum_32(a): the butterfly `for m = 16, 8, 4, 2, 1: a += __shfl_xor(a, m, 32)` with the same
// partner, order and rounding at every lane (so the same bits), on VALU lane exchanges
// instead of LDS-crossbar ds_bpermute round trips: xor 16 by v_permlane16_swap (odd and even
// 16-lane rows of a half-wave exchanged), xor 8 by DPP row_ror:8, xor 4 by DPP row_half_mirror
// (lane ^ 7) then quad_perm [3,2,1,0] (lane ^ 3), xor 2 / xor 1 by quad_perm.  Every partner
// stays inside the lane's half-wave (a half-wave whose row is past N is inactive as a whole).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// the value of lane ^ 16 (v_permlane16_swap of v with itself: lanes 0-15 of the pair's first
// result hold their own values, lanes 16-31 lanes 0-15's; the second result the other way)
__device__ __forceinline__ float xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float sum_32(float a) {
  a += xor16(a);
  a += dpp_mov<0x128>(a);                     // row_ror:8       lane ^ 8
  a += dpp_mov<0x1B>(dpp_mov<0x141>(a));      // half_mirror, quad_perm [3,2,1,0]: lane ^ 4
  a += dpp_mov<0x4E>(a);                      // quad_perm [2,3,0,1]: lane ^ 2
  a += dpp_mov<0xB1>(a);                      // quad_perm [1,0,3,2]: lane ^ 1
  return a;
}

// The half-wave sums of four outputs a0..a3 at once, reduce-scattered: at xor 16 each lane
// keeps the pair of outputs of its half of the half-wave ({0,1} for lanes 0-15, {2,3} for
// 16-31) and receives its partner's values of that pair, at xor 8 it keeps one output
// ((lane >> 3) & 3) and receives the partner's, then xor 4 / 2 / 1 sum the eight lanes of that
// output.  Returns output ((lane >> 3) & 3)'s total, the same bits at all eight lanes of the
// group (every step adds own + partner, and float addition commutes).  6 lane exchanges for
// four outputs against 20 for four sum_32.  Every sum is own value + partner's, the same
// order in the head kernel and in the layer epilogue that folds it (gine_mpmlp.hip).
__device__ __forceinline__ float sum4_32(float a0, float a1, float a2, float a3) {
  const bool b4 = threadIdx.x & 16, b3 = threadIdx.x & 8;
  const float r0 = xor16(b4 ? a0 : a2), r1 = xor16(b4 ? a1 : a3);
  const float c0 = (b4 ? a2 : a0) + r0, c1 = (b4 ? a3 : a1) + r1;
  float d = (b3 ? c1 : c0) + dpp_mov<0x128>(b3 ? c0 : c1);  // lane ^ 8
  d += dpp_mov<0x1B>(dpp_mov<0x141>(d));                     // lane ^ 4
  d += dpp_mov<0x4E>(d);                                     // lane ^ 2
  d += dpp_mov<0xB1>(d);                                     // lane ^ 1
  return d;
}

// Column roles of the K outputs for each loss (models/model_utils.py:80-111).
enum Role { R_ID = 0, R_SOFTPLUS = 1, R_SIGMOID = 2, R_SIGMOID_U = 3 };

__device__ __forceinline__ int role_of(int kind, int k) {
  if (k == 0) return R_ID;                              // mu
  if (k == 1 || k == 3) return R_SOFTPLUS;              // sigma, sigma_u
  if (k == 2) return R_SIGMOID;                         // p
  return kind == GINE_LOSS_MIXED_U ? R_SIGMOID_U : R_ID;  // u (learned threshold)
}

// torch.nn.functional.softplus(beta=1, threshold=20)
__device__ __forceinline__ float softplus_f(float x) {
  return x > 20.f ? x : log1pf(expf(x));
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ float post(int role, float x) {
  switch (role) {
    case R_SOFTPLUS: return softplus_f(x) + 1e-6f;
    case R_SIGMOID: return sigmoid_f(x);
    case R_SIGMOID_U: return sigmoid_f(x) * 2.12f;
    default: return x;
  }
}

// d post / d x applied to g (ATen: softplus_backward z = exp(x), g*z/(z+1) below the
// threshold; sigmoid_backward g*(1-s)*s from the output s)
__device__ __forceinline__ float post_bwd(int role, float x, float g) {
  switch (role) {
    case R_SOFTPLUS: {
      if (x > 20.f) return g;
      const float z = expf(x);
      return g * z / (z + 1.f);
    }
    case R_SIGMOID: {
      const float s = sigmoid_f(x);
      return g * (1.f - s) * s;
    }
    case R_SIGMOID_U: {
      const float s = sigmoid_f(x);
      return (g * 2.12f) * (1.f - s) * s;
    }
    default: return g;
  }
}

// The slab row of a workgroup: LDS partial rows [0, rows) summed in fixed order (fp64), by
// all kThreads threads (after the __syncthreads that published the rows).
template <int K>
__device__ __forceinline__ void reduce_rows(float* __restrict__ out, int D,
                                            const float (*s_part)[kMaxK * 256 + kMaxK],
                                            int rows) {
  const int per = K * D + K;
  for (int e = threadIdx.x; e < per; e += kThreads) {
    double s = 0.0;
    for (int r = 0; r < rows; ++r) s += (double)s_part[r][e];
    out[e] = (float)s;
  }
}

// One workgroup's share of the head backward: half-wave hw takes the nodes n = first + hw +
// stride j (n < N), U rows per batch of loads; d raw = graw(n) [K floats] -> dh[n] = d raw W
// (written), and the K x D dW / K db partials of these nodes, summed over the 8 half-waves
// in fixed order (fp64) into the slab row `out` (K*D + K floats).  256 threads; s_part:
// kRowsPerBlock * (kMaxK*256 + kMaxK) floats of LDS.  load() issues a batch's row loads and
// step() consumes them, so a caller can put other work between the two (the CRPS pass
// evaluates the loss while its rows arrive).  C: float4 column chunks per lane (1 when
// D <= 128; the registers of a second chunk are not held for nothing).
template <int K, int U, int C = kMaxChunks>
struct HeadRows {
  static_assert(C >= 1 && C <= kMaxChunks, "column chunks per lane");
  float4 wk[C][K];
  float4 aw[C][K];  // sum over this half-wave's nodes of d raw[k] * h[n, cols]
  float ab[K];
  float4 x[U][C];
  int t, hw, D4;

  __device__ __forceinline__ void init(const float* __restrict__ w, int D) {
    t = threadIdx.x & 31;
    hw = threadIdx.x / 32;
    D4 = D / 4;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      ab[k] = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) aw[c][k] = f4_zero();
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int q = min(t + 32 * c, D4 - 1);
#pragma unroll
      for (int k = 0; k < K; ++k)
        wk[c][k] = reinterpret_cast<const float4*>(w + (size_t)k * D)[q];
    }
  }
  // the h rows n0 + u*stride (u < U) of this half-wave
  __device__ __forceinline__ void load(int64_t n0, int64_t stride, int64_t N,
                                       const float* __restrict__ h, int D) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t n = n0 + u * stride;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const int q = t + 32 * c;
        x[u][c] = (n < N && q < D4) ? reinterpret_cast<const float4*>(h + n * D)[q] : f4_zero();
      }
    }
  }
  template <class GRaw>
  __device__ __forceinline__ void step(GRaw&& graw, int64_t n0, int64_t stride, int64_t N,
                                       float* __restrict__ dh, int D) {
    float g[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t n = n0 + u * stride;
      if (n < N) {
        graw(n, g[u]);
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) g[u][k] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t n = n0 + u * stride;
      if (n >= N) break;
#pragma unroll
      for (int k = 0; k < K; ++k) ab[k] += g[u][k];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const int q = t + 32 * c;
        if (q < D4) {
          float4 o = f4_zero();
#pragma unroll
          for (int k = 0; k < K; ++k) {
            o.x = __builtin_fmaf(g[u][k], wk[c][k].x, o.x);
            o.y = __builtin_fmaf(g[u][k], wk[c][k].y, o.y);
            o.z = __builtin_fmaf(g[u][k], wk[c][k].z, o.z);
            o.w = __builtin_fmaf(g[u][k], wk[c][k].w, o.w);
            aw[c][k].x = __builtin_fmaf(g[u][k], x[u][c].x, aw[c][k].x);
            aw[c][k].y = __builtin_fmaf(g[u][k], x[u][c].y, aw[c][k].y);
            aw[c][k].z = __builtin_fmaf(g[u][k], x[u][c].z, aw[c][k].z);
            aw[c][k].w = __builtin_fmaf(g[u][k], x[u][c].w, aw[c][k].w);
          }
          reinterpret_cast<float4*>(dh + n * D)[q] = o;
        }
      }
    }
  }
  // this half-wave's partial into LDS row `row`
  __device__ __forceinline__ void put(float (*s_part)[kMaxK * 256 + kMaxK], int row, int D) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int q = t + 32 * c;
      if (q < D4) {
#pragma unroll
        for (int k = 0; k < K; ++k)
          *reinterpret_cast<float4*>(&s_part[row][k * D + 4 * q]) = aw[c][k];
      }
    }
    if (t < K) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) v = (t == k) ? ab[k] : v;
      s_part[row][K * D + t] = v;
    }
  }
  // workgroup partial: the 8 half-waves summed in fixed order (fp64) -> one slab row
  __device__ __forceinline__ void flush(float* __restrict__ out, int D,
                                        float (*s_part)[kMaxK * 256 + kMaxK]) {
    put(s_part, hw, D);
    __syncthreads();
    reduce_rows<K>(out, D, s_part, kRowsPerBlock);
  }
};

// The whole share in batches of U rows (gine_head_bwd).
template <int K, int U, class GRaw>
__device__ __forceinline__ void bwd_rows(GRaw&& graw, int64_t first, int64_t stride, int64_t N,
                                         const float* __restrict__ h,
                                         const float* __restrict__ w, float* __restrict__ dh,
                                         float* __restrict__ out, int D,
                                         float (*s_part)[kMaxK * 256 + kMaxK]) {
  HeadRows<K, U> r;
  r.init(w, D);
  for (int64_t n0 = first + r.hw; n0 < N; n0 += U * stride) {
    r.load(n0, stride, N, h, D);
    r.step(graw, n0, stride, N, dh, D);
  }
  r.flush(out, D, s_part);
}

}  // namespace head
}  // namespace gine
