// DeepSetEncoder phi, first layer + ReLU + member sum, fused (models/gnn.py:48-68):
//   r[n, :] = sum_m relu(ens[n, m, :] W1^T + b1)          ens [N, M, F], W1 [H, F]
// and its backward for the weights:
//   dh[n, m, :] = dr[n, :] * 1[ens[n, m, :] W1^T + b1 > 0]
//   dW1 = sum_{n,m} dh[n, m, :]^T ens[n, m, :],   db1 = sum_{n,m} dh[n, m, :]
// The reference materialises the [N, M, H] pre-activation (90 MB at the 24h_mixed
// benchmark shape) three times per step (Linear output, ReLU output, ReLU gradient).  Here
// it never leaves the MFMA accumulators: rows are (node, member) pairs, a workgroup walks
// groups of 32 nodes = M tiles of 32 rows; per tile the v_mfma_f32_32x32x2_f32 chain over
// the (padded) features yields the pre-activations of 32 rows x 32 hidden units per wave.
//  * forward: bias + ReLU in registers, member sums accumulated per node in LDS (fixed
//    order, deterministic);
//  * backward: the same chain is recomputed, masked with dr of the row's node, and the
//    masked accumulator registers are fed straight back as the A operand of the dW1 MFMA
//    (lane (c, h) holds rows (r&3)+8(r>>2)+4h of hidden unit c -- exactly a 32x32x2 A
//    fragment under a k-permutation that B, read from the staged ens tile, follows too).
#include "gine_common.hpp"

#include <algorithm>

namespace gine {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kNodes = 32;  // nodes per group; a group is exactly M tiles of 32 rows

__device__ __forceinline__ floatx16 zero16() {
  floatx16 v;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = 0.f;
  return v;
}

__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Stage rows [row0, row0+32) of ens (contiguous: 32*F floats) into s_e[32][KP+4], zero
// padded beyond F and beyond the valid rows.  `vals` is the register copy (prefetch).
template <int NT, int KP>
struct Stager {
  static constexpr int PER = (32 * 64 + NT - 1) / NT;  // >= 32*F / NT for F <= 64
  float vals[PER];
  __device__ __forceinline__ void load(const float* __restrict__ ens, int64_t row0,
                                       int64_t row_end, int F) {
    const int64_t base = row0 * F;
    const int64_t lim = (row_end > row0 ? (row_end - row0) : 0) * F;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + i * NT;
      const bool ok = e < 32 * F && e < lim;
      const float v = ens[base + (ok ? e : 0)];
      vals[i] = ok ? v : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* s_e, int F) const {
    constexpr int LD = KP + 4;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + i * NT;
      if (e < 32 * F) s_e[(e / F) * LD + e % F] = vals[i];
    }
  }
};

template <int KP>
__device__ __forceinline__ void zero_pad(float* s_e, int F) {
  constexpr int LD = KP + 4;
  for (int i = threadIdx.x; i < 32 * (LD - F); i += blockDim.x) {
    const int r = i / (LD - F), c = F + i % (LD - F);
    s_e[r * LD + c] = 0.f;
  }
}

// Pre-activation chain of one 32-row tile for this wave's 32 hidden units.
template <int KP>
__device__ __forceinline__ floatx16 pre_tile(const float* s_e, const float (&bf)[KP / 2],
                                             int c32, int h) {
  constexpr int LD = KP + 4;
  constexpr int KS = KP / 2;
  floatx16 acc = zero16();
  const float* arow = s_e + c32 * LD + h * KS;
#pragma unroll
  for (int q = 0; q < KS / 4; ++q) {
    const float4 a4 = *reinterpret_cast<const float4*>(arow + 4 * q);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, bf[4 * q], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, bf[4 * q + 1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, bf[4 * q + 2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, bf[4 * q + 3], acc, 0, 0, 0);
  }
  return acc;
}

template <int KP>
__device__ __forceinline__ void load_b(const float* __restrict__ w1, int col, int h, int F,
                                       float (&bf)[KP / 2]) {
  constexpr int KS = KP / 2;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = h * KS + s;
    bf[s] = k < F ? w1[(size_t)col * F + k] : 0.f;
  }
}

// groups of one XCD form a contiguous range walked by that XCD's workgroups
struct Range {
  int first, end, step;
};
__device__ __forceinline__ Range xcd_range(int n) {
  const int nb = gridDim.x;
  const int xcd = blockIdx.x % kNumXcd, pos = blockIdx.x / kNumXcd;
  const int here = nb / kNumXcd + (xcd < nb % kNumXcd ? 1 : 0);
  const int span = (n + kNumXcd - 1) / kNumXcd;
  return Range{xcd * span + pos, min(n, xcd * span + span), here};
}

// ---------------------------------------------------------------------------------------
template <int H, int KP>
__global__ __launch_bounds__(2 * H) void k_deepset_fwd(const float* __restrict__ ens,
                                                       const float* __restrict__ w1,
                                                       const float* __restrict__ b1,
                                                       float* __restrict__ r, int64_t N,
                                                       int M, int F, int num_groups) {
  constexpr int NT = 2 * H;
  __shared__ __attribute__((aligned(16))) float s_e[32 * (KP + 4)];
  __shared__ float s_sum[kNodes * H];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  float bf[KP / 2];
  load_b<KP>(w1, col, h, F, bf);
  const float bias = b1[col];
  zero_pad<KP>(s_e, F);

  const int64_t rows_total = N * M;
  Stager<NT, KP> st;
  const Range rg = xcd_range(num_groups);
  if (rg.first < rg.end) st.load(ens, (int64_t)rg.first * kNodes * M, rows_total, F);
  for (int g = rg.first; g < rg.end; g += rg.step) {
    const int64_t node0 = (int64_t)g * kNodes;
    const int64_t row_base = node0 * M;
    for (int i = lane; i < kNodes * 32; i += kWave)  // this wave's 32 columns
      s_sum[(i >> 5) * H + wave * 32 + (i & 31)] = 0.f;
    for (int t = 0; t < M; ++t) {
      const int64_t row0 = row_base + 32 * t;
      __syncthreads();
      st.store(s_e, F);
      __syncthreads();
      // prefetch the next tile (of this group, or the first of the next group)
      if (t + 1 < M) st.load(ens, row0 + 32, rows_total, F);
      else if (g + rg.step < rg.end)
        st.load(ens, (int64_t)(g + rg.step) * kNodes * M, rows_total, F);
      const floatx16 acc = pre_tile<KP>(s_e, bf, c32, h);
      // member sums: the two lane halves in turn (they can share a node), rows in order
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if (h == hh) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int64_t row = row0 + acc_row(q, h);
            if (row < rows_total) {
              const int slot = (int)(row / M - node0);
              const float v = relu_nan(acc[q] + bias);
              s_sum[slot * H + col] += v;
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    for (int i = lane; i < kNodes * 32; i += kWave) {
      const int64_t n = node0 + (i >> 5);
      const int c = wave * 32 + (i & 31);
      if (n < N) r[n * H + c] = s_sum[(i >> 5) * H + c];
    }
  }
}

// ---------------------------------------------------------------------------------------
template <int H, int KP>
__global__ __launch_bounds__(2 * H) void k_deepset_bwd(const float* __restrict__ ens,
                                                       const float* __restrict__ w1,
                                                       const float* __restrict__ b1,
                                                       const float* __restrict__ dr,
                                                       float* __restrict__ slab, int64_t N,
                                                       int M, int F, int num_groups) {
  constexpr int NT = 2 * H;
  constexpr int LD = KP + 4;
  constexpr int NI = (KP + 31) / 32;  // 32-wide feature tiles of dW1
  __shared__ __attribute__((aligned(16))) float s_e[32 * LD];
  __shared__ float s_dr[kNodes * H];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  float bf[KP / 2];
  load_b<KP>(w1, col, h, F, bf);
  const float bias = b1[col];
  zero_pad<KP>(s_e, F);

  floatx16 gw[NI];
#pragma unroll
  for (int it = 0; it < NI; ++it) gw[it] = zero16();
  double gb = 0.0;

  const int64_t rows_total = N * M;
  Stager<NT, KP> st;
  const Range rg = xcd_range(num_groups);
  if (rg.first < rg.end) st.load(ens, (int64_t)rg.first * kNodes * M, rows_total, F);
  for (int g = rg.first; g < rg.end; g += rg.step) {
    const int64_t node0 = (int64_t)g * kNodes;
    const int64_t row_base = node0 * M;
    for (int i = lane; i < kNodes * 32; i += kWave) {  // dr of this group, own columns
      const int64_t n = node0 + (i >> 5);
      const int c = wave * 32 + (i & 31);
      s_dr[(i >> 5) * H + c] = n < N ? dr[n * H + c] : 0.f;
    }
    for (int t = 0; t < M; ++t) {
      const int64_t row0 = row_base + 32 * t;
      __syncthreads();
      st.store(s_e, F);
      __syncthreads();
      if (t + 1 < M) st.load(ens, row0 + 32, rows_total, F);
      else if (g + rg.step < rg.end)
        st.load(ens, (int64_t)(g + rg.step) * kNodes * M, rows_total, F);
      floatx16 dh = pre_tile<KP>(s_e, bf, c32, h);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = row0 + acc_row(q, h);
        float v = 0.f;
        if (row < rows_total) {
          const int slot = (int)(row / M - node0);
          v = (dh[q] + bias > 0.f) ? s_dr[slot * H + col] : 0.f;  // ReLU backward
        }
        dh[q] = v;
        gb += (double)v;
      }
      // dW1[o][i] += sum_rows dh[row][o] ens[row][i]: A = dh (registers), B = staged ens
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float* erow = s_e + acc_row(q, h) * LD;
#pragma unroll
        for (int it = 0; it < NI; ++it) {
          const int i = 32 * it + c32;
          const float b = i < KP ? erow[i] : 0.f;
          gw[it] = __builtin_amdgcn_mfma_f32_32x32x2f32(dh[q], b, gw[it], 0, 0, 0);
        }
      }
    }
  }
  // slab row of this workgroup: [H*F weights | H bias]
  float* out = slab + (size_t)blockIdx.x * ((size_t)H * F + H);
#pragma unroll
  for (int it = 0; it < NI; ++it) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int o = wave * 32 + acc_row(q, h);
      const int i = 32 * it + c32;
      if (i < F) out[(size_t)o * F + i] = gw[it][q];
    }
  }
  gb += shfl_xor_d(gb, 32);
  if (h == 0) out[(size_t)H * F + col] = (float)gb;
}

__global__ __launch_bounds__(256) void k_deepset_slab_reduce(const float* __restrict__ slab,
                                                             int chunks, int64_t per,
                                                             int64_t wsize,
                                                             float* __restrict__ dw,
                                                             float* __restrict__ db) {
  __shared__ double s_part[4][64];
  const int64_t e = blockIdx.x * (int64_t)64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  double acc = 0.0;
  if (e < per) {
    for (int c = g; c < chunks; c += 4) acc += (double)slab[(size_t)c * per + e];
  }
  s_part[g][threadIdx.x & 63] = acc;
  __syncthreads();
  if (g != 0 || e >= per) return;
  const int j = threadIdx.x & 63;
  const float v = (float)((s_part[0][j] + s_part[1][j]) + (s_part[2][j] + s_part[3][j]));
  if (e < wsize) dw[e] = v;
  else if (db) db[e - wsize] = v;
}

inline int pad_features(int F) {
  if (F <= 16) return 16;
  if (F <= 32) return 32;
  if (F <= 40) return 40;
  if (F <= 48) return 48;
  if (F <= 64) return 64;
  return -1;
}

inline bool hidden_ok(int H) { return H == 32 || H == 64 || H == 128 || H == 256; }

inline int bwd_grid(int64_t N) {
  const int64_t groups = ceil_div(N > 0 ? N : 1, kNodes);
  return (int)std::min<int64_t>(groups, 256);
}

#define DS_DISPATCH(H_, KP_, MACRO)                       \
  switch (KP_) {                                          \
    case 16: MACRO(H_, 16); break;                        \
    case 32: MACRO(H_, 32); break;                        \
    case 40: MACRO(H_, 40); break;                        \
    case 48: MACRO(H_, 48); break;                        \
    default: MACRO(H_, 64); break;                        \
  }

#define DS_DISPATCH_H(H, KP, MACRO)                       \
  switch (H) {                                            \
    case 32: DS_DISPATCH(32, KP, MACRO); break;           \
    case 64: DS_DISPATCH(64, KP, MACRO); break;           \
    case 128: DS_DISPATCH(128, KP, MACRO); break;         \
    default: DS_DISPATCH(256, KP, MACRO); break;          \
  }

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_deepset_fwd(const float* ens, const float* w1, const float* b1, float* r,
                                int64_t num_nodes, int32_t members, int32_t in_features,
                                int32_t hidden, void* stream) {
  const int KP = pad_features(in_features);
  if (!hidden_ok(hidden) || KP < 0 || in_features <= 0) return GINE_ERR_DIM;
  if (num_nodes < 0 || members <= 0) return GINE_ERR_INVALID;
  if (num_nodes == 0) return GINE_OK;
  if (!ens || !w1 || !b1 || !r) return GINE_ERR_INVALID;
  if (num_nodes * members >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  const int groups = (int)ceil_div(num_nodes, kNodes);
  const int grid = std::min(groups, 1024);
  hipStream_t s = as_stream(stream);
#define LAUNCH_FWD(H_, KP_)                                                                 \
  hipLaunchKernelGGL((k_deepset_fwd<H_, KP_>), dim3(grid), dim3(2 * H_), 0, s, ens, w1, b1, \
                     r, num_nodes, members, in_features, groups)
  DS_DISPATCH_H(hidden, KP, LAUNCH_FWD);
#undef LAUNCH_FWD
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_deepset_bwd_num_partials(int64_t num_nodes, int32_t* num_partials) {
  if (!num_partials || num_nodes < 0) return GINE_ERR_INVALID;
  *num_partials = bwd_grid(num_nodes);
  return GINE_OK;
}

extern "C" int gine_deepset_bwd(const float* ens, const float* w1, const float* b1,
                                const float* dr, float* slab, float* dw1, float* db1,
                                int64_t num_nodes, int32_t members, int32_t in_features,
                                int32_t hidden, void* stream) {
  const int KP = pad_features(in_features);
  if (!hidden_ok(hidden) || KP < 0 || in_features <= 0) return GINE_ERR_DIM;
  if (num_nodes < 0 || members <= 0 || !slab || !dw1) return GINE_ERR_INVALID;
  if (num_nodes > 0 && (!ens || !w1 || !b1 || !dr)) return GINE_ERR_INVALID;
  if (num_nodes * members >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  const int groups = (int)ceil_div(num_nodes > 0 ? num_nodes : 1, kNodes);
  const int grid = bwd_grid(num_nodes);
  const int64_t per = (int64_t)hidden * in_features + hidden;
  hipStream_t s = as_stream(stream);
  if (num_nodes == 0) {
    GINE_RETURN_IF_HIP(hipMemsetAsync(slab, 0, sizeof(float) * per * grid, s));
  } else {
#define LAUNCH_BWD(H_, KP_)                                                                 \
  hipLaunchKernelGGL((k_deepset_bwd<H_, KP_>), dim3(grid), dim3(2 * H_), 0, s, ens, w1, b1, \
                     dr, slab, num_nodes, members, in_features, groups)
    DS_DISPATCH_H(hidden, KP, LAUNCH_BWD);
#undef LAUNCH_BWD
    GINE_LAUNCH_STATUS();
  }
  hipLaunchKernelGGL(k_deepset_slab_reduce, dim3((unsigned)ceil_div(per, 64)), dim3(256), 0, s,
                     slab, grid, per, (int64_t)hidden * in_features, dw1, db1);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
