// DeepSetEncoder phi, first layer + ReLU + member sum, fused (models/gnn.py:48-68):
//   r[n, :] = sum_m relu(ens[n, m, :] W1^T + b1)          ens [N, M, F], W1 [H, F]
// and its backward for the weights:
//   dh[n, m, :] = dr[n, :] * 1[ens[n, m, :] W1^T + b1 > 0]
//   dW1 = sum_{n,m} dh[n, m, :]^T ens[n, m, :],   db1 = sum_{n,m} dh[n, m, :]
// The reference materialises the [N, M, H] pre-activation (90 MB at the 24h_mixed
// benchmark shape) three times per step (Linear output, ReLU output, ReLU gradient).  Here
// it never leaves the MFMA accumulators.  Rows are (node, member) pairs; a workgroup walks
// groups of 32 nodes = 32*M rows as M tiles of 32 rows, and each wave owns 32 hidden units.
// Row placement: the accumulator register q of lane half h (v_mfma_f32_32x32x2_f32 output
// row (q&3)+8(q>>2)+4h) holds group row 16*M*h + 16*t + q in tile t, i.e. half 0 walks the
// rows of nodes 0-15 and half 1 those of nodes 16-31, both in member order.  So
//  * forward: bias + ReLU in registers and a running per-node sum per lane, written once
//    when the node changes (wave-uniform: both halves are at the same local row) -- no
//    LDS read-modify-write, deterministic member order;
//  * backward: the chain is recomputed, masked with dr of the row's node, and the masked
//    accumulator registers are fed straight back as the A operand of the dW1 MFMA (a lane
//    half's 16 registers are 16 distinct k of a 32x32x2 A fragment under a k-permutation
//    that B -- read from the staged ens rows 16h+q -- follows too).
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

// LDS row holding MFMA output row i (see the row placement above): 16*h + q.
__device__ __forceinline__ int staged_row(int i) {
  return 16 * ((i >> 2) & 1) + (i & 3) + 4 * (i >> 3);
}

// Tile t of a group stages, into an LDS tile [32][KP+4], rows 16c+j <- group row
// 16*M*c + 16*t + j (c = lane half, j < 16): two contiguous runs of 16*F floats.  Offsets
// depend only on the thread, so they are computed once.
template <int NT, int KP>
struct Stager {
  static constexpr int PER = (32 * KP + NT - 1) / NT;  // >= 32*F / NT
  static constexpr int LD = KP + 4;
  int src[PER];  // float offset from the tile's first row; -1: thread has no element
  int row[PER];  // group-row offset from the tile's first row
  int dst[PER];  // LDS offset
  __device__ __forceinline__ void init(int F, int M) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + i * NT;
      const int c = e >= 16 * F ? 1 : 0;
      const int off = e - c * 16 * F;
      const int j = off / F, f = off - j * F;
      const bool has = e < 32 * F;
      src[i] = has ? c * 16 * M * F + off : -1;
      row[i] = c * 16 * M + j;
      dst[i] = has ? (16 * c + j) * LD + f : -1;
    }
  }
  // row0: first group row of the tile (group base + 16 t)
  __device__ __forceinline__ void load(float (&v)[PER], const float* __restrict__ ens,
                                       int64_t row0, int64_t rows_total, int F) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const bool ok = src[i] >= 0 && row0 + row[i] < rows_total;
      const float x = ens[ok ? row0 * F + src[i] : 0];  // clamped: every lane loads
      v[i] = ok ? x : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* s_e, const float (&v)[PER]) const {
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (dst[i] >= 0) s_e[dst[i]] = v[i];
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
  const float* arow = s_e + staged_row(c32) * LD + h * KS;
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

// node (within a lane half's 16) of half-local row l < 16*M: exact for M < 2^16 (the
// fractional part of (l + 0.5)/M is at least 0.5/M from an integer)
__device__ __forceinline__ int node_of(int l, float inv_m) {
  return (int)(((float)l + 0.5f) * inv_m);
}

// The tiles of this workgroup: groups first, first+step, ... < end (one XCD's groups form a
// contiguous range walked by that XCD's workgroups), M tiles each, as one flat sequence so
// that loads run two tiles ahead across group boundaries.
struct Tiles {
  int first, step, M, count;
  __device__ __forceinline__ Tiles(int num_groups, int M_) : M(M_) {
    const int nb = gridDim.x;
    const int xcd = blockIdx.x % kNumXcd, pos = blockIdx.x / kNumXcd;
    const int here = nb / kNumXcd + (xcd < nb % kNumXcd ? 1 : 0);
    const int span = (num_groups + kNumXcd - 1) / kNumXcd;
    const int end = min(num_groups, xcd * span + span);
    first = xcd * span + pos;
    step = here;
    count = first < end ? ((end - first + step - 1) / step) * M : 0;
  }
  __device__ __forceinline__ int group(int k) const { return first + (k / M) * step; }
  __device__ __forceinline__ int64_t row0(int k) const {  // first group row of tile k
    const int gi = k / M;
    return (int64_t)(first + gi * step) * kNodes * M + 16 * (k - gi * M);
  }
};

// Drive `tile(k, buf)` over the workgroup's tiles with a two-deep register ring and a
// double-buffered LDS tile: tile k+2 is loaded while tile k computes, tile k+1 is stored
// after it, one barrier per tile.
template <int NT, int KP, class Body>
__device__ __forceinline__ void walk_tiles(const Tiles& tl, const Stager<NT, KP>& st,
                                           const float* __restrict__ ens, int64_t rows_total,
                                           int F, float* buf0, float* buf1, Body&& tile) {
  constexpr int PER = Stager<NT, KP>::PER;
  float va[PER], vb[PER];
  if (tl.count > 0) {
    st.load(va, ens, tl.row0(0), rows_total, F);
    st.store(buf0, va);
  }
  if (tl.count > 1) st.load(vb, ens, tl.row0(1), rows_total, F);
  __syncthreads();
  auto step = [&](int k, float (&cur)[PER], float (&nxt)[PER], float* bcur, float* bnxt) {
    if (k + 2 < tl.count) st.load(cur, ens, tl.row0(k + 2), rows_total, F);
    tile(k, bcur);
    if (k + 1 < tl.count) st.store(bnxt, nxt);
    __syncthreads();
  };
  for (int k = 0; k < tl.count; k += 2) {
    step(k, va, vb, buf0, buf1);
    if (k + 1 < tl.count) step(k + 1, vb, va, buf1, buf0);
  }
}

// ---------------------------------------------------------------------------------------
template <int H, int KP>
__global__ __launch_bounds__(2 * H) void k_deepset_fwd(const float* __restrict__ ens,
                                                       const float* __restrict__ w1,
                                                       const float* __restrict__ b1,
                                                       float* __restrict__ r, int64_t N,
                                                       int M, int F, int num_groups) {
  constexpr int NT = 2 * H;
  constexpr int LD = KP + 4;
  __shared__ __attribute__((aligned(16))) float s_e[2][32 * LD];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  const float inv_m = 1.f / (float)M;
  float bf[KP / 2];
  load_b<KP>(w1, col, h, F, bf);
  const float bias = b1[col];
  zero_pad<KP>(s_e[0], F);
  zero_pad<KP>(s_e[1], F);

  Stager<NT, KP> st;
  st.init(F, M);
  const Tiles tl(num_groups, M);
  int cur = 0;
  float run = 0.f;
  walk_tiles(tl, st, ens, N * M, F, s_e[0], s_e[1], [&](int k, const float* buf) {
    const int gi = k / M, t = k - gi * M;
    const int64_t my_node0 = (int64_t)(tl.first + gi * tl.step) * kNodes + 16 * h;
    const floatx16 acc = pre_tile<KP>(buf, bf, c32, h);
    if (t == 0) {
      cur = 0;
      run = 0.f;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int node = node_of(16 * t + q, inv_m);  // wave-uniform
      if (node != cur) {
        if (my_node0 + cur < N) r[(my_node0 + cur) * H + col] = run;
        cur = node;
        run = 0.f;
      }
      run += relu_nan(acc[q] + bias);
    }
    if (t == M - 1 && my_node0 + cur < N) r[(my_node0 + cur) * H + col] = run;
  });
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
  __shared__ __attribute__((aligned(16))) float s_e[2][32 * LD];
  __shared__ float s_dr[kNodes * H];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  const float inv_m = 1.f / (float)M;
  float bf[KP / 2];
  load_b<KP>(w1, col, h, F, bf);
  const float bias = b1[col];
  zero_pad<KP>(s_e[0], F);
  zero_pad<KP>(s_e[1], F);

  floatx16 gw[NI];
#pragma unroll
  for (int it = 0; it < NI; ++it) gw[it] = zero16();
  double gb = 0.0;

  Stager<NT, KP> st;
  st.init(F, M);
  const Tiles tl(num_groups, M);
  walk_tiles(tl, st, ens, N * M, F, s_e[0], s_e[1], [&](int k, const float* buf) {
    const int gi = k / M, t = k - gi * M;
    if (t == 0) {  // dr of this group, this wave's columns (read by this wave only)
      const int64_t node0 = (int64_t)(tl.first + gi * tl.step) * kNodes;
      for (int i = lane; i < kNodes * 32; i += kWave) {
        const int64_t n = node0 + (i >> 5);
        const int c = wave * 32 + (i & 31);
        s_dr[(i >> 5) * H + c] = n < N ? dr[n * H + c] : 0.f;
      }
    }
    floatx16 dh = pre_tile<KP>(buf, bf, c32, h);
#pragma unroll
    for (int q = 0; q < 16; ++q) {  // independent LDS reads: no branch on the node change
      const float d = s_dr[(16 * h + node_of(16 * t + q, inv_m)) * H + col];  // 0 if >= N
      const float v = (dh[q] + bias > 0.f) ? d : 0.f;  // ReLU backward
      dh[q] = v;
      gb += (double)v;
    }
    // dW1[o][i] += sum_rows dh[row][o] ens[row][i]: A = dh (registers), B = staged rows
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float* erow = buf + (16 * h + q) * LD;
#pragma unroll
      for (int it = 0; it < NI; ++it) {
        const int i = 32 * it + c32;
        const float b = (32 * it + 32 <= KP || i < KP) ? erow[i] : 0.f;
        gw[it] = __builtin_amdgcn_mfma_f32_32x32x2f32(dh[q], b, gw[it], 0, 0, 0);
      }
    }
  });
  // slab row of this workgroup: [H*F weights | H bias]
  float* out = slab + (size_t)blockIdx.x * ((size_t)H * F + H);
#pragma unroll
  for (int it = 0; it < NI; ++it) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int o = wave * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
      const int i = 32 * it + c32;
      if (i < F) out[(size_t)o * F + i] = gw[it][q];
    }
  }
  gb += shfl_xor_d(gb, 32);
  if (h == 0) out[(size_t)H * F + col] = (float)gb;
}

// 16 consecutive slab elements x 16 chunk groups per workgroup (many workgroups for the
// few thousand elements of dW1), fixed summation order, fp64.
__global__ __launch_bounds__(256) void k_deepset_slab_reduce(const float* __restrict__ slab,
                                                             int chunks, int64_t per,
                                                             int64_t wsize,
                                                             float* __restrict__ dw,
                                                             float* __restrict__ db) {
  __shared__ double s_part[16][17];
  const int j = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t e = blockIdx.x * (int64_t)16 + j;
  double acc = 0.0;
  if (e < per) {
#pragma unroll 4
    for (int c = g; c < chunks; c += 16) acc += (double)slab[(size_t)c * per + e];
  }
  s_part[g][j] = acc;
  __syncthreads();
  if (g != 0 || e >= per) return;
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) v += s_part[k][j];
  if (e < wsize) dw[e] = (float)v;
  else if (db) db[e - wsize] = (float)v;
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
  return (int)std::min<int64_t>(groups, 512);
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
  hipLaunchKernelGGL(k_deepset_slab_reduce, dim3((unsigned)ceil_div(per, 16)), dim3(256), 0, s,
                     slab, grid, per, (int64_t)hidden * in_features, dw1, db1);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
