// GINEConv message passing on gfx950: gather -> edge-MLP -> deterministic scatter-add.
//
// Replaces (torch_geometric, called from models/gnn.py:41,44):
//   x_j = x.index_select(0, edge_index[0])                 MessagePassing._collect
//   m   = (x_j + Linear(1,D)(edge_attr)).relu()            GINEConv.message
//   agg = zeros(N,D).scatter_add_(0, edge_index[1], m)     SumAggregation
//   z   = agg + (1 + eps) * x                              GINEConv.forward
// and the autograd of that chain.
//
// Layout: one "row group" of L lanes owns one node; lane t holds float4 chunks
// t, t+L, ... of the node's D channels, so every row read/written is a run of D*4
// contiguous bytes (512 B at D=128: two nodes per wave, 16 B per lane).  The node's edge
// list (neighbour id + edge attribute) is staged through LDS (one coalesced load by the
// group's lanes, then broadcast reads), and U neighbour rows are kept in flight per lane
// before the sequential accumulation, so the gather is latency-hidden without splitting a
// destination's sum.  Accumulation order is the CSR order = original edge order, hence
// bit-identical to CPU scatter_add_ / index_add_.
#include "gine_common.hpp"
#include "gine_edge.hpp"
#include "gine_reduce.hpp"
#include "gine_slab.hpp"


namespace gine {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;

// Neighbour rows in flight per lane.  (16 -- one round for k <= 15 -- was measured slower
// at cfg2: the extra VGPRs halve the waves per SIMD, and those hide more latency.)
#ifndef GINE_MPFWD_U
#define GINE_MPFWD_U 6
#endif
template <int C>
struct MpUnroll {
  static constexpr int value = C == 1 ? GINE_MPFWD_U : (C == 2 ? 4 : 2);
};
#ifndef GINE_MPBWD_U
#define GINE_MPBWD_U 6
#endif
template <int C>
struct MpUnrollBwd {
  static constexpr int value = C == 1 ? GINE_MPBWD_U : (C == 2 ? 4 : 2);
};

// ----------------------------------------------------------------------------------------
// Forward
// ----------------------------------------------------------------------------------------
template <int L, int C, bool FMA>
__global__ __launch_bounds__(kThreads) void k_mp_fwd(
    const float4* __restrict__ x4, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ nbr, const float* __restrict__ attr,
    const float4* __restrict__ lw4, const float4* __restrict__ lb4,
    const float* __restrict__ eps, float4* __restrict__ z4, int64_t N, int D4) {
  constexpr int GPW = kWave / L;  // nodes per wave
  constexpr int U = MpUnroll<C>::value;
  __shared__ int32_t s_nbr[kWaves][kWave];
  __shared__ float s_attr[kWaves][kWave];

  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int g = lane / L, t = lane % L;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t node = (int64_t)tile * (kWaves * GPW) + wave * GPW + g;
  if (node >= N) return;  // whole row group leaves together; no block barrier below

  // Lanes past the last float4 (D/4 not a multiple of L) duplicate the last chunk so that
  // every load is issued unconditionally; only their stores are masked.  Neighbour rows
  // are addressed by 32-bit byte offsets from the table base (N*D*4 < 2^32, host-checked).
  const char* xb = reinterpret_cast<const char*>(x4);
  const uint32_t rowb = (uint32_t)D4 * 16u;
  f4v w[C], b[C], self[C], acc[C];
  uint32_t qb[C];
  const uint32_t own = (uint32_t)node * rowb;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int q = min(t + c * L, D4 - 1);
    qb[c] = (uint32_t)q * 16u;
    acc[c] = f4v_zero();
    w[c] = ld_f4v(reinterpret_cast<const char*>(lw4), qb[c]);
    b[c] = ld_f4v(reinterpret_cast<const char*>(lb4), qb[c]);
    self[c] = ld_f4v(xb, own + qb[c]);
  }
  const float ope = 1.0f + eps[0];
  const int beg = rowptr[node], end = rowptr[node + 1];
  int32_t* my_nbr = &s_nbr[wave][g * L];
  float* my_attr = &s_attr[wave][g * L];

  for (int base = beg; base < end; base += L) {
    const int cnt = min(L, end - base);
    if (t < cnt) {
      my_nbr[t] = (int32_t)((uint32_t)nbr[base + t] * rowb);  // row byte offset
      my_attr[t] = attr[base + t];
    }
    __builtin_amdgcn_wave_barrier();
    int j = 0;
    // full batches of U neighbours: no per-edge test
    for (; j + U <= cnt; j += U) {
      f4v r[U][C];
      float a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t ro = (uint32_t)my_nbr[j + u];
        a[u] = my_attr[j + u];
#pragma unroll
        for (int c = 0; c < C; ++c) r[u][c] = ld_f4v(xb, ro + qb[c]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c) fwd_edge<FMA>(acc[c], r[u][c], a[u], w[c], b[c]);
    }
    // tail: loads clamped to the last neighbour (always issued), sums tested
    if (j < cnt) {
      f4v r[U][C];
      float a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = min(j + u, cnt - 1);
        const uint32_t ro = (uint32_t)my_nbr[jj];
        a[u] = my_attr[jj];
#pragma unroll
        for (int c = 0; c < C; ++c) r[u][c] = ld_f4v(xb, ro + qb[c]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j + u < cnt) {
#pragma unroll
          for (int c = 0; c < C; ++c) fwd_edge<FMA>(acc[c], r[u][c], a[u], w[c], b[c]);
        }
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int q = t + c * L;
    if (q < D4) z4[node * D4 + q] = to_float4(add_scaled(acc[c], ope, self[c]));
  }
}

// ----------------------------------------------------------------------------------------
// Backward over the out-edge CSR (source-sorted, stable)
// ----------------------------------------------------------------------------------------
// (C == 1: 4 workgroups per CU, i.e. the kernel fits 128 VGPRs = 4 waves per SIMD)
template <int L, int C, bool FMA>
__global__ __launch_bounds__(kThreads, C == 1 ? 4 : 2) void k_mp_bwd(
    const float4* __restrict__ dz4, const float4* __restrict__ x4,
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ nbr,
    const float* __restrict__ attr, const float4* __restrict__ lw4,
    const float4* __restrict__ lb4, const float* __restrict__ eps,
    const float4* __restrict__ dres4, float4* __restrict__ dx4, double* __restrict__ partials,
    int64_t N, int D4, int num_tiles, int flags, MlpSlabJob job) {
  constexpr int GPW = kWave / L;
  constexpr int U = MpUnrollBwd<C>::value;
  __shared__ int32_t s_nbr[kWaves][kWave];
  __shared__ float s_attr[kWaves][kWave];
  extern __shared__ __attribute__((aligned(16))) double s_red[];  // [3][D]
  // side job: the first job.nblocks workgroups reduce the preceding weight-gradient slabs
  if ((int)blockIdx.x < job.nblocks) {
    __shared__ double s_job[kSlabGroups][kSlabQuads * 4 + 1];
    job.run(blockIdx.x, s_job);
    return;
  }
  const int vb = blockIdx.x - job.nblocks, nb = gridDim.x - job.nblocks;

  const int D = D4 * 4;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int g = lane / L, t = lane % L;
  const float ope = 1.0f + eps[0];
  const bool add_self = (flags & GINE_MP_BWD_SELF) != 0;
  const char* dzb = reinterpret_cast<const char*>(dz4);
  const char* xb = reinterpret_cast<const char*>(x4);
  // the residual gradient row is loaded with the node's own rows (unconditionally, from
  // dz when there is none): a load behind the gather would add a round trip per tile
  const char* rb = reinterpret_cast<const char*>(dres4 != nullptr ? dres4 : dz4);
  const uint32_t rowb = (uint32_t)D4 * 16u;

  f4v w[C], b[C];
  uint32_t qb[C];
  double pw[C][4], pb[C][4];  // sum dm*a, sum dm (per channel, per-node terms)
  double pe = 0.0;            // sum over nodes and channels of dz*x
#pragma unroll
  for (int c = 0; c < C; ++c) {
    qb[c] = (uint32_t)min(t + c * L, D4 - 1) * 16u;
    w[c] = ld_f4v(reinterpret_cast<const char*>(lw4), qb[c]);
    b[c] = ld_f4v(reinterpret_cast<const char*>(lb4), qb[c]);
#pragma unroll
    for (int k = 0; k < 4; ++k) pw[c][k] = pb[c][k] = 0.0;
  }
  int32_t* my_nbr = &s_nbr[wave][g * L];
  float* my_attr = &s_attr[wave][g * L];

  // Tiles are split into 8 contiguous XCD ranges; the blocks of one XCD stride its range.
  const int xcd = vb % kNumXcd, pos = vb / kNumXcd;
  const int blocks_here = nb / kNumXcd + (xcd < nb % kNumXcd ? 1 : 0);
  const int span = (num_tiles + kNumXcd - 1) / kNumXcd;
  const int t_begin = xcd * span, t_end = min(num_tiles, t_begin + span);

  for (int tile = t_begin + pos; tile < t_end; tile += blocks_here) {
    const int64_t node = (int64_t)tile * (kWaves * GPW) + wave * GPW + g;
    if (node >= N) continue;
    const uint32_t own = (uint32_t)node * rowb;
    f4v h[C], g_self[C], acc[C], accw[C], r_self[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      acc[c] = f4v_zero();
      accw[c] = f4v_zero();
      h[c] = ld_f4v(xb, own + qb[c]);
      g_self[c] = ld_f4v(dzb, own + qb[c]);
      r_self[c] = ld_f4v(rb, own + qb[c]);
    }
    // pre-activation of this node's outgoing messages: h + (a*W + b) depends on the edge
    // only through a, so h is loaded once per source node.
    const int beg = rowptr[node], end = rowptr[node + 1];
    for (int base = beg; base < end; base += L) {
      const int cnt = min(L, end - base);
      if (t < cnt) {
        my_nbr[t] = (int32_t)((uint32_t)nbr[base + t] * rowb);  // row byte offset
        my_attr[t] = attr[base + t];
      }
      __builtin_amdgcn_wave_barrier();
      int j = 0;
      // full batches of U neighbours: no per-edge test
      for (; j + U <= cnt; j += U) {
        f4v r[U][C];
        float a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t ro = (uint32_t)my_nbr[j + u];
          a[u] = my_attr[j + u];
#pragma unroll
          for (int c = 0; c < C; ++c) r[u][c] = ld_f4v(dzb, ro + qb[c]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int c = 0; c < C; ++c)
            bwd_edge<FMA>(acc[c], accw[c], r[u][c], a[u], h[c], w[c], b[c]);
      }
      // tail: loads clamped to the last neighbour (always issued), sums tested
      if (j < cnt) {
        f4v r[U][C];
        float a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int jj = min(j + u, cnt - 1);
          const uint32_t ro = (uint32_t)my_nbr[jj];
          a[u] = my_attr[jj];
#pragma unroll
          for (int c = 0; c < C; ++c) r[u][c] = ld_f4v(dzb, ro + qb[c]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (j + u < cnt) {
#pragma unroll
            for (int c = 0; c < C; ++c)
              bwd_edge<FMA>(acc[c], accw[c], r[u][c], a[u], h[c], w[c], b[c]);
          }
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int q = t + c * L;
      if (q < D4) {
        // db_e = sum_e dm_e: each source node contributes its message-gradient sum
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          pb[c][k] += (double)acc[c][k];
          pw[c][k] += (double)accw[c][k];
        }
        f4v o = add_self ? add_scaled(acc[c], ope, g_self[c]) : acc[c];
        if (dres4 != nullptr) {
          o.xy = o.xy + r_self[c].xy;
          o.zw = o.zw + r_self[c].zw;
        }
        dx4[node * D4 + q] = to_float4(o);
        pe += ((double)g_self[c].x * (double)h[c].x + (double)g_self[c].y * (double)h[c].y) +
              ((double)g_self[c].z * (double)h[c].z + (double)g_self[c].w * (double)h[c].w);
      }
    }
  }

  // Block reduction of the parameter-gradient partials: row groups of a wave first
  // (butterfly over lanes t, t+L, ...), then the waves in fixed order through LDS.
#pragma unroll
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int m = L; m < kWave; m <<= 1) {
        pw[c][k] += shfl_xor_d(pw[c][k], m);
        pb[c][k] += shfl_xor_d(pb[c][k], m);
      }
    }
  }
#pragma unroll
  for (int m = 1; m < kWave; m <<= 1) pe += shfl_xor_d(pe, m);
  for (int wv = 0; wv < kWaves; ++wv) {
    if (wave == wv && g == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const int q = t + c * L;
        if (q < D4) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int ch = q * 4 + k;
            if (wv == 0) {
              s_red[ch] = pw[c][k];
              s_red[D + ch] = pb[c][k];
            } else {
              s_red[ch] += pw[c][k];
              s_red[D + ch] += pb[c][k];
            }
          }
        }
      }
      if (lane == 0) s_red[2 * D + wv] = pe;
    }
    __syncthreads();
  }
  // row layout [dW_e (D) | db_e (D) | sum over nodes and channels of dz*x (1) | unused]
  if (threadIdx.x == 0) {
    double e = 0.0;
    for (int wv = 0; wv < kWaves; ++wv) e += s_red[2 * D + wv];
    s_red[2 * D] = e;
  }
  __syncthreads();
  double* out = partials + (size_t)vb * 3 * D;
  for (int i = threadIdx.x; i <= 2 * D; i += kThreads) out[i] = s_red[i];
}

// Finish of the parameter-gradient partials (k_colsum_fin<4>): workgroups b < nb-1 own 4
// of the 2D columns [dW_e | db_e]; the last one reduces the per-block eps column (2D).
constexpr int kMpFinCols = 4;
struct MpBwdFin {
  float *dlin_w, *dlin_b, *deps;
  int D, nb;
  __device__ int col(int b, int j) const {
    if (b == nb - 1) return j == 0 ? 2 * D : -1;
    const int c = kMpFinCols * b + j;
    return c < 2 * D ? c : -1;
  }
  __device__ void finish(int b, const double* tot) const {
    const int t = threadIdx.x;
    if (b == nb - 1) {
      if (t == 0) deps[0] = (float)tot[0];
      return;
    }
    const int c = kMpFinCols * b + t;
    if (t >= kMpFinCols || c >= 2 * D) return;
    if (c < D) dlin_w[c] = (float)tot[t];
    else dlin_b[c - D] = (float)tot[t];
  }
};

// ----------------------------------------------------------------------------------------
// Host dispatch
// ----------------------------------------------------------------------------------------
struct Shape {
  int L, C;
};

inline bool pick_shape(int D, Shape* s) {
  if (D <= 0 || D % 4 != 0 || D > 1024) return false;
  const int D4 = D / 4;
  if (D4 <= 64) {
    int L = 1;
    while (L < D4) L <<= 1;
    s->L = L;
    s->C = 1;
  } else {
    s->L = 64;
    s->C = (D4 + 63) / 64;
  }
  return true;
}

inline int nodes_per_block(const Shape& s) { return kWaves * (kWave / s.L); }

// Persistent grid cap (512 - 4096 measured within noise at cfg2).
inline int64_t max_bwd_blocks() { return 1024; }

inline int bwd_grid(int64_t N, const Shape& s) {
  const int64_t tiles = ceil_div(N, nodes_per_block(s));
  const int64_t cap = max_bwd_blocks();
  int64_t g = tiles < cap ? tiles : cap;
  return (int)(g > 0 ? g : 1);
}

#define GINE_MP_DISPATCH_L(SHAPE, MACRO, F)                                     \
  switch ((SHAPE).C) {                                                          \
    case 1:                                                                     \
      switch ((SHAPE).L) {                                                      \
        case 1: MACRO(1, 1, F); break;                                          \
        case 2: MACRO(2, 1, F); break;                                          \
        case 4: MACRO(4, 1, F); break;                                          \
        case 8: MACRO(8, 1, F); break;                                          \
        case 16: MACRO(16, 1, F); break;                                        \
        case 32: MACRO(32, 1, F); break;                                        \
        default: MACRO(64, 1, F); break;                                        \
      }                                                                         \
      break;                                                                    \
    case 2: MACRO(64, 2, F); break;                                             \
    case 3: MACRO(64, 3, F); break;                                             \
    default: MACRO(64, 4, F); break;                                            \
  }

#define GINE_MP_DISPATCH(SHAPE, FMA_FLAG, MACRO)                                \
  if (FMA_FLAG) {                                                               \
    GINE_MP_DISPATCH_L(SHAPE, MACRO, true)                                      \
  } else {                                                                      \
    GINE_MP_DISPATCH_L(SHAPE, MACRO, false)                                     \
  }

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_mp_fwd(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                           const float* in_attr, const float* lin_w, const float* lin_b,
                           const float* eps, float* z, int64_t num_nodes, int32_t channels,
                           int32_t flags, void* stream) {
  Shape sh;
  if (!pick_shape(channels, &sh)) return GINE_ERR_DIM;
  if (num_nodes < 0 || (flags & ~GINE_MP_LIN_MULADD) != 0) return GINE_ERR_INVALID;
  if (num_nodes * channels * 4 >= (int64_t(1) << 32)) return GINE_ERR_TOO_LARGE;
  if (num_nodes == 0) return GINE_OK;
  if (!x || !in_rowptr || !lin_w || !lin_b || !eps || !z) return GINE_ERR_INVALID;
  const int D4 = channels / 4;
  const int64_t tiles = ceil_div(num_nodes, nodes_per_block(sh));
  hipStream_t s = as_stream(stream);
  const bool fma = (flags & GINE_MP_LIN_MULADD) == 0;
#define LAUNCH_FWD(L_, C_, F_)                                                              \
  hipLaunchKernelGGL((k_mp_fwd<L_, C_, F_>), dim3((unsigned)tiles), dim3(kThreads), 0, s,      \
                     (const float4*)x, in_rowptr, in_src, in_attr, (const float4*)lin_w,    \
                     (const float4*)lin_b, eps, (float4*)z, num_nodes, D4)
  GINE_MP_DISPATCH(sh, fma, LAUNCH_FWD);
#undef LAUNCH_FWD
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_mp_bwd_num_partials(int64_t num_nodes, int32_t channels,
                                        int32_t* num_partials) {
  Shape sh;
  if (!num_partials) return GINE_ERR_INVALID;
  if (!pick_shape(channels, &sh)) return GINE_ERR_DIM;
  if (num_nodes < 0) return GINE_ERR_INVALID;
  *num_partials = bwd_grid(num_nodes, sh);
  return GINE_OK;
}

static int mp_bwd_launch(const float* dz, const float* x, const int32_t* out_rowptr,
                         const int32_t* out_dst, const float* out_attr, const float* lin_w,
                         const float* lin_b, const float* eps, const float* dres, float* dx,
                         double* partials, int64_t num_nodes, int32_t channels, int32_t flags,
                         const MlpSlabJob& job, void* stream) {
  Shape sh;
  if (!pick_shape(channels, &sh)) return GINE_ERR_DIM;
  if (num_nodes < 0 || (flags & ~(GINE_MP_BWD_SELF | GINE_MP_LIN_MULADD)) != 0)
    return GINE_ERR_INVALID;
  if (num_nodes * channels * 4 >= (int64_t(1) << 32)) return GINE_ERR_TOO_LARGE;
  if (!dz || !x || !out_rowptr || !lin_w || !lin_b || !eps || !dx || !partials)
    return GINE_ERR_INVALID;
  const int D4 = channels / 4;
  const int grid = bwd_grid(num_nodes, sh);
  const int tiles = (int)ceil_div(num_nodes, nodes_per_block(sh));
  int m = 1;
  while (m < channels) m <<= 1;  // tree-sum scratch of the eps column
  const size_t smem = sizeof(double) * (2 * (size_t)channels + (size_t)m);
  hipStream_t s = as_stream(stream);
  const bool fma = (flags & GINE_MP_LIN_MULADD) == 0;
#define LAUNCH_BWD(L_, C_, F_)                                                               \
  hipLaunchKernelGGL((k_mp_bwd<L_, C_, F_>), dim3((unsigned)(grid + job.nblocks)),            \
                     dim3(kThreads), smem, s, (const float4*)dz, (const float4*)x, out_rowptr,  \
                     out_dst, out_attr, (const float4*)lin_w, (const float4*)lin_b, eps,       \
                     (const float4*)dres, (float4*)dx, partials, num_nodes, D4, tiles, flags,  \
                     job)
  GINE_MP_DISPATCH(sh, fma, LAUNCH_BWD);
#undef LAUNCH_BWD
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_mp_bwd(const float* dz, const float* x, const int32_t* out_rowptr,
                           const int32_t* out_dst, const float* out_attr, const float* lin_w,
                           const float* lin_b, const float* eps, const float* dres, float* dx,
                           double* partials, int64_t num_nodes, int32_t channels, int32_t flags,
                           void* stream) {
  const MlpSlabJob none{nullptr, 0, 0, 0, MlpWgradOut{nullptr, nullptr, nullptr, nullptr, 0}};
  return mp_bwd_launch(dz, x, out_rowptr, out_dst, out_attr, lin_w, lin_b, eps, dres, dx,
                       partials, num_nodes, channels, flags, none, stream);
}

extern "C" int gine_mp_bwd_side(const float* dz, const float* x, const int32_t* out_rowptr,
                                const int32_t* out_dst, const float* out_attr,
                                const float* lin_w, const float* lin_b, const float* eps,
                                const float* dres, float* dx, double* partials,
                                int64_t num_nodes, int32_t channels, int32_t flags,
                                const float* wg_slab, int32_t wg_chunks, int32_t mlp_channels,
                                float* dw1, float* db1, float* dw2, float* db2, void* stream) {
  if (!wg_slab || wg_chunks <= 0 || mlp_channels <= 0) return GINE_ERR_INVALID;
  const int64_t per = (int64_t)mlp_channels * mlp_channels + mlp_channels;
  if (per % 4 != 0 || (reinterpret_cast<uintptr_t>(wg_slab) & 15) != 0) return GINE_ERR_INVALID;
  const int cols = (int)ceil_div(per, kSlabQuads * 4);
  const MlpSlabJob job{wg_slab, wg_chunks, cols, 2 * cols,
                       MlpWgradOut{dw2, db2, dw1, db1, mlp_channels}};
  return mp_bwd_launch(dz, x, out_rowptr, out_dst, out_attr, lin_w, lin_b, eps, dres, dx,
                       partials, num_nodes, channels, flags, job, stream);
}

extern "C" int gine_mp_bwd_finalize(const double* partials, int32_t num_partials,
                                    int32_t channels, float* dlin_w, float* dlin_b,
                                    float* deps, void* stream) {
  if (num_partials < 0 || channels <= 0) return GINE_ERR_INVALID;
  if (!partials || !dlin_w || !dlin_b || !deps) return GINE_ERR_INVALID;
  const int nb = (int)ceil_div(2 * channels, kMpFinCols) + 1;
  const MpBwdFin fin{dlin_w, dlin_b, deps, channels, nb};
  hipLaunchKernelGGL((k_colsum_fin<kMpFinCols, MpBwdFin>), dim3(nb), dim3(256), 0,
                     as_stream(stream), partials, num_partials, 3 * channels, fin);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
