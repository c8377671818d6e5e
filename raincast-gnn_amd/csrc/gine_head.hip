// Output head of the station-graph GNN on gfx950: aggr = Linear(D, K) followed by
// PostProcess, forward and backward, one kernel each.
//
// Replaces (models/gnn.py:123,125,140-141 and models/model_utils.py:42-113):
//   raw  = h W^T + b                      GNN.aggr (Linear(hidden, out_channels))
//   pred = PostProcess(raw):  column 0 (mu) as is; sigma, sigma_u -> softplus(.) + 1e-6;
//          p -> sigmoid(.); u -> sigmoid(.) * 2.12  (per loss, see gine_hip.h)
// and their autograd, which the reference runs as one library GEMV, ~5 elementwise kernels
// and a concatenation each way.  K <= 5 outputs per node, so the head is a row-streaming
// kernel bound by reading h [N, D] once: one 32-lane half-wave per node, lane t holding
// float4 columns t, t+32, ... of the row; the K dot products are reduced across the
// half-wave in a fixed order on VALU lane exchanges (gine_headrow.hpp sum4_32 / sum_32).  softplus / sigmoid and their derivatives follow
// ATen's formulas (threshold 20 for softplus, sigmoid backward from the saved output).
//
// Backward: d raw = PostProcess'(raw) * d pred; dh = d raw W (written once); dW = d raw^T h
// and db = sum d raw as fp32 per-workgroup partials in a slab, reduced in fixed order by
// k_slab_sum (deterministic).
#include "gine_common.hpp"
#include "gine_headrow.hpp"
#include "gine_slab.hpp"

#include <algorithm>

namespace gine {
namespace {

using namespace head;

template <int K, bool COUNT>
__global__ __launch_bounds__(kThreads) void k_head_fwd(const float* __restrict__ h,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ b,
                                                       float* __restrict__ raw,
                                                       float* __restrict__ pred, int64_t N,
                                                       int D, int kind,
                                                       const float* __restrict__ y,
                                                       uint32_t* __restrict__ count_parts) {
  static_assert(kThreads == 256, "count_valid_parts takes 256-thread blocks");
  if constexpr (COUNT) count_valid_parts(y, N, count_parts);
  const int t = threadIdx.x & 31;
  const int D4 = D / 4;
  for (int64_t n = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / 32; n < N;
       n += (int64_t)gridDim.x * kRowsPerBlock) {
    float acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.f;
#pragma unroll
    for (int c = 0; c < kMaxChunks; ++c) {
      const int q = t + 32 * c;
      if (q < D4) {
        const float4 x = reinterpret_cast<const float4*>(h + n * D)[q];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float4 wk = reinterpret_cast<const float4*>(w + (size_t)k * D)[q];
          acc[k] = __builtin_fmaf(x.x, wk.x, acc[k]);
          acc[k] = __builtin_fmaf(x.y, wk.y, acc[k]);
          acc[k] = __builtin_fmaf(x.z, wk.z, acc[k]);
          acc[k] = __builtin_fmaf(x.w, wk.w, acc[k]);
        }
      }
    }
    // outputs 0-3 reduce-scattered (sum4_32; output o at lanes 8 o .. 8 o + 7, finalised by
    // lane 8 o), output 4 by a full butterfly (finalised by lane 1)
    const float d = sum4_32(acc[0], K > 1 ? acc[1] : 0.f, K > 2 ? acc[2] : 0.f,
                            K > 3 ? acc[3] : 0.f);
    const int o = (t >> 3) & 3;
    if ((t & 7) == 0 && o < K) {
      const float v = d + b[o];
      raw[n * K + o] = v;
      pred[n * K + o] = post(role_of(kind, o), v);
    }
    if constexpr (K == 5) {
      const float e = sum_32(acc[4]);
      if (t == 1) {
        const float v = e + b[4];
        raw[n * K + 4] = v;
        pred[n * K + 4] = post(role_of(kind, 4), v);
      }
    }
  }
}

template <int K>
__global__ __launch_bounds__(kThreads) void k_head_bwd(const float* __restrict__ gpred,
                                                       const float* __restrict__ raw,
                                                       const float* __restrict__ h,
                                                       const float* __restrict__ w,
                                                       float* __restrict__ dh,
                                                       float* __restrict__ slab, int64_t N,
                                                       int D, int kind) {
  __shared__ float s_part[kRowsPerBlock][kMaxK * 256 + kMaxK];
  bwd_rows<K, 8>(
      [&](int64_t n, float (&g)[K]) {
#pragma unroll
        for (int k = 0; k < K; ++k)
          g[k] = post_bwd(role_of(kind, k), raw[n * K + k], gpred[n * K + k]);
      },
      (int64_t)blockIdx.x * kRowsPerBlock, (int64_t)gridDim.x * kRowsPerBlock, N, h, w, dh,
      slab + (size_t)blockIdx.x * (K * D + K), D, s_part);
}

// gine_testing_sum_32: sum_32 against the __shfl_xor butterfly it stands for, per lane
__global__ __launch_bounds__(64) void k_testing_sum_32(const float* __restrict__ in,
                                                       float* __restrict__ out, int mode) {
  float a = in[blockIdx.x * 64 + threadIdx.x];
  if (mode == 1) {
    a = sum_32(a);
  } else {
#pragma unroll
    for (int m = 16; m >= 1; m >>= 1) a += __shfl_xor(a, m, 32);
  }
  out[blockIdx.x * 64 + threadIdx.x] = a;
}

struct HeadOut {
  float* dw;
  float* db;
  int64_t wsize;
  __device__ void operator()(int, int64_t e, double v) const {
    if (e < wsize) dw[e] = (float)v;
    else if (db) db[e - wsize] = (float)v;
  }
};

inline int k_of(int kind) {
  switch (kind) {
    case GINE_LOSS_NORMAL: return 2;
    case GINE_LOSS_MIXED_NORMAL: return 3;
    case GINE_LOSS_MIXED: return 4;
    case GINE_LOSS_MIXED_U: return 5;
    default: return -1;
  }
}

inline bool head_dim_ok(int D) { return D > 0 && D % 4 == 0 && D <= 32 * 4 * kMaxChunks; }

inline int head_bwd_grid(int64_t N) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(kHeadBlocks, ceil_div(N, kRowsPerBlock)));
}

}  // namespace
}  // namespace gine

using namespace gine;

namespace {
int head_fwd(const float* h, const float* w, const float* b, float* raw, float* pred,
             int64_t num_nodes, int32_t channels, int32_t kind, const float* y,
             uint32_t* count_parts, void* stream) {
  const int K = k_of(kind);
  if (K < 0 || num_nodes < 0) return GINE_ERR_INVALID;
  if (!head_dim_ok(channels)) return GINE_ERR_DIM;
  if (count_parts && num_nodes > 0 && !y) return GINE_ERR_INVALID;
  if (num_nodes == 0) {
    if (count_parts) return gine_count_valid(y, 0, count_parts, stream);
    return GINE_OK;
  }
  if (!h || !w || !b || !raw || !pred) return GINE_ERR_INVALID;
  const int grid = (int)std::min<int64_t>(2048, ceil_div(num_nodes, kRowsPerBlock));
  hipStream_t s = as_stream(stream);
#define HEAD_FWD(KK)                                                                         \
  do {                                                                                       \
    if (count_parts)                                                                         \
      hipLaunchKernelGGL((k_head_fwd<KK, true>), dim3(grid), dim3(kThreads), 0, s, h, w, b,  \
                         raw, pred, num_nodes, channels, kind, y, count_parts);              \
    else                                                                                     \
      hipLaunchKernelGGL((k_head_fwd<KK, false>), dim3(grid), dim3(kThreads), 0, s, h, w, b, \
                         raw, pred, num_nodes, channels, kind, nullptr, nullptr);            \
  } while (0)
  switch (K) {
    case 2: HEAD_FWD(2); break;
    case 3: HEAD_FWD(3); break;
    case 4: HEAD_FWD(4); break;
    default: HEAD_FWD(5); break;
  }
#undef HEAD_FWD
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
}  // namespace

extern "C" int gine_testing_sum_32(const float* in, float* out, int32_t waves, int32_t mode,
                                   void* stream) {
  if (!in || !out || waves <= 0 || (mode != 0 && mode != 1)) return GINE_ERR_INVALID;
  hipLaunchKernelGGL(k_testing_sum_32, dim3((unsigned)waves), dim3(64), 0, as_stream(stream), in,
                     out, (int)mode);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_head_fwd(const float* h, const float* w, const float* b, float* raw,
                             float* pred, int64_t num_nodes, int32_t channels, int32_t kind,
                             void* stream) {
  return head_fwd(h, w, b, raw, pred, num_nodes, channels, kind, nullptr, nullptr, stream);
}

extern "C" int gine_head_fwd_count(const float* h, const float* w, const float* b, float* raw,
                                   float* pred, int64_t num_nodes, int32_t channels,
                                   int32_t kind, const float* y, uint32_t* count_parts,
                                   void* stream) {
  if (!count_parts) return GINE_ERR_INVALID;
  return head_fwd(h, w, b, raw, pred, num_nodes, channels, kind, y, count_parts, stream);
}

extern "C" int gine_head_bwd_slab_floats(int64_t num_nodes, int32_t channels, int32_t kind,
                                         size_t* floats) {
  const int K = k_of(kind);
  if (K < 0 || num_nodes < 0 || !floats) return GINE_ERR_INVALID;
  if (!head_dim_ok(channels)) return GINE_ERR_DIM;
  *floats = (size_t)head_bwd_grid(num_nodes) * (size_t)(K * channels + K);
  return GINE_OK;
}

extern "C" int gine_head_bwd(const float* grad_pred, const float* raw, const float* h,
                             const float* w, float* dh, float* slab, float* dw, float* db,
                             int64_t num_nodes, int32_t channels, int32_t kind, void* stream) {
  const int K = k_of(kind);
  if (K < 0 || num_nodes < 0) return GINE_ERR_INVALID;
  if (!head_dim_ok(channels)) return GINE_ERR_DIM;
  if (!w || !slab) return GINE_ERR_INVALID;
  if (num_nodes > 0 && (!grad_pred || !raw || !h || !dh)) return GINE_ERR_INVALID;
  const int grid = head_bwd_grid(num_nodes);
  const int64_t per = (int64_t)K * channels + K;
  hipStream_t s = as_stream(stream);
  if (num_nodes == 0) {
    GINE_RETURN_IF_HIP(hipMemsetAsync(slab, 0, sizeof(float) * per, s));
  } else {
#define HEAD_BWD(KK)                                                                          \
  hipLaunchKernelGGL(k_head_bwd<KK>, dim3(grid), dim3(kThreads), 0, s, grad_pred, raw, h, w, \
                     dh, slab, num_nodes, channels, kind)
    switch (K) {
      case 2: HEAD_BWD(2); break;
      case 3: HEAD_BWD(3); break;
      case 4: HEAD_BWD(4); break;
      default: HEAD_BWD(5); break;
    }
#undef HEAD_BWD
    GINE_LAUNCH_STATUS();
  }
  if (!dw) return GINE_OK;  // slab left for gine_head_bwd_reduce
  return launch_slab_sum(slab, num_nodes == 0 ? 1 : grid, per, (size_t)per, 0, 1,
                         HeadOut{dw, db, (int64_t)K * channels}, s);
}

extern "C" int gine_head_bwd_reduce(const float* slab, float* dw, float* db, int64_t num_nodes,
                                    int32_t channels, int32_t kind, void* stream) {
  const int K = k_of(kind);
  if (K < 0 || num_nodes < 0 || !slab || !dw) return GINE_ERR_INVALID;
  if (!head_dim_ok(channels)) return GINE_ERR_DIM;
  const int64_t per = (int64_t)K * channels + K;
  return launch_slab_sum(slab, num_nodes == 0 ? 1 : head_bwd_grid(num_nodes), per, (size_t)per,
                         0, 1, HeadOut{dw, db, (int64_t)K * channels}, as_stream(stream));
}

extern "C" int gine_head_bwd_grad_job(int64_t num_nodes, int32_t channels, int32_t kind,
                                      const float* slab, float* dw, float* db,
                                      gine_grad_job* job) {
  const int K = k_of(kind);
  if (K < 0 || num_nodes < 0 || !head_dim_ok(channels) || !slab || !dw || !job)
    return GINE_ERR_INVALID;
  const int64_t per = (int64_t)K * channels + K;
  *job = gine_grad_job{};
  job->kind = GINE_GRAD_JOB_SLAB;
  job->src = slab;
  job->rows = num_nodes == 0 ? 1 : head_bwd_grid(num_nodes);
  job->cstride = per;
  job->nz = 1;
  job->per[0] = per;
  job->wsize[0] = (int64_t)K * channels;
  job->w[0] = dw;
  job->b[0] = db;
  job->bscale[0] = 1.0f;
  return GINE_OK;
}
