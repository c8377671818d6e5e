// Weight / bias gradients of a plain Linear over MANY rows: dW = dY^T X, db = sum_rows dY.
//
// The model around the GINE stack (DeepSetEncoder phi/rho, dim_red, aggr: models/gnn.py:
// 48-68, 112-123) has tiny weights ([128 x 35] ... [4 x 128]) but reduces over 16,000 nodes
// or 176,000 node x member rows per step.  Library GEMMs tile the small [O x I] output into
// only 8-16 workgroups for these shapes and run at a few TFLOP/s; the engine of
// gine_wgrad.hpp splits the ROWS (the contraction) instead, with fp32 partial slabs reduced
// over chunks in fixed order in fp64 (deterministic).
#include "gine_common.hpp"
#include "gine_wgrad.hpp"

namespace gine {
namespace {

// Operand source of the engine: P = dy [R, O], Q = x [R, I], plain row-major fp32.
// VEC: rows are whole float4s (ld % 4 == 0, 16-B aligned base); otherwise (dim_red's input
// row is 35 + 128 = 163 floats) four scalar loads at clamped addresses, zeroed past ld.
template <bool VEC>
__device__ __forceinline__ float4 row_quad(const float* __restrict__ a, int64_t n, int ld,
                                           int q) {
  const float* row = a + n * ld;
  const int c = 4 * q;
  if constexpr (VEC) {
    return *reinterpret_cast<const float4*>(row + c);
  } else {
    const float v0 = row[min(c, ld - 1)], v1 = row[min(c + 1, ld - 1)];
    const float v2 = row[min(c + 2, ld - 1)], v3 = row[min(c + 3, ld - 1)];
    return make_float4(v0, c + 1 < ld ? v1 : 0.f, c + 2 < ld ? v2 : 0.f, c + 3 < ld ? v3 : 0.f);
  }
}

template <bool VP, bool VQ>
struct LinWgradSrc {
  const float* dy;
  const float* x;
  int O, I;
  struct Raw {
    float4 v;
  };
  struct Col {};
  template <int Z> __device__ Col p_col(int) const { return Col{}; }
  template <int Z> __device__ Col q_col(int) const { return Col{}; }
  template <int Z> __device__ Raw p_load(int64_t n, int q) const { return Raw{row_quad<VP>(dy, n, O, q)}; }
  template <int Z> __device__ Raw q_load(int64_t n, int q) const { return Raw{row_quad<VQ>(x, n, I, q)}; }
  template <int Z> __device__ float4 p_xform(const Raw& r, const Col&) const { return r.v; }
  template <int Z> __device__ float4 q_xform(const Raw& r, const Col&) const { return r.v; }
};

inline bool vec_ok(const float* p, int ld) {
  return ld % 4 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

// 64 consecutive slab elements x 4 chunk groups per workgroup (fixed order, see gine_mlp).
__global__ __launch_bounds__(256) void k_linear_slab_reduce(const float* __restrict__ slab,
                                                            int chunks, int64_t per,
                                                            int64_t wsize,
                                                            float* __restrict__ dw,
                                                            float* __restrict__ db,
                                                            float bias_scale) {
  __shared__ double s_part[4][64];
  const int64_t e = blockIdx.x * (int64_t)64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  double acc = 0.0;
  if (e < per) {
    const float* base = slab + e;
    for (int c = g; c < chunks; c += 4) acc += (double)base[(size_t)c * per];
  }
  s_part[g][threadIdx.x & 63] = acc;
  __syncthreads();
  if (g != 0 || e >= per) return;
  const int j = threadIdx.x & 63;
  const double v = (s_part[0][j] + s_part[1][j]) + (s_part[2][j] + s_part[3][j]);
  if (e < wsize) {
    dw[e] = (float)v;
  } else if (db != nullptr) {
    db[e - wsize] = (float)(v * (double)bias_scale);
  }
}

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_linear_wgrad_num_chunks(int64_t rows, int32_t out_features,
                                            int32_t in_features, int32_t* num_chunks) {
  if (!num_chunks || rows < 0 || out_features <= 0 || in_features <= 0)
    return GINE_ERR_INVALID;
  *num_chunks = wg_plan(rows, out_features, in_features, 1).chunks;
  return GINE_OK;
}

extern "C" int gine_linear_wgrad(const float* dy, const float* x, int64_t rows,
                                 int32_t out_features, int32_t in_features, float* slab,
                                 float* dw, float* db, float bias_scale, void* stream) {
  if (rows < 0 || out_features <= 0 || in_features <= 0 || !dw || !slab)
    return GINE_ERR_INVALID;
  if (rows > 0 && (!dy || !x)) return GINE_ERR_INVALID;
  const int O = out_features, I = in_features;
  const WgPlan p = wg_plan(rows, O, I, 1);
  hipStream_t s = as_stream(stream);
  const int64_t per = (int64_t)O * I + O;
  if (rows == 0) {
    GINE_RETURN_IF_HIP(hipMemsetAsync(slab, 0, sizeof(float) * per, s));
  } else {
    const bool vp = vec_ok(dy, O), vq = vec_ok(x, I);
    int st;
    if (vp && vq) {
      st = launch_wgrad_engine(LinWgradSrc<true, true>{dy, x, O, I}, rows, O, I, 1, p, 0,
                               (size_t)per, slab, s);
    } else if (vp) {
      st = launch_wgrad_engine(LinWgradSrc<true, false>{dy, x, O, I}, rows, O, I, 1, p, 0,
                               (size_t)per, slab, s);
    } else if (vq) {
      st = launch_wgrad_engine(LinWgradSrc<false, true>{dy, x, O, I}, rows, O, I, 1, p, 0,
                               (size_t)per, slab, s);
    } else {
      st = launch_wgrad_engine(LinWgradSrc<false, false>{dy, x, O, I}, rows, O, I, 1, p, 0,
                               (size_t)per, slab, s);
    }
    if (st != GINE_OK) return st;
  }
  hipLaunchKernelGGL(k_linear_slab_reduce, dim3((unsigned)ceil_div(per, 64)), dim3(256), 0, s,
                     slab, rows == 0 ? 1 : p.chunks, per, (int64_t)O * I, dw, db, bias_scale);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
