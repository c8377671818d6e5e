// Weight / bias gradients of a plain Linear over MANY rows: dW = dY^T X, db = sum_rows dY.
//
// The model around the GINE stack (DeepSetEncoder phi/rho, dim_red, aggr: models/gnn.py:
// 48-68, 112-123) has tiny weights ([128 x 35] ... [4 x 128]) but reduces over 16,000 nodes
// or 176,000 node x member rows per step.  Library GEMMs tile the small [O x I] output into
// only 8-16 workgroups for these shapes and run at a few TFLOP/s; the engine of
// gine_wgrad.hpp splits the ROWS (the contraction) instead, with fp32 partial slabs reduced
// over chunks in fixed order in fp64 (deterministic).
#include "gine_common.hpp"
#include "gine_slab.hpp"
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
  static constexpr int kZ = 1;
  const float* dy;
  const float* x;
  int O, I;
  struct Raw {
    float4 v;
  };
  struct Col {};
  template <int Z> __device__ int i_dim(int I) const { return I; }
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

struct LinWgradOut {
  float* dw;
  float* db;
  int64_t wsize;
  float bias_scale;
  __device__ void operator()(int, int64_t e, double v) const {
    if (e < wsize) dw[e] = (float)v;
    else if (db) db[e - wsize] = (float)(v * (double)bias_scale);
  }
};

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_linear_wgrad_num_chunks(int64_t rows, int32_t out_features,
                                            int32_t in_features, int32_t* num_chunks) {
  if (!num_chunks || rows < 0 || out_features <= 0 || in_features <= 0)
    return GINE_ERR_INVALID;
  *num_chunks = wg_plan(rows, out_features, in_features, 1, 64).chunks;
  return GINE_OK;
}

extern "C" int gine_linear_wgrad(const float* dy, const float* x, int64_t rows,
                                 int32_t out_features, int32_t in_features, float* slab,
                                 float* dw, float* db, float bias_scale, void* stream) {
  if (rows < 0 || out_features <= 0 || in_features <= 0 || !dw || !slab)
    return GINE_ERR_INVALID;
  if (rows > 0 && (!dy || !x)) return GINE_ERR_INVALID;
  const int O = out_features, I = in_features;
  const WgPlan p = wg_plan(rows, O, I, 1, 64);
  hipStream_t s = as_stream(stream);
  const int64_t per = (int64_t)O * I + O;
  if (rows == 0) {
    GINE_RETURN_IF_HIP(hipMemsetAsync(slab, 0, sizeof(float) * per, s));
  } else {
    const bool vp = vec_ok(dy, O), vq = vec_ok(x, I);
    int st;
    if (vp && vq) {
      st = launch_wgrad_engine<64>(LinWgradSrc<true, true>{dy, x, O, I}, rows, O, I, p.tiles_o * p.tiles_i, p, 0,
                               (size_t)per, slab, s);
    } else if (vp) {
      st = launch_wgrad_engine<64>(LinWgradSrc<true, false>{dy, x, O, I}, rows, O, I, p.tiles_o * p.tiles_i, p, 0,
                               (size_t)per, slab, s);
    } else if (vq) {
      st = launch_wgrad_engine<64>(LinWgradSrc<false, true>{dy, x, O, I}, rows, O, I, p.tiles_o * p.tiles_i, p, 0,
                               (size_t)per, slab, s);
    } else {
      st = launch_wgrad_engine<64>(LinWgradSrc<false, false>{dy, x, O, I}, rows, O, I, p.tiles_o * p.tiles_i, p, 0,
                               (size_t)per, slab, s);
    }
    if (st != GINE_OK) return st;
  }
  return launch_slab_sum(slab, rows == 0 ? 1 : p.chunks, per, (size_t)per, 0, 1,
                         LinWgradOut{dw, db, (int64_t)O * I, bias_scale}, s);
}
