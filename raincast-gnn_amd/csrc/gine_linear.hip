// Weight / bias gradients of a plain Linear over MANY rows: dW = dY^T X, db = sum_rows dY.
//
// The model around the GINE stack (DeepSetEncoder phi/rho, dim_red, aggr: models/gnn.py:
// 48-68, 112-123) has tiny weights ([128 x 35] ... [4 x 128]) but reduces over 16,000 nodes
// or 176,000 node x member rows per step.  Library GEMMs tile the small [O x I] output into
// only 8-16 workgroups for these shapes and run at a few TFLOP/s; this kernel splits the
// ROWS (the contraction) instead: grid = (row chunks) x (64x64 output tiles), one 32x32
// v_mfma_f32_32x32x2_f32 tile per wave, 32-row sub-tiles staged through LDS with the next
// sub-tile prefetched into registers during the MFMAs, fp32 partial slabs reduced over
// chunks in fixed order in fp64 (deterministic).
#include "gine_common.hpp"

namespace gine {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kRows = 32;         // rows per staged sub-tile
constexpr int kTile = 64;         // output tile edge
constexpr int kLds = kTile + 1;   // padded LDS row
constexpr int kPer = kRows * kTile / 256;  // elements per thread per array per sub-tile
constexpr int kTargetBlocks = 256;
constexpr int kMinSubtiles = 8;  // per chunk: keeps the partial slab small next to the GEMM

struct Plan {
  int tiles_o, tiles_i, chunks, rows_per_chunk;
};

inline Plan plan(int64_t R, int O, int I) {
  Plan p;
  p.tiles_o = (int)ceil_div(O, kTile);
  p.tiles_i = (int)ceil_div(I, kTile);
  const int64_t subtiles = ceil_div(R > 0 ? R : 1, kRows);
  int64_t chunks = ceil_div(kTargetBlocks, (int64_t)p.tiles_o * p.tiles_i);
  if (chunks > ceil_div(subtiles, kMinSubtiles)) chunks = ceil_div(subtiles, kMinSubtiles);
  if (chunks < 1) chunks = 1;
  const int64_t per = ceil_div(subtiles, chunks);  // sub-tiles per chunk
  p.rows_per_chunk = (int)(per * kRows);
  p.chunks = (int)ceil_div(R > 0 ? R : 1, p.rows_per_chunk);
  return p;
}

__device__ __forceinline__ void load_subtile(const float* __restrict__ a, int64_t n0,
                                             int64_t r_end, int ld, int c0, int ncols,
                                             float (&v)[kPer]) {
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int idx = threadIdx.x + k * 256;
    const int r = idx / kTile, c = idx % kTile;
    const int64_t n = n0 + r;
    const bool ok = (n < r_end) && (c0 + c < ncols);
    const int64_t nn = ok ? n : n0;          // clamped: every lane issues its load
    const int cc = ok ? c0 + c : c0;
    const float x = a[nn * ld + cc];
    v[k] = ok ? x : 0.f;
  }
}

__device__ __forceinline__ void store_subtile(float* s, const float (&v)[kPer]) {
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int idx = threadIdx.x + k * 256;
    s[(idx / kTile) * kLds + idx % kTile] = v[k];
  }
}

__global__ __launch_bounds__(256) void k_linear_wgrad(const float* __restrict__ dy,
                                                      const float* __restrict__ x, int64_t R,
                                                      int O, int I, int rows_per_chunk,
                                                      int tiles_i, float* __restrict__ slab) {
  __shared__ float sA[kRows * kLds];
  __shared__ float sB[kRows * kLds];
  const int chunk = blockIdx.x;
  const int to = blockIdx.y / tiles_i, ti = blockIdx.y % tiles_i;
  const int o0 = to * kTile, i0 = ti * kTile;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int wr = wave >> 1, wc = wave & 1;
  const bool active = (o0 + 32 * wr < O) && (i0 + 32 * wc < I);
  const bool do_bias = (ti == 0) && (wc == 0) && (o0 + 32 * wr < O);

  const int64_t r_begin = (int64_t)chunk * rows_per_chunk;
  const int64_t r_end = min<int64_t>(R, r_begin + rows_per_chunk);
  floatx16 acc;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;
  double bsum = 0.0;

  float va[kPer], vb[kPer];
  load_subtile(dy, r_begin, r_end, O, o0, O, va);
  load_subtile(x, r_begin, r_end, I, i0, I, vb);
  for (int64_t n0 = r_begin; n0 < r_end; n0 += kRows) {
    store_subtile(sA, va);
    store_subtile(sB, vb);
    __syncthreads();
    if (n0 + kRows < r_end) {  // prefetch the next sub-tile under this one's MFMAs
      load_subtile(dy, n0 + kRows, r_end, O, o0, O, va);
      load_subtile(x, n0 + kRows, r_end, I, i0, I, vb);
    }
    if (active) {
#pragma unroll
      for (int s = 0; s < kRows / 2; ++s) {
        const int rr = h * (kRows / 2) + s;  // lane half h takes rows [16h, 16h+16)
        const float a = sA[rr * kLds + 32 * wr + c32];
        const float b = sB[rr * kLds + 32 * wc + c32];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      }
    }
    if (do_bias) {
#pragma unroll
      for (int s = 0; s < kRows / 2; ++s) bsum += (double)sA[(h * (kRows / 2) + s) * kLds + 32 * wr + c32];
    }
    __syncthreads();
  }

  float* out = slab + (size_t)chunk * ((size_t)O * I + O);
  if (active) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = o0 + 32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int i = i0 + 32 * wc + c32;
      if (o < O && i < I) out[(size_t)o * I + i] = acc[r];
    }
  }
  bsum += shfl_xor_d(bsum, 32);
  const int ob = o0 + 32 * wr + c32;
  if (do_bias && h == 0 && ob < O) out[(size_t)O * I + ob] = (float)bsum;
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
  *num_chunks = plan(rows, out_features, in_features).chunks;
  return GINE_OK;
}

extern "C" int gine_linear_wgrad(const float* dy, const float* x, int64_t rows,
                                 int32_t out_features, int32_t in_features, float* slab,
                                 float* dw, float* db, float bias_scale, void* stream) {
  if (rows < 0 || out_features <= 0 || in_features <= 0 || !dw || !slab)
    return GINE_ERR_INVALID;
  if (rows > 0 && (!dy || !x)) return GINE_ERR_INVALID;
  const int O = out_features, I = in_features;
  const Plan p = plan(rows, O, I);
  hipStream_t s = as_stream(stream);
  const int64_t per = (int64_t)O * I + O;
  if (rows == 0) {
    GINE_RETURN_IF_HIP(hipMemsetAsync(slab, 0, sizeof(float) * per, s));
  } else {
    hipLaunchKernelGGL(k_linear_wgrad, dim3(p.chunks, p.tiles_o * p.tiles_i), dim3(256), 0, s,
                       dy, x, rows, O, I, p.rows_per_chunk, p.tiles_i, slab);
    GINE_LAUNCH_STATUS();
  }
  hipLaunchKernelGGL(k_linear_slab_reduce, dim3((unsigned)ceil_div(per, 64)), dim3(256), 0, s,
                     slab, rows == 0 ? 1 : p.chunks, per, (int64_t)O * I, dw, db, bias_scale);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
