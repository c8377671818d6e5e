// Deterministic (run-to-run bit-identical) reductions of per-workgroup fp64 partials.
//
// Kernels that reduce over nodes (parameter gradients, BatchNorm statistics) write one row
// of partial sums per workgroup; a finalize kernel then sums the rows.  The order of every
// addition depends only on the shapes, never on scheduling, so results are reproducible
// without float atomics.  One workgroup of kColsumThreads threads: G = 1024 / W row groups,
// each thread sums every G-th row with 4 interleaved accumulators (independent loads in
// flight, short dependent add chains), then the G group sums are added in group order.
#pragma once

#include "gine_common.hpp"

namespace gine {

constexpr int kColsumThreads = 1024;

// s_tmp: >= kColsumThreads doubles of LDS; s_out: >= W doubles of LDS.
__device__ inline void block_colsum(const double* __restrict__ a, int P, int W, int ld,
                                    double* s_tmp, double* s_out) {
  const int t = threadIdx.x;
  for (int c0 = 0; c0 < W; c0 += kColsumThreads) {
    const int wc = min(kColsumThreads, W - c0);
    const int G = max(1, kColsumThreads / wc);
    const int g = t / wc, c = t % wc;
    if (g < G) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      const double* col = a + c0 + c;
      const size_t step = (size_t)G * ld;
      int p = g;
      for (; p + 3 * G < P; p += 4 * G) {
        const double* r = col + (size_t)p * ld;
        a0 += r[0];
        a1 += r[step];
        a2 += r[2 * step];
        a3 += r[3 * step];
      }
      for (; p < P; p += G) a0 += col[(size_t)p * ld];
      s_tmp[g * wc + c] = (a0 + a1) + (a2 + a3);
    }
    __syncthreads();
    if (t < wc) {
      double s = 0.0;
      for (int gg = 0; gg < G; ++gg) s += s_tmp[gg * wc + t];
      s_out[c0 + t] = s;
    }
    __syncthreads();
  }
}

// Stage 1 of a two-stage fixed-order column reduction of a row-major [P][W] fp64 matrix:
// workgroup (column slab x, row slice y) sums rows [y*L, y*L+L) of 64 columns and writes
// the result IN PLACE into row y*L (the first row of its own slice -- no other workgroup
// reads it).  Stage 2 then reduces the S = ceil(P/L) slice heads with block_colsum using
// row stride L*W.  Pulls the partials through many CUs instead of one.
constexpr int kSliceRows = 32;

namespace {  // one private copy of the kernel per translation unit

__global__ __launch_bounds__(256) void k_colsum_slices(double* __restrict__ a, int P, int W) {
  __shared__ double s_part[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane4 = threadIdx.x >> 6;  // 4 row lanes
  const int r0 = blockIdx.y * kSliceRows;
  const int r1 = min(P, r0 + kSliceRows);
  double acc = 0.0;
  if (c < W) {
    for (int r = r0 + lane4; r < r1; r += 4) acc += a[(size_t)r * W + c];
  }
  s_part[lane4][threadIdx.x & 63] = acc;
  __syncthreads();
  if (lane4 == 0 && c < W) {
    const int j = threadIdx.x & 63;
    a[(size_t)r0 * W + c] = (s_part[0][j] + s_part[1][j]) + (s_part[2][j] + s_part[3][j]);
  }
}

inline int colsum_slices(int P) { return (P + kSliceRows - 1) / kSliceRows; }

// Launch stage 1 on `s`; returns the number of slice heads (stage-2 rows).
inline int launch_colsum_slices(double* a, int P, int W, hipStream_t s) {
  const int S = colsum_slices(P);
  hipLaunchKernelGGL(k_colsum_slices, dim3((W + 63) / 64, S), dim3(256), 0, s, a, P, W);
  return S;
}

}  // namespace

// Fixed-order tree sum of v[0..n) (LDS, clobbered) by one workgroup; result in v[0].
__device__ inline void block_tree_sum(double* v, int n) {
  int m = 1;
  while (m < n) m <<= 1;
  for (int i = n + threadIdx.x; i < m; i += blockDim.x) v[i] = 0.0;
  __syncthreads();
  for (int s = m >> 1; s > 0; s >>= 1) {
    for (int i = threadIdx.x; i < s; i += blockDim.x) v[i] += v[i + s];
    __syncthreads();
  }
}

// Single-launch fixed-order column reduction + finish.  Workgroup b reduces the COLS
// columns fin.col(b, j) (j < COLS; -1 = none) of a row-major [P][ld] fp64 matrix: 256
// threads = COLS columns x (256 / COLS) interleaved row groups, 4 independent accumulators
// per thread, the group sums added in group order through LDS; then fin.finish(b, tot)
// runs with tot[j] = total of column j (LDS, all threads of the workgroup).  Narrow
// workgroups (few columns, many row groups) keep each thread's dependent chain short, so
// one launch of many small workgroups replaces the slice + single-block two-launch form.
template <int COLS, class Fin>
__device__ __forceinline__ void colsum_fin_block(const double* __restrict__ a, int P, int ld,
                                                 const Fin& fin, int b,
                                                 double (*s_part)[COLS], double* s_tot) {
  constexpr int G = 256 / COLS;
  const int j = threadIdx.x % COLS, g = threadIdx.x / COLS;
  const int c = fin.col(b, j);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (c >= 0) {
    const double* colp = a + c;
    const size_t step = (size_t)G * ld;
    int p = g;
    for (; p + 3 * G < P; p += 4 * G) {
      const double* r = colp + (size_t)p * ld;
      a0 += r[0];
      a1 += r[step];
      a2 += r[2 * step];
      a3 += r[3 * step];
    }
    for (; p < P; p += G) a0 += colp[(size_t)p * ld];
  }
  s_part[g][j] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (threadIdx.x < COLS) {
    double t = 0.0;
#pragma unroll 8
    for (int k = 0; k < G; ++k) t += s_part[k][threadIdx.x];
    s_tot[threadIdx.x] = t;
  }
  __syncthreads();
  fin.finish(b, s_tot);
}

template <int COLS, class Fin>
__global__ __launch_bounds__(256) void k_colsum_fin(const double* __restrict__ a, int P, int ld,
                                                    Fin fin) {
  __shared__ double s_part[256 / COLS][COLS];
  __shared__ double s_tot[COLS];
  colsum_fin_block<COLS, Fin>(a, P, ld, fin, blockIdx.x, s_part, s_tot);
}

}  // namespace gine
