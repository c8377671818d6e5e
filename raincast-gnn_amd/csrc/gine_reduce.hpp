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

}  // namespace gine
