// BatchNorm1d batch statistics without a finish launch (training mode, momentum given).
//
// The producer of the statistics (the first node-MLP GEMM: k_rowgemm EPI_A1STATS or the
// fused gather kernel) adds each workgroup's fp64 per-column sums into a device-wide
// accumulator as 2-word fixed-point integers (hi = v * 2^16 rounded, lo = the remainder *
// 2^32 rounded) with agent-scope integer atomics: integer addition is order-independent, so
// the totals -- and everything computed from them -- are the same bits on every run, with
// no release fence (an agent-scope release writes the XCD's L2 back).  The consumer (the
// second GEMM, whose prologue needs alpha / shift) reads the 2-word totals in every
// workgroup and finishes the statistics itself (workgroup 0 also writes bn_save and the
// running statistics); the accumulator is never reset (see bnacc_total).
// Exact for |sum| < 2^37 per column (beyond that the conversion to double rounds, still
// deterministically); the per-workgroup rounding is below 2^-49.
// Layout of acc (int64): [replica: 8][hi: W][lo: W], [snapshot: 2][hi: W][lo: W], phase;
// W = 2 * D (sum | sum of squares).  Every producer launch must be followed by exactly one
// consumer launch on the same accumulator.
#pragma once

#include "gine_common.hpp"

namespace gine {

// Workgroups of one XCD (blockIdx % 8 under round-robin dispatch) add into their own
// replica: same-address atomics serialise at the memory side, and 256 workgroups on one
// copy cost ~4 us at the end of the producer; 8 replicas make 32-deep chains.  The consumer
// sums the replicas' integers (exact) before the one conversion to double.
constexpr int kBnAccReplicas = 8;

// Word offsets after the replicas: snapshots [2][hi W | lo W], then the phase counter.
__device__ __forceinline__ long long* bnacc_snap(long long* acc, int W) {
  return acc + (size_t)kBnAccReplicas * 2 * W;
}
__device__ __forceinline__ long long* bnacc_phase(long long* acc, int W) {
  return acc + (size_t)kBnAccReplicas * 2 * W + 4 * W;
}

__device__ __forceinline__ void bnacc_add(long long* acc, int W, int c, double v) {
  long long* r = acc + (size_t)(blockIdx.x % kBnAccReplicas) * 2 * W;
  const double sv = v * 65536.0;                  // 2^16
  const double h = rint(sv);
  const double l = rint((sv - h) * 4294967296.0);  // 2^32: |l| <= 2^31
  __hip_atomic_fetch_add(r + c, (long long)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(r + W + c, (long long)l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x == 0 && c == 0) {  // one producer launch = one phase (read by the consumer)
    long long* ph = bnacc_phase(acc, W);
    *ph = *ph + 1;
  }
}

// This step's total of word t (< W).  The replicas only ever grow (mod 2^64): the step's sum
// is the replicas' total minus the snapshot the previous consumer took.  The snapshot slot
// alternates with the phase, so workgroup 0 (write_snap) stores this step's totals into the
// slot nobody reads in this launch -- no atomics, no reset, nothing host-side (HIP-graph
// replays keep working).  Plain (L2-cached) loads: the producer's atomics were performed at
// the memory side and the consumer is a later kernel on the stream, whose start invalidates
// the L2s.
__device__ __forceinline__ double bnacc_total(long long* acc, int W, int t, bool write_snap) {
  unsigned long long h = 0, l = 0;
#pragma unroll
  for (int r = 0; r < kBnAccReplicas; ++r) {
    h += (unsigned long long)acc[(size_t)r * 2 * W + t];
    l += (unsigned long long)acc[(size_t)r * 2 * W + W + t];
  }
  const long long ph = *bnacc_phase(acc, W);
  long long* prev = bnacc_snap(acc, W) + ((ph - 1) & 1) * 2 * W;
  long long* cur = bnacc_snap(acc, W) + (ph & 1) * 2 * W;
  const long long dh = (long long)(h - (unsigned long long)prev[t]);
  const long long dl = (long long)(l - (unsigned long long)prev[W + t]);
  if (write_snap) {
    cur[t] = (long long)h;
    cur[W + t] = (long long)l;
  }
  return (double)dh * (1.0 / 65536.0) + (double)dl * (1.0 / 281474976710656.0);
}

struct BnFwdParams {
  const float *gamma, *beta;
  float *rmean, *rvar;
  int64_t* nbt;
  float* bn_save;
  int64_t N;
  float momentum, bn_eps;
  int update_running;
};

// mean / biased var -> (alpha, shift); workgroup 0 (write) also stores bn_save
// [mean | invstd | alpha | shift] and the running statistics (momentum, unbiased var) --
// the arithmetic of gine_bn_fwd_finalize.
__device__ __forceinline__ void bn_finish_channel(const BnFwdParams& q, int D, int c,
                                                  double s1, double s2, bool write,
                                                  float* alpha_out, float* shift_out) {
  const double mean = s1 / (double)q.N;
  double var = s2 / (double)q.N - mean * mean;
  if (var < 0.0) var = 0.0;
  const double invstd = 1.0 / sqrt(var + (double)q.bn_eps);
  const double g = q.gamma ? (double)q.gamma[c] : 1.0;
  const double bt = q.beta ? (double)q.beta[c] : 0.0;
  const double alpha = g * invstd;
  const float alpha_f = (float)alpha, shift_f = (float)(bt - mean * alpha);
  *alpha_out = alpha_f;
  *shift_out = shift_f;
  if (!write) return;
  if (q.update_running && q.rmean != nullptr) {
    const double f = (double)q.momentum;
    const double unbiased = q.N > 1 ? var * (double)q.N / (double)(q.N - 1) : var;
    q.rmean[c] = (float)(f * mean + (1.0 - f) * (double)q.rmean[c]);
    q.rvar[c] = (float)(f * unbiased + (1.0 - f) * (double)q.rvar[c]);
  }
  q.bn_save[c] = (float)mean;
  q.bn_save[D + c] = (float)invstd;
  q.bn_save[2 * D + c] = alpha_f;
  q.bn_save[3 * D + c] = shift_f;
}

}  // namespace gine
