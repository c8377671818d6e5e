// BatchNorm1d batch statistics without a finish launch (training mode, momentum given).
//
// The producer of the statistics (the first node-MLP GEMM: k_rowgemm EPI_A1STATS or the
// fused gather kernel; in the backward the dbn GEMM, EPI_DBN) adds each workgroup's fp64
// per-column sums into a device-wide accumulator as 3-word fixed-point integers
//   v = hi + mid * 2^-32 + lo * 2^-64   (hi = rint(v), then the remainder in two words)
// with agent-scope integer atomics: integer addition is order-independent, so the totals --
// and everything computed from them -- are the same bits on every run, with no release
// fence (an agent-scope release writes the XCD's L2 back).  The consumer (the next GEMM,
// whose prologue needs the finished statistics) reads the totals in every workgroup and
// finishes the statistics itself; the accumulator is never reset (see bnacc_total).
// Range and resolution: a per-step column total must stay below 2^63 in magnitude
// (guaranteed: a workgroup sum of 2^52 or more is not added, see below, and grids are
// <= 2048 workgroups); the resolution is 2^-64 absolute, so a column sum of 1e-10 (tiny
// gradients in the backward) keeps ~31 significant bits.
// Non-finite sums follow IEEE/ATen: a NaN, +Inf or -Inf workgroup sum is counted (one
// count word per column, single copy, rare: three 21-bit fields, nan | +inf << 21 |
// -inf << 42 -- the per-step difference of the word is exact mod 2^64 whatever the running
// total, and a step adds at most 2048 per field) instead of being converted, and the consumer rebuilds the
// column total as NaN (a NaN, or both infinities), +Inf or -Inf -- so mean / var / alpha
// come out non-finite exactly where ATen's batch_norm does.  A finite workgroup sum of
// magnitude >= 2^52 (an activation column far beyond fp32 BatchNorm's useful range) is
// counted as NaN: the statistics turn NaN, loudly, instead of wrapping.
// Pairing: every producer launch must be followed by exactly one consumer launch on the
// same accumulator.  The producer bumps a phase word; the consumer records the phase it
// consumed and, if the phase moved by anything but 1 since the last consumer (a producer
// ran without its consumer, e.g. after a host-side error between the two), emits NaN
// statistics for that step instead of silently mixing steps.
// Layout of acc (int64), W = 2 * D words per quantity (sum | sum of squares, or in the
// backward sum dbn | sum dbn * xhat):
//   [replica: R][hi | mid | lo: W]   [count: W]
//   [snapshot: 2][hi | mid | lo | count: W]   phase   consumed[2]   barrier[kBarWords]
// The barrier words (zero at allocation) belong to the one-launch layer forward
// (gine_mp_fwd_layer), whose producer and consumer halves are separated by a grid barrier
// instead of a launch boundary (grid_barrier below); one of them counts barrier failures.
#pragma once

#include "gine_common.hpp"

namespace gine {

// Workgroups add into replica blockIdx % R: same-address atomics serialise at the memory
// side (256 workgroups on one copy cost ~4 us at the end of the producer), while every
// consumer workgroup reads every replica.  Measured on the cfg2 step (r02_s21, A/B twice):
// R = 2 / 4 / 8 / 16 -> 0.579 / 0.572 / 0.586 / 0.605 ms.  The consumer sums the replicas'
// integers (exact) before the one conversion to double.
#ifndef GINE_BNACC_REPLICAS
#define GINE_BNACC_REPLICAS 4
#endif
constexpr int kBnAccReplicas = GINE_BNACC_REPLICAS;
constexpr int kBnAccWords = 3;   // hi, mid, lo
constexpr int kBnAccCounts = 1;  // nan | +inf << 21 | -inf << 42
constexpr int kBnAccCountBits = 21;
constexpr int kBnAccSnap = kBnAccWords + kBnAccCounts;
// grid barrier: one 128-byte line each for the global arrival count, the failure count, the
// 8 per-XCD arrival counts and the 8 per-XCD generations
constexpr int kBarLine = 16;  // int64 words per line
constexpr int kBarWords = (2 + 2 * kNumXcd) * kBarLine;
constexpr int kBarFailWord = kBarLine;  // (barrier-area word index: the failure count)

__host__ __device__ constexpr int64_t bnacc_words(int D) {
  return (int64_t)(kBnAccReplicas * kBnAccWords + kBnAccCounts + 2 * kBnAccSnap) * 2 * D + 3 +
         kBarWords;
}

__device__ __forceinline__ long long* bnacc_counts(long long* acc, int W) {
  return acc + (size_t)kBnAccReplicas * kBnAccWords * W;
}
__device__ __forceinline__ long long* bnacc_snap(long long* acc, int W) {
  return acc + (size_t)(kBnAccReplicas * kBnAccWords + kBnAccCounts) * W;
}
__device__ __forceinline__ long long* bnacc_phase(long long* acc, int W) {
  return acc + (size_t)(kBnAccReplicas * kBnAccWords + kBnAccCounts + 2 * kBnAccSnap) * W;
}

__device__ __forceinline__ long long* bnacc_barrier(long long* acc, int W) {
  return bnacc_phase(acc, W) + 3;
}

// A grid barrier of this accumulator has failed (its failure word is non-zero) since the host
// last zeroed it (raincast_gnn.functional.check_grid_barriers): sticky -- every consumer then
// finishes NaN statistics and leaves the running statistics alone (see bnacc_total).  LIVE:
// an agent-scope atomic load (inside the launch whose workgroups may be adding to it).
template <bool LIVE = false>
__device__ __forceinline__ bool bnacc_poisoned(long long* acc, int W) {
  long long* w = bnacc_barrier(acc, W) + kBarFailWord;
  if constexpr (LIVE) return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  else return *w != 0;
}

// PHASE = false: the caller (gine_mp_fwd_layer) keeps the phase word itself.
template <bool PHASE = true>
__device__ __forceinline__ void bnacc_add(long long* acc, int W, int c, double v) {
  if (__builtin_fabs(v) < 4503599627370496.0) {  // 2^52; false for NaN
    long long* r = acc + (size_t)(blockIdx.x % kBnAccReplicas) * kBnAccWords * W;
    const double h = __builtin_rint(v);
    const double f = (v - h) * 4294967296.0;  // exact: |v - h| <= 1/2, power-of-2 scale
    const double m = __builtin_rint(f);
    const double l = __builtin_rint((f - m) * 4294967296.0);
    // a zero word is not added (the identity; the backward's sums of small gradients mostly
    // have hi == 0): fewer same-address atomics for the memory side to serialise
    if (h != 0.0)
      __hip_atomic_fetch_add(r + c, (long long)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (m != 0.0)
      __hip_atomic_fetch_add(r + W + c, (long long)m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (l != 0.0)
      __hip_atomic_fetch_add(r + 2 * W + c, (long long)l, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  } else {  // NaN, +-Inf, or out of range (counted as NaN)
    const int k = (v == __builtin_inf()) ? 1 : (v == -__builtin_inf()) ? 2 : 0;
    __hip_atomic_fetch_add(bnacc_counts(acc, W) + c, 1ll << (kBnAccCountBits * k),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (PHASE && blockIdx.x == 0 && c == 0) {  // one producer launch = one phase (read by the consumer)
    long long* ph = bnacc_phase(acc, W);
    *ph = *ph + 1;
  }
}

// This step's total of word t (< W).  The replicas and counts only ever grow (mod 2^64):
// the step's sum is the current total minus the snapshot the previous consumer took.  The
// snapshot slot alternates with the phase, so workgroup 0 (write_snap) stores this step's
// totals into the slot nobody reads in this launch -- no atomics, no reset, nothing
// host-side (HIP-graph replays keep working).  Plain (L2-cached) loads: the producer's
// atomics were performed at the memory side and the consumer is a later kernel on the
// stream, whose start invalidates the L2s.  The consumed phase is kept the same way: a
// consumer at phase p checks slot (p-1)&1 == p-1 (what a correctly paired previous
// consumer wrote) and workgroup 0 writes p into slot p&1 (bnacc_mark_consumed).
// LIVE (the one-launch layer forward, after its grid barrier): the replica and count words
// are read with agent-scope atomic loads -- the producer's atomics of the same launch were
// performed at the memory side, and no launch boundary has invalidated this XCD's L2 since
// -- and the phase / consumed words come from the caller (read before the barrier).
template <bool LIVE = false>
__device__ __forceinline__ double bnacc_total(long long* acc, int W, int t, bool write_snap,
                                              long long ph_live = 0,
                                              long long consumed_live = 0) {
  auto rd = [](long long* p) -> unsigned long long {
    if constexpr (LIVE)
      return (unsigned long long)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      return (unsigned long long)*p;
  };
  unsigned long long cur_v[kBnAccSnap];
#pragma unroll
  for (int k = 0; k < kBnAccSnap; ++k) cur_v[k] = 0;
#pragma unroll
  for (int r = 0; r < kBnAccReplicas; ++r) {
#pragma unroll
    for (int k = 0; k < kBnAccWords; ++k)
      cur_v[k] += rd(acc + (size_t)(r * kBnAccWords + k) * W + t);
  }
  long long* cnt = bnacc_counts(acc, W);
#pragma unroll
  for (int k = 0; k < kBnAccCounts; ++k) cur_v[kBnAccWords + k] = rd(cnt + k * W + t);
  long long* phw = bnacc_phase(acc, W);
  const long long ph = LIVE ? ph_live : phw[0];
  const long long consumed = LIVE ? consumed_live : phw[1 + ((ph - 1) & 1)];
  long long* prev = bnacc_snap(acc, W) + ((ph - 1) & 1) * kBnAccSnap * W;
  long long* cur = bnacc_snap(acc, W) + (ph & 1) * kBnAccSnap * W;
  long long d[kBnAccSnap];
#pragma unroll
  for (int k = 0; k < kBnAccSnap; ++k)
    d[k] = (long long)(cur_v[k] - (unsigned long long)prev[k * W + t]);
  if (write_snap) {
    // read-before-write within the thread: slot `cur` is not read in this launch
#pragma unroll
    for (int k = 0; k < kBnAccSnap; ++k) cur[k * W + t] = (long long)cur_v[k];
  }
  const unsigned long long fm = (1ull << kBnAccCountBits) - 1, cnt_d = (unsigned long long)d[3];
  const bool n_nan = (cnt_d & fm) != 0, n_pinf = ((cnt_d >> kBnAccCountBits) & fm) != 0,
             n_ninf = ((cnt_d >> (2 * kBnAccCountBits)) & fm) != 0;
  // a grid barrier of this accumulator has failed since the host last zeroed it: its
  // snapshot and phase words may have been written from incomplete totals (workgroup 0 of
  // the failed launch) while late workgroups' atomics landed after them, so every later
  // statistic of this accumulator is NaN until the host's reset (check_grid_barriers) --
  // never finite but wrong
  const bool poisoned = bnacc_poisoned<LIVE>(acc, W);
  const bool nan = n_nan || (n_pinf && n_ninf) || ph - consumed != 1 || poisoned;
  double v;
  if (nan) v = __builtin_nan("");
  else if (n_pinf) v = __builtin_inf();
  else if (n_ninf) v = -__builtin_inf();
  else
    v = ((double)d[2] * 5.421010862427522e-20 + (double)d[1] * 2.3283064365386963e-10) +
        (double)d[0];  // lo * 2^-64 + mid * 2^-32 + hi, smallest first
  return v;
}

// Grid-wide barrier of a launch whose workgroups are all resident at once (one per CU; the
// host checks the occupancy before choosing such a launch): one thread per workgroup, after a
// __syncthreads.  Two levels, every word on its own 128-byte line: a workgroup arrives on its
// XCD's count (blocks are dealt round-robin, so b % 8 is its XCD), the last arriver of each
// XCD on the global count, and the last of those bumps the 8 per-XCD generations, which each
// workgroup polls on its own XCD's line.  Same-address atomics serialise at the memory side
// (256 arrivals on one word cost ~4 us, gine_bnacc.hpp replicas), and 256 pollers on one
// line contend with the arrivals; this way at most 32 + 8 arrivals and 32 pollers share a
// line.  Counts are reset by their last arriver, generations only grow, so the words serve
// any grid size launch after launch (HIP-graph replays included).  Relaxed agent-scope
// atomics: the barrier orders only the producer's fixed-point atomics (performed at the
// memory side; the arriving thread waited for every one of its workgroup's before the
// __syncthreads, see the callers) against the consumer's atomic loads -- no L2 write-back or
// invalidate.
// A grid that was not co-resident after all (other work holding CUs: another process on the
// device, a kernel on another stream) cannot complete: a watchdog on the constant 100 MHz
// clock gives up after ~2 s rather than hanging the device, adds 1 to the launch's failure
// word (kBarFailWord, line 1 of the barrier area) and returns false.  The caller then
// poisons what it computes from the incomplete totals (NaN BatchNorm statistics, no running
// statistics update), and the host turns a non-zero failure word into GineError
// (gine_bn_acc_barrier_failures, raincast_gnn.functional.check_grid_barriers).  The late
// workgroups of such a launch complete the barrier among themselves (their arrival completes
// the counts) and see complete totals.
__device__ __forceinline__ bool grid_barrier(long long* bar, int nblocks) {
  const int b = blockIdx.x, x = b % kNumXcd;
  long long* glob = bar;
  long long* cnt = bar + (2 + x) * kBarLine;
  long long* gen = bar + (2 + kNumXcd + x) * kBarLine;
  const int here = nblocks / kNumXcd + (x < nblocks % kNumXcd ? 1 : 0);
  const int xcds = nblocks < kNumXcd ? nblocks : kNumXcd;
  const long long g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the generation is read before the arrival is performed (else the last arriver's bump
  // could be seen here as the old generation)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (__hip_atomic_fetch_add(cnt, 1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == here - 1) {
    __hip_atomic_store(cnt, 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(glob, 1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        xcds - 1) {
      __hip_atomic_store(glob, 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int y = 0; y < xcds; ++y)
        __hip_atomic_fetch_add(bar + (2 + kNumXcd + y) * kBarLine, 1ll, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // ~2 s: give up, loudly
      __hip_atomic_fetch_add(bar + kBarFailWord, 1ll, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return false;
    }
  }
  return true;
}

// Record the consumed phase (one thread of workgroup 0 of the consumer).
__device__ __forceinline__ void bnacc_mark_consumed(long long* acc, int W) {
  long long* phw = bnacc_phase(acc, W);
  const long long ph = phw[0];
  phw[1 + (ph & 1)] = ph;
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
