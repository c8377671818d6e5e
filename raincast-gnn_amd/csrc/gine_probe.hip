// Measurement utility: the HBM copy ceiling that bench.py prices the message-passing kernels
// against (roofline.measured_copy_GBps).  A plain 16-byte-per-lane streaming copy -- the
// form MI355X_MICROARCH.md's measured 6.29 TB/s ceiling comes from -- instead of a torch
// copy_, whose elementwise kernel reached 4.8-5.5 TB/s on the same boxes.
#include "gine_common.hpp"
#include "gine_bf16x3.hpp"

namespace gine {
namespace {

constexpr int kCopyThreads = 256;
constexpr int kCopyUnroll = 4;

// One workgroup moves one contiguous 16 KiB block (kCopyUnroll float4 per thread, lane-
// consecutive 16-byte chunks, every load issued before the first store): the fastest of the
// forms measured with tools/copy_probe.py (profiles/r05_s06_copy_forms.txt, 1 and 4 GiB):
// 5.75-5.79 TB/s, against 5.0-5.5 for 32-64 KiB blocks, non-temporal loads / stores, 512-1024
// threads, and 4.4-4.9 for grid-stride loops (the round-4 form) and 4.6-4.8 for torch's
// copy_.  None reached the guide's 6.29 TB/s float4-copy figure on these boxes.
typedef float f4n __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(kCopyThreads) void k_copy_f4(const f4n* __restrict__ src,
                                                           f4n* __restrict__ dst, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * kCopyThreads * kCopyUnroll + threadIdx.x;
  f4n v[kCopyUnroll];
#pragma unroll
  for (int u = 0; u < kCopyUnroll; ++u) {
    const int64_t i = base + (int64_t)u * kCopyThreads;
    v[u] = i < n ? src[i] : f4n{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < kCopyUnroll; ++u) {
    const int64_t i = base + (int64_t)u * kCopyThreads;
    if (i < n) dst[i] = v[u];
  }
}

// Measurement utility: the cost of one 32x32 output block of the row GEMMs' split-bf16 chain
// (K = 128: 8 steps of split8 + 6 v_mfma_f32_32x32x16_bf16), per wave, in shader-clock
// ticks, for the forms a kernel can take (tools/chain_micro.py):
//   0: A rows read from LDS and split in the loop (the row GEMMs / layer kernels);
//   1: A pre-split bf16 planes read from LDS (a staging pass would split them once);
//   2: MFMAs only (A planes held in registers);
//   3: form 0 over two tiles with the two chains interleaved step by step;
//   4: form 0 software-pipelined: the split of step s+1 scheduled between the dependent
//      MFMAs of step s (sched_group_barrier).
typedef float floatx16p __attribute__((ext_vector_type(16)));
constexpr int kChainLD = 132;
template <int V>
__global__ __launch_bounds__(256) void k_chain_probe(int reps, float* __restrict__ sink,
                                                     long long* __restrict__ ticks) {
  __shared__ __attribute__((aligned(16))) float s_x[2][32 * kChainLD];
  __shared__ __attribute__((aligned(16))) uint16_t s_p[3][32 * 136];
  const int lane = threadIdx.x % kWave, wave = threadIdx.x / kWave;
  const int h = lane >> 5, c32 = lane & 31;
  for (int i = threadIdx.x; i < 2 * 32 * kChainLD; i += 256)
    (&s_x[0][0])[i] = (float)((i * 2654435761u) >> 8) * 1e-7f - 0.8f;
  for (int i = threadIdx.x; i < 3 * 32 * 136; i += 256) (&s_p[0][0])[i] = (uint16_t)(i * 77);
  float bf[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) bf[k] = 0.01f * (float)((k * 7 + c32 + wave) % 13) - 0.06f;
  BPlanes<64> bp;
  bp.from(bf);
  __syncthreads();
  floatx16p tot;
#pragma unroll
  for (int i = 0; i < 16; ++i) tot[i] = 0.f;
  Bf16x3 areg[8];
  if constexpr (V == 2) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float* ar = &s_x[0][c32 * kChainLD + h * 64 + 8 * s];
      areg[s] = split8(*reinterpret_cast<const float4*>(ar),
                       *reinterpret_cast<const float4*>(ar + 4));
    }
  }
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    floatx16p acc, acc2;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = acc2[i] = 0.f;
    const float* arow = &s_x[r & 1][c32 * kChainLD + h * 64];
    const float* brow = &s_x[(r + 1) & 1][c32 * kChainLD + h * 64];
    if constexpr (V == 4) {
      // split of step s+1 issued between the dependent MFMAs of step s
      Bf16x3 cur = split8(*reinterpret_cast<const float4*>(&arow[0]),
                          *reinterpret_cast<const float4*>(&arow[4]));
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        Bf16x3 nxt = cur;
        if (s + 1 < 8)
          nxt = split8(*reinterpret_cast<const float4*>(&arow[8 * s + 8]),
                       *reinterpret_cast<const float4*>(&arow[8 * s + 12]));
        acc = mfma_bf16x3(cur, bp.f[s], acc);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);  // up to 8 VALU
        }
        cur = nxt;
      }
    }
#pragma unroll
    for (int s = 0; s < (V == 4 ? 0 : 8); ++s) {
      if constexpr (V == 0 || V == 3) {
        acc = mfma_bf16x3(split8(*reinterpret_cast<const float4*>(&arow[8 * s]),
                                 *reinterpret_cast<const float4*>(&arow[8 * s + 4])),
                          bp.f[s], acc);
        if constexpr (V == 3)
          acc2 = mfma_bf16x3(split8(*reinterpret_cast<const float4*>(&brow[8 * s]),
                                    *reinterpret_cast<const float4*>(&brow[8 * s + 4])),
                             bp.f[s], acc2);
      } else if constexpr (V == 4) {
        // (the pipelined form is the loop below; this branch is not taken)
      } else if constexpr (V == 1) {
        const uint16_t* pr = &s_p[0][c32 * 136 + h * 64 + 8 * s] + (r & 1) * 8;
        Bf16x3 a;
        a.h = *reinterpret_cast<const bf16x8_t*>(pr);
        a.m = *reinterpret_cast<const bf16x8_t*>(pr + 32 * 136);
        a.l = *reinterpret_cast<const bf16x8_t*>(pr + 2 * 32 * 136);
        acc = mfma_bf16x3(a, bp.f[s], acc);
      } else {
        acc = mfma_bf16x3(areg[s], bp.f[s], acc);
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) tot[i] += acc[i] + acc2[i];
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) sum += tot[i];
  sink[blockIdx.x * 256 + threadIdx.x] = sum;
  if (lane == 0) ticks[blockIdx.x * 4 + wave] = t1 - t0;
}

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_probe_chain(int32_t variant, int32_t reps, int32_t blocks, float* sink,
                                long long* ticks, void* stream) {
  if (!sink || !ticks || reps <= 0 || blocks <= 0 || blocks > 4096) return GINE_ERR_INVALID;
  hipStream_t s = as_stream(stream);
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_chain_probe<0>, dim3(blocks), dim3(256), 0, s, reps, sink, ticks); break;
    case 1: hipLaunchKernelGGL(k_chain_probe<1>, dim3(blocks), dim3(256), 0, s, reps, sink, ticks); break;
    case 2: hipLaunchKernelGGL(k_chain_probe<2>, dim3(blocks), dim3(256), 0, s, reps, sink, ticks); break;
    case 3: hipLaunchKernelGGL(k_chain_probe<3>, dim3(blocks), dim3(256), 0, s, reps, sink, ticks); break;
    case 4: hipLaunchKernelGGL(k_chain_probe<4>, dim3(blocks), dim3(256), 0, s, reps, sink, ticks); break;
    default: return GINE_ERR_INVALID;
  }
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_copy_f4(const void* src, void* dst, int64_t bytes, void* stream) {
  if (!src || !dst || bytes < 0 || bytes % 16 != 0) return GINE_ERR_INVALID;
  const int64_t n = bytes / 16;
  if (n == 0) return GINE_OK;
  const int64_t grid = ceil_div(n, (int64_t)kCopyThreads * kCopyUnroll);
  if (grid >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  hipLaunchKernelGGL(k_copy_f4, dim3(grid), dim3(kCopyThreads), 0, as_stream(stream),
                     reinterpret_cast<const f4n*>(src), reinterpret_cast<f4n*>(dst), n);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
