// Measurement utility: the HBM copy ceiling that bench.py prices the message-passing kernels
// against (roofline.measured_copy_GBps).  A plain 16-byte-per-lane streaming copy -- the
// form MI355X_MICROARCH.md's measured 6.29 TB/s ceiling comes from -- instead of a torch
// copy_, whose elementwise kernel reached 4.8-5.5 TB/s on the same boxes.
#include "gine_common.hpp"

namespace gine {
namespace {

constexpr int kCopyThreads = 256;
constexpr int kCopyUnroll = 4;

// Each thread moves kCopyUnroll float4 per pass, all loads issued before the stores; the
// passes stride the whole grid, so consecutive lanes touch consecutive 16-byte chunks.
__global__ __launch_bounds__(kCopyThreads) void k_copy_f4(const float4* __restrict__ src,
                                                           float4* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kCopyThreads;
  int64_t i = (int64_t)blockIdx.x * kCopyThreads + threadIdx.x;
  for (; i + (kCopyUnroll - 1) * stride < n; i += kCopyUnroll * stride) {
    float4 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) dst[i + u * stride] = v[u];
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_copy_f4(const void* src, void* dst, int64_t bytes, void* stream) {
  if (!src || !dst || bytes < 0 || bytes % 16 != 0) return GINE_ERR_INVALID;
  const int64_t n = bytes / 16;
  if (n == 0) return GINE_OK;
  const int64_t want = ceil_div(n, (int64_t)kCopyThreads * kCopyUnroll);
  const int grid = (int)(want < 8 * kNumCu ? want : 8 * kNumCu);
  hipLaunchKernelGGL(k_copy_f4, dim3(grid), dim3(kCopyThreads), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), n);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
