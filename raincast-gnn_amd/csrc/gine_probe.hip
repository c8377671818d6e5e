// Measurement utility: the HBM copy ceiling that bench.py prices the message-passing kernels
// against (roofline.measured_copy_GBps).  A plain 16-byte-per-lane streaming copy -- the
// form MI355X_MICROARCH.md's measured 6.29 TB/s ceiling comes from -- instead of a torch
// copy_, whose elementwise kernel reached 4.8-5.5 TB/s on the same boxes.
#include "gine_common.hpp"

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

}  // namespace
}  // namespace gine

using namespace gine;

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
