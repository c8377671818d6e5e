// Probe (not part of the library): forms of a 16-byte-per-lane HBM copy, for choosing the
// copy-ceiling kernel bench.py prices the message-passing kernels against (csrc/gine_probe.hip).
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/copy_probe.hip -o <dir>/copy_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int T, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(T) void k_block(const f4* __restrict__ s, f4* __restrict__ d, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * T * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * T;
    if (NTL) v[u] = i < n ? __builtin_nontemporal_load(s + i) : f4{0, 0, 0, 0};
    else v[u] = i < n ? s[i] : f4{0, 0, 0, 0};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * T;
    if (i < n) {
      if (NTS) __builtin_nontemporal_store(v[u], d + i);
      else d[i] = v[u];
    }
  }
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_stride(const f4* __restrict__ s, f4* __restrict__ d, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * T;
  int64_t i = (int64_t)blockIdx.x * T + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = s[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * stride] = v[u];
  }
  for (; i < n; i += stride) d[i] = s[i];
}

extern "C" int copy_probe(int mode, const void* src, void* dst, int64_t bytes, void* stream) {
  const int64_t n = bytes / 16;
  const f4* s = (const f4*)src;
  f4* d = (f4*)dst;
  hipStream_t st = (hipStream_t)stream;
  auto blocks = [&](int T, int U) { return dim3((unsigned)((n + (int64_t)T * U - 1) / ((int64_t)T * U))); };
  switch (mode) {
    case 0: hipLaunchKernelGGL((k_block<256, 8, true, true>), blocks(256, 8), dim3(256), 0, st, s, d, n); break;
    case 1: hipLaunchKernelGGL((k_block<256, 8, false, false>), blocks(256, 8), dim3(256), 0, st, s, d, n); break;
    case 2: hipLaunchKernelGGL((k_block<256, 8, false, true>), blocks(256, 8), dim3(256), 0, st, s, d, n); break;
    case 3: hipLaunchKernelGGL((k_block<512, 4, false, false>), blocks(512, 4), dim3(512), 0, st, s, d, n); break;
    case 4: hipLaunchKernelGGL((k_block<256, 4, false, false>), blocks(256, 4), dim3(256), 0, st, s, d, n); break;
    case 5: hipLaunchKernelGGL((k_block<256, 16, false, false>), blocks(256, 16), dim3(256), 0, st, s, d, n); break;
    case 6: hipLaunchKernelGGL((k_stride<256, 4>), dim3(2048), dim3(256), 0, st, s, d, n); break;
    case 7: hipLaunchKernelGGL((k_stride<256, 8>), dim3(8192), dim3(256), 0, st, s, d, n); break;
    case 8: hipLaunchKernelGGL((k_block<1024, 4, false, false>), blocks(1024, 4), dim3(1024), 0, st, s, d, n); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
