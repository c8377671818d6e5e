// Precision of the split-bf16 MFMA product (gine_bf16x3.hpp) against fp64, next to the fp32
// MFMA chain: C[32x32] = A[32xK] B[Kx32] for random operands, K = 128, one wave.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../raincast-gnn_amd/csrc -I../include
//         bf16x3_precision.hip -o bin/bf16x3_precision
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gine_bf16x3.hpp"

using namespace gine;
constexpr int K = 128;

// A row-major [32][K], B row-major [K][32]; mode 0: fp32 MFMA, 1: bf16x3 (6), 2: 8 products
__global__ void k_gemm(const float* A, const float* B, float* C, int mode) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f32x16_t acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  if (mode == 0) {
    for (int s = 0; s < K / 2; ++s)  // lane half h: k = h*K/2 + s
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[r * K + h * (K / 2) + s],
                                                 B[(h * (K / 2) + s) * 32 + r], acc, 0, 0, 0);
  } else {
    for (int s = 0; s < K / 16; ++s) {
      float a[8], b[8];
      for (int j = 0; j < 8; ++j) {
        a[j] = A[r * K + h * (K / 2) + 8 * s + j];
        b[j] = B[(h * (K / 2) + 8 * s + j) * 32 + r];
      }
      const Bf16x3 x = split8(make_float4(a[0], a[1], a[2], a[3]), make_float4(a[4], a[5], a[6], a[7]));
      const Bf16x3 y = split8(make_float4(b[0], b[1], b[2], b[3]), make_float4(b[4], b[5], b[6], b[7]));
      if (mode == 2) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x.l, y.m, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x.m, y.l, acc, 0, 0, 0);
      }
      acc = mfma_bf16x3(x, y, acc);
    }
  }
  for (int i = 0; i < 16; ++i) C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[i];
}

int main() {
  srand(1);
  std::vector<float> A(32 * K), B(K * 32), C(32 * 32);
  double worst[3] = {0, 0, 0}, norm_err[3] = {0, 0, 0}, norm_ref = 0;
  float *dA, *dB, *dC;
  hipMalloc(&dA, A.size() * 4);
  hipMalloc(&dB, B.size() * 4);
  hipMalloc(&dC, C.size() * 4);
  for (int trial = 0; trial < 20; ++trial) {
    for (auto& v : A) v = (float)((rand() / (double)RAND_MAX - 0.5) * 4.0);
    for (auto& v : B) v = (float)((rand() / (double)RAND_MAX - 0.5) * 0.2);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 3; ++mode) {
      hipLaunchKernelGGL(k_gemm, dim3(1), dim3(64), 0, 0, dA, dB, dC, mode);
      hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          double ref = 0, mag = 0;
          for (int k = 0; k < K; ++k) {
            ref += (double)A[i * K + k] * B[k * 32 + j];
            mag += fabs((double)A[i * K + k] * B[k * 32 + j]);
          }
          const double e = fabs(C[i * 32 + j] - ref) / mag;
          worst[mode] = e > worst[mode] ? e : worst[mode];
          norm_err[mode] += (C[i * 32 + j] - ref) * (C[i * 32 + j] - ref);
          if (mode == 0) norm_ref += ref * ref;
        }
    }
  }
  const char* names[3] = {"fp32 mfma 32x32x2", "bf16x3 (6 products)", "bf16x3 (8 products)"};
  for (int m = 0; m < 3; ++m)
    printf("%-22s max |err| / sum|a b| = %.3e   normwise rel = %.3e\n", names[m], worst[m],
           sqrt(norm_err[m] * 3 / norm_ref));
  return 0;
}
