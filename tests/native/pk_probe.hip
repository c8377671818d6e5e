// Detector probe for tests/test_isa.py: the forward message's per-edge arithmetic
// (gine_edge.hpp fwd_edge) on f4v vectors -- code the compiler turns into packed-FP32 VALU
// instructions unless the library's NOPK feature switch (csrc/Makefile) is on the command line.
#include "gine_edge.hpp"

__global__ void pk_probe(const float4* __restrict__ x, const float* __restrict__ a,
                         const float4* __restrict__ w, const float4* __restrict__ b,
                         float4* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  gine::f4v acc = gine::f4v_zero();
  const gine::f4v wv = *reinterpret_cast<const gine::f4v*>(&w[threadIdx.x & 31]);
  const gine::f4v bv = *reinterpret_cast<const gine::f4v*>(&b[threadIdx.x & 31]);
  for (int j = 0; j < n; ++j)
    gine::fwd_edge<true>(acc, *reinterpret_cast<const gine::f4v*>(&x[i + j]), a[i + j], wv, bv);
  out[i] = gine::to_float4(acc);
}
