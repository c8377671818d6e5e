// Microbenchmark of the weight-gradient engine (raincast-gnn_amd/csrc/gine_wgrad.hpp) on
// the node-MLP shape: Z = 2 products [128 x 128] over N rows, plain fp32 operands.
// Build variants with -DGINE_WG_VARIANT=<bits> (see the header) to attribute the time:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I raincast-gnn_amd/csrc \
//         -DGINE_WG_VARIANT=1 tools/wg_micro.hip -o /tmp/wg1 && /tmp/wg1 16000
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gine_slab.hpp"
#include "gine_wgrad.hpp"

using namespace gine;

struct PlainSrc {
  static constexpr int kZ = 2;
  const float* p[2];
  const float* q[2];
  int D;
  struct Raw {
    float4 v;
  };
  struct Col {};
  template <int Z> __device__ int i_dim(int I) const { return I; }
  template <int Z> __device__ Col p_col(int) const { return Col{}; }
  template <int Z> __device__ Col q_col(int) const { return Col{}; }
  template <int Z> __device__ Raw p_load(int64_t n, int c) const {
    return Raw{reinterpret_cast<const float4*>(p[Z] + n * D)[c]};
  }
  template <int Z> __device__ Raw q_load(int64_t n, int c) const {
    return Raw{reinterpret_cast<const float4*>(q[Z] + n * D)[c]};
  }
  template <int Z> __device__ float4 p_xform(const Raw& r, const Col&) const { return r.v; }
  template <int Z> __device__ float4 q_xform(const Raw& r, const Col&) const { return r.v; }
};

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 16000;
  const int D = 128, reps = 50;
  std::vector<float> h(N * D);
  for (auto& v : h) v = (float)(rand() % 1000) / 1000.f - 0.5f;
  float* buf[4];
  for (auto& b : buf) {
    CK(hipMalloc(&b, sizeof(float) * N * D));
    CK(hipMemcpy(b, h.data(), sizeof(float) * N * D, hipMemcpyHostToDevice));
  }
  const WgPlan p = wg_plan(N, D, D, 2, 64);
  const size_t per = (size_t)D * D + D;
  float* slab;
  CK(hipMalloc(&slab, sizeof(float) * per * p.chunks * 2));
  PlainSrc src{{buf[0], buf[1]}, {buf[2], buf[3]}, D};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    launch_wgrad_engine<64>(src, N, D, D, 2 * p.tiles_o * p.tiles_i, p, per * p.chunks, per, slab, 0);
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i)
    launch_wgrad_engine<64>(src, N, D, D, 2 * p.tiles_o * p.tiles_i, p, per * p.chunks, per, slab, 0);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps;
#if (GINE_WG_VARIANT & 8) != 0
  {
    static unsigned long long clk[4096][4];
    CK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(gine_wg_clock), sizeof(clk)));
    const int nb = p.chunks * 2 * p.tiles_o * p.tiles_i;
    double cyc = 0, rt = 0;
    for (int i = 0; i < nb && i < 4096; ++i) {
      cyc += (double)(clk[i][2] - clk[i][0]);
      rt += (double)(clk[i][3] - clk[i][1]);
    }
    printf("  mean block body: %.0f cycles over %.2f us -> clock %.2f GHz\n", cyc / nb,
           rt / nb / 100.0, cyc / rt * 0.1);
  }
#endif
  printf("variant %d N=%lld chunks=%d rows/chunk=%d blocks=%d: %.2f us  (%.1f TFLOP/s)\n",
         GINE_WG_VARIANT, (long long)N, p.chunks, p.rows_per_chunk,
         p.chunks * 2 * p.tiles_o * p.tiles_i, us, 4.0 * N * D * D / us * 1e-6);
  return 0;
}
