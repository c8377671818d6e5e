// AdamW over ONE flat fp32 buffer holding every parameter of the model (the benchmarked
// training step, train.py:67-69: zero_grad / backward / AdamW.step, lr from params.json).
//
// torch.optim.AdamW (amsgrad=False, maximize=False) per element, default (non-capturable)
// formulation, with the scalar bias corrections computed in double and applied in fp32 the
// way torch applies Python scalars to fp32 tensors:
//   step += 1
//   p  *= 1 - lr*wd
//   m   = m + (1-b1)*(g - m)                 (lerp, weight < 0.5 branch)
//   v   = v*b2 + (1-b2)*g*g
//   p  += -(lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// The step counter lives on the device, so the update is legal inside a captured HIP graph
// and replays correctly: every workgroup uses step[0] + 1, and the workgroup that finishes
// last stores the bump -- one launch per optimizer step.  "Last" is found by a two-level
// ticket: workgroup b draws from sub-ticket b % 8 (step[32 + 32 g], one 128-byte line each),
// the last of each group draws from the top ticket (step[1]); every ticket word is re-armed
// to 0 by its last drawer.  The step buffer is kAdamStateFloats = 288 floats
// (gine_adamw_state_floats), all zero at allocation.
#include "gine_common.hpp"


namespace gine {
namespace {

constexpr int kAdamGroups = 8;     // sub-tickets (one per XCD's share of the grid)
constexpr int kAdamSubBase = 32;   // floats: sub-ticket g at step[32 + 32 g]
constexpr int kAdamStateFloats = kAdamSubBase + 32 * kAdamGroups;

struct AdamW {
  float decay, neg_step_size, bc2_sqrt, w1, w2, beta2, eps;
  __device__ __forceinline__ void operator()(float gi, float& pi, float& mi, float& vi) const {
    pi = pi * decay;
    mi = mi + w1 * (gi - mi);
    vi = vi * beta2;
    vi = vi + w2 * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi + neg_step_size * (mi / denom);  // addcdiv: p + value * (m / denom)
  }
};

// One float4 of every buffer per thread (16-byte loads, all four issued before any use);
// the last n % 4 elements by the first threads of the grid.
__global__ __launch_bounds__(256) void k_adamw(float* __restrict__ p, const float* __restrict__ g,
                                               float* __restrict__ m, float* __restrict__ v,
                                               float* __restrict__ step, int64_t n,
                                               float lr, float beta1, float beta2, float eps,
                                               float weight_decay) {
  const float t_new = step[0] + 1.0f;
  const double t = (double)t_new;
  const AdamW op{(float)(1.0 - (double)lr * (double)weight_decay),
                 (float)(-((double)lr / (1.0 - pow((double)beta1, t)))),
                 (float)sqrt(1.0 - pow((double)beta2, t)), 1.0f - beta1, 1.0f - beta2, beta2,
                 eps};
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int64_t i = tid; i < n4; i += stride) {
    const float4 gi = reinterpret_cast<const float4*>(g)[i];
    float4 pi = reinterpret_cast<float4*>(p)[i];
    float4 mi = reinterpret_cast<float4*>(m)[i];
    float4 vi = reinterpret_cast<float4*>(v)[i];
    op(gi.x, pi.x, mi.x, vi.x);
    op(gi.y, pi.y, mi.y, vi.y);
    op(gi.z, pi.z, mi.z, vi.z);
    op(gi.w, pi.w, mi.w, vi.w);
    reinterpret_cast<float4*>(p)[i] = pi;
    reinterpret_cast<float4*>(m)[i] = mi;
    reinterpret_cast<float4*>(v)[i] = vi;
  }
  if (tid < n - 4 * n4) {
    const int64_t i = 4 * n4 + tid;
    float pi = p[i], mi = m[i], vi = v[i];
    op(g[i], pi, mi, vi);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
  __syncthreads();  // every thread of this workgroup has read step[0]
  if (threadIdx.x == 0) {
    unsigned int* ticket = reinterpret_cast<unsigned int*>(&step[1]);  // 0.0f == 0u
    // two-level ticket: same-word returning atomics serialise (~88 per us on one word,
    // MI355X_MICROARCH.md "dequeue"), so 512 workgroups on one ticket cost ~6 us at the
    // end of the launch; workgroup b draws from sub-ticket b % 8 (own 128-byte line),
    // the last of each group from the top ticket (one word: 6.81 -> 5.46 us, r02_s84)
    const unsigned int g = blockIdx.x % kAdamGroups;
    const unsigned int groups = min(gridDim.x, (unsigned)kAdamGroups);
    const unsigned int size = (gridDim.x - g + kAdamGroups - 1) / kAdamGroups;
    unsigned int* sub = reinterpret_cast<unsigned int*>(step + kAdamSubBase) + 32 * g;
    if (atomicAdd(sub, 1u) == size - 1) {
      *sub = 0u;  // re-armed (the next launch is ordered after this one)
      if (atomicAdd(ticket, 1u) == groups - 1) {
        step[0] = t_new;
        *ticket = 0u;
      }
    }
  }
}

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_adamw_step(float* param, const float* grad, float* exp_avg,
                               float* exp_avg_sq, float* step, int64_t n, float lr,
                               float beta1, float beta2, float eps, float weight_decay,
                               void* stream) {
  if (n < 0 || !step) return GINE_ERR_INVALID;
  if (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq)) return GINE_ERR_INVALID;
  hipStream_t s = as_stream(stream);
  // one float4 per thread up to 512 workgroups (few tickets to serialise on one word);
  // 16-byte accesses need 16-byte aligned buffers
  const uintptr_t al = reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                       reinterpret_cast<uintptr_t>(exp_avg) |
                       reinterpret_cast<uintptr_t>(exp_avg_sq);
  if (n > 0 && (al & 15) != 0) return GINE_ERR_INVALID;
  int64_t blocks = ceil_div(n > 0 ? ceil_div(n, 4) : 1, 256);
  if (blocks > 512) blocks = 512;
  hipLaunchKernelGGL(k_adamw, dim3((unsigned)blocks), dim3(256), 0, s, param, grad, exp_avg,
                     exp_avg_sq, step, n, lr, beta1, beta2, eps, weight_decay);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_adamw_state_floats(int64_t* floats) {
  if (!floats) return GINE_ERR_INVALID;
  *floats = kAdamStateFloats;
  return GINE_OK;
}
