// Fused CRPS losses of the reference (models/loss.py) on gfx950: one pass computes, per
// station-node, the closed-form CRPS and its exact gradient w.r.t. the K distribution
// parameters (forward-mode dual numbers), then the NaN-masked mean over nodes.
//
// Replaces the ~700 elementwise launches per training step that the torch formulation of
// MixedLoss.crps (loss.py:203-272) + its autograd takes.  Evaluated in fp64 (the reference
// promotes the mixed losses to fp64 through c = tensor([log 0.01]), loss.py:33-34,230-231;
// its remaining fp32 sub-expressions are reproduced to within their fp32 rounding).
//   NormalCRPS      loss.py:335-369   pred = [mu, sigma]
//   MixedNormalCRPS loss.py:6-68      pred = [mu, sigma, p]
//   MixedLoss       loss.py:71-272    pred = [mu, sigma, p, sigma_u] (+ u if grad_u)
#include "gine_common.hpp"
#include "gine_headrow.hpp"
#include "gine_reduce.hpp"

namespace gine {
namespace {

constexpr double kInvSqrtPi = 0.56418958354775628695;   // 1/sqrt(pi)
constexpr double kLogSqrt2Pi = 0.91893853320467274178;  // log(sqrt(2 pi))
constexpr double kSqrt2 = 1.41421356237309504880;
constexpr int kThreads = 256;
constexpr int kHeadNodes = 64;  // nodes per workgroup of the pass that runs the head backward

// ---------------------------------------------------------------------------------------
// forward-mode dual numbers: value + gradient w.r.t. the K prediction columns
// ---------------------------------------------------------------------------------------
template <int K>
struct Dual {
  double v;
  double d[K];
};

template <int K>
__device__ __forceinline__ Dual<K> cst(double v) {
  Dual<K> r;
  r.v = v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = 0.0;
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> var(double v, int i) {
  Dual<K> r = cst<K>(v);
  r.d[i] = 1.0;
  return r;
}
// f(x) with derivative f'(x): chain rule
template <int K>
__device__ __forceinline__ Dual<K> apply(const Dual<K>& x, double f, double df) {
  Dual<K> r;
  r.v = f;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = df * x.d[i];
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator+(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v + b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] + b.d[i];
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator-(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v - b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] - b.d[i];
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator-(const Dual<K>& a) {
  return apply(a, -a.v, -1.0);
}
template <int K>
__device__ __forceinline__ Dual<K> operator*(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v * b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator/(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v / b.v;
  const double inv = 1.0 / b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) * inv;
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator*(double s, const Dual<K>& a) {
  return apply(a, s * a.v, s);
}
template <int K>
__device__ __forceinline__ Dual<K> operator+(double s, const Dual<K>& a) {
  return apply(a, s + a.v, 1.0);
}
template <int K>
__device__ __forceinline__ Dual<K> operator-(double s, const Dual<K>& a) {
  return apply(a, s - a.v, -1.0);
}
template <int K>
__device__ __forceinline__ Dual<K> sq(const Dual<K>& a) {
  return apply(a, a.v * a.v, 2.0 * a.v);
}
template <int K>
__device__ __forceinline__ Dual<K> dabs(const Dual<K>& a) {  // torch: d|x| = sign(x)
  return apply(a, fabs(a.v), a.v > 0.0 ? 1.0 : (a.v < 0.0 ? -1.0 : 0.0));
}
template <int K>
__device__ __forceinline__ Dual<K> powc(const Dual<K>& a, double c) {  // constant exponent
  const double p = pow(a.v, c);
  return apply(a, p, c * pow(a.v, c - 1.0));
}
// the two powers of pareto_crps at the experiments' xi = 0.5 (params.json "xi": 0.5):
// x^-2 and x^0.5 without pow() -- fp64 pow is the longest routine of the pass, and eight of
// them per node dominated its dependent chain.  Same values and derivatives as powc up to
// the last-bit rounding of pow (inf / NaN / signed-zero cases as pow for every argument
// the pass can produce: 1 + xi*yt and 1 - cdf with cdf <= 1).
template <int K>
__device__ __forceinline__ Dual<K> pow_m2(const Dual<K>& a) {  // a^-2, d = -2 a^-3
  const double p = 1.0 / (a.v * a.v);
  return apply(a, p, -2.0 * (p / a.v));
}
template <int K>
__device__ __forceinline__ Dual<K> pow_half(const Dual<K>& a) {  // a^0.5, d = 0.5 a^-0.5
  const double p = sqrt(a.v);
  return apply(a, p, 0.5 / p);
}
// standard normal cdf / pdf (torch.distributions.Normal(0, 1))
template <int K>
__device__ __forceinline__ Dual<K> Phi(const Dual<K>& z) {
  const double pdf = exp(-0.5 * z.v * z.v - kLogSqrt2Pi);
  return apply(z, 0.5 * (1.0 + erf(z.v / kSqrt2)), pdf);
}
template <int K>
__device__ __forceinline__ Dual<K> phi(const Dual<K>& z) {
  const double pdf = exp(-0.5 * z.v * z.v - kLogSqrt2Pi);
  return apply(z, pdf, -z.v * pdf);
}
template <int K>
__device__ __forceinline__ Dual<K> sigmoid(const Dual<K>& a) {
  const double s = 1.0 / (1.0 + exp(-a.v));
  return apply(a, s, s * (1.0 - s));
}
template <int K>
__device__ __forceinline__ Dual<K> select(bool c, const Dual<K>& a, const Dual<K>& b) {
  return c ? a : b;  // torch.where: gradient flows to the selected branch only
}

// ---------------------------------------------------------------------------------------
// closed forms (restated from models/loss.py)
// ---------------------------------------------------------------------------------------
template <int K>
__device__ Dual<K> crps_normal(const Dual<K>& mu, const Dual<K>& sigma, double y) {
  const Dual<K> z = (cst<K>(y) - mu) / sigma;
  return sigma * (z * (2.0 * Phi(z) - cst<K>(1.0)) + 2.0 * phi(z) - cst<K>(kInvSqrtPi));
}

template <int K>
__device__ Dual<K> crps_mixed_normal(const Dual<K>& mu, const Dual<K>& sigma, const Dual<K>& p,
                                     double y, double c) {
  const Dual<K> yt = (cst<K>(y) - mu) / sigma;
  const Dual<K> ct = (cst<K>(c) - mu) / sigma;
  const Dual<K> q = 1.0 - p;
  const Dual<K> Pc = p + q * Phi(ct);
  const Dual<K> t1 = yt * (2.0 * (p + q * Phi(yt)) - cst<K>(1.0));
  const Dual<K> t2 = -(ct * sq(Pc));
  const Dual<K> t3 = 2.0 * (q * (-phi(ct)) * Pc);
  const Dual<K> t4 = -2.0 * (q * (-phi(yt)));
  const Dual<K> t5 = (-kInvSqrtPi) * (sq(q) * (1.0 - Phi(kSqrt2 * ct)));
  return sigma * (t1 + t2 + t3 + t4 + t5);
}

template <int K>
__device__ Dual<K> pareto_crps(const Dual<K>& y, const Dual<K>& u, const Dual<K>& m,
                               const Dual<K>& s, double xi) {
  const Dual<K> yt = (y - u) / s;
  const bool half = xi == 0.5;  // a kernel argument: uniform
  const Dual<K> base = 1.0 + xi * yt;
  const Dual<K> cdf =
      select(yt.v <= 0.0, cst<K>(0.0), 1.0 - (half ? pow_m2(base) : powc(base, -1.0 / xi)));
  const Dual<K> om = 1.0 - m;
  const Dual<K> tail = 1.0 - cdf;
  return s * (dabs(yt) -
              (2.0 / (1.0 - xi)) * (om * (1.0 - (half ? pow_half(tail) : powc(tail, 1.0 - xi)))) +
              (1.0 / (2.0 - xi)) * sq(om));
}

template <int K, bool GRAD_U>
__device__ Dual<K> crps_mixed(const Dual<K>& mu, const Dual<K>& sigma, const Dual<K>& p,
                              const Dual<K>& su, const Dual<K>& u, double y, double c,
                              double xi, double t) {
  const Dual<K> yy = cst<K>(y);
  const Dual<K> ct = (cst<K>(c) - mu) / sigma;
  const Dual<K> ut = (u - mu) / sigma;
  const Dual<K> yt = (yy - mu) / sigma;
  const Dual<K> q = 1.0 - p;
  const Dual<K> m_u = p + q * Phi(ut);
  const Dual<K> Pc = p + q * Phi(ct);
  const Dual<K> Pu = q * (1.0 - Phi(ut));
  const Dual<K> t2 = ut * sq(Pu) - ct * sq(Pc);
  const Dual<K> t3 = -2.0 * (q * phi(ct) * Pc + q * phi(ut) * Pu);
  const Dual<K> t5 = (-kInvSqrtPi) * (sq(q) * (Phi(kSqrt2 * ut) - Phi(kSqrt2 * ct)));
  const Dual<K> mixed = sigma * (yt * (2.0 * (p + q * Phi(yt)) - cst<K>(1.0)) + t2 + t3 +
                                 2.0 * (q * phi(yt)) + t5);
  const Dual<K> upper = sigma * (ut + t2 + t3 + (-2.0) * (q * (-phi(ut)) + ut * Pu) + t5);
  const Dual<K> loss1 = mixed + pareto_crps(u, u, m_u, su, xi);
  const Dual<K> loss2 = pareto_crps(yy, u, m_u, su, xi) + upper;
  if constexpr (GRAD_U) {
    return sigmoid(t * (u - yy)) * (loss1 - loss2) + loss2;
  } else {
    return select(y < u.v, loss1, loss2);
  }
}

template <int KIND>
struct LossK {
  static constexpr int value = KIND == GINE_LOSS_NORMAL ? 2
                               : KIND == GINE_LOSS_MIXED_NORMAL ? 3
                               : KIND == GINE_LOSS_MIXED ? 4 : 5;
};

// The output head's backward run by the CRPS pass for a unit loss seed (gine_crps_head_fwd_grad):
// raw = the head's pre-PostProcess output, h / w its input and weight; dh and the dW | db
// partial row of each workgroup (gine_headrow.hpp) are written beside grad_unit.
struct HeadBwdArgs {
  const float* raw;
  const float* h;
  const float* w;
  float* dh;
  float* slab;
  int D;
};

// One thread per node.  Writes d crps_n / d pred_n (0 for NaN targets) and per-block
// [sum crps, count] partials; the workgroup that finishes last (ticket) reduces the partials
// into the loss -- no separate finalize launch.  HC > 0 (the head backward of these nodes
// from grad_unit, HC float4 column chunks per lane): kHeadNodes nodes per workgroup (the
// CRPS evaluation is latency-bound: one busy wave per CU costs what four do), evaluated by
// wave 0 alone, while the other waves load the head's weight and the nodes' h rows; after
// one barrier those waves run the head backward, the nodes spread over their half-waves
// (gine_headrow.hpp).  The roles stay in branches of their own: h rows held through the
// loss evaluation had pushed it past 256 registers into scratch.
template <int KIND, int HC = 0>
__global__ __launch_bounds__(kThreads) void k_crps(const float* __restrict__ pred,
                                                   const float* __restrict__ y, int64_t n,
                                                   double u_fixed, double xi, double c,
                                                   double t, double* __restrict__ dpred,
                                                   double* __restrict__ partials,
                                                   double* __restrict__ loss_out,
                                                   double* __restrict__ count_out,
                                                   unsigned int* __restrict__ ticket,
                                                   const uint32_t* __restrict__ count_parts,
                                                   float* __restrict__ grad_unit,
                                                   HeadBwdArgs hb) {
  constexpr bool HEAD = HC > 0;
  constexpr int K = LossK<KIND>::value;
  static_assert(kThreads == head::kThreads, "one CRPS node per head-backward thread");
  // the head backward's half-waves (waves 1..3) and the rows each walks
  constexpr int kHelpHW = (kThreads - kHeadNodes) / 32;
  constexpr int kHelpU = (kHeadNodes + kHelpHW - 1) / kHelpHW;
  static_assert(kHeadNodes % kWave == 0 && kHelpHW > 0, "wave 0 evaluates the loss");
  __shared__ float s_graw[HEAD ? kHeadNodes : 1][K];
  __shared__ float s_part[HEAD ? kHelpHW : 1][head::kMaxK * 256 + head::kMaxK];
  __shared__ double s_sum[kThreads];
  __shared__ double s_cnt[kThreads];
  __shared__ int s_last;
  __shared__ double s_count;
  constexpr int NPB = HEAD ? kHeadNodes : kThreads;
  static_assert(GINE_COUNT_PARTS == kWave, "one partial count per lane of wave 0");
  if (grad_unit != nullptr) {  // the count of valid targets: wave 0 sums the partials
    if (threadIdx.x < kWave) {
      uint32_t c = count_parts[threadIdx.x];
      for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
      if (threadIdx.x == 0) s_count = (double)c;
    }
    __syncthreads();
  }
  const int64_t i = blockIdx.x * (int64_t)NPB + threadIdx.x;
  const int64_t first = blockIdx.x * (int64_t)NPB;
  const int64_t n_blk = min<int64_t>(n, first + NPB);
  double val = 0.0, cnt = 0.0;
  if (!HEAD || (int)threadIdx.x < NPB) {  // the loss (wave 0 when HEAD)
    if (i < n) {
      const float yf = y[i];
      double g[K];
#pragma unroll
      for (int k = 0; k < K; ++k) g[k] = 0.0;
      if (yf == yf) {  // NaN targets are masked out (loss.py:22,220)
        const double yy = (double)yf;
        Dual<K> v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = var<K>((double)pred[i * K + k], k);
        Dual<K> r;
        if constexpr (KIND == GINE_LOSS_NORMAL) {
          r = crps_normal(v[0], v[1], yy);
        } else if constexpr (KIND == GINE_LOSS_MIXED_NORMAL) {
          r = crps_mixed_normal(v[0], v[1], v[2], yy, c);
        } else if constexpr (KIND == GINE_LOSS_MIXED) {
          r = crps_mixed<K, false>(v[0], v[1], v[2], v[3], cst<K>(u_fixed), yy, c, xi, t);
        } else {
          r = crps_mixed<K, true>(v[0], v[1], v[2], v[3], v[4], yy, c, xi, t);
        }
        val = r.v;
        cnt = 1.0;
#pragma unroll
        for (int k = 0; k < K; ++k) g[k] = r.d[k];
      }
#pragma unroll
      for (int k = 0; k < K; ++k) dpred[i * K + k] = g[k];
      if (grad_unit != nullptr) {  // d loss / d pred for gloss = 1, as k_crps_bwd rounds it
        const double cnt_all = s_count;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float gu = (float)(1.0 * g[k] / cnt_all);
          grad_unit[i * K + k] = gu;
          if constexpr (HEAD)  // d raw, as k_head_bwd forms it from grad_pred
            s_graw[threadIdx.x][k] =
                head::post_bwd(head::role_of(KIND, k), hb.raw[i * K + k], gu);
        }
      }
    }
    if constexpr (HEAD) {
      __syncthreads();  // d raw in LDS
      __syncthreads();  // the helpers' partial rows in LDS
    }
  } else if constexpr (HEAD) {  // waves 1..3: the head backward of the workgroup's nodes
    head::HeadRows<K, kHelpU, HC> rows;
    const int hw = threadIdx.x / 32 - NPB / 32;
    rows.init(hb.w, hb.D);
    rows.load(first + hw, kHelpHW, n_blk, hb.h, hb.D);  // arriving under the evaluation
    __syncthreads();  // d raw in LDS
    rows.step([&](int64_t nd, float (&gr)[K]) {
#pragma unroll
                for (int k = 0; k < K; ++k) gr[k] = s_graw[nd - first][k];
              },
              first + hw, kHelpHW, n_blk, hb.dh, hb.D);
    rows.put(s_part, hw, hb.D);
    __syncthreads();  // the partial rows in LDS
  }
  if constexpr (HEAD)
    head::reduce_rows<K>(hb.slab + (size_t)blockIdx.x * (K * hb.D + K), hb.D, s_part, kHelpHW);
  s_sum[threadIdx.x] = val;
  s_cnt[threadIdx.x] = cnt;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {  // fixed-order tree
    if (threadIdx.x < s) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + s];
      s_cnt[threadIdx.x] += s_cnt[threadIdx.x + s];
    }
    __syncthreads();
  }
  // publish the partial, then draw a ticket.  The partial goes out as agent-scope atomic
  // exchanges (performed at the memory side, like the BatchNorm accumulator's adds) and the
  // last arriver reads the partials with agent-scope atomic loads: no release / acquire
  // fence -- an agent-scope release writes the XCD's whole L2 back, and with the head
  // backward's dh rows just written that write-back sat in every workgroup's tail.
  if (threadIdx.x == 0) {
    __hip_atomic_exchange(&partials[2 * blockIdx.x], s_sum[0], __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_exchange(&partials[2 * blockIdx.x + 1], s_cnt[0], __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned int prev =
        __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // fixed order: thread j sums partial rows j, j + 256, ... then the same tree as above
  const int P = gridDim.x;
  double a = 0.0, b = 0.0;
  for (int p = threadIdx.x; p < P; p += kThreads) {
    a += __hip_atomic_load(&partials[2 * p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b += __hip_atomic_load(&partials[2 * p + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  s_sum[threadIdx.x] = a;
  s_cnt[threadIdx.x] = b;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + s];
      s_cnt[threadIdx.x] += s_cnt[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss_out[0] = s_sum[0] / s_cnt[0];  // NaN when no target is valid (torch.mean of empty)
    count_out[0] = s_cnt[0];
    *ticket = 0u;  // re-armed for the next call (stream order)
  }
}

// Number of non-NaN targets (the size of the reference's y[mask], loss.py:39-42, 234-239)
// as GINE_COUNT_PARTS partial counts: the unit-seed gradient of the CRPS pass divides by
// their sum before any workgroup of that pass could know the total.  Recounted every step
// (a replayed graph counts whatever y holds now).  The training step gets the same partials
// from the head forward (gine_head_fwd_count); this launch is the stand-alone form.
__global__ __launch_bounds__(256) void k_count_valid(const float* __restrict__ y, int64_t n,
                                                     uint32_t* __restrict__ parts) {
  count_valid_parts(y, n, parts);
}

// grad_pred = gloss * dpred / count
__global__ __launch_bounds__(kThreads) void k_crps_bwd(const double* __restrict__ dpred,
                                                       const double* __restrict__ count,
                                                       const double* __restrict__ gloss,
                                                       int64_t total, float* __restrict__ grad) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i >= total) return;
  grad[i] = (float)(gloss[0] * dpred[i] / count[0]);
}

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_crps_num_partials(int64_t num_nodes, int32_t* num_partials) {
  if (!num_partials || num_nodes < 0) return GINE_ERR_INVALID;
  const int64_t p = ceil_div(num_nodes, kHeadNodes);  // enough for either workgroup size
  *num_partials = (int32_t)(p > 0 ? p : 1);
  return GINE_OK;
}

namespace {
int crps_fwd_launch(const float* pred, const float* y, int64_t num_nodes, int32_t kind, double u,
                    double xi, double c, double t, double* dpred, double* partials,
                    double* loss_out, double* count_out, uint32_t* ticket,
                    const uint32_t* count_parts, float* grad_unit, void* stream,
                    const HeadBwdArgs* hb = nullptr) {
  if (num_nodes < 0 || !partials || !loss_out || !count_out || !ticket) return GINE_ERR_INVALID;
  if ((count_parts == nullptr) != (grad_unit == nullptr)) return GINE_ERR_INVALID;
  if (num_nodes > 0 && (!pred || !y || !dpred)) return GINE_ERR_INVALID;
  if (kind < GINE_LOSS_NORMAL || kind > GINE_LOSS_MIXED_U) return GINE_ERR_INVALID;
  hipStream_t s = as_stream(stream);
  const int npb = hb ? kHeadNodes : kThreads;
  const int64_t blocks = ceil_div(num_nodes, npb) > 0 ? ceil_div(num_nodes, npb) : 1;
#define LAUNCH_CRPS_H(KIND_, H_)                                                               \
  hipLaunchKernelGGL((k_crps<KIND_, H_>), dim3((unsigned)blocks), dim3(kThreads), 0, s, pred, y, \
                     num_nodes, u, xi, c, t, dpred, partials, loss_out, count_out, ticket,      \
                     count_parts, grad_unit, hb ? *hb : HeadBwdArgs{})
#define LAUNCH_CRPS(KIND_)                                 \
  do {                                                     \
    if (!hb) LAUNCH_CRPS_H(KIND_, 0);                      \
    else if (hb->D <= 128) LAUNCH_CRPS_H(KIND_, 1);        \
    else LAUNCH_CRPS_H(KIND_, 2);                          \
  } while (0)
  switch (kind) {
    case GINE_LOSS_NORMAL: LAUNCH_CRPS(GINE_LOSS_NORMAL); break;
    case GINE_LOSS_MIXED_NORMAL: LAUNCH_CRPS(GINE_LOSS_MIXED_NORMAL); break;
    case GINE_LOSS_MIXED: LAUNCH_CRPS(GINE_LOSS_MIXED); break;
    default: LAUNCH_CRPS(GINE_LOSS_MIXED_U); break;
  }
#undef LAUNCH_CRPS
#undef LAUNCH_CRPS_H
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
}  // namespace

extern "C" int gine_crps_fwd(const float* pred, const float* y, int64_t num_nodes, int32_t kind,
                             double u, double xi, double c, double t, double* dpred,
                             double* partials, double* loss_out, double* count_out,
                             uint32_t* ticket, void* stream) {
  return crps_fwd_launch(pred, y, num_nodes, kind, u, xi, c, t, dpred, partials, loss_out,
                         count_out, ticket, nullptr, nullptr, stream);
}

extern "C" int gine_crps_fwd_grad(const float* pred, const float* y, int64_t num_nodes,
                                  int32_t kind, double u, double xi, double c, double t,
                                  double* dpred, double* partials, double* loss_out,
                                  double* count_out, uint32_t* ticket,
                                  const uint32_t* count_parts, float* grad_unit, void* stream) {
  if (!count_parts || !grad_unit) return GINE_ERR_INVALID;
  return crps_fwd_launch(pred, y, num_nodes, kind, u, xi, c, t, dpred, partials, loss_out,
                         count_out, ticket, count_parts, grad_unit, stream);
}

namespace {
int loss_k(int kind) {
  return kind == GINE_LOSS_NORMAL ? 2 : kind == GINE_LOSS_MIXED_NORMAL ? 3
         : kind == GINE_LOSS_MIXED ? 4 : kind == GINE_LOSS_MIXED_U ? 5 : -1;
}
int64_t crps_head_blocks(int64_t num_nodes) {
  const int64_t b = ceil_div(num_nodes, kHeadNodes);
  return b > 0 ? b : 1;
}
}  // namespace

extern "C" int gine_crps_head_slab_floats(int64_t num_nodes, int32_t channels, int32_t kind,
                                          size_t* floats) {
  const int K = loss_k(kind);
  if (K < 0 || num_nodes < 0 || !floats) return GINE_ERR_INVALID;
  if (channels <= 0 || channels % 4 != 0 || channels > 32 * 4 * head::kMaxChunks)
    return GINE_ERR_DIM;
  *floats = (size_t)crps_head_blocks(num_nodes) * (size_t)(K * channels + K);
  return GINE_OK;
}

extern "C" int gine_crps_head_fwd_grad(const float* pred, const float* y, int64_t num_nodes,
                                       int32_t kind, double u, double xi, double c, double t,
                                       double* dpred, double* partials, double* loss_out,
                                       double* count_out, uint32_t* ticket,
                                       const uint32_t* count_parts, float* grad_unit,
                                       const float* raw, const float* h, const float* w,
                                       int32_t channels, float* dh, float* head_slab,
                                       void* stream) {
  size_t floats = 0;
  const int rc = gine_crps_head_slab_floats(num_nodes, channels, kind, &floats);
  if (rc != GINE_OK) return rc;
  if (!count_parts || !grad_unit || !head_slab || !w) return GINE_ERR_INVALID;
  if (num_nodes > 0 && (!raw || !h || !dh)) return GINE_ERR_INVALID;
  const HeadBwdArgs hb{raw, h, w, dh, head_slab, channels};
  return crps_fwd_launch(pred, y, num_nodes, kind, u, xi, c, t, dpred, partials, loss_out,
                         count_out, ticket, count_parts, grad_unit, stream, &hb);
}

extern "C" int gine_crps_head_grad_job(int64_t num_nodes, int32_t channels, int32_t kind,
                                       const float* head_slab, float* dw, float* db,
                                       gine_grad_job* job) {
  size_t floats = 0;
  const int rc = gine_crps_head_slab_floats(num_nodes, channels, kind, &floats);
  if (rc != GINE_OK) return rc;
  if (!head_slab || !dw || !job) return GINE_ERR_INVALID;
  const int K = loss_k(kind);
  const int64_t per = (int64_t)K * channels + K;
  *job = gine_grad_job{};
  job->kind = GINE_GRAD_JOB_SLAB;
  job->src = head_slab;
  job->rows = (int32_t)crps_head_blocks(num_nodes);
  job->cstride = per;
  job->nz = 1;
  job->per[0] = per;
  job->wsize[0] = (int64_t)K * channels;
  job->w[0] = dw;
  job->b[0] = db;
  job->bscale[0] = 1.0f;
  return GINE_OK;
}

extern "C" int gine_count_valid(const float* y, int64_t num_nodes, uint32_t* count_parts,
                                void* stream) {
  if (num_nodes < 0 || !count_parts || (num_nodes > 0 && !y)) return GINE_ERR_INVALID;
  if (num_nodes > ((int64_t)1 << 32) - 1) return GINE_ERR_DIM;  // 32-bit counts
  hipLaunchKernelGGL(k_count_valid, dim3(GINE_COUNT_PARTS), dim3(256), 0, as_stream(stream), y,
                     num_nodes, count_parts);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_crps_bwd(const double* dpred, const double* count, const double* gloss,
                             int64_t num_nodes, int32_t kind, float* grad_pred, void* stream) {
  if (num_nodes < 0 || !count || !gloss) return GINE_ERR_INVALID;
  if (kind < GINE_LOSS_NORMAL || kind > GINE_LOSS_MIXED_U) return GINE_ERR_INVALID;
  const int K = kind == GINE_LOSS_NORMAL ? 2 : kind == GINE_LOSS_MIXED_NORMAL ? 3
              : kind == GINE_LOSS_MIXED ? 4 : 5;
  const int64_t total = num_nodes * K;
  if (total == 0) return GINE_OK;
  if (!dpred || !grad_pred) return GINE_ERR_INVALID;
  hipLaunchKernelGGL(k_crps_bwd, dim3((unsigned)ceil_div(total, kThreads)), dim3(kThreads), 0,
                     as_stream(stream), dpred, count, gloss, total, grad_pred);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
