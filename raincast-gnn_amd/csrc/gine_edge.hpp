// Per-edge arithmetic of GINEConv message passing on packed fp32 pairs.
//
// A lane owns 4 consecutive channels (one 16-byte chunk of a feature row).  The per-edge
// work is elementwise, so it runs on the packed-fp32 VALU (v_pk_mul/add/fma_f32: two
// channels per instruction) with the exact rounding sequence of the CPU path:
//   forward   acc += relu(x_j + lin(a))             lin(a) = a*w + b (fma or mul, add)
//   backward  dm = (x_i + lin(a) <= 0) ? 0 : dz_j   (ATen threshold_backward on relu(pre))
//             acc += dm;  accw = fma(dm, a, accw)   (this node's share of dW_e)
// -ffp-contract=off keeps every unfused mul/add separately rounded.
#pragma once

#include "gine_common.hpp"

namespace gine {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v f4v_zero() { return f4v{0.f, 0.f, 0.f, 0.f}; }

__device__ __forceinline__ f4v ld_f4v(const char* base, uint32_t byte_off) {
  return *reinterpret_cast<const f4v*>(base + byte_off);
}

template <bool FMA>
__device__ __forceinline__ f2v edge_lin2(float a, f2v w, f2v b) {
  const f2v av = {a, a};
  if constexpr (FMA) return __builtin_elementwise_fma(av, w, b);
  return av * w + b;  // two roundings
}

__device__ __forceinline__ f2v relu2(f2v v) {
  return __builtin_elementwise_maximum(v, f2v{0.f, 0.f});  // NaN-propagating, -0 < +0
}

template <bool FMA>
__device__ __forceinline__ void fwd_edge(f4v& acc, f4v r, float a, f4v w, f4v b) {
  acc.xy = acc.xy + relu2(r.xy + edge_lin2<FMA>(a, w.xy, b.xy));
  acc.zw = acc.zw + relu2(r.zw + edge_lin2<FMA>(a, w.zw, b.zw));
}

template <bool FMA>
__device__ __forceinline__ void bwd_edge(f4v& acc, f4v& accw, f4v r, float a, f4v h, f4v w,
                                         f4v b) {
  const f2v plo = h.xy + edge_lin2<FMA>(a, w.xy, b.xy);
  const f2v phi = h.zw + edge_lin2<FMA>(a, w.zw, b.zw);
  f4v dm;
  dm.x = plo.x <= 0.f ? 0.f : r.x;
  dm.y = plo.y <= 0.f ? 0.f : r.y;
  dm.z = phi.x <= 0.f ? 0.f : r.z;
  dm.w = phi.y <= 0.f ? 0.f : r.w;
  acc.xy = acc.xy + dm.xy;
  acc.zw = acc.zw + dm.zw;
  const f2v av = {a, a};
  accw.xy = __builtin_elementwise_fma(dm.xy, av, accw.xy);
  accw.zw = __builtin_elementwise_fma(dm.zw, av, accw.zw);
}

// o = acc + s * v (the (1 + eps) terms: mul rounds, then add)
__device__ __forceinline__ f4v add_scaled(f4v acc, float s, f4v v) {
  const f2v sv = {s, s};
  f4v o;
  o.xy = acc.xy + sv * v.xy;
  o.zw = acc.zw + sv * v.zw;
  return o;
}

__device__ __forceinline__ float4 to_float4(f4v v) { return make_float4(v.x, v.y, v.z, v.w); }

}  // namespace gine
