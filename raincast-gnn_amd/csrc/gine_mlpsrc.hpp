// Node-MLP operand sources (prologue transforms of the row-tile GEMM, the weight-gradient
// engine's MlpWgradSrc), shared by gine_mlp.hip and the message-passing backward of
// gine_mpwin.hip, which can run the node-MLP weight-gradient engine in its own launch.
#pragma once

#include "gine_common.hpp"

namespace gine {
namespace {

// Compile-time variants only: a runtime branch between loads makes the compiler drain the
// memory queue (s_waitcnt vmcnt(0)) at the merge, serialising what should be in flight.
//   PRO_DOR: do = dy * 1[y > 0]  (ReLU epilogue)     PRO_DOM: do = dy * mask (residual)
//   (no epilogue: do = dy, PRO_PLAIN)
enum Pro { PRO_PLAIN = 0, PRO_BNRELU = 1, PRO_DA1 = 3, PRO_DOR = 4, PRO_DOM = 5 };
//   EPI_OUT / EPI_OUT_RELU / EPI_OUT_RES: y = o | relu(o) | x + relu(o) (+ mask)
enum Epi { EPI_A1STATS = 0, EPI_OUT = 1, EPI_DBN = 2, EPI_PLAIN = 3, EPI_OUT_RELU = 4,
           EPI_OUT_RES = 5 };


// bn_save layout: [mean | invstd | alpha | shift], each [D]
struct BnView {
  const float* mean;
  const float* invstd;
  const float* alpha;
  const float* shift;
};
__device__ __forceinline__ BnView bn_view(const float* s, int D) {
  return BnView{s, s + D, s + 2 * D, s + 3 * D};
}

struct ProArgs {
  const float* x;        // primary [N][D]: z | a1 | dy | dbn
  const float* aux;      // a1 for PRO_DA1; y for PRO_DOR
  const uint8_t* mask;   // PRO_DOM
  const float* bn;       // bn_save
  const float* coef;     // [c1 | c2 | c3] (PRO_DA1)
};

// Same rounding sequence wherever bn is recomputed (forward GEMM2 prologue, backward
// ReLU mask, dW2 prologue): mul then add, no contraction.
__device__ __forceinline__ float bn_apply(float a, float alpha, float shift) {
  return a * alpha + shift;
}

// Prologue value of float4 column-group q of row n.
template <int PRO>
__device__ __forceinline__ float4 prologue(const ProArgs& p, int D, int64_t n, int q) {
  const int64_t off = n * D + 4 * q;
  const float4 v = *reinterpret_cast<const float4*>(p.x + off);
  if constexpr (PRO == PRO_PLAIN) {
    return v;
  } else if constexpr (PRO == PRO_BNRELU) {
    const BnView b = bn_view(p.bn, D);
    const float4 al = *reinterpret_cast<const float4*>(b.alpha + 4 * q);
    const float4 sh = *reinterpret_cast<const float4*>(b.shift + 4 * q);
    return make_float4(relu_nan(bn_apply(v.x, al.x, sh.x)), relu_nan(bn_apply(v.y, al.y, sh.y)),
                       relu_nan(bn_apply(v.z, al.z, sh.z)), relu_nan(bn_apply(v.w, al.w, sh.w)));
  } else if constexpr (PRO == PRO_DOR) {
    const float4 y = *reinterpret_cast<const float4*>(p.aux + off);
    return make_float4(y.x > 0.f ? v.x : 0.f, y.y > 0.f ? v.y : 0.f, y.z > 0.f ? v.z : 0.f,
                       y.w > 0.f ? v.w : 0.f);
  } else if constexpr (PRO == PRO_DOM) {
    const uchar4 m = *reinterpret_cast<const uchar4*>(p.mask + off);
    return make_float4(m.x ? v.x : 0.f, m.y ? v.y : 0.f, m.z ? v.z : 0.f, m.w ? v.w : 0.f);
  } else {  // PRO_DA1: da1 = c1*dbn + c2*xhat + c3, xhat = (a1 - mean)*invstd
    const BnView b = bn_view(p.bn, D);
    const float4 a1 = *reinterpret_cast<const float4*>(p.aux + off);
    const float4 mu = *reinterpret_cast<const float4*>(b.mean + 4 * q);
    const float4 is = *reinterpret_cast<const float4*>(b.invstd + 4 * q);
    const float4 c1 = *reinterpret_cast<const float4*>(p.coef + 4 * q);
    const float4 c2 = *reinterpret_cast<const float4*>(p.coef + D + 4 * q);
    const float4 c3 = *reinterpret_cast<const float4*>(p.coef + 2 * D + 4 * q);
    float4 r;
    r.x = c1.x * v.x + c2.x * ((a1.x - mu.x) * is.x) + c3.x;
    r.y = c1.y * v.y + c2.y * ((a1.y - mu.y) * is.y) + c3.y;
    r.z = c1.z * v.z + c2.z * ((a1.z - mu.z) * is.z) + c3.z;
    r.w = c1.w * v.w + c2.w * ((a1.w - mu.w) * is.w) + c3.w;
    return r;
  }
}

// Raw (pre-prologue) values of one staged float4 item, loaded a tile ahead.
struct RawItem {
  float4 v;    // primary input
  float4 aux;  // y (PRO_DOR) | a1 (PRO_DA1)
  uchar4 m;    // ReLU mask (PRO_DOM)
};

// Per-thread column constants of the prologue (a thread always stages the same column
// group q = tid % (D/4), so these are loaded once per workgroup).
struct ColConst {
  float4 a, b, c, d, e;
};

template <int PRO>
__device__ __forceinline__ ColConst col_const(const ProArgs& p, int D, int q) {
  ColConst k;
  k.a = k.b = k.c = k.d = k.e = f4_zero();
  if constexpr (PRO == PRO_BNRELU) {
    const BnView b = bn_view(p.bn, D);
    k.a = *reinterpret_cast<const float4*>(b.alpha + 4 * q);
    k.b = *reinterpret_cast<const float4*>(b.shift + 4 * q);
  } else if constexpr (PRO == PRO_DA1) {
    const BnView b = bn_view(p.bn, D);
    k.a = *reinterpret_cast<const float4*>(p.coef + 4 * q);
    k.b = *reinterpret_cast<const float4*>(p.coef + D + 4 * q);
    k.c = *reinterpret_cast<const float4*>(p.coef + 2 * D + 4 * q);
    k.d = *reinterpret_cast<const float4*>(b.mean + 4 * q);
    k.e = *reinterpret_cast<const float4*>(b.invstd + 4 * q);
  }
  return k;
}

template <int PRO>
__device__ __forceinline__ RawItem raw_load(const ProArgs& p, int D, int64_t n, int q) {
  RawItem r;
  const int64_t off = n * D + 4 * q;
  r.v = *reinterpret_cast<const float4*>(p.x + off);
  r.aux = f4_zero();
  r.m = make_uchar4(1, 1, 1, 1);
  if constexpr (PRO == PRO_DOR) {
    r.aux = *reinterpret_cast<const float4*>(p.aux + off);
  } else if constexpr (PRO == PRO_DOM) {
    r.m = *reinterpret_cast<const uchar4*>(p.mask + off);
  } else if constexpr (PRO == PRO_DA1) {
    r.aux = *reinterpret_cast<const float4*>(p.aux + off);
  }
  return r;
}

// Same arithmetic as prologue<PRO>() (the weight-gradient kernel recomputes through that).
template <int PRO>
__device__ __forceinline__ float4 transform(const ProArgs& p, const RawItem& r,
                                            const ColConst& k) {
  const float4 v = r.v;
  if constexpr (PRO == PRO_PLAIN) {
    return v;
  } else if constexpr (PRO == PRO_BNRELU) {
    return make_float4(relu_nan(bn_apply(v.x, k.a.x, k.b.x)), relu_nan(bn_apply(v.y, k.a.y, k.b.y)),
                       relu_nan(bn_apply(v.z, k.a.z, k.b.z)), relu_nan(bn_apply(v.w, k.a.w, k.b.w)));
  } else if constexpr (PRO == PRO_DOR) {
    const float4 y = r.aux;
    return make_float4(y.x > 0.f ? v.x : 0.f, y.y > 0.f ? v.y : 0.f, y.z > 0.f ? v.z : 0.f,
                       y.w > 0.f ? v.w : 0.f);
  } else if constexpr (PRO == PRO_DOM) {
    const uchar4 m = r.m;
    return make_float4(m.x ? v.x : 0.f, m.y ? v.y : 0.f, m.z ? v.z : 0.f, m.w ? v.w : 0.f);
  } else {  // PRO_DA1
    const float4 a1 = r.aux;
    float4 o;
    o.x = k.a.x * v.x + k.b.x * ((a1.x - k.d.x) * k.e.x) + k.c.x;
    o.y = k.a.y * v.y + k.b.y * ((a1.y - k.d.y) * k.e.y) + k.c.y;
    o.z = k.a.z * v.z + k.b.z * ((a1.z - k.d.z) * k.e.z) + k.c.z;
    o.w = k.a.w * v.w + k.b.w * ((a1.w - k.d.w) * k.e.w) + k.c.w;
    return o;
  }
}

// ----------------------------------------------------------------------------------------
// Weight gradients: dW[o][i] = sum_n P[n][o] * Q[n][i], db[o] = sum_n P[n][o]
//   z = 0: P = do (PRO_DO of dy), Q = r = relu(bn(a1))  -> dW2, db2
//   z = 1: P = da1 (PRO_DA1 of dbn), Q = z               -> dW1, db1
// on the shared engine (gine_wgrad.hpp); this is its operand source.
// ----------------------------------------------------------------------------------------
// Output-tile height of the node-MLP weight gradients (experiment switch: TO = 128 reads
// each operand row once per chunk, TO = 64 twice, with twice the workgroups; at cfg2
// TO = 128 measured 28.2 vs 25.0 us for gine_mlp_bwd1_wgrad, 26.3 vs 22.1 standalone).
#ifndef GINE_MLP_WG_TO
#define GINE_MLP_WG_TO 64
#endif
constexpr int kMlpWgTO = GINE_MLP_WG_TO;
// The node-MLP weight-gradient engines -- stand-alone (gine_mlp_wgrad), beside the dz GEMM
// (gine_mlp_bwd1_wgrad) and inside the window backward (gine_mp_bwd_win_mlp_wgrad) -- all run
// the split-bf16 chain (gine_wgrad.hpp wgrad_body_x3), so the three give the same bits
// (tests/test_gpu_fuzz.py, test_gpu_training.py).  0: the fp32 chain everywhere (A/B builds).
#ifndef GINE_MLP_ENG_X3
#define GINE_MLP_ENG_X3 1
#endif
constexpr bool kMlpEngX3 = GINE_MLP_ENG_X3 != 0;

template <int PDO>  // PRO_PLAIN | PRO_DOR | PRO_DOM: how do is formed from dy
struct MlpWgradSrc {
  static constexpr int kZ = 2;
  ProArgs p_do, q_r, p_da1, q_z;
  int D;
  using Raw = RawItem;
  using Col = ColConst;
  template <int Z> __device__ int i_dim(int I) const { return I; }
  template <int Z> __device__ Col p_col(int q) const {
    if constexpr (Z == 0) return col_const<PDO>(p_do, D, q);
    else return col_const<PRO_DA1>(p_da1, D, q);
  }
  template <int Z> __device__ Col q_col(int q) const {
    if constexpr (Z == 0) return col_const<PRO_BNRELU>(q_r, D, q);
    else return col_const<PRO_PLAIN>(q_z, D, q);
  }
  template <int Z> __device__ Raw p_load(int64_t n, int q) const {
    if constexpr (Z == 0) return raw_load<PDO>(p_do, D, n, q);
    else return raw_load<PRO_DA1>(p_da1, D, n, q);
  }
  template <int Z> __device__ Raw q_load(int64_t n, int q) const {
    if constexpr (Z == 0) return raw_load<PRO_BNRELU>(q_r, D, n, q);
    else return raw_load<PRO_PLAIN>(q_z, D, n, q);
  }
  template <int Z> __device__ float4 p_xform(const Raw& r, const Col& c) const {
    if constexpr (Z == 0) return transform<PDO>(p_do, r, c);
    else return transform<PRO_DA1>(p_da1, r, c);
  }
  template <int Z> __device__ float4 q_xform(const Raw& r, const Col& c) const {
    if constexpr (Z == 0) return transform<PRO_BNRELU>(q_r, r, c);
    else return transform<PRO_PLAIN>(q_z, r, c);
  }
};

}  // namespace
}  // namespace gine
