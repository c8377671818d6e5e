// The dense layers between the DeepSet member sum and the GINE stack, fused on gfx950.
//
// Replaces (models/gnn.py:48-68, 112-113, 132-135; phi's last Linear applied after the
// member sum, see raincast_gnn/models.py DeepSetEncoder):
//   s  = r Wp2^T + M bp2          phi[2] (member-summed)
//   u  = relu(s Wr0^T + br0)      rho[0], rho[1]
//   e  = u Wr1^T + br1            rho[2]           (the DeepSet embedding)
//   h0 = [x | e] Wdr^T + bdr      dim_red(cat([x, emb], 1))
// which the reference runs as four library GEMMs, a ReLU and a concatenation forward and
// four input-gradient GEMMs, four weight-gradient GEMMs, a ReLU backward and a split
// backward.  Here: two 2-stage row-chain kernels forward (F1: s, u; F2: e, h0), two
// backward (B1: de, dt; B2: ds, dr), one weight-gradient launch for all four Linears
// (gine_wgrad.hpp, Z = 4) and one fixed-order slab reduction.
//
// Row-chain kernel: a workgroup of D/32 waves walks 32-row tiles (persistent, XCD-local
// tile ranges).  Both stages' weight fragments live in VGPRs (loaded once per workgroup);
// stage 1 reads its A tile from LDS (staged from HBM with the next tile's raw rows in
// flight), writes its output both to HBM (saved for the backward) and to a second LDS
// tile, which is stage 2's A operand -- the intermediate never round-trips through HBM
// between the two GEMMs.  The MFMA layout and the lane-half k split are k_rowgemm's
// (gine_mlp.hip): lane half h contracts k in [h*K/2, (h+1)*K/2), A fragments read as
// ds_read_b128 from rows padded by 4 floats.
#include "gine_common.hpp"
#include "gine_slab.hpp"
#include "gine_wgrad.hpp"

#include <algorithm>
#include <cstdlib>

namespace gine {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kRowTile = 32;

enum ChainKind { CH_F1 = 0, CH_F2 = 1, CH_B1 = 2, CH_B2 = 3 };

struct ChainArgs {
  const float* in;   // stage-1 A rows [N, D]: r | u | dh0 | dt
  const float* x;    // F2: node features [N, F]
  const float* aux;  // B1: u (ReLU mask of rho[1])
  const float* w1;   // stage-1 weight
  const float* b1;   // stage-1 bias (forward)
  const float* w2;   // stage-2 weight
  const float* b2;   // stage-2 bias (forward)
  float* out1;       // stage-1 output [N, D]: s | e | de | ds
  float* out2;       // stage-2 output [N, D]: u | h0 | dt | dr
  float bias1_scale; // F1: M (phi[2]'s bias summed over members)
  int F;             // F2 / B1: dim_red's x width
};

__device__ __forceinline__ floatx16 zero16() {
  floatx16 v;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = 0.f;
  return v;
}

// acc = A[32 x K] (LDS rows, stride lda) x B-fragments (K/2 per lane half)
template <int K>
__device__ __forceinline__ floatx16 tile_mma(const float* sA, int lda, const float (&bf)[K / 2],
                                             int c32, int h) {
  constexpr int KS = K / 2;
  floatx16 acc = zero16();
  const float* arow = sA + c32 * lda + h * KS;
#pragma unroll
  for (int q = 0; q < KS / 4; ++q) {
    const float4 a4 = *reinterpret_cast<const float4*>(&arow[4 * q]);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, bf[4 * q], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, bf[4 * q + 1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, bf[4 * q + 2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, bf[4 * q + 3], acc, 0, 0, 0);
  }
  return acc;
}

// Y = X W^T fragment: bf[s] = W[col][h*KS + s]  (W row-major [*, ldw])
template <int K>
__device__ __forceinline__ void frag_t(float (&bf)[K / 2], const float* W, int ldw, int col,
                                       int h) {
  constexpr int KS = K / 2;
#pragma unroll
  for (int s = 0; s < KS; ++s) bf[s] = W[(size_t)col * ldw + h * KS + s];
}
// dX = dY W fragment: bf[s] = W[h*KS + s][coff + col]
template <int K>
__device__ __forceinline__ void frag_n(float (&bf)[K / 2], const float* W, int ldw, int coff,
                                       int col, int h) {
  constexpr int KS = K / 2;
#pragma unroll
  for (int s = 0; s < KS; ++s) bf[s] = W[(size_t)(h * KS + s) * ldw + coff + col];
}
// dim_red's weight [D][F + D] seen on the padded k axis [x (F) | 0 (FP - F) | e (D)]
template <int FP, int D>
__device__ __forceinline__ void frag_dimred(float (&bf)[(FP + D) / 2], const float* W, int F,
                                            int col, int h) {
  constexpr int KS = (FP + D) / 2;
  const int ldw = F + D;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = h * KS + s;
    const int c = k < F ? k : (k < FP ? 0 : k - FP + F);
    const float v = W[(size_t)col * ldw + c];
    bf[s] = (k >= F && k < FP) ? 0.f : v;
  }
}

// Per-XCD contiguous tile ranges (as k_rowgemm).
struct TileRange {
  int first, end, step;
};
__device__ __forceinline__ TileRange tile_range(int num_tiles) {
  const int nb = gridDim.x;
  const int xcd = blockIdx.x % kNumXcd, pos = blockIdx.x / kNumXcd;
  const int here = nb / kNumXcd + (xcd < nb % kNumXcd ? 1 : 0);
  const int span = (num_tiles + kNumXcd - 1) / kNumXcd;
  const int b = xcd * span;
  return TileRange{b + pos, min(num_tiles, b + span), here};
}

template <int D, int FP, int KIND>
__global__ __launch_bounds__(2 * D) void k_chain(ChainArgs a, int64_t N, int num_tiles) {
  constexpr int NT = 2 * D;
  constexpr int D4 = D / 4;
  constexpr int LDA = D + 4;
  constexpr int K2 = KIND == CH_F2 ? FP + D : D;    // stage-2 contraction length
  constexpr int LDB = K2 + 4;
  constexpr int BOFF = KIND == CH_F2 ? FP : 0;      // stage-1 output column offset in sB
  constexpr int ITEMS = kRowTile * D4 / NT;         // 4
  constexpr int RSTEP = NT / D4;                    // 8
  constexpr int XITEMS = (kRowTile * FP + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) float sA[kRowTile * LDA];
  __shared__ __attribute__((aligned(16))) float sB[kRowTile * LDB];

  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  const int q_me = threadIdx.x % D4, r_me = threadIdx.x / D4;

  // both stages' weight fragments, once per workgroup
  float bf1[D / 2], bf2[K2 / 2];
  if constexpr (KIND == CH_F1 || KIND == CH_F2) {
    frag_t<D>(bf1, a.w1, D, col, h);
  } else if constexpr (KIND == CH_B1) {
    frag_n<D>(bf1, a.w1, a.F + D, a.F, col, h);     // dim_red weight, e columns
  } else {
    frag_n<D>(bf1, a.w1, D, 0, col, h);
  }
  if constexpr (KIND == CH_F1) {
    frag_t<D>(bf2, a.w2, D, col, h);
  } else if constexpr (KIND == CH_F2) {
    frag_dimred<FP, D>(bf2, a.w2, a.F, col, h);
  } else {
    frag_n<D>(bf2, a.w2, D, 0, col, h);
  }
  float bias1 = 0.f, bias2 = 0.f;
  if constexpr (KIND == CH_F1 || KIND == CH_F2) {
    bias1 = a.b1[col] * a.bias1_scale;
    bias2 = a.b2[col];
  }

  auto load_tile = [&](int tile, float4 (&raw)[ITEMS], float (&xr)[XITEMS]) {
    const int64_t n0 = (int64_t)tile * kRowTile;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      int64_t n = n0 + r_me + i * RSTEP;
      n = n < N ? n : N - 1;  // clamped: always issued
      raw[i] = reinterpret_cast<const float4*>(a.in + n * D)[q_me];
    }
    if constexpr (KIND == CH_F2) {
#pragma unroll
      for (int i = 0; i < XITEMS; ++i) {
        const int idx = threadIdx.x + i * NT;      // over [32][FP]
        const int r = idx / FP, c = idx % FP;
        int64_t n = n0 + r;
        n = n < N ? n : N - 1;
        // raw value only: the padding columns are zeroed at the LDS store (a select right
        // behind the load would make the compiler wait for it here, ending the prefetch)
        xr[i] = a.x[n * a.F + min(c, a.F - 1)];
      }
    }
  };

  const TileRange tr = tile_range(num_tiles);
  float4 raw[ITEMS];
  float xr[XITEMS];
  if (tr.first < tr.end) load_tile(tr.first, raw, xr);
  for (int tile = tr.first; tile < tr.end; tile += tr.step) {
    const int64_t n0 = (int64_t)tile * kRowTile;
    __syncthreads();  // previous tile's reads of sA / sB are done
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int r = r_me + i * RSTEP;
      const float4 v = (n0 + r < N) ? raw[i] : f4_zero();
      *reinterpret_cast<float4*>(&sA[r * LDA + 4 * q_me]) = v;
    }
    if constexpr (KIND == CH_F2) {
#pragma unroll
      for (int i = 0; i < XITEMS; ++i) {
        const int idx = threadIdx.x + i * NT;
        if (idx < kRowTile * FP) sB[(idx / FP) * LDB + idx % FP] = idx % FP < a.F ? xr[i] : 0.f;
      }
    }
    __syncthreads();
    if (tile + tr.step < tr.end) load_tile(tile + tr.step, raw, xr);  // next tile in flight
    float ep[16];
    if constexpr (KIND == CH_B1) {  // ReLU mask operand of stage 2, in flight too
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int64_t n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        n = n < N ? n : N - 1;
        ep[r] = a.aux[n * D + col];
      }
    }

    // stage 1
    floatx16 acc = tile_mma<D>(sA, LDA, bf1, c32, h);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t n = n0 + rr;
      const float v = acc[r] + bias1;
      sB[rr * LDB + BOFF + col] = v;
      if (n < N) a.out1[n * D + col] = v;
    }
    __syncthreads();

    // stage 2
    acc = tile_mma<K2>(sB, LDB, bf2, c32, h);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t n = n0 + rr;
      float v = acc[r] + bias2;
      if constexpr (KIND == CH_F1) v = relu_nan(v);              // u = relu(rho[0](s))
      if constexpr (KIND == CH_B1) v = ep[r] > 0.f ? v : 0.f;   // dt = du * 1[u > 0]
      if (n < N) a.out2[n * D + col] = v;
    }
  }
}

// Persistent grid, one workgroup per CU (two per CU measured slower at cfg2: 0.614 vs
// 0.589 ms per step).  GINE_CHAIN_BLOCKS (tuning experiments only) overrides the cap.
inline int chain_grid(int64_t N) {
  static const int cap = [] {
    const char* e = getenv("GINE_CHAIN_BLOCKS");
    return e && atoi(e) > 0 ? atoi(e) : kNumCu;
  }();
  const int64_t tiles = ceil_div(N, kRowTile);
  return (int)std::max<int64_t>(1, std::min<int64_t>(tiles, cap));
}

template <int D, int FP, int KIND>
int launch_chain(const ChainArgs& a, int64_t N, hipStream_t s) {
  const int tiles = (int)ceil_div(N, kRowTile);
  hipLaunchKernelGGL((k_chain<D, FP, KIND>), dim3(chain_grid(N)), dim3(2 * D), 0, s, a, N,
                     tiles);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

// ----------------------------------------------------------------------------------------
// weight gradients of the four Linears, one engine launch (Z = 4)
//   z = 0: dWdr [D x (F+D)] = dh0^T [x | e]     z = 1: dWr1 = de^T u
//   z = 2: dWr0 = dt^T s                         z = 3: dWp2 = ds^T r
// ----------------------------------------------------------------------------------------
struct ChainWgradSrc {
  static constexpr int kZ = 4;
  const float *dh0, *de, *dt, *ds;  // P
  const float *x, *e, *u, *s, *r;   // Q
  int D, F;
  struct Raw {
    float4 v;
  };
  struct Col {
    float keep[4];  // Q of z = 0: 1 for the columns inside [x | e], 0 for the padding
  };
  template <int Z> __device__ int i_dim(int) const { return Z == 0 ? F + D : D; }
  template <int Z> __device__ Col p_col(int) const { return Col{{1.f, 1.f, 1.f, 1.f}}; }
  template <int Z> __device__ Col q_col(int q) const {
    Col c{{1.f, 1.f, 1.f, 1.f}};
    if constexpr (Z == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) c.keep[j] = 4 * q + j < F + D ? 1.f : 0.f;
    }
    return c;
  }
  template <int Z> __device__ Raw p_load(int64_t n, int q) const {
    const float* p = Z == 0 ? dh0 : (Z == 1 ? de : (Z == 2 ? dt : ds));
    return Raw{reinterpret_cast<const float4*>(p + n * D)[q]};
  }
  template <int Z> __device__ Raw q_load(int64_t n, int q) const {
    if constexpr (Z == 0) {  // [x | e]: F + D columns, x rows are not float4-aligned
      const int I = F + D;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = min(4 * q + j, I - 1);
        const float* src = c < F ? x + n * F + c : e + n * D + (c - F);
        v[j] = *src;  // raw: the padding is zeroed in q_xform, when the tile is staged
      }
      return Raw{make_float4(v[0], v[1], v[2], v[3])};
    } else {
      const float* p = Z == 1 ? u : (Z == 2 ? s : r);
      return Raw{reinterpret_cast<const float4*>(p + n * D)[q]};
    }
  }
  template <int Z> __device__ float4 p_xform(const Raw& r, const Col&) const { return r.v; }
  template <int Z> __device__ float4 q_xform(const Raw& r, const Col& c) const {
    if constexpr (Z == 0)
      return make_float4(c.keep[0] != 0.f ? r.v.x : 0.f, c.keep[1] != 0.f ? r.v.y : 0.f,
                         c.keep[2] != 0.f ? r.v.z : 0.f, c.keep[3] != 0.f ? r.v.w : 0.f);
    return r.v;
  }
};

struct ChainWgradOut {
  float* w[4];  // dWdr, dWr1, dWr0, dWp2 (product order)
  float* b[4];
  int D, F;
  float bias_scale;  // phi[2]'s bias enters M times
  __device__ void operator()(int z, int64_t e, double v) const {
    const int64_t I = z == 0 ? F + D : D;
    const int64_t ws = (int64_t)D * I;
    if (e < ws) {
      w[z][e] = (float)v;
    } else if (e < ws + D && b[z] != nullptr) {
      b[z][e - ws] = (float)(z == 3 ? v * (double)bias_scale : v);
    }
  }
};

// output tiles: dim_red's [D x (F+D)] plus three [D x D]
inline int chain_wgrad_tiles(int D, int F) {
  const int to = (int)ceil_div(D, 64);
  return to * (int)ceil_div(F + D, kWgTI) + 3 * to * (int)ceil_div(D, kWgTI);
}
inline WgPlan chain_wgrad_plan(int64_t N, int D, int F) {
  return wg_plan(N, D, F + D, 4, 64, chain_wgrad_tiles(D, F));
}

inline bool chain_dims_ok(int D, int F) { return (D == 64 || D == 128) && F >= 1 && F <= 64; }

#define GINE_CHAIN_DISPATCH(D_, F_, CALL)                          \
  do {                                                             \
    if ((D_) == 64) {                                              \
      if ((F_) <= 40) { CALL(64, 40); } else { CALL(64, 64); }     \
    } else {                                                       \
      if ((F_) <= 40) { CALL(128, 40); } else { CALL(128, 64); }   \
    }                                                              \
  } while (0)

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_chain_fwd(const float* r, const float* x, const float* wp2, const float* bp2,
                              float bias_scale, const float* wr0, const float* br0,
                              const float* wr1, const float* br1, const float* wdr,
                              const float* bdr, float* s, float* u, float* e, float* h0,
                              int64_t num_nodes, int32_t hidden, int32_t in_features,
                              void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes < 0) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  if (num_nodes == 0) return GINE_OK;
  if (!r || !x || !wp2 || !bp2 || !wr0 || !br0 || !wr1 || !br1 || !wdr || !bdr || !s || !u ||
      !e || !h0)
    return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const ChainArgs f1{r, nullptr, nullptr, wp2, bp2, wr0, br0, s, u, bias_scale, in_features};
  const ChainArgs f2{u, x, nullptr, wr1, br1, wdr, bdr, e, h0, 1.f, in_features};
  int rc = GINE_OK;
#define CALL_F(DD, FF)                                                  \
  rc = launch_chain<DD, FF, CH_F1>(f1, num_nodes, st);                  \
  if (rc == GINE_OK) rc = launch_chain<DD, FF, CH_F2>(f2, num_nodes, st)
  GINE_CHAIN_DISPATCH(hidden, in_features, CALL_F);
#undef CALL_F
  return rc;
}

extern "C" int gine_chain_bwd_slab_floats(int64_t num_nodes, int32_t hidden,
                                          int32_t in_features, size_t* floats) {
  if (!floats || num_nodes < 0) return GINE_ERR_INVALID;
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  const WgPlan p = chain_wgrad_plan(num_nodes, hidden, in_features);
  const size_t per = (size_t)hidden * (hidden + in_features) + hidden;
  *floats = 4 * (size_t)p.chunks * per;
  return GINE_OK;
}

extern "C" int gine_chain_bwd(const float* dh0, const float* x, const float* r, const float* s,
                              const float* u, const float* e, const float* wp2,
                              const float* wr0, const float* wr1, const float* wdr, float* de,
                              float* dt, float* ds, float* dr, float* slab, float* dwp2,
                              float* dbp2, float bias_scale, float* dwr0, float* dbr0,
                              float* dwr1, float* dbr1, float* dwdr, float* dbdr,
                              int64_t num_nodes, int32_t hidden, int32_t in_features,
                              void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  if (!dh0 || !x || !r || !s || !u || !e || !wp2 || !wr0 || !wr1 || !wdr || !de || !dt ||
      !ds || !dr)
    return GINE_ERR_INVALID;
  if (slab && (!dwp2 || !dwr0 || !dwr1 || !dwdr)) return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int D = hidden, F = in_features;
  const ChainArgs b1{dh0, nullptr, u, wdr, nullptr, wr1, nullptr, de, dt, 1.f, F};
  const ChainArgs b2{dt, nullptr, nullptr, wr0, nullptr, wp2, nullptr, ds, dr, 1.f, F};
  int rc = GINE_OK;
#define CALL_B(DD, FF)                                                  \
  rc = launch_chain<DD, FF, CH_B1>(b1, num_nodes, st);                  \
  if (rc == GINE_OK) rc = launch_chain<DD, FF, CH_B2>(b2, num_nodes, st)
  GINE_CHAIN_DISPATCH(D, F, CALL_B);
#undef CALL_B
  if (rc != GINE_OK || !slab) return rc;  // no slab: weight gradients via gine_chain_wgrad
  return gine_chain_wgrad(dh0, x, r, s, u, e, de, dt, ds, slab, dwp2, dbp2, bias_scale, dwr0,
                          dbr0, dwr1, dbr1, dwdr, dbdr, num_nodes, hidden, in_features, stream);
}

extern "C" int gine_chain_wgrad(const float* dh0, const float* x, const float* r,
                                const float* s, const float* u, const float* e,
                                const float* de, const float* dt, const float* ds, float* slab,
                                float* dwp2, float* dbp2, float bias_scale, float* dwr0,
                                float* dbr0, float* dwr1, float* dbr1, float* dwdr, float* dbdr,
                                int64_t num_nodes, int32_t hidden, int32_t in_features,
                                void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0) return GINE_ERR_INVALID;
  if (!dh0 || !x || !r || !s || !u || !e || !de || !dt || !ds || !slab) return GINE_ERR_INVALID;
  // all four weight outputs NULL: the slab is left for gine_grad_finalize_batch
  const bool reduce = dwp2 || dwr0 || dwr1 || dwdr;
  if (reduce && (!dwp2 || !dwr0 || !dwr1 || !dwdr)) return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int D = hidden, F = in_features;
  int rc;
  const WgPlan p = chain_wgrad_plan(num_nodes, D, F);
  const size_t per = (size_t)D * (D + F) + D;
  const ChainWgradSrc src{dh0, de, dt, ds, x, e, u, s, r, D, F};
  rc = launch_wgrad_engine<64>(src, num_nodes, D, D + F, chain_wgrad_tiles(D, F), p,
                                per * p.chunks, per, slab, st);
  if (rc != GINE_OK) return rc;
  if (!reduce) return GINE_OK;
  return launch_slab_sum(slab, p.chunks, (int64_t)per, per, per * p.chunks, 4,
                         ChainWgradOut{{dwdr, dwr1, dwr0, dwp2}, {dbdr, dbr1, dbr0, dbp2}, D,
                                       F, bias_scale},
                         st);
}

extern "C" int gine_chain_wgrad_grad_job(int64_t num_nodes, int32_t hidden, int32_t in_features,
                                         const float* slab, float bias_scale, float* dwp2,
                                         float* dbp2, float* dwr0, float* dbr0, float* dwr1,
                                         float* dbr1, float* dwdr, float* dbdr,
                                         gine_grad_job* job) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !slab || !dwp2 || !dwr0 || !dwr1 || !dwdr || !job)
    return GINE_ERR_INVALID;
  const int64_t D = hidden, F = in_features;
  const WgPlan p = chain_wgrad_plan(num_nodes, hidden, in_features);
  const int64_t per = D * (D + F) + D;
  *job = gine_grad_job{};
  job->kind = GINE_GRAD_JOB_SLAB;
  job->src = slab;
  job->rows = p.chunks;
  job->cstride = per;
  job->zstride = per * p.chunks;
  job->nz = 4;
  float* w[4] = {dwdr, dwr1, dwr0, dwp2};  // product order of ChainWgradSrc
  float* b[4] = {dbdr, dbr1, dbr0, dbp2};
  for (int z = 0; z < 4; ++z) {
    const int64_t ws = D * (z == 0 ? F + D : D);
    job->per[z] = ws + D;
    job->wsize[z] = ws;
    job->w[z] = w[z];
    job->b[z] = b[z];
    job->bscale[z] = z == 3 ? bias_scale : 1.0f;
  }
  return GINE_OK;
}
