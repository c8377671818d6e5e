// The node-MLP backward of a GINE layer in one launch (gine_mlp_bwd_layer), D = 128:
//   phase A = gine_mlp_bwd2_acc: do = PRO(dy) (residual mask / ReLU of y / none),
//             dbn = (do W2) * 1[bn(a1) > 0], the BatchNorm-backward sums
//             [sum dbn | sum dbn * xhat] into the fixed-point accumulator (gine_bnacc.hpp);
//   grid barrier (every workgroup resident: one per CU, host-checked);
//   phase B = gine_mlp_bwd1_bn: coef = [c1 | c2 | c3] from the totals (workgroup 0 also
//             writes coef, dgamma, dbeta and the consumed phase), da1 = c1 dbn + c2 xhat + c3,
//             dz = da1 W1.
// Replaces models/gnn.py:21-26's autograd through Linear2 -> ReLU -> BatchNorm1d -> Linear1
// (torch: addmm backward, threshold_backward, native_batch_norm_backward, addmm backward),
// which the two launches above run with a launch boundary where this one has a barrier.
// Same layout as the one-launch forward (gine_mpmlp.hip): 768 threads, waves 0-3 multiply
// ("matrix"), waves 4-11 stage ("helpers"):
//   * the helpers stage both of the workgroup's tiles at once -- do as split-bf16 planes
//     into xp[t] (split once here, not inside the chains), the a1 rows into o[t] -- and W2
//     (then W1, loaded under phase A's chains) through the padded LDS image w;
//   * the matrix waves keep the weight planes in registers (the row GEMM's split-bf16 chain,
//     gine_bf16x3.hpp) and transpose each 32x32 accumulator block through a tile of their
//     own; the helpers run the EPI_DBN epilogue of tile t beside the chain of tile t + 1
//     (double-buffered transposition tiles): dbn overwrites the a1 rows in o[t] and goes to
//     HBM for the weight-gradient engine, and the BatchNorm-backward sums accumulate in the
//     row GEMM's thread mapping;
//   * after the barrier the helpers read the totals beside the matrix waves' W1 fragments
//     (x-hat of their items computed before the totals arrive), then stage da1 as planes --
//     tile 1's beside the chain of tile 0 -- and store the dz rows the matrix waves transpose.
// Bit-identical to the pair: same tile -> workgroup map (xcd tile ranges, grid =
// gine_mlp_num_partials), the same chains (k order, NaN redo on the fp32 chain), the same
// epilogue and prologue arithmetic, the per-workgroup sums in the row GEMM's order (row groups
// r % 8, then the 8 groups in order), integer totals.
#include "gine_common.hpp"
#include "gine_mlpsrc.hpp"
#include "gine_bnacc.hpp"
#include "gine_bf16x3.hpp"

#include <algorithm>
#include <atomic>
#include <mutex>

namespace gine {
namespace {

constexpr int kD = 128, kD4 = kD / 4, kLD = kD + 4, kKS = kD / 2;
constexpr int kRows = 32;                 // rows per tile
constexpr int kMat = 256;                 // waves 0-3
constexpr int kThreads = 768;             // + waves 4-11
constexpr int kHelp = kThreads - kMat;    // 512 helper threads
constexpr int kTiles = 2;                 // tiles a workgroup holds
constexpr int kTLD = 36;                  // per-wave transposition tile row (floats)
constexpr int kItems = kRows * kD4 / kHelp;  // float4 items per helper thread per tile (2)
constexpr int kWPer = kD * kD4 / kHelp;      // float4 of a weight per helper thread (8)
static_assert(kItems == 2 && kWPer == 8 && kTiles == 2, "staging shares");

typedef float floatx16 __attribute__((ext_vector_type(16)));

#ifdef GINE_LAYER_PROFILE
// Debug build only (make variant VDEFS=-DGINE_LAYER_PROFILE): thread 0 of every workgroup
// stamps s_memtime at its phase boundaries (tools/layer_bwd_prof.py): 0 entry, 1 tiles
// staged, 2 W2 planes ready, 3 / 4 tile 1 / 2 epilogue done, 5 sums in the accumulator,
// 6 barrier passed, 7 W1 planes ready, 8 totals read, 9 coef ready, 10 da1 staged, 11 end;
// 16-19 s_memrealtime at entry, arrival, release and the end.
__device__ long long g_bwd_layer_prof[1024][24];
#define BL_MARK(i)                                                                  \
  do {                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < 1024)                                      \
      g_bwd_layer_prof[blockIdx.x][i] = (long long)__builtin_amdgcn_s_memtime();     \
  } while (0)
#define BL_RT(i)                                                                    \
  do {                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < 1024)                                      \
      g_bwd_layer_prof[blockIdx.x][i] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define BL_MARK(i) do {} while (0)
#define BL_RT(i) do {} while (0)
#endif

struct BwdLayerArgs {
  const float* dy;
  const float* y;        // PRO_DOR
  const uint8_t* mask;   // PRO_DOM
  const float* a1;
  const float* bn_save;  // [mean | invstd | alpha | shift]
  const float* W2;
  const float* W1;
  const float* gamma;
  float* dbn;
  float* dz;
  float* coef;
  float* dgamma;
  float* dbeta;
  long long* acc;
  int N, num_tiles;
};

constexpr int kPS = kD + 8;  // plane row stride (bf16): 272-byte rows, conflict-free b128 reads
struct BwdLayerLds {
  float w[kD * kLD];              // W2 image; per-wave transposition tiles + sums; W1 image
  // the staged A operands -- do (phase A), da1 (phase B) -- as split-bf16 planes hi | mid | lo
  // (gine_bf16x3.hpp split2), split once by the helpers: a matrix wave's chain then reads
  // them (2,046 instead of 3,081 shader ticks per 32x32 block at one wave per SIMD, where
  // the in-loop split's VALU work adds to the MFMA chain instead of hiding under it;
  // tools/chain_micro.py, profiles/r05_s18_chain_micro.txt)
  uint16_t xp[kTiles][3][kRows * kPS];
  float o[kTiles][kRows * kLD];   // a1 rows, overwritten in place by dbn
  float bnp[4 * kD];              // bn_save: mean | invstd | alpha | shift
  double tot[2 * kD];
  float coef[3 * kD];
  int barrier_failed;
};
static_assert(kTiles * 4 * 32 * kTLD * 4 + 2 * 8 * kD * 8 <= kD * kLD * 4, "scratch fits in w");

// The row GEMM's tile -> workgroup assignment (gine_mlp.hip xcd_tile_range).
struct Tiles {
  int first, end, step;
  __device__ int count() const { return first < end ? (end - first + step - 1) / step : 0; }
  __device__ int at(int k) const { return first + k * step; }
};
__device__ __forceinline__ Tiles tiles_of(int num_tiles, int vb, int nb) {
  const int xcd = vb % kNumXcd, pos = vb / kNumXcd;
  const int here = nb / kNumXcd + (xcd < nb % kNumXcd ? 1 : 0);
  const int span = (num_tiles + kNumXcd - 1) / kNumXcd;
  const int b = xcd * span;
  return Tiles{b + pos, min(num_tiles, b + span), here};
}

// A weight (row-major [D][D], 16 KB-float image) staged by the helpers: 8 float4 per thread.
struct WRegs {
  float4 v0, v1, v2, v3, v4, v5, v6, v7;
  __device__ __forceinline__ void load(const float4* __restrict__ w4, int p) {
    v0 = w4[p]; v1 = w4[p + kHelp]; v2 = w4[p + 2 * kHelp]; v3 = w4[p + 3 * kHelp];
    v4 = w4[p + 4 * kHelp]; v5 = w4[p + 5 * kHelp]; v6 = w4[p + 6 * kHelp];
    v7 = w4[p + 7 * kHelp];
  }
  __device__ __forceinline__ void put(float* w, int idx, float4 v) const {
    *reinterpret_cast<float4*>(&w[(idx / kD4) * kLD + 4 * (idx % kD4)]) = v;
  }
  __device__ __forceinline__ void store(float* w, int p) const {
    put(w, p, v0); put(w, p + kHelp, v1); put(w, p + 2 * kHelp, v2); put(w, p + 3 * kHelp, v3);
    put(w, p + 4 * kHelp, v4); put(w, p + 5 * kHelp, v5); put(w, p + 6 * kHelp, v6);
    put(w, p + 7 * kHelp, v7);
  }
};

// dX = dY W fragments (B[k][j] = W[k][j]): lane half h takes k in [h*64, h*64 + 64) of
// column col, read down the staged image (the row GEMM's BT = false fragment).
__device__ __forceinline__ void w_fragments(const float* w, int col, int h, float (&bf)[kKS]) {
#pragma unroll
  for (int s = 0; s < kKS; ++s) bf[s] = w[(h * kKS + s) * kLD + col];
}

// Split a staged float4 item (row r, k = 4q .. 4q + 3) into the three planes of tile t.
__device__ __forceinline__ void put_planes(uint16_t (*xp)[kRows * kPS], int r, int q, float4 v) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split2(v.x, v.y, h0, m0, l0);
  split2(v.z, v.w, h1, m1, l1);
  const int e = r * kPS + 4 * q;
  *reinterpret_cast<uint2*>(&xp[0][e]) = make_uint2(h0, h1);
  *reinterpret_cast<uint2*>(&xp[1][e]) = make_uint2(m0, m1);
  *reinterpret_cast<uint2*>(&xp[2][e]) = make_uint2(l0, l1);
}

// One 32x32 block of a tile: A = the staged planes, B = the lane's weight planes (the row
// GEMM's split chain, the same k order and products).  A wave whose accumulators see a NaN
// redoes the block on the fp32 chain of the row GEMM's redo (mfma_f32_row_mem's order), with
// A[row c32][h*64 + k] from `aval(k)` -- the staged values recomputed from their sources.
template <class AVal>
__device__ __forceinline__ floatx16 chain(const uint16_t (*xp)[kRows * kPS],
                                          const BPlanes<kKS>& bp, const float* __restrict__ W,
                                          int col, int h, int c32, const AVal& aval) {
  const int e = c32 * kPS + h * kKS;
  floatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
  for (int s = 0; s < kKS / 8; ++s) {
    Bf16x3 a;
    a.h = *reinterpret_cast<const bf16x8_t*>(&xp[0][e + 8 * s]);
    a.m = *reinterpret_cast<const bf16x8_t*>(&xp[1][e + 8 * s]);
    a.l = *reinterpret_cast<const bf16x8_t*>(&xp[2][e + 8 * s]);
    acc = mfma_bf16x3(a, bp.f[s], acc);
  }
  if (wave_any_nan(acc)) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const float* wp = W + (size_t)h * kKS * kD + col;
#pragma unroll 1
    for (int q = 0; q < kKS / 4; ++q) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(aval(4 * q), wp[(4 * q) * kD], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(aval(4 * q + 1), wp[(4 * q + 1) * kD], acc, 0,
                                                 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(aval(4 * q + 2), wp[(4 * q + 2) * kD], acc, 0,
                                                 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(aval(4 * q + 3), wp[(4 * q + 3) * kD], acc, 0,
                                                 0, 0);
    }
  }
  return acc;
}

// Transposition tiles in w, one per (tile, matrix wave): the helpers finish tile t while the
// matrix waves chain tile t + 1.  Then the epilogue's sums scratch.
__device__ __forceinline__ float* tt_of(float* w, int t, int wave) {
  return w + (t * 4 + wave) * 32 * kTLD;
}
__device__ __forceinline__ double* sums_of(float* w) {
  return reinterpret_cast<double*>(w + kTiles * 4 * 32 * kTLD);
}

// this wave's 32x32 block -> row-major through its own LDS tile
__device__ __forceinline__ void transpose_in(float* tt, const floatx16& acc, int h, int c32) {
#pragma unroll
  for (int r = 0; r < 16; ++r) tt[((r & 3) + 8 * (r >> 2) + 4 * h) * kTLD + c32] = acc[r];
  __builtin_amdgcn_wave_barrier();
}

template <int PRO>
__global__ __launch_bounds__(kThreads, 1) void k_mlp_bwd_layer(BwdLayerArgs A) {
  __shared__ __attribute__((aligned(16))) BwdLayerLds L;
  const Tiles ts = tiles_of(A.num_tiles, blockIdx.x, gridDim.x);
  const int nt = ts.count();
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const bool mat = wave < kMat / kWave;
  const int lane = tid % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = 32 * wave + c32;           // (matrix waves)
  const int p = tid - kMat;                   // (helpers)
  long long* phw = bnacc_phase(A.acc, 2 * kD);
  // written by earlier launches only (workgroup 0 moves them after the barrier)
  const long long ph = phw[0] + 1, consumed = phw[1 + ((ph - 1) & 1)];
  const BnView bv = bn_view(A.bn_save, kD);
  BL_MARK(0);
  BL_RT(16);

  // ---- phase A staging: W2 and both tiles (helpers) ----
  if (!mat) {
    WRegs w2;
    w2.load(reinterpret_cast<const float4*>(A.W2), p);
    ProArgs pa{A.dy, A.y, A.mask, nullptr, nullptr};
    RawItem raw[kTiles][kItems];
    float4 a1v[kTiles][kItems];
#pragma unroll
    for (int t = 0; t < kTiles; ++t)
#pragma unroll
      for (int j = 0; j < kItems; ++j) {
        const int e = p + kHelp * j, r = e / kD4, q = e % kD4;
        int64_t n = (int64_t)ts.at(t < nt ? t : 0) * kRows + r;
        n = n < A.N ? n : A.N - 1;
        raw[t][j] = raw_load<PRO>(pa, kD, n, q);
        a1v[t][j] = *reinterpret_cast<const float4*>(A.a1 + n * kD + 4 * q);
      }
    w2.store(L.w, p);
    if (p < kD) *reinterpret_cast<float4*>(&L.bnp[4 * p]) =
        *reinterpret_cast<const float4*>(A.bn_save + 4 * p);
    const ColConst kc{};
#pragma unroll
    for (int t = 0; t < kTiles; ++t)
#pragma unroll
      for (int j = 0; j < kItems; ++j) {
        const int e = p + kHelp * j, r = e / kD4, q = e % kD4;
        float4 v = transform<PRO>(pa, raw[t][j], kc);
        if (t >= nt || (int64_t)ts.at(t) * kRows + r >= A.N) v = f4_zero();
        put_planes(L.xp[t], r, q, v);
        *reinterpret_cast<float4*>(&L.o[t][r * kLD + 4 * q]) = a1v[t][j];
      }
  }
  __syncthreads();  // S1: W2 and the tiles staged
  BL_MARK(1);

  if (mat) {
    // ---- phase A: dbn = (do W2) * 1[bn(a1) > 0], BatchNorm-backward sums ----
    float bf[kKS];
    w_fragments(L.w, col, h, bf);
    BPlanes<kKS> bp;
    bp.from(bf);
    __syncthreads();  // S2: every wave's fragment reads of w are done (transposition tiles)
    BL_MARK(2);
    for (int t = 0; t < kTiles; ++t) {  // (the barriers are uniform: kTiles of them)
      if (t < nt) {
        const int64_t nrow = (int64_t)ts.at(t) * kRows + c32;  // this lane's A row
        const floatx16 acc = chain(L.xp[t], bp, A.W2, col, h, c32, [&](int k) -> float {
          if (nrow >= A.N) return 0.f;  // (rows past N are staged as zero)
          const int64_t off = nrow * kD + h * kKS + k;
          const float v = A.dy[off];
          if constexpr (PRO == PRO_DOM) return A.mask[off] ? v : 0.f;
          else if constexpr (PRO == PRO_DOR) return A.y[off] > 0.f ? v : 0.f;
          else return v;
        });
        transpose_in(tt_of(L.w, t, wave), acc, h, c32);
      }
      __syncthreads();  // E_t: tile t's blocks transposed (the helpers' epilogue follows)
      BL_MARK(3 + t);
    }
    __syncthreads();  // X: the epilogue's sums in sr
    BL_MARK(5);
    __syncthreads();  // S3: phase A's use of w is over (the accumulator holds the sums)
  } else {
    __syncthreads();  // S2
    // W1, in flight under phase A's chains
    WRegs w1;
    w1.load(reinterpret_cast<const float4*>(A.W1), p);
    // The EPI_DBN epilogue of tile t beside the matrix waves' chain of tile t + 1: thread
    // p < 256 takes the (row group, column chunk) slot of lane p % 64 of matrix wave p / 64
    // -- the row GEMM's thread mapping, so the BatchNorm-backward sums accumulate in its order
    const bool epi = p < kMat;
    const int ew = p >> 6, el = p & 63;
    const int eg = el >> 3, ecq = el & 7;
    const int c0 = 32 * ew + 4 * ecq;
    double st1[4] = {0.0, 0.0, 0.0, 0.0}, st2[4] = {0.0, 0.0, 0.0, 0.0};
    for (int t = 0; t < kTiles; ++t) {
      __syncthreads();  // E_t
      if (!epi || t >= nt) continue;
      const float* tt = tt_of(L.w, t, ew);
      const float4 mu4 = *reinterpret_cast<const float4*>(&L.bnp[c0]);
      const float4 is4 = *reinterpret_cast<const float4*>(&L.bnp[kD + c0]);
      const float4 al4 = *reinterpret_cast<const float4*>(&L.bnp[2 * kD + c0]);
      const float4 sh4 = *reinterpret_cast<const float4*>(&L.bnp[3 * kD + c0]);
      const float al[4] = {al4.x, al4.y, al4.z, al4.w}, sh[4] = {sh4.x, sh4.y, sh4.z, sh4.w};
      const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, is[4] = {is4.x, is4.y, is4.z, is4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = eg + 8 * i;
        const int64_t n = (int64_t)ts.at(t) * kRows + row;
        const float4 v = *reinterpret_cast<const float4*>(&tt[row * kTLD + 4 * ecq]);
        if (n >= A.N) continue;
        float* slot = &L.o[t][row * kLD + c0];
        const float4 a14 = *reinterpret_cast<const float4*>(slot);
        const float vv[4] = {v.x, v.y, v.z, v.w};
        const float a1[4] = {a14.x, a14.y, a14.z, a14.w};
        float o4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // EPI_DBN of the row GEMM
          const float bn = bn_apply(a1[k], al[k], sh[k]);
          o4[k] = (bn > 0.f) ? vv[k] : 0.f;
          const double xhat = (double)((a1[k] - mu[k]) * is[k]);
          st1[k] += (double)o4[k];
          st2[k] += (double)o4[k] * xhat;
        }
        const float4 ov = make_float4(o4[0], o4[1], o4[2], o4[3]);
        *reinterpret_cast<float4*>(slot) = ov;
        *reinterpret_cast<float4*>(A.dbn + n * kD + c0) = ov;
      }
    }
    // per-column sums: the 8 row groups added in fixed order (row-tile GEMM order)
    double* sr = sums_of(L.w);  // [2][8][kD]
    if (epi) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sr[(0 * 8 + eg) * kD + c0 + k] = st1[k];
        sr[(1 * 8 + eg) * kD + c0 + k] = st2[k];
      }
    }
    __syncthreads();  // X
    if (epi) {
      const int which = el >> 5, cc = 32 * ew + (el & 31);
      double sum = 0.0;
#pragma unroll
      for (int g = 0; g < 8; ++g) sum += sr[(which * 8 + g) * kD + cc];
      bnacc_add<false>(A.acc, 2 * kD, which * kD + cc, sum);
      // the atomics are performed before this workgroup arrives at the grid barrier
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // S3
    w1.store(L.w, p);
  }

  BL_RT(17);
  if (tid == 0)
    L.barrier_failed = grid_barrier(bnacc_barrier(A.acc, 2 * kD), gridDim.x) ? 0 : 1;
  __syncthreads();  // S4: barrier passed; W1 staged
  BL_MARK(6);
  BL_RT(18);
  // a timed-out barrier (the grid was not co-resident): the totals are incomplete, so this
  // workgroup's coefficients and outputs are NaN; the failure word tells the host
  const bool failed = L.barrier_failed != 0;

  // ---- phase B: W1's fragments (matrix) beside the totals, coef and the da1 planes
  // (helpers); each role in a branch of its own, so that neither holds the other's registers
  if (mat) {
    float bf1[kKS];
    w_fragments(L.w, col, h, bf1);
    BPlanes<kKS> bp1;
    bp1.from(bf1);
    BL_MARK(7);
    __syncthreads();  // S5: totals in LDS
    BL_MARK(8);
    if (blockIdx.x == 0 && tid == 0) {
      phw[0] = ph;
      phw[1 + (ph & 1)] = ph;  // bnacc_mark_consumed
    }
    __syncthreads();  // S6: coef in LDS
    BL_MARK(9);
    __syncthreads();  // S7: tile 0's da1 staged (tile 1's follows beside chain 0)
    BL_MARK(10);
    for (int t = 0; t < kTiles; ++t) {  // dz = da1 W1 (EPI_PLAIN: stored by the helpers)
      if (t < nt) {
        const int64_t nrow = (int64_t)ts.at(t) * kRows + c32;
        const floatx16 acc = chain(L.xp[t], bp1, A.W1, col, h, c32, [&](int k) -> float {
          if (nrow >= A.N) return 0.f;
          const int kk = h * kKS + k;
          const float v = L.o[t][c32 * kLD + kk];
          const float a1 = A.a1[nrow * kD + kk];
          return L.coef[kk] * v + L.coef[kD + kk] * ((a1 - L.bnp[kk]) * L.bnp[kD + kk]) +
                 L.coef[2 * kD + kk];  // transform<PRO_DA1>'s expression
        });
        transpose_in(tt_of(L.w, t, wave), acc, h, c32);
      }
      __syncthreads();  // F_t: tile t's dz blocks transposed (F_0: tile 1's da1 staged)
    }
  } else {
    // the a1 rows of this thread's items, in flight under the totals (named registers: an
    // array held across the barriers went to scratch)
    auto a1_at = [&](int t, int j) {
      const int e = p + kHelp * j, r = e / kD4, q = e % kD4;
      int64_t n = (int64_t)ts.at(t < nt ? t : 0) * kRows + r;
      n = n < A.N ? n : A.N - 1;
      return *reinterpret_cast<const float4*>(A.a1 + n * kD + 4 * q);
    };
    // xhat = (a1 - mean) * invstd of these items now (transform<PRO_DA1>'s inner product,
    // the same operations), so that the staging behind the totals is three FMAs' worth
    auto xhat_of = [&](int j, float4 a) {
      const int q = (p + kHelp * j) % kD4;
      const float4 mu = *reinterpret_cast<const float4*>(&L.bnp[4 * q]);
      const float4 is = *reinterpret_cast<const float4*>(&L.bnp[kD + 4 * q]);
      return make_float4((a.x - mu.x) * is.x, (a.y - mu.y) * is.y, (a.z - mu.z) * is.z,
                         (a.w - mu.w) * is.w);
    };
    const float4 xh00 = xhat_of(0, a1_at(0, 0)), xh01 = xhat_of(1, a1_at(0, 1)),
                 xh10 = xhat_of(0, a1_at(1, 0)), xh11 = xhat_of(1, a1_at(1, 1));
    if (p < 2 * kD) {
      const double t = bnacc_total<true>(A.acc, 2 * kD, p, blockIdx.x == 0, ph, consumed);
      L.tot[p] = failed ? __builtin_nan("") : t;
    }
    __syncthreads();  // S5
    if (p < kD) {  // the arithmetic of k_bwd1_bnacc's prologue
      const double sd = L.tot[p], sx = L.tot[kD + p];
      const double g = A.gamma ? (double)A.gamma[p] : 1.0;
      const double c1 = g * (double)bv.invstd[p];
      const float k1 = (float)c1, k2 = (float)(-c1 * sx / (double)A.N),
                  k3 = (float)(-c1 * sd / (double)A.N);
      L.coef[p] = k1;
      L.coef[kD + p] = k2;
      L.coef[2 * kD + p] = k3;
      if (blockIdx.x == 0) {
        if (A.dgamma) A.dgamma[p] = (float)sx;
        if (A.dbeta) A.dbeta[p] = (float)sd;
        A.coef[p] = k1;
        A.coef[kD + p] = k2;
        A.coef[2 * kD + p] = k3;
      }
    }
    __syncthreads();  // S6
    // da1 = PRO_DA1(dbn) as split planes (rows past N zero, as the row GEMM stages them):
    // c1 dbn + c2 xhat + c3, transform<PRO_DA1>'s expression.  Tile 0 first; tile 1 beside
    // the matrix waves' chain of tile 0.
    auto stage = [&](int t, int j, float4 xh) {
      const int e = p + kHelp * j, r = e / kD4, q = e % kD4;
      const float4 v0 = *reinterpret_cast<const float4*>(&L.o[t][r * kLD + 4 * q]);
      const float4 c1 = *reinterpret_cast<const float4*>(&L.coef[4 * q]);
      const float4 c2 = *reinterpret_cast<const float4*>(&L.coef[kD + 4 * q]);
      const float4 c3 = *reinterpret_cast<const float4*>(&L.coef[2 * kD + 4 * q]);
      float4 v = make_float4(c1.x * v0.x + c2.x * xh.x + c3.x, c1.y * v0.y + c2.y * xh.y + c3.y,
                             c1.z * v0.z + c2.z * xh.z + c3.z, c1.w * v0.w + c2.w * xh.w + c3.w);
      if (t >= nt || (int64_t)ts.at(t) * kRows + r >= A.N) v = f4_zero();
      put_planes(L.xp[t], r, q, v);
    };
    stage(0, 0, xh00);
    stage(0, 1, xh01);
    __syncthreads();  // S7
    stage(1, 0, xh10);
    stage(1, 1, xh11);
    for (int t = 0; t < kTiles; ++t) {  // dz rows of tile t beside the chain of tile t + 1
      __syncthreads();  // F_t
      if (p >= kMat || t >= nt) continue;
      const int ew = p >> 6, el = p & 63, eg = el >> 3, ecq = el & 7;
      const float* tt = tt_of(L.w, t, ew);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = eg + 8 * i;
        const int64_t n = (int64_t)ts.at(t) * kRows + row;
        const float4 v = *reinterpret_cast<const float4*>(&tt[row * kTLD + 4 * ecq]);
        if (n < A.N) *reinterpret_cast<float4*>(A.dz + n * kD + 32 * ew + 4 * ecq) = v;
      }
    }
  }
  BL_MARK(11);
  BL_RT(19);
}

int bwd_layer_capacity() {
  static std::mutex mu;
  static int cap[64];
  static bool known[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  std::lock_guard<std::mutex> lock(mu);
  if (!known[dev]) {
    int cus = 0, c = 1 << 30;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    const void* ks[] = {(const void*)k_mlp_bwd_layer<PRO_PLAIN>,
                        (const void*)k_mlp_bwd_layer<PRO_DOR>,
                        (const void*)k_mlp_bwd_layer<PRO_DOM>};
    for (const void* k : ks) {
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kThreads, 0) != hipSuccess)
        return 0;
      c = std::min(c, nb * cus);
    }
    cap[dev] = c;
    known[dev] = true;
  }
  return cap[dev];
}

// Largest number of tiles one workgroup walks (tiles_of).
int max_tiles(int tiles, int grid) {
  const int span = (tiles + kNumXcd - 1) / kNumXcd;
  int worst = 0;
  for (int xcd = 0; xcd < kNumXcd; ++xcd) {
    const int here = grid / kNumXcd + (xcd < grid % kNumXcd ? 1 : 0);
    const int range = std::max(0, std::min(tiles, (xcd + 1) * span) - xcd * span);
    if (range > 0 && here == 0) return 1 << 30;
    if (range > 0) worst = std::max(worst, (range + here - 1) / here);
  }
  return worst;
}

// gine_testing_bwd_layer_extra_workgroups: workgroups added to the grid (0 in production),
// for the test of the grid barrier's failure path
std::atomic<int> g_bwd_layer_extra{0};

bool bwd_layer_ok(int64_t num_nodes, int32_t channels) {
  if (channels != kD || num_nodes <= 0 || num_nodes * channels * 4 >= (int64_t(1) << 32))
    return false;
  int32_t grid = 0;
  if (gine_mlp_num_partials(num_nodes, channels, &grid) != GINE_OK) return false;
  const int tiles = (int)ceil_div(num_nodes, kRows);
  return grid <= bwd_layer_capacity() && max_tiles(tiles, grid) <= kTiles;
}

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_testing_bwd_layer_extra_workgroups(int32_t extra) {
  if (extra < 0 || extra > 4096) return GINE_ERR_INVALID;
  g_bwd_layer_extra.store(extra);
  return GINE_OK;
}

extern "C" int gine_mlp_bwd_layer_ok(int64_t num_nodes, int32_t channels, int32_t* ok) {
  if (!ok) return GINE_ERR_INVALID;
  *ok = bwd_layer_ok(num_nodes, channels) ? 1 : 0;
  return GINE_OK;
}

extern "C" int gine_mlp_bwd_layer(const float* dy, const float* y, const uint8_t* mask,
                                  const float* a1, const float* bn_save, const float* w2,
                                  float* dbn, int64_t* bn_acc, const float* gamma,
                                  float* dgamma, float* dbeta, float* coef, const float* w1,
                                  float* dz, int64_t num_nodes, int32_t channels,
                                  int32_t epilogue, void* stream) {
  if (channels != kD) return GINE_ERR_DIM;
  if (!dy || !a1 || !bn_save || !w2 || !dbn || !bn_acc || !coef || !w1 || !dz)
    return GINE_ERR_INVALID;
  if (epilogue < GINE_EPI_NONE || epilogue > GINE_EPI_RESIDUAL_RELU) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RELU && !y) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && !mask) return GINE_ERR_INVALID;
  if (!bwd_layer_ok(num_nodes, channels)) return GINE_ERR_INVALID;
  int32_t grid = 0;
  const int st = gine_mlp_num_partials(num_nodes, channels, &grid);
  if (st != GINE_OK) return st;
  grid += g_bwd_layer_extra.load();
  const BwdLayerArgs A{dy,  y,    mask,  a1,     bn_save, w2, w1, gamma,
                       dbn, dz,   coef,  dgamma, dbeta,   reinterpret_cast<long long*>(bn_acc),
                       (int)num_nodes, (int)ceil_div(num_nodes, kRows)};
  hipStream_t s = as_stream(stream);
  switch (epilogue) {
    case GINE_EPI_NONE:
      hipLaunchKernelGGL(k_mlp_bwd_layer<PRO_PLAIN>, dim3((unsigned)grid), dim3(kThreads), 0, s,
                         A);
      break;
    case GINE_EPI_RELU:
      hipLaunchKernelGGL(k_mlp_bwd_layer<PRO_DOR>, dim3((unsigned)grid), dim3(kThreads), 0, s, A);
      break;
    default:
      hipLaunchKernelGGL(k_mlp_bwd_layer<PRO_DOM>, dim3((unsigned)grid), dim3(kThreads), 0, s, A);
  }
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

#ifdef GINE_LAYER_PROFILE
extern "C" int gine_debug_bwd_layer_prof(long long* out) {  // [1024][24] host buffer
  GINE_RETURN_IF_HIP(hipDeviceSynchronize());
  GINE_RETURN_IF_HIP(
      hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd_layer_prof), sizeof(g_bwd_layer_prof)));
  return GINE_OK;
}
#endif
