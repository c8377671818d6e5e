// Node MLP of the GINE layer on gfx950 fp32 matrix cores.
//
// Replaces nn = Sequential(Linear(D,D), BatchNorm1d(D), ReLU(), Linear(D,D))
// (models/gnn.py:21-26) applied by GINEConv to z, plus ResGnn's outer ReLU / residual
// (models/gnn.py:38-44), forward (train and eval BN) and backward.
//
// All four node GEMMs are [N x D] x [D x D] with D <= 256: tall-skinny.  One kernel shape
// serves them all (k_rowgemm): a workgroup of D/32 waves, wave w owns output columns
// [32w, 32w+32); the whole [D x 32] slice of the weight for that wave lives in VGPRs as
// v_mfma_f32_32x32x2_f32 B fragments (D/2 registers), loaded once per workgroup; 32-row
// tiles of the activation are staged through LDS by the workgroup with the elementwise
// prologue fused (BN-normalise + ReLU, ReLU-mask of the upstream gradient, BN backward),
// and the epilogue is fused too (bias, BN statistics, ReLU / residual, ReLU mask).
//
// The contraction index k is split between the two lane halves of the MFMA operand
// (lane half h takes k in [h*D/2, (h+1)*D/2)); A and B use the same permutation so the
// product is unchanged, and each lane's A fragments become contiguous in LDS, so four
// k-steps are fetched with one ds_read_b128 (row stride D+4 floats: conflict-free).
//
// Weight gradients (K = N rows) run on the shared engine of gine_wgrad.hpp (64x128 output
// tiles x row chunks, fp32 partial slabs) and are reduced in fixed chunk order in fp64 by
// k_slab_sum (gine_slab.hpp) -> deterministic.
#include "gine_common.hpp"
#include "gine_reduce.hpp"
#include "gine_slab.hpp"
#include "gine_wgrad.hpp"
#include "gine_mlpsrc.hpp"
#include "gine_bnacc.hpp"
#include "gine_bf16x3.hpp"

#include <algorithm>
#include <mutex>
#include <type_traits>

namespace gine {
namespace {

#ifdef GINE_RG_PROFILE
// Debug build only (make rgprof): workgroup 0 / thread 0 stamps s_memtime at the phase
// boundaries of the row-tile GEMM into LDS (no global access between the stamps, so no
// vmcnt wait is introduced) and flushes them at the end; tools/rg_prof.py reads them.
__device__ long long g_rg_prof[4096];
__device__ int g_rg_prof_n;
#define RG_DECL                    \
  __shared__ long long s_rgp[64];  \
  int rg_n = 0
#define RG_MARK(tag)                                                                  \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    if (vb == 0 && threadIdx.x == 0 && rg_n < 32) {                                   \
      long long t_;                                                                   \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_));              \
      s_rgp[2 * rg_n] = (tag);                                                        \
      s_rgp[2 * rg_n + 1] = t_;                                                       \
      ++rg_n;                                                                         \
    }                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                \
  } while (0)
#define RG_FLUSH()                                                                    \
  do {                                                                                \
    if (vb == 0 && threadIdx.x == 0) {                                                \
      const int b_ = atomicAdd(&g_rg_prof_n, rg_n);                                   \
      for (int i_ = 0; i_ < rg_n && b_ + i_ < 2040; ++i_) {                           \
        g_rg_prof[2 * (b_ + i_)] = s_rgp[2 * i_];                                     \
        g_rg_prof[2 * (b_ + i_) + 1] = s_rgp[2 * i_ + 1];                             \
      }                                                                               \
    }                                                                                 \
  } while (0)
#else
#define RG_DECL do {} while (0)
#define RG_MARK(tag) do {} while (0)
#define RG_FLUSH() do {} while (0)
#endif

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ floatx16 zero16() {
  floatx16 v;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = 0.f;
  return v;
}

constexpr int kRowTile = 32;

struct EpiArgs {
  const float* bias;   // b1 (A1STATS) / b2 (OUT)
  float* out;          // a1 | y | dbn | dz
  uint8_t* mask_out;   // OUT, residual epilogue
  const float* resid;  // OUT, residual epilogue: the layer input x
  const float* a1;     // DBN
  const float* bn;     // DBN
  double* partials;    // A1STATS / DBN: [grid][2][D]  (A1STATS: may be NULL with bnacc)
  int mode;            // OUT: GINE_EPI_*
  long long* bnacc = nullptr;  // A1STATS / DBN: fixed-point accumulator (gine_bnacc.hpp)
};

// Tiles of one XCD form a contiguous range; its blocks stride that range.
struct TileRange {
  int first, end, step;
};
__device__ __forceinline__ TileRange xcd_tile_range(int num_tiles, int vb, int nb) {
  const int xcd = vb % kNumXcd, pos = vb / kNumXcd;
  const int here = nb / kNumXcd + (xcd < nb % kNumXcd ? 1 : 0);
  const int span = (num_tiles + kNumXcd - 1) / kNumXcd;
  const int b = xcd * span;
  return TileRange{b + pos, min(num_tiles, b + span), here};
}

// ----------------------------------------------------------------------------------------
// Row-tile GEMM: out[n][j] = epi( sum_k pro(X)[n][k] * B[k][j] )
//   BT = true : B[k][j] = W[j][k]   (Y = X W^T, forward Linear)
//   BT = false: B[k][j] = W[k][j]   (dX = dY W, backward Linear)
// ----------------------------------------------------------------------------------------
// ----------------------------------------------------------------------------------------
// Row-tile GEMM: out[n][j] = epi( sum_k pro(X)[n][k] * B[k][j] )
//   BT = true : B[k][j] = W[j][k]   (Y = X W^T, forward Linear)
//   BT = false: B[k][j] = W[k][j]   (dX = dY W, backward Linear)
// Persistent: about one workgroup per CU walks a contiguous (XCD-local) range of 32-row
// tiles.  Per tile: the raw inputs of the NEXT tile and the epilogue operands of THIS tile
// are loaded into registers before this tile's 64-long MFMA chain, so HBM latency hides
// under the matrix pipe instead of serialising with it.
// ----------------------------------------------------------------------------------------
// One persistent workgroup (virtual index vb of vgrid) of the row-tile GEMM; s_x: LDS of
// kRowTile * (D + 4) floats.
// The fp32 re-do of a non-finite tile (gine_bf16x3.hpp) with the lane's B fragment read
// from W: W^T fragment (BT / WL: b[s] = W[col][h*KS + s]) or W fragment (b[s] = W[h*KS + s][col]).
template <int D, int KS, bool BT>
__device__ __forceinline__ floatx16 redo_fp32(const float* arow, const float* __restrict__ W,
                                              int col, int h) {
  return BT ? mfma_f32_row_mem<KS>(arow, W + (size_t)col * D + h * KS, 1, zero16())
            : mfma_f32_row_mem<KS>(arow, W + (size_t)h * KS * D + col, D, zero16());
}

struct NoHook {
  __device__ void operator()() const {}
};

// hook: runs once per workgroup after the weight staging and before the prologue constants
// are read (k_fwd2_bnacc: the BatchNorm finish, overlapping the first tile's loads).
template <int D, int PRO, int EPI, bool BT, bool WL = false, class Hook = NoHook>
__device__ __forceinline__ void rowgemm_body(const float* __restrict__ W, const ProArgs& pa,
                                             const EpiArgs& ea, int64_t N, int num_tiles,
                                             float* __restrict__ s_x, int vb, int vgrid,
                                             const Hook& hook = Hook{}) {
  constexpr int NT = 2 * D;      // threads: D/32 waves
  constexpr int KS = D / 2;      // k-steps per lane half
  constexpr int LD = D + 4;      // padded LDS row (floats)
  constexpr int D4 = D / 4;
  constexpr int ITEMS = kRowTile * D4 / NT;  // float4 staged per thread (= 4)
  constexpr int RSTEP = NT / D4;             // row step between a thread's items (= 8)
  constexpr bool IS_OUT = (EPI == EPI_OUT) || (EPI == EPI_OUT_RELU) || (EPI == EPI_OUT_RES);
  constexpr bool EPI_LOAD = (EPI == EPI_DBN) || (EPI == EPI_OUT_RES);

  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  const int q_me = threadIdx.x % D4, r_me = threadIdx.x / D4;
  RG_DECL;
  RG_MARK(0);

  float bf[KS];
  // WL: W^T fragments via LDS.  A lane's fragment is 64 consecutive floats of ONE row of W,
  // so direct loads touch 64 cache lines per instruction (16 B used of each): ~4K line
  // lookups per workgroup, the bulk of the kernel's start-up.  Instead the workgroup reads
  // W with unit-stride 16-byte loads (8 lines per instruction), writes it to the padded
  // LDS tile (s_x holds D*(D+4) floats in this variant) and reads the fragments from there.
  constexpr int WCH = D * D4 / NT;  // float4 chunks of W per thread
  float4 wtmp[WL ? WCH : 1];
  if constexpr (WL) {
    const float4* w4 = reinterpret_cast<const float4*>(W);
#pragma unroll
    for (int j = 0; j < WCH; ++j) wtmp[j] = w4[threadIdx.x + NT * j];
  } else if constexpr (BT) {
    const float4* wr = reinterpret_cast<const float4*>(W + (size_t)col * D + h * KS);
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
      const float4 v = wr[q];
      bf[4 * q] = v.x;
      bf[4 * q + 1] = v.y;
      bf[4 * q + 2] = v.z;
      bf[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) bf[s] = W[(size_t)(h * KS + s) * D + col];
  }
  // With a hook the prologue constants come after the weight staging: the hook's barriers
  // and stores in the middle of the live weight registers put them in scratch.
  constexpr bool kHook = !std::is_same<Hook, NoHook>::value;
  ColConst kc;
  if constexpr (!kHook) kc = col_const<PRO>(pa, D, q_me);

  // Epilogue in the row-major domain: after the MFMA chain the accumulator tile goes
  // through LDS (s_x, free by then), and each thread finishes the float4 column group q_me
  // of rows r_me + RSTEP*i -- 16-byte loads of the epilogue operands and 16-byte stores
  // (4-byte stores of the ReLU mask) instead of 16 scalar accesses per lane.
  float4 bias4 = f4_zero();
  if constexpr (EPI == EPI_A1STATS || IS_OUT)
    bias4 = *reinterpret_cast<const float4*>(ea.bias + 4 * q_me);
  float4 al4 = f4_zero(), sh4 = f4_zero(), mu4 = f4_zero(), is4 = f4_zero();
  if constexpr (EPI == EPI_DBN) {
    const BnView b = bn_view(ea.bn, D);
    al4 = *reinterpret_cast<const float4*>(b.alpha + 4 * q_me);
    sh4 = *reinterpret_cast<const float4*>(b.shift + 4 * q_me);
    mu4 = *reinterpret_cast<const float4*>(b.mean + 4 * q_me);
    is4 = *reinterpret_cast<const float4*>(b.invstd + 4 * q_me);
  }
  double st1[4] = {0.0, 0.0, 0.0, 0.0}, st2[4] = {0.0, 0.0, 0.0, 0.0};

  auto load_tile = [&](int tile, RawItem (&raw)[ITEMS]) {
    const int64_t n0 = (int64_t)tile * kRowTile;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int64_t n = n0 + r_me + i * RSTEP;
      raw[i] = raw_load<PRO>(pa, D, n < N ? n : N - 1, q_me);  // clamped: always issued
    }
  };

  const TileRange tr = xcd_tile_range(num_tiles, vb, vgrid);
  RawItem raw[ITEMS];
  if (tr.first < tr.end) load_tile(tr.first, raw);
  if constexpr (WL) {
#pragma unroll
    for (int j = 0; j < WCH; ++j) {
      const int idx = threadIdx.x + NT * j;
      *reinterpret_cast<float4*>(&s_x[(idx / D4) * LD + 4 * (idx % D4)]) = wtmp[j];
    }
    __syncthreads();
    const float* wr = &s_x[col * LD + h * KS];
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(&wr[4 * q]);
      bf[4 * q] = v.x;
      bf[4 * q + 1] = v.y;
      bf[4 * q + 2] = v.z;
      bf[4 * q + 3] = v.w;
    }
    // the first tile's __syncthreads() below orders these reads before the staging writes
  }
  if constexpr (kHook) {
    hook();
    kc = col_const<PRO>(pa, D, q_me);
  }
  BPlanes<KS> bp;
  if constexpr (GINE_GEMM_BF16X3 && KS <= 64) bp.from(bf);
  for (int tile = tr.first; tile < tr.end; tile += tr.step) {
    const int64_t n0 = (int64_t)tile * kRowTile;
    RG_MARK(1);
    __syncthreads();  // previous tile's epilogue reads of s_x are done
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int r = r_me + i * RSTEP;
      float4 v = transform<PRO>(pa, raw[i], kc);
      if (n0 + r >= N) v = f4_zero();
      *reinterpret_cast<float4*>(&s_x[r * LD + 4 * q_me]) = v;
    }
    __syncthreads();
    if (tile + tr.step < tr.end) load_tile(tile + tr.step, raw);  // next tile, in flight
    float4 ep[ITEMS];
    if constexpr (EPI_LOAD) {  // epilogue operands of this tile, in flight too
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        int64_t n = n0 + r_me + i * RSTEP;
        n = n < N ? n : N - 1;
        const float* src = EPI == EPI_DBN ? ea.a1 : ea.resid;
        ep[i] = *reinterpret_cast<const float4*>(src + n * D + 4 * q_me);
      }
    }
    RG_MARK(2);
    floatx16 acc = zero16();
    const float* arow = &s_x[c32 * LD + h * KS];
    if constexpr (GINE_GEMM_BF16X3 && KS <= 64) {
#pragma unroll
      for (int s = 0; s < KS / 8; ++s) {
        const float4 a0 = *reinterpret_cast<const float4*>(&arow[8 * s]);
        const float4 a1 = *reinterpret_cast<const float4*>(&arow[8 * s + 4]);
        acc = mfma_bf16x3(split8(a0, a1), bp.f[s], acc);
      }
      if (wave_any_nan(acc)) acc = redo_fp32<D, KS, BT || WL>(arow, W, col, h);
    } else {
      acc = mfma_f32_row<KS>(arow, bf, acc);
    }
#ifdef GINE_RG_PROFILE
    if (acc[0] == 1.2345e-30f) s_x[0] = 0.f;  // the stamp below waits for the chain
#endif
    RG_MARK(3);
    __syncthreads();  // every wave's A-fragment reads of s_x are done
#pragma unroll
    for (int r = 0; r < 16; ++r) s_x[((r & 3) + 8 * (r >> 2) + 4 * h) * LD + col] = acc[r];
    __syncthreads();

#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int r = r_me + i * RSTEP;
      const int64_t n = n0 + r;
      const float4 v = *reinterpret_cast<const float4*>(&s_x[r * LD + 4 * q_me]);
      const float vv[4] = {v.x, v.y, v.z, v.w};
      if (n >= N) continue;
      const int64_t off = n * D + 4 * q_me;
      float o4[4];
      if constexpr (EPI == EPI_A1STATS) {
        const float bb[4] = {bias4.x, bias4.y, bias4.z, bias4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o4[k] = vv[k] + bb[k];
          st1[k] += (double)o4[k];
          st2[k] += (double)o4[k] * (double)o4[k];
        }
      } else if constexpr (IS_OUT) {
        const float bb[4] = {bias4.x, bias4.y, bias4.z, bias4.w};
        if constexpr (EPI == EPI_OUT_RES) {
          const float xr[4] = {ep[i].x, ep[i].y, ep[i].z, ep[i].w};
          uchar4 m;
          unsigned char mk[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float o = vv[k] + bb[k];
            o4[k] = xr[k] + relu_nan(o);
            mk[k] = (o > 0.f) ? 1 : 0;
          }
          m.x = mk[0];
          m.y = mk[1];
          m.z = mk[2];
          m.w = mk[3];
          *reinterpret_cast<uchar4*>(ea.mask_out + off) = m;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float o = vv[k] + bb[k];
            o4[k] = (EPI == EPI_OUT_RELU) ? relu_nan(o) : o;
          }
        }
      } else if constexpr (EPI == EPI_DBN) {
        const float a1[4] = {ep[i].x, ep[i].y, ep[i].z, ep[i].w};
        const float al[4] = {al4.x, al4.y, al4.z, al4.w}, sh[4] = {sh4.x, sh4.y, sh4.z, sh4.w};
        const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, is[4] = {is4.x, is4.y, is4.z, is4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float bn = bn_apply(a1[k], al[k], sh[k]);
          o4[k] = (bn > 0.f) ? vv[k] : 0.f;
          const double xhat = (double)((a1[k] - mu[k]) * is[k]);
          st1[k] += (double)o4[k];
          st2[k] += (double)o4[k] * xhat;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) o4[k] = vv[k];
      }
      *reinterpret_cast<float4*>(ea.out + off) = make_float4(o4[0], o4[1], o4[2], o4[3]);
    }
    RG_MARK(4);
  }

  if constexpr (EPI == EPI_A1STATS || EPI == EPI_DBN) {
    // per-column partials of the workgroup: the RSTEP row groups added in fixed order
    __syncthreads();
    double* sr = reinterpret_cast<double*>(s_x);  // [2][RSTEP][D] (fits: 16*D*8 <= 32*LD*4)
    static_assert(2 * RSTEP * D * 8 <= kRowTile * LD * 4, "partials fit in the tile");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sr[(0 * RSTEP + r_me) * D + 4 * q_me + k] = st1[k];
      sr[(1 * RSTEP + r_me) * D + 4 * q_me + k] = st2[k];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * D; c += NT) {
      const int which = c / D, cc = c % D;
      double t = 0.0;
#pragma unroll
      for (int g = 0; g < RSTEP; ++g) t += sr[(which * RSTEP + g) * D + cc];
      if (ea.partials) ea.partials[(size_t)vb * 2 * D + c] = t;
      if (ea.bnacc) bnacc_add(ea.bnacc, 2 * D, c, t);
    }
  }
  RG_MARK(5);
  RG_FLUSH();
}

// ----------------------------------------------------------------------------------------
// Software-pipelined row-tile GEMM: the same arithmetic as rowgemm_body (same MFMA chains,
// same epilogue rounding -> identical outputs), with the per-tile work that is not matrix
// work moved INTO the next tile's MFMA chain.  One wave per SIMD issues a 64-cycle
// v_mfma_f32_32x32x2_f32 every 64 cycles; the matrix pipe runs asynchronously, so the gaps
// between MFMA issues hold other instructions for free.  Per 32-row tile k the chain of
// tile k carries, in fixed slots of its 16 four-MFMA steps:
//   step 0      the accumulator of tile k-1 -> the LDS output tile (transpose)
//   steps 1-2   staging of tile k+1 (prologue transform) into the other A buffer
//   step 3      the raw loads of tile k+2 (in flight for a whole chain)
//   step 4      barrier (every wave's tile k-1 rows are in LDS)
//   steps 5-11  the epilogue of tile k-1: bias / BN statistics / residual / ReLU mask,
//               16-byte global stores
//   step 13     the epilogue operands of tile k (consumed one chain later)
// so a workgroup's tiles cost one MFMA chain each, plus one staging and one epilogue for
// the whole range, instead of (staging + chain + epilogue) per tile.  Loads are never
// conditional (clamped to the last tile: a branch around a load drains the memory queue).
// LDS: A buffers [2][32][D+4], output tile [32][D+4] (aliasing the W^T staging area).
template <int D>
constexpr int rowgemm_pipe_lds_floats(bool wl) {
  return (wl && D * (D + 4) > 3 * kRowTile * (D + 4)) ? D * (D + 4) : 3 * kRowTile * (D + 4);
}

template <int D, int PRO, int EPI, bool BT, bool WL = false, class Hook = NoHook>
__device__ __forceinline__ void rowgemm_pipe(const float* __restrict__ W, const ProArgs& pa,
                                             const EpiArgs& ea, int64_t N, int num_tiles,
                                             float* __restrict__ s_lds, int vb, int vgrid,
                                             const Hook& hook = Hook{}) {
  constexpr int NT = 2 * D;
  constexpr int KS = D / 2;
  constexpr int LD = D + 4;
  constexpr int D4 = D / 4;
  constexpr int ITEMS = kRowTile * D4 / NT;
  constexpr int RSTEP = NT / D4;
  constexpr int NQ = KS / 4;  // four-MFMA steps per chain
  // rgprof build: 0 start, 1 tile 0 staged (prologue done), 2 first chain done, 3 each later
  // chain done, 4 last epilogue done, 5 statistics written
  RG_DECL;
  RG_MARK(0);
  constexpr bool IS_OUT = (EPI == EPI_OUT) || (EPI == EPI_OUT_RELU) || (EPI == EPI_OUT_RES);
  constexpr bool EPI_LOAD = (EPI == EPI_DBN) || (EPI == EPI_OUT_RES);
  static_assert(NQ >= 8, "the pipeline slots need at least 8 steps (D >= 64)");
  // slots: item i of the epilogue at step Q_EPI0 + i * (Q_EPLOAD - Q_EPI0) / ITEMS
  constexpr int Q_STAGE0 = 1, Q_STAGE1 = 2, Q_LOAD = 3, Q_SYNC = 4, Q_EPI0 = 5;
  constexpr int Q_EPLOAD = NQ - 2;
  constexpr int EPI_SLOTS = Q_EPLOAD - Q_EPI0;

  // A buffer b at s_lds + b * kRowTile * LD (arithmetic, not a pointer table: a runtime
  // index into a table of pointers loses the LDS address space -> flat loads)
  float* sO = s_lds + 2 * kRowTile * LD;

  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  const int q_me = threadIdx.x % D4, r_me = threadIdx.x / D4;

  float bf[KS];
  constexpr int WCH = D * D4 / NT;
  float4 wtmp[WL ? WCH : 1];
  if constexpr (WL) {
    const float4* w4 = reinterpret_cast<const float4*>(W);
#pragma unroll
    for (int j = 0; j < WCH; ++j) wtmp[j] = w4[threadIdx.x + NT * j];
  } else if constexpr (BT) {
    const float4* wr = reinterpret_cast<const float4*>(W + (size_t)col * D + h * KS);
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
      const float4 v = wr[q];
      bf[4 * q] = v.x;
      bf[4 * q + 1] = v.y;
      bf[4 * q + 2] = v.z;
      bf[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) bf[s] = W[(size_t)(h * KS + s) * D + col];
  }
  constexpr bool kHook = !std::is_same<Hook, NoHook>::value;
  ColConst kc;
  if constexpr (!kHook) kc = col_const<PRO>(pa, D, q_me);

  float4 bias4 = f4_zero();
  if constexpr (EPI == EPI_A1STATS || IS_OUT)
    bias4 = *reinterpret_cast<const float4*>(ea.bias + 4 * q_me);
  float4 al4 = f4_zero(), sh4 = f4_zero(), mu4 = f4_zero(), is4 = f4_zero();
  if constexpr (EPI == EPI_DBN) {
    const BnView b = bn_view(ea.bn, D);
    al4 = *reinterpret_cast<const float4*>(b.alpha + 4 * q_me);
    sh4 = *reinterpret_cast<const float4*>(b.shift + 4 * q_me);
    mu4 = *reinterpret_cast<const float4*>(b.mean + 4 * q_me);
    is4 = *reinterpret_cast<const float4*>(b.invstd + 4 * q_me);
  }
  double st1[4] = {0.0, 0.0, 0.0, 0.0}, st2[4] = {0.0, 0.0, 0.0, 0.0};

  const TileRange tr = xcd_tile_range(num_tiles, vb, vgrid);
  const int count = tr.first < tr.end ? (tr.end - tr.first + tr.step - 1) / tr.step : 0;
  auto tile_of = [&](int i) { return tr.first + min(i, count - 1) * tr.step; };

  auto load_tile = [&](int tile, RawItem (&raw)[ITEMS]) {
    const int64_t n0 = (int64_t)tile * kRowTile;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int64_t n = n0 + r_me + i * RSTEP;
      raw[i] = raw_load<PRO>(pa, D, n < N ? n : N - 1, q_me);
    }
  };
  auto load_ep = [&](int tile, float4 (&ep)[ITEMS]) {
    if constexpr (EPI_LOAD) {
      const int64_t n0 = (int64_t)tile * kRowTile;
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        int64_t n = n0 + r_me + i * RSTEP;
        n = n < N ? n : N - 1;
        const float* src = EPI == EPI_DBN ? ea.a1 : ea.resid;
        ep[i] = *reinterpret_cast<const float4*>(src + n * D + 4 * q_me);
      }
    }
  };
  auto stage_item = [&](int tile, const RawItem& raw, int i, float* dst) {
    const int r = r_me + i * RSTEP;
    float4 v = transform<PRO>(pa, raw, kc);
    if ((int64_t)tile * kRowTile + r >= N) v = f4_zero();
    *reinterpret_cast<float4*>(&dst[r * LD + 4 * q_me]) = v;
  };
  auto acc_to_lds = [&](const floatx16& acc) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sO[((r & 3) + 8 * (r >> 2) + 4 * h) * LD + col] = acc[r];
  };
  // epilogue of one item (rows r_me + i*RSTEP of tile `tile`), from the LDS output tile
  auto epi_item = [&](int tile, int i, const float4 (&ep)[ITEMS]) {
    const int r = r_me + i * RSTEP;
    const int64_t n = (int64_t)tile * kRowTile + r;
    const float4 v = *reinterpret_cast<const float4*>(&sO[r * LD + 4 * q_me]);
    const float vv[4] = {v.x, v.y, v.z, v.w};
    if (n >= N) return;
    const int64_t off = n * D + 4 * q_me;
    float o4[4];
    if constexpr (EPI == EPI_A1STATS) {
      const float bb[4] = {bias4.x, bias4.y, bias4.z, bias4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o4[k] = vv[k] + bb[k];
        st1[k] += (double)o4[k];
        st2[k] += (double)o4[k] * (double)o4[k];
      }
    } else if constexpr (IS_OUT) {
      const float bb[4] = {bias4.x, bias4.y, bias4.z, bias4.w};
      if constexpr (EPI == EPI_OUT_RES) {
        const float xr[4] = {ep[i].x, ep[i].y, ep[i].z, ep[i].w};
        unsigned char mk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float o = vv[k] + bb[k];
          o4[k] = xr[k] + relu_nan(o);
          mk[k] = (o > 0.f) ? 1 : 0;
        }
        *reinterpret_cast<uchar4*>(ea.mask_out + off) = make_uchar4(mk[0], mk[1], mk[2], mk[3]);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float o = vv[k] + bb[k];
          o4[k] = (EPI == EPI_OUT_RELU) ? relu_nan(o) : o;
        }
      }
    } else if constexpr (EPI == EPI_DBN) {
      const float a1[4] = {ep[i].x, ep[i].y, ep[i].z, ep[i].w};
      const float al[4] = {al4.x, al4.y, al4.z, al4.w}, sh[4] = {sh4.x, sh4.y, sh4.z, sh4.w};
      const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, is[4] = {is4.x, is4.y, is4.z, is4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float bn = bn_apply(a1[k], al[k], sh[k]);
        o4[k] = (bn > 0.f) ? vv[k] : 0.f;
        const double xhat = (double)((a1[k] - mu[k]) * is[k]);
        st1[k] += (double)o4[k];
        st2[k] += (double)o4[k] * xhat;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) o4[k] = vv[k];
    }
    *reinterpret_cast<float4*>(ea.out + off) = make_float4(o4[0], o4[1], o4[2], o4[3]);
  };

  RawItem raw[ITEMS];
  float4 ep_prev[ITEMS], ep_cur[ITEMS];
  floatx16 accp = zero16();
  if (count > 0) {
    load_tile(tile_of(0), raw);
    if constexpr (WL) {
#pragma unroll
      for (int j = 0; j < WCH; ++j) {
        const int idx = threadIdx.x + NT * j;
        *reinterpret_cast<float4*>(&s_lds[(idx / D4) * LD + 4 * (idx % D4)]) = wtmp[j];
      }
      __syncthreads();
      const float* wr = &s_lds[col * LD + h * KS];
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(&wr[4 * q]);
        bf[4 * q] = v.x;
        bf[4 * q + 1] = v.y;
        bf[4 * q + 2] = v.z;
        bf[4 * q + 3] = v.w;
      }
    }
    if constexpr (kHook) {
      hook();
      kc = col_const<PRO>(pa, D, q_me);
    }
    BPlanes<KS> bp;
    if constexpr (GINE_GEMM_BF16X3 && KS <= 64) bp.from(bf);
    __syncthreads();  // W^T fragment reads (WL) are done before the A buffers overwrite them
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) stage_item(tile_of(0), raw[i], i, s_lds);
    load_tile(tile_of(1), raw);
    __syncthreads();  // tile 0 staged
    RG_MARK(1);

    // tile k's chain (A = sA[k & 1]) carrying the pipeline slots; EPI_ON: the epilogue of
    // tile k-1 (every iteration but the first)
    auto chain = [&](int k, auto epi_on) -> floatx16 {
      constexpr bool EPI_ON = decltype(epi_on)::value;
      const float* arow = s_lds + (k & 1) * (kRowTile * LD) + c32 * LD + h * KS;
      float* snext = s_lds + ((k + 1) & 1) * (kRowTile * LD);
      const int tprev = tile_of(k - 1), tnext = tile_of(k + 1);
      floatx16 acc = zero16();
      // each step's A fragment is read one step ahead (the step boundaries are scheduling
      // barriers: a read issued in the same step would expose the LDS latency every step)
      float4 a4 = *reinterpret_cast<const float4*>(&arow[0]);
      float4 aprev = a4;  // (split-bf16: the even step's four k values, used by the odd step)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const float4 an =
            *reinterpret_cast<const float4*>(&arow[4 * (q + 1 < NQ ? q + 1 : q)]);
        if constexpr (GINE_GEMM_BF16X3 && KS <= 64) {
          if (q % 2 == 0) aprev = a4;
          else acc = mfma_bf16x3(split8(aprev, a4), bp.f[q / 2], acc);
        } else {
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, bf[4 * q], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, bf[4 * q + 1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, bf[4 * q + 2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, bf[4 * q + 3], acc, 0, 0, 0);
        }
        if (q == 0 && EPI_ON) acc_to_lds(accp);
        if (q == Q_STAGE0) {
#pragma unroll
          for (int i = 0; i < ITEMS / 2; ++i) stage_item(tnext, raw[i], i, snext);
        }
        if (q == Q_STAGE1) {
#pragma unroll
          for (int i = ITEMS / 2; i < ITEMS; ++i) stage_item(tnext, raw[i], i, snext);
        }
        if (q == Q_LOAD) load_tile(tile_of(k + 2), raw);
        if (q == Q_SYNC && EPI_ON) __syncthreads();
        if (EPI_ON) {
#pragma unroll
          for (int i = 0; i < ITEMS; ++i)
            if (q == Q_EPI0 + i * EPI_SLOTS / ITEMS) epi_item(tprev, i, ep_prev);
        }
        if (q == Q_EPLOAD) load_ep(tile_of(k), ep_cur);  // tile k's operands, for next chain
        __builtin_amdgcn_sched_barrier(0);
        a4 = an;
      }
      // (the A buffer of tile k stays until the barrier before chain k + 1)
      if constexpr (GINE_GEMM_BF16X3 && KS <= 64)
        if (wave_any_nan(acc)) acc = redo_fp32<D, KS, BT || WL>(arow, W, col, h);
      return acc;
    };

    auto rotate_ep = [&]() {
      if constexpr (EPI_LOAD) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) ep_prev[i] = ep_cur[i];
      }
    };
    // peeled first chain: no previous tile to finish
    accp = chain(0, std::false_type{});
    rotate_ep();
    RG_MARK(2);
    for (int k = 1; k < count; ++k) {
      __syncthreads();  // tile k staged; the output tile and the other A buffer are free
      accp = chain(k, std::true_type{});
      rotate_ep();
      RG_MARK(3);
    }
    // the last tile's epilogue
    __syncthreads();
    acc_to_lds(accp);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) epi_item(tile_of(count - 1), i, ep_prev);
    RG_MARK(4);
  } else if constexpr (kHook) {
    hook();  // (no tiles: the hook still runs its workgroup-0 duties)
  }

  if constexpr (EPI == EPI_A1STATS || EPI == EPI_DBN) {
    __syncthreads();
    double* sr = reinterpret_cast<double*>(s_lds);
    static_assert(2 * RSTEP * D * 8 <= kRowTile * LD * 4, "partials fit in the tile");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sr[(0 * RSTEP + r_me) * D + 4 * q_me + k] = st1[k];
      sr[(1 * RSTEP + r_me) * D + 4 * q_me + k] = st2[k];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * D; c += NT) {
      const int which = c / D, cc = c % D;
      double t = 0.0;
#pragma unroll
      for (int g = 0; g < RSTEP; ++g) t += sr[(which * RSTEP + g) * D + cc];
      if (ea.partials) ea.partials[(size_t)vb * 2 * D + c] = t;
      if (ea.bnacc) bnacc_add(ea.bnacc, 2 * D, c, t);
    }
  }
  RG_MARK(5);
  RG_FLUSH();
}

#ifndef GINE_ROWGEMM_PIPE
#define GINE_ROWGEMM_PIPE 1
#endif

template <int D, int PRO, int EPI, bool BT>
__global__ __launch_bounds__(2 * D) void k_rowgemm(const float* __restrict__ W, ProArgs pa,
                                                   EpiArgs ea, int64_t N, int num_tiles) {
  constexpr bool WL = BT && D <= 128;  // W^T staged through LDS (fits: 128*132*4 B)
  if constexpr (GINE_ROWGEMM_PIPE && D >= 64) {
    __shared__ __attribute__((aligned(16))) float s_x[rowgemm_pipe_lds_floats<D>(WL)];
    rowgemm_pipe<D, PRO, EPI, BT, WL>(W, pa, ea, N, num_tiles, s_x, blockIdx.x, gridDim.x);
  } else {
    __shared__ __attribute__((aligned(16))) float s_x[(WL ? D : kRowTile) * (D + 4)];
    rowgemm_body<D, PRO, EPI, BT, WL>(W, pa, ea, N, num_tiles, s_x, blockIdx.x, gridDim.x);
  }
}

// Persistent grid.  One workgroup per CU while each has at most 4 tiles; past that two
// per CU, so one workgroup's epilogue and staging run beside the other's MFMA chain (cfg3,
// 4,000 tiles: 48 -> 44 us fwd1, 65 -> 54 us bwd2; at cfg2, 500 tiles, the second
// workgroup's weight staging costs more than the overlap gains; 512 / 1024 workgroups at
// cfg2 measured no better, r02_s61).
inline int rowgemm_cap(int D, int64_t tiles) {
  const int per_cu = (D == 128 && tiles > 4 * kNumCu) ? 2 : 1;
  return std::max(kNumCu * per_cu, 1024 / (D / 32));
}

inline int rowgemm_grid(int64_t N, int D) {
  const int64_t tiles = ceil_div(N, kRowTile);
  const int64_t cap = rowgemm_cap(D, tiles);
  const int64_t g = tiles < cap ? tiles : cap;
  return (int)(g > 0 ? g : 1);
}

template <int PRO, int EPI, bool BT>
int launch_rowgemm(int D, const float* W, const ProArgs& pa, const EpiArgs& ea, int64_t N,
                   hipStream_t s) {
  const int grid = rowgemm_grid(N, D);
  const int tiles = (int)ceil_div(N, kRowTile);
  switch (D) {
    case 32:
      hipLaunchKernelGGL((k_rowgemm<32, PRO, EPI, BT>), dim3(grid), dim3(64), 0, s, W, pa, ea,
                         N, tiles);
      break;
    case 64:
      hipLaunchKernelGGL((k_rowgemm<64, PRO, EPI, BT>), dim3(grid), dim3(128), 0, s, W, pa, ea,
                         N, tiles);
      break;
    case 128:
      hipLaunchKernelGGL((k_rowgemm<128, PRO, EPI, BT>), dim3(grid), dim3(256), 0, s, W, pa,
                         ea, N, tiles);
      break;
    case 256:
      hipLaunchKernelGGL((k_rowgemm<256, PRO, EPI, BT>), dim3(grid), dim3(512), 0, s, W, pa,
                         ea, N, tiles);
      break;
    default:
      return GINE_ERR_DIM;
  }
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

// Second GEMM with the BatchNorm finish in its prologue (training, momentum given): every
// workgroup turns the fixed-point totals of gine_bnacc.hpp into alpha / shift in LDS
// (workgroup 0 also writes bn_save, the running statistics and num_batches_tracked -- the
// arithmetic of BnFwdFin -- and its snapshot / consumed-phase words), then the row-tile
// GEMM runs with its prologue constants read from LDS.
template <int D, int EPI>
__global__ __launch_bounds__(2 * D) void k_fwd2_bnacc(const float* __restrict__ W, ProArgs pa,
                                                      EpiArgs ea, BnFwdParams q,
                                                      long long* acc, int64_t N,
                                                      int num_tiles) {
  constexpr bool WL = D <= 128;
  constexpr bool PIPE = GINE_ROWGEMM_PIPE && D >= 64;
  __shared__ __attribute__((aligned(16)))
  float s_x[PIPE ? rowgemm_pipe_lds_floats<D>(WL) : (WL ? D : kRowTile) * (D + 4)];
  __shared__ __attribute__((aligned(16))) float s_bn[4 * D];
  __shared__ double s_tot[2 * D];
  auto finish = [=]() {  // by value: a reference to a kernel argument puts it in scratch
    const int t = threadIdx.x;  // 2D threads: word t = (sum | sum of squares) of column t % D
    s_tot[t] = bnacc_total(acc, 2 * D, t, blockIdx.x == 0);
    // a failed grid barrier on this accumulator (sticky until the host's reset): NaN
    // statistics from bnacc_total, running statistics untouched
    BnFwdParams qq = q;
    if (bnacc_poisoned(acc, 2 * D)) qq.update_running = 0;
    __syncthreads();
    if (t < D)
      bn_finish_channel(qq, D, t, s_tot[t], s_tot[D + t], blockIdx.x == 0, &s_bn[2 * D + t],
                        &s_bn[3 * D + t]);
    if (blockIdx.x == 0 && t == 0) {
      if (qq.update_running && qq.nbt != nullptr) qq.nbt[0] = qq.nbt[0] + 1;
      bnacc_mark_consumed(acc, 2 * D);
    }
    __syncthreads();
  };
  ProArgs p2 = pa;
  p2.bn = s_bn;
  if constexpr (PIPE)
    rowgemm_pipe<D, PRO_BNRELU, EPI, true, WL>(W, p2, ea, N, num_tiles, s_x, blockIdx.x,
                                               gridDim.x, finish);
  else
    rowgemm_body<D, PRO_BNRELU, EPI, true, WL>(W, p2, ea, N, num_tiles, s_x, blockIdx.x,
                                               gridDim.x, finish);
}

// dz = da1 W1 with the BatchNorm backward finish in its prologue (training): the totals
// [sum dbn | sum dbn*xhat] of gine_bnacc.hpp -> coef = [c1 | c2 | c3] in LDS (workgroup 0
// also writes coef, dgamma, dbeta -- the arithmetic of BnBwdFin).
template <int D>
__global__ __launch_bounds__(2 * D) void k_bwd1_bnacc(const float* __restrict__ W, ProArgs pa,
                                                      EpiArgs ea, const float* gamma,
                                                      float* dgamma, float* dbeta, float* coef,
                                                      long long* acc, int64_t N,
                                                      int num_tiles) {
  constexpr bool PIPE = GINE_ROWGEMM_PIPE && D >= 64;
  __shared__ __attribute__((aligned(16)))
  float s_x[PIPE ? rowgemm_pipe_lds_floats<D>(false) : kRowTile * (D + 4)];
  __shared__ __attribute__((aligned(16))) float s_coef[3 * D];
  __shared__ double s_tot[2 * D];
  const float* bn_save = pa.bn;
  auto finish = [=]() {  // by value: a reference to a kernel argument puts it in scratch
    const int t = threadIdx.x;
    s_tot[t] = bnacc_total(acc, 2 * D, t, blockIdx.x == 0);
    __syncthreads();
    if (t < D) {
      const double sd = s_tot[t], sx = s_tot[D + t];
      const double g = gamma ? (double)gamma[t] : 1.0;
      const double c1 = g * (double)bn_save[D + t];
      const float k1 = (float)c1, k2 = (float)(-c1 * sx / (double)N),
                  k3 = (float)(-c1 * sd / (double)N);
      s_coef[t] = k1;
      s_coef[D + t] = k2;
      s_coef[2 * D + t] = k3;
      if (blockIdx.x == 0) {
        if (t == 0) bnacc_mark_consumed(acc, 2 * D);
        if (dgamma) dgamma[t] = (float)sx;
        if (dbeta) dbeta[t] = (float)sd;
        coef[t] = k1;
        coef[D + t] = k2;
        coef[2 * D + t] = k3;
      }
    }
    __syncthreads();
  };
  ProArgs p2 = pa;
  p2.coef = s_coef;
  if constexpr (PIPE)
    rowgemm_pipe<D, PRO_DA1, EPI_PLAIN, false, false>(W, p2, ea, N, num_tiles, s_x,
                                                      blockIdx.x, gridDim.x, finish);
  else
    rowgemm_body<D, PRO_DA1, EPI_PLAIN, false, false>(W, p2, ea, N, num_tiles, s_x,
                                                      blockIdx.x, gridDim.x, finish);
}

template <int EPI>
int launch_fwd2_bnacc(int D, const float* W, const ProArgs& pa, const EpiArgs& ea,
                      const BnFwdParams& q, long long* acc, int64_t N, hipStream_t s) {
  const int grid = rowgemm_grid(N, D);
  const int tiles = (int)ceil_div(N, kRowTile);
  switch (D) {
    case 32:
      hipLaunchKernelGGL((k_fwd2_bnacc<32, EPI>), dim3(grid), dim3(64), 0, s, W, pa, ea, q, acc,
                         N, tiles);
      break;
    case 64:
      hipLaunchKernelGGL((k_fwd2_bnacc<64, EPI>), dim3(grid), dim3(128), 0, s, W, pa, ea, q,
                         acc, N, tiles);
      break;
    case 128:
      hipLaunchKernelGGL((k_fwd2_bnacc<128, EPI>), dim3(grid), dim3(256), 0, s, W, pa, ea, q,
                         acc, N, tiles);
      break;
    case 256:
      hipLaunchKernelGGL((k_fwd2_bnacc<256, EPI>), dim3(grid), dim3(512), 0, s, W, pa, ea, q,
                         acc, N, tiles);
      break;
    default:
      return GINE_ERR_DIM;
  }
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

// ----------------------------------------------------------------------------------------
// BatchNorm1d finalize kernels (one thread per channel, partials summed in fixed order)
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(kColsumThreads) void k_bn_fwd_finalize(
    const double* __restrict__ partials, int P, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
    int64_t* __restrict__ nbt, float* __restrict__ bn_save, int64_t N, int D, float momentum,
    float bn_eps, int training, int update_running) {
  __shared__ double s_tmp[kColsumThreads];
  __shared__ double s_sum[2 * 256];  // [sum | sumsq], D <= 256
  __shared__ double s_factor;
  if (training) block_colsum(partials, P, 2 * D, 2 * D * kSliceRows, s_tmp, s_sum);
  if (threadIdx.x == 0) {
    double f = (double)momentum;
    if (training && update_running && nbt != nullptr) {
      const int64_t t = nbt[0] + 1;
      nbt[0] = t;
      if (momentum < 0.f) f = 1.0 / (double)t;  // momentum=None: cumulative average
    }
    s_factor = f;
  }
  __syncthreads();
  const double factor = s_factor;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    double mean, var;
    if (training) {
      mean = s_sum[c] / (double)N;
      var = s_sum[D + c] / (double)N - mean * mean;
      if (var < 0.0) var = 0.0;
      if (update_running && rmean != nullptr) {
        const double unbiased = N > 1 ? var * (double)N / (double)(N - 1) : var;
        rmean[c] = (float)(factor * mean + (1.0 - factor) * (double)rmean[c]);
        rvar[c] = (float)(factor * unbiased + (1.0 - factor) * (double)rvar[c]);
      }
    } else {
      mean = (double)rmean[c];
      var = (double)rvar[c];
    }
    const double invstd = 1.0 / sqrt(var + (double)bn_eps);
    const double g = gamma ? (double)gamma[c] : 1.0;
    const double bt = beta ? (double)beta[c] : 0.0;
    const double alpha = g * invstd;
    bn_save[c] = (float)mean;
    bn_save[D + c] = (float)invstd;
    bn_save[2 * D + c] = (float)alpha;
    bn_save[3 * D + c] = (float)(bt - mean * alpha);
  }
}



// Finish of the BatchNorm statistics (k_colsum_fin<4>): workgroup b owns channels 2b, 2b+1;
// column j < 2 is the sum of a1 of channel 2b+j, j >= 2 its sum of squares.
constexpr int kBnFinCh = 2;  // channels per finish workgroup
struct BnFwdFin {
  const float *gamma, *beta;
  float *rmean, *rvar;
  int64_t* nbt;
  float* bn_save;
  int64_t N;
  int D;
  float momentum, bn_eps;
  int update_running;
  __device__ int col(int b, int j) const {
    const int c = kBnFinCh * b + (j % kBnFinCh);
    if (c >= D) return -1;
    return j < kBnFinCh ? c : D + c;
  }
  __device__ void finish(int b, const double* tot) const {
    const int t = threadIdx.x;
    if (b == 0 && t == 0 && update_running && nbt != nullptr) nbt[0] = nbt[0] + 1;
    const int c = kBnFinCh * b + t;
    if (t >= kBnFinCh || c >= D) return;
    const double mean = tot[t] / (double)N;
    double var = tot[kBnFinCh + t] / (double)N - mean * mean;
    if (var < 0.0) var = 0.0;
    if (update_running && rmean != nullptr) {  // momentum >= 0 here (None: other path)
      const double f = (double)momentum;
      const double unbiased = N > 1 ? var * (double)N / (double)(N - 1) : var;
      rmean[c] = (float)(f * mean + (1.0 - f) * (double)rmean[c]);
      rvar[c] = (float)(f * unbiased + (1.0 - f) * (double)rvar[c]);
    }
    const double invstd = 1.0 / sqrt(var + (double)bn_eps);
    const double g = gamma ? (double)gamma[c] : 1.0;
    const double bt = beta ? (double)beta[c] : 0.0;
    const double alpha = g * invstd;
    bn_save[c] = (float)mean;
    bn_save[D + c] = (float)invstd;
    bn_save[2 * D + c] = (float)alpha;
    bn_save[3 * D + c] = (float)(bt - mean * alpha);
  }
};

// Finish of the BatchNorm backward sums (k_colsum_fin<4>): column j < 2 = sum dbn of
// channel 2b+j, j >= 2 = sum dbn * xhat.
struct BnBwdFin {
  const float* gamma;
  const float* bn_save;
  float *dgamma, *dbeta, *coef;
  int64_t N;
  int D;
  int training;
  __device__ int col(int b, int j) const {
    const int c = kBnFinCh * b + (j % kBnFinCh);
    if (c >= D) return -1;
    return j < kBnFinCh ? c : D + c;
  }
  __device__ void finish(int b, const double* tot) const {
    const int t = threadIdx.x;
    const int c = kBnFinCh * b + t;
    if (t >= kBnFinCh || c >= D) return;
    const double sd = tot[t], sx = tot[kBnFinCh + t];
    if (dgamma) dgamma[c] = (float)sx;
    if (dbeta) dbeta[c] = (float)sd;
    const double g = gamma ? (double)gamma[c] : 1.0;
    const double c1 = g * (double)bn_save[D + c];
    coef[c] = (float)c1;
    coef[D + c] = training ? (float)(-c1 * sx / (double)N) : 0.f;
    coef[2 * D + c] = training ? (float)(-c1 * sd / (double)N) : 0.f;
  }
};

// Backward GEMM dz = da1 W1 and the weight gradients (dW1, dW2, biases) in ONE launch: they
// read the same inputs (dy, the ReLU mask, a1, dbn, z) and are independent, so the first
// eng_blocks workgroups run the weight-gradient engine (the longer job starts first) and
// the rest run the row-tile GEMM, sharing the CUs instead of taking two launches.  D = 128
// (both parts then use 256-thread workgroups).
template <int PDO>
__global__ __launch_bounds__(256) void k_bwd1_wgrad(const float* __restrict__ w1, ProArgs pa,
                                                    EpiArgs ea, int64_t N, int num_tiles,
                                                    int rg_grid, MlpWgradSrc<PDO> src,
                                                    int chunks, int rows_per_chunk,
                                                    size_t zstride, size_t cstride,
                                                    float* __restrict__ slab, int eng_blocks) {
  // one region: the engine's operand images (fp32 tiles or split planes, wg_lds_bytes),
  // or the row GEMM's A tile in its sQ part
  __shared__ __attribute__((aligned(16))) float s_eng[wg_lds_bytes<kMlpWgTO>() / sizeof(float)];
  float* sP = s_eng;
  float* sQ = s_eng + kWgRows * (kMlpWgTO + 4);
  const int b = blockIdx.x;
  if (b < eng_blocks) {
    // the output tiles of one row chunk run back to back on ONE XCD: they read the same
    // rows (a1 by all four, z by the two dW1 tiles), which that XCD's L2 then serves
    const int lb = xcd_remap(b, eng_blocks), tiles = eng_blocks / chunks;
    wgrad_block<MlpWgradSrc<PDO>, kMlpWgTO, 4, kMlpEngX3>(src, N, 128, 128, lb / tiles,
                                                          lb % tiles, rows_per_chunk, zstride,
                                                          cstride, slab, sP, sQ);
  } else {
    static_assert(kRowTile * (128 + 4) <= kWgRows * kWgLdQ, "row tile fits in sQ");
    rowgemm_body<128, PRO_DA1, EPI_PLAIN, false>(w1, pa, ea, N, num_tiles, sQ,
                                                 b - eng_blocks, rg_grid);
  }
}


inline bool mlp_dim_ok(int D) { return D == 32 || D == 64 || D == 128 || D == 256; }

inline WgPlan mlp_wgrad_plan(int64_t N, int D) { return wg_plan(N, D, D, 2, kMlpWgTO); }

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_mlp_num_partials(int64_t num_nodes, int32_t channels,
                                     int32_t* num_partials) {
  if (!num_partials || num_nodes < 0) return GINE_ERR_INVALID;
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  *num_partials = rowgemm_grid(num_nodes, channels);
  return GINE_OK;
}

extern "C" int gine_mlp_fwd1(const float* z, const float* w1, const float* b1, float* a1,
                             double* partials, int64_t num_nodes, int32_t channels,
                             void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !z || !w1 || !b1 || !a1 || !partials) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  ProArgs pa{z, nullptr, nullptr, nullptr, nullptr};
  EpiArgs ea{b1, a1, nullptr, nullptr, nullptr, nullptr, partials, 0};
  return launch_rowgemm<PRO_PLAIN, EPI_A1STATS, true>(channels, w1, pa, ea, num_nodes,
                                                      as_stream(stream));
}

extern "C" int gine_bn_acc_words(int32_t channels, int64_t* words) {
  if (!words || channels <= 0) return GINE_ERR_INVALID;
  *words = bnacc_words(channels);
  return GINE_OK;
}

extern "C" int gine_bn_acc_barrier_failures_index(int32_t channels, int64_t* index) {
  if (!index || channels <= 0) return GINE_ERR_INVALID;
  // the barrier area follows the phase word and the two consumed words (gine_bnacc.hpp)
  *index = (int64_t)(kBnAccReplicas * kBnAccWords + kBnAccCounts + 2 * kBnAccSnap) * 2 *
               channels + 3 + kBarFailWord;
  return GINE_OK;
}

extern "C" int gine_mlp_fwd1_acc(const float* z, const float* w1, const float* b1, float* a1,
                                 double* partials, int64_t* bn_acc, int64_t num_nodes,
                                 int32_t channels, void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !z || !w1 || !b1 || !a1 || !bn_acc) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  ProArgs pa{z, nullptr, nullptr, nullptr, nullptr};
  EpiArgs ea{b1, a1, nullptr, nullptr, nullptr, nullptr, partials, 0,
             reinterpret_cast<long long*>(bn_acc)};
  return launch_rowgemm<PRO_PLAIN, EPI_A1STATS, true>(channels, w1, pa, ea, num_nodes,
                                                      as_stream(stream));
}

extern "C" int gine_mlp_fwd2_bn(const float* a1, int64_t* bn_acc, const float* gamma,
                                const float* beta, float* running_mean, float* running_var,
                                int64_t* num_batches_tracked, float* bn_save, float momentum,
                                float bn_eps, int32_t update_running, const float* w2,
                                const float* b2, const float* x, float* y, uint8_t* mask,
                                int64_t num_nodes, int32_t channels, int32_t epilogue,
                                void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !a1 || !bn_acc || !bn_save || !w2 || !b2 || !y) return GINE_ERR_INVALID;
  if (!(momentum >= 0.f)) return GINE_ERR_INVALID;  // momentum=None: gine_bn_fwd_finalize
  if (update_running && (!running_mean || !running_var)) return GINE_ERR_INVALID;
  if (epilogue < GINE_EPI_NONE || epilogue > GINE_EPI_RESIDUAL_RELU) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && (!x || !mask)) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  ProArgs pa{a1, nullptr, nullptr, nullptr, nullptr};
  EpiArgs ea{b2, y, mask, x, nullptr, nullptr, nullptr, epilogue};
  const BnFwdParams q{gamma,   beta,      running_mean, running_var,   num_batches_tracked,
                      bn_save, num_nodes, momentum,     bn_eps,        update_running};
  long long* acc = reinterpret_cast<long long*>(bn_acc);
  hipStream_t s = as_stream(stream);
  switch (epilogue) {
    case GINE_EPI_NONE:
      return launch_fwd2_bnacc<EPI_OUT>(channels, w2, pa, ea, q, acc, num_nodes, s);
    case GINE_EPI_RELU:
      return launch_fwd2_bnacc<EPI_OUT_RELU>(channels, w2, pa, ea, q, acc, num_nodes, s);
    default:
      return launch_fwd2_bnacc<EPI_OUT_RES>(channels, w2, pa, ea, q, acc, num_nodes, s);
  }
}

extern "C" int gine_bn_fwd_finalize(const double* partials, int32_t num_partials,
                                    const float* gamma, const float* beta, float* running_mean,
                                    float* running_var, int64_t* num_batches_tracked,
                                    float* bn_save, int64_t num_nodes, int32_t channels,
                                    float momentum, float bn_eps, int32_t training,
                                    int32_t update_running, void* stream) {
  if (channels <= 0 || !bn_save || num_nodes <= 0) return GINE_ERR_INVALID;
  if (training && (!partials || num_partials <= 0)) return GINE_ERR_INVALID;
  if (!training && (!running_mean || !running_var)) return GINE_ERR_INVALID;
  if (update_running && training && (!running_mean || !running_var)) return GINE_ERR_INVALID;
  if (channels > 256) return GINE_ERR_DIM;
  hipStream_t s = as_stream(stream);
  const bool cumulative = training && update_running && momentum < 0.f;
  if (training && !cumulative) {
    // one launch: workgroup b owns two channels (their sums and sums of squares)
    const BnFwdFin fin{gamma, beta, running_mean, running_var, num_batches_tracked, bn_save,
                       num_nodes, channels, momentum, bn_eps, update_running};
    hipLaunchKernelGGL((k_colsum_fin<2 * kBnFinCh, BnFwdFin>),
                       dim3((unsigned)ceil_div(channels, kBnFinCh)),
                       dim3(256), 0, s, partials, num_partials, 2 * channels, fin);
    GINE_LAUNCH_STATUS();
    return GINE_OK;
  }
  int S = num_partials;
  if (training) {  // momentum=None: every channel needs the one num_batches_tracked bump
    S = launch_colsum_slices(const_cast<double*>(partials), num_partials, 2 * channels, s);
    GINE_LAUNCH_STATUS();
  }
  hipLaunchKernelGGL(k_bn_fwd_finalize, dim3(1), dim3(kColsumThreads), 0, s, partials, S,
                     gamma, beta, running_mean, running_var, num_batches_tracked, bn_save,
                     num_nodes, channels, momentum, bn_eps, training, update_running);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_mlp_fwd2(const float* a1, const float* bn_save, const float* w2,
                             const float* b2, const float* x, float* y, uint8_t* mask,
                             int64_t num_nodes, int32_t channels, int32_t epilogue,
                             void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !a1 || !bn_save || !w2 || !b2 || !y) return GINE_ERR_INVALID;
  if (epilogue < GINE_EPI_NONE || epilogue > GINE_EPI_RESIDUAL_RELU) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && (!x || !mask)) return GINE_ERR_INVALID;
  ProArgs pa{a1, nullptr, nullptr, bn_save, nullptr};
  EpiArgs ea{b2, y, mask, x, nullptr, nullptr, nullptr, epilogue};
  hipStream_t s = as_stream(stream);
  switch (epilogue) {
    case GINE_EPI_NONE:
      return launch_rowgemm<PRO_BNRELU, EPI_OUT, true>(channels, w2, pa, ea, num_nodes, s);
    case GINE_EPI_RELU:
      return launch_rowgemm<PRO_BNRELU, EPI_OUT_RELU, true>(channels, w2, pa, ea, num_nodes, s);
    default:
      return launch_rowgemm<PRO_BNRELU, EPI_OUT_RES, true>(channels, w2, pa, ea, num_nodes, s);
  }
}

extern "C" int gine_mlp_bwd2(const float* dy, const float* y, const uint8_t* mask,
                             const float* a1, const float* bn_save, const float* w2, float* dbn,
                             double* partials, int64_t num_nodes, int32_t channels,
                             int32_t epilogue, void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !dy || !a1 || !bn_save || !w2 || !dbn || !partials)
    return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RELU && !y) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && !mask) return GINE_ERR_INVALID;
  ProArgs pa{dy, y, mask, nullptr, nullptr};
  EpiArgs ea{nullptr, dbn, nullptr, nullptr, a1, bn_save, partials, 0};
  hipStream_t s = as_stream(stream);
  switch (epilogue) {
    case GINE_EPI_NONE:
      return launch_rowgemm<PRO_PLAIN, EPI_DBN, false>(channels, w2, pa, ea, num_nodes, s);
    case GINE_EPI_RELU:
      return launch_rowgemm<PRO_DOR, EPI_DBN, false>(channels, w2, pa, ea, num_nodes, s);
    default:
      return launch_rowgemm<PRO_DOM, EPI_DBN, false>(channels, w2, pa, ea, num_nodes, s);
  }
}

extern "C" int gine_bn_bwd_finalize(const double* partials, int32_t num_partials,
                                    const float* gamma, const float* bn_save, float* dgamma,
                                    float* dbeta, float* coef, int64_t num_nodes,
                                    int32_t channels, int32_t training, void* stream) {
  if (channels <= 0 || !partials || num_partials <= 0 || !bn_save || !coef || num_nodes <= 0)
    return GINE_ERR_INVALID;
  if (channels > 256) return GINE_ERR_DIM;
  const BnBwdFin fin{gamma, bn_save, dgamma, dbeta, coef, num_nodes, channels, training};
  hipLaunchKernelGGL((k_colsum_fin<2 * kBnFinCh, BnBwdFin>),
                     dim3((unsigned)ceil_div(channels, kBnFinCh)), dim3(256), 0,
                     as_stream(stream), partials, num_partials, 2 * channels, fin);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_mlp_bwd1(const float* dbn, const float* a1, const float* bn_save,
                             const float* coef, const float* w1, float* dz, int64_t num_nodes,
                             int32_t channels, void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !dbn || !a1 || !bn_save || !coef || !w1 || !dz)
    return GINE_ERR_INVALID;
  ProArgs pa{dbn, a1, nullptr, bn_save, coef};
  EpiArgs ea{nullptr, dz, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  return launch_rowgemm<PRO_DA1, EPI_PLAIN, false>(channels, w1, pa, ea, num_nodes,
                                                   as_stream(stream));
}

extern "C" int gine_mlp_bwd2_acc(const float* dy, const float* y, const uint8_t* mask,
                                 const float* a1, const float* bn_save, const float* w2,
                                 float* dbn, double* partials, int64_t* bn_acc,
                                 int64_t num_nodes, int32_t channels, int32_t epilogue,
                                 void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !dy || !a1 || !bn_save || !w2 || !dbn || !bn_acc)
    return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RELU && !y) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && !mask) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  ProArgs pa{dy, y, mask, nullptr, nullptr};
  EpiArgs ea{nullptr, dbn, nullptr, nullptr, a1, bn_save, partials, 0,
             reinterpret_cast<long long*>(bn_acc)};
  hipStream_t s = as_stream(stream);
  switch (epilogue) {
    case GINE_EPI_NONE:
      return launch_rowgemm<PRO_PLAIN, EPI_DBN, false>(channels, w2, pa, ea, num_nodes, s);
    case GINE_EPI_RELU:
      return launch_rowgemm<PRO_DOR, EPI_DBN, false>(channels, w2, pa, ea, num_nodes, s);
    default:
      return launch_rowgemm<PRO_DOM, EPI_DBN, false>(channels, w2, pa, ea, num_nodes, s);
  }
}

extern "C" int gine_mlp_bwd1_bn(const float* dbn, const float* a1, const float* bn_save,
                                int64_t* bn_acc, const float* gamma, float* dgamma,
                                float* dbeta, float* coef, const float* w1, float* dz,
                                int64_t num_nodes, int32_t channels, void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !dbn || !a1 || !bn_save || !bn_acc || !coef || !w1 || !dz)
    return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  ProArgs pa{dbn, a1, nullptr, bn_save, nullptr};
  EpiArgs ea{nullptr, dz, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  long long* acc = reinterpret_cast<long long*>(bn_acc);
  const int grid = rowgemm_grid(num_nodes, channels);
  const int tiles = (int)ceil_div(num_nodes, kRowTile);
  hipStream_t s = as_stream(stream);
  switch (channels) {
    case 32:
      hipLaunchKernelGGL(k_bwd1_bnacc<32>, dim3(grid), dim3(64), 0, s, w1, pa, ea, gamma,
                         dgamma, dbeta, coef, acc, num_nodes, tiles);
      break;
    case 64:
      hipLaunchKernelGGL(k_bwd1_bnacc<64>, dim3(grid), dim3(128), 0, s, w1, pa, ea, gamma,
                         dgamma, dbeta, coef, acc, num_nodes, tiles);
      break;
    case 128:
      hipLaunchKernelGGL(k_bwd1_bnacc<128>, dim3(grid), dim3(256), 0, s, w1, pa, ea, gamma,
                         dgamma, dbeta, coef, acc, num_nodes, tiles);
      break;
    default:
      hipLaunchKernelGGL(k_bwd1_bnacc<256>, dim3(grid), dim3(512), 0, s, w1, pa, ea, gamma,
                         dgamma, dbeta, coef, acc, num_nodes, tiles);
      break;
  }
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_mlp_wgrad_num_chunks(int64_t num_nodes, int32_t channels,
                                         int32_t* num_chunks) {
  if (!num_chunks || num_nodes < 0) return GINE_ERR_INVALID;
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  *num_chunks = mlp_wgrad_plan(num_nodes, channels).chunks;
  return GINE_OK;
}

extern "C" int gine_mlp_wgrad(const float* dy, const float* y, const uint8_t* mask,
                              const float* a1, const float* bn_save, const float* dbn,
                              const float* coef, const float* z, float* slab, float* dw1,
                              float* db1, float* dw2, float* db2, int64_t num_nodes,
                              int32_t channels, int32_t epilogue, void* stream) {
  if (!mlp_dim_ok(channels)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !dy || !a1 || !bn_save || !dbn || !coef || !z || !slab)
    return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RELU && !y) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && !mask) return GINE_ERR_INVALID;
  const int D = channels;
  const ProArgs p_do{dy, y, mask, nullptr, nullptr};
  const ProArgs q_r{a1, nullptr, nullptr, bn_save, nullptr};
  const ProArgs p_da1{dbn, a1, nullptr, bn_save, coef};
  const ProArgs q_z{z, nullptr, nullptr, nullptr, nullptr};
  const WgPlan p = mlp_wgrad_plan(num_nodes, D);
  const size_t per = (size_t)D * D + D;
  hipStream_t s = as_stream(stream);
  int st;
  if (epilogue == GINE_EPI_NONE) {
    const MlpWgradSrc<PRO_PLAIN> src{p_do, q_r, p_da1, q_z, D};
    st = launch_wgrad_engine<kMlpWgTO, MlpWgradSrc<PRO_PLAIN>, kMlpEngX3>(src, num_nodes, D, D, 2 * p.tiles_o * p.tiles_i, p,
                                       per * p.chunks, per, slab, s);
  } else if (epilogue == GINE_EPI_RELU) {
    const MlpWgradSrc<PRO_DOR> src{p_do, q_r, p_da1, q_z, D};
    st = launch_wgrad_engine<kMlpWgTO, MlpWgradSrc<PRO_DOR>, kMlpEngX3>(src, num_nodes, D, D, 2 * p.tiles_o * p.tiles_i, p,
                                       per * p.chunks, per, slab, s);
  } else {
    const MlpWgradSrc<PRO_DOM> src{p_do, q_r, p_da1, q_z, D};
    st = launch_wgrad_engine<kMlpWgTO, MlpWgradSrc<PRO_DOM>, kMlpEngX3>(src, num_nodes, D, D, 2 * p.tiles_o * p.tiles_i, p,
                                       per * p.chunks, per, slab, s);
  }
  if (st != GINE_OK) return st;
  if (!dw1 && !db1 && !dw2 && !db2) return GINE_OK;  // slab left for a batched reduction
  return launch_slab_sum(slab, p.chunks, (int64_t)per, per, per * p.chunks, 2,
                         MlpWgradOut{dw2, db2, dw1, db1, D}, s);
}

extern "C" int gine_mlp_bwd1_wgrad(const float* dy, const float* y, const uint8_t* mask,
                                   const float* a1, const float* bn_save, const float* dbn,
                                   const float* coef, const float* z, const float* w1, float* dz,
                                   float* slab, float* dw1, float* db1, float* dw2, float* db2,
                                   int64_t num_nodes, int32_t channels, int32_t epilogue,
                                   void* stream) {
  if (channels != 128) {  // fused launch for the 256-thread shapes; two launches otherwise
    int rc = gine_mlp_bwd1(dbn, a1, bn_save, coef, w1, dz, num_nodes, channels, stream);
    if (rc != GINE_OK) return rc;
    return gine_mlp_wgrad(dy, y, mask, a1, bn_save, dbn, coef, z, slab, dw1, db1, dw2, db2,
                          num_nodes, channels, epilogue, stream);
  }
  if (num_nodes <= 0 || !dy || !a1 || !bn_save || !dbn || !coef || !z || !w1 || !dz || !slab)
    return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  if (epilogue == GINE_EPI_RELU && !y) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && !mask) return GINE_ERR_INVALID;
  const int D = channels;
  const ProArgs pa{dbn, a1, nullptr, bn_save, coef};
  const EpiArgs ea{nullptr, dz, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  const ProArgs p_do{dy, y, mask, nullptr, nullptr};
  const ProArgs q_r{a1, nullptr, nullptr, bn_save, nullptr};
  const ProArgs p_da1{dbn, a1, nullptr, bn_save, coef};
  const ProArgs q_z{z, nullptr, nullptr, nullptr, nullptr};
  const WgPlan p = mlp_wgrad_plan(num_nodes, D);
  const size_t per = (size_t)D * D + D;
  const int eng = p.chunks * 2 * p.tiles_o * p.tiles_i;
  const int rg = rowgemm_grid(num_nodes, D);
  const int tiles = (int)ceil_div(num_nodes, kRowTile);
  hipStream_t s = as_stream(stream);
#define BWD1_WGRAD(PD)                                                                        \
  hipLaunchKernelGGL(k_bwd1_wgrad<PD>, dim3(eng + rg), dim3(256), 0, s, w1, pa, ea, num_nodes, \
                     tiles, rg, MlpWgradSrc<PD>{p_do, q_r, p_da1, q_z, D}, p.chunks,           \
                     p.rows_per_chunk, per * p.chunks, per, slab, eng)
  if (epilogue == GINE_EPI_NONE) BWD1_WGRAD(PRO_PLAIN);
  else if (epilogue == GINE_EPI_RELU) BWD1_WGRAD(PRO_DOR);
  else BWD1_WGRAD(PRO_DOM);
#undef BWD1_WGRAD
  GINE_LAUNCH_STATUS();
  if (!dw1 && !dw2 && !db1 && !db2) return GINE_OK;  // slab left for gine_mp_bwd_side
  return launch_slab_sum(slab, p.chunks, (int64_t)per, per, per * p.chunks, 2,
                         MlpWgradOut{dw2, db2, dw1, db1, D}, s);
}

#ifdef GINE_RG_PROFILE
extern "C" int gine_debug_rg_prof(long long* out, int* n) {
  GINE_RETURN_IF_HIP(hipDeviceSynchronize());
  GINE_RETURN_IF_HIP(hipMemcpyFromSymbol(n, HIP_SYMBOL(g_rg_prof_n), sizeof(int)));
  GINE_RETURN_IF_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rg_prof), sizeof(long long) * 4096));
  const int zero = 0;
  GINE_RETURN_IF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_rg_prof_n), &zero, sizeof(int)));
  return GINE_OK;
}
#endif
