// GINEConv forward message passing fused with the first node-MLP Linear (D = 128).
//
// Replaces, in one launch (models/gnn.py:41,44 -> PyG GINEConv.forward -> nn[0]):
//   z  = scatter_add(relu(x[src] + Linear(1,D)(edge_attr)), dst) + (1 + eps) x
//   a1 = z W1^T + b1,   per-workgroup fp64 partial sums of a1 and a1^2 (BatchNorm1d stats)
// which otherwise are gine_mp_fwd (gather, L2-bound, no matrix work) followed by
// gine_mlp_fwd1 (row-tile GEMM, matrix-bound, one HBM read of z).  The two are
// complementary, so one 768-thread workgroup per CU runs both on the same 32-row tiles,
// split by wave role:
//   waves 4-11 ("gather"): tile k+1's destinations -- each half-wave owns 2 rows, lane t
//            the 16-byte column chunk t; edge lists run two stages ahead, 22 neighbour
//            rows in flight per lane -- written to an LDS z tile and to HBM;
//   waves 0-3 ("matrix"): tile k's 64-step v_mfma_f32_32x32x2_f32 chain against W1
//            fragments held in VGPRs, then bias + BN statistics + a1 store, transposed
//            through a per-wave LDS tile (no cross-wave barrier).
// One __syncthreads per tile hands the z tile over (double-buffered).
//
// Measured (tools/fused_micro.py, HIP-graph replay, MI355X): cfg1 7.5 us vs 8.1 for the
// pair, cfg2 15.1 vs 16.9; at cfg3 (4,000 tiles) 121 vs 96 -- the gather waves keep fewer
// loads in flight than the standalone gather kernel's 32 waves per CU, which only the
// short per-workgroup tile runs hide.  The host uses it up to 2 tiles per workgroup.
//
// Results are bit-identical to the unfused pair: z follows k_mp_fwd's per-edge rounding
// sequence in CSR order (gine_edge.hpp), a1 the row-tile GEMM's MFMA order, and the BN
// partials its row-group summation order over the same tile -> workgroup assignment
// (xcd_tile_range, grid = gine_mlp_num_partials).  Every in-degree must be at most
// GINE_MP_FUSED_MAX_DEGREE (one 32-slot edge list per row; the host checks).
#include "gine_common.hpp"
#include "gine_bnacc.hpp"
#include "gine_edge.hpp"
#include "gine_bf16x3.hpp"
#include "gine_headrow.hpp"
#include "gine_mlpsrc.hpp"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <type_traits>

namespace gine {
namespace {

constexpr int kD = 128, kD4 = kD / 4;
constexpr int kTileRows = 32;
constexpr int kLD = kD + 4;                 // padded z-tile / W row (floats)
constexpr int kKS = kD / 2;                 // MFMA k-steps per lane half
#ifndef GINE_FUSED_GATHER_WAVES
#define GINE_FUSED_GATHER_WAVES 8
#endif
constexpr int kMatThreads = 256;                                 // waves 0-3
constexpr int kGatherWaves = GINE_FUSED_GATHER_WAVES;            // waves 4-...
constexpr int kThreads = kMatThreads + kWave * kGatherWaves;
constexpr int kHalves = 2 * kGatherWaves;                        // gather half-waves
constexpr int kRowsPerHalf = kTileRows / kHalves;
static_assert(kRowsPerHalf % 2 == 0, "rows are gathered in pairs");
constexpr int kSlots = GINE_MP_FUSED_MAX_DEGREE;
constexpr int kU = 11;  // neighbour rows in flight per row, 2 rows per round (k=10: one)
constexpr int kTLD = 36;                    // per-wave transposition tile row (floats)
constexpr uint32_t kRowBytes = kD * 4;
// experiment builds only (make variant VDEFS=-DGINE_FUSED_DBG=n): 1 = no neighbour loads,
// 2 = no MFMA chain -- the two roles timed without each other
#ifndef GINE_FUSED_DBG
#define GINE_FUSED_DBG 0
#endif

typedef float floatx16 __attribute__((ext_vector_type(16)));

#ifdef GINE_LAYER_PROFILE
// Debug build only (make layerprof): thread 0 of every workgroup of the one-launch layer
// forward stamps s_memtime at its phase boundaries (tools/layer_prof.py):
// 0 entry, 1 matrix role done, 2 phase A done (block), 3 barrier arrival, 4 grid barrier
// passed, 5 BatchNorm finish + W2 fragments done, 6 r = relu(bn(a1)) done, 7 last Linear2
// chain done.
// Phase A detail: 8 W1 planes ready, 9 / 11 tile 1 / 2 chain done, 10 / 12 tile 1 / 2
// epilogue done, 13 statistics in the accumulator (matrix role, thread 0); 14 / 15 tile 1 /
// 2 gathered (gather role, thread 256).
// 16-19: s_memrealtime (the 100 MHz clock every XCD shares) at entry, barrier arrival,
// barrier release and the end, for the arrival skew across workgroups.
// 20 / 21: tile 1 / 2's planes in LDS (matrix role); 22 / 23: the window form's tile 1 / 2
// staged (gather role, thread 256, after G).
__device__ long long g_layer_prof[1024][24];
#define LAYER_RT(i)                                                              \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 1024)                                   \
      g_layer_prof[blockIdx.x][i] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define LAYER_MARK_T(t, i)                                                       \
  do {                                                                           \
    if (threadIdx.x == (t) && blockIdx.x < 1024)                                 \
      g_layer_prof[blockIdx.x][i] = (long long)__builtin_amdgcn_s_memtime();    \
  } while (0)
#else
#define LAYER_MARK_T(t, i) do {} while (0)
#define LAYER_RT(i) do {} while (0)
#endif
#define LAYER_MARK(i) LAYER_MARK_T(0, i)

struct TileSeq {
  int first, end, step;
  __device__ int count() const { return first < end ? (end - first + step - 1) / step : 0; }
  __device__ int at(int k) const { return first + k * step; }
};
// The row-tile GEMM's tile -> workgroup assignment (gine_mlp.hip xcd_tile_range): the tiles
// of one XCD form a contiguous range, its workgroups stride it.
__device__ __forceinline__ TileSeq tile_seq(int num_tiles, int vb, int nb) {
  const int xcd = vb % kNumXcd, pos = vb / kNumXcd;
  const int here = nb / kNumXcd + (xcd < nb % kNumXcd ? 1 : 0);
  const int span = (num_tiles + kNumXcd - 1) / kNumXcd;
  const int b = xcd * span;
  return TileSeq{b + pos, min(num_tiles, b + span), here};
}

// Edge lists run two stages ahead of their use, with nothing waiting on a load until the
// tile that consumes it: rowptr of tile k+2 and the edge slots of tile k+1 are issued while
// tile k is gathered.  Lane t keeps slot t of each of its half-wave's 4 rows; the selects
// that depend on loaded values (slot past the in-degree -> the row itself, a valid index)
// run when the slots are written to LDS, not right behind the loads.
struct RowptrStage {
  int32_t beg[kRowsPerHalf], end[kRowsPerHalf];
};
struct EdgeStage {
  int32_t nbr[kRowsPerHalf];
  float attr[kRowsPerHalf];
  int cnt[kRowsPerHalf];
};

// acc += relu(r + lin(a)) when ok (else + 0: acc is never -0, so adding +0 is exact)
template <bool FMA>
__device__ __forceinline__ void edge_acc(f4v& acc, f4v r, float a, f4v w, f4v b, bool ok) {
  const f2v lo = relu2(r.xy + edge_lin2<FMA>(a, w.xy, b.xy));
  const f2v hi = relu2(r.zw + edge_lin2<FMA>(a, w.zw, b.zw));
  const f2v zero = {0.f, 0.f};
  acc.xy = acc.xy + (ok ? lo : zero);
  acc.zw = acc.zw + (ok ? hi : zero);
}

struct FusedArgs {
  const float* x;
  const int32_t* rowptr;
  const int32_t* nbr;
  const float* attr;
  const float* lin_w;
  const float* lin_b;
  const float* eps;
  const float* W1;
  const float* b1;
  float* z;
  float* a1;
  double* partials;      // NULL: bnacc only
  long long* bnacc;      // NULL: partials only (gine_bnacc.hpp)
  int N, num_tiles;
};

struct FusedLds {
  // W1 staging (prologue only), then the matrix waves' transposition tiles and, at the end,
  // their statistics scratch (disjoint regions)
  float w[kD * kLD];
  float z[2][kTileRows * kLD];  // z tiles, gather -> matrix, double-buffered
  int32_t nbr[kHalves][kRowsPerHalf][kSlots];
  float attr[kHalves][kRowsPerHalf][kSlots];
};
static_assert(4 * 32 * kTLD * 4 + 2 * 8 * kD * 8 <= kD * kLD * 4, "scratch fits in w");

// The one-launch layer's phase A hands each z tile from the gather waves to the matrix waves
// as split-bf16 planes (hi | mid | lo, gine_bf16x3.hpp split2), split ONCE by the producers:
// in the pair form every matrix wave splits the whole 32x128 A tile inside its chain (4x the
// work, on the SIMDs the gather waves issue from: the 4 matrix waves' in-loop split is ~450
// VALU instructions each per tile against the gather waves' ~570).  The fp32 z tile is not
// kept in LDS (the rare non-finite redo reads z back from HBM): tile it's planes live in the
// z region (it even) or in the w region past the matrix waves' transposition tiles and
// statistics scratch (it odd; W1's staging there is over by then).
constexpr int kPS = kD + 8;  // split-plane row stride (bf16): conflict-free 16-byte reads
constexpr int kPlaneBytes = 3 * kTileRows * kPS * 2;
constexpr int kPlaneOffW = 4 * 32 * kTLD * 4 + 2 * 8 * kD * 8;  // bytes into w
static_assert(kPlaneOffW + kPlaneBytes <= kD * kLD * 4, "odd tiles' planes fit in w");
static_assert(kPlaneBytes <= 2 * kTileRows * kLD * 4, "even tiles' planes fit in the z tiles");
__device__ __forceinline__ uint16_t* tile_planes(FusedLds& L, int it) {
  return (it & 1) ? reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(L.w) + kPlaneOffW)
                  : reinterpret_cast<uint16_t*>(&L.z[0][0]);
}

// Matrix role (waves 0-3).  Barriers: 1 + (nt + 1), as the gather role.
// LAYER (gine_mp_fwd_layer): every a1 tile is also kept in LDS (a1k[it], row-major, at most
// kLayerTiles of them) for the second half of the layer, and the producer's phase word is
// left to the caller.
template <bool LAYER = false>
__device__ __forceinline__ void matrix_role(const FusedArgs& A, FusedLds& L, const TileSeq& ts,
                                            int nt, float* a1k = nullptr) {
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int cq = lane & 7, grp = lane >> 3;  // transposed epilogue: 4-column chunk, row group
  {
    const float4* w4 = reinterpret_cast<const float4*>(A.W1);
    float4 wt[kD * kD4 / kMatThreads];
#pragma unroll
    for (int j = 0; j < kD * kD4 / kMatThreads; ++j) wt[j] = w4[tid + kMatThreads * j];
#pragma unroll
    for (int j = 0; j < kD * kD4 / kMatThreads; ++j) {
      const int idx = tid + kMatThreads * j;
      *reinterpret_cast<float4*>(&L.w[(idx / kD4) * kLD + 4 * (idx % kD4)]) = wt[j];
    }
  }
  const float4 bias4 = *reinterpret_cast<const float4*>(A.b1 + 32 * wave + 4 * cq);
  __syncthreads();
  // W1^T fragments: B[k][j] = W1[j][k], lane half h takes k in [h*64, h*64+64)
  float bf[kKS];
  {
    const float* wr = &L.w[(32 * wave + c32) * kLD + h * kKS];
#pragma unroll
    for (int q = 0; q < kKS / 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(&wr[4 * q]);
      bf[4 * q] = v.x;
      bf[4 * q + 1] = v.y;
      bf[4 * q + 2] = v.z;
      bf[4 * q + 3] = v.w;
    }
  }
  BPlanes<kKS> bp;
  if constexpr (GINE_GEMM_BF16X3) bp.from(bf);
  __syncthreads();  // (iteration 0: the gather role stages the first tile)
  if constexpr (LAYER) LAYER_MARK(8);
  // per-column BatchNorm sums of this lane's (row group, 4 columns), kept in the statistics
  // scratch of LDS between tiles rather than in 16 VGPRs beside the B planes (the lane's own
  // slots, brought into registers for each tile's rows: the same sequential order, the same
  // bits); W1's staging is over
  double* sr = reinterpret_cast<double*>(&L.w[4 * 32 * kTLD]);  // [2][8][kD]
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 32 * wave + 4 * cq + k;
    sr[(0 * 8 + grp) * kD + c] = 0.0;
    sr[(1 * 8 + grp) * kD + c] = 0.0;
  }
  const float bb[4] = {bias4.x, bias4.y, bias4.z, bias4.w};
  float* tt = &L.w[wave * 32 * kTLD];
  for (int it = 1; it <= nt; ++it) {
    const int T = ts.at(it - 1);
    if constexpr (LAYER) {
      if (it <= 2) LAYER_MARK(19 + it);  // (profile builds) tile it's z is in LDS
    }
    const float* arow = &L.z[(it - 1) & 1][c32 * kLD + h * kKS];
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if constexpr (LAYER) {  // the same chain from the gather waves' split planes
      static_assert(GINE_GEMM_BF16X3, "the layer forward reads split planes");
      const uint16_t* pa = tile_planes(L, it - 1) + c32 * kPS + h * kKS;
      auto frag = [&](int s8) {
        Bf16x3 a;
        a.h = *reinterpret_cast<const bf16x8_t*>(pa + 8 * s8);
        a.m = *reinterpret_cast<const bf16x8_t*>(pa + kTileRows * kPS + 8 * s8);
        a.l = *reinterpret_cast<const bf16x8_t*>(pa + 2 * kTileRows * kPS + 8 * s8);
        return a;
      };
      // one fragment in flight beside the current block's six MFMAs (192 cycles hide the LDS
      // latency): with all eight hoisted the matrix waves' B planes (96 VGPRs) spilled
      Bf16x3 a = frag(0);
#pragma unroll
      for (int s8 = 0; s8 < (GINE_FUSED_DBG == 2 ? 1 : kKS / 8); ++s8) {
        Bf16x3 an = a;
        if (s8 + 1 < kKS / 8) an = frag(s8 + 1);
        acc = mfma_bf16x3(a, bp.f[s8], acc);
        __builtin_amdgcn_sched_barrier(0);
        a = an;
      }
      if (wave_any_nan(acc)) {  // non-finite operands: the fp32 chain on z read back from HBM
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the gather waves' z stores
        const int64_t zr = min((int64_t)T * kTileRows + c32, (int64_t)A.N - 1);
        acc = mfma_f32_row_mem<kKS>(A.z + zr * kD + h * kKS,
                                    A.W1 + (size_t)(32 * wave + c32) * kD + h * kKS, 1, acc);
      }
    } else if constexpr (GINE_GEMM_BF16X3) {  // the row-tile GEMM's split-bf16 chain (gine_mlp.hip)
#pragma unroll
      for (int s = 0; s < (GINE_FUSED_DBG == 2 ? 1 : kKS / 8); ++s) {
        const float4 a0 = *reinterpret_cast<const float4*>(&arow[8 * s]);
        const float4 a1 = *reinterpret_cast<const float4*>(&arow[8 * s + 4]);
        acc = mfma_bf16x3(split8(a0, a1), bp.f[s], acc);
      }
      if (wave_any_nan(acc)) {  // non-finite operands: the fp32 chain (gine_bf16x3.hpp)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
        acc = mfma_f32_row_mem<kKS>(arow, A.W1 + (size_t)(32 * wave + c32) * kD + h * kKS, 1,
                                    acc);
      }
    } else {
#pragma unroll
      for (int q = 0; q < (GINE_FUSED_DBG == 2 ? 1 : kKS / 4); ++q) {
        const float4 a4 = *reinterpret_cast<const float4*>(&arow[4 * q]);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, bf[4 * q], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, bf[4 * q + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, bf[4 * q + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, bf[4 * q + 3], acc, 0, 0, 0);
      }
    }
#ifdef GINE_LAYER_PROFILE
    if constexpr (LAYER) {
      if (it <= 2 && acc[0] == 1.2345e-30f) tt[0] = 0.f;  // the stamp waits for the chain
      if (it <= 2) LAYER_MARK(7 + 2 * it);
    }
#endif
    // this wave's 32x32 block -> row-major through its own LDS tile
#pragma unroll
    for (int r = 0; r < 16; ++r) tt[((r & 3) + 8 * (r >> 2) + 4 * h) * kTLD + c32] = acc[r];
    __builtin_amdgcn_wave_barrier();
    // the running sums come into registers for the tile's 4 rows (same order, same bits)
    double st1[4], st2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      st1[k] = sr[(0 * 8 + grp) * kD + 32 * wave + 4 * cq + k];
      st2[k] = sr[(1 * 8 + grp) * kD + 32 * wave + 4 * cq + k];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = grp + 8 * i;
      const int64_t n = (int64_t)T * kTileRows + row;
      const float4 v = *reinterpret_cast<const float4*>(&tt[row * kTLD + 4 * cq]);
      if (n >= A.N) continue;
      const float vv[4] = {v.x, v.y, v.z, v.w};
      float o4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o4[k] = vv[k] + bb[k];
        st1[k] += (double)o4[k];
        st2[k] += (double)o4[k] * (double)o4[k];
      }
      *reinterpret_cast<float4*>(A.a1 + n * kD + 32 * wave + 4 * cq) =
          make_float4(o4[0], o4[1], o4[2], o4[3]);
      if constexpr (LAYER)
        *reinterpret_cast<float4*>(&a1k[(it - 1) * kTileRows * kLD + row * kLD + 32 * wave +
                                        4 * cq]) = make_float4(o4[0], o4[1], o4[2], o4[3]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sr[(0 * 8 + grp) * kD + 32 * wave + 4 * cq + k] = st1[k];
      sr[(1 * 8 + grp) * kD + 32 * wave + 4 * cq + k] = st2[k];
    }
    __builtin_amdgcn_wave_barrier();  // the next tile's transposition writes come after
    if constexpr (LAYER) {
      if (it <= 2) LAYER_MARK(8 + 2 * it);
    }
    __syncthreads();
  }
  // per-column partials: the 8 row groups added in fixed order (row-tile GEMM order)
  __builtin_amdgcn_wave_barrier();
  const int which = lane >> 5, cc = 32 * wave + (lane & 31);
  double s = 0.0;
#pragma unroll
  for (int g = 0; g < 8; ++g) s += sr[(which * 8 + g) * kD + cc];
  if (A.partials) A.partials[(size_t)blockIdx.x * 2 * kD + which * kD + cc] = s;
  if constexpr (LAYER) {
    bnacc_add<false>(A.bnacc, 2 * kD, which * kD + cc, s);
    // the atomics are performed before this workgroup arrives at the grid barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LAYER_MARK(13);
  } else if (A.bnacc) {
    bnacc_add(A.bnacc, 2 * kD, which * kD + cc, s);
  }
}

// Gather role (waves 4-11).  Barriers: 1 + (nt + 1), as the matrix role; without LAST_SYNC
// the caller runs the last one (after work of its own beside the matrix role's last tile).
// PLANES (the one-launch layer): the tile goes to the matrix waves as split-bf16 planes
// (tile_planes) instead of an fp32 LDS tile.
template <bool FMA, bool LAST_SYNC = true, bool PLANES = false>
__device__ __forceinline__ void gather_role(const FusedArgs& A, FusedLds& L, const TileSeq& ts,
                                            int nt) {
  const int p = threadIdx.x - kMatThreads;
  const int hw = p >> 5, t = p & 31;
  const int N = A.N;
  const uint32_t qb = (uint32_t)t * 16u;
  const char* xb = reinterpret_cast<const char*>(A.x);
  RowptrStage rp;
  EdgeStage es;
#pragma unroll
  for (int i = 0; i < kRowsPerHalf; ++i) {
    rp.beg[i] = rp.end[i] = 0;
    es.nbr[i] = 0;
    es.attr[i] = 0.f;
    es.cnt[i] = 0;
  }
  auto row_of = [&](int T, int i) { return T * kTileRows + hw + kHalves * i; };
  auto clamp_row = [&](int n) { return n < N ? n : N - 1; };
  auto issue_rowptr = [&](int T) {  // -> rp (no wait)
#pragma unroll
    for (int i = 0; i < kRowsPerHalf; ++i) {
      const int n = clamp_row(row_of(T, i));
      rp.beg[i] = A.rowptr[n];
      rp.end[i] = A.rowptr[n + 1];
    }
  };
  auto issue_edges = [&](int T) {  // rp (of tile T, arrived) -> es (no wait)
#pragma unroll
    for (int i = 0; i < kRowsPerHalf; ++i) {
      const int cnt = row_of(T, i) < N ? min(rp.end[i] - rp.beg[i], kSlots) : 0;
      const int e = cnt > 0 ? rp.beg[i] + min(t, cnt - 1) : 0;  // always a valid index
      es.nbr[i] = A.nbr[e];
      es.attr[i] = A.attr[e];
      es.cnt[i] = cnt;
    }
  };
  const f4v lw = ld_f4v(reinterpret_cast<const char*>(A.lin_w), qb);
  const f4v lb = ld_f4v(reinterpret_cast<const char*>(A.lin_b), qb);
  const float ope = 1.0f + A.eps[0];
  if (nt > 0) {
    issue_rowptr(ts.at(0));
    issue_edges(ts.at(0));
  }
  if (nt > 1) issue_rowptr(ts.at(1));
  __syncthreads();

  for (int it = 0; it < nt; ++it) {
    const int T = ts.at(it);
    float* sz = L.z[it & 1];
    int cnt[kRowsPerHalf];
#pragma unroll
    for (int i = 0; i < kRowsPerHalf; ++i) {
      L.nbr[hw][i][t] = t < es.cnt[i] ? es.nbr[i] : clamp_row(row_of(T, i));
      L.attr[hw][i][t] = es.attr[i];
      cnt[i] = es.cnt[i];
    }
    __builtin_amdgcn_wave_barrier();
    if (it + 1 < nt) issue_edges(ts.at(it + 1));
    if (it + 2 < nt) issue_rowptr(ts.at(it + 2));
    f4v self[kRowsPerHalf], acc[kRowsPerHalf];
#pragma unroll
    for (int i = 0; i < kRowsPerHalf; ++i) {
      self[i] = ld_f4v(xb, (uint32_t)clamp_row(row_of(T, i)) * kRowBytes + qb);
      acc[i] = f4v_zero();
    }
#pragma unroll
    for (int pr = 0; pr < kRowsPerHalf; pr += 2) {
      const int m = GINE_FUSED_DBG == 1 ? 0 : max(cnt[pr], cnt[pr + 1]);
      for (int j0 = 0; j0 < m; j0 += kU) {
        f4v r0[kU], r1[kU];
        float a0[kU], a1v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int j = min(j0 + u, kSlots - 1);
          r0[u] = ld_f4v(xb, (uint32_t)L.nbr[hw][pr][j] * kRowBytes + qb);
          r1[u] = ld_f4v(xb, (uint32_t)L.nbr[hw][pr + 1][j] * kRowBytes + qb);
          a0[u] = L.attr[hw][pr][j];
          a1v[u] = L.attr[hw][pr + 1][j];
        }
        // (an unmasked copy of this loop for full batches -- the common case -- spilled: 292 B of
        // scratch in k_mp_fwd_mlp1, which then ran 34 instead of 14 us; profiles/r05_s15)
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          edge_acc<FMA>(acc[pr], r0[u], a0[u], lw, lb, j0 + u < cnt[pr]);
          edge_acc<FMA>(acc[pr + 1], r1[u], a1v[u], lw, lb, j0 + u < cnt[pr + 1]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kRowsPerHalf; ++i) {
      const int r = hw + kHalves * i;
      const int64_t n = (int64_t)T * kTileRows + r;
      const f4v zv = add_scaled(acc[i], ope, self[i]);
      if constexpr (PLANES) {
        uint32_t h0, m0, l0, h1, m1, l1;
        split2(zv.x, zv.y, h0, m0, l0);
        split2(zv.z, zv.w, h1, m1, l1);
        uint16_t* pl = tile_planes(L, it) + r * kPS + 4 * t;
        *reinterpret_cast<uint2*>(pl) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(pl + kTileRows * kPS) = make_uint2(m0, m1);
        *reinterpret_cast<uint2*>(pl + 2 * kTileRows * kPS) = make_uint2(l0, l1);
      } else {
        *reinterpret_cast<f4v*>(&sz[r * kLD + 4 * t]) = zv;
      }
      if (n < N) *reinterpret_cast<f4v*>(A.z + n * kD + 4 * t) = zv;
    }
    if (it < 2) LAYER_MARK_T(kMatThreads, 14 + it);
    __builtin_amdgcn_wave_barrier();  // edge-list reads done before the next tile's writes
    __syncthreads();
  }
  if constexpr (LAST_SYNC) __syncthreads();  // (iteration nt: the matrix role multiplies the last tile)
}

template <bool FMA>
__global__ __launch_bounds__(kThreads, 1) void k_mp_fwd_mlp1(FusedArgs A) {
  __shared__ __attribute__((aligned(16))) FusedLds L;
  const TileSeq ts = tile_seq(A.num_tiles, blockIdx.x, gridDim.x);
  const int nt = ts.count();
  // the role is wave-uniform (an SGPR): each wave branches, none runs the other's barriers
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  if (wave < kMatThreads / kWave) matrix_role(A, L, ts, nt);
  else gather_role<FMA>(A, L, ts, nt);
}

// ---------------------------------------------------------------------------------------
// The whole node-MLP forward of the layer in one launch (gine_mp_fwd_layer):
//   phase A = k_mp_fwd_mlp1 (gather -> z, Linear1 -> a1, BatchNorm sums into the fixed-point
//             accumulator), a1 tiles also kept in LDS;
//   grid barrier (every workgroup resident: one per CU, host-checked);
//   phase B = k_fwd2_bnacc on the workgroup's own tiles: BatchNorm finish from the
//             accumulator totals, r = relu(bn(a1)) from the LDS tiles, split once into
//             split-bf16 planes by the gather waves (the matrix waves' Linear2 chains read
//             them instead of splitting inside the chain), epilogue (bias, ResGnn ReLU /
//             residual + mask) on the gather waves.
// W2 is loaded by the gather waves under the matrix role's last chain and staged in LDS
// before the barrier; its fragments are read after it, beside the BatchNorm totals (gather
// waves), so a workgroup arrives as soon as its phase A is done; the residual rows are
// loaded under the BatchNorm finish.
// Same tile -> workgroup map, same arithmetic and order as the two-launch pair (bit-identical:
// the BatchNorm totals are integer sums, the MFMA chains and epilogues are the row GEMM's).
// ---------------------------------------------------------------------------------------
constexpr int kLayerTiles = 2;  // a1 tiles a workgroup keeps in LDS
static_assert(kLayerTiles * 3 * kTileRows * kPS * 2 <= kD * kLD * 4, "planes fit in w");

// W2 in flight in the gather waves' registers: 8 float4 per thread (element idx = t + n*j,
// row idx / kD4, column chunk idx % kD4), staged into the padded LDS image.
template <int PER>
struct W2Regs {
  static_assert(PER == 8, "eight float4 per gather thread");
  float4 v0, v1, v2, v3, v4, v5, v6, v7;
  __device__ __forceinline__ void load(const float4* __restrict__ w4, int t, int n) {
    v0 = w4[t]; v1 = w4[t + n]; v2 = w4[t + 2 * n]; v3 = w4[t + 3 * n];
    v4 = w4[t + 4 * n]; v5 = w4[t + 5 * n]; v6 = w4[t + 6 * n]; v7 = w4[t + 7 * n];
  }
  __device__ __forceinline__ void put(float* w, int idx, float4 v) const {
    *reinterpret_cast<float4*>(&w[(idx / kD4) * kLD + 4 * (idx % kD4)]) = v;
  }
  __device__ __forceinline__ void store(float* w, int t, int n) const {
    put(w, t, v0); put(w, t + n, v1); put(w, t + 2 * n, v2); put(w, t + 3 * n, v3);
    put(w, t + 4 * n, v4); put(w, t + 5 * n, v5); put(w, t + 6 * n, v6); put(w, t + 7 * n, v7);
  }
};

struct LayerArgs {
  const float* W2;
  const float* b2;
  float* y;
  uint8_t* mask;
  BnFwdParams q;
  const int2* win;     // WIN: per 32-row tile (first window row, window rows)
  int win_rows;        // WIN: max window rows over the tiles (the dummy row's index)
  int win_slots;       // WIN: slots per row of the padded slot table (lw_slots)
  gine_layer_head hd;  // the output head folded into the epilogue (hk > 0)
  int hk;              // head outputs per node (2..5), 0: no head
};

// The output head's LDS block (gine_layer_head): weights [kMaxK][kD] | bias [8] | raw outputs
// of the workgroup's tiles [kLayerTiles][32][K] (PostProcess and the stores after the tile
// loop, one element per thread) | valid-target counts per part [GINE_COUNT_PARTS] (uint32)
constexpr int kHB = head::kMaxK * kD;
constexpr int kHR = kHB + 8;
constexpr int kHRTile = kTileRows * head::kMaxK;
constexpr int kHC = kHR + kLayerTiles * kHRTile;
constexpr int kHeadFloats = kHC + GINE_COUNT_PARTS;

struct LayerLds {
  FusedLds f;
  float a1k[kLayerTiles][kTileRows * kLD];
  float bn[2 * kD];  // alpha | shift
  double tot[2 * kD];
  float hd[kHeadFloats];  // the output head (gine_layer_head)
  int barrier_failed;  // this workgroup's grid barrier timed out (gine_bnacc.hpp)
};

// ---------------------------------------------------------------------------------------
// WIN: phase A with LDS staging of each tile's neighbour rows (north star: per-destination
// LDS staging of neighbour features).  A PyG batch is block-diagonal and the stations are in
// the locality order, so the in-neighbours of a 32-row tile lie in one short run of rows --
// the tile's window [lo, lo + rows) (gine_graph_plan_layer_windows; cfg2: ~100 rows, at most
// 129, against 352 neighbour reads).  The gather waves stage the window (coalesced, each row
// once), the tile's CSR segment (window byte offset | attribute) and its local rowptr in LDS,
// then sum every destination's messages from LDS in edge order -- the same per-edge rounding
// sequence as gine_mp_fwd, so z is bit-identical.  Tile k+1's staging loads are in flight in
// registers while tile k is summed (one window in LDS).  A dummy row of -inf and a dummy edge
// pointing at it stand in for past-the-degree slots (masked, so any weights give the gather's
// bits).  The rest of the workgroup's LDS: the matrix waves' transposition tiles and BatchNorm
// sums, two tiles of split planes; W1's fragments come straight from memory (no staging
// image) and a1 is read back from memory in phase B (no a1 tiles kept).
// Barriers: two per tile in both roles (G: window staged | S: tile summed and planes written),
// for it = 0 .. nt (the matrix role multiplies tile it - 1).
// ---------------------------------------------------------------------------------------
#ifndef GINE_LW_U  // (experiments)
#define GINE_LW_U 4
#endif
constexpr int kLwU = GINE_LW_U;             // slots per row and group (LDS reads in flight)
constexpr int kLwRowLoads = 9;              // float4 per gather thread: windows <= 144 rows
constexpr int kLwRowsMax = kLwRowLoads * (kThreads - kMatThreads) / kD4;
constexpr int kLwRegion = 73712;            // window | slot table | rowptr (phase B: W2's image)
struct LayerWinLds {
  float tt[4 * 32 * kTLD];                  // transposition tiles | phase B: output tiles
  double sr[2 * 8 * kD];                    // BatchNorm sums     | (output tiles, cont.)
  uint16_t planes[2][3 * kTileRows * kPS];  // z planes of tiles it & 1 | phase B: relu planes
  float4 win[kLwRegion / 16];
  float bn[2 * kD];
  double tot[2 * kD];
  int barrier_failed;
};
static_assert(sizeof(LayerWinLds) <= 160 * 1024, "one workgroup per CU");
static_assert(kD * kLD * 4 <= kLwRegion, "W2's image fits the window region");
// phase B: the output head's weights and valid-target counts behind W2's image
constexpr int kLwHeadOff = kD * kLD;  // floats into the window region
static_assert((kLwHeadOff + kHeadFloats) * 4 <= kLwRegion,
              "the head's weights and counts fit behind W2's image");
static_assert(2 * kTileRows * kLD * 4 <= sizeof(float) * 4 * 32 * kTLD + sizeof(double) * 2 * 8 * kD,
              "phase B's output tiles fit the transposition + statistics region");
// Slots per row of the padded slot table: the in-degree bound rounded up to whole groups.
__host__ __device__ constexpr int lw_slots(int max_in_degree) {
  return (max_in_degree + kLwU - 1) / kLwU * kLwU;
}
__host__ __device__ constexpr int lw_table_off(int win_rows) { return (win_rows + 1) * kRowBytes; }
__host__ __device__ constexpr int lw_rowptr_off(int win_rows, int slots) {
  return lw_table_off(win_rows) + kTileRows * slots * 8;
}
__host__ __device__ constexpr bool lw_fits(int win_rows, int max_in_degree) {
  return win_rows >= 1 && win_rows <= kLwRowsMax && max_in_degree >= 0 &&
         max_in_degree <= GINE_MP_FUSED_MAX_DEGREE &&
         lw_rowptr_off(win_rows, lw_slots(max_in_degree)) + (kTileRows + 1) * 4 <= kLwRegion;
}
static_assert(kTileRows * lw_slots(GINE_MP_FUSED_MAX_DEGREE) <= 2 * (kThreads - kMatThreads),
              "two slot-table entries per gather thread");

// The gather waves' staging of one tile in two dependent levels, each a tile ahead of its
// use, so that nothing waits on a load until the tile that consumes it:
//   level A (tile it + 2): the window (plan), the row pointers of this thread's slot-table
//            entries (entry e = p, p + 512: row e / SP, slot e % SP) and local rowptr word p;
//   level B (tile it + 1): the window rows and the entries' edges, from level A's values.
// Named scalars written out member by member: an array (or an accessor returning references,
// or HIP's float4 union) held across the barriers stays a private-memory object -- scratch
// stores right behind the loads, which serialise the prefetch.
struct LwLevelA {
  int lo, rows, ra0, rb0, ra1, rb1, rpx;
  __device__ __forceinline__ void load(const FusedArgs& A, const int2* win, int T, int p,
                                       int SP, int kG) {
    const int2 w = win[T];
    lo = w.x;
    rows = w.y;
    const int n0 = T * kTileRows;
    const int r0 = min(p / SP, kTileRows - 1), r1 = min((p + kG) / SP, kTileRows - 1);
    ra0 = A.rowptr[min(n0 + r0, A.N)];
    rb0 = A.rowptr[min(n0 + r0 + 1, A.N)];
    ra1 = A.rowptr[min(n0 + r1, A.N)];
    rb1 = A.rowptr[min(n0 + r1 + 1, A.N)];
    rpx = A.rowptr[min(n0 + min(p, kTileRows), A.N)];
  }
};
struct LwStage {
  f4v v0, v1, v2, v3, v4, v5, v6, v7, v8;
  int32_t nb0, nb1;
  float at0, at1;
  int lo, rows, ra0, rb0, ra1, rb1, rpx;
  // window element p + k * 512 (row-major float4 of the window rows): row p / 32 + 16 k,
  // chunk p % 32 -- one base offset, the rows as immediate steps, and a predicate per k (the
  // stores below use the same one)
  __device__ __forceinline__ void load(const FusedArgs& A, const LwLevelA& a, int p, int SP,
                                       int kG) {
    static_assert(kLwRowLoads == 9, "the members below");
    static_assert(kThreads - kMatThreads == 16 * kD4, "16 window rows per load round");
    lo = a.lo;
    rows = a.rows;
    ra0 = a.ra0;
    rb0 = a.rb0;
    ra1 = a.ra1;
    rb1 = a.rb1;
    rpx = a.rpx;
    // the edges first: their indices use level A's values, and a wait for those placed
    // after the window loads would count the window loads too (vmcnt is in issue order)
    const int j0 = p % SP, j1 = (p + kG) % SP;
    if (j0 < rb0 - ra0) {
      nb0 = A.nbr[ra0 + j0];
      at0 = A.attr[ra0 + j0];
    }
    if (j1 < rb1 - ra1) {
      nb1 = A.nbr[ra1 + j1];
      at1 = A.attr[ra1 + j1];
    }
    const char* xb = reinterpret_cast<const char*>(A.x);
    const uint32_t off0 = ((uint32_t)(lo + (p >> 5)) * kD4 + (p & 31)) * 16u;
    const int lim = rows - (p >> 5);
#define LW_LD(K, V) \
  if (16 * (K) < lim) V = *reinterpret_cast<const f4v*>(xb + off0 + (K) * 8192u);
    LW_LD(0, v0) LW_LD(1, v1) LW_LD(2, v2) LW_LD(3, v3) LW_LD(4, v4) LW_LD(5, v5)
    LW_LD(6, v6) LW_LD(7, v7) LW_LD(8, v8)
#undef LW_LD
  }
  // window rows, the padded slot table (past-the-degree slots: the dummy row R, attribute 0)
  // and the local rowptr into LDS
  __device__ __forceinline__ void store(float4* win, int2* tab, int* rpl, int p, int SP, int kG,
                                        int R) const {
    f4v* w = reinterpret_cast<f4v*>(win) + p;
    const int lim = rows - (p >> 5);
#define LW_ST(K, V) if (16 * (K) < lim) w[(K) * 512] = V;
    LW_ST(0, v0) LW_ST(1, v1) LW_ST(2, v2) LW_ST(3, v3) LW_ST(4, v4) LW_ST(5, v5)
    LW_ST(6, v6) LW_ST(7, v7) LW_ST(8, v8)
#undef LW_ST
    const int2 dummy = make_int2(R * (int)kRowBytes, 0);
    if (p < kTileRows * SP)
      tab[p] = p % SP < rb0 - ra0
                   ? make_int2((nb0 - lo) * (int)kRowBytes, __float_as_int(at0))
                   : dummy;
    if (p + kG < kTileRows * SP)
      tab[p + kG] = (p + kG) % SP < rb1 - ra1
                        ? make_int2((nb1 - lo) * (int)kRowBytes, __float_as_int(at1))
                        : dummy;
    if (p <= kTileRows) rpl[p] = rpx;  // (absolute: only differences are read)
  }
};

// Matrix role of the window form.  Barriers: 2 (nt + 1).
__device__ __forceinline__ void matrix_role_win(const FusedArgs& A, LayerWinLds& L,
                                                const TileSeq& ts, int nt) {
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int cq = lane & 7, grp = lane >> 3;
  // W1^T fragments straight from memory: lane (h, c32) reads W1[32 wave + c32][h*64 ..+64)
  float bf[kKS];
  {
    const float4* wr = reinterpret_cast<const float4*>(A.W1 + (size_t)(32 * wave + c32) * kD +
                                                       h * kKS);
#pragma unroll
    for (int q = 0; q < kKS / 4; ++q) {
      const float4 v = wr[q];
      bf[4 * q] = v.x;
      bf[4 * q + 1] = v.y;
      bf[4 * q + 2] = v.z;
      bf[4 * q + 3] = v.w;
    }
  }
  const float4 bias4 = *reinterpret_cast<const float4*>(A.b1 + 32 * wave + 4 * cq);
  BPlanes<kKS> bp;
  bp.from(bf);
  double* sr = L.sr;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    sr[(0 * 8 + grp) * kD + 32 * wave + 4 * cq + k] = 0.0;
    sr[(1 * 8 + grp) * kD + 32 * wave + 4 * cq + k] = 0.0;
  }
  LAYER_MARK(8);
  const float bb[4] = {bias4.x, bias4.y, bias4.z, bias4.w};
  float* tt = &L.tt[wave * 32 * kTLD];
  for (int it = 0; it <= nt; ++it) {
    __syncthreads();  // G_it
    if (it >= 1) {
      const int T = ts.at(it - 1);
      if (it <= 2) LAYER_MARK(19 + it);
      floatx16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
      const uint16_t* pa = L.planes[(it - 1) & 1] + c32 * kPS + h * kKS;
      auto frag = [&](int s8) {
        Bf16x3 a;
        a.h = *reinterpret_cast<const bf16x8_t*>(pa + 8 * s8);
        a.m = *reinterpret_cast<const bf16x8_t*>(pa + kTileRows * kPS + 8 * s8);
        a.l = *reinterpret_cast<const bf16x8_t*>(pa + 2 * kTileRows * kPS + 8 * s8);
        return a;
      };
      Bf16x3 a = frag(0);
#pragma unroll
      for (int s8 = 0; s8 < kKS / 8; ++s8) {
        Bf16x3 an = a;
        if (s8 + 1 < kKS / 8) an = frag(s8 + 1);
        acc = mfma_bf16x3(a, bp.f[s8], acc);
        __builtin_amdgcn_sched_barrier(0);
        a = an;
      }
      if (wave_any_nan(acc)) {  // non-finite operands: the fp32 chain on z read back from HBM
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the gather waves' z stores
        const int64_t zr = min((int64_t)T * kTileRows + c32, (int64_t)A.N - 1);
        acc = mfma_f32_row_mem<kKS>(A.z + zr * kD + h * kKS,
                                    A.W1 + (size_t)(32 * wave + c32) * kD + h * kKS, 1, acc);
      }
#ifdef GINE_LAYER_PROFILE
      if (it <= 2 && acc[0] == 1.2345e-30f) tt[0] = 0.f;
      if (it <= 2) LAYER_MARK(7 + 2 * it);
#endif
#pragma unroll
      for (int r = 0; r < 16; ++r) tt[((r & 3) + 8 * (r >> 2) + 4 * h) * kTLD + c32] = acc[r];
      __builtin_amdgcn_wave_barrier();
      double st1[4], st2[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        st1[k] = sr[(0 * 8 + grp) * kD + 32 * wave + 4 * cq + k];
        st2[k] = sr[(1 * 8 + grp) * kD + 32 * wave + 4 * cq + k];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = grp + 8 * i;
        const int64_t n = (int64_t)T * kTileRows + row;
        const float4 v = *reinterpret_cast<const float4*>(&tt[row * kTLD + 4 * cq]);
        if (n >= A.N) continue;
        const float vv[4] = {v.x, v.y, v.z, v.w};
        float o4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o4[k] = vv[k] + bb[k];
          st1[k] += (double)o4[k];
          st2[k] += (double)o4[k] * (double)o4[k];
        }
        *reinterpret_cast<float4*>(A.a1 + n * kD + 32 * wave + 4 * cq) =
            make_float4(o4[0], o4[1], o4[2], o4[3]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sr[(0 * 8 + grp) * kD + 32 * wave + 4 * cq + k] = st1[k];
        sr[(1 * 8 + grp) * kD + 32 * wave + 4 * cq + k] = st2[k];
      }
      __builtin_amdgcn_wave_barrier();
      if (it <= 2) LAYER_MARK(8 + 2 * it);
    }
    __syncthreads();  // S_it+1
  }
  // per-column partials: the 8 row groups added in fixed order (row-tile GEMM order)
  __builtin_amdgcn_wave_barrier();
  const int which = lane >> 5, cc = 32 * wave + (lane & 31);
  double s = 0.0;
#pragma unroll
  for (int g = 0; g < 8; ++g) s += sr[(which * 8 + g) * kD + cc];
  bnacc_add<false>(A.bnacc, 2 * kD, which * kD + cc, s);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // performed before the barrier arrival
  LAYER_MARK(13);
}

// Gather role of the window form (waves 4-11).  Barriers: 2 (nt + 1).  In the last round
// (it = nt) W2 is loaded and staged into the window region under the matrix role's last
// chain.
// The sums: a half-wave owns rows hw and hw + 16 of the tile, lane t the 16-byte chunk t, and
// walks both rows' SP slots in groups of kLwU (slot entry -> neighbour row, both from LDS).
// Where the edge Linear's weights are finite in every lane (the wave checks) the padded slots
// need no mask: the dummy row is -inf and its attribute 0, so relu(-inf + lin(0)) = +0 and
// acc + 0 = acc (acc is never -0); otherwise each slot is masked by its row's in-degree, as
// the gather does.
template <bool FMA>
__device__ __forceinline__ void lw_sum(f4v (&acc)[kRowsPerHalf], const char* wb, const int2* t0,
                                       const int2* t1, uint32_t qb, int SP, f4v lw, f4v lb,
                                       bool masked, int c0, int c1) {
  for (int j0 = 0; j0 < SP; j0 += kLwU) {
    int2 q0[kLwU], q1[kLwU];
#pragma unroll
    for (int u = 0; u < kLwU; ++u) {
      q0[u] = t0[j0 + u];
      q1[u] = t1[j0 + u];
    }
    f4v r0[kLwU], r1[kLwU];
#pragma unroll
    for (int u = 0; u < kLwU; ++u) {
      r0[u] = *reinterpret_cast<const f4v*>(wb + q0[u].x + qb);
      r1[u] = *reinterpret_cast<const f4v*>(wb + q1[u].x + qb);
    }
    if (masked) {
#pragma unroll
      for (int u = 0; u < kLwU; ++u) {
        edge_acc<FMA>(acc[0], r0[u], __int_as_float(q0[u].y), lw, lb, j0 + u < c0);
        edge_acc<FMA>(acc[1], r1[u], __int_as_float(q1[u].y), lw, lb, j0 + u < c1);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kLwU; ++u) {
        fwd_edge<FMA>(acc[0], r0[u], __int_as_float(q0[u].y), lw, lb);
        fwd_edge<FMA>(acc[1], r1[u], __int_as_float(q1[u].y), lw, lb);
      }
    }
  }
}

template <bool FMA>
__device__ __forceinline__ void gather_role_win(const FusedArgs& A, const LayerArgs& B,
                                                LayerWinLds& L, const TileSeq& ts, int nt) {
  const int p = threadIdx.x - kMatThreads;  // 0 .. 511
  constexpr int kG = kThreads - kMatThreads;
  const int hw = p >> 5, t = p & 31;
  const int N = A.N;
  const uint32_t qb = (uint32_t)t * 16u;
  char* wb = reinterpret_cast<char*>(L.win);
  const int R = B.win_rows, SP = B.win_slots;
  int2* tab = reinterpret_cast<int2*>(wb + lw_table_off(R));
  int* rpl = reinterpret_cast<int*>(wb + lw_rowptr_off(R, SP));
  // (member functions, not lambdas: a lambda called from two sites is not inlined, and what
  // it captures by reference then lives in scratch)
  LwLevelA la;
  LwStage st;
  // the dummy row (-inf), once (nothing else writes there in phase A)
  if (p < kD4) L.win[R * kD4 + p] = make_float4(-__builtin_inff(), -__builtin_inff(),
                                                -__builtin_inff(), -__builtin_inff());
  const f4v lw = ld_f4v(reinterpret_cast<const char*>(A.lin_w), qb);
  const f4v lb = ld_f4v(reinterpret_cast<const char*>(A.lin_b), qb);
  const float ope = 1.0f + A.eps[0];
  static_assert(kLayerTiles == 2, "the tile rounds below are unrolled for two tiles");
  if (nt > 0) la.load(A, B.win, ts.at(0), p, SP, kG);
  if (nt > 0) st.load(A, la, p, SP, kG);
  if (nt > 1) la.load(A, B.win, ts.at(1), p, SP, kG);
  // padded slots unmasked only where every lane's Linear(1, D) weights are finite
  const bool fin = __builtin_isfinite(lw.x) && __builtin_isfinite(lw.y) &&
                   __builtin_isfinite(lw.z) && __builtin_isfinite(lw.w) &&
                   __builtin_isfinite(lb.x) && __builtin_isfinite(lb.y) &&
                   __builtin_isfinite(lb.z) && __builtin_isfinite(lb.w);
  const bool masked = __builtin_amdgcn_readfirstlane(__any(!fin) ? 1 : 0) != 0;
  // the tile rounds unrolled (nt <= kLayerTiles = 2, host-checked): in a rolled loop the
  // stage registers loaded in round it and stored in round it + 1 are copied at the back
  // edge, and each copy waits for its load (s_waitcnt vmcnt(0) right behind the issue)
#pragma unroll
  for (int it = 0; it < kLayerTiles; ++it) {
    if (it >= nt) break;
    const int T = ts.at(it);
    const int lo = st.lo;
    st.store(L.win, tab, rpl, p, SP, kG, R);
    __syncthreads();  // G_it: window, slot table and rowptr of tile it staged
    LAYER_MARK_T(kMatThreads, 22 + it);
    if (it + 1 < nt) st.load(A, la, p, SP, kG);             // level B of tile it + 1
    f4v self[kRowsPerHalf], acc[kRowsPerHalf];
    int c[kRowsPerHalf];
#pragma unroll
    for (int i = 0; i < kRowsPerHalf; ++i) {
      const int r = hw + kHalves * i;
      const int n = T * kTileRows + r;
      c[i] = rpl[r + 1] - rpl[r];
      self[i] = *reinterpret_cast<const f4v*>(wb + (min(n, N - 1) - lo) * (int)kRowBytes + qb);
      acc[i] = f4v_zero();
    }
    if (GINE_FUSED_DBG != 1)
      lw_sum<FMA>(acc, wb, tab + hw * SP, tab + (hw + kHalves) * SP, qb, SP, lw, lb, masked,
                  c[0], c[1]);
#pragma unroll
    for (int i = 0; i < kRowsPerHalf; ++i) {
      const int r = hw + kHalves * i;
      const int64_t n = (int64_t)T * kTileRows + r;
      const f4v zv = add_scaled(acc[i], ope, self[i]);
      uint32_t h0, m0, l0, h1, m1, l1;
      split2(zv.x, zv.y, h0, m0, l0);
      split2(zv.z, zv.w, h1, m1, l1);
      uint16_t* pl = L.planes[it & 1] + r * kPS + 4 * t;
      *reinterpret_cast<uint2*>(pl) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(pl + kTileRows * kPS) = make_uint2(m0, m1);
      *reinterpret_cast<uint2*>(pl + 2 * kTileRows * kPS) = make_uint2(l0, l1);
      if (n < N) *reinterpret_cast<f4v*>(A.z + n * kD + 4 * t) = zv;
    }
    LAYER_MARK_T(kMatThreads, 14 + it);
    __syncthreads();  // S_it+1: tile it summed, its planes written
  }
  // round nt: W2 under the matrix role's last chain, into the (free) window region
  constexpr int kW2Per = kD * kD4 / kG;
  W2Regs<kW2Per> w2r;
  w2r.load(reinterpret_cast<const float4*>(B.W2), p, kG);
  __syncthreads();  // G_nt: every gather wave is done with the last window
  w2r.store(reinterpret_cast<float*>(L.win), p, kG);
  if (p < GINE_COUNT_PARTS)  // the head's valid-target counts (k_mp_fwd_layer)
    reinterpret_cast<uint32_t*>(reinterpret_cast<float*>(L.win) + kLwHeadOff + kHC)[p] = 0;
  __syncthreads();  // S_nt+1
}

// Element e of the head's outputs of 32-row tile T from its raw values in LDS (rt: [32][K],
// written by the epilogue's half-waves): raw stored and PostProcess applied once per element
// after the tile loop (coalesced rows of raw / pred), instead of on the K lanes of every row's
// half-wave inside it.
__device__ __forceinline__ void head_finish(const LayerArgs& B, const float* rt, int T, int N,
                                            int e) {
  const int64_t base = (int64_t)T * kTileRows * B.hk;
  if (base + e < (int64_t)N * B.hk) {
    const float v = rt[e];
    B.hd.raw[base + e] = v;
    B.hd.pred[base + e] = head::post(head::role_of(B.hd.kind, e % B.hk), v);
  }
}

template <bool FMA, int EPI, bool WIN = false>
__global__ __launch_bounds__(kThreads, 1) void k_mp_fwd_layer(FusedArgs A, LayerArgs B) {
  using Lds = std::conditional_t<WIN, LayerWinLds, LayerLds>;
  __shared__ __attribute__((aligned(16))) Lds L;
  const TileSeq ts = tile_seq(A.num_tiles, blockIdx.x, gridDim.x);
  const int nt = ts.count();
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const bool mat = wave < kMatThreads / kWave;
  long long* phw = bnacc_phase(A.bnacc, 2 * kD);
  // written by earlier launches only (workgroup 0 moves them after the barrier)
  const long long ph = phw[0] + 1, consumed = phw[1 + ((ph - 1) & 1)];
  // the output head's weights and valid-target counts (gine_layer_head)
  float* hwl;
  if constexpr (WIN) {
    hwl = reinterpret_cast<float*>(L.win) + kLwHeadOff;  // counts zeroed by gather_role_win
  } else {
    hwl = L.hd;
  }
  uint32_t* const cwl = reinterpret_cast<uint32_t*>(hwl + kHC);
  if constexpr (!WIN)
    if (tid < GINE_COUNT_PARTS) cwl[tid] = 0;  // (phase A's barriers publish it)

  // ---- phase A ----
  LAYER_MARK(0);
  LAYER_RT(16);
  // W2 for the second half: the gather waves load it (coalesced, 8 float4 per thread) once
  // their last tile is gathered, so its latency hides under the matrix role's last chain
  // and statistics, and stage it in LDS when phase A's use of L.f.w is over
  constexpr int kW2Per = kD * kD4 / (kThreads - kMatThreads);
  static_assert(kD * kD4 % (kThreads - kMatThreads) == 0, "W2 in whole float4 per thread");
  // phase B's LDS: W2's image, the relu planes, the output tiles
  float* w2img;
  uint16_t* rp;  // [kLayerTiles][3][kTileRows * kPS]
  float* sOb;    // [2][kTileRows * kLD]
  if constexpr (WIN) {
    w2img = reinterpret_cast<float*>(L.win);
    rp = &L.planes[0][0];
    sOb = L.tt;
    if (mat) {
      matrix_role_win(A, L, ts, nt);
      LAYER_MARK(1);
    } else {
      gather_role_win<FMA>(A, B, L, ts, nt);
    }
    __syncthreads();  // every matrix wave's statistics atomics performed (before the arrival)
    LAYER_MARK(2);
  } else {
    w2img = L.f.w;
    rp = reinterpret_cast<uint16_t*>(L.f.w);
    sOb = &L.f.z[0][0];
    if (mat) {
      matrix_role<true>(A, L.f, ts, nt, &L.a1k[0][0]);
      LAYER_MARK(1);
      __syncthreads();  // phase A's LDS use is over (L.f.w is free)
      LAYER_MARK(2);
    } else {
      // (W2Regs is confined to this branch -- live across the matrix role it would spill --
      // and a struct of scalars: an array held across the barriers went to scratch)
      gather_role<FMA, false, true>(A, L.f, ts, nt);
      W2Regs<kW2Per> w2r;
      w2r.load(reinterpret_cast<const float4*>(B.W2), tid - kMatThreads, kThreads - kMatThreads);
      __syncthreads();  // gather_role's last barrier (the matrix role multiplies the last tile)
      __syncthreads();  // phase A's LDS use is over (L.f.w is free)
      w2r.store(L.f.w, tid - kMatThreads, kThreads - kMatThreads);
    }
  }

  const int lane = tid % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = 32 * wave + c32;  // (matrix waves)
  // epilogue items of the gather waves: rows p / 32 and p / 32 + 16 of a tile, column chunk
  // p % 32 (p = tid - 256 < 512)
  const int p = tid - kMatThreads;
  const int eq = p & 31, er = p >> 5;
  // the output head (gine_layer_head): its weights staged in LDS, and the loss's valid-target
  // partial counts (count_valid_parts' parts: part q counts [q * chunk, min(N, q * chunk +
  // chunk)), integer, any order) summed into L.cw -- gather waves, in the shadow of the grid
  // barrier's wait
  if (!mat && B.hk) {
    if (p < B.hk * kD4)
      *reinterpret_cast<float4*>(&hwl[4 * p]) =
          *reinterpret_cast<const float4*>(B.hd.weight + 4 * p);
    else if (p < B.hk * kD4 + B.hk)
      hwl[kHB + p - B.hk * kD4] = B.hd.bias[p - B.hk * kD4];
    if (B.hd.count_parts) {
      const int64_t chunk = ((int64_t)A.N + GINE_COUNT_PARTS - 1) / GINE_COUNT_PARTS;
      for (int q = blockIdx.x; q < GINE_COUNT_PARTS; q += gridDim.x) {
        const int64_t lo = (int64_t)q * chunk, hi = min(lo + chunk, (int64_t)A.N);
        uint32_t c = 0;
        for (int64_t i = lo + p; i < hi; i += kThreads - kMatThreads)
          c += B.hd.y_target[i] == B.hd.y_target[i];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
        if (lane == 0) atomicAdd(&cwl[q], c);
      }
    }
  }
  LAYER_MARK(3);
  LAYER_RT(17);
  // the workgroup arrives as soon as phase A is done; W2's fragments are read after the
  // barrier, beside the BatchNorm totals
  // (a barrier that failed earlier on this accumulator, before the host's reset, counts too:
  // bnacc_poisoned is sticky)
  if (tid == 0)
    L.barrier_failed = grid_barrier(bnacc_barrier(A.bnacc, 2 * kD), gridDim.x) &&
                               !bnacc_poisoned<true>(A.bnacc, 2 * kD)
                           ? 0
                           : 1;
  __syncthreads();  // (also: W2 staged by the gather waves)
  LAYER_MARK(4);
  LAYER_RT(18);
  // a timed-out barrier (the grid was not co-resident): the totals are incomplete, so this
  // workgroup's statistics and outputs are NaN and the running statistics stay as they were;
  // the failure word tells the host
  const bool failed = L.barrier_failed != 0;
  // WIN: a1 (kept in memory, not in LDS) for the relu pass, in flight under the BatchNorm
  // finish: element e = tid + kThreads * j of the workgroup's tiles (row-major float4)
  constexpr int kA1Per = (kLayerTiles * kTileRows * kD4 + kThreads - 1) / kThreads;
  float4 a1v[WIN ? kA1Per : 1];
  if constexpr (WIN) {
#pragma unroll
    for (int j = 0; j < kA1Per; ++j) {
      const int e = tid + kThreads * j;
      const int k = e / (kTileRows * kD4), r = (e / kD4) % kTileRows, q4 = e % kD4;
      int64_t n = (int64_t)ts.at(k < nt ? k : 0) * kTileRows + r;
      n = n < A.N ? n : A.N - 1;
      a1v[j] = e < nt * kTileRows * kD4
                   ? *reinterpret_cast<const float4*>(A.a1 + n * kD + 4 * q4)
                   : f4_zero();
    }
  }
  // the gather waves' epilogue operands, in flight under the BatchNorm finish
  float4 xres[kLayerTiles][2];
  float4 bias2 = f4_zero();
  if (!mat) {
    bias2 = *reinterpret_cast<const float4*>(B.b2 + 4 * eq);
#pragma unroll
    for (int k = 0; k < kLayerTiles; ++k)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        xres[k][i] = f4_zero();
        if constexpr (EPI == EPI_OUT_RES) {
          int64_t n = (int64_t)ts.at(k < nt ? k : 0) * kTileRows + er + 16 * i;
          n = n < A.N ? n : A.N - 1;
          xres[k][i] = *reinterpret_cast<const float4*>(A.x + n * kD + 4 * eq);
        }
      }
  }

  // the loss's valid-target partial counts, summed above by the gather waves
  if (!mat && B.hk && B.hd.count_parts) {
    const int q = (int)blockIdx.x + p * (int)gridDim.x;
    if (q < GINE_COUNT_PARTS) B.hd.count_parts[q] = cwl[q];
  }

  // ---- phase B: BatchNorm finish (the arithmetic of k_fwd2_bnacc's prologue) on the
  // gather waves, W2's fragments on the matrix waves ----
  float bf[kKS];
  BPlanes<kKS> bp;
  if (mat) {
    const float* wr = &w2img[col * kLD + h * kKS];
#pragma unroll
    for (int q = 0; q < kKS / 4; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(&wr[4 * q]);
      bf[4 * q] = v.x;
      bf[4 * q + 1] = v.y;
      bf[4 * q + 2] = v.z;
      bf[4 * q + 3] = v.w;
    }
    if constexpr (GINE_GEMM_BF16X3) bp.from(bf);
  } else if (p < 2 * kD) {
    const double t = bnacc_total<true>(A.bnacc, 2 * kD, p, blockIdx.x == 0, ph, consumed);
    L.tot[p] = failed ? __builtin_nan("") : t;
  }
  __syncthreads();
  if (!mat && p < kD) {
    BnFwdParams q = B.q;
    if (failed) q.update_running = 0;
    bn_finish_channel(q, kD, p, L.tot[p], L.tot[kD + p], blockIdx.x == 0, &L.bn[p],
                      &L.bn[kD + p]);
  }
  if (blockIdx.x == 0 && tid == 0) {
    if (B.q.update_running && B.q.nbt != nullptr && !failed) B.q.nbt[0] = B.q.nbt[0] + 1;
    phw[0] = ph;
    phw[1 + (ph & 1)] = ph;  // bnacc_mark_consumed
  }
  __syncthreads();
  LAYER_MARK(5);
  // r = relu(bn(a1)) as split-bf16 planes (hi | mid | lo, gine_bf16x3.hpp split2) in the
  // w region (free since W2's fragments were read): split once here by all 12 waves, the
  // matrix waves' chains then only read them (a wave's in-loop split adds to its MFMA chain:
  // 3,081 against 2,046 shader ticks per 32x32 block, tools/chain_micro.py).  a1k keeps a1
  // for the rare fp32 redo.  Rows past N are zero (the row GEMM stages them as zero).
#pragma unroll
  for (int j = 0; j < (WIN ? kA1Per : (kLayerTiles * kTileRows * kD4 + kThreads - 1) / kThreads);
       ++j) {
    const int e = tid + kThreads * j;
    if (e >= nt * kTileRows * kD4) break;
    const int k = e / (kTileRows * kD4), r = (e / kD4) % kTileRows, q4 = e % kD4;
    float4 v;
    if constexpr (WIN) v = a1v[j];
    else v = *reinterpret_cast<const float4*>(&L.a1k[k][r * kLD + 4 * q4]);
    const float4 al = *reinterpret_cast<const float4*>(&L.bn[4 * q4]);
    const float4 sh = *reinterpret_cast<const float4*>(&L.bn[kD + 4 * q4]);
    v = make_float4(relu_nan(bn_apply(v.x, al.x, sh.x)), relu_nan(bn_apply(v.y, al.y, sh.y)),
                    relu_nan(bn_apply(v.z, al.z, sh.z)), relu_nan(bn_apply(v.w, al.w, sh.w)));
    if ((int64_t)ts.at(k) * kTileRows + r >= A.N) v = f4_zero();
    uint32_t h0, m0, l0, h1, m1, l1;
    split2(v.x, v.y, h0, m0, l0);
    split2(v.z, v.w, h1, m1, l1);
    uint16_t* pl = rp + k * 3 * kTileRows * kPS + r * kPS + 4 * q4;
    *reinterpret_cast<uint2*>(pl) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(pl + kTileRows * kPS) = make_uint2(m0, m1);
    *reinterpret_cast<uint2*>(pl + 2 * kTileRows * kPS) = make_uint2(l0, l1);
  }
  __syncthreads();
  LAYER_MARK(6);
  for (int k = 0; k < nt; ++k) {
    float* sO = sOb + (k & 1) * kTileRows * kLD;
    if (mat) {  // Linear2 chain of tile k (the row GEMM's split-bf16 chain and k order)
      floatx16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
      if constexpr (GINE_GEMM_BF16X3) {
        const uint16_t* pa = rp + k * 3 * kTileRows * kPS + c32 * kPS + h * kKS;
#pragma unroll
        for (int s8 = 0; s8 < kKS / 8; ++s8) {
          Bf16x3 a;
          a.h = *reinterpret_cast<const bf16x8_t*>(pa + 8 * s8);
          a.m = *reinterpret_cast<const bf16x8_t*>(pa + kTileRows * kPS + 8 * s8);
          a.l = *reinterpret_cast<const bf16x8_t*>(pa + 2 * kTileRows * kPS + 8 * s8);
          acc = mfma_bf16x3(a, bp.f[s8], acc);
        }
        if (wave_any_nan(acc)) {  // the fp32 chain, r recomputed from a1 (mfma_f32_row_mem's order)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[i] = 0.f;
          const bool live = (int64_t)ts.at(k) * kTileRows + c32 < A.N;
          const float* arow;
          if constexpr (WIN)
            arow = A.a1 + min((int64_t)ts.at(k) * kTileRows + c32, (int64_t)A.N - 1) * kD +
                   h * kKS;
          else
            arow = &L.a1k[k][c32 * kLD + h * kKS];
          const float* wp = B.W2 + (size_t)col * kD + h * kKS;
          auto rv = [&](int kk) -> float {
            const int c = h * kKS + kk;
            return live ? relu_nan(bn_apply(arow[kk], L.bn[c], L.bn[kD + c])) : 0.f;
          };
#pragma unroll 1
          for (int q = 0; q < kKS / 4; ++q) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(rv(4 * q), wp[4 * q], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(rv(4 * q + 1), wp[4 * q + 1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(rv(4 * q + 2), wp[4 * q + 2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(rv(4 * q + 3), wp[4 * q + 3], acc, 0, 0, 0);
          }
        }
      } else {
        static_assert(GINE_GEMM_BF16X3, "the layer forward's second half reads split planes");
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sO[((r & 3) + 8 * (r >> 2) + 4 * h) * kLD + col] = acc[r];
    }
    __syncthreads();  // output tile k in LDS
    if (!mat) {  // epilogue of tile k (beside the matrix waves' next chain)
      const int T = ts.at(k);
      const float bb[4] = {bias2.x, bias2.y, bias2.z, bias2.w};
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = er + 16 * i;
        const int64_t n = (int64_t)T * kTileRows + r;
        const float4 v = *reinterpret_cast<const float4*>(&sO[r * kLD + 4 * eq]);
        if (n >= A.N) continue;
        const float vv[4] = {v.x, v.y, v.z, v.w};
        const int64_t off = n * kD + 4 * eq;
        float o4[4];
        if constexpr (EPI == EPI_OUT_RES) {
          const float4 xv = k == 0 ? xres[0][i] : xres[1][i];
          const float xr[4] = {xv.x, xv.y, xv.z, xv.w};
          unsigned char mk[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float o = vv[c] + bb[c];
            o4[c] = xr[c] + relu_nan(o);
            mk[c] = (o > 0.f) ? 1 : 0;
          }
          *reinterpret_cast<uchar4*>(B.mask + off) = make_uchar4(mk[0], mk[1], mk[2], mk[3]);
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float o = vv[c] + bb[c];
            o4[c] = (EPI == EPI_OUT_RELU) ? relu_nan(o) : o;
          }
        }
        *reinterpret_cast<float4*>(B.y + off) = make_float4(o4[0], o4[1], o4[2], o4[3]);
        if (B.hk) {  // the head on this row: k_head_fwd's fma order and reduction
          // (outputs 0-3 always -- independent chains; outputs past K are never stored --
          // and output 4 when K = 5); raw into the LDS tile, finished after the tile loop
          float a[4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const float4 wk = *reinterpret_cast<const float4*>(&hwl[kk * kD + 4 * eq]);
            a[kk] = 0.f;
            a[kk] = __builtin_fmaf(o4[0], wk.x, a[kk]);
            a[kk] = __builtin_fmaf(o4[1], wk.y, a[kk]);
            a[kk] = __builtin_fmaf(o4[2], wk.z, a[kk]);
            a[kk] = __builtin_fmaf(o4[3], wk.w, a[kk]);
          }
          const float d = head::sum4_32(a[0], a[1], a[2], a[3]);
          const int o = (eq >> 3) & 3;
          float* rt = hwl + kHR + k * kHRTile + r * B.hk;
          if ((eq & 7) == 0 && o < B.hk) rt[o] = d + hwl[kHB + o];
          if (B.hk == 5) {
            const float4 wk = *reinterpret_cast<const float4*>(&hwl[4 * kD + 4 * eq]);
            float a4 = 0.f;
            a4 = __builtin_fmaf(o4[0], wk.x, a4);
            a4 = __builtin_fmaf(o4[1], wk.y, a4);
            a4 = __builtin_fmaf(o4[2], wk.z, a4);
            a4 = __builtin_fmaf(o4[3], wk.w, a4);
            a4 = head::sum_32(a4);
            if (eq == 1) rt[4] = a4 + hwl[kHB + 4];
          }
        }
      }
    }
  }
  if (B.hk) {  // the head's PostProcess and stores of both tiles (nt <= kLayerTiles = 2)
    __syncthreads();
    static_assert(kLayerTiles * kHRTile <= kThreads - kMatThreads, "one element per thread");
    const int kt = p / (kTileRows * B.hk), e = p - kt * kTileRows * B.hk;
    if (!mat && kt < nt) head_finish(B, hwl + kHR + kt * kHRTile, ts.at(kt), A.N, e);
  }
  LAYER_MARK(7);
  LAYER_RT(19);
}

}  // namespace
}  // namespace gine

using namespace gine;

namespace {
int mp_fwd_mlp1(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                const float* in_attr, const float* lin_w, const float* lin_b, const float* eps,
                const float* w1, const float* b1, float* z, float* a1, double* partials,
                int64_t* bn_acc, int64_t num_nodes, int32_t channels, int32_t max_in_degree,
                int32_t flags, void* stream) {
  if (channels != kD) return GINE_ERR_DIM;
  if ((flags & ~GINE_MP_LIN_MULADD) != 0) return GINE_ERR_INVALID;
  if (max_in_degree < 0 || max_in_degree > GINE_MP_FUSED_MAX_DEGREE) return GINE_ERR_INVALID;
  if (num_nodes <= 0 || !x || !in_rowptr || !in_src || !in_attr || !lin_w || !lin_b || !eps ||
      !w1 || !b1 || !z || !a1 || (!partials && !bn_acc))
    return GINE_ERR_INVALID;
  if (num_nodes * channels * 4 >= (int64_t(1) << 32)) return GINE_ERR_TOO_LARGE;
  int32_t grid = 0;
  const int st = gine_mlp_num_partials(num_nodes, channels, &grid);
  if (st != GINE_OK) return st;
  const int tiles = (int)ceil_div(num_nodes, kTileRows);
  hipStream_t s = as_stream(stream);
  const FusedArgs A{x,  in_rowptr, in_src, in_attr,  lin_w, lin_b,
                    eps, w1,       b1,     z,        a1,    partials,
                    reinterpret_cast<long long*>(bn_acc), (int)num_nodes, tiles};
  if (flags & GINE_MP_LIN_MULADD)
    hipLaunchKernelGGL(k_mp_fwd_mlp1<false>, dim3((unsigned)grid), dim3(kThreads), 0, s, A);
  else
    hipLaunchKernelGGL(k_mp_fwd_mlp1<true>, dim3((unsigned)grid), dim3(kThreads), 0, s, A);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
}  // namespace

namespace {
// Workgroups of k_mp_fwd_layer the device holds at once (one per CU at most): its grid
// barrier needs every workgroup resident.  Queried once per device.
int layer_capacity() {
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
    const void* ks[] = {(const void*)k_mp_fwd_layer<true, EPI_OUT>,
                        (const void*)k_mp_fwd_layer<true, EPI_OUT_RELU>,
                        (const void*)k_mp_fwd_layer<true, EPI_OUT_RES>,
                        (const void*)k_mp_fwd_layer<false, EPI_OUT>,
                        (const void*)k_mp_fwd_layer<false, EPI_OUT_RELU>,
                        (const void*)k_mp_fwd_layer<false, EPI_OUT_RES>,
                        (const void*)k_mp_fwd_layer<true, EPI_OUT, true>,
                        (const void*)k_mp_fwd_layer<true, EPI_OUT_RELU, true>,
                        (const void*)k_mp_fwd_layer<true, EPI_OUT_RES, true>,
                        (const void*)k_mp_fwd_layer<false, EPI_OUT, true>,
                        (const void*)k_mp_fwd_layer<false, EPI_OUT_RELU, true>,
                        (const void*)k_mp_fwd_layer<false, EPI_OUT_RES, true>};
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

// Largest number of tiles one workgroup of the fused grid walks (tile_seq).
int max_tiles_per_block(int tiles, int grid) {
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

// gine_testing_layer_extra_workgroups: workgroups added to k_mp_fwd_layer's grid (0 in
// production) -- a grid the device cannot hold at once, for the test of the grid barrier's
// failure path
std::atomic<int> g_layer_extra{0};

bool layer_ok(int64_t num_nodes, int32_t channels, int32_t max_in_degree) {
  if (channels != kD || num_nodes <= 0 || max_in_degree < 0 ||
      max_in_degree > GINE_MP_FUSED_MAX_DEGREE || num_nodes * channels * 4 >= (int64_t(1) << 32))
    return false;
  int32_t grid = 0;
  if (gine_mlp_num_partials(num_nodes, channels, &grid) != GINE_OK) return false;
  const int tiles = (int)ceil_div(num_nodes, kTileRows);
  return grid <= layer_capacity() && max_tiles_per_block(tiles, grid) <= kLayerTiles;
}
}  // namespace

extern "C" int gine_testing_layer_extra_workgroups(int32_t extra) {
  if (extra < 0 || extra > 4096) return GINE_ERR_INVALID;
  g_layer_extra.store(extra);
  return GINE_OK;
}

extern "C" int gine_mp_fwd_layer_ok(int64_t num_nodes, int32_t channels, int32_t max_in_degree,
                                    int32_t* ok) {
  if (!ok) return GINE_ERR_INVALID;
  *ok = layer_ok(num_nodes, channels, max_in_degree) ? 1 : 0;
  return GINE_OK;
}

// One wave per 32-row tile: the window [lo, lo + rows) covering the tile's own rows and
// every in-neighbour, and the maxima (window rows, in-edges) over the tiles.
__global__ __launch_bounds__(64) void k_plan_layer_windows(const int32_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ src,
                                                           int N, int tiles, int2* win,
                                                           int32_t* maxima) {
  const int T = blockIdx.x;
  if (T >= tiles) return;
  const int n0 = T * kTileRows, n1 = min(n0 + kTileRows, N);
  const int e0 = rowptr[n0], e1 = rowptr[n1];
  int lo = n0, hi = n1 - 1;
  for (int e = e0 + (int)threadIdx.x; e < e1; e += 64) {
    const int s = src[e];
    lo = min(lo, s);
    hi = max(hi, s);
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o, 64));
    hi = max(hi, __shfl_xor(hi, o, 64));
  }
  if (threadIdx.x == 0) {
    win[T] = make_int2(lo, hi - lo + 1);
    atomicMax(&maxima[0], hi - lo + 1);
    atomicMax(&maxima[1], e1 - e0);
  }
}

extern "C" int gine_graph_plan_layer_windows(const int32_t* in_rowptr, const int32_t* in_src,
                                             int64_t num_nodes, int32_t* tile_windows,
                                             int32_t* maxima, void* stream) {
  if (num_nodes <= 0 || num_nodes >= (int64_t(1) << 31) || !in_rowptr || !in_src ||
      !tile_windows || !maxima)
    return GINE_ERR_INVALID;
  const int tiles = (int)ceil_div(num_nodes, kTileRows);
  hipStream_t s = as_stream(stream);
  GINE_RETURN_IF_HIP(hipMemsetAsync(maxima, 0, 2 * sizeof(int32_t), s));
  hipLaunchKernelGGL(k_plan_layer_windows, dim3((unsigned)tiles), dim3(64), 0, s, in_rowptr,
                     in_src, (int)num_nodes, tiles, reinterpret_cast<int2*>(tile_windows),
                     maxima);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_mp_fwd_layer_windows_fit(int32_t window_rows, int32_t max_in_degree,
                                             int32_t* ok) {
  if (!ok) return GINE_ERR_INVALID;
  *ok = lw_fits(window_rows, max_in_degree) ? 1 : 0;
  return GINE_OK;
}

extern "C" int gine_mp_fwd_layer(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                                 const float* in_attr, const float* lin_w, const float* lin_b,
                                 const float* eps, const float* w1, const float* b1, float* z,
                                 float* a1, int64_t* bn_acc, const float* gamma,
                                 const float* beta, float* running_mean, float* running_var,
                                 int64_t* num_batches_tracked, float* bn_save, float momentum,
                                 float bn_eps, int32_t update_running, const float* w2,
                                 const float* b2, float* y, uint8_t* mask, int64_t num_nodes,
                                 int32_t channels, int32_t max_in_degree, int32_t flags,
                                 int32_t epilogue, const int32_t* tile_windows,
                                 int32_t window_rows, const gine_layer_head* head,
                                 void* stream) {
  if (channels != kD) return GINE_ERR_DIM;
  if ((flags & ~GINE_MP_LIN_MULADD) != 0) return GINE_ERR_INVALID;
  if (!x || !in_rowptr || !in_src || !in_attr || !lin_w || !lin_b || !eps || !w1 || !b1 || !z ||
      !a1 || !bn_acc || !bn_save || !w2 || !b2 || !y)
    return GINE_ERR_INVALID;
  if (!(momentum >= 0.f)) return GINE_ERR_INVALID;
  if (update_running && (!running_mean || !running_var)) return GINE_ERR_INVALID;
  if (epilogue < GINE_EPI_NONE || epilogue > GINE_EPI_RESIDUAL_RELU) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && !mask) return GINE_ERR_INVALID;
  if (!layer_ok(num_nodes, channels, max_in_degree)) return GINE_ERR_INVALID;
  int hk = 0;
  if (head) {
    switch (head->kind) {
      case GINE_LOSS_NORMAL: hk = 2; break;
      case GINE_LOSS_MIXED_NORMAL: hk = 3; break;
      case GINE_LOSS_MIXED: hk = 4; break;
      case GINE_LOSS_MIXED_U: hk = 5; break;
      default: return GINE_ERR_INVALID;
    }
    if (!head->weight || !head->bias || !head->raw || !head->pred ||
        (head->count_parts && !head->y_target))
      return GINE_ERR_INVALID;
  }
  int32_t grid = 0;
  const int st = gine_mlp_num_partials(num_nodes, channels, &grid);
  if (st != GINE_OK) return st;
  grid += g_layer_extra.load();
  const int tiles = (int)ceil_div(num_nodes, kTileRows);
  hipStream_t s = as_stream(stream);
  const FusedArgs A{x,  in_rowptr, in_src, in_attr, lin_w, lin_b,
                    eps, w1,       b1,     z,       a1,    nullptr,
                    reinterpret_cast<long long*>(bn_acc), (int)num_nodes, tiles};
  const bool win = tile_windows != nullptr;
  if (win && !lw_fits(window_rows, max_in_degree)) return GINE_ERR_INVALID;
  const LayerArgs B{w2, b2, y, mask,
                    BnFwdParams{gamma, beta, running_mean, running_var, num_batches_tracked,
                                bn_save, num_nodes, momentum, bn_eps, update_running},
                    reinterpret_cast<const int2*>(tile_windows), window_rows,
                    lw_slots(max_in_degree), head ? *head : gine_layer_head{}, hk};
  const bool fma = !(flags & GINE_MP_LIN_MULADD);
#define LAYER_LAUNCH(F_, E_)                                                                   \
  do {                                                                                         \
    if (win)                                                                                   \
      hipLaunchKernelGGL((k_mp_fwd_layer<F_, E_, true>), dim3((unsigned)grid), dim3(kThreads), \
                         0, s, A, B);                                                          \
    else                                                                                       \
      hipLaunchKernelGGL((k_mp_fwd_layer<F_, E_>), dim3((unsigned)grid), dim3(kThreads), 0, s, \
                         A, B);                                                                \
  } while (0)
  switch (epilogue) {
    case GINE_EPI_NONE:
      if (fma) LAYER_LAUNCH(true, EPI_OUT); else LAYER_LAUNCH(false, EPI_OUT);
      break;
    case GINE_EPI_RELU:
      if (fma) LAYER_LAUNCH(true, EPI_OUT_RELU); else LAYER_LAUNCH(false, EPI_OUT_RELU);
      break;
    default:
      if (fma) LAYER_LAUNCH(true, EPI_OUT_RES); else LAYER_LAUNCH(false, EPI_OUT_RES);
  }
#undef LAYER_LAUNCH
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_mp_fwd_mlp1(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                                const float* in_attr, const float* lin_w, const float* lin_b,
                                const float* eps, const float* w1, const float* b1, float* z,
                                float* a1, double* partials, int64_t num_nodes,
                                int32_t channels, int32_t max_in_degree, int32_t flags,
                                void* stream) {
  if (!partials) return GINE_ERR_INVALID;
  return mp_fwd_mlp1(x, in_rowptr, in_src, in_attr, lin_w, lin_b, eps, w1, b1, z, a1, partials,
                     nullptr, num_nodes, channels, max_in_degree, flags, stream);
}

extern "C" int gine_mp_fwd_mlp1_acc(const float* x, const int32_t* in_rowptr,
                                    const int32_t* in_src, const float* in_attr,
                                    const float* lin_w, const float* lin_b, const float* eps,
                                    const float* w1, const float* b1, float* z, float* a1,
                                    double* partials, int64_t* bn_acc, int64_t num_nodes,
                                    int32_t channels, int32_t max_in_degree, int32_t flags,
                                    void* stream) {
  if (!bn_acc) return GINE_ERR_INVALID;
  return mp_fwd_mlp1(x, in_rowptr, in_src, in_attr, lin_w, lin_b, eps, w1, b1, z, a1, partials,
                     bn_acc, num_nodes, channels, max_in_degree, flags, stream);
}

#ifdef GINE_LAYER_PROFILE
extern "C" int gine_debug_layer_prof(long long* out) {  // [1024][24] host buffer
  GINE_RETURN_IF_HIP(hipDeviceSynchronize());
  GINE_RETURN_IF_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_layer_prof), sizeof(g_layer_prof)));
  return GINE_OK;
}
#endif
