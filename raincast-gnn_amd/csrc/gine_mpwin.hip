// Window-staged GINEConv message passing: neighbour feature rows gathered from LDS.
//
// Same arithmetic as gine_mp.hip (PyG GINEConv.message + SumAggregation, models/gnn.py:41,44;
// bit-identical forward z and backward dx), different data movement.  A PyG batch is a
// block-diagonal union of station graphs (Batch.from_data_list), so the in-neighbours of a
// run of consecutive destination nodes all lie in one short run of source rows -- the
// node's own graph.  gine_graph_plan_windows cuts the destinations into tiles whose source
// window [lo, lo + rows) fits in LDS; a workgroup then owns (tile, column slice):
//   1. stages the window's CS-channel slice of x (rows x CS x 4 bytes) and the tile's edge
//      list (source offset in the window + attribute) in LDS with coalesced loads,
//   2. walks the tile's destinations, Q = CS/4 lanes per destination (one float4 each),
//      reading every neighbour row from LDS in the original edge order.
// The per-edge gather of 512-byte rows from L2/MALL (11 neighbours per destination) becomes
// one streaming read of each window slice per tile: HBM/L2 bytes per layer fall from
// E*D*4 gathered to about (tiles per window) * N*D*4 staged.
#include "gine_common.hpp"
#include "gine_edge.hpp"
#include "gine_slab.hpp"
#include "gine_wgrad.hpp"
#include "gine_mlpsrc.hpp"
#include "gine_reduce.hpp"

#include <algorithm>
#include <climits>
#include <vector>

namespace gine {
namespace {

constexpr int kWinThreads = 512;
constexpr int kWinWaves = kWinThreads / kWave;
constexpr int kWinMaxSlices = 8;    // column slices per tile (= finalize columns per block)
#ifndef GINE_WIN_UNROLL  // tuning experiments
#define GINE_WIN_UNROLL 6
#endif
#ifndef GINE_WIN_ROW_BYTES
#define GINE_WIN_ROW_BYTES (64 * 1024)
#endif
constexpr int kWinUnroll = GINE_WIN_UNROLL;  // neighbour rows in flight per lane (LDS reads)
constexpr int kWinTileNodes = 128;  // planner cap on nodes per tile
constexpr int kWinRowBytes = GINE_WIN_ROW_BYTES;
// every thread's share of a tile's global loads, issued in one batch (bounds by construction:
// window slice <= kWinRowBytes, tile edges <= kWinEdgeLoads * kWinThreads)
constexpr int kWinRowLoads = kWinRowBytes / 16 / kWinThreads;  // float4 per thread
constexpr int kWinEdgeLoads = 4;

#ifdef GINE_WIN_PROFILE
// Debug build only (make winprof): s_memtime at the phase boundaries of the window backward,
// per workgroup: [block][8] (entry, loads issued, staged, edges done, reduced, end).
__device__ long long g_win_prof[4096][8];
#define WIN_MARK(i)                                                                   \
  do {                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                                        \
      g_win_prof[blockIdx.x][i] = (long long)__builtin_amdgcn_s_memtime();           \
  } while (0)
#else
#define WIN_MARK(i) do {} while (0)
#endif

struct WinPlan {
  const int32_t* tile_begin;  // [T + 1]
  const int32_t* win_lo;      // [T]
  const int32_t* win_rows;    // [T]
  int max_rows, max_edges, max_nodes;
  const int16_t* slot;        // [N] or null: tile-local node at each work position
  const int32_t* edge_begin;  // [T + 1] or null: rowptr at the tile starts
};

// Dynamic LDS: window [max_rows][Q] float4 | nbr [max_edges] | attr [max_edges] | rp [nodes+1]
__host__ __device__ inline size_t win_lds_bytes(int cs, int max_rows, int max_edges,
                                                int max_nodes) {
  return (size_t)max_rows * cs * 4 + (size_t)max_edges * 8 + (size_t)(max_nodes + 1) * 4;
}

struct WinLds {
  float4* win;
  int32_t* nbr;  // neighbour's byte offset in the window (row * Q * 16)
  float* attr;
  int32_t* rp;
  __device__ WinLds(float4* base, const WinPlan& p, int Q) {
    win = base;
    nbr = reinterpret_cast<int32_t*>(base + (size_t)p.max_rows * Q);
    attr = reinterpret_cast<float*>(nbr + p.max_edges);
    rp = reinterpret_cast<int32_t*>(attr + p.max_edges);
  }
};

// One tile's staging: every global load of the window slice, the CSR segment and the row
// pointers is issued before the first LDS store, so the tile pays one memory latency.
// The tile's global loads, held in registers until stage_store: window rows, the edge list
// (from e0 / ne: the plan's edge offsets, or rowptr) and the local rowptr.
struct StageRegs {
  float4 v[kWinRowLoads];
  int32_t nb[kWinEdgeLoads];
  float at[kWinEdgeLoads];
  int rp, e0, ne;
};
template <int Q>
__device__ __forceinline__ void stage_load(StageRegs& r, const float4* __restrict__ tab4, int D4,
                                           int col4, const int32_t* __restrict__ rowptr,
                                           const int32_t* __restrict__ nbr,
                                           const float* __restrict__ attr, int n0, int nodes,
                                           int lo, int rows, int e0, int ne) {
  const int tid = threadIdx.x;
  const int n = rows * Q;
#pragma unroll
  for (int k = 0; k < kWinRowLoads; ++k) {
    const int i = min(tid + k * kWinThreads, max(n - 1, 0));
    r.v[k] = n > 0 ? tab4[(int64_t)(lo + i / Q) * D4 + col4 + i % Q] : f4_zero();
  }
  r.rp = rowptr[n0 + min(tid, nodes)];
  r.e0 = e0;
  r.ne = ne;
#pragma unroll
  for (int k = 0; k < kWinEdgeLoads; ++k) {
    const int i = min(tid + k * kWinThreads, max(ne - 1, 0));
    r.nb[k] = ne > 0 ? nbr[e0 + i] : 0;
    r.at[k] = ne > 0 ? attr[e0 + i] : 0.f;
  }
}
template <int Q>
__device__ __forceinline__ void stage_store(const StageRegs& r, int nodes, int lo, int rows,
                                            const WinLds& lds) {
  const int tid = threadIdx.x;
  const int n = rows * Q;
#pragma unroll
  for (int k = 0; k < kWinRowLoads; ++k) {
    const int i = tid + k * kWinThreads;
    if (i < n) lds.win[i] = r.v[k];
  }
  if (tid <= nodes) lds.rp[tid] = r.rp - r.e0;
#pragma unroll
  for (int k = 0; k < kWinEdgeLoads; ++k) {
    const int i = tid + k * kWinThreads;
    if (i < r.ne) {
      lds.nbr[i] = (r.nb[k] - lo) * Q * 16;
      lds.attr[i] = r.at[k];
    }
  }
}
// Stage tile t's window slice, edge list and local rowptr into LDS.  Every global load of
// the tile is issued before the first LDS store, so the tile pays the edge list's
// dependent latency (rowptr -> edges) once.
template <int Q>
__device__ __forceinline__ void stage_tile(const float4* __restrict__ tab4, int D4, int col4,
                                           const int32_t* __restrict__ rowptr,
                                           const int32_t* __restrict__ nbr,
                                           const float* __restrict__ attr, int n0, int nodes,
                                           int lo, int rows, const WinLds& lds) {
  const int e0 = rowptr[n0];
  const int ne = rowptr[n0 + nodes] - e0;
  StageRegs r;
  stage_load<Q>(r, tab4, D4, col4, rowptr, nbr, attr, n0, nodes, lo, rows, e0, ne);
  stage_store<Q>(r, nodes, lo, rows, lds);
}

// ----------------------------------------------------------------------------------------
// Forward: z = sum_{in-edges, edge order} relu(x[src] + lin(a)) + (1 + eps) x
// ----------------------------------------------------------------------------------------
template <int CS, bool FMA>
__global__ __launch_bounds__(kWinThreads, CS == 32 ? 2 : 3) void k_mp_fwd_win(
    const float4* __restrict__ x4, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ nbr, const float* __restrict__ attr,
    const float4* __restrict__ lw4, const float4* __restrict__ lb4,
    const float* __restrict__ eps, float4* __restrict__ z4, WinPlan plan, int D4, int S) {
  constexpr int Q = CS / 4, G = kWinThreads / Q, U = kWinUnroll;
  constexpr int P = (kWinTileNodes + G - 1) / G;  // destination passes per lane group
  extern __shared__ float4 s_dyn[];
  const WinLds lds(s_dyn, plan, Q);
  // consecutive logical blocks (the slices of a tile, then the next tile of the same
  // graph: the same window rows) stay on one XCD
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lb / S, col4 = (lb % S) * Q;
  const int n0 = plan.tile_begin[tile], nodes = plan.tile_begin[tile + 1] - n0;
  const int lo = plan.win_lo[tile];
  const int g = threadIdx.x / Q, t = threadIdx.x % Q;
  // the lane's own rows (x_i for the (1+eps) x_i term) join the staging batch
  const char* xb = reinterpret_cast<const char*>(x4);
  const uint32_t rowb = (uint32_t)D4 * 16u, tb = (uint32_t)(col4 + t) * 16u;
  f4v self[P];
#pragma unroll
  for (int p = 0; p < P; ++p)
    self[p] = ld_f4v(xb, (uint32_t)(n0 + min(g + p * G, nodes - 1)) * rowb + tb);
  const f4v w = ld_f4v(reinterpret_cast<const char*>(lw4), tb);
  const f4v b = ld_f4v(reinterpret_cast<const char*>(lb4), tb);
  const float ope = 1.0f + eps[0];
  stage_tile<Q>(x4, D4, col4, rowptr, nbr, attr, n0, nodes, lo, plan.win_rows[tile], lds);
  __syncthreads();
  const char* wb = reinterpret_cast<const char*>(lds.win) + t * 16;

#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int d = g + p * G;
    if (d >= nodes) break;
    const int eb = lds.rp[d], ee = lds.rp[d + 1];
    f4v acc = f4v_zero();
    int j = eb;
    for (; j + U <= ee; j += U) {
      f4v r[U];
      float a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        r[u] = *reinterpret_cast<const f4v*>(wb + lds.nbr[j + u]);
        a[u] = lds.attr[j + u];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) fwd_edge<FMA>(acc, r[u], a[u], w, b);
    }
    if (j < ee) {
      f4v r[U];
      float a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = min(j + u, ee - 1);
        r[u] = *reinterpret_cast<const f4v*>(wb + lds.nbr[jj]);
        a[u] = lds.attr[jj];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j + u < ee) fwd_edge<FMA>(acc, r[u], a[u], w, b);
    }
    z4[(int64_t)(n0 + d) * D4 + col4 + t] = to_float4(add_scaled(acc, ope, self[p]));
  }
}

// ----------------------------------------------------------------------------------------
// Backward over the out-edge CSR: the window holds dz rows of the tile's destinations.
// partials row `tile` (fp64 [3][D]): columns [slice] of sum dm*a and sum dm, and at
// 2D + slice the slice's sum of dz*x.
// ----------------------------------------------------------------------------------------
// The node-MLP weight-gradient engine (dW1 = da1^T z, dW2 = do^T r of this GINE layer,
// gine_wgrad.hpp with 8 waves) as extra workgroups of the message-passing backward: the
// engine is matrix- and HBM-bound, the window kernel LDS- and VALU-bound, so they share
// the CUs instead of the engine sharing them with the dz GEMM (gine_mlp_bwd1_wgrad).
template <int PDO>
struct WinEngine {
  MlpWgradSrc<PDO> src;
  float* slab;
  int64_t N;
  size_t zstride, cstride;
  int nblocks, tiles, rows_per_chunk;
  int D;  // node-MLP width (64 or 128): the engine's O = I
};
// The engine in this launch runs the split-bf16 chain, as the stand-alone node-MLP engines do
// (kMlpEngX3: the same bits), at two workgroups per CU (128 registers).  Round 4 found this
// build's message-passing half wrong and varying from run to run (even float columns of dx);
// round 5 traced it to the packed-FP32 VALU instructions of the message-passing waves beside
// the engine's v_mfma_f32_32x32x16_bf16 waves (gine_common.hpp __global__):
// every kernel is now compiled without packed FP32, and the split chain here is bit-exact
// run after run (tools/determinism_layer.py --flat, tests/test_gpu_layer.py).  Measured
// 26.5-27.0 -> 24.1-24.2 us per launch at cfg2 (profiles/r05_s05).
#ifndef GINE_WIN_ENG_LDS  // (experiments: a larger floor limits workgroups per CU)
#define GINE_WIN_ENG_LDS 0
#endif
constexpr size_t kWinEngineLdsNeed =
    kMlpEngX3 ? wg_lds_bytes<64>() : sizeof(float) * kWgRows * ((64 + 4) + kWgLdQ);
constexpr size_t kWinEngineLds =
    kWinEngineLdsNeed > GINE_WIN_ENG_LDS ? kWinEngineLdsNeed : GINE_WIN_ENG_LDS;

// GINE_WIN_ENG_OCC (tuning experiments): waves per SIMD the combined launch is compiled
// for (register budget: 4 = two 512-thread workgroups per CU, 128 VGPRs); the plan's LDS
// must allow as many workgroups.
// Cross-lane double sums for the block reduction of the window backward, without the LDS
// round trip of ds_bpermute: DPP within a row of 16 lanes, v_permlane16/32_swap across rows.
// Each returns, in every lane, the same-order sum of the two lanes it pairs (so all lanes
// agree bit for bit).
template <int CTRL>
__device__ __forceinline__ double dpp_mov_d(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf, 0xf,
                                                            false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL,
                                                            0xf, 0xf, false);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// lanes i and i^8 (same row of 16): DPP row_ror:8
__device__ __forceinline__ double sum_x8(double v) { return v + dpp_mov_d<0x128>(v); }
// lanes i and i^1 / i^2: DPP quad_perm [1,0,3,2] / [2,3,0,1]; the two quads of an 8-lane
// half row: DPP row_half_mirror
__device__ __forceinline__ double sum_x1(double v) { return v + dpp_mov_d<0xB1>(v); }
__device__ __forceinline__ double sum_x2(double v) { return v + dpp_mov_d<0x4E>(v); }
__device__ __forceinline__ double sum_x4(double v) { return v + dpp_mov_d<0x141>(v); }
// row pairs (lanes i and i^16) / wave halves (i and i^32): even + odd in every lane
__device__ __forceinline__ double sum_x16(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const auto a = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32),
                                                  false, false);
  const double even = __builtin_bit_cast(double, ((uint64_t)b[0] << 32) | (uint32_t)a[0]);
  const double odd = __builtin_bit_cast(double, ((uint64_t)b[1] << 32) | (uint32_t)a[1]);
  return even + odd;
}
__device__ __forceinline__ double sum_x32(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const auto a = __builtin_amdgcn_permlane32_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32),
                                                  false, false);
  const double low = __builtin_bit_cast(double, ((uint64_t)b[0] << 32) | (uint32_t)a[0]);
  const double high = __builtin_bit_cast(double, ((uint64_t)b[1] << 32) | (uint32_t)a[1]);
  return low + high;
}

#ifndef GINE_WIN_ENG_OCC
#define GINE_WIN_ENG_OCC 4
#endif
template <int CS, bool FMA, bool ENG = false, int PDO = PRO_PLAIN>
__global__ __launch_bounds__(kWinThreads, ENG ? GINE_WIN_ENG_OCC : 2) void k_mp_bwd_win(
    const float4* __restrict__ dz4, const float4* __restrict__ x4,
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ nbr,
    const float* __restrict__ attr, const float4* __restrict__ lw4,
    const float4* __restrict__ lb4, const float* __restrict__ eps,
    const float4* __restrict__ dres4, float4* __restrict__ dx4, double* __restrict__ partials,
    WinPlan plan, int D4, int S, int flags, MlpSlabJob job, WinEngine<PDO> eng) {
  constexpr int Q = CS / 4, G = kWinThreads / Q, U = kWinUnroll;
  constexpr int P = (kWinTileNodes + G - 1) / G;
  extern __shared__ float4 s_dyn[];
  int eb = 0;  // engine workgroups (first: the longest job starts first)
  if constexpr (ENG) {
    static_assert(kWinThreads == 512, "the engine runs 8 waves");
    if ((int)blockIdx.x < eng.nblocks) {
      float* sP = reinterpret_cast<float*>(s_dyn);
      float* sQ = sP + kWgRows * (64 + 4);
      const int e = xcd_remap(blockIdx.x, eng.nblocks);
      wgrad_block<MlpWgradSrc<PDO>, 64, 8, kMlpEngX3>(eng.src, eng.N, eng.D, eng.D,
                                                      e / eng.tiles, e % eng.tiles,
                                                      eng.rows_per_chunk, eng.zstride,
                                                      eng.cstride, eng.slab, sP, sQ);
      return;
    }
    eb = eng.nblocks;
  }
  if ((int)blockIdx.x - eb < job.nblocks) {  // side job: the node-MLP weight-gradient slab
    if (threadIdx.x < 256)
      job.run(blockIdx.x - eb, reinterpret_cast<double(*)[kSlabQuads * 4 + 1]>(s_dyn));
    return;
  }
  WIN_MARK(0);
  const WinLds lds(s_dyn, plan, Q);
  const int lb = xcd_remap(blockIdx.x - eb - job.nblocks, gridDim.x - eb - job.nblocks);
  const int tile = lb / S, slice = lb % S, col4 = slice * Q;
  const int n0 = plan.tile_begin[tile], nodes = plan.tile_begin[tile + 1] - n0;
  const int lo = plan.win_lo[tile];
  const int g = threadIdx.x / Q, t = threadIdx.x % Q;
  const char* xb = reinterpret_cast<const char*>(x4);
  const char* dzb = reinterpret_cast<const char*>(dz4);
  const char* rb = reinterpret_cast<const char*>(dres4 != nullptr ? dres4 : dz4);
  const uint32_t rowb = (uint32_t)D4 * 16u, tb = (uint32_t)(col4 + t) * 16u;
  // The tile's staging loads first (the edge range from the plan: no dependent rowptr read),
  // then the work order, then this thread's own rows: the staging pays about one memory
  // latency after the plan's, and the own rows arrive under the LDS stores and barrier.
  const int e0 = plan.edge_begin != nullptr ? plan.edge_begin[tile] : rowptr[n0];
  const int ne = (plan.edge_begin != nullptr ? plan.edge_begin[tile + 1] : rowptr[n0 + nodes]) - e0;
  StageRegs sr;
  stage_load<Q>(sr, dz4, D4, col4, rowptr, nbr, attr, n0, nodes, lo, plan.win_rows[tile], e0,
                ne);
  // work position g + p*G -> tile-local node (the plan's degree-balanced order, if any)
  int dn[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int d = min(g + p * G, nodes - 1);
    dn[p] = plan.slot != nullptr ? (int)plan.slot[n0 + d] : d;
  }
  stage_store<Q>(sr, nodes, lo, plan.win_rows[tile], lds);
  f4v h[P], gs[P], rs[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const uint32_t off = (uint32_t)(n0 + dn[p]) * rowb + tb;
    h[p] = ld_f4v(xb, off);
    gs[p] = ld_f4v(dzb, off);
    rs[p] = ld_f4v(rb, off);
  }
  const f4v w = ld_f4v(reinterpret_cast<const char*>(lw4), tb);
  const f4v b = ld_f4v(reinterpret_cast<const char*>(lb4), tb);
  const float ope = 1.0f + eps[0];
  const bool add_self = (flags & GINE_MP_BWD_SELF) != 0;
  WIN_MARK(1);
  __syncthreads();
  WIN_MARK(2);
  const char* wb = reinterpret_cast<const char*>(lds.win) + t * 16;

  double pw[4] = {0.0, 0.0, 0.0, 0.0}, pb[4] = {0.0, 0.0, 0.0, 0.0};
  double pe = 0.0;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    if (g + p * G >= nodes) break;
    const int d = dn[p];
    const int eb = lds.rp[d], ee = lds.rp[d + 1];
    f4v acc = f4v_zero(), accw = f4v_zero();
    int j = eb;
    for (; j + U <= ee; j += U) {
      f4v r[U];
      float a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        r[u] = *reinterpret_cast<const f4v*>(wb + lds.nbr[j + u]);
        a[u] = lds.attr[j + u];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) bwd_edge<FMA>(acc, accw, r[u], a[u], h[p], w, b);
    }
    if (j < ee) {
      f4v r[U];
      float a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = min(j + u, ee - 1);
        r[u] = *reinterpret_cast<const f4v*>(wb + lds.nbr[jj]);
        a[u] = lds.attr[jj];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (j + u < ee) bwd_edge<FMA>(acc, accw, r[u], a[u], h[p], w, b);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pb[k] += (double)acc[k];
      pw[k] += (double)accw[k];
    }
    f4v o = add_self ? add_scaled(acc, ope, gs[p]) : acc;
    if (dres4 != nullptr) {
      o.xy = o.xy + rs[p].xy;
      o.zw = o.zw + rs[p].zw;
    }
    dx4[(int64_t)(n0 + d) * D4 + col4 + t] = to_float4(o);
    pe += ((double)gs[p].x * (double)h[p].x + (double)gs[p].y * (double)h[p].y) +
          ((double)gs[p].z * (double)h[p].z + (double)gs[p].w * (double)h[p].w);
  }

#ifdef GINE_WIN_PROFILE
  __syncthreads();
#endif
  WIN_MARK(3);
  // Fixed-order block reduction: the G destination groups of a wave by a butterfly over the
  // lane bits above Q, then the waves in order through LDS (the window is dead by now).
  if constexpr (Q == 8) {  // the 32-channel slice: DPP / permlane swaps, no LDS round trips
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pw[k] = sum_x32(sum_x16(sum_x8(pw[k])));
      pb[k] = sum_x32(sum_x16(sum_x8(pb[k])));
    }
    pe = sum_x4(sum_x2(sum_x1(sum_x32(sum_x16(sum_x8(pe))))));
  } else {
#pragma unroll
    for (int m = Q; m < kWave; m <<= 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        pw[k] += shfl_xor_d(pw[k], m);
        pb[k] += shfl_xor_d(pb[k], m);
      }
    }
#pragma unroll
    for (int m = 1; m < kWave; m <<= 1) pe += shfl_xor_d(pe, m);
  }
  __syncthreads();
  double* s_red = reinterpret_cast<double*>(s_dyn);  // [kWinWaves][2 * CS + 1]
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane < Q) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s_red[wave * (2 * CS + 1) + 4 * lane + k] = pw[k];
      s_red[wave * (2 * CS + 1) + CS + 4 * lane + k] = pb[k];
    }
  }
  if (lane == 0) s_red[wave * (2 * CS + 1) + 2 * CS] = pe;
  __syncthreads();
  WIN_MARK(4);
  const int D = D4 * 4;
  double* out = partials + (size_t)tile * 3 * D;
  for (int i = threadIdx.x; i <= 2 * CS; i += kWinThreads) {
    double v = 0.0;
#pragma unroll
    for (int wv = 0; wv < kWinWaves; ++wv) v += s_red[wv * (2 * CS + 1) + i];
    if (i < CS) out[slice * CS + i] = v;
    else if (i < 2 * CS) out[D + slice * CS + (i - CS)] = v;
    else out[2 * D + slice] = v;
  }
  WIN_MARK(5);
}

// Finish: blocks b < nb-1 own kWinMaxSlices of the 2D columns [dW_e | db_e]; the last one
// sums the S eps columns of every tile, then the S totals in slice order.
struct MpWinFin {
  float *dlin_w, *dlin_b, *deps;
  int D, S, nb;
  __device__ int col(int b, int j) const {
    if (b == nb - 1) return j < S ? 2 * D + j : -1;
    const int c = kWinMaxSlices * b + j;
    return c < 2 * D ? c : -1;
  }
  __device__ void finish(int b, const double* tot) const {
    const int t = threadIdx.x;
    if (b == nb - 1) {
      if (t == 0) {
        double s = 0.0;
        for (int j = 0; j < S; ++j) s += tot[j];
        deps[0] = (float)s;
      }
      return;
    }
    const int c = kWinMaxSlices * b + t;
    if (t >= kWinMaxSlices || c >= 2 * D) return;
    if (c < D) dlin_w[c] = (float)tot[t];
    else dlin_b[c - D] = (float)tot[t];
  }
};

// ----------------------------------------------------------------------------------------
// Host side
// ----------------------------------------------------------------------------------------
bool valid_plan(const gine_window_plan* p, int64_t num_nodes, int32_t channels) {
  if (!p || !p->tile_begin || !p->win_lo || !p->win_rows || p->num_tiles <= 0) return false;
  const int cs = p->slice_channels;
  if (!(cs == 8 || cs == 16 || cs == 32) || channels % cs != 0) return false;
  if (channels / cs > kWinMaxSlices) return false;
  if (p->max_rows < 0 || p->max_edges < 0 || p->max_nodes <= 0) return false;
  if ((int64_t)p->max_rows * cs * 4 > kWinRowBytes) return false;
  if (p->max_edges > kWinEdgeLoads * kWinThreads || p->max_nodes > kWinTileNodes) return false;
  if (num_nodes <= 0 || num_nodes * channels * 4 >= (int64_t(1) << 32)) return false;
  return win_lds_bytes(cs, p->max_rows, p->max_edges, p->max_nodes) <= GINE_WINDOW_LDS_BYTES;
}

WinPlan device_plan(const gine_window_plan* p) {
  return WinPlan{p->tile_begin, p->win_lo, p->win_rows, p->max_rows, p->max_edges,
                 p->max_nodes, p->slot, p->edge_begin};
}

// Raise the kernel's dynamic-LDS ceiling once per instantiation (thread-safe static init).

// (the whole 160 KiB less the kernel's static LDS, which the attribute must leave room for)
template <auto K>
int set_lds_limit() {
  static const hipError_t e = [] {
    hipFuncAttributes fa{};
    hipError_t r = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(K));
    if (r != hipSuccess) return r;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(K),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024 - (int)fa.sharedSizeBytes);
  }();
  return e == hipSuccess ? GINE_OK : GINE_ERR_HIP_BASE + (int)e;
}

#define GINE_WIN_DISPATCH(CS_, FMA_FLAG, MACRO) \
  switch (CS_) {                                \
    case 8:                                     \
      if (FMA_FLAG) MACRO(8, true);             \
      else MACRO(8, false);                     \
      break;                                    \
    case 16:                                    \
      if (FMA_FLAG) MACRO(16, true);            \
      else MACRO(16, false);                    \
      break;                                    \
    default:                                    \
      if (FMA_FLAG) MACRO(32, true);            \
      else MACRO(32, false);                    \
      break;                                    \
  }

template <int PDO>
int mp_bwd_win_launch(const float* dz, const float* x, const int32_t* out_rowptr,
                      const int32_t* out_dst, const float* out_attr, const float* lin_w,
                      const float* lin_b, const float* eps, const float* dres, float* dx,
                      double* partials, int64_t num_nodes, int32_t channels, int32_t flags,
                      const gine_window_plan* plan, const MlpSlabJob& job,
                      const WinEngine<PDO>* eng, void* stream) {
  if (!valid_plan(plan, num_nodes, channels)) return GINE_ERR_INVALID;
  if ((flags & ~(GINE_MP_BWD_SELF | GINE_MP_LIN_MULADD)) != 0) return GINE_ERR_INVALID;
  if (!dz || !x || !out_rowptr || !out_dst || !out_attr || !lin_w || !lin_b || !eps || !dx ||
      !partials)
    return GINE_ERR_INVALID;
  const int cs = plan->slice_channels, S = channels / cs, D4 = channels / 4;
  size_t smem = win_lds_bytes(cs, plan->max_rows, plan->max_edges, plan->max_nodes);
  const size_t red = sizeof(double) * kWinWaves * (2 * (size_t)cs + 1);
  const size_t jobb = job.nblocks > 0 ? sizeof(double) * kSlabGroups * (kSlabQuads * 4 + 1) : 0;
  smem = smem > red ? smem : red;
  smem = smem > jobb ? smem : jobb;
  if (eng) {  // the engine: D = 64 / 128, 32-channel slices, no slab side job in the launch
    if ((channels != 128 && channels != 64) || eng->D != channels || cs != 32 ||
        job.nblocks != 0 || eng->nblocks <= 0)
      return GINE_ERR_INVALID;
    smem = smem > kWinEngineLds ? smem : kWinEngineLds;
  }
  if (smem > GINE_WINDOW_LDS_BYTES) return GINE_ERR_INVALID;
  const unsigned grid =
      (unsigned)(plan->num_tiles * S + job.nblocks + (eng ? eng->nblocks : 0));
  const WinPlan wp = device_plan(plan);
  hipStream_t s = as_stream(stream);
  const bool fma = (flags & GINE_MP_LIN_MULADD) == 0;
  int st = GINE_OK;
  const WinEngine<PDO> e0 = eng ? *eng : WinEngine<PDO>{};
#define LAUNCH_BWD_WIN_K(KER)                                                                 \
  do {                                                                                       \
    st = set_lds_limit<KER>();                                                               \
    if (st == GINE_OK)                                                                       \
      hipLaunchKernelGGL((KER), dim3(grid), dim3(kWinThreads), smem, s, (const float4*)dz,   \
                         (const float4*)x, out_rowptr, out_dst, out_attr,                    \
                         (const float4*)lin_w, (const float4*)lin_b, eps, (const float4*)dres, \
                         (float4*)dx, partials, wp, D4, S, flags, job, e0);                  \
  } while (0)
#define LAUNCH_BWD_WIN(CS_, F_) LAUNCH_BWD_WIN_K((k_mp_bwd_win<CS_, F_, false, PDO>))
  if (eng) {
    if (fma) LAUNCH_BWD_WIN_K((k_mp_bwd_win<32, true, true, PDO>));
    else LAUNCH_BWD_WIN_K((k_mp_bwd_win<32, false, true, PDO>));
  } else if constexpr (PDO == PRO_PLAIN) {  // (the engine's type is unused here)
    GINE_WIN_DISPATCH(cs, fma, LAUNCH_BWD_WIN);
  } else {
    return GINE_ERR_INVALID;
  }
#undef LAUNCH_BWD_WIN
#undef LAUNCH_BWD_WIN_K
  if (st != GINE_OK) return st;
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_graph_plan_windows(const int32_t* rowptr, const int32_t* nbr,
                                       int64_t num_nodes, int32_t max_rows, int32_t max_nodes,
                                       int32_t max_edges, int32_t* tile_begin, int32_t* win_lo,
                                       int32_t* win_rows, int32_t* num_tiles,
                                       int32_t* maxima) {
  if (!rowptr || !tile_begin || !win_lo || !win_rows || !num_tiles || !maxima)
    return GINE_ERR_INVALID;
  if (num_nodes < 0 || max_rows <= 0 || max_nodes <= 0 || max_edges <= 0)
    return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  *num_tiles = 0;
  maxima[0] = maxima[1] = maxima[2] = 0;
  if (num_nodes == 0) return GINE_OK;
  if (rowptr[num_nodes] > 0 && !nbr) return GINE_ERR_INVALID;
  int T = 0, begin = 0, lo = INT_MAX, hi = -1, cnt = 0, ecnt = 0;
  int mrows = 0, medges = 0, mnodes = 0;
  auto close_tile = [&]() {
    tile_begin[T] = begin;
    win_lo[T] = hi >= lo ? lo : 0;
    win_rows[T] = hi >= lo ? hi - lo + 1 : 0;
    mrows = win_rows[T] > mrows ? win_rows[T] : mrows;
    medges = ecnt > medges ? ecnt : medges;
    mnodes = cnt > mnodes ? cnt : mnodes;
    ++T;
  };
  for (int v = 0; v < (int)num_nodes; ++v) {
    const int e0 = rowptr[v], e1 = rowptr[v + 1], deg = e1 - e0;
    int vlo = INT_MAX, vhi = -1;
    for (int e = e0; e < e1; ++e) {
      vlo = nbr[e] < vlo ? nbr[e] : vlo;
      vhi = nbr[e] > vhi ? nbr[e] : vhi;
    }
    if (deg > max_edges || (deg > 0 && vhi - vlo + 1 > max_rows)) return GINE_OK;  // no plan
    const int nlo = vlo < lo ? vlo : lo, nhi = vhi > hi ? vhi : hi;
    const bool too_wide = nhi >= nlo && nhi - nlo + 1 > max_rows;
    if (cnt > 0 && (cnt == max_nodes || ecnt + deg > max_edges || too_wide)) {
      close_tile();
      begin = v;
      lo = vlo;
      hi = vhi;
      cnt = 0;
      ecnt = 0;
    } else {
      lo = nlo;
      hi = nhi;
    }
    ++cnt;
    ecnt += deg;
  }
  close_tile();
  tile_begin[T] = (int32_t)num_nodes;
  *num_tiles = T;
  maxima[0] = mrows;
  maxima[1] = medges;
  maxima[2] = mnodes;
  return GINE_OK;
}

extern "C" int gine_graph_plan_window_slots(const int32_t* rowptr, const int32_t* tile_begin,
                                            int32_t num_tiles, int16_t* slot) {
  if (!rowptr || !tile_begin || !slot || num_tiles < 0) return GINE_ERR_INVALID;
  constexpr int G = kWinThreads / 8;  // lane groups of the 32-channel backward
  std::vector<int> idx;
  for (int t = 0; t < num_tiles; ++t) {
    const int n0 = tile_begin[t], n = tile_begin[t + 1] - n0;
    if (n < 0 || n > kWinTileNodes) return GINE_ERR_INVALID;
    idx.resize(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
      return rowptr[n0 + a + 1] - rowptr[n0 + a] > rowptr[n0 + b + 1] - rowptr[n0 + b];
    });
    // positions [0, G): the heaviest nodes; position G + g: the (g+1)-th lightest, so the
    // lane group that runs the heaviest node runs the lightest second
    const int first = n < G ? n : G;
    for (int s = 0; s < first; ++s) slot[n0 + s] = (int16_t)idx[s];
    for (int g = 0; G + g < n; ++g) slot[n0 + G + g] = (int16_t)idx[n - 1 - g];
  }
  return GINE_OK;
}

extern "C" int gine_mp_fwd_win(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                               const float* in_attr, const float* lin_w, const float* lin_b,
                               const float* eps, float* z, int64_t num_nodes, int32_t channels,
                               int32_t flags, const gine_window_plan* plan, void* stream) {
  if (!valid_plan(plan, num_nodes, channels)) return GINE_ERR_INVALID;
  if ((flags & ~GINE_MP_LIN_MULADD) != 0) return GINE_ERR_INVALID;
  if (!x || !in_rowptr || !in_src || !in_attr || !lin_w || !lin_b || !eps || !z)
    return GINE_ERR_INVALID;
  const int cs = plan->slice_channels, S = channels / cs, D4 = channels / 4;
  const size_t smem = win_lds_bytes(cs, plan->max_rows, plan->max_edges, plan->max_nodes);
  const unsigned grid = (unsigned)(plan->num_tiles * S);
  const WinPlan wp = device_plan(plan);
  hipStream_t s = as_stream(stream);
  const bool fma = (flags & GINE_MP_LIN_MULADD) == 0;
  int st = GINE_OK;
#define LAUNCH_FWD_WIN(CS_, F_)                                                              \
  do {                                                                                       \
    st = set_lds_limit<k_mp_fwd_win<CS_, F_>>();                                               \
    if (st == GINE_OK)                                                                       \
      hipLaunchKernelGGL((k_mp_fwd_win<CS_, F_>), dim3(grid), dim3(kWinThreads), smem, s,    \
                         (const float4*)x, in_rowptr, in_src, in_attr, (const float4*)lin_w, \
                         (const float4*)lin_b, eps, (float4*)z, wp, D4, S);                  \
  } while (0)
  GINE_WIN_DISPATCH(cs, fma, LAUNCH_FWD_WIN);
#undef LAUNCH_FWD_WIN
  if (st != GINE_OK) return st;
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_mp_bwd_win(const float* dz, const float* x, const int32_t* out_rowptr,
                               const int32_t* out_dst, const float* out_attr,
                               const float* lin_w, const float* lin_b, const float* eps,
                               const float* dres, float* dx, double* partials,
                               int64_t num_nodes, int32_t channels, int32_t flags,
                               const gine_window_plan* plan, void* stream) {
  const MlpSlabJob none{nullptr, 0, 0, 0, MlpWgradOut{nullptr, nullptr, nullptr, nullptr, 0}};
  return mp_bwd_win_launch<PRO_PLAIN>(dz, x, out_rowptr, out_dst, out_attr, lin_w, lin_b, eps,
                                      dres, dx, partials, num_nodes, channels, flags, plan,
                                      none, nullptr, stream);
}

extern "C" int gine_mp_bwd_win_side(const float* dz, const float* x, const int32_t* out_rowptr,
                                    const int32_t* out_dst, const float* out_attr,
                                    const float* lin_w, const float* lin_b, const float* eps,
                                    const float* dres, float* dx, double* partials,
                                    int64_t num_nodes, int32_t channels, int32_t flags,
                                    const gine_window_plan* plan, const float* wg_slab,
                                    int32_t wg_chunks, int32_t mlp_channels, float* dw1,
                                    float* db1, float* dw2, float* db2, void* stream) {
  if (!wg_slab || wg_chunks <= 0 || mlp_channels <= 0) return GINE_ERR_INVALID;
  const int64_t per = (int64_t)mlp_channels * mlp_channels + mlp_channels;
  if (per % 4 != 0 || (reinterpret_cast<uintptr_t>(wg_slab) & 15) != 0) return GINE_ERR_INVALID;
  const int cols = (int)ceil_div(per, kSlabQuads * 4);
  const MlpSlabJob job{wg_slab, wg_chunks, cols, 2 * cols,
                       MlpWgradOut{dw2, db2, dw1, db1, mlp_channels}};
  return mp_bwd_win_launch<PRO_PLAIN>(dz, x, out_rowptr, out_dst, out_attr, lin_w, lin_b, eps,
                                      dres, dx, partials, num_nodes, channels, flags, plan,
                                      job, nullptr, stream);
}

extern "C" int gine_mp_bwd_win_mlp_wgrad(
    const float* dz, const float* x, const int32_t* out_rowptr, const int32_t* out_dst,
    const float* out_attr, const float* lin_w, const float* lin_b, const float* eps,
    const float* dres, float* dx, double* partials, int64_t num_nodes, int32_t channels,
    int32_t flags, const gine_window_plan* plan, const float* dy, const float* y,
    const uint8_t* mask, const float* a1, const float* bn_save, const float* dbn,
    const float* coef, const float* z, float* slab, int32_t epilogue, void* stream) {
  if (!dy || !a1 || !bn_save || !dbn || !coef || !z || !slab) return GINE_ERR_INVALID;
  if (epilogue < GINE_EPI_NONE || epilogue > GINE_EPI_RESIDUAL_RELU) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RELU && !y) return GINE_ERR_INVALID;
  if (epilogue == GINE_EPI_RESIDUAL_RELU && !mask) return GINE_ERR_INVALID;
  if (channels != 128 && channels != 64) return GINE_ERR_DIM;
  static_assert(kMlpWgTO == 64, "the fused engine runs 64-row output tiles");
  const int D = channels;
  const WgPlan p = wg_plan(num_nodes, D, D, 2, kMlpWgTO);  // = gine_mlp_wgrad's plan
  const size_t per = (size_t)D * D + D;
  const int tiles = 2 * p.tiles_o * p.tiles_i;
  const ProArgs p_do{dy, y, mask, nullptr, nullptr};
  const ProArgs q_r{a1, nullptr, nullptr, bn_save, nullptr};
  const ProArgs p_da1{dbn, a1, nullptr, bn_save, coef};
  const ProArgs q_z{z, nullptr, nullptr, nullptr, nullptr};
  const MlpSlabJob none{nullptr, 0, 0, 0, MlpWgradOut{nullptr, nullptr, nullptr, nullptr, 0}};
#define MP_ENG(PD)                                                                           \
  do {                                                                                       \
    const WinEngine<PD> e{MlpWgradSrc<PD>{p_do, q_r, p_da1, q_z, D}, slab, num_nodes,        \
                          per * p.chunks, per, p.chunks * tiles, tiles, p.rows_per_chunk, D};\
    return mp_bwd_win_launch<PD>(dz, x, out_rowptr, out_dst, out_attr, lin_w, lin_b, eps,    \
                                 dres, dx, partials, num_nodes, channels, flags, plan, none,  \
                                 &e, stream);                                                \
  } while (0)
  if (epilogue == GINE_EPI_NONE) MP_ENG(PRO_PLAIN);
  if (epilogue == GINE_EPI_RELU) MP_ENG(PRO_DOR);
  MP_ENG(PRO_DOM);
#undef MP_ENG
}

extern "C" int gine_mp_bwd_win_finalize(const double* partials, int32_t num_tiles,
                                        int32_t channels, int32_t slice_channels,
                                        float* dlin_w, float* dlin_b, float* deps,
                                        void* stream) {
  if (num_tiles <= 0 || channels <= 0 || slice_channels <= 0) return GINE_ERR_INVALID;
  if (channels % slice_channels != 0 || channels / slice_channels > kWinMaxSlices)
    return GINE_ERR_INVALID;
  if (!partials || !dlin_w || !dlin_b || !deps) return GINE_ERR_INVALID;
  const int nb = (int)ceil_div(2 * channels, kWinMaxSlices) + 1;
  const MpWinFin fin{dlin_w, dlin_b, deps, channels, channels / slice_channels, nb};
  hipLaunchKernelGGL((k_colsum_fin<kWinMaxSlices, MpWinFin>), dim3(nb), dim3(256), 0,
                     as_stream(stream), partials, num_tiles, 3 * channels, fin);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

#ifdef GINE_WIN_PROFILE
extern "C" int gine_debug_win_prof(long long* out) {  // [4096][8] host buffer
  GINE_RETURN_IF_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_win_prof), sizeof(g_win_prof)));
  return GINE_OK;
}
#endif
