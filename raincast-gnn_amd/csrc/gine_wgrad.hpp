// Weight-gradient engine: dW[o][i] = sum_n P[n][o] * Q[n][i], db[o] = sum_n P[n][o],
// over MANY rows n (16,000 - 128,000 nodes) into a small [O x I] output (O, I <= 256).
//
// Used by the node-MLP backward (dW2 = do^T r, dW1 = da1^T z; models/gnn.py:21-26 via
// autograd) and by the plain Linears around the GINE stack (DeepSet rho/phi, dim_red,
// aggr: models/gnn.py:48-68,112-123).  P and Q come from "source" policies that load raw
// operands and apply the elementwise prologue (ReLU masks, BatchNorm backward, ...) when
// the tile is staged, so the [N x D] operands are never materialised.
//
// Decomposition: grid = (row chunks, TO x 128 output tiles, Z independent products).  A
// 256-thread workgroup owns one TO(o) x 128(i) output tile of one row chunk, as
// v_mfma_f32_32x32x2_f32 accumulators spread over its 4 waves (see wgrad_body for TO = 64
// and 128).  64-row sub-tiles of P and Q are staged through LDS;
// the RAW operands of the next sub-tile are loaded into registers before this sub-tile's
// 64-long MFMA chain and transformed only when staged, so their HBM latency hides under
// the matrix pipe.  Each (chunk, tile) writes an fp32 partial slab; slabs are reduced over
// chunks in fixed order in fp64 (deterministic, no float atomics).
//
// The chain runs on the bf16 matrix cores in three-way split form (gine_bf16x3.hpp,
// wgrad_body_x3): each staged value is split ONCE, by the thread that stages it, into three
// bf16 planes kept in LDS column-major (a thread stages consecutive rows of one float4
// column quad, so each column gets its k run in one store per plane), and the waves read
// their MFMA fragments as plain 16-byte LDS reads -- no per-wave re-split (the form measured
// slower in round 3) and 2.7x the MFMA rate of v_mfma_f32_32x32x2_f32.  A workgroup whose
// accumulators see a NaN (a non-finite operand) redoes its tile with the fp32 chain.
#pragma once

#include "gine_common.hpp"
#include "gine_bf16x3.hpp"

// Diagnostic switches (tools/wg_micro.hip only; 0 in the library): bit 0 skips the MFMA
// chain, bit 1 replaces the operand loads by zeros, bit 2 skips the slab stores, bit 3
// stamps s_memtime / s_memrealtime at body entry and exit into gine_wg_clock[block][4],
// bit 4 replaces the chain's LDS operand reads by register values.
#ifndef GINE_WG_VARIANT
#define GINE_WG_VARIANT 0
#endif

namespace gine {

#if (GINE_WG_VARIANT & 8) != 0
__device__ unsigned long long gine_wg_clock[4096][4];
#endif

typedef float wg_floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWgRows = 64;                   // rows per staged sub-tile
constexpr int kWgTI = 128;                    // i-columns per workgroup tile
constexpr int kWgLdQ = kWgTI + 4;             // padded LDS rows (floats)
#ifndef GINE_WG_TARGET_BLOCKS
#define GINE_WG_TARGET_BLOCKS 256
#endif
constexpr int kWgTargetBlocks = GINE_WG_TARGET_BLOCKS;  // one workgroup per CU
constexpr int kWgMinSubtiles = 2;             // per chunk
#ifndef GINE_WG_WAVES64
#define GINE_WG_WAVES64 8
#endif
constexpr int kWgWaves64 = GINE_WG_WAVES64;   // waves per workgroup of the 64-row tiles

// GINE_WG_BF16X3=0 (A/B builds) keeps the fp32 chain.
#ifndef GINE_WG_BF16X3
#define GINE_WG_BF16X3 1
#endif

// LDS image of one staged operand for the split chain: three bf16 planes (h, m, l), each
// COLUMN-major -- C columns of kWgRows (64) k values, 128 bytes per column -- so an MFMA
// fragment (8 consecutive k of one column) is one 16-byte ds_read_b128.  The 16-byte chunks
// of a column are XOR-swizzled by (column >> 1) & 7, so the reads of 16 consecutive columns
// at one k offset land on 16 different bank groups.
template <int C>
struct WgImg {
  static constexpr int kPlane = C * kWgRows * 2;
  static constexpr int kBytes = 3 * kPlane;
  // byte offset of (column c, k) in a plane
  __device__ static __forceinline__ int off(int c, int k) {
    return c * (kWgRows * 2) + 16 * ((k >> 3) ^ ((c >> 1) & 7)) + 2 * (k & 7);
  }
};

// Bytes of LDS one engine workgroup needs (sP followed by sQ in ONE region: the fp32
// layout, or the split planes, whichever is larger).
template <int TO>
constexpr size_t wg_lds_bytes() {
  constexpr size_t f32 = sizeof(float) * kWgRows * ((TO + 4) + kWgLdQ);
  constexpr size_t x3 = (size_t)3 * kWgRows * 2 * (TO + kWgTI);
  return GINE_WG_BF16X3 ? (f32 > x3 ? f32 : x3) : f32;
}

struct WgPlan {
  int tiles_o, tiles_i, chunks, rows_per_chunk;
};

// Z products of [O x I] over R rows in TO x 128 output tiles: about one workgroup per CU,
// >= 2 sub-tiles per chunk.  total_tiles: output tiles of all Z products together
// (default Z * tiles_o * tiles_i; less when a policy gives some products a narrower I).
inline WgPlan wg_plan(int64_t R, int O, int I, int Z, int TO, int total_tiles = 0) {
  WgPlan p;
  p.tiles_o = (int)ceil_div(O, TO);
  p.tiles_i = (int)ceil_div(I, kWgTI);
  const int64_t subtiles = ceil_div(R > 0 ? R : 1, kWgRows);
  if (total_tiles <= 0) total_tiles = Z * p.tiles_o * p.tiles_i;
  int64_t chunks = ceil_div(kWgTargetBlocks, (int64_t)total_tiles);
  const int64_t cap = ceil_div(subtiles, kWgMinSubtiles);
  if (chunks > cap) chunks = cap;
  if (chunks < 1) chunks = 1;
  const int64_t per = ceil_div(subtiles, chunks);
  p.rows_per_chunk = (int)(per * kWgRows);
  p.chunks = (int)ceil_div(R > 0 ? R : 1, p.rows_per_chunk);
  return p;
}

// Src policy (see the users in gine_mlp.hip / gine_linear.hip); every member is a
// template on the product index Z, so each body is free of runtime branches between loads
// (a branch merge makes the compiler drain the memory queue, serialising the prefetch):
//   typename Src::Raw, Src::Col
//   Col p_col<Z>(q4) / q_col<Z>(q4)          per-column constants (q4 = float4 column)
//   Raw p_load<Z>(n, q4) / q_load<Z>(n, q4)  raw operands of row n (n always in range)
//   float4 p_xform<Z>(raw, col) / q_xform<Z> the staged value
//   int i_dim<Z>(I)                          I of product Z (<= the launch's I)
//   static constexpr int kZ                  number of products (<= 4)
//
// TO = 128: wave w holds the 64x64 quadrant (o-half w>>1, i-half w&1) as 2x2 32x32
//           accumulators (P and Q each read once per chunk; for the Z=2 node-MLP products).
// TO = 64:  wave w holds i-columns [32w, 32w+32) x all 64 o-rows (2x1 accumulators; twice
//           the workgroups for a single product).
template <class Src, int Z, int TO, int NW>
__device__ __forceinline__ void wgrad_body(const Src& src, int64_t R, int O, int I, int chunk,
                                           int tile, int rows_per_chunk, size_t zstride,
                                           size_t cstride, float* __restrict__ slab,
                                           float* __restrict__ sP, float* __restrict__ sQ) {
  using Raw = typename Src::Raw;
  using Col = typename Src::Col;
#if (GINE_WG_VARIANT & 8) != 0
  const int blin = blockIdx.x + gridDim.x * blockIdx.y + gridDim.x * gridDim.y * blockIdx.z;
  if (threadIdx.x == 0 && blin < 4096) {
    gine_wg_clock[blin][0] = __builtin_amdgcn_s_memtime();
    gine_wg_clock[blin][1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  constexpr int NT = 64 * NW;                // threads
  constexpr int LDP = TO + 4;
  constexpr int PQ = TO / 4;                 // float4 columns of the P tile
  constexpr int PG = NT / PQ;                // P row groups (rows pr + PG*k)
  constexpr int PITEMS = kWgRows / PG;
  constexpr int QQ = kWgTI / 4, QG = NT / QQ;
  constexpr int QITEMS = kWgRows / QG;
  // accumulators per wave: NJ 32-row o-tiles x NI 32-col i-tiles
  constexpr int NJ = NW == 8 ? 1 : 2;
  constexpr int NI = (NW == 4 && TO == 128) ? 2 : 1;
  static_assert(NW == 4 || (NW == 8 && TO == 64), "engine shapes");

  const int tiles_i = (int)ceil_div(I, kWgTI);
  const int o0 = (tile / tiles_i) * TO, i0 = (tile % tiles_i) * kWgTI;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  // wave's o / i origin in the tile
  const int ob = NW == 8 ? 32 * (wave >> 2) : (TO == 128 ? 64 * (wave >> 1) : 0);
  const int ib = NW == 8 ? 32 * (wave & 3) : (TO == 128 ? 64 * (wave & 1) : 32 * wave);
  const bool bias_block = (i0 == 0);

  // staging coordinates: a thread always stages the same float4 column of P and of Q
  const int pq = threadIdx.x % PQ, pr = threadIdx.x / PQ;
  const int qq = threadIdx.x % QQ, qr = threadIdx.x / QQ;
  const bool p_ok = o0 + 4 * pq < O, q_ok = i0 + 4 * qq < I;
  const int pqa = p_ok ? o0 / 4 + pq : 0, qqa = q_ok ? i0 / 4 + qq : 0;
  const Col pc = src.template p_col<Z>(pqa);
  const Col qc = src.template q_col<Z>(qqa);

  const int64_t r_begin = (int64_t)chunk * rows_per_chunk;
  const int64_t r_end = min<int64_t>(R, r_begin + rows_per_chunk);

  wg_floatx16 acc[NJ][NI];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int k = 0; k < NI; ++k)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][k][e] = 0.f;
  double bsum[4] = {0.0, 0.0, 0.0, 0.0};  // bias partials of this thread's P column quad

  Raw rp[PITEMS]{}, rq[QITEMS]{};
  // raw operands of staged item j (P items first, then Q) for the sub-tile at row n0;
  // rows past the chunk clamp to its last row (always issued: no branch around a load)
  auto load_item = [&](int j, int64_t n0) {
    if constexpr ((GINE_WG_VARIANT & 2) != 0) return;
    if (j < PITEMS) {
      const int64_t n = n0 + pr + PG * j;
      rp[j] = src.template p_load<Z>(n < r_end ? n : r_end - 1, pqa);
    } else {
      const int k = j - PITEMS;
      const int64_t n = n0 + qr + QG * k;
      rq[k] = src.template q_load<Z>(n < r_end ? n : r_end - 1, qqa);
    }
  };
  constexpr int NITEMS = PITEMS + QITEMS;     // <= 16: one per SP k-steps below
  constexpr int SP = (kWgRows / 2) / NITEMS;
  static_assert(SP >= 2, "at most one raw load per two k-steps");

  if (r_begin < r_end) {
#pragma unroll
    for (int j = 0; j < NITEMS; ++j) load_item(j, r_begin);
  }
  for (int64_t n0 = r_begin; n0 < r_end; n0 += kWgRows) {
#pragma unroll
    for (int k = 0; k < PITEMS; ++k) {
      const int r = pr + PG * k;
      float4 v = src.template p_xform<Z>(rp[k], pc);
      if (n0 + r >= r_end || !p_ok) v = f4_zero();
      *reinterpret_cast<float4*>(&sP[r * LDP + 4 * pq]) = v;
      bsum[0] += (double)v.x;
      bsum[1] += (double)v.y;
      bsum[2] += (double)v.z;
      bsum[3] += (double)v.w;
    }
#pragma unroll
    for (int k = 0; k < QITEMS; ++k) {
      const int r = qr + QG * k;
      float4 v = src.template q_xform<Z>(rq[k], qc);
      if (n0 + r >= r_end || !q_ok) v = f4_zero();
      *reinterpret_cast<float4*>(&sQ[r * kWgLdQ + 4 * qq]) = v;
    }
    __syncthreads();
    // MFMA chain over the 64 staged rows (lane half h contracts rows [32h, 32h+32): the
    // same permutation for A and B).  The next sub-tile's raw loads are spread over the
    // chain, one every other k-step: a wave that issued them all at once would stall on
    // the memory queue before its first MFMA (no second wave on the SIMD to cover it).
    // Each k-step's LDS operands are read one step ahead; sched_barrier keeps the order.
    const int64_t n1 = n0 + kWgRows;
    const float* pa = &sP[(32 * h) * LDP + ob + c32];
    const float* qb = &sQ[(32 * h) * kWgLdQ + ib + c32];
    float a[NJ], b[NI], an[NJ], bn[NI];
#pragma unroll
    for (int j = 0; j < NJ; ++j) a[j] = pa[32 * j];
#pragma unroll
    for (int k = 0; k < NI; ++k) b[k] = qb[32 * k];
#pragma unroll
    for (int s = 0; s < kWgRows / 2; ++s) {
      if (s + 1 < kWgRows / 2) {
        if constexpr ((GINE_WG_VARIANT & 16) != 0) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) an[j] = a[j] * 0.5f;
#pragma unroll
          for (int k = 0; k < NI; ++k) bn[k] = b[k] * 0.5f;
        } else {
#pragma unroll
          for (int j = 0; j < NJ; ++j) an[j] = pa[(s + 1) * LDP + 32 * j];
#pragma unroll
          for (int k = 0; k < NI; ++k) bn[k] = qb[(s + 1) * kWgLdQ + 32 * k];
        }
      }
      if (s % SP == 0 && s / SP < NITEMS) load_item(s / SP, n1);
      if constexpr ((GINE_WG_VARIANT & 1) == 0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int k = 0; k < NI; ++k)
            acc[j][k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[k], acc[j][k], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NJ; ++j) a[j] = an[j];
#pragma unroll
      for (int k = 0; k < NI; ++k) b[k] = bn[k];
    }
    __syncthreads();
  }

  float* out = slab + (size_t)Z * zstride + (size_t)chunk * cstride;
  if constexpr ((GINE_WG_VARIANT & 4) != 0) {
    if (acc[0][0][0] != 12345.f) return;  // keeps the accumulators live
  }
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    const int i = i0 + ib + 32 * k + c32;
    if (i >= I) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + ob + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o < O) out[(size_t)o * I + i] = acc[j][k][r];
      }
    }
  }
#if (GINE_WG_VARIANT & 8) != 0
  if (threadIdx.x == 0 && blin < 4096) {
    gine_wg_clock[blin][2] = __builtin_amdgcn_s_memtime();
    gine_wg_clock[blin][3] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if (bias_block) {  // fixed-order sum of the row groups' partials through LDS
    double* sb = reinterpret_cast<double*>(sQ);  // [PG][TO], sQ is free after the loop
#pragma unroll
    for (int j = 0; j < 4; ++j) sb[pr * TO + 4 * pq + j] = bsum[j];
    __syncthreads();
    if ((int)threadIdx.x < TO && o0 + (int)threadIdx.x < O) {
      double t = 0.0;
#pragma unroll 8
      for (int g = 0; g < PG; ++g) t += sb[g * TO + threadIdx.x];
      out[(size_t)O * I + o0 + threadIdx.x] = (float)t;
    }
  }
}

// ITEMS consecutive rows (k0 .. k0+ITEMS-1, ITEMS in {2, 4, 8}, k0 % ITEMS == 0) of one
// float4 column quad (columns 4cq .. 4cq+3): per column and plane one store of ITEMS bf16.
template <int C, int ITEMS>
__device__ __forceinline__ void wg_store_cols(char* img, int cq, int k0, const float4 (&v)[ITEMS]) {
  static_assert(ITEMS == 2 || ITEMS == 4 || ITEMS == 8, "column runs");
  using Img = WgImg<C>;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    uint32_t ph[ITEMS / 2], pm[ITEMS / 2], pl[ITEMS / 2];
#pragma unroll
    for (int k = 0; k < ITEMS; k += 2) {
      const float a = e == 0 ? v[k].x : e == 1 ? v[k].y : e == 2 ? v[k].z : v[k].w;
      const float b = e == 0 ? v[k + 1].x : e == 1 ? v[k + 1].y : e == 2 ? v[k + 1].z : v[k + 1].w;
      split2(a, b, ph[k / 2], pm[k / 2], pl[k / 2]);
    }
    const int o = Img::off(4 * cq + e, k0);
    char* d[3] = {img + o, img + Img::kPlane + o, img + 2 * Img::kPlane + o};
    const uint32_t* src[3] = {ph, pm, pl};
#pragma unroll
    for (int pl3 = 0; pl3 < 3; ++pl3) {
      if constexpr (ITEMS == 2) {
        *reinterpret_cast<uint32_t*>(d[pl3]) = src[pl3][0];
      } else if constexpr (ITEMS == 4) {
        *reinterpret_cast<uint2*>(d[pl3]) = make_uint2(src[pl3][0], src[pl3][1]);
      } else {
        *reinterpret_cast<uint4*>(d[pl3]) =
            make_uint4(src[pl3][0], src[pl3][1], src[pl3][2], src[pl3][3]);
      }
    }
  }
}

// The split fragment (8 consecutive k from k0, column c) from a column-major plane image.
template <int C>
__device__ __forceinline__ Bf16x3 wg_col_frag(const char* img, int c, int k0) {
  using Img = WgImg<C>;
  const int o = Img::off(c, k0);
  Bf16x3 f;
  f.h = *reinterpret_cast<const bf16x8_t*>(img + o);
  f.m = *reinterpret_cast<const bf16x8_t*>(img + Img::kPlane + o);
  f.l = *reinterpret_cast<const bf16x8_t*>(img + 2 * Img::kPlane + o);
  return f;
}

// wgrad_body on the split chain.  Staging as there (same transforms; the bias partials
// from the fp32 values), but a thread stages ITEMS CONSECUTIVE rows of its column quad and
// stores them as three bf16 planes column-major; per 64-row sub-tile every wave runs 4
// K-blocks of 16 rows, each 6 bf16 MFMAs (mfma_bf16x3) per accumulator, its fragments plain
// 16-byte reads of the plane images (element j of lane half h: row 16b + 8h + j -- the same
// k order for both operands).  The next sub-tile's raw loads are spread over the K-blocks.
template <class Src, int Z, int TO, int NW>
__device__ __forceinline__ void wgrad_body_x3(const Src& src, int64_t R, int O, int I,
                                              int chunk, int tile, int rows_per_chunk,
                                              size_t zstride, size_t cstride,
                                              float* __restrict__ slab, float* __restrict__ sP,
                                              float* __restrict__ sQ) {
  using Raw = typename Src::Raw;
  using Col = typename Src::Col;
  using IP = WgImg<TO>;
  char* imgP = reinterpret_cast<char*>(sP);  // sP.. is one region (wg_lds_bytes)
  char* imgQ = imgP + IP::kBytes;
  constexpr int NT = 64 * NW;
  constexpr int PQ = TO / 4;
  constexpr int PG = NT / PQ;
  constexpr int PITEMS = kWgRows / PG;
  constexpr int QQ = kWgTI / 4, QG = NT / QQ;
  constexpr int QITEMS = kWgRows / QG;
  constexpr int NJ = NW == 8 ? 1 : 2;
  constexpr int NI = (NW == 4 && TO == 128) ? 2 : 1;
  static_assert(NW == 4 || (NW == 8 && TO == 64), "engine shapes");

  const int tiles_i = (int)ceil_div(I, kWgTI);
  const int o0 = (tile / tiles_i) * TO, i0 = (tile % tiles_i) * kWgTI;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int ob = NW == 8 ? 32 * (wave >> 2) : (TO == 128 ? 64 * (wave >> 1) : 0);
  const int ib = NW == 8 ? 32 * (wave & 3) : (TO == 128 ? 64 * (wave & 1) : 32 * wave);
  const bool bias_block = (i0 == 0);

  const int pq = threadIdx.x % PQ, pr = threadIdx.x / PQ;
  const int qq = threadIdx.x % QQ, qr = threadIdx.x / QQ;
  const bool p_ok = o0 + 4 * pq < O, q_ok = i0 + 4 * qq < I;
  const int pqa = p_ok ? o0 / 4 + pq : 0, qqa = q_ok ? i0 / 4 + qq : 0;
  const Col pc = src.template p_col<Z>(pqa);
  const Col qc = src.template q_col<Z>(qqa);
  static_assert(PITEMS % 2 == 0 && QITEMS % 2 == 0, "column runs of 2, 4 or 8 rows");

  const int64_t r_begin = (int64_t)chunk * rows_per_chunk;
  const int64_t r_end = min<int64_t>(R, r_begin + rows_per_chunk);

  wg_floatx16 acc[NJ][NI];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int k = 0; k < NI; ++k)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][k][e] = 0.f;
  double bsum[4] = {0.0, 0.0, 0.0, 0.0};

  Raw rp[PITEMS]{}, rq[QITEMS]{};
  // this thread's rows: pr * PITEMS + k (P) and qr * QITEMS + k (Q)
  auto load_item = [&](int j, int64_t n0) {
    if (j < PITEMS) {
      const int64_t n = n0 + pr * PITEMS + j;
      rp[j] = src.template p_load<Z>(n < r_end ? n : r_end - 1, pqa);
    } else {
      const int k = j - PITEMS;
      const int64_t n = n0 + qr * QITEMS + k;
      rq[k] = src.template q_load<Z>(n < r_end ? n : r_end - 1, qqa);
    }
  };
  constexpr int NITEMS = PITEMS + QITEMS;
  constexpr int KB = kWgRows / 16;             // K-blocks per sub-tile

  if (r_begin < r_end) {
#pragma unroll
    for (int j = 0; j < NITEMS; ++j) load_item(j, r_begin);
  }
  for (int64_t n0 = r_begin; n0 < r_end; n0 += kWgRows) {
    {
      float4 vp[PITEMS], vq[QITEMS];
#pragma unroll
      for (int k = 0; k < PITEMS; ++k) {
        const int r = pr * PITEMS + k;
        float4 v = src.template p_xform<Z>(rp[k], pc);
        if (n0 + r >= r_end || !p_ok) v = f4_zero();
        vp[k] = v;
        bsum[0] += (double)v.x;
        bsum[1] += (double)v.y;
        bsum[2] += (double)v.z;
        bsum[3] += (double)v.w;
      }
      wg_store_cols<TO, PITEMS>(imgP, pq, pr * PITEMS, vp);
#pragma unroll
      for (int k = 0; k < QITEMS; ++k) {
        const int r = qr * QITEMS + k;
        float4 v = src.template q_xform<Z>(rq[k], qc);
        if (n0 + r >= r_end || !q_ok) v = f4_zero();
        vq[k] = v;
      }
      wg_store_cols<kWgTI, QITEMS>(imgQ, qq, qr * QITEMS, vq);
    }
    __syncthreads();
    const int64_t n1 = n0 + kWgRows;
#pragma unroll
    for (int b = 0; b < KB; ++b) {
      const int k0 = 16 * b + 8 * h;
      Bf16x3 fa[NJ], fb[NI];
#pragma unroll
      for (int j = 0; j < NJ; ++j) fa[j] = wg_col_frag<TO>(imgP, ob + 32 * j + c32, k0);
#pragma unroll
      for (int k = 0; k < NI; ++k) fb[k] = wg_col_frag<kWgTI>(imgQ, ib + 32 * k + c32, k0);
#pragma unroll
      for (int j = 0; j < NITEMS; ++j)
        if (j % KB == b) load_item(j, n1);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int k = 0; k < NI; ++k) acc[j][k] = mfma_bf16x3(fa[j], fb[k], acc[j][k]);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  }

  // a NaN in any wave's accumulators (non-finite operand): the tile again on the fp32 chain
  bool bad = false;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int k = 0; k < NI; ++k) bad = bad || wave_any_nan(acc[j][k]);
#ifndef GINE_WG_X3_NANCHECK
#define GINE_WG_X3_NANCHECK 1
#endif
  if (GINE_WG_X3_NANCHECK && block_any(bad, reinterpret_cast<int*>(imgP))) {
    wgrad_body<Src, Z, TO, NW>(src, R, O, I, chunk, tile, rows_per_chunk, zstride, cstride,
                               slab, sP, sQ);
    return;
  }

  float* out = slab + (size_t)Z * zstride + (size_t)chunk * cstride;
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    const int i = i0 + ib + 32 * k + c32;
    if (i >= I) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + ob + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o < O) out[(size_t)o * I + i] = acc[j][k][r];
      }
    }
  }
  if (bias_block) {  // fixed-order sum of the row groups' partials through LDS
    double* sb = reinterpret_cast<double*>(imgQ);  // [PG][TO], the planes are free now
#pragma unroll
    for (int j = 0; j < 4; ++j) sb[pr * TO + 4 * pq + j] = bsum[j];
    __syncthreads();
    if ((int)threadIdx.x < TO && o0 + (int)threadIdx.x < O) {
      double t = 0.0;
#pragma unroll 8
      for (int g = 0; g < PG; ++g) t += sb[g * TO + threadIdx.x];
      out[(size_t)O * I + o0 + threadIdx.x] = (float)t;
    }
  }
}

template <bool X3, class Src, int Z, int TO, int NW>
__device__ __forceinline__ void wg_body(const Src& src, int64_t R, int O, int I, int chunk,
                                        int tile, int rows_per_chunk, size_t zstride,
                                        size_t cstride, float* __restrict__ slab, float* sP,
                                        float* sQ) {
  if constexpr (X3)
    wgrad_body_x3<Src, Z, TO, NW>(src, R, O, I, chunk, tile, rows_per_chunk, zstride, cstride,
                                  slab, sP, sQ);
  else
    wgrad_body<Src, Z, TO, NW>(src, R, O, I, chunk, tile, rows_per_chunk, zstride, cstride,
                               slab, sP, sQ);
}

// Output tiles of product z: tiles_o * ceil(I_z / 128).
template <class Src, int Z>
__device__ __forceinline__ int wg_tiles(const Src& src, int O, int I, int TO) {
  return (int)(ceil_div(O, TO) * ceil_div(src.template i_dim<Z>(I), kWgTI));
}

// One engine workgroup: output tile y of the concatenated per-product tile lists, rows of
// chunk `chunk`.  sP / sQ: ONE LDS region of wg_lds_bytes<TO>(), sQ = sP + kWgRows * (TO + 4)
// (the fp32 body's two arrays; the split body uses the region as its plane images).
// X3: the split chain (wgrad_body_x3) or the fp32 one (wgrad_body).
template <class Src, int TO, int NW, bool X3 = GINE_WG_BF16X3 != 0>
__device__ __forceinline__ void wgrad_block(const Src& src, int64_t R, int O, int I, int chunk,
                                            int y, int rows_per_chunk, size_t zstride,
                                            size_t cstride, float* __restrict__ slab,
                                            float* sP, float* sQ) {
  const int t0 = wg_tiles<Src, 0>(src, O, I, TO);
  if (y < t0) {
    wg_body<X3, Src, 0, TO, NW>(src, R, O, src.template i_dim<0>(I), chunk, y, rows_per_chunk,
                               zstride, cstride, slab, sP, sQ);
    return;
  }
  y -= t0;
  if constexpr (Src::kZ > 1) {
    const int t1 = wg_tiles<Src, 1>(src, O, I, TO);
    if (y < t1) {
      wg_body<X3, Src, 1, TO, NW>(src, R, O, src.template i_dim<1>(I), chunk, y,
                                 rows_per_chunk, zstride, cstride, slab, sP, sQ);
      return;
    }
    y -= t1;
  }
  if constexpr (Src::kZ > 2) {
    const int t2 = wg_tiles<Src, 2>(src, O, I, TO);
    if (y < t2) {
      wg_body<X3, Src, 2, TO, NW>(src, R, O, src.template i_dim<2>(I), chunk, y,
                                 rows_per_chunk, zstride, cstride, slab, sP, sQ);
      return;
    }
    y -= t2;
  }
  if constexpr (Src::kZ > 3) {
    wg_body<X3, Src, 3, TO, NW>(src, R, O, src.template i_dim<3>(I), chunk, y, rows_per_chunk,
                               zstride, cstride, slab, sP, sQ);
  }
}

// 1-D grid of chunks x tiles (tiles = sum over z of the product's output tiles).  The
// tiles of one row chunk run back to back on ONE XCD (xcd_remap): they read the same rows,
// which that XCD's L2 then serves.
template <class Src, int TO, int NW, bool X3>
__global__ __launch_bounds__(64 * NW) void k_wgrad_engine(Src src, int64_t R, int O, int I,
                                                          int rows_per_chunk, size_t zstride,
                                                          size_t cstride,
                                                          float* __restrict__ slab,
                                                          int total_tiles) {
  constexpr size_t kBytes =
      X3 ? wg_lds_bytes<TO>() : sizeof(float) * kWgRows * ((TO + 4) + kWgLdQ);
  __shared__ __attribute__((aligned(16))) float s_eng[kBytes / sizeof(float)];
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  wgrad_block<Src, TO, NW, X3>(src, R, O, I, lb / total_tiles, lb % total_tiles,
                               rows_per_chunk, zstride, cstride, slab, s_eng,
                               s_eng + kWgRows * (TO + 4));
}

// Z must equal Src::kZ; total_tiles = sum of the products' output tiles (the plan's).
// X3: the split chain (the node-MLP engines keep the fp32 one, so the stand-alone engine
// and the one inside the window backward give the same bits).
template <int TO, class Src, bool X3 = GINE_WG_BF16X3 != 0>
inline int launch_wgrad_engine(const Src& src, int64_t R, int O, int I, int total_tiles,
                               const WgPlan& p, size_t zstride, size_t cstride, float* slab,
                               hipStream_t s) {
  constexpr int NW = TO == 64 ? kWgWaves64 : 4;
  hipLaunchKernelGGL((k_wgrad_engine<Src, TO, NW, X3>), dim3(p.chunks * total_tiles),
                     dim3(64 * NW), 0, s, src, R, O, I, p.rows_per_chunk, zstride, cstride,
                     slab, total_tiles);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

}  // namespace gine
