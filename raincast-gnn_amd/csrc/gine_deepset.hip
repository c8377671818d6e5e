// DeepSetEncoder phi, first layer + ReLU + member sum, fused (models/gnn.py:48-68):
//   r[n, :] = sum_m relu(ens[n, m, :] W1^T + b1)          ens [N, M, F], W1 [H, F]
// and its backward for the weights:
//   dh[n, m, :] = dr[n, :] * 1[ens[n, m, :] W1^T + b1 > 0]
//   dW1 = sum_{n,m} dh[n, m, :]^T ens[n, m, :],   db1 = sum_{n,m} dh[n, m, :]
// The reference materialises the [N, M, H] pre-activation (90 MB at the 24h_mixed
// benchmark shape) three times per step (Linear output, ReLU output, ReLU gradient).  Here
// it never leaves the MFMA accumulators.  Rows are (node, member) pairs; a workgroup walks
// groups of 2G nodes (G = 16; 8 or 4 for small batches) = 2G*M rows as ceil(G*M/16) tiles of
// 32 rows, and each wave owns 32 hidden units.
// Row placement: the accumulator register q of lane half h (v_mfma_f32_32x32x2_f32 output
// row (q&3)+8(q>>2)+4h) holds group row G*M*h + 16*t + q in tile t, i.e. half 0 walks the
// rows of nodes 0..G-1 and half 1 those of nodes G..2G-1, both in member order.  So
//  * forward: bias + ReLU in registers and a running per-node sum per lane, written once
//    when the node changes (wave-uniform: both halves are at the same local row) -- no
//    LDS read-modify-write, deterministic member order;
//  * backward: the chain is recomputed, masked with dr of the row's node, and the masked
//    accumulator registers are fed straight back as the A operand of the dW1 MFMA (a lane
//    half's 16 registers are 16 distinct k of a 32x32x2 A fragment under a k-permutation
//    that B -- read from the staged ens rows 16h+q -- follows too).
#include "gine_common.hpp"
#include "gine_chainfold.hpp"
#include "gine_bf16x3.hpp"

#include <algorithm>

namespace gine {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// A group is 2G nodes (G per lane half), walked as TPG = ceil(G*M/16) tiles of 32 rows:
// half c's 16 rows of tile t are the group's rows c*G*M + 16t + j (j < 16), and rows with
// 16t + j >= G*M are padding (staged as zero, ReLU bit cleared, sum not kept).  G = 16 (no
// padding) when there are enough nodes to fill the chip; G = 8 doubles the workgroups of a
// small batch (cfg2: 1,000 instead of 500) at the cost of <= 15 padding rows per half.
__host__ __device__ constexpr int tiles_per_group(int G, int M) { return (G * M + 15) / 16; }

// The forward's pre-activation chain on the bf16 matrix cores in three-way split form
// (gine_bf16x3.hpp): each staged ens value is split ONCE, by the thread that stages it, into
// three bf16 planes (images [32][RS] per plane, k padded to a multiple of 16 with zeros;
// rows of RS*2 = 16 x odd bytes, so the 16-byte row reads of 16 consecutive rows cover all
// banks), W1 is split once per workgroup into register planes, and a 32-row tile costs
// ceil(K/16) x 6 v_mfma_f32_32x32x16_bf16 (192 cycles per 16 k) instead of K/2
// v_mfma_f32_32x32x2_f32 (64 cycles per 2 k): 576 instead of 1,280 cycles at K = 35.  A
// wave whose accumulators see a NaN (a non-finite ens value or weight) redoes its tile on
// the fp32 chain from global memory, which is the fp32 form's exact result.
// GINE_DS_BF16X3=0 (A/B builds) keeps the fp32 chain.
#ifndef GINE_DS_BF16X3
#define GINE_DS_BF16X3 1
#endif
template <int KP>
struct DsImg {
  static constexpr int KX = (KP + 15) / 16 * 16;  // k of the split chain
  static constexpr int RS = KX + 8;               // row stride (bf16 elements)
  static constexpr int PLANE = 32 * RS;           // elements per plane
  static constexpr int FLOATS = 3 * PLANE / 2;    // one tile's three planes, in floats
};
// The backward's images: COLUMN-major planes, one column of 32 staged rows (+ 8 padding,
// 80 bytes: 16-byte reads of 16 consecutive columns hit 16 different bank groups) per
// feature, 32 or 64 features (all on the matrix cores; zero past F).
template <int KI>
struct DsBwdImg {
  static_assert(KI == 32 || KI == 64, "feature tiles");
  static constexpr int RS = 40;                   // column stride (bf16 elements)
  static constexpr int PLANE = KI * RS;
  static constexpr int FLOATS = 3 * PLANE / 2;
};
constexpr int ds_bwd_ki(int KP) { return KP <= 32 ? 32 : 64; }
template <int KP, bool X3, int KI>
constexpr int stager_ld() {
  if constexpr (!X3) return KP + 4;
  else if constexpr (KI == 0) return DsImg<KP>::RS;
  else return DsBwdImg<KI>::RS;
}
template <int KP, bool X3, int KI>
constexpr int stager_plane() {
  if constexpr (!X3) return 0;
  else if constexpr (KI == 0) return DsImg<KP>::PLANE;
  else return DsBwdImg<KI>::PLANE;
}

#ifdef GINE_DS_PROFILE
// Debug build only: block 0 / thread 0 records s_memtime at phase boundaries of its tiles.
__device__ long long g_ds_prof[4096];
__device__ int g_ds_prof_n;
#define DS_MARK(tag)                                                          \
  do {                                                                        \
    if (blockIdx.x == 0 && threadIdx.x == 0 && g_ds_prof_n < 2040) {          \
      g_ds_prof[2 * g_ds_prof_n] = (tag);                                     \
      g_ds_prof[2 * g_ds_prof_n + 1] = (long long)__builtin_amdgcn_s_memtime(); \
      ++g_ds_prof_n;                                                          \
    }                                                                         \
  } while (0)
#else
#define DS_MARK(tag) do {} while (0)
#endif

__device__ __forceinline__ floatx16 zero16() {
  floatx16 v;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = 0.f;
  return v;
}

// LDS row holding MFMA output row i (see the row placement above): 16*h + q.
__device__ __forceinline__ int staged_row(int i) {
  return 16 * ((i >> 2) & 1) + (i & 3) + 4 * (i >> 3);
}

// Tile t of a group stages, into an LDS tile [32][KP+4], rows 16c+j <- group row
// G*M*c + 16*t + j (c = lane half, j < 16): two contiguous runs of 16*F floats.  Offsets
// depend only on the thread, so they are computed once; the loads address a uniform
// (scalar) tile base plus a 32-bit lane offset.
// X3: the staged tile is three bf16 planes (dst in bf16 elements): DsImg<KP>'s (the
// forward, KI = 0) or DsBwdImg<KI>'s (the backward)
// Stores of the stagers without a branch per element (bit 0: the backward's, bit 1: the
// forward's): backward 40.4 -> 39.3 us, forward 27.8 -> 27.3 us at 16,000 nodes
// (profiles/r05_s08_ds_ab_branchless.txt)
#ifndef GINE_DS_BRANCHLESS
#define GINE_DS_BRANCHLESS 3
#endif
// PAD: G*M % 16 != 0 possible; BWD: the backward's stager
template <int NT, int KP, bool PAD, bool X3 = false, int KI = 0, bool BWD = false>
struct Stager {
  static constexpr int PER = (32 * KP + NT - 1) / NT;  // >= 32*F / NT
  static constexpr int LD = stager_ld<KP, X3, KI>();
  static constexpr int kPlane = stager_plane<KP, X3, KI>();
  // A thread without an element stores its zero to a padding slot no chain reads instead
  // of branching around the store (GINE_DS_BRANCHLESS bit 0: the backward's stager, bit 1:
  // the forward's): row t % 32 past the k range of the row-major images (columns KX.. /
  // KP..), rows 32.. of feature t % 32 in the column-major ones -- a slot per thread, so no
  // two lanes of a store share an address
  static constexpr bool kBranchless = (GINE_DS_BRANCHLESS & (BWD ? 1 : 2)) != 0;
  __device__ static int dummy_slot() {
    const int r = threadIdx.x & 31, u = threadIdx.x >> 5;
    if constexpr (X3 && KI != 0) return r * LD + 32 + (u & 7);
    else if constexpr (X3) return r * LD + DsImg<KP>::KX + (u & 7);
    else return r * LD + KP + (u & 3);
  }
  int src[PER];  // float offset from the tile's first row (0 if the thread has no element)
  int row[PER];  // group-row offset from the tile's first row (INT_MAX: no element)
  int dst[PER];  // LDS offset (-1: no element)
  uint32_t jrow[PAD ? PER : 1];
  __device__ __forceinline__ void init(int F, int M, int G) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + i * NT;
      const int c = e >= 16 * F ? 1 : 0;
      const int off = e - c * 16 * F;
      const int j = off / F, f = off - j * F;
      const bool has = e < 32 * F;
      src[i] = has ? c * G * M * F + off : 0;
      row[i] = has ? c * G * M + j : 0x7fffffff;
      if constexpr (X3 && KI != 0)
        dst[i] = has ? f * LD + (16 * c + j) : (kBranchless ? dummy_slot() : -1);  // col-major
      else
        dst[i] = has ? (16 * c + j) * LD + f : (kBranchless ? dummy_slot() : -1);
      if constexpr (PAD) jrow[i] = has ? (uint32_t)j : 0u;
    }
  }
  // Stage the tile whose first group row is `row0` (rows_total = N*M rows exist); rows
  // j >= half_lim of each lane half are padding (half_lim = G*M - 16t).
  // Returns the rows-in-range bits: the zeroing of out-of-range rows waits for store(), so
  // nothing consumes the loaded registers before the tile is staged -- a select right
  // behind each load made the compiler wait for it there and serialised the prefetch.
  // A short last group has whole tiles past rows_total: their base is clamped to `ens`
  // (every lane then loads ens[0], which exists since N*M > 0), so no address outside
  // [ens, ens + N*M*F) is ever formed.
  __device__ __forceinline__ uint32_t load(float (&v)[PER], const float* __restrict__ ens,
                                           int64_t row0, int64_t rows_total, int F,
                                           int half_lim) const {
    const int64_t d = rows_total - row0;
    const int lim = d <= 0 ? 0 : (d > 0x7fffffff ? 0x7fffffff : (int)d);
    const float* __restrict__ base = lim > 0 ? ens + row0 * F : ens;
    uint32_t ok = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      bool in = row[i] < lim;
      if constexpr (PAD) in = in && (int)jrow[i] < half_lim;
      const int off = in ? src[i] : 0;
#ifdef GINE_BOUNDS_CHECK
      const int64_t a = (base - ens) + off;
      if (a < 0 || a >= rows_total * F) {
        printf("GINE_BOUNDS_CHECK deepset Stager::load: block %d thread %d reads ens[%lld] "
               "outside [0, %lld)\n", (int)blockIdx.x, (int)threadIdx.x, (long long)a,
               (long long)(rows_total * F));
        __builtin_trap();
      }
#endif
      v[i] = base[off];
      ok |= (in ? 1u : 0u) << i;
    }
    return ok;
  }
  __device__ __forceinline__ void store(float* s_e, const float (&v)[PER], uint32_t ok) const {
    if constexpr (X3) {
      constexpr int PL = kPlane;
      uint16_t* img = reinterpret_cast<uint16_t*>(s_e);
#pragma unroll
      for (int i = 0; i < PER; i += 2) {  // values split in pairs (v_cvt_pk_bf16_f32)
        const int i1 = i + 1 < PER ? i + 1 : i;
        const float a = ((ok >> i) & 1u) ? v[i] : 0.f;
        const float b = ((ok >> i1) & 1u) ? v[i1] : 0.f;
        uint32_t ph, pm, pl;
        split2(a, b, ph, pm, pl);
        if (kBranchless || dst[i] >= 0) {
          img[dst[i]] = (uint16_t)ph;
          img[PL + dst[i]] = (uint16_t)pm;
          img[2 * PL + dst[i]] = (uint16_t)pl;
        }
        if (i + 1 < PER && (kBranchless || dst[i1] >= 0)) {
          img[dst[i1]] = (uint16_t)(ph >> 16);
          img[PL + dst[i1]] = (uint16_t)(pm >> 16);
          img[2 * PL + dst[i1]] = (uint16_t)(pl >> 16);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (kBranchless || dst[i] >= 0) s_e[dst[i]] = ((ok >> i) & 1u) ? v[i] : 0.f;
    }
  }
};

template <int KP>
__device__ __forceinline__ void zero_pad(float* s_e, int F) {
  constexpr int LD = KP + 4;
  for (int i = threadIdx.x; i < 32 * (LD - F); i += blockDim.x) {
    const int r = i / (LD - F), c = F + i % (LD - F);
    s_e[r * LD + c] = 0.f;
  }
}
// The planes' columns F.. of every row (never written by the stager)
template <int KP>
__device__ __forceinline__ void zero_pad_x3(float* s_e, int F) {
  using I = DsImg<KP>;
  uint16_t* img = reinterpret_cast<uint16_t*>(s_e);
  const int w = I::RS - F;
  for (int i = threadIdx.x; i < 3 * 32 * w; i += blockDim.x) {
    const int pr = i / w, c = F + i % w;  // pr = plane * 32 + row
    img[pr * I::RS + c] = 0;
  }
}

// Pre-activation chain of one 32-row tile for this wave's 32 hidden units.
template <int KP>
__device__ __forceinline__ floatx16 pre_tile(const float* s_e, const float (&bf)[KP / 2],
                                             int c32, int h) {
  constexpr int LD = KP + 4;
  constexpr int KS = KP / 2;
  floatx16 acc = zero16();
  const float* arow = s_e + staged_row(c32) * LD + h * KS;
#pragma unroll
  for (int q = 0; q < KS / 4; ++q) {
    const float4 a4 = *reinterpret_cast<const float4*>(arow + 4 * q);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, bf[4 * q], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, bf[4 * q + 1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, bf[4 * q + 2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, bf[4 * q + 3], acc, 0, 0, 0);
  }
  return acc;
}

// The split chain: A fragments (ds_read_b128 of 8 k per plane) from the tile's planes, B =
// W1's register planes (wb[b]: k = 16b + 8h + j of this lane's column).
template <int KP>
__device__ __forceinline__ floatx16 pre_tile_x3(const float* s_e,
                                                const Bf16x3 (&wb)[DsImg<KP>::KX / 16],
                                                int c32, int h) {
  using I = DsImg<KP>;
  const uint16_t* img = reinterpret_cast<const uint16_t*>(s_e) + staged_row(c32) * I::RS + 8 * h;
  floatx16 acc = zero16();
#pragma unroll
  for (int b = 0; b < I::KX / 16; ++b) {
    Bf16x3 a;
    a.h = *reinterpret_cast<const bf16x8_t*>(img + 16 * b);
    a.m = *reinterpret_cast<const bf16x8_t*>(img + I::PLANE + 16 * b);
    a.l = *reinterpret_cast<const bf16x8_t*>(img + 2 * I::PLANE + 16 * b);
    acc = mfma_bf16x3(a, wb[b], acc);
  }
  return acc;
}
template <int KP>
__device__ __forceinline__ void load_b_x3(const float* __restrict__ w1, int col, int h, int F,
                                          Bf16x3 (&wb)[DsImg<KP>::KX / 16]) {
#pragma unroll
  for (int b = 0; b < DsImg<KP>::KX / 16; ++b) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * b + 8 * h + j;
      v[j] = k < F ? w1[(size_t)col * F + k] : 0.f;
    }
    wb[b] = split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
  }
}
// The rare path: this wave's tile on the fp32 chain, A rows and W1 read from global memory
// (same operands and k order as pre_tile, so the same bits as the fp32 form).
template <int KP>
__device__ __noinline__ floatx16 pre_tile_mem(const float* __restrict__ ens,
                                              const float* __restrict__ w1, int64_t row0,
                                              int64_t rows_total, int GM, int half_lim, int F,
                                              int col, int c32, int h) {
  constexpr int KS = KP / 2;
  const int tr = staged_row(c32), c = tr >> 4, j = tr & 15;
  const int64_t grow = row0 + (int64_t)c * GM + j;
  const bool valid = grow < rows_total && j < half_lim;
  floatx16 acc = zero16();
#pragma unroll 1
  for (int s = 0; s < KS; ++s) {
    const int k = h * KS + s;
    const float a = (valid && k < F) ? ens[grow * F + k] : 0.f;
    const float b = k < F ? w1[(size_t)col * F + k] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  return acc;
}

template <int KP>
__device__ __forceinline__ void load_b(const float* __restrict__ w1, int col, int h, int F,
                                       float (&bf)[KP / 2]) {
  constexpr int KS = KP / 2;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = h * KS + s;
    bf[s] = k < F ? w1[(size_t)col * F + k] : 0.f;
  }
}

// The groups of this workgroup: each XCD owns a contiguous range of groups proportional to
// the number of workgroups it holds (blocks are dealt round-robin over the XCDs), walked by
// its workgroups with stride = that number.
struct Groups {
  int first, step, end;
  // nb: the walking workgroups; b: this one's index among them (blockIdx.x unless other
  // workgroups are dealt first -- a multiple of kNumXcd of them keeps the XCD of each)
  __device__ __forceinline__ Groups(int num_groups, int nb, int b = (int)blockIdx.x) {
    const int xcd = b % kNumXcd, pos = b / kNumXcd;
    const int q = nb / kNumXcd, rm = nb % kNumXcd;
    const int here = q + (xcd < rm ? 1 : 0);
    const int before = xcd * q + min(xcd, rm);  // workgroups on lower XCDs
    const int lo = (int)((int64_t)num_groups * before / nb);
    end = (int)((int64_t)num_groups * (before + here) / nb);
    first = lo + pos;
    step = here;
  }
};

// Position of a tile in the flat walk over (group, tile-in-group), advanced incrementally.
struct Cursor {
  int g, t;     // group index, tile within the group
  int64_t row;  // first group row of the tile: g*2G*M + 16*t
  __device__ __forceinline__ void start(int g0, int GM) {
    g = g0;
    t = 0;
    row = (int64_t)g0 * 2 * GM;
  }
  __device__ __forceinline__ void advance(int GM, int tpg, int step) {
    if (++t == tpg) {
      t = 0;
      g += step;
      row = (int64_t)g * 2 * GM;
    } else {
      row += 16;
    }
  }
};

// Drive `tile(cursor, buf, mbits)` over the workgroup's tiles with a two-deep register ring
// and a double-buffered LDS tile: tile k+2 is loaded while tile k computes, tile k+1 is
// stored after it, one barrier per tile.  With `mask_in`, each thread's 16-bit ReLU mask
// word of the tile rides in the same ring (registers only: a thread reads its own word).
// UNCOND (the backward): the ring loads past the walk's last tile reload the current tile
// (never consumed) instead of being skipped, so no register merge at the loop's back edge
// waits for them (backward 41.4 -> 39.0 us at 16,000 nodes; the forward, whose ring holds
// no mask word, runs 0.9 us slower that way: profiles/r03_s35).
template <bool UNCOND, bool MASKIN, int NT, int KP, bool PAD, bool X3, int KI, bool BWD,
          class Body>
__device__ __forceinline__ void walk_tiles(const Groups& gr, int GM, int tpg,
                                           const Stager<NT, KP, PAD, X3, KI, BWD>& st,
                                           const float* __restrict__ ens, int64_t rows_total,
                                           int F, float* buf0, float* buf1,
                                           const uint16_t* __restrict__ mask_in, Body&& tile) {
  constexpr int PER = Stager<NT, KP, PAD, X3, KI, BWD>::PER;
  if (gr.first >= gr.end) return;
  const int count = ((gr.end - gr.first + gr.step - 1) / gr.step) * tpg;
  Cursor cur, pf;  // tile being computed, tile being loaded
  cur.start(gr.first, GM);
  pf = cur;
  // the mask ring is a compile-time property of the walk: a run-time null test made the
  // mask load conditional, and the s_waitcnt at the staging store below then assumed the
  // path without it -- waiting for the first load of tile k+2, i.e. a one-deep ring
  auto mload = [&](const Cursor& c) -> uint32_t {
    if constexpr (MASKIN) return (uint32_t)mask_in[((int64_t)c.g * tpg + c.t) * NT + threadIdx.x];
    else return 0u;
  };
  auto sload = [&](float (&v)[PER], const Cursor& c) -> uint32_t {
    return st.load(v, ens, c.row, rows_total, F, GM - 16 * c.t);
  };
  float va[PER], vb[PER];
  uint32_t ma = 0, mb = 0, oa = 0, ob = 0;
  oa = sload(va, pf);
  ma = mload(pf);
  st.store(buf0, va, oa);
  if (count > 1) {
    pf.advance(GM, tpg, gr.step);
    ob = sload(vb, pf);
    mb = mload(pf);
  }
  pf.advance(GM, tpg, gr.step);  // pf: tile k+2
  __syncthreads();
  auto step = [&](int k, float (&vcur)[PER], uint32_t& mcur, uint32_t& ocur,
                  float (&vnxt)[PER], uint32_t onxt, float* bcur, float* bnxt) {
    const uint32_t bits = mcur;
    DS_MARK(0);
    if constexpr (UNCOND) {
      const bool more = k + 2 < count;
      ocur = sload(vcur, more ? pf : cur);
      mcur = mload(more ? pf : cur);
    } else if (k + 2 < count) {
      ocur = sload(vcur, pf);
      mcur = mload(pf);
    }
    DS_MARK(1);
    tile(cur, bcur, bits);
    DS_MARK(4);
    if (k + 1 < count) st.store(bnxt, vnxt, onxt);
    DS_MARK(5);
    __syncthreads();
    DS_MARK(6);
    cur.advance(GM, tpg, gr.step);
    pf.advance(GM, tpg, gr.step);
  };
  for (int k = 0; k < count; k += 2) {
    step(k, va, ma, oa, vb, ob, buf0, buf1);
    if (k + 1 < count) step(k + 1, vb, mb, ob, va, oa, buf1, buf0);
  }
}

// ---------------------------------------------------------------------------------------
// Forward.  mask_out (MASK): bit q of word [(g*TPG + t)*NT + thread] = ReLU active for the
// row in accumulator register q (0 for padding rows) -- what the backward needs instead of
// the activation.
// Node sums go to LDS as nodes complete and to HBM once per group (2G nodes): no global
// store sits in a data-dependent branch of the tile loop, so the compiler can count the
// memory operations in flight and the next tiles' loads stay in flight under the MFMAs
// (a conditional store there made it drain the whole queue -- s_waitcnt vmcnt(0) -- every
// tile).
// FOLD (gine_deepset_fwd_fold): the first kFoldBlocks<H> workgroups fold the dense chain's
// dim_red weight (gine_chainfold.hpp) beside the member sums, for the chain's one-launch
// forward that follows.  They are dealt first (so they never wait for a free slot behind the
// walk) and share one LDS buffer with the walk's tiles (so the walk's occupancy is that of
// the larger of the two, not of their sum).
// (experiments) the forward's ring loads unconditional, as the backward's: the compiler then
// waits for the ring at the loop head instead (register reuse), 27.5 vs 27.8 us at 16,000
// nodes and 14.7 vs 13.9 at 4,000 (profiles/r05_s07_ds_ab_ring_branchless.txt): off
#ifndef GINE_DS_FWD_UNCOND
#define GINE_DS_FWD_UNCOND 0
#endif
template <int H, int KP, int G, bool MASK, bool FOLD = false>
__global__ __launch_bounds__(2 * H, 4) void k_deepset_fwd(const float* __restrict__ ens,
                                                       const float* __restrict__ w1,
                                                       const float* __restrict__ b1,
                                                       float* __restrict__ r,
                                                       uint16_t* __restrict__ mask_out,
                                                       int64_t N, int M, int F,
                                                       int num_groups, FoldArgs fold,
                                                       Fold2Args fold2) {
  constexpr int NT = 2 * H;
  // the split chain for the large-batch group size only: at 4,000 nodes (8-node groups) it
  // measured 16.2 against 14.1 us, at 16,000 27.7 against 31.3 (profiles/r04_s15_ds_*.txt)
  constexpr bool X3 = GINE_DS_BF16X3 != 0 && G == 16;
  constexpr int TILEF = X3 ? DsImg<KP>::FLOATS : 32 * (KP + 4);  // one staged tile (floats)
  constexpr int kWalk = 2 * TILEF + 2 * G * H;  // two staged tiles + the group's node sums
  constexpr int kFold = FOLD ? 32 * (H + 4) + (H / 32) * kSR : 0;
  __shared__ __attribute__((aligned(16))) float s_lds[kWalk > kFold ? kWalk : kFold];
  int nbw = gridDim.x, bw = blockIdx.x;  // workgroups walking the groups, this one's index
  if constexpr (FOLD) {
    const int nfold = kFoldBlocks<H> * (fold2.wfold2 != nullptr ? 2 : 1);
    nbw -= nfold;
    bw -= nfold;
    if (bw < 0) {
      const int lane = threadIdx.x % kWave;
      if ((int)blockIdx.x < kFoldBlocks<H>)
        fold_tile<H>(fold, blockIdx.x, s_lds, s_lds + 32 * (H + 4), lane & 31, lane >> 5);
      else
        fold2_tile<H>(fold2, blockIdx.x - kFoldBlocks<H>, s_lds, s_lds + 32 * (H + 4),
                      lane & 31, lane >> 5);
      return;
    }
  }
  float(*s_e)[TILEF] = reinterpret_cast<float(*)[TILEF]>(s_lds);
  float* s_r = s_lds + 2 * TILEF;  // node sums of the current group
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  float bf[X3 ? 1 : KP / 2];
  Bf16x3 wb[X3 ? DsImg<KP>::KX / 16 : 1];
  if constexpr (X3) {
    load_b_x3<KP>(w1, col, h, F, wb);
    zero_pad_x3<KP>(s_e[0], F);
    zero_pad_x3<KP>(s_e[1], F);
  } else {
    load_b<KP>(w1, col, h, F, bf);
    zero_pad<KP>(s_e[0], F);
    zero_pad<KP>(s_e[1], F);
  }
  const float bias = b1[col];

  Stager<NT, KP, G != 16, X3> st;
  st.init(F, M, G);
  const Groups gr(num_groups, nbw, bw);
  const int GM = G * M, tpg = tiles_per_group(G, M);
  float run = 0.f;
  float* s_mine = s_r + (G * h) * H + col;  // this lane's column of its half's G nodes
  // uniform walk state: node (0..G-1 within each half's G; G: padding) and rows left in it
  int node = 0, rem = M;
  walk_tiles<GINE_DS_FWD_UNCOND != 0, false>(gr, GM, tpg, st, ens, N * M, F, s_e[0], s_e[1],
                                             nullptr,
             [&](const Cursor& c, const float* buf, uint32_t) {
    if (c.t == 0) {
      node = 0;
      rem = M;
      run = 0.f;
    }
    floatx16 acc;
    if constexpr (X3) {
      acc = pre_tile_x3<KP>(buf, wb, c32, h);
      if (wave_any_nan(acc))  // non-finite operand: the fp32 chain's result instead
        acc = pre_tile_mem<KP>(ens, w1, c.row, N * M, GM, GM - 16 * c.t, F, col, c32, h);
    } else {
      acc = pre_tile<KP>(buf, bf, c32, h);
    }
    DS_MARK(2 + 0 * (int)acc[15]);
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float v = acc[q] + bias;
      bits |= (v > 0.f ? 1u : 0u) << q;
      run += relu_nan(v);
      // (a branch-free form -- every row storing the running sum to its node's slot --
      // measured 4.4 us slower at 16,000 nodes: profiles/r05_s07_ds_ab_ring_branchless.txt)
      if (--rem == 0) {  // last member of this node: keep its sum
        if (node < G) s_mine[node * H] = run;
        run = 0.f;
        ++node;
        rem = M;
      }
    }
    DS_MARK(3 + 0 * (int)run);
    if (G * M % 16 != 0 && c.t == tpg - 1) {  // padding rows: no ReLU bit
      const int live = GM - 16 * c.t;
      bits &= live >= 16 ? 0xffffu : (1u << live) - 1u;
    }
    if constexpr (MASK) mask_out[((int64_t)c.g * tpg + c.t) * NT + threadIdx.x] = (uint16_t)bits;
    if (c.t == tpg - 1) {  // the group is complete: its 2 x G node sums to HBM
      const int64_t n0 = (int64_t)c.g * 2 * G + G * h;
      const int64_t nvalid = N - n0;
#pragma unroll
      for (int n = 0; n < G; ++n)
        if (n < nvalid) r[(n0 + n) * H + col] = s_mine[n * H];
    }
  });
}

// ---------------------------------------------------------------------------------------
// Backward for the weights from the forward's ReLU mask:
//   dh = dr[node] * mask;  dW1 += dh^T ens;  db1 += sum dh.
// fp32 form: MFMA over 32-feature tiles, A = dh straight from registers, B = staged rows;
// the last F % 32 features as fp32 FMAs.
// Split form (X3): A = dh split into bf16 planes in registers (k-block s, element j of lane
// half h = staged row 16h + 8s + j), B = the staged ens planes, stored column-major by the
// stager, so this lane's 8 rows of its feature are one 16-byte read per plane; all features
// on the matrix cores (the planes are zero past F).  A workgroup whose
// accumulators see a NaN (non-finite ens or dr) writes nothing and runs the fp32 form
// instead, which gives the fp32 result.

template <int H, int KP, int G, bool X3>
__device__ __forceinline__ bool ds_bwd_body(const float* __restrict__ ens,
                                            const uint16_t* __restrict__ mask,
                                            const float* __restrict__ dr,
                                            float* __restrict__ slab, int64_t N, int M, int F,
                                            int num_groups, float* s_lds) {
  constexpr int NT = 2 * H;
  constexpr int KI = ds_bwd_ki(KP);
  using I = DsBwdImg<KI>;
  constexpr int LD = X3 ? I::RS : KP + 4;
  constexpr int TILEF = X3 ? I::FLOATS : 32 * (KP + 4);
  constexpr int NIF = X3 ? KI / 32 : KP / 32;  // 32-wide feature tiles on the matrix cores
  constexpr int TAIL = X3 ? 0 : KP - 32 * NIF; // fp32 form: remaining features (VALU)
  float* s_e0 = s_lds;
  float* s_e1 = s_lds + TILEF;
  float* s_dr = s_lds + 2 * TILEF;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  if constexpr (X3) {  // the feature columns F.. of every plane (never staged)
    uint16_t* i0 = reinterpret_cast<uint16_t*>(s_e0);
    uint16_t* i1 = reinterpret_cast<uint16_t*>(s_e1);
    const int w = (KI - F) * I::RS;
    for (int i = threadIdx.x; i < 3 * w; i += blockDim.x) {
      const int pl = i / w, e = F * I::RS + i % w;
      i0[pl * I::PLANE + e] = 0;
      i1[pl * I::PLANE + e] = 0;
    }
  } else {
    zero_pad<KP>(s_e0, F);
    zero_pad<KP>(s_e1, F);
  }

  floatx16 gw[NIF > 0 ? NIF : 1];
#pragma unroll
  for (int it = 0; it < NIF; ++it) gw[it] = zero16();
  float tw[TAIL > 0 ? TAIL : 1];
#pragma unroll
  for (int j = 0; j < TAIL; ++j) tw[j] = 0.f;
  double gb = 0.0;

  Stager<NT, KP, G != 16, X3, KI, true> st;
  st.init(F, M, G);
  const Groups gr(num_groups, gridDim.x);
  const int GM = G * M, tpg = tiles_per_group(G, M);
  const float* my_dr = s_dr + G * h * H + col;  // this lane: node j of its half at j*H
  int node = 0, rem = M;
  walk_tiles<true, true>(gr, GM, tpg, st, ens, N * M, F, s_e0, s_e1, mask,
             [&](const Cursor& c, const float* buf, uint32_t bits) {
    if (c.t == 0) {  // dr of this group, this wave's columns (read by this wave only)
      const int64_t node0 = (int64_t)c.g * 2 * G;
      // all loads in flight before the first LDS store (clamped rows, zero past N)
      constexpr int kPer = 2 * G * 32 / kWave;
      float v[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int i = lane + j * kWave;
        const int64_t n = node0 + (i >> 5);
        v[j] = dr[(n < N ? n : N - 1) * H + wave * 32 + (i & 31)];
      }
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int i = lane + j * kWave;
        s_dr[(i >> 5) * H + wave * 32 + (i & 31)] = node0 + (i >> 5) < N ? v[j] : 0.f;
      }
      node = 0;
      rem = M;
    }
    float dh[16];
    float gsum = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {  // independent LDS reads, uniform node walk
      const float d = my_dr[(node < G ? node : G - 1) * H];  // 0 for nodes >= N
      const float v = ((bits >> q) & 1u) ? d : 0.f;
      dh[q] = v;
      gsum += v;
      if (--rem == 0) {
        ++node;
        rem = M;
      }
    }
    gb += (double)gsum;
    DS_MARK(2 + 0 * (int)gsum);
    if constexpr (X3) {
      const uint16_t* img = reinterpret_cast<const uint16_t*>(buf);
#pragma unroll
      for (int s8 = 0; s8 < 2; ++s8) {
        const Bf16x3 a = split8(make_float4(dh[8 * s8], dh[8 * s8 + 1], dh[8 * s8 + 2],
                                            dh[8 * s8 + 3]),
                                make_float4(dh[8 * s8 + 4], dh[8 * s8 + 5], dh[8 * s8 + 6],
                                            dh[8 * s8 + 7]));
#pragma unroll
        for (int it = 0; it < NIF; ++it) {  // B: rows 16h + 8s8 .. +7 of feature 32it + c32
          const uint16_t* col = img + (32 * it + c32) * I::RS + 16 * h + 8 * s8;
          Bf16x3 b;
          b.h = *reinterpret_cast<const bf16x8_t*>(col);
          b.m = *reinterpret_cast<const bf16x8_t*>(col + I::PLANE);
          b.l = *reinterpret_cast<const bf16x8_t*>(col + 2 * I::PLANE);
          gw[it] = mfma_bf16x3(a, b, gw[it]);
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float* erow = buf + (16 * h + q) * LD;
#pragma unroll
        for (int it = 0; it < NIF; ++it)
          gw[it] = __builtin_amdgcn_mfma_f32_32x32x2f32(dh[q], erow[32 * it + c32], gw[it], 0,
                                                        0, 0);
#pragma unroll
        for (int j = 0; j < TAIL; j += 4) {
          const float4 e4 = *reinterpret_cast<const float4*>(erow + 32 * NIF + j);
          tw[j] = __builtin_fmaf(dh[q], e4.x, tw[j]);
          tw[j + 1] = __builtin_fmaf(dh[q], e4.y, tw[j + 1]);
          tw[j + 2] = __builtin_fmaf(dh[q], e4.z, tw[j + 2]);
          tw[j + 3] = __builtin_fmaf(dh[q], e4.w, tw[j + 3]);
        }
      }
    }
    DS_MARK(3 + 0 * (int)gw[0][0]);
  });
  if constexpr (X3) {
    bool bad = false;
#pragma unroll
    for (int it = 0; it < NIF; ++it) bad = bad || wave_any_nan(gw[it]);
    if (block_any(bad, reinterpret_cast<int*>(s_e0))) return false;
  }
  // slab row of this workgroup: [H*F weights | H bias]
  float* out = slab + (size_t)blockIdx.x * ((size_t)H * F + H);
#pragma unroll
  for (int it = 0; it < NIF; ++it) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int o = wave * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (32 * it + c32 < F) out[(size_t)o * F + 32 * it + c32] = gw[it][q];
    }
  }
#pragma unroll
  for (int j = 0; j < TAIL; ++j) {
    const float v = tw[j] + __shfl_xor(tw[j], 32, kWave);
    if (h == 0 && 32 * NIF + j < F) out[(size_t)col * F + 32 * NIF + j] = v;
  }
  gb += shfl_xor_d(gb, 32);
  if (h == 0) out[(size_t)H * F + col] = (float)gb;
  return true;
}

// The split backward (GINE_DS_BWD_BF16X3=1) measured no faster than the fp32 one (16,000
// nodes 39.5 vs 40.1 us, 4,000 nodes 22.8 vs 22.0; profiles/r04_s15_ds_*.txt): off.
#ifndef GINE_DS_BWD_BF16X3
#define GINE_DS_BWD_BF16X3 0
#endif
template <int H, int KP, int G>
constexpr int ds_bwd_lds_floats() {
  constexpr int f32 = 2 * 32 * (KP + 4);
  constexpr int x3 = GINE_DS_BWD_BF16X3 ? 2 * DsBwdImg<ds_bwd_ki(KP)>::FLOATS : 0;
  return (f32 > x3 ? f32 : x3) + 2 * G * H;
}

template <int H, int KP, int G>
__global__ __launch_bounds__(2 * H) void k_deepset_bwd(const float* __restrict__ ens,
                                                       const uint16_t* __restrict__ mask,
                                                       const float* __restrict__ dr,
                                                       float* __restrict__ slab, int64_t N,
                                                       int M, int F, int num_groups) {
  __shared__ __attribute__((aligned(16))) float s_lds[ds_bwd_lds_floats<H, KP, G>()];
#if GINE_DS_BWD_BF16X3
  if (ds_bwd_body<H, KP, G, true>(ens, mask, dr, slab, N, M, F, num_groups, s_lds)) return;
  __syncthreads();  // a non-finite operand: the fp32 form
#endif
  ds_bwd_body<H, KP, G, false>(ens, mask, dr, slab, N, M, F, num_groups, s_lds);
}

// 16 consecutive slab elements x 16 chunk groups per workgroup (many workgroups for the
// few thousand elements of dW1), fixed summation order, fp64.
__global__ __launch_bounds__(256) void k_deepset_slab_reduce(const float* __restrict__ slab,
                                                             int chunks, int64_t per,
                                                             int64_t wsize,
                                                             float* __restrict__ dw,
                                                             float* __restrict__ db) {
  __shared__ double s_part[16][17];
  const int j = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t e = blockIdx.x * (int64_t)16 + j;
  double acc = 0.0;
  if (e < per) {
#pragma unroll 4
    for (int c = g; c < chunks; c += 16) acc += (double)slab[(size_t)c * per + e];
  }
  s_part[g][j] = acc;
  __syncthreads();
  if (g != 0 || e >= per) return;
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) v += s_part[k][j];
  if (e < wsize) dw[e] = (float)v;
  else if (db) db[e - wsize] = (float)v;
}

// forward: the MFMA k-split needs KP % 8 == 0; backward: rows stage as float4, KP % 4 == 0
inline int pad_fwd(int F) {
  if (F <= 16) return 16;
  if (F <= 32) return 32;
  if (F <= 40) return 40;
  if (F <= 48) return 48;
  if (F <= 64) return 64;
  return -1;
}
inline int pad_bwd(int F) {
  if (F <= 16) return 16;
  if (F <= 32) return 32;
  if (F <= 36) return 36;
  if (F <= 40) return 40;
  if (F <= 48) return 48;
  if (F <= 64) return 64;
  return -1;
}

inline bool hidden_ok(int H) { return H == 32 || H == 64 || H == 128 || H == 256; }

// Nodes per lane half: 8 while 16 would leave at most one wave per SIMD (H/32 waves per
// group; H = 128: <= 8,192 nodes; at 4,000 nodes forward 21.4 -> 14.8 us, backward 28.4 ->
// 20.9 us); at 16,000 nodes and H = 128 8 is no faster (forward 31.5 vs 33.3 us: two waves
// per SIMD already keep it busy; profiles/r03_s35); at 16,000 nodes and H = 64 forward
// 31.9 -> 22.9 us, backward (1,000 partials) 38.6 -> 32.7 us (profiles/r03_s38, r03_s39).
// G = 4 at a quarter wave per SIMD or less, i.e. N <= 2,048 nodes at H = 128 and <= 4,096 at
// H = 64 (cfg1's single 500-station graph: forward / backward 13.1 / 17.1 -> 8.6 / 12.9 us,
// profiles/r03_s42).  The earlier bound of half a wave per SIMD also put 4,000-node batches
// at H = 128 on G = 4, where the backward measured slower (21.5 -> 22.4 us), so it stops
// below that size.
#ifndef GINE_DS_G8_WAVES  // (experiments)
#define GINE_DS_G8_WAVES 1024
#endif
inline int nodes_per_half(int64_t N, int H) {
  const int64_t waves16 = ceil_div(N > 0 ? N : 1, 32) * (H / 32);
  return waves16 <= 256 ? 4 : (waves16 <= GINE_DS_G8_WAVES ? 8 : 16);
}
inline int num_groups(int64_t N, int H) {
  return (int)ceil_div(N > 0 ? N : 1, 2 * nodes_per_half(N, H));
}
// Backward partials (slab rows): one per group up to 512 (H >= 128) or 1,024 (H <= 64: the
// same slab bytes) workgroups; a smaller grid walks several groups per workgroup.
inline int bwd_grid(int64_t N, int H) {
  return std::min(num_groups(N, H), H >= 128 ? 512 : 1024);
}

#define DS_FWD_KP(H_, KP_, MACRO)                         \
  switch (KP_) {                                          \
    case 16: MACRO(H_, 16); break;                        \
    case 32: MACRO(H_, 32); break;                        \
    case 40: MACRO(H_, 40); break;                        \
    case 48: MACRO(H_, 48); break;                        \
    default: MACRO(H_, 64); break;                        \
  }

#define DS_BWD_KP(H_, KP_, MACRO)                         \
  switch (KP_) {                                          \
    case 16: MACRO(H_, 16); break;                        \
    case 32: MACRO(H_, 32); break;                        \
    case 36: MACRO(H_, 36); break;                        \
    case 40: MACRO(H_, 40); break;                        \
    case 48: MACRO(H_, 48); break;                        \
    default: MACRO(H_, 64); break;                        \
  }

#define DS_DISPATCH_H(H, KP, KPSWITCH, MACRO)             \
  switch (H) {                                            \
    case 32: KPSWITCH(32, KP, MACRO); break;              \
    case 64: KPSWITCH(64, KP, MACRO); break;              \
    case 128: KPSWITCH(128, KP, MACRO); break;            \
    default: KPSWITCH(256, KP, MACRO); break;             \
  }

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_deepset_mask_bytes(int64_t num_nodes, int32_t members, int32_t hidden,
                                       size_t* bytes) {
  if (!bytes || num_nodes < 0 || members <= 0 || !hidden_ok(hidden)) return GINE_ERR_INVALID;
  const int G = nodes_per_half(num_nodes, hidden);
  *bytes = num_nodes == 0 ? 0
                          : (size_t)num_groups(num_nodes, hidden) * tiles_per_group(G, members) * 2 *
                                hidden * sizeof(uint16_t);
  return GINE_OK;
}

extern "C" int gine_deepset_mask_layout(int64_t num_nodes, int32_t hidden,
                                        int32_t* nodes_per_half_out) {
  if (!nodes_per_half_out || num_nodes < 0 || !hidden_ok(hidden)) return GINE_ERR_INVALID;
  *nodes_per_half_out = nodes_per_half(num_nodes, hidden);
  return GINE_OK;
}

extern "C" int gine_deepset_fwd(const float* ens, const float* w1, const float* b1, float* r,
                                uint16_t* mask, int64_t num_nodes, int32_t members,
                                int32_t in_features, int32_t hidden, void* stream) {
  const int KP = pad_fwd(in_features);
  if (!hidden_ok(hidden) || KP < 0 || in_features <= 0) return GINE_ERR_DIM;
  if (num_nodes < 0 || members <= 0) return GINE_ERR_INVALID;
  if (num_nodes == 0) return GINE_OK;
  if (!ens || !w1 || !b1 || !r) return GINE_ERR_INVALID;
  if (num_nodes * members >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  const int groups = num_groups(num_nodes, hidden);
  const int grid = std::min(groups, 1024);
  const int G = nodes_per_half(num_nodes, hidden);
  hipStream_t s = as_stream(stream);
#define LAUNCH_FWD_M(H_, KP_, G_, MK_)                                                        \
  hipLaunchKernelGGL((k_deepset_fwd<H_, KP_, G_, MK_>), dim3(grid), dim3(2 * H_), 0, s, ens, w1, \
                     b1, r, mask, num_nodes, members, in_features, groups, FoldArgs{},       \
                     Fold2Args{})
#define LAUNCH_FWD_G(H_, KP_, G_)                             \
  do {                                                        \
    if (mask) LAUNCH_FWD_M(H_, KP_, G_, true);                \
    else LAUNCH_FWD_M(H_, KP_, G_, false);                    \
  } while (0)
#define LAUNCH_FWD(H_, KP_)                                   \
  do {                                                        \
    if (G == 4) LAUNCH_FWD_G(H_, KP_, 4);                     \
    else if (G == 8) LAUNCH_FWD_G(H_, KP_, 8);                \
    else LAUNCH_FWD_G(H_, KP_, 16);                           \
  } while (0)
  DS_DISPATCH_H(hidden, KP, DS_FWD_KP, LAUNCH_FWD);
#undef LAUNCH_FWD
#undef LAUNCH_FWD_G
#undef LAUNCH_FWD_M
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_deepset_bwd_num_partials(int64_t num_nodes, int32_t hidden,
                                             int32_t* num_partials) {
  if (!num_partials || num_nodes < 0) return GINE_ERR_INVALID;
  if (!hidden_ok(hidden)) return GINE_ERR_DIM;
  *num_partials = bwd_grid(num_nodes, hidden);
  return GINE_OK;
}

extern "C" int gine_deepset_bwd(const float* ens, const uint16_t* mask, const float* dr,
                                float* slab, float* dw1, float* db1, int64_t num_nodes,
                                int32_t members, int32_t in_features, int32_t hidden,
                                void* stream) {
  const int KP = pad_bwd(in_features);
  if (!hidden_ok(hidden) || KP < 0 || in_features <= 0) return GINE_ERR_DIM;
  if (num_nodes < 0 || members <= 0 || !slab) return GINE_ERR_INVALID;
  if (num_nodes > 0 && (!ens || !mask || !dr)) return GINE_ERR_INVALID;
  if (num_nodes * members >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  const int groups = num_groups(num_nodes, hidden);
  const int grid = bwd_grid(num_nodes, hidden);
  const int G = nodes_per_half(num_nodes, hidden);
  const int64_t per = (int64_t)hidden * in_features + hidden;
  hipStream_t s = as_stream(stream);
  if (num_nodes == 0) {
    GINE_RETURN_IF_HIP(hipMemsetAsync(slab, 0, sizeof(float) * per * grid, s));
  } else {
#define LAUNCH_BWD_G(H_, KP_, G_)                                                             \
  hipLaunchKernelGGL((k_deepset_bwd<H_, KP_, G_>), dim3(grid), dim3(2 * H_), 0, s, ens, mask,  \
                     dr, slab, num_nodes, members, in_features, groups)
#define LAUNCH_BWD(H_, KP_)                       \
  do {                                            \
    if (G == 4) LAUNCH_BWD_G(H_, KP_, 4);         \
    else if (G == 8) LAUNCH_BWD_G(H_, KP_, 8);    \
    else LAUNCH_BWD_G(H_, KP_, 16);               \
  } while (0)
    DS_DISPATCH_H(hidden, KP, DS_BWD_KP, LAUNCH_BWD);
#undef LAUNCH_BWD
#undef LAUNCH_BWD_G
    GINE_LAUNCH_STATUS();
  }
  if (!dw1) return GINE_OK;  // slab left for gine_grad_finalize_batch
  hipLaunchKernelGGL(k_deepset_slab_reduce, dim3((unsigned)ceil_div(per, 16)), dim3(256), 0, s,
                     slab, grid, per, (int64_t)hidden * in_features, dw1, db1);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

extern "C" int gine_deepset_bwd_grad_job(int64_t num_nodes, int32_t in_features, int32_t hidden,
                                         const float* slab, float* dw1, float* db1,
                                         gine_grad_job* job) {
  if (!hidden_ok(hidden) || pad_bwd(in_features) < 0 || in_features <= 0) return GINE_ERR_DIM;
  if (num_nodes < 0 || !slab || !dw1 || !job) return GINE_ERR_INVALID;
  const int64_t per = (int64_t)hidden * in_features + hidden;
  *job = gine_grad_job{};
  job->kind = GINE_GRAD_JOB_SLAB;
  job->src = slab;
  job->rows = bwd_grid(num_nodes, hidden);
  job->cstride = per;
  job->nz = 1;
  job->per[0] = per;
  job->wsize[0] = (int64_t)hidden * in_features;
  job->w[0] = dw1;
  job->b[0] = db1;
  job->bscale[0] = 1.0f;
  return GINE_OK;
}

#ifdef GINE_DS_PROFILE
extern "C" int gine_debug_ds_prof(long long* out, int* n) {
  GINE_RETURN_IF_HIP(hipDeviceSynchronize());
  GINE_RETURN_IF_HIP(hipMemcpyFromSymbol(n, HIP_SYMBOL(g_ds_prof_n), sizeof(int)));
  GINE_RETURN_IF_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ds_prof), sizeof(long long) * 4096));
  const int zero = 0;
  GINE_RETURN_IF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ds_prof_n), &zero, sizeof(int)));
  return GINE_OK;
}
#endif

namespace {
int deepset_fwd_fold(const float* ens, const float* w1, const float* b1, float* r,
                     uint16_t* mask, int64_t num_nodes, int32_t members, int32_t in_features,
                     int32_t hidden, const FoldArgs& fold, const Fold2Args& fold2,
                     void* stream) {
  const int KP = pad_fwd(in_features);
  if ((hidden != 64 && hidden != 128) || KP < 0 || in_features <= 0) return GINE_ERR_DIM;
  if (fold.F < 1 || fold.F > 64) return GINE_ERR_DIM;
  if (num_nodes < 0 || members <= 0) return GINE_ERR_INVALID;
  if (!fold.fw_r1 || !fold.fb_r1 || !fold.fw_dr || !fold.fb_dr || !fold.wfold)
    return GINE_ERR_INVALID;
  if (num_nodes > 0 && (!ens || !w1 || !b1 || !r)) return GINE_ERR_INVALID;
  if (num_nodes * members >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  const int groups = num_groups(num_nodes, hidden);
  const int walk = num_nodes > 0 ? std::min(groups, 1024) : 0;
  const int G = nodes_per_half(num_nodes, hidden);
  const int nfold = (hidden == 64 ? kFoldBlocks<64> : kFoldBlocks<128>) *
                    (fold2.wfold2 != nullptr ? 2 : 1);
  hipStream_t s = as_stream(stream);
#define LAUNCH_FWD_F(H_, KP_, G_, MK_)                                                        \
  hipLaunchKernelGGL((k_deepset_fwd<H_, KP_, G_, MK_, true>), dim3(walk + nfold),             \
                     dim3(2 * H_), 0, s, ens, w1, b1, r, mask, num_nodes, members, in_features, \
                     groups, fold, fold2)
#define LAUNCH_FWD_G(H_, KP_, G_)                             \
  do {                                                        \
    if (mask) LAUNCH_FWD_F(H_, KP_, G_, true);                \
    else LAUNCH_FWD_F(H_, KP_, G_, false);                    \
  } while (0)
#define LAUNCH_FWD(H_, KP_)                                   \
  do {                                                        \
    if (G == 4) LAUNCH_FWD_G(H_, KP_, 4);                     \
    else if (G == 8) LAUNCH_FWD_G(H_, KP_, 8);                \
    else LAUNCH_FWD_G(H_, KP_, 16);                           \
  } while (0)
  if (hidden == 64) {
    DS_FWD_KP(64, KP, LAUNCH_FWD);
  } else {
    DS_FWD_KP(128, KP, LAUNCH_FWD);
  }
#undef LAUNCH_FWD
#undef LAUNCH_FWD_G
#undef LAUNCH_FWD_F
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
}  // namespace

extern "C" int gine_deepset_fwd_fold(const float* ens, const float* w1, const float* b1,
                                     float* r, uint16_t* mask, int64_t num_nodes,
                                     int32_t members, int32_t in_features, int32_t hidden,
                                     const float* wr1, const float* br1, const float* wdr,
                                     const float* bdr, float* wfold, int32_t x_features,
                                     void* stream) {
  return deepset_fwd_fold(ens, w1, b1, r, mask, num_nodes, members, in_features, hidden,
                          FoldArgs{wr1, br1, wdr, bdr, wfold, x_features}, Fold2Args{},
                          stream);
}

extern "C" int gine_deepset_fwd_fold2(const float* ens, const float* w1, const float* b1,
                                      float* r, uint16_t* mask, int64_t num_nodes,
                                      int32_t members, int32_t in_features, int32_t hidden,
                                      const float* wr1, const float* br1, const float* wdr,
                                      const float* bdr, float* wfold, int32_t x_features,
                                      const float* wr0, const float* br0, const float* wp2,
                                      const float* bp2, float* wfold2, void* stream) {
  if (!wr0 || !br0 || !wp2 || !bp2 || !wfold2) return GINE_ERR_INVALID;
  return deepset_fwd_fold(ens, w1, b1, r, mask, num_nodes, members, in_features, hidden,
                          FoldArgs{wr1, br1, wdr, bdr, wfold, x_features},
                          Fold2Args{wr0, br0, wp2, bp2, (float)members, wfold2}, stream);
}
