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
#include "gine_chainfold.hpp"

#include <algorithm>

namespace gine {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kRowTile = 32;
#ifndef GINE_CHAIN_EP_EARLY
#define GINE_CHAIN_EP_EARLY 1
#endif

#ifdef GINE_CHAIN_PROFILE
// Debug build only (make variant V=chainprof VSRC=gine_chain.hip VDEFS=-DGINE_CHAIN_PROFILE,
// tools/chain_prof.py): thread 0 of every workgroup of the two-stage chain kernels stamps
// s_memtime: 0 entry, 1 weight fragments issued, then per tile k < 2 at 2 + 4k: A tile
// staged (after the barrier), 3 + 4k: stage 1 done, 4 + 4k: stage-2 A tile complete (after
// the barrier), 5 + 4k: stage 2 done; 10 end; 11 / 12: s_memrealtime at entry / end.
__device__ long long g_chain_prof[1024][16];
#define CHAIN_MARK(i)                                                          \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 1024)                                 \
      g_chain_prof[blockIdx.x][i] = (long long)__builtin_amdgcn_s_memtime();  \
  } while (0)
#define CHAIN_RT(i)                                                            \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 1024)                                 \
      g_chain_prof[blockIdx.x][i] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define CHAIN_MARK(i) do {} while (0)
#define CHAIN_RT(i) do {} while (0)
#endif

// F2F / B1F: the one-stage kernels of the folded chain (rho[2] folded into dim_red, see
// gine_chain_fwd_folded): F2F h0 = [x | u] W'^T + b', B1F dt = (dh0 Wc) * 1[u > 0].
// B3: the folded chain's whole input-gradient backward in one launch (B1F's stage, then B2's
// two: dt -> ds -> dr, each stage's output the next one's A tile in LDS).
// F3: the folded chain's whole forward in one launch (s -> u -> h0 = [x | u] W'^T + b',
// with W' folded beforehand by gine_deepset_fwd_fold).
// F2D / B2D: the doubly folded chain (gine_chain_fwd_folded2): phi[2] folded into rho[0]
// as well (Wf = Wr0 Wp2, bf = M Wr0 bp2 + br0, gine_deepset_fwd_fold2), F2D: u = relu(r Wf^T
// + bf) -> h0 = [x | u] W'^T + b', B2D: dt = (dh0 Wc) * 1[u > 0] -> dr = dt Wf.
enum ChainKind {
  CH_F1 = 0, CH_F2 = 1, CH_B1 = 2, CH_B2 = 3, CH_F2F = 4, CH_B1F = 5, CH_B3 = 6, CH_F3 = 7,
  CH_F2D = 8, CH_B2D = 9
};

struct ChainArgs {
  const float* in;   // stage-1 A rows [N, D]: r | u | dh0 | dt | u (F2F) | dh0 (B1F)
  const float* x;    // F2 / F2F: node features [N, F]
  const float* aux;  // B1 / B1F: u (ReLU mask of rho[1])
  const float* w1;   // stage-1 weight (B1F: W')
  const float* b1;   // stage-1 bias (forward)
  const float* w2;   // stage-2 weight (F2F: W')
  const float* b2;   // stage-2 bias (forward; F2F: b')
  float* out1;       // stage-1 output [N, D]: s | e | de | ds
  float* out2;       // stage-2 output [N, D]: u | h0 | dt | dr
  float bias1_scale; // F1: M (phi[2]'s bias summed over members)
  int F;             // F2 / B1: dim_red's x width
  // F1 of the folded chain: W' = [Wdr_x | Wdr_e Wr1] and b' = Wdr_e br1 + bdr into wfold
  // ([D][F + D] then [D]) once the tiles are done (NULL: not folded)
  const float *fw_r1, *fb_r1, *fw_dr, *fb_dr;
  float* wfold;
  const float* w3;  // B3: stage-3 weight (Wp2); F3 / F2D: W'^T
  float* out3;      // B3: stage-3 output (dr); F3 / F2D: h0
  const float* b3;  // F3 / F2D: b'
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
// The same in 16-byte vectors (W 16-byte aligned, ldw % 4 == 0): a lane's fragment is
// KS consecutive floats of one row of W, so a wave's load touches 64 rows either way, but
// with a quarter of the load instructions (measured: the scalar form costs ~0.05 us per
// instruction and workgroup in the chain kernels).
template <int K>
__device__ __forceinline__ void frag_t4(float (&bf)[K / 2], const float* W, int ldw, int col,
                                        int h) {
  constexpr int KS = K / 2;
  const float4* row = reinterpret_cast<const float4*>(W + (size_t)col * ldw + h * KS);
#pragma unroll
  for (int s = 0; s < KS / 4; ++s) {
    const float4 v = row[s];
    bf[4 * s] = v.x;
    bf[4 * s + 1] = v.y;
    bf[4 * s + 2] = v.z;
    bf[4 * s + 3] = v.w;
  }
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

// The same from W^T [F + D][D] (the folded chain's W'^T): lanes read consecutive columns.
template <int FP, int D>
__device__ __forceinline__ void frag_dimred_t(float (&bf)[(FP + D) / 2], const float* WT, int F,
                                              int col, int h) {
  constexpr int KS = (FP + D) / 2;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = h * KS + s;
    const int c = k < F ? k : (k < FP ? 0 : k - FP + F);
    const float v = WT[(size_t)c * D + col];
    bf[s] = (k >= F && k < FP) ? 0.f : v;
  }
}

// Per-XCD contiguous tile ranges (as k_rowgemm).
struct TileRange {
  int first, end, step;
};
__device__ __forceinline__ TileRange tile_range(int num_tiles, int nb) {
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
  constexpr bool kDimRed = KIND == CH_F2 || KIND == CH_F2F;
  constexpr int K2 = kDimRed ? FP + D : D;          // stage-2 contraction length
  constexpr int LDB = K2 + 4;
  constexpr int BOFF = kDimRed ? FP : 0;            // stage-1 output column offset in sB
  constexpr int ITEMS = kRowTile * D4 / NT;         // 4
  constexpr int RSTEP = NT / D4;                    // 8
  constexpr int XITEMS = (kRowTile * FP + NT - 1) / NT;
  constexpr bool kF3 = KIND == CH_F3;
  constexpr bool kF2D = KIND == CH_F2D, kB2D = KIND == CH_B2D;
  constexpr bool kLast = kF3 || kF2D;               // last stage h0 = [x | u] W'^T + b'
  constexpr bool kMaskIn = KIND == CH_B3 || kB2D;   // stage 1 dt = (dh0 Wc) * 1[u > 0]
  constexpr bool kX = kDimRed || kLast;             // stages x rows
  constexpr int LDC = FP + D + 4;                   // F3 / F2D: last stage's A tile [x | u]
  __shared__ __attribute__((aligned(16))) float sA[kRowTile * LDA];
  __shared__ __attribute__((aligned(16))) float sB[kF2D ? 4 : kRowTile * LDB];
  __shared__ __attribute__((aligned(16))) float sC[kLast ? kRowTile * LDC : 4];

  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  const int q_me = threadIdx.x % D4, r_me = threadIdx.x / D4;
  CHAIN_RT(11);
  CHAIN_MARK(0);
  int nb = gridDim.x;  // chain workgroups
  if constexpr (KIND == CH_F1) {
    if (a.wfold != nullptr) {
      nb -= kFoldBlocks<D>;
      if ((int)blockIdx.x >= nb) {
        fold_tile<D>(FoldArgs{a.fw_r1, a.fb_r1, a.fw_dr, a.fb_dr, a.wfold, a.F},
                     blockIdx.x - nb, sA, sB, c32, h);
        return;
      }
    }
  }

  // both stages' weight fragments, once per workgroup (F2F: stage 2 only, B1F: stage 1)
  float bf1[D / 2], bf2[K2 / 2];
  const bool w16 =
      ((reinterpret_cast<uintptr_t>(a.w1) | reinterpret_cast<uintptr_t>(a.w2)) & 15) == 0;
  if constexpr (KIND == CH_F1 || kF3) {
    if (w16) {
      frag_t4<D>(bf1, a.w1, D, col, h);
      frag_t4<D>(bf2, a.w2, D, col, h);
    } else {
      frag_t<D>(bf1, a.w1, D, col, h);
      frag_t<D>(bf2, a.w2, D, col, h);
    }
  } else if constexpr (kF2D) {
    if (w16) frag_t4<D>(bf1, a.w1, D, col, h);
    else frag_t<D>(bf1, a.w1, D, col, h);
  } else if constexpr (KIND == CH_F2) {
    frag_t<D>(bf1, a.w1, D, col, h);
  } else if constexpr (KIND == CH_B1 || KIND == CH_B1F || kMaskIn) {
    frag_n<D>(bf1, a.w1, a.F + D, a.F, col, h);     // dim_red (B1F / B3: W') weight, e columns
  } else if constexpr (KIND == CH_B2) {
    frag_n<D>(bf1, a.w1, D, 0, col, h);
  }
  if constexpr (KIND == CH_F2) {
    frag_dimred<FP, D>(bf2, a.w2, a.F, col, h);
  } else if constexpr (KIND == CH_F2F) {
    frag_dimred_t<FP, D>(bf2, a.w2, a.F, col, h);  // w2 = W'^T
  } else if constexpr (KIND == CH_B1 || KIND == CH_B2 || kMaskIn) {
    frag_n<D>(bf2, a.w2, D, 0, col, h);   // B2D: w2 = Wf
  }
  float bf3[KIND == CH_B3 ? D / 2 : (kLast ? (FP + D) / 2 : 1)];
  if constexpr (KIND == CH_B3) frag_n<D>(bf3, a.w3, D, 0, col, h);
  if constexpr (kLast) frag_dimred_t<FP, D>(bf3, a.w3, a.F, col, h);  // w3 = W'^T
  float bias1 = 0.f, bias2 = 0.f, bias3 = 0.f;
  if constexpr (KIND == CH_F1 || KIND == CH_F2 || kLast) bias1 = a.b1[col] * a.bias1_scale;
  if constexpr (KIND == CH_F1 || kDimRed || kF3) bias2 = a.b2[col];
  if constexpr (kLast) bias3 = a.b3[col];
  CHAIN_MARK(1);

  auto load_tile = [&](int tile, float4 (&raw)[ITEMS], float (&xr)[XITEMS]) {
    const int64_t n0 = (int64_t)tile * kRowTile;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      int64_t n = n0 + r_me + i * RSTEP;
      n = n < N ? n : N - 1;  // clamped: always issued
      raw[i] = reinterpret_cast<const float4*>(a.in + n * D)[q_me];
    }
    if constexpr (kX) {
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

  const TileRange tr = tile_range(num_tiles, nb);
  float4 raw[ITEMS];
  float xr[XITEMS];
  if (tr.first < tr.end) load_tile(tr.first, raw, xr);
  int kt = 0;  // (profile stamps) tile index of this workgroup
  for (int tile = tr.first; tile < tr.end; tile += tr.step, ++kt) {
    const int64_t n0 = (int64_t)tile * kRowTile;
    float ep[16];
    if constexpr ((KIND == CH_B1 || KIND == CH_B1F || kMaskIn) && GINE_CHAIN_EP_EARLY) {
      // the ReLU mask, in flight under the staging and stage 1 -- issued before the next
      // tile's rows, so the epilogue's wait for it (vector-memory counts retire in order)
      // does not also wait for that prefetch
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int64_t n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        n = n < N ? n : N - 1;
        ep[r] = a.aux[n * D + col];
      }
    }
    __syncthreads();  // previous tile's reads of sA / sB are done
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int r = r_me + i * RSTEP;
      const float4 v = (n0 + r < N) ? raw[i] : f4_zero();
      float* dst = KIND == CH_F2F ? &sB[r * LDB + BOFF + 4 * q_me] : &sA[r * LDA + 4 * q_me];
      *reinterpret_cast<float4*>(dst) = v;
    }
    if constexpr (kX) {
      float* sx = kLast ? sC : sB;
      constexpr int LDX = kLast ? LDC : LDB;
#pragma unroll
      for (int i = 0; i < XITEMS; ++i) {
        const int idx = threadIdx.x + i * NT;
        if (idx < kRowTile * FP) sx[(idx / FP) * LDX + idx % FP] = idx % FP < a.F ? xr[i] : 0.f;
      }
    }
    __syncthreads();
    if (kt < 2) CHAIN_MARK(2 + 4 * kt);
    if (tile + tr.step < tr.end) load_tile(tile + tr.step, raw, xr);  // next tile in flight
    if constexpr ((KIND == CH_B1 || KIND == CH_B1F || kMaskIn) && !GINE_CHAIN_EP_EARLY) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {  // (A/B builds: the mask behind the prefetch)
        int64_t n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        n = n < N ? n : N - 1;
        ep[r] = a.aux[n * D + col];
      }
    }

    floatx16 acc;
    if constexpr (KIND == CH_B1F) {  // the one stage: dt = (dh0 Wc) * 1[u > 0]
      acc = tile_mma<D>(sA, LDA, bf1, c32, h);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = ep[r] > 0.f ? acc[r] : 0.f;
        if (n < N) a.out2[n * D + col] = v;
      }
      continue;
    }
    if constexpr (KIND != CH_F2F) {  // stage 1
      acc = tile_mma<D>(sA, LDA, bf1, c32, h);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t n = n0 + rr;
        float v = acc[r] + bias1;
        if constexpr (kMaskIn) v = ep[r] > 0.f ? acc[r] : 0.f;  // dt = du * 1[u > 0]
        if constexpr (kF2D) {
          v = relu_nan(v);                                       // u = relu(r Wf^T + bf)
          sC[rr * LDC + FP + col] = v;                           // the last stage's A tile
        } else {
          sB[rr * LDB + BOFF + col] = v;
        }
        if (n < N) a.out1[n * D + col] = v;
      }
      if (kt < 2) CHAIN_MARK(3 + 4 * kt);
      __syncthreads();
      if (kt < 2) CHAIN_MARK(4 + 4 * kt);
    }

    // stage 2
    if constexpr (!kF2D) {
      acc = tile_mma<K2>(sB, LDB, bf2, c32, h);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t n = n0 + rr;
        float v = acc[r] + bias2;
        if constexpr (KIND == CH_F1 || kF3) v = relu_nan(v);      // u = relu(rho[0](s))
        if constexpr (kF3) sC[rr * LDC + FP + col] = v;           // stage 3's A tile
        if constexpr (KIND == CH_B1) v = ep[r] > 0.f ? v : 0.f;   // dt = du * 1[u > 0]
        if constexpr (KIND == CH_B3) sA[rr * LDA + col] = v;      // stage 3's A tile
        if (n < N) a.out2[n * D + col] = v;
      }
    }
    if constexpr (kLast) {  // last stage: h0 = [x | u] W'^T + b'
      if constexpr (kF3) __syncthreads();
      acc = tile_mma<FP + D>(sC, LDC, bf3, c32, h);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (n < N) a.out3[n * D + col] = acc[r] + bias3;
      }
      if (kt < 2) CHAIN_MARK(5 + 4 * kt);
    }
    if constexpr (KIND == CH_B3) {  // stage 3: dr = ds Wp2 (sA: every wave is past stage 1)
      __syncthreads();
      acc = tile_mma<D>(sA, LDA, bf3, c32, h);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (n < N) a.out3[n * D + col] = acc[r];
      }
    }
    if constexpr (!kLast)
      if (kt < 2) CHAIN_MARK(5 + 4 * kt);
  }
  CHAIN_MARK(10);
  CHAIN_RT(12);
}

// ---------------------------------------------------------------------------------------
// The doubly folded chain's two row stages on the bf16 matrix cores (gine_bf16x3.hpp split
// form, fp32-class products):
//   FWD  (F2D): u  = relu(r Wf^T + bf)        -> h0 = [x | u] W'^T + b'
//   !FWD (B2D): dt = (dh0 Wc) * 1[u > 0]      -> dr = dt Wf
// k_chain's F2D / B2D ran both stages on v_mfma_f32_32x32x2_f32: at one wave per SIMD, K = 128
// costs 64 x 64 = 4,096 MFMA cycles per 32x32 block, against 8 x 192 = 1,536 for the split
// chain.  Both weights are split once per workgroup into register planes (BPlanes); every
// A tile is split once, by the threads that stage it, into three bf16 planes in LDS (the
// stage-1 input from HBM, x beside it; stage 1's output by the lanes that produce it, one
// bf16 per plane), so the chains only read fragments (tools/chain_micro.py: a block with
// pre-split planes 2,046 ticks, split in the loop 3,081).  x's columns are padded to a
// multiple of 16 (FPX) so both stages run whole K = 16 blocks.  A wave whose accumulators
// see a NaN (a non-finite input or weight) redoes its tile on the fp32 chain from memory:
// non-finite values propagate as in the fp32 GEMM.  Same tile walk, grid and outputs as
// k_chain.
// Measured (profiles/r06_s21): correct (the chain, training and head tests green on it) but
// SLOWER in the step -- forward 23.4 vs 20.4 us, backward 16.2 vs 16.4, step 0.4482 vs
// 0.4432 ms interleaved: the fp32 chain is not MFMA-bound at one workgroup per CU (its
// 2 x 9,472 MFMA cycles are ~8 of the 20 us), and the split form's 228 weight-plane
// registers spill into AGPR copies and just-in-time fragment reads.  With the weights split
// in the loop instead (fp32 fragments, as k_chain; the split hidden from loop-invariant code
// motion) and two accumulators per stage: forward 22.0-25.5 vs 20.8 us standalone
// (profiles/r06_s28-s30, tools/chain_prof.py stamps: the stages take as long as the fp32
// ones -- the chain is bound by more than its MFMA issue).  Off (GINE_CHAIN_X3=1 builds it
// into the dispatch).
// ---------------------------------------------------------------------------------------
#ifndef GINE_CHAIN_X3
#define GINE_CHAIN_X3 0
#endif

// The split planes of eight fp32 weights, computed where they are used: the (empty) asm
// hides the values' loop invariance, so the split is not hoisted out of the tile loop into
// 228 live plane registers.
__device__ __forceinline__ Bf16x3 split_w8(const float* w) {
  float w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4], w5 = w[5], w6 = w[6], w7 = w[7];
  asm volatile("" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3), "+v"(w4), "+v"(w5), "+v"(w6),
               "+v"(w7));
  return split8(make_float4(w0, w1, w2, w3), make_float4(w4, w5, w6, w7));
}

template <int D, int FP, bool FWD>
__global__ __launch_bounds__(2 * D) void k_chain2_x3(ChainArgs a, int64_t N, int num_tiles) {
  constexpr int NT = 2 * D, D4 = D / 4;
  constexpr int FPX = FWD ? (FP + 15) / 16 * 16 : 0;  // stage 2's x columns, whole 16-k blocks
  constexpr int K1 = D, K2 = FPX + D;
  constexpr int KS1 = K1 / 2, KS2 = K2 / 2;
  static_assert(KS1 % 8 == 0 && KS2 % 8 == 0, "whole split fragments per lane half");
  constexpr int RS1 = K1 + 8, RS2 = K2 + 8;  // plane row strides (bf16): 16 x odd bytes
  constexpr int P1 = kRowTile * RS1, P2 = kRowTile * RS2;
  constexpr int ITEMS = kRowTile * D4 / NT;  // stage-1 A float4 per thread
  constexpr int RSTEP = NT / D4;
  constexpr int XP = FWD ? FPX / 2 : 1;  // x column pairs per row
  constexpr int XITEMS = FWD ? (kRowTile * XP + NT - 1) / NT : 1;
  __shared__ __attribute__((aligned(16))) uint16_t pa[3 * P1];
  __shared__ __attribute__((aligned(16))) uint16_t pb[3 * P2];

  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const int col = wave * 32 + c32;
  const int q_me = threadIdx.x % D4, r_me = threadIdx.x / D4;
  const int F = a.F;
  CHAIN_RT(11);
  CHAIN_MARK(0);

  const TileRange tr = tile_range(num_tiles, gridDim.x);
  float4 raw[ITEMS];
  float xr[2 * XITEMS];
  auto load_tile = [&](int tile) {
    const int64_t n0 = (int64_t)tile * kRowTile;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      int64_t n = n0 + r_me + i * RSTEP;
      n = n < N ? n : N - 1;
      raw[i] = reinterpret_cast<const float4*>(a.in + n * D)[q_me];
    }
    if constexpr (FWD) {
#pragma unroll
      for (int i = 0; i < XITEMS; ++i) {
        const int idx = min((int)threadIdx.x + i * NT, kRowTile * XP - 1);
        int64_t n = n0 + idx / XP;
        n = n < N ? n : N - 1;
        const int c = 2 * (idx % XP);
        xr[2 * i] = a.x[n * F + min(c, F - 1)];  // padding columns zeroed at the store
        xr[2 * i + 1] = a.x[n * F + min(c + 1, F - 1)];
      }
    }
  };
  // the first tile's rows first (its staging waits for them only), then both weights' fp32
  // fragments (lane half h: k = h*KS + s), split per K = 16 block inside the chains: held
  // as split planes (228 registers at D = 128) they spilled into AGPR copies
  if (tr.first < tr.end) load_tile(tr.first);
  float bf1[KS1], bf2[KS2];
  if constexpr (FWD) {
    frag_t4<D>(bf1, a.w1, D, col, h);              // Wf
    frag_dimred_t<FPX, D>(bf2, a.w3, F, col, h);   // W'^T, x columns padded to FPX
  } else {
    frag_n<D>(bf1, a.w1, F + D, F, col, h);        // W' e-columns (Wc)
    frag_n<D>(bf2, a.w2, D, 0, col, h);            // Wf
  }
  const float bias1 = FWD ? a.b1[col] * a.bias1_scale : 0.f;
  const float bias2 = FWD ? a.b3[col] : 0.f;
  float* out1 = a.out1;
  float* out2 = FWD ? a.out3 : a.out2;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) before the loop (see k_chain)
  CHAIN_MARK(1);
  int kt = 0;
  for (int tile = tr.first; tile < tr.end; tile += tr.step, ++kt) {
    const int64_t n0 = (int64_t)tile * kRowTile;
    __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {  // stage-1 A planes (rows past N: zero)
      const int r = r_me + i * RSTEP;
      const float4 v = (n0 + r < N) ? raw[i] : f4_zero();
      uint32_t h0, m0, l0, h1, m1, l1;
      split2(v.x, v.y, h0, m0, l0);
      split2(v.z, v.w, h1, m1, l1);
      uint16_t* d = pa + r * RS1 + 4 * q_me;
      *reinterpret_cast<uint2*>(d) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(d + P1) = make_uint2(m0, m1);
      *reinterpret_cast<uint2*>(d + 2 * P1) = make_uint2(l0, l1);
    }
    if constexpr (FWD) {
#pragma unroll
      for (int i = 0; i < XITEMS; ++i) {  // x planes: columns [0, FPX) of stage 2's A
        const int idx = threadIdx.x + i * NT;
        if (idx < kRowTile * XP) {
          const int r = idx / XP, c = 2 * (idx % XP);
          const bool live = n0 + r < N;
          const float v0 = live && c < F ? xr[2 * i] : 0.f;
          const float v1 = live && c + 1 < F ? xr[2 * i + 1] : 0.f;
          uint32_t hh, mm, ll;
          split2(v0, v1, hh, mm, ll);
          uint16_t* d = pb + r * RS2 + c;
          *reinterpret_cast<uint32_t*>(d) = hh;
          *reinterpret_cast<uint32_t*>(d + P2) = mm;
          *reinterpret_cast<uint32_t*>(d + 2 * P2) = ll;
        }
      }
    }
    __syncthreads();
    if (kt < 2) CHAIN_MARK(2 + 4 * kt);
    if (tile + tr.step < tr.end) load_tile(tile + tr.step);  // next tile in flight
    float ep[FWD ? 1 : 16];
    if constexpr (!FWD) {  // the ReLU mask of u, in flight under stage 1
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int64_t n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        n = n < N ? n : N - 1;
        ep[r] = a.aux[n * D + col];
      }
    }

    // stage 1 (two accumulators over alternate K = 16 blocks: independent MFMA chains)
    floatx16 acc = zero16();
    {
      floatx16 acc2 = zero16();
      const uint16_t* pr = pa + c32 * RS1 + h * KS1;
#pragma unroll
      for (int s8 = 0; s8 < KS1 / 8; ++s8) {
        Bf16x3 f;
        f.h = *reinterpret_cast<const bf16x8_t*>(pr + 8 * s8);
        f.m = *reinterpret_cast<const bf16x8_t*>(pr + P1 + 8 * s8);
        f.l = *reinterpret_cast<const bf16x8_t*>(pr + 2 * P1 + 8 * s8);
        const Bf16x3 b = split_w8(bf1 + 8 * s8);
        if (s8 & 1) acc2 = mfma_bf16x3(f, b, acc2);
        else acc = mfma_bf16x3(f, b, acc);
      }
      acc = acc + acc2;
      if (wave_any_nan(acc)) {  // fp32 chain from memory (the fp32 GEMM's non-finite values)
        const int64_t n = min(n0 + c32, N - 1);
        acc = zero16();
        if constexpr (FWD)
          acc = mfma_f32_row_mem<KS1>(a.in + n * D + h * KS1, a.w1 + (size_t)col * D + h * KS1,
                                      1, acc);
        else
          acc = mfma_f32_row_mem<KS1>(a.in + n * D + h * KS1,
                                      a.w1 + (size_t)(h * KS1) * (F + D) + F + col, F + D, acc);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t n = n0 + rr;
      float v;
      if constexpr (FWD) v = relu_nan(acc[r] + bias1);   // u = relu(r Wf^T + bf)
      else v = ep[r] > 0.f ? acc[r] : 0.f;               // dt = du * 1[u > 0]
      if (n < N) out1[n * D + col] = v;
      else v = 0.f;
      uint32_t hh, mm, ll;
      split2(v, 0.f, hh, mm, ll);
      uint16_t* d = pb + rr * RS2 + FPX + col;
      d[0] = (uint16_t)hh;
      d[P2] = (uint16_t)mm;
      d[2 * P2] = (uint16_t)ll;
    }
    if (kt < 2) CHAIN_MARK(3 + 4 * kt);
    __syncthreads();  // stage 2's A planes complete (and stage 1's outputs written)
    if (kt < 2) CHAIN_MARK(4 + 4 * kt);

    // stage 2 (two accumulators, as stage 1)
    acc = zero16();
    {
      floatx16 acc2 = zero16();
      const uint16_t* pr = pb + c32 * RS2 + h * KS2;
#pragma unroll
      for (int s8 = 0; s8 < KS2 / 8; ++s8) {
        Bf16x3 f;
        f.h = *reinterpret_cast<const bf16x8_t*>(pr + 8 * s8);
        f.m = *reinterpret_cast<const bf16x8_t*>(pr + P2 + 8 * s8);
        f.l = *reinterpret_cast<const bf16x8_t*>(pr + 2 * P2 + 8 * s8);
        const Bf16x3 b = split_w8(bf2 + 8 * s8);
        if (s8 & 1) acc2 = mfma_bf16x3(f, b, acc2);
        else acc = mfma_bf16x3(f, b, acc);
      }
      acc = acc + acc2;
      if (wave_any_nan(acc)) {
        const int64_t n = min(n0 + c32, N - 1);
        acc = zero16();
        if constexpr (FWD) {  // A = [x | 0 | u] of row n, B = W'^T on the same padded k axis
#pragma unroll 1
          for (int s = 0; s < KS2; ++s) {
            const int k = h * KS2 + s;
            float av, bv;
            if (k < FPX) {
              av = k < F ? a.x[n * F + k] : 0.f;
              bv = k < F ? a.w3[(size_t)k * D + col] : 0.f;
            } else {
              av = out1[n * D + (k - FPX)];
              bv = a.w3[(size_t)(k - FPX + F) * D + col];
            }
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
          }
        } else {
          acc = mfma_f32_row_mem<KS2>(out1 + n * D + h * KS2, a.w2 + (size_t)(h * KS2) * D + col,
                                      D, acc);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t n = n0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (n < N) out2[n * D + col] = acc[r] + bias2;
    }
    if (kt < 2) CHAIN_MARK(5 + 4 * kt);
  }
  CHAIN_MARK(10);
  CHAIN_RT(12);
}

template <int D, int FP, bool FWD>
int launch_chain2_x3(const ChainArgs& a, int64_t N, hipStream_t s);

// Persistent grid, one workgroup per CU (two per CU measured slower at cfg2: 0.614 vs
// 0.589 ms per step).
inline int chain_grid(int64_t N) {
  const int64_t tiles = ceil_div(N, kRowTile);
  return (int)std::max<int64_t>(1, std::min<int64_t>(tiles, kNumCu));
}

template <int D, int FP, int KIND>
int launch_chain(const ChainArgs& a, int64_t N, hipStream_t s) {
  const int tiles = (int)ceil_div(N, kRowTile);
  const int fold = (KIND == CH_F1 && a.wfold != nullptr) ? kFoldBlocks<D> : 0;
  hipLaunchKernelGGL((k_chain<D, FP, KIND>), dim3(chain_grid(N) + fold), dim3(2 * D), 0, s, a,
                     N, tiles);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

template <int D, int FP, bool FWD>
int launch_chain2_x3(const ChainArgs& a, int64_t N, hipStream_t s) {
  const int tiles = (int)ceil_div(N, kRowTile);
  hipLaunchKernelGGL((k_chain2_x3<D, FP, FWD>), dim3(chain_grid(N)), dim3(2 * D), 0, s, a, N,
                     tiles);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

// ----------------------------------------------------------------------------------------
// weight gradients, one engine launch
//   NZ = 4 (unfolded):  z = 0: dWdr [D x (F+D)] = dh0^T [x | e]   z = 1: dWr1 = de^T u
//                       z = 2: dWr0 = dt^T s                       z = 3: dWp2 = ds^T r
//   NZ = 3 (folded):    z = 0: G = dh0^T [x | u]   z = 1: dWr0 = dt^T s   z = 2: dWp2 = ds^T r
//                       (dWdr / dWr1 follow from G in gine_chain_unfold_grads)
// ----------------------------------------------------------------------------------------
template <int NZ>
struct ChainWgradSrc {
  static constexpr int kZ = NZ;
  const float* p[4];  // P rows [N, D] of product z
  const float* q[4];  // Q rows [N, D] of product z (z = 0: the D columns after x)
  const float* x;
  int D, F;
  struct Raw {
    float4 v;
  };
  struct Col {
    float keep[4];  // Q of z = 0: 1 for the columns inside [x | .], 0 for the padding
  };
  template <int Z> __device__ int i_dim(int) const { return Z == 0 ? F + D : D; }
  template <int Z> __device__ Col p_col(int) const { return Col{{1.f, 1.f, 1.f, 1.f}}; }
  template <int Z> __device__ Col q_col(int q4) const {
    Col c{{1.f, 1.f, 1.f, 1.f}};
    if constexpr (Z == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) c.keep[j] = 4 * q4 + j < F + D ? 1.f : 0.f;
    }
    return c;
  }
  template <int Z> __device__ Raw p_load(int64_t n, int q4) const {
    return Raw{reinterpret_cast<const float4*>(p[Z] + n * D)[q4]};
  }
  template <int Z> __device__ Raw q_load(int64_t n, int q4) const {
    if constexpr (Z == 0) {  // [x | q0]: F + D columns, x rows are not float4-aligned
      const int I = F + D;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = min(4 * q4 + j, I - 1);
        const float* src = c < F ? x + n * F + c : q[0] + n * D + (c - F);
        v[j] = *src;  // raw: the padding is zeroed in q_xform, when the tile is staged
      }
      return Raw{make_float4(v[0], v[1], v[2], v[3])};
    } else {
      return Raw{reinterpret_cast<const float4*>(q[Z] + n * D)[q4]};
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
  float* w[4];  // product order of ChainWgradSrc
  float* b[4];
  int D, F, nz;
  float bias_scale;  // phi[2]'s bias (the last product) enters M times
  __device__ void operator()(int z, int64_t e, double v) const {
    const int64_t I = z == 0 ? F + D : D;
    const int64_t ws = (int64_t)D * I;
    if (e < ws) {
      w[z][e] = (float)v;
    } else if (e < ws + D && b[z] != nullptr) {
      b[z][e - ws] = (float)(z == nz - 1 ? v * (double)bias_scale : v);
    }
  }
};

// output tiles: dim_red's [D x (F+D)] plus nz - 1 [D x D]
inline int chain_wgrad_tiles(int D, int F, int nz) {
  const int to = (int)ceil_div(D, 64);
  return to * (int)ceil_div(F + D, kWgTI) + (nz - 1) * to * (int)ceil_div(D, kWgTI);
}
inline WgPlan chain_wgrad_plan(int64_t N, int D, int F, int nz) {
  return wg_plan(N, D, F + D, nz, 64, chain_wgrad_tiles(D, F, nz));
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
  // enough for either chain (4 products unfolded, 3 folded)
  const WgPlan p4 = chain_wgrad_plan(num_nodes, hidden, in_features, 4);
  const WgPlan p3 = chain_wgrad_plan(num_nodes, hidden, in_features, 3);
  const size_t per = (size_t)hidden * (hidden + in_features) + hidden;
  *floats = std::max(4 * (size_t)p4.chunks, 3 * (size_t)p3.chunks) * per;
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
  const WgPlan p = chain_wgrad_plan(num_nodes, D, F, 4);
  const size_t per = (size_t)D * (D + F) + D;
  const ChainWgradSrc<4> src{{dh0, de, dt, ds}, {e, u, s, r}, x, D, F};
  rc = launch_wgrad_engine<64>(src, num_nodes, D, D + F, chain_wgrad_tiles(D, F, 4), p,
                                per * p.chunks, per, slab, st);
  if (rc != GINE_OK) return rc;
  if (!reduce) return GINE_OK;
  return launch_slab_sum(slab, p.chunks, (int64_t)per, per, per * p.chunks, 4,
                         ChainWgradOut{{dwdr, dwr1, dwr0, dwp2}, {dbdr, dbr1, dbr0, dbp2}, D,
                                       F, 4, bias_scale},
                         st);
}

namespace {
// the slab job of either chain; w / b in product order
void chain_slab_job(int64_t N, int D, int F, int nz, const float* slab, float bias_scale,
                    float* const* w, float* const* b, gine_grad_job* job) {
  const WgPlan p = chain_wgrad_plan(N, D, F, nz);
  const int64_t per = (int64_t)D * (D + F) + D;
  *job = gine_grad_job{};
  job->kind = GINE_GRAD_JOB_SLAB;
  job->src = slab;
  job->rows = p.chunks;
  job->cstride = per;
  job->zstride = per * p.chunks;
  job->nz = nz;
  for (int z = 0; z < nz; ++z) {
    const int64_t ws = (int64_t)D * (z == 0 ? F + D : D);
    job->per[z] = ws + D;
    job->wsize[z] = ws;
    job->w[z] = w[z];
    job->b[z] = b[z];
    job->bscale[z] = z == nz - 1 ? bias_scale : 1.0f;
  }
}
}  // namespace

extern "C" int gine_chain_wgrad_grad_job(int64_t num_nodes, int32_t hidden, int32_t in_features,
                                         const float* slab, float bias_scale, float* dwp2,
                                         float* dbp2, float* dwr0, float* dbr0, float* dwr1,
                                         float* dbr1, float* dwdr, float* dbdr,
                                         gine_grad_job* job) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !slab || !dwp2 || !dwr0 || !dwr1 || !dwdr || !job)
    return GINE_ERR_INVALID;
  float* w[4] = {dwdr, dwr1, dwr0, dwp2};  // product order of ChainWgradSrc<4>
  float* b[4] = {dbdr, dbr1, dbr0, dbp2};
  chain_slab_job(num_nodes, hidden, in_features, 4, slab, bias_scale, w, b, job);
  return GINE_OK;
}

// ---------------------------------------------------------------------------------------
// Folded chain.  rho[2] is followed by dim_red with no nonlinearity between them, so
//   h0 = [x | u Wr1^T + br1] Wdr^T + bdr = [x | u] W'^T + b',
//   W' = [Wdr_x | Wc], Wc = Wdr_e Wr1, b' = Wdr_e br1 + bdr,
// and the backward needs neither e nor de: dt = (dh0 Wc) * 1[u > 0], and with
// G = dh0^T [x | u] and g = sum_n dh0 (one engine product instead of two):
//   dWdr = [G_x | G_u Wr1^T + g br1^T], dbdr = g, dWr1 = Wdr_e^T G_u, dbr1 = Wdr_e^T g.
// One GEMM fewer forward, one fewer input-gradient GEMM and one fewer weight-gradient
// product backward; W' is folded by the first chain kernel's workgroups after their tiles,
// G is unfolded by one small launch (2 (D/32)^2 workgroups) after the slab reduction.
// ---------------------------------------------------------------------------------------
namespace gine {
namespace {

// One unfold job: G = gf ([D][F + D] then g [D]) of the product dY^T [x | q] where the
// rows of q feed a Linear (w1, bias b1 * bscale) whose output meets Wdr's q columns, e.g.
//   h0 = [x | u Wr1^T + br1] Wdr^T + bdr:   dWdr = [G_x | G_u Wr1^T + g br1^T], dbdr = g,
//                                           dWr1 = Wdr_e^T G_u, dbr1 = Wdr_e^T g,
// and the same with F = 0 for pre = (r Wp2^T + M bp2) Wr0^T + br0 (the double fold):
//   dWr0 = G2 Wp2^T + M g2 bp2^T, dbr0 = g2, dWp2 = Wr0^T G2, dbp2 = M Wr0^T g2.
struct UnfoldJob {
  const float *gf, *w1, *b1, *wdr;  // w1 [D][D]; wdr [D][F + D] (its last D columns used)
  float *dwdr, *dbdr, *dw1, *db1;
  int F;
  float bscale;
};

// 2 (D/32)^2 workgroups per job, one [32 x 32] tile each (ksplit_tile): tiles of dWdr's q
// columns, G_q W1^T + g (bscale b1)^T (G_q rows staged, B = W1^T read along W1's rows), then
// tiles of dW1 = Wdr_q^T G_q (Wdr_q columns staged as rows, B = G_q); the x columns and dbdr
// (resp. db1) by the tiles of column 0.
template <int D>
__global__ __launch_bounds__(2 * D) void k_chain_unfold(UnfoldJob j0, UnfoldJob j1) {
  constexpr int NT = 2 * D, LDA = D + 4, T = D / 32, TT = T * T;
  constexpr int SI = 32 * D / NT, XI = 32 * 64 / NT;
  __shared__ __attribute__((aligned(16))) float sA[32 * LDA];
  __shared__ float sR[T * kSR];
  __shared__ float svec[D];
  const bool second = (int)blockIdx.x >= 2 * TT;
  // field by field (uniform selects; no private copy of a kernel argument)
  const UnfoldJob J{second ? j1.gf : j0.gf,     second ? j1.w1 : j0.w1,
                    second ? j1.b1 : j0.b1,     second ? j1.wdr : j0.wdr,
                    second ? j1.dwdr : j0.dwdr, second ? j1.dbdr : j0.dbdr,
                    second ? j1.dw1 : j0.dw1,   second ? j1.db1 : j0.db1,
                    second ? j1.F : j0.F,       second ? j1.bscale : j0.bscale};
  const int blk = (int)blockIdx.x - (second ? 2 * TT : 0);
  const float* __restrict__ gf = J.gf;
  const int F = J.F;
  const int LW = F + D;
  const float* g = gf + (size_t)D * LW;
  const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int h = lane >> 5, c32 = lane & 31;
  const bool e_cols = blk < TT;
  const int t = e_cols ? blk : blk - TT;
  const int r0 = 32 * (t / T), c0 = 32 * (t % T);
  float bf[16], st[SI];
  if (e_cols) {
#pragma unroll
    for (int s = 0; s < 16; ++s) bf[s] = J.w1[(size_t)(c0 + c32) * D + w * 32 + h * 16 + s];
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int idx = threadIdx.x + i * NT;
      st[i] = gf[(size_t)(r0 + idx / D) * LW + F + idx % D];
    }
    if (c0 == 0) {
      if (F > 0) {
        float xv[XI];
#pragma unroll
        for (int i = 0; i < XI; ++i) {
          const int idx = min(threadIdx.x + i * NT, 32 * F - 1);
          xv[i] = gf[(size_t)(r0 + idx / F) * LW + idx % F];
        }
#pragma unroll
        for (int i = 0; i < XI; ++i) {
          const int idx = threadIdx.x + i * NT;
          if (idx < 32 * F) J.dwdr[(size_t)(r0 + idx / F) * LW + idx % F] = xv[i];
        }
      }
      if (threadIdx.x < 32 && J.dbdr != nullptr) J.dbdr[r0 + threadIdx.x] = g[r0 + threadIdx.x];
    }
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int idx = threadIdx.x + i * NT;
      sA[(idx / D) * LDA + idx % D] = st[i];
    }
  } else {
#pragma unroll
    for (int s = 0; s < 16; ++s)
      bf[s] = gf[(size_t)(w * 32 + h * 16 + s) * LW + F + c0 + c32];  // G_q[k][c0 + c32]
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int idx = threadIdx.x + i * NT;
      st[i] = J.wdr[(size_t)(idx / 32) * LW + F + r0 + idx % 32];
    }
    const float gv = threadIdx.x < D ? g[threadIdx.x] : 0.f;
#pragma unroll
    for (int i = 0; i < SI; ++i) {
      const int idx = threadIdx.x + i * NT;
      sA[(idx % 32) * LDA + idx / 32] = st[i];
    }
    if (threadIdx.x < D) svec[threadIdx.x] = gv;
  }
  __syncthreads();
  ksplit_tile<D>(sA, bf, sR, c32, h);
  if (!e_cols && c0 == 0) {
    const float v = rows_dot<D>(sA, svec);  // (Wdr_q^T g)[r0 + r]
    constexpr int TPR = NT / 32;
    if (threadIdx.x % TPR == 0 && J.db1 != nullptr) J.db1[r0 + threadIdx.x / TPR] = v * J.bscale;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int o = threadIdx.x + i * NT, rr = o / 32, cc = o % 32;
    const float v = ksplit_sum<D>(sR, rr, cc);
    if (e_cols)
      J.dwdr[(size_t)(r0 + rr) * LW + F + c0 + cc] =
          fmaf(g[r0 + rr], J.b1[c0 + cc] * J.bscale, v);
    else
      J.dw1[(size_t)(r0 + rr) * D + c0 + cc] = v;
  }
}

int launch_unfold(int D, const UnfoldJob& j0, const UnfoldJob* j1, hipStream_t st) {
  const int jobs = j1 ? 2 : 1;
  const UnfoldJob second = j1 ? *j1 : j0;
  if (D == 64)
    hipLaunchKernelGGL((k_chain_unfold<64>), dim3(jobs * 2 * 4), dim3(128), 0, st, j0, second);
  else
    hipLaunchKernelGGL((k_chain_unfold<128>), dim3(jobs * 2 * 16), dim3(256), 0, st, j0,
                       second);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}

}  // namespace
}  // namespace gine

extern "C" int gine_chain_fwd_folded(const float* r, const float* x, const float* wp2,
                                     const float* bp2, float bias_scale, const float* wr0,
                                     const float* br0, const float* wr1, const float* br1,
                                     const float* wdr, const float* bdr, float* wfold, float* s,
                                     float* u, float* h0, int64_t num_nodes, int32_t hidden,
                                     int32_t in_features, void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes < 0) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  if (num_nodes == 0) return GINE_OK;
  if (!r || !x || !wp2 || !bp2 || !wr0 || !br0 || !wr1 || !br1 || !wdr || !bdr || !wfold ||
      !s || !u || !h0)
    return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int D = hidden, F = in_features;
  const float* bfold = wfold + (size_t)D * (F + D);
  const float* wfold_t = bfold + D;
  const ChainArgs f1{r,  nullptr, nullptr, wp2, bp2, wr0, br0, s,
                     u,  bias_scale, F,    wr1, br1, wdr, bdr, wfold};
  const ChainArgs f2{u, x, nullptr, nullptr, nullptr, wfold_t, bfold, nullptr, h0, 1.f, F};
  int rc = GINE_OK;
#define CALL_F(DD, FF)                                                  \
  rc = launch_chain<DD, FF, CH_F1>(f1, num_nodes, st);                  \
  if (rc == GINE_OK) rc = launch_chain<DD, FF, CH_F2F>(f2, num_nodes, st)
  GINE_CHAIN_DISPATCH(D, F, CALL_F);
#undef CALL_F
  return rc;
}

extern "C" int gine_chain_fwd_folded3(const float* r, const float* x, const float* wp2,
                                      const float* bp2, float bias_scale, const float* wr0,
                                      const float* br0, const float* wfold, float* s, float* u,
                                      float* h0, int64_t num_nodes, int32_t hidden,
                                      int32_t in_features, void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes < 0) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  if (num_nodes == 0) return GINE_OK;
  if (!r || !x || !wp2 || !bp2 || !wr0 || !br0 || !wfold || !s || !u || !h0)
    return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int D = hidden, F = in_features;
  const float* bfold = wfold + (size_t)D * (F + D);
  ChainArgs f{r, x, nullptr, wp2, bp2, wr0, br0, s, u, bias_scale, F};
  f.w3 = bfold + D;  // W'^T
  f.b3 = bfold;
  f.out3 = h0;
  int rc = GINE_OK;
#define CALL_F(DD, FF) rc = launch_chain<DD, FF, CH_F3>(f, num_nodes, st)
  GINE_CHAIN_DISPATCH(D, F, CALL_F);
#undef CALL_F
  return rc;
}

extern "C" int gine_chain_bwd_folded(const float* dh0, const float* u, const float* wp2,
                                     const float* wr0, const float* wfold, float* dt, float* ds,
                                     float* dr, int64_t num_nodes, int32_t hidden,
                                     int32_t in_features, void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  if (!dh0 || !u || !wp2 || !wr0 || !wfold || !dt || !ds || !dr) return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int F = in_features;
  int rc = GINE_OK;
  // one launch: dt -> ds -> dr (two launches, B1F + B2, measured slower: r02_s43)
  ChainArgs b{dh0, nullptr, u, wfold, nullptr, wr0, nullptr, dt, ds, 1.f, F};
  b.w3 = wp2;
  b.out3 = dr;
#define CALL_B(DD, FF) rc = launch_chain<DD, FF, CH_B3>(b, num_nodes, st)
  GINE_CHAIN_DISPATCH(hidden, F, CALL_B);
#undef CALL_B
  return rc;
}

extern "C" int gine_chain_wgrad_folded(const float* dh0, const float* x, const float* r,
                                       const float* s, const float* u, const float* dt,
                                       const float* ds, float* slab, float* gfold, float* dwr0,
                                       float* dbr0, float* dwp2, float* dbp2, float bias_scale,
                                       int64_t num_nodes, int32_t hidden, int32_t in_features,
                                       void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0) return GINE_ERR_INVALID;
  if (!dh0 || !x || !r || !s || !u || !dt || !ds || !slab) return GINE_ERR_INVALID;
  // gfold, dwr0, dwp2 all NULL: the slab is left for gine_grad_finalize_batch
  const bool reduce = gfold || dwr0 || dwp2;
  if (reduce && (!gfold || !dwr0 || !dwp2)) return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int D = hidden, F = in_features;
  const WgPlan p = chain_wgrad_plan(num_nodes, D, F, 3);
  const size_t per = (size_t)D * (D + F) + D;
  const ChainWgradSrc<3> src{{dh0, dt, ds, nullptr}, {u, s, r, nullptr}, x, D, F};
  int rc = launch_wgrad_engine<64>(src, num_nodes, D, D + F, chain_wgrad_tiles(D, F, 3), p,
                                   per * p.chunks, per, slab, st);
  if (rc != GINE_OK || !reduce) return rc;
  return launch_slab_sum(slab, p.chunks, (int64_t)per, per, per * p.chunks, 3,
                         ChainWgradOut{{gfold, dwr0, dwp2, nullptr},
                                       {gfold + (size_t)D * (F + D), dbr0, dbp2, nullptr}, D,
                                       F, 3, bias_scale},
                         st);
}

extern "C" int gine_chain_wgrad_folded_grad_job(int64_t num_nodes, int32_t hidden,
                                                int32_t in_features, const float* slab,
                                                float bias_scale, float* gfold, float* dwr0,
                                                float* dbr0, float* dwp2, float* dbp2,
                                                gine_grad_job* job) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !slab || !gfold || !dwr0 || !dwp2 || !job) return GINE_ERR_INVALID;
  float* w[3] = {gfold, dwr0, dwp2};  // product order of ChainWgradSrc<3>
  float* b[3] = {gfold + (size_t)hidden * (hidden + in_features), dbr0, dbp2};
  chain_slab_job(num_nodes, hidden, in_features, 3, slab, bias_scale, w, b, job);
  return GINE_OK;
}

extern "C" int gine_chain_unfold_grads(const float* gfold, const float* wr1, const float* br1,
                                       const float* wdr, float* dwdr, float* dbdr, float* dwr1,
                                       float* dbr1, int32_t hidden, int32_t in_features,
                                       void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (!gfold || !wr1 || !br1 || !wdr || !dwdr || !dwr1) return GINE_ERR_INVALID;
  return launch_unfold(hidden,
                       UnfoldJob{gfold, wr1, br1, wdr, dwdr, dbdr, dwr1, dbr1, in_features, 1.f},
                       nullptr, as_stream(stream));
}

// ---------------------------------------------------------------------------------------
// Doubly folded chain: phi[2] folded into rho[0] as well,
//   pre = s Wr0^T + br0 = r Wf^T + bf,  Wf = Wr0 Wp2,  bf = M Wr0 bp2 + br0
// (wfold2 = [Wf | bf], folded by gine_deepset_fwd_fold2's workgroups), so neither s nor ds is
// formed: forward u -> h0 in one 2-stage launch, backward dt -> dr in one, the weight
// gradients from two engine products, G = dh0^T [x | u] and G2 = dt^T r (+ g2 = sum dt),
// unfolded together: dWdr, dWr1 from G as before, dWr0 = G2 Wp2^T + M g2 bp2^T,
// dbr0 = g2, dWp2 = Wr0^T G2, dbp2 = M Wr0^T g2.
// ---------------------------------------------------------------------------------------
extern "C" int gine_chain_fwd_folded2(const float* r, const float* x, const float* wfold,
                                      const float* wfold2, float* u, float* h0,
                                      int64_t num_nodes, int32_t hidden, int32_t in_features,
                                      void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes < 0) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  if (num_nodes == 0) return GINE_OK;
  if (!r || !x || !wfold || !wfold2 || !u || !h0) return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int D = hidden, F = in_features;
  const float* bfold = wfold + (size_t)D * (F + D);
  ChainArgs f{r, x, nullptr, wfold2, wfold2 + (size_t)D * D, nullptr, nullptr, u, nullptr,
              1.f, F};
  f.w3 = bfold + D;  // W'^T
  f.b3 = bfold;
  f.out3 = h0;
  int rc = GINE_OK;
#define CALL_F(DD, FF)                                                                  \
  rc = GINE_CHAIN_X3 ? launch_chain2_x3<DD, FF, true>(f, num_nodes, st)                   \
                     : launch_chain<DD, FF, CH_F2D>(f, num_nodes, st)
  GINE_CHAIN_DISPATCH(D, F, CALL_F);
#undef CALL_F
  return rc;
}

extern "C" int gine_chain_bwd_folded2(const float* dh0, const float* u, const float* wfold,
                                      const float* wfold2, float* dt, float* dr,
                                      int64_t num_nodes, int32_t hidden, int32_t in_features,
                                      void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0) return GINE_ERR_INVALID;
  if (num_nodes >= (int64_t(1) << 31)) return GINE_ERR_TOO_LARGE;
  if (!dh0 || !u || !wfold || !wfold2 || !dt || !dr) return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int F = in_features;
  const ChainArgs b{dh0, nullptr, u, wfold, nullptr, wfold2, nullptr, dt, dr, 1.f, F};
  int rc = GINE_OK;
#define CALL_B(DD, FF)                                                                  \
  rc = GINE_CHAIN_X3 ? launch_chain2_x3<DD, FF, false>(b, num_nodes, st)                  \
                     : launch_chain<DD, FF, CH_B2D>(b, num_nodes, st)
  GINE_CHAIN_DISPATCH(hidden, F, CALL_B);
#undef CALL_B
  return rc;
}

extern "C" int gine_chain_wgrad_folded2(const float* dh0, const float* x, const float* r,
                                        const float* u, const float* dt, float* slab,
                                        float* gfold, float* g2fold, int64_t num_nodes,
                                        int32_t hidden, int32_t in_features, void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0) return GINE_ERR_INVALID;
  if (!dh0 || !x || !r || !u || !dt || !slab) return GINE_ERR_INVALID;
  // gfold, g2fold both NULL: the slab is left for gine_grad_finalize_batch
  const bool reduce = gfold || g2fold;
  if (reduce && (!gfold || !g2fold)) return GINE_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  const int D = hidden, F = in_features;
  const WgPlan p = chain_wgrad_plan(num_nodes, D, F, 2);
  const size_t per = (size_t)D * (D + F) + D;
  const ChainWgradSrc<2> src{{dh0, dt, nullptr, nullptr}, {u, r, nullptr, nullptr}, x, D, F};
  int rc = launch_wgrad_engine<64>(src, num_nodes, D, D + F, chain_wgrad_tiles(D, F, 2), p,
                                   per * p.chunks, per, slab, st);
  if (rc != GINE_OK || !reduce) return rc;
  return launch_slab_sum(slab, p.chunks, (int64_t)per, per, per * p.chunks, 2,
                         ChainWgradOut{{gfold, g2fold, nullptr, nullptr},
                                       {gfold + (size_t)D * (F + D), g2fold + (size_t)D * D,
                                        nullptr, nullptr},
                                       D, F, 2, 1.f},
                         st);
}

extern "C" int gine_chain_wgrad_folded2_grad_job(int64_t num_nodes, int32_t hidden,
                                                 int32_t in_features, const float* slab,
                                                 float* gfold, float* g2fold,
                                                 gine_grad_job* job) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (num_nodes <= 0 || !slab || !gfold || !g2fold || !job) return GINE_ERR_INVALID;
  float* w[2] = {gfold, g2fold};  // product order of ChainWgradSrc<2>
  float* b[2] = {gfold + (size_t)hidden * (hidden + in_features),
                 g2fold + (size_t)hidden * hidden};
  chain_slab_job(num_nodes, hidden, in_features, 2, slab, 1.f, w, b, job);
  return GINE_OK;
}

extern "C" int gine_chain_unfold_grads2(const float* gfold, const float* wr1, const float* br1,
                                        const float* wdr, float* dwdr, float* dbdr, float* dwr1,
                                        float* dbr1, const float* g2fold, const float* wp2,
                                        const float* bp2, const float* wr0, float* dwr0,
                                        float* dbr0, float* dwp2, float* dbp2, float members,
                                        int32_t hidden, int32_t in_features, void* stream) {
  if (!chain_dims_ok(hidden, in_features)) return GINE_ERR_DIM;
  if (!gfold || !wr1 || !br1 || !wdr || !dwdr || !dwr1) return GINE_ERR_INVALID;
  if (!g2fold || !wp2 || !bp2 || !wr0 || !dwr0 || !dwp2) return GINE_ERR_INVALID;
  const UnfoldJob j1{g2fold, wp2, bp2, wr0, dwr0, dbr0, dwp2, dbp2, 0, members};
  return launch_unfold(hidden,
                       UnfoldJob{gfold, wr1, br1, wdr, dwdr, dbdr, dwr1, dbr1, in_features, 1.f},
                       &j1, as_stream(stream));
}

#ifdef GINE_CHAIN_PROFILE
extern "C" int gine_debug_chain_prof(long long* out) {  // [1024][16] host buffer
  GINE_RETURN_IF_HIP(hipDeviceSynchronize());
  GINE_RETURN_IF_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain_prof), sizeof(g_chain_prof)));
  return GINE_OK;
}
#endif
