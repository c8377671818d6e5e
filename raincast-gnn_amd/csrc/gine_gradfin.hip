// Batched gradient finish: every parameter-gradient reduction that only the optimizer reads,
// in one launch at the end of the backward (gine_grad_finalize_batch, include/gine_hip.h).
//
// Per GINE layer the message-passing backward leaves fp64 partial rows of dW_e, db_e and
// d eps; the output head, the dense chain and the DeepSet backward leave fp32 split-K slabs
// of their weight gradients.  Reduced one launch each they cost ~3 us apiece in a replayed
// step (a kernel boundary plus a short dependent read); here the workgroups of all jobs
// share one grid.  The per-element summation order is the one of the single-job kernels'
// block functions (colsum_fin_block, slab_sum_block): fixed, so a rerun is bit-identical.
#include "gine_common.hpp"
#include "gine_reduce.hpp"
#include "gine_slab.hpp"

namespace gine {
namespace {

constexpr int kFinCols = 8;  // MP jobs: columns per workgroup; also the eps-column limit

struct GradBatch {
  gine_grad_job job[GINE_GRAD_MAX_JOBS];
  int first[GINE_GRAD_MAX_JOBS + 1];     // first workgroup of each job
  int zfirst[GINE_GRAD_MAX_JOBS][5];     // SLAB: first workgroup of product z in the job
  int vec[GINE_GRAD_MAX_JOBS];           // SLAB: 16-byte loads allowed
  int n;
};

// [dW_e (D) | db_e (D)] in kFinCols-column workgroups, then one workgroup for the eps
// columns, whose totals are added in column order.
struct MpJobFin {
  float *dlin_w, *dlin_b, *deps;
  int D, neps, nb;
  __device__ int col(int b, int j) const {
    if (b == nb - 1) return j < neps ? 2 * D + j : -1;
    const int c = kFinCols * b + j;
    return c < 2 * D ? c : -1;
  }
  __device__ void finish(int b, const double* tot) const {
    const int t = threadIdx.x;
    if (b == nb - 1) {
      if (t == 0) {
        double s = 0.0;
        for (int j = 0; j < neps; ++j) s += tot[j];
        deps[0] = (float)s;
      }
      return;
    }
    const int c = kFinCols * b + t;
    if (t >= kFinCols || c >= 2 * D) return;
    if (c < D) dlin_w[c] = (float)tot[t];
    else dlin_b[c - D] = (float)tot[t];
  }
};

struct SlabJobOut {
  float* w;
  float* b;
  int64_t wsize, bsize;
  double bscale;
  __device__ void operator()(int, int64_t e, double v) const {
    if (e < wsize) w[e] = (float)v;
    else if (b != nullptr && e < wsize + bsize) b[e - wsize] = (float)(v * bscale);
  }
};

__host__ __device__ inline int mp_blocks(int D) { return (int)ceil_div(2 * D, kFinCols) + 1; }

__global__ __launch_bounds__(256) void k_grad_batch(GradBatch gb) {
  __shared__ __attribute__((aligned(16))) double s_mem[kSlabGroups * (kSlabQuads * 4 + 1)];
  int j = 0;
  while (j + 1 < gb.n && (int)blockIdx.x >= gb.first[j + 1]) ++j;
  const gine_grad_job& J = gb.job[j];
  const int lb = blockIdx.x - gb.first[j];
  if (J.kind == GINE_GRAD_JOB_MP) {
    const MpJobFin fin{J.w[0], J.w[1], J.w[2], J.channels, J.eps_cols, mp_blocks(J.channels)};
    constexpr int G = 256 / kFinCols;
    static_assert(G * kFinCols + kFinCols <= kSlabGroups * (kSlabQuads * 4 + 1), "LDS");
    colsum_fin_block<kFinCols, MpJobFin>(static_cast<const double*>(J.src), J.rows,
                                         3 * J.channels, fin, lb,
                                         reinterpret_cast<double(*)[kFinCols]>(s_mem),
                                         s_mem + G * kFinCols);
    return;
  }
  int z = 0;
  while (z + 1 < J.nz && lb >= gb.zfirst[j][z + 1]) ++z;
  const int bx = lb - gb.zfirst[j][z];
  const SlabJobOut out{J.w[z], J.b[z], J.wsize[z], J.per[z] - J.wsize[z], (double)J.bscale[z]};
  auto* s_part = reinterpret_cast<double(*)[kSlabQuads * 4 + 1]>(s_mem);
  const float* slab = static_cast<const float*>(J.src);
  if (gb.vec[j])
    slab_sum_block<true, SlabJobOut>(slab, J.rows, J.per[z], (size_t)J.cstride,
                                     (size_t)J.zstride, out, bx, z, s_part);
  else
    slab_sum_block<false, SlabJobOut>(slab, J.rows, J.per[z], (size_t)J.cstride,
                                      (size_t)J.zstride, out, bx, z, s_part);
}

int slab_job(gine_grad_job* job, const float* slab, int chunks, int64_t cstride,
             int64_t zstride, int nz) {
  if (!job || !slab || chunks <= 0 || nz <= 0 || nz > 4) return GINE_ERR_INVALID;
  *job = gine_grad_job{};
  job->kind = GINE_GRAD_JOB_SLAB;
  job->src = slab;
  job->rows = chunks;
  job->cstride = cstride;
  job->zstride = zstride;
  job->nz = nz;
  return GINE_OK;
}

void slab_product(gine_grad_job* job, int z, int64_t wsize, int64_t bsize, float* w, float* b,
                  float bscale = 1.0f) {
  job->per[z] = wsize + bsize;
  job->wsize[z] = wsize;
  job->w[z] = w;
  job->b[z] = b;
  job->bscale[z] = bscale;
}

}  // namespace
}  // namespace gine

using namespace gine;

extern "C" int gine_grad_finalize_batch(const gine_grad_job* jobs, int32_t num_jobs,
                                        void* stream) {
  if (num_jobs < 0 || num_jobs > GINE_GRAD_MAX_JOBS) return GINE_ERR_INVALID;
  if (num_jobs == 0) return GINE_OK;
  if (!jobs) return GINE_ERR_INVALID;
  GradBatch gb{};
  gb.n = num_jobs;
  int total = 0;
  for (int j = 0; j < num_jobs; ++j) {
    const gine_grad_job& J = jobs[j];
    gb.job[j] = J;
    gb.first[j] = total;
    if (!J.src || J.rows <= 0) return GINE_ERR_INVALID;
    if (J.kind == GINE_GRAD_JOB_MP) {
      if (J.channels <= 0 || J.eps_cols < 1 || J.eps_cols > kFinCols) return GINE_ERR_INVALID;
      if (!J.w[0] || !J.w[1] || !J.w[2]) return GINE_ERR_INVALID;
      total += mp_blocks(J.channels);
    } else if (J.kind == GINE_GRAD_JOB_SLAB) {
      if (J.nz < 1 || J.nz > 4 || J.cstride <= 0 || (J.nz > 1 && J.zstride <= 0))
        return GINE_ERR_INVALID;
      bool vec = (reinterpret_cast<uintptr_t>(J.src) & 15) == 0 && J.cstride % 4 == 0 &&
                 J.zstride % 4 == 0;
      int zb = 0;
      for (int z = 0; z < J.nz; ++z) {
        if (J.per[z] <= 0 || J.wsize[z] < 0 || J.wsize[z] > J.per[z] || !J.w[z])
          return GINE_ERR_INVALID;
        vec = vec && J.per[z] % 4 == 0;
        gb.zfirst[j][z] = zb;
        zb += (int)ceil_div(J.per[z], kSlabQuads * 4);
      }
      gb.zfirst[j][J.nz] = zb;
      gb.vec[j] = vec ? 1 : 0;
      total += zb;
    } else {
      return GINE_ERR_INVALID;
    }
  }
  gb.first[num_jobs] = total;
  hipLaunchKernelGGL(k_grad_batch, dim3((unsigned)total), dim3(256), 0, as_stream(stream), gb);
  GINE_LAUNCH_STATUS();
  return GINE_OK;
}
