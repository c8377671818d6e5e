/*
 * gine_hip.h -- C ABI of the MI355X (gfx950) GINEConv message-passing engine.
 *
 * This is the drop-in boundary for the hot path of SohirMaskey/raincast-gnn:
 *   models/gnn.py:20-29   ResGnn builds GINEConv(nn=Linear->BatchNorm1d->ReLU->Linear,
 *                          train_eps=True, edge_dim=1)
 *   models/gnn.py:41,44   conv(x, edge_index, edge_attr)   (called once per layer per step)
 * The arithmetic behind that call lives in torch_geometric (GINEConv.message /
 * MessagePassing.propagate / SumAggregation -> scatter_add_), which is not vendored in the
 * reference (environment.yml:29-31).  Every entry point below names the reference-side
 * operation it replaces.
 *
 * Conventions
 *   - All tensors are device pointers (HBM), row-major, contiguous, fp32 unless stated.
 *   - Every buffer (outputs and workspace) is allocated by the caller; no entry point
 *     allocates, frees or synchronises, so every call is legal inside hipGraph capture.
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).
 *   - Return value: GINE_OK, a GINE_ERR_* code, or GINE_ERR_HIP_BASE + hipError_t.
 *   - No hidden global state: the library holds nothing but its immutable kernels, so
 *     calls are re-entrant from any host thread (PyTorch runs backward on its autograd
 *     device thread).
 */
#ifndef GINE_HIP_H_
#define GINE_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GINE_ABI_VERSION 8  /* 2: adamw step-state query, gine_count_valid, window plan slot/edge_begin;
                              3: gine_deepset_bwd_num_partials takes the hidden width;
                              4: bn_acc grows two grid-barrier words (gine_mp_fwd_layer);
                              5: grid-barrier failure count (gine_bn_acc_barrier_failures_index),
                                 gine_mlp_bwd_layer removed;
                              6: gine_mlp_bwd_layer again, in the forward layer's role-split form;
                              7: gine_mp_fwd_layer takes the layer window plan
                                 (gine_graph_plan_layer_windows, gine_mp_fwd_layer_windows_fit);
                              8: gine_mp_fwd_layer can also run the output head (gine_layer_head) */

#define GINE_OK 0
#define GINE_ERR_INVALID 1    /* null pointer, negative size, bad flag */
#define GINE_ERR_DIM 2        /* unsupported channel count */
#define GINE_ERR_WORKSPACE 3  /* workspace smaller than gine_graph_workspace_bytes() */
#define GINE_ERR_TOO_LARGE 4  /* num_nodes or num_edges >= 2^31 */
#define GINE_ERR_HIP_BASE 1000

/* Library identity. */
int gine_abi_version(void);
const char* gine_status_string(int status);

/* ------------------------------------------------------------------------------------
 * Graph preparation.  Replaces the implicit per-call work of PyG's gather/scatter
 * (x.index_select(0, edge_index[0]) and zeros.scatter_add_(0, edge_index[1], .)) with
 * two stable counting structures built once per distinct edge_index:
 *   CSR by destination (in-edges):  in_rowptr[N+1], in_src[E], in_attr[E]
 *   CSR by source      (out-edges): out_rowptr[N+1], out_dst[E], out_attr[E]
 * Within a node's segment edges keep their original order (stable), which is exactly
 * the order in which CPU scatter_add_ / index_add_ accumulate.
 *   edge_index: int64 [2, E] (row 0 = source j, row 1 = target i; flow source_to_target)
 *   edge_attr : fp32 [E] (edge_dim = 1) or NULL (then in_attr/out_attr are not written)
 *   d_error   : device int32, OR-ed with 1 when an index lies outside [0, N); the caller
 *               zeroes it before the call and reads it when convenient.
 * Reference: utils/data.py:261-284 (edge layout), models/gnn.py:41,44 (consumer).
 * ---------------------------------------------------------------------------------- */
int gine_graph_workspace_bytes(int64_t num_nodes, int64_t num_edges, size_t* bytes);
int gine_graph_build(const int64_t* edge_index, const float* edge_attr, int64_t num_nodes,
                     int64_t num_edges, int32_t* in_rowptr, int32_t* in_src, float* in_attr,
                     int32_t* out_rowptr, int32_t* out_dst, float* out_attr, int32_t* d_error,
                     void* workspace, size_t workspace_bytes, void* stream);
/* Content check for the graph cache: *differ = 1 when edge_index_a [2, E] (int64, 16-byte
 * aligned) differs from edge_index_b or, if given, edge_attr_a [E] from edge_attr_b (bit
 * patterns); *differ is zeroed by the caller and otherwise left alone.  Lets a caller that
 * copies the same static graph to the device every step (train.py:62) reuse its CSRs and
 * window plans instead of rebuilding them.  differ may be mapped host memory: */
int gine_graph_same_edges(const int64_t* edge_index_a, const int64_t* edge_index_b,
                          const float* edge_attr_a, const float* edge_attr_b, int64_t num_edges,
                          int32_t* differ, void* stream);
/* the device address of pinned (page-locked) host memory (hipHostGetDevicePointer); an error
 * status when the memory is not mapped for the device. */
int gine_host_device_ptr(void* host_ptr, void** device_ptr);

/* ------------------------------------------------------------------------------------
 * Message passing forward.  Replaces GINEConv.forward up to (excluding) self.nn:
 *   m_e  = relu(x[src_e] + lin(a_e))                      (GINEConv.message, lin=Linear(1,D))
 *   agg_i = sum over in-edges of i, original edge order   (SumAggregation / scatter_add_)
 *   z_i  = agg_i + (1 + eps) * x_i                         (out + (1 + self.eps) * x_r)
 * Bit-identical to the CPU path (sequential per-destination order, no contraction).
 * The K=1 Linear's rounding is host-dependent in the reference itself: MKL's sgemm rounds
 * a*w+b once (fma) on Intel CPUs and twice (mul, then add) on AMD EPYC hosts, so the mode
 * is a flag: GINE_MP_LIN_MULADD selects mul-then-add, otherwise fma.
 *   x [N, D], lin_w [D] (Linear(1,D).weight flattened), lin_b [D], eps [1] (device), z [N, D]
 * Supported D: multiple of 4, 4 <= D <= 1024.
 * ---------------------------------------------------------------------------------- */
#define GINE_MP_LIN_MULADD 2
int gine_mp_fwd(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                const float* in_attr, const float* lin_w, const float* lin_b, const float* eps,
                float* z, int64_t num_nodes, int32_t channels, int32_t flags, void* stream);

/* ------------------------------------------------------------------------------------
 * Message passing backward (autograd of gine_mp_fwd), over the out-edge CSR:
 *   dm_e   = dz[dst_e] * 1[x[j] + lin(a_e) > 0]                    (gather + relu bwd)
 *   dx_j   = sum over out-edges of j in original order of dm_e   (index_add_, bit-exact)
 *            [+ (1 + eps) * dz_j  if flags & GINE_MP_BWD_SELF]
 *            [+ dres_j            if dres != NULL]
 *   partials[b] (fp64, a [3][D] row per block b): sum dm*a [D], sum dm [D], then the
 *            block's sum over channels of dz*x (one value; the rest of the row unused)
 *   flags may also carry GINE_MP_LIN_MULADD (must match the forward).
 * gine_mp_bwd_finalize reduces the partials in fixed block order into
 *   dlin_w [D], dlin_b [D], deps [1] (one launch).  Finalize calls may reduce IN PLACE:
 *   treat the partials buffer as consumed -- true of every *_finalize below too.
 * ---------------------------------------------------------------------------------- */
#define GINE_MP_BWD_SELF 1
int gine_mp_bwd_num_partials(int64_t num_nodes, int32_t channels, int32_t* num_partials);
int gine_mp_bwd(const float* dz, const float* x, const int32_t* out_rowptr,
                const int32_t* out_dst, const float* out_attr, const float* lin_w,
                const float* lin_b, const float* eps, const float* dres, float* dx,
                double* partials, int64_t num_nodes, int32_t channels, int32_t flags,
                void* stream);
int gine_mp_bwd_finalize(const double* partials, int32_t num_partials, int32_t channels,
                         float* dlin_w, float* dlin_b, float* deps, void* stream);
/* gine_mp_bwd plus, in the same launch, the fixed-order reduction of the node-MLP
 * weight-gradient slab that gine_mlp_bwd1_wgrad left when called with NULL dw1/db1/dw2/db2
 * (wg_chunks = gine_mlp_wgrad_num_chunks(num_nodes, mlp_channels)); writes dw1, db1, dw2,
 * db2 exactly as gine_mlp_wgrad would. */
int gine_mp_bwd_side(const float* dz, const float* x, const int32_t* out_rowptr,
                     const int32_t* out_dst, const float* out_attr, const float* lin_w,
                     const float* lin_b, const float* eps, const float* dres, float* dx,
                     double* partials, int64_t num_nodes, int32_t channels, int32_t flags,
                     const float* wg_slab, int32_t wg_chunks, int32_t mlp_channels, float* dw1,
                     float* db1, float* dw2, float* db2, void* stream);

/* ------------------------------------------------------------------------------------
 * Window-staged message passing (same results as gine_mp_fwd / gine_mp_bwd, bit for bit
 * for z and dx).  A PyG batch is a block-diagonal union of graphs (Batch.from_data_list,
 * train.py:155), so the neighbours of a run of consecutive nodes lie in one short run of
 * rows.  gine_graph_plan_windows (HOST pointers: a host copy of a CSR) cuts the nodes into
 * tiles of at most max_nodes nodes / max_edges edges whose neighbour window
 * [win_lo, win_lo + win_rows) spans at most max_rows rows; maxima[3] = the largest window
 * rows, tile edges and tile nodes.  *num_tiles = 0 means no plan (some node's own neighbour
 * span exceeds max_rows or its degree max_edges): use the gather entry points.
 * The kernels stage each tile's window slice of slice_channels (8, 16 or 32) channels in
 * LDS and read every neighbour row from there; channels % slice_channels == 0 and
 * channels / slice_channels <= 8.  The plan arrays are device copies.
 * gine_mp_bwd_win partials: num_tiles rows of fp64 [3][D]; gine_mp_bwd_win_finalize
 * reduces them (fixed order) into dlin_w, dlin_b, deps.
 * Replaces the same reference ops as gine_mp_fwd / gine_mp_bwd (models/gnn.py:41,44).
 * ---------------------------------------------------------------------------------- */
#define GINE_WINDOW_LDS_BYTES (80 * 1024)  /* two workgroups per CU (160 KiB LDS) */
typedef struct gine_window_plan {
  const int32_t* tile_begin; /* device [num_tiles + 1] */
  const int32_t* win_lo;     /* device [num_tiles] */
  const int32_t* win_rows;   /* device [num_tiles] */
  int32_t num_tiles;
  int32_t slice_channels;
  int32_t max_rows, max_edges, max_nodes;
  const int16_t* slot;       /* device [num_nodes] or NULL: gine_graph_plan_window_slots */
  const int32_t* edge_begin; /* device [num_tiles + 1] or NULL: rowptr[tile_begin[t]] */
} gine_window_plan;
int gine_graph_plan_windows(const int32_t* rowptr, const int32_t* nbr, int64_t num_nodes,
                            int32_t max_rows, int32_t max_nodes, int32_t max_edges,
                            int32_t* tile_begin, int32_t* win_lo, int32_t* win_rows,
                            int32_t* num_tiles, int32_t* maxima);
/* Work order inside the tiles of a backward (out-CSR) window plan (HOST pointers):
 * slot[tile_begin[t] + s] = the tile-local node a workgroup processes at position s.  A
 * lane group takes positions g and g + 64 one after the other; the order pairs each tile's
 * nodes by out-degree (heaviest with lightest, ties by index), so the groups of a wave run
 * chains of similar length.  Per-node results are unchanged (each node's edges are still
 * summed in their own order). */
int gine_graph_plan_window_slots(const int32_t* rowptr, const int32_t* tile_begin,
                                 int32_t num_tiles, int16_t* slot);
/* Locality order of a graph's nodes (HOST pointers: a host copy of a CSR, either
 * direction; the adjacency is symmetrised).  order[i] = the node placed at position i:
 * reverse Cuthill-McKee, deterministic.  Relabelling a static station graph this way before
 * batching (raincast_gnn.data.relabel_stations) narrows every tile's neighbour window (the
 * reference's dataset order, utils/data.py:261-284, scatters k-NN neighbours over the whole
 * graph).  Per-node results are unchanged: each node keeps its in/out edges in their
 * original relative order. */
int gine_graph_order_locality(const int32_t* rowptr, const int32_t* nbr, int64_t num_nodes,
                              int32_t* order);
int gine_mp_fwd_win(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                    const float* in_attr, const float* lin_w, const float* lin_b,
                    const float* eps, float* z, int64_t num_nodes, int32_t channels,
                    int32_t flags, const gine_window_plan* plan, void* stream);
int gine_mp_bwd_win(const float* dz, const float* x, const int32_t* out_rowptr,
                    const int32_t* out_dst, const float* out_attr, const float* lin_w,
                    const float* lin_b, const float* eps, const float* dres, float* dx,
                    double* partials, int64_t num_nodes, int32_t channels, int32_t flags,
                    const gine_window_plan* plan, void* stream);
int gine_mp_bwd_win_side(const float* dz, const float* x, const int32_t* out_rowptr,
                         const int32_t* out_dst, const float* out_attr, const float* lin_w,
                         const float* lin_b, const float* eps, const float* dres, float* dx,
                         double* partials, int64_t num_nodes, int32_t channels, int32_t flags,
                         const gine_window_plan* plan, const float* wg_slab, int32_t wg_chunks,
                         int32_t mlp_channels, float* dw1, float* db1, float* dw2, float* db2,
                         void* stream);
/* gine_mp_bwd_win + the node-MLP weight-gradient engine of the same GINE layer in ONE launch
 * (D = 64 or 128, slice_channels = 32): extra workgroups write the fp32 slab
 * [2][gine_mlp_wgrad_num_chunks][D*D + D] exactly as gine_mlp_wgrad does with NULL outputs
 * (operands dy, y, mask, a1, bn_save, dbn, coef, z, epilogue as for gine_mlp_wgrad), while
 * the window workgroups run the message-passing backward; the slab is then reduced by
 * gine_grad_finalize_batch.  Replaces the same reference ops as gine_mp_bwd and
 * gine_mlp_wgrad (models/gnn.py:21-26,41,44 autograd).  GINE_ERR_INVALID when the plan's
 * slice is not 32 channels. */
int gine_mp_bwd_win_mlp_wgrad(const float* dz, const float* x, const int32_t* out_rowptr,
                              const int32_t* out_dst, const float* out_attr,
                              const float* lin_w, const float* lin_b, const float* eps,
                              const float* dres, float* dx, double* partials,
                              int64_t num_nodes, int32_t channels, int32_t flags,
                              const gine_window_plan* plan, const float* dy, const float* y,
                              const uint8_t* mask, const float* a1, const float* bn_save,
                              const float* dbn, const float* coef, const float* z, float* slab,
                              int32_t epilogue, void* stream);
int gine_mp_bwd_win_finalize(const double* partials, int32_t num_tiles, int32_t channels,
                             int32_t slice_channels, float* dlin_w, float* dlin_b,
                             float* deps, void* stream);

/* ------------------------------------------------------------------------------------
 * Batched gradient finish.  The parameter-gradient reductions that nothing reads before
 * the optimizer -- dW_e/db_e/eps of every GINE layer (gine_mp_bwd*_finalize), the head's
 * and the dense chain's weight-gradient slabs, the DeepSet dW1 slab -- in ONE launch at the
 * end of the backward instead of one launch each (autograd of the Linear/GINEConv
 * parameters, models/gnn.py; reduced by the reference's autograd as separate mm/sum ops).
 *   GINE_GRAD_JOB_MP:   src = fp64 partial rows [rows][3*channels] as gine_mp_bwd (eps at
 *                       column 2D, eps_cols = 1) or gine_mp_bwd_win (eps at 2D + slice,
 *                       eps_cols = slices) write them; w[0] = dlin_w [D], w[1] = dlin_b
 *                       [D], w[2] = deps [1].
 *   GINE_GRAD_JOB_SLAB: src = fp32 slab, element e of product z < nz at
 *                       src + z*zstride + c*cstride + e for chunks c < rows; product z has
 *                       per[z] elements: e < wsize[z] -> w[z][e], else b[z][e - wsize[z]]
 *                       (times bscale[z]).  Sums in fp64, fixed order.
 * The *_grad_job entry points (host only) describe the slab a producer left when called
 * with NULL gradient outputs.  At most GINE_GRAD_MAX_JOBS jobs per launch.
 * ---------------------------------------------------------------------------------- */
#define GINE_GRAD_JOB_MP 1
#define GINE_GRAD_JOB_SLAB 2
#define GINE_GRAD_MAX_JOBS 12
typedef struct gine_grad_job {
  int32_t kind;
  int32_t rows;      /* MP: partial rows; SLAB: chunks */
  int32_t channels;  /* MP: D */
  int32_t eps_cols;  /* MP: eps columns */
  int32_t nz;        /* SLAB: products (<= 4) */
  int32_t pad_;
  const void* src;
  int64_t cstride, zstride;  /* SLAB, in floats */
  int64_t per[4];
  int64_t wsize[4];
  float bscale[4];
  float* w[4];
  float* b[4];
} gine_grad_job;
int gine_grad_finalize_batch(const gine_grad_job* jobs, int32_t num_jobs, void* stream);
int gine_head_bwd_grad_job(int64_t num_nodes, int32_t channels, int32_t kind, const float* slab,
                           float* dw, float* db, gine_grad_job* job);
int gine_chain_wgrad_grad_job(int64_t num_nodes, int32_t hidden, int32_t in_features,
                              const float* slab, float bias_scale, float* dwp2, float* dbp2,
                              float* dwr0, float* dbr0, float* dwr1, float* dbr1, float* dwdr,
                              float* dbdr, gine_grad_job* job);
int gine_deepset_bwd_grad_job(int64_t num_nodes, int32_t in_features, int32_t hidden,
                              const float* slab, float* dw1, float* db1, gine_grad_job* job);

/* ------------------------------------------------------------------------------------
 * Node MLP  nn = Sequential(Linear(D,D), BatchNorm1d(D), ReLU(), Linear(D,D))
 * (models/gnn.py:21-26), plus the ResGnn epilogue (models/gnn.py:38-44).
 * fp32 MFMA (v_mfma_f32_32x32x2_f32) row-tile GEMMs with fused prologues/epilogues.
 * Supported D: 32, 64, 128, 256.
 *
 * Forward, training mode:
 *   gine_mlp_fwd1:      a1 = z W1^T + b1; per-block fp64 partial sums of a1 and a1^2
 *   gine_bn_fwd_finalize: mean, biased var -> invstd; running stats update
 *                       (momentum, unbiased var); bn_save = [mean | invstd | alpha | shift]
 *                       with alpha = gamma*invstd, shift = beta - mean*alpha
 *                       (eval mode: from running stats, partials unused)
 *   gine_mlp_fwd2:      r = relu(a1*alpha + shift); o = r W2^T + b2;
 *                       y = o | relu(o) | x + relu(o)   (epilogue 0 | 1 | 2)
 *                       mask[n,c] = (o > 0) stored as uint8 for epilogue 2 (may be NULL else)
 * Backward:
 *   gine_mlp_bwd2:      do = dy*1[o>0] (per epilogue); dr = do W2; dbn = dr*1[bn>0];
 *                       partials of sum dbn, sum dbn*xhat
 *   gine_bn_bwd_finalize: dgamma, dbeta, and coef = [c1 | c2 | c3] with
 *                       da1 = c1*dbn + c2*xhat + c3
 *   gine_mlp_bwd1:      dz = da1 W1
 *   gine_mlp_wgrad:     dW2 = do^T r, db2 = sum do, dW1 = da1^T z, db1 = sum da1
 *                       (split over row chunks; fp32 partial slabs reduced in fixed order)
 * ---------------------------------------------------------------------------------- */
#define GINE_EPI_NONE 0
#define GINE_EPI_RELU 1
#define GINE_EPI_RESIDUAL_RELU 2

int gine_mlp_num_partials(int64_t num_nodes, int32_t channels, int32_t* num_partials);
int gine_mlp_fwd1(const float* z, const float* w1, const float* b1, float* a1, double* partials,
                  int64_t num_nodes, int32_t channels, void* stream);
int gine_bn_fwd_finalize(const double* partials, int32_t num_partials, const float* gamma,
                         const float* beta, float* running_mean, float* running_var,
                         int64_t* num_batches_tracked, float* bn_save, int64_t num_nodes,
                         int32_t channels, float momentum, float bn_eps, int32_t training,
                         int32_t update_running, void* stream);
int gine_mlp_fwd2(const float* a1, const float* bn_save, const float* w2, const float* b2,
                  const float* x, float* y, uint8_t* mask, int64_t num_nodes, int32_t channels,
                  int32_t epilogue, void* stream);

/* Fused forward message passing + first Linear (D = 128 only): z exactly as gine_mp_fwd and
 * a1 / partials exactly as gine_mlp_fwd1 (bit-identical; partials has gine_mlp_num_partials
 * rows), in one launch whose workgroups gather the next 32-row tile of z while the matrix
 * cores multiply the current one (csrc/gine_mpmlp.hip).  Requires every in-degree <=
 * GINE_MP_FUSED_MAX_DEGREE: the caller passes the graph's maximum in-degree and gets
 * GINE_ERR_INVALID above it (-> the unfused pair); GINE_ERR_DIM for channels != 128.
 * flags: GINE_MP_LIN_MULADD as for gine_mp_fwd.
 * Replaces models/gnn.py:41,44 (GINEConv.propagate + nn[0] Linear + BN batch statistics). */
#define GINE_MP_FUSED_MAX_DEGREE 32
int gine_mp_fwd_mlp1(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                     const float* in_attr, const float* lin_w, const float* lin_b,
                     const float* eps, const float* w1, const float* b1, float* z, float* a1,
                     double* partials, int64_t num_nodes, int32_t channels,
                     int32_t max_in_degree, int32_t flags, void* stream);

/* BatchNorm statistics without a finish launch (training, momentum >= 0; csrc/gine_bnacc.hpp).
 * bn_acc: int64[gine_bn_acc_words(D)] (query it: the size follows the build-time replica count
 * R = GINE_BNACC_REPLICAS, (3R + 1 + 8) * 2D + 3 + 288 words, the 288 being the one-launch
 * layer's grid barrier: 18 lines of 16 words), zeroed once by the caller at allocation,
 * then owned by the kernels (the sums only grow; each consumer differences them against a
 * snapshot the previous consumer left), so one buffer serves every step of one BatchNorm,
 * HIP-graph replays included.  Every producer launch must be followed by exactly one
 * gine_mlp_fwd2_bn on the same buffer; not shared by layers whose launches interleave.  A
 * consumer that finds the pairing broken (the producer's phase moved by more than one since
 * the last consumer) emits NaN statistics for that step; re-zero the buffer to recover.
 *   gine_mlp_fwd1_acc / gine_mp_fwd_mlp1_acc: as gine_mlp_fwd1 / gine_mp_fwd_mlp1, and the
 *     per-workgroup sums are also added into bn_acc as 3-word fixed point (2^0 / 2^-32 /
 *     2^-64) with integer atomics (order-independent: same bits every run); NaN / +Inf /
 *     -Inf workgroup sums are counted instead and give NaN / +Inf / -Inf column sums, as
 *     ATen's do.  partials may be NULL.
 *   gine_mlp_fwd2_bn: gine_bn_fwd_finalize (from bn_acc) + gine_mlp_fwd2 in one launch;
 *     writes bn_save, the running statistics and num_batches_tracked as the finalize does.
 * The statistics agree with the partials path to ~1e-15 relative (sums are rounded to
 * 2^-64 per workgroup), so bn_save can differ from it in the last fp32 bit. */
int gine_bn_acc_words(int32_t channels, int64_t* words);
/* Index (int64 words into bn_acc) of the grid-barrier failure count: gine_mp_fwd_layer adds 1
 * there for every workgroup whose grid barrier timed out (~2 s: the grid was not resident at
 * once -- other work held CUs).  Such a launch's outputs are NaN in those workgroups' rows,
 * bn_save is NaN if workgroup 0 failed, and the running statistics are left as they were.
 * The caller reads the word at its synchronisation points and raises on a non-zero value;
 * re-zero the buffer afterwards (raincast_gnn.functional.check_grid_barriers). */
int gine_bn_acc_barrier_failures_index(int32_t channels, int64_t* index);
/* Backward, same scheme (a second accumulator per BatchNorm): gine_mlp_bwd2_acc = gine_mlp_bwd2
 * with the [sum dbn | sum dbn*xhat] sums into bn_acc (partials may be NULL);
 * gine_mlp_bwd1_bn = gine_bn_bwd_finalize (training) + gine_mlp_bwd1 in one launch (writes
 * coef, dgamma, dbeta; dgamma / dbeta may be NULL). */
int gine_mlp_bwd2_acc(const float* dy, const float* y, const uint8_t* mask, const float* a1,
                      const float* bn_save, const float* w2, float* dbn, double* partials,
                      int64_t* bn_acc, int64_t num_nodes, int32_t channels, int32_t epilogue,
                      void* stream);
int gine_mlp_bwd1_bn(const float* dbn, const float* a1, const float* bn_save, int64_t* bn_acc,
                     const float* gamma, float* dgamma, float* dbeta, float* coef,
                     const float* w1, float* dz, int64_t num_nodes, int32_t channels,
                     void* stream);
/* The backward pair in ONE launch (csrc/gine_mlpbwd.hip k_mlp_bwd_layer; replaces
 * gine_mlp_bwd2_acc followed by gine_mlp_bwd1_bn, models/gnn.py:21-26 autograd): phase A =
 * dbn and the BatchNorm-backward sums, grid barrier, phase B = coef (workgroup 0 also writes
 * coef, dgamma, dbeta) and dz = da1 W1 -- both row tiles of a workgroup stay in LDS, W1 is
 * loaded under phase A.  Same outputs, bit for bit, as the pair (dbn, dz, coef, dgamma,
 * dbeta) and the same pairing protocol on bn_acc (the backward accumulator); a barrier that
 * cannot complete is counted at gine_bn_acc_barrier_failures_index and makes that launch's
 * coef / dz NaN.  Applies where gine_mlp_bwd_layer_ok says so: channels = 128, at most 2
 * row tiles per workgroup and the whole grid resident at once (occupancy query, cached per
 * device); GINE_ERR_INVALID otherwise.  gamma, dgamma, dbeta may be NULL; y (GINE_EPI_RELU)
 * and mask (GINE_EPI_RESIDUAL_RELU) as for gine_mlp_bwd2. */
int gine_mlp_bwd_layer_ok(int64_t num_nodes, int32_t channels, int32_t* ok);
int gine_mlp_bwd_layer(const float* dy, const float* y, const uint8_t* mask, const float* a1,
                       const float* bn_save, const float* w2, float* dbn, int64_t* bn_acc,
                       const float* gamma, float* dgamma, float* dbeta, float* coef,
                       const float* w1, float* dz, int64_t num_nodes, int32_t channels,
                       int32_t epilogue, void* stream);
/* Testing only: `extra` workgroups added to every later gine_mlp_bwd_layer grid (0 restores
 * production), for the barrier-failure test. */
int gine_testing_bwd_layer_extra_workgroups(int32_t extra);
int gine_mlp_fwd1_acc(const float* z, const float* w1, const float* b1, float* a1,
                      double* partials, int64_t* bn_acc, int64_t num_nodes, int32_t channels,
                      void* stream);
int gine_mp_fwd_mlp1_acc(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                         const float* in_attr, const float* lin_w, const float* lin_b,
                         const float* eps, const float* w1, const float* b1, float* z,
                         float* a1, double* partials, int64_t* bn_acc, int64_t num_nodes,
                         int32_t channels, int32_t max_in_degree, int32_t flags, void* stream);
/* The whole node-MLP forward of a GINE layer in ONE launch (models/gnn.py:41-44: propagate +
 * nn + ResGnn's ReLU / residual): gine_mp_fwd_mlp1_acc and gine_mlp_fwd2_bn on the same
 * workgroups, separated by a grid barrier (csrc/gine_mpmlp.hip k_mp_fwd_layer) -- every a1
 * tile stays in LDS between the halves, W2 is staged under the barrier's wait.  Same
 * outputs, bit for bit, as the pair (z, a1, bn_save, running statistics, y, mask), same
 * pairing protocol on bn_acc (the barrier words at its end, gine_bn_acc_words; a barrier that
 * cannot complete is counted there, gine_bn_acc_barrier_failures_index).
 * Applies where gine_mp_fwd_layer_ok says so: channels = 128, max_in_degree <=
 * GINE_MP_FUSED_MAX_DEGREE, at most 2 row tiles per workgroup and the whole grid resident
 * on the device at once (occupancy query, cached per device); GINE_ERR_INVALID otherwise. */
int gine_mp_fwd_layer_ok(int64_t num_nodes, int32_t channels, int32_t max_in_degree, int32_t* ok);
/* Testing only: `extra` workgroups added to every later gine_mp_fwd_layer grid (0 restores
 * production), so a test can launch a grid the device cannot hold at once and check that the
 * barrier's failure reaches the host (gine_bn_acc_barrier_failures_index). */
int gine_testing_layer_extra_workgroups(int32_t extra);
/* Testing only: the output head's 32-lane butterfly sum (csrc/gine_headrow.hpp sum_32; mode 1)
 * against the __shfl_xor butterfly it stands for (mode 0), on `waves` x 64 floats. */
int gine_testing_sum_32(const float* in, float* out, int32_t waves, int32_t mode, void* stream);
/* With a layer window plan (tile_windows != NULL; ABI 7) every workgroup stages each of its
 * 32-row tiles' neighbour rows -- the tile's window, one contiguous run of rows -- in LDS once
 * and sums the messages from there (per-destination LDS staging; same bits as the gather);
 * window_rows is the plan's largest window and (window_rows, max_in_degree) must pass
 * gine_mp_fwd_layer_windows_fit (GINE_ERR_INVALID otherwise).  NULL: neighbour rows are
 * gathered from L2 (any graph). */
/* The output head folded into the last layer's launch (ABI 8; models/gnn.py:140-141,
 * GNN.aggr + PostProcess): with head != NULL the epilogue also evaluates gine_head_fwd on the
 * rows it writes -- raw = y W^T + b, pred = PostProcess(raw) -- with the same lane layout,
 * fma order and butterfly as k_head_fwd (same bits), and, with y_target != NULL, the loss's
 * GINE_COUNT_PARTS valid-target partial counts (gine_head_fwd_count).  One launch fewer
 * and h is not read back.  kind: GINE_LOSS_* (K = 2..5 outputs per node). */
typedef struct gine_layer_head {
  const float* weight;    /* [K, 128] (GNN.aggr.weight) */
  const float* bias;      /* [K] */
  float* raw;             /* [N, K] pre-PostProcess output (what gine_head_bwd reads) */
  float* pred;            /* [N, K] */
  const float* y_target;  /* [N] batch targets, or NULL */
  uint32_t* count_parts;  /* GINE_COUNT_PARTS partial counts (with y_target), or NULL */
  int32_t kind;           /* GINE_LOSS_* */
} gine_layer_head;
int gine_mp_fwd_layer(const float* x, const int32_t* in_rowptr, const int32_t* in_src,
                      const float* in_attr, const float* lin_w, const float* lin_b,
                      const float* eps, const float* w1, const float* b1, float* z, float* a1,
                      int64_t* bn_acc, const float* gamma, const float* beta,
                      float* running_mean, float* running_var, int64_t* num_batches_tracked,
                      float* bn_save, float momentum, float bn_eps, int32_t update_running,
                      const float* w2, const float* b2, float* y, uint8_t* mask,
                      int64_t num_nodes, int32_t channels, int32_t max_in_degree, int32_t flags,
                      int32_t epilogue, const int32_t* tile_windows, int32_t window_rows,
                      const gine_layer_head* head, void* stream);
/* The layer window plan of a graph (built once per graph, like its CSRs): for every 32-row
 * tile of destinations, tile_windows[2T] = first row and tile_windows[2T + 1] = number of rows
 * of the run [lo, lo + rows) holding the tile's own rows and all their in-neighbours (int32
 * [ceil(N / 32)][2], device), and maxima[0] / maxima[1] = the largest window and the largest
 * number of in-edges of a tile (int32[2], device; zeroed by the call).  The caller reads the
 * maxima back once and asks gine_mp_fwd_layer_windows_fit (largest window, the graph's largest
 * in-degree) whether the plan fits the launch's LDS: (rows + 1) x 512 B of window rows (a -inf
 * dummy row last), 32 x round_up(max_in_degree, 4) x 8 B of padded slot table and 33 rowptr
 * words within 73,712 B, rows <= 144 (cfg2's 500-station k = 10 graphs in the locality order:
 * about 129 rows, in-degree 11).
 * Replaces nothing in the reference: the data movement of PyG's x.index_select per tile. */
int gine_graph_plan_layer_windows(const int32_t* in_rowptr, const int32_t* in_src,
                                  int64_t num_nodes, int32_t* tile_windows, int32_t* maxima,
                                  void* stream);
int gine_mp_fwd_layer_windows_fit(int32_t window_rows, int32_t max_in_degree, int32_t* ok);
int gine_mlp_fwd2_bn(const float* a1, int64_t* bn_acc, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, int64_t* num_batches_tracked,
                     float* bn_save, float momentum, float bn_eps, int32_t update_running,
                     const float* w2, const float* b2, const float* x, float* y,
                     uint8_t* mask, int64_t num_nodes, int32_t channels, int32_t epilogue,
                     void* stream);

int gine_mlp_bwd2(const float* dy, const float* y, const uint8_t* mask, const float* a1,
                  const float* bn_save, const float* w2, float* dbn, double* partials,
                  int64_t num_nodes, int32_t channels, int32_t epilogue, void* stream);
int gine_bn_bwd_finalize(const double* partials, int32_t num_partials, const float* gamma,
                         const float* bn_save, float* dgamma, float* dbeta, float* coef,
                         int64_t num_nodes, int32_t channels, int32_t training, void* stream);
int gine_mlp_bwd1(const float* dbn, const float* a1, const float* bn_save, const float* coef,
                  const float* w1, float* dz, int64_t num_nodes, int32_t channels,
                  void* stream);
int gine_mlp_wgrad_num_chunks(int64_t num_nodes, int32_t channels, int32_t* num_chunks);
/* dw1, db1, dw2, db2 all NULL: only the fp32 slab [2][chunks][D*D + D] is written (for a
 * batched reduction, gine_grad_finalize_batch). */
int gine_mlp_wgrad(const float* dy, const float* y, const uint8_t* mask, const float* a1,
                   const float* bn_save, const float* dbn, const float* coef, const float* z,
                   float* slab, float* dw1, float* db1, float* dw2, float* db2,
                   int64_t num_nodes, int32_t channels, int32_t epilogue, void* stream);

/* gine_mlp_bwd1 + gine_mlp_wgrad in one launch (same arguments as the two; the weight
 * gradients and dz are computed side by side on the CUs).  Same results bit for bit. */
int gine_mlp_bwd1_wgrad(const float* dy, const float* y, const uint8_t* mask, const float* a1,
                        const float* bn_save, const float* dbn, const float* coef,
                        const float* z, const float* w1, float* dz, float* slab, float* dw1,
                        float* db1, float* dw2, float* db2, int64_t num_nodes,
                        int32_t channels, int32_t epilogue, void* stream);

/* ------------------------------------------------------------------------------------
 * AdamW over one flat fp32 parameter buffer (the optimizer of the benchmarked training
 * step, train.py:67-69 with torch.optim.AdamW, lr from params.json).  Bumps the device
 * step counter `step` (fp32 [288]: the count, a ticket word, and at floats 32 + 32 g
 * (g < 8) the sub-tickets of a two-level ticket, one per 128-byte line; every ticket word
 * must start at 0 and is left at 0) and updates param / exp_avg / exp_avg_sq in place with torch.optim.AdamW's
 * default (amsgrad=False) formulation.  One launch, graph-safe; the four buffers must be
 * 16-byte aligned (float4 accesses).
 * ---------------------------------------------------------------------------------- */
int gine_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                    float* step, int64_t n, float lr, float beta1, float beta2, float eps,
                    float weight_decay, void* stream);
/* Length in floats of gine_adamw_step's `step` buffer (288 since ABI 2). */
int gine_adamw_state_floats(int64_t* floats);

/* ------------------------------------------------------------------------------------
 * Fused CRPS losses (models/loss.py) over the post-processed predictions pred [N, K]
 * (models/model_utils.py PostProcess output) and targets y [N] (NaN = missing):
 *   GINE_LOSS_NORMAL        NormalCRPS.crps         (loss.py:335-369)   K = 2
 *   GINE_LOSS_MIXED_NORMAL  MixedNormalCRPS.crps    (loss.py:6-68)      K = 3
 *   GINE_LOSS_MIXED         MixedLoss(grad_u=False) (loss.py:71-272)    K = 4, u fixed
 *   GINE_LOSS_MIXED_U       MixedLoss(grad_u=True)                      K = 5, u learned
 * gine_crps_fwd: per node the closed form and its exact gradient w.r.t. pred (fp64
 * forward-mode duals) into dpred [N, K]; per-block partials [P][2]; loss_out[0] = mean over
 * non-NaN targets, count_out[0] = their number, written by the workgroup that finishes
 * last (ticket: a device uint32 the caller zeroes ONCE; every call leaves it at 0 again;
 * calls sharing a ticket must not overlap).  c = censoring point (log 0.01), t = sigmoid
 * temperature of grad_u, xi = GPD shape, u = fixed threshold.
 * gine_crps_bwd: grad_pred = gloss[0] * dpred / count (fp32).
 * gine_count_valid: the number of non-NaN y as GINE_COUNT_PARTS uint32 partial counts
 * (count_parts; their sum is the count) -- the count_parts of gine_crps_fwd_grad, recounted
 * every step (inside a captured step too).  gine_head_fwd_count writes the same partials
 * beside the head forward, so a training step needs no launch for them.
 * ---------------------------------------------------------------------------------- */
#define GINE_LOSS_NORMAL 0
#define GINE_LOSS_MIXED_NORMAL 1
#define GINE_LOSS_MIXED 2
#define GINE_LOSS_MIXED_U 3
int gine_crps_num_partials(int64_t num_nodes, int32_t* num_partials);
int gine_crps_fwd(const float* pred, const float* y, int64_t num_nodes, int32_t kind, double u,
                  double xi, double c, double t, double* dpred, double* partials,
                  double* loss_out, double* count_out, uint32_t* ticket, void* stream);
int gine_crps_bwd(const double* dpred, const double* count, const double* gloss,
                  int64_t num_nodes, int32_t kind, float* grad_pred, void* stream);
#define GINE_COUNT_PARTS 64
int gine_count_valid(const float* y, int64_t num_nodes, uint32_t* count_parts, void* stream);
/* gine_crps_fwd that also writes grad_unit = (float)(dpred / count), the gradient for
 * gloss = 1 exactly as gine_crps_bwd would round it, given the count of non-NaN targets
 * up front (count_parts: GINE_COUNT_PARTS device uint32 partial counts of y, from
 * gine_count_valid or gine_head_fwd_count) -- a backward seeded with 1 then needs no launch. */
int gine_crps_fwd_grad(const float* pred, const float* y, int64_t num_nodes, int32_t kind,
                       double u, double xi, double c, double t, double* dpred, double* partials,
                       double* loss_out, double* count_out, uint32_t* ticket,
                       const uint32_t* count_parts, float* grad_unit, void* stream);
/* gine_crps_fwd_grad that also runs the output head's backward for that unit seed (the head
 * of gine_head_fwd: raw [N, K], its input h [N, channels], weight w [K, channels]): dh
 * [N, channels] as gine_head_bwd writes it from grad_pred = grad_unit, and per-workgroup dW |
 * db partials in head_slab (gine_crps_head_slab_floats() floats; gine_crps_head_grad_job
 * describes them for gine_grad_finalize_batch).  One launch instead of three (crps, crps_bwd,
 * head_bwd) for a training step's loss.backward() seeded with 1. */
int gine_crps_head_slab_floats(int64_t num_nodes, int32_t channels, int32_t kind,
                               size_t* floats);
int gine_crps_head_fwd_grad(const float* pred, const float* y, int64_t num_nodes, int32_t kind,
                            double u, double xi, double c, double t, double* dpred,
                            double* partials, double* loss_out, double* count_out,
                            uint32_t* ticket, const uint32_t* count_parts, float* grad_unit,
                            const float* raw, const float* h, const float* w, int32_t channels,
                            float* dh, float* head_slab, void* stream);
int gine_crps_head_grad_job(int64_t num_nodes, int32_t channels, int32_t kind,
                            const float* head_slab, float* dw, float* db, gine_grad_job* job);

/* ------------------------------------------------------------------------------------
 * Weight/bias gradient of a plain Linear y = x W^T + b over many rows (the DeepSet,
 * dim_red and aggr layers around the GINE stack, models/gnn.py:48-68,112-123):
 *   dw [O, I] = dy^T x,  db [O] = bias_scale * sum_rows dy  (db may be NULL)
 * (bias_scale: y = x W^T + bias_scale * b, e.g. the DeepSet member sum of a bias)
 * dy [rows, O], x [rows, I] row-major fp32.  Rows are split into chunks
 * (gine_linear_wgrad_num_chunks); slab holds chunks * (O*I + O) floats of partials,
 * reduced in fixed order (deterministic).
 * ---------------------------------------------------------------------------------- */
int gine_linear_wgrad_num_chunks(int64_t rows, int32_t out_features, int32_t in_features,
                                 int32_t* num_chunks);
int gine_linear_wgrad(const float* dy, const float* x, int64_t rows, int32_t out_features,
                      int32_t in_features, float* slab, float* dw, float* db, float bias_scale,
                      void* stream);

/* ------------------------------------------------------------------------------------
 * DeepSetEncoder phi first layer + ReLU + member sum, fused (models/gnn.py:48-68,
 * replaces phi[0](x) -> phi[1] ReLU -> .sum(dim=1) of the reference's Sequential; the
 * member-sum moves before phi[2] because a Linear commutes with the sum):
 *   r [N, H] = sum_m relu(ens[n, m, :] w1^T + b1)
 * ens [N, M, F] (row-major, contiguous), w1 [H, F], b1 [H], fp32.
 * H in {32, 64, 128, 256}; 1 <= F <= 64; M >= 1.  The [N, M, H] activation is never
 * written to memory; mask (optional, gine_deepset_mask_bytes bytes) receives its ReLU
 * pattern as bits, for the backward.
 * gine_deepset_bwd: weight gradients for dr = d loss / d r from the forward's mask:
 *   dw1 [H, F] = sum_{n,m} (dr[n] * 1[pre > 0])^T ens[n, m],  db1 [H] likewise summed
 * slab: gine_deepset_bwd_num_partials(N, H) * (H*F + H) floats of per-workgroup partials,
 * reduced in fixed order (deterministic).  db1 may be NULL.
 * ---------------------------------------------------------------------------------- */
int gine_deepset_mask_bytes(int64_t num_nodes, int32_t members, int32_t hidden, size_t* bytes);
/* Layout of the mask (for test-side decoding of the forward's ReLU decisions): nodes are
 * walked in groups of 2G (*nodes_per_half = G); the uint16 word
 * [(g * ceil(G*M/16) + t) * 2H + (c / 32) * 64 + 32 * h + c % 32] holds in bit q the decision
 * for hidden unit c of group row G*M*h + 16*t + q, i.e. node 2G*g + G*h + (16t+q) / M,
 * member (16t+q) % M (rows past G*M or past N are padding, bit 0). */
int gine_deepset_mask_layout(int64_t num_nodes, int32_t hidden, int32_t* nodes_per_half);
int gine_deepset_fwd(const float* ens, const float* w1, const float* b1, float* r,
                     uint16_t* mask, int64_t num_nodes, int32_t members, int32_t in_features,
                     int32_t hidden, void* stream);
/* gine_deepset_fwd plus the dense chain's folded dim_red weight (W' | b' | W'^T of
 * gine_chain_fwd_folded, hidden in {64, 128}, x_features <= 64) into wfold, computed by
 * extra workgroups of the same launch for gine_chain_fwd_folded3. */
int gine_deepset_fwd_fold(const float* ens, const float* w1, const float* b1, float* r,
                          uint16_t* mask, int64_t num_nodes, int32_t members,
                          int32_t in_features, int32_t hidden, const float* wr1,
                          const float* br1, const float* wdr, const float* bdr, float* wfold,
                          int32_t x_features, void* stream);
/* gine_deepset_fwd_fold plus the doubly folded chain's [Wf | bf] (Wf = Wr0 Wp2 [D][D],
 * bf = members * Wr0 bp2 + br0 [D]) into wfold2 [D*D + D], by a second set of extra
 * workgroups, for gine_chain_fwd_folded2 (wr0 / br0 = rho[0], wp2 / bp2 = phi[2]). */
int gine_deepset_fwd_fold2(const float* ens, const float* w1, const float* b1, float* r,
                           uint16_t* mask, int64_t num_nodes, int32_t members,
                           int32_t in_features, int32_t hidden, const float* wr1,
                           const float* br1, const float* wdr, const float* bdr, float* wfold,
                           int32_t x_features, const float* wr0, const float* br0,
                           const float* wp2, const float* bp2, float* wfold2, void* stream);
int gine_deepset_bwd_num_partials(int64_t num_nodes, int32_t hidden, int32_t* num_partials);
int gine_deepset_bwd(const float* ens, const uint16_t* mask, const float* dr, float* slab,
                     float* dw1, float* db1, int64_t num_nodes, int32_t members,
                     int32_t in_features, int32_t hidden, void* stream);

/* ------------------------------------------------------------------------------------
 * Output head: aggr = Linear(D, K) + PostProcess (models/gnn.py:123,125,140-141;
 * models/model_utils.py:42-113), K and the column transforms given by the loss `kind`
 * (GINE_LOSS_*, K = 2, 3, 4, 5):  pred[:, 0] = raw (mu); sigma, sigma_u -> softplus + 1e-6;
 * p -> sigmoid; u (GINE_LOSS_MIXED_U) -> 2.12 * sigmoid.
 *   gine_head_fwd: raw [N, K] = h [N, D] W^T + b;  pred [N, K] = PostProcess(raw)
 *   gine_head_bwd: d raw = PostProcess'(raw) * grad_pred;  dh [N, D] = d raw W;
 *                  dw [K, D] = d raw^T h, db [K] = sum d raw (db may be NULL), through
 *                  gine_head_bwd_slab_floats() floats of per-workgroup partials, reduced
 *                  in fixed order (deterministic).
 * D multiple of 4, D <= 256.
 * ---------------------------------------------------------------------------------- */
int gine_head_fwd(const float* h, const float* w, const float* b, float* raw, float* pred,
                  int64_t num_nodes, int32_t channels, int32_t kind, void* stream);
/* gine_head_fwd that also counts the batch's non-NaN targets y [N] into count_parts
 * (GINE_COUNT_PARTS uint32, as gine_count_valid) for the loss pass that follows. */
int gine_head_fwd_count(const float* h, const float* w, const float* b, float* raw,
                        float* pred, int64_t num_nodes, int32_t channels, int32_t kind,
                        const float* y, uint32_t* count_parts, void* stream);
int gine_head_bwd_slab_floats(int64_t num_nodes, int32_t channels, int32_t kind,
                              size_t* floats);
int gine_head_bwd(const float* grad_pred, const float* raw, const float* h, const float* w,
                  float* dh, float* slab, float* dw, float* db, int64_t num_nodes,
                  int32_t channels, int32_t kind, void* stream);
/* dw = NULL in gine_head_bwd leaves the partial slab; this reduces it (another stream). */
int gine_head_bwd_reduce(const float* slab, float* dw, float* db, int64_t num_nodes,
                         int32_t channels, int32_t kind, void* stream);

/* ------------------------------------------------------------------------------------
 * Dense layers between the DeepSet member sum and the GINE stack (models/gnn.py:48-68,
 * 112-113, 132-135), phi's last Linear applied after the member sum:
 *   s = r Wp2^T + bias_scale * bp2;  u = relu(s Wr0^T + br0);  e = u Wr1^T + br1;
 *   h0 = [x | e] Wdr^T + bdr
 * r [N, D] = gine_deepset_fwd output, x [N, F] node features, D in {64, 128}, F <= 64.
 * gine_chain_fwd writes s, u, e (saved for the backward) and h0.
 * gine_chain_bwd, from dh0 = d loss / d h0: de = dh0 Wdr[:, F:], dt = (de Wr1) * 1[u > 0],
 *   ds = dt Wr0, dr = ds Wp2 (dr feeds gine_deepset_bwd), and all eight parameter
 *   gradients (dbp2 scaled by bias_scale; bias pointers may be NULL) through
 *   gine_chain_bwd_slab_floats() floats of partials reduced in fixed order.
 * ---------------------------------------------------------------------------------- */
int gine_chain_fwd(const float* r, const float* x, const float* wp2, const float* bp2,
                   float bias_scale, const float* wr0, const float* br0, const float* wr1,
                   const float* br1, const float* wdr, const float* bdr, float* s, float* u,
                   float* e, float* h0, int64_t num_nodes, int32_t hidden,
                   int32_t in_features, void* stream);
int gine_chain_bwd_slab_floats(int64_t num_nodes, int32_t hidden, int32_t in_features,
                               size_t* floats);
int gine_chain_bwd(const float* dh0, const float* x, const float* r, const float* s,
                   const float* u, const float* e, const float* wp2, const float* wr0,
                   const float* wr1, const float* wdr, float* de, float* dt, float* ds,
                   float* dr, float* slab, float* dwp2, float* dbp2, float bias_scale,
                   float* dwr0, float* dbr0, float* dwr1, float* dbr1, float* dwdr,
                   float* dbdr, int64_t num_nodes, int32_t hidden, int32_t in_features,
                   void* stream);
/* The parameter-gradient half of gine_chain_bwd on its own (call gine_chain_bwd with
 * slab = NULL for the input-gradient half): lets it run on another stream, beside the
 * DeepSet backward that consumes dr. */
int gine_chain_wgrad(const float* dh0, const float* x, const float* r, const float* s,
                     const float* u, const float* e, const float* de, const float* dt,
                     const float* ds, float* slab, float* dwp2, float* dbp2, float bias_scale,
                     float* dwr0, float* dbr0, float* dwr1, float* dbr1, float* dwdr,
                     float* dbdr, int64_t num_nodes, int32_t hidden, int32_t in_features,
                     void* stream);

/* Folded chain (the default path of raincast_gnn.chain): rho[2] and dim_red have no
 * nonlinearity between them, so h0 = [x | u] W'^T + b' with W' = [Wdr_x | Wdr_e Wr1],
 * b' = Wdr_e br1 + bdr, and e / de are never formed.
 * gine_chain_fwd_folded writes s, u, h0 and W' [D][F+D] | b' [D] | W'^T [F+D][D] into
 *   wfold [2*D*(F+D) + D] (saved for the backward; folded from the current weights by every
 *   call).
 * gine_chain_bwd_folded: dt = (dh0 Wc) * 1[u > 0] (Wc = W'[:, F:]), ds = dt Wr0, dr = ds Wp2.
 * gine_chain_wgrad_folded: one engine launch for G = dh0^T [x | u] | g = sum_n dh0 (into
 *   gfold [D*(F+D) + D]), dWr0 | dbr0 and dWp2 | dbp2 (dbp2 scaled by bias_scale); slab of
 *   gine_chain_bwd_slab_floats() floats.  gfold = dwr0 = dwp2 = NULL leaves the slab for
 *   gine_grad_finalize_batch (job from gine_chain_wgrad_folded_grad_job).
 * gine_chain_unfold_grads, after the reduction: dWdr = [G_x | G_u Wr1^T + g br1^T],
 *   dbdr = g, dWr1 = Wdr_e^T G_u, dbr1 = Wdr_e^T g (fp32 MFMA; bias outputs may be NULL).
 * Replaces the same reference modules as gine_chain_fwd / gine_chain_bwd. */
int gine_chain_fwd_folded(const float* r, const float* x, const float* wp2, const float* bp2,
                          float bias_scale, const float* wr0, const float* br0,
                          const float* wr1, const float* br1, const float* wdr,
                          const float* bdr, float* wfold, float* s, float* u, float* h0,
                          int64_t num_nodes, int32_t hidden, int32_t in_features, void* stream);
/* The folded forward in ONE launch (s -> u -> h0), W' | b' | W'^T already in wfold (folded
 * by gine_deepset_fwd_fold in the launch before). */
int gine_chain_fwd_folded3(const float* r, const float* x, const float* wp2, const float* bp2,
                           float bias_scale, const float* wr0, const float* br0,
                           const float* wfold, float* s, float* u, float* h0, int64_t num_nodes,
                           int32_t hidden, int32_t in_features, void* stream);
int gine_chain_bwd_folded(const float* dh0, const float* u, const float* wp2, const float* wr0,
                          const float* wfold, float* dt, float* ds, float* dr,
                          int64_t num_nodes, int32_t hidden, int32_t in_features, void* stream);
int gine_chain_wgrad_folded(const float* dh0, const float* x, const float* r, const float* s,
                            const float* u, const float* dt, const float* ds, float* slab,
                            float* gfold, float* dwr0, float* dbr0, float* dwp2, float* dbp2,
                            float bias_scale, int64_t num_nodes, int32_t hidden,
                            int32_t in_features, void* stream);
int gine_chain_wgrad_folded_grad_job(int64_t num_nodes, int32_t hidden, int32_t in_features,
                                     const float* slab, float bias_scale, float* gfold,
                                     float* dwr0, float* dbr0, float* dwp2, float* dbp2,
                                     gine_grad_job* job);
int gine_chain_unfold_grads(const float* gfold, const float* wr1, const float* br1,
                            const float* wdr, float* dwdr, float* dbdr, float* dwr1,
                            float* dbr1, int32_t hidden, int32_t in_features, void* stream);

/* Doubly folded chain (raincast_gnn.chain.FOLD2): phi[2] is followed by rho[0] with only the
 * member sum between them, so pre = s Wr0^T + br0 = r Wf^T + bf with Wf = Wr0 Wp2,
 * bf = M Wr0 bp2 + br0 (wfold2, from gine_deepset_fwd_fold2); s / ds are never formed.
 * gine_chain_fwd_folded2: u = relu(r Wf^T + bf), h0 = [x | u] W'^T + b' (one launch).
 * gine_chain_bwd_folded2: dt = (dh0 Wc) * 1[u > 0], dr = dt Wf (one launch).
 * gine_chain_wgrad_folded2: one engine launch for G = dh0^T [x | u] | g (gfold
 *   [D*(F+D) + D]) and G2 = dt^T r | g2 = sum_n dt (g2fold [D*D + D]); gfold = g2fold = NULL
 *   leaves the slab for gine_grad_finalize_batch (job: gine_chain_wgrad_folded2_grad_job).
 * gine_chain_unfold_grads2, after the reduction, one launch: gine_chain_unfold_grads's
 *   outputs plus dWr0 = G2 Wp2^T + M g2 bp2^T, dbr0 = g2, dWp2 = Wr0^T G2,
 *   dbp2 = M Wr0^T g2 (M = members; bias outputs may be NULL). */
int gine_chain_fwd_folded2(const float* r, const float* x, const float* wfold,
                           const float* wfold2, float* u, float* h0, int64_t num_nodes,
                           int32_t hidden, int32_t in_features, void* stream);
int gine_chain_bwd_folded2(const float* dh0, const float* u, const float* wfold,
                           const float* wfold2, float* dt, float* dr, int64_t num_nodes,
                           int32_t hidden, int32_t in_features, void* stream);
int gine_chain_wgrad_folded2(const float* dh0, const float* x, const float* r, const float* u,
                             const float* dt, float* slab, float* gfold, float* g2fold,
                             int64_t num_nodes, int32_t hidden, int32_t in_features,
                             void* stream);
int gine_chain_wgrad_folded2_grad_job(int64_t num_nodes, int32_t hidden, int32_t in_features,
                                      const float* slab, float* gfold, float* g2fold,
                                      gine_grad_job* job);
int gine_chain_unfold_grads2(const float* gfold, const float* wr1, const float* br1,
                             const float* wdr, float* dwdr, float* dbdr, float* dwr1,
                             float* dbr1, const float* g2fold, const float* wp2,
                             const float* bp2, const float* wr0, float* dwr0, float* dbr0,
                             float* dwp2, float* dbp2, float members, int32_t hidden,
                             int32_t in_features, void* stream);

/* Measurement utility (not on the hot path): copy `bytes` (a multiple of 16) from src to dst
 * with 16-byte-per-lane streaming loads and stores -- the HBM copy ceiling bench.py prices
 * the message-passing kernels against (csrc/gine_probe.hip). */
int gine_copy_f4(const void* src, void* dst, int64_t bytes, void* stream);
/* Measurement utility (tools/chain_micro.py): `reps` 32x32 blocks of the split-bf16 row-GEMM
 * chain (K = 128) per wave in `blocks` 256-thread workgroups, in form `variant` (0: A split
 * in the loop, 1: pre-split A planes from LDS, 2: MFMAs only, 3: two chains interleaved);
 * ticks[block * 4 + wave] = shader-clock ticks of the loop, sink = [blocks * 256] sums. */
int gine_probe_chain(int32_t variant, int32_t reps, int32_t blocks, float* sink,
                     long long* ticks, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GINE_HIP_H_ */
