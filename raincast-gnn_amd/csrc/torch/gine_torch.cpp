// PyTorch binding of the GINE layer for the drop-in path (raincast_gnn.nn.GINEConv called
// from the reference's own models/gnn.py structure and train.py loop, without HIP graphs).
//
// The same launches as raincast_gnn/functional.py's GineLayer (forward: the one-launch layer,
// the fused gather + Linear1 or the unfused pair, BatchNorm sums through the fixed-point
// accumulator or fp64 partials; backward, the non-deferred form: where a 32-channel window
// plan exists, dbn GEMM + BatchNorm sums and BatchNorm finish + dz GEMM (accumulator pair),
// the window message passing with the node-MLP weight-gradient engine in one launch, and
// one batch launch for the engine's slab and the message passing's partials; otherwise dbn
// GEMM, BatchNorm backward finish, dz GEMM beside the engine, message-passing backward
// reducing that slab in the same launch, then its own finish), issued from a C++
// torch::autograd::Function: one Python call per layer forward and none in backward, where
// the Python Function spends ~50 us and ~190 us of host time per layer on argument
// marshalling, allocations and per-launch ctypes calls (profiles/r04_s02_dropin_prof.txt).
// The kernels and their order are unchanged, so the results are the same bits as the
// Python path's (tests/test_gpu_dropin.py).  Everything goes through the C ABI of
// include/gine_hip.h; this file owns no kernels.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <vector>

#include "gine_hip.h"

namespace {

using torch::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::tensor_list;

void* P(const Tensor& t) { return t.defined() ? t.data_ptr() : nullptr; }

void ok(int st, const char* what) {
  TORCH_CHECK(st == GINE_OK, what, " failed with status ", st, ": ", gine_status_string(st));
}

void* stream_of(const Tensor& t) {
  return reinterpret_cast<void*>(at::hip::getCurrentHIPStream(t.device().index()).stream());
}

int32_t query(int (*fn)(int64_t, int32_t, int32_t*), int64_t n, int32_t d, const char* what) {
  int32_t v = 0;
  ok(fn(n, d, &v), what);
  return v;
}

// Indices into the integer / float option vectors the Python side passes.
enum IntOpt {
  kEpi = 0,        // GINE_EPI_*
  kLinFlag,        // 0 | GINE_MP_LIN_MULADD (the host CPU's Linear(1,D) rounding)
  kBatchStats,     // BatchNorm uses batch statistics
  kUpdateRunning,  // ... and updates the running buffers
  kFused,          // gine_mp_fwd_mlp1 applies
  kLayer,          // gine_mp_fwd_layer applies
  kMaxInDegree,
  kEngine,         // gine_mp_bwd_win_mlp_wgrad applies (functional.engine_in_mp_ok)
  kLayerBwd,       // gine_mlp_bwd_layer applies (functional.layer_backward_ok)
  // the window plans' scalars, kPlanFields each: num_tiles (0: no plan), slice_channels,
  // max_rows, max_edges, max_nodes -- the plan's device arrays come in the graph list, so the
  // autograd node holds them (a plan's addresses alone would dangle once the graph cache
  // evicts the graph between forward and backward)
  kPlanIn,
  kPlanOut = kPlanIn + 5,
  // the layer window plan (gine_graph_plan_layer_windows): its largest window; its tile
  // array is the graph list's last entry (undefined: the L2 gather)
  kLayerWinRows = kPlanOut + 5,
  kIntOpts
};
constexpr int kPlanFields = 5;
// graph list: the two CSRs, then per plan (in, out) its device arrays
enum GraphArg { kInRowptr = 0, kInSrc, kInAttr, kOutRowptr, kOutDst, kOutAttr, kGraphCsr };
enum PlanArray { kTileBegin = 0, kWinLo, kWinRows, kSlot, kEdgeBegin, kPlanArrays };
constexpr int kLayerWinTiles = kGraphCsr + 2 * kPlanArrays;
constexpr int kGraphArgs = kLayerWinTiles + 1;

// The window plan of side `which` (0: in, 1: out) rebuilt from its scalars and its arrays
// (a struct on the caller's stack: the library reads it only during the call).
bool plan_of(const std::vector<int64_t>& io, const Tensor* arrays, int which,
             gine_window_plan* out) {
  const int64_t* f = io.data() + (which == 0 ? kPlanIn : kPlanOut);
  if (f[0] <= 0) return false;
  auto p32 = [&](int k) { return static_cast<const int32_t*>(arrays[k].defined() ? arrays[k].data_ptr() : nullptr); };
  out->tile_begin = p32(kTileBegin);
  out->win_lo = p32(kWinLo);
  out->win_rows = p32(kWinRows);
  out->num_tiles = (int32_t)f[0];
  out->slice_channels = (int32_t)f[1];
  out->max_rows = (int32_t)f[2];
  out->max_edges = (int32_t)f[3];
  out->max_nodes = (int32_t)f[4];
  out->slot = static_cast<const int16_t*>(arrays[kSlot].defined() ? arrays[kSlot].data_ptr() : nullptr);
  out->edge_begin = p32(kEdgeBegin);
  return true;
}
enum FloatOpt { kMomentum = 0, kBnEps, kFloatOpts };

// Several tensors from ONE allocation (each 256-byte aligned): the caching allocator's
// per-call cost dominates the drop-in path's host time, and these are internal buffers or
// gradients handed to autograd (a view with the parameter's shape and strides is adopted as
// .grad without a copy).  An empty shape list entry gives an undefined tensor.
struct Spec {
  std::vector<int64_t> shape;
  c10::ScalarType dtype;
  bool want;
};
std::vector<Tensor> carve(const Tensor& like, const std::vector<Spec>& specs) {
  std::vector<int64_t> off(specs.size(), 0), bytes(specs.size(), 0);
  int64_t total = 0;
  for (size_t i = 0; i < specs.size(); ++i) {
    if (!specs[i].want) continue;
    int64_t n = (int64_t)c10::elementSize(specs[i].dtype);
    for (int64_t d : specs[i].shape) n *= d;
    bytes[i] = n;
    off[i] = total;
    total += (n + 255) / 256 * 256;
  }
  Tensor buf = torch::empty({std::max<int64_t>(total, 256)}, like.options().dtype(torch::kUInt8));
  std::vector<Tensor> out(specs.size());
  for (size_t i = 0; i < specs.size(); ++i)
    if (specs[i].want)
      out[i] = buf.narrow(0, off[i], bytes[i]).view(specs[i].dtype).view(specs[i].shape);
  return out;
}

struct ZeroOnError {  // csrc/gine_bnacc.hpp pairing: re-zero the accumulator if a launch fails
  Tensor acc;
  bool armed = true;
  ~ZeroOnError() {
    if (armed && acc.defined()) acc.zero_();
  }
};

class GineLayerFn : public torch::autograd::Function<GineLayerFn> {
 public:
  // graph: in_rowptr, in_src, in_attr, out_rowptr, out_dst, out_attr, the two plans' arrays
  // bn: running_mean, running_var, num_batches_tracked, accumulator, backward accumulator
  // (undefined: partials)
  static Tensor forward(AutogradContext* ctx, Tensor x, Tensor lin_w, Tensor lin_b, Tensor eps,
                        Tensor w1, Tensor b1, Tensor gamma, Tensor beta, Tensor w2, Tensor b2,
                        std::vector<Tensor> graph, std::vector<Tensor> bn,
                        std::vector<int64_t> io, std::vector<double> fo) {
    x = x.contiguous();
    const int64_t N = x.size(0);
    const int32_t D = (int32_t)x.size(1);
    void* s = stream_of(x);
    Tensor lw = lin_w.reshape({-1}).contiguous(), lb = lin_b.reshape({-1}).contiguous();
    Tensor ep = eps.contiguous();
    Tensor w1c = w1.contiguous(), b1c = b1.contiguous(), w2c = w2.contiguous(),
           b2c = b2.contiguous();
    Tensor g = gamma.defined() ? gamma.contiguous() : gamma;
    Tensor bt = beta.defined() ? beta.contiguous() : beta;
    const int epi = (int)io[kEpi], lin_flag = (int)io[kLinFlag];
    const bool batch_stats = io[kBatchStats] != 0;
    const int update_running = (int)io[kUpdateRunning];
    const bool fused = io[kFused] != 0, layer = io[kLayer] != 0;
    const int32_t max_deg = (int32_t)io[kMaxInDegree];
    gine_window_plan plan_in_v{};
    const gine_window_plan* plan_in =
        plan_of(io, graph.data() + kGraphCsr, 0, &plan_in_v) ? &plan_in_v : nullptr;
    const Tensor &in_rowptr = graph[kInRowptr], &in_src = graph[kInSrc], &in_attr = graph[kInAttr];
    const Tensor &rmean = bn[0], &rvar = bn[1], &nbt = bn[2], &acc = bn[3];
    TORCH_CHECK_VALUE(!(batch_stats && N <= 1), "Expected more than 1 value per channel when "
                "training, got input size [", N, ", ", D, "]");
    const float momentum = (float)fo[kMomentum], bn_eps = (float)fo[kBnEps];

    Tensor y = torch::empty_like(x);  // the user's tensor: its own storage
    int32_t Pn = 0;
    if (!acc.defined()) Pn = query(gine_mlp_num_partials, N, D, "gine_mlp_num_partials");
    // saved for the backward / scratch: one allocation
    std::vector<Tensor> t = carve(x, {{{N, D}, torch::kFloat32, true},
                                      {{N, D}, torch::kFloat32, true},
                                      {{4, D}, torch::kFloat32, true},
                                      {{N, D}, torch::kUInt8, epi == GINE_EPI_RESIDUAL_RELU},
                                      {{Pn, 2, D}, torch::kFloat64, !acc.defined()}});
    Tensor a1 = t[0], z = t[1], bn_save = t[2], mask = t[3], partials = t[4];
    void* nbt_p = update_running ? P(nbt) : nullptr;
    const int upd = (update_running && rmean.defined()) ? 1 : 0;
    if (!fused) {  // the gather (or window) forward, unpaired
      if (plan_in)
        ok(gine_mp_fwd_win((const float*)P(x), (const int32_t*)P(in_rowptr),
                           (const int32_t*)P(in_src), (const float*)P(in_attr),
                           (const float*)P(lw), (const float*)P(lb), (const float*)P(ep),
                           (float*)P(z), N, D, lin_flag, plan_in, s),
           "gine_mp_fwd_win");
      else
        ok(gine_mp_fwd((const float*)P(x), (const int32_t*)P(in_rowptr),
                       (const int32_t*)P(in_src), (const float*)P(in_attr),
                       (const float*)P(lw), (const float*)P(lb), (const float*)P(ep),
                       (float*)P(z), N, D, lin_flag, s),
           "gine_mp_fwd");
    }
    {
      ZeroOnError guard{acc};
      if (layer) {
        ok(gine_mp_fwd_layer((const float*)P(x), (const int32_t*)P(in_rowptr),
                             (const int32_t*)P(in_src), (const float*)P(in_attr),
                             (const float*)P(lw), (const float*)P(lb), (const float*)P(ep),
                             (const float*)P(w1c), (const float*)P(b1c), (float*)P(z),
                             (float*)P(a1), (int64_t*)P(acc), (const float*)P(g),
                             (const float*)P(bt), (float*)P(rmean), (float*)P(rvar),
                             (int64_t*)nbt_p, (float*)P(bn_save), momentum, bn_eps, upd,
                             (const float*)P(w2c), (const float*)P(b2c), (float*)P(y),
                             (uint8_t*)P(mask), N, D, max_deg, lin_flag, epi,
                             graph[kLayerWinTiles].defined()
                                 ? (const int32_t*)graph[kLayerWinTiles].data_ptr()
                                 : nullptr,
                             (int32_t)io[kLayerWinRows], /*head=*/nullptr, s),
           "gine_mp_fwd_layer");
      } else {
        if (fused) {
          if (acc.defined())
            ok(gine_mp_fwd_mlp1_acc((const float*)P(x), (const int32_t*)P(in_rowptr),
                                    (const int32_t*)P(in_src), (const float*)P(in_attr),
                                    (const float*)P(lw), (const float*)P(lb),
                                    (const float*)P(ep), (const float*)P(w1c),
                                    (const float*)P(b1c), (float*)P(z), (float*)P(a1),
                                    (double*)P(partials), (int64_t*)P(acc), N, D, max_deg,
                                    lin_flag, s),
               "gine_mp_fwd_mlp1_acc");
          else
            ok(gine_mp_fwd_mlp1((const float*)P(x), (const int32_t*)P(in_rowptr),
                                (const int32_t*)P(in_src), (const float*)P(in_attr),
                                (const float*)P(lw), (const float*)P(lb), (const float*)P(ep),
                                (const float*)P(w1c), (const float*)P(b1c), (float*)P(z),
                                (float*)P(a1), (double*)P(partials), N, D, max_deg, lin_flag,
                                s),
               "gine_mp_fwd_mlp1");
        } else if (acc.defined()) {
          ok(gine_mlp_fwd1_acc((const float*)P(z), (const float*)P(w1c), (const float*)P(b1c),
                               (float*)P(a1), nullptr, (int64_t*)P(acc), N, D, s),
             "gine_mlp_fwd1_acc");
        } else {
          ok(gine_mlp_fwd1((const float*)P(z), (const float*)P(w1c), (const float*)P(b1c),
                           (float*)P(a1), (double*)P(partials), N, D, s),
             "gine_mlp_fwd1");
        }
        if (acc.defined()) {
          ok(gine_mlp_fwd2_bn((const float*)P(a1), (int64_t*)P(acc), (const float*)P(g),
                              (const float*)P(bt), (float*)P(rmean), (float*)P(rvar),
                              (int64_t*)nbt_p, (float*)P(bn_save), momentum, bn_eps, upd,
                              (const float*)P(w2c), (const float*)P(b2c), (const float*)P(x),
                              (float*)P(y), (uint8_t*)P(mask), N, D, epi, s),
             "gine_mlp_fwd2_bn");
        } else {
          ok(gine_bn_fwd_finalize((const double*)P(partials), Pn, (const float*)P(g),
                                  (const float*)P(bt), (float*)P(rmean), (float*)P(rvar),
                                  (int64_t*)nbt_p, (float*)P(bn_save), N, D, momentum, bn_eps,
                                  batch_stats ? 1 : 0, upd, s),
             "gine_bn_fwd_finalize");
          ok(gine_mlp_fwd2((const float*)P(a1), (const float*)P(bn_save),
                           (const float*)P(w2c), (const float*)P(b2c), (const float*)P(x),
                           (float*)P(y), (uint8_t*)P(mask), N, D, epi, s),
             "gine_mlp_fwd2");
        }
      }
      guard.armed = false;
    }
    const Tensor* po = graph.data() + kGraphCsr + kPlanArrays;  // the backward's plan arrays
    ctx->save_for_backward({x, z, a1, epi == GINE_EPI_RELU ? y : Tensor(), mask, bn_save, lw,
                            lb, ep, w1c, w2c, g, graph[kOutRowptr], graph[kOutDst],
                            graph[kOutAttr], po[0], po[1], po[2], po[3], po[4], bn[4]});
    ctx->saved_data["io"] = io;
    ctx->saved_data["beta"] = beta.defined();
    ctx->saved_data["lin_w_shape"] = lin_w.sizes().vec();
    return y;
  }

  static tensor_list backward(AutogradContext* ctx, tensor_list grads) {
    auto sv = ctx->get_saved_variables();
    Tensor x = sv[0], z = sv[1], a1 = sv[2], y = sv[3], mask = sv[4], bn_save = sv[5],
           lw = sv[6], lb = sv[7], ep = sv[8], w1c = sv[9], w2c = sv[10], g = sv[11];
    const Tensor &out_rowptr = sv[12], &out_dst = sv[13], &out_attr = sv[14];
    const std::vector<int64_t> io = ctx->saved_data["io"].toIntVector();
    const bool has_beta = ctx->saved_data["beta"].toBool();
    const std::vector<int64_t> lin_w_shape = ctx->saved_data["lin_w_shape"].toIntVector();
    Tensor dy = grads[0].contiguous();
    const int64_t N = x.size(0);
    const int32_t D = (int32_t)x.size(1);
    void* s = stream_of(x);
    const int epi = (int)io[kEpi], lin_flag = (int)io[kLinFlag];
    gine_window_plan plan_out_v{};
    const gine_window_plan* plan_out =
        plan_of(io, sv.data() + 15, 1, &plan_out_v) ? &plan_out_v : nullptr;
    auto fo = x.options();
    const int32_t C = query(gine_mlp_wgrad_num_chunks, N, D, "gine_mlp_wgrad_num_chunks");
    const int32_t Pn = query(gine_mlp_num_partials, N, D, "gine_mlp_num_partials");
    const int32_t P2 = plan_out ? plan_out->num_tiles
                                : query(gine_mp_bwd_num_partials, N, D, "gine_mp_bwd_num_partials");
    // the parameter gradients from one allocation, the scratch from another
    std::vector<Tensor> gr = carve(x, {{{D}, torch::kFloat32, g.defined()},
                                       {{D}, torch::kFloat32, has_beta},
                                       {{D, D}, torch::kFloat32, true},
                                       {{D}, torch::kFloat32, true},
                                       {{D, D}, torch::kFloat32, true},
                                       {{D}, torch::kFloat32, true},
                                       {{D}, torch::kFloat32, true},
                                       {{D}, torch::kFloat32, true},
                                       {{1}, torch::kFloat32, true}});
    Tensor dgamma = gr[0], dbeta = gr[1], dw1 = gr[2], db1 = gr[3], dw2 = gr[4], db2 = gr[5];
    Tensor dlw = gr[6], dlb = gr[7], deps = gr[8];
    std::vector<Tensor> sc = carve(x, {{{N, D}, torch::kFloat32, true},
                                       {{3, D}, torch::kFloat32, true},
                                       {{N, D}, torch::kFloat32, true},
                                       {{2 * (int64_t)C * ((int64_t)D * D + D)}, torch::kFloat32, true},
                                       {{Pn, 2, D}, torch::kFloat64, true},
                                       {{P2, 3, D}, torch::kFloat64, true}});
    Tensor dbn = sc[0], coef = sc[1], dz = sc[2], slab = sc[3], partials = sc[4], part2 = sc[5];
    Tensor dres = epi == GINE_EPI_RESIDUAL_RELU ? dy : Tensor();
    Tensor dx = torch::empty_like(x);
    const int32_t flags = GINE_MP_BWD_SELF | lin_flag;
    if (plan_out && io[kEngine]) {
      const Tensor& bacc = sv[20];  // the BatchNorm-backward accumulator (undefined: partials)
      if (bacc.defined()) {
        ZeroOnError guard{bacc};
        if (io[kLayerBwd]) {  // the pair in one launch (grid barrier)
          ok(gine_mlp_bwd_layer((const float*)P(dy), (const float*)P(y),
                                (const uint8_t*)P(mask), (const float*)P(a1),
                                (const float*)P(bn_save), (const float*)P(w2c), (float*)P(dbn),
                                (int64_t*)P(bacc), (const float*)P(g), (float*)P(dgamma),
                                (float*)P(dbeta), (float*)P(coef), (const float*)P(w1c),
                                (float*)P(dz), N, D, epi, s),
             "gine_mlp_bwd_layer");
        } else {
          ok(gine_mlp_bwd2_acc((const float*)P(dy), (const float*)P(y), (const uint8_t*)P(mask),
                               (const float*)P(a1), (const float*)P(bn_save),
                               (const float*)P(w2c), (float*)P(dbn), nullptr, (int64_t*)P(bacc),
                               N, D, epi, s),
             "gine_mlp_bwd2_acc");
          ok(gine_mlp_bwd1_bn((const float*)P(dbn), (const float*)P(a1),
                              (const float*)P(bn_save), (int64_t*)P(bacc), (const float*)P(g),
                              (float*)P(dgamma), (float*)P(dbeta), (float*)P(coef),
                              (const float*)P(w1c), (float*)P(dz), N, D, s),
             "gine_mlp_bwd1_bn");
        }
        guard.armed = false;
      } else {
        ok(gine_mlp_bwd2((const float*)P(dy), (const float*)P(y), (const uint8_t*)P(mask),
                         (const float*)P(a1), (const float*)P(bn_save), (const float*)P(w2c),
                         (float*)P(dbn), (double*)P(partials), N, D, epi, s),
           "gine_mlp_bwd2");
        ok(gine_bn_bwd_finalize((const double*)P(partials), Pn, (const float*)P(g),
                                (const float*)P(bn_save), (float*)P(dgamma), (float*)P(dbeta),
                                (float*)P(coef), N, D, io[kBatchStats] ? 1 : 0, s),
           "gine_bn_bwd_finalize");
        ok(gine_mlp_bwd1((const float*)P(dbn), (const float*)P(a1), (const float*)P(bn_save),
                         (const float*)P(coef), (const float*)P(w1c), (float*)P(dz), N, D, s),
           "gine_mlp_bwd1");
      }
      // message passing + the dW1 / dW2 engine in one launch, then both reductions in one
      ok(gine_mp_bwd_win_mlp_wgrad((const float*)P(dz), (const float*)P(x),
                                   (const int32_t*)P(out_rowptr), (const int32_t*)P(out_dst),
                                   (const float*)P(out_attr), (const float*)P(lw),
                                   (const float*)P(lb), (const float*)P(ep), (const float*)P(dres),
                                   (float*)P(dx), (double*)P(part2), N, D, flags, plan_out,
                                   (const float*)P(dy), (const float*)P(y),
                                   (const uint8_t*)P(mask), (const float*)P(a1),
                                   (const float*)P(bn_save), (const float*)P(dbn),
                                   (const float*)P(coef), (const float*)P(z), (float*)P(slab), epi,
                                   s),
         "gine_mp_bwd_win_mlp_wgrad");
      gine_grad_job jobs[2] = {};
      const int64_t per = (int64_t)D * D + D;
      jobs[0].kind = GINE_GRAD_JOB_SLAB;  // [dW2 | db2], [dW1 | db1] (MlpWgradOut order)
      jobs[0].src = P(slab);
      jobs[0].rows = C;
      jobs[0].nz = 2;
      jobs[0].cstride = per;
      jobs[0].zstride = per * C;
      float* wz[2][2] = {{(float*)P(dw2), (float*)P(db2)}, {(float*)P(dw1), (float*)P(db1)}};
      for (int zi = 0; zi < 2; ++zi) {
        jobs[0].per[zi] = per;
        jobs[0].wsize[zi] = (int64_t)D * D;
        jobs[0].bscale[zi] = 1.f;
        jobs[0].w[zi] = wz[zi][0];
        jobs[0].b[zi] = wz[zi][1];
      }
      jobs[1].kind = GINE_GRAD_JOB_MP;   // dW_e, db_e, eps from the window partials
      jobs[1].src = P(part2);
      jobs[1].rows = P2;
      jobs[1].channels = D;
      jobs[1].eps_cols = D / plan_out->slice_channels;
      jobs[1].w[0] = (float*)P(dlw);
      jobs[1].w[1] = (float*)P(dlb);
      jobs[1].w[2] = (float*)P(deps);
      ok(gine_grad_finalize_batch(jobs, 2, s), "gine_grad_finalize_batch");
      return {dx,    dlw.view(lin_w_shape), dlb, deps.view_as(ep), dw1,      db1,     dgamma,
              dbeta, dw2,                   db2, Tensor(),          Tensor(), Tensor(), Tensor()};
    }
    ok(gine_mlp_bwd2((const float*)P(dy), (const float*)P(y), (const uint8_t*)P(mask),
                     (const float*)P(a1), (const float*)P(bn_save), (const float*)P(w2c),
                     (float*)P(dbn), (double*)P(partials), N, D, epi, s),
       "gine_mlp_bwd2");
    ok(gine_bn_bwd_finalize((const double*)P(partials), Pn, (const float*)P(g),
                            (const float*)P(bn_save), (float*)P(dgamma), (float*)P(dbeta),
                            (float*)P(coef), N, D, io[kBatchStats] ? 1 : 0, s),
       "gine_bn_bwd_finalize");
    // dz = da1 W1 and the dW1 / dW2 partial slab side by side in one launch
    ok(gine_mlp_bwd1_wgrad((const float*)P(dy), (const float*)P(y), (const uint8_t*)P(mask),
                           (const float*)P(a1), (const float*)P(bn_save), (const float*)P(dbn),
                           (const float*)P(coef), (const float*)P(z), (const float*)P(w1c),
                           (float*)P(dz), (float*)P(slab), nullptr, nullptr, nullptr, nullptr,
                           N, D, epi, s),
       "gine_mlp_bwd1_wgrad");
    // message-passing backward; its extra workgroups reduce the slab
    if (plan_out) {
      ok(gine_mp_bwd_win_side((const float*)P(dz), (const float*)P(x),
                              (const int32_t*)P(out_rowptr), (const int32_t*)P(out_dst),
                              (const float*)P(out_attr), (const float*)P(lw),
                              (const float*)P(lb), (const float*)P(ep), (const float*)P(dres),
                              (float*)P(dx), (double*)P(part2), N, D, flags, plan_out,
                              (const float*)P(slab), C, D, (float*)P(dw1), (float*)P(db1),
                              (float*)P(dw2), (float*)P(db2), s),
         "gine_mp_bwd_win_side");
      ok(gine_mp_bwd_win_finalize((const double*)P(part2), P2, D, plan_out->slice_channels,
                                  (float*)P(dlw), (float*)P(dlb), (float*)P(deps), s),
         "gine_mp_bwd_win_finalize");
    } else {
      ok(gine_mp_bwd_side((const float*)P(dz), (const float*)P(x), (const int32_t*)P(out_rowptr),
                          (const int32_t*)P(out_dst), (const float*)P(out_attr),
                          (const float*)P(lw), (const float*)P(lb), (const float*)P(ep),
                          (const float*)P(dres), (float*)P(dx), (double*)P(part2), N, D, flags,
                          (const float*)P(slab), C, D, (float*)P(dw1), (float*)P(db1),
                          (float*)P(dw2), (float*)P(db2), s),
         "gine_mp_bwd_side");
      ok(gine_mp_bwd_finalize((const double*)P(part2), P2, D, (float*)P(dlw), (float*)P(dlb),
                              (float*)P(deps), s),
         "gine_mp_bwd_finalize");
    }
    // x, lin_w, lin_b, eps, w1, b1, gamma, beta, w2, b2, graph, bn, io, fo
    return {dx,     dlw.view(lin_w_shape), dlb,  deps.view_as(ep), dw1,      db1,     dgamma,
            dbeta,  dw2,                   db2,  Tensor(),          Tensor(), Tensor(), Tensor()};
  }
};

Tensor opt(const c10::optional<Tensor>& t) { return t.has_value() ? *t : Tensor(); }

// The Python entry point: one call per layer forward.
Tensor gine_layer(Tensor x, Tensor lin_w, Tensor lin_b, Tensor eps, Tensor w1, Tensor b1,
                  c10::optional<Tensor> gamma, c10::optional<Tensor> beta, Tensor w2, Tensor b2,
                  std::vector<c10::optional<Tensor>> graph_opt,
                  std::vector<c10::optional<Tensor>> bn, std::vector<int64_t> io,
                  std::vector<double> fo) {
  std::vector<Tensor> graph;
  for (const auto& t : graph_opt) graph.push_back(opt(t));
  TORCH_CHECK(graph.size() == kGraphArgs, "graph: in_rowptr, in_src, in_attr, out_rowptr, "
              "out_dst, out_attr, then the in and out window plans' tile_begin, win_lo, "
              "win_rows, slot, edge_begin, then the layer window plan's tiles");
  TORCH_CHECK(bn.size() == 5, "bn: running_mean, running_var, num_batches_tracked, acc, "
              "backward acc");
  TORCH_CHECK(io.size() == kIntOpts && fo.size() == kFloatOpts, "option vectors");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kFloat32 && x.dim() == 2,
              "x: fp32 [N, D] on a HIP device");
  std::vector<Tensor> bnt;
  for (const auto& t : bn) bnt.push_back(opt(t));
  return GineLayerFn::apply(x, lin_w, lin_b, eps, w1, b1, opt(gamma), opt(beta), w2, b2,
                            graph, bnt, io, fo);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "C++ autograd binding of the GINE layer (drop-in path; include/gine_hip.h)";
  m.def("gine_layer", &gine_layer, "GINE layer forward (autograd: the non-deferred backward)");
  m.attr("ABI_VERSION") = GINE_ABI_VERSION;
}
