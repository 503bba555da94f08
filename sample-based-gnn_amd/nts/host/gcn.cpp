// Model drivers: the GPU-sampled GCN / GraphSAGE toolkits.
//   GCN_SAMPLE_ALLGPU_impl   toolkits/GCN_SAMPLE_ALLGPU.hpp  (GPU sampler, 1 GPU)
//   GS_SAMPLE_ALLGPU         toolkits/GS_SAMPLE_ALLGPU.hpp   (same pipeline, Mean weights, :296)
//   GCN_SAMPLE_ALL_MULTI     toolkits/GCN_SAMPLE_ALL_MULTI.hpp (data parallel, grad SUM all-reduce)
// One class covers the three: the weight type and the optional communicator
// select the variant.  Per batch: sample_gpu_fast -> load_label_gpu ->
// [fused feature gather +] graph op -> vertexForward ... -> Loss ->
// self_backward -> Update (all-reduce + Adam) -> zero_grad.
#include "gcn.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <cstdio>
#include <cstdlib>

namespace nts {

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

GCN_SAMPLE_ALLGPU_impl::GCN_SAMPLE_ALLGPU_impl(std::shared_ptr<FullyRepGraph> g, NtsVar feature,
                                               NtsVar label, std::vector<VertexId> train_nids,
                                               GCNConfig c, std::shared_ptr<Communicator> comm_)
    : graph(std::move(g)), F(std::move(feature)), L_GT(std::move(label)), cfg(std::move(c)),
      comm(std::move(comm_)) {
  TORCH_CHECK(cfg.layer_size.size() >= 2, "need at least one layer");
  TORCH_CHECK(cfg.fanout.size() == cfg.layer_size.size() - 1, "fanout per layer");
  TORCH_CHECK(F.is_cuda() && F.dtype() == torch::kFloat32 && F.size(1) == cfg.layer_size[0],
              "feature table must be fp32 [V, layer_size[0]] on the GPU");
  if (cfg.sample_gpu) {
    TORCH_CHECK(!cfg.gat && !cfg.pd_cache, "GCN_SAMPLE_GPU: GCN / GraphSAGE layers");
    TORCH_CHECK(cfg.rng_mode != NTS_RNG_PHILOX,
                "GCN_SAMPLE_GPU samples with the reference's mt19937 stream (rng_mode MT19937)");
    cfg.deterministic_backward = true;  // the CSR exists for every graph-op backward
  }
  // sampler_cus n > 0: the sampler's stream on n CUs, the training stream on
  // the others; n < 0: the sampler on |n| CUs, the training stream on all
  if (cfg.pipeline && cfg.sampler_cus > 0)
    cs = std::make_unique<NtsStream>(graph->device,
                                     cu_mask_spread(graph->device, cfg.sampler_cus, true),
                                     (uint64_t)cfg.seed);
  else
    cs = std::make_unique<NtsStream>(graph->device, nullptr, (uint64_t)cfg.seed,
                                     cfg.pipeline && cfg.sampler_priority < 0);
  hip_check(nts_hip_ctx_set_gemm_mode(cs->ctx(), cfg.gemm_mode), "nts_hip_ctx_set_gemm_mode");
  // inputs were produced on other streams: order them before our stream
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
  auto guard = cs->guard();
  // Wide feature rows are re-laid with a 128-byte aligned pitch (one copy,
  // +1% memory): a gathered row then spans the minimum number of cache lines
  // (19 instead of ~19.8 for 602 floats), ~2% less traffic in the bottom
  // aggregation, which reads every sampled row once per edge.
  if (cfg.pad_features && F.size(1) >= 256 && F.size(1) % 32 != 0 && F.stride(1) == 1) {
    NtsVar Fp = row_padded_empty(F.size(0), F.size(1), graph->device);
    Fp.copy_(F);
    F = Fp;
  }
  if (cfg.cache_rate >= 0.0) {
    TORCH_CHECK(cfg.cache_rate <= 1.0, "cache_rate must be in [0, 1]");
    const uint64_t V = graph->global_vertices;
    const uint64_t n_cache = std::min<uint64_t>(V, (uint64_t)(cfg.cache_rate * (double)V));
    fcache = std::make_unique<FeatureCache>(*cs, *graph, F, n_cache);
    F = torch::empty({0, F.size(1)}, f32_opts(graph->device));  // HBM table released
  }
  if (cfg.shuffle) {  // shuffle_vec (toolkits/GCN_SAMPLE_GPU.hpp:175-180): mt19937(2000)
    std::mt19937 gen(2000);
    std::shuffle(train_nids.begin(), train_nids.end(), gen);
  }
  const int L = (int)cfg.fanout.size();
  // Bottom layer order: transform first when the first layer
  // narrows the rows — the aggregation then gathers F_out-wide rows of X W
  // (a table that stays in the Infinity Cache) instead of F_in-wide feature
  // rows, at the price of a GEMM over the src rows instead of the dst rows.
  const bool tf_ok = L >= 2 && !cfg.gat && !fcache && cfg.hip_gemm && cfg.fuse_activation &&
                     !cfg.pd_cache;
  if (cfg.transform_first == 1)
    TORCH_CHECK(tf_ok, "transform_first needs >= 2 layers, the MFMA GEMMs with the fused "
                       "activation, no GAT and no feature cache");
  // auto (-1): transform first where the first layer narrows the rows at
  // least 4x and its GEMMs run on the whole-row fp32-exact kernels
  // (csrc/gemmx3.hip, split-bf16) or the f16 pair tables (C2: 602 -> 128,
  // 0.93 vs 1.04 ms/step fp32-exact); the reference's order elsewhere
  tf_ = tf_ok && (cfg.transform_first == 1 ||
                  (cfg.transform_first < 0 &&
                   (cfg.pair_table >= 3 || cfg.gemm_mode == NTS_GEMM_SPLIT3) &&
                   cfg.layer_size[0] >= 4 * cfg.layer_size[1]));
  if (tf_ && cfg.pair_table > 0) {
    // the feature table is static: its rows are split into f16 pairs once,
    // in ONE layout — planar where the planar kernels take the shape (both
    // GEMMs: every dW output row in one block, K <= 640, N % 128 == 0),
    // interleaved otherwise
    const int64_t V = F.size(0), K = F.size(1), Kp = (K + 31) / 32 * 32;
    const int64_t Nh = cfg.layer_size[1];
    pairs_ = std::make_unique<PairTable>();
    pairs_->rs = torch::empty({V}, f32_opts(graph->device));
    pairs_->tn = cfg.pair_table >= 2;
    if (cfg.pair_table >= 3 && Kp <= 640 && Nh % 128 == 0) {
      // rows padded to 2560 bytes where that leaves a tail for the row scale
      // (the four-stage forward GEMM reads it with the row); Q is the [V, 2 Kp]
      // view of the padded rows
      const int64_t ldq = 4 * Kp + 8 <= 2560 ? 1280 : 2 * Kp;
      pairs_->Q = torch::empty({V, ldq}, torch::TensorOptions().dtype(torch::kInt16).device(F.device()))
                      .narrow(1, 0, 2 * Kp);
      hip_check(nts_hip_h2_split_rows_planar(cs->ctx(), (uint64_t)V, (uint32_t)K, F.data_ptr<float>(),
                                             (uint64_t)F.stride(0), (uint32_t)Kp,
                                             reinterpret_cast<uint16_t*>(pairs_->Q.data_ptr<int16_t>()),
                                             (uint64_t)ldq, pairs_->rs.data_ptr<float>()),
                "nts_hip_h2_split_rows_planar");
    } else {
      pairs_->P = torch::empty({V, Kp}, torch::TensorOptions().dtype(torch::kInt32).device(F.device()));
      hip_check(nts_hip_h2_split_rows(cs->ctx(), (uint64_t)V, (uint32_t)K, F.data_ptr<float>(),
                                      (uint64_t)F.stride(0), (uint32_t)Kp,
                                      reinterpret_cast<uint32_t*>(pairs_->P.data_ptr<int32_t>()),
                                      (uint64_t)Kp, pairs_->rs.data_ptr<float>()),
                "nts_hip_h2_split_rows");
    }
  }
  // CSR transposes only where a graph-op backward runs (every hop but the
  // outermost, whose backward the context skips — unless the bottom layer is
  // transform-first: its aggregation then has a backward, dH = A^T dZ)
  std::vector<bool> csr(L, cfg.deterministic_backward);
  csr[L - 1] = tf_;
  if (cfg.gat) csr.assign(L, true);  // every layer's backward runs over its CSR
  // Pipelined: three sampler slots.  Batch k+1 is sampled into the slot of
  // batch k-2, whose training finished before batch k-1's began, so the
  // sampling stream never waits on an unfinished event when its kernels are
  // launched (with two slots it waits on batch k-1's training, and ROCm then
  // blocks every launch on that stream in the host for ~60 us).
  nslots_ = cfg.pipeline ? kSlots : 1;
  sampler = std::make_unique<FastSampler>(graph, train_nids, L, cfg.batch_size, cfg.fanout,
                                          nslots_, csr,
                                          !cfg.gat && cfg.weight_type != WeightType::None,
                                          cfg.gat);
  sampler->rng_mode = cfg.rng_mode;
  sampler->up_degree = cfg.up_degree;
  if (cfg.pipeline && cfg.sampler_cus != 0)
    ss = std::make_unique<NtsStream>(graph->device,
                                     cu_mask_spread(graph->device, std::abs(cfg.sampler_cus), false),
                                     (uint64_t)cfg.seed);
  else if (cfg.pipeline)
    ss = std::make_unique<NtsStream>(graph->device, nullptr, (uint64_t)cfg.seed,
                                     cfg.sampler_priority == 1 ||
                                         (cfg.sampler_priority == 2 && cfg.rng_mode != NTS_RNG_PHILOX));
  // size the scratch arenas once so the training loop never allocates
  uint64_t items = graph->global_vertices;
  for (auto* s : sampler->ssg->sampled_sgs) items = std::max<uint64_t>({items, s->e_cap, s->v_cap});
  hip_check(nts_hip_ctx_reserve(cs->ctx(), graph->global_vertices, items), "nts_hip_ctx_reserve");
  if (ss) {
    hip_check(nts_hip_ctx_reserve(ss->ctx(), graph->global_vertices, items), "nts_hip_ctx_reserve");
    hip_check(nts_hip_ctx_set_gemm_mode(ss->ctx(), cfg.gemm_mode), "nts_hip_ctx_set_gemm_mode");
  }
  // The bottom graph op Y_0 = A_0 X depends on the sampled graph and the
  // feature table only (not on the weights), so it is issued right behind the
  // sampling, on the sampling stream: with the pipeline it runs while the
  // previous batch trains (HBM-bound gather next to MFMA-bound GEMMs).
  early_ = cfg.early_aggregate && cfg.fused_gather && !cfg.gat && !tf_ && !cfg.pd_cache;
  sampler->rerun_ok = !early_;  // (an MT re-run would leave the early aggregation stale)
  if (cfg.pd_cache) {
    TORCH_CHECK(!cfg.gat && L >= 2 && cfg.hip_gemm && cfg.pd_super_batch >= 1 &&
                    cfg.pd_rate >= 0.0,
                "PD cache: GCN/GraphSAGE with >= 2 layers on the MFMA GEMMs");
    pd_cache_map_ = torch::full({(int64_t)graph->global_vertices}, -1, u32_opts(graph->device));
    pd_cache_loc_ = torch::zeros({(int64_t)graph->global_vertices}, u32_opts(graph->device));
  }
  for (int i = 0; i < nslots_; ++i) {
    TORCH_CHECK(hipEventCreateWithFlags(&ready_[i], hipEventDisableTiming) == hipSuccess,
                "hipEventCreate");
    if (early_)
      pre_y_[i] = row_padded_empty((int64_t)sampler->ssgs[i]->sampled_sgs[L - 1]->v_cap,
                                   F.size(1), graph->device);
    if (early_ && fcache)
      stage_[i] = torch::empty({(int64_t)std::max<uint32_t>(sampler->ssgs[i]->sampled_sgs[L - 1]->s_cap, 1),
                                (int64_t)fcache->ld},
                               f32_opts(graph->device));
  }
  correct_ = torch::zeros({1}, u32_opts(graph->device));
  init_nn();
  defer_ = comm && (cfg.overlap_allreduce == 1 || (cfg.overlap_allreduce < 0 && comm->nranks > 1));
  if (defer_) {
    TORCH_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking) == hipSuccess,
                "hipStreamCreate");
    TORCH_CHECK(hipEventCreateWithFlags(&grads_packed_, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&grads_reduced_, hipEventDisableTiming) == hipSuccess,
                "hipEventCreate");
  }
  if (cfg.pd_cache) {  // preSample on the device (the Python runner may replace it)
    auto hot = presample();
    set_presample(hot.first, hot.second);
  }
}

GCN_SAMPLE_ALLGPU_impl::~GCN_SAMPLE_ALLGPU_impl() {
  if (!tl_.empty()) {
    (void)hipDeviceSynchronize();
    const size_t from = tl_.size() > 80 ? tl_.size() - 80 : 0;
    for (size_t i = from; i < tl_.size(); ++i) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, tl_[from].second, tl_[i].second);
      fprintf(stderr, "[timeline] %s %9.1f us\n", tl_[i].first, ms * 1e3);
    }
    for (auto& e : tl_) (void)hipEventDestroy(e.second);
  }
  for (auto* e : ready_)
    if (e) (void)hipEventDestroy(e);
  if (defer_) {
    (void)hipDeviceSynchronize();
    (void)hipEventDestroy(grads_packed_);
    (void)hipEventDestroy(grads_reduced_);
    (void)hipStreamDestroy(comm_stream_);
  }
  for (auto* p : P) delete p;
}

// Sampling of one batch into `slot` (sample_gpu_fast's device part), then —
// with early aggregation — the bottom graph op (fused feature gather +
// aggregation, SingleGPUAllSampleGraphOp::forward on the feature table) on
// the same stream.  Sizes are device-side: nothing here waits for the host.
// NTS_TIMELINE=1: timing events at the start/end of every sampling and
// training launch sequence, printed (relative to the first) at destruction —
// the unperturbed GPU timeline of the two streams (a profiler slows the host).
static bool timeline_on() {
  static const bool on = getenv("NTS_TIMELINE") != nullptr;
  return on;
}
void GCN_SAMPLE_ALLGPU_impl::mark(const char* what, NtsStream& st) {
  if (!timeline_on() || tl_.size() > 4000) return;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return;
  (void)hipEventRecord(e, (hipStream_t)st.stream());
  tl_.push_back({what, e});
}

void GCN_SAMPLE_ALLGPU_impl::issue(int slot, NtsStream& st) {
  mark("S<", st);
  if (cfg.pd_cache) pd_issue(slot, st);
  sampler->issue_gpu_sample(cfg.batch_size, slot, st,
                            cfg.gat ? WeightType::None : cfg.weight_type);
  sampler->omit_map = nullptr;
  {  // load_label_gpu for this batch, on the sampling stream next to its
     // subgraph (off the training stream; ordered by ready_[slot] below)
    SampledSubgraph* q = sampler->ssgs[slot];
    const int64_t n = q->pending_batch;
    NtsVar& t = lbl_[slot];
    if (!t.defined() || t.size(0) < n)
      t = torch::empty({std::max<int64_t>(n, cfg.batch_size)},
                       torch::TensorOptions().dtype(torch::kInt64).device(torch::kCUDA, graph->device));
    if (n > 0)
      hip_check(nts_hip_gather_labels(st.ctx(), L_GT.data_ptr<int64_t>(),
                                      q->sampled_sgs[0]->dev_dst(), nullptr, (uint32_t)n,
                                      t.data_ptr<int64_t>()),
                "nts_hip_gather_labels");
  }
  if (early_) {
    auto guard = st.guard();
    const int L = (int)P.size();
    sampCSC* s = sampler->ssgs[slot]->sampled_sgs[L - 1];
    if (cfg.profile) prof.begin(KernelProfiler::BOTTOM_AGG, (hipStream_t)st.stream());
    NtsVar& y = pre_y_[slot];
    if (fcache)
      fcache->aggregate(st.ctx(), s, dptr<uint32_t>(s->sizes), s->v_cap,
                        dptr<uint32_t>(s->sizes) + 2, s->s_cap, stage_[slot].data_ptr<float>(),
                        y.data_ptr<float>(), (uint64_t)y.stride(0));
    else
      hip_check(nts_hip_spmm_csc_fwd(st.ctx(), s->dev_c_o(), s->dev_r_i(), s->dev_e_w_f(),
                                     dptr<uint32_t>(s->sizes), s->v_cap, F.data_ptr<float>(),
                                     (uint64_t)F.stride(0), s->dev_src(), (uint32_t)F.size(1),
                                     y.data_ptr<float>(), (uint64_t)y.stride(0)),
                "nts_hip_spmm_csc_fwd(early)");
    // bytes are added when the batch's sizes are known (train_batch)
    if (cfg.profile) prof.end(KernelProfiler::BOTTOM_AGG, (hipStream_t)st.stream(), 0.0);
  }
  TORCH_CHECK(hipEventRecord(ready_[slot], (hipStream_t)st.stream()) == hipSuccess,
              "hipEventRecord");
  mark("S>", st);
}

// compulsory bytes of the bottom aggregation: distinct src rows once, index +
// weight per edge, offsets, output rows (+ source map when fused)  
double GCN_SAMPLE_ALLGPU_impl::bottom_bytes(SampledSubgraph* sg, bool fused_map) const {
  sampCSC* s = sg->sampled_sgs[sg->layers - 1];
  const double Fd = (double)(fcache ? fcache->F : F.size(1));
  return Fd * 4.0 * s->src_size + 8.0 * s->e_size + 4.0 * (s->v_size + 1) +
         Fd * 4.0 * s->v_size + (fused_map ? 4.0 * s->src_size : 0.0);
}

void GCN_SAMPLE_ALLGPU_impl::init_nn() {
  for (size_t i = 0; i + 1 < cfg.layer_size.size(); ++i) {
    P.push_back(new Parameter(cfg.layer_size[i], cfg.layer_size[i + 1], cfg.learn_rate, cfg.beta1,
                              cfg.beta2, cfg.epsilon, cfg.weight_decay, graph->device,
                              cfg.seed + (int64_t)i));
    if (cfg.gat)  // attention vector W_att [2 F_{l+1}, 1] (GAT_SAMPLE_ALL_GPU.hpp:141-147)
      P.push_back(new Parameter(2 * cfg.layer_size[i + 1], 1, cfg.learn_rate, cfg.beta1,
                                cfg.beta2, cfg.epsilon, cfg.weight_decay, graph->device,
                                cfg.seed + 1000 + (int64_t)i));
  }
  if (cfg.hip_gemm)
    for (auto* p : P) p->cs = cs.get();
  int64_t n = 0;
  for (auto* p : P) n += p->W.numel();
  grad_bucket = torch::zeros({n}, f32_opts(graph->device));
  if (comm) {  // identical initial weights on every rank (init_parameter / Bcast)
    torch::NoGradGuard ng;
    // the initialisation ran on libtorch's current stream: order it before the
    // broadcast on the driver stream (construction time only)
    TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
    for (auto* p : P) comm->broadcast(p->W.data_ptr<float>(), (uint64_t)p->W.numel(), 0, cs->stream());
  }
}

void GCN_SAMPLE_ALLGPU_impl::set_weights(const std::vector<NtsVar>& ws) {
  flush_update();
  auto guard = cs->guard();
  TORCH_CHECK(ws.size() == P.size(), "one tensor per layer");
  torch::NoGradGuard ng;
  for (size_t i = 0; i < P.size(); ++i) P[i]->W.copy_(ws[i]);
}

std::vector<NtsVar> GCN_SAMPLE_ALLGPU_impl::weights() {
  flush_update();
  std::vector<NtsVar> out;
  for (auto* p : P) out.push_back(p->W.detach().clone());
  return out;
}

// vertexForward (toolkits/GCN_SAMPLE_GPU.hpp:252-266): hidden layers
// dropout(relu(XW)), the last layer log_softmax(XW).
NtsVar GCN_SAMPLE_ALLGPU_impl::vertexForward(int l, NtsVar& a) {
  const int L = (int)P.size();
  if (l == L - 1) return P[l]->forward(a).log_softmax(1);
  if (cfg.hip_gemm && cfg.fuse_activation) {
    const double p = ctx.is_train() ? cfg.drop_rate : 0.0;
    return hip_linear_act(a, P[l]->W, p, (uint64_t)cfg.seed * 0x9E3779B97F4A7C15ull + 1,
                          dropout_calls_++, cs.get(), cfg.pair_table > 0);
  }
  return torch::dropout(torch::relu(P[l]->forward(a)), cfg.drop_rate, ctx.is_train());
}

std::vector<NtsVar> GCN_SAMPLE_ALLGPU_impl::forward(SampledSubgraph* sg, bool keep,
                                                     const NtsVar* pre_y,
                                                     const NtsVar* loss_target) {
  const int L = (int)P.size();
  std::vector<NtsVar> acts;
  NtsVar X0;
  if (!cfg.fused_gather && !tf_) {
    if (fcache)
      sampler->load_feature_gpu_cache(*cs, sg, X0, *fcache);
    else
      sampler->load_feature_gpu(*cs, sg, X0, F);
  }
  int l0 = 0;
  NtsVar X;
  if (pre_y) {  // bottom graph op already ran on the sampling stream (issue())
    NtsVar Y = pre_y->narrow(0, 0, (int64_t)sg->sampled_sgs[L - 1]->v_size);
    flush_update();
    X = ctx.runVertexForward([&](NtsVar& a) { return vertexForward(0, a); }, Y);
    if (keep) {
      acts.push_back(Y.detach());
      acts.push_back(X.detach());
    }
    l0 = 1;
  } else {
    X = X0;
  }
  for (int l = l0; l < L; ++l) {
    const int hop = L - 1 - l;
    NtsVar Y;
    const bool bottom = (l == 0);
    if (bottom && tf_) {  // transform-first: H = X[src] W, X1 = act(A H) (one NN op)
      flush_update();
      sampCSC* s = sg->sampled_sgs[hop];
      const double p = ctx.is_train() ? cfg.drop_rate : 0.0;
      NtsVar h;
      if (keep) h = torch::empty({(int64_t)std::max<uint32_t>(s->src_size, 1), P[0]->W.size(1)},
                                 f32_opts(graph->device));
      const uint64_t off = dropout_calls_++;
      X = ctx.runVertexForward(
          [&](NtsVar& t) {
            return hip_bottom_transform(t, P[0]->W, s, p,
                                        (uint64_t)cfg.seed * 0x9E3779B97F4A7C15ull + 1, off,
                                        cs.get(), profiler(),
                                        keep ? h.data_ptr<float>() : nullptr, pairs_.get());
          },
          F);
      // training: the graph op above applies this layer's relu/dropout
      // backward to its own backward output (one CSR pass instead of the CSR
      // gather + nts_hip_act_backward; same arithmetic); the A/B build
      // -DNTS_TF_MASKED_BWD keeps the unfused masked gather
      // (only over a CSR: with the atomic CSC backward the layer above has
      // none, and this layer then runs nts_hip_act_backward itself)
#ifdef NTS_TF_MASKED_BWD
      constexpr bool masked_env = true;
#else
      constexpr bool masked_env = false;
#endif
      const bool fuse = ctx.is_train() && !masked_env && hop >= 1 &&
                        sg->sampled_sgs[hop - 1]->has_csr;
      if (hop >= 1) {
        sampCSC* up = sg->sampled_sgs[hop - 1];
        up->post_mask = fuse ? X.data_ptr<float>() : nullptr;
        // (A/B build -DNTS_TF_MASK_FLOAT: the mask read from X1's rows)
#ifdef NTS_TF_MASK_FLOAT
        constexpr bool mask_float_env = true;
#else
        constexpr bool mask_float_env = false;
#endif
        up->post_mask_bits = fuse && !mask_float_env && s->act_bits.defined() &&
                                     nts_hip_act_bits_words((uint32_t)X.size(1))
                                 ? reinterpret_cast<const uint32_t*>(s->act_bits.data_ptr<int32_t>())
                                 : nullptr;
        up->post_mask_ld = (uint64_t)X.stride(0);
        up->post_mask_scale = p < 1.0 ? 1.0f / (1.0f - (float)p) : 0.f;
      }
      s->grad_premasked = fuse;
      if (keep) {
        acts.push_back(h.narrow(0, 0, (int64_t)s->src_size));
        acts.push_back(X.detach());
      }
      continue;
    }
    if (bottom && cfg.profile) prof.begin(KernelProfiler::BOTTOM_AGG, (hipStream_t)cs->stream());
    if (cfg.sample_gpu && bottom && cfg.fused_gather)
      Y = ctx.runGraphOp<op::SingleGPUSampleGraphOp>(F, sg, graph.get(), hop, cs.get(), true,
                                                     fcache.get());
    else if (cfg.sample_gpu)
      Y = ctx.runGraphOp<op::SingleGPUSampleGraphOp>(X, sg, graph.get(), hop, cs.get(), false);
    else if (bottom && cfg.fused_gather)
      Y = ctx.runGraphOp<op::SingleGPUAllSampleGraphOp>(F, sg, graph.get(), hop, cs.get(), true,
                                                        fcache.get());
    else
      Y = ctx.runGraphOp<op::SingleGPUAllSampleGraphOp>(X, sg, graph.get(), hop, cs.get(), false);
    if (bottom && cfg.profile)
      prof.end(KernelProfiler::BOTTOM_AGG, (hipStream_t)cs->stream(),
               bottom_bytes(sg, cfg.fused_gather));
    // the previous step's all-reduce ran beside this bottom aggregation,
    // which does not read W; its optimizer step goes in here
    if (bottom) flush_update();
    if (bottom && pd_active_) {
      // GCN_SAMPLE_PD_CACHE::Forward (toolkits/GCN_SAMPLE_PD_CACHE.hpp:916-945):
      // Y W, the cached dsts' rows replaced by the super-batch's (A X) W
      // (load_share_embedding), then relu + dropout.  The omitted dsts have no
      // sampled edges, so their rows of Y are zero and add nothing to dW.
      sampCSC* s = sg->sampled_sgs[hop];
      const uint64_t off = dropout_calls_++;
      const double p = ctx.is_train() ? cfg.drop_rate : 0.0;
      X = ctx.runVertexForward(
          [&](NtsVar& a) {
            NtsVar Z = P[0]->forward(a);
            hip_check(nts_hip_pd_load_share(cs->ctx(), dptr<uint32_t>(s->omit_row), nullptr,
                                            s->v_size, pd_share_.data_ptr<float>(),
                                            (uint64_t)pd_share_.stride(0), (uint32_t)Z.size(1),
                                            Z.data_ptr<float>(), (uint64_t)Z.stride(0)),
                      "nts_hip_pd_load_share");
            if (l == L - 1) return Z.log_softmax(1);
            return hip_relu_dropout(Z, p, (uint64_t)cfg.seed * 0x9E3779B97F4A7C15ull + 1, off,
                                    cs.get());
          },
          Y);
      if (keep) {
        acts.push_back(Y.detach());
        acts.push_back(X.detach());
      }
      continue;
    }
    if (loss_target && l == L - 1)  // vertexForward + Loss of the last layer, fused
      X = ctx.runVertexForward(
          [&](NtsVar& a) {
            return hip_linear_xent(a, P[l]->W, *loss_target, cs.get(), count_to_);
          },
          Y);
    else
      X = ctx.runVertexForward([&](NtsVar& a) { return vertexForward(l, a); }, Y);
    if (keep) {
      acts.push_back(Y.detach());
      acts.push_back(X.detach());
    }
  }
  acts.push_back(X);
  return acts;
}

std::vector<NtsVar> GCN_SAMPLE_ALLGPU_impl::forward_gat(SampledSubgraph* sg) {
  flush_update();
  const int L = (int)sg->layers;
  NtsVar X;
  if (fcache)
    sampler->load_feature_gpu_cache(*cs, sg, X, *fcache);
  else
    sampler->load_feature_gpu(*cs, sg, X, F);
  std::vector<NtsVar> acts;
  for (int l = 0; l < L; ++l) {
    const int hop = L - 1 - l;  // X_{l+1} = relu(attention aggregate of X_l W_l)
    X = hip_gat_layer(X, P[2 * l]->W, P[2 * l + 1]->W, sg->sampled_sgs[hop], cs.get(),
                      profiler());
    acts.push_back(X);
  }
  return acts;
}

void GCN_SAMPLE_ALLGPU_impl::Loss(NtsVar& left, NtsVar& right) {
  NtsVar a = left.log_softmax(1);
  loss = torch::nll_loss(a, right);
  if (ctx.training) ctx.appendNNOp(left, loss);
}

void GCN_SAMPLE_ALLGPU_impl::Update() {
  // GCN_SAMPLE_ALL_MULTI::Update (toolkits/GCN_SAMPLE_ALL_MULTI.hpp:367-377):
  // SUM all-reduce of every W.grad — one fused RCCL call over a flat bucket.
  if (defer_) {
    // pack on the training stream, reduce on the comm stream; the Adam step
    // runs in flush_update() once the next batch first needs W
    TORCH_CHECK(!pending_update_, "deferred update still pending");
    torch::NoGradGuard ng;
    int64_t off = 0;
    for (auto* p : P) {
      const int64_t n = p->W.numel();
      grad_bucket.narrow(0, off, n).copy_(p->W.grad().reshape({-1}));
      off += n;
    }
    TORCH_CHECK(hipEventRecord(grads_packed_, (hipStream_t)cs->stream()) == hipSuccess &&
                    hipStreamWaitEvent(comm_stream_, grads_packed_, 0) == hipSuccess,
                "hipEventRecord/hipStreamWaitEvent");
    comm->allreduce_sum(grad_bucket.data_ptr<float>(), (uint64_t)grad_bucket.numel(), comm_stream_);
    TORCH_CHECK(hipEventRecord(grads_reduced_, comm_stream_) == hipSuccess, "hipEventRecord");
    pending_update_ = true;
    return;
  }
  if (comm) {  // also at one rank: the same bucket, all-reduce and unpack run
    torch::NoGradGuard ng;
    int64_t off = 0;
    for (auto* p : P) {
      const int64_t n = p->W.numel();
      grad_bucket.narrow(0, off, n).copy_(p->W.grad().reshape({-1}));
      off += n;
    }
    comm->allreduce_sum(grad_bucket.data_ptr<float>(), (uint64_t)grad_bucket.numel(), cs->stream());
    off = 0;
    for (auto* p : P) {
      const int64_t n = p->W.numel();
      p->W.mutable_grad().copy_(grad_bucket.narrow(0, off, n).view(p->W.sizes()));
      off += n;
    }
  }
  for (auto* p : P) {
    if (cfg.bias_correction) p->learnC2C_with_decay_Adam(*cs);
    else p->learn_local_with_decay_Adam(*cs);
    p->next();
  }
}

void GCN_SAMPLE_ALLGPU_impl::flush_update() {
  if (!pending_update_) return;
  pending_update_ = false;
  auto guard = cs->guard();
  TORCH_CHECK(hipStreamWaitEvent((hipStream_t)cs->stream(), grads_reduced_, 0) == hipSuccess,
              "hipStreamWaitEvent");
  int64_t off = 0;
  for (auto* p : P) {
    p->adam_from(*cs, grad_bucket.data_ptr<float>() + off, cfg.bias_correction != 0);
    p->next();
    off += p->W.numel();
  }
}

float GCN_SAMPLE_ALLGPU_impl::train_batch() {
  auto guard = cs->guard();
  double t0 = now_s();
  if (cfg.profile) prof.next_step();  // (one kernel class timed per step)
  NtsStream& sst = ss ? *ss : *cs;
  // set_diag_reuse_sample (diagnostic only, not a valid measurement): sample
  // once and train every step on that batch — the training stream's time
  // without the sampler beside it
  const bool diag_reuse = diag_reuse_;
  int slot;
  SampledSubgraph* sg;
  if (diag_reuse && reuse_slot_ >= 0) {
    slot = reuse_slot_;
    sg = sampler->ssgs[slot];
  } else {
    if (prefetched_ >= 0) {
      slot = prefetched_;
      prefetched_ = -1;
    } else {
      slot = next_slot_;
      issue(slot, sst);
    }
    sg = sampler->finish_gpu_sample(slot);
    if (diag_reuse) {
      reuse_slot_ = slot;
    } else if (ss) {
      next_slot_ = (slot + 1) % nslots_;
      if (cfg.sampler_gate > 0 && tf_) {
        // issued from the bottom layer's forward GEMM hook (below), behind it
        deferred_issue_ = [this] { prefetch_next(); };
      } else {
        prefetch_next();
      }
    }
  }
  if (deferred_issue_) {
    if (!gate_ev_)
      TORCH_CHECK(hipEventCreateWithFlags(&gate_ev_, hipEventDisableTiming) == hipSuccess,
                  "hipEventCreate");
    set_bottom_gemm_hooks(
        [this] {
          if (!deferred_issue_) return;
          TORCH_CHECK(hipEventRecord(gate_ev_, (hipStream_t)cs->stream()) == hipSuccess &&
                          hipStreamWaitEvent((hipStream_t)ss->stream(), gate_ev_, 0) == hipSuccess,
                      "hipEventRecord/hipStreamWaitEvent");
          auto f = std::move(deferred_issue_);
          deferred_issue_ = nullptr;
          f();
        },
        cfg.sampler_gate >= 2
            ? std::function<void()>([this] {
                if (gated_slot_ >= 0)
                  TORCH_CHECK(hipStreamWaitEvent((hipStream_t)cs->stream(), ready_[gated_slot_], 0) ==
                                  hipSuccess,
                              "hipStreamWaitEvent");
              })
            : std::function<void()>());
  }
  fresh_pass_ = false;
  last_sg = sg;
  TORCH_CHECK(hipStreamWaitEvent((hipStream_t)cs->stream(), ready_[slot], 0) == hipSuccess,
              "hipStreamWaitEvent");
  double t1 = now_s();
  if (cfg.pd_cache) pd_train(slot);
  mark("T<", *cs);
  target = lbl_[slot].narrow(0, 0, (int64_t)sg->sampled_sgs[0]->v_size);
  ctx.train();
  if (early_ && cfg.profile) prof.add_units(KernelProfiler::BOTTOM_AGG, bottom_bytes(sg, true));
  const int L = (int)P.size();
  if (cfg.gat) {  // GAT_SAMPLE_ALL_GPU::Loss + loss.backward() (toolkits/GAT_SAMPLE_ALL_GPU.hpp:393-399)
    auto acts = forward_gat(sg);
    loss = torch::nll_loss(acts.back().log_softmax(1), target);
    count_correct(acts.back(), target);
    loss.backward();
    ctx.reset();
  } else {
    const bool fuse_loss = cfg.fuse_loss && cfg.hip_gemm && L >= 2 &&
                           hip_linear_xent_supported(P[L - 1]->W.size(0), P[L - 1]->W.size(1));
    count_to_ = dptr<uint32_t>(correct_);
    auto acts = forward(sg, false, early_ ? &pre_y_[slot] : nullptr, fuse_loss ? &target : nullptr);
    count_to_ = nullptr;
    if (fuse_loss) {
      loss = acts.back();
    } else {
      NtsVar out = acts.back();
      count_correct(out, target);
      Loss(out, target);
    }
    ctx.self_backward(false);
  }
  pd_active_ = false;
  if (deferred_issue_) {  // (the hook did not run: issue behind the step's kernels so far)
    auto f = std::move(deferred_issue_);
    deferred_issue_ = nullptr;
    f();
  }
  set_bottom_gemm_hooks(nullptr, nullptr);
  gated_slot_ = -1;
  Update();
  for (auto* p : P) p->zero_grad();
  TORCH_CHECK(hipEventRecord(sg->consumed, (hipStream_t)cs->stream()) == hipSuccess,
              "hipEventRecord");
  mark("T>", *cs);
  double t2 = now_s();
  sample_time += t1 - t0;
  train_time += t2 - t1;
  for (int l = 0; l < sg->layers; ++l) batch_edges += sg->sampled_sgs[l]->e_size;
  ++batches;
  return 0.f;  // the loss stays on the device (no per-step host sync)
}

// the pipelined sampler's next batch (issued behind the batch being trained)
void GCN_SAMPLE_ALLGPU_impl::prefetch_next() {
  if (!pass_done_ && sampler->sample_not_finished()) {
    issue(next_slot_, *ss);  // prefetch the next batch behind this one
    prefetched_ = next_slot_;
    gated_slot_ = next_slot_;
  } else if (!pass_done_) {
    // last batch of the pass: sample the first batch of the next pass now
    // (same seeds, same stream position as after restart()), so the
    // pipeline does not drain at every pass boundary
    sampler->restart();
    issue(next_slot_, *ss);
    carry_ = next_slot_;
    gated_slot_ = next_slot_;
    pass_done_ = true;
  }
}

void GCN_SAMPLE_ALLGPU_impl::restart() {
  if (fresh_pass_) return;  // nothing trained since the last restart
  fresh_pass_ = true;
  if (carry_ >= 0) {  // the next pass's first batch is already in flight
    TORCH_CHECK(prefetched_ < 0, "pipeline state");
    prefetched_ = carry_;
    carry_ = -1;
    pass_done_ = false;
    return;
  }
  pass_done_ = false;
  if (prefetched_ >= 0) {  // drop a prefetched batch of the previous pass
    sampler->finish_gpu_sample(prefetched_);
    prefetched_ = -1;
  }
  sampler->restart();
}

float GCN_SAMPLE_ALLGPU_impl::run_epoch() {
  restart();
  float l = 0;
  while (has_batch()) l = train_batch();
  return l;
}

std::vector<NtsVar> GCN_SAMPLE_ALLGPU_impl::forward_eval(const std::vector<VertexId>& seeds,
                                                         uint64_t batch_seq) {
  flush_update();
  auto guard = cs->guard();
  const int L = (int)cfg.fanout.size();
  std::vector<bool> csr(L, cfg.gat);
  FastSampler s(graph, seeds, L, (int)seeds.size(), cfg.fanout, 1, csr,
                !cfg.gat && cfg.weight_type != WeightType::None, cfg.gat);
  s.rng_mode = cfg.rng_mode;
  s.up_degree = cfg.up_degree;
  s.batch_seq = batch_seq;
  SampledSubgraph* sg = s.sample_gpu_fast((int)seeds.size(), 0, *cs,
                                          cfg.gat ? WeightType::None : cfg.weight_type);
  ctx.eval();
  torch::NoGradGuard ng;
  std::vector<NtsVar> acts;
  if (cfg.gat) {
    acts = forward_gat(sg);
  } else {
    acts = forward(sg, true);
    acts.pop_back();
  }
  ctx.train();
  cs->synchronize();
  return acts;
}

void GCN_SAMPLE_ALLGPU_impl::count_correct(const NtsVar& out, const NtsVar& tgt) {
  torch::NoGradGuard ng;
  correct_.add_(out.argmax(1).eq(tgt).sum().to(torch::kInt32));
}

uint64_t GCN_SAMPLE_ALLGPU_impl::train_correct() {
  cs->synchronize();
  return (uint64_t)(uint32_t)correct_.cpu().item<int32_t>();
}

void GCN_SAMPLE_ALLGPU_impl::reset_correct() {
  auto guard = cs->guard();
  correct_.zero_();
}

double GCN_SAMPLE_ALLGPU_impl::evaluate(const std::vector<VertexId>& nids) {
  flush_update();
  if (nids.empty()) return 0.0;
  auto guard = cs->guard();
  const int L = (int)cfg.fanout.size();
  const WeightType wt = cfg.gat ? WeightType::None : cfg.weight_type;
  std::vector<bool> csr(L, cfg.gat);
  FastSampler s(graph, nids, L, cfg.batch_size, cfg.fanout, 1, csr, wt != WeightType::None,
                cfg.gat);
  s.rng_mode = cfg.rng_mode;
  s.up_degree = cfg.up_degree;
  s.batch_seq = eval_seq;
  NtsVar correct = torch::zeros({1}, u32_opts(graph->device));
  const bool fuse_loss = !cfg.gat && cfg.fuse_loss && cfg.hip_gemm && L >= 2 &&
                         hip_linear_xent_supported(P[L - 1]->W.size(0), P[L - 1]->W.size(1));
  ctx.eval();
  {
    torch::NoGradGuard ng;
    NtsVar tgt;
    while (s.sample_not_finished()) {
      SampledSubgraph* sg = s.sample_gpu_fast(cfg.batch_size, 0, *cs, wt);
      s.load_label_gpu(*cs, sg, tgt, L_GT);
      if (cfg.gat) {
        auto acts = forward_gat(sg);
        correct.add_(acts.back().argmax(1).eq(tgt).sum().to(torch::kInt32));
      } else if (fuse_loss) {
        count_to_ = dptr<uint32_t>(correct);
        forward(sg, false, nullptr, &tgt);
        count_to_ = nullptr;
      } else {
        auto acts = forward(sg, false);
        correct.add_(acts.back().argmax(1).eq(tgt).sum().to(torch::kInt32));
      }
      // the sampler slot is reused by the next batch: order it behind this forward
      TORCH_CHECK(hipEventRecord(sg->consumed, (hipStream_t)cs->stream()) == hipSuccess,
                  "hipEventRecord");
    }
  }
  ctx.train();
  eval_seq = s.batch_seq;
  cs->synchronize();
  return (double)(uint32_t)correct.cpu().item<int32_t>() / (double)nids.size();
}

// ---------------------------------------------------------------------------
// PD cache
std::pair<std::vector<uint32_t>, std::vector<uint32_t>> GCN_SAMPLE_ALLGPU_impl::presample() {
  auto guard = cs->guard();
  const std::vector<VertexId>& ids = sampler->sample_nids;  // shuffled like training
  const uint64_t sbs = (uint64_t)cfg.batch_size * (uint64_t)cfg.pd_super_batch;
  const uint64_t n_sb = (ids.size() + sbs - 1) / sbs;
  const uint64_t V = graph->global_vertices;
  NtsVar seeds = torch::empty({(int64_t)std::max<size_t>(ids.size(), 1)}, u32_opts(graph->device));
  if (!ids.empty())
    seeds.narrow(0, 0, (int64_t)ids.size())
        .copy_(torch::from_blob((void*)ids.data(), {(int64_t)ids.size()}, torch::kInt32));
  NtsVar counts = torch::empty({(int64_t)V}, u32_opts(graph->device));
  NtsVar tmp = torch::empty({(int64_t)V}, u32_opts(graph->device));
  NtsVar out = torch::empty({(int64_t)V}, u32_opts(graph->device));
  NtsVar n_dev = torch::empty({1}, u32_opts(graph->device));
  const nts_graph_dev g = graph->dev();
  std::vector<uint32_t> cnt(n_sb), all;
  // get_most_neighbor over `layers` = the number of GNN layers (the driver's
  // gnnctx->layer_size.size() - 1, toolkits/GCN_SAMPLE_PD_CACHE.hpp:989)
  const int layers = (int)cfg.fanout.size();
  for (uint64_t b = 0; b < n_sb; ++b) {
    const uint64_t beg = b * sbs, n = std::min<uint64_t>(sbs, ids.size() - beg);
    hip_check(nts_hip_presample_counts(cs->ctx(), &g, dptr<uint32_t>(seeds) + beg, (uint32_t)n,
                                       layers, dptr<uint32_t>(counts), dptr<uint32_t>(tmp)),
              "nts_hip_presample_counts");
    hip_check(nts_hip_presample_select(cs->ctx(), dptr<uint32_t>(counts), V, (float)cfg.pd_rate,
                                       dptr<uint32_t>(out), dptr<uint32_t>(n_dev)),
              "nts_hip_presample_select");
    cs->synchronize();
    cnt[b] = (uint32_t)n_dev.cpu().item<int32_t>();
    auto h = out.narrow(0, 0, (int64_t)cnt[b]).cpu();
    const uint32_t* hp = reinterpret_cast<const uint32_t*>(h.data_ptr<int32_t>());
    all.insert(all.end(), hp, hp + cnt[b]);
  }
  return {cnt, all};
}

void GCN_SAMPLE_ALLGPU_impl::set_presample(const std::vector<uint32_t>& counts,
                                           const std::vector<uint32_t>& ids) {
  TORCH_CHECK(cfg.pd_cache, "set_presample needs the PD cache (cfg.pd_cache)");
  auto guard = cs->guard();
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
  pd_counts_ = counts;
  pd_offset_.assign(counts.size() + 1, 0);
  for (size_t i = 0; i < counts.size(); ++i) pd_offset_[i + 1] = pd_offset_[i] + counts[i];
  TORCH_CHECK(pd_offset_.back() == ids.size(), "PD cache: ids must hold sum(counts) vertices");
  // the ids index cache_map / cache_location on the device: a stale or
  // mismatched PRE_SAMPLE_FILE must not write past them
  for (uint32_t id : ids)
    TORCH_CHECK(id < graph->global_vertices, "PD cache: hot vertex id ", id,
                " >= vertex count ", graph->global_vertices, " (stale PRE_SAMPLE_FILE?)");
  uint32_t mx = 1;
  for (uint32_t c : counts) mx = std::max(mx, c);
  std::vector<VertexId> hot(ids.begin(), ids.end());
  if (hot.empty()) hot.push_back(0);  // a sampler needs a non-empty id list
  const int L = (int)cfg.fanout.size();
  // CPU side of the reference (:740-745): a 1-layer sampler over the hot ids
  // with the bottom layer's fanout, consumed super-batch by super-batch
  pd_sampler_ = std::make_unique<FastSampler>(graph, hot, 1, (int)mx,
                                              std::vector<int>{cfg.fanout[L - 1]}, kPdRing,
                                              std::vector<bool>{false},
                                              cfg.weight_type != WeightType::None, false);
  pd_sampler_->rng_mode = cfg.rng_mode;
  pd_sampler_->batch_seq = uint64_t(1) << 48;  // a PHILOX stream of its own
  const int64_t Fin = cfg.layer_size[0];
  for (int i = 0; i < kPdRing; ++i) {
    pd_y_[i] = torch::empty({(int64_t)mx, Fin}, f32_opts(graph->device));
    if (fcache)  // the hot rows' neighbours may be spilled to the host table
      pd_stage_[i] = torch::empty(
          {(int64_t)std::max<uint32_t>(pd_sampler_->ssgs[i]->sampled_sgs[0]->s_cap, 1),
           (int64_t)fcache->ld},
          f32_opts(graph->device));
  }
  pd_share_ = torch::empty({(int64_t)mx, (int64_t)cfg.layer_size[1]}, f32_opts(graph->device));
  pd_ids_ = torch::empty({(int64_t)std::max<size_t>(ids.size(), 1)}, u32_opts(graph->device));
  if (!ids.empty())
    pd_ids_.narrow(0, 0, (int64_t)ids.size())
        .copy_(torch::from_blob((void*)ids.data(), {(int64_t)ids.size()}, torch::kInt32));
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
}

// At sampling time, for a batch that opens a super-batch: its hot vertices get
// the next key in cache_map / cache_location (set_cache_index), their
// 1-layer neighbourhoods are sampled and aggregated (PushDownBatchOp: the
// reference's CPU thread; here the fused gather on the sampling stream).  Every
// batch then samples its bottom layer with the super-batch's key omitted.
void GCN_SAMPLE_ALLGPU_impl::pd_issue(int slot, NtsStream& st) {
  const uint64_t bip = (sampler->work_offset - sampler->work_range[0]) / (uint64_t)cfg.batch_size;
  const int sb = (int)(bip / (uint64_t)cfg.pd_super_batch);
  const bool first = bip % (uint64_t)cfg.pd_super_batch == 0;
  TORCH_CHECK(sb < (int)pd_counts_.size(), "PD cache: more super-batches than preSampled");
  if (first) {
    pd_next_key_++;
    const uint32_t n = pd_counts_[sb];
    auto guard = st.guard();
    hip_check(nts_hip_pd_set_cache(st.ctx(), dptr<uint32_t>(pd_ids_) + pd_offset_[sb], n,
                                   pd_next_key_, dptr<uint32_t>(pd_cache_map_),
                                   dptr<uint32_t>(pd_cache_loc_)),
              "nts_hip_pd_set_cache");
    if (n) {
      const int ring = (int)(pd_next_key_ % kPdRing);
      pd_sampler_->work_offset = (VertexId)pd_offset_[sb];
      pd_sampler_->issue_gpu_sample((int)n, ring, st, cfg.weight_type);
      sampCSC* h = pd_sampler_->ssgs[ring]->sampled_sgs[0];
      NtsVar& y = pd_y_[ring];
      if (fcache)  // two-tier table: cached rows from HBM, the rest staged once from the host
        fcache->aggregate(st.ctx(), h, dptr<uint32_t>(h->sizes), h->v_cap,
                          dptr<uint32_t>(h->sizes) + 2, h->s_cap, pd_stage_[ring].data_ptr<float>(),
                          y.data_ptr<float>(), (uint64_t)y.stride(0));
      else
        hip_check(nts_hip_spmm_csc_fwd(st.ctx(), h->dev_c_o(), h->dev_r_i(), h->dev_e_w_f(),
                                       dptr<uint32_t>(h->sizes), h->v_cap, F.data_ptr<float>(),
                                       (uint64_t)F.stride(0), h->dev_src(), (uint32_t)F.size(1),
                                       y.data_ptr<float>(), (uint64_t)y.stride(0)),
                  "nts_hip_spmm_csc_fwd(pd)");
    }
  }
  pd_slot_key_[slot] = (int)pd_next_key_;
  pd_slot_sb_[slot] = sb;
  pd_slot_first_[slot] = first;
  sampler->omit_map = dptr<uint32_t>(pd_cache_map_);
  sampler->omit_key = pd_next_key_;
  sampler->omit_loc = dptr<uint32_t>(pd_cache_loc_);
}

// Before the forward of a batch: at the super-batch's first batch, the shared
// embedding = (A X) W with the current weights (the reference's CPU GEMM with
// the W of shared_W_queue, :821-840); later batches of the super-batch reuse it.
void GCN_SAMPLE_ALLGPU_impl::pd_train(int slot) {
  flush_update();
  pd_key_ = (uint32_t)pd_slot_key_[slot];
  pd_active_ = true;
  if (!pd_slot_first_[slot]) return;
  const int sb = pd_slot_sb_[slot];
  const uint32_t n = pd_counts_[sb];
  if (n == 0) return;
  const int ring = (int)(pd_key_ % kPdRing);
  pd_sampler_->finish_gpu_sample(ring);  // its sizes (the batch's own sync already covered it)
  auto guard = cs->guard();
  torch::NoGradGuard ng;
  NtsVar Wc = P[0]->W.contiguous();
  hip_check(nts_hip_gemm_f32(cs->ctx(), 0, (int)n, (int)Wc.size(1), (int)Wc.size(0),
                             pd_y_[ring].data_ptr<float>(), (uint64_t)pd_y_[ring].stride(0),
                             Wc.data_ptr<float>(), (uint64_t)Wc.size(1),
                             pd_share_.data_ptr<float>(), (uint64_t)pd_share_.stride(0)),
            "nts_hip_gemm_f32(pd share)");
  TORCH_CHECK(hipEventRecord(pd_sampler_->ssgs[ring]->consumed, (hipStream_t)cs->stream()) ==
                  hipSuccess,
              "hipEventRecord");
}

void GCN_SAMPLE_ALLGPU_impl::reset_stats() {
  prof.reset();
  sample_time = train_time = 0;
  batch_edges = 0;
  batches = 0;
}

SamplerRate sampler_throughput(std::shared_ptr<FullyRepGraph> g, const std::vector<VertexId>& seeds,
                               int batch_size, const std::vector<int>& fanout, WeightType w,
                               int rng_mode, int n_batches, const std::vector<bool>& csr_layers) {
  constexpr int kS = 3;
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
  NtsStream st(g->device, nullptr, 2000);
  auto guard = st.guard();
  const int L = (int)fanout.size();
  FastSampler s(g, seeds, L, batch_size, fanout, kS, csr_layers, w != WeightType::None, false);
  s.rng_mode = rng_mode;
  uint64_t items = g->global_vertices;
  for (auto* x : s.ssg->sampled_sgs) items = std::max<uint64_t>({items, x->e_cap, x->v_cap});
  hip_check(nts_hip_ctx_reserve(st.ctx(), g->global_vertices, items), "nts_hip_ctx_reserve");
  SamplerRate r;
  auto run = [&](int n, bool count) {
    int pending[kS] = {0, 0, 0};
    for (int i = 0; i < n + kS; ++i) {
      const int slot = i % kS;
      if (pending[slot]) {
        // (no consumer: the slot is free once its sizes are read.  Recording
        // `consumed` here, at the stream's tail, made the next issue into the
        // slot wait for every batch in flight — one batch at a time, the GPU
        // idle while the host issued the next: 5.7 G edges/s)
        SampledSubgraph* sg = s.finish_gpu_sample(slot);
        pending[slot] = 0;
        if (count) {
          for (auto* x : sg->sampled_sgs) r.edges += x->e_size;
          ++r.batches;
        }
      }
      if (i >= n) continue;
      if (!s.sample_not_finished()) s.restart();
      s.issue_gpu_sample(batch_size, slot, st, w);
      pending[slot] = 1;
    }
  };
  run(std::min(n_batches, 4), false);  // warm-up (first-touch, code objects)
  st.synchronize();
  const auto t0 = std::chrono::steady_clock::now();
  run(n_batches, true);
  st.synchronize();
  r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

}  // namespace nts
