// C++ host layer: streams, graph, sampler, graph ops, autodiff context,
// parameters and the RCCL communicator.  See nts_host.hpp for the reference
// classes each of these mirrors.
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>

#include "nts_host.hpp"

namespace nts {

void hip_check(int rc, const char* what) {
  if (rc != NTS_OK)
    throw std::runtime_error(std::string(what) + ": nts_hip error " + std::to_string(rc) + ": " +
                             nts_hip_last_error());
}

static void hip_rt(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// NTS_HOST_PROFILE=1: host-side durations of the sampler issue/finish calls
static bool host_profile() {
  static const bool on = getenv("NTS_HOST_PROFILE") != nullptr;
  return on;
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------------------
// The structs of include/nts_hip.h are passed by pointer: a host layer built
// against another header revision must not reach the kernels.
static void check_abi() {
  TORCH_CHECK(nts_hip_abi_version() == NTS_HIP_ABI_VERSION, "libnts_hip.so ABI ",
              nts_hip_abi_version(), " != host layer ABI ", NTS_HIP_ABI_VERSION,
              ": rebuild (python -c 'import __graft_entry__ as g; g.build()')");
}

NtsStream::NtsStream(int device, void* stream, uint64_t seed, bool high_priority)
    : device_(device),
      torch_stream_(stream ? c10::hip::getStreamFromExternal((hipStream_t)stream, (c10::DeviceIndex)device)
                           : c10::hip::getStreamFromPool(high_priority, (c10::DeviceIndex)device)) {
  // a pool stream, never the legacy NULL stream: our kernels must not
  // serialise with every other blocking stream of the device
  check_abi();
  hip_check(nts_hip_ctx_create(&ctx_, device, (void*)torch_stream_.stream(), seed),
            "nts_hip_ctx_create");
}
static hipStream_t create_masked(int device, const std::vector<uint32_t>& mask) {
  hip_rt(hipSetDevice(device), "hipSetDevice");
  hipStream_t s = nullptr;
  hip_rt(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()),
         "hipExtStreamCreateWithCUMask");
  return s;
}
NtsStream::NtsStream(int device, const std::vector<uint32_t>& cu_mask, uint64_t seed)
    : device_(device),
      torch_stream_(c10::hip::getStreamFromExternal(create_masked(device, cu_mask),
                                                    (c10::DeviceIndex)device)) {
  check_abi();
  owned_ = torch_stream_.stream();
  hip_check(nts_hip_ctx_create(&ctx_, device, (void*)owned_, seed), "nts_hip_ctx_create");
}
NtsStream::~NtsStream() {
  nts_hip_ctx_destroy(ctx_);
  if (owned_) (void)hipStreamDestroy(owned_);
}

std::vector<uint32_t> cu_mask_spread(int device, int n, bool complement) {
  hipDeviceProp_t prop;
  hip_rt(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
  const int total = prop.multiProcessorCount;
  TORCH_CHECK(n > 0 && n < total, "CU partition size must be in (0, ", total, ")");
  const int step = total / n;
  std::vector<uint32_t> mask((total + 31) / 32, 0u);
  int taken = 0;
  for (int i = 0; i < total; ++i) {
    const bool in = (i % step == 0) && taken < n;
    if (in) ++taken;
    if (in != complement) mask[i / 32] |= 1u << (i % 32);
  }
  return mask;
}
void NtsStream::setNewStream(void* stream) {
  hip_check(nts_hip_ctx_set_stream(ctx_, stream), "setNewStream");
  torch_stream_ = c10::hip::getStreamFromExternal((hipStream_t)stream, (c10::DeviceIndex)device_);
}
void* NtsStream::stream() const { return nts_hip_ctx_get_stream(ctx_); }
void NtsStream::synchronize() const {
  hip_rt(hipStreamSynchronize((hipStream_t)stream()), "hipStreamSynchronize");
}

// ---------------------------------------------------------------------------
std::shared_ptr<FullyRepGraph> FullyRepGraph::from_edges(NtsStream& cs, const torch::Tensor& src,
                                                         const torch::Tensor& dst,
                                                         VertexId vertices) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.dtype() == torch::kInt32 &&
                  dst.dtype() == torch::kInt32 && src.numel() == dst.numel(),
              "from_edges: src/dst must be int32 CUDA tensors of equal length");
  hip_rt(hipDeviceSynchronize(), "hipDeviceSynchronize");  // inputs may come from any stream
  auto guard = cs.guard();
  auto g = std::make_shared<FullyRepGraph>();
  g->device = cs.device();
  g->global_vertices = vertices;
  g->global_edges = (uint64_t)src.numel();
  auto s = src.contiguous(), d = dst.contiguous();
  g->column_offset = torch::empty({(int64_t)vertices + 1},
                                  torch::TensorOptions().dtype(torch::kInt64).device(torch::kCUDA, g->device));
  g->row_indices = torch::empty({(int64_t)std::max<uint64_t>(g->global_edges, 1)}, u32_opts(g->device));
  g->in_degree = torch::empty({(int64_t)vertices}, u32_opts(g->device));
  g->out_degree = torch::empty({(int64_t)vertices}, u32_opts(g->device));
  hip_check(nts_hip_build_csc(cs.ctx(), dptr<uint32_t>(s), dptr<uint32_t>(d), g->global_edges,
                              vertices, dptr<uint64_t>(g->column_offset),
                              dptr<uint32_t>(g->row_indices)),
            "nts_hip_build_csc");
  hip_check(nts_hip_degrees(cs.ctx(), dptr<uint32_t>(s), dptr<uint32_t>(d), g->global_edges,
                            vertices, dptr<uint32_t>(g->out_degree), dptr<uint32_t>(g->in_degree)),
            "nts_hip_degrees");
  cs.synchronize();
  return g;
}

std::shared_ptr<FullyRepGraph> FullyRepGraph::from_csc(torch::Tensor column_offset,
                                                       torch::Tensor row_indices,
                                                       torch::Tensor in_degree,
                                                       torch::Tensor out_degree) {
  auto g = std::make_shared<FullyRepGraph>();
  TORCH_CHECK(column_offset.dtype() == torch::kInt64 && row_indices.dtype() == torch::kInt32,
              "from_csc: column_offset int64, row_indices int32");
  g->device = column_offset.device().index();
  g->global_vertices = (VertexId)(column_offset.numel() - 1);
  g->global_edges = (uint64_t)row_indices.numel();
  g->column_offset = column_offset.contiguous();
  g->row_indices = row_indices.contiguous();
  g->in_degree = in_degree.contiguous();
  g->out_degree = out_degree.contiguous();
  return g;
}

nts_graph_dev FullyRepGraph::dev() const {
  nts_graph_dev d;
  d.n_vertices = global_vertices;
  d.n_edges = global_edges;
  d.column_offset = dptr<uint64_t>(column_offset);
  d.row_indices = dptr<uint32_t>(row_indices);
  d.in_degree = dptr<uint32_t>(in_degree);
  d.out_degree = dptr<uint32_t>(out_degree);
  return d;
}

// ---------------------------------------------------------------------------
void sampCSC::set_merge_src_dst() {
  dst_local_id = torch::empty({std::max<int64_t>(v_cap, 1)}, u32_opts(column_offset.device().index()));
  if (has_csr)
    csr_edge_id = torch::empty({std::max<int64_t>(e_cap, 1)}, u32_opts(column_offset.device().index()));
}

sampCSC::sampCSC(int device, VertexId vc, VertexId ec, VertexId sc, bool csr, bool weights)
    : v_cap(vc), e_cap(ec), s_cap(sc), has_csr(csr) {
  auto U = u32_opts(device);
  auto F = f32_opts(device);
  const int64_t e1 = std::max<int64_t>(ec, 1), s1 = std::max<int64_t>(sc, 1);
  column_offset = torch::empty({(int64_t)vc + 1}, U);
  row_indices = torch::empty({e1}, U);
  sample_ans = torch::empty({e1}, U);
  edge_dst = torch::empty({e1}, U);
  source = torch::empty({s1}, U);
  sizes = torch::zeros({4}, U);
  if (weights) edge_weight_forward = torch::empty({e1}, F);
  if (csr) {
    row_offset = torch::empty({(int64_t)sc + 1}, U);
    column_indices = torch::empty({e1}, U);
    if (weights) edge_weight_backward = torch::empty({e1}, F);
  }
}

std::vector<VertexId> sampCSC::host_u32(const torch::Tensor& t, size_t n) const {
  auto c = t.narrow(0, 0, (int64_t)n).cpu();
  std::vector<VertexId> out(n);
  if (n) std::memcpy(out.data(), c.data_ptr(), n * 4);
  return out;
}

static std::vector<std::array<uint64_t, 3>> layer_caps(VertexId batch,
                                                       const std::vector<int>& fanout,
                                                       VertexId V, uint64_t E, bool merge) {
  std::vector<std::array<uint64_t, 3>> caps;
  uint64_t v = batch;
  for (int f : fanout) {
    uint64_t e = f < 0 ? E : std::min<uint64_t>(v * (uint64_t)f, E);
    uint64_t s = std::min<uint64_t>(e + (merge ? v : 0), V);
    TORCH_CHECK(e <= 0xFFFFFFFFull, "sampled layer exceeds 2^32 edges");
    caps.push_back({v, e, s});
    v = s;
  }
  return caps;
}

SampledSubgraph::SampledSubgraph(int device, int layers_, const std::vector<int>& fanout_,
                                 VertexId batch, VertexId vertices, uint64_t edges,
                                 const std::vector<bool>& csr, bool weights, bool merge)
    : layers(layers_), fanout(fanout_) {
  auto caps = layer_caps(batch, fanout, vertices, edges, merge);
  for (int l = 0; l < layers; ++l) {
    bool c = csr.empty() ? true : (bool)csr[l];
    sampled_sgs.push_back(new sampCSC(device, (VertexId)caps[l][0], (VertexId)caps[l][1],
                                      (VertexId)caps[l][2], c, weights));
    if (merge) sampled_sgs.back()->set_merge_src_dst();
  }
  // every layer's sizes[4] as a view of one device array: one D2H per batch
  dev_sizes = torch::zeros({std::max(layers, 1) * 4}, u32_opts(device));
  for (int l = 0; l < layers; ++l) sampled_sgs[l]->sizes = dev_sizes.narrow(0, 4 * l, 4);
  void* hs = nullptr;
  hip_rt(hipHostMalloc(&hs, 16 * (size_t)std::max(layers, 1), hipHostMallocMapped | hipHostMallocCoherent),
         "hipHostMalloc(sizes)");
  host_sizes = static_cast<int32_t*>(hs);
  std::fill(host_sizes, host_sizes + 4 * std::max(layers, 1), 0);
  void* hd = nullptr;
  hip_rt(hipHostGetDevicePointer(&hd, hs, 0), "hipHostGetDevicePointer(sizes)");
  host_sizes_dev = static_cast<uint32_t*>(hd);
  hip_rt(hipEventCreateWithFlags(&sampled, hipEventDisableTiming), "hipEventCreate");
  hip_rt(hipEventCreateWithFlags(&consumed, hipEventDisableTiming), "hipEventCreate");
}

SampledSubgraph::~SampledSubgraph() {
  for (auto* s : sampled_sgs) delete s;
  (void)hipHostFree(host_sizes);
  (void)hipEventDestroy(sampled);
  (void)hipEventDestroy(consumed);
}

// ---------------------------------------------------------------------------
FastSampler::FastSampler(std::shared_ptr<FullyRepGraph> g, const std::vector<VertexId>& index,
                         int layers, int batch_size, const std::vector<int>& fanout_,
                         int pipeline_num, std::vector<bool> csr_layers, bool weights,
                         bool merge_src_dst)
    : whole_graph(g), layer(layers), fanout(fanout_), batch_cap_((VertexId)batch_size) {
  TORCH_CHECK((int)fanout.size() == layers, "fanout size != layers");
  if (pipeline_num < 1) pipeline_num = 1;
  for (int i = 0; i < pipeline_num; ++i)
    ssgs.push_back(new SampledSubgraph(g->device, layers, fanout, batch_cap_, g->global_vertices,
                                       g->global_edges, csr_layers, weights, merge_src_dst));
  ssg = ssgs[0];
  recs_.resize(ssgs.size());
  set_sample_nids(index);
  dev_iota_ = torch::arange((int64_t)batch_cap_ + 1, u32_opts(g->device));
}

FastSampler::~FastSampler() {
  for (auto* s : ssgs) delete s;
}

void FastSampler::set_sample_nids(const std::vector<VertexId>& ids) {
  sample_nids = ids;
  work_range[0] = 0;
  work_range[1] = (VertexId)sample_nids.size();
  work_offset = 0;
  dev_nids_ = torch::empty({(int64_t)std::max<size_t>(ids.size(), 1)}, u32_opts(whole_graph->device));
  if (!ids.empty()) {
    auto h = torch::from_blob((void*)sample_nids.data(), {(int64_t)ids.size()}, torch::kInt32);
    dev_nids_.narrow(0, 0, (int64_t)ids.size()).copy_(h);
  }
}

SampledSubgraph* FastSampler::sample_gpu_fast(int batch_size, int ssg_id, NtsStream& cs,
                                              WeightType w) {
  issue_gpu_sample(batch_size, ssg_id, cs, w);
  return finish_gpu_sample(ssg_id);
}

void FastSampler::issue_gpu_sample(int batch_size, int ssg_id, NtsStream& cs, WeightType w) {
  double t0 = now_s();
  TORCH_CHECK(work_offset < work_range[1], "sample_gpu_fast: no work left");
  TORCH_CHECK((VertexId)batch_size <= batch_cap_, "batch larger than the sampler's capacity");
  TORCH_CHECK(ssg_id >= 0 && ssg_id < (int)ssgs.size(), "ssg_id out of range");
  ssg = ssgs[ssg_id];
  const VertexId actual = std::min<VertexId>((VertexId)batch_size, work_range[1] - work_offset);
  hipStream_t st = (hipStream_t)cs.stream();
  // The slot's previous batch must be trained before it is overwritten.  With
  // several slots (pipelined sampler on its own stream) wait for that on the
  // host: ROCm blocks every kernel launch on a stream whose queue waits on an
  // unfinished event of another stream (~60 us each here), which would stall
  // the whole issue loop; the event is normally complete already.
  if (ssgs.size() > 1) hip_rt(hipEventSynchronize(ssg->consumed), "hipEventSynchronize");
  hip_rt(hipStreamWaitEvent(st, ssg->consumed, 0), "hipStreamWaitEvent");
  int wt = w == WeightType::Sum           ? NTS_WEIGHT_SUM
           : w == WeightType::Mean        ? NTS_WEIGHT_MEAN
           : w == WeightType::MeanSampled ? NTS_WEIGHT_MEAN_SAMPLED
                                          : NTS_WEIGHT_NONE;
  if (up_degree && wt != NTS_WEIGHT_NONE) wt |= NTS_WEIGHT_UP_DEGREE;
  // what a re-run of this batch needs (MT19937 modes: a short word stream)
  IssueRec& r = recs_[ssg_id];
  r.offset = work_offset;
  r.actual = actual;
  r.batch_seq = batch_seq;
  r.wt = wt;
  r.omit_map = omit_map;
  r.omit_key = omit_key;
  r.omit_loc = omit_loc;
  r.cs = &cs;
  if (rng_mode != NTS_RNG_PHILOX) {
    if (!r.mt_ckpt.defined())
      r.mt_ckpt = torch::empty({625}, u32_opts(whole_graph->device));
    // the generator state before the batch's first layer (stream order)
    hip_check(nts_hip_mt_checkpoint(cs.ctx(), dptr<uint32_t>(r.mt_ckpt)), "nts_hip_mt_checkpoint");
  }
  issued_.push_back(ssg_id);
  enqueue_layers(ssg_id, r);
  if (host_profile()) fprintf(stderr, "[host] issue total: %.1f us\n", (now_s() - t0) * 1e6);
  ssg->pending_batch = (int)actual;
  work_offset += actual;
  ++batch_seq;
  all_time += now_s() - t0;
}

// the batch's sampling kernels (every layer) on the record's stream
void FastSampler::enqueue_layers(int ssg_id, const IssueRec& r) {
  ssg = ssgs[ssg_id];
  NtsStream& cs = *r.cs;
  hipStream_t st = (hipStream_t)cs.stream();
  const nts_graph_dev g = whole_graph->dev();
  const int wt = r.wt;
  const VertexId actual = r.actual;
  const uint64_t bseq = r.batch_seq;
  const VertexId* dst = dptr<VertexId>(dev_nids_) + r.offset;
  sampCSC* s0 = ssg->sampled_sgs[0];
  // layer-0 v_size as a device scalar without a per-batch memset: entry
  // `actual` of the device table 0..batch_cap
  (void)s0;
  const VertexId* vsz = dptr<VertexId>(dev_iota_) + actual;
  for (int l = 0; l < layer; ++l) {
    sampCSC* s = ssg->sampled_sgs[l];
    nts_sampcsc_dev o{};
    o.v_cap = s->v_cap;
    o.e_cap = s->e_cap;
    o.s_cap = s->s_cap;
    o.destination = dst;
    o.v_size = vsz;
    o.column_offset = dptr<uint32_t>(s->column_offset);
    o.row_indices = dptr<uint32_t>(s->row_indices);
    o.sample_ans = dptr<uint32_t>(s->sample_ans);
    o.edge_dst = dptr<uint32_t>(s->edge_dst);
    o.source = dptr<uint32_t>(s->source);
    o.edge_weight_forward = wt == NTS_WEIGHT_NONE ? nullptr : dptr<float>(s->edge_weight_forward);
    o.row_offset = s->has_csr ? dptr<uint32_t>(s->row_offset) : nullptr;
    o.column_indices = s->has_csr ? dptr<uint32_t>(s->column_indices) : nullptr;
    o.edge_weight_backward =
        (s->has_csr && wt != NTS_WEIGHT_NONE) ? dptr<float>(s->edge_weight_backward) : nullptr;
    o.sizes = dptr<uint32_t>(s->sizes);
    o.dst_local_id = dptr<uint32_t>(s->dst_local_id);  // undefined (NULL) unless merged
    o.csr_edge_id = dptr<uint32_t>(s->csr_edge_id);
    o.sizes_host = ssg->host_sizes_dev + 4 * l;
    if (l == layer - 1 && r.omit_map) {
      if (!s->omit_row.defined())
        s->omit_row = torch::empty({std::max<int64_t>(s->v_cap, 1)}, u32_opts(whole_graph->device));
      o.omit_map = r.omit_map;
      o.omit_key = r.omit_key;
      o.omit_loc = r.omit_loc;
      o.omit_row = dptr<uint32_t>(s->omit_row);
    }
    const double tl = now_s();
    hip_check(nts_hip_sample_layer(cs.ctx(), &g, fanout[l], l, bseq, rng_mode, wt, &o),
              "nts_hip_sample_layer");
    if (host_profile()) fprintf(stderr, "[host] sample_layer %d: %.1f us\n", l, (now_s() - tl) * 1e6);
    // the reference keeps the destination as a view of the previous source
    if (l == 0)
      s->destination = dev_nids_.narrow(0, r.offset, std::max<int64_t>(actual, 0));
    else
      s->destination = ssg->sampled_sgs[l - 1]->source;
    dst = o.source;
    vsz = o.sizes + 2;
  }
  // the layers' sizes reach host_sizes from their last kernels (the reference
  // syncs twice per layer; a D2H copy here cost a blit kernel per batch)
  hip_rt(hipEventRecord(ssg->sampled, st), "hipEventRecord");
}

void FastSampler::set_mt_budget_scale(NtsStream& cs, double scale) {
  mt_budget_ = scale;
  hip_check(nts_hip_mt_budget_scale(cs.ctx(), scale), "nts_hip_mt_budget_scale");
}

// MT19937 modes: a layer's draws passed the words generated for it (its
// bound, nts_hip_mt_budget_scale).  That layer left the generator where it
// began, so every layer after it — of this batch and of the batches issued
// behind it — read the stream from the wrong word.  Re-run from the batch's
// checkpoint with every bound scaled up: the batch and each one issued after
// it, in order (the same stream, so the same, reference-exact sets).
void FastSampler::rerun_from(int ssg_id) {
  TORCH_CHECK(rng_mode != NTS_RNG_PHILOX, "only the MT19937 modes can fall short");
  TORCH_CHECK(rerun_ok, "a short MT19937 stream with work chained to the sampled batches "
              "(early aggregation): cannot re-run");
  auto it = std::find(issued_.begin(), issued_.end(), ssg_id);
  TORCH_CHECK(it != issued_.end(), "re-run of a batch that is not pending");
  IssueRec& r0 = recs_[ssg_id];
  NtsStream& cs = *r0.cs;
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
  mt_budget_ = std::min(mt_budget_ * 4.0, 1e4);
  hip_check(nts_hip_mt_budget_scale(cs.ctx(), mt_budget_), "nts_hip_mt_budget_scale");
  hip_check(nts_hip_mt_rewind(cs.ctx(), dptr<uint32_t>(r0.mt_ckpt)), "nts_hip_mt_rewind");
  ++mt_reruns;
  for (auto j = it; j != issued_.end(); ++j) {
    IssueRec& r = recs_[*j];
    hip_check(nts_hip_mt_checkpoint(r.cs->ctx(), dptr<uint32_t>(r.mt_ckpt)), "nts_hip_mt_checkpoint");
    enqueue_layers(*j, r);
  }
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
}

SampledSubgraph* FastSampler::finish_gpu_sample(int ssg_id) {
  double t0 = now_s();
  ssg = ssgs[ssg_id];
  TORCH_CHECK(ssg->pending_batch > 0, "finish_gpu_sample without a pending issue");
  hip_rt(hipEventSynchronize(ssg->sampled), "hipEventSynchronize");
  if (host_profile()) fprintf(stderr, "[host] finish wait: %.1f us\n", (now_s() - t0) * 1e6);
  const volatile int32_t* hs = ssg->host_sizes;
  for (int attempt = 0;; ++attempt) {
    bool short_stream = false;
    for (int l = 0; l < layer; ++l) short_stream |= (hs[4 * l + 3] & 4) != 0;
    if (!short_stream) break;
    TORCH_CHECK(attempt < 8, "the MT19937 word stream fell short ", attempt + 1,
                " times for one batch (bound scale ", mt_budget_, ")");
    rerun_from(ssg_id);  // synchronises (and moves `ssg` to the last slot it re-ran)
    ssg = ssgs[ssg_id];
  }
  ssg->pending_batch = 0;
  issued_.erase(std::find(issued_.begin(), issued_.end(), ssg_id));
  for (int l = 0; l < layer; ++l) {
    sampCSC* s = ssg->sampled_sgs[l];
    s->v_size = (VertexId)hs[4 * l];
    s->e_size = (VertexId)hs[4 * l + 1];
    s->src_size = (VertexId)hs[4 * l + 2];
    TORCH_CHECK(hs[4 * l + 3] == 0, "sampled layer ", l, " exceeded its capacity");
    sampled_edges += s->e_size;
  }
  all_time += now_s() - t0;
  return ssg;
}

void FastSampler::load_feature_gpu(NtsStream& cs, SampledSubgraph* sg, NtsVar& local_feature,
                                   const NtsVar& global_feature) {
  sampCSC* top = sg->sampled_sgs[layer - 1];
  const int64_t F = global_feature.size(1);
  if (!local_feature.defined() || local_feature.size(0) != (int64_t)top->src_size ||
      local_feature.size(1) != F)  // 128-byte row pitch: float4 rows for the GEMMs
    local_feature = row_padded_empty((int64_t)top->src_size, F, whole_graph->device);
  hip_check(nts_hip_gather_rows(cs.ctx(), global_feature.data_ptr<float>(),
                                (uint64_t)global_feature.stride(0), top->dev_src(), nullptr,
                                top->src_size, (uint32_t)F, local_feature.data_ptr<float>(),
                                (uint64_t)local_feature.stride(0)),
            "nts_hip_gather_rows");
}

void FastSampler::load_feature_gpu_cache(NtsStream& cs, SampledSubgraph* sg,
                                         NtsVar& local_feature, const FeatureCache& fc) {
  sampCSC* top = sg->sampled_sgs[layer - 1];
  if (!local_feature.defined() || local_feature.size(0) != (int64_t)top->src_size ||
      local_feature.size(1) != fc.F)
    local_feature = torch::empty({(int64_t)top->src_size, fc.F}, f32_opts(whole_graph->device));
  hip_check(nts_hip_gather_rows_cached(cs.ctx(), fc.cache_ptr(), fc.ld,
                                       dptr<uint32_t>(fc.cache_map), fc.host_dev, fc.ld,
                                       top->dev_src(), nullptr, top->src_size, (uint32_t)fc.F,
                                       local_feature.data_ptr<float>(),
                                       (uint64_t)local_feature.stride(0)),
            "nts_hip_gather_rows_cached");
}

FeatureCache::FeatureCache(NtsStream& cs, const FullyRepGraph& g, const NtsVar& table,
                           uint64_t n_cache_)
    : n_vertices(g.global_vertices), n_cache(n_cache_), F(table.size(1)) {
  TORCH_CHECK(table.is_cuda() && table.dtype() == torch::kFloat32 && table.dim() == 2 &&
                  table.stride(1) == 1 && (uint64_t)table.size(0) == n_vertices,
              "feature table must be fp32 [V, F] on the GPU");
  TORCH_CHECK(n_cache <= n_vertices, "n_cache > V");
  ld = (uint64_t)(F + 31) / 32 * 32;  // 128-byte rows in both tiers
  void* hp = nullptr;
  hip_check(nts_hip_host_alloc(n_vertices * ld * sizeof(float), &hp), "nts_hip_host_alloc");
  host = static_cast<float*>(hp);
  void* dp = nullptr;
  hip_check(nts_hip_host_device_pointer(hp, &dp), "nts_hip_host_device_pointer");
  host_dev = static_cast<const float*>(dp);
  // spill: the whole table to the host (the reference's pinned
  // local_feature, core/ntsDataloador.hpp:483), then the hot rows back to HBM
  TORCH_CHECK(hipMemcpy2DAsync(host, ld * sizeof(float), table.data_ptr<float>(),
                               (size_t)table.stride(0) * sizeof(float), (size_t)F * sizeof(float),
                               (size_t)n_vertices, hipMemcpyDeviceToHost,
                               (hipStream_t)cs.stream()) == hipSuccess,
              "hipMemcpy2DAsync");
  cache_map = torch::empty({(int64_t)n_vertices}, u32_opts(g.device));
  if (n_cache) {
    cache_ids = torch::empty({(int64_t)n_cache}, u32_opts(g.device));
    cache = torch::empty({(int64_t)n_cache, (int64_t)ld}, f32_opts(g.device)).narrow(1, 0, F);
  }
  hip_check(nts_hip_cache_select(cs.ctx(), dptr<uint32_t>(g.out_degree), n_vertices, n_cache,
                                 dptr<uint32_t>(cache_map), dptr<uint32_t>(cache_ids)),
            "nts_hip_cache_select");
  if (n_cache)  // gater_cpu_cache_feature_and_trans_to_gpu
    hip_check(nts_hip_gather_rows(cs.ctx(), table.data_ptr<float>(), (uint64_t)table.stride(0),
                                  dptr<uint32_t>(cache_ids), nullptr, (uint32_t)n_cache,
                                  (uint32_t)F, cache.data_ptr<float>(), ld),
              "nts_hip_gather_rows");
  cs.synchronize();
}

void FeatureCache::aggregate(nts_hip_ctx* ctx, const sampCSC* s, const uint32_t* v_dev,
                             uint32_t v_cap, const uint32_t* s_dev, uint32_t s_cap, float* stage,
                             float* y, uint64_t ldy) const {
  hip_check(nts_hip_stage_uncached_rows(ctx, dptr<uint32_t>(cache_map), host_dev, ld,
                                        s->dev_src(), s_dev, s_cap, (uint32_t)F, stage, ld),
            "nts_hip_stage_uncached_rows");
  hip_check(nts_hip_spmm_csc_fwd_cached(ctx, s->dev_c_o(), s->dev_r_i(), s->dev_e_w_f(), v_dev,
                                        v_cap, cache_ptr(), ld, dptr<uint32_t>(cache_map), stage,
                                        ld, 1, s->dev_src(), (uint32_t)F, y, ldy),
            "nts_hip_spmm_csc_fwd_cached");
}

FeatureCache::~FeatureCache() {
  if (host) (void)nts_hip_host_free(host);
}

void FastSampler::load_label_gpu(NtsStream& cs, SampledSubgraph* sg, NtsVar& local_label,
                                 const NtsVar& global_label) {
  sampCSC* s0 = sg->sampled_sgs[0];
  if (!local_label.defined() || local_label.size(0) != (int64_t)s0->v_size)
    local_label = torch::empty({(int64_t)s0->v_size},
                               torch::TensorOptions().dtype(torch::kInt64).device(torch::kCUDA, whole_graph->device));
  hip_check(nts_hip_gather_labels(cs.ctx(), global_label.data_ptr<int64_t>(), s0->dev_dst(),
                                  nullptr, s0->v_size, local_label.data_ptr<int64_t>()),
            "nts_hip_gather_labels");
}

// ---------------------------------------------------------------------------
namespace op {

SingleGPUAllSampleGraphOp::SingleGPUAllSampleGraphOp(SampledSubgraph* sgs, FullyRepGraph* graph,
                                                     int layer_, NtsStream* cs, bool gather,
                                                     const FeatureCache* fc)
    : subgraphs(sgs), layer(layer_), cuda_stream(cs), gather_from_table(gather),
      feature_cache(fc) {
  (void)graph;
  TORCH_CHECK(!fc || gather, "a feature cache needs gather_from_table");
}

NtsVar SingleGPUAllSampleGraphOp::forward(NtsVar& f_input) {
  sampCSC* sg = subgraphs->sampled_sgs[layer];
  if (feature_cache) {  // two-tier table: f_input only carries the width
    const FeatureCache& fc = *feature_cache;
    NtsVar f_output = row_padded_empty((int64_t)sg->v_size, fc.F, cuda_stream->device());
    NtsVar stage = torch::empty({(int64_t)std::max<uint32_t>(sg->src_size, 1), (int64_t)fc.ld},
                                f32_opts(cuda_stream->device()));
    fc.aggregate(cuda_stream->ctx(), sg, nullptr, sg->v_size, nullptr, sg->src_size,
                 stage.data_ptr<float>(), f_output.data_ptr<float>(), (uint64_t)f_output.stride(0));
    if (output_requires_grad) f_output.set_requires_grad(true);
    return f_output;
  }
  TORCH_CHECK(f_input.is_cuda() && f_input.dtype() == torch::kFloat32 && f_input.dim() == 2 &&
                  f_input.stride(1) == 1,
              "graph op input must be a row-major fp32 CUDA matrix");
  TORCH_CHECK(gather_from_table || f_input.size(0) >= (int64_t)sg->src_size,
              "graph op input has fewer rows than src_size");
  const int64_t F = f_input.size(1);
  NtsVar f_output = row_padded_empty((int64_t)sg->v_size, F, cuda_stream->device());
  hip_check(nts_hip_spmm_csc_fwd(cuda_stream->ctx(), sg->dev_c_o(), sg->dev_r_i(), sg->dev_e_w_f(),
                                 nullptr, sg->v_size, f_input.data_ptr<float>(),
                                 (uint64_t)f_input.stride(0),
                                 gather_from_table ? sg->dev_src() : nullptr, (uint32_t)F,
                                 f_output.data_ptr<float>(), (uint64_t)f_output.stride(0)),
            "nts_hip_spmm_csc_fwd");
  if (output_requires_grad) f_output.set_requires_grad(true);
  return f_output;
}

NtsVar SingleGPUAllSampleGraphOp::backward(NtsVar& g) {
  sampCSC* sg = subgraphs->sampled_sgs[layer];
  NtsVar go = g.contiguous();
  const int64_t F = go.size(1);
  TORCH_CHECK(go.size(0) == (int64_t)sg->v_size, "output grad rows != v_size");
  if (sg->has_csr) {
    NtsVar gi = torch::empty({(int64_t)sg->src_size, F}, f32_opts(cuda_stream->device()));
    if (sg->post_mask_bits)  // the same, the mask read as bits
      hip_check(nts_hip_spmm_csr_bwd_postmask_bits(
                    cuda_stream->ctx(), sg->dev_r_o(), sg->dev_c_i(), sg->dev_e_w_b(), nullptr,
                    sg->src_size, go.data_ptr<float>(), (uint64_t)F, sg->post_mask_bits,
                    sg->post_mask_scale, (uint32_t)F, gi.data_ptr<float>(), (uint64_t)F),
                "nts_hip_spmm_csr_bwd_postmask_bits");
    else if (sg->post_mask)  // the transform-first bottom layer's activation backward fused
      hip_check(nts_hip_spmm_csr_bwd_postmask(cuda_stream->ctx(), sg->dev_r_o(), sg->dev_c_i(),
                                              sg->dev_e_w_b(), nullptr, sg->src_size,
                                              go.data_ptr<float>(), (uint64_t)F, sg->post_mask,
                                              sg->post_mask_ld, sg->post_mask_scale, (uint32_t)F,
                                              gi.data_ptr<float>(), (uint64_t)F),
                "nts_hip_spmm_csr_bwd_postmask");
    else
      hip_check(nts_hip_spmm_csr_bwd(cuda_stream->ctx(), sg->dev_r_o(), sg->dev_c_i(),
                                     sg->dev_e_w_b(), nullptr, sg->src_size, go.data_ptr<float>(),
                                     (uint64_t)F, (uint32_t)F, gi.data_ptr<float>(), (uint64_t)F),
                "nts_hip_spmm_csr_bwd");
    return gi;
  }
  TORCH_CHECK(!sg->post_mask, "a fused activation backward needs the CSR backward");
  NtsVar gi = torch::zeros({(int64_t)sg->src_size, F}, f32_opts(cuda_stream->device()));
  hip_check(nts_hip_spmm_csc_bwd_atomic(cuda_stream->ctx(), sg->dev_c_o(), sg->dev_r_i(),
                                        sg->dev_e_w_f(), nullptr, sg->v_size, go.data_ptr<float>(),
                                        (uint64_t)F, (uint32_t)F, gi.data_ptr<float>(), (uint64_t)F),
            "nts_hip_spmm_csc_bwd_atomic");
  return gi;
}

NtsVar SingleGPUSampleGraphOp::backward(NtsVar& g) {
  TORCH_CHECK(subgraphs->sampled_sgs[layer]->has_csr,
              "SingleGPUSampleGraphOp needs the CSR transpose");
  return SingleGPUAllSampleGraphOp::backward(g);
}

}  // namespace op

// ---------------------------------------------------------------------------
// A persistent fp32 scalar 1 per device: the seed gradient of a scalar loss.
// Kernels that precompute their backward for d loss = 1 recognise it by
// identity (HipLinearXentFn); no fill kernel per step.
const NtsVar& unit_scalar(const torch::Device& dev) {
  static std::mutex mu;
  static std::map<std::string, NtsVar> units;
  std::lock_guard<std::mutex> lk(mu);
  NtsVar& u = units[dev.str()];
  if (!u.defined()) u = torch::ones({}, torch::TensorOptions().dtype(torch::kFloat32).device(dev));
  return u;
}

namespace ctx {

NtsContext::NtsContext() {}
NtsContext::~NtsContext() { reset(); }

void NtsContext::push_graph_op(op::ntsGraphOp* op, NtsVar& in, NtsVar& out) {
  if (!training) {  // eval: ops are not recorded (and not leaked, unlike the reference)
    delete op;
    return;
  }
  ops_.push_back(Entry{GRAPHOP, op, in, out, NtsVar(), in.data_ptr(), out.data_ptr()});
  ++count;
}

NtsVar NtsContext::runVertexForward(const std::function<NtsVar(NtsVar&, NtsVar&)>& fn,
                                    NtsVar& nbr_input, NtsVar& vtx_input) {
  NtsVar out = fn(nbr_input, vtx_input);
  if (training) appendNNOp(nbr_input, out);
  return out;
}

NtsVar NtsContext::runVertexForward(const std::function<NtsVar(NtsVar&)>& fn, NtsVar& nbr_input) {
  NtsVar out = fn(nbr_input);
  if (training) appendNNOp(nbr_input, out);
  return out;
}

// core/ntsContext.hpp:384-405: consecutive NN ops are chained (libtorch
// handles their backward), so only the segment's last output is kept.
void NtsContext::appendNNOp(NtsVar& input_t, NtsVar& output_t) {
  TORCH_CHECK(training, "appendNNOp in eval mode");
  if (count > 0 && ops_.back().type == NNOP) {
    ops_.back().output = output_t;
    ops_.back().out_id = output_t.data_ptr();
  } else {
    ops_.push_back(Entry{NNOP, nullptr, input_t, output_t, NtsVar(), input_t.data_ptr(),
                         output_t.data_ptr()});
    ++count;
  }
}

void NtsContext::pop_one_op() {
  delete ops_.back().op;
  ops_.pop_back();
  --count;
}

// core/ntsContext.hpp:436-508: loss backward through libtorch, then walk the
// stack alternating graph-op backward and libtorch backward; the bottom graph
// op's backward is skipped.
void NtsContext::self_backward(bool retain_graph) {
  TORCH_CHECK(training && count > 0, "self_backward outside training");
  Entry& top = ops_.back();
  const bool unit = top.output.dim() == 0 && top.output.scalar_type() == torch::kFloat32;
  top.output.backward(unit ? unit_scalar(top.output.device()) : torch::ones_like(top.output), {},
                      retain_graph);
  if (count >= 2) ops_[count - 2].output_grad = top.input.grad();
  pop_one_op();
  while (count > 1 || (count == 1 && ops_.back().type == NNOP)) {
    Entry& e = ops_.back();
    const int t = count - 1;
    if (e.type == GRAPHOP) {
      if (!e.output_grad.defined()) e.output_grad = e.output.grad();
      int pre = t;
      for (; pre >= 0; --pre)
        if (ops_[pre].out_id == e.in_id) break;
      TORCH_CHECK(pre >= 0, "graph op input has no producer on the stack");
      ops_[pre].output_grad = e.op->backward(e.output_grad);
      pop_one_op();
    } else {
      if (!e.output_grad.defined()) e.output_grad = e.output.grad();
      if (e.output_grad.defined() && e.output_grad.dim() > 1)
        e.output.backward(e.output_grad, {}, retain_graph);
      pop_one_op();
    }
  }
  reset();
}

void NtsContext::reset() {
  while (!ops_.empty()) pop_one_op();
  count = 0;
}

}  // namespace ctx

// ---------------------------------------------------------------------------
// Row-major with unit column stride (rows may be padded); copies otherwise.
NtsVar row_major(const NtsVar& x) {
  return (x.dim() == 2 && x.stride(1) == 1 && x.stride(0) >= x.size(1)) ? x : x.contiguous();
}

// [rows, F] fp32 whose rows start on 128-byte boundaries for wide F (the
// bottom aggregation output: aligned row writes, 16-byte A loads in the
// GEMMs that consume it).
NtsVar row_padded_empty(int64_t rows, int64_t F, int device) {
  // (F >= 64: whole 32-float k-steps for k_x3_tn's row reads, C3 / C4's F = 100)
  const int64_t ld = F >= 64 ? (F + 31) / 32 * 32 : F;
  if (ld == F) return torch::empty({rows, F}, f32_opts(device));
  return torch::empty_strided({rows, F}, {ld, 1}, f32_opts(device));
}

namespace {
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

struct HipLinearFn : public torch::autograd::Function<HipLinearFn> {
  static NtsVar forward(AutogradContext* ctx, NtsVar x, NtsVar W, int64_t cs_ptr) {
    auto* cs = reinterpret_cast<NtsStream*>(cs_ptr);
    NtsVar xc = row_major(x), Wc = W.contiguous();
    const int64_t M = xc.size(0), K = xc.size(1), N = Wc.size(1);
    TORCH_CHECK(Wc.size(0) == K, "hip_linear: shape mismatch");
    NtsVar Z = torch::empty({M, N}, xc.options());
    hip_check(nts_hip_gemm_f32(cs->ctx(), 0, (int)M, (int)N, (int)K, xc.data_ptr<float>(),
                               (uint64_t)xc.stride(0), Wc.data_ptr<float>(), (uint64_t)N,
                               Z.data_ptr<float>(), (uint64_t)N),
              "nts_hip_gemm_f32(nn)");
    ctx->save_for_backward({xc, Wc});
    ctx->saved_data["cs"] = cs_ptr;
    return Z;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto saved = ctx->get_saved_variables();
    NtsVar x = saved[0], W = saved[1];
    auto* cs = reinterpret_cast<NtsStream*>(ctx->saved_data["cs"].toInt());
    NtsVar g = grads[0].contiguous();
    const int64_t M = x.size(0), K = x.size(1), N = W.size(1);
    NtsVar dx, dW;
    if (ctx->needs_input_grad(1)) {
      dW = torch::empty({K, N}, W.options());
      hip_check(nts_hip_gemm_f32(cs->ctx(), 1, (int)K, (int)N, (int)M, x.data_ptr<float>(),
                                 (uint64_t)x.stride(0), g.data_ptr<float>(), (uint64_t)N,
                                 dW.data_ptr<float>(), (uint64_t)N),
                "nts_hip_gemm_f32(tn)");
    }
    if (ctx->needs_input_grad(0)) dx = g.matmul(W.t());
    return {dx, dW, NtsVar()};
  }
};
// dropout(relu(x W)) with the activation in the GEMM epilogue and its
// backward in the weight-gradient GEMM's operand load (nts_hip.h).
struct HipLinearActFn : public torch::autograd::Function<HipLinearActFn> {
  static NtsVar forward(AutogradContext* ctx, NtsVar x, NtsVar W, double p, int64_t seed,
                        int64_t offset, int64_t cs_ptr, bool pair_split) {
    auto* cs = reinterpret_cast<NtsStream*>(cs_ptr);
    NtsVar xc = row_major(x), Wc = W.contiguous();
    const int64_t M = xc.size(0), K = xc.size(1), N = Wc.size(1);
    TORCH_CHECK(Wc.size(0) == K, "hip_linear_act: shape mismatch");
    NtsVar X = torch::empty({M, N}, xc.options());
    // a narrow input (K <= 128, N 128 or 256: the products / papers-shaped
    // aggregate-first bottom layer) on the in-kernel f16 pair split
    // (nts_hip_gemm_h2d_act) when the config allows pair-split
    // arithmetic (GCNConfig::pair_table > 0); otherwise the GEMM mode's kernel
    if (pair_split && K <= 128 && K % 4 == 0 && (N == 128 || N == 256) && xc.stride(0) % 4 == 0 &&
        (uintptr_t)xc.data_ptr<float>() % 16 == 0)
      hip_check(nts_hip_gemm_h2d_act(cs->ctx(), 1, (int)M, (int)N, (int)K, xc.data_ptr<float>(),
                                     (uint64_t)xc.stride(0), Wc.data_ptr<float>(), (uint64_t)N,
                                     X.data_ptr<float>(), (uint64_t)N, (float)p, (uint64_t)seed,
                                     (uint64_t)offset, nullptr, 0, nullptr),
                "nts_hip_gemm_h2d_act");
    else
      hip_check(nts_hip_gemm_relu_dropout_f32(cs->ctx(), (int)M, (int)N, (int)K,
                                              xc.data_ptr<float>(), (uint64_t)xc.stride(0),
                                              Wc.data_ptr<float>(), (uint64_t)N, X.data_ptr<float>(),
                                              (uint64_t)N, (float)p, (uint64_t)seed,
                                              (uint64_t)offset),
                "nts_hip_gemm_relu_dropout_f32");
    ctx->save_for_backward({xc, Wc, X});
    ctx->saved_data["cs"] = cs_ptr;
    ctx->saved_data["scale"] = p < 1.0 ? (double)(1.0f / (1.0f - (float)p)) : 0.0;
    return X;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto saved = ctx->get_saved_variables();
    NtsVar x = saved[0], W = saved[1], X = saved[2];
    auto* cs = reinterpret_cast<NtsStream*>(ctx->saved_data["cs"].toInt());
    const float scale = (float)ctx->saved_data["scale"].toDouble();
    NtsVar g = grads[0].contiguous();
    const int64_t M = x.size(0), K = x.size(1), N = W.size(1);
    NtsVar dx, dW;
    if (ctx->needs_input_grad(1)) {
      dW = torch::empty({K, N}, W.options());
      hip_check(nts_hip_gemm_tn_masked_f32(cs->ctx(), (int)K, (int)N, (int)M, x.data_ptr<float>(),
                                           (uint64_t)x.stride(0), g.data_ptr<float>(), (uint64_t)N,
                                           X.data_ptr<float>(), (uint64_t)N, scale,
                                           dW.data_ptr<float>(), (uint64_t)N),
                "nts_hip_gemm_tn_masked_f32");
    }
    if (ctx->needs_input_grad(0)) {
      // dx = (g ⊙ [X > 0] / (1-p)) W^T: the activation backward
      // (nts_hip_act_backward) and the layer GEMM, not three torch
      // elementwise kernels and a library GEMM
      NtsVar dZ = torch::empty({M, N}, g.options());
      hip_check(nts_hip_act_backward(cs->ctx(), (uint32_t)M, (uint32_t)N, g.data_ptr<float>(),
                                     (uint64_t)N, X.data_ptr<float>(), (uint64_t)N, scale,
                                     dZ.data_ptr<float>(), (uint64_t)N),
                "nts_hip_act_backward");
      NtsVar Wt = W.t().contiguous();
      dx = torch::empty({M, K}, g.options());
      hip_check(nts_hip_gemm_f32(cs->ctx(), 0, (int)M, (int)K, (int)N, dZ.data_ptr<float>(),
                                 (uint64_t)N, Wt.data_ptr<float>(), (uint64_t)K,
                                 dx.data_ptr<float>(), (uint64_t)K),
                "nts_hip_gemm_f32(dx)");
    }
    return {dx, dW, NtsVar(), NtsVar(), NtsVar(), NtsVar(), NtsVar()};
  }
};

// Transform-first bottom layer (nts_hip.h):
//   H = X[source] W      (row-gathered MFMA GEMM: load_feature_gpu fused away)
//   X1 = dropout(relu(A H))  (the graph op over F_out-wide rows, activation in
//                             the epilogue with the GEMM epilogue's mask keys)
// backward: dH = A^T (dX1 ⊙ [X1 > 0] / (1-p)) over the CSR, dW = X[source]^T dH.
// Recorded as one NN op whose input is the feature table (the bottom graph
// op has no backward, core/ntsContext.hpp:443-444).
std::function<void()> g_after_fwd_gemm, g_before_bwd_gemm;  // set_bottom_gemm_hooks

struct HipBottomTFFn : public torch::autograd::Function<HipBottomTFFn> {
  static NtsVar forward(AutogradContext* ctx, NtsVar table, NtsVar W, int64_t sg_ptr,
                        int64_t cs_ptr, double p, int64_t seed, int64_t offset, int64_t prof_ptr,
                        int64_t h_out, int64_t pairs_ptr) {
    const auto* pairs = reinterpret_cast<const PairTable*>(pairs_ptr);
    auto* cs = reinterpret_cast<NtsStream*>(cs_ptr);
    auto* sg = reinterpret_cast<sampCSC*>(sg_ptr);
    auto* prof = reinterpret_cast<KernelProfiler*>(prof_ptr);
    NtsVar Wc = W.contiguous();
    const int64_t F = table.size(1), N = Wc.size(1);
    const int64_t s = sg->src_size, v = sg->v_size, e = sg->e_size;
    TORCH_CHECK(Wc.size(0) == F && table.stride(1) == 1, "transform-first: shape mismatch");
    const int dev = cs->device();
    hipStream_t st = (hipStream_t)cs->stream();
    NtsVar H = h_out ? NtsVar() : torch::empty({std::max<int64_t>(s, 1), N}, f32_opts(dev));
    float* hp = h_out ? reinterpret_cast<float*>(h_out) : H.data_ptr<float>();
    if (prof) prof->begin(KernelProfiler::GATHER_GEMM, st);
    if (pairs && pairs->Q.defined())
      hip_check(nts_hip_gemm_h2p_gather(cs->ctx(), 0, (int)s, (int)N, (int)(pairs->Q.size(1) / 2),
                                        reinterpret_cast<const uint16_t*>(pairs->Q.data_ptr<int16_t>()),
                                        (uint64_t)pairs->Q.stride(0), pairs->rs.data_ptr<float>(),
                                        sg->dev_src(), Wc.data_ptr<float>(), (uint64_t)N, (int)F, hp,
                                        (uint64_t)N, 0.f, 0, 0),
                "nts_hip_gemm_h2p_gather");
    else if (pairs && pairs->P.defined())
      hip_check(nts_hip_gemm_h2_gather(cs->ctx(), 0, (int)s, (int)N, (int)pairs->P.size(1),
                                       reinterpret_cast<const uint32_t*>(pairs->P.data_ptr<int32_t>()),
                                       (uint64_t)pairs->P.stride(0), pairs->rs.data_ptr<float>(),
                                       sg->dev_src(), Wc.data_ptr<float>(), (uint64_t)N, (int)F, hp,
                                       (uint64_t)N, 0.f, 0, 0),
                "nts_hip_gemm_h2_gather");
    else
      hip_check(nts_hip_gemm_gather_f32(cs->ctx(), (int)s, (int)N, (int)F, table.data_ptr<float>(),
                                        (uint64_t)table.stride(0), sg->dev_src(),
                                        Wc.data_ptr<float>(), (uint64_t)N, hp, (uint64_t)N),
                "nts_hip_gemm_gather_f32");
    if (prof) prof->end(KernelProfiler::GATHER_GEMM, st, 2.0 * (double)s * F * N);
    if (g_after_fwd_gemm) g_after_fwd_gemm();
    NtsVar X1 = torch::empty({v, N}, f32_opts(dev));
    if (prof) prof->begin(KernelProfiler::BOTTOM_AGG, st);
    // the keep mask [X1 > 0] also as bits (16 B a 128-float row), which the
    // graph op above reads in its fused activation backward instead of X1
    const uint32_t words = nts_hip_act_bits_words((uint32_t)N);
    if (words) {
      const int64_t need = std::max<int64_t>((int64_t)sg->v_cap, 1) * words;
      if (!sg->act_bits.defined() || sg->act_bits.numel() < need)
        sg->act_bits = torch::empty({need}, torch::TensorOptions().dtype(torch::kInt32).device(
                                                torch::kCUDA, dev));
      hip_check(nts_hip_spmm_csc_fwd_act_bits(
                    cs->ctx(), sg->dev_c_o(), sg->dev_r_i(), sg->dev_e_w_f(), nullptr, (uint32_t)v,
                    hp, (uint64_t)N, (uint32_t)N, X1.data_ptr<float>(), (uint64_t)N, (float)p,
                    (uint64_t)seed, (uint64_t)offset,
                    reinterpret_cast<uint32_t*>(sg->act_bits.data_ptr<int32_t>())),
                "nts_hip_spmm_csc_fwd_act_bits");
    } else {
      hip_check(nts_hip_spmm_csc_fwd_act(cs->ctx(), sg->dev_c_o(), sg->dev_r_i(), sg->dev_e_w_f(),
                                         nullptr, (uint32_t)v, hp, (uint64_t)N, (uint32_t)N,
                                         X1.data_ptr<float>(), (uint64_t)N, (float)p,
                                         (uint64_t)seed, (uint64_t)offset),
                "nts_hip_spmm_csc_fwd_act");
    }
    // compulsory bytes: each H row once, index + weight per edge, offsets, output
    if (prof)
      prof->end(KernelProfiler::BOTTOM_AGG, st,
                4.0 * N * s + 8.0 * e + 4.0 * (v + 1) + 4.0 * N * v);
    ctx->save_for_backward({table, Wc, X1});
    ctx->saved_data["sg"] = sg_ptr;
    ctx->saved_data["cs"] = cs_ptr;
    ctx->saved_data["prof"] = prof_ptr;
    ctx->saved_data["pairs"] = pairs_ptr;
    ctx->saved_data["scale"] = p < 1.0 ? (double)(1.0f / (1.0f - (float)p)) : 0.0;
    return X1;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto saved = ctx->get_saved_variables();
    NtsVar table = saved[0], W = saved[1], X1 = saved[2];
    auto* cs = reinterpret_cast<NtsStream*>(ctx->saved_data["cs"].toInt());
    auto* sg = reinterpret_cast<sampCSC*>(ctx->saved_data["sg"].toInt());
    auto* prof = reinterpret_cast<KernelProfiler*>(ctx->saved_data["prof"].toInt());
    TORCH_CHECK(sg->has_csr, "transform-first backward needs the bottom layer's CSR");
    NtsVar g = grads[0].contiguous();
    const int64_t F = table.size(1), N = W.size(1), s = sg->src_size, v = sg->v_size;
    const int dev = cs->device();
    hipStream_t st = (hipStream_t)cs->stream();
    NtsVar dH = torch::empty({std::max<int64_t>(s, 1), N}, f32_opts(dev));
    const float scale = (float)ctx->saved_data["scale"].toDouble();
    const auto* pairs = reinterpret_cast<const PairTable*>(ctx->saved_data["pairs"].toInt());
    const PairTable* pairs_q = pairs && pairs->tn && pairs->Q.defined() ? pairs : nullptr;
    NtsVar colmax;  // dH's per-part column maxima (int32 bits), when the gather produced them
    uint32_t rpp = 0;
    // dZ = dX1 ⊙ mask once per dst row, then the plain CSR gather (measured
    // faster than applying the mask to every gathered row:
    // nts_hip_spmm_csr_bwd_masked reads two rows per edge); the A/B build
    // -DNTS_TF_MASKED_BWD selects the fused form
#ifdef NTS_TF_MASKED_BWD
    constexpr bool fused_mask = true;
#else
    constexpr bool fused_mask = false;
#endif
    if (fused_mask && !sg->grad_premasked) {
      if (prof) prof->begin(KernelProfiler::BOTTOM_BWD, st);
      hip_check(nts_hip_spmm_csr_bwd_masked(cs->ctx(), sg->dev_r_o(), sg->dev_c_i(),
                                            sg->dev_e_w_b(), nullptr, (uint32_t)s,
                                            g.data_ptr<float>(), (uint64_t)N, X1.data_ptr<float>(),
                                            (uint64_t)N, scale, (uint32_t)N, dH.data_ptr<float>(),
                                            (uint64_t)N),
                "nts_hip_spmm_csr_bwd_masked");
      if (prof)
        prof->end(KernelProfiler::BOTTOM_BWD, st,
                  8.0 * N * v + 8.0 * sg->e_size + 4.0 * (s + 1) + 4.0 * N * s);
    } else {
      // the graph op above applied the activation backward already (post_mask)
      NtsVar dZ = sg->grad_premasked ? g : torch::empty({std::max<int64_t>(v, 1), N}, f32_opts(dev));
      if (!sg->grad_premasked)
        hip_check(nts_hip_act_backward(cs->ctx(), (uint32_t)v, (uint32_t)N, g.data_ptr<float>(),
                                       (uint64_t)N, X1.data_ptr<float>(), (uint64_t)N, scale,
                                       dZ.data_ptr<float>(), (uint64_t)N),
                  "nts_hip_act_backward");
      if (prof) prof->begin(KernelProfiler::BOTTOM_BWD, st);
      // the planar-table TN GEMM takes dH's column maxima per part of rows
      // from this gather's epilogue (one read of dH instead of two); the A/B
      // build -DNTS_TN_CHUNK_SCALES keeps its own per-chunk pre-pass
#ifdef NTS_TN_CHUNK_SCALES
      constexpr bool chunk_scales = true;
#else
      constexpr bool chunk_scales = false;
#endif
      // (its float4 rows need 16-byte aligned dZ / dH rows: else the plain gather)
      const bool cm_rows = N <= 512 && N % 4 == 0 && (uintptr_t)dZ.data_ptr<float>() % 16 == 0 &&
                           (uintptr_t)dH.data_ptr<float>() % 16 == 0;
      if (pairs_q && !chunk_scales && cm_rows) {
        rpp = nts_hip_csr_bwd_colmax_rows_per_part((uint32_t)N);
        const int64_t nparts = (std::max<int64_t>(s, 1) + rpp - 1) / rpp;
        colmax = torch::empty({nparts, N}, torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, dev));
        hip_check(nts_hip_spmm_csr_bwd_colmax(
                      cs->ctx(), sg->dev_r_o(), sg->dev_c_i(), sg->dev_e_w_b(), nullptr, (uint32_t)s,
                      dZ.data_ptr<float>(), (uint64_t)N, (uint32_t)N, dH.data_ptr<float>(), (uint64_t)N,
                      reinterpret_cast<uint32_t*>(colmax.data_ptr<int32_t>()),
                      pairs_q->rs.data_ptr<float>(), sg->dev_src()),
                  "nts_hip_spmm_csr_bwd_colmax");
      } else {
        hip_check(nts_hip_spmm_csr_bwd(cs->ctx(), sg->dev_r_o(), sg->dev_c_i(), sg->dev_e_w_b(),
                                       nullptr, (uint32_t)s, dZ.data_ptr<float>(), (uint64_t)N,
                                       (uint32_t)N, dH.data_ptr<float>(), (uint64_t)N),
                  "nts_hip_spmm_csr_bwd");
      }
      if (prof)
        prof->end(KernelProfiler::BOTTOM_BWD, st,
                  4.0 * N * v + 8.0 * sg->e_size + 4.0 * (s + 1) + 4.0 * N * s);
    }
    NtsVar dW = torch::empty({F, N}, W.options());
    if (g_before_bwd_gemm) g_before_bwd_gemm();
    if (prof) prof->begin(KernelProfiler::GATHER_GEMM_TN, st);
    if (pairs_q && colmax.defined())
      hip_check(nts_hip_gemm_h2p_tn_gather_cm(cs->ctx(), (int)F, (int)N, (int)s,
                                              reinterpret_cast<const uint16_t*>(pairs->Q.data_ptr<int16_t>()),
                                              (uint64_t)pairs->Q.stride(0), (int)(pairs->Q.size(1) / 2),
                                              pairs->rs.data_ptr<float>(), sg->dev_src(),
                                              dH.data_ptr<float>(), (uint64_t)N, dW.data_ptr<float>(),
                                              (uint64_t)N,
                                              reinterpret_cast<const uint32_t*>(colmax.data_ptr<int32_t>()),
                                              rpp),
                "nts_hip_gemm_h2p_tn_gather_cm");
    else if (pairs_q)
      hip_check(nts_hip_gemm_h2p_tn_gather(cs->ctx(), (int)F, (int)N, (int)s,
                                           reinterpret_cast<const uint16_t*>(pairs->Q.data_ptr<int16_t>()),
                                           (uint64_t)pairs->Q.stride(0), (int)(pairs->Q.size(1) / 2),
                                           pairs->rs.data_ptr<float>(), sg->dev_src(),
                                           dH.data_ptr<float>(), (uint64_t)N, dW.data_ptr<float>(),
                                           (uint64_t)N),
                "nts_hip_gemm_h2p_tn_gather");
    else if (pairs && pairs->tn && pairs->P.defined())
      hip_check(nts_hip_gemm_h2_tn_gather(cs->ctx(), (int)F, (int)N, (int)s,
                                          reinterpret_cast<const uint32_t*>(pairs->P.data_ptr<int32_t>()),
                                          (uint64_t)pairs->P.stride(0), pairs->rs.data_ptr<float>(),
                                          sg->dev_src(), dH.data_ptr<float>(), (uint64_t)N, nullptr, 0,
                                          1.f, dW.data_ptr<float>(), (uint64_t)N),
                "nts_hip_gemm_h2_tn_gather");
    else
      hip_check(nts_hip_gemm_tn_gather_f32(cs->ctx(), (int)F, (int)N, (int)s, table.data_ptr<float>(),
                                           (uint64_t)table.stride(0), sg->dev_src(),
                                           dH.data_ptr<float>(), (uint64_t)N, dW.data_ptr<float>(),
                                           (uint64_t)N),
                "nts_hip_gemm_tn_gather_f32");
    if (prof) prof->end(KernelProfiler::GATHER_GEMM_TN, st, 2.0 * (double)s * F * N);
    return {NtsVar(), dW,       NtsVar(), NtsVar(), NtsVar(), NtsVar(),
            NtsVar(), NtsVar(), NtsVar(), NtsVar()};
  }
};
// Output layer + loss in fused kernels (nts_hip.h).  Under grad mode the
// forward runs the training kernel: loss, dY and dW for d loss = 1 in one pass
// over Y; the backward returns them when the upstream gradient is the unit
// seed of self_backward (exactly 1), and otherwise runs the backward kernel.
struct HipLinearXentFn : public torch::autograd::Function<HipLinearXentFn> {
  static NtsVar forward(AutogradContext* ctx, NtsVar y, NtsVar W, NtsVar target, int64_t cs_ptr,
                        bool train, int64_t correct_ptr) {
    auto* correct = reinterpret_cast<uint32_t*>(correct_ptr);
    auto* cs = reinterpret_cast<NtsStream*>(cs_ptr);
    NtsVar yc = row_major(y), Wc = W.contiguous(), tc = target.contiguous();
    const int64_t n = yc.size(0), K = yc.size(1), C = Wc.size(1);
    TORCH_CHECK(Wc.size(0) == K && tc.numel() == n && tc.scalar_type() == torch::kInt64,
                "hip_linear_xent: shape mismatch");
    NtsVar loss = torch::empty({}, yc.options());
    if (train) {
      NtsVar dY = torch::empty({n, K}, yc.options());
      NtsVar dW = torch::empty({K, C}, Wc.options());
      hip_check(nts_hip_linear_xent_train(cs->ctx(), yc.data_ptr<float>(), (uint64_t)yc.stride(0),
                                          (int)n, (int)K, Wc.data_ptr<float>(), (int)C,
                                          tc.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                          dY.data_ptr<float>(), dW.data_ptr<float>(), correct),
                "nts_hip_linear_xent_train");
      ctx->saved_data["dY"] = dY;
      ctx->saved_data["dW"] = dW;
    } else {
      hip_check(nts_hip_linear_xent_fwd(cs->ctx(), yc.data_ptr<float>(), (uint64_t)yc.stride(0),
                                        (int)n, (int)K, Wc.data_ptr<float>(), (int)C,
                                        tc.data_ptr<int64_t>(), loss.data_ptr<float>(), correct),
                "nts_hip_linear_xent_fwd");
    }
    ctx->save_for_backward({yc, Wc, tc});
    ctx->saved_data["cs"] = cs_ptr;
    return loss;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto saved = ctx->get_saved_variables();
    NtsVar y = saved[0], W = saved[1], t = saved[2];
    auto* cs = reinterpret_cast<NtsStream*>(ctx->saved_data["cs"].toInt());
    NtsVar g = grads[0];
    NtsVar dY, dW;
    if (ctx->saved_data.count("dY") &&
        g.data_ptr() == unit_scalar(g.device()).data_ptr()) {  // d loss == 1: precomputed
      dY = ctx->saved_data["dY"].toTensor();
      dW = ctx->saved_data["dW"].toTensor();
    } else {
      g = g.contiguous();
      const int64_t n = y.size(0), K = y.size(1), C = W.size(1);
      dY = torch::empty({n, K}, y.options());
      dW = torch::empty({K, C}, W.options());
      hip_check(nts_hip_linear_xent_bwd(cs->ctx(), y.data_ptr<float>(), (uint64_t)y.stride(0),
                                        (int)n, (int)K, W.data_ptr<float>(), (int)C,
                                        t.data_ptr<int64_t>(), g.data_ptr<float>(),
                                        dY.data_ptr<float>(), dW.data_ptr<float>()),
                "nts_hip_linear_xent_bwd");
    }
    ctx->saved_data.erase("dY");
    ctx->saved_data.erase("dW");
    return {ctx->needs_input_grad(0) ? dY : NtsVar(), dW, NtsVar(), NtsVar(), NtsVar(), NtsVar()};
  }
};
}  // namespace

NtsVar hip_linear_act(const NtsVar& x, const NtsVar& W, double p, uint64_t seed, uint64_t offset,
                      NtsStream* cs, bool pair_split) {
  return HipLinearActFn::apply(x, W, p, (int64_t)seed, (int64_t)offset,
                               reinterpret_cast<int64_t>(cs), pair_split);
}

// dropout(relu(x)) on its own (nts_hip_relu_dropout_f32, the GEMM epilogue's
// keep bits); backward dx = dy ⊙ [y > 0] / (1-p) (nts_hip_act_backward)
struct HipActFn : public torch::autograd::Function<HipActFn> {
  static NtsVar forward(AutogradContext* ctx, NtsVar x, double p, int64_t seed, int64_t offset,
                        int64_t cs_ptr) {
    auto* cs = reinterpret_cast<NtsStream*>(cs_ptr);
    NtsVar xc = row_major(x);
    NtsVar y = torch::empty({xc.size(0), xc.size(1)}, xc.options());
    hip_check(nts_hip_relu_dropout_f32(cs->ctx(), (uint32_t)xc.size(0), (uint32_t)xc.size(1),
                                       xc.data_ptr<float>(), (uint64_t)xc.stride(0), (float)p,
                                       (uint64_t)seed, (uint64_t)offset, y.data_ptr<float>(),
                                       (uint64_t)y.size(1)),
              "nts_hip_relu_dropout_f32");
    ctx->save_for_backward({y});
    ctx->saved_data["cs"] = cs_ptr;
    ctx->saved_data["scale"] = p < 1.0 ? (double)(1.0f / (1.0f - (float)p)) : 0.0;
    return y;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    NtsVar y = ctx->get_saved_variables()[0];
    auto* cs = reinterpret_cast<NtsStream*>(ctx->saved_data["cs"].toInt());
    NtsVar g = grads[0].contiguous();
    NtsVar dx = torch::empty_like(y);
    hip_check(nts_hip_act_backward(cs->ctx(), (uint32_t)y.size(0), (uint32_t)y.size(1),
                                   g.data_ptr<float>(), (uint64_t)g.size(1), y.data_ptr<float>(),
                                   (uint64_t)y.size(1),
                                   (float)ctx->saved_data["scale"].toDouble(),
                                   dx.data_ptr<float>(), (uint64_t)dx.size(1)),
              "nts_hip_act_backward");
    return {dx, NtsVar(), NtsVar(), NtsVar(), NtsVar()};
  }
};

NtsVar hip_relu_dropout(const NtsVar& x, double p, uint64_t seed, uint64_t offset, NtsStream* cs) {
  return HipActFn::apply(x, p, (int64_t)seed, (int64_t)offset, reinterpret_cast<int64_t>(cs));
}

void set_bottom_gemm_hooks(std::function<void()> after_fwd_gemm,
                           std::function<void()> before_bwd_gemm) {
  g_after_fwd_gemm = std::move(after_fwd_gemm);
  g_before_bwd_gemm = std::move(before_bwd_gemm);
}

NtsVar hip_bottom_transform(const NtsVar& table, const NtsVar& W, sampCSC* sg, double p,
                            uint64_t seed, uint64_t offset, NtsStream* cs, KernelProfiler* prof,
                            float* h_out, const PairTable* pairs) {
  return HipBottomTFFn::apply(table, W, reinterpret_cast<int64_t>(sg),
                              reinterpret_cast<int64_t>(cs), p, (int64_t)seed, (int64_t)offset,
                              reinterpret_cast<int64_t>(prof), reinterpret_cast<int64_t>(h_out),
                              reinterpret_cast<int64_t>(pairs));
}

// ---------------------------------------------------------------------------
KernelProfiler::~KernelProfiler() {
  for (auto& e : pool_) {
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
}
const char* KernelProfiler::name(int id) {
  static const char* n[kCount] = {"bottom_aggregation", "gather_gemm", "gather_gemm_tn",
                                  "bottom_backward", "gat_forward"};
  return n[id];
}
void KernelProfiler::begin(Id id, hipStream_t st) {
  if (open_[id] >= 0) return;  // nested begin: keep the outer interval
  if (!active(id)) return;     // another class is timed this step
  if (used_ >= 4096) resolve();
  if (used_ == pool_.size()) {
    Slot sl;
    // timing-only events: no system-scope fence (an L2 writeback + invalidate
    // per record, ~5 us of gap each in the training stream's trace)
    hip_rt(hipEventCreateWithFlags(&sl.a, hipEventDisableSystemFence), "hipEventCreate");
    hip_rt(hipEventCreateWithFlags(&sl.b, hipEventDisableSystemFence), "hipEventCreate");
    pool_.push_back(sl);
  }
  Slot& sl = pool_[used_];
  sl.id = id;
  sl.units = 0;
  hip_rt(hipEventRecord(sl.a, st), "hipEventRecord");
  open_[id] = (int)used_++;
}
void KernelProfiler::end(Id id, hipStream_t st, double units) {
  const int k = open_[id];
  if (k < 0) return;
  hip_rt(hipEventRecord(pool_[k].b, st), "hipEventRecord");
  pool_[k].units = units;
  open_[id] = -1;
}
void KernelProfiler::resolve() {
  for (size_t i = 0; i < used_; ++i) {
    Slot& sl = pool_[i];
    if (open_[sl.id] == (int)i) continue;  // never closed (exception): drop it
    hip_rt(hipEventSynchronize(sl.b), "hipEventSynchronize");
    float ms = 0;
    hip_rt(hipEventElapsedTime(&ms, sl.a, sl.b), "hipEventElapsedTime");
    stat[sl.id].ms += ms;
    stat[sl.id].units += sl.units;
    stat[sl.id].calls += 1;
  }
  used_ = 0;
  for (int& o : open_) o = -1;
}
void KernelProfiler::reset() {
  resolve();
  for (auto& x : stat) x = Stat();
}

// GAT layer on a merged src/dst sampled block (GAT_SAMPLE_ALL_GPU's chain,
// toolkits/GAT_SAMPLE_ALL_GPU.hpp:322-388): H = X W on the MFMA GEMM, then
// the fused attention/softmax/aggregation/relu kernel; the backward runs the
// two deterministic GAT backward passes and three GEMMs (dW = X^T dH,
// dW_att = H^T dS, dX = dH W^T).
struct HipGATLayerFn : public torch::autograd::Function<HipGATLayerFn> {
  static NtsVar forward(AutogradContext* ctx, NtsVar X, NtsVar W, NtsVar Watt, int64_t sg_ptr,
                        int64_t cs_ptr, int64_t prof_ptr) {
    auto* sg = reinterpret_cast<sampCSC*>(sg_ptr);
    auto* cs = reinterpret_cast<NtsStream*>(cs_ptr);
    auto* prof = reinterpret_cast<KernelProfiler*>(prof_ptr);
    TORCH_CHECK(sg->dst_local_id.defined() && sg->csr_edge_id.defined(),
                "GAT needs a merged src/dst layer with its CSR (set_merge_src_dst)");
    NtsVar Xc = row_major(X), Wc = W.contiguous(), Ac = Watt.contiguous();
    const int64_t s = sg->src_size, v = sg->v_size, e = sg->e_size;
    const int64_t Fin = Xc.size(1), F = Wc.size(1);
    TORCH_CHECK(Xc.size(0) == s && Wc.size(0) == Fin && Ac.numel() == 2 * F, "GAT layer shapes");
    const int dev = cs->device();
    NtsVar H = torch::empty({s, F}, f32_opts(dev));
    hip_check(nts_hip_gemm_f32(cs->ctx(), 0, (int)s, (int)F, (int)Fin, Xc.data_ptr<float>(),
                               (uint64_t)Xc.stride(0), Wc.data_ptr<float>(), (uint64_t)F,
                               H.data_ptr<float>(), (uint64_t)F),
              "nts_hip_gemm_f32(H)");
    NtsVar m = torch::empty({std::max<int64_t>(e, 1)}, f32_opts(dev));
    NtsVar a = torch::empty({std::max<int64_t>(e, 1)}, f32_opts(dev));
    NtsVar Y = torch::empty({v, F}, f32_opts(dev));
    hipStream_t st = (hipStream_t)cs->stream();
    if (prof) prof->begin(KernelProfiler::GAT_FWD, st);
    hip_check(nts_hip_gat_forward(cs->ctx(), sg->dev_c_o(), sg->dev_r_i(), sg->dev_dst_local_id(),
                                  (uint32_t)v, H.data_ptr<float>(), (uint64_t)F, (uint32_t)F,
                                  Ac.data_ptr<float>(), m.data_ptr<float>(), a.data_ptr<float>(),
                                  Y.data_ptr<float>(), (uint64_t)F),
              "nts_hip_gat_forward");
    // compulsory bytes: H rows once, offsets, row index + score + weight per
    // edge, dst local ids, W_att, output rows
    if (prof)
      prof->end(KernelProfiler::GAT_FWD, st,
                4.0 * F * s + 4.0 * (v + 1) + 12.0 * e + 4.0 * v + 8.0 * F + 4.0 * F * v);
    ctx->save_for_backward({Xc, Wc, Ac, H, Y, m, a});
    ctx->saved_data["sg"] = sg_ptr;
    ctx->saved_data["cs"] = cs_ptr;
    ctx->saved_data["x_grad"] = X.requires_grad();
    return Y;
  }
  static torch::autograd::variable_list backward(AutogradContext* ctx,
                                                 torch::autograd::variable_list grads) {
    auto v_ = ctx->get_saved_variables();
    NtsVar X = v_[0], W = v_[1], A = v_[2], H = v_[3], Y = v_[4], m = v_[5], a = v_[6];
    auto* sg = reinterpret_cast<sampCSC*>(ctx->saved_data["sg"].toInt());
    auto* cs = reinterpret_cast<NtsStream*>(ctx->saved_data["cs"].toInt());
    NtsVar GY = grads[0].contiguous();
    const int64_t s = H.size(0), F = H.size(1), Fin = X.size(1), v = Y.size(0);
    const int64_t e = sg->e_size;
    const int dev = cs->device();
    auto guard = cs->guard();
    NtsVar du = torch::empty({std::max<int64_t>(e, 1)}, f32_opts(dev));
    NtsVar ds2 = torch::empty({std::max<int64_t>(s, 1)}, f32_opts(dev));
    NtsVar dH = torch::empty({s, F}, f32_opts(dev));
    NtsVar dS = torch::empty({s, 2}, f32_opts(dev));
    NtsVar GM = torch::empty({std::max<int64_t>(v, 1), F}, f32_opts(dev));
    hip_check(nts_hip_gat_backward(cs->ctx(), sg->dev_c_o(), sg->dev_r_i(), sg->dev_dst_local_id(),
                                   (uint32_t)v, sg->dev_r_o(), sg->dev_c_i(),
                                   dptr<uint32_t>(sg->csr_edge_id), (uint32_t)s, H.data_ptr<float>(),
                                   (uint64_t)F, (uint32_t)F, A.data_ptr<float>(), a.data_ptr<float>(),
                                   m.data_ptr<float>(), Y.data_ptr<float>(), (uint64_t)F,
                                   GY.data_ptr<float>(), (uint64_t)F, du.data_ptr<float>(),
                                   ds2.data_ptr<float>(), GM.data_ptr<float>(), (uint64_t)F,
                                   dH.data_ptr<float>(), (uint64_t)F, dS.data_ptr<float>()),
              "nts_hip_gat_backward");
    NtsVar dW = torch::empty({Fin, F}, f32_opts(dev));
    hip_check(nts_hip_gemm_f32(cs->ctx(), 1, (int)Fin, (int)F, (int)s, X.data_ptr<float>(),
                               (uint64_t)X.stride(0), dH.data_ptr<float>(), (uint64_t)F,
                               dW.data_ptr<float>(), (uint64_t)F),
              "nts_hip_gemm_f32(dW)");
    NtsVar T = torch::empty({F, 2}, f32_opts(dev));
    hip_check(nts_hip_gemm_f32(cs->ctx(), 1, (int)F, 2, (int)s, H.data_ptr<float>(), (uint64_t)F,
                               dS.data_ptr<float>(), 2, T.data_ptr<float>(), 2),
              "nts_hip_gemm_f32(dW_att)");
    NtsVar dA = T.t().contiguous().view({2 * F, 1});  // [a1 | a2] as W_att's rows
    NtsVar dX;
    if (ctx->saved_data["x_grad"].toBool()) {
      NtsVar Wt = W.t().contiguous();
      dX = torch::empty({s, Fin}, f32_opts(dev));
      hip_check(nts_hip_gemm_f32(cs->ctx(), 0, (int)s, (int)Fin, (int)F, dH.data_ptr<float>(),
                                 (uint64_t)F, Wt.data_ptr<float>(), (uint64_t)Fin,
                                 dX.data_ptr<float>(), (uint64_t)Fin),
                "nts_hip_gemm_f32(dX)");
    }
    return {dX, dW, dA.view(A.sizes()), NtsVar(), NtsVar(), NtsVar()};
  }
};

NtsVar hip_gat_layer(const NtsVar& x, const NtsVar& W, const NtsVar& Watt, sampCSC* sg,
                     NtsStream* cs, KernelProfiler* prof) {
  return HipGATLayerFn::apply(x, W, Watt, reinterpret_cast<int64_t>(sg),
                              reinterpret_cast<int64_t>(cs), reinterpret_cast<int64_t>(prof));
}

NtsVar hip_linear(const NtsVar& x, const NtsVar& W, NtsStream* cs) {
  return HipLinearFn::apply(x, W, reinterpret_cast<int64_t>(cs));
}

bool hip_linear_xent_supported(int64_t K, int64_t C) {
  // mirrors the argument checks of nts_hip_linear_xent_fwd/bwd (C <= 64,
  // K % 16 == 0, W, 64 Y rows and 64 dZ rows in LDS)
  const int64_t Cp = (C + 15) / 16 * 16;
  return K >= 16 && K % 16 == 0 && C >= 1 && C <= 64 &&
         (K * Cp + 64 * (K + 4) + 64 * Cp) * 4 <= 160 * 1024;
}

NtsVar hip_linear_xent(const NtsVar& y, const NtsVar& W, const NtsVar& target, NtsStream* cs,
                       uint32_t* correct) {
  // a backward follows only under grad mode with an input requiring grad
  const bool train = torch::GradMode::is_enabled() && (y.requires_grad() || W.requires_grad());
  return HipLinearXentFn::apply(y, W, target, reinterpret_cast<int64_t>(cs), train,
                                reinterpret_cast<int64_t>(correct));
}

// ---------------------------------------------------------------------------
Parameter::Parameter(size_t w, size_t h, ValueType alpha_, ValueType beta1_, ValueType beta2_,
                     ValueType epsilon_, ValueType weight_decay_, int device, int64_t init_seed)
    : row((int)w), col((int)h), alpha(alpha_), beta1(beta1_), beta2(beta2_), epsilon(epsilon_),
      weight_decay(weight_decay_), beta1_t(beta1_), beta2_t(beta2_) {
  // xavier_uniform_ (core/NtsScheduler.hpp:731-733), seeded for reproducibility
  auto gen = at::detail::createCPUGenerator(init_seed);
  const double a = std::sqrt(6.0 / (double)(w + h));
  auto Wc = torch::empty({(int64_t)w, (int64_t)h}, torch::kFloat32).uniform_(-a, a, gen);
  W = Wc.to(torch::Device(torch::kCUDA, device)).set_requires_grad(true);
  M = torch::zeros_like(W).set_requires_grad(false);
  V = torch::zeros_like(W).set_requires_grad(false);
}

static void adam_step(Parameter& p, NtsStream& cs, int bias_correction) {
  TORCH_CHECK(p.W.grad().defined(), "Parameter has no gradient");
  NtsVar g = p.W.grad().contiguous();
  torch::NoGradGuard ng;
  hip_check(nts_hip_adam(cs.ctx(), p.W.data_ptr<float>(), g.data_ptr<float>(),
                         p.M.data_ptr<float>(), p.V.data_ptr<float>(), (uint64_t)p.W.numel(),
                         p.alpha, p.beta1, p.beta2, p.epsilon, p.weight_decay, p.beta1_t,
                         p.beta2_t, bias_correction),
            "nts_hip_adam");
}

void Parameter::adam_from(NtsStream& cs, const float* grad, bool bias_correction) {
  torch::NoGradGuard ng;
  hip_check(nts_hip_adam(cs.ctx(), W.data_ptr<float>(), grad, M.data_ptr<float>(),
                         V.data_ptr<float>(), (uint64_t)W.numel(), alpha, beta1, beta2, epsilon,
                         weight_decay, beta1_t, beta2_t, bias_correction ? 1 : 0),
            "nts_hip_adam");
}

void Parameter::learnC2C_with_decay_Adam(NtsStream& cs) { adam_step(*this, cs, 1); }
void Parameter::learn_local_with_decay_Adam(NtsStream& cs) { adam_step(*this, cs, 0); }

void Parameter::next() {
  beta1_t *= beta1;
  beta2_t *= beta2;
  ++curr_epoch;
}

// The gradient is dropped rather than zero-filled: the next backward then
// assigns W.grad instead of accumulating into zeros (no fill + add kernels).
void Parameter::zero_grad() {
  if (W.grad().defined()) W.mutable_grad() = NtsVar();
}

// ---------------------------------------------------------------------------
Communicator::Communicator(int n, int r, const std::vector<uint8_t>& uid, int device)
    : nranks(n), rank(r) {
  TORCH_CHECK(uid.size() == 128, "RCCL unique id must be 128 bytes");
  hip_check(nts_hip_comm_init(&comm_, n, r, uid.data(), device), "nts_hip_comm_init");
}
Communicator::Communicator(int n, int r, HostCollective host)
    : nranks(n), rank(r), host_(std::move(host)) {
  TORCH_CHECK(host_ && n >= 1 && r >= 0 && r < n, "host collective: ranks");
}
Communicator::~Communicator() {
  for (auto& e : tev_) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (comm_) nts_hip_comm_destroy(comm_);
}
void Communicator::timing_reset() {
  if (tused_) TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
  tused_ = 0;
  host_us_ = 0;
  host_calls_ = 0;
}
std::tuple<double, uint64_t, std::string> Communicator::timing_stats() {
  if (host_) return {host_calls_ ? host_us_ / (double)host_calls_ : 0.0, host_calls_, "host-wall"};
  double us = 0;
  for (size_t i = 0; i < tused_; ++i) {
    TORCH_CHECK(hipEventSynchronize(tev_[i].second) == hipSuccess, "hipEventSynchronize");
    float ms = 0;
    TORCH_CHECK(hipEventElapsedTime(&ms, tev_[i].first, tev_[i].second) == hipSuccess,
                "hipEventElapsedTime");
    us += 1e3 * ms;
  }
  return {tused_ ? us / (double)tused_ : 0.0, (uint64_t)tused_, "hip-events"};
}
void Communicator::host_call(float* buf, uint64_t n, void* stream, int op, int root) {
  TORCH_CHECK(hipStreamSynchronize((hipStream_t)stream) == hipSuccess, "hipStreamSynchronize");
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice");
  host_(torch::from_blob(buf, {(int64_t)n}, f32_opts(dev)), op, root);
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
}
void Communicator::allreduce_sum(float* buf, uint64_t n, void* stream) {
  if (host_) {
    const double t0 = now_s();
    host_call(buf, n, stream, 0, 0);
    if (timing_) {
      host_us_ += 1e6 * (now_s() - t0);
      ++host_calls_;
    }
    return;
  }
  if (timing_) {
    if (tused_ == tev_.size()) {
      hipEvent_t a, b;
      TORCH_CHECK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence) == hipSuccess &&
                      hipEventCreateWithFlags(&b, hipEventDisableSystemFence) == hipSuccess,
                  "hipEventCreateWithFlags");
      tev_.push_back({a, b});
    }
    TORCH_CHECK(hipEventRecord(tev_[tused_].first, (hipStream_t)stream) == hipSuccess, "hipEventRecord");
  }
  hip_check(nts_hip_allreduce_sum_f32(comm_, buf, n, stream), "nts_hip_allreduce_sum_f32");
  if (timing_) {
    TORCH_CHECK(hipEventRecord(tev_[tused_].second, (hipStream_t)stream) == hipSuccess, "hipEventRecord");
    ++tused_;
  }
}
void Communicator::broadcast(float* buf, uint64_t n, int root, void* stream) {
  if (host_) return host_call(buf, n, stream, 1, root);
  hip_check(nts_hip_broadcast_f32(comm_, buf, n, root, stream), "nts_hip_broadcast_f32");
}
std::pair<int, int> Communicator::rccl_count() const {
  if (host_) return {-1, -1};
  int n = 0, r = 0;
  hip_check(nts_hip_comm_count(comm_, &n, &r), "nts_hip_comm_count");
  return {n, r};
}
std::vector<uint8_t> Communicator::unique_id() {
  std::vector<uint8_t> id(128);
  hip_check(nts_hip_comm_unique_id(id.data()), "nts_hip_comm_unique_id");
  return id;
}

}  // namespace nts
