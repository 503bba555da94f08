// C++ host layer (libtorch-ROCm) over the C-ABI in include/nts_hip.h.
//
// Mirrors the reference's operator / sampler surface so a toolkit written
// against it reads the same:
//   FullyRepGraph           core/FullyRepGraph.hpp:682-798   (HBM-resident here)
//   sampCSC / SampledSubgraph core/coocsc.hpp:24-462, core/FullyRepGraph.hpp:30-681
//   FastSampler             core/ntsFastSampler.hpp:28-1326  (GPU ctor + sample_gpu_fast)
//   nts::op::ntsGraphOp     core/ntsBaseOp.hpp:28-45
//   SingleGPUAllSampleGraphOp / SingleGPUSampleGraphOp  core/ntsSingleGPUSampleGraphOp.hpp:50-294
//   nts::ctx::NtsContext    core/ntsContext.hpp:95-680
//   Parameter               core/NtsScheduler.hpp:680-1029
//   Cuda_Stream             cuda/ntsCUDA.hpp:177-595  -> NtsStream (one nts_hip_ctx)
// Errors from the C-ABI throw std::runtime_error (the reference aborts).
#pragma once

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/torch.h>

#include <functional>
#include <memory>
#include <stack>
#include <string>
#include <deque>
#include <vector>

#include "nts_hip.h"

typedef uint32_t VertexId;
typedef float ValueType;
typedef torch::Tensor NtsVar;

// Sum / Mean / None: core/ntsFastSampler.hpp:27.  MeanSampled: the reference GPU
// kernel get_mean_weight's formula (NTS_WEIGHT_MEAN_SAMPLED, nts_hip.h).
enum class WeightType { Sum, Mean, None, MeanSampled };

namespace nts {

void hip_check(int rc, const char* what);

// torch dtype used to store uint32 vertex ids (bit pattern kept)
inline torch::TensorOptions u32_opts(int device) {
  return torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, device);
}
inline torch::TensorOptions f32_opts(int device) {
  return torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, device);
}
template <typename T>
inline T* dptr(const torch::Tensor& t) {
  return t.defined() ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}

// ---------------------------------------------------------------------------
// Cuda_Stream equivalent: one C-ABI context bound to one HIP stream.
// ---------------------------------------------------------------------------
class NtsStream {
 public:
  // stream == nullptr: a dedicated stream from torch's pool; torch work that
  // must be ordered with our kernels runs under guard() (the reference binds
  // a pool stream per pipeline thread, toolkits/GCN_SAMPLE_GPU.hpp:444-466).
  // high_priority: the pool's high-priority stream (the pipelined sampler:
  // its short, latency-bound kernels are dispatched ahead of the training
  // stream's long ones, which fill the remaining CU slots)
  NtsStream(int device, void* stream, uint64_t seed, bool high_priority = false);
  // an owned stream restricted to the CUs set in `cu_mask` (one bit per CU,
  // hipExtStreamCreateWithCUMask): partitions the device between streams
  NtsStream(int device, const std::vector<uint32_t>& cu_mask, uint64_t seed);
  ~NtsStream();
  NtsStream(const NtsStream&) = delete;
  NtsStream& operator=(const NtsStream&) = delete;
  void setNewStream(void* stream);  // Cuda_Stream::setNewStream
  void* stream() const;
  nts_hip_ctx* ctx() const { return ctx_; }
  int device() const { return device_; }
  void synchronize() const;
  // make this stream torch's current stream for the guard's lifetime
  c10::hip::HIPStreamGuard guard() const { return c10::hip::HIPStreamGuard(torch_stream_); }
  c10::hip::HIPStream torch_stream() const { return torch_stream_; }

 private:
  nts_hip_ctx* ctx_ = nullptr;
  hipStream_t owned_ = nullptr;
  int device_ = 0;
  c10::hip::HIPStream torch_stream_;
};

// ---------------------------------------------------------------------------
// FullyRepGraph: replicated global CSC + degrees in HBM.
// ---------------------------------------------------------------------------
class FullyRepGraph {
 public:
  VertexId global_vertices = 0;
  uint64_t global_edges = 0;
  int device = 0;
  torch::Tensor column_offset;  // int64 [V+1]
  torch::Tensor row_indices;    // int32 [E]
  torch::Tensor in_degree;      // int32 [V]  in_degree_for_backward
  torch::Tensor out_degree;     // int32 [V]  out_degree_for_backward

  // GenerateAll/ReadRepGraphFromRawFile from an edge list already on the device
  // (src/dst int32 tensors in file order), degrees from the same list.
  static std::shared_ptr<FullyRepGraph> from_edges(NtsStream& cs, const torch::Tensor& src,
                                                   const torch::Tensor& dst, VertexId vertices);
  // Wrap an existing device CSC (+ degrees).
  static std::shared_ptr<FullyRepGraph> from_csc(torch::Tensor column_offset,
                                                 torch::Tensor row_indices,
                                                 torch::Tensor in_degree, torch::Tensor out_degree);
  nts_graph_dev dev() const;
};

// ---------------------------------------------------------------------------
// sampCSC: one sampled layer, device arrays sized by capacity (the
// reference's dev_* mirrors + its global_data_buffer arena in one).
// ---------------------------------------------------------------------------
class sampCSC {
 public:
  VertexId v_size = 0, e_size = 0, src_size = 0;  // live sizes (host copy)
  VertexId v_cap = 0, e_cap = 0, s_cap = 0;
  bool has_csr = false;
  torch::Tensor destination, column_offset, row_indices, sample_ans, edge_dst, source,
      edge_weight_forward, row_offset, column_indices, edge_weight_backward, sizes;
  // is_merge_src_dst (GAT): dst d is local src dst_local_id[d]; CSR slot j is
  // CSC edge csr_edge_id[j] (both undefined unless set_merge_src_dst())
  torch::Tensor dst_local_id, csr_edge_id;
  // PD cache (sampled with an omit map): per dst its cache row or NTS_NOT_CACHED
  torch::Tensor omit_row;
  // transform-first training: this layer's graph-op backward also applies the
  // bottom layer's relu/dropout backward to its output (rows of post_mask =
  // the bottom activation X1, > 0 kept, times post_mask_scale), and the
  // bottom layer then receives dZ instead of dX1 (grad_premasked on it)
  const float* post_mask = nullptr;
  uint64_t post_mask_ld = 0;
  float post_mask_scale = 1.f;
  const uint32_t* post_mask_bits = nullptr;  // that mask as bits (act_bits of the layer below)
  torch::Tensor act_bits;  // transform-first bottom layer: its output's keep mask as bits
  bool grad_premasked = false;

  sampCSC(int device, VertexId v_cap, VertexId e_cap, VertexId s_cap, bool csr, bool weights);
  void set_merge_src_dst();  // core/coocsc.hpp:405-411
  VertexId* dev_dst_local_id() const { return dptr<VertexId>(dst_local_id); }
  // the reference accessor names
  VertexId* dev_dst() const { return dptr<VertexId>(destination); }
  VertexId* dev_src() const { return dptr<VertexId>(source); }
  VertexId* dev_c_o() const { return dptr<VertexId>(column_offset); }
  VertexId* dev_r_i() const { return dptr<VertexId>(row_indices); }
  VertexId* dev_r_o() const { return dptr<VertexId>(row_offset); }
  VertexId* dev_c_i() const { return dptr<VertexId>(column_indices); }
  ValueType* dev_e_w_f() const { return dptr<ValueType>(edge_weight_forward); }
  ValueType* dev_e_w_b() const { return dptr<ValueType>(edge_weight_backward); }
  ValueType* dev_e_w() const { return dptr<ValueType>(edge_weight_forward); }
  const VertexId* dev_v_size() const { return dptr<VertexId>(sizes); }
  const VertexId* dev_e_size() const { return dptr<VertexId>(sizes) + 1; }
  const VertexId* dev_src_size() const { return dptr<VertexId>(sizes) + 2; }
  // host copies (debug / tests): destination(), src(), c_o(), r_i(), ...
  std::vector<VertexId> host_u32(const torch::Tensor& t, size_t n) const;
};

class SampledSubgraph {
 public:
  std::vector<sampCSC*> sampled_sgs;
  int layers = 0;
  std::vector<int> fanout;
  torch::Tensor dev_sizes;   // device u32 [layers*4]: the layers' sizes (views)
  // int32 [layers*4] in mapped, coherent host memory: each layer's last
  // kernel stores its sizes words there (nts_sampcsc_dev::sizes_host)
  int32_t* host_sizes = nullptr;
  uint32_t* host_sizes_dev = nullptr;  // its device-visible address
  hipEvent_t sampled = nullptr;   // recorded after the last issue's kernels
  hipEvent_t consumed = nullptr;  // recorded by the trainer once it is done with the slot
  int pending_batch = 0;          // seeds of the issued, not yet finished batch
  SampledSubgraph(int device, int layers, const std::vector<int>& fanout, VertexId batch,
                  VertexId vertices, uint64_t edges, const std::vector<bool>& csr,
                  bool weights,
                  bool merge = false);
  ~SampledSubgraph();
  SampledSubgraph(const SampledSubgraph&) = delete;
  SampledSubgraph& operator=(const SampledSubgraph&) = delete;
};

// ---------------------------------------------------------------------------
// HBM feature cache + host-pinned spill (GS_SAMPLE_PD_CACHE:
// determine_cache_node_idx / cache_high_degree / mark_cache_node /
// gater_cpu_cache_feature_and_trans_to_gpu, toolkits/GS_SAMPLE_PD_CACHE.hpp:1019-1112).
// The full table moves to pinned host memory (device-mapped, zero-copy reads);
// the rows of the n_cache highest-out-degree vertices stay in HBM.
// ---------------------------------------------------------------------------
class FeatureCache {
 public:
  // table: fp32 [V, F] on the GPU (any row pitch); n_cache <= V rows cached
  FeatureCache(NtsStream& cs, const FullyRepGraph& g, const NtsVar& table, uint64_t n_cache);
  ~FeatureCache();
  FeatureCache(const FeatureCache&) = delete;
  FeatureCache& operator=(const FeatureCache&) = delete;
  uint64_t n_vertices = 0, n_cache = 0;
  int64_t F = 0;
  uint64_t ld = 0;               // row pitch (floats) of both tiers
  float* host = nullptr;         // pinned host table [V, ld] (owned)
  const float* host_dev = nullptr;  // its device-visible address
  NtsVar cache;                  // HBM [n_cache, F] (pitch ld), undefined when n_cache == 0
  NtsVar cache_map;              // u32 [V]: slot or NTS_NOT_CACHED
  NtsVar cache_ids;              // u32 [n_cache]
  const float* cache_ptr() const { return cache.defined() ? cache.data_ptr<float>() : nullptr; }
  // the fused bottom graph op on the two-tier table: the layer's non-cached
  // source rows are staged once into `stage` ([s_cap, ld] floats, HBM), then
  // Y = A X reads cached rows from the cache and the others from the stage.
  // v_dev / s_dev: device v_size / src_size (NULL: v_cap / s_cap are exact).
  void aggregate(nts_hip_ctx* ctx, const sampCSC* s, const uint32_t* v_dev, uint32_t v_cap,
                 const uint32_t* s_dev, uint32_t s_cap, float* stage, float* y,
                 uint64_t ldy) const;
};

// ---------------------------------------------------------------------------
// FastSampler (GPU form): sample_gpu_fast runs every hop on the device, with
// one D2H copy of the layer sizes per batch.
// ---------------------------------------------------------------------------
class FastSampler {
 public:
  std::shared_ptr<FullyRepGraph> whole_graph;
  VertexId work_range[2] = {0, 0};
  VertexId work_offset = 0;
  int layer = 0;
  std::vector<int> fanout;
  std::vector<VertexId> sample_nids;
  SampledSubgraph* ssg = nullptr;
  std::vector<SampledSubgraph*> ssgs;
  int rng_mode = NTS_RNG_PHILOX;
  bool up_degree = false;  // UP_DEGREE: weights from each sampled layer's own degrees
  uint64_t batch_seq = 0;  // keys the PHILOX stream (one per sampled batch)
  // sample_gpu_fast_omit (core/ntsFastSampler.hpp:711-915): when set, the
  // bottom layer skips the dsts with omit_map[d] == omit_key
  const uint32_t* omit_map = nullptr;
  uint32_t omit_key = 0;
  const uint32_t* omit_loc = nullptr;  // cache rows; recorded in the layer's omit_row
  double all_time = 0;     // sampler wall time (reference `all_time`)
  uint64_t sampled_edges = 0;

  // GPU ctor (core/ntsFastSampler.hpp:125-176).  csr_layers: which hops need
  // the CSR transpose (backward); empty = all.
  FastSampler(std::shared_ptr<FullyRepGraph> g, const std::vector<VertexId>& index, int layers,
              int batch_size, const std::vector<int>& fanout, int pipeline_num = 1,
              std::vector<bool> csr_layers = {}, bool weights = true,
              bool merge_src_dst = false);
  ~FastSampler();

  SampledSubgraph* sample_gpu_fast(int batch_size, int ssg_id, NtsStream& cs,
                                   WeightType w = WeightType::Sum);
  // Split form for pipelining (the reference overlaps with PIPELINE_NUM host
  // threads, toolkits/GCN_SAMPLE_GPU.hpp:289-394): issue enqueues every hop
  // and the size copy on `cs` without blocking; finish waits for that batch
  // and publishes v/e/src sizes.  A slot is reused only after its `consumed`
  // event (recorded by the trainer) — issue makes `cs` wait for it.
  void issue_gpu_sample(int batch_size, int ssg_id, NtsStream& cs, WeightType w);
  SampledSubgraph* finish_gpu_sample(int ssg_id);
  // MT19937 modes: a batch whose word stream fell short is sampled again
  // from its checkpoint with larger bounds (finish_gpu_sample does it; the
  // batches issued behind it are re-run too).  rerun_ok = false when work
  // chained to the sampled batches on the sampler stream (the driver's early
  // aggregation) would have to be re-done as well: then a short stream throws.
  bool rerun_ok = true;
  uint64_t mt_reruns = 0;  // batches re-run so far (tests)
  bool sample_not_finished() const { return work_offset < work_range[1]; }
  void restart() { work_offset = work_range[0]; }
  void set_sample_nids(const std::vector<VertexId>& ids);

  // load_feature_gpu / load_label_gpu (core/ntsFastSampler.hpp:244-261, 414-426)
  void load_feature_gpu(NtsStream& cs, SampledSubgraph* sg, NtsVar& local_feature,
                        const NtsVar& global_feature);
  void load_label_gpu(NtsStream& cs, SampledSubgraph* sg, NtsVar& local_label,
                      const NtsVar& global_label);
  // load_feature_gpu_cache (core/ntsFastSampler.hpp:263-317): cached rows from
  // HBM, the rest zero-copy from the pinned host table, in one kernel
  void load_feature_gpu_cache(NtsStream& cs, SampledSubgraph* sg, NtsVar& local_feature,
                              const FeatureCache& cache);
  // MT19937 modes: every later layer's word bound x scale (tests force a short
  // first stream with a small one; each re-run multiplies it by 4)
  void set_mt_budget_scale(NtsStream& cs, double scale);
  double mt_budget_scale() const { return mt_budget_; }

 private:
  struct IssueRec {  // one pending batch per slot: what a re-run needs
    VertexId offset = 0, actual = 0;
    uint64_t batch_seq = 0;
    int wt = 0;
    const uint32_t* omit_map = nullptr;
    uint32_t omit_key = 0;
    const uint32_t* omit_loc = nullptr;
    NtsStream* cs = nullptr;
    torch::Tensor mt_ckpt;  // device u32 [625]: the generator before the batch
  };
  std::vector<IssueRec> recs_;
  std::deque<int> issued_;  // slots issued and not yet finished, in issue order
  double mt_budget_ = 1.0;
  void enqueue_layers(int ssg_id, const IssueRec& r);
  void rerun_from(int ssg_id);
  torch::Tensor dev_nids_;  // device copy of sample_nids
  torch::Tensor dev_iota_;  // 0, 1, ..., batch_cap: device scalars for the layer-0 v_size
  VertexId batch_cap_ = 0;
};

// ---------------------------------------------------------------------------
// graph operators
// ---------------------------------------------------------------------------
namespace op {

class ntsGraphOp {
 public:
  virtual ~ntsGraphOp() = default;
  virtual NtsVar forward(NtsVar& f_input) = 0;
  virtual NtsVar forward(NtsVar& f_input, std::vector<VertexId> cacheflag) {
    (void)cacheflag;
    return forward(f_input);
  }
  virtual NtsVar backward(NtsVar& output_grad) = 0;
  bool output_requires_grad = true;
};

// SingleGPUAllSampleGraphOp (core/ntsSingleGPUSampleGraphOp.hpp:195-294):
// forward Y = A^T X over the sampled CSC (hand kernel instead of cuSPARSE);
// backward through the CSR transpose when the sampler built it
// (deterministic), otherwise the atomic CSC scatter (Push_From_Dst_To_Src).
// With `gather_from_table`, f_input is the global feature table and rows are
// fetched through the layer's `source` (fused load_feature_gpu + aggregate).
class SingleGPUAllSampleGraphOp : public ntsGraphOp {
 public:
  // feature_cache: with gather_from_table, rows come from the two-tier table
  // (HBM cache + host spill) instead of f_input
  SingleGPUAllSampleGraphOp(SampledSubgraph* subgraphs, FullyRepGraph* graph, int layer,
                            NtsStream* cs, bool gather_from_table = false,
                            const FeatureCache* feature_cache = nullptr);
  NtsVar forward(NtsVar& f_input) override;
  NtsVar backward(NtsVar& f_output_grad) override;

  SampledSubgraph* subgraphs;
  int layer;
  NtsStream* cuda_stream;
  bool gather_from_table;
  const FeatureCache* feature_cache;
};

// SingleGPUSampleGraphOp (core/ntsSingleGPUSampleGraphOp.hpp:50-176): same
// forward; backward always through the CSR (row_offset/column_indices/e_w_b).
class SingleGPUSampleGraphOp : public SingleGPUAllSampleGraphOp {
 public:
  using SingleGPUAllSampleGraphOp::SingleGPUAllSampleGraphOp;
  NtsVar backward(NtsVar& f_output_grad) override;
};

}  // namespace op

// ---------------------------------------------------------------------------
// autodiff context (core/ntsContext.hpp)
// ---------------------------------------------------------------------------
namespace ctx {

enum OpType { NNOP = 0, GRAPHOP = 1 };

class NtsContext {
 public:
  NtsContext();
  ~NtsContext();

  template <typename GOPT, typename... Args>
  NtsVar runGraphOp(NtsVar& f_input, Args&&... args) {
    auto* curr = new GOPT(std::forward<Args>(args)...);
    // The bottom graph op's input never needs a gradient (its backward is
    // skipped, core/ntsContext.hpp:443-444); its output then needs none either,
    // which spares autograd the dense dY of the first GEMM.
    curr->output_requires_grad = !(training && count == 0);
    NtsVar f_output = curr->forward(f_input);
    push_graph_op(curr, f_input, f_output);
    return f_output;
  }
  NtsVar runVertexForward(const std::function<NtsVar(NtsVar&, NtsVar&)>& fn, NtsVar& nbr_input,
                          NtsVar& vtx_input);
  NtsVar runVertexForward(const std::function<NtsVar(NtsVar&)>& fn, NtsVar& nbr_input);
  void appendNNOp(NtsVar& input_t, NtsVar& output_t);
  void self_backward(bool retain_graph = true);
  void reset();
  void train() { training = true; }
  void eval() { training = false; }
  bool is_train() const { return training; }

  bool training = true;
  int count = 0;

 private:
  struct Entry {
    OpType type;
    op::ntsGraphOp* op;  // owned (GRAPHOP)
    NtsVar input, output, output_grad;
    void* in_id;
    void* out_id;
  };
  void push_graph_op(op::ntsGraphOp* op, NtsVar& in, NtsVar& out);
  void pop_one_op();
  std::vector<Entry> ops_;
};

}  // namespace ctx

// ---------------------------------------------------------------------------
// Parameter (core/NtsScheduler.hpp:680-1029), Adam via the fused HIP kernel.
// ---------------------------------------------------------------------------
// x.matmul(W) on the MFMA fp32 kernels (nts_hip_gemm_f32) with its own
// backward: dW = x^T dZ (split-reduction, deterministic), dx = dZ W^T.
NtsVar hip_linear(const NtsVar& x, const NtsVar& W, NtsStream* cs);
// one GAT layer (H = X W, attention softmax over each dst's sampled edges,
// relu(sum a H[src])) on a merged src/dst layer: [src_size, F_in] -> [v_size, F]
class KernelProfiler;
NtsVar hip_gat_layer(const NtsVar& x, const NtsVar& W, const NtsVar& Watt, sampCSC* sg,
                     NtsStream* cs, KernelProfiler* prof = nullptr);
// CU masks splitting the device: `n` CUs spread evenly over the chip
// (every (total/n)-th CU) and the complement
std::vector<uint32_t> cu_mask_spread(int device, int n, bool complement);
// training output layer + loss: nll_loss(log_softmax(log_softmax(y W)), target)
// in two fused kernels (nts_hip_linear_xent_fwd/bwd); returns the scalar loss
// Persistent fp32 scalar 1 on `dev` (the loss-backward seed).
const NtsVar& unit_scalar(const torch::Device& dev);
bool hip_linear_xent_supported(int64_t K, int64_t C);
// correct != NULL: *correct += rows whose argmax is the target (getCorrect)
NtsVar hip_linear_xent(const NtsVar& y, const NtsVar& W, const NtsVar& target, NtsStream* cs,
                       uint32_t* correct = nullptr);
// row-major fp32 views the HIP GEMMs take without a copy (unit column stride)
NtsVar row_major(const NtsVar& x);
// [rows, F] with 128-byte aligned rows when F >= 64 (padded leading dimension)
NtsVar row_padded_empty(int64_t rows, int64_t F, int device);
// dropout(relu(x W), p) in one MFMA GEMM (activation in the epilogue, Philox
// mask of (seed, offset)); autograd: dW = x^T (dX ⊙ [X > 0] / (1-p)) fused.
// pair_split: narrow inputs (K <= 128, N 128 | 256) may use the in-kernel f16
// pair split (nts_hip_gemm_h2d_act) instead of the GEMM mode's kernel.
NtsVar hip_linear_act(const NtsVar& x, const NtsVar& W, double p, uint64_t seed, uint64_t offset,
                      NtsStream* cs, bool pair_split);

// Device time of selected kernels on the stream that launches them (HIP
// events; resolve() synchronises — call outside timed regions).  `units` are
// the algorithmic bytes (aggregations) or flops (GEMMs) of one launch.
// One kernel class per step is timed, rotating over the classes the driver
// has launched (next_step() per training step): each event pair costs the
// training stream ~4-5 us of gap, so timing every class every step added ~36
// us to a 0.9 ms step; a quarter of the launches of each class is the sample.
class KernelProfiler {
 public:
  enum Id { BOTTOM_AGG = 0, GATHER_GEMM, GATHER_GEMM_TN, BOTTOM_BWD, GAT_FWD, kCount };
  struct Stat {
    double ms = 0, units = 0;
    uint64_t calls = 0;
  };
  KernelProfiler() { for (int& o : open_) o = -1; }
  ~KernelProfiler();
  KernelProfiler(const KernelProfiler&) = delete;
  KernelProfiler& operator=(const KernelProfiler&) = delete;
  void begin(Id id, hipStream_t st);
  void end(Id id, hipStream_t st, double units);
  void resolve();
  void reset();
  void add_units(Id id, double units) {
    if (active(id)) stat[id].units += units;
  }
  // a new step: its timed class is the (step % #seen)-th of the classes seen
  // in the steps before it, frozen for the whole step (a class
  // first seen mid-step no longer changes the choice between begin, add_units
  // and end of one step); before any class was seen, the step's first caller
  void next_step() {
    ++step_;
    sel_ = -1;
    if (seen_) {
      uint32_t m = seen_;
      for (int k = (int)(step_ % (uint64_t)__builtin_popcount(seen_)); k > 0; --k) m &= m - 1;
      sel_ = __builtin_ctz(m);
    }
  }
  static const char* name(int id);
  Stat stat[kCount];

 private:
  bool active(Id id) {
    seen_ |= 1u << id;
    if (sel_ < 0) sel_ = (int)id;
    return sel_ == (int)id;
  }
  uint32_t seen_ = 0;
  uint64_t step_ = 0;
  int sel_ = -1;  // this step's timed class
  struct Slot {
    Id id = BOTTOM_AGG;
    hipEvent_t a = nullptr, b = nullptr;
    double units = 0;
  };
  std::vector<Slot> pool_;
  size_t used_ = 0;
  int open_[kCount];
};

// dropout(relu(x), p) as its own autograd op (the GEMM epilogue's mask keys)
NtsVar hip_relu_dropout(const NtsVar& x, double p, uint64_t seed, uint64_t offset, NtsStream* cs);

// Transform-first bottom layer (nts_hip.h): X1 = dropout(relu(A (X[source] W)))
// on the layer's sampled block `sg` (its CSR is needed for the backward);
// autograd returns dW = X[source]^T (A^T (dX1 ⊙ mask)).  h_out != NULL: H =
// X[source] W is written there ([src_size, F_out], eval / tests).
// pairs != NULL: the table's f16 pair table (nts_hip_h2_split_rows, built once
// by the driver) — the forward GEMM runs on it, and the weight-gradient GEMM
// too when pairs->tn.
struct PairTable {
  NtsVar P;   // int32 [V, Kp] pair words
  NtsVar rs;  // fp32 [V] row scales
  bool tn = true;
  NtsVar Q;   // int16 [V, 2 Kp] planar form (defined: the weight gradient on k_h2_tn3)
};
// Stream-phase hooks of the transform-first bottom layer (the driver's
// sampler gating, GCNConfig::sampler_gate): called on the host right after
// the forward gather GEMM is enqueued, and right before the backward one.
void set_bottom_gemm_hooks(std::function<void()> after_fwd_gemm,
                           std::function<void()> before_bwd_gemm);
NtsVar hip_bottom_transform(const NtsVar& table, const NtsVar& W, sampCSC* sg, double p,
                            uint64_t seed, uint64_t offset, NtsStream* cs, KernelProfiler* prof,
                            float* h_out = nullptr, const PairTable* pairs = nullptr);

struct Parameter {
  NtsVar W, M, V;
  NtsStream* cs = nullptr;  // set -> forward runs on the hand-written MFMA GEMM
  int row, col;
  ValueType alpha, beta1, beta2, epsilon, weight_decay;
  ValueType beta1_t, beta2_t;
  int curr_epoch = 0;
  Parameter(size_t w, size_t h, ValueType alpha, ValueType beta1, ValueType beta2,
            ValueType epsilon, ValueType weight_decay, int device, int64_t init_seed);
  NtsVar forward(const NtsVar& x) const { return cs ? hip_linear(x, W, cs) : x.matmul(W); }
  // Parameter::learnC2C_with_decay_Adam (bias-corrected, CPU driver semantics)
  void learnC2C_with_decay_Adam(NtsStream& cs);
  // Parameter::learn_local_with_decay_Adam (GPU drivers, no bias correction)
  void learn_local_with_decay_Adam(NtsStream& cs);
  // either variant with the gradient taken from `grad` (a reduced bucket slice)
  void adam_from(NtsStream& cs, const float* grad, bool bias_correction);
  void next();
  void zero_grad();
};

// RCCL communicator (NCCL_Communicator replacement) — one per process.
// Host transport for the same two collectives (tests and the one-GPU
// rehearsal of the multi-rank path): called with a tensor viewing the device
// buffer after its stream is synchronised; op 0 = SUM all-reduce in place,
// op 1 = broadcast from `root`.  The result must be in the buffer when it
// returns.
using HostCollective = std::function<void(torch::Tensor, int op, int root)>;

class Communicator {
 public:
  Communicator(int nranks, int rank, const std::vector<uint8_t>& uid, int device);
  Communicator(int nranks, int rank, HostCollective host);
  ~Communicator();
  void allreduce_sum(float* buf, uint64_t n, void* stream);
  void broadcast(float* buf, uint64_t n, int root, void* stream);
  static std::vector<uint8_t> unique_id();
  bool host_transport() const { return (bool)host_; }
  // (ranks, this rank) as RCCL reports them (ncclCommCount / ncclCommUserRank);
  // (-1, -1) for the host transport
  std::pair<int, int> rccl_count() const;
  int nranks, rank;
  // Per-call timing of allreduce_sum (bench.py's allreduce_us_per_step):
  // RCCL — a HIP event pair (no system fence) around the call on the stream it
  // is enqueued on; host transport — the host wall time of the blocking call.
  // timing_stats() synchronises the events: call outside timed regions.
  void set_timing(bool on) { timing_ = on; }
  void timing_reset();
  // (mean microseconds per call, calls, "hip-events" | "host-wall")
  std::tuple<double, uint64_t, std::string> timing_stats();

 private:
  void host_call(float* buf, uint64_t n, void* stream, int op, int root);
  nts_hip_comm* comm_ = nullptr;
  HostCollective host_;
  bool timing_ = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> tev_;
  size_t tused_ = 0;
  double host_us_ = 0;
  uint64_t host_calls_ = 0;
};

}  // namespace nts
