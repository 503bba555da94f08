#pragma once
#include <hip/hip_runtime_api.h>

#include "nts_host.hpp"

namespace nts {

struct GCNConfig {
  std::vector<int> layer_size;  // LAYERS, e.g. 602-128-41
  std::vector<int> fanout;      // FANOUT, layer 0 = nearest the seeds
  int batch_size = 1024;        // BATCH_SIZE
  float learn_rate = 0.01f, weight_decay = 1e-4f, drop_rate = 0.5f;
  float beta1 = 0.9f, beta2 = 0.999f, epsilon = 1e-9f;  // toolkits/GCN_SAMPLE_GPU.hpp:115-117
  int rng_mode = NTS_RNG_PHILOX;
  // GCN_SAMPLE_GPU (toolkits/GCN_SAMPLE_GPU.hpp:289-394): the CPU sampler's
  // blocks (sample_fast: the reference's mt19937 stream, here replayed on the
  // device, NTS_RNG_MT19937_LEMIRE) through SingleGPUSampleGraphOp, whose
  // backward always runs over the sampled CSR (Gather_By_Src_From_Dst_Spmm)
  bool sample_gpu = false;
  WeightType weight_type = WeightType::Sum;  // GraphSAGE toolkits: Mean
  bool up_degree = false;             // UP_DEGREE cfg key (core/GraphSegment.cpp:273-276)
  bool gat = false;                   // GAT_SAMPLE_ALL_GPU model (attention layers)
  bool fused_gather = true;           // gather features inside the bottom aggregation
  bool bias_correction = false;       // false: learn_local_with_decay_Adam (GPU drivers)
  bool deterministic_backward = true; // CSR transpose gather instead of atomics
  bool hip_gemm = true;               // layer GEMMs on the hand-written MFMA kernels
  bool pipeline = true;               // sample batch i+1 on its own stream while i trains
  bool fuse_activation = true;        // hidden layers: relu + dropout in the MFMA GEMM
  bool fuse_loss = true;              // training: output layer + log_softmax x2 + nll in 2 kernels
  // pipelined sampler's stream priority: 1 = sampler stream high, 0 = both
  // normal, -1 = the training stream high (the sampler's blocks dispatched
  // after the training stream's), 2 = auto: high for the MT19937 stream (its
  // chain is the step's critical path), normal for Philox (its ~0.2 ms of
  // kernels a batch fit beside the training step: C2 0.819-0.823 vs
  // 0.830-0.832 ms/step with the sampler high, scripts/ab/r06_u.sh)
  int sampler_priority = 2;
  // CUs of the pipelined sampler's stream: n > 0 reserves n CUs for it (the
  // training stream on the rest), n < 0 confines it to |n| CUs and leaves the
  // training stream on all; 0: no CU masks
  int sampler_cus = 0;
  // pipelined sampler, transform-first bottom layer: 0 = the next batch's
  // sampling is issued ahead of the training step; 1 = behind the forward
  // gather GEMM (it starts once that GEMM ends); 2 = also the backward gather
  // GEMM waits for it (neither GEMM shares CUs with the sampler)
  int sampler_gate = 0;
  bool pad_features = true;           // copy wide feature tables to a 128-byte row pitch
  bool early_aggregate = true;        // bottom aggregation issued with the sampling (see issue())
  // bottom layer order: 1 = transform first, A (X W) (rows narrowed before the
  // aggregation), 0 = aggregate first, (A X) W (the reference's order),
  // -1 = auto: transform first where F_in >= 4 F_out and the split-bf16
  // (fp32-exact) or pair-table GEMMs apply, aggregate first elsewhere
  int transform_first = -1;
  // layer GEMM arithmetic (nts_hip_ctx_set_gemm_mode): NTS_GEMM_F32 (fp32-input
  // MFMA) or NTS_GEMM_SPLIT3 (fp32-accurate three-piece bf16 split)
  int gemm_mode = NTS_GEMM_SPLIT3;
  // transform-first GEMMs on the feature table's f16 pair table (csrc/gemmh2.hip,
  // built once at construction; 22-bit significand inputs, narrower than
  // fp32: opt-in): 0 = off (gemm_mode: fp32-exact split-bf16), 1 = the
  // forward GEMM, 2 = the forward and the weight-gradient GEMMs, 3 = 2 with
  // the weight gradient on the planar table's whole-row kernel where the
  // shape allows
  int pair_table = 0;
  // data parallel: the gradient all-reduce of step k runs on a stream of its
  // own and the optimizer step waits for it only where step k+1 first reads
  // W (after its bottom aggregation, which does not depend on W): -1 = on with
  // more than one rank, 1 = always (also at one rank, for tests), 0 = off
  int overlap_allreduce = -1;
  bool shuffle = true;
  bool profile = false;               // HIP events around the bottom aggregation
  // CACHE_RATE in [0, 1): the feature table moves to pinned host memory and
  // the rows of the cache_rate * V highest-degree vertices stay in HBM
  // (GS_SAMPLE_PD_CACHE's placement); < 0: the whole table in HBM
  double cache_rate = -1.0;
  // NeutronOrch PD cache (GCN_SAMPLE_PD_CACHE): training seeds in
  // super-batches of pd_super_batch mini-batches (PIPELINE_NUM); per
  // super-batch the hot vertices (preSample, rate pd_rate = CACHE_RATE) get
  // their bottom-layer embedding (A X) W once, at the super-batch's first
  // batch, and every batch of the super-batch skips sampling their bottom
  // neighbourhoods and takes those rows instead.  Training only; aggregate-first.
  bool pd_cache = false;
  double pd_rate = 0.2;
  int pd_super_batch = 4;
  int64_t seed = 2000;
};

// Sampler-only throughput of the GPU sampler (SURVEY §8d "sampler-only"
// sampled-edges/s): FastSampler::sample_gpu_fast over `n_batches` batches of
// `seeds` on its own stream, three slots in flight (issue / finish as the
// pipelined driver does), nothing else on the device.  csr_layers as the
// training driver builds them.
struct SamplerRate {
  double seconds = 0;
  uint64_t edges = 0, batches = 0;
};
SamplerRate sampler_throughput(std::shared_ptr<FullyRepGraph> g, const std::vector<VertexId>& seeds,
                               int batch_size, const std::vector<int>& fanout, WeightType w,
                               int rng_mode, int n_batches, const std::vector<bool>& csr_layers);

class GCN_SAMPLE_ALLGPU_impl {
 public:
  GCN_SAMPLE_ALLGPU_impl(std::shared_ptr<FullyRepGraph> g, NtsVar feature, NtsVar label,
                         std::vector<VertexId> train_nids, GCNConfig cfg,
                         std::shared_ptr<Communicator> comm = nullptr);
  ~GCN_SAMPLE_ALLGPU_impl();

  void init_nn();
  float train_batch();
  float run_epoch();
  // Diagnostic (bench.py's training-stream-alone probe, never the headline):
  // on = sample one batch and train every later step on it, so the training
  // stream runs without the sampler beside it; off = back to sampling.
  void set_diag_reuse_sample(bool on) {
    diag_reuse_ = on;
    reuse_slot_ = -1;
  }
  bool has_batch() const {
    return prefetched_ >= 0 || (!pass_done_ && sampler->sample_not_finished());
  }
  void restart();
  // eval-mode forward over a given seed batch: [Y_0, X_1, Y_1, X_2, ...]
  std::vector<NtsVar> forward_eval(const std::vector<VertexId>& seeds, uint64_t batch_seq);
  void set_weights(const std::vector<NtsVar>& ws);
  // Accuracy (getCorrect / Test, toolkits/GCN_SAMPLE_ALLGPU.hpp:166-213,361-383):
  // training batches count their correct rows on the device as they train
  // (no per-batch sync); train_correct() reads the count (synchronises).
  uint64_t train_correct();
  void reset_correct();
  // Forward(eval_sampler, 1/2): eval mode over `nids` in batches of the
  // training batch size, sampled like training (the reference's eval/test
  // samplers); returns correct / |nids|.
  double evaluate(const std::vector<VertexId>& nids);
  // PD cache: the hot vertices of every super-batch (preSample on the device,
  // per super-batch counts + their concatenated ids, the PRE_SAMPLE_FILE
  // layout), or replace them (e.g. read from a PRE_SAMPLE_FILE)
  std::pair<std::vector<uint32_t>, std::vector<uint32_t>> presample();
  void set_presample(const std::vector<uint32_t>& counts, const std::vector<uint32_t>& ids);
  uint64_t pd_hits = 0;  // bottom-layer dsts served from the PD cache (host count, sampled batches)
  std::vector<NtsVar> weights();
  void reset_stats();
  void resolve_profile() { prof.resolve(); }

  std::shared_ptr<FullyRepGraph> graph;
  NtsVar F, L_GT, target, loss, grad_bucket;
  GCNConfig cfg;
  std::shared_ptr<Communicator> comm;
  std::unique_ptr<NtsStream> cs;  // training stream
  std::unique_ptr<NtsStream> ss;  // sampling stream (pipeline) — own scratch arena
  std::unique_ptr<FastSampler> sampler;
  std::unique_ptr<FeatureCache> fcache;  // two-tier feature table (cache_rate)
  std::vector<Parameter*> P;
  ctx::NtsContext ctx;
  // statistics
  double sample_time = 0, train_time = 0;
  uint64_t batch_edges = 0, batches = 0;
  KernelProfiler prof;  // device time of the bottom-layer kernels (cfg.profile)
  bool transform_first() const { return tf_; }
  uint64_t eval_seq = uint64_t(1) << 40;  // PHILOX stream of the evaluation batches

  SampledSubgraph* last_sg = nullptr;  // the batch the last train_batch() trained on
  // finish a deferred optimizer step (overlap_allreduce); every public entry
  // that reads or writes the weights calls it
  void flush_update();
  void sync() {
    flush_update();
    cs->synchronize();
  }

 private:
  NtsVar vertexForward(int l, NtsVar& a);
  // with `loss_target` (training), the last element is the fused scalar loss
  std::vector<NtsVar> forward(SampledSubgraph* sg, bool keep, const NtsVar* pre_y = nullptr,
                              const NtsVar* loss_target = nullptr);
  void issue(int slot, NtsStream& st);
  // GAT_SAMPLE_ALL_GPU::Forward (toolkits/GAT_SAMPLE_ALL_GPU.hpp:308-391)
  std::vector<NtsVar> forward_gat(SampledSubgraph* sg);
  double bottom_bytes(SampledSubgraph* sg, bool fused_map) const;
  KernelProfiler* profiler() { return cfg.profile ? &prof : nullptr; }
  void Loss(NtsVar& left, NtsVar& right);
  void Update();
  bool defer_ = false;            // overlap_allreduce in effect
  bool pending_update_ = false;   // an all-reduce is in flight, its Adam not yet run
  hipStream_t comm_stream_ = nullptr;
  hipEvent_t grads_packed_ = nullptr, grads_reduced_ = nullptr;
  std::pair<hipEvent_t, hipEvent_t>& next_events();
  void mark(const char* what, NtsStream& st);
  void count_correct(const NtsVar& out, const NtsVar& tgt);  // non-fused output layers
  NtsVar correct_;        // int32 [1]: correct rows of the training batches since reset
  uint32_t* count_to_ = nullptr;  // where forward's fused loss adds its correct count
  // ---- PD cache state ----
  static constexpr int kPdRing = 4;  // super-batches in flight (sampler lookahead)
  void pd_issue(int slot, NtsStream& st);  // per batch, at sampling time
  void pd_train(int slot);                 // per batch, before its forward
  std::vector<uint32_t> pd_counts_;   // hot vertices per super-batch
  std::vector<uint64_t> pd_offset_;   // their offsets in the concatenated id list
  NtsVar pd_ids_, pd_cache_map_, pd_cache_loc_;  // device: ids; u32 [V] map / location
  std::unique_ptr<FastSampler> pd_sampler_;      // 1 layer (bottom fanout) over the hot ids
  NtsVar pd_y_[kPdRing];              // their aggregation A X, per ring slot
  NtsVar pd_stage_[kPdRing];          // spilled feature rows of that aggregation (feature cache)
  NtsVar pd_share_;                   // (A X) W of the current super-batch
  uint32_t pd_next_key_ = 0;
  int pd_slot_key_[3] = {0, 0, 0};    // per sampler slot (kSlots): its super-batch key
  int pd_slot_sb_[3] = {-1, -1, -1};  // ... its super-batch index in the pass
  bool pd_slot_first_[3] = {false, false, false};
  uint32_t pd_key_ = 0;               // key of the batch being trained (forward)
  bool pd_active_ = false;
  std::vector<std::pair<const char*, hipEvent_t>> tl_;  // NTS_TIMELINE events
  bool tf_ = false;  // transform-first bottom layer (cfg.transform_first)
  std::unique_ptr<PairTable> pairs_;  // the feature table's f16 pair table (cfg.pair_table)
  // early aggregation: per sampler slot, the bottom graph op's output and the
  // event after which it (and the slot's sampled graph) is ready
  static constexpr int kSlots = 3;  // sampler slots when pipelined (see the constructor)
  int nslots_ = 1;
  NtsVar pre_y_[kSlots];
  NtsVar lbl_[kSlots];  // each slot's batch labels, gathered on the sampling stream
  NtsVar stage_[kSlots];  // early aggregation + feature cache: staged spill rows
  hipEvent_t ready_[kSlots] = {nullptr, nullptr, nullptr};
  bool early_ = false;
  uint64_t dropout_calls_ = 0;  // Philox offset of the fused dropout masks
  int prefetched_ = -1;  // slot holding an issued, not yet trained batch
  int next_slot_ = 0;
  bool diag_reuse_ = false;
  int reuse_slot_ = -1;  // set_diag_reuse_sample
  // pass boundary: the next pass's first batch is issued behind the current
  // pass's last one (carry_), handed over by restart()
  int carry_ = -1;
  bool pass_done_ = false;
  bool fresh_pass_ = true;
  // cfg.sampler_gate: the next batch's issue, deferred to the bottom layer's
  // forward GEMM hook, and the event it waits on
  std::function<void()> deferred_issue_;
  hipEvent_t gate_ev_ = nullptr;
  int gated_slot_ = -1;
  void prefetch_next();
};

}  // namespace nts
