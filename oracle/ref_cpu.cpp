// ============================================================================
//  ORACLE — test infrastructure only.
//  A CPU restatement of the reference's sampled-GCN hot path
//  (AiX-im/Sample-based-GNN @ 2024-10-08), used as the checker by tests/,
//  __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product path
//  (sample-based-gnn_amd/) never links or calls this file.
//
//  Parity pinning: the reference ships no tests or golden vectors (SURVEY §4,
//  §8c) and may not be compiled or run here (recorded denial), so
//  this restatement is pinned by (i) RNG-independent known-answer tests
//  (full-neighbourhood fanout, all-ones features, a hand-computed 5-vertex
//  graph) and (ii) the reference's own Cora data files (tests/golden/).
//  The sampler uses the same std::mt19937 / std::uniform_int_distribution /
//  std::unordered_map as the reference, so its draws are the reference's
//  draws for a single sampler thread.
//
//  Each function cites the reference lines it restates.
// ============================================================================
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <sstream>
#include <unordered_map>
#include <vector>

extern "C" {

// ---- graph ------------------------------------------------------------------
// FullyRepGraph::ReadRepGraphFromRawFile (core/FullyRepGraph.hpp:724-798):
// pass 1 counts edges per dst, prefix sum; pass 2 appends src in file order.
int orc_build_csc(uint64_t V, uint64_t E, const uint32_t* src, const uint32_t* dst,
                  uint64_t* column_offset, uint32_t* row_indices) {
  std::vector<uint64_t> tmp(V + 1, 0);
  for (uint64_t e = 0; e < E; ++e) tmp[dst[e] + 1]++;
  for (uint64_t i = 0; i < V; ++i) tmp[i + 1] += tmp[i];
  std::memcpy(column_offset, tmp.data(), (V + 1) * sizeof(uint64_t));
  for (uint64_t e = 0; e < E; ++e) row_indices[tmp[dst[e]]++] = src[e];
  return 0;
}

// Graph::load_directed out/in degree (core/graph.hpp:1157-1186, 1420-1425)
// + clamp to >= 1 (core/graph.hpp:4525-4530).
int orc_degrees(uint64_t V, uint64_t E, const uint32_t* src, const uint32_t* dst,
                uint32_t* out_degree, uint32_t* in_degree) {
  std::fill(out_degree, out_degree + V, 0u);
  std::fill(in_degree, in_degree + V, 0u);
  for (uint64_t e = 0; e < E; ++e) {
    out_degree[src[e]]++;
    in_degree[dst[e]]++;
  }
  for (uint64_t v = 0; v < V; ++v) {
    if (in_degree[v] < 1) in_degree[v] = 1;
    if (out_degree[v] < 1) out_degree[v] = 1;
  }
  return 0;
}

}  // extern "C"

namespace {

// nts_norm_degree (core/ntsBaseOp.hpp:652-657): std::sqrt of an integer is the
// double overload, each factor is rounded to float, then 1 / (a*b) in float.
inline float norm_degree(uint32_t out_src, uint32_t in_dst) {
  float a = (float)std::sqrt(out_src);
  float b = (float)std::sqrt(in_dst);
  return 1 / (a * b);
}

// Philox4x32-10 counter stream of the product's PHILOX mode (restated from
// its published definition; keyed exactly like sampler.hip).
inline void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
inline uint32_t philox_word(uint64_t seed, uint32_t d, uint32_t layer, uint64_t bs, uint32_t j) {
  uint32_t c[4] = {j >> 2, d, layer, (uint32_t)bs};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(bs >> 32));
  return c[j & 3];
}

struct Layer {
  std::vector<uint32_t> destination, column_offset, row_indices, sample_ans, source;
  std::vector<uint32_t> row_offset, column_indices, csr_edge_id, dst_local_id;
  std::vector<float> edge_weight_forward, edge_weight_backward;
  uint32_t v_size = 0, e_size = 0, src_size = 0;
};

enum { RNG_PHILOX = 0, RNG_MT_LEMIRE = 1, RNG_MT_DIV = 2 };
enum { ORDER_DRAW = 0, ORDER_UNORDERED_MAP = 1 };
// W_MEAN_SAMPLED: the reference GPU kernel get_mean_weight
// (cuda/ntsCUDATransferKernel.cuh:319-342): norm / (sampled edges of the dst).
// Its GPU toolkits never reach it (sample_gpu_fast drops the weight type,
// core/ntsFastSampler.hpp:944-948).
enum { W_SUM = 0, W_MEAN = 1, W_NONE = 2, W_MEAN_SAMPLED = 3, W_UP_DEGREE = 0x10,
       F_MERGE_SRC_DST = 0x20 };

struct Sampler {
  uint64_t V;
  const uint64_t* off;
  const uint32_t* rows;
  const uint32_t* indeg;
  const uint32_t* outdeg;
  std::vector<int> fanout;
  uint64_t seed;
  int rng_mode, order_mode;
  std::mt19937 gen;  // `static thread_local std::mt19937 generator(2000)` (core/ntsFastSampler.hpp:202)
  std::vector<Layer> layers;
  std::vector<uint32_t> src_index;
  std::vector<uint64_t> bitmap;
  // sample_gpu_fast_omit (core/ntsFastSampler.hpp:711-915): in the LAST layer a
  // dst with omit_map[dst] == omit_key samples nothing
  const uint32_t* omit_map = nullptr;
  uint32_t omit_key = 0;
};

// std::uniform_int_distribution<int>(0, range-1) in its libstdc++ <= 10 form
// (two divisions) for the MT19937_DIV mode.
inline uint32_t uniform_div(std::mt19937& g, uint32_t range) {
  const uint32_t scaling = 0xFFFFFFFFu / range;
  const uint32_t past = range * scaling;
  uint32_t r;
  do r = (uint32_t)g(); while (r >= past);
  return r / scaling;
}

// The `num` distinct draws of one dst, in draw order and in the order the
// reference emits them (std::unordered_map iteration, core/ntsFastSampler.hpp:1026-1038).
void draw_distinct(Sampler& s, std::mt19937& gen, uint32_t d, uint32_t layer, uint64_t bs,
                   uint32_t deg, uint32_t num, std::vector<uint32_t>& out_pos) {
  out_pos.clear();
  std::unordered_map<uint32_t, int> sampled;  // reference key type: VertexId
  std::vector<uint32_t> order;
  uint32_t j = 0;
  while (sampled.size() < num) {
    uint32_t r;
    if (s.rng_mode == RNG_MT_LEMIRE) {
      std::uniform_int_distribution<int> dist(0, (int)deg - 1);  // random_uniform_int (:200-205)
      r = (uint32_t)dist(gen);
    } else if (s.rng_mode == RNG_MT_DIV) {
      r = uniform_div(gen, deg);
    } else {
      // PHILOX: word-wise Lemire acceptance on the per-dst counter stream
      const uint32_t thr = (0u - deg) % deg;
      for (;;) {
        uint64_t m = (uint64_t)philox_word(s.seed, d, layer, bs, j++) * deg;
        if ((uint32_t)m >= thr) { r = (uint32_t)(m >> 32); break; }
      }
    }
    if (sampled.insert(std::pair<uint32_t, int>(r, 1)).second) order.push_back(r);
  }
  if (s.order_mode == ORDER_UNORDERED_MAP) {
    for (auto& kv : sampled) out_pos.push_back(kv.first);
  } else {
    out_pos = order;
  }
}

}  // namespace

extern "C" {

void* orc_sampler_new(uint64_t V, const uint64_t* off, const uint32_t* rows,
                      const uint32_t* indeg, const uint32_t* outdeg, int layers,
                      const int* fanout, uint64_t seed, int rng_mode, int order_mode) {
  Sampler* s = new Sampler();
  s->V = V;
  s->off = off;
  s->rows = rows;
  s->indeg = indeg;
  s->outdeg = outdeg;
  s->fanout.assign(fanout, fanout + layers);
  s->seed = seed;
  s->rng_mode = rng_mode;
  s->order_mode = order_mode;
  s->gen.seed((std::mt19937::result_type)seed);
  s->layers.resize(layers);
  s->src_index.assign(V, 0);
  s->bitmap.assign(V / 64 + 1, 0);
  return s;
}

void orc_sampler_free(void* h) { delete (Sampler*)h; }

void orc_sampler_set_omit(void* h, const uint32_t* omit_map, uint32_t omit_key) {
  Sampler& s = *(Sampler*)h;
  s.omit_map = omit_map;
  s.omit_key = omit_key;
}

// FastSampler::sample_fast (core/ntsFastSampler.hpp:962-1140) for one batch,
// single sampler thread.  threads > 1 runs the dst loops under OpenMP with a
// thread-local generator per worker like the reference (timing baseline only;
// results then depend on the thread count, as the reference's do).
int orc_sample_batch(void* h, const uint32_t* seeds, uint32_t B, uint64_t batch_seq,
                     int weight_flags, int build_csr, int threads) {
  Sampler& s = *(Sampler*)h;
  // UP_DEGREE (cfg key, core/GraphSegment.cpp:273-276): degrees recomputed from
  // each sampled layer before its weights (SampledSubgraph::update_degrees,
  // core/FullyRepGraph.hpp:189-207, called at core/ntsFastSampler.hpp:1107-1108)
  const bool up_degree = (weight_flags & W_UP_DEGREE) != 0;
  // is_merge_src_dst (core/coocsc.hpp:405-411, set by the GAT drivers): every
  // dst is marked in the frontier too (core/ntsFastSampler.hpp:1050-1052) and
  // dst_local_id[d] = its local src id (:1095-1097)
  const bool merge = (weight_flags & F_MERGE_SRC_DST) != 0;
  const int weight_type = weight_flags & 0xF;
  const int L = (int)s.layers.size();
  for (int i = 0; i < L; ++i) {
    Layer& ly = s.layers[i];
    // destination: seeds (i == 0) or the previous layer's source (:984-995)
    if (i == 0) ly.destination.assign(seeds, seeds + B);
    else ly.destination = s.layers[i - 1].source;
    const uint32_t v = (uint32_t)ly.destination.size();
    ly.v_size = v;
    // init_co_only (core/FullyRepGraph.hpp:530-539) with the lambda at :1001-1009
    ly.column_offset.assign(v + 1, 0);
    uint32_t acc = 0;
    for (uint32_t k = 0; k < v; ++k) {
      ly.column_offset[k] = acc;
      uint32_t d = ly.destination[k];
      uint32_t nbrs = (uint32_t)(s.off[d + 1] - s.off[d]);
      if (s.omit_map && i == L - 1 && s.omit_map[d] == s.omit_key) nbrs = 0;  // omit
      int f = s.fanout[i];
      uint32_t ret = (f < 0) ? nbrs : std::min(nbrs, (uint32_t)f);
      acc += ret;
    }
    ly.column_offset[v] = acc;
    const uint32_t e = acc;
    ly.e_size = e;
    ly.sample_ans.assign(e, 0);
    ly.row_indices.assign(e, 0);
    std::fill(s.bitmap.begin(), s.bitmap.end(), 0ull);  // samp_bitmap->clear()
    // sample_processing1 with the lambda at :1020-1054
    const uint32_t fan_u = (uint32_t)s.fanout[i];      // VertexId fanout_i: -1 -> 0xFFFFFFFF
    auto per_dst = [&](uint32_t k, std::mt19937& gen, std::vector<uint32_t>& pos) {
      uint32_t d = ly.destination[k];
      uint64_t beg = s.off[d];
      uint32_t deg = (uint32_t)(s.off[d + 1] - beg);
      uint32_t c = ly.column_offset[k];
      uint32_t num = ly.column_offset[k + 1] - c;
      if (num == 0) return;
      if (deg > fan_u) {
        draw_distinct(s, gen, d, (uint32_t)i, batch_seq, deg, num, pos);
        for (uint32_t p = 0; p < num; ++p) ly.sample_ans[c + p] = s.rows[beg + pos[p]];
      } else {
        for (uint32_t p = 0; p < num; ++p) ly.sample_ans[c + p] = s.rows[beg + p];
      }
      for (uint32_t p = 0; p < num; ++p) {
        uint32_t g = ly.sample_ans[c + p];
        __atomic_fetch_or(&s.bitmap[g >> 6], 1ull << (g & 63), __ATOMIC_RELAXED);
      }
    };
    if (threads <= 1) {
      std::vector<uint32_t> pos;
      for (uint32_t k = 0; k < v; ++k) per_dst(k, s.gen, pos);
    } else {
#pragma omp parallel num_threads(threads)
      {
        static thread_local std::mt19937 tgen(2000);
        std::vector<uint32_t> pos;
#pragma omp for
        for (uint32_t k = 0; k < v; ++k) per_dst(k, tgen, pos);
      }
    }
    if (merge)
      for (uint32_t k = 0; k < v; ++k) {
        const uint32_t g = ly.destination[k];
        s.bitmap[g >> 6] |= 1ull << (g & 63);
      }
    // bitmap scan in ascending order -> source, src_index (:1064-1083)
    ly.source.clear();
    for (uint64_t w = 0; w < s.bitmap.size(); ++w) {
      uint64_t word = s.bitmap[w];
      uint32_t bit = 0;
      while (word) {
        if (word & 1ull) {
          uint32_t g = (uint32_t)(w * 64 + bit);
          s.src_index[g] = (uint32_t)ly.source.size();
          ly.source.push_back(g);
        }
        ++bit;
        word >>= 1;
      }
    }
    const uint32_t src_size = (uint32_t)ly.source.size();
    ly.src_size = src_size;
    ly.dst_local_id.clear();
    // dst_local_id[k] = src_index[destination[k]] — indexed by the dst k.  The
    // reference writes dst_local_id[id] = src_index_array[dst()[i]] with i the
    // LAYER (core/ntsFastSampler.hpp:1096), which stores
    // the local id of the i-th dst for every dst; this restatement (and the
    // product) follows the evident intent (set_dst_local_index,
    // cuda/ntsCUDAGraphOP.cu:1696) instead of replicating that defect.
    if (merge) {
      ly.dst_local_id.resize(v);
      for (uint32_t k = 0; k < v; ++k) ly.dst_local_id[k] = s.src_index[ly.destination[k]];
    }
    // relabel (:1085-1099)
#pragma omp parallel for num_threads(threads > 1 ? threads : 1)
    for (uint32_t k = 0; k < e; ++k) ly.row_indices[k] = s.src_index[ly.sample_ans[k]];
    // csc_to_csr (core/coocsc.hpp:82-111), serial fill -> ascending dst per src
    if (build_csr || weight_type != W_NONE) {
      ly.row_offset.assign(src_size + 1, 0);
      ly.column_indices.assign(e, 0);
      for (uint32_t k = 0; k < e; ++k) ly.row_offset[ly.row_indices[k]]++;
      uint32_t run = 0;
      for (uint32_t r = 0; r < src_size; ++r) {
        uint32_t t = ly.row_offset[r];
        ly.row_offset[r] = run;
        run += t;
      }
      ly.row_offset[src_size] = e;
      std::vector<uint32_t> cursor(ly.row_offset.begin(), ly.row_offset.end());
      ly.csr_edge_id.assign(e, 0);
      for (uint32_t k = 0; k < v; ++k)
        for (uint32_t j = ly.column_offset[k]; j < ly.column_offset[k + 1]; ++j) {
          const uint32_t slot = cursor[ly.row_indices[j]]++;
          ly.column_indices[slot] = k;
          ly.csr_edge_id[slot] = j;
        }
    }
    // WeightCompute (core/coocsc.hpp:301-324) with Sum / Mean lambdas (:1111-1119)
    std::vector<uint32_t> up_out, up_in;  // per local src / local dst (UP_DEGREE)
    if (up_degree) {
      up_out.assign(src_size, 0);
      up_in.assign(v, 0);
      for (uint32_t k = 0; k < v; ++k) up_in[k] = ly.column_offset[k + 1] - ly.column_offset[k];
      for (uint32_t k = 0; k < e; ++k) up_out[ly.row_indices[k]]++;
    }
    auto wfun2 = [&](uint32_t src_l, uint32_t dst_l) -> float {
      const uint32_t od = up_degree ? up_out[src_l] : s.outdeg[ly.source[src_l]];
      const uint32_t id = up_degree ? up_in[dst_l] : s.indeg[ly.destination[dst_l]];
      float w = norm_degree(od, id);
      if (weight_type == W_MEAN) w = w / id;
      if (weight_type == W_MEAN_SAMPLED)
        w = w / (float)(ly.column_offset[dst_l + 1] - ly.column_offset[dst_l]);
      return w;
    };
    if (weight_type != W_NONE) {
      ly.edge_weight_backward.assign(e, 0.f);
      ly.edge_weight_forward.assign(e, 0.f);
      for (uint32_t r = 0; r < src_size; ++r)
        for (uint32_t j = ly.row_offset[r]; j < ly.row_offset[r + 1]; ++j)
          ly.edge_weight_backward[j] = wfun2(r, ly.column_indices[j]);
      for (uint32_t k = 0; k < v; ++k)
        for (uint32_t j = ly.column_offset[k]; j < ly.column_offset[k + 1]; ++j)
          ly.edge_weight_forward[j] = wfun2(ly.row_indices[j], k);
    } else {
      ly.edge_weight_backward.clear();
      ly.edge_weight_forward.clear();
    }
  }
  return 0;
}

int orc_layer_size(void* h, int l, uint32_t* out3) {
  Sampler& s = *(Sampler*)h;
  const Layer& ly = s.layers[l];
  out3[0] = ly.v_size;
  out3[1] = ly.e_size;
  out3[2] = ly.src_size;
  return 0;
}

static void cp(void* dst, const void* src, size_t bytes) {
  if (dst && bytes) std::memcpy(dst, src, bytes);
}

int orc_layer_copy(void* h, int l, uint32_t* destination, uint32_t* column_offset,
                   uint32_t* row_indices, uint32_t* sample_ans, uint32_t* source,
                   float* edge_weight_forward, uint32_t* row_offset, uint32_t* column_indices,
                   float* edge_weight_backward) {
  Sampler& s = *(Sampler*)h;
  const Layer& ly = s.layers[l];
  cp(destination, ly.destination.data(), ly.v_size * 4);
  cp(column_offset, ly.column_offset.data(), (ly.v_size + 1) * 4);
  cp(row_indices, ly.row_indices.data(), ly.e_size * 4);
  cp(sample_ans, ly.sample_ans.data(), ly.e_size * 4);
  cp(source, ly.source.data(), ly.src_size * 4);
  if (!ly.edge_weight_forward.empty()) cp(edge_weight_forward, ly.edge_weight_forward.data(), ly.e_size * 4);
  if (!ly.row_offset.empty()) {
    cp(row_offset, ly.row_offset.data(), (ly.src_size + 1) * 4);
    cp(column_indices, ly.column_indices.data(), ly.e_size * 4);
  }
  if (!ly.edge_weight_backward.empty())
    cp(edge_weight_backward, ly.edge_weight_backward.data(), ly.e_size * 4);
  return 0;
}

// merge-mode / CSR extras of layer l: dst_local_id [v_size] (if merged),
// csr_edge_id [e_size] (if the CSR was built)
int orc_layer_extra(void* h, int l, uint32_t* dst_local_id, uint32_t* csr_edge_id) {
  Sampler& s = *(Sampler*)h;
  const Layer& ly = s.layers[l];
  if (!ly.dst_local_id.empty()) cp(dst_local_id, ly.dst_local_id.data(), ly.v_size * 4);
  if (!ly.csr_edge_id.empty()) cp(csr_edge_id, ly.csr_edge_id.data(), ly.e_size * 4);
  return (ly.dst_local_id.empty() ? 0 : 1) | (ly.csr_edge_id.empty() ? 0 : 2);
}

// Serialized std::mt19937 state (624 words + position), libstdc++ operator<<.
int orc_mt_state(void* h, uint32_t* out625) {
  Sampler& s = *(Sampler*)h;
  std::stringstream ss;
  ss << s.gen;
  for (int i = 0; i < 625; ++i) {
    unsigned long x;
    ss >> x;
    out625[i] = (uint32_t)x;
  }
  return 0;
}

// nts::op::PushDownBatchOp::forward (core/ntsPushdownGraphOp.hpp:108-160): rows
// [v_begin, v_end) of one sampled layer, Y[d - v_begin] = sum_e e_w_f[e] *
// X[source[row_indices[e]]] (the GLOBAL feature table, the sampled forward
// weights), zero-initialised, nts_comp arithmetic (mul then add)
int orc_pushdown_fwd(uint32_t v_begin, uint32_t v_end, const uint32_t* co, const uint32_t* ri,
                     const uint32_t* source, const float* ewf, const float* X, uint32_t F,
                     float* Y) {
  for (uint32_t d = v_begin; d < v_end; ++d) {
    float* out = Y + (uint64_t)(d - v_begin) * F;
    std::fill(out, out + F, 0.0f);
    for (uint32_t e = co[d]; e < co[d + 1]; ++e) {
      const float* in = X + (uint64_t)source[ri[e]] * F;
      const float w = ewf[e];
      for (uint32_t k = 0; k < F; ++k) out[k] = in[k] * w + out[k];
    }
  }
  return 0;
}

// preSample's get_most_neighbor (core/ntsBaseOp.hpp:330-404, the cache_rate
// overload) for one super-batch, single thread:
//   old[seeds] = 1; (layers-1) x { new = 0; new[u] += old[v] for u in the CSC
//   segment of v with old[v] > 0; swap }; counts = new
//   sorted = counts descending; total = (index of the first 0) + 1
//   (V when there is none — the reference leaves it unset); n = (VertexId)
//   (total * cache_rate) (float product); pivot = sorted[n] (clamped: n <= V,
//   pivot 0 at n == V); ids = the first n vertices, ascending, with
//   counts >= pivot (the reference's OpenMP loop visits them in this order
//   on one thread)
int orc_presample(uint64_t V, const uint64_t* off, const uint32_t* rows, const uint32_t* seeds,
                  uint32_t n_seeds, int layers, float cache_rate, uint32_t* counts_out,
                  uint32_t* ids_out, uint32_t* n_out) {
  std::vector<uint32_t> oldc(V, 0), newc(V, 0);
  for (uint32_t i = 0; i < n_seeds; ++i) oldc[seeds[i]] = 1;
  for (int layer = 1; layer < layers; ++layer) {
    if (layer != 1) {
      std::swap(oldc, newc);
      std::fill(newc.begin(), newc.end(), 0u);
    }
    for (uint64_t v = 0; v < V; ++v)
      if (oldc[v] > 0)
        for (uint64_t e = off[v]; e < off[v + 1]; ++e) newc[rows[e]] += oldc[v];
  }
  std::vector<uint32_t> sorted(newc);
  std::sort(sorted.begin(), sorted.end(), [](uint32_t a, uint32_t b) { return a > b; });
  uint64_t total = V;
  for (uint64_t i = 0; i < V; ++i)
    if (sorted[i] == 0) {
      total = i + 1;
      break;
    }
  uint64_t n = (uint64_t)((float)total * cache_rate);
  if (n > V) n = V;
  const uint32_t pivot = n < V ? sorted[n] : 0u;
  uint64_t k = 0;
  for (uint64_t v = 0; v < V && k < n; ++v)
    if (newc[v] >= pivot) ids_out[k++] = (uint32_t)v;
  *n_out = (uint32_t)n;
  if (counts_out) std::memcpy(counts_out, newc.data(), V * sizeof(uint32_t));
  return 0;
}

// nts::op::get_feature (core/ntsMiniBatchGraphOp.hpp:45-60)
int orc_get_feature(uint32_t n, const uint32_t* idx, const float* table, uint32_t F,
                    float* out, int threads) {
#pragma omp parallel for num_threads(threads > 1 ? threads : 1)
  for (uint32_t i = 0; i < n; ++i)
    std::memcpy(out + (uint64_t)i * F, table + (uint64_t)idx[i] * F, F * sizeof(float));
  return 0;
}

// MiniBatchFuseOp::forward (core/ntsMiniBatchGraphOp.hpp:153-182): output zeroed
// (NewKeyTensor = torch::zeros), then for every dst, for every edge in CSC
// order, out += in * w with w recomputed by nts_norm_degree (nts_comp,
// core/ntsBaseOp.hpp:546-562: mul then add, no FMA — build with -ffp-contract=off).
int orc_fuse_fwd(uint32_t v, const uint32_t* co, const uint32_t* ri, const uint32_t* source,
                 const uint32_t* destination, const uint32_t* outdeg, const uint32_t* indeg,
                 const float* X, uint32_t F, float* Y, int weight_mean, int threads) {
#pragma omp parallel for schedule(static) num_threads(threads > 1 ? threads : 1)
  for (uint32_t d = 0; d < v; ++d) {
    float* out = Y + (uint64_t)d * F;
    std::fill(out, out + F, 0.0f);
    const uint32_t dg = destination[d];
    for (uint32_t e = co[d]; e < co[d + 1]; ++e) {
      const uint32_t ls = ri[e];
      float w = norm_degree(outdeg[source[ls]], indeg[dg]);
      if (weight_mean) w = w / indeg[dg];
      const float* in = X + (uint64_t)ls * F;
      for (uint32_t k = 0; k < F; ++k) out[k] = in[k] * w + out[k];
    }
  }
  return 0;
}

static inline void cas_add(float* p, float x) {
  // write_add (dep/gemini/atomic.hpp:54-60): CAS loop on the float bits
  std::atomic_ref<float> a(*p);
  float old = a.load(std::memory_order_relaxed);
  while (!a.compare_exchange_weak(old, old + x, std::memory_order_relaxed)) {
  }
}

// MiniBatchFuseOp::backward (core/ntsMiniBatchGraphOp.hpp:214-268):
// G_in[src,:] += G_out[dst,:] * w (nts_acc, core/ntsBaseOp.hpp:579-584).
// threads == 1: dst-ascending order (the deterministic restatement);
// threads > 1 : CAS per float like the reference (timing only).
int orc_fuse_bwd(uint32_t v, uint32_t s, const uint32_t* co, const uint32_t* ri,
                 const uint32_t* source, const uint32_t* destination, const uint32_t* outdeg,
                 const uint32_t* indeg, const float* G, uint32_t F, float* Gin, int weight_mean,
                 int threads) {
  std::fill(Gin, Gin + (uint64_t)s * F, 0.0f);
  auto body = [&](uint32_t d, bool atomic) {
    const uint32_t dg = destination[d];
    const float* g = G + (uint64_t)d * F;
    for (uint32_t e = co[d]; e < co[d + 1]; ++e) {
      const uint32_t ls = ri[e];
      float w = norm_degree(outdeg[source[ls]], indeg[dg]);
      if (weight_mean) w = w / indeg[dg];
      float* out = Gin + (uint64_t)ls * F;
      if (atomic)
        for (uint32_t k = 0; k < F; ++k) cas_add(&out[k], g[k] * w);
      else
        for (uint32_t k = 0; k < F; ++k) out[k] = out[k] + g[k] * w;
    }
  };
  if (threads <= 1) {
    for (uint32_t d = 0; d < v; ++d) body(d, false);
  } else {
#pragma omp parallel for num_threads(threads)
    for (uint32_t d = 0; d < v; ++d) body(d, true);
  }
  return 0;
}

}  // extern "C"
