// pybind11 bindings of the C++ host layer (tests, bench.py, smoke()).
#include <torch/extension.h>

#include "gcn.hpp"

namespace py = pybind11;
using namespace nts;

static std::vector<VertexId> to_ids(const torch::Tensor& t) {
  auto c = t.to(torch::kCPU).to(torch::kInt64).contiguous();
  std::vector<VertexId> v(c.numel());
  const int64_t* p = c.data_ptr<int64_t>();
  for (size_t i = 0; i < v.size(); ++i) v[i] = (VertexId)p[i];
  return v;
}

static py::list layers_of(SampledSubgraph* sg) {
  py::list out;
  for (auto* s : sg->sampled_sgs) {
    py::dict d;
    auto n = [](const torch::Tensor& t, int64_t k) {
      return t.defined() ? t.narrow(0, 0, std::min<int64_t>(k, t.size(0))) : torch::Tensor();
    };
    d["v_size"] = s->v_size;
    d["e_size"] = s->e_size;
    d["src_size"] = s->src_size;
    d["destination"] = n(s->destination, s->v_size);
    d["column_offset"] = n(s->column_offset, s->v_size + 1);
    d["row_indices"] = n(s->row_indices, s->e_size);
    d["sample_ans"] = n(s->sample_ans, s->e_size);
    d["source"] = n(s->source, s->src_size);
    d["edge_weight_forward"] = n(s->edge_weight_forward, s->e_size);
    if (s->has_csr) {
      d["row_offset"] = n(s->row_offset, s->src_size + 1);
      d["column_indices"] = n(s->column_indices, s->e_size);
      d["edge_weight_backward"] = n(s->edge_weight_backward, s->e_size);
    }
    out.append(d);
  }
  return out;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "nts C++ host layer (libtorch-ROCm) over libnts_hip.so";

  py::enum_<WeightType>(m, "WeightType")
      .value("Sum", WeightType::Sum)
      .value("Mean", WeightType::Mean)
      .value("None", WeightType::None)
      .value("MeanSampled", WeightType::MeanSampled);

  py::class_<FullyRepGraph, std::shared_ptr<FullyRepGraph>>(m, "FullyRepGraph")
      .def_static(
          "from_edges",
          [](const torch::Tensor& src, const torch::Tensor& dst, VertexId V) {
            NtsStream cs(src.device().index(), nullptr, 2000);
            return FullyRepGraph::from_edges(cs, src, dst, V);
          },
          py::arg("src"), py::arg("dst"), py::arg("vertices"))
      .def_static("from_csc", &FullyRepGraph::from_csc)
      .def_readonly("global_vertices", &FullyRepGraph::global_vertices)
      .def_readonly("global_edges", &FullyRepGraph::global_edges)
      .def_readonly("column_offset", &FullyRepGraph::column_offset)
      .def_readonly("row_indices", &FullyRepGraph::row_indices)
      .def_readonly("in_degree", &FullyRepGraph::in_degree)
      .def_readonly("out_degree", &FullyRepGraph::out_degree);

  // FastSampler driven from Python (tests): owns its own stream context.
  struct PySampler {
    std::unique_ptr<NtsStream> cs;
    std::unique_ptr<FastSampler> s;
  };
  py::class_<PySampler>(m, "FastSampler")
      .def(py::init([](std::shared_ptr<FullyRepGraph> g, const torch::Tensor& seeds, int layers,
                       int batch, std::vector<int> fanout, int rng_mode, uint64_t seed,
                       bool csr, int pipeline) {
             auto p = new PySampler();
             TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize");
             p->cs = std::make_unique<NtsStream>(g->device, nullptr, seed);
             auto guard = p->cs->guard();
             std::vector<bool> c(layers, csr);
             p->s = std::make_unique<FastSampler>(g, to_ids(seeds), layers, batch, fanout, pipeline,
                                                  c, true);
             p->s->rng_mode = rng_mode;
             return p;
           }),
           py::arg("graph"), py::arg("seeds"), py::arg("layers"), py::arg("batch_size"),
           py::arg("fanout"), py::arg("rng_mode") = (int)NTS_RNG_PHILOX, py::arg("seed") = 2000,
           py::arg("csr") = true, py::arg("pipeline") = 1)
      // the split form (several slots in flight, finished in issue order)
      .def("issue",
           [](PySampler& p, int batch, int slot, WeightType w) {
             auto guard = p.cs->guard();
             p.s->issue_gpu_sample(batch, slot, *p.cs, w);
           },
           py::arg("batch_size"), py::arg("slot"), py::arg("weight_type") = WeightType::Sum)
      .def("finish",
           [](PySampler& p, int slot) {
             auto guard = p.cs->guard();
             auto out = layers_of(p.s->finish_gpu_sample(slot));
             p.cs->synchronize();
             return out;
           },
           py::arg("slot"))
      // MT19937 modes: scale every later layer's word bound (tests force a
      // short stream with a small scale; a re-run multiplies it by 4)
      .def("set_mt_budget_scale",
           [](PySampler& p, double scale) { p.s->set_mt_budget_scale(*p.cs, scale); })
      .def_property_readonly("mt_budget_scale", [](PySampler& p) { return p.s->mt_budget_scale(); })
      .def_property_readonly("mt_reruns", [](PySampler& p) { return p.s->mt_reruns; })
      .def("sample_gpu_fast",
           [](PySampler& p, int batch, WeightType w) {
             auto guard = p.cs->guard();
             auto out = layers_of(p.s->sample_gpu_fast(batch, 0, *p.cs, w));
             p.cs->synchronize();
             return out;
           },
           py::arg("batch_size"), py::arg("weight_type") = WeightType::Sum)
      .def("sample_not_finished", [](PySampler& p) { return p.s->sample_not_finished(); })
      .def("restart", [](PySampler& p) { p.s->restart(); })
      .def("rng_state",
           [](PySampler& p) {
             // the MT19937 modes' generator (624 words + _M_p), as std::mt19937 holds it
             auto out = torch::empty({625}, torch::kInt32);
             p.cs->synchronize();
             TORCH_CHECK(nts_hip_rng_state(p.cs->ctx(), (uint32_t*)out.data_ptr<int32_t>()) == 0,
                         nts_hip_last_error());
             return out;
           })
      .def_property("batch_seq", [](PySampler& p) { return p.s->batch_seq; },
                    [](PySampler& p, uint64_t v) { p.s->batch_seq = v; })
      .def_property_readonly("work_offset", [](PySampler& p) { return p.s->work_offset; })
      .def_property_readonly("sampled_edges", [](PySampler& p) { return p.s->sampled_edges; });

  m.def(
      "sampler_throughput",
      [](std::shared_ptr<FullyRepGraph> g, const torch::Tensor& seeds, int batch,
         std::vector<int> fanout, WeightType w, int rng_mode, int n_batches,
         std::vector<bool> csr) {
        SamplerRate r;
        {
          py::gil_scoped_release nogil;
          r = sampler_throughput(g, to_ids(seeds), batch, fanout, w, rng_mode, n_batches, csr);
        }
        py::dict d;
        d["seconds"] = r.seconds;
        d["edges"] = r.edges;
        d["batches"] = r.batches;
        return d;
      },
      py::arg("graph"), py::arg("seeds"), py::arg("batch_size"), py::arg("fanout"),
      py::arg("weight_type") = WeightType::Sum, py::arg("rng_mode") = (int)NTS_RNG_PHILOX,
      py::arg("n_batches") = 16, py::arg("csr_layers") = std::vector<bool>());

  py::class_<Communicator, std::shared_ptr<Communicator>>(m, "Communicator")
      .def(py::init([](int n, int r, py::bytes uid, int dev) {
        std::string s = uid;
        return std::make_shared<Communicator>(n, r, std::vector<uint8_t>(s.begin(), s.end()), dev);
      }))
      .def_static(
          "host",
          [](int n, int r, py::function fn) {
            // the Python callable runs with the GIL (pybind11's std::function
            // wrapper acquires it); train_batch releases it
            HostCollective h = [fn](torch::Tensor t, int op, int root) {
              py::gil_scoped_acquire g;
              fn(t, op, root);
            };
            return std::make_shared<Communicator>(n, r, h);
          },
          py::arg("nranks"), py::arg("rank"), py::arg("collective"))
      .def_property_readonly("host_transport", &Communicator::host_transport)
      .def("rccl_count", &Communicator::rccl_count)
      .def_static("unique_id",
                  []() {
                    auto v = Communicator::unique_id();
                    return py::bytes(std::string(v.begin(), v.end()));
                  })
      .def("allreduce_sum",
           [](Communicator& c, torch::Tensor t, uint64_t stream) {
             c.allreduce_sum(t.data_ptr<float>(), (uint64_t)t.numel(), (void*)stream);
           },
           py::arg("tensor"), py::arg("stream"))
      .def("set_timing", &Communicator::set_timing, py::arg("on"))
      .def("timing_reset", &Communicator::timing_reset)
      .def("timing_stats",
           [](Communicator& c) {
             auto t = c.timing_stats();
             py::dict d;
             d["us_per_call"] = std::get<0>(t);
             d["calls"] = std::get<1>(t);
             d["how"] = std::get<2>(t);
             return d;
           })
      .def_readonly("nranks", &Communicator::nranks)
      .def_readonly("rank", &Communicator::rank);

  py::class_<GCNConfig>(m, "GCNConfig")
      .def(py::init<>())
      .def_readwrite("layer_size", &GCNConfig::layer_size)
      .def_readwrite("fanout", &GCNConfig::fanout)
      .def_readwrite("batch_size", &GCNConfig::batch_size)
      .def_readwrite("learn_rate", &GCNConfig::learn_rate)
      .def_readwrite("weight_decay", &GCNConfig::weight_decay)
      .def_readwrite("drop_rate", &GCNConfig::drop_rate)
      .def_readwrite("beta1", &GCNConfig::beta1)
      .def_readwrite("beta2", &GCNConfig::beta2)
      .def_readwrite("epsilon", &GCNConfig::epsilon)
      .def_readwrite("rng_mode", &GCNConfig::rng_mode)
      .def_readwrite("sample_gpu", &GCNConfig::sample_gpu)
      .def_readwrite("weight_type", &GCNConfig::weight_type)
      .def_readwrite("fused_gather", &GCNConfig::fused_gather)
      .def_readwrite("bias_correction", &GCNConfig::bias_correction)
      .def_readwrite("deterministic_backward", &GCNConfig::deterministic_backward)
      .def_readwrite("hip_gemm", &GCNConfig::hip_gemm)
      .def_readwrite("pipeline", &GCNConfig::pipeline)
      .def_readwrite("transform_first", &GCNConfig::transform_first)
      .def_readwrite("gemm_mode", &GCNConfig::gemm_mode)
      .def_readwrite("pair_table", &GCNConfig::pair_table)
      .def_readwrite("overlap_allreduce", &GCNConfig::overlap_allreduce)
      .def_readwrite("pd_cache", &GCNConfig::pd_cache)
      .def_readwrite("pd_rate", &GCNConfig::pd_rate)
      .def_readwrite("pd_super_batch", &GCNConfig::pd_super_batch)
      .def_readwrite("early_aggregate", &GCNConfig::early_aggregate)
      .def_readwrite("sampler_priority", &GCNConfig::sampler_priority)
      .def_readwrite("fuse_loss", &GCNConfig::fuse_loss)
      .def_readwrite("sampler_cus", &GCNConfig::sampler_cus)
      .def_readwrite("sampler_gate", &GCNConfig::sampler_gate)
      .def_readwrite("pad_features", &GCNConfig::pad_features)
      .def_readwrite("cache_rate", &GCNConfig::cache_rate)
      .def_readwrite("up_degree", &GCNConfig::up_degree)
      .def_readwrite("gat", &GCNConfig::gat)
      .def_readwrite("fuse_activation", &GCNConfig::fuse_activation)
      .def_readwrite("shuffle", &GCNConfig::shuffle)
      .def_readwrite("profile", &GCNConfig::profile)
      .def_readwrite("seed", &GCNConfig::seed);

  py::class_<GCN_SAMPLE_ALLGPU_impl>(m, "GCN_SAMPLE_ALLGPU_impl")
      .def(py::init([](std::shared_ptr<FullyRepGraph> g, torch::Tensor feature,
                       torch::Tensor label, const torch::Tensor& train_nids, GCNConfig cfg,
                       std::shared_ptr<Communicator> comm) {
             return new GCN_SAMPLE_ALLGPU_impl(g, feature, label, to_ids(train_nids), cfg, comm);
           }),
           py::arg("graph"), py::arg("feature"), py::arg("label"), py::arg("train_nids"),
           py::arg("cfg"), py::arg("comm") = nullptr)
      .def("train_batch", &GCN_SAMPLE_ALLGPU_impl::train_batch,
           py::call_guard<py::gil_scoped_release>())
      .def("run_epoch", &GCN_SAMPLE_ALLGPU_impl::run_epoch,
           py::call_guard<py::gil_scoped_release>())
      .def("forward_eval",
           [](GCN_SAMPLE_ALLGPU_impl& d, const torch::Tensor& seeds, uint64_t bs) {
             return d.forward_eval(to_ids(seeds), bs);
           },
           py::arg("seeds"), py::arg("batch_seq") = 0)
      .def("set_weights", &GCN_SAMPLE_ALLGPU_impl::set_weights)
      .def("train_correct", &GCN_SAMPLE_ALLGPU_impl::train_correct)
      .def("presample", &GCN_SAMPLE_ALLGPU_impl::presample)
      .def("set_presample", &GCN_SAMPLE_ALLGPU_impl::set_presample)
      .def("reset_correct", &GCN_SAMPLE_ALLGPU_impl::reset_correct)
      .def("evaluate",
           [](GCN_SAMPLE_ALLGPU_impl& d, const torch::Tensor& nids) {
             auto ids = to_ids(nids);
             py::gil_scoped_release nogil;
             return d.evaluate(ids);
           },
           py::arg("nids"))
      .def("weights", &GCN_SAMPLE_ALLGPU_impl::weights)
      .def("reset_stats", &GCN_SAMPLE_ALLGPU_impl::reset_stats)
      .def("set_diag_reuse_sample", &GCN_SAMPLE_ALLGPU_impl::set_diag_reuse_sample)
      .def("resolve_profile",
           [](GCN_SAMPLE_ALLGPU_impl& d) {
             // {kernel: {"ms": total device ms, "calls": n, "units": algorithmic
             //  bytes (aggregations) or flops (GEMMs) summed over the calls}}
             d.resolve_profile();
             py::dict out;
             for (int i = 0; i < KernelProfiler::kCount; ++i) {
               const auto& st = d.prof.stat[i];
               if (!st.calls) continue;
               py::dict e;
               e["ms"] = st.ms;
               e["calls"] = st.calls;
               e["units"] = st.units;
               out[KernelProfiler::name(i)] = e;
             }
             return out;
           })
      .def_property_readonly("transform_first", &GCN_SAMPLE_ALLGPU_impl::transform_first)
      .def("sample_not_finished", &GCN_SAMPLE_ALLGPU_impl::has_batch)
      .def("restart", &GCN_SAMPLE_ALLGPU_impl::restart)
      .def("synchronize", [](GCN_SAMPLE_ALLGPU_impl& d) { d.sync(); })
      .def_property_readonly("loss", [](GCN_SAMPLE_ALLGPU_impl& d) { return d.loss; })
      .def_property_readonly("n_train", [](GCN_SAMPLE_ALLGPU_impl& d) { return d.sampler->work_range[1]; })
      .def_property_readonly("last_layers",
                             [](GCN_SAMPLE_ALLGPU_impl& d) {
                               // the last TRAINED batch (the sampler's current
                               // slot may already hold the next, in flight)
                               return layers_of(d.last_sg ? d.last_sg : d.sampler->ssg);
                             })
      .def_readonly("sample_time", &GCN_SAMPLE_ALLGPU_impl::sample_time)
      .def_readonly("train_time", &GCN_SAMPLE_ALLGPU_impl::train_time)
      .def_readonly("batch_edges", &GCN_SAMPLE_ALLGPU_impl::batch_edges)
      .def_readonly("batches", &GCN_SAMPLE_ALLGPU_impl::batches);
}
